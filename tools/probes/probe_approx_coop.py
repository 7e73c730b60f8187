"""GPU probe: the estimators' per-lane form against the cooperative form (one
wave per sample, approx.hip approx_coop) on grid graphs; same bits, samples/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

for (m, n) in ((8, 8), (12, 12), (14, 14), (16, 16), (20, 20), (24, 24), (36, 36)):
    g = S.grid_graph(m, n)
    for algo in (1, 2):
        res = {}
        for form in ("0", "1"):
            os.environ["SUP_APPROX_COOP"] = form
            samples = 1 << 16 if form == "1" or m <= 16 else 1 << 12
            if algo == 2 and form == "0" and m >= 24:
                samples = 1 << 10
            S.approx(g, algo, samples=1024, seed=1)
            est, st = S.approx(g, algo, samples=samples, seed=2, return_stats=True)
            res[form] = (est, st["samples"] / (st["kernel_ms"] * 1e-3))
        same = S.approx(g, algo, samples=1024, seed=3) == (os.environ.update(SUP_APPROX_COOP="0") or
                                                           S.approx(g, algo, samples=1024, seed=3))
        print(f"grid {m}x{n} (nov {g.shape[0]}) algo {algo}: per-lane {res['0'][1]:.3e} samples/s, "
              f"cooperative {res['1'][1]:.3e} samples/s ({res['1'][1] / res['0'][1]:.2f}x), same bits {same}",
              flush=True)
