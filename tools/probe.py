"""Quick GPU probe: correctness on a small case, then throughput per n."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import superman_amd as S
import oracle
rng = np.random.default_rng(0)
a = rng.random((16, 16))
g, st = S.perman(a, return_stats=True)
print("n16 dense", g, oracle.engine_perman(a, "dense", 4), st, flush=True)
for kind, algo, sp in (("sparse", 4, True), ("skip", 7, True)):
    g = S.perman(a, algo=algo, sparse=sp)
    print("n16", kind, g, oracle.engine_perman(a, kind, 4), flush=True)
for path in ("double__32_0.50_0", "double__36_0.20_0", "double__40_0.50_0"):
    m, _, _ = S.read_matrix(os.path.join("tests/fixtures", path))
    n = m.shape[0]
    for kind, algo, sp in (("dense", 4, False), ("sparse", 4, True)):
        mm = S.sort_order(m)[0] if sp else m
        S.perman(mm, algo=algo, sparse=sp)
        t = time.perf_counter()
        v, st = S.perman(mm, algo=algo, sparse=sp, return_stats=True)
        dt = time.perf_counter() - t
        steps = 2 ** (n - 1)
        print(f"{path} {kind}: perm={v:.17e} wall={dt*1e3:.1f}ms kernel={st['kernel_ms']:.1f}ms "
              f"steps/s={steps/(st['kernel_ms']*1e-3):.3e} fp64 frac={2*n*steps/(st['kernel_ms']*1e-3)/78.6e12:.3f} "
              f"grid={st['grid']}", flush=True)
