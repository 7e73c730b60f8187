#!/usr/bin/env python3
"""which dense (n, d) patterns get a segmented plan.

For n in {44,...,64} x d in {0.5, 0.9} (seeded random matrices, the corpus
style: Bernoulli(d) pattern, U(0,5) values, a permutation diagonal so no row
or column is empty) plan the segmented walk (sup_plan_info kernel "seg",
jit 1: walk-order search + the compiler check's hiprtc compiles + the code
scan) on the CPU — no GPU needed — and report the kind, cached bits, pair bits,
modelled ops per Gray step, the prefix-blocked walk's ops for comparison, and
the error when the engine refuses.  usage: sweep_large_n.py [n,...] [d,...]"""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402


def mat(n, d, seed):
    rng = np.random.default_rng(seed)
    a = np.where(rng.random((n, n)) < d, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0 + rng.random(n)
    return a


def main():
    ns = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [44, 46, 48, 52, 56, 60, 64]
    ds = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.5, 0.9]
    if "SUP_JIT_CACHE_DIR" not in os.environ:
        os.environ["SUP_JIT_CACHE_DIR"] = tempfile.mkdtemp(prefix="sup_sweep_")
    for n in ns:
        for d in ds:
            a = mat(n, d, 1000 * n + int(round(100 * d)))
            aot = S.plan_info(a, "dense", jit=-1)
            t = time.perf_counter()
            try:
                info = S.plan_info(a, "seg", jit=1)
                res = (f"seg cc={info['cached']} b={info['pair_bits']} m={info['m']} "
                       f"ops={info['est_ops_per_step']:.2f} ratio={info['est_ops_per_step'] / aot['est_ops_per_step']:.3f}")
            except S.SupError as e:
                res = "REFUSED " + str(e).splitlines()[0][:200]
            print(f"n={n} d={d} aot={aot['kind']}:{aot['est_ops_per_step']:.2f} {res} "
                  f"plan_s={time.perf_counter() - t:.1f}", flush=True)


if __name__ == "__main__":
    main()
