"""GPU probe of the exact integer path (sup_perman_exact): time and primes on
the corpus int matrices and on the n = 40 bench pattern read with -b."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

FIX = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "fixtures")
for name, binary in (("int__30_0.50_0", False), ("int__36_0.20_0", False), ("double__32_0.50_0", True),
                     ("double__40_0.50_0", True)):
    a = S.read_matrix(os.path.join(FIX, name), binary=binary)[0]
    n = a.shape[0]
    t = time.perf_counter()
    e, st = S.perman_exact(a, return_stats=True)
    dt = time.perf_counter() - t
    f = S.perman(a, algo=4, jit=1)
    print(f"{name}{' -b' if binary else ''} n={n}: exact={e} kernel={st['kernel_ms']:.1f}ms wall={dt*1e3:.1f}ms "
          f"gray-steps/s={2**(n-1)/(st['kernel_ms']*1e-3):.3e} fp64-seg rel.err={abs(f-e)/abs(e):.2e}", flush=True)
