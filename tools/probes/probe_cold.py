"""Cold segmented-plan cost (walk-order search + the compiler check's compiles)
per matrix and host thread count: the data auto mode's cold bar is fitted to
(VERDICT r4 next-2).  Each matrix is planned with an empty disk cache; a small
plan first loads the library and hiprtc.  No device needed."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import superman_amd as sup  # noqa: E402

os.environ["SUP_JIT_CACHE_DIR"] = tempfile.mkdtemp(prefix="cold_")
rng = np.random.default_rng(5)
w = np.where(rng.random((24, 24)) < 0.5, rng.random((24, 24)), 0.0) + np.eye(24)
sup.prepare(w, "dense", jit=1)
for name in sys.argv[1:]:
    os.environ["SUP_JIT_CACHE_DIR"] = tempfile.mkdtemp(prefix="cold_")
    a = sup.read_matrix(name)[0]
    t0 = time.time()
    info = sup.plan_info(a, "dense", jit=1)
    t1 = time.time()
    p = sup.prepare(a, "dense", jit=1)
    t2 = time.time()
    print(f"{os.path.basename(name)} n={a.shape[0]} threads={os.environ.get('OMP_NUM_THREADS')} cpus={os.cpu_count()}"
          f" plan {t1 - t0:.3f} s then compile {t2 - t1:.3f} s kind {info['kind']}"
          f" ops {info['est_ops_per_step']:.3f}", flush=True)
