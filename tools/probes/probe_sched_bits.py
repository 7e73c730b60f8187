"""where do the bits of the n = 28 walk of
test_seg_codegen_schedule_invariance_gpu differ under SUP_JIT_SCHED=max-ilp
with SUP_JIT_KP=1?  For each code-generation setting: the plan the engine
walks (plan_info, plan_key), the full permanent three times (determinism), and
every wave-chunk's partial (perman_shard with one shard per chunk) against the
oracle's engine-schedule mirror of the same chunk.  GPU probe; the oracle is
the checker only."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import superman_amd as sup  # noqa: E402

os.environ.setdefault("SUP_JIT_CACHE_DIR", tempfile.mkdtemp(prefix="supjit_"))
rng = np.random.default_rng(91)
n = 28
a = np.where(rng.random((n, n)) < 0.5, rng.random((n, n)) * 5, 0.0)
a[np.arange(n), rng.permutation(n)] = 1.0

SETTINGS = [dict(), dict(SUP_JIT_KP="1"), dict(SUP_JIT_SCHED="max-ilp"), dict(SUP_JIT_SCHED="max-ilp", SUP_JIT_KP="1")]
if len(sys.argv) > 1:
    SETTINGS = [dict(kv.split("=") for kv in arg.split(",") if kv) for arg in sys.argv[1:]]
mirror_full = None
for s in SETTINGS:
    for k in ("SUP_JIT_SCHED", "SUP_JIT_KP"):
        os.environ.pop(k, None)
    os.environ.update(s)
    info = sup.plan_info(a, "seg", jit=1)
    key = sup.plan_key(a, "seg", jit=1)
    L, m, cc, pb = info["L"], info["m"], info["cached"], info["pair_bits"]
    h = n - 1 - L - m
    want = oracle.engine_perman_as(sup, a, "seg", threads=16, jit=1)
    got = [sup.perman(a, algo=4, kernel="seg", jit=1) for _ in range(3)]
    print(f"setting {s or 'default'}: key {key:#x} L {L} m {m} cc {cc} b {pb} ops {info['est_ops_per_step']:.4f}"
          f" colmap {info['colmap'].tolist()}", flush=True)
    print(f"  full: got {[repr(g) for g in got]} mirror {want!r} equal {[g == want for g in got]}", flush=True)
    nch = 1 << h
    parts = np.array([sup.perman_shard(a, c, nch, kernel="seg", jit=1) for c in range(nch)])
    parts2 = np.array([sup.perman_shard(a, c, nch, kernel="seg", jit=1) for c in range(nch)])
    mir = np.array([oracle.engine_range(a, "seg", c, c + 1, L, m, info["colmap"], 16, cc, pb)[0] for c in range(nch)])
    bad = np.nonzero(parts != mir)[0]
    rep = np.nonzero(parts != parts2)[0]
    print(f"  chunks: {nch}, differing from mirror {len(bad)}, differing between two runs {len(rep)}", flush=True)
    for c in bad[:12]:
        rel = abs(parts[c] - mir[c]) / max(abs(mir[c]), 1e-300)
        print(f"    chunk {c} ({c:#x}): got {parts[c]!r} mirror {mir[c]!r} rel {rel:.3e}", flush=True)
