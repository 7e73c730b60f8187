"""A/B of one SUP_JIT_* code-generation knob on the walk kernels the bench
times: each (matrix, setting) is planned and compiled, then timed (median of
5 launches through sup_perman_shard).  A setting is one or more env
assignments joined by commas; '-' is the default.  PROBE_CASES (comma-separated
fixture names) restricts the matrices; PROBE_TORCH=1 imports torch first (its
bundled HIP runtime, hiprtc and comgr then compile the kernels, as in bench.py).

    python3 tools/probes/probe_ab.py KNOB=val[,KNOB2=val] [...]
"""
import os
import statistics
import sys

if os.environ.get("PROBE_TORCH") == "1":
    import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

CASES = [("double__40_0.50_0", 0, "dense"), ("double__36_0.20_0", 1, "sparse"), ("double__32_0.50_0", 0, "dense"),
         ("double__40_0.20_0", 0, "dense"), ("synth44_0.15_int", 2, "skip")]
settings = ["-"] + sys.argv[1:]
if os.environ.get("PROBE_CASES"):  # fixture names; ones not listed above run as dense requests
    want = os.environ["PROBE_CASES"].split(",")
    CASES = [c for c in CASES if c[0] in want] + [(w, 0, "dense") for w in want if w not in [c[0] for c in CASES]]
for name, prep, kernel in CASES:
    a = S.read_matrix(os.path.join("tests", "fixtures", name))[0]
    if prep == 1:
        a = S.sort_order(a)[0]
    elif prep == 2:
        a = S.skip_order(a)[0]
    for st in settings:
        env = {}
        if st != "-":
            for kv in st.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        for k, v in env.items():
            os.environ[k] = v
        info = S.plan_info(a, kernel, jit=1)
        S.perman_shard(a, 0, 1, kernel=kernel, jit=1)
        ks = []
        for _ in range(5):
            v, stt = S.perman_shard(a, 0, 1, kernel=kernel, jit=1, return_stats=True)
            ks.append(stt["kernel_ms"])
        print(f"{name} {st}: ops {info['est_ops_per_step']:.3f} kernel median {statistics.median(ks):.3f} ms "
              f"(min {min(ks):.3f}) sum {v!r}", flush=True)
        for k in env:
            del os.environ[k]
