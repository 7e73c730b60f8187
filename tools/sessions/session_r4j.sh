# round-4 session J: hoisting the piece-free statements of a region ahead of its pin (SUP_JIT_HOIST, default on)
# and the prefetch / cross-step knobs, re-measured now that the generator reads them per kernel (session F read
# them once per process: its PF / XSTEP legs had compiled the default kernel); interleaved on one box
bash tools/gpu_session.sh r4j \
 "ab_hoist=env PROBE_TORCH=1 PROBE_CASES=double__40_0.50_0,double__40_0.90_0,double__40_0.20_0,double__36_0.20_0 python3 tools/probe_ab.py SUP_JIT_HOIST=0 SUP_JIT_PF=0 SUP_JIT_XSTEP=0 - SUP_JIT_HOIST=0" \
 "seg_tests=python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_seg.py tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu"
