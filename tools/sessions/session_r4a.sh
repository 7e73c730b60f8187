# round-4 session A: the new launcher / checkpoint / RCCL-map / large-n / auto-mode / stream-sharing tests, the
# bench entry point with --gpus 2 (rehearsal), the per-call host cost, A/Bs of the SGPR piece budget
# (readlane-free loops) and of constant-stream sharing (d = 0.9), the counter list
bash tools/gpu_session.sh r4a \
 "newtests=python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py tests/test_gpu_checkpoint.py tests/test_capi.py tests/test_bench_launch.py tests/test_gpu_maxsize.py tests/test_gpu_seg.py" \
 "bench2=python3 bench.py --gpus 2 --rehearse --steps 2 --warmup 1 --configs 0 --cpu-seconds 0 --pmc 0 --cold 0" \
 "bench1=python3 bench.py --gpus 1 --steps 2 --warmup 1 --configs 0 --cpu-seconds 0 --pmc 0 --cold 0" \
 "overhead=python3 tools/probe_overhead.py" \
 "ab_kp=PROBE_TORCH=1 PROBE_CASES=double__40_0.50_0 python3 tools/probe_ab.py SUP_JIT_BUDGET=214 SUP_JIT_KP=3,SUP_JIT_BUDGET=206 SUP_JIT_KP=3,SUP_JIT_BUDGET=198 SUP_JIT_BUDGET=214 SUP_JIT_KP=3,SUP_JIT_BUDGET=206 SUP_JIT_KP=3,SUP_JIT_BUDGET=198" \
 "ab_share=PROBE_TORCH=1 PROBE_CASES=double__40_0.90_0 python3 tools/probe_ab.py SUP_JIT_NOSHARE=1 SUP_JIT_BUDGET=110 - SUP_JIT_NOSHARE=1" \
 "counters=rocprofv3 -L"
