# round-3 session S: leaf memo on the GPU — the reduction tests (workers and callback path), then dwt_59 with
# 4 workers (memo) for the timing
bash tools/gpu_session.sh r3s \
 "reduce_tests=python3 -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_reduce_workers.py tests/test_gpu_exact.py tests/test_gpu_quad.py -m gpu" \
 "probe_reduce=python3 -u tools/probe_reduce.py chesapeake.mtx will57.mtx dwt_59.mtx"
