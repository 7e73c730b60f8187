# round-3 session T: per-call overhead with the tables staged through pinned memory (A: previous commit's
# library built as superman_amd/lib_prev, B: this tree), -o probe, and the GPU parity + reduction tests
bash tools/gpu_session.sh r3t \
 "overhead=python3 -u tools/probe_overhead.py" \
 "reduce_tests=python3 -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_reduce_workers.py tests/test_gpu_seg.py tests/test_gpu_pinned.py -m gpu" \
 "probe_reduce=python3 -u tools/probe_reduce.py chesapeake.mtx will57.mtx dwt_59.mtx"
