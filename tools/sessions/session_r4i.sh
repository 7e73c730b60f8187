# round-4 session I: the per-call path with the host waiting on
# the reduction's sequence flag (mapped memory) — overhead probe new vs old path (SUP_FLAG_WAIT=0),
# dwt_59 with 8 leaf workers both ways (8 spinning waits), the GPU suite, and the bench line with its config lines
OLD="env SUP_FLAG_WAIT=0"
bash tools/gpu_session.sh r4i \
 "overhead_new=python3 tools/probe_overhead.py" \
 "overhead_old=$OLD python3 tools/probe_overhead.py" \
 "overhead_new2=python3 tools/probe_overhead.py" \
 "reduce_new=env PROBE_SPARSE=0 PROBE_BATCHES=1 PROBE_WORKERS=1,8 python3 tools/probe_reduce.py will57.mtx dwt_59.mtx" \
 "reduce_old=$OLD PROBE_SPARSE=0 PROBE_BATCHES=1 PROBE_WORKERS=1,8 python3 tools/probe_reduce.py will57.mtx dwt_59.mtx" \
 "pytest_gpu=python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "bench=python3 bench.py --steps 3 --warmup 1"
