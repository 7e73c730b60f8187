# round-4 session D: the per-call path without the counter memset and the result copy (the reduction zeroes the
# queue head and writes the result to mapped host memory) — whole GPU suite, the overhead probe, the bench line
bash tools/gpu_session.sh r4d \
 "pytest_gpu=python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "overhead=python3 tools/probe_overhead.py" \
 "smoke=python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench=python3 bench.py --steps 3 --warmup 1"
