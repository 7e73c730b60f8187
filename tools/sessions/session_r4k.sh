# round-4 session K, the final tree: whole GPU suite, smoke, the default bench line, and the bench's
# rocprofv3 --kernel-trace --stats summary (headline only, counters off)
OUT=gpurun_out/r4k
bash tools/gpu_session.sh r4k \
 "pytest_gpu=python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 smoke \
 "bench=python3 bench.py" \
 "prof=rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
