# round-3 session L (re-entry after the container was re-created): the tree with the
# hiprtc-file cache keys — GPU suite, smoke, bench line, rocprofv3 stats of the headline
bash tools/gpu_session.sh r3l \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 smoke \
 "bench=python3 bench.py" \
 "prof=rocprofv3 --kernel-trace --stats -d gpurun_out/r3l/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --configs 0 --also= --pmc 0 --cold 0"
