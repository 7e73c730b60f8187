# round-3 session C: whole GPU suite (pinned seg-walk tests included), the
# default bench line (live PMC flops, cold/warm CLI), rocprofv3 stats of it
bash tools/gpu_session.sh r3c \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "bench=python3 bench.py" \
 "prof=rocprofv3 --kernel-trace --stats -d gpurun_out/r3c/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --configs 0 --pmc 0 --cold 0"
