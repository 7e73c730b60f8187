# round-4 session A: the new launcher / checkpoint / RCCL-map / large-n tests, the bench entry point with --gpus 2 (rehearsal)
bash tools/gpu_session.sh r4a \
 "newtests=python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py tests/test_gpu_checkpoint.py tests/test_capi.py tests/test_bench_launch.py tests/test_gpu_maxsize.py" \
 "bench2=python3 bench.py --gpus 2 --rehearse --steps 2 --warmup 1 --configs 0 --cpu-seconds 0 --pmc 0 --cold 0" \
 "bench1=python3 bench.py --gpus 1 --steps 2 --warmup 1 --configs 0 --cpu-seconds 0 --pmc 0 --cold 0"
