# round-4 session N: visited states summed on the device (8 bytes back instead of a 4-byte count per wave-chunk):
# the tests that read visited counts, and the bench's config lines (config 5 -p8 is the one that changes)
bash tools/gpu_session.sh r4n \
 "vis_tests=python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_multidev.py tests/test_gpu_checkpoint.py tests/test_gpu_seg.py tests/test_gpu_callpath.py -m gpu" \
 "bench_cfg=python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --pmc 0 --cold 0 --also="
