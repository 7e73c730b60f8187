# round-3 session U (final tree): GPU suite, smoke, bench line
bash tools/gpu_session.sh r3u \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 smoke \
 "bench=python3 bench.py"
