# round-4 session Q, the final tree again (visited sums on the device, one-item queues, n = 64 parity): the whole
# GPU suite and smoke, as the driver runs them at round end
bash tools/gpu_session.sh r4q \
 "pytest_gpu=python3 -u -m pytest -q -x --timeout 600 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 smoke
