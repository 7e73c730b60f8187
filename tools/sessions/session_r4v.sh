# round-4 session V: after reverting the scheduler default — the segmented-walk GPU tests and smoke on the tree as
# committed
bash tools/gpu_session.sh r4v \
 "seg_tests=python3 -u -m pytest -q -x --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_seg.py tests/test_gpu_pinned.py tests/test_gpu_callpath.py -m gpu" \
 smoke
