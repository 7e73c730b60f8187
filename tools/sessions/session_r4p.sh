# round-4 session P: the segmented walk at the maximum order (n = 64, d = 0.5 and 0.9) against the oracle's mirror
bash tools/gpu_session.sh r4p \
 "maxsize=python3 -u -m pytest -v -x --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_maxsize.py -m gpu -k seg_large"
