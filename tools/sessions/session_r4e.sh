# round-4 session E: which hiprtc compiles the faster segmented walks — torch's bundled copy (what bench.py
# gets, since it imports torch first) against /opt/rocm's — on the bench matrices and configs 2, 3, 5
bash tools/gpu_session.sh r4e \
 "ab_rocm=python3 tools/probe_ab.py -" \
 "ab_torch=env PROBE_TORCH=1 python3 tools/probe_ab.py -" \
 "ab_rocm2=python3 tools/probe_ab.py -" \
 "ab_torch2=env PROBE_TORCH=1 python3 tools/probe_ab.py -"
