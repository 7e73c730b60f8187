# round-3 session P: -o reductions on the GPU (wall vs walk-kernel time), before batching the leaves
bash tools/gpu_session.sh r3p "probe_reduce=python3 -u tools/probe_reduce.py"
