# round-3 session N: the tree with per-process auto-mode decisions, the measured cold bar and rank 0's
# auto decision in bench.py — GPU suite, then the N-rank bench path rehearsed on one GPU (gloo, all ranks on
# device 0) at 2 and 4 ranks with every leg (configs included: config 5's auto leg goes through auto_decision)
R="python3 -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_session.sh r3n \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "rehearse2=$R --nproc-per-node 2 --master-port 29521 bench.py --gpus 2 --rehearse --steps 2 --warmup 1" \
 "rehearse4=$R --nproc-per-node 4 --master-port 29523 bench.py --gpus 4 --rehearse --steps 2 --warmup 1"
