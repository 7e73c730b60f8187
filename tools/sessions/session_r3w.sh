# round-3 session W: the 8-rank bench path rehearsed on one GPU (gloo, all ranks on device 0), every leg
bash tools/gpu_session.sh r3w \
 "rehearse8=python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --rehearse --steps 2 --warmup 1"
