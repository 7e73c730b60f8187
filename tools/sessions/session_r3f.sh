# round-3 session F: the queue's tail phase (generated walk), whole GPU suite,
# and the N-rank bench path rehearsed on one GPU (2 ranks, gloo)
bash tools/gpu_session.sh r3f \
 "group=python3 -u tools/probe_group.py double__40_0.50_0 t0 t4 t2 t1 4" \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "rehearse2=python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --rehearse --configs 0 --cpu-seconds 0"
