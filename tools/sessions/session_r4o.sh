# round-4 session O: the launcher's 2- and 4-rank rehearsals on the final tree (gloo, all ranks on GPU 0; each leg's
# permanent must equal the one-rank line's bits), then the one-rank default bench line
bash tools/gpu_session.sh r4o \
 "rehearse2=python3 bench.py --gpus 2 --rehearse --steps 2 --warmup 1 --cpu-seconds 0 --pmc 0 --cold 0" \
 "rehearse4=python3 bench.py --gpus 4 --rehearse --steps 2 --warmup 1 --cpu-seconds 0 --pmc 0 --cold 0" \
 "bench=python3 bench.py"
