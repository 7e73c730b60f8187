# Step-region size of the segmented walk (SGPR pieces per region, Plan::seg_kp; default 4) on the bench matrix.
mkdir -p gpurun_out/kp
for kp in 3 4 5 6; do
  SUP_JIT_KP=$kp timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 > gpurun_out/kp/kp$kp.log 2>&1 || exit $?
  echo "kp $kp: $(grep '^{' gpurun_out/kp/kp$kp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"], d["roofline"]["flops_definition"][:12])')"
done
