# round-4 session U: the max-ilp scheduler is the default now, so the walks have new plan keys: the counter
# profiles bench.py looks up by plan key (fp64 flops; FETCH_SIZE / WRITE_SIZE), the whole GPU suite, smoke, and the
# default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4u
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "STOP: $name exit $rc"; exit $rc; fi
}
P="rocprofv3 --kernel-trace -o run --output-format csv"
for d in 20 50 90; do
  M=tests/fixtures/double__40_0.${d}_0
  CHILD="python3 bench.py --pmc-child --kernel dense --jit 1 --prep 0 --matrix $M"
  step f64_$d 180 $P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/f64_$d -- $CHILD
  step fetch_$d 180 $P --pmc FETCH_SIZE -d $O/fetch_$d -- $CHILD
  step write_$d 180 $P --pmc WRITE_SIZE -d $O/write_$d -- $CHILD
  step sum_f64_$d 300 python3 tools/pmc_r4.py $O/pmc_f64_d0$d.json $M $O/f64_$d $O/fetch_$d $O/write_$d
  step sum_hbm_$d 300 python3 tools/pmc_r4.py $O/pmc_hbm_d0$d.json $M $O/fetch_$d $O/write_$d
done
step pytest_gpu 1200 python3 -u -m pytest -q -x --timeout 600 --timeout-method thread -p no:cacheprovider tests -m gpu
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python3 bench.py
step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0
echo "== done"
