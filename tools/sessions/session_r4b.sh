# round-4 session B: the named north-star counters on the final kernels (LDS bank conflicts, LDS instructions,
# occupancy; scalar-cache hits at d = 0.9), one pass each per density through bench.py --pmc-child, then the
# whole GPU suite and the default bench line with its rocprofv3 --stats summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
have() { grep -qw "$1" "$OUT/counters.txt"; }
pick() { local out=""; for c in "$@"; do have "$c" && out="$out $c"; done; echo $out; }
LDSOCC=$(pick SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT)
SQC=$(pick SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE)
echo "lds/occ counters: $LDSOCC"; echo "sqc counters: $SQC"
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "STOP: $name exit $rc"; exit $rc; fi
}
CHILD="python3 bench.py --pmc-child --kernel dense --jit 1 --prep 0 --matrix"
for d in 020 050 090; do
  M=tests/fixtures/double__40_0.${d:1:2}_0
  step "pmc_lds_d$d" 120 rocprofv3 --pmc $LDSOCC --kernel-trace -d "$OUT/pmc_lds_d$d" -o run --output-format csv -- $CHILD $M
  # achieved occupancy: rocprofv3's derived MeanOccupancyPerCU / PerActiveCU (SQ_LEVEL_WAVES accumulated), one per pass
  have MeanOccupancyPerCU && step "pmc_occ_d$d" 120 rocprofv3 --pmc MeanOccupancyPerCU --kernel-trace -d "$OUT/pmc_occ_d$d" -o run --output-format csv -- $CHILD $M
  have MeanOccupancyPerActiveCU && step "pmc_occa_d$d" 120 rocprofv3 --pmc MeanOccupancyPerActiveCU --kernel-trace -d "$OUT/pmc_occa_d$d" -o run --output-format csv -- $CHILD $M
done
# HBM bytes of the final kernels (FETCH_SIZE and WRITE_SIZE cannot share a pass)
for d in 020 050 090; do
  M=tests/fixtures/double__40_0.${d:1:2}_0
  step "pmc_fetch_d$d" 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch_d$d" -o run --output-format csv -- $CHILD $M
  step "pmc_write_d$d" 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write_d$d" -o run --output-format csv -- $CHILD $M
  step "pmc_f64_d$d" 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/pmc_f64_d$d" -o run --output-format csv -- $CHILD $M
done
step pmc_sqc_d090 120 rocprofv3 --pmc $SQC --kernel-trace -d "$OUT/pmc_sqc_d090" -o run --output-format csv -- $CHILD tests/fixtures/double__40_0.90_0
step pmc_sqc_d050 120 rocprofv3 --pmc $SQC --kernel-trace -d "$OUT/pmc_sqc_d050" -o run --output-format csv -- $CHILD tests/fixtures/double__40_0.50_0
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py --steps 3 --warmup 1
step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0
echo "== done"
