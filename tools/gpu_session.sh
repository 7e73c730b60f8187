#!/bin/bash
# One GPU session on the MI355X box: each step under its own time limit; stop
# at the first crash/timeout (exit codes 124/134/137/139 or signals), keep
# going after plain test failures (exit 1) so the bench still runs.
# usage: tools/gpu_session.sh <tag> [steps...]   steps: test bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 "$OUT/$name.log"
  case $rc in 0|1|5) return 0;; *) echo "STOP: $name exit $rc"; exit $rc;; esac
}
rocm-smi --showproductname --showclocks > "$OUT/rocm_smi.log" 2>&1 || true
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()";;
    test)  run pytest_gpu 1200 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider;;
    testall) run pytest_gpu 1200 python3 -m pytest tests -m gpu -q -p no:cacheprovider;;
    bench) run bench 600 python3 bench.py --steps 3 --warmup 1;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0;;
    pmc)   run pmc 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0
           run pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0;;
    probe) run probe 300 python3 tools/probe.py;;
  esac
done
echo "== done"
