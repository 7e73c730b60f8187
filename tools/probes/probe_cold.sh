#!/bin/bash
# Cold segmented-plan cost on this host: every matrix in a fresh process with
# an empty plan cache AND an empty comgr cache (hiprtc's compiles are cached by
# comgr under ~/.cache/comgr: a "cold" plan after another process compiled the
# same kernel is not cold).  usage: tools/probes/probe_cold.sh <out.log> <threads...> -- <matrices...>
set -u
OUT=$1; shift
TS=()
while [ "$1" != "--" ]; do TS+=("$1"); shift; done; shift
for T in "${TS[@]}"; do
  for M in "$@"; do
    D=$(mktemp -d)
    OMP_NUM_THREADS=$T AMD_COMGR_CACHE_DIR=$D/comgr SUP_JIT_CACHE_DIR=$D/plans SUP_JIT_VERBOSE=1 \
      timeout -k 10 120 python3 -u tools/probes/probe_cold.py "$M" > $D/log 2>&1 || { echo "FAIL $M"; cat $D/log; exit 1; }
    grep -E "^cold segmented|threads=" $D/log | tr '\n' ' ' >> "$OUT"; echo >> "$OUT"
    rm -rf "$D"
  done
done
