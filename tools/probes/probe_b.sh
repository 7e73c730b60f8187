#!/bin/bash
# Specialised pair bits (SUP_JIT_B) and cached bits (SUP_JIT_CC) sweep of the
# segmented walk: one process per setting (plans are cached per process).
# usage: tools/probes/probe_b.sh "<fixture prep>"... ; env B_LIST / CC_LIST
set -u
for spec in "$@"; do
  set -- $spec
  for b in ${B_LIST:-5 6 7}; do
    for cc in ${CC_LIST:-auto}; do
      if [ "$cc" = auto ]; then unset SUP_JIT_CC; else export SUP_JIT_CC=$cc; fi
      echo -n "b=$b cc=$cc: "
      SUP_JIT_B=$b SUP_JIT_VERBOSE=1 timeout -k 10 120 python3 tools/probes/run_one.py "$1" "$2" seg 3 2>&1 | grep -v amdgpu.ids | tr '\n' ' '
      rc=${PIPESTATUS[0]}
      echo
      if [ "$rc" -ne 0 ]; then echo "STOP rc=$rc"; exit "$rc"; fi
    done
  done
done
