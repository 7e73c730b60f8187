#!/bin/bash
# The fused fold against the reduction launches (SUP_FOLD=0) on one box, alternately, same build:
# config 2 and config 3's bench steps (tools/probes/probe_defer.py's eager leg).
set -e
for i in 1 2; do
  for f in 1 0; do
    echo "SUP_FOLD=$f"
    SUP_FOLD=$f timeout -k 10 120 python3 tools/probes/probe_defer.py | grep eager
  done
done
