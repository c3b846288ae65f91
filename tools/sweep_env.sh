#!/bin/bash
# Sweep one environment knob over values for tools/bench_build.py (single GPU).
# Usage: tools/sweep_env.sh VAR "v1 v2 ..." [bench_build.py args...]
var=$1; vals=$2; shift 2
for v in $vals; do
  echo "$var=$v"
  env "$var=$v" python tools/bench_build.py "$@" 2>&1 | grep '"n"' || exit 1
done
