#!/bin/bash
# A/B/A/B of environment variants on bench.py (every run checks its tree). Usage:
#   ab_env.sh OUT ROUNDS "VAR=a VAR=b,VAR2=c ..." [bench.py args...]   (comma: several variables)
set -e
OUT=$1; ROUNDS=$2; VARS=$3; shift 3
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARS; do
    echo "== round $r $v" >> "$OUT"
    env PKD_AB=1 $(echo "$v" | tr , " ") PKD_SKIP_BUILD=1 timeout -k 10 150 python bench.py "$@" 2>&1 | grep -v amdgpu.ids >> "$OUT"
  done
done
