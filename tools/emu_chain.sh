#!/bin/bash
# Distributed-path checks + the emulated P = 8 rank's chain (phase JSON and per-kernel timeline of
# the last replay) on one GPU box; each step under its own time limit, chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread ${DIST_TESTS:-tests/test_gpu_dist_ops.py tests/test_gpu_multirank.py} > $O/dist_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/emulate_rank.py --reps 5 > $O/emu.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/prof_emu -o emu --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/emulate_rank.py --reps 3 > $GRAFT_REPO_ROOT/$O/prof_emu.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/chain_timeline.py $O/prof_emu/emu_kernel_trace.csv > $O/emu_timeline.txt
