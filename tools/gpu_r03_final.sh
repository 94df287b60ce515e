#!/bin/bash
# Round 3 final evidence: the full GPU suite, then the default bench (every leg, CPU baselines).
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=16
start=$(date +%s)
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --durations=15 --timeout 400 --timeout-method thread \
  > $O/r03_gputests.log 2>&1; rc=$?
echo "suite $(( $(date +%s) - start )) s rc=$rc"; tail -22 $O/r03_gputests.log
exit $rc
