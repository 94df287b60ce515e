#!/bin/bash
# r03 session 2 evidence: the full GPU suite, then the default bench (every leg, CPU baselines).
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=16
start=$(date +%s)
timeout -k 10 950 python3 -u -m pytest tests -m gpu -x -q --durations=15 --timeout 400 --timeout-method thread \
  > $O/r03_gputests.log 2>&1; rc=$?
echo "suite $(( $(date +%s) - start )) s rc=$rc"; tail -4 $O/r03_gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1; rc=$?
tail -1 $O/bench_default.log | cut -c1-250; exit $rc
