#!/bin/bash
# Round-4 evidence: the full GPU suite, then the default bench (every leg, CPU baselines).
set -u
O=gpurun_out; mkdir -p $O
start=$(date +%s)
SEL=${SEL:-tests}
timeout -k 10 1050 python3 -u -m pytest $SEL -m gpu -x -v -s --durations=20 --timeout 420 --timeout-method thread \
  > $O/r04_gputests.log 2>&1; rc=$?
echo "suite $(( $(date +%s) - start )) s rc=$rc"; tail -28 $O/r04_gputests.log
exit $rc
