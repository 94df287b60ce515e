#!/bin/bash
# Round 4 GPU session script: tools/gpu_r04.sh TAG "pytest selection" [bench args...]
#   1. the named GPU tests (skipped when the selection is "-")
#   2. bench.py with the given arguments (skipped when none), JSON line to gpurun_out/r04_TAG_bench.json
# Every GPU step under its own time limit; the script stops at the first failure.
set -u
O=gpurun_out; mkdir -p $O
TAG=$1; SEL=$2; shift 2
start=$(date +%s)
if [ "$SEL" != "-" ]; then
  timeout -k 10 900 python3 -u -m pytest $SEL -m gpu -x -v --timeout 400 --timeout-method thread \
    > $O/r04_${TAG}_tests.log 2>&1; rc=$?
  echo "tests $(( $(date +%s) - start )) s rc=$rc"; tail -15 $O/r04_${TAG}_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 python3 -u bench.py --json-out $O/r04_${TAG}_bench.json "$@" > $O/r04_${TAG}_bench.log 2>&1; rc=$?
  echo "bench $(( $(date +%s) - start )) s rc=$rc"; tail -4 $O/r04_${TAG}_bench.log
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
