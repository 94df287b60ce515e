#!/bin/bash
# Round-5 GPU session steps: a selection of the GPU tests (SEL, pytest -k KEXPR), then optional
# commands (PROBE).  Every GPU step runs under its own time limit; the script stops at the first
# failing step.
set -u
O=gpurun_out; mkdir -p $O
TAG=${TAG:-r05}
if [ -n "${SEL:-}" ]; then
  start=$(date +%s)
  timeout -k 10 ${TEST_LIMIT:-900} python3 -u -m pytest $SEL -m gpu -x -v --durations=15 --timeout 420 \
    --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $O/${TAG}_tests.log 2>&1; rc=$?
  echo "tests $(( $(date +%s) - start )) s rc=$rc"; tail -22 $O/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROBE:-}" ]; then
  timeout -k 10 ${PROBE_LIMIT:-600} bash -c "$PROBE" > $O/${TAG}_probe.log 2>&1; rc=$?
  echo "probe rc=$rc"; tail -25 $O/${TAG}_probe.log
  exit $rc
fi
