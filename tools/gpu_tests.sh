#!/bin/bash
# GPU test suite on the box (stops at the first failure).
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
tail -5 $O/gputests.log; exit $rc
