#!/bin/bash
# add_batch rework: build parity (unit, key-range passes, colliding ids, rank groups), then the default bench
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_multirank.py -m gpu -x -v -s --timeout 400 \
  --timeout-method thread > $O/r04_m_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r04_m_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 800 python3 -u bench.py --json-out $O/r04_m_default.json > $O/r04_m_default.log 2>&1; rc=$?
echo "bench rc=$rc"; exit $rc
