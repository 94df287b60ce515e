#!/bin/bash
# r03 session 2: routing default 16384 -- the build parity tests (C3 slice included), then the
# default bench (every leg, CPU baselines).
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=16
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_scale.py::test_c2_build_bit_exact \
  tests/test_gpu_c3.py -x -v --timeout 400 --timeout-method thread > $O/t_route.log 2>&1; rc=$?
tail -3 $O/t_route.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1; rc=$?
tail -2 $O/bench_default.log | cut -c1-300; exit $rc
