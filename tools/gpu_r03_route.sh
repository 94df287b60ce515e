#!/bin/bash
# Round 3: heavy-key routing parity (synthetic, C2, C3 at default settings), then the C3 headline
# bench (short) with the per-kernel table and the chain tail.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -v --durations=0 --timeout 400 --timeout-method thread \
  "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py \
  > $O/r03_route.log 2>&1; rc=$?
tail -30 $O/r03_route.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --annot-queries 0 --matrix-seqs 0 \
  --json-out $O/r03_bench_route.json > $O/r03_bench_route.log 2>&1; rc=$?
tail -5 $O/r03_bench_route.log; exit $rc
