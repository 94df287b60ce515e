#!/bin/bash
# Round 3 (b): multi-rank matrix distance (gloo 2/4 processes, CLI --comm host), matrix parity,
# heavy-key routing at C2/C3, then a short C3 bench with the per-kernel table and the chain tail.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 1000 python3 -u -m pytest -x -v --durations=0 --timeout 400 --timeout-method thread \
  tests/test_transport_gloo.py tests/test_gpu_matrix.py \
  "tests/test_gpu_cli.py::test_matrix_distance_row_bands_multi_rank" \
  "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py \
  > $O/r03_b.log 2>&1; rc=$?
tail -40 $O/r03_b.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --annot-queries 0 --matrix-seqs 0 \
  --json-out $O/r03_bench_b.json > $O/r03_bench_b.log 2>&1; rc=$?
tail -5 $O/r03_bench_b.log; exit $rc
