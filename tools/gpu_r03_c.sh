#!/bin/bash
# Round 3 (c): device-planned multi-rank exchange (in-process groups, gloo processes), heavy-key
# routing at C2/C3, a short C3 bench (kernel table, chain tail), the bucket-kernel phase stamps.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 1000 python3 -u -m pytest -x -v --durations=0 --timeout 400 --timeout-method thread \
  tests/test_gpu_multirank.py tests/test_transport_gloo.py \
  "tests/test_gpu_cli.py::test_build_signatures_multi_rank_host_comm" \
  "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py \
  > $O/r03_c.log 2>&1; rc=$?
tail -40 $O/r03_c.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --annot-queries 0 --matrix-seqs 0 \
  --json-out $O/r03_bench_c.json > $O/r03_bench_c.log 2>&1; rc=$?
tail -5 $O/r03_bench_c.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/diag_build.py --steps 1 > $O/r03_diag_c2.log 2>&1; rc=$?
tail -30 $O/r03_diag_c2.log; exit $rc
