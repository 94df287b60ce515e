#!/bin/bash
# k_calls_scan in length order: annotate parity (unit + C4 + recall) and the legs bench
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_annotate.py tests/test_gpu_scale.py::test_c4_db_calls_bit_exact \
  tests/test_gpu_scale.py::test_c2_recall_bit_exact tests/test_gpu_cli.py -m gpu -x -v -s --timeout 400 \
  --timeout-method thread > $O/r04_n_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r04_n_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u bench.py --json-out $O/r04_n_legs.json --seqs-total 1000000 --steps 3 --warmup 1 \
  --no-cpu-baseline --matrix-seqs 0 > $O/r04_n_legs.log 2>&1; rc=$?
echo "legs rc=$rc"; exit $rc
