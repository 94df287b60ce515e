#!/bin/bash
# Round 3 (d): bucket-kernel changes -- parity (build suite subset + C2), stamps, short C3 bench.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -q --durations=5 --timeout 400 --timeout-method thread \
  tests/test_gpu_build.py "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_multirank.py \
  > $O/r03_d.log 2>&1; rc=$?
tail -12 $O/r03_d.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/diag_build.py --steps 1 > $O/r03_diag_d.log 2>&1; rc=$?
grep -A 14 "^stamps" $O/r03_diag_d.log; grep "^timings" $O/r03_diag_d.log | tail -1
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --annot-queries 0 --matrix-seqs 0 --no-cpu-baseline \
  --json-out $O/r03_bench_d.json > $O/r03_bench_d.log 2>&1; rc=$?
python3 -c "
import json; d=json.load(open('$O/r03_bench_d.json')); print('C3', round(d['ms_per_step'],1), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_launch_ms'],2), d['roofline']['kernels_ms_per_step']); w=d['weak']; print('C2', round(w['ms_per_step'],2), w['roofline']['kernels_ms_per_step'])"
exit $rc
