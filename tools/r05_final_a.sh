#!/bin/bash
# round-5 final measurements, part a: the default bench line, then the C3/C2 kernel traces
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python3 -u bench.py --json-out $O/r05_bench_final.json > $O/r05_bench_final.log 2>&1 \
  || { tail -20 $O/r05_bench_final.log; exit 1; }
tail -1 $O/r05_bench_final.log | cut -c1-400
PHASE=trace bash tools/gpu_profile.sh
