#!/bin/bash
# round-5 final measurements on the final sources: the default bench line, kernel traces (C3, C2),
# FETCH/WRITE counter passes (C3, C2), SQ counters at C3, and the legs' trace + counters
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python3 -u bench.py --json-out $O/r05_bench_final.json > $O/r05_bench_final.log 2>&1 \
  || { tail -20 $O/r05_bench_final.log; exit 1; }
tail -1 $O/r05_bench_final.log | cut -c1-300
PHASE=trace bash tools/gpu_profile.sh || exit 1
PHASE=pmc bash tools/gpu_profile.sh || exit 1
PHASE=sq bash tools/gpu_profile.sh || exit 1
PHASE=legs bash tools/gpu_profile.sh
