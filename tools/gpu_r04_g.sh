#!/bin/bash
# full GPU suite, then the default bench (every leg, CPU baselines)
set -u
bash tools/gpu_r04_final.sh || exit $?
timeout -k 10 900 python3 -u bench.py --json-out gpurun_out/r04_g_bench.json > gpurun_out/r04_g_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/r04_g_bench.log | cut -c1-400
exit $rc
