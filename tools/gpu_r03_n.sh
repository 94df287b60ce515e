#!/bin/bash
# Round 3 (n): routing spread (route_vacate) parity + C3 A/B; wave priorities.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_build.py::test_heavy_key_routing" > $O/r03_n.log 2>&1; rc=$?
tail -3 $O/r03_n.log
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "route_vacate=4" "route_vacate=2" "route_vacate=6" "bucket_prio=3" "overflow_inline_prio=0"
