#!/bin/bash
# Round 3 (h): partition round variants (parity + C3 A/B) and C3 option A/B -- heavy-routing
# threshold, long-chain batches.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_build.py::test_key_range_passes" > $O/r03_h.log 2>&1; rc=$?
tail -3 $O/r03_h.log
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "partition_round=1" "partition_round=2" "route_heavy_min=16384" "route_heavy_min=262144" "chain_batches=8"
