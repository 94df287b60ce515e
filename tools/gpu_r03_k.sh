#!/bin/bash
# Round 3 (k): CU-masked side streams -- parity of chain_cus / side_cus, then C3 A/B.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_build.py::test_key_range_passes" > $O/r03_k.log 2>&1; rc=$?
tail -3 $O/r03_k.log
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "chain_cus=32" "chain_cus=64" "side_cus=128" "side_cus=64" "side_cus=128 chain_cus=32" "side_cus=192" "prefetch=0"
