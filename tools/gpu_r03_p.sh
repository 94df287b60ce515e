#!/bin/bash
# r03 session 2: C3 A/B of flag_bits, then the build parity tests (per-lane long chains default).
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=16
bash tools/c3_ab2.sh "" "flag_bits=1" || exit 1
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_scale.py::test_c2_build_bit_exact \
  tests/test_gpu_c3.py -x -v --timeout 600 --timeout-method thread > $O/t_lane.log 2>&1; rc=$?
tail -4 $O/t_lane.log; exit $rc
