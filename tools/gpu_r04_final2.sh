#!/bin/bash
# final evidence: the default bench, then the GPU suite without the C3 test (run with the parity set)
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python3 -u bench.py --json-out $O/r04_final_bench.json > $O/r04_final_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
SEL="tests --deselect tests/test_gpu_c3.py::test_c3_slice_bit_exact_and_whole_build_properties" bash tools/gpu_r04_final.sh
