#!/bin/bash
# HitSet: parity (unit + C4), then the annotate leg with the default library and without the
# selects (libskm_seg2, diagnostics only)
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_annotate.py tests/test_gpu_scale.py::test_c4_db_calls_bit_exact \
  -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/r04_l_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 $O/r04_l_tests.log
[ $rc -ne 0 ] && exit $rc
A="--seqs-total 1000000 --cache-dir /tmp/legs --no-cpu-baseline --matrix-seqs 0 --recall 0 --steps 3 --warmup 1"
timeout -k 10 400 python3 -u bench.py --seqs-total 1000000 --cache-dir /tmp/legs --cache-only > $O/r04_l_cache.log 2>&1 || exit $?
for V in "" seg2; do
  L=signature_kmers_amd/libskm.so; [ -n "$V" ] && L=signature_kmers_amd/libskm_$V.so
  SKM_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py $A --json-out $O/r04_l_${V:-default}.json > $O/r04_l_${V:-default}.log 2>&1; rc=$?
  echo "${V:-default} rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
