#!/bin/bash
# HitSet rework: annotate parity (unit + C4), the annotate / recall legs, then a C3 A/B of k_bucket_process
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = 0 ]; then
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_annotate.py tests/test_gpu_scale.py::test_c4_db_calls_bit_exact \
  -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/r04_i_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -6 $O/r04_i_tests.log
[ $rc -ne 0 ] && exit $rc
fi
# the annotate / recall legs (the headline at 1 M proteins: the legs' inputs do not depend on it)
timeout -k 10 600 python3 -u bench.py --json-out $O/r04_i_legs.json --seqs-total 1000000 --steps 3 --warmup 1 \
  --no-cpu-baseline --matrix-seqs 0 > $O/r04_i_legs.log 2>&1; rc=$?
echo "legs rc=$rc"; tail -2 $O/r04_i_legs.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
# C3 A/B: k_bucket_process as 256-thread workgroups (libskm_bp256.so) vs the default 512
A="--steps 3 --warmup 1 --no-cpu-baseline --annot-queries 0 --matrix-seqs 0 --weak-seqs 0 --recall 0 --cache-dir /tmp/c3cache"
i=0; for V in 512 256 512; do i=$((i+1))
  L=signature_kmers_amd/libskm.so; [ $V = 256 ] && L=signature_kmers_amd/libskm_bp256.so
  SKM_LIB_PATH=$L timeout -k 10 600 python3 -u bench.py $A --json-out $O/r04_i_bp${V}_$i.json > $O/r04_i_bp${V}_$i.log 2>&1; rc=$?
  echo "bp$V rc=$rc"; tail -1 $O/r04_i_bp${V}_$i.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
exit 0
