#!/bin/bash
# HitSet diagnosis: the annotate leg with the default library and the diagnostic variants
# (libskm_seg1: no mean, seg2: no median / MAD, seg3: neither -- results wrong by design), then
# the legs' kernel trace on the default library
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
A="--seqs-total 1000000 --cache-dir /tmp/legs --no-cpu-baseline --matrix-seqs 0 --recall 0 --steps 3 --warmup 1"
timeout -k 10 400 python3 -u bench.py --seqs-total 1000000 --cache-dir /tmp/legs --cache-only > $O/r04_k_cache.log 2>&1 || exit $?
echo cached
for V in "" seg1 seg2 seg3; do
  L=signature_kmers_amd/libskm.so; [ -n "$V" ] && L=signature_kmers_amd/libskm_$V.so
  SKM_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py $A --json-out $O/r04_k_${V:-default}.json > $O/r04_k_${V:-default}.log 2>&1; rc=$?
  echo "${V:-default} rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/r04_k_prof -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py $A --json-out $GRAFT_REPO_ROOT/$O/r04_k_trace.json > $GRAFT_REPO_ROOT/$O/r04_k_trace.log 2>&1; rc=$?
echo "trace rc=$rc"; exit $rc
