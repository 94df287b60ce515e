#!/bin/bash
# C3 A/B of two libraries on one box: signature_kmers_amd/libskm_base.so (a saved build of the
# previous sources) against the current libskm.so, three alternating pairs, C3 cached under /tmp/c3.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/ab_cache.log 2>&1 || exit 1
i=0
for V in base new base new base new; do i=$((i+1))
  L=signature_kmers_amd/libskm.so; [ $V = base ] && L=signature_kmers_amd/libskm_base.so
  SKM_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --steps 5 --warmup 1 --weak-seqs 0 --annot-queries 0 \
    --matrix-seqs 0 --cli-seqs 0 --finish 0 --no-cpu-baseline --recall 0 --json-out $O/ab_$i.json > $O/ab_$i.log 2>&1 || exit 1
  python3 -c "
import json; d=json.load(open('$O/ab_$i.json')); k=d['roofline']['kernels_ms_per_step']
print('$V', round(d['ms_per_step'],1), 'bucket', k.get('k_bucket_process'), 'avg', round(d['roofline']['avg_launch_ms'],2))"
done
