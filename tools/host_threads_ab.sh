#!/bin/bash
# one-shot (PCIe-inclusive) host phases of the C3 build over host-pool sizes (SKM_HOST_THREADS);
# the inputs generated in memory as in the default bench (a memory-mapped cache would add page
# faults to the packing)
set -u
O=gpurun_out; mkdir -p $O
for T in ${THREADS:-16 8 4}; do
  SKM_HOST_THREADS=$T timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --weak-seqs 0 \
    --annot-queries 0 --matrix-seqs 0 --cli-seqs 0 --finish 0 --no-cpu-baseline --json-out $O/ht_$T.json > $O/ht_$T.log 2>&1 || exit 1
  python3 -c "
import json; d=json.load(open('$O/ht_$T.json')); p=d['pcie_inclusive']; print('threads $T', round(p['value']/1e9,3), p['phases'])"
done
