#!/bin/bash
# (1) world-2 rehearsal on the one GPU over the gloo host transport, 2 key-range passes per rank with
#     heavy-key routing at world > 1; (2) C3 A/B: heavy_min 512 (the heavy path's new cost)
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 2 --comm host --seqs-total 4000000 --steps 3 --warmup 1 --annot-queries 0 \
  --matrix-seqs 0 --weak-seqs 0 --recall 0 --no-cpu-baseline --option key_range_passes=2 --option route_heavy_min=4096 \
  --json-out $O/r04_h_world2.json > $O/r04_h_world2.log 2>&1; rc=$?
echo "world2 rc=$rc"; tail -2 $O/r04_h_world2.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --json-out $O/r04_h_hm512.json --steps 4 --warmup 2 --no-cpu-baseline \
  --annot-queries 0 --matrix-seqs 0 --weak-seqs 0 --recall 0 --option heavy_min=512 > $O/r04_h_hm512.log 2>&1; rc=$?
echo "hm512 rc=$rc"; exit $rc
