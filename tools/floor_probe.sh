#!/bin/bash
# The multi-GPU chain floor (verdict r04 #4), run via gpurun from the repo root:
#  1. C3 on one GPU, giant chains on (giant_class=14), heavy keys of >= route_heavy_min occurrences
#     routed into a heavy-only pass 0 (route_first=1): when do the giant chains start / end
#     (C3_SETS: the option sets, tools/c3_opts.sh arguments);
#  2. the world-2 host-transport rehearsal (both ranks on this GPU, 4 M proteins, a memory budget
#     that makes each rank plan two passes -- the 8-GPU C3 shape), route_first default (on) vs 0
#     (W2_OPTS: extra bench options of both runs).
set -u
O=gpurun_out; mkdir -p $O
if [ -n "${C3_SETS:-}" ]; then
  eval "bash tools/c3_opts.sh $C3_SETS" || exit 1
fi
for RF in ${W2_RF:-1 0}; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2953$RF bench.py --gpus 2 --comm host --seqs-total 4000000 --steps 3 --warmup 1 --weak-seqs 0 \
    --annot-queries 0 --matrix-seqs 0 --cli-seqs 0 --finish 0 --option device_memory_budget_mb=80000 \
    --option route_first=$RF ${W2_OPTS:-} --json-out $O/r05_world2_rf$RF.json > $O/r05_world2_rf$RF.log 2>&1 \
    || { tail -20 $O/r05_world2_rf$RF.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/r05_world2_rf$RF.json'))
print('world2 route_first=$RF', round(d['ms_per_step'],1), 'passes', d['config'].get('key_range_passes'), 'tail', d.get('chain_tail_ms'), 'giant', d.get('giant_chains'))"
done
