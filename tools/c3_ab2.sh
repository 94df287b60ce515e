#!/bin/bash
# C3 headline A/B over build options and environment (run via gpurun from the repo root):
#   bash tools/c3_ab2.sh "" "lane_long=131072" "GPU_MAX_HW_QUEUES=8 lane_long=131072" ...
# Each argument is one set: UPPERCASE=value words are environment variables of that run, the
# others build options (name=value).  The shard is generated once and cached under /tmp/c3.
# Results: gpurun_out/ab2_<i>.json, one summary line per set on stdout.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/ab2_cache.log 2>&1 || { tail -5 $O/ab2_cache.log; exit 1; }
i=0
for set in "$@"; do
  args=""; envs=""
  for kv in $set; do
    case "$kv" in
      [A-Z]*=*) envs="$envs $kv" ;;
      *) args="$args --option $kv" ;;
    esac
  done
  env $envs timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --steps 5 --warmup 1 --weak-seqs 0 --annot-queries 0 \
    --matrix-seqs 0 --no-cpu-baseline $args --json-out $O/ab2_$i.json > $O/ab2_$i.log 2>&1 \
    || { tail -5 $O/ab2_$i.log; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/ab2_$i.json')); r=d['roofline']; k=r.get('kernels_ms_per_step') or {}
print(sys.argv[1] or 'defaults', round(d['ms_per_step'],1), 'tail', round(d.get('chain_tail_ms') or 0,1), {n: round(v) for n, v in sorted(k.items(), key=lambda x: -x[1])[:9]})" "$set"
  i=$((i+1))
done
