#!/bin/bash
# C3 headline A/B over build options (run via gpurun from the repo root):
#   bash tools/c3_opts.sh "" "giant_class=14 giant_passes=1" ...
# Each argument is one option set (space-separated name=value, "" = defaults); the shard is
# generated once and cached under /tmp/c3.  Results: gpurun_out/c3_opts_<i>.json.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/c3_opts_cache.log 2>&1 || { tail -5 $O/c3_opts_cache.log; exit 1; }
i=0
for set in "$@"; do
  args=""
  for kv in $set; do args="$args --option $kv"; done
  timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --steps 5 --warmup 1 --weak-seqs 0 --annot-queries 0 \
    --matrix-seqs 0 --cli-seqs 0 --finish 0 --no-cpu-baseline $args --json-out $O/c3_opts_$i.json > $O/c3_opts_$i.log 2>&1 \
    || { tail -5 $O/c3_opts_$i.log; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/c3_opts_$i.json')); r=d['roofline']; k=r.get('kernels_ms_per_step') or {}
print(sys.argv[1] or 'defaults', round(d['ms_per_step'],1), 'tail', round(d.get('chain_tail_ms') or 0,1), 'giant', d.get('giant_chains'), {n: round(v) for n, v in sorted(k.items(), key=lambda x: -x[1])[:10]})" "$set"
  i=$((i+1))
done
