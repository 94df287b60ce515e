#!/bin/bash
# C3 diagnostics A/B on one GPU (cached inputs): VARIANTS="'' 'heavy_min=512 split_min=2049'"
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/cache.log 2>&1 || { tail -5 $O/cache.log; exit 1; }
i=0
eval "set -- $VARIANTS"
for v in "$@"; do
  opts=""
  for kv in $v; do opts="$opts --option $kv"; done
  timeout -k 10 300 python3 -u tools/c3_diag.py --cache-dir /tmp/c3 --steps 2 ${DIAG_ARGS:-} $opts > $O/c3v$i.log 2>&1 || { tail -5 $O/c3v$i.log; exit 1; }
  python3 - "$O/c3v$i.log" "$v" "$i" <<'PY'
import json, re, sys
rows = [json.loads(l.split("wall; ", 1)[1]) for l in open(sys.argv[1]) if "] run " in l]
rows = rows[1:] if len(rows) > 2 else rows  # drop the first (cold) run
t = [r["total"] for r in rows]
keys = ("extract_count", "extract_scatter", "partition", "bucket_kernel", "big_groups", "overflow", "chains")
print(f"variant {sys.argv[3]} [{sys.argv[2]}]: total mean {sum(t)/len(t):.1f} ms (min {min(t):.1f}, n={len(t)}) " +
      " ".join(f"{k}={sum(r[k] for r in rows)/len(rows):.1f}" for k in keys))
PY
  i=$((i+1))
done
