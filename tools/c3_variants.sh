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
  echo "variant $i [$v]: $(grep 'run ' $O/c3v$i.log | tail -1)"
  i=$((i+1))
done
