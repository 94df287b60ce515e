#!/bin/bash
# C3 headline A/B on one GPU: cache the 50M-protein inputs once, then one bench run per variant.
#   VARIANTS="'' 'main_long_class=12'"  (each a space-separated list of name=value options)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
STEPS=${STEPS:-2}
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > "$O/c3_cache.log" 2>&1 || { tail -5 "$O/c3_cache.log"; exit 1; }
i=0
eval "set -- $VARIANTS"
for v in "$@"; do
  opts=""
  for kv in $v; do opts="$opts --option $kv"; done
  echo "[$(date +%T)] variant $i: $v"
  timeout -k 10 400 python3 bench.py --cache-dir /tmp/c3 --steps "$STEPS" --warmup 1 --weak-seqs 0 --annot-queries 0 \
    --matrix-seqs 0 --no-cpu-baseline $opts --json-out "$O/c3_v$i.json" > "$O/c3_v$i.log" 2>&1
  rc=$?
  echo "[$(date +%T)] variant $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/c3_v$i.log"; exit $rc; fi
  python3 -c "import json; d=json.load(open('$O/c3_v$i.json')); p=d['pipeline']['phase_ms_rank0']; print('  %.1f ms/step  %.2f G/s' % (d['ms_per_step'], d['value']/1e9), {k: round(v,1) for k,v in p.items()})"
  i=$((i+1))
done
