#!/bin/bash
# Annotate-leg timings of several libskm builds (ab/libskm_<name>.so), twice each, interleaved.
#   bash tools/ab_annot_multi.sh name1 name2 ...
set -u
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    SKM_LIB_PATH=ab/libskm_$v.so timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
       --matrix-seqs 0 --json-out $O/abx_$v.json > $O/abx_$v.log 2>&1 || { tail -20 $O/abx_$v.log; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/abx_$v.json'));a=d['annotate']
print('$v',round(a['ms_per_step'],2),{k:round(x,2) for k,x in a['phase_ms'].items()})"
  done
done
