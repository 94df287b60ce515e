#!/bin/bash
# Bench several libskm builds (ab/libskm_<name>.so), twice each, interleaved.
#   bash tools/ab_multi.sh name1 name2 ...
set -u
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    L=ab/libskm_$v.so
    SKM_LIB_PATH=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --annot-queries 0 \
       --matrix-seqs 0 --json-out $O/abm_$v.json > $O/abm_$v.log 2>&1 || { tail -20 $O/abm_$v.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/abm_$v.json'));p=d['pipeline']['phase_ms'];c=d['config'];print('$v',round(d['ms_per_step'],3),{k:round(x,3) for k,x in p.items() if k in ('bucket_kernel','overflow','partition','big_groups','total')})"
  done
done
