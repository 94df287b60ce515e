#!/bin/bash
# Bench the build under several env settings, twice each: bash tools/exp_env.sh "A=1" "A=0 B=2" ...
set -u
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --annot-queries 0 \
       --matrix-seqs 0 --json-out $O/exe_$i.json > $O/exe_$i.log 2>&1 || { tail -20 $O/exe_$i.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/exe_$i.json'));p=d['pipeline']['phase_ms'];print('$cfg',round(d['ms_per_step'],3),{k:round(x,3) for k,x in p.items() if k in ('bucket_kernel','overflow','partition','big_groups','chains','total')})"
  done
done
