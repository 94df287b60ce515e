#!/bin/bash
# A/B of two libskm builds on the build bench (no cpu baseline, no annotate leg).
#   A = signature_kmers_amd/libskm.so, B = $1 (default ab/libskm_base.so)
set -u
O=gpurun_out; mkdir -p $O
B=${1:-ab/libskm_base.so}
for v in A B A B; do
  if [ $v = A ]; then L=signature_kmers_amd/libskm.so; else L=$B; fi
  SKM_LIB_PATH=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --annot-queries 0 \
     --json-out $O/ab_$v.json > $O/ab_$v.log 2>&1 || { tail -20 $O/ab_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));p=d['pipeline']['phase_ms'];print('$v',round(d['ms_per_step'],3),{k:round(x,3) for k,x in p.items()})"
done
