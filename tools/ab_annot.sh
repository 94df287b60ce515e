#!/bin/bash
# A/B of two libskm builds on the annotate + matrix legs (build leg at 200K sequences to save time).
#   A = signature_kmers_amd/libskm.so, B = $1 (default ab/libskm_base.so)
set -u
O=gpurun_out; mkdir -p $O
B=${1:-ab/libskm_base.so}
for v in A B A B; do
  if [ $v = A ]; then L=signature_kmers_amd/libskm.so; else L=$B; fi
  SKM_LIB_PATH=$L timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --seqs 1000000 \
     --json-out $O/aba_$v.json > $O/aba_$v.log 2>&1 || { tail -20 $O/aba_$v.log; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/aba_$v.json'))
a=d['annotate'];m=d['matrix']
print('$v','annot',round(a['ms_per_step'],2),{k:round(x,2) for k,x in a['phase_ms'].items()},'matrix',round(m['ms_per_step'],2),{k:round(x,2) for k,x in m['phase_ms'].items()})"
done
