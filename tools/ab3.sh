#!/bin/bash
# C3: saved variant libraries (LIBS="base nostride ...": signature_kmers_amd/libskm_<name>.so) once
# each with the defaults, then the current library over option sets (tools/c3_opts.sh arguments).
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/ab_cache.log 2>&1 || exit 1
for V in ${LIBS:-base}; do
  SKM_LIB_PATH=signature_kmers_amd/libskm_$V.so timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --steps 5 --warmup 1 \
    --weak-seqs 0 --annot-queries 0 --matrix-seqs 0 --cli-seqs 0 --finish 0 --no-cpu-baseline --recall 0 \
    --json-out $O/ab_$V.json > $O/ab_$V.log 2>&1 || exit 1
  python3 -c "
import json; d=json.load(open('$O/ab_$V.json')); k=d['roofline']['kernels_ms_per_step']
print('$V', round(d['ms_per_step'],1), 'tail', round(d['chain_tail_ms'],1), {n: round(v) for n, v in sorted(k.items(), key=lambda x: -x[1])[:10]})"
done
bash tools/c3_opts.sh "$@"
