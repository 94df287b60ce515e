#!/bin/bash
# C4 annotate A/B over variant libraries (LIBS="libskm libskm_wave": signature_kmers_amd/<name>.so),
# each under a rocprofv3 kernel trace (run via gpurun from the repo root).  Results:
# gpurun_out/hs_<name>.json and gpurun_out/prof_hs_<name>/ (kernel stats).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python3 -u bench.py --seqs-total 1000000 --cache-dir /tmp/legs --cache-only > $O/hs_cache.log 2>&1 || { tail -5 $O/hs_cache.log; exit 1; }
cd /tmp
for V in ${LIBS:-libskm}; do
  SKM_LIB_PATH=$R/signature_kmers_amd/$V.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/prof_hs_$V -o run -- python3 -u $R/bench.py --seqs-total 1000000 --cache-dir /tmp/legs --cli-seqs 0 --finish 0 \
    --no-cpu-baseline --matrix-seqs 0 --recall 0 --steps 3 --warmup 1 --json-out $O/hs_$V.json > $O/hs_$V.log 2>&1 \
    || { tail -5 $O/hs_$V.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/hs_$V.json')); print('$V', d['annotate']['phase_ms'])"
done
