# A/B of two libskm builds on the C3 step (record of the k_pass_compact experiment):
# 'new' = signature_kmers_amd/libskm.so, 'old' = ab/libskm_oldcompact.so (build it from the variant
# source with the Makefile's hipcc flags first); plus a rocprof kernel-stats run of 'old'.
set -u
O=gpurun_out; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/abc_cache.log 2>&1 || { tail -5 $O/abc_cache.log; exit 1; }
for v in new old new old; do
  L=$R/signature_kmers_amd/libskm.so; [ $v = old ] && L=$R/ab/libskm_oldcompact.so
  SKM_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --steps 5 --warmup 1 --weak-seqs 0 --annot-queries 0 --matrix-seqs 0 --no-cpu-baseline --json-out $O/abc_$v.json > $O/abc_$v.log 2>&1 || { tail -5 $O/abc_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/abc_$v.json'));print('$v',round(d['ms_per_step'],1))"
done
cd /tmp
SKM_LIB_PATH=$R/ab/libskm_oldcompact.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/abc_prof_old -o run -- python3 $R/bench.py --cache-dir /tmp/c3 --steps 2 --warmup 1 --weak-seqs 0 --annot-queries 0 --matrix-seqs 0 --no-cpu-baseline > $R/$O/abc_prof_old.log 2>&1 || exit 1
grep -h "k_pass_compact\|k_bucket_process" $R/$O/abc_prof_old/run_kernel_stats.csv | cut -c1-160
