set -u
O=gpurun_out
for v in 0 1 0 1; do
  SKM_DBG_SKIP_OVERFLOW=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --annot-queries 0 --matrix-seqs 0 --json-out $O/exp_$v.json > $O/exp_$v.log 2>&1 || { tail -5 $O/exp_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp_$v.json'));p=d['pipeline']['phase_ms'];print('skip=$v',round(d['ms_per_step'],3),{k:round(x,3) for k,x in p.items()})"
done
