#!/bin/bash
# Profile set (run via gpurun from the repo root; inputs cached under /tmp/c3; tools/pmc_summary.py folds it):
#   c3_stamps.log  k_bucket_process phase stamps of one C3 build (tools/c3_diag.py --stamps)
#   prof_c3/  rocprofv3 kernel trace + stats, C3 headline build (bench.py, 1 warmup + 2 steps)
#   prof_c2/  the same for the C2 workload (first 250 files; tools/c3_diag.py, 3 runs)
#   prof_legs/  annotate (10M queries) + matrix (100K) legs (bench.py on the C2 proteome)
#   pmc_{c3,c2,legs}_{fetch,write}/   FETCH_SIZE / WRITE_SIZE, one counter per pass
# FETCH_SIZE calibration: profiles/r02_fetch_calib.json (streaming x2, gathers x1).
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$O/$name.log"; exit $rc; fi
}
cd "$R"
python3 -c "import bench; print(bench.src_sha16())" > "$O/src_sha16.txt"
P=${PHASE:-all}
case "$P" in legs*) ;; *) step cache 300 python3 bench.py --cache-dir /tmp/c3 --cache-only ;; esac
cd /tmp
C3="python3 -u $R/bench.py --cache-dir /tmp/c3 --weak-seqs 0 --annot-queries 0 --matrix-seqs 0 --cli-seqs 0 --finish 0 --no-cpu-baseline"
C2="python3 -u $R/tools/c3_diag.py --cache-dir /tmp/c3 --files 250"
LEGS="python3 -u $R/bench.py --seqs-total 1000000 --cache-dir /tmp/legs --cli-seqs 0 --finish 0 --no-cpu-baseline"
# PHASE: all | trace (stamps + C3/C2 traces) | pmc (C3/C2 counters) | legs (legs trace + counters)
#        | legs_trace (the legs' kernel trace only) | sq (SQ counters of a C3 build)
if [ "$P" = all ] || [ "$P" = trace ]; then
  step c3_stamps 300 python3 -u $R/tools/c3_diag.py --cache-dir /tmp/c3 --runs 1 --stamps
  step prof_c3 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c3" -o run -- $C3 --steps 2 --warmup 1 --json-out "$O/bench_c3_trace.json"
  step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c2" -o run -- $C2 --runs 3
fi
if [ "$P" = all ] || [ "$P" = pmc ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    step pmc_c3_$lc 500 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_c3_$lc" -o run -- python3 -u $R/tools/c3_diag.py --cache-dir /tmp/c3 --runs 1
    step pmc_c2_$lc 300 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_c2_$lc" -o run -- $C2 --runs 1
  done
fi
if [ "$P" = sq ]; then  # SQ counters of one C3 build (k_bucket_process at C3 size; dispatches serialised)
  cd "$R"
  SQ_CMD="python3 -u $R/tools/c3_diag.py --cache-dir /tmp/c3 --runs 1" SQ_OUT=pmc_sq_c3 SKM_PROBE_ANNOT=0 \
    bash tools/pmc_sq.sh || exit 1
  echo done; exit 0
fi
if [ "$P" = all ] || [ "$P" = legs ] || [ "$P" = legs_trace ]; then
  cd "$R"
  step legs_cache 400 python3 -u $R/bench.py --seqs-total 1000000 --cache-dir /tmp/legs --cache-only
  cd /tmp
  step prof_legs 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_legs" -o run -- $LEGS --steps 3 --warmup 1 --json-out "$O/bench_legs_trace.json"
  [ "$P" = legs_trace ] && { echo done; exit 0; }
  for c in FETCH_SIZE WRITE_SIZE; do
    lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    step pmc_legs_$lc 500 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_legs_$lc" -o run -- $LEGS --steps 1 --warmup 1
  done
fi
echo done
