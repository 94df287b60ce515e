#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   1. bench line with cpu_baseline                          -> gpurun_out/bench.json
#   2. rocprofv3 kernel trace + stats, build leg alone       -> gpurun_out/prof_trace/
#      (the headline kernels: averages over the C2 launches only)
#   3. rocprofv3 kernel trace + stats, annotate + matrix legs -> gpurun_out/prof_trace_legs/
#      (their kernels; the build kernels in this trace also include the matrix leg's small
#      training build and are not cited)
#   4. rocprofv3 PMC FETCH_SIZE / WRITE_SIZE, one pass each, build leg alone and legs
#                                                            -> gpurun_out/prof_{fetch,write}[_legs]/
# Every GPU step has its own time limit; the script stops at the first failure.
# PHASE=trace runs 1-3, PHASE=pmc runs 4, PHASE=all (default) everything.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
STEPS=${STEPS:-5}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$O/$name.log"; exit $rc; fi
}
PHASE=${PHASE:-all}
cd "$R"
export TMPDIR=/tmp
if [ "$PHASE" != pmc ]; then
  step bench 500 python3 bench.py --steps "$STEPS" --warmup 2 --json-out "$O/bench.json"
  cd /tmp
  step prof_trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_trace" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --annot-queries 0 --matrix-seqs 0 \
    --json-out "$O/bench_trace.json"
  step prof_trace_legs 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_trace_legs" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --json-out "$O/bench_trace_legs.json"
fi
if [ "$PHASE" != trace ]; then
  cd /tmp
  for leg in build legs; do
    if [ $leg = build ]; then X="--annot-queries 0 --matrix-seqs 0"; S=""; else X=""; S="_legs"; fi
    step prof_fetch$S 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/prof_fetch$S" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline $X
    step prof_write$S 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/prof_write$S" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline $X
  done
fi
echo done
