#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   1. bench line with cpu_baseline            -> gpurun_out/bench.json
#   2. rocprofv3 kernel trace + stats          -> gpurun_out/prof_trace/
#   3. rocprofv3 PMC FETCH_SIZE (own pass)     -> gpurun_out/prof_fetch/
#   4. rocprofv3 PMC WRITE_SIZE (own pass)     -> gpurun_out/prof_write/
# Every GPU step has its own time limit; the script stops at the first failure.
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
PHASE=${PHASE:-all}   # all | trace (bench + kernel trace) | pmc (FETCH_SIZE, WRITE_SIZE passes)
cd "$R"
export TMPDIR=/tmp
if [ "$PHASE" != pmc ]; then
  step bench 500 python3 bench.py --steps "$STEPS" --warmup 2 --json-out "$O/bench.json"
  cd /tmp
  step prof_trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_trace" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --json-out "$O/bench_trace.json"
fi
if [ "$PHASE" != trace ]; then
  cd /tmp
  step prof_fetch 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/prof_fetch" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline
  step prof_write 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/prof_write" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline
fi
echo done
