#!/bin/bash
# HIP runtime API call counts of one build step: the C2 probe (tools/pmc_probe.py) with 1 and 3
# runs under rocprofv3 --hip-runtime-trace --stats; (calls(3) - calls(1)) / 2 = calls per step.
# Summarised by tools/sync_summary.py into profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/syncs
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for n in 1 3; do
  SKM_PROBE_RUNS=$n timeout -k 10 300 rocprofv3 --hip-runtime-trace --stats --output-format csv -d "$O/r$n" -o run -- python3 "$R/tools/pmc_probe.py" > "$O/r$n.log" 2>&1 || { tail -5 "$O/r$n.log"; exit 1; }
done
echo syncs done
