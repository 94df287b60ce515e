#!/bin/bash
# kernel trace of the probe workload (one build, two runs)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace_probe
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- python3 "$R/tools/pmc_probe.py" > "$O/log.txt" 2>&1
echo "rc=$?"
