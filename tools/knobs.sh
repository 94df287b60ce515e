#!/bin/bash
# run the probe under several knob settings; prints the timings of each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CFGS=${CFGS:-"SKM_OVF_HEAVY=8192"}
IFS='|' read -ra ARR <<< "$CFGS"
for cfg in "${ARR[@]}"; do
  echo "== $cfg"
  env SKM_PROBE_RUNS=4 $cfg timeout -k 10 120 python tools/pmc_probe.py 2>&1 | tail -1
done
