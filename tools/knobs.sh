#!/bin/bash
# run the probe under several knob settings; prints the timings of each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
CFGS=${CFGS:-"SKM_OVF_LONG_CLASS=15|SKM_OVF_LONG_CLASS=14|SKM_OVF_LONG_CLASS=13|SKM_OVF_LONG_CLASS=12"}
IFS='|' read -ra ARR <<< "$CFGS"
for cfg in "${ARR[@]}"; do
  echo "== $cfg"
  env SKM_PROBE_RUNS=4 $cfg timeout -k 10 120 python tools/pmc_probe.py 2>&1 | tail -1
done
