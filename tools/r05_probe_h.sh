#!/bin/bash
# C3 A/B: the stashed-chain grid (lane_grid: fewer resident waves beside the group-by)
set -u
bash tools/c3_opts.sh "" "lane_grid=128" "lane_grid=64" "lane_grid=512" ""
