#!/bin/bash
# C3 A/B: k_big_groups grids on the tail stream (beside the next pass's staging)
set -u
bash tools/c3_opts.sh "" "big_grid_large=128" "big_grid=512 big_grid_large=128" "big_grid=1024 big_grid_large=256" ""
