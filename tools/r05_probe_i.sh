#!/bin/bash
# C3 A/B: smaller persistent grids for the overflow path beside the group-by (it has until the
# next pass's split with tail_async)
set -u
bash tools/c3_opts.sh "" "heavy_grid=256 overflow_grid=256" "heavy_grid=128 overflow_grid=128 split_grid=128" "heavy_grid=512 overflow_grid=512 split_grid=256" ""
