#!/bin/bash
# Round 3 (m): side-stream persistent grid sizes (with and without pipelined passes), C3 A/B.
set -u
export GPU_MAX_HW_QUEUES=8
bash tools/c3_opts.sh "" "overflow_grid=256" "overflow_grid=256 overlap=1" "overflow_grid=256 split_grid=128 heavy_grid=128 overlap=1" "heavy_grid=128" "overflow_grid=512 heavy_grid=256"
