#!/bin/bash
# C3 A/B: the overflow / emission side streams confined to a CU subset (side_cus), now that the
# main stream only waits for them at the next pass's split (tail_async)
set -u
bash tools/c3_opts.sh "" "side_cus=128" "side_cus=96" "side_cus=64" ""
