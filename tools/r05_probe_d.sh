#!/bin/bash
# round-5 session probe: HitSet A/B (branchless k_seg_process vs round 4's annotate), then the
# chain-floor C3 run with the giant chains at the highest wave priority
set -u
LIBS="libskm libskm_prev" bash tools/hitset_ab.sh || exit 1
C3_SETS='"giant_class=14 route_first=1 route_first_min=131072 chain_prio=3"' W2_RF=" " bash tools/floor_probe.sh
