#!/bin/bash
# round-5 session probe: HitSet A/B (current vs previous annotate library), then the chain-floor probe
set -u
LIBS="libskm libskm_prev" bash tools/hitset_ab.sh || exit 1
C3_SETS='"giant_class=14 route_first=1 route_first_min=131072"' \
  W2_OPTS="--option route_heavy_min=8192 --option route_first_min=8192" bash tools/floor_probe.sh
