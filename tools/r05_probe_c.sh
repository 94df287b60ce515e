#!/bin/bash
# round-5 session probe: the chain-floor C3 run (giant chains sorted longest first)
set -u
C3_SETS='"giant_class=14 route_first=1 route_first_min=131072"' W2_RF=" " bash tools/floor_probe.sh
