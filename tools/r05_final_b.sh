#!/bin/bash
# round-5 final measurements, part b: FETCH/WRITE counter passes (C3, C2), then the SQ counters at C3
set -u
PHASE=pmc bash tools/gpu_profile.sh || exit 1
PHASE=sq bash tools/gpu_profile.sh
