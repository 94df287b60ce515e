#!/bin/bash
# quick check of the emit placement (C3 bench), then the SQ counter passes (C2 probe build + annotate)
set -u
bash tools/gpu_r04.sh f "tests/test_gpu_build.py::test_key_range_passes" --steps 4 --warmup 2 --no-cpu-baseline \
  --annot-queries 0 --matrix-seqs 0 --weak-seqs 0 --recall 0 || exit $?
bash tools/pmc_sq.sh
