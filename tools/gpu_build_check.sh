#!/bin/bash
# build-path GPU tests, then the C3 diagnostics (cached inputs) -- one gpurun call
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread > $O/t_build.log 2>&1 || { tail -30 $O/t_build.log; exit 1; }
tail -2 $O/t_build.log
timeout -k 10 300 python3 bench.py --cache-dir /tmp/c3 --cache-only > $O/cache.log 2>&1 || { tail -5 $O/cache.log; exit 1; }
timeout -k 10 400 python3 -u tools/c3_diag.py --cache-dir /tmp/c3 --steps 2 ${DIAG_ARGS:-} > $O/c3diag.log 2>&1; rc=$?
cat $O/c3diag.log | grep -v "^\[diag\]   >=" ; exit $rc
