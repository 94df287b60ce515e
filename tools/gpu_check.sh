set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
tail -5 $O/gputests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --json-out $O/bench.json > $O/bench.log 2>&1; rc=$?
tail -3 $O/bench.log; exit $rc
