#!/bin/bash
# Two ranks of bench.py on whatever GPUs are visible (device = local_rank % device_count), small
# shards: exercises the RCCL exchange path end to end.  Output under gpurun_out/rccl/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rccl
mkdir -p "$O"
cd "$R"
NCCL_DEBUG=WARN timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --seqs-total 400000 --weak-seqs 100000 --annot-queries 0 --matrix-seqs 20000 \
  --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench2.log" 2>&1
rc=$?
echo "rc=$rc"
tail -30 "$O/bench2.log" | cut -c1-400
exit $rc
