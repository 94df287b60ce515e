#!/bin/bash
# SQ counter passes on the build kernels (own passes, kernel-trace only; no sys/runtime trace).
# SQ_CMD: the profiled program (default: the C2 probe build, tools/pmc_probe.py); SQ_OUT: the
# output directory under gpurun_out (default pmc_sq).  rocprofv3 collects counters per dispatch,
# so the profiled kernels run one at a time (no side-stream overlap) in these passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${SQ_OUT:-pmc_sq}
mkdir -p "$O"
export TMPDIR=/tmp
export SKM_PROBE_ANNOT=${SKM_PROBE_ANNOT:-1}
cd /tmp
timeout -k 10 300 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$O/p$i" -o run -- ${SQ_CMD:-python3 $R/tools/pmc_probe.py} > "$O/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/p$i.log"; exit $rc; fi
done
