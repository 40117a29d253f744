#!/bin/bash
# Instruction-mix / utilisation counters for the crypto kernels, one
# counter set per rocprofv3 pass (<= 8 SQ, <= 2 GRBM counters each).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM GRBM_COUNT" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -f csv -d $R/gpurun_out/pmcsq_$i -o run -- python3 $R/bench.py --no-cpu-baseline --no-verify --steps 2 --warmup 1 ${BENCH_ARGS:-} > $R/gpurun_out/pmcsq_$i.log 2>&1 || exit $?
done
