#!/bin/bash
# PMC passes for bench.py's roofline annotations (profiles/r03_pmc.json):
# per workload ($WLS: tag=bench args;...), one pass each for FETCH_SIZE,
# WRITE_SIZE and the SQ/GRBM set (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE cannot share a pass; <= 8 SQ, <= 2 GRBM counters), kernel
# trace only beside --pmc.  Each pass under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc3
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra W <<< "${WLS:-config2=}"
for tw in "${W[@]}"; do
  t=${tw%%=*}; a=${tw#*=}
  for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"; do
    n=${C%% *}
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -f csv -d $R/gpurun_out/pmc3/${t}_$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-verify --steps 2 --warmup 1 $a > $R/gpurun_out/pmc3/${t}_$n.log 2>&1 || exit $?
  done
done
