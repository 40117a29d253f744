#!/bin/bash
# Round-6 profile set (the round-5 recipe on the round-6 build).  Per workload ($WLS: tag=bench args;...): HBM
# traffic passes (FETCH_SIZE, WRITE_SIZE: one counter each,
# MI355X_MICROARCH.md), one SQ/GRBM pass, summarised on the box by
# scripts/pmc_r05.py into gpurun_out/prof_r06/r06_pmc.json (kernel name +
# workload keys), then the kernel-trace --stats run of bench.py whose JSON
# line carries the annotations from that file.  Every GPU step under its
# own time limit; the first failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r06
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
BA="--no-cpu-baseline --no-verify --steps 2 --warmup 1"
IFS=';' read -ra W <<< "${WLS:-config2=--config 2;config3=--config 3;config4=--config 4;config2_rtcp=--config 2 --rtcp;config3_rtcp=--config 3 --rtcp}"
for tw in "${W[@]}"; do
  t=${tw%%=*}; a=${tw#*=}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -f csv -d $O/${t}_$C -o run -- python3 $R/bench.py $a $BA > $O/${t}_$C.log 2>&1 || exit $?
  done
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/${t}_SQ -o run -- python3 $R/bench.py $a $BA > $O/${t}_SQ.log 2>&1 || exit $?
  python3 $R/scripts/pmc_r05.py $O/r06_pmc.json $t $O/${t}_FETCH_SIZE $O/${t}_WRITE_SIZE $O/${t}_SQ > $O/${t}_pmc.txt || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/stats_$t -o run -- python3 $R/bench.py $a --no-cpu-baseline --steps 20 --warmup 5 --traffic-json $O/r06_pmc.json > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
done
