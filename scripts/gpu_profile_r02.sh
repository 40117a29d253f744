#!/bin/bash
# Round profile set per BASELINE config (default 2 3 4): HBM traffic passes
# (FETCH_SIZE, WRITE_SIZE: one counter each, MI355X_MICROARCH.md), one SQ
# pass (VALU / LDS issue), summarised on the box into
# gpurun_out/prof_r02/{pmc_traffic,pmc_sq}.json, then the kernel-trace
# --stats run of bench.py whose JSON line (roofline with traffic and
# int_frac attached from those summaries) is kept beside its rocprof
# summary.  Every GPU step under its own time limit; the first failure ends
# the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r02
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
BA="--no-cpu-baseline --no-verify --steps 2 --warmup 1"
for c in ${CONFIGS:-2 3 4}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace -f csv -d $O/pmc_c${c}_$C -o run -- python3 $R/bench.py --config $c $BA ${BENCH_ARGS:-} > $O/pmc_c${c}_$C.log 2>&1 || exit $?
  done
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/pmcsq_c$c -o run -- python3 $R/bench.py --config $c $BA ${BENCH_ARGS:-} > $O/pmcsq_c$c.log 2>&1 || exit $?
  python3 $R/scripts/pmc_summary.py $O/pmc_traffic.json config$c $O/pmc_c${c}_FETCH_SIZE $O/pmc_c${c}_WRITE_SIZE > $O/pmc_c$c.txt || exit $?
  python3 $R/scripts/pmc_sq_summary.py --json $O/pmc_sq.json config$c $O/pmcsq_c$c > $O/pmcsq_c$c.txt || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/stats_c$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 --traffic-json $O/pmc_traffic.json --sq-json $O/pmc_sq.json ${BENCH_ARGS:-} > $O/bench_c$c.json 2> $O/bench_c$c.err || exit $?
done
