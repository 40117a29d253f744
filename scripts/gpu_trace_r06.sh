#!/bin/bash
# Round-6 kernel traces: per workload ($WLS: tag=bench args;...) one
# rocprofv3 --kernel-trace --stats run of bench.py (the bench line beside
# it), then the per-step split (scripts/step_gaps.py) and the last kernels
# with their gaps (scripts/timeline.py), into gpurun_out/r06/trace_$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/trace_${TAG:-run}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra W <<< "${WLS:-config4=--config 4}"
for tw in "${W[@]}"; do
  t=${tw%%=*}; a=${tw#*=}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/$t -o run -- python3 $R/bench.py $a --no-cpu-baseline --steps ${STEPS:-20} --warmup ${WARM:-5} > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
  kt=$(find $O/$t -name '*kernel_trace.csv' | head -1)
  ks=$(find $O/$t -name '*kernel_stats.csv' | head -1)
  cp $ks $O/${t}_kernel_stats.csv
  python3 $R/scripts/step_gaps.py $kt 10 > $O/${t}_step_split.txt 2>&1 || exit $?
  python3 $R/scripts/timeline.py $kt ${TL:-40} --crypto > $O/${t}_timeline.txt 2>&1 || exit $?
done
echo done > $O/done
