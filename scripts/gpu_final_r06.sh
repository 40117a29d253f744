#!/bin/bash
# Round-6 final set on the final build: the GPU suite, smoke, the driver's
# default bench command, every config's bench line at the driver's step
# counts (--steps 20 --warmup 5), the per-packet API, the 8-rank
# same-device rehearsal of config 5.  Into gpurun_out/final_r06/; every
# GPU step under its own time limit, the first failure ends the script.
# NOTESTS=1 skips the suite and smoke; BENCHES overrides the bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final_r06
mkdir -p $O
cd $R
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
timeout -k 10 300 python3 bench.py --gpus 1 > $O/default.json 2> $O/default.err || exit $?
S="--steps 20 --warmup 5 --no-cpu-baseline"
IFS=';' read -ra BS <<< "${BENCHES:-c2=--config 2 $S;c3=--config 3 $S;c4=--config 4 $S;c2_rtcp=--config 2 --rtcp $S;c3_rtcp=--config 3 --rtcp $S;percall=--percall;percall_gcm=--percall --percall-suite 4 --no-cpu-baseline}"
for nb in "${BS[@]}"; do
  n=${nb%%=*}; a=${nb#*=}
  timeout -k 10 300 python3 bench.py $a > $O/$n.json 2> $O/$n.err || exit $?
done
if [ -z "$NOREH" ]; then
  timeout -k 10 600 python3 bench.py --gpus 8 --same-device --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/config5_8ranks_same_gpu.json 2> $O/config5_8ranks_same_gpu.err || exit $?
fi
echo done > $O/done
