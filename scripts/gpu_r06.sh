#!/bin/bash
# Round-6 GPU checks: the named test files ($TESTS), then bench lines
# ($BENCHES: name=args;name=args, each a bench.py run), optionally the
# 8-rank same-device rehearsal ($REH8=1), into gpurun_out/r06/$TAG/.
# Every GPU step under its own time limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/${TAG:-run}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || exit $?
fi
IFS=';' read -ra BS <<< "${BENCHES:-}"
for nb in "${BS[@]}"; do
  n=${nb%%=*}; a=${nb#*=}
  timeout -k 10 300 python bench.py $a > $O/$n.json 2> $O/$n.err || exit $?
done
if [ -n "$REH8" ]; then
  timeout -k 10 600 python bench.py --gpus 8 --same-device --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/config5_8ranks_same_gpu.json 2> $O/config5_8ranks_same_gpu.err || exit $?
fi
echo done > $O/done
