#!/bin/bash
# Reusable GPU lease script (round 5 on).  Into gpurun_out/$TAG/ (default
# "run"):
#   TESTS="file::test ..."        pytest -m gpu of those, tests.log
#   BENCHES="name=args;..."       bench.py lines, name.json / name.err
#   TRACES="name=args;..."        rocprofv3 --kernel-trace --stats of a
#                                 bench.py run: trace_name/ (csv) + name.json
# Every GPU step runs under its own time limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-run}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || exit $?
fi
IFS=';' read -ra BS <<< "${BENCHES:-}"
for nb in "${BS[@]}"; do
  n=${nb%%=*}; a=${nb#*=}
  timeout -k 10 ${BENCH_TIMEOUT:-150} python bench.py $a > $O/$n.json 2> $O/$n.err || exit $?
done
IFS=';' read -ra TS <<< "${TRACES:-}"
for nb in "${TS[@]}"; do
  n=${nb%%=*}; a=${nb#*=}
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$n -o run -- python3 $R/bench.py $a > $O/$n.json 2> $O/$n.err) || exit $?
done
echo done > $O/done
