#!/bin/bash
# Quick GPU check: the named test files ($TESTS), then bench lines ($BENCHES:
# name=args;name=args, each a bench.py run), into gpurun_out/quick/.
set -o pipefail
O=gpurun_out/quick
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || exit $?
fi
IFS=';' read -ra BS <<< "${BENCHES:-}"
for nb in "${BS[@]}"; do
  n=${nb%%=*}; a=${nb#*=}
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > $O/$n.json 2> $O/$n.err || exit $?
done
