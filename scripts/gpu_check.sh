#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, kernel-trace profile.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest_rc=$rc" >> gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-verify --steps 3 --warmup 1 ${BENCH_ARGS:-} > $R/gpurun_out/prof.log 2>&1 || exit $?
fi
exit ${rc:-0}
