#!/bin/bash
# Full GPU suite + smoke on the final build; kernel-trace of config 4.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4v
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/stats_c4 -o run -- python3 $R/bench.py --config 4 --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
