#!/bin/bash
# Full GPU suite + smoke after the late planner-hint change.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4r
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
