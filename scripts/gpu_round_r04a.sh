#!/bin/bash
# Round-4 end measurement set, part A: the full GPU suite, smoke, the
# BASELINE configs and their SRTCP lines.  Every GPU step under its own
# time limit; the first failure ends the script.
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c2
b c3 --config 3
b c4 --config 4
b c2_rtcp --rtcp --no-cpu-baseline
b c3_rtcp --config 3 --rtcp --no-cpu-baseline
