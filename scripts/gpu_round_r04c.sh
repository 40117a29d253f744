#!/bin/bash
# Round-4 end set, part C (after the per-call, GCM-store and rx-walk
# changes): full GPU suite, smoke, the lines those changes move.
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c2
b c3 --config 3 --no-cpu-baseline
b c3_rtcp --config 3 --rtcp --no-cpu-baseline
b c2_percall --percall --no-cpu-baseline
b c3_percall_gcm128 --percall --percall-suite 4 --no-cpu-baseline
b c3_percall_gcm256 --percall --percall-suite 5 --no-cpu-baseline
timeout -k 10 300 python scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
