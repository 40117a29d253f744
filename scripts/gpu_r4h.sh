#!/bin/bash
# Per-call A/B: slot streams created together (default) vs lazily (the
# variant library found first through LD_LIBRARY_PATH: percall's RUNPATH).
set -o pipefail
O=gpurun_out/r4h2
mkdir -p $O
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/re_amd/lib/variants/slots_lazy
b() { local n=$1 lp=$2; shift 2; LD_LIBRARY_PATH=$lp timeout -k 10 300 python bench.py --percall --no-cpu-baseline --percall-calls 8000 "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b eager1 ""
b lazy1 $V
b eager2 ""
b lazy2 $V
b eager3 ""
b lazy3 $V
