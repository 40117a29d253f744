#!/bin/bash
# Per-call A/B: completion word vs stream sync, interleaved.
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py --percall --no-cpu-baseline --percall-calls 8000 "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b flag1
b sync1 --tune smallsync=1
b flag2
b sync2 --tune smallsync=1
