#!/bin/bash
# Per-call A/B: runners 4 / 6 / 8 (8 slots), interleaved.
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py --percall --no-cpu-baseline --percall-calls 8000 "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b r4a --tune pcrunners=4
b r6a --tune pcrunners=6
b r8a --tune pcrunners=8
b r4b --tune pcrunners=4
b r6b --tune pcrunners=6
b r8b --tune pcrunners=8
