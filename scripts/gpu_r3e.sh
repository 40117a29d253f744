#!/bin/bash
# round-3 measurements, part 2
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit $?; }

b c4_forge1 --config 4 --forge 1
b c4_forge001 --config 4 --forge 0.001
b c2_forge1 --forge 1
b c4_nopipe --config 4 --no-pipeline
b c2 --steps 10
RE_SRTP_LIB=$PWD/re_amd/lib/variants/b1bitop3.so b c2_b1 --steps 10
b c3 --config 3 --steps 10
RE_SRTP_LIB=$PWD/re_amd/lib/variants/b1bitop3.so b c3_b1 --config 3 --steps 10
timeout -k 10 300 python bench.py --percall > $O/percall.json 2> $O/percall.err || exit $?
timeout -k 10 200 python bench.py --udp --udp-seconds 4 > $O/udp.json 2> $O/udp.err || exit $?
timeout -k 10 200 python bench.py --udp --udp-seconds 4 --udp-pairs 1 --udp-sync > $O/udp_sync1.json 2> $O/udp_sync1.err || exit $?
