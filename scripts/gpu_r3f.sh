#!/bin/bash
# round-3 re-measurement after the container restart: the round bench set,
# config-4 forged lines, per-call latency, UDP, byte-1 bitop3 A/B.
# Each GPU step under its own limit; the first failure ends the script.
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
timeout -k 10 120 scripts/ubench_sdwa.bin > $O/ubench_sdwa.txt 2>&1 || exit $?
b c2 --steps 10
RE_SRTP_LIB=$PWD/re_amd/lib/variants/b1bitop3.so b c2_b1 --steps 10
b c2b --steps 10
b c3 --config 3 --steps 10
RE_SRTP_LIB=$PWD/re_amd/lib/variants/b1bitop3.so b c3_b1 --config 3 --steps 10
b c4 --config 4 --steps 10
b c4_forge1 --config 4 --forge 1
b c4_forge001 --config 4 --forge 0.001
b c2_forge1 --forge 1
b c2_rtcp --rtcp
b c3_rtcp --config 3 --rtcp
b c2_ssrc2 --ssrcs 2
b c2_fresh2 --ssrcs 2 --fresh-streams
b c2_host --host-arrays
b c2_e2e --e2e
timeout -k 10 300 python bench.py --percall --no-cpu-baseline > $O/percall.json 2> $O/percall.err || exit $?
timeout -k 10 200 python bench.py --udp --udp-seconds 4 > $O/udp.json 2> $O/udp.err || exit $?
timeout -k 10 200 python bench.py --udp --udp-seconds 4 --udp-pairs 1 --udp-sync > $O/udp_sync1.json 2> $O/udp_sync1.err || exit $?
