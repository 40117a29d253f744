#!/bin/bash
# Round-end measurement set: the bench lines committed under profiles/
# (configs 2/3/4, SRTCP, host-array API, end-to-end, socket to socket,
# adversarial receive, several SSRCs).  Every GPU step under its own
# time limit; the first failure ends the script.
set -o pipefail
O=gpurun_out/round
mkdir -p $O
b() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?
}
b c2
b c3 --config 3
b c4 --config 4
b c2_rtcp --rtcp --no-cpu-baseline
b c3_rtcp --config 3 --rtcp --no-cpu-baseline
b c2_host --host-arrays --no-cpu-baseline
b c2_sync --sync --no-cpu-baseline
b c2_e2e --e2e --no-cpu-baseline
b c2_udp --udp
b c2_forge1 --forge 1 --no-cpu-baseline
b c2_ssrc2 --ssrcs 2 --no-cpu-baseline
