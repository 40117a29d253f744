#!/bin/bash
# RTCP goldens from the reference itself (oracle/gen_rtcp_golden.c linked
# against /root/reference/src/rtp/pkt.c, rr.c, sdes.c, fb.c by
# `make -C oracle ref`): decode loop outputs (descriptors, items, errno,
# stop) and rtcp_encode outputs.
set -e -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle ref
./oracle/_ref/gen_rtcp_golden 2>/dev/null | gzip -9n > tests/golden/rtcp_decode_golden.json.gz
./oracle/_ref/gen_rtcp_golden encode 2>/dev/null | gzip -9n > tests/golden/rtcp_encode_golden.json.gz
ls -la tests/golden/rtcp_*_golden.json.gz
