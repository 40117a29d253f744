#!/bin/bash
# The CPU suite against the host C built under gcc's sanitizers
# (make -C re_amd SAN=address,undefined): the library the tests load is the
# instrumented one (RE_SRTP_LIB), the runtime preloaded into python.
# Leak detection is off (the interpreter itself is not leak-clean); UBSan
# aborts on the first report (-fno-sanitize-recover=all).
#   scripts/san_check.sh [pytest args]    (default: -m "not gpu")
# On a GPU box the same with -m gpu runs the threaded paths instrumented.
set -e -o pipefail
cd "$(dirname "$0")/.."
make -s -j8 -C re_amd SAN=address,undefined
LIB=re_amd/lib/libre_srtp_amd_san-address-undefined.so
export RE_SRTP_LIB=$PWD/$LIB
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
  python -u -m pytest -q -p no:cacheprovider "${@:--m not gpu}"
