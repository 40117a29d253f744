#!/bin/sh
# Regenerate tests/golden/fullsize_digests.json: the reference src/srtp
# (oracle/_ref/ref_digest, built by `make -C oracle ref` from the sources
# under /root/reference) over the full BASELINE.json configs 1-4 and the shapes 5-12
# (ref_digest.c).
# Build container only (needs /root/reference); ~3 min (SHARDS=0 skips
# the config-5 shard file, ~2 min more).
set -e
cd "$(dirname "$0")/.."
make -s -C oracle ref
{
	echo '{"generator": "oracle/ref_digest.c (reference src/srtp + OpenSSL)",'
	echo ' "configs": ['
	oracle/_ref/ref_digest 1; echo ','
	oracle/_ref/ref_digest 2; echo ','
	oracle/_ref/ref_digest 3; echo ','
	oracle/_ref/ref_digest 4; echo ','
	oracle/_ref/ref_digest 5; echo ','
	oracle/_ref/ref_digest 6; echo ','
	oracle/_ref/ref_digest 7; echo ','
	oracle/_ref/ref_digest 8; echo ','
	oracle/_ref/ref_digest 9; echo ','
	oracle/_ref/ref_digest 10; echo ','
	oracle/_ref/ref_digest 11; echo ','
	oracle/_ref/ref_digest 12
	echo ']}'
} > tests/golden/fullsize_digests.json
python -c "import json; json.load(open('tests/golden/fullsize_digests.json'))"
[ "${SHARDS:-1}" = 0 ] && exit 0
# config 5 whole: 8 shards of 1M of the one 8M-packet stream, per-shard
# digests and the reference's boundary states (~2 min)
oracle/_ref/ref_digest shards 8 1048576 > tests/golden/config5_shards.json
python -c "import json; json.load(open('tests/golden/config5_shards.json'))"
