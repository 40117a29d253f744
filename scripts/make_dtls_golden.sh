#!/bin/sh
# Regenerate tests/golden/dtls_srtp_keying.json (OpenSSL's TLS 1.2 PRF as
# used by SSL_export_keying_material for tls_srtp_keyinfo, see
# oracle/gen_dtls_prf.c).  Build container only.
set -e
cd "$(dirname "$0")/.."
make -s -C oracle dtls
oracle/_build/gen_dtls_prf > tests/golden/dtls_srtp_keying.json
python -c "import json; json.load(open('tests/golden/dtls_srtp_keying.json'))"
