"""DTLS-SRTP keying on the GPU (include/re_srtp_keying.h, dtls_prf.hip)
through the C-ABI library:

  * srtp_dtls_keying_many() on all 64 golden connections (OpenSSL's TLS 1.2
    PRF with the "EXTRACTOR-dtls_srtp" label, P_SHA256 and P_SHA384, split
    like tls_srtp_keyinfo, src/tls/openssl/tls.c:1083-1157): bit-exact
    client/server keys, per PRF and with both PRFs mixed in one call;
  * srtp_alloc_dtls_many(): the client's sender interoperates with the
    server's receiver and back (test/dtls.c:346-368 checks the same with a
    real handshake), and a protected packet equals the oracle's
    srtp_encrypt under the golden client key;
  * a 64K-connection burst keyed and set up in one call each way.
"""
import json
import os

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    P.load()
    return torch


@pytest.fixture(scope="module")
def cases():
    with open(os.path.join(ROOT, "tests", "golden",
                           "dtls_srtp_keying.json")) as f:
        return json.load(f)["cases"]


def items(cs):
    return [(bytes.fromhex(c["master"]), bytes.fromhex(c["client_random"]),
             bytes.fromhex(c["server_random"]), c["prf"]) for c in cs]


@pytest.mark.parametrize("prf", [0, 1, "mixed"])
def test_keying_many_vs_golden(torch_cuda, cases, prf):
    for suite in sorted({c["suite"] for c in cases}):
        cs = [c for c in cases if c["suite"] == suite and
              (prf == "mixed" or c["prf"] == prf)]
        if prf == "mixed":          # interleave the two PRFs in one call
            cs = cs[0::2] + cs[1::2]
            assert {c["prf"] for c in cs} == {0, 1}
        e, cli, srv = P.dtls_keying_many(suite, items(cs))
        assert e == 0, P.lib().srtp_gpu_error()
        assert [k.hex() for k in cli] == [c["cli_key"] for c in cs]
        assert [k.hex() for k in srv] == [c["srv_key"] for c in cs]


def test_keying_bad_prf(torch_cuda, cases):
    import errno
    it = items(cases[:2])
    it[1] = it[1][:3] + (2,)
    e, _, _ = P.dtls_keying_many(1, it)
    assert e == errno.EINVAL


def rtp(seq, n=200):
    return bytes([0x80, 0, seq >> 8, seq & 0xff]) + bytes(4) + \
        (0x0BADCAFE).to_bytes(4, "big") + bytes(range(256))[:n - 12]


def test_alloc_dtls_endpoints_interoperate(torch_cuda, cases):
    ob = O.OracleBackend()
    for suite in sorted({c["suite"] for c in cases}):
        cs = [c for c in cases if c["suite"] == suite]
        e1, ctx_c, crx_c = P.alloc_dtls_many(suite, items(cs), True)
        e2, ctx_s, crx_s = P.alloc_dtls_many(suite, items(cs), False)
        assert e1 == 0 and e2 == 0
        for i, c in enumerate(cs):
            for seq in (7, 8):
                pkt = rtp(seq)
                # client -> server, checked against the oracle under the
                # golden client key
                mb = P.new_mbuf(pkt, 512)
                assert ctx_c[i].encrypt(mb) == 0
                wire = P.mbuf_bytes(mb)
                octx = ob.alloc(suite, bytes.fromhex(c["cli_key"]), 0)[0]
                if seq == 7:
                    r = ob.call(octx, "srtp_encrypt", 512, 0, len(pkt), pkt,
                                0)
                    assert r[0] == 0 and r[4][:r[2]] == wire
                ob.free(octx)
                mb.contents.pos = 0
                assert crx_s[i].decrypt(mb) == 0
                assert P.mbuf_bytes(mb) == pkt
                P.free_mbuf(mb)
                # server -> client
                mb = P.new_mbuf(pkt, 512)
                assert ctx_s[i].encrypt(mb) == 0
                mb.contents.pos = 0
                assert crx_c[i].decrypt(mb) == 0
                assert P.mbuf_bytes(mb) == pkt
                P.free_mbuf(mb)
        for s in ctx_c + crx_c + ctx_s + crx_s:
            s.close()


def test_keying_burst_64k(torch_cuda):
    rng = np.random.default_rng(17)
    n = 1 << 16
    raw = rng.integers(0, 256, size=(n, 112), dtype=np.uint8)
    its = [(r[:48].tobytes(), r[48:80].tobytes(), r[80:].tobytes())
           for r in raw]
    e, tx, rx = P.alloc_dtls_many(1, its, True)
    assert e == 0 and len(tx) == n and len(rx) == n
    # spot check three connections against the restated PRF
    from tests.test_keying_cpu import p_sha256
    e, cli, srv = P.dtls_keying_many(1, [its[0], its[n // 2], its[-1]])
    for (m, c, s), k1, k2 in zip([its[0], its[n // 2], its[-1]], cli, srv):
        km = p_sha256(m, b"EXTRACTOR-dtls_srtp" + c + s, 60)
        assert k1 == km[:16] + km[32:46] and k2 == km[16:32] + km[46:60]
    for s in tx + rx:
        s.close()
