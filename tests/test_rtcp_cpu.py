"""RTCP compound decode, CPU side: the C restatement (oracle/rtcp_oracle.c)
against the reference itself -- tests/golden/rtcp_decode_golden.json.gz,
written by oracle/gen_rtcp_golden.c running libre's receive loop
(`while (0 == rtcp_decode(&msg, mb))`, /root/reference/src/rtp/rtp.c:164,
pkt.c:337-551) over 2032 packets: every message type pkt.c decodes, well
formed compounds, truncations, bad versions / lengths / counts, junk.
Per message: [off, size, pt, count, length, ssrc, aux]; per packet the
errno that ended the loop and the offset where that call began.
"""
import ctypes
import errno
import gzip
import json
import os

import pytest

from tests import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "rtcp_decode_golden.json.gz")


def load_cases():
    with gzip.open(GOLDEN, "rt") as f:
        return json.load(f)["cases"]


def oracle_walk(pkt, maxmsg=64):
    L = O.lib()
    f = L.oracle_rtcp_walk
    u32p = ctypes.POINTER(ctypes.c_uint32)
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u32p, ctypes.c_uint32,
                  u32p, u32p]
    f.restype = ctypes.c_int
    desc = (ctypes.c_uint32 * (7 * maxmsg))()
    nmsg, stop = ctypes.c_uint32(), ctypes.c_uint32()
    err = f(pkt, len(pkt), desc, maxmsg, ctypes.byref(nmsg),
            ctypes.byref(stop))
    msgs = [list(desc[7 * k:7 * k + 7]) for k in range(min(nmsg.value,
                                                           maxmsg))]
    return msgs, err, stop.value, nmsg.value


@pytest.fixture(scope="module")
def cases():
    return load_cases()


def test_golden_shape(cases):
    assert len(cases) == 2032
    pts = {m[2] for c in cases for m in c["msgs"]}
    assert {192, 193, 200, 201, 202, 203, 204, 205, 206, 207} <= pts
    # both whole-packet walks and walks ended by a malformed message
    assert any(c["stop"] * 2 == len(c["pkt"]) for c in cases)
    assert any(c["stop"] * 2 < len(c["pkt"]) for c in cases)


def test_oracle_vs_reference(cases):
    for i, c in enumerate(cases):
        pkt = bytes.fromhex(c["pkt"])
        msgs, err, stop, n = oracle_walk(pkt)
        assert (msgs, err, stop) == (c["msgs"], c["err"], c["stop"]), i


ENC_GOLDEN = os.path.join(ROOT, "tests", "golden", "rtcp_encode_golden.json.gz")


def load_encode_cases():
    """rtcp_encode goldens (oracle/gen_rtcp_golden.c encode: the
    reference's rtcp_encode calls, src/rtp/pkt.c:136-335)"""
    with gzip.open(ENC_GOLDEN, "rt") as f:
        return json.load(f)["cases"]


def test_encode_golden_decodes_back(cases):
    """the encode goldens are well-formed compounds: the reference-pinned
    decode restatement walks every successful packet made of messages whose
    body it parses whole (SR/RR/SDES with count = blocks / chunks, BYE,
    (a reason of at most 255 bytes: the length byte is (uint8_t)str_len,
    pkt.c:181-183), APP, FIR, NACK; header count < 32) to its end, one message per
    rtcp_encode call with the spec's type, count and sender; and the
    decode goldens carry the contents of every item kind"""
    enc = load_encode_cases()
    assert len(enc) == 1500
    assert {c["err"] for c in enc} == {0, errno.EINVAL, errno.EBADMSG}
    checked = 0
    for i, c in enumerate(enc):
        if c["err"]:
            assert c["out"] == ""
            continue
        whole = all(m[0] in (192, 193, 204) or
                    (m[0] == 203 and not (m[2] and m[13] > 255)) or
                    (m[0] in (200, 201, 202) and m[1] == m[10])
                    for m in c["msgs"]) and \
            all(m[1] < 32 for m in c["msgs"])
        if not whole:
            continue
        pkt = bytes.fromhex(c["out"])
        msgs, e, s, n = oracle_walk(pkt, 64)
        assert (e, s, n) == (errno.EBADMSG, len(pkt), len(c["msgs"])), i
        for m, spec in zip(msgs, c["msgs"]):
            assert m[2] == spec[0] and m[3] == spec[1], i
            if spec[0] in (192, 193, 200, 201, 204):
                assert m[5] == spec[3], i
        checked += 1
    assert checked > 200
    kinds = {it[1] for c in cases for it in c["items"]}
    assert kinds == set(range(1, 19))
