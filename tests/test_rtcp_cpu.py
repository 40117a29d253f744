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
