"""The LIBRE=1 library inside libre's own event loop and UDP layer
(§8(f)1: the transform on libre's helper chain, include/re_srtp_libre.h).

tests/libre_udp_driver.py runs in a fresh process: libre's src/main,
src/udp, src/net, src/sa and src/tmr compiled from the reference sources
without src/srtp (oracle/_ref/libre_net.so) host re_amd/lib/
libre_srtp_amd_libre.so, whose helper is registered on a udp_sock with
udp_register_helper (/root/reference/src/udp/udp.c:830).  Checked against
the reference's own results (tests/golden/fullsize_digests.json config 1,
oracle/ref_digest.c):

  * udp_send() of the 1024 config-1 packets: the datagrams on the wire are
    the reference's protected arena, and the sender state is its state;
  * those datagrams received through udp_read(): the socket's handler gets
    every plaintext in order at the reference's pos/end, a replayed and a
    forged datagram are dropped (EALREADY / EAUTH), and the receiver state
    is the reference's;
  * rtcp-mux (RTP and RTCP on one socket, libre's src/rtp/rtp.c:184-196):
    the RTCP datagrams take the SRTCP transform in datagram order -- the
    wire equals the oracle's srtp_encrypt / srtcp_encrypt sequence, and the
    handler gets every plaintext back in order.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from re_amd import workload as W
from tests import fullsize_util as F

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_libre_helper_chain_vs_reference():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for p in ("oracle/_ref/libre_net.so", "re_amd/lib/libre_srtp_amd_libre.so"):
        assert os.path.exists(os.path.join(ROOT, p)), p
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests",
                                                     "libre_udp_driver.py")],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    ref = F.load()[1]
    arena, pos, end, cap, _, _ = W.build_config(1)
    n, slot = ref["n"], ref["slot"]

    # send: the wire is the reference's protected arena
    wire = [bytes.fromhex(w) for w in out["wire"]]
    assert len(wire) == n
    prot = np.zeros(n * slot, dtype=np.uint8)
    pend = np.zeros(n, dtype=np.uint32)
    for i, d in enumerate(wire):
        prot[i * slot:i * slot + len(d)] = np.frombuffer(d, dtype=np.uint8)
        pend[i] = i * slot + len(d)
    bad = F.compare(ref["protect"], prot, n, slot, pend,
                    np.zeros(n, dtype=np.int32),
                    F.state_bytes([tuple(out["tx_state"])]))
    assert not bad, bad

    # receive: every authentic packet's plaintext in order, at pos 0
    keep = [i for i in range(n) if i != 900]
    got = out["got"]
    assert len(got) == len(keep)
    for (p, e, b), i in zip(got, keep):
        pkt = arena[pos[i]:end[i]].tobytes()
        assert (p, e, bytes.fromhex(b)) == (0, len(pkt), pkt), i
    st = F.state_bytes([tuple(out["rx_state"])])
    assert hashlib.sha256(st).hexdigest() == ref["unprotect"]["states"]
    assert out["stats"] == [n + 1, n - 1, n, 2]

    # rtcp-mux: the oracle's per-packet sequence on one context pair
    from tests import oracle_lib as O
    from tests.libre_udp_driver import mux_packets
    mux = mux_packets(arena, pos, end)
    ob = O.OracleBackend()
    otx = ob.alloc(1, W.CONFIG1_KEY, 0)[0]
    wire2 = [bytes.fromhex(w) for w in out["mux_wire"]]
    assert len(wire2) == len(mux)
    for i, (pkt, w) in enumerate(zip(mux, wire2)):
        op = "srtcp_encrypt" if i % 10 == 9 else "srtp_encrypt"
        e, _, en, _, buf = ob.call(otx, op, 256, 0, len(pkt), pkt,
                                   len(pkt) + 20)
        assert e == 0 and buf[:en] == w, (i, op)
    got2 = out["mux_got"]
    assert [(p, e, bytes.fromhex(b)) for p, e, b in got2] == \
        [(0, len(m), m) for m in mux]
