"""The batched SRTP UDP helper (include/re_srtp_udp.h) over loopback,
through the C-ABI library on the GPU.

  * send: the config-1 workload (test/srtp.c key, 1024 x 160 B) protected
    by srtp_udp_send() (GPU protect + sendmmsg) arrives on a plain socket;
    the datagrams, laid out as the reference's arena, match the reference
    digests of tests/golden/fullsize_digests.json (oracle/ref_digest.c:
    src/srtp compiled from the reference sources) -- bytes, ends, final
    sender state;
  * receive: those reference-exact datagrams, sent from a plain socket to
    srtp_udp_recv() (recvmmsg + GPU unprotect), reach the handler as the
    plaintext packets with err 0, and the receive slots and final receiver
    state match the reference's unprotect digests;
  * errors: forged and replayed datagrams reach the handler with the
    oracle's errno (EAUTH, EALREADY), in datagram order;
  * both synchronous and pipelined (srtp_udp_pipeline: batch k+1 read
    while batch k is on the GPU; chunk j+1 protected while chunk j is
    sent);
  * send argument checks: a bad mbuf anywhere fails the call before any
    packet is protected or sent.
"""
import socket

import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import workload as W
from tests import fullsize_util as F
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

CHUNK = 128              # datagrams in flight (default socket buffers)


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    P.load()
    return torch


def udp_pair():
    a = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    b = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    a.bind(("127.0.0.1", 0))
    b.bind(("127.0.0.1", 0))
    for s in (a, b):
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 21)
    return a, b


def slot_view(mb, err, slot=256):
    """(err, pos, end relative to the datagram's slot, slot bytes)"""
    m = mb.contents
    base = m.size - slot                       # the view ends at its slot
    addr = P.ctypes.addressof(m.buf.contents) + base
    return (err, m.pos - base, m.end - base, P.ctypes.string_at(addr, slot))


def state_of(ctx):
    e, st = ctx.export(W.SSRC_BASE)
    assert e == 0
    return F.state_bytes([(st.roc, st.s_l, st.replay_rtp_lix,
                           st.replay_rtp_bitmap)])


def drain(sr, got, want):
    """srtp_udp_recv rounds until `want` datagrams reached the handler
    (pipelined: a round hands over the previous round's batch; a round
    that receives nothing flushes the batch in flight)"""
    for _ in range(10000):
        if len(got) >= want:
            return
        assert sr.recv(200) >= 0
    raise AssertionError("datagrams missing: %d of %d" % (len(got), want))


@pytest.mark.parametrize("pipeline", [False, True])
def test_udp_send_and_receive_vs_reference(torch_cuda, pipeline):
    ref = F.load()[1]
    arena, pos, end, cap, _, keys = W.build_config(1)
    n, slot = ref["n"], ref["slot"]
    key = keys[0].tobytes()
    a, b = udp_pair()
    addr_b = P.sockaddr_in(*b.getsockname())

    # ---- send: GPU protect + sendmmsg -> plain socket ----
    tx = P.Srtp(1, key)
    su = P.SrtpUdp(a.fileno(), tx=tx, batch=64, slot=256,
                   pipeline=pipeline)
    assert su.err == 0, P.lib().srtp_gpu_error()
    wire = []
    for c0 in range(0, n, CHUNK):
        mbs = [P.new_mbuf(arena[pos[i]:end[i]].tobytes(), 256)
               for i in range(c0, min(n, c0 + CHUNK))]
        sent, errs = su.send(addr_b, mbs)
        assert sent == len(mbs) and not any(errs), errs
        for mb in mbs:
            P.free_mbuf(mb)
        for _ in range(len(mbs)):
            wire.append(b.recv(2048))
    assert su.stats()[2] == n
    prot = np.zeros(n * slot, dtype=np.uint8)
    pend = np.zeros(n, dtype=np.uint32)
    for i, d in enumerate(wire):
        prot[i * slot:i * slot + len(d)] = np.frombuffer(d, dtype=np.uint8)
        pend[i] = i * slot + len(d)
    bad = F.compare(ref["protect"], prot, n, slot, pend,
                    np.zeros(n, dtype=np.int32), state_of(tx))
    assert not bad, bad
    su.close()

    # ---- receive: plain socket -> recvmmsg + GPU unprotect -> handler --
    got = []

    def handler(src, mb, err):
        got.append(slot_view(mb, err))

    rx = P.Srtp(1, key)
    sr = P.SrtpUdp(b.fileno(), rx=rx, batch=64, slot=256, handler=handler,
                   pipeline=pipeline)
    assert sr.err == 0
    addr_a = b.getsockname()
    for c0 in range(0, n, CHUNK):
        for d in wire[c0:c0 + CHUNK]:
            a.sendto(d, addr_a)
        drain(sr, got, min(n, c0 + CHUNK))
    assert [g[0] for g in got] == [0] * n
    unp = np.zeros(n * slot, dtype=np.uint8)
    uend = np.zeros(n, dtype=np.uint32)
    for i, (e, p0, e0, sb) in enumerate(got):
        L = len(wire[i])
        assert p0 == 0
        assert sb[:e0] == arena[pos[i]:end[i]].tobytes()
        unp[i * slot:i * slot + L] = np.frombuffer(sb[:L], dtype=np.uint8)
        uend[i] = i * slot + e0
    bad = F.compare(ref["unprotect"], unp, n, slot, uend,
                    np.zeros(n, dtype=np.int32), state_of(rx))
    assert not bad, bad
    assert sr.stats()[:2] == (n, n)
    sr.close()
    a.close()
    b.close()


@pytest.mark.parametrize("pipeline", [False, True])
def test_udp_receive_errors_vs_oracle(torch_cuda, pipeline):
    key = W.CONFIG1_KEY
    arena, pos, end, cap, _, _ = W.build_config(1, n=300)
    ob = O.OracleBackend()
    otx = ob.alloc(1, key, 0)[0]
    wire = []
    for i in range(300):
        p = arena[pos[i]:end[i]].tobytes()
        e, _, en, _, buf = ob.call(otx, "srtp_encrypt", 256, 0, len(p), p,
                                   len(p) + 16)
        wire.append(buf[:en])
    wire.insert(150, wire[100])                       # replay
    q = bytearray(wire[200])
    q[-1] ^= 1
    wire[200] = bytes(q)                              # forgery
    orx = ob.alloc(1, key, 0)[0]
    want = []
    for d in wire:
        e, po, en, _, buf = ob.call(orx, "srtp_decrypt", 256, 0, len(d), d,
                                    len(d))
        want.append((e, po, en, buf[:max(en, len(d))]))
    a, b = udp_pair()
    got = []

    def handler(src, mb, err):
        got.append(slot_view(mb, err))

    rx = P.Srtp(1, key)
    sr = P.SrtpUdp(b.fileno(), rx=rx, batch=100, slot=256, handler=handler,
                   pipeline=pipeline)
    for c0 in range(0, len(wire), CHUNK):
        for d in wire[c0:c0 + CHUNK]:
            a.sendto(d, b.getsockname())
        drain(sr, got, min(len(wire), c0 + CHUNK))
    for i, (g, w) in enumerate(zip(got, want)):
        assert g[:3] == w[:3], i
        assert g[3][:len(w[3])] == w[3], i
    assert sorted({g[0] for g in got}) == sorted({0, P.EAUTH, 114}) or \
        sorted({g[0] for g in got}) == sorted({0, P.EAUTH, 215})
    sr.close()
    a.close()
    b.close()


def test_udp_send_checks_every_mbuf_first(torch_cuda):
    a, b = udp_pair()
    tx = P.Srtp(1, W.CONFIG1_KEY)
    su = P.SrtpUdp(a.fileno(), tx=tx, batch=4, slot=256)
    pkt = bytes([0x80, 0, 0, 1]) + bytes(8) + bytes(100)
    mbs = [P.new_mbuf(pkt, 512) for _ in range(9)]
    big = P.new_mbuf(bytes([0x80, 0, 0, 2]) + bytes(400), 512)
    r, errs = su.send(P.sockaddr_in(*b.getsockname()), mbs + [big])
    assert r == -22                       # -EINVAL, nothing went out
    assert su.stats()[2] == 0
    e, st = tx.export(0)
    assert e != 0                         # no stream created: nothing ran
    for m in mbs + [big]:
        P.free_mbuf(m)
    su.close()
    a.close()
    b.close()


@pytest.mark.parametrize("pipeline", [True])
def test_udp_receive_failure_delivers_each_datagram_once(torch_cuda,
                                                         pipeline):
    """a batch whose GPU issue or completion fails (allocation failure
    injected, srtp_gpu_tune "fail_alloc") still reaches the handler, once,
    with the errno; the batch in flight before it is completed and
    delivered first, and later batches run normally.  Each attempt runs in
    a fresh thread: batch 0 has 16 datagrams, batch 1 (the faulted one)
    64.  Pipelined only: the synchronous device call on warm workspaces
    allocates nothing, so nothing can be injected there (its failure
    path, rx_fail, is the same code)"""
    import errno
    import threading
    key = W.CONFIG1_KEY
    arena, pos, end, cap, _, _ = W.build_config(1, n=192)
    ob = O.OracleBackend()
    otx = ob.alloc(1, key, 0)[0]
    wire = []
    for i in range(192):
        p = arena[pos[i]:end[i]].tobytes()
        e, _, en, _, buf = ob.call(otx, "srtp_encrypt", 256, 0, len(p), p,
                                   len(p) + 16)
        wire.append(buf[:en])
    a, b = udp_pair()

    def attempt(k):
        got = []

        def handler(src, mb, err):
            got.append(slot_view(mb, err)[0])

        rx = P.Srtp(1, key)
        sr = P.SrtpUdp(b.fileno(), rx=rx, batch=64, slot=256,
                       handler=handler, pipeline=pipeline)
        assert sr.err == 0
        for d in wire[:16]:
            a.sendto(d, b.getsockname())
        rets = [sr.recv(200)]
        for d in wire[16:80]:
            a.sendto(d, b.getsockname())
        P.lib().srtp_gpu_tune(b"fail_alloc", k)
        try:
            rets.append(sr.recv(200))
        finally:
            left = P.counter("fail_alloc")
            P.lib().srtp_gpu_tune(b"fail_alloc", 0)
        for d in wire[80:]:
            a.sendto(d, b.getsockname())
        for _ in range(100):
            if len(got) >= 192:
                break
            rets.append(sr.recv(200))
        st = sr.stats()
        sr.close()
        rx.close()
        return got, rets, left, st

    for k in range(1, 30):
        out = {}
        t = threading.Thread(target=lambda: out.update(r=attempt(k)))
        t.start()
        t.join(120)
        assert not t.is_alive() and "r" in out, k
        errs, rets, left, st = out["r"]
        assert len(errs) == 192 and st[0] == 192, (k, len(errs), rets)
        if left:                      # the fault was never reached
            assert errs == [0] * 192 and min(rets) >= 0
            continue
        assert min(rets) == -errno.ENOMEM, (k, rets)
        # batch 0 authentic; batch 1 failed as a whole; the rest authentic
        assert errs[:16] == [0] * 16 and errs[80:] == [0] * 112, k
        assert errs[16:80] == [errno.ENOMEM] * 64, (k, errs[16:80])
        break
    else:
        raise AssertionError("no allocation fault reached")
    a.close()
    b.close()
