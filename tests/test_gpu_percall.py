"""Per-packet calls (the unchanged re_srtp.h API) from many threads at once
share GPU launches (srtp.c `one`: a runner takes every queued packet and
runs them as one multi-session batch per operation).  Each of 16 threads
owns its context pair (struct srtp is single-threaded, like the
reference's) and runs an interleaved srtp_encrypt / srtp_decrypt /
srtcp_encrypt / srtcp_decrypt sequence with ROC wrap, a replay and a
forgery; every call's errno, pos/end and bytes must equal the oracle's
(the C restatement, pinned to the reference goldens), whatever packets of
other threads shared its launch.
"""
import threading

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_fastpath import rtp_packet

pytestmark = pytest.mark.gpu

SUITES = [1, 0, 5, 4]


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def rtcp_packet(rng, ssrc, n):
    return bytes([0x80, 200, 0, (8 + n) // 4 - 1]) + ssrc.to_bytes(4, "big") \
        + rng.integers(0, 256, n, dtype=np.uint8).tobytes()


def script(t):
    """thread t's call sequence: (op, packet bytes or index of an earlier
    protected packet to replay / forge)"""
    rng = np.random.default_rng(100 + t)
    ssrc = 0x10000 + t
    out = []
    for k in range(120):
        seq = (65500 + k) & 0xffff
        out.append(("srtp_encrypt", rtp_packet(rng, seq, ssrc,
                                               plen=int(rng.integers(0, 300)))))
        out.append(("srtp_decrypt", ("prot", len(out) - 1)))
        if k % 10 == 3:
            out.append(("srtcp_encrypt", rtcp_packet(rng, ssrc, 4 * int(
                rng.integers(1, 20)))))
            out.append(("srtcp_decrypt", ("prot", len(out) - 1)))
    out.append(("srtp_decrypt", ("prot", 0)))              # replay
    out.append(("srtp_decrypt", ("forge", 2)))             # forgery
    return out


def run_thread(t, suite, key, backend, results):
    tx, rx = backend(suite, key)
    res, prot = [], {}
    for i, (op, arg) in enumerate(script(t)):
        if isinstance(arg, tuple):
            kind, j = arg
            data = bytearray(prot[j])
            if kind == "forge":
                data[-1] ^= 1
            data = bytes(data)
        else:
            data = arg
        ctx = tx if op.endswith("encrypt") else rx
        e, po, en, b = ctx(op, data)
        prot[i] = b[:en] if op.endswith("encrypt") else None
        res.append((e, po, en, b[:max(en, len(data))]))
    results[t] = res


def dev_backend(suite, key):
    def ctx_of(c):
        def call(op, data):
            mb = P.new_mbuf(data, len(data) + 64)
            e = c._op(op, mb)
            m = mb.contents
            out = (e, m.pos, m.end, P.mbuf_bytes(mb, m.size))
            P.free_mbuf(mb)
            return out
        return call
    return ctx_of(P.Srtp(suite, key)), ctx_of(P.Srtp(suite, key))


def oracle_backend(suite, key):
    ob = O.OracleBackend()

    def ctx_of(c):
        def call(op, data):
            e, po, en, so, buf = ob.call(c, op, len(data) + 64, 0,
                                         len(data), data, len(data) + 64)
            return (e, po, en, bytes(buf[:so]))
        return call
    return ctx_of(ob.alloc(suite, key, 0)[0]), ctx_of(ob.alloc(suite, key,
                                                               0)[0])


@pytest.mark.parametrize("suites,fuse,runners,hold,linger", [
    (SUITES, 1, 0, 0, 0), (SUITES, 0, 0, 0, 0), (SUITES, 1, 1, 0, 0),
    # CTR suites only, one runner (its queue gathers every thread's next
    # call): lists mixing operations run as one fused launch
    ([1, 0, 3, 2], 1, 1, 0, 0), ([1, 0, 3, 2], 0, 1, 0, 0),
    ([1, 0, 3, 2], 1, 0, 0, 0),
    # a new runner holding its launch 20 us while others run (pchold)
    (SUITES, 1, 0, 20, 0),
    # the lingering small kernel (pclinger): batches posted to a launch
    # already on the GPU, relaunched when it left
    (SUITES, 1, 0, 0, 100), ([1, 0, 3, 2], 1, 1, 0, 30),
    (SUITES, 0, 0, 0, 5)])
def test_threads_share_launches_exactly(torch_cuda, suites, fuse, runners,
                                        hold, linger):
    T = 16
    keys = [bytes((13 * t + i) & 0xff for i in range(46)) for t in range(T)]
    want, got = {}, {}
    for t in range(T):
        s = suites[t % 4]
        k = keys[t][:P.key_len(s) + P.salt_len(s)]
        run_thread(t, s, k, oracle_backend, want)
    b0, p0 = P.counter("pcbatches"), P.counter("pcpackets")
    f0 = P.counter("pcfused")
    ths = []
    for t in range(T):
        s = suites[t % 4]
        k = keys[t][:P.key_len(s) + P.salt_len(s)]
        ths.append(threading.Thread(target=run_thread,
                                    args=(t, s, k, dev_backend, got)))
    with P.tune(nofuse=0 if fuse else 1, pcrunners=runners, pchold=hold,
                pclinger=linger):
        for th in ths:
            th.start()
        for th in ths:
            th.join(120)
    assert len(got) == T
    for t in range(T):
        for i, (g, w) in enumerate(zip(got[t], want[t])):
            assert g[:3] == w[:3], (t, i)
            assert g[3][:len(w[3])] == w[3][:len(g[3])], (t, i)
    batches = P.counter("pcbatches") - b0
    packets = P.counter("pcpackets") - p0
    assert packets == sum(len(v) for v in got.values())
    assert batches <= packets
    fused = P.counter("pcfused") - f0
    if not fuse:
        assert fused == 0
    elif suites[2] == 3 and runners == 1:
        # 16 threads alternating protect and unprotect: some lists mix them
        assert fused > 0


def test_helper_thread_handoff_stress(torch_cuda):
    """The runners' helper threads (lists pc_run_fused rejects: nofuse=1)
    under many short alternating calls: a post of the runner between the
    helper's check and its futex wait once left the helper asleep on a word
    already posted, hanging every caller queued behind the slot.
    32 threads x 300 protect/unprotect pairs must all finish, every packet
    back to its plaintext."""
    T, N = 32, 300
    done, bad = [], []

    def worker(t):
        rng = np.random.default_rng(900 + t)
        key = bytes((7 * t + i) & 0xff for i in range(30))
        tx, rx = P.Srtp(1, key), P.Srtp(1, key)
        try:
            for k in range(N):
                pkt = rtp_packet(rng, (1000 + k) & 0xffff, 0x500 + t,
                                 plen=int(rng.integers(0, 200)))
                mb = P.new_mbuf(pkt, len(pkt) + 64)
                e1 = tx._op("srtp_encrypt", mb)
                m = mb.contents
                m.pos = 0
                e2 = rx._op("srtp_decrypt", mb)
                m = mb.contents
                out = P.mbuf_bytes(mb, m.end)
                P.free_mbuf(mb)
                if e1 or e2 or out != pkt:
                    bad.append((t, k, e1, e2))
                    return
            done.append(t)
        finally:
            tx.close()
            rx.close()

    ths = [threading.Thread(target=worker, args=(t,), daemon=True)
           for t in range(T)]
    with P.tune(nofuse=1, pcspin=1, pcrunners=4):
        for th in ths:
            th.start()
        for th in ths:
            th.join(90)
    assert not bad, bad[:4]
    assert sorted(done) == list(range(T)), "threads hung: %d of %d done" % (
        len(done), T)


def test_linger_sequence_and_other_streams(torch_cuda):
    """One thread's calls through the lingering small kernel (pclinger):
    exact against the oracle across its gaps (calls spaced past the linger
    time, so the kernel leaves and is launched again), a staging pool that
    grows under it (the kernel is stopped before the workspace's stream is
    synchronised), and a device batch on another stream right after a call
    (it runs while the kernel lingers, or behind it: at most the linger
    time on a shared hardware queue)."""
    import time
    torch = torch_cuda
    key = bytes(range(30))
    want = {}
    run_thread(0, 1, key, oracle_backend, want)
    got = {}
    with P.tune(pclinger=200):
        tx, rx = dev_backend(1, key)
        rng = np.random.default_rng(5)
        res, prot = [], {}
        for i, (op, arg) in enumerate(script(0)):
            if isinstance(arg, tuple):
                kind, j = arg
                data = bytearray(prot[j])
                if kind == "forge":
                    data[-1] ^= 1
                data = bytes(data)
            else:
                data = arg
            ctx = tx if op.endswith("encrypt") else rx
            e, po, en, b = ctx(op, data)
            prot[i] = b[:en] if op.endswith("encrypt") else None
            res.append((e, po, en, b[:max(en, len(data))]))
            if i % 37 == 5:
                time.sleep(0.002)       # past the linger: the kernel left
            if i == 50:
                # a device batch of another session right behind a call
                from tests.test_gpu_fastpath import run_dev
                pk = [rtp_packet(rng, k, 0x77, plen=100) for k in range(64)]
                arena = np.zeros(64 * 256, dtype=np.uint8)
                pos = np.arange(64, dtype=np.int64) * 256
                end = pos.copy()
                for k, q in enumerate(pk):
                    arena[k * 256:k * 256 + len(q)] = np.frombuffer(
                        q, dtype=np.uint8)
                    end[k] = k * 256 + len(q)
                s = P.Srtp(1, key)
                t0 = time.perf_counter()
                _, _, _, err = run_dev(torch, "srtp_encrypt", [s], arena,
                                       pos, end, pos + 256, None)
                assert time.perf_counter() - t0 < 0.5
                assert not err.any()
                s.close()
        got[0] = res
    for i, (g, w) in enumerate(zip(got[0], want[0])):
        assert g[:3] == w[:3], i
        assert g[3][:len(w[3])] == w[3][:len(g[3])], i
