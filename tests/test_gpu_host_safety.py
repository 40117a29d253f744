"""Host-side safety of the batch API (GPU, through the C-ABI library):

  * aliased sessions: a session array naming one context twice
    ({A, B, A}) must behave like the pointers it holds -- one stream, one
    state machine -- on every batch path (device arrays, host arrays), ROC
    wrap, replayed and forged packets included; checked against the
    oracle called one packet at a time;
  * concurrency: srtp_alloc_many on one thread (growing, i.e. moving, the
    device session table) while another thread runs batches must neither
    corrupt the batches nor the new sessions.
"""
import threading

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_fastpath import rtp_packet, to_arena

pytestmark = pytest.mark.gpu

KEY_A = bytes(range(30))
KEY_B = bytes(range(100, 130))


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    P.load()
    return torch


def oracle_seq(ob, ctxs, op, pkts):
    """sequential oracle calls: [(err, pos_rel, end_rel, bytes)]"""
    out = []
    for s, p in pkts:
        e, po, eo, so, buf = ob.call(ctxs[s], op, len(p) + 64, 0, len(p), p,
                                     len(p) + 16)
        out.append((e, po, eo, buf[:max(eo, len(p))]))
    return out


def product(torch, api, op, sessions, pkts):
    arena, pos, end, cap, sess = to_arena(pkts)
    dev = torch.from_numpy(arena).cuda()
    if api == "dev":
        i32 = lambda a: torch.from_numpy(a.astype(np.uint32).view(np.int32)
                                         ).cuda()
        p_d, e_d, c_d, s_d = i32(pos), i32(end), i32(cap), i32(sess)
        err_d = torch.full((len(pkts),), -1, dtype=torch.int32,
                           device="cuda")
        torch.cuda.synchronize()
        rc = P.device_batch_dev(op, sessions, dev.data_ptr(), dev.numel(),
                                p_d.data_ptr(), e_d.data_ptr(),
                                c_d.data_ptr(), err_d.data_ptr(), len(pkts),
                                s_d.data_ptr() if len(sessions) > 1
                                else None)
        assert rc == 0, (rc, P.lib().srtp_gpu_error())
        torch.cuda.synchronize()
        po = p_d.cpu().numpy().view(np.uint32)
        eo = e_d.cpu().numpy().view(np.uint32)
        err = err_d.cpu().numpy()
    else:
        po, eo = pos.copy(), end.copy()
        torch.cuda.synchronize()
        rc, err = P.device_batch(op, sessions, dev.data_ptr(), dev.numel(),
                                 po, eo, cap,
                                 sess if len(sessions) > 1 else None)
        assert rc == 0, (rc, P.lib().srtp_gpu_error())
    a = dev.cpu().numpy()
    res = []
    for i, (_, p) in enumerate(pkts):
        n = max(int(eo[i] - pos[i]), len(p))
        res.append((int(err[i]), int(po[i] - pos[i]), int(eo[i] - pos[i]),
                    a[pos[i]:pos[i] + n].tobytes()))
    return res


def alias_traffic(rng):
    """(sender packets, receive order) of streams A (via session index 0
    or 2) and B (index 1): ROC wrap, a replay and a forged packet"""
    seqs_a = [(65530 + k) & 0xffff for k in range(40)]
    seqs_b = [(1000 + k) for k in range(20)]
    pa = [rtp_packet(rng, q, 0xAAAA, plen=int(rng.integers(10, 300)))
          for q in seqs_a]
    pb = [rtp_packet(rng, q, 0xBBBB, plen=int(rng.integers(10, 300)))
          for q in seqs_b]
    order, ia, ib = [], 0, 0
    while ia < len(pa) or ib < len(pb):
        if ib >= len(pb) or (ia < len(pa) and rng.random() < 0.66):
            order.append(("A", ia, 0 if rng.random() < 0.5 else 2))
            ia += 1
        else:
            order.append(("B", ib, 1))
            ib += 1
    return pa, pb, order


@pytest.mark.parametrize("api", ["dev", "host"])
@pytest.mark.parametrize("suite", [1, 5])
def test_aliased_sessions(torch_cuda, api, suite):
    torch = torch_cuda
    rng = np.random.default_rng(99 + suite)
    klen = P.key_len(suite) + P.salt_len(suite)
    ka, kb = KEY_A[:klen] if klen <= 30 else (KEY_A * 2)[:klen], \
        KEY_B[:klen] if klen <= 30 else (KEY_B * 2)[:klen]
    pa, pb, order = alias_traffic(rng)
    ob = O.OracleBackend()

    # protect: sessv = {txA, txB, txA}
    send = [(k, pa[i] if s == "A" else pb[i]) for s, i, k in order]
    oa, _ = ob.alloc(suite, ka, 0)
    obb, _ = ob.alloc(suite, kb, 0)
    want = oracle_seq(ob, [oa, obb, oa], "srtp_encrypt", send)
    ta, tb = P.Srtp(suite, ka), P.Srtp(suite, kb)
    got = product(torch, api, "srtp_encrypt", [ta, tb, ta], send)
    assert got == want

    # unprotect the protected packets, plus a replay and a forgery
    recv = [(k, w[3][:w[2]]) for (k, _), w in zip(send, want)]
    dup = next(j for j, (s, _, _) in enumerate(order) if s == "A" and j > 10)
    recv.insert(len(recv) - 3, (2, recv[dup][1]))           # replay of A
    fj = next(j for j, (s, _, _) in enumerate(order) if s == "A" and j > 20)
    q = bytearray(recv[fj][1])
    q[-1] ^= 0x40
    recv[fj] = (recv[fj][0], bytes(q))                       # forged A
    ra, _ = ob.alloc(suite, ka, 0)
    rb, _ = ob.alloc(suite, kb, 0)
    want = oracle_seq(ob, [ra, rb, ra], "srtp_decrypt", recv)
    xa, xb = P.Srtp(suite, ka), P.Srtp(suite, kb)
    got = product(torch, api, "srtp_decrypt", [xa, xb, xa], recv)
    assert [g[0] for g in got] == [w[0] for w in want]
    assert got == want
    assert sum(1 for w in want if w[0] == P.EAUTH) == 1
    assert any(w[0] == 114 or w[0] == 215 for w in want)     # EALREADY
    for c in (ta, tb, xa, xb):
        c.close()
    for c in (oa, obb, ra, rb):
        ob.free(c)


def test_alloc_while_batching(torch_cuda):
    """the table grows (moves) under running batches of other sessions"""
    torch = torch_cuda
    rng = np.random.default_rng(7)
    pkts = [(0, rtp_packet(rng, 500 + k, 0x4242, plen=180))
            for k in range(4096)]
    ref = None
    errors = []
    stop = threading.Event()

    def batches():
        nonlocal ref
        try:
            it = 0
            while not stop.is_set() or it < 3:
                tx = P.Srtp(1, KEY_A)
                got = product(torch, "dev", "srtp_encrypt", [tx], pkts)
                tx.close()
                if ref is None:
                    ref = got
                elif got != ref:
                    errors.append("batch %d differs" % it)
                    return
                it += 1
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    t = threading.Thread(target=batches)
    t.start()
    keep = []
    try:
        for r in range(6):
            e, ss = P.alloc_many(40000, 1,
                                 bytes(rng.integers(0, 256, 40000 * 30,
                                                    dtype=np.uint8)))
            assert e == 0
            keep.append(ss)
    finally:
        stop.set()
        t.join(timeout=300)
    assert not errors, errors
    # a session created by the growing thread works like a fresh one
    ob = O.OracleBackend()
    key = bytes(range(30))
    e, ss = P.alloc_many(1, 1, key)
    want = oracle_seq(ob, [ob.alloc(1, key, 0)[0]], "srtp_encrypt", pkts[:64])
    assert product(torch, "dev", "srtp_encrypt", ss, pkts[:64]) == want
    # the first batch against the oracle
    want = oracle_seq(ob, [ob.alloc(1, KEY_A, 0)[0]], "srtp_encrypt", pkts)
    assert ref == want
    for ss in keep:
        for s in ss:
            s.close()
