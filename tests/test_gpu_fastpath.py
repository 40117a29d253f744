"""GPU parity of the compact descriptor path (srtp_*_batch fast path).

The fast path (re_amd/csrc/host/srtp.c run_fast) must give exactly the
results of the general engine (srtp_gpu_tune general), which the golden
replays pin to the reference, and of the oracle called one packet at a
time: same errno, pos/end, bytes and stream state.  Batches are adversarial:
CSRC/extension headers (mixed kernel classes), 9 SSRCs in one session
(ENOSR), seq jumps past 32768 (ETIMEDOUT), ROC wraps, reordering,
truncated packets (EBADMSG), short capacity (ENOMEM), replays (EALREADY)
and forged packets (EAUTH -> speculation miss -> undo + exact fold), with
tiny chunks so the host/GPU pipeline crosses many chunk boundaries.
"""
import errno

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def rtp_packet(rng, seq, ssrc, cc=0, x=False, plen=None):
    b = bytearray([0x80 | (0x10 if x else 0) | cc, 96,
                   (seq >> 8) & 0xff, seq & 0xff])
    b += int(rng.integers(0, 1 << 32)).to_bytes(4, "big")
    b += ssrc.to_bytes(4, "big")
    for _ in range(cc):
        b += int(rng.integers(0, 1 << 32)).to_bytes(4, "big")
    if x:
        xl = int(rng.integers(0, 4))
        b += b"\xbe\xde" + xl.to_bytes(2, "big")
        b += rng.integers(0, 256, 4 * xl, dtype=np.uint8).tobytes()
    if plen is None:
        plen = int(rng.integers(0, 300))
    b += rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
    return bytes(b)


def make_traffic(rng, n, nsess, enosr=True):
    """[(session, packet bytes)] with per-stream sequence evolution"""
    streams = {}
    out = []
    for _ in range(n):
        s = int(rng.integers(0, nsess))
        k = int(rng.integers(0, 9 if (enosr and s == 0) else 2))
        ssrc = 0x1000 * (s + 1) + k
        seq = streams.get(ssrc, int(rng.integers(0, 65536)))
        r = rng.random()
        if r < 0.80:
            seq = (seq + 1) & 0xffff
        elif r < 0.88:
            seq = (seq + int(rng.integers(2, 200))) & 0xffff
        elif r < 0.95:
            seq = (seq - int(rng.integers(1, 40))) & 0xffff
        elif r < 0.98:
            seq = (seq + int(rng.integers(32769, 40000))) & 0xffff
        else:
            seq = (seq + 65000) & 0xffff
        streams[ssrc] = seq
        cc = int(rng.integers(0, 4)) if rng.random() < 0.3 else 0
        x = rng.random() < 0.2
        pkt = rtp_packet(rng, seq, ssrc, cc, x)
        if rng.random() < 0.03:
            pkt = pkt[:int(rng.integers(0, len(pkt)))]
        out.append((s, pkt))
    return out


def to_arena(pkts, short_cap=()):
    """(arena, pos, end, cap, sess) with 4-aligned starts and tag room"""
    sizes = [len(p) + 80 for _, p in pkts]
    base, off = [], 0
    for sz in sizes:
        base.append(off)
        off += (sz + 15) & ~15
    arena = np.zeros(off, dtype=np.uint8)
    pos = np.zeros(len(pkts), dtype=np.uint32)
    end = np.zeros(len(pkts), dtype=np.uint32)
    cap = np.zeros(len(pkts), dtype=np.uint32)
    for i, (_, p) in enumerate(pkts):
        st = base[i] + 4 * (i % 3)
        arena[st:st + len(p)] = np.frombuffer(p, dtype=np.uint8)
        pos[i], end[i] = st, st + len(p)
        cap[i] = end[i] + (2 if i in short_cap else 60)
    sess = np.array([s for s, _ in pkts], dtype=np.uint32)
    return arena, pos, end, cap, sess


def run(torch, opname, sessions, arena, pos, end, cap, sess, general,
        chunk=None):
    with P.tune(general=1 if general else 0, chunk=chunk or 0):
        dev = torch.from_numpy(arena.copy()).cuda()
        p, e = pos.copy(), end.copy()
        torch.cuda.synchronize()
        rc, err = P.device_batch(opname, sessions, dev.data_ptr(),
                                 arena.nbytes, p, e, cap, sess)
        assert rc == 0, (rc, P.lib().srtp_gpu_error())
        return dev.cpu().numpy(), p, e, err


def states(sessions, ssrcs):
    out = []
    for s in sessions:
        for x in ssrcs:
            e, st = s.export(x)
            out.append((e,) if e else (st.roc, st.s_l, st.s_l_set,
                                       st.replay_rtp_bitmap,
                                       st.replay_rtp_lix))
    return out


def keys_for(suite, nsess):
    klen = P.key_len(suite) + P.salt_len(suite)
    return [bytes((7 * s + i) & 0xff for i in range(klen))
            for s in range(nsess)]


@pytest.mark.parametrize("suite", list(range(6)))
def test_fast_equals_general_and_oracle(suite, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(100 + suite)
    nsess, n = 3, 1500
    keys = keys_for(suite, nsess)
    pkts = make_traffic(rng, n, nsess)
    ssrcs = sorted({int.from_bytes(p[8:12], "big") for _, p in pkts
                    if len(p) >= 12})
    short = set()
    arena, pos, end, cap, sess = to_arena(pkts, short)

    txa = [P.Srtp(suite, k) for k in keys]
    txb = [P.Srtp(suite, k) for k in keys]
    ra = run(torch, "srtp_encrypt", txa, arena, pos, end, cap, sess, False,
             chunk=200)
    rb = run(torch, "srtp_encrypt", txb, arena, pos, end, cap, sess, True)
    assert (ra[3] == rb[3]).all() and (ra[1] == rb[1]).all() and \
        (ra[2] == rb[2]).all()
    assert (ra[0] == rb[0]).all()
    assert states(txa, ssrcs) == states(txb, ssrcs)
    errs = ra[3]
    assert (errs == 0).sum() > n // 2
    assert {int(e) for e in errs} >= {0}

    # oracle, one call at a time, on the packets with enough capacity
    be = O.OracleBackend()
    octx = [be.alloc(suite, k, 0)[0] for k in keys]
    for i, (s, p) in enumerate(pkts):
        if i in short:
            continue
        e, po, en, _, buf = be.call(octx[s], "srtp_encrypt", len(p) + 64, 0,
                                    len(p), p, len(p) + 16)
        got = (int(errs[i]), int(ra[1][i] - pos[i]), int(ra[2][i] - pos[i]))
        assert got == (e, po, en), (i, got, (e, po, en))
        if e == 0:
            assert ra[0][pos[i]:ra[2][i]].tobytes() == buf[:en], i
    for c in octx:
        be.free(c)

    # receive: protected packets, plus replays and forgeries
    prot = []
    for i, (s, _) in enumerate(pkts):
        if errs[i] == 0:
            prot.append((s, ra[0][pos[i]:ra[2][i]].tobytes()))
    rx_pkts = []
    for k, (s, p) in enumerate(prot):
        rx_pkts.append((s, p))
        r = rng.random()
        if r < 0.03:
            rx_pkts.append(prot[int(rng.integers(0, k + 1))])
        elif r < 0.05:
            q = bytearray(p)
            q[int(rng.integers(12, len(q)))] ^= 0x40
            rx_pkts.append((s, bytes(q)))
    arena2, pos2, end2, cap2, sess2 = to_arena(rx_pkts)
    rxa = [P.Srtp(suite, k) for k in keys]
    rxb = [P.Srtp(suite, k) for k in keys]
    da = run(torch, "srtp_decrypt", rxa, arena2, pos2, end2, cap2, sess2,
             False, chunk=128)
    db = run(torch, "srtp_decrypt", rxb, arena2, pos2, end2, cap2, sess2,
             True)
    assert (da[3] == db[3]).all(), np.flatnonzero(da[3] != db[3])[:10]
    assert (da[1] == db[1]).all() and (da[2] == db[2]).all()
    assert (da[0] == db[0]).all()
    assert states(rxa, ssrcs) == states(rxb, ssrcs)
    codes = {int(e) for e in da[3]}
    assert {0, P.EAUTH, errno.EALREADY} <= codes, codes

    # and against the oracle receiver
    octx = [be.alloc(suite, k, 0)[0] for k in keys]
    for i, (s, p) in enumerate(rx_pkts):
        e, po, en, _, buf = be.call(octx[s], "srtp_decrypt", len(p) + 64, 0,
                                    len(p), p, len(p))
        got = (int(da[3][i]), int(da[1][i] - pos2[i]),
               int(da[2][i] - pos2[i]))
        assert got == (e, po, en), (i, got, (e, po, en))
        assert da[0][pos2[i]:pos2[i] + len(buf)].tobytes() == buf, i
    for c in octx:
        be.free(c)
    for c in txa + txb + rxa + rxb:
        c.close()


def test_fast_all_forged_single_chunk(torch_cuda):
    """every packet forged: one speculation miss per packet, one undo"""
    torch = torch_cuda
    suite = 1
    key = keys_for(suite, 1)[0]
    rng = np.random.default_rng(5)
    pkts = [(0, rtp_packet(rng, (65530 + i) & 0xffff, 0x42, plen=200))
            for i in range(300)]
    arena, pos, end, cap, sess = to_arena(pkts)
    tx = P.Srtp(suite, key)
    enc = run(torch, "srtp_encrypt", [tx], arena, pos, end, cap, None, False)
    assert not enc[3].any()
    forged = []
    for i in range(300):
        q = bytearray(enc[0][pos[i]:enc[2][i]].tobytes())
        q[-1] ^= 1
        forged.append((0, bytes(q)))
    a2, p2, e2, c2, _ = to_arena(forged)
    rxa, rxb = P.Srtp(suite, key), P.Srtp(suite, key)
    da = run(torch, "srtp_decrypt", [rxa], a2, p2, e2, c2, None, False)
    db = run(torch, "srtp_decrypt", [rxb], a2, p2, e2, c2, None, True)
    assert (da[3] == P.EAUTH).all()
    for x, y in zip(da, db):
        assert (x == y).all()
    assert states([rxa], [0x42]) == states([rxb], [0x42])


@pytest.mark.parametrize("suite", [1, 5])
def test_fast_short_capacity(suite, torch_cuda):
    """device arenas cannot grow: ENOMEM, identical in both engines"""
    torch = torch_cuda
    rng = np.random.default_rng(33 + suite)
    keys = keys_for(suite, 2)
    pkts = make_traffic(rng, 400, 2, enosr=False)
    short = set(rng.choice(400, 40, replace=False).tolist())
    arena, pos, end, cap, sess = to_arena(pkts, short)
    ssrcs = sorted({int.from_bytes(p[8:12], "big") for _, p in pkts
                    if len(p) >= 12})
    txa = [P.Srtp(suite, k) for k in keys]
    txb = [P.Srtp(suite, k) for k in keys]
    ra = run(torch, "srtp_encrypt", txa, arena, pos, end, cap, sess, False,
             chunk=64)
    rb = run(torch, "srtp_encrypt", txb, arena, pos, end, cap, sess, True)
    assert errno.ENOMEM in {int(e) for e in ra[3]}
    for x, y in zip(ra, rb):
        assert (x == y).all()
    assert states(txa, ssrcs) == states(txb, ssrcs)


def seq_batch(rng, seqs, ssrc=0x5151, plen=160, csrc_at=()):
    return [(0, rtp_packet(rng, s & 0xffff, ssrc, cc=1 if i in csrc_at else 0,
                           plen=plen)) for i, s in enumerate(seqs)]


@pytest.mark.parametrize("suite", [1, 5])
def test_device_planner_and_its_fallbacks(suite, torch_cuda):
    """Single-stream batches take the device planner; every broken
    speculation (reorder, replay, ETIMEDOUT, mixed header classes, second
    SSRC) must fall back with identical results.  Compared against the
    host-planned fast path (srtp_gpu_tune noplan) and the general engine, with
    state carried across consecutive batches."""
    torch = torch_cuda
    rng = np.random.default_rng(77 + suite)
    key = keys_for(suite, 1)[0]
    base = list(range(65000, 65000 + 3000))            # ROC wrap inside
    cases = {
        "inorder": (base, ()),
        "reorder": (base[:700] + [base[701], base[700]] + base[702:], ()),
        "classes": (base, (5, 900)),
        "jump": (base[:1000] + [base[999] + 40000] + base[1000:], ()),
        "dup": (base[:1500] + [base[1200]] + base[1500:], ()),
    }
    for name, (seqs, csrc_at) in cases.items():
        pkts = seq_batch(rng, seqs, csrc_at=csrc_at)
        if name == "dup":
            pkts[1500] = pkts[1200]
        arena, pos, end, cap, _ = to_arena(pkts)
        half = len(pkts) // 2
        parts = [(0, half), (half, len(pkts))]
        res = {}
        for mode in ("plan", "noplan", "general"):
            tx, rx = P.Srtp(suite, key), P.Srtp(suite, key)
            outs = []
            for a, b in parts:
                P.lib().srtp_gpu_tune(b"noplan", 0)
                if mode == "noplan":
                    P.lib().srtp_gpu_tune(b"noplan", 1)
                sl = slice(a, b)
                enc = run(torch, "srtp_encrypt", [tx], arena, pos[sl],
                          end[sl], cap[sl], None, mode == "general")
                P.lib().srtp_gpu_tune(b"noplan", 0)
                outs.append(enc)
            # receive what was sent (protected windows), same split
            prot = []
            for (a, b), enc in zip(parts, outs):
                for j in range(b - a):
                    i = a + j
                    if enc[3][j] == 0:
                        prot.append((0, enc[0][pos[i]:enc[2][j]].tobytes()))
            a2, p2, e2, c2, _ = to_arena(prot)
            h = len(prot) // 2
            douts = []
            for a, b in ((0, h), (h, len(prot))):
                if mode == "noplan":
                    P.lib().srtp_gpu_tune(b"noplan", 1)
                sl = slice(a, b)
                douts.append(run(torch, "srtp_decrypt", [rx], a2, p2[sl],
                                 e2[sl], c2[sl], None, mode == "general"))
                P.lib().srtp_gpu_tune(b"noplan", 0)
            res[mode] = (outs, douts, states([tx], [0x5151]),
                         states([rx], [0x5151]))
            tx.close()
            rx.close()
        for mode in ("noplan", "general"):
            A, B = res["plan"], res[mode]
            for x, y in zip(A[0] + A[1], B[0] + B[1]):
                for u, v in zip(x, y):
                    assert (u == v).all(), (name, mode)
            assert A[2] == B[2] and A[3] == B[3], (name, mode)


def run_dev(torch, opname, sessions, arena, pos, end, cap, sess):
    """srtp_*_batch_dev with every per-packet array in HBM"""
    dev = torch.from_numpy(arena.copy()).cuda()
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).cuda()
    p = t(pos.astype(np.int64), np.int64).to(torch.int32)
    e = t(end.astype(np.int64), np.int64).to(torch.int32)
    c = t(cap.astype(np.int64), np.int64).to(torch.int32)
    er = torch.full((len(pos),), -1, dtype=torch.int32, device="cuda")
    s = t(sess.astype(np.int64), np.int64).to(torch.int32) \
        if sess is not None else None
    torch.cuda.synchronize()
    rc = P.device_batch_dev(opname, sessions, dev.data_ptr(), arena.nbytes,
                            p.data_ptr(), e.data_ptr(), c.data_ptr(),
                            er.data_ptr(), len(pos),
                            s.data_ptr() if s is not None else None)
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    u32 = lambda x: x.cpu().numpy().view(np.uint32)
    return dev.cpu().numpy(), u32(p), u32(e), er.cpu().numpy()


@pytest.mark.parametrize("suite", [1, 4])
def test_device_resident_api(suite, torch_cuda):
    """srtp_*_batch_dev == srtp_*_batch: planned single stream, forged
    packet (undo + fold), multi-session (staged), SRTCP (staged)"""
    torch = torch_cuda
    rng = np.random.default_rng(9 + suite)
    key = keys_for(suite, 1)[0]
    seqs = list(range(65300, 65300 + 2000))
    pkts = seq_batch(rng, seqs)
    arena, pos, end, cap, _ = to_arena(pkts)
    txa, txb = P.Srtp(suite, key), P.Srtp(suite, key)
    a = run_dev(torch, "srtp_encrypt", [txa], arena, pos, end, cap, None)
    b = run(torch, "srtp_encrypt", [txb], arena, pos, end, cap, None, False)
    for x, y in zip(a, b):
        assert (x == y).all()
    assert states([txa], [0x5151]) == states([txb], [0x5151])
    # receive with one forged packet
    prot = [(0, a[0][pos[i]:a[2][i]].tobytes()) for i in range(len(pkts))]
    q = bytearray(prot[700][1])
    q[40] ^= 1
    prot[700] = (0, bytes(q))
    a2, p2, e2, c2, _ = to_arena(prot)
    rxa, rxb = P.Srtp(suite, key), P.Srtp(suite, key)
    da = run_dev(torch, "srtp_decrypt", [rxa], a2, p2, e2, c2, None)
    db = run(torch, "srtp_decrypt", [rxb], a2, p2, e2, c2, None, True)
    for x, y in zip(da, db):
        assert (x == y).all()
    assert da[3][700] == P.EAUTH and (np.delete(da[3], 700) == 0).all()
    assert states([rxa], [0x5151]) == states([rxb], [0x5151])
    # multi-session: staged through the host engine
    keys = keys_for(suite, 3)
    mp = make_traffic(rng, 600, 3, enosr=False)
    ma, mpos, mend, mcap, msess = to_arena(mp)
    sa = [P.Srtp(suite, k) for k in keys]
    sb = [P.Srtp(suite, k) for k in keys]
    x = run_dev(torch, "srtp_encrypt", sa, ma, mpos, mend, mcap, msess)
    y = run(torch, "srtp_encrypt", sb, ma, mpos, mend, mcap, msess, True)
    for u, v in zip(x, y):
        assert (u == v).all()
    for c in [txa, txb, rxa, rxb] + sa + sb:
        c.close()


def multi_session_traffic(rng, n, nsess, s0=None, forge=()):
    """in-order traffic of nsess sessions, one SSRC each, interleaved at
    random (the multi-session device planner's case)"""
    nxt = {}
    out = []
    for _ in range(n):
        s = int(rng.integers(0, nsess))
        seq = nxt.get(s, (s0 if s0 is not None else
                          int(rng.integers(0, 65536))))
        nxt[s] = (seq + 1) & 0xffff
        out.append((s, rtp_packet(rng, seq, 0x7000 + s,
                                  plen=int(rng.integers(0, 400)))))
    return out


@pytest.mark.parametrize("suite", [1, 5])
def test_multi_session_device_planner(suite, torch_cuda):
    """many sessions, one SSRC each: planned on the device (sort by
    session + per-session speculation); must equal the host scan
    (srtp_gpu_tune noplan) and the general engine, across two consecutive
    batches, with a forged packet forcing undo + exact fold"""
    torch = torch_cuda
    rng = np.random.default_rng(55 + suite)
    nsess = 40
    keys = keys_for(suite, nsess)
    ssrcs = [0x7000 + s for s in range(nsess)]
    batches = [multi_session_traffic(rng, 2500, nsess, s0=65400)]
    # second batch continues every session (ROC wraps inside)
    last = {}
    for s, p in batches[0]:
        last[s] = int.from_bytes(p[2:4], "big")
    nb = []
    for _ in range(2500):
        s = int(rng.integers(0, nsess))
        last[s] = (last.get(s, 0) + 1) & 0xffff
        nb.append((s, rtp_packet(rng, last[s], 0x7000 + s, plen=120)))
    batches.append(nb)
    res = {}
    for mode in ("plan", "noplan", "general"):
        tx = [P.Srtp(suite, k) for k in keys]
        rx = [P.Srtp(suite, k) for k in keys]
        outs = []
        for bi, pk in enumerate(batches):
            arena, pos, end, cap, sess = to_arena(pk)
            if mode == "noplan":
                P.lib().srtp_gpu_tune(b"noplan", 1)
            enc = run(torch, "srtp_encrypt", tx, arena, pos, end, cap, sess,
                      mode == "general")
            P.lib().srtp_gpu_tune(b"noplan", 0)
            prot = [(s, enc[0][pos[i]:enc[2][i]].tobytes())
                    for i, (s, _) in enumerate(pk)]
            if bi == 1:
                q = bytearray(prot[1234][1])
                q[-3] ^= 0x10
                prot[1234] = (prot[1234][0], bytes(q))
            a2, p2, e2, c2, s2 = to_arena(prot)
            if mode == "noplan":
                P.lib().srtp_gpu_tune(b"noplan", 1)
            dec = run(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2,
                      mode == "general")
            P.lib().srtp_gpu_tune(b"noplan", 0)
            outs.append((enc, dec))
        res[mode] = (outs, states(tx, ssrcs), states(rx, ssrcs))
        for c in tx + rx:
            c.close()
    A = res["plan"]
    assert int(A[0][1][1][3][1234]) == P.EAUTH
    for mode in ("noplan", "general"):
        B = res[mode]
        for (ea, da), (eb, db) in zip(A[0], B[0]):
            for x, y in zip(ea + da, eb + db):
                assert (x == y).all(), mode
        assert A[1] == B[1] and A[2] == B[2], mode


@pytest.mark.parametrize("suite", list(range(6)))
@pytest.mark.parametrize("cc", [0, 1, 3])
def test_every_length_single_session(suite, cc, torch_cuda):
    """one session, one header class, every payload length 0..260: the
    single-key kernels' head/steady/tail chunk split and partial last
    words (k_ctr_hmac UNI, k_gcmu) against the oracle, both directions"""
    torch = torch_cuda
    rng = np.random.default_rng(900 + 10 * suite + cc)
    key = keys_for(suite, 1)[0]
    pkts = [(0, rtp_packet(rng, (65500 + i) & 0xffff, 0x2468, cc=cc,
                           plen=plen)) for i, plen in enumerate(range(261))]
    arena, pos, end, cap, _ = to_arena(pkts)
    tx = P.Srtp(suite, key)
    enc = run(torch, "srtp_encrypt", [tx], arena, pos, end, cap, None, False)
    be = O.OracleBackend()
    octx = be.alloc(suite, key, 0)[0]
    prot = []
    for i, (_, p) in enumerate(pkts):
        e, po, en, _, buf = be.call(octx, "srtp_encrypt", len(p) + 64, 0,
                                    len(p), p, len(p) + 16)
        assert (int(enc[3][i]), int(enc[1][i] - pos[i]),
                int(enc[2][i] - pos[i])) == (e, po, en), i
        assert enc[0][pos[i]:enc[2][i]].tobytes() == buf[:en], (i, len(p))
        prot.append((0, bytes(buf[:en])))
    be.free(octx)
    a2, p2, e2, c2, _ = to_arena(prot)
    rx = P.Srtp(suite, key)
    dec = run(torch, "srtp_decrypt", [rx], a2, p2, e2, c2, None, False)
    assert not dec[3].any(), np.flatnonzero(dec[3])[:8]
    # whole buffer vs the oracle receiver: plaintext, and the tag bytes
    # (the HMAC suites leave the ROC over them, srtp.c:342-344)
    octx = be.alloc(suite, key, 0)[0]
    for i, (_, q) in enumerate(prot):
        e, po, en, _, buf = be.call(octx, "srtp_decrypt", len(q) + 64, 0,
                                    len(q), q, len(q))
        assert e == 0 and dec[0][p2[i]:dec[2][i]].tobytes() == pkts[i][1]
        assert dec[0][p2[i]:p2[i] + len(buf)].tobytes() == buf, (i, len(q))
    be.free(octx)
    tx.close()
    rx.close()


@pytest.mark.parametrize("suite", [1, 5])
def test_device_resident_multi_session(suite, torch_cuda):
    """srtp_*_batch_dev with a session array (multi-session device plan,
    every array in HBM) == srtp_*_batch (host arrays) == general engine,
    over two consecutive batches; a forged packet forces undo + fold"""
    torch = torch_cuda
    rng = np.random.default_rng(77 + suite)
    nsess = 50
    keys = keys_for(suite, nsess)
    ssrcs = [0x7000 + s for s in range(nsess)]
    batches = [multi_session_traffic(rng, 1500, nsess, s0=65500)]
    last = {}
    for s, p in batches[0]:
        last[s] = int.from_bytes(p[2:4], "big")
    nb = []
    for _ in range(1500):   # continues every session (ROC wraps inside)
        s = int(rng.integers(0, nsess))
        last[s] = (last.get(s, 0) + 1) & 0xffff
        nb.append((s, rtp_packet(rng, last[s], 0x7000 + s,
                                 plen=int(rng.integers(0, 400)))))
    batches.append(nb)
    res = {}
    # dev_par: the session gather/apply passes split over the host pool
    # (par_min 4 -> parts of >= 4 sessions)
    for mode in ("dev", "dev_par", "host", "general"):
        tx = [P.Srtp(suite, k) for k in keys]
        rx = [P.Srtp(suite, k) for k in keys]
        outs = []
        if mode == "dev_par":
            P.lib().srtp_gpu_tune(b"par_min", 4)
        for bi, pk in enumerate(batches):
            arena, pos, end, cap, sess = to_arena(pk)
            if mode.startswith("dev"):
                enc = run_dev(torch, "srtp_encrypt", tx, arena, pos, end,
                              cap, sess)
            else:
                enc = run(torch, "srtp_encrypt", tx, arena, pos, end, cap,
                          sess, mode == "general")
            prot = [(s, enc[0][pos[i]:enc[2][i]].tobytes())
                    for i, (s, _) in enumerate(pk)]
            if bi == 1:
                q = bytearray(prot[321][1])
                q[-2] ^= 0x08
                prot[321] = (prot[321][0], bytes(q))
            a2, p2, e2, c2, s2 = to_arena(prot)
            if mode.startswith("dev"):
                dec = run_dev(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2)
            else:
                dec = run(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2,
                          mode == "general")
            outs.append((enc, dec))
        P.lib().srtp_gpu_tune(b"par_min", 0)
        res[mode] = (outs, states(tx, ssrcs), states(rx, ssrcs))
        for c in tx + rx:
            c.close()
    A = res["dev"]
    assert int(A[0][1][1][3][321]) == P.EAUTH
    for mode in ("dev_par", "host", "general"):
        B = res[mode]
        for (ea, da), (eb, db) in zip(A[0], B[0]):
            for x, y in zip(ea + da, eb + db):
                assert (x == y).all(), mode
        assert A[1] == B[1] and A[2] == B[2], mode


@pytest.mark.parametrize("suite", [1, 2, 5])
@pytest.mark.parametrize("big", [False, True])
def test_cached_size_boundary(suite, big, torch_cuda):
    """packets either side of the compact kernels' size bound
    (SGPU_CACHED_MAX_CTR = 4032 B: AES-CM caches rounds 1-2 only while the
    keystream block index stays < 256, kern_common.h CTR_B15).  big=False:
    every packet just under the bound, so the whole batch takes the
    device-planned compact kernels; big=True: packets up to 9000 B, so the
    batch goes to the plain kernels.  Device-resident and host-array APIs
    against the oracle, both directions."""
    torch = torch_cuda
    rng = np.random.default_rng(1300 + suite + 7 * big)
    key = keys_for(suite, 1)[0]
    lens = ([4031 - 12, 4030 - 12, 3800, 4000 - 12, 4016 - 12] if not big
            else [4032 - 12, 4033 - 12, 4095 - 12, 4096 - 12, 4100, 9000])
    pkts = [(0, rtp_packet(rng, (65530 + i) & 0xffff, 0x4242,
                           plen=lens[i % len(lens)])) for i in range(24)]
    arena, pos, end, cap, _ = to_arena(pkts)
    txa, txb = P.Srtp(suite, key), P.Srtp(suite, key)
    a = run_dev(torch, "srtp_encrypt", [txa], arena, pos, end, cap, None)
    b = run(torch, "srtp_encrypt", [txb], arena, pos, end, cap, None, False)
    for x, y in zip(a, b):
        assert (x == y).all()
    be = O.OracleBackend()
    octx = be.alloc(suite, key, 0)[0]
    prot = []
    for i, (_, p) in enumerate(pkts):
        e, po, en, _, buf = be.call(octx, "srtp_encrypt", len(p) + 64, 0,
                                    len(p), p, len(p) + 16)
        assert (int(a[3][i]), int(a[2][i] - pos[i])) == (e, en), i
        assert a[0][pos[i]:a[2][i]].tobytes() == buf[:en], (i, len(p))
        prot.append((0, bytes(buf[:en])))
    be.free(octx)
    a2, p2, e2, c2, _ = to_arena(prot)
    rxa, rxb = P.Srtp(suite, key), P.Srtp(suite, key)
    da = run_dev(torch, "srtp_decrypt", [rxa], a2, p2, e2, c2, None)
    db = run(torch, "srtp_decrypt", [rxb], a2, p2, e2, c2, None, False)
    for x, y in zip(da, db):
        assert (x == y).all()
    assert not da[3].any()
    for i in range(len(pkts)):
        assert da[0][p2[i]:da[2][i]].tobytes() == pkts[i][1], i
    for c in (txa, txb, rxa, rxb):
        c.close()


@pytest.mark.parametrize("suite", [1, 5])
@pytest.mark.parametrize("shape", ["skewed", "few_sessions", "bad_session"])
def test_multi_session_shapes(suite, shape, torch_cuda):
    """multi-session device plan (plan_multi.hip) over session shapes:
    one session far longer than the rest (skewed), few long sessions
    (few_sessions) -- srtp_*_batch_dev results and final stream states
    equal the general engine's -- and an out-of-range session index
    (bad_session: the device plan fails with every sort key clamped in
    bounds, the staged path rejects the call with EINVAL)"""
    torch = torch_cuda
    rng = np.random.default_rng(1234 + suite)
    nsess = {"skewed": 64, "few_sessions": 3, "bad_session": 40}[shape]
    n = {"skewed": 3000, "few_sessions": 1500, "bad_session": 800}[shape]
    keys = keys_for(suite, nsess)
    ssrcs = [0x7000 + s for s in range(nsess)]
    pk = multi_session_traffic(rng, n, nsess, s0=65300)
    if shape == "skewed":     # session 5 gets 400 extra packets
        for j in range(400):
            pk.insert(int(rng.integers(0, len(pk))),
                      (5, None))
        out, seqs = [], {}
        for s, p in pk:       # renumber every session in array order
            q = seqs.get(s, 65300)
            seqs[s] = (q + 1) & 0xffff
            out.append((s, rtp_packet(rng, q, 0x7000 + s,
                                      plen=int(rng.integers(0, 300)))))
        pk = out
    if shape == "bad_session":
        # the device plan fails (SPF_BAD, every key clamped so the plan's
        # reads stay in bounds) and the staged path rejects the call
        # with EINVAL before touching any state -- for both sorts
        for _ in range(2):
            tx = [P.Srtp(suite, k) for k in keys]
            arena, pos, end, cap, sess = to_arena(pk)
            sess = sess.copy()
            sess[17] = nsess + 3
            dev = torch.from_numpy(arena.copy()).cuda()
            i32 = lambda a: torch.from_numpy(
                np.asarray(a, dtype=np.uint32).view(np.int32)).cuda()
            p, e, c, sd = i32(pos), i32(end), i32(cap), i32(sess)
            er = torch.full((len(pos),), -1, dtype=torch.int32,
                            device="cuda")
            torch.cuda.synchronize()
            rc = P.device_batch_dev("srtp_encrypt", tx, dev.data_ptr(),
                                    arena.nbytes, p.data_ptr(),
                                    e.data_ptr(), c.data_ptr(),
                                    er.data_ptr(), len(pos), sd.data_ptr())
            torch.cuda.synchronize()
            assert rc == errno.EINVAL, rc
            assert (dev.cpu().numpy() == arena).all()
            # no stream was created (export fails for every SSRC)
            assert all(len(x) == 1 for x in states(tx, ssrcs))
            for t in tx:
                t.close()
        return
    res = {}
    for mode in ("dev", "general"):
        tx = [P.Srtp(suite, k) for k in keys]
        rx = [P.Srtp(suite, k) for k in keys]
        arena, pos, end, cap, sess = to_arena(pk)
        if mode == "general":
            enc = run(torch, "srtp_encrypt", tx, arena, pos, end, cap,
                      sess, True)
        else:
            enc = run_dev(torch, "srtp_encrypt", tx, arena, pos, end, cap,
                          sess)
        prot = [(s, enc[0][pos[i]:enc[2][i]].tobytes())
                for i, (s, _) in enumerate(pk)]
        a2, p2, e2, c2, s2 = to_arena(prot)
        if mode == "general":
            dec = run(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2, True)
        else:
            dec = run_dev(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2)
        assert not dec[3].any()
        res[mode] = ((enc, dec), states(tx, ssrcs), states(rx, ssrcs))
        for c in tx + rx:
            c.close()
    A = res["general"]
    for mode in ("dev",):
        B = res[mode]
        for x, y in zip(A[0][0] + A[0][1], B[0][0] + B[0][1]):
            assert (x == y).all(), mode
        assert A[1] == B[1] and A[2] == B[2], mode


def next_batch(rng, last, n, nsess, plen=None):
    """continue every session's sequence (ROC wraps inside)"""
    out = []
    for _ in range(n):
        s = int(rng.integers(0, nsess))
        last[s] = (last.get(s, 0) + 1) & 0xffff
        out.append((s, rtp_packet(rng, last[s], 0x7000 + s,
                                  plen=int(rng.integers(0, 300))
                                  if plen is None else plen)))
    return out


@pytest.mark.parametrize("suite", [1, 4])
def test_resident_state_across_paths(suite, torch_cuda):
    """Multi-session device batches keep stream states in HBM across calls
    (sgpu_sst_*); any host-side path reads them back first.  Sessions
    driven through: device multi-session batch, per-packet srtp_encrypt /
    srtp_decrypt on some sessions, another device batch, export + import
    of one session, a host-array batch, a device batch, a forged packet in
    a device batch, and again a device batch -- against twin sessions
    driven only by the general engine (golden-pinned)."""
    torch = torch_cuda
    rng = np.random.default_rng(4242 + suite)
    nsess = 24
    keys = keys_for(suite, nsess)
    ssrcs = [0x7000 + s for s in range(nsess)]
    last = {s: 65400 + 7 * s for s in range(nsess)}
    plan = [("dev", next_batch(rng, last, 900, nsess)),
            ("one", next_batch(rng, last, 40, 5)),
            ("dev", next_batch(rng, last, 900, nsess)),
            ("xport", None),
            ("host", next_batch(rng, last, 600, nsess)),
            ("dev", next_batch(rng, last, 900, nsess)),
            ("forge", next_batch(rng, last, 900, nsess)),
            ("dev", next_batch(rng, last, 900, nsess))]
    res = {}
    for mode in ("resident", "general"):
        tx = [P.Srtp(suite, k) for k in keys]
        rx = [P.Srtp(suite, k) for k in keys]
        outs = []
        for kind, pk in plan:
            if kind == "xport":
                for ctx in (tx[3], rx[3]):
                    e, st = ctx.export(0x7000 + 3)
                    assert e == 0
                    assert ctx.import_(st) == 0
                continue
            if kind == "one":
                for s, p in pk:
                    mb = P.new_mbuf(p, len(p) + 64)
                    e1 = tx[s].encrypt(mb)
                    q = P.mbuf_bytes(mb)
                    P.free_mbuf(mb)
                    mb = P.new_mbuf(q, len(q) + 64)
                    e2 = rx[s].decrypt(mb)
                    outs.append((e1, q, e2, P.mbuf_bytes(mb)))
                    P.free_mbuf(mb)
                continue
            arena, pos, end, cap, sess = to_arena(pk)
            dev = mode == "resident" and kind != "host"
            if dev:
                enc = run_dev(torch, "srtp_encrypt", tx, arena, pos, end,
                              cap, sess)
            else:
                enc = run(torch, "srtp_encrypt", tx, arena, pos, end, cap,
                          sess, mode == "general")
            prot = [(s, enc[0][pos[i]:enc[2][i]].tobytes())
                    for i, (s, _) in enumerate(pk)]
            if kind == "forge":
                q = bytearray(prot[77][1])
                q[-1] ^= 0x01
                prot[77] = (prot[77][0], bytes(q))
            a2, p2, e2, c2, s2 = to_arena(prot)
            if dev:
                dec = run_dev(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2)
            else:
                dec = run(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2,
                          mode == "general")
            outs.append((enc, dec))
        res[mode] = (outs, states(tx, ssrcs), states(rx, ssrcs))
        for c in tx + rx:
            c.close()
    A, B = res["resident"], res["general"]
    for x, y in zip(A[0], B[0]):
        if isinstance(x[0], int):
            assert x == y
            continue
        for u, v in zip(x[0] + x[1], y[0] + y[1]):
            assert (u == v).all()
    assert A[1] == B[1] and A[2] == B[2]


def hot_session_traffic(rng, n, nsess, hot, s0=65000):
    """multi-session traffic where session 0 carries `hot` of the n
    packets (in order per session, interleaved at random)"""
    owner = np.concatenate([np.zeros(hot, dtype=np.int64),
                            rng.integers(1, nsess, n - hot)])
    rng.shuffle(owner)
    nxt, out = {}, []
    for s in owner.tolist():
        seq = nxt.get(s, s0)
        nxt[s] = (seq + 1) & 0xffff
        out.append((s, rtp_packet(rng, seq, 0x7000 + s,
                                  plen=int(rng.integers(0, 300)))))
    return out


@pytest.mark.parametrize("suite", [1, 5])
def test_multi_session_counting_grouping(suite, torch_cuda):
    """the multi-session planner groups packets by session with a counting
    pass (stable rank among a session's packets); a session with more than
    SGPU_MP_SEGMAX (1024) packets rejects that grouping (SPF_SEG) and the
    call is re-planned with the radix sort.  Both must equal the radix-sort
    grouping (srtp_gpu_tune mpradix) and the general engine, protect and
    unprotect, with a forged packet in the hot session"""
    torch = torch_cuda
    rng = np.random.default_rng(404 + suite)
    nsess = 12
    keys = keys_for(suite, nsess)
    ssrcs = [0x7000 + s for s in range(nsess)]
    batches = [hot_session_traffic(rng, 3000, nsess, 1500),   # SPF_SEG
               hot_session_traffic(rng, 3000, nsess, 900, s0=2000)]
    res = {}
    for mode in ("count", "radix", "general"):
        if mode == "radix":
            P.lib().srtp_gpu_tune(b"mpradix", 1)
        tx = [P.Srtp(suite, k) for k in keys]
        rx = [P.Srtp(suite, k) for k in keys]
        outs, rej = [], []
        for bi, pk in enumerate(batches):
            r0 = P.counter("rejects")
            arena, pos, end, cap, sess = to_arena(pk)
            if mode == "general":
                enc = run(torch, "srtp_encrypt", tx, arena, pos, end, cap,
                          sess, True)
            else:
                enc = run_dev(torch, "srtp_encrypt", tx, arena, pos, end,
                              cap, sess)
            prot = [(s, enc[0][pos[i]:enc[2][i]].tobytes())
                    for i, (s, _) in enumerate(pk)]
            hot = next(i for i, (s, _) in enumerate(pk) if s == 0 and i > 700)
            q = bytearray(prot[hot][1])
            q[-1] ^= 0x04
            prot[hot] = (prot[hot][0], bytes(q))
            a2, p2, e2, c2, s2 = to_arena(prot)
            if mode == "general":
                dec = run(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2,
                          True)
            else:
                dec = run_dev(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2)
            assert int(dec[3][hot]) == P.EAUTH
            outs.append((enc, dec))
            rej.append(P.counter("rejects") - r0)
        P.lib().srtp_gpu_tune(b"mpradix", 0)
        res[mode] = (outs, states(tx, ssrcs), states(rx, ssrcs), rej)
        for c in tx + rx:
            c.close()
    # the hot batch re-planned (one reject per direction), the other not
    assert res["count"][3][0] == 2 and res["count"][3][1] == 0
    assert res["radix"][3] == [0, 0]
    A = res["count"]
    for mode in ("radix", "general"):
        B = res[mode]
        for (ea, da), (eb, db) in zip(A[0], B[0]):
            for x, y in zip(ea + da, eb + db):
                assert (x == y).all(), mode
        assert A[1] == B[1] and A[2] == B[2], mode
