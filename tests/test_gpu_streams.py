"""GPU parity of the per-stream device planner (re_amd/csrc/hip/
plan_streams.hip): one session (struct srtp) carrying several SSRCs through
srtp_*_batch_dev.

The reference finds or creates the stream by SSRC for every packet
(stream_get_seq, /root/reference/src/srtp/stream.c:87-109; at most 8
streams, stream.c:16-17,50-51 -> ENOSR) and runs each stream's ROC / s_l /
replay state machine on its own (srtp.c:203-215, 279-280, 310-321,
426-427).  The planner must give exactly the results of the general engine
(srtp_gpu_tune general, pinned to the reference by the golden replays) and
of the oracle called one packet at a time: errno, pos/end, bytes and every
stream's exported state, over consecutive batches (streams created in the
first, continued and extended in the second).  Broken speculation
(reordering inside a stream, a replay, a 9th SSRC, a forged packet) must
fall back with identical results.
"""
import errno

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_async import Dev, run_chain
from tests.test_gpu_fastpath import keys_for, rtp_packet, run_dev, states

pytestmark = pytest.mark.gpu

SSRC0 = 0x7000


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def interleaved(rng, which, seq0, plen=None):
    """packets of one session: packet i belongs to stream which[i]
    (SSRC0 + k), each stream's seq runs on from seq0[k]"""
    nxt = dict(seq0)
    out = []
    for k in which:
        k = int(k)
        out.append((0, rtp_packet(rng, nxt[k] & 0xffff, SSRC0 + k,
                                  plen=plen)))
        nxt[k] += 1
    return out, nxt


def arena_of(pkts, room=80):
    sizes = [len(p) + room for _, p in pkts]
    off, base = 0, []
    for sz in sizes:
        base.append(off)
        off += (sz + 15) & ~15
    arena = np.zeros(off, dtype=np.uint8)
    pos = np.array(base, dtype=np.uint32)
    end = pos + np.array([len(p) for _, p in pkts], dtype=np.uint32)
    cap = end + 60
    for i, (_, p) in enumerate(pkts):
        arena[pos[i]:end[i]] = np.frombuffer(p, dtype=np.uint8)
    return arena, pos, end, cap.astype(np.uint32)


def protected(res, pos):
    arena, _, end, err = res
    return [(0, arena[pos[i]:end[i]].tobytes())
            for i in range(len(pos)) if err[i] == 0]


def run_mode(torch, mode, suite, key, batches, ssrcs, rx_mutate=None):
    """batches: packet lists sent through one tx context, then the
    protected packets through one rx context, batch by batch"""
    knobs = {"plan": {}, "general": {"general": 1},
             "forced": {"splan": 1}}[mode]
    tx, rx = P.Srtp(suite, key), P.Srtp(suite, key)
    outs = []
    with P.tune(**knobs):
        for pk in batches:
            a, p, e, c = arena_of(pk)
            r = run_dev(torch, "srtp_encrypt", [tx], a, p, e, c, None)
            outs.append(r)
            rp = protected(r, p)
            if rx_mutate:
                rp = rx_mutate(rp)
            a2, p2, e2, c2 = arena_of(rp)
            outs.append(run_dev(torch, "srtp_decrypt", [rx], a2, p2, e2, c2,
                                None))
    st = (states([tx], ssrcs), states([rx], ssrcs))
    tx.close()
    rx.close()
    return outs, st


def same(A, B, what):
    for x, y in zip(A[0], B[0]):
        for u, v in zip(x, y):
            assert (u == v).all(), what
    assert A[1] == B[1], what


@pytest.mark.parametrize("suite", [0, 1, 3, 4, 5])
@pytest.mark.parametrize("nstreams", [2, 3, 8])
def test_streams_planner_equals_general_and_oracle(suite, nstreams,
                                                   torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(500 + 10 * suite + nstreams)
    key = keys_for(suite, 1)[0]
    n = 2400
    seq0 = {k: int(65000 + 333 * k) if k % 2 == 0 else int(rng.integers(0,
            65536)) for k in range(8)}
    # batch 1: all but the last stream (nstreams - 1 of them when 8, so
    # batch 2 adds one); batch 2: every stream, wraps on the way
    k1 = nstreams - 1 if nstreams > 2 else nstreams
    b1, nxt = interleaved(rng, rng.integers(0, k1, n), seq0)
    b2, _ = interleaved(rng, rng.integers(0, nstreams, n), nxt)
    ssrcs = [SSRC0 + k for k in range(nstreams)]
    s0 = P.counter("splans")
    res = {m: run_mode(torch, m, suite, key, [b1, b2], ssrcs)
           for m in ("plan", "general")}
    # each of the 4 calls took the per-stream planner
    assert P.counter("splans") - s0 == 4
    same(res["plan"], res["general"], "plan vs general")
    outs = res["plan"][0]
    for r in outs:
        assert (r[3] == 0).all()

    # the oracle, one packet at a time, same call order
    be = O.OracleBackend()
    otx, _ = be.alloc(suite, key, 0)
    orx, _ = be.alloc(suite, key, 0)
    for bi, pk in enumerate((b1, b2)):
        enc = outs[2 * bi]
        a, p, e, c = arena_of(pk)
        sent = []
        for i, (_, pkt) in enumerate(pk):
            er, po, en, _, buf = be.call(otx, "srtp_encrypt", len(pkt) + 64,
                                         0, len(pkt), pkt, len(pkt) + 16)
            assert (int(enc[3][i]), int(enc[1][i] - p[i]),
                    int(enc[2][i] - p[i])) == (er, po, en), (bi, i)
            assert enc[0][p[i]:enc[2][i]].tobytes() == buf[:en], (bi, i)
            sent.append(buf[:en])
        dec = outs[2 * bi + 1]
        a2, p2, e2, c2 = arena_of([(0, x) for x in sent])
        for i, pkt in enumerate(sent):
            er, po, en, _, buf = be.call(orx, "srtp_decrypt", len(pkt) + 64,
                                         0, len(pkt), pkt, len(pkt))
            assert (int(dec[3][i]), int(dec[1][i] - p2[i]),
                    int(dec[2][i] - p2[i])) == (er, po, en), (bi, i)
            assert dec[0][p2[i]:p2[i] + en].tobytes() == buf[:en], (bi, i)
    be.free(otx)
    be.free(orx)


@pytest.mark.parametrize("suite", [1, 5])
def test_streams_forced_single_stream(suite, torch_cuda):
    """srtp_gpu_tune splan: a one-SSRC batch through the per-stream planner
    equals the single-stream planner (ROC wrap inside)"""
    torch = torch_cuda
    rng = np.random.default_rng(61 + suite)
    key = keys_for(suite, 1)[0]
    b1, nxt = interleaved(rng, np.zeros(1500, dtype=int), {0: 65200})
    b2, _ = interleaved(rng, np.zeros(1500, dtype=int), nxt)
    s0 = P.counter("splans")
    A = run_mode(torch, "forced", suite, key, [b1, b2], [SSRC0])
    assert P.counter("splans") - s0 == 4
    B = run_mode(torch, "plan", suite, key, [b1, b2], [SSRC0])
    same(A, B, "forced splan vs single-stream plan")


def test_fresh_sessions_learn_the_per_stream_planner(torch_cuda):
    """a session's first batch (no stream yet) with several SSRCs: the
    one-stream plan is rejected once (g_fresh_multi set), later fresh
    sessions go to the per-stream planner directly (no reject, same bytes
    and states as the general engine); a fresh one-SSRC session clears the
    hint again"""
    torch = torch_cuda
    rng = np.random.default_rng(808)
    key = keys_for(1, 1)[0]
    b2, _ = interleaved(rng, rng.integers(0, 2, 3000), {0: 65300, 1: 900})
    b1, _ = interleaved(rng, np.zeros(3000, dtype=int), {0: 65300})
    ss2, ss1 = [SSRC0, SSRC0 + 1], [SSRC0]
    assert P.counter("freshmulti") == 0
    r0, s0 = P.counter("rejects"), P.counter("splans")
    A = run_mode(torch, "plan", 1, key, [b2], ss2)
    assert P.counter("rejects") - r0 == 1          # tx: rejected once
    assert P.counter("splans") - s0 == 2
    assert P.counter("freshmulti") == 1
    r1 = P.counter("rejects")
    B = run_mode(torch, "plan", 1, key, [b2], ss2)
    assert P.counter("rejects") == r1              # planned directly
    G = run_mode(torch, "general", 1, key, [b2], ss2)
    same(A, G, "first fresh session vs general")
    same(B, G, "hinted fresh session vs general")
    C = run_mode(torch, "plan", 1, key, [b1], ss1)
    assert P.counter("freshmulti") == 0
    D = run_mode(torch, "plan", 1, key, [b1], ss1)
    same(C, D, "one SSRC: per-stream vs single-stream plan")
    for r in A[0] + B[0] + C[0]:
        assert (r[3] == 0).all()


@pytest.mark.parametrize("suite", [1, 4])
@pytest.mark.parametrize("case", ["reorder", "replay", "ninth", "forged",
                                  "timeout"])
def test_streams_fallbacks(suite, case, torch_cuda):
    """broken speculation falls back to the host engines, same results"""
    torch = torch_cuda
    rng = np.random.default_rng(91 + suite)
    key = keys_for(suite, 1)[0]
    n = 1200
    nst = 9 if case == "ninth" else 3
    which = rng.integers(0, nst, n)
    if case == "ninth":
        which[1000] = 8
    seq0 = {k: 65100 + 50 * k for k in range(9)}
    pk, _ = interleaved(rng, which, seq0)
    if case == "reorder":
        j = [i for i in range(n) if which[i] == 1][100:102]
        pk[j[0]], pk[j[1]] = pk[j[1]], pk[j[0]]
    if case == "timeout":
        i = [i for i in range(n) if which[i] == 2][200]
        b = bytearray(pk[i][1])
        s = ((b[2] << 8 | b[3]) + 40000) & 0xffff
        b[2], b[3] = s >> 8, s & 0xff
        pk[i] = (0, bytes(b))

    def mutate(rp):
        rp = list(rp)
        if case == "replay":
            rp.insert(700, rp[650])
        if case == "forged":
            q = bytearray(rp[500][1])
            q[40] ^= 1
            rp[500] = (0, bytes(q))
        return rp

    ssrcs = [SSRC0 + k for k in range(nst)]
    A = run_mode(torch, "plan", suite, key, [pk], ssrcs, mutate)
    B = run_mode(torch, "general", suite, key, [pk], ssrcs, mutate)
    same(A, B, case)
    codes = {int(x) for r in A[0] for x in r[3]}
    if case == "ninth":
        assert errno.ENOSR in codes
    if case == "forged":
        assert P.EAUTH in codes
    if case == "replay":
        assert errno.EALREADY in codes


@pytest.mark.parametrize("suite", [1, 5])
def test_streams_async_chain(suite, torch_cuda):
    """asynchronous calls on a multi-SSRC session equal the synchronous
    ones (the chain issues the per-stream planner without a host sync)"""
    torch = torch_cuda
    rng = np.random.default_rng(3 + suite)
    key = keys_for(suite, 1)[0]
    seq0 = {k: 65400 + k for k in range(4)}
    b1, nxt = interleaved(rng, rng.integers(0, 4, 1000), seq0)
    b2, _ = interleaved(rng, rng.integers(0, 4, 1000), nxt)
    outs = {}
    for mode in ("sync", "async"):
        tx = P.Srtp(suite, key)
        calls = []
        for pk in (b1, b2):
            a, p, e, c = arena_of(pk)
            calls.append(("srtp_encrypt", [tx],
                          Dev(torch, a, p, e, c, None)))
        outs[mode] = (run_chain(torch, calls, mode),
                      states([tx], [SSRC0 + k for k in range(4)]))
        tx.close()
    for x, y in zip(outs["sync"][0], outs["async"][0]):
        for u, v in zip(x, y):
            assert (u == v).all()
    assert outs["sync"][1] == outs["async"][1]


@pytest.mark.parametrize("suite", [1, 4])
def test_streams_edge_shapes(suite, torch_cuda):
    """per-stream planner edge shapes, each vs the general engine: batches
    of 1, 255, 257 and 1025 packets; an 8th stream joining 7 existing
    ones; a 9th SSRC in a later batch (ENOSR); a stream whose s_l is not
    set yet (created by SRTCP first); a ROC wrap exactly at the batch
    boundary; a replay of the previous batch's last packet"""
    torch = torch_cuda
    rng = np.random.default_rng(1234 + suite)
    key = keys_for(suite, 1)[0]

    def run_both(batches, ssrcs, pre=None, rx_mutate=None):
        res = []
        for mode in ("plan", "general"):
            knobs = {"plan": {}, "general": {"general": 1}}[mode]
            tx, rx = P.Srtp(suite, key), P.Srtp(suite, key)
            if pre:
                pre(tx, rx)
            outs = []
            with P.tune(**knobs):
                for bi, pk in enumerate(batches):
                    a, p, e, c = arena_of(pk)
                    r = run_dev(torch, "srtp_encrypt", [tx], a, p, e, c,
                                None)
                    outs.append(r)
                    rp = protected(r, p)
                    if rx_mutate:
                        rp = rx_mutate(bi, rp)
                    a2, p2, e2, c2 = arena_of(rp)
                    outs.append(run_dev(torch, "srtp_decrypt", [rx], a2, p2,
                                        e2, c2, None))
            res.append((outs, (states([tx], ssrcs), states([rx], ssrcs))))
            tx.close()
            rx.close()
        same(res[0], res[1], "edge")
        return res[0]

    # sizes around the planner's block (1024) and the LDS scan width
    for n in (1, 255, 257, 1025):
        which = rng.integers(0, 3, n)
        pk, _ = interleaved(rng, which, {k: 65530 + k for k in range(3)})
        run_both([pk], [SSRC0 + k for k in range(3)])

    # 7 streams, then an 8th joins; then a 9th SSRC (ENOSR) in batch 3
    b1, nxt = interleaved(rng, rng.integers(0, 7, 700),
                          {k: 100 * k for k in range(9)})
    b2, nxt = interleaved(rng, rng.integers(0, 8, 700), nxt)
    b3, _ = interleaved(rng, rng.integers(0, 9, 700), nxt)
    out, _ = run_both([b1, b2, b3], [SSRC0 + k for k in range(9)])
    assert errno.ENOSR in {int(x) for x in out[4][3]}

    # a stream created by SRTCP (s_l not set), then RTP on it and another
    def rtcp_first(tx, rx):
        for ctx in (tx, rx):
            st = P.StreamState()
            st.ssrc = SSRC0 + 1
            assert ctx.import_(st) == 0     # exists, s_l_set = 0
    pk, _ = interleaved(rng, rng.integers(0, 2, 600), {0: 5, 1: 65000})
    run_both([pk], [SSRC0, SSRC0 + 1], pre=rtcp_first)

    # a ROC wrap exactly at the batch boundary, and a replayed last packet
    b1, nxt = interleaved(rng, np.array([0, 1] * 268),
                          {0: 65536 - 268, 1: 65536 - 268})
    b2, _ = interleaved(rng, np.array([0, 1] * 300), nxt)

    saved = []

    def replay_last(bi, rp):
        if bi == 0:
            saved[:] = [rp[-1]]         # the batch's last packet ...
            return rp
        return saved + rp               # ... received again first
    out, _ = run_both([b1, b2], [SSRC0, SSRC0 + 1], rx_mutate=replay_last)
    assert errno.EALREADY in {int(x) for x in out[3][3]}


def test_streams_full_size(torch_cuda):
    """BASELINE size through the per-stream planner: 1M x 1200-B packets of
    one session over two SSRCs (bench.py --ssrcs 2: packet i on stream
    i mod 2, each stream's seq from 65000 -- eight ROC wraps), protect and
    unprotect, against the reference itself (tests/golden/
    fullsize_digests.json shape 6, oracle/ref_digest.c): the whole arena,
    every end and errno and both streams' final states after each
    direction; the general engine must agree too"""
    from re_amd import workload as W
    from tests import fullsize_util as F
    torch = torch_cuda
    ref = F.load()[6]
    arena, pos, end, cap, _, keys = W.build_config(6)
    n, slot = ref["n"], ref["slot"]
    assert F.sha(arena) == ref["plain"]
    key = keys[0].tobytes()
    ssrcs = [W.SSRC_BASE, W.SSRC_BASE + 1]

    def st_bytes(ctx):
        rows = []
        for x in ssrcs:
            e, st = ctx.export(x)
            assert e == 0
            rows.append((st.roc, st.s_l, st.replay_rtp_lix,
                         st.replay_rtp_bitmap))
        return F.state_bytes(rows)

    for mode in ("plan", "general"):
        knobs = {"plan": {}, "general": {"general": 1}}[mode]
        tx, rx = P.Srtp(1, key), P.Srtp(1, key)
        s0 = P.counter("splans")
        with P.tune(**knobs):
            a, p, e, err = run_dev(torch, "srtp_encrypt", [tx], arena, pos,
                                   end, cap, None)
            bad_p = F.compare(ref["protect"], a, n, slot, e, err,
                              st_bytes(tx))
            d, p2, e2, err2 = run_dev(torch, "srtp_decrypt", [rx], a, pos,
                                      e, cap, None)
            bad_u = F.compare(ref["unprotect"], d, n, slot, e2, err2,
                              st_bytes(rx))
        if mode == "plan":
            assert P.counter("splans") - s0 == 2
        tx.close()
        rx.close()
        assert not bad_p and not bad_u, (mode, bad_p, bad_u)
