"""Cross-rank replay fold of one stream split across ranks (SURVEY 8(e);
include/re_srtp_batch.h srtp_rx_index / srtp_rx_fold, re_amd/shard.py).

A stream with a ROC wrap, loss, reordering, replays, forged packets, a
header-truncated packet and an out-of-window jump is protected by the
oracle sender.  The truth is the oracle receiver over the whole stream in
arrival order (the C restatement pinned to the reference's goldens,
tests/test_oracle.py).  Each "rank" then unprotects its contiguous shard
with its own oracle receiver started from an ASSUMED boundary state
(the closed form re_amd/shard.py uses: highest index so far, full replay
window), records what it did with the product's srtp_rx_index, and the
product's srtp_rx_fold replays the reference receiver over the gathered
records: every verdict it keeps must equal the truth, the state it returns
must be the exact state before the first voided packet, and re-running
from there must reproduce the truth to the end.  A world-size-2 gloo run
checks the gather.  No GPU: both entry points are host code.
"""
import ctypes
import errno
import multiprocessing as mp
import socket

import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import shard as S

from oracle_lib import OracleBackend

SSRC = 0x5a5a0001
EAUTH = 217
CM80, GCM128 = 1, 4


def key_for(suite):
    n = P.key_len(suite) + P.salt_len(suite)
    return bytes((7 * i + 3) & 0xff for i in range(n))


def rtp(seq, k):
    hdr = bytes([0x80, 96, seq >> 8, seq & 0xff]) + \
        (k * 160 & 0xffffffff).to_bytes(4, "big") + SSRC.to_bytes(4, "big")
    return hdr + bytes((k + i) & 0xff for i in range(40 + k % 23))


def protect_stream(O, suite, ixs):
    """oracle sender over indices ixs (monotone, gaps = loss)"""
    ctx, e = O.alloc(suite, key_for(suite), 0)
    assert e == 0
    out = {}
    for ix in ixs:
        p = rtp(ix & 0xffff, ix)
        e, pos, end, _, buf = O.call(ctx, "srtp_encrypt", len(p) + 32, 0,
                                     len(p), p, len(p) + 32)
        assert e == 0
        out[ix] = buf[pos:end]
    O.free(ctx)
    return out


def arrival(suite, O, s0=65400, n=900, seed=1):
    """arrival-order packets: loss, adjacent swaps, late packets, replays
    (some across any boundary), forgeries, one truncated header and one
    out-of-window jump"""
    rng = np.random.default_rng(seed)
    ixs = [s0 + i for i in range(n) if rng.random() > 0.05]
    ixs.append(s0 + n + 40000)               # jump: ETIMEDOUT at the receiver
    pk = protect_stream(O, suite, ixs)
    order = ixs[:-1]
    for i in range(1, len(order) - 1, 17):   # adjacent swaps
        order[i], order[i + 1] = order[i + 1], order[i]
    pkts = [pk[ix] for ix in order]
    for j in range(40, len(pkts), 61):       # late packets (within window)
        pkts.insert(j, pk[order[j - 30]])
    for j in range(25, len(pkts), 97):       # far replays (outside window)
        pkts.insert(j + 300 if j + 300 < len(pkts) else j, pk[order[j // 3]])
    for j in range(11, len(pkts), 131):      # forged copies
        b = bytearray(pkts[j])
        b[20] ^= 0x40
        pkts.insert(j, bytes(b))
    pkts.insert(333, pkts[333][:9])          # truncated header
    pkts.insert(500, pk[ixs[-1]])            # out-of-window jump
    return pkts


def receive(O, suite, pkts, st=None, outs=None):
    """oracle receiver over pkts; st = (roc, s_l, s_l_set, lix, bitmap) to
    start from.  Returns (errs, (roc, s_l, lix, bitmap)); each packet's
    side effects (pos, end, bytes) are appended to the list outs."""
    ctx, e = O.alloc(suite, key_for(suite), 0)
    assert e == 0
    if st is not None:
        assert O.l.oracle_stream_set(ctx, SSRC, *st) == 0
    errs = []
    for p in pkts:
        e, pos, end, _, buf = O.call(ctx, "srtp_decrypt", len(p) + 32, 0,
                                     len(p), p, len(p))
        errs.append(e)
        if outs is not None:
            outs.append((pos, end, buf[:len(p)]))
    fin = O.export(ctx, SSRC)
    O.free(ctx)
    return np.array(errs, dtype=np.int32), fin


def arena_of(pkts):
    pos, end, buf = [], [], bytearray()
    for p in pkts:
        pos.append(len(buf))
        buf += p
        end.append(len(buf))
        buf += bytes(-len(buf) % 16)
    return (np.frombuffer(bytes(buf), dtype=np.uint8),
            np.array(pos, dtype=np.uint32), np.array(end, dtype=np.uint32))


def state(roc=0, s_l=0, s_l_set=0, lix=0, bitmap=0):
    st = P.StreamState()
    st.ssrc = SSRC
    st.roc, st.s_l, st.s_l_set = roc, s_l, s_l_set
    st.replay_rtp_lix, st.replay_rtp_bitmap = lix, bitmap
    return st


def assumed_boundary(pkts):
    """the guess a rank makes without the previous shards' verdicts: their
    packets' headers run through the receiver's index rules as if every
    packet were authentic (srtp.c:313-321, misc.c:22-41), the highest index
    as the window top and every packet below it seen"""
    roc, s_l, hi = 0, None, None
    for p in pkts:
        if len(p) < 12:
            continue
        seq = p[2] << 8 | p[3]
        if s_l is None:
            s_l = seq
        d = seq - s_l
        if d > 32768:
            continue
        if d <= -32768:
            roc, s_l = roc + 1, 0
        v = roc
        if s_l < 32768 and seq - s_l > 32768:
            v = roc - 1
        elif s_l >= 32768 and s_l - 32768 > seq:
            v = roc + 1
        ix = (v << 16) + seq
        if seq > s_l:
            s_l = seq
        hi = ix if hi is None or ix > hi else hi
    if hi is None:
        return (0, 0, 0, 0, 0)
    return (roc, s_l, 1, hi, (1 << 64) - 1)


def fold_check(O, suite, pkts, bounds, guess=assumed_boundary):
    """the ranks' results folded, voided tails re-run from the fold's
    state: the verdicts, the final state and every packet's side effects
    (pos, end, bytes: the ranks' where their verdict stands, the re-run's
    after a void) equal the one receiver's"""
    want = []
    truth, fin = receive(O, suite, pkts, outs=want)
    recs = []
    got = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        st0 = guess(pkts[:a]) if a else None
        res, _ = receive(O, suite, pkts[a:b], st0, outs=got)
        arena, pos, end = arena_of(pkts[a:b])
        recs.append(S.rx_records(state(*st0) if st0 else state(), arena,
                                 pos, end, res))
    rec = np.concatenate(recs)
    st = state()
    done = 0
    err_all = []
    while True:
        err, nd = S.rx_fold(st, suite, rec[done:] if done else rec)
        err_all.append(err)
        assert (err == truth[done:done + nd]).all()
        done += nd
        if done == len(pkts):
            break
        # a voided verdict: re-run the rest from the fold's state, as one
        # rank would (its records are then exact)
        st0 = (st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
               st.replay_rtp_bitmap)
        del got[done:]
        res, _ = receive(O, suite, pkts[done:], st0, outs=got)
        arena, pos, end = arena_of(pkts[done:])
        rec = np.concatenate([rec[:done],
                              S.rx_records(state(*st0), arena, pos, end,
                                           res)])
    assert (np.concatenate(err_all) == truth).all()
    assert (st.roc, st.s_l, st.replay_rtp_lix, st.replay_rtp_bitmap) == fin
    assert got == want
    return truth


@pytest.mark.parametrize("suite", [CM80, GCM128])
def test_fold_single_rank_is_the_receiver(suite):
    O = OracleBackend()
    pkts = arrival(suite, O)
    truth = fold_check(O, suite, pkts, [0, len(pkts)])
    # the stream exercises every verdict the fold produces
    codes = set(truth.tolist())
    assert {0, EAUTH, errno.ETIMEDOUT, errno.EBADMSG, errno.EALREADY} <= codes


@pytest.mark.parametrize("suite", [CM80, GCM128])
@pytest.mark.parametrize("nshard", [2, 3, 8])
def test_fold_across_ranks_matches_sequential_receiver(suite, nshard):
    O = OracleBackend()
    pkts = arrival(suite, O, seed=nshard)
    n = len(pkts)
    bounds = [n * r // nshard for r in range(nshard)] + [n]
    fold_check(O, suite, pkts, bounds)


def local_and_fold(O, suite, pkts, b, st1):
    """rank 0 = pkts[:b] fresh, rank 1 = pkts[b:] from st1: (local
    results, folded results, ndone)"""
    res0, _ = receive(O, suite, pkts[:b])
    res1, _ = receive(O, suite, pkts[b:], st1)
    a0, p0, e0 = arena_of(pkts[:b])
    a1, p1, e1 = arena_of(pkts[b:])
    rec = np.concatenate([S.rx_records(state(), a0, p0, e0, res0),
                          S.rx_records(state(*st1), a1, p1, e1, res1)])
    err, nd = S.rx_fold(state(), suite, rec)
    return np.concatenate([res0, res1]), err, nd


@pytest.mark.parametrize("suite", [CM80, GCM128])
def test_fold_fixes_reorder_across_the_boundary(suite):
    """packet 100 arrives after 101..104 and the shard boundary falls
    between them: rank 1 assumed 'everything up to 102 seen' and gave
    EALREADY; the one receiver accepts it.  The rank's bytes for it are
    those of a rejected packet (HMAC: still ciphertext), so the fold stops
    there with the exact state and the re-run accepts it"""
    O = OracleBackend()
    pk = protect_stream(O, suite, range(65500, 65700))
    order = list(range(65500, 65700))
    order.remove(65600)
    order.insert(order.index(65604) + 1, 65600)
    pkts = [pk[i] for i in order]
    b = order.index(65602) + 1
    truth, fin = receive(O, suite, pkts)
    st1 = assumed_boundary(pkts[:b])
    local, err, nd = local_and_fold(O, suite, pkts, b, st1)
    k = order.index(65600)
    assert local[k] == errno.EALREADY and truth[k] == 0
    assert nd == k and (err == truth[:k]).all()
    fold_check(O, suite, pkts, [0, b, len(pkts)])


@pytest.mark.parametrize("suite", [CM80, GCM128])
def test_fold_voids_a_wrong_boundary_state(suite):
    """rank 1 starts one ROC off: every verdict it made is void, the fold
    stops at its first packet with the exact state there, and the re-run
    from that state reproduces the one receiver"""
    O = OracleBackend()
    pkts = arrival(suite, O, n=600, seed=5)[:500]
    b = 250
    roc, s_l, set_, lix, bm = assumed_boundary(pkts[:b])
    st1 = (roc + 1, s_l, set_, lix + (1 << 16), bm)
    truth, _ = receive(O, suite, pkts)
    local, err, nd = local_and_fold(O, suite, pkts, b, st1)
    assert (local[b:] != truth[b:]).any()
    assert nd == b and (err == truth[:b]).all()
    fold_check(O, suite, pkts, [0, b, len(pkts)], lambda _: st1)


def test_fold_rejects_other_ssrc_and_bad_args():
    O = OracleBackend()
    pkts = arrival(CM80, O)
    arena, pos, end = arena_of(pkts)
    res = np.zeros(len(pkts), dtype=np.int32)
    st = state()
    st.ssrc = SSRC + 1
    with pytest.raises(OSError):
        S.rx_records(st, arena, pos, end, res)
    e = P.lib().srtp_rx_fold(None, CM80, None, 0, None, None)
    assert e == errno.EINVAL
    nd = ctypes.c_size_t(7)
    assert P.lib().srtp_rx_fold(ctypes.byref(state()), CM80, None, 0, None,
                                ctypes.byref(nd)) == 0 and nd.value == 0
    assert P.lib().srtp_rx_fold(ctypes.byref(state()), 9, None, 0, None,
                                ctypes.byref(nd)) == errno.EINVAL


def _gather_worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" %
                                port, rank=rank, world_size=world)
        dt = S._rx_rec_dtype()
        mine = np.zeros(3 + 5 * rank, dtype=dt)
        mine["ix"] = np.arange(len(mine)) + 1000 * rank
        mine["res"] = rank
        mine["stage"] = 2
        got = S.gather_records(dist, mine)
        want = []
        for r in range(world):
            w = np.zeros(3 + 5 * r, dtype=dt)
            w["ix"] = np.arange(len(w)) + 1000 * r
            w["res"] = r
            w["stage"] = 2
            want.append(w)
        want = np.concatenate(want)
        assert got.dtype == dt and (got == want).all()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_gloo_world2_gather_records():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
