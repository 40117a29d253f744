"""srtp_rx_index's receiver walk runs in parallel parts on long streams
(re_amd/csrc/host/rxfold.c rx_walk_packed: each part guesses its start
state from a cold walk over the packets before it, the guesses are checked
in order against the previous part's true end state, a wrong one is walked
again, a right one gets its ROC base added).  The records must be those of
the sequential walk -- restated here from the reference receiver's index
step (src/srtp/srtp.c:310-321, the s_l update of :426-427, srtp_get_index
misc.c:22-41) -- on streams with ROC wraps, loss, reordering, replays,
long runs of failed packets at part boundaries, headers that do not parse
and a ROC near the signed-int range.  CPU only (no device call).
"""
import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import shard as S

SSRC = 0x5EED0042
PARTS = 16          # RXW_PARTS


def get_index(roc, s_l, seq):
    if s_l < 32768:
        v = roc - 1 if seq - s_l > 32768 else roc
    else:
        v = roc + 1 if s_l - 32768 > seq else roc
    v = ((v & 0xffffffff) ^ 0x80000000) - 0x80000000      # int32_t
    return (seq + v * 65536) & 0xffffffffffffffff


def walk(roc, s_l, sset, oks, seqs, res):
    """the sequential walk (rx_step): (ix, res, seq, stage) per packet"""
    out = []
    for ok, seq, r in zip(oks, seqs, res):
        if not ok:
            out.append((0, r, 0, P.RX_NOHDR))
            continue
        if not sset:
            s_l, sset = seq, 1
        diff = seq - s_l
        if diff > 32768:
            out.append((0, r, seq, P.RX_NOIX))
            continue
        if diff <= -32768:
            roc = (roc + 1) & 0xffffffff
            s_l = 0
        out.append((get_index(roc, s_l, seq), r, seq, P.RX_IX))
        if r == 0 and seq > s_l:
            s_l = seq
    return out


def stream(n, seed, s0=65000):
    """arrival order of a lossy, reordered stream with replays: global
    packet numbers"""
    rng = np.random.default_rng(seed)
    g = np.arange(n, dtype=np.int64)
    g = g[rng.random(n) > 0.02]                             # loss
    sw = rng.integers(0, len(g) - 1, len(g) // 50)          # local swaps
    g[sw], g[sw + 1] = g[sw + 1].copy(), g[sw].copy()
    # a block delivered late, deeper than the parts' warm-up
    b = len(g) // 3
    g = np.concatenate([g[:b], g[b + 3000:b + 9000], g[b:b + 3000],
                        g[b + 9000:]])
    dup = rng.integers(0, len(g), len(g) // 100)            # replays
    g = np.insert(g, np.sort(dup), g[dup])
    return (g + s0) & 0xffff, rng


def arena_of(seqs, rng, bad_frac=0.005):
    m = len(seqs)
    arena = np.zeros((m, 16), dtype=np.uint8)
    arena[:, 0] = 0x80
    arena[:, 2] = (seqs >> 8) & 0xff
    arena[:, 3] = seqs & 0xff
    for k in range(4):
        arena[:, 8 + k] = (SSRC >> (24 - 8 * k)) & 0xff
    pos = np.arange(m, dtype=np.uint32) * 16
    end = pos + 16
    bad = rng.random(m) < bad_frac
    end[bad] = pos[bad] + 7                                 # no header
    return arena.reshape(-1), pos, end, ~bad


def results(m, rng, fail_runs):
    res = np.where(rng.random(m) < 0.03, 80, 0).astype(np.int32)  # EAUTH
    res[rng.random(m) < 0.01] = 114                         # EALREADY
    for a, ln in fail_runs:                                 # failed runs
        res[a:a + ln] = 80
    return res


def check(st, seqs, arena, pos, end, ok, res):
    st0 = P.StreamState()
    st0.ssrc = SSRC
    st0.roc, st0.s_l, st0.s_l_set = st
    rec = S.rx_records(st0, arena, pos, end, res)
    want = walk(st[0], st[1], st[2], ok, seqs.tolist(), res.tolist())
    got = list(zip(rec["ix"].tolist(), rec["res"].tolist(),
                   rec["seq"].tolist(), rec["stage"].tolist()))
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[:5], got[bad[0]], want[bad[0]])


@pytest.mark.parametrize("seed,st", [
    (1, (0, 0, 0)),
    (2, (7, 65000, 1)),
    (3, (0x7ffe0000, 100, 1)),       # ROC near the int32 range
])
def test_parallel_walk_equals_sequential(seed, st):
    P.load()
    seqs, rng = stream(300000, seed)
    arena, pos, end, ok = arena_of(seqs, rng)
    m = len(seqs)
    # runs of failures longer than the warm-up across part boundaries
    runs = [(m * k // PARTS - 700, 1400) for k in (3, 7, 11)]
    res = results(m, rng, runs)
    r0 = P.counter("rxw_redos")
    check(st, seqs, arena, pos, end, ok, res)
    if st[0] < 0x70000000:
        # the parts after the failure runs guessed wrong and were re-walked
        assert P.counter("rxw_redos") - r0 >= 3


def test_parallel_walk_other_ssrc_is_einval():
    P.load()
    seqs, rng = stream(200000, 5)
    arena, pos, end, ok = arena_of(seqs, rng, bad_frac=0)
    a = arena.reshape(-1, 16)
    a[150000, 11] ^= 1                                      # another SSRC
    st0 = P.StreamState()
    st0.ssrc = SSRC
    with pytest.raises(OSError):
        S.rx_records(st0, arena, pos, end, np.zeros(len(seqs), np.int32))


EALREADY, ETIMEDOUT, EAUTH = 114, 110, 80


def receiver(st, oks, seqs, forged):
    """the reference receiver's results (srtp.c:310-368 with the 64-packet
    window of replay.c:32-62) for a packet sequence: what every rank of a
    correct split would report"""
    roc, s_l, sset = st
    lix, bm = 0, 0
    out = []
    for ok, seq, bad in zip(oks, seqs, forged):
        if not ok:
            out.append(74)                                   # EBADMSG
            continue
        if not sset:
            s_l, sset = seq, 1
        diff = seq - s_l
        if diff > 32768:
            out.append(ETIMEDOUT)
            continue
        if diff <= -32768:
            roc = (roc + 1) & 0xffffffff
            s_l = 0
        ix = get_index(roc, s_l, seq)
        if bad:
            out.append(EAUTH)
            continue
        if ix > lix:
            d = ix - lix
            bm = ((bm << d) | 1) & (2**64 - 1) if d < 64 else 1
            lix = ix
        else:
            d = lix - ix
            if d >= 64 or (bm >> d) & 1:
                out.append(EALREADY)
                continue
            bm |= 1 << d
        out.append(0)
        if seq > s_l:
            s_l = seq
    return np.array(out, dtype=np.int32)


def fold_both(st, rec):
    """srtp_rx_fold in one pass (rxseq) and in parallel parts"""
    outs = []
    for seq in (1, 0):
        s = P.StreamState()
        s.ssrc = SSRC
        s.roc, s.s_l, s.s_l_set = st
        with P.tune(rxseq=seq):
            e, nd = S.rx_fold(s, 1, rec)
        outs.append((e.tolist(), nd, s.roc, s.s_l, s.s_l_set,
                     s.replay_rtp_lix, s.replay_rtp_bitmap))
    return outs


@pytest.mark.parametrize("seed,st", [(11, (0, 0, 0)), (12, (3, 40000, 1))])
def test_parallel_fold_equals_sequential(seed, st):
    P.load()
    seqs, rng = stream(300000, seed)
    arena, pos, end, ok = arena_of(seqs, rng)
    forged = rng.random(len(seqs)) < 0.02
    res = receiver(st, ok.tolist(), seqs.tolist(), forged.tolist())
    st0 = P.StreamState()
    st0.ssrc = SSRC
    st0.roc, st0.s_l, st0.s_l_set = st
    rec = S.rx_records(st0, arena, pos, end, res)
    r0 = P.counter("rxw_redos")
    a, b = fold_both(st, rec)
    assert a == b
    assert a[1] == len(rec) and a[0] == res.tolist()       # every verdict
    m = len(rec)
    # a replay verdict the window contradicts, and an index the rank got
    # wrong, late in the stream: the fold stops there, in both forms
    for p0, how in ((int(m * 0.71), "res"), (int(m * 0.83), "ix")):
        r = rec.copy()
        p = p0 + int(np.flatnonzero((r["stage"][p0:] == P.RX_IX) &
                                    (r["res"][p0:] == 0))[0])
        if how == "res":
            r["res"][p] = EALREADY
        else:
            r["ix"][p] += 65536
        a, b = fold_both(st, r)
        assert a == b and a[1] == p, (how, p, a[1], b[1])
    assert P.counter("rxw_redos") >= r0                     # (diagnostic)
