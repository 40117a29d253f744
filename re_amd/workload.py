"""Synthetic SRTP workloads (BASELINE.json configs).

Packets are full RTP packets: 12-byte header (V=2, CC=0, X=0, PT=0),
seq = (s0 + i) mod 2^16 with s0 = 65000 (ROC wraps every 65536 packets),
ts = 160*i, one SSRC per session; payload bytes from a seeded generator.
Each packet sits in a 16-byte aligned slot with room for the tag, so the
arena can be handed to srtp_*_batch as-is.
"""
import numpy as np

SEED_PAYLOAD = 0x5EED5EED
SEED_KEYS = 0xC0FFEE
SSRC_BASE = 0x01020304


def slot_size(max_len):
    return (max_len + 16 + 15) & ~15


def make_keys(nsess, klen, seed=SEED_KEYS):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(nsess, klen), dtype=np.uint8)


def make_arena(npkts, lengths, s0=65000, sess=None, seed=SEED_PAYLOAD,
               payload=True):
    """Returns (arena uint8[n*slot], pos, end, cap) numpy arrays.

    lengths: int or uint32 array (RTP packet length incl. 12-B header).
    sess: optional per-packet session index (SSRC = SSRC_BASE + sess).
    """
    lengths = np.broadcast_to(np.asarray(lengths, dtype=np.uint32),
                              (npkts,)).copy()
    slot = slot_size(int(lengths.max()))
    arena = np.zeros((npkts, slot), dtype=np.uint8)
    if payload:
        rng = np.random.default_rng(seed)
        arena[:, 12:int(lengths.max())] = rng.integers(
            0, 256, size=(npkts, int(lengths.max()) - 12), dtype=np.uint8)
        # zero bytes past each packet's end (mixed lengths)
        if lengths.min() != lengths.max():
            col = np.arange(slot, dtype=np.uint32)[None, :]
            arena[col >= lengths[:, None]] = 0
    i = np.arange(npkts, dtype=np.uint64)
    if sess is not None:
        # per-session sequence numbers: ordinal of the packet within its
        # session, so every SSRC sends seq s0, s0+1, ... in array order
        sarr = np.asarray(sess, dtype=np.int64)
        order = np.argsort(sarr, kind="stable")
        ss = sarr[order]
        first = np.r_[0, np.flatnonzero(np.diff(ss)) + 1]
        run_start = np.repeat(first, np.diff(np.r_[first, len(ss)]))
        ordinal = np.empty(npkts, dtype=np.uint64)
        ordinal[order] = (np.arange(npkts) - run_start).astype(np.uint64)
        seq = ((s0 + ordinal) & 0xffff).astype(np.uint16)
    else:
        seq = ((s0 + i) & 0xffff).astype(np.uint16)
    ts = (160 * i & 0xffffffff).astype(np.uint32)
    ssrc = np.full(npkts, SSRC_BASE, dtype=np.uint32)
    if sess is not None:
        ssrc = (SSRC_BASE + np.asarray(sess, dtype=np.uint32)).astype(np.uint32)
    arena[:, 0] = 0x80
    arena[:, 1] = 0
    arena[:, 2] = (seq >> 8).astype(np.uint8)
    arena[:, 3] = (seq & 0xff).astype(np.uint8)
    for k in range(4):
        arena[:, 4 + k] = ((ts >> (24 - 8 * k)) & 0xff).astype(np.uint8)
        arena[:, 8 + k] = ((ssrc >> (24 - 8 * k)) & 0xff).astype(np.uint8)
    pos = (np.arange(npkts, dtype=np.uint64) * slot).astype(np.uint32)
    end = (pos + lengths).astype(np.uint32)
    cap = (pos + slot).astype(np.uint32)
    return arena.reshape(-1), pos, end, cap


def mixed_lengths(npkts, seed=SEED_PAYLOAD + 1):
    """config 4: Bernoulli(0.5) -> 200 or 1400 B"""
    rng = np.random.default_rng(seed)
    return np.where(rng.integers(0, 2, size=npkts) == 1, 1400,
                    200).astype(np.uint32)


def random_sessions(npkts, nsess, seed=SEED_PAYLOAD + 2):
    rng = np.random.default_rng(seed)
    return rng.integers(0, nsess, size=npkts, dtype=np.uint32)
