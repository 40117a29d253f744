"""Synthetic SRTP workloads (BASELINE.json configs).

Packets are full RTP packets: 12-byte header (V=2, CC=0, X=0, PT=0),
seq = (s0 + i) mod 2^16 (per session: s0 + the packet's ordinal in its
session), ts = 160*i, SSRC = SSRC_BASE + session; each packet sits in a
16-byte aligned slot with room for the tag, so the arena can be handed to
srtp_*_batch as-is.

Every random byte comes from xorshift64* (SURVEY.md 8(d)), one generator
per packet / per session so the arena builds vectorised here and packet by
packet in C (oracle/ref_digest.c rebuilds the identical arenas to compute
the reference digests in tests/golden/fullsize_digests.json):

  xs64(s):        s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
                  return s * 0x2545F4914F6CDD1D
  state(seed, i): seed ^ (0x9E3779B97F4A7C15 * (i + 1))   (0 -> GOLDEN)
  payload of packet i:  bytes [12, L) = LE bytes of xs64 outputs of
                        state(SEED_PAYLOAD, i)
  key of session k:     LE bytes of xs64 outputs of state(SEED_KEYS, k)
  length (config 4):    first output of state(SEED_PAYLOAD + 1, i):
                        top bit set -> 1400 B, else 200 B
  session (config 4):   (first output of state(SEED_PAYLOAD + 2, i)
                         >> 32) % nsess
"""
import numpy as np

SEED_PAYLOAD = 0x5EED5EED
SEED_KEYS = 0xC0FFEE
SSRC_BASE = 0x01020304
GOLDEN = 0x9E3779B97F4A7C15
XS_MUL = 0x2545F4914F6CDD1D

# config 1: test/srtp.c:524-528 key, SSRC 0x01020304
CONFIG1_KEY = b"\x22" * 16 + b"\x44" * 14


def slot_size(max_len, room=16, align=16):
    """packet slot: the packet, `room` bytes for what protect appends (the
    SRTP tag: <= 16 B; SRTCP: E||index + tag, <= 20 B), `align`-B aligned
    (SRTCP arenas: 64, so every packet starts on a 64-B line boundary like
    the RTP configs' 1216-B slots -- the kernels walk packet-aligned 64-B
    chunks)"""
    return (max_len + room + align - 1) & ~(align - 1)


def xs_state(seed, idx):
    """initial xorshift64* states of generators idx (uint64 array)"""
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        s = np.uint64(seed) ^ (np.uint64(GOLDEN) * (idx + np.uint64(1)))
    s[s == 0] = np.uint64(GOLDEN)
    return s


def xs_next(s):
    """advance states in place, return the xorshift64* outputs"""
    s ^= s >> np.uint64(12)
    s ^= s << np.uint64(25)
    s ^= s >> np.uint64(27)
    with np.errstate(over="ignore"):
        return s * np.uint64(XS_MUL)


def xs_bytes(seed, idx, nbytes):
    """uint8[len(idx), nbytes]: LE bytes of each generator's outputs"""
    s = xs_state(seed, idx)
    nw = (nbytes + 7) // 8
    out = np.empty((len(s), nw), dtype=np.uint64)
    for w in range(nw):
        out[:, w] = xs_next(s)
    return out.view(np.uint8)[:, :nbytes]


def make_keys(nsess, klen, seed=SEED_KEYS, ids=None):
    """keys of sessions 0..nsess-1, or of the global session ids `ids`"""
    ids = np.arange(nsess) if ids is None else np.asarray(ids)
    return np.ascontiguousarray(xs_bytes(seed, ids, klen))


def make_arena(npkts, lengths, s0=65000, sess=None, seed=SEED_PAYLOAD,
               payload=True, first=0, room=16, idx=None, align=None):
    """Returns (arena uint8[n*slot], pos, end, cap) numpy arrays.

    lengths: int or uint32 array (RTP packet length incl. 12-B header).
    sess: optional per-packet session index (SSRC = SSRC_BASE + sess).
    first: global index of packet 0 (a shard of a longer stream: payload
    generators and ts continue the stream).
    idx: or the global index of every packet (a session-hashed shard of a
    longer workload, re_amd/shard.py shard_sessions).
    """
    # mixed lengths (config 4): 64-B aligned slots, so every packet starts
    # on a line boundary (oracle/ref_digest.c applies the same rule)
    if align is None:
        align = 16 if np.ndim(lengths) == 0 else 64
    lengths = np.broadcast_to(np.asarray(lengths, dtype=np.uint32),
                              (npkts,)).copy()
    maxlen = int(lengths.max())
    slot = slot_size(maxlen, room, align)
    arena = np.zeros((npkts, slot), dtype=np.uint8)
    gidx = np.arange(first, first + npkts, dtype=np.uint64) if idx is None \
        else np.asarray(idx, dtype=np.uint64)
    assert len(gidx) == npkts
    if payload and maxlen > 12:
        # in chunks: the uint64 word matrix of 1M packets is ~1.2 GB
        step = 1 << 16
        for a in range(0, npkts, step):
            b = min(npkts, a + step)
            arena[a:b, 12:maxlen] = xs_bytes(seed, gidx[a:b], maxlen - 12)
        # zero bytes past each packet's end (mixed lengths)
        if lengths.min() != maxlen:
            col = np.arange(slot, dtype=np.uint32)[None, :]
            arena[col >= lengths[:, None]] = 0
    if sess is not None:
        # per-session sequence numbers: ordinal of the packet within its
        # session, so every SSRC sends seq s0, s0+1, ... in array order
        sarr = np.asarray(sess, dtype=np.int64)
        order = np.argsort(sarr, kind="stable")
        ss = sarr[order]
        firsts = np.r_[0, np.flatnonzero(np.diff(ss)) + 1]
        run_start = np.repeat(firsts, np.diff(np.r_[firsts, len(ss)]))
        ordinal = np.empty(npkts, dtype=np.uint64)
        ordinal[order] = (np.arange(npkts) - run_start).astype(np.uint64)
        seq = ((s0 + ordinal) & 0xffff).astype(np.uint16)
    else:
        seq = ((np.uint64(s0) + np.arange(npkts, dtype=np.uint64))
               & np.uint64(0xffff)).astype(np.uint16)
    ts = ((np.uint64(160) * gidx) & np.uint64(0xffffffff)).astype(np.uint32)
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


def make_rtcp_arena(npkts, length, seed=SEED_PAYLOAD, first=0):
    """SRTCP workload: RTCP packets of `length` bytes (one SR-typed message
    header V=2, PT=200, length field = length/4 - 1, SSRC_BASE), payload
    from the same generators as make_arena.  Returns (arena, pos, end, cap).
    """
    arena, pos, end, cap = make_arena(npkts, length, seed=seed, first=first,
                                      room=20, align=64)
    a = arena.reshape(npkts, -1)
    words = (int(length) // 4 - 1) & 0xffff
    a[:, 0] = 0x80
    a[:, 1] = 200
    a[:, 2] = words >> 8
    a[:, 3] = words & 0xff
    for k in range(4):
        a[:, 4 + k] = (SSRC_BASE >> (24 - 8 * k)) & 0xff
    return arena, pos, end, cap


def mixed_lengths(npkts, seed=SEED_PAYLOAD + 1):
    """config 4: Bernoulli(0.5) -> 200 or 1400 B"""
    v = xs_next(xs_state(seed, np.arange(npkts)))
    return np.where(v >> np.uint64(63), 1400, 200).astype(np.uint32)


def random_sessions(npkts, nsess, seed=SEED_PAYLOAD + 2):
    v = xs_next(xs_state(seed, np.arange(npkts)))
    return ((v >> np.uint64(32)) % np.uint64(nsess)).astype(np.uint32)


# BASELINE.json configs as workloads (oracle/ref_digest.c mirrors this),
# plus the full-size shapes beyond them that the reference digests pin:
#   5  the config-5 stream, 2M packets (two 1M shards of it)
#   6  config 2 over 2 SSRCs of one session (packet i -> SSRC i mod 2)
#   7  SRTCP in the config-2 shape, 8  SRTCP in the config-3 shape
#   9  config 2, 10 config 4, 11 config 3, with the packets
#      i % 1000 == 999 forged between protect and unprotect (FORGE_AT:
#      payload byte 20 ^ 0x40)
#  12  shape 7 (SRTCP) with the same forgeries, and every packet
#      i % 1000 == 499 replaced after protect by a copy of protected packet
#      i - 1 (replay_targets: a replayed SRTCP index)
FORGE_AT = 32


def replay_targets(n, replay):
    """packets overwritten by a copy of their predecessor (ref_digest.c:
    i % replay == replay / 2 - 1, i >= 1)"""
    i = np.arange(1, n)
    return i[i % replay == replay // 2 - 1]

CONFIGS = {
    1: dict(suite=1, n=1024, length=160, nsess=1, s0=1, key=CONFIG1_KEY),
    2: dict(suite=1, n=1 << 20, length=1200, nsess=1, s0=65000),
    3: dict(suite=5, n=1 << 20, length=1200, nsess=1, s0=65000),
    4: dict(suite=1, n=1 << 20, length=None, nsess=1 << 16, s0=65000),
    5: dict(suite=1, n=2 << 20, length=1200, nsess=1, s0=65000),
    6: dict(suite=1, n=1 << 20, length=1200, nsess=1, s0=65000, nssrc=2),
    7: dict(suite=1, n=1 << 20, length=1200, nsess=1, s0=65000, rtcp=True),
    8: dict(suite=5, n=1 << 20, length=1200, nsess=1, s0=65000, rtcp=True),
    9: dict(suite=1, n=1 << 20, length=1200, nsess=1, s0=65000, forge=1000),
    10: dict(suite=1, n=1 << 20, length=None, nsess=1 << 16, s0=65000,
             forge=1000),
    11: dict(suite=5, n=1 << 20, length=1200, nsess=1, s0=65000, forge=1000),
    12: dict(suite=1, n=1 << 20, length=1200, nsess=1, s0=65000, rtcp=True,
             forge=1000, replay=1000),
}

KEY_LEN = {0: 30, 1: 30, 2: 46, 3: 46, 4: 28, 5: 44}


def build_config(cfg_id, n=None):
    """(arena, pos, end, cap, sess or None, keys uint8[nsess, klen])"""
    c = CONFIGS[cfg_id]
    n = n or c["n"]
    lengths = c["length"] if c["length"] else mixed_lengths(n)
    sess = random_sessions(n, c["nsess"]) if c["nsess"] > 1 else None
    if c.get("rtcp"):
        arena, pos, end, cap = make_rtcp_arena(n, lengths)
    elif c.get("nssrc", 1) > 1:
        # one session, packet i on stream i mod nssrc (SSRC_BASE + k)
        arena, pos, end, cap = make_arena(
            n, lengths, s0=c["s0"],
            sess=np.arange(n, dtype=np.uint32) % c["nssrc"])
    else:
        arena, pos, end, cap = make_arena(n, lengths, s0=c["s0"], sess=sess)
    klen = KEY_LEN[c["suite"]]
    if c.get("key"):
        keys = np.frombuffer(c["key"], dtype=np.uint8).reshape(1, klen)
    else:
        keys = make_keys(c["nsess"], klen)
    return arena, pos, end, cap, sess, keys
