"""Multi-GPU sharding of one SRTP stream (BASELINE config 5).

Packets are independent once their index is known, so a stream of
world * n packets with monotone seq = (s0 + i) mod 2^16 shards into
contiguous ranges, one per rank, with no data collective: rank r starts
from the stream state the sequential reference would hold after packets
0 .. r*n-1 (src/srtp/srtp.c:203-213, 279-280 sender; 310-321, 426-427
receiver; src/srtp/replay.c:32-62 window), handed to its contexts with
srtp_stream_import().  RCCL (or gloo on CPU) only reduces the counters.
"""


def shard_state(rank, per_rank, s0, ssrc, receiver, state_cls=None):
    """Stream state after a sequential sender (receiver) processed packets
    0 .. rank*per_rank-1 with seq = (s0 + i) mod 2^16, starting from a
    fresh stream.  Returns a StreamState (re_amd.srtp) or a dict.

    Precondition (the only stream shape this closed form covers -- the
    config-5 workload, re_amd/workload.py): ONE SSRC, a fresh stream at
    packet 0, seq strictly +1 per packet (mod 2^16), every packet authentic
    and none lost.  Other shapes (several SSRCs, reordering, loss, forged
    packets) have no closed form: hand the state over with
    srtp_stream_export() of the previous shard's contexts instead, which
    serialises the shards.  tests/test_shard_cpu.py checks this function
    against a sequential model, tests/test_gpu_shard.py against the library.
    """
    if not (isinstance(rank, int) and isinstance(per_rank, int) and
            rank >= 0 and per_rank > 0 and 0 <= s0 <= 0xffff):
        raise ValueError("shard_state: rank >= 0, per_rank > 0, "
                         "0 <= s0 < 65536 (monotone single stream only)")
    k = rank * per_rank
    st = {"ssrc": ssrc, "roc": 0, "s_l": 0, "s_l_set": 0,
          "replay_rtp_lix": 0, "replay_rtp_bitmap": 0}
    if k:
        last = s0 + k - 1            # 48-bit index of the last packet
        st["roc"] = last >> 16
        st["s_l"] = last & 0xffff
        st["s_l_set"] = 1
        if receiver:
            st["replay_rtp_lix"] = last
            st["replay_rtp_bitmap"] = (1 << 64) - 1 if k >= 64 else \
                (1 << k) - 1
    if state_cls is None:
        return st
    o = state_cls()
    for f, v in st.items():
        setattr(o, f, v)
    return o


def session_rank(sess, world):
    """rank owning each session of a multi-session workload (SURVEY 8(e):
    shard by session id): the id modulo the world size.  Every packet of a
    session -- so every stream's ROC, s_l and replay state -- stays on one
    rank, with no hand-off; the generated ids are uniform, so ranks get
    equal shares."""
    import numpy as np
    if world < 1:
        raise ValueError("session_rank: world >= 1")
    return (np.asarray(sess, dtype=np.uint64) %
            np.uint64(world)).astype(np.int64)


def shard_sessions(sess, world, rank):
    """rank's shard of a multi-session workload: (global indices of its
    packets in arrival order, their dense local session ids
    global // world).  Local id k is global session k * world + rank."""
    import numpy as np
    sess = np.asarray(sess)
    mine = np.flatnonzero(session_rank(sess, world) == rank)
    return mine, (sess[mine] // world).astype(np.uint32)


def shard_seq0(rank, per_rank, s0):
    """first sequence number of rank's shard"""
    return (s0 + rank * per_rank) & 0xffff


def reduce_results(dist, counters, elapsed):
    """whole-job counters (sum over ranks) and step time (max over ranks)
    -- the only collectives of the sharded run.  counters / elapsed are
    torch tensors on the rank's device (float64)."""
    if dist is not None and dist.is_initialized() and \
            dist.get_world_size() > 1:
        cpu = dist.get_backend() == "gloo" and counters.is_cuda
        c = counters.cpu() if cpu else counters
        e = elapsed.cpu() if cpu else elapsed
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        if cpu:
            counters.copy_(c)
            elapsed.copy_(e)
    return counters, elapsed
