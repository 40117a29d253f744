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


# ---- cross-rank replay fold --------------------------------
#
# When one stream's unprotect is split across ranks and its shape has no
# closed form (loss, reordering, replays or forged packets across a shard
# boundary), each rank unprotects its shard from an assumed boundary state,
# records per packet what its receiver did (16 B: index, result, seq,
# stage), the ranks all-gather the records, and every rank replays the
# reference receiver over the whole stream (srtp_rx_fold): one all-gather
# of 16 B per packet (16 MB per 1M) is the only data collective.

def _rx_rec_dtype():
    import numpy as np
    # struct srtp_rx_rec (include/re_srtp_batch.h)
    return np.dtype([("ix", "<u8"), ("res", "<i4"), ("seq", "<u2"),
                     ("stage", "u1"), ("pad", "u1")])


def rx_records(st0, arena, pos, end, res):
    """the rank's records (srtp_rx_index): arena a host uint8 array,
    pos/end uint32 arrays, res the int32 results of the rank's decrypt call,
    st0 the StreamState it imported before the call."""
    import ctypes
    import numpy as np
    from . import srtp as S
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    pos = np.ascontiguousarray(pos, dtype=np.uint32)
    end = np.ascontiguousarray(end, dtype=np.uint32)
    res = np.ascontiguousarray(res, dtype=np.int32)
    n = len(pos)
    if len(end) != n or len(res) != n:
        raise ValueError("rx_records: pos, end and res differ in length")
    if n and int(end.max()) > arena.size:
        raise ValueError("rx_records: end beyond the arena")
    rec = np.zeros(n, dtype=_rx_rec_dtype())
    e = S.lib().srtp_rx_index(ctypes.byref(st0), arena.ctypes.data,
                              pos.ctypes.data, end.ctypes.data,
                              res.ctypes.data, n, rec.ctypes.data)
    if e:
        raise OSError(e, "srtp_rx_index")
    return rec


def rx_records_dev(st0, arena, pos, end, res, stream=None, out=None):
    """the rank's records from its DEVICE outputs (srtp_rx_index_dev): arena
    a torch uint8 CUDA tensor, pos/end/res int32 CUDA tensors of the rank's
    srtp_decrypt_batch_dev call (the arena never leaves the device); out: a
    record array of that length to fill (else a new one)"""
    import ctypes
    import numpy as np
    from . import srtp as S
    n = int(pos.numel())
    if int(end.numel()) != n or int(res.numel()) != n:
        raise ValueError("rx_records_dev: pos, end and res differ in length")
    rec = np.zeros(n, dtype=_rx_rec_dtype()) if out is None else out
    if rec.dtype != _rx_rec_dtype() or len(rec) != n or \
            not rec.flags["C_CONTIGUOUS"]:
        raise ValueError("rx_records_dev: out is not n contiguous records")
    e = S.lib().srtp_rx_index_dev(ctypes.byref(st0), arena.data_ptr(),
                                  arena.numel(), pos.data_ptr(),
                                  end.data_ptr(), res.data_ptr(), n,
                                  rec.ctypes.data, stream)
    if e:
        raise OSError(e, "srtp_rx_index_dev")
    return rec


def rx_fold(st, suite, rec):
    """fold the whole stream's records from StreamState st (the true state
    before its first packet; updated in place).  Returns (err int32 array
    of the packets folded, ndone): ndone < len(rec) when packet ndone was
    authenticated at an index its rank's boundary state got wrong -- re-run
    packets ndone.. from st."""
    import ctypes
    import numpy as np
    from . import srtp as S
    rec = np.ascontiguousarray(rec, dtype=_rx_rec_dtype())
    err = np.zeros(len(rec), dtype=np.int32)
    nd = ctypes.c_size_t(0)
    e = S.lib().srtp_rx_fold(ctypes.byref(st), suite, rec.ctypes.data,
                             len(rec), err.ctypes.data, ctypes.byref(nd))
    if e:
        raise OSError(e, "srtp_rx_fold")
    return err[:nd.value], nd.value


def gather_records(dist, rec):
    """all-gather every rank's records in rank order (shards are
    contiguous, so rank order is arrival order); ranks may hold different
    counts.  One all_gather of the counts, one of the padded records."""
    import numpy as np
    import torch
    if dist is None or not dist.is_initialized() or \
            dist.get_world_size() == 1:
        return rec
    world = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend() == "nccl" else torch.device("cpu")
    cnt = torch.tensor([len(rec)], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    cnts = [int(c.item()) for c in cnts]
    m = max(cnts)
    raw = np.zeros(m * rec.dtype.itemsize, dtype=np.uint8)
    raw[:rec.nbytes] = rec.view(np.uint8)
    t = torch.from_numpy(raw).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    parts = [o.cpu().numpy()[:c * rec.dtype.itemsize].view(rec.dtype)
             for o, c in zip(outs, cnts)]
    return np.concatenate(parts)
