"""Full-size parity at BASELINE.json's sizes, through the C-ABI library
(srtp_*_batch_dev, every array in HBM):

  config 2  AES_CM_128_HMAC_SHA1_80, 1M x 1200-B packets, one stream
  config 3  AEAD_AES_256_GCM,        1M x 1200-B packets, one stream
  config 4  AES_CM_128_HMAC_SHA1_80, 1M packets of 200/1400 B over 64K
            sessions

The oracle is sequential and slow at 1M packets, so full size is checked
through size-independent properties plus a sample:
  * protect: every result code 0 and every end grown by the tag; a sample
    of packets (both sides of the ROC wrap at packet 536, the last packet,
    random others) equals the oracle's srtp_encrypt of the same packet
    with the same ROC -- the oracle context is walked to that ROC with
    header-only packets (a seq drop of 32768 or more is a rollover,
    src/srtp/srtp.c:207-210);
  * unprotect of the whole protected batch: every result 0, every end back
    to the plaintext end, every plaintext byte equal to the input
    (round trip over all 1.2 GB);
  * final stream states (ROC, s_l, replay index) equal the closed form of
    the sequential reference after n packets.
"""
import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import workload as W
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

N = 1 << 20
S0 = 65000


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def oracle_protect(be, suite, key, pkt, roc):
    """srtp_encrypt of pkt by an oracle sender whose ROC is roc"""
    ctx = be.alloc(suite, key, 0)[0]
    for _ in range(roc):
        for s in (40000, 0):
            h = bytearray(pkt[:12])
            h[2], h[3] = s >> 8, s & 0xff
            e = be.call(ctx, "srtp_encrypt", 128, 0, 12, bytes(h), 0)[0]
            assert e == 0
    e, _, en, _, buf = be.call(ctx, "srtp_encrypt", len(pkt) + 64, 0,
                               len(pkt), pkt, len(pkt) + 16)
    be.free(ctx)
    assert e == 0
    return buf[:en]


def run_dev(torch, opname, sessions, arena_d, pos_d, end_d, cap_d, sess_d,
            n):
    err = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    rc = P.device_batch_dev(opname, sessions, arena_d.data_ptr(),
                            arena_d.numel(), pos_d.data_ptr(),
                            end_d.data_ptr(), cap_d.data_ptr(),
                            err.data_ptr(), n,
                            sess_d.data_ptr() if sess_d is not None
                            else None)
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    return err


def i32(torch, a):
    return torch.from_numpy(
        np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).cuda()


def check_batch(torch, suite, lengths, nsess, nsample):
    klen = P.key_len(suite) + P.salt_len(suite)
    tag = P.tag_len(suite)
    keys = W.make_keys(nsess, klen)
    sess = W.random_sessions(N, nsess) if nsess > 1 else None
    arena, pos, end, cap = W.make_arena(N, lengths, s0=S0, sess=sess)
    slot = int(cap[0] - pos[0])
    plain = torch.from_numpy(arena).cuda()
    dev = plain.clone()
    pos_d, end_d, cap_d = i32(torch, pos), i32(torch, end), i32(torch, cap)
    sess_d = i32(torch, sess) if sess is not None else None
    if nsess > 1:
        e1, tx = P.alloc_many(nsess, suite, keys.tobytes())
        e2, rx = P.alloc_many(nsess, suite, keys.tobytes())
        assert not e1 and not e2
    else:
        tx, rx = [P.Srtp(suite, keys[0].tobytes())], \
                 [P.Srtp(suite, keys[0].tobytes())]

    # ---- protect: results, ends, sample vs the oracle ----
    err = run_dev(torch, "srtp_encrypt", tx, dev, pos_d, end_d, cap_d,
                  sess_d, N)
    assert int(torch.count_nonzero(err)) == 0
    ends = end_d.cpu().numpy().view(np.uint32)
    assert (ends == end + tag).all()
    prot = dev.cpu().numpy()
    rng = np.random.default_rng(4242 + suite + nsess)
    idx = sorted(set([0, 1, 535, 536, 537, N - 1] +
                     rng.integers(0, N, size=nsample).tolist()))
    if sess is not None:      # per-session seq: ordinal within its session
        seqs = ((arena.reshape(N, slot)[:, 2].astype(np.uint32) << 8) |
                arena.reshape(N, slot)[:, 3])
    be = O.OracleBackend()
    for i in idx:
        pkt = arena[pos[i]:end[i]].tobytes()
        if sess is None:
            roc = (S0 + i) >> 16
            key = keys[0].tobytes()
        else:
            roc = 0           # every session stays below the wrap
            assert int(seqs[i]) >= S0
            key = keys[int(sess[i])].tobytes()
        ref = oracle_protect(be, suite, key, pkt, roc)
        assert prot[pos[i]:ends[i]].tobytes() == ref, i

    # ---- unprotect of the whole batch: round trip over every byte ----
    err = run_dev(torch, "srtp_decrypt", rx, dev, pos_d, end_d, cap_d,
                  sess_d, N)
    assert int(torch.count_nonzero(err)) == 0
    assert (end_d.cpu().numpy().view(np.uint32) == end).all()
    L = torch.from_numpy(np.asarray(end - pos, dtype=np.int64)).cuda()
    col = torch.arange(slot, device="cuda")[None, :]
    mask = col < L[:, None]
    diff = (dev.view(N, slot) != plain.view(N, slot)) & mask
    assert int(torch.count_nonzero(diff)) == 0

    # ---- final stream states (closed form of the sequential reference) --
    if sess is None:
        last = S0 + N - 1
        for ctx, is_rx in ((tx[0], False), (rx[0], True)):
            e, st = ctx.export(W.SSRC_BASE)
            assert e == 0
            assert (st.roc, st.s_l) == (last >> 16, last & 0xffff)
            if is_rx:
                assert st.replay_rtp_lix == last
    else:
        counts = np.bincount(sess.astype(np.int64), minlength=nsess)
        for s in rng.integers(0, nsess, size=64).tolist():
            if not counts[s]:
                continue
            last = S0 + int(counts[s]) - 1
            for ctx, is_rx in ((tx[s], False), (rx[s], True)):
                e, st = ctx.export(W.SSRC_BASE + s)
                assert e == 0
                assert (st.roc, st.s_l) == (last >> 16, last & 0xffff)
                if is_rx:
                    assert st.replay_rtp_lix == last
    for c in tx + rx:
        c.close()


def test_config2_full_size(torch_cuda):
    check_batch(torch_cuda, 1, 1200, 1, 300)


def test_config3_full_size(torch_cuda):
    check_batch(torch_cuda, 5, 1200, 1, 300)


def test_config4_full_size(torch_cuda):
    check_batch(torch_cuda, 1, W.mixed_lengths(N), 65536, 300)
