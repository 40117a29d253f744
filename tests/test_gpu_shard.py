"""Config 5 (one stream sharded over GPUs) on one GPU, through the C-ABI
library: a 2M-packet stream (seq from 65000, the ROC wraps 32 times) is
protected and unprotected in one call per direction by one context pair,
and separately as two 1M-packet shards -- shard 0 by fresh contexts, shard
1 by fresh contexts that srtp_stream_import() the state re_amd/shard.py
computes for the boundary (what bench.py --gpus N hands each rank).  The
shards must produce byte-identical arenas, identical per-packet errnos and
ends, and the same final exported stream states as the unsharded run.
"""
import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import shard as S
from re_amd import workload as W

pytestmark = pytest.mark.gpu

PER = 1 << 20
S0 = 65000


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def i32(torch, a):
    return torch.from_numpy(
        np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).cuda()


def run(torch, op, ctx, dev, pos, end, cap, a, b):
    """srtp_*_batch_dev over packets [a, b) of the arena"""
    n = b - a
    pos_d, end_d, cap_d = i32(torch, pos[a:b]), i32(torch, end[a:b]), \
        i32(torch, cap[a:b])
    err = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    rc = P.device_batch_dev(op, [ctx], dev.data_ptr(), dev.numel(),
                            pos_d.data_ptr(), end_d.data_ptr(),
                            cap_d.data_ptr(), err.data_ptr(), n)
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    end[a:b] = end_d.cpu().numpy().view(np.uint32)
    return err.cpu().numpy()


def state(ctx):
    e, st = ctx.export(W.SSRC_BASE)
    assert e == 0
    return (st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
            st.replay_rtp_bitmap)


def test_two_shards_equal_one_stream(torch_cuda):
    torch = torch_cuda
    n = 2 * PER
    arena, pos, end, cap = W.make_arena(n, 1200, s0=S0)
    key = W.make_keys(1, 30)[0].tobytes()
    one = torch.from_numpy(arena).cuda()
    two = one.clone()
    end1, end2 = end.copy(), end.copy()

    # unsharded: one context pair, one call per direction
    tx, rx = P.Srtp(1, key), P.Srtp(1, key)
    e1p = run(torch, "srtp_encrypt", tx, one, pos, end1, cap, 0, n)
    e1u = run(torch, "srtp_decrypt", rx, one, pos, end1, cap, 0, n)

    # sharded: rank r's contexts start from the closed-form boundary state
    errs, finals = [], []
    for r in range(2):
        a, b = r * PER, (r + 1) * PER
        assert (int(arena[pos[a] + 2]) << 8 | int(arena[pos[a] + 3])) == \
            S.shard_seq0(r, PER, S0)
        stx, srx = P.Srtp(1, key), P.Srtp(1, key)
        if r:
            for c, recv in ((stx, False), (srx, True)):
                assert c.import_(S.shard_state(r, PER, S0, W.SSRC_BASE,
                                               recv, P.StreamState)) == 0
        ep = run(torch, "srtp_encrypt", stx, two, pos, end2, cap, a, b)
        eu = run(torch, "srtp_decrypt", srx, two, pos, end2, cap, a, b)
        errs.append((ep, eu))
        finals.append((state(stx), state(srx)))
        stx.close()
        srx.close()

    assert not e1p.any() and not e1u.any()
    assert np.array_equal(np.concatenate([e[0] for e in errs]), e1p)
    assert np.array_equal(np.concatenate([e[1] for e in errs]), e1u)
    assert np.array_equal(end1, end2)
    assert torch.equal(one, two)
    # the last shard ends where the single stream ends
    assert finals[1] == (state(tx), state(rx))
    # and the closed form agrees with the exported unsharded state
    last = S.shard_state(2, PER, S0, W.SSRC_BASE, True)
    assert state(rx)[:2] == (last["roc"], last["s_l"])
    assert state(rx)[3:] == (last["replay_rtp_lix"],
                             last["replay_rtp_bitmap"])
    tx.close()
    rx.close()
