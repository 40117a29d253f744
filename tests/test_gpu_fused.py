"""Single-stream batches planned by the decoupled look-back plan of
k_ctr_fused.h (parse, every check, the ROC prefix over 1024-packet
workgroups), in its two forms:

  fused   the AES-CM default: the plan inside the crypto launch
          (k_ctr_fused, host dev_fused);
  lplan   the plan as a launch of its own (k_lp_plan, host lp_issue /
          lp_finish) in front of the lean crypto kernel -- AES-GCM always,
          AES-CM with srtp_gpu_tune lplan (k_ctr_fast_any);
  *_copy  either with the plan out brought back by a blit copy
          (srtp_gpu_tune nopost) instead of the k_plan_post launch.

Both must give exactly the separate device planner's results
(srtp_gpu_tune noplanfuse: k_parse + k_plan_* + the lean kernel, pinned by
the reference digests in earlier rounds) and the general engine's: arena,
pos, end, errno and stream state -- for batches the plan accepts and for
every rejection, wherever in the batch the broken assumption sits (first,
middle or last workgroup), which each path must leave undone before the
host re-plans (srtp.c:183-432, misc.c:22-41, replay.c:32-62 of the
reference).
"""
import numpy as np
import pytest

import re_amd.srtp as P
from tests.test_gpu_fastpath import keys_for, rtp_packet, run_dev, states, \
    to_arena

pytestmark = pytest.mark.gpu

SSRC = 0x5151
N = 5000                # five workgroups of 1024 packets


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def batch(rng, seqs, ssrc_at=(), csrc_at=(), short_at=(), plen=64):
    out = []
    for i, s in enumerate(seqs):
        pkt = rtp_packet(rng, s & 0xffff, 0x7777 if i in ssrc_at else SSRC,
                         cc=1 if i in csrc_at else 0, plen=plen)
        if i in short_at:
            pkt = pkt[:7]
        out.append((0, pkt))
    return out


def cases(s0):
    base = list(range(s0, s0 + N))
    mid, last = 2600, N - 3
    return {
        "inorder": (base, {}),
        "reorder_first": (base[:5] + [base[6], base[5]] + base[7:], {}),
        "reorder_mid": (base[:mid] + [base[mid + 1], base[mid]] +
                        base[mid + 2:], {}),
        "reorder_last": (base[:last] + [base[last + 1], base[last]] +
                         base[last + 2:], {}),
        "replay_mid": (base[:mid] + [base[mid - 10]] + base[mid + 1:], {}),
        "jump_last": (base[:last] + [base[last] + 40000] + base[last + 1:],
                      {}),
        "class_mid": (base, {"csrc_at": (mid,)}),
        "ssrc_last": (base, {"ssrc_at": (N - 1,)}),
        "short_mid": (base, {"short_at": (mid,)}),
    }


GCM = (4, 5)


def modes(suite):
    """(mode, tune knobs, the counter its accepted plans move)"""
    m = [("lplan", {"lplan": 1}, "lplans"),
         # the plan out back by a blit copy instead of the post launch
         ("lplan_copy", {"lplan": 1, "nopost": 1}, "lplans")]
    if suite not in GCM:
        m.append(("fused", {}, "fused"))
        m.append(("fused_copy", {"nopost": 1}, "fused"))
        # waited for by the post's completion word, not the stream
        m.append(("fused_spin", {"syncspin": 1}, "fused"))
    return m + [("planner", {"noplanfuse": 1}, None),
                ("general", {"general": 1}, None)]


PLANNED = ("lplan", "fused", "lplan_copy", "fused_copy", "fused_spin")


def run_modes(torch, suite, key, op, pkts, state_from=None, cap_short=()):
    """the batch through the one-launch plan, the fused path, the separate
    planner and the general engine; returns {mode: (outputs, state,
    (accepted plans of the mode's kind, rejects))}"""
    arena, pos, end, cap, _ = to_arena(pkts, short_cap=cap_short)
    res = {}
    for mode, tune, cname in modes(suite):
        ctx = P.Srtp(suite, key)
        if state_from is not None:
            assert ctx.import_(state_from) == 0
        f0 = P.counter(cname) if cname else 0
        r0 = P.counter("rejects")
        # every mode from the same first-batch hint (a rejected plan for a
        # second SSRC of a fresh session sets it, re_srtp_batch.h)
        P.lib().srtp_gpu_tune(b"freshmulti", 0)
        with P.tune(**tune):
            out = run_dev(torch, op, [ctx], arena, pos, end, cap, None)
        res[mode] = (out, states([ctx], [SSRC]),
                     ((P.counter(cname) - f0) if cname else 0,
                      P.counter("rejects") - r0))
        ctx.close()
    return res


def same(res, name):
    for a in PLANNED:
        if a not in res:
            continue
        A = res[a]
        for mode in ("planner", "general"):
            B = res[mode]
            for k, (x, y) in enumerate(zip(A[0], B[0])):
                assert (x == y).all(), (name, a, mode,
                                        ("arena", "pos", "end", "err")[k])
            assert A[1] == B[1], (name, a, mode, A[1], B[1])


def planned(res, want, name):
    for a in PLANNED:
        if a in res:
            assert res[a][2] == want, (name, a, res[a][2])


@pytest.mark.parametrize("suite", [1, 0, 2, 4, 5])
@pytest.mark.parametrize("s0", [65000, 100])
def test_fused_equals_planner_and_general(suite, s0, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(1000 + suite + s0)
    key = keys_for(suite, 1)[0]
    for name, (seqs, kw) in cases(s0).items():
        pkts = batch(rng, seqs, **kw)
        res = run_modes(torch, suite, key, "srtp_encrypt", pkts)
        same(res, name + "/protect")
        # a forward jump of 40000 is only ETIMEDOUT for the receiver
        accepted = name in ("inorder", "jump_last")
        planned(res, (1, 0) if accepted else (0, 1), name)
        # receive what the accepted protect produced (in-order stream),
        # with the same defect injected on the protected packets
        out = res["lplan"][0]
        prot = [(0, out[0][out[1][i]:out[2][i]].tobytes())
                for i in range(len(pkts)) if out[3][i] == 0]
        if name == "reorder_mid":
            prot = prot[:2600] + [prot[2601], prot[2600]] + prot[2602:]
        elif name == "replay_mid":
            prot = prot[:2600] + [prot[2590]] + prot[2601:]
        dres = run_modes(torch, suite, key, "srtp_decrypt", prot)
        same(dres, name + "/unprotect")


@pytest.mark.parametrize("suite", [1, 2, 5])
def test_fused_forged_packets_fold_on_device(suite, torch_cuda):
    """forged packets in several workgroups: the crypto launch counts the
    misses, the host then restores their ciphertext (AES-CM) and folds the
    verdicts on the device (no rejection)"""
    torch = torch_cuda
    rng = np.random.default_rng(33 + suite)
    key = keys_for(suite, 1)[0]
    seqs = list(range(65500, 65500 + N))
    pkts = batch(rng, seqs)
    res = run_modes(torch, suite, key, "srtp_encrypt", pkts)
    same(res, "protect")
    out = res["lplan"][0]
    prot = [(0, out[0][out[1][i]:out[2][i]].tobytes())
            for i in range(len(pkts))]
    for forged in ([17], [36], [3, 1500, 4096, N - 1], list(range(0, N, 97))):
        q = list(prot)
        for i in forged:
            b = bytearray(q[i][1])
            b[20] ^= 0x10
            q[i] = (0, bytes(b))
        dres = run_modes(torch, suite, key, "srtp_decrypt", q)
        same(dres, "forged %d" % len(forged))
        errs = dres["lplan"][0][3]
        assert (errs[forged] == P.EAUTH).all()
        planned(dres, (1, 0), "forged")


def test_fused_short_capacity_and_continuation(torch_cuda):
    """protect with one packet short of tag room (ENOMEM on the host
    re-plan) in the last workgroup, then a second batch continuing the
    stream from the first one's state (the fused path's state update)"""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    key = keys_for(1, 1)[0]
    seqs = list(range(65530, 65530 + N))
    pkts = batch(rng, seqs)
    res = run_modes(torch, 1, key, "srtp_encrypt", pkts, cap_short=(N - 2,))
    same(res, "short cap")
    assert res["lplan"][0][3][N - 2] != 0
    # two accepted batches back to back on one context, against one
    # batch of both through the separate planner
    a, b = batch(rng, seqs[:2100]), batch(rng, seqs[2100:])
    ctx = P.Srtp(1, key)
    outs = []
    for part in (a, b):
        ar, pos, end, cap, _ = to_arena(part)
        outs.append(run_dev(torch, "srtp_encrypt", [ctx], ar, pos, end, cap,
                            None))
    st = states([ctx], [SSRC])
    ctx.close()
    ref = P.Srtp(1, key)
    with P.tune(noplanfuse=1):
        routs = []
        for part in (a, b):
            ar, pos, end, cap, _ = to_arena(part)
            routs.append(run_dev(torch, "srtp_encrypt", [ref], ar, pos, end,
                                 cap, None))
    assert states([ref], [SSRC]) == st
    ref.close()
    for x, y in zip(outs, routs):
        for u, v in zip(x, y):
            assert (u == v).all()


def test_fused_many_launches_sizes_and_epoch_wrap(torch_cuda):
    """one stream continued over many fused launches of every workgroup
    shape (1 packet, a partial, exactly one, one past, several) -- the
    ticket base, the double-buffered plan out and the look-back epoch move
    on every launch -- and across the epoch's wrap (the host zeroes the
    look-back words and counters, srtp_gpu_tune fzepoch starts it just
    short of 0xffff): every batch equal to the separate planner's, and the
    final stream state too"""
    torch = torch_cuda
    rng = np.random.default_rng(77)
    key = keys_for(1, 1)[0]
    sizes = [1, 2, 1023, 1024, 1025, 3000, 1, 700, 2049, 5]
    seq = 65400
    parts = []
    for n in sizes:
        parts.append(batch(rng, list(range(seq, seq + n))))
        seq += n
    outs = {}
    for mode, tune, cname in (("lplan", {"lplan": 1}, "lplans"),
                              ("fused", {}, "fused"),
                              ("planner", {"noplanfuse": 1}, "dplans")):
        ctx = P.Srtp(1, key)
        res = []
        f0 = P.counter(cname)
        with P.tune(**tune):
            for k, part in enumerate(parts):
                if mode != "planner" and k == 3:
                    P.lib().srtp_gpu_tune(b"fzepoch", 0xfffe)
                ar, pos, end, cap, _ = to_arena(part)
                res.append(run_dev(torch, "srtp_encrypt", [ctx], ar, pos,
                                   end, cap, None))
        outs[mode] = (res, states([ctx], [SSRC]), P.counter(cname) - f0)
        ctx.close()
    for mode in ("lplan", "fused", "planner"):
        assert outs[mode][2] == len(sizes), mode
    for mode in ("lplan", "fused"):
        assert outs[mode][1] == outs["planner"][1]
        for x, y in zip(outs[mode][0], outs["planner"][0]):
            for u, v in zip(x, y):
                assert (u == v).all()
