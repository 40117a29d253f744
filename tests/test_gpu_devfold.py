"""GPU parity of the device verdict fold (sgpu_fold_rtp, srtp.c dev_planned).

A device-planned single-stream unprotect speculates that every tag
verifies.  When some do not, the fold on the device decides whether the
speculation still holds under the true s_l (forged packets bump the ROC
but never set s_l: reference src/srtp/srtp.c:313-321, 358-359, 426-427)
and, if so, writes the EAUTH results, s_l and replay window without
re-running the batch; otherwise the call is undone and re-run on the host
engine.  Either way the results must be the reference's: every packet's
errno, pos/end and bytes, and the final stream state, are compared here
with the oracle called one packet at a time (tests/oracle_lib.py, pinned
to reference-generated goldens in tests/test_oracle.py).
"""

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_fastpath import keys_for, rtp_packet, run_dev, to_arena

pytestmark = pytest.mark.gpu

SSRC = 0x5151


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def protect(ob, suite, key, seqs, rng, plen=160):
    """protected packets of one stream (oracle sender)"""
    tx, e = ob.alloc(suite, key, 0)
    assert e == 0
    out = []
    for s in seqs:
        p = rtp_packet(rng, s & 0xffff, SSRC, plen=plen)
        r = ob.call(tx, "srtp_encrypt", len(p) + 64, 0, len(p), p, 0)
        assert r[0] == 0
        out.append(r[4][:r[2]])
    ob.free(tx)
    return out


def forge(pkts, idx, rng):
    pkts = list(pkts)
    for i in idx:
        q = bytearray(pkts[i])
        q[12 + int(rng.integers(0, len(q) - 12))] ^= 0x40
        pkts[i] = bytes(q)
    return pkts


def oracle_rx(ob, rx, pkts):
    res = []
    for p in pkts:
        r = ob.call(rx, "srtp_decrypt", len(p) + 64, 0, len(p), p, len(p))
        res.append((r[0], r[1], r[2], r[4][:len(p)]))
    return res


def check(torch, suite, key, batches, label):
    """batches: lists of protected packets, received in order by one rx
    context on the device and one in the oracle"""
    ob = O.OracleBackend()
    orx, e = ob.alloc(suite, key, 0)
    assert e == 0
    rx = P.Srtp(suite, key)
    try:
        for b, pkts in enumerate(batches):
            arena, pos, end, cap, _ = to_arena([(0, p) for p in pkts])
            da, dp, de, derr = run_dev(torch, "srtp_decrypt", [rx], arena,
                                       pos, end, cap, None)
            want = oracle_rx(ob, orx, pkts)
            for i, (err, wp, we, wb) in enumerate(want):
                got = (int(derr[i]), int(dp[i] - pos[i]), int(de[i] - pos[i]))
                assert got == (err, wp, we), (label, b, i, got, want[i][:3])
                assert da[pos[i]:end[i]].tobytes() == wb, (label, b, i)
            e, st = rx.export(SSRC)
            assert e == 0
            assert (st.roc, st.s_l, st.replay_rtp_lix,
                    st.replay_rtp_bitmap) == ob.export(orx, SSRC), (label, b)
    finally:
        rx.close()
        ob.free(orx)


def cases(rng, n=3000):
    base = list(range(65300, 65300 + n))            # ROC wrap at 236
    wrap = base.index(65536)
    mid = [1000, 20000, 40000] + list(range(40001, 40001 + 200))
    return {
        # (seqs, forged indices, expect a device fold)
        "one": (base, [700], True),
        "first": (base, [0], True),
        "last": (base, [n - 1], True),
        "all": (base, list(range(n)), True),
        "wrap": (base, [wrap], True),
        "wrap_next": (base, [wrap, wrap + 1], True),
        "sparse": (base, sorted(rng.choice(n, 5, replace=False).tolist()),
                   True),
        "window": (base, [n - 65, n - 64, n - 63, n - 2], True),
        # the forged packet carried the s_l the next one needs: ETIMEDOUT
        # under the true s_l -> the host folds
        "timeout": (mid, [1], False),
        # a forged packet hides a rollover's s_l: the next packet's
        # rollover differs -> the host folds
        "rollover": ([30000, 50000, 10] + list(range(11, 300)), [1], False),
    }


@pytest.mark.parametrize("suite", [0, 1, 3, 4, 5])
def test_device_fold_vs_oracle(suite, torch_cuda):
    rng = np.random.default_rng(123 + suite)
    key = keys_for(suite, 1)[0]
    ob = O.OracleBackend()
    for name, (seqs, bad, devfold) in cases(rng).items():
        pkts = forge(protect(ob, suite, key, seqs, rng), bad, rng)
        f0, h0 = P.counter("devfolds"), P.counter("folds")
        check(torch_cuda, suite, key, [pkts], name)
        if devfold:
            assert P.counter("devfolds") == f0 + 1, name
            assert P.counter("folds") == h0, name
        else:
            assert P.counter("folds") > h0, name
            assert P.counter("devfolds") == f0, name


@pytest.mark.parametrize("suite", [1, 4])
def test_device_fold_across_batches(suite, torch_cuda):
    """state after a folded batch (s_l, replay window built from the
    authentic packets only) is what the next batch starts from; a forged
    packet 0 of a fresh stream still sets s_l (stream.c:64-78)"""
    rng = np.random.default_rng(7 + suite)
    key = keys_for(suite, 1)[0]
    ob = O.OracleBackend()
    seqs = list(range(65400, 65400 + 900))
    pkts = protect(ob, suite, key, seqs, rng)
    b1 = forge(pkts[:300], [0, 299], rng)
    b2 = forge(pkts[300:590] + pkts[592:600], [10, 11, 250], rng)
    # late packets below the window's lix first (the host plans), then a
    # folded batch again
    b3 = [pkts[590], pkts[591], pkts[590]] + forge(pkts[600:], [5], rng)
    check(torch_cuda, suite, key, [b1, b2, b3], "batches")


@pytest.mark.parametrize("suite", [1])
def test_host_fold_knob_same_results(suite, torch_cuda):
    """RE_SRTP_NODEVFOLD (srtp_gpu_tune nodevfold): the host engine folds
    the same batches to the same results"""
    rng = np.random.default_rng(99)
    key = keys_for(suite, 1)[0]
    ob = O.OracleBackend()
    seqs = list(range(65300, 67300))
    pkts = forge(protect(ob, suite, key, seqs, rng), [3, 236, 1999], rng)
    f0 = P.counter("devfolds")
    with P.tune(nodevfold=1):
        check(torch_cuda, suite, key, [pkts], "nodevfold")
    assert P.counter("devfolds") == f0
