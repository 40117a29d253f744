"""The four-launch multi-session planner (plan_buckets.hip, srtpgpu.h
struct sgpu_bplan) against the counting-grouping planner it replaces
(plan_multi.hip, srtp_gpu_tune nobucket) and the general engine (pinned to
the reference by the golden replays), through srtp_*_batch_dev:

  * many sessions of random in-order traffic, two consecutive batches with
    ROC rollovers inside, AES-CM/HMAC and AES-GCM, with and without forged
    packets (the verdict fold in k_bp_finish: EAUTH, post-error bytes,
    s_l and replay windows of the touched sessions);
  * bucket geometries: sessions not a multiple of the bucket width, empty
    sessions and empty buckets, one session per bucket;
  * a bucket over its capacity and a session over SGPU_BP_SEGMAX in one
    bucket: SPF_SEG, the radix-sort re-plan;
  * a forged packet the fold must reject (its s_l carried the next
    packets' estimate): the host folds.

Every case compares whole arenas, pos, end, errno and every session's
exported state, and asserts which planner ran (srtp_gpu_counter "mplans",
"rejects", "devfolds", "folds").  The reference semantics are
src/srtp/srtp.c:183-432 per session, sessions independent."""
import errno

import numpy as np
import pytest

import re_amd.srtp as P
from tests.test_gpu_fastpath import keys_for, rtp_packet, run, run_dev, \
    to_arena

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def traffic(rng, n, owner_p, s0, last=None, plen=(0, 400)):
    """n packets; session of each drawn from owner_p (probabilities);
    per-session seq continues `last` (or starts at s0[s])"""
    last = {} if last is None else last
    owners = rng.choice(len(owner_p), size=n, p=owner_p)
    out = []
    for s in owners.tolist():
        seq = (last[s] + 1) & 0xffff if s in last else s0[s]
        last[s] = seq
        out.append((s, rtp_packet(rng, seq, 0x7000 + s,
                                  plen=int(rng.integers(*plen)))))
    return out, last


def forge(prot, idx):
    out = list(prot)
    for i in idx:
        q = bytearray(out[i][1])
        q[-1] ^= 0x20                   # the tag's last byte
        out[i] = (out[i][0], bytes(q))
    return out


COUNTERS = ("mplans", "rejects", "devfolds", "folds")


def states(sessions):
    """session s's stream state (its one SSRC, 0x7000 + s)"""
    out = []
    for k, s in enumerate(sessions):
        e, st = s.export(0x7000 + k)
        out.append((e,) if e else (st.roc, st.s_l, st.s_l_set,
                                   st.replay_rtp_bitmap, st.replay_rtp_lix))
    return out


def counters():
    return {c: P.counter(c) for c in COUNTERS}


def run_modes(torch, suite, nsess, batches, forged=None, modes=None):
    """run every batch (protect, then unprotect with the forged packets of
    forged[bi]) in each mode; returns {mode: (outs, tx states, rx states,
    counter deltas per call)}"""
    keys = keys_for(suite, nsess)
    res = {}
    for mode in modes or ("bucket", "count", "general"):
        # bucket_copy: the outcome back by a blit copy, not by k_bp_finish
        knobs = ({"nobucket": 1} if mode == "count" else
                 {"nopost": 1} if mode == "bucket_copy" else {})
        tx = [P.Srtp(suite, k) for k in keys]
        rx = [P.Srtp(suite, k) for k in keys]
        outs, deltas = [], []
        with P.tune(**knobs):
            for bi, pk in enumerate(batches):
                arena, pos, end, cap, sess = to_arena(pk)
                c0 = counters()
                if mode == "general":
                    enc = run(torch, "srtp_encrypt", tx, arena, pos, end, cap,
                              sess, True)
                else:
                    enc = run_dev(torch, "srtp_encrypt", tx, arena, pos, end,
                                  cap, sess)
                c1 = counters()
                prot = [(s, enc[0][pos[i]:enc[2][i]].tobytes())
                        for i, (s, _) in enumerate(pk)]
                if forged and forged.get(bi):
                    prot = forge(prot, forged[bi])
                a2, p2, e2, c2, s2 = to_arena(prot)
                if mode == "general":
                    dec = run(torch, "srtp_decrypt", rx, a2, p2, e2, c2, s2,
                              True)
                else:
                    dec = run_dev(torch, "srtp_decrypt", rx, a2, p2, e2, c2,
                                  s2)
                c2_ = counters()
                outs.append((enc, dec))
                deltas.append(({k: c1[k] - c0[k] for k in COUNTERS},
                               {k: c2_[k] - c1[k] for k in COUNTERS}))
        res[mode] = (outs, states(tx), states(rx), deltas)
        for c in tx + rx:
            c.close()
    ref = res["general"]
    for mode, got in res.items():
        if mode == "general":
            continue
        for bi, ((ea, da), (eb, db)) in enumerate(zip(got[0], ref[0])):
            for name, x, y in zip(("arena", "pos", "end", "err") * 2,
                                  ea + da, eb + db):
                assert (x == y).all(), (mode, bi, name)
        assert got[1] == ref[1], (mode, "tx states")
        assert got[2] == ref[2], (mode, "rx states")
    return res


@pytest.mark.parametrize("suite", [1, 5])
@pytest.mark.parametrize("frac", [0.0, 0.002, 0.03])
def test_bucket_planner_many_sessions(suite, frac, torch_cuda):
    """600 sessions (5 buckets of 128, the last part-full), 2 x 12000
    packets with ROC rollovers inside; forged packets scattered over the
    second batch's unprotect (not at a rollover: the fold keeps them)"""
    rng = np.random.default_rng(int(frac * 1000) + 31 * suite)
    nsess = 600
    s0 = [int(x) for x in rng.integers(65400, 65536, nsess)]
    p = np.full(nsess, 1.0 / nsess)
    b1, last = traffic(rng, 12000, p, s0)
    b2, _ = traffic(rng, 12000, p, s0, last)
    forged = {}
    if frac:
        cand = [i for i, (_, q) in enumerate(b2) if q[2:4] != b"\x00\x00"]
        forged[1] = sorted(rng.choice(cand, max(1, int(frac * len(b2))),
                                      replace=False).tolist())
    res = run_modes(torch_cuda, suite, nsess, [b1, b2], forged,
                    ("bucket", "bucket_copy", "count", "general"))
    d = res["bucket"][3]
    assert res["bucket_copy"][3] == d
    for bi in range(2):
        assert d[bi][0] == {"mplans": 1, "rejects": 0, "devfolds": 0,
                            "folds": 0}, d
    assert d[0][1] == {"mplans": 1, "rejects": 0, "devfolds": 0, "folds": 0}
    assert d[1][1] == {"mplans": 1, "rejects": 0,
                       "devfolds": 1 if frac else 0, "folds": 0}, d
    err = res["bucket"][0][1][1][3]
    assert set(np.flatnonzero(err).tolist()) == set(forged.get(1, []))
    assert all(int(err[i]) == P.EAUTH for i in forged.get(1, []))


@pytest.mark.parametrize("suite", [1, 4])
@pytest.mark.parametrize("shape", ["sparse", "narrow", "wide"])
def test_bucket_geometries(suite, shape, torch_cuda):
    """sparse: 1000 sessions, a third of them silent (empty sessions and
    an empty bucket); narrow: 5000 packets over 70 sessions (buckets of
    fewer sessions); wide: 6000 sessions, two packets each on average
    (bucket width 256, 24 buckets); each with a few forged packets"""
    rng = np.random.default_rng({"sparse": 1, "narrow": 2, "wide": 3}[shape]
                                + 10 * suite)
    nsess, n = {"sparse": (1000, 9000), "narrow": (70, 5000),
                "wide": (6000, 12000)}[shape]
    p = np.ones(nsess)
    if shape == "sparse":
        p[rng.choice(nsess, nsess // 3, replace=False)] = 0
        p[256:512] = 0                  # bucket 1 empty
    p /= p.sum()
    s0 = [int(x) for x in rng.integers(0, 65536, nsess)]
    b1, _ = traffic(rng, n, p, s0, plen=(0, 200))
    cand = [i for i, (_, q) in enumerate(b1) if q[2:4] != b"\x00\x00"]
    forged = {0: sorted(rng.choice(cand, 5, replace=False).tolist())}
    res = run_modes(torch_cuda, suite, nsess, [b1], forged,
                    modes=("bucket", "general"))
    d = res["bucket"][3][0]
    assert d[0]["mplans"] == 1 and d[0]["rejects"] == 0, d
    assert d[1] == {"mplans": 1, "rejects": 0, "devfolds": 1, "folds": 0}, d


@pytest.mark.parametrize("suite", [1, 5])
def test_bucket_overflow_and_hot_session_replan(suite, torch_cuda):
    """batch 0: one session carries 1500 of 3000 packets (over
    SGPU_BP_SEGMAX in its bucket: SPF_SEG); batch 1: 9000 of 12000 packets
    fall on the first 64 of 512 sessions (the first bucket over its
    capacity: SPF_SEG).  Both re-planned by the radix grouping, equal to
    the general engine; batch 2 is uniform again and takes the buckets"""
    rng = np.random.default_rng(808 + suite)
    nsess = 512
    s0 = [65000] * nsess
    p0 = np.full(nsess, 0.5 / (nsess - 1))
    p0[0] = 0.5
    b0, last = traffic(rng, 3000, p0, s0)
    p1 = np.full(nsess, 0.25 / (nsess - 64))
    p1[:64] = 0.75 / 64
    b1, last = traffic(rng, 12000, p1, s0, last)
    b2, _ = traffic(rng, 6000, np.full(nsess, 1.0 / nsess), s0, last)
    res = run_modes(torch_cuda, suite, nsess, [b0, b1, b2],
                    modes=("bucket", "general"))
    d = res["bucket"][3]
    for bi in (0, 1):
        for dr in range(2):
            assert d[bi][dr]["rejects"] == 1 and \
                d[bi][dr]["mplans"] == 1, (bi, d)
    assert d[2][0]["rejects"] == 0 and d[2][1]["rejects"] == 0, d


def test_bucket_fold_rejected_falls_back(torch_cuda):
    """a forged packet whose s_l the next packets of its session depend
    on (as tests/test_gpu_mfold.py): session 0 sends 100, 101, 32869
    (forged), 32870, 32871; the reference gives ETIMEDOUT for the last two
    (srtp.c:313-315) -- the bucket fold rejects, the host folds"""
    rng = np.random.default_rng(5)
    nsess = 300
    pk = [(0, rtp_packet(rng, seq, 0x7000, plen=100))
          for seq in (100, 101, 101 + 32768, 101 + 32769, 101 + 32770)]
    for s in range(1, nsess):
        for q in range(3):
            pk.append((s, rtp_packet(rng, 500 + q, 0x7000 + s, plen=50)))
    res = run_modes(torch_cuda, 1, nsess, [pk], {0: [2]},
                    modes=("bucket", "general"))
    err = res["bucket"][0][0][1][3]
    assert {int(i): int(err[i]) for i in np.flatnonzero(err)} == \
        {2: P.EAUTH, 3: errno.ETIMEDOUT, 4: errno.ETIMEDOUT}
    d = res["bucket"][3][0][1]
    # the device fold gave up (one host fold), the host engine folded
    # (it counts its own)
    assert d["mplans"] == 1 and d["folds"] >= 1 and d["devfolds"] == 0, d
