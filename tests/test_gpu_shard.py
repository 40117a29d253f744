"""Config 5 (one stream sharded over GPUs) on one GPU, through the C-ABI
library: a 2M-packet stream (seq from 65000, the ROC wraps 32 times) is
protected and unprotected in one call per direction by one context pair,
and separately as two 1M-packet shards -- shard 0 by fresh contexts, shard
1 by fresh contexts that srtp_stream_import() the state re_amd/shard.py
computes for the boundary (what bench.py --gpus N hands each rank).  The
shards must produce byte-identical arenas, identical per-packet errnos and
ends, and the same final exported stream states as the unsharded run --
and both must equal the reference itself: whole-arena, end, errno and
final-state digests of the reference src/srtp over the same 2M-packet
stream after each direction (tests/golden/fullsize_digests.json shape 5,
oracle/ref_digest.c).
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


def run(torch, op, ctx, dev, pos, end, cap, a, b, pos_out=None):
    """srtp_*_batch_dev over packets [a, b) of the arena (the windows
    after the call: end in place, pos into pos_out)"""
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
    if pos_out is not None:
        pos_out[a:b] = pos_d.cpu().numpy().view(np.uint32)
    return err.cpu().numpy()


def state(ctx):
    e, st = ctx.export(W.SSRC_BASE)
    assert e == 0
    return (st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
            st.replay_rtp_bitmap)


def test_two_shards_equal_one_stream(torch_cuda):
    from tests import fullsize_util as F
    torch = torch_cuda
    ref = F.load()[5]
    n = 2 * PER
    arena, pos, end, cap, _, keys = W.build_config(5)
    assert ref["n"] == n and F.sha(arena) == ref["plain"]
    slot = ref["slot"]
    key = keys[0].tobytes()
    one = torch.from_numpy(arena).cuda()
    del arena
    two = one.clone()
    end1, end2 = end.copy(), end.copy()

    def st_bytes(ctx):
        return F.state_bytes([state(ctx)[:2] + state(ctx)[3:]])

    # unsharded: one context pair, one call per direction
    tx, rx = P.Srtp(1, key), P.Srtp(1, key)
    e1p = run(torch, "srtp_encrypt", tx, one, pos, end1, cap, 0, n)
    bad = F.compare(ref["protect"], one.cpu().numpy(), n, slot, end1, e1p,
                    st_bytes(tx))
    assert not bad, ("unsharded protect", bad)
    e1u = run(torch, "srtp_decrypt", rx, one, pos, end1, cap, 0, n)
    bad = F.compare(ref["unprotect"], one.cpu().numpy(), n, slot, end1, e1u,
                    st_bytes(rx))
    assert not bad, ("unsharded unprotect", bad)

    # sharded: rank r's contexts start from the closed-form boundary state;
    # all shards protect, then all shards unprotect
    ctxs = []
    for r in range(2):
        a = r * PER
        assert (int(one[pos[a] + 2]) << 8 | int(one[pos[a] + 3])) == \
            S.shard_seq0(r, PER, S0)
        stx, srx = P.Srtp(1, key), P.Srtp(1, key)
        if r:
            for c, recv in ((stx, False), (srx, True)):
                assert c.import_(S.shard_state(r, PER, S0, W.SSRC_BASE,
                                               recv, P.StreamState)) == 0
        ctxs.append((stx, srx))
    errs = {}
    for d, (op, k) in enumerate((("srtp_encrypt", 0), ("srtp_decrypt", 1))):
        errs[op] = np.concatenate([
            run(torch, op, ctxs[r][k], two, pos, end2, cap, r * PER,
                (r + 1) * PER) for r in range(2)])
        direction = ("protect", "unprotect")[d]
        bad = F.compare(ref[direction], two.cpu().numpy(), n, slot, end2,
                        errs[op], st_bytes(ctxs[1][k]))
        assert not bad, ("sharded " + direction, bad)
    finals = [(state(stx), state(srx)) for stx, srx in ctxs]
    for stx, srx in ctxs:
        stx.close()
        srx.close()

    assert not e1p.any() and not e1u.any()
    assert np.array_equal(errs["srtp_encrypt"], e1p)
    assert np.array_equal(errs["srtp_decrypt"], e1u)
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


def test_config5_all_eight_shards_match_reference(torch_cuda):
    """BASELINE config 5 whole: the 8M-packet stream as the 8 ranks of
    bench.py --gpus 8 hold it, run shard after shard on one GPU.  Rank r's
    fresh contexts import shard_state(r) (the closed-form boundary state
    bench.py hands each rank), protect its 1M packets, and unprotect them;
    every shard's arena, end, errno digests and exported final states must
    equal the reference src/srtp's over the same stream
    (tests/golden/config5_shards.json: one reference sender and receiver over
    all 8M packets in order, `oracle/_ref/ref_digest shards 8 1048576`)."""
    import hashlib
    import json
    import os
    import sys
    torch = torch_cuda
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                        "config5_shards.json")
    with open(path) as f:
        ref = json.load(f)
    per, s0 = ref["per"], ref["s0"]
    assert (ref["world"], per) == (8, PER)
    key = W.make_keys(1, W.KEY_LEN[1])[0].tobytes()

    def sha(a):
        return hashlib.sha256(memoryview(np.ascontiguousarray(a)).cast("B")
                              ).hexdigest()

    def want_state(row):
        return (row["roc"], row["s_l"], row["s_l_set"], row["lix"],
                row["bitmap"])

    for sh in ref["shards"]:
        r = sh["rank"]
        arena, pos, end, cap = W.make_arena(per, 1200,
                                            s0=S.shard_seq0(r, per, s0),
                                            first=r * per)
        assert sha(arena) == sh["plain"], r
        dev = torch.from_numpy(arena).cuda()
        del arena
        tx, rx = P.Srtp(1, key), P.Srtp(1, key)
        if r:
            for c, recv in ((tx, False), (rx, True)):
                assert c.import_(S.shard_state(r, per, s0, W.SSRC_BASE, recv,
                                               P.StreamState)) == 0
        for op, ctx, direction in (("srtp_encrypt", tx, "protect"),
                                   ("srtp_decrypt", rx, "unprotect")):
            err = run(torch, op, ctx, dev, pos, end, cap, 0, per)
            want = sh[direction]
            bad = []
            if sha(dev.cpu().numpy()) != want["arena"]:
                bad.append("arena")
            if sha(end.astype("<u4")) != want["end"]:
                bad.append("end")
            if sha(err.astype("<i4")) != want["err"]:
                bad.append(("err", int(np.count_nonzero(err))))
            if state(ctx) != want_state(want["state"]):
                bad.append(("state", state(ctx), want["state"]))
            assert not bad, (r, direction, bad)
        tx.close()
        rx.close()
        del dev
        print("config 5 shard %d/8: protect + unprotect equal to the "
              "reference" % (r + 1), file=sys.stderr, flush=True)


def test_bench_spawns_two_gpu_ranks():
    """`bench.py --gpus 2` without a launcher runs two real ranks (here both
    on cuda:0 with gloo counters, --same-device): config 5 shards, the
    round trip verifies on each rank and rank 0 reports n_gpus 2"""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                        "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"),
                        "--gpus", "2", "--same-device", "--packets", "8192",
                        "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True,
                       env=env, timeout=180, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines()
             if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["dist_world"] == 2
    assert ln["verified_roundtrip"] is True and ln["errors"] == 0
    assert ln["config"]["workload"].startswith("config5")


def test_split_stream_fold_on_device_results(torch_cuda):
    """one stream with loss, reordering across the shard boundary, replays
    and forged packets, unprotected on the GPU as two shards (rank 1 from
    the header-only boundary guess) and folded with srtp_rx_index /
    srtp_rx_fold (re_amd/shard.py): equal to the same stream unprotected
    in one call, and to the oracle receiver (tests/test_rxfold_cpu.py
    covers the fold against the oracle on the CPU)"""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_rxfold_cpu as X
    from oracle_lib import OracleBackend
    torch = torch_cuda
    O = OracleBackend()
    suite = X.CM80
    key = X.key_for(suite)
    ixs = [65000 + i for i in range(3000) if i % 37 != 5]
    # protect on the GPU, in index order, slot per packet
    plain = [X.rtp(ix & 0xffff, ix) for ix in ixs]

    def arena_dev(pkts, room):
        slot = (max(len(p) for p in pkts) + room + 15) & ~15
        buf = np.zeros(slot * len(pkts), dtype=np.uint8)
        pos = np.arange(len(pkts), dtype=np.uint32) * slot
        end = pos + np.array([len(p) for p in pkts], dtype=np.uint32)
        for i, p in enumerate(pkts):
            buf[pos[i]:end[i]] = np.frombuffer(p, dtype=np.uint8)
        return buf, pos, end, pos + slot

    buf, pos, end, cap = arena_dev(plain, 16)
    dev = torch.from_numpy(buf).cuda()
    tx = P.Srtp(suite, key)
    assert not run(torch, "srtp_encrypt", tx, dev, pos, end, cap, 0,
                   len(plain)).any()
    host = dev.cpu().numpy()
    prot = {ix: host[pos[i]:end[i]].tobytes() for i, ix in enumerate(ixs)}
    tx.close()
    # rank 0 gets the first half minus one late packet, which arrives as
    # rank 1's third packet, below the top rank 1 guesses as seen
    L, R = list(ixs[:len(ixs) // 2]), list(ixs[len(ixs) // 2:])
    late = L.pop(-3)
    R.insert(2, late)
    left = [prot[ix] for ix in L]
    left.insert(len(left) - 20, prot[L[-40]])        # replay inside rank 0
    right = [prot[ix] for ix in R]
    right.insert(5, prot[L[-10]])                    # replay across it
    f = bytearray(right[30])
    f[24] ^= 1
    right.insert(31, bytes(f))                       # forged
    pkts = left + right
    b = len(left)
    n = len(pkts)
    truth, fin = X.receive(O, suite, pkts)

    # unsharded on the GPU
    buf, pos, end, cap = arena_dev(pkts, 0)
    one = torch.from_numpy(buf).cuda()
    rx = P.Srtp(suite, key)
    pos1 = pos.copy()
    end1 = end.copy()
    e1 = run(torch, "srtp_decrypt", rx, one, pos, end1, cap, 0, n, pos1)
    assert (e1 == truth).all()
    e, so = rx.export(X.SSRC)
    assert e == 0
    st_one = (so.roc, so.s_l, so.s_l_set, so.replay_rtp_lix,
              so.replay_rtp_bitmap)
    rx.close()

    # two shards on the GPU, then the fold; a voided tail re-runs from the
    # fold's state on its received bytes (what the rank holding it does)
    two = torch.from_numpy(buf).cuda()
    end2 = end.copy()
    pos2 = pos.copy()
    guess = X.assumed_boundary(pkts[:b])
    recs = []
    for r, (a, z) in enumerate(((0, b), (b, n))):
        c = P.Srtp(suite, key)
        st0 = X.state(*guess) if r else X.state()
        if r:
            assert c.import_(st0) == 0
        res = run(torch, "srtp_decrypt", c, two, pos, end2, cap, a, z, pos2)
        recs.append(S.rx_records(st0, buf, pos[a:z], end[a:z], res))
        # the same records from the device outputs (the arena stays there)
        dv = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(
            np.int32)).cuda()
        recd = S.rx_records_dev(st0, two, dv(pos[a:z]), dv(end[a:z]),
                                dv(res))
        assert (recd == recs[-1]).all(), r
        c.close()
    rec = np.concatenate(recs)
    assert (rec["res"] != truth).any()     # the ranks alone disagree
    st = X.state()
    done, reruns, errs = 0, 0, []
    while True:
        err, nd = S.rx_fold(st, suite, rec[done:])
        errs.append(err)
        done += nd
        if done == n:
            break
        reruns += 1
        assert reruns <= 4
        lo, hi = int(pos[done]), int(cap[n - 1])
        two[lo:hi] = torch.from_numpy(buf[lo:hi]).cuda()
        end2[done:] = end[done:]
        st0 = X.state(st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
                      st.replay_rtp_bitmap)
        c = P.Srtp(suite, key)
        assert c.import_(st0) == 0
        res = run(torch, "srtp_decrypt", c, two, pos, end2, cap, done, n,
                  pos2)
        c.close()
        rec = np.concatenate([rec[:done],
                              S.rx_records(st0, buf, pos[done:], end[done:],
                                           res)])
    # the late packet the rank rejected as a replay is accepted by the one
    # receiver: its bytes were voided and re-run
    assert reruns >= 1
    assert (np.concatenate(errs) == truth).all()
    assert (st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
            st.replay_rtp_bitmap) == st_one
    assert (st.roc, st.s_l, st.replay_rtp_lix, st.replay_rtp_bitmap) == fin
    assert (end2 == end1).all() and (pos2 == pos1).all()
    assert torch.equal(two, one)


def test_split_stream_fold_full_size(torch_cuda):
    """the split-stream fold at shard size: a 512K-packet config-2-shape
    stream (1200-B packets, the ROC wraps) with 1 % loss, local swaps, late
    packets across the shard boundary, replays and forged packets,
    unprotected on the GPU as two shards (rank 1 from the header-only
    boundary guess), records from the device outputs, the parallel fold
    (srtp_rx_fold in parts), voided tails re-run from the fold's state:
    arena, ends, errnos and final state equal to the same stream
    unprotected in one call"""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_rxfold_cpu as X
    torch = torch_cuda
    suite = 1                                   # AES_CM_128_HMAC_SHA1_80
    N = 1 << 19
    key = W.make_keys(1, 30)[0].tobytes()
    arena, pos, end, cap = W.make_arena(N, 1200, s0=S0)
    slot = int(cap[0] - pos[0])
    dev = torch.from_numpy(arena).cuda()
    tx = P.Srtp(suite, key)
    e = run(torch, "srtp_encrypt", tx, dev, pos, end, cap, 0, N)
    assert not e.any()
    tx.close()
    prot = dev.cpu().numpy().reshape(N, slot)
    plen = int(end[0] - pos[0])                 # protected length
    # arrival order
    rng = np.random.default_rng(7)
    g = np.arange(N)
    g = g[rng.random(N) > 0.01]
    sw = rng.integers(0, len(g) - 1, len(g) // 100)
    g[sw], g[sw + 1] = g[sw + 1].copy(), g[sw].copy()
    m0 = len(g) // 2
    late = g[m0 - 5:m0 - 2].copy()              # three arrive in rank 1
    g = np.concatenate([g[:m0 - 5], g[m0 - 2:m0 + 7], late, g[m0 + 7:]])
    dup = np.sort(rng.integers(0, len(g), 200))
    g = np.insert(g, dup, g[dup])               # replays
    m = len(g)
    arr = prot[g].copy()
    forged = rng.integers(0, m, 40)
    arr[forged, 40] ^= 1
    buf = arr.reshape(-1)
    apos = np.arange(m, dtype=np.uint32) * slot
    aend = apos + plen
    acap = apos + slot
    del prot, arr

    # one call
    one = torch.from_numpy(buf).cuda()
    rx = P.Srtp(suite, key)
    end1, pos1 = aend.copy(), apos.copy()
    e1 = run(torch, "srtp_decrypt", rx, one, apos, end1, acap, 0, m, pos1)
    st_one = state(rx)
    rx.close()
    assert (e1 != 0).sum() >= 40

    # two shards, device records, the fold, voided tails re-run
    b = m // 2
    hdrs = [buf[int(apos[i]):int(apos[i]) + 12].tobytes() for i in range(b)]
    guess = X.assumed_boundary(hdrs)
    two = torch.from_numpy(buf).cuda()
    end2, pos2 = aend.copy(), apos.copy()
    dv = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(
        np.int32)).cuda()
    recs = []
    for r, (a, z) in enumerate(((0, b), (b, m))):
        c = P.Srtp(suite, key)
        st0 = X.state(*guess) if r else X.state()
        st0.ssrc = W.SSRC_BASE
        if r:
            assert c.import_(st0) == 0
        res = run(torch, "srtp_decrypt", c, two, apos, end2, acap, a, z, pos2)
        recs.append(S.rx_records_dev(st0, two, dv(apos[a:z]), dv(aend[a:z]),
                                     dv(res)))
        c.close()
    rec = np.concatenate(recs)
    st = X.state()
    st.ssrc = W.SSRC_BASE
    done, reruns, errs = 0, 0, []
    while True:
        err, nd = S.rx_fold(st, suite, rec[done:])
        errs.append(err)
        done += nd
        if done == m:
            break
        reruns += 1
        assert reruns <= 8
        lo, hi = int(apos[done]), int(acap[m - 1])
        two[lo:hi] = torch.from_numpy(buf[lo:hi]).cuda()
        end2[done:] = aend[done:]
        st0 = X.state(st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
                      st.replay_rtp_bitmap)
        st0.ssrc = W.SSRC_BASE
        c = P.Srtp(suite, key)
        assert c.import_(st0) == 0
        res = run(torch, "srtp_decrypt", c, two, apos, end2, acap, done, m,
                  pos2)
        c.close()
        rec = np.concatenate([rec[:done],
                              S.rx_records_dev(st0, two, dv(apos[done:]),
                                               dv(aend[done:]), dv(res))])
    # the late packets rank 1 took for replays are accepted by the one
    # receiver: voided and re-run
    assert reruns >= 1
    assert (np.concatenate(errs) == e1).all()
    assert (st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
            st.replay_rtp_bitmap) == st_one
    assert (end2 == end1).all() and (pos2 == pos1).all()
    assert torch.equal(two, one)
