"""GPU parity: the HIP path (through the C-ABI library) against the golden
vectors recorded from the reference and against the C restatement oracle.

Bit-exact is the bar (integer/byte work): errno, mbuf pos/end/size and
every buffer byte the reference call leaves.
"""
import ctypes
from itertools import groupby

import numpy as np
import pytest

import re_amd.srtp as P
from tests import oracle_lib as O
from tests.golden_util import replay_scenario
from tests.product_backend import ProductBackend

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("path", ["small", "coop", "general"])
def test_per_call_golden(golden, path, torch_cuda):
    """Every recorded reference call, replayed one srtp_* call at a time --
    through the fused small kernel over pinned memory (small.hip, the
    default for packets up to SGPU_SMALL_MAX), through the copy path with
    the small-launch split (nosmall: the cipher regions by k_ctr_coop /
    k_gcm_coop, the general kernel MAC-only), and with the cipher fused
    into the one-packet-per-lane general kernel (nosmall + nocoop)."""
    be = ProductBackend()
    with P.tune(nosmall=0 if path == "small" else 1,
                nocoop=1 if path == "general" else 0):
        bad = [m for m in (replay_scenario(be, s)
                           for s in golden["scenarios"]) if m]
    assert not bad, bad[:5]


def test_libsrtp_known_answer(torch_cuda):
    # test/srtp.c:514-570
    key = b"\x22" * 16 + b"\x44" * 14
    s = P.Srtp(1, key)
    assert s.err == 0
    mb = P.new_mbuf(bytes.fromhex("800000010000000001020304") + b"\xa5" * 20,
                    512)
    assert s.encrypt(mb) == 0
    assert P.mbuf_bytes(mb) == bytes.fromhex(
        "800000010000000001020304f5b44b7e3ad4eb057bc6480c45df6547bb70bcc2"
        "7b136e1f3d3a62821b15")
    P.free_mbuf(mb)


def _groups(scn):
    """maximal runs of consecutive ops on the same context and op"""
    ops = list(enumerate(scn["ops"]))
    return [list(g) for _, g in groupby(ops, key=lambda t: (t[1]["ctx"],
                                                             t[1]["op"]))]


def test_batched_mbufs_golden(golden, torch_cuda):
    """Runs of consecutive calls as ONE srtp_*_mbufs batch: same results as
    the sequential reference calls (forged/replayed packets mid-batch)."""
    bad = []
    for scn in golden["scenarios"]:
        ctxs = [P.Srtp(c["suite"], bytes.fromhex(c["key"]), c["flags"])
                for c in scn["ctxs"]]
        for grp in _groups(scn):
            ctx = ctxs[grp[0][1]["ctx"]]
            mbs = [P.new_mbuf(bytes.fromhex(op["in"]), op["size"] or 512,
                              op["pos"]) for _, op in grp]
            rc, errs = P.batch_run(ctx, grp[0][1]["op"], mbs)
            assert rc == 0
            for (k, op), mb, e in zip(grp, mbs, errs):
                m = mb.contents
                out = bytes.fromhex(op["out"])
                got = (e, m.pos, m.end, m.size)
                want = (op["err"], op["pos_o"], op["end_o"], op["size_o"])
                if got != want or ctypes.string_at(m.buf, len(out)) != out:
                    bad.append("%s op#%d %s got %r want %r" % (
                        scn["name"], k, op["op"], got, want))
                P.free_mbuf(mb)
        for c in ctxs:
            c.close()
    assert not bad, bad[:5]


def test_device_batch_golden(golden, torch_cuda):
    """Same runs through the device-resident srtp_*_batch API (packets in
    an HBM arena, in-place results)."""
    torch = torch_cuda
    bad = []
    for scn in golden["scenarios"]:
        ctxs = [P.Srtp(c["suite"], bytes.fromhex(c["key"]), c["flags"])
                for c in scn["ctxs"]]
        for grp in _groups(scn):
            ctx = ctxs[grp[0][1]["ctx"]]
            n = len(grp)
            sizes = [max(op["size"] or 512, op["size_o"]) for _, op in grp]
            base = np.zeros(n, dtype=np.uint64)
            off = 0
            for i, sz in enumerate(sizes):
                base[i] = off
                off += (sz + 64 + 15) & ~15
            host = np.zeros(off, dtype=np.uint8)
            pos = np.zeros(n, dtype=np.uint32)
            end = np.zeros(n, dtype=np.uint32)
            cap = np.zeros(n, dtype=np.uint32)
            for i, (_, op) in enumerate(grp):
                inb = np.frombuffer(bytes.fromhex(op["in"]), dtype=np.uint8)
                host[base[i]:base[i] + len(inb)] = inb
                pos[i] = base[i] + op["pos"]
                end[i] = base[i] + op["end"]
                cap[i] = base[i] + sizes[i]
            dev = torch.from_numpy(host).cuda()
            torch.cuda.synchronize()
            rc, err = P.device_batch(grp[0][1]["op"], [ctx], dev.data_ptr(),
                                     off, pos, end, cap)
            assert rc == 0
            res = dev.cpu().numpy()
            for i, (k, op) in enumerate(grp):
                out = bytes.fromhex(op["out"])
                got = (int(err[i]), int(pos[i] - base[i]),
                       int(end[i] - base[i]))
                want = (op["err"], op["pos_o"], op["end_o"])
                gb = res[base[i]:base[i] + len(out)].tobytes()
                if got != want or gb != out:
                    bad.append("%s op#%d %s got %r want %r bytes_ok=%s" % (
                        scn["name"], k, op["op"], got, want, gb == out))
        for c in ctxs:
            c.close()
    assert not bad, bad[:5]


@pytest.mark.parametrize("suite", list(range(6)))
def test_stream_vs_oracle(suite, torch_cuda):
    """A 3000-packet stream (ROC wrap, mixed lengths incl. 1200 B) through
    the device batch API vs the oracle, bit-exact, then decrypt back."""
    from re_amd import workload as W
    torch = torch_cuda
    n = 3000
    rng = np.random.default_rng(7 + suite)
    lens = rng.integers(12, 1401, size=n).astype(np.uint32)
    lens[::5] = 1200
    arena, pos, end, cap = W.make_arena(n, lens, s0=64000)
    key = bytes(range(1, 1 + P.key_len(suite) + P.salt_len(suite)))
    tx = P.Srtp(suite, key)
    rx = P.Srtp(suite, key)
    otx, _ = O.OracleBackend().alloc(suite, key, 0)
    be = O.OracleBackend()
    # oracle, sequentially
    want = []
    slot = int(cap[0] - pos[0])
    for i in range(n):
        pkt = arena[pos[i]:end[i]].tobytes()
        e, p, en, sz, buf = be.call(otx, "srtp_encrypt", slot, 0, len(pkt),
                                    pkt, 0)
        assert e == 0
        want.append(buf[:en])
    dev = torch.from_numpy(arena.copy()).cuda()
    p2, e2 = pos.copy(), end.copy()
    rc, err = P.device_batch("srtp_encrypt", [tx], dev.data_ptr(),
                             arena.nbytes, p2, e2, cap)
    assert rc == 0 and not err.any()
    res = dev.cpu().numpy()
    for i in range(n):
        assert res[p2[i]:e2[i]].tobytes() == want[i], i
    rc, err = P.device_batch("srtp_decrypt", [rx], dev.data_ptr(),
                             arena.nbytes, p2, e2, cap)
    assert rc == 0 and not err.any()
    res = dev.cpu().numpy()
    for i in range(0, n, 7):
        assert res[p2[i]:e2[i]].tobytes() == arena[pos[i]:end[i]].tobytes()
    be.free(otx)
