"""SRTCP batches planned on the device (srtcp_*_batch_dev, dev_planned_rtcp:
the one-launch plan k_rp_plan, and with srtp_gpu_tune noplanfuse k_parse +
k_plan_rtcp), through the C-ABI library, against the oracle called one
packet at a time (srtcp_encrypt srtcp.c:31-140, srtcp_decrypt
srtcp.c:143-287): every suite, SRTP_UNENCRYPTED_SRTCP, two consecutive
batches per direction (the SRTCP index and replay window carried over),
and the planner's fallbacks -- a replayed and a forged packet (exact fold
through the host engine), a second SSRC, a truncated packet.
"""
import errno

import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import workload as W
from tests import oracle_lib as O
from tests.test_gpu_fastpath import keys_for, to_arena
from tests.test_gpu_fastpath import run_dev as run_dev_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    P.load()
    return torch


def rtcp_packet(rng, ssrc, body):
    words = (8 + body) // 4 - 1
    return bytes([0x81, 200 + int(rng.integers(0, 5)), words >> 8,
                  words & 0xff]) + ssrc.to_bytes(4, "big") + \
        rng.integers(0, 256, body, dtype=np.uint8).tobytes()


def run_dev(torch, op, ctx, pkts):
    arena, pos, end, cap, _ = to_arena([(0, p) for p in pkts])
    dev = torch.from_numpy(arena).cuda()
    i32 = lambda a: torch.from_numpy(a.astype(np.uint32).view(np.int32)
                                     ).cuda()
    p_d, e_d, c_d = i32(pos), i32(end), i32(cap)
    err = torch.full((len(pkts),), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    rc = P.device_batch_dev(op, [ctx], dev.data_ptr(), dev.numel(),
                            p_d.data_ptr(), e_d.data_ptr(), c_d.data_ptr(),
                            err.data_ptr(), len(pkts))
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    a = dev.cpu().numpy()
    po = p_d.cpu().numpy().view(np.uint32)
    eo = e_d.cpu().numpy().view(np.uint32)
    er = err.cpu().numpy()
    return [(int(er[i]), int(po[i] - pos[i]), int(eo[i] - pos[i]),
             a[pos[i]:pos[i] + max(int(eo[i] - pos[i]), len(p))].tobytes())
            for i, p in enumerate(pkts)]


def oracle_run(ob, ctx, op, pkts):
    out = []
    for p in pkts:
        e, po, en, _, buf = ob.call(ctx, op, len(p) + 64, 0, len(p), p,
                                    len(p) + 32)
        out.append((e, po, en, buf[:max(en, len(p))]))
    return out


def counters():
    return P.counter("rejects"), P.counter("folds")


@pytest.mark.parametrize("sep", [0, 1])
@pytest.mark.parametrize("flags", [0, P.SRTP_UNENCRYPTED_SRTCP])
@pytest.mark.parametrize("suite", list(range(6)))
def test_srtcp_device_planned_vs_oracle(torch_cuda, suite, flags, sep):
    """sep: the separate planner launches (noplanfuse) instead of the
    one-launch plan"""
    with P.tune(noplanfuse=sep):
        srtcp_planned_vs_oracle(torch_cuda, suite, flags)


def srtcp_planned_vs_oracle(torch_cuda, suite, flags):
    torch = torch_cuda
    rng = np.random.default_rng(31 + suite + 7 * flags)
    key = keys_for(suite, 1)[0]
    ob = O.OracleBackend()
    otx, orx = ob.alloc(suite, key, flags)[0], ob.alloc(suite, key, flags)[0]
    tx, rx = P.Srtp(suite, key, flags), P.Srtp(suite, key, flags)
    for batch in range(2):
        pkts = [rtcp_packet(rng, 0xC0FFEE01, 4 * int(rng.integers(0, 80)))
                for _ in range(700)]
        r0 = counters()
        got = run_dev(torch, "srtcp_encrypt", tx, pkts)
        want = oracle_run(ob, otx, "srtcp_encrypt", pkts)
        assert got == want
        wire = [w[3][:w[2]] for w in want]
        got = run_dev(torch, "srtcp_decrypt", rx, wire)
        want = oracle_run(ob, orx, "srtcp_decrypt", wire)
        assert got == want
        assert all(g[0] == 0 for g in got)
        assert counters() == r0, "expected the device planner, no fallback"
    e, st = rx.export(0xC0FFEE01)
    assert e == 0 and st.rtcp_index == 0
    e, st = tx.export(0xC0FFEE01)
    assert e == 0 and st.rtcp_index == 1400
    for c in (otx, orx):
        ob.free(c)


@pytest.mark.parametrize("sep", [0, 1])
@pytest.mark.parametrize("suite", [1, 4])
def test_srtcp_fallbacks_vs_oracle(torch_cuda, suite, sep):
    with P.tune(noplanfuse=sep):
        srtcp_fallbacks_vs_oracle(torch_cuda, suite)


def srtcp_fallbacks_vs_oracle(torch_cuda, suite):
    torch = torch_cuda
    rng = np.random.default_rng(77 + suite)
    key = keys_for(suite, 1)[0]
    ob = O.OracleBackend()
    otx = ob.alloc(suite, key, 0)[0]
    pkts = [rtcp_packet(rng, 0xABCD0001, 4 * int(rng.integers(0, 40)))
            for _ in range(400)]
    wire = [w[3][:w[2]] for w in oracle_run(ob, otx, "srtcp_encrypt", pkts)]
    cases = {
        "replay": wire[:200] + [wire[150]] + wire[200:],
        "forged": wire[:100] + [bytes(wire[100][:-1]) +
                                bytes([wire[100][-1] ^ 1])] + wire[101:],
        "truncated": wire[:50] + [wire[50][:6]] + wire[51:],
        "second_ssrc": wire[:30] + [rtcp_packet(rng, 0x5555, 40)] + wire[30:],
    }
    for name, w in cases.items():
        orx = ob.alloc(suite, key, 0)[0]
        want = oracle_run(ob, orx, "srtcp_decrypt", w)
        rx = P.Srtp(suite, key)
        got = run_dev(torch, "srtcp_decrypt", rx, w)
        assert [g[0] for g in got] == [x[0] for x in want], name
        assert got == want, name
        ob.free(orx)
    # protect fallback: a packet too short to hold an RTCP header
    o2 = ob.alloc(suite, key, 0)[0]
    pk = pkts[:10] + [b"\x81\xc8\x00"] + pkts[10:20]
    tx = P.Srtp(suite, key)
    assert run_dev(torch, "srtcp_encrypt", tx, pk) == \
        oracle_run(ob, o2, "srtcp_encrypt", pk)
    assert run_dev(torch, "srtcp_encrypt", tx, pk)[10][0] == errno.EBADMSG


@pytest.mark.parametrize("suite", [1, 5])
def test_srtcp_large_packets(suite, torch_cuda):
    """SRTCP packets either side of the counter-cached kernels' size bound
    (SGPU_CACHED_MAX, 4032 B): the device planner sends the large ones to
    the plain kernels; every packet matches the oracle both ways"""
    torch = torch_cuda
    rng = np.random.default_rng(4040 + suite)
    key = keys_for(suite, 1)[0]
    lens = [4000, 4028, 4032, 4100, 6000, 200]
    pkts = []
    for i in range(24):
        L = lens[i % len(lens)]
        b = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        b[0], b[1] = 0x80, 200
        b[2], b[3] = ((L // 4 - 1) >> 8) & 0xff, (L // 4 - 1) & 0xff
        b[4:8] = (0x5150).to_bytes(4, "big")
        pkts.append((0, bytes(b)))
    arena, pos, end, cap, _ = to_arena(pkts)
    tx, rx = P.Srtp(suite, key), P.Srtp(suite, key)
    a = run_dev_arrays(torch, "srtcp_encrypt", [tx], arena, pos, end, cap,
                       None)
    be = O.OracleBackend()
    octx = be.alloc(suite, key, 0)[0]
    orx = be.alloc(suite, key, 0)[0]
    prot = []
    for i, (_, p) in enumerate(pkts):
        e, po, en, _, buf = be.call(octx, "srtcp_encrypt", len(p) + 64, 0,
                                    len(p), p, len(p) + 20)
        assert (int(a[3][i]), int(a[2][i] - pos[i])) == (e, en), i
        assert a[0][pos[i]:a[2][i]].tobytes() == buf[:en], (i, len(p))
        prot.append((0, bytes(buf[:en])))
    a2, p2, e2, c2, _ = to_arena(prot)
    d = run_dev_arrays(torch, "srtcp_decrypt", [rx], a2, p2, e2, c2, None)
    for i, (_, p) in enumerate(prot):
        e, po, en, _, buf = be.call(orx, "srtcp_decrypt", len(p) + 64, 0,
                                    len(p), p, len(p))
        assert (int(d[3][i]), int(d[2][i] - p2[i])) == (e, en), i
        assert d[0][p2[i]:p2[i] + en].tobytes() == buf[:en], i
    be.free(octx)
    be.free(orx)
    tx.close()
    rx.close()
