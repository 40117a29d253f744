"""RTCP compound decode on the GPU (include/re_rtcp_batch.h,
re_amd/csrc/hip/rtcp_walk.hip) through the C-ABI library:

  * all 2032 golden packets of the reference receive loop
    (tests/golden/rtcp_decode_golden.json.gz, oracle/gen_rtcp_golden.c
    running `while (0 == rtcp_decode(&msg, mb))`, src/rtp/rtp.c:164,
    pkt.c:337-551) in one batch: every descriptor, errno and stop offset
    bit-exact;
  * 200K mutated compounds against the C restatement (oracle/
    rtcp_oracle.c, itself pinned to the golden file), with maxmsg smaller
    than some packets' message counts (counted, not written);
  * the SRTCP path end to end: config-2-shape SRTCP arena protected and
    unprotected on the GPU, then decoded in place, against the oracle;
  * windows outside the arena give EINVAL, never a read out of bounds.
"""
import errno

import numpy as np
import pytest

import re_amd.srtp as P
from tests.test_rtcp_cpu import load_cases, oracle_walk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def pack(pkts, align=4):
    pos, off = [], 0
    for p in pkts:
        pos.append(off)
        off += (len(p) + align - 1) // align * align + align
    arena = np.zeros(max(off, 4), dtype=np.uint8)
    for o, p in zip(pos, pkts):
        arena[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    pos = np.array(pos, dtype=np.uint32)
    end = pos + np.array([len(p) for p in pkts], dtype=np.uint32)
    return arena, pos, end


def decode_dev(torch, arena, pos, end, maxmsg):
    n = len(pos)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    d_arena = t(arena)
    d_pos = t(pos.view(np.int32))
    d_end = t(end.view(np.int32))
    desc = torch.full((n * maxmsg * 5 + 1,), -1, dtype=torch.int32,
                      device="cuda")
    nmsg = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    err = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    stop = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    rc = P.rtcp_decode_dev(d_arena.data_ptr(), d_arena.numel(),
                           d_pos.data_ptr(), d_end.data_ptr(), n,
                           desc.data_ptr(), maxmsg, nmsg.data_ptr(),
                           err.data_ptr(), stop.data_ptr())
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    d = desc.cpu().numpy()[:-1].view(np.uint32).reshape(n, maxmsg, 5)
    return d, nmsg.cpu().numpy(), err.cpu().numpy(), \
        stop.cpu().numpy().view(np.uint32)


def rows(d, k):
    """descriptor k as the golden's [off, size, pt, count, length, ssrc,
    aux]"""
    w = [int(x) for x in d[k]]
    return [w[0], w[1], w[2] & 0xff, (w[2] >> 8) & 0xff, w[2] >> 16, w[3],
            w[4]]


def test_rtcp_decode_vs_reference(torch_cuda):
    cases = load_cases()
    pkts = [bytes.fromhex(c["pkt"]) for c in cases]
    arena, pos, end = pack(pkts)
    maxmsg = max(len(c["msgs"]) for c in cases)
    d, nmsg, err, stop = decode_dev(torch_cuda, arena, pos, end, maxmsg)
    for i, c in enumerate(cases):
        got = [rows(d[i], k) for k in range(nmsg[i])]
        assert (got, int(err[i]), int(stop[i])) == \
            (c["msgs"], c["err"], c["stop"]), i


def mutate(rng, cases, n):
    """compounds of golden packets, then one random mutation each"""
    base = [bytes.fromhex(c["pkt"]) for c in cases]
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 4))
        b = bytearray(b"".join(base[int(j)] for j in
                               rng.integers(0, len(base), k)))
        kind = int(rng.integers(0, 5))
        if b and kind == 0:
            del b[int(rng.integers(0, len(b))):]
        elif b and kind == 1:
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
        elif b and kind == 2:
            at = int(rng.integers(0, len(b))) & ~3
            if at + 3 < len(b):
                b[at + 3] = int(rng.integers(0, 256))
        elif kind == 3:
            b += bytes(rng.integers(0, 256, int(rng.integers(1, 9)),
                                    dtype=np.uint8))
        out.append(bytes(b))
    return out


def test_rtcp_decode_fuzz_vs_oracle(torch_cuda):
    rng = np.random.default_rng(2032)
    pkts = mutate(rng, load_cases(), 200000)
    arena, pos, end = pack(pkts)
    maxmsg = 6                  # fewer than some packets carry
    d, nmsg, err, stop = decode_dev(torch_cuda, arena, pos, end, maxmsg)
    over = 0
    for i in range(0, len(pkts), 1 if len(pkts) < 50000 else 7):
        msgs, e, s, n = oracle_walk(pkts[i], 64)
        over += n > maxmsg
        assert int(nmsg[i]) == n, i
        assert (int(err[i]), int(stop[i])) == (e, s), i
        assert [rows(d[i], k) for k in range(min(n, maxmsg))] == \
            msgs[:maxmsg], i
    assert over > 0


def test_srtcp_then_rtcp_decode(torch_cuda):
    """the receive path: SRTCP-unprotect a config-2-shape arena on the
    GPU, then decode the compounds where they lie"""
    from re_amd import workload as W
    torch = torch_cuda
    n = 1 << 16
    arena, pos, end, cap = W.make_rtcp_arena(n, 1200)
    key = W.make_keys(1, 30)[0].tobytes()
    tx, rx = P.Srtp(1, key), P.Srtp(1, key)
    dev = torch.from_numpy(arena.copy()).cuda()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(
        np.int32)).cuda()
    p_d, e_d, c_d = t(pos), t(end), t(cap)
    er = torch.zeros(n, dtype=torch.int32, device="cuda")
    for op, ctx in (("srtcp_encrypt", tx), ("srtcp_decrypt", rx)):
        rc = P.device_batch_dev(op, [ctx], dev.data_ptr(), dev.numel(),
                                p_d.data_ptr(), e_d.data_ptr(),
                                c_d.data_ptr(), er.data_ptr(), n)
        assert rc == 0 and not bool(er.any())
    torch.cuda.synchronize()
    slot = int(pos[1] - pos[0])          # make_rtcp_arena's slot
    assert slot % 64 == 0 and arena.size == n * slot
    assert torch.equal(dev[:n * slot].view(n, slot)[:, :1200],
                       torch.from_numpy(arena).cuda().view(n, slot)[:, :1200])
    maxmsg = 4
    desc = torch.zeros(n * maxmsg * 5, dtype=torch.int32, device="cuda")
    nm, ee, st = (torch.zeros(n, dtype=torch.int32, device="cuda")
                  for _ in range(3))
    rc = P.rtcp_decode_dev(dev.data_ptr(), dev.numel(), p_d.data_ptr(),
                           e_d.data_ptr(), n, desc.data_ptr(), maxmsg,
                           nm.data_ptr(), ee.data_ptr(), st.data_ptr())
    assert rc == 0
    d = desc.cpu().numpy().view(np.uint32).reshape(n, maxmsg, 5)
    nm, ee, st = nm.cpu().numpy(), ee.cpu().numpy(), st.cpu().numpy()
    for i in range(0, n, 997):
        pk = arena[pos[i]:end[i]].tobytes()
        msgs, e, s, k = oracle_walk(pk, 64)
        assert (int(nm[i]), int(ee[i]), int(st[i])) == (k, e, s), i
        assert [rows(d[i], j) for j in range(min(k, maxmsg))] == \
            msgs[:maxmsg], i
        assert msgs[0][2] == 200 and msgs[0][5] == W.SSRC_BASE
    tx.close()
    rx.close()


def test_rtcp_decode_bad_windows(torch_cuda):
    torch = torch_cuda
    arena = np.zeros(64, dtype=np.uint8)
    pos = np.array([0, 40, 8], dtype=np.uint32)
    end = np.array([8, 80, 4], dtype=np.uint32)   # past the arena; pos>end
    d, nmsg, err, stop = decode_dev(torch, arena, pos, end, 2)
    assert list(err[1:]) == [errno.EINVAL, errno.EINVAL]
    assert list(nmsg[1:]) == [0, 0]
    assert err[0] == errno.EBADMSG                 # zeros: version 0
    L = P.lib()
    assert L.rtcp_decode_batch_dev(None, 0, None, None, 1, None, 0, None,
                                   None, None, None) == errno.EINVAL
    assert L.rtcp_decode_batch_dev(None, 0, None, None, 0, None, 0, None,
                                   None, None, None) == 0
