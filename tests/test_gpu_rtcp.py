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
  * windows outside the arena give EINVAL, never a read out of bounds;
  * message contents (rtcp_decode_full_batch_dev): every golden packet's
    items equal the reference's struct rtcp_msg fields and copied data;
  * compound encode (rtcp_encode_batch_dev): the 1500 reference
    rtcp_encode goldens byte-exact (or their errno), ENOMEM past cap;
  * the report path at scale: 256K SR + SDES CNAME compounds encoded,
    SRTCP-protected and -unprotected, decoded back field for field.
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


# ---- message contents (rtcp_decode_full_batch_dev) ------------------------

def decode_full_dev(torch, arena, pos, end, maxmsg, maxitem):
    n = len(pos)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    d_arena, d_pos, d_end = t(arena), t(pos.view(np.int32)), \
        t(end.view(np.int32))
    desc = torch.full((n * maxmsg * 5 + 1,), -1, dtype=torch.int32,
                      device="cuda")
    item = torch.full((n * maxitem * 8 + 1,), -1, dtype=torch.int32,
                      device="cuda")
    nmsg, nitem, err, stop = (torch.full((n,), -1, dtype=torch.int32,
                                         device="cuda") for _ in range(4))
    torch.cuda.synchronize()
    rc = P.rtcp_decode_full_dev(d_arena.data_ptr(), d_arena.numel(),
                                d_pos.data_ptr(), d_end.data_ptr(), n,
                                desc.data_ptr(), maxmsg, nmsg.data_ptr(),
                                item.data_ptr(), maxitem, nitem.data_ptr(),
                                err.data_ptr(), stop.data_ptr())
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    u = lambda x: x.cpu().numpy().view(np.uint32)
    return (u(desc)[:-1].reshape(n, maxmsg, 5), u(nmsg),
            u(item)[:-1].reshape(n, maxitem, 8), u(nitem),
            err.cpu().numpy(), u(stop))


# item kinds whose data the reference copies out (offset word, data length
# word): SDES item data, BYE reason, APP data
COPIED = {4: (1, 0), 6: (1, 0), 7: (2, 3)}


def item_row(pkt, w):
    """a device item as the golden's [msg, kind, sub, v0..v6, hex]"""
    w = [int(x) for x in w]
    msg, kind, sub = w[0] & 0xffff, (w[0] >> 16) & 0xff, w[0] >> 24
    v = w[1:8]
    data = b""
    if kind in COPIED:
        o, ln = COPIED[kind]
        data = pkt[v[o]:v[o] + v[ln]]
        if kind == 6:           # a C string: the reference's strlen
            data = data.split(b"\0")[0]
            v[ln] = len(data)
        v[o] = 0
    return [msg, kind, sub] + v + [data.hex()]


def test_rtcp_decode_items_vs_reference(torch_cuda):
    """every golden packet's message contents (report blocks, SDES chunks
    and items, BYE sources and reason, APP data, NACK / GNACK / TWCC / SLI
    / AFB / FIR FCI, XR blocks) equal what the reference's rtcp_decode put
    in struct rtcp_msg"""
    cases = load_cases()
    pkts = [bytes.fromhex(c["pkt"]) for c in cases]
    arena, pos, end = pack(pkts)
    maxmsg = max(len(c["msgs"]) for c in cases)
    maxitem = max(len(c["items"]) for c in cases)
    d, nmsg, it, nitem, err, stop = decode_full_dev(torch_cuda, arena, pos,
                                                    end, maxmsg, maxitem)
    total = 0
    for i, c in enumerate(cases):
        assert [rows(d[i], k) for k in range(nmsg[i])] == c["msgs"], i
        assert (int(err[i]), int(stop[i])) == (c["err"], c["stop"]), i
        assert int(nitem[i]) == len(c["items"]), i
        got = [item_row(pkts[i], it[i, k]) for k in range(nitem[i])]
        assert got == c["items"], (i, got, c["items"])
        total += len(got)
    assert total > 6000
    # maxitem smaller than some packets need: counted, the first written
    d2, nm2, it2, ni2, e2, s2 = decode_full_dev(torch_cuda, arena, pos, end,
                                                maxmsg, 3)
    assert (ni2 == nitem).all()
    for i in range(len(cases)):
        k = min(3, int(nitem[i]))
        assert (it2[i, :k] == it[i, :k]).all(), i


# ---- compound encode (rtcp_encode_batch_dev) -------------------------------

def encode_inputs(cases, slot=1024):
    """the golden specs as one batch: arrays concatenated, references
    rebased"""
    from tests.test_rtcp_cpu import load_encode_cases  # noqa: F401
    dm, drb, dch, dsd = P.rtcp_enc_dtypes()
    msgs, rbs, chs, sds, srcs, pool, mfirst = [], [], [], [], [], [], [0]
    for c in cases:
        b_rb, b_ch, b_sd, b_src = len(rbs), len(chs), len(sds), len(srcs)
        b_pool = sum(len(x) for x in pool)
        for m in c["msgs"]:
            pt = m[0]
            first = m[9] + (b_rb if pt in (200, 201) else
                            b_ch if pt == 202 else
                            b_src if pt == 203 else 0)
            msgs.append((pt, m[1], m[2], m[3:9], first, m[10],
                         m[12] + b_pool, m[13]))
        rbs += [tuple(r) for r in c["rb"]]
        chs += [(ch[0], ch[1] + b_sd, ch[2]) for ch in c["chunks"]]
        sds += [(s[0], 0, s[1], s[2] + b_pool) for s in c["sdes"]]
        srcs += c["srcs"]
        pool.append(bytes.fromhex(c["pool"]))
        mfirst.append(len(msgs))
    n = len(cases)
    A = dict(msg=np.array(msgs, dtype=dm), rb=np.array(rbs, dtype=drb),
             chunk=np.array(chs, dtype=dch), sdes=np.array(sds, dtype=dsd),
             src=np.array(srcs, dtype=np.uint32),
             pool=np.frombuffer(b"".join(pool) or b"\0", dtype=np.uint8),
             mfirst=np.array(mfirst, dtype=np.uint32))
    pos = np.arange(n, dtype=np.uint32) * slot
    return A, pos, pos + slot


def encode_dev(torch, A, pos, cap, arena_bytes):
    n = len(pos)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(
        np.uint8)).cuda()
    dA = {k: t(v) for k, v in A.items()}
    arena = torch.full((arena_bytes,), 0xEE, dtype=torch.uint8,
                       device="cuda")
    d_pos, d_cap = t(pos), t(cap)
    d_end = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    err = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    rc = P.rtcp_encode_dev(arena.data_ptr(), arena.numel(), d_pos.data_ptr(),
                           d_end.data_ptr(), d_cap.data_ptr(), n,
                           dA["mfirst"].data_ptr(), dA["msg"].data_ptr(),
                           len(A["msg"]), dA["rb"].data_ptr(), len(A["rb"]),
                           dA["chunk"].data_ptr(), len(A["chunk"]),
                           dA["sdes"].data_ptr(), len(A["sdes"]),
                           dA["src"].data_ptr(), len(A["src"]),
                           dA["pool"].data_ptr(), len(A["pool"]),
                           err.data_ptr())
    assert rc == 0, (rc, P.lib().srtp_gpu_error())
    torch.cuda.synchronize()
    return arena, d_end.cpu().numpy().view(np.uint32), err.cpu().numpy()


def test_rtcp_encode_vs_reference(torch_cuda):
    """1500 compounds in one batch, each byte-exact with the reference's
    rtcp_encode calls (tests/golden/rtcp_encode_golden.json.gz: SR/RR with
    report blocks, SDES chunks, BYE with and without reason -- also one
    over 255 bytes --, APP, FIR, NACK, RTPFB/PSFB/XR handler bytes, header
    counts past 31), or its errno (EINVAL, EBADMSG) with nothing written"""
    from tests.test_rtcp_cpu import load_encode_cases
    cases = load_encode_cases()
    A, pos, cap = encode_inputs(cases)
    arena, end, err = encode_dev(torch_cuda, A, pos, cap, int(cap[-1]))
    host = arena.cpu().numpy()
    for i, c in enumerate(cases):
        assert int(err[i]) == c["err"], i
        if c["err"]:
            assert end[i] == pos[i], i
            assert (host[pos[i]:cap[i]] == 0xEE).all(), i
            continue
        assert host[pos[i]:end[i]].tobytes().hex() == c["out"], i
        assert (host[end[i]:cap[i]] == 0xEE).all(), i
    # room short by one byte: ENOMEM for exactly the packets that needed
    # it all, nothing written
    need = np.array([len(c["out"]) // 2 for c in cases], dtype=np.uint32)
    ok = np.array([c["err"] == 0 for c in cases])
    cap2 = pos + np.where(ok, need - 1, 1024).astype(np.uint32)
    arena2, end2, err2 = encode_dev(torch_cuda, A, pos, cap2, int(cap[-1]))
    assert (err2[ok & (need > 0)] == errno.ENOMEM).all()
    assert (end2[ok] == pos[ok]).all()


def test_rtcp_encode_bad_arguments(torch_cuda):
    import ctypes
    L = P.lib()
    assert L.rtcp_encode_batch_dev(None) == errno.EINVAL
    b = P.RtcpEncBatch()
    assert L.rtcp_encode_batch_dev(ctypes.byref(b)) == 0          # n = 0
    b.n = 1
    assert L.rtcp_encode_batch_dev(ctypes.byref(b)) == errno.EINVAL


def test_rtcp_report_round_trip(torch_cuda):
    """the sender's report path on the device at scale: 256K SR + report
    block + SDES CNAME compounds (libre's rtcp_sess report shape) encoded,
    SRTCP-protected and -unprotected in place on one stream, then decoded
    with their contents: every field and CNAME byte comes back"""
    torch = torch_cuda
    n = 1 << 18
    rng = np.random.default_rng(314)
    dm, drb, dch, dsd = P.rtcp_enc_dtypes()
    msg = np.zeros(2 * n, dtype=dm)
    msg["pt"][0::2], msg["pt"][1::2] = 200, 202
    msg["count"][0::2] = 1
    msg["count"][1::2] = 1
    w = rng.integers(0, 2**32, (n, 6), dtype=np.uint64).astype(np.uint32)
    w[:, 0] = 0x5EED0001        # one sender: the session's one SSRC
    msg["w"][0::2] = w
    msg["first"][0::2] = np.arange(n)
    msg["num"][0::2] = 1
    msg["first"][1::2] = np.arange(n)
    msg["num"][1::2] = 1
    rb = np.zeros(n, dtype=drb)
    for f in drb.names:
        rb[f] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    cname_len = rng.integers(1, 40, n).astype(np.uint32)
    pool_off = np.concatenate([[0], np.cumsum(cname_len)[:-1]]).astype(
        np.uint32)
    pool = rng.integers(33, 127, int(cname_len.sum()), dtype=np.uint8)
    chunk = np.zeros(n, dtype=dch)
    chunk["src"] = w[:, 0]
    chunk["first"] = np.arange(n)
    chunk["num"] = 1
    sdes = np.zeros(n, dtype=dsd)
    sdes["type"] = 1                        # CNAME
    sdes["len"] = cname_len
    sdes["off"] = pool_off
    A = dict(msg=msg, rb=rb, chunk=chunk, sdes=sdes,
             src=np.zeros(1, dtype=np.uint32), pool=pool,
             mfirst=np.arange(0, 2 * n + 1, 2, dtype=np.uint32))
    slot = 192
    pos = np.arange(n, dtype=np.uint32) * slot
    arena, end, err = encode_dev(torch, A, pos, pos + slot, n * slot)
    assert not err.any()
    cl = cname_len.astype(np.int64)
    L = 4 + 24 + 24 + ((4 + 4 + 2 + cl + 1 + 3) & ~3)
    assert (end - pos == L).all()
    # SRTCP protect + unprotect in place
    key = bytes(range(30))
    tx, rx = P.Srtp(1, key), P.Srtp(1, key)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(
        np.int32)).cuda()
    p_d, e_d, c_d = t(pos), t(end), t(pos + slot)
    er = torch.zeros(n, dtype=torch.int32, device="cuda")
    plain = arena.clone()
    for op, ctx in (("srtcp_encrypt", tx), ("srtcp_decrypt", rx)):
        rc = P.device_batch_dev(op, [ctx], arena.data_ptr(), arena.numel(),
                                p_d.data_ptr(), e_d.data_ptr(),
                                c_d.data_ptr(), er.data_ptr(), n)
        assert rc == 0 and not bool(er.any()), op
    torch.cuda.synchronize()
    assert (e_d.cpu().numpy().view(np.uint32) == end).all()
    host = arena.cpu().numpy()
    ref = plain.cpu().numpy()
    win = np.arange(slot)[None, :] < (end - pos)[:, None]
    assert (host.reshape(n, slot)[win] == ref.reshape(n, slot)[win]).all()
    d, nmsg, it, nitem, e, s = decode_full_dev(torch, host, pos, end, 2, 5)
    assert (nmsg == 2).all() and (nitem == 4).all()
    assert (e == errno.EBADMSG).all() and (s == end - pos).all()
    kinds = (it[:, :4, 0] >> 16) & 0xff
    assert (kinds == np.array([1, 2, 3, 4])[None, :]).all()
    assert (it[:, :2, 0] & 0xffff == 0).all() and \
        (it[:, 2:4, 0] & 0xffff == 1).all()
    assert (it[:, 0, 1:6] == w[:, 1:6]).all()           # SR sender info
    assert (it[:, 1, 1] == rb["ssrc"]).all()
    assert (it[:, 1, 2] == rb["fraction"] & 0xff).all()
    assert (it[:, 1, 3] == rb["lost"] & 0xffffff).all()
    assert (it[:, 1, 4:8] == np.stack([rb[f] for f in
                                       ("last_seq", "jitter", "lsr",
                                        "dlsr")], 1)).all()
    assert (it[:, 2, 1] == w[:, 0]).all() and (it[:, 2, 2] == 1).all()
    assert (it[:, 3, 1] == cname_len).all()
    for i in range(0, n, 4099):
        o = int(pos[i] + it[i, 3, 2])
        assert host[o:o + cname_len[i]].tobytes() == \
            pool[pool_off[i]:pool_off[i] + cname_len[i]].tobytes(), i
    tx.close()
    rx.close()
