#!/usr/bin/env python3
"""Debug helper: single-session GCM protect/unprotect of packets of every
length 12..MAXL through the device batch API vs the oracle, one packet per
length; prints the lengths (and first byte offsets) that differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import re_amd.srtp as P
    from tests import oracle_lib as O
    suite = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    maxl = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    P.load()
    key = bytes(range(P.key_len(suite) + P.salt_len(suite)))
    rng = np.random.default_rng(1)
    lens = list(range(12, maxl + 1))
    n = len(lens)
    slot = ((maxl + 64 + 15) // 16) * 16
    arena = np.zeros(n * slot, dtype=np.uint8)
    pos = np.zeros(n, dtype=np.uint32)
    end = np.zeros(n, dtype=np.uint32)
    cap = np.zeros(n, dtype=np.uint32)
    for i, L in enumerate(lens):
        p = bytearray([0x80, 96, (i >> 8) & 0xff, i & 0xff, 0, 0, 0, 0,
                       0x12, 0x34, 0x56, 0x78])
        p += rng.integers(0, 256, L - 12, dtype=np.uint8).tobytes()
        arena[i * slot:i * slot + L] = np.frombuffer(bytes(p), np.uint8)
        pos[i], end[i], cap[i] = i * slot, i * slot + L, (i + 1) * slot
    tx = P.Srtp(suite, key)
    ob = O.OracleBackend()
    octx, _ = ob.alloc(suite, key, 0)
    dev = torch.from_numpy(arena.copy()).cuda()
    p2, e2 = pos.copy(), end.copy()
    rc, err = P.device_batch("srtp_encrypt", [tx], dev.data_ptr(),
                             arena.nbytes, p2, e2, cap)
    res = dev.cpu().numpy()
    bad = 0
    for i, L in enumerate(lens):
        pkt = arena[pos[i]:end[i]].tobytes()
        e, _, en, _, buf = ob.call(octx, "srtp_encrypt", 2048, 0, len(pkt),
                                   pkt, 0)
        got = res[p2[i]:e2[i]].tobytes()
        want = buf[:en]
        if e != err[i] or got != want:
            bad += 1
            if bad <= 12:
                diff = [k for k in range(min(len(got), len(want)))
                        if got[k] != want[k]]
                print("protect L=%d err %d/%d len %d/%d first diffs %s" % (
                    L, err[i], e, len(got), len(want), diff[:6]))
    print("protect: %d of %d lengths differ" % (bad, n))
    # unprotect the oracle's protected packets
    rx = P.Srtp(suite, key)
    octx2, _ = ob.alloc(suite, key, 0)
    arena2 = np.zeros_like(arena)
    e3 = end.copy()
    for i, L in enumerate(lens):
        pkt = arena[pos[i]:end[i]].tobytes()
        e, _, en, _, buf = ob.call(octx2, "srtp_encrypt", 2048, 0, len(pkt),
                                   pkt, 0)
        arena2[pos[i]:pos[i] + en] = np.frombuffer(buf[:en], np.uint8)
        e3[i] = pos[i] + en
    dev2 = torch.from_numpy(arena2.copy()).cuda()
    p4, e4 = pos.copy(), e3.copy()
    rc, err = P.device_batch("srtp_decrypt", [rx], dev2.data_ptr(),
                             arena2.nbytes, p4, e4, cap)
    res = dev2.cpu().numpy()
    bad = 0
    for i, L in enumerate(lens):
        got = res[p4[i]:e4[i]].tobytes()
        want = arena[pos[i]:end[i]].tobytes()
        if err[i] or got != want:
            bad += 1
            if bad <= 12:
                diff = [k for k in range(min(len(got), len(want)))
                        if got[k] != want[k]]
                print("unprotect L=%d err %d len %d/%d first diffs %s" % (
                    L, err[i], len(got), len(want), diff[:6]))
                if bad == 1:
                    print("  got  ", got[:24].hex(), "...", got[-24:].hex())
                    print("  want ", want[:24].hex(), "...", want[-24:].hex())
                    ct = arena2[pos[i]:e3[i]].tobytes()
                    print("  ct   ", ct[:24].hex(), "...", ct[-28:].hex())
                    raw = res[pos[i]:e3[i]].tobytes()
                    print("  raw  ", raw[:24].hex(), "...", raw[-28:].hex())
    for i, L in enumerate(lens):
        if L in (64, 65, 66, 68, 129):
            print("  L=%d raw tail %s | ct tail %s" % (
                L, res[pos[i] + 56:e3[i]].tobytes().hex(),
                arena2[pos[i] + 56:e3[i]].tobytes().hex()))
    print("unprotect: %d of %d lengths differ" % (bad, n))


if __name__ == "__main__":
    main()
