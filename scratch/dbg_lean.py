"""debug: lean CTR kernel unprotect vs oracle, per length, batch and single"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_fastpath import rtp_packet, to_arena, run

torch.cuda.set_device(0)
P.load()
key = bytes(range(30))
rng = np.random.default_rng(5)
be = O.OracleBackend()
for cc in (0, 1):
    pkts = [(0, rtp_packet(rng, 100 + i, 0x2468, cc=cc, plen=plen))
            for i, plen in enumerate(range(261))]
    octx = be.alloc(1, key, 0)[0]
    prot = []
    for _, p in pkts:
        e, po, en, _, buf = be.call(octx, "srtp_encrypt", len(p) + 64, 0, len(p), p, len(p) + 16)
        prot.append((0, bytes(buf[:en])))
    a2, p2, e2, c2, _ = to_arena(prot)
    for mode in ("lean", "nolean"):
        with P.tune(nolean=1 if mode == "nolean" else 0):
            rx = P.Srtp(1, key)
            dec = run(torch, "srtp_decrypt", [rx], a2, p2, e2, c2, None, False)
        bad = np.flatnonzero(dec[3])
        print("cc", cc, mode, "batch errors at", bad.tolist(), flush=True)
    for mode in ("lean", "nolean"):
        badl = []
        for i, q in enumerate(prot):
            a3, p3, e3, c3, _ = to_arena([q])
            rx = P.Srtp(1, key)
            with P.tune(nolean=1 if mode == "nolean" else 0, trace=1):
                d = run(torch, "srtp_decrypt", [rx], a3, p3, e3, c3, None, False)
            if d[3][0]:
                badl.append(i)
        print("cc", cc, mode, "single-packet errors", badl, flush=True)
