import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_fastpath import rtp_packet, to_arena, run
torch.cuda.set_device(0)
P.load()
be = O.OracleBackend()
for suite in (0, 1):
    key = bytes(range(30))
    rng = np.random.default_rng(5)
    res = []
    for plen in list(range(0, 40)) + [53, 54, 57]:
        p = rtp_packet(rng, 100, 0x2468, plen=plen)
        octx = be.alloc(suite, key, 0)[0]
        e, po, en, _, buf = be.call(octx, "srtp_encrypt", len(p) + 64, 0, len(p), p, len(p) + 16)
        q = bytes(buf[:en])
        a3, p3, e3, c3, _ = to_arena([(0, q)])
        m0 = P.counter("misses")
        rx = P.Srtp(suite, key)
        d = run(torch, "srtp_decrypt", [rx], a3, p3, e3, c3, None, False)
        res.append((plen, int(d[3][0]), P.counter("misses") - m0))
    print("suite", suite, "failing (plen, err, misses):", [r for r in res if r[1] or r[2]])
