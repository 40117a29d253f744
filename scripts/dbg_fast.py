"""debug helper: fast path vs general engine vs oracle on the adversarial
batch of tests/test_gpu_fastpath.py (suite 0), printing mismatches"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import re_amd.srtp as P
from tests import oracle_lib as O
from tests.test_gpu_fastpath import make_traffic, keys_for, to_arena, run

suite = int(sys.argv[1]) if len(sys.argv) > 1 else 0
rng = np.random.default_rng(100 + suite)
keys = keys_for(suite, 3)
pkts = make_traffic(rng, 1500, 3)
arena, pos, end, cap, sess = to_arena(pkts)
for chunk in (None, 200):
    txa = [P.Srtp(suite, k) for k in keys]
    txb = [P.Srtp(suite, k) for k in keys]
    ra = run(torch, "srtp_encrypt", txa, arena, pos, end, cap, sess, False, chunk=chunk)
    rb = run(torch, "srtp_encrypt", txb, arena, pos, end, cap, sess, True)
    be = O.OracleBackend()
    octx = [be.alloc(suite, k, 0)[0] for k in keys]
    bad_a = bad_b = 0
    first = None
    for i, (s, p) in enumerate(pkts):
        e, po, en, _, buf = be.call(octx[s], "srtp_encrypt", len(p) + 64, 0, len(p), p, len(p) + 16)
        for name, r in (("fast", ra), ("gen", rb)):
            got = (int(r[3][i]), int(r[1][i] - pos[i]), int(r[2][i] - pos[i]))
            ok = got == (e, po, en) and (e != 0 or r[0][pos[i]:r[2][i]].tobytes() == buf[:en])
            if not ok:
                if name == "fast": bad_a += 1
                else: bad_b += 1
                if first is None:
                    first = (name, i, got, (e, po, en))
    print("chunk", chunk, "fast bad", bad_a, "general bad", bad_b, "first", first)
