"""Debug helper: replay tests/test_gpu_fastpath.py's mixed-traffic receive
case for one suite and report packets whose bytes differ from the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import re_amd.srtp as P
from tests import oracle_lib as O
from tests import test_gpu_fastpath as T

suite = int(sys.argv[1]) if len(sys.argv) > 1 else 0
rng = np.random.default_rng(100 + suite)
nsess, n = 3, 1500
keys = T.keys_for(suite, nsess)
pkts = T.make_traffic(rng, n, nsess)
arena, pos, end, cap, sess = T.to_arena(pkts, set())
txa = [P.Srtp(suite, k) for k in keys]
ra = T.run(torch, "srtp_encrypt", txa, arena, pos, end, cap, sess, False,
           chunk=200)
errs = ra[3]
prot = [(s, ra[0][pos[i]:ra[2][i]].tobytes()) for i, (s, _) in enumerate(pkts)
        if errs[i] == 0]
rx = []
for k, (s, p) in enumerate(prot):
    rx.append((s, p))
    r = rng.random()
    if r < 0.03:
        rx.append(prot[int(rng.integers(0, k + 1))])
    elif r < 0.05:
        q = bytearray(p)
        q[int(rng.integers(12, len(q)))] ^= 0x40
        rx.append((s, bytes(q)))
arena2, pos2, end2, cap2, sess2 = T.to_arena(rx)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/rx_%d.npz" % suite,
         data=np.frombuffer(b"".join(p for _, p in rx), dtype=np.uint8),
         lens=np.array([len(p) for _, p in rx]),
         sess=np.array([s for s, _ in rx]),
         tx=np.frombuffer(b"".join(p for _, p in pkts), dtype=np.uint8),
         txlens=np.array([len(p) for _, p in pkts]),
         txsess=np.array([s for s, _ in pkts]))
for label, env in (("any", {}), ("perclass", {"RE_SRTP_PERCLASS": "1"}),
                   ("general", {"RE_SRTP_GENERAL": "1"}),
                   ("general2", {"RE_SRTP_GENERAL": "1"}), ("any2", {})):
    for k in ("RE_SRTP_PERCLASS",):
        os.environ.pop(k, None)
    os.environ.update(env)
    rxs = [P.Srtp(suite, k) for k in keys]
    da = T.run(torch, "srtp_decrypt", rxs, arena2, pos2, end2, cap2, sess2,
               "RE_SRTP_GENERAL" in env, chunk=128)
    os.environ.pop("RE_SRTP_GENERAL", None)
    be = O.OracleBackend()
    octx = [be.alloc(suite, k, 0)[0] for k in keys]
    bad = 0
    for i, (s, p) in enumerate(rx):
        e, po, en, _, buf = be.call(octx[s], "srtp_decrypt", len(p) + 64, 0,
                                    len(p), p, len(p))
        got = da[0][pos2[i]:pos2[i] + len(buf)].tobytes()
        if got != buf or int(da[3][i]) != e:
            d = [j for j in range(len(buf)) if got[j] != buf[j]]
            if bad < 8:
                print(label, "pkt", i, "len", len(p), "err", int(da[3][i]), e,
                      "sess", s, "ndiff", len(d), "first", d[:4], "last", d[-2:],
                      "hdr", p[:2].hex())
                print("   gpu", got[max(0, d[0] - 8):d[-1] + 4].hex(),
                      "\n   ora", buf[max(0, d[0] - 8):d[-1] + 4].hex(),
                      "\n   in ", p[max(0, d[0] - 8):d[-1] + 4].hex())
            bad += 1
    print(label, "bad packets:", bad, "of", len(rx))
