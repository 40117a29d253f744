"""Golden-vector loading and replay (test infrastructure).

tests/golden/srtp_golden.json.gz is produced by oracle/gen_golden.c, which
drives the reference libre src/srtp (compiled from /root/reference by
oracle/Makefile) exactly as test/srtp.c does, recording every call's inputs
and outputs.  `replay_scenario` re-runs a scenario through any backend that
exposes the re_srtp.h API shape and reports the first mismatch.
"""
import gzip
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "srtp_golden.json.gz")

_cache = None


def load_golden():
    global _cache
    if _cache is None:
        with gzip.open(GOLDEN, "rt") as f:
            _cache = json.load(f)
    return _cache


OPS = ("srtp_encrypt", "srtp_decrypt", "srtcp_encrypt", "srtcp_decrypt")


def replay_scenario(backend, scn):
    """backend: object with alloc(suite, key, flags)->ctx, free(ctx),
    call(ctx, opname, size, pos, end, inbytes)->(err,pos,end,size,bytes).
    Returns None on success, else a description of the first mismatch."""
    ctxs = []
    try:
        for c in scn["ctxs"]:
            ctx, err = backend.alloc(c["suite"], bytes.fromhex(c["key"]),
                                     c["flags"])
            if err:
                return "%s: alloc err %d" % (scn["name"], err)
            ctxs.append(ctx)
        for i, op in enumerate(scn["ops"]):
            inb = bytes.fromhex(op["in"])
            out = bytes.fromhex(op["out"])
            # gen_golden builds the mbuf with mbuf_alloc(size), which turns
            # size 0 into DEFAULT_SIZE=512 (src/mbuf/mbuf.c:18,44)
            err, pos, end, size, buf = backend.call(
                ctxs[op["ctx"]], op["op"], op["size"] or 512, op["pos"],
                op["end"], inb, len(out))
            exp = (op["err"], op["pos_o"], op["end_o"], op["size_o"])
            got = (err, pos, end, size)
            if got != exp:
                return "%s op#%d %s: (err,pos,end,size) got %r want %r" % (
                    scn["name"], i, op["op"], got, exp)
            if buf[:len(out)] != out:
                j = next(k for k in range(len(out)) if buf[k] != out[k])
                return "%s op#%d %s: byte %d differs (len %d)" % (
                    scn["name"], i, op["op"], j, len(out))
    finally:
        for c in ctxs:
            backend.free(c)
    return None
