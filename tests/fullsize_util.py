"""Whole-arena digests of BASELINE.json configs (tests/golden/
fullsize_digests.json, written by scripts/make_fullsize_digests.sh from
the reference src/srtp -- oracle/ref_digest.c).  Shared by the CPU tests
(workload generator and oracle vs the reference) and the -m gpu tests
(the HIP path vs the reference at full size)."""
import hashlib
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "tests", "golden", "fullsize_digests.json")
BLOCK = 65536          # packets per block digest (ref_digest.c BLOCK_PKTS)


def load():
    with open(PATH) as f:
        return {c["config"]: c for c in json.load(f)["configs"]}


def sha(b):
    return hashlib.sha256(memoryview(np.ascontiguousarray(b)).cast("B")
                          ).hexdigest()


def block_digests(arena, n, slot):
    a = arena.reshape(n, slot)
    return [sha(a[k:k + BLOCK]) for k in range(0, n, BLOCK)]


def state_bytes(rows):
    """rows: [(roc, s_l, lix, bitmap)] per session -> ref_digest layout"""
    dt = np.dtype([("roc", "<u4"), ("s_l", "<u4"), ("lix", "<u8"),
                   ("bitmap", "<u8")])
    a = np.zeros(len(rows), dtype=dt)
    for k, r in enumerate(rows):
        a[k] = r
    return a.tobytes()


def compare(ref, arena, n, slot, end, err, states):
    """list of mismatch descriptions (empty: identical to the reference)"""
    bad = []
    if sha(arena) != ref["arena"]:
        blocks = block_digests(arena, n, slot)
        bad.append(("arena", [k for k, (x, y) in
                              enumerate(zip(blocks, ref["blocks"]))
                              if x != y]))
    if sha(np.asarray(end, dtype="<u4")) != ref["end"]:
        bad.append("end")
    if sha(np.asarray(err, dtype="<i4")) != ref["err"]:
        bad.append(("err", int(np.count_nonzero(err)), ref["nerr"]))
    if hashlib.sha256(states).hexdigest() != ref["states"]:
        bad.append(("states", states[:24].hex(), ref.get("state0")))
    return bad
