"""CPU checks of the full-size reference digests (tests/golden/
fullsize_digests.json, from the reference src/srtp via oracle/ref_digest.c):

  * re_amd/workload.py builds byte-identical input arenas to the C
    generator the reference digests were computed on (configs 1-4), so the
    -m gpu full-size tests compare like with like;
  * config 1 (AES_CM_128_HMAC_SHA1_80, 1024 x 160 B, the test/srtp.c:524-528
    key, SSRC 0x01020304, seq 1..1024 -- CPU plumbing in BASELINE.json)
    through the C restatement oracle, packet by packet: protected arena,
    ends, errnos, final stream states and the unprotect round trip equal
    the reference's.
"""
import numpy as np
import pytest

from re_amd import workload as W
from tests import fullsize_util as F
from tests import oracle_lib as O


@pytest.fixture(scope="module")
def digests():
    return F.load()


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 8])
def test_workload_matches_reference_generator(digests, cfg):
    ref = digests[cfg]
    arena, pos, end, cap, sess, keys = W.build_config(cfg)
    assert len(pos) == ref["n"] and int(cap[0] - pos[0]) == ref["slot"]
    assert F.sha(arena) == ref["plain"]


def test_config1_oracle_vs_reference(digests):
    ref = digests[1]
    arena, pos, end, cap, sess, keys = W.build_config(1)
    n, slot = ref["n"], ref["slot"]
    be = O.OracleBackend()
    key = keys[0].tobytes()
    for direction in ("protect", "unprotect"):
        op = "srtp_encrypt" if direction == "protect" else "srtp_decrypt"
        ctx, e = be.alloc(1, key, 0)
        assert e == 0
        err = np.zeros(n, dtype=np.int32)
        for i in range(n):
            pkt = arena[pos[i]:end[i]].tobytes()
            e, po, eo, so, buf = be.call(ctx, op, slot, 0, len(pkt), pkt,
                                         slot)
            assert so == slot          # the slot always has room
            arena[pos[i]:pos[i] + slot] = np.frombuffer(buf[:slot],
                                                        dtype=np.uint8)
            err[i] = e
            end[i] = pos[i] + eo
        st = be.export(ctx, W.SSRC_BASE)
        be.free(ctx)
        bad = F.compare(ref[direction], arena, n, slot, end, err,
                        F.state_bytes([st]))
        assert not bad, (direction, bad)
