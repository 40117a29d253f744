"""Fault injection on the batch paths (srtp_gpu_tune "fail_grow": the k-th
workspace growth from now fails with ENOMEM -- the analogue of the
reference's mem_threshold_set / `retest -o`, src/mem/mem.c:45,156,
test/test.c:468-560).  A call that fails must return the errno and leave
the caller's windows exactly as it found them; the next call (no
injection) must succeed and be exact.
"""
import threading

import numpy as np
import pytest

import re_amd.srtp as P
from re_amd import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    P.load()
    return torch


def _in_thread(fn):
    """run fn in a fresh thread (fresh per-thread workspaces)"""
    out = {}

    def body():
        try:
            out["r"] = fn()
        except BaseException as e:          # noqa: B902
            out["e"] = e
    t = threading.Thread(target=body)
    t.start()
    t.join(120)
    assert not t.is_alive()
    if "e" in out:
        raise out["e"]
    return out["r"]


@pytest.mark.parametrize("op", ["srtp_encrypt", "srtp_decrypt"])
def test_failed_growth_leaves_windows(torch_cuda, op):
    torch = torch_cuda
    nsess = 256
    keys = W.make_keys(nsess, 30)
    seen = set()
    for k in range(1, 13):
        def body():
            e1, ctx = P.alloc_many(nsess, 1, keys.tobytes())
            assert not e1
            # call 1: small, 4 sessions, windows A (warms some pools)
            n1 = 64
            s1 = np.arange(n1, dtype=np.uint32) % 4
            a1, p1, q1, c1 = W.make_arena(n1, 200, sess=s1)
            d1 = torch.from_numpy(a1).cuda()
            p1 = p1 + 0
            rc, err = P.device_batch(op, ctx, d1.data_ptr(), d1.numel(),
                                     p1, q1, c1, s1)
            assert rc == 0
            # call 2: larger, all sessions, windows B; the k-th growth
            # fails
            n2 = 4096
            s2 = W.random_sessions(n2, nsess)
            a2, p2, q2, c2 = W.make_arena(n2, 1200, sess=s2)
            d2 = torch.from_numpy(a2).cuda()
            p0, q0 = p2.copy(), q2.copy()
            assert P.lib().srtp_gpu_tune(b"fail_grow", k) == 0
            try:
                rc, err = P.device_batch(op, ctx, d2.data_ptr(), d2.numel(),
                                         p2, q2, c2, s2)
            finally:
                P.lib().srtp_gpu_tune(b"fail_grow", 0)
            if rc:
                assert np.array_equal(p2, p0) and np.array_equal(q2, q0), k
            else:
                assert not err.any() or op == "srtp_decrypt"
            # and without injection the same call goes through
            if rc:
                rc2, err2 = P.device_batch(op, ctx, d2.data_ptr(),
                                           d2.numel(), p2, q2, c2, s2)
                assert rc2 == 0
            for c in ctx:
                c.close()
            return rc
        seen.add(_in_thread(body))
    import errno
    assert errno.ENOMEM in seen       # some growth was hit
