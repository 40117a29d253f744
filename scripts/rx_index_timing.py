"""Cost of the cross-rank fold's index pass per 1M packets:
srtp_rx_index over a host arena vs srtp_rx_index_dev over the device
outputs of the rank's unprotect (config-2 shape, 1M x 1200 B), and
srtp_rx_fold over the records.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import re_amd.srtp as P  # noqa: E402
from re_amd import shard as S  # noqa: E402
from re_amd import workload as W  # noqa: E402

P.load()
n = 1 << 20
arena, pos, end, cap = W.make_arena(n, 1200, s0=65000)
key = W.make_keys(1, 30)[0].tobytes()
tx, rx = P.Srtp(1, key), P.Srtp(1, key)
dev = torch.from_numpy(arena).cuda()
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()
p_d, e_d, c_d = t(pos), t(end), t(cap)
err = torch.zeros(n, dtype=torch.int32, device="cuda")
for op, ctx in (("srtp_encrypt", tx), ("srtp_decrypt", rx)):
    if op == "srtp_decrypt":
        p_in, e_in = p_d.clone(), e_d.clone()
        host = dev.cpu().numpy()
        hp = p_in.cpu().numpy().view(np.uint32)
        he = e_in.cpu().numpy().view(np.uint32)
    assert P.device_batch_dev(op, [ctx], dev.data_ptr(), dev.numel(),
                              p_d.data_ptr(), e_d.data_ptr(), c_d.data_ptr(),
                              err.data_ptr(), n) == 0
torch.cuda.synchronize()
res = err.cpu().numpy()
st0 = P.StreamState()
st0.ssrc = W.SSRC_BASE
out = {"packets": n}
# the records land in a warm array (the rank's gather buffer): the C call's
# own cost, not the first touch of 16 MB of fresh pages
rec_d = np.zeros(n, dtype=S._rx_rec_dtype())
rec_d.view(np.uint8).fill(0)
for rep in range(3):
    t0 = time.perf_counter()
    rec_h = S.rx_records(st0, host, hp, he, res)
    t1 = time.perf_counter()
    S.rx_records_dev(st0, dev, p_in, e_in, err, out=rec_d)
    t2 = time.perf_counter()
    st = P.StreamState()
    st.ssrc = W.SSRC_BASE
    e, nd = S.rx_fold(st, 1, rec_d)
    t3 = time.perf_counter()
out.update(rx_index_host_ms=round((t1 - t0) * 1e3, 2),
           rx_index_dev_ms=round((t2 - t1) * 1e3, 2),
           rx_fold_ms=round((t3 - t2) * 1e3, 2),
           records_equal=bool((rec_h == rec_d).all()), ndone=int(nd),
           errors=int(np.count_nonzero(e)))
print(json.dumps(out))
