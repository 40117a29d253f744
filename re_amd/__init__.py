"""re_amd -- MI355X-native SRTP/SRTCP (drop-in for libre src/srtp).

The product is the C-ABI shared library ``re_amd/lib/libre_srtp_amd.so``
(host C state machine + hand-written gfx950 HIP kernels) exporting exactly
libre's ``include/re_srtp.h`` API plus the batch extension in
``include/re_srtp_batch.h``.  This Python package is a thin ctypes mirror of
that interface used by the tests and ``bench.py``; it never computes any
cipher or MAC itself and refuses to run when the library is missing.
"""
from .srtp import (  # noqa: F401
    LIB_PATH, lib, load, Mbuf, Srtp, SrtpBatch, StreamState, SUITES,
    SRTP_UNENCRYPTED_SRTCP, EAUTH, suite_name, key_len, salt_len, tag_len,
    batch_run, device_batch, alloc_many,
)
