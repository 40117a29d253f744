"""ctypes mirror of include/re_srtp.h + include/re_srtp_batch.h.

Names, argument meaning and errno results follow the reference interface
(/root/reference/include/re_srtp.h:8-30).  Errors from the C library are
returned as errno integers exactly as the C functions return them.
"""
import ctypes
import errno
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RE_SRTP_LIB: an alternative build of the same library (kernel variant
# experiments, scripts/build_variants.sh); default the in-tree build
LIB_PATH = os.environ.get("RE_SRTP_LIB") or os.path.join(
    HERE, "lib", "libre_srtp_amd.so")

SRTP_AES_CM_128_HMAC_SHA1_32 = 0
SRTP_AES_CM_128_HMAC_SHA1_80 = 1
SRTP_AES_256_CM_HMAC_SHA1_32 = 2
SRTP_AES_256_CM_HMAC_SHA1_80 = 3
SRTP_AES_128_GCM = 4
SRTP_AES_256_GCM = 5
SUITES = range(6)
SRTP_UNENCRYPTED_SRTCP = 1 << 1
EAUTH = 217
EBUSY = 16      # Linux errno.h

_KEY = {0: 16, 1: 16, 2: 32, 3: 32, 4: 16, 5: 32}
_SALT = {0: 14, 1: 14, 2: 14, 3: 14, 4: 12, 5: 12}
_TAG = {0: 4, 1: 10, 2: 4, 3: 10, 4: 16, 5: 16}


def key_len(s):
    return _KEY[s]


def salt_len(s):
    return _SALT[s]


def tag_len(s):
    return _TAG[s]


class Mbuf(ctypes.Structure):
    """struct mbuf (include/re_mbuf.h:43-48)"""
    _fields_ = [("buf", ctypes.POINTER(ctypes.c_uint8)),
                ("size", ctypes.c_size_t),
                ("pos", ctypes.c_size_t),
                ("end", ctypes.c_size_t)]


class SrtpBatch(ctypes.Structure):
    """struct srtp_batch (include/re_srtp_batch.h)"""
    _fields_ = [("arena", ctypes.c_void_p),
                ("arena_size", ctypes.c_size_t),
                ("pos", ctypes.POINTER(ctypes.c_uint32)),
                ("end", ctypes.POINTER(ctypes.c_uint32)),
                ("cap", ctypes.POINTER(ctypes.c_uint32)),
                ("err", ctypes.POINTER(ctypes.c_int32)),
                ("sess", ctypes.POINTER(ctypes.c_uint32)),
                ("n", ctypes.c_size_t),
                ("stream", ctypes.c_void_p)]


class SrtpBatchDev(ctypes.Structure):
    """struct srtp_batch_dev (include/re_srtp_batch.h): every per-packet
    array is a device pointer"""
    _fields_ = [("arena", ctypes.c_void_p),
                ("arena_size", ctypes.c_size_t),
                ("pos", ctypes.c_void_p),
                ("end", ctypes.c_void_p),
                ("cap", ctypes.c_void_p),
                ("err", ctypes.c_void_p),
                ("sess", ctypes.c_void_p),
                ("n", ctypes.c_size_t),
                ("stream", ctypes.c_void_p)]


class DtlsSecret(ctypes.Structure):
    """struct srtp_dtls_secret (include/re_srtp_keying.h)"""
    _fields_ = [("master", ctypes.c_uint8 * 48),
                ("client_random", ctypes.c_uint8 * 32),
                ("server_random", ctypes.c_uint8 * 32),
                ("prf", ctypes.c_uint32)]


PRF_SHA256, PRF_SHA384 = 0, 1


class StreamState(ctypes.Structure):
    _fields_ = [("replay_rtp_bitmap", ctypes.c_uint64),
                ("replay_rtp_lix", ctypes.c_uint64),
                ("replay_rtcp_bitmap", ctypes.c_uint64),
                ("replay_rtcp_lix", ctypes.c_uint64),
                ("ssrc", ctypes.c_uint32),
                ("roc", ctypes.c_uint32),
                ("s_l", ctypes.c_uint16),
                ("s_l_set", ctypes.c_uint8),
                ("pad", ctypes.c_uint8),
                ("rtcp_index", ctypes.c_uint32)]


# enum srtp_rx_stage (include/re_srtp_batch.h)
RX_NOHDR, RX_NOIX, RX_IX = 0, 1, 2


EXPORTS = (
    "srtp_alloc", "srtp_encrypt", "srtp_decrypt", "srtcp_encrypt",
    "srtcp_decrypt", "srtp_suite_name",
    "srtp_encrypt_mbufs", "srtp_decrypt_mbufs", "srtcp_encrypt_mbufs",
    "srtcp_decrypt_mbufs", "srtp_encrypt_batch", "srtp_decrypt_batch",
    "srtcp_encrypt_batch", "srtcp_decrypt_batch", "srtp_encrypt_batch_dev",
    "srtp_decrypt_batch_dev", "srtcp_encrypt_batch_dev",
    "srtcp_decrypt_batch_dev", "srtp_encrypt_batch_dev_async",
    "srtp_decrypt_batch_dev_async", "srtp_batch_wait", "srtp_stream_export",
    "srtp_stream_import", "srtp_rx_index", "srtp_rx_fold", "srtp_alloc_many", "srtp_gpu_error",
    "srtp_gpu_prof", "srtp_gpu_prof_read", "srtp_gpu_prof_read_named",
    "srtp_gpu_tune", "srtp_gpu_counter",
    "rtcp_decode_batch_dev",
    "srtp_udp_alloc", "srtp_udp_recv", "srtp_udp_send", "srtp_udp_stats",
    "srtp_udp_pipeline", "srtp_udp_times",
    "srtp_dtls_key_size", "srtp_keyinfo_split", "srtp_dtls_keying_many",
    "srtp_alloc_dtls_many",
    "mbuf_alloc", "mbuf_resize", "mbuf_write_mem", "mem_deref", "mem_zalloc",
)

# srtp_udp_recv_h (include/re_srtp_udp.h)
UDP_RECV_H = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32,
                              ctypes.POINTER(Mbuf), ctypes.c_int,
                              ctypes.c_void_p)

_lib = None


def load():
    """Load the C-ABI library; raise (loudly) if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            "re_amd: %s missing -- run `make -C re_amd` (or "
            "__graft_entry__.build()); there is no CPU fallback" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.srtp_alloc.argtypes = [ctypes.POINTER(vp), ctypes.c_int,
                             ctypes.c_char_p, sz, ctypes.c_int]
    for f in ("srtp_encrypt", "srtp_decrypt", "srtcp_encrypt",
              "srtcp_decrypt"):
        getattr(L, f).argtypes = [vp, ctypes.POINTER(Mbuf)]
        getattr(L, f + "_mbufs").argtypes = [
            vp, ctypes.POINTER(ctypes.POINTER(Mbuf)),
            ctypes.POINTER(ctypes.c_int), sz]
        getattr(L, f + "_batch").argtypes = [
            ctypes.POINTER(vp), sz, ctypes.POINTER(SrtpBatch)]
        getattr(L, f + "_batch_dev").argtypes = [
            ctypes.POINTER(vp), sz, ctypes.POINTER(SrtpBatchDev)]
    for f in ("srtp_encrypt", "srtp_decrypt"):
        getattr(L, f + "_batch_dev_async").argtypes = [
            ctypes.POINTER(vp), sz, ctypes.POINTER(SrtpBatchDev),
            ctypes.POINTER(vp)]
    L.srtp_batch_wait.argtypes = [vp]
    L.srtp_suite_name.restype = ctypes.c_char_p
    L.srtp_suite_name.argtypes = [ctypes.c_int]
    L.srtp_gpu_error.restype = ctypes.c_char_p
    L.srtp_stream_export.argtypes = [vp, ctypes.c_uint32,
                                     ctypes.POINTER(StreamState)]
    L.srtp_stream_import.argtypes = [vp, ctypes.POINTER(StreamState)]
    L.srtp_alloc_many.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_int,
                                  ctypes.c_char_p, sz, ctypes.c_int]
    L.srtp_rx_index.argtypes = [ctypes.POINTER(StreamState), vp, vp, vp, vp,
                                sz, vp]
    L.srtp_rx_index_dev.argtypes = [ctypes.POINTER(StreamState), vp, sz, vp,
                                    vp, vp, sz, vp, vp]
    L.srtp_rx_fold.argtypes = [ctypes.POINTER(StreamState), ctypes.c_int, vp,
                               sz, vp, ctypes.POINTER(sz)]
    L.srtp_gpu_prof.argtypes = [ctypes.c_int]
    L.srtp_gpu_tune.argtypes = [ctypes.c_char_p, ctypes.c_long]
    L.srtp_gpu_counter.argtypes = [ctypes.c_char_p]
    L.srtp_gpu_counter.restype = ctypes.c_uint64
    L.srtp_gpu_prof_read.argtypes = [ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_uint64)]
    L.rtcp_decode_batch_dev.argtypes = [vp, sz, vp, vp, sz, vp,
                                        ctypes.c_uint32, vp, vp, vp, vp]
    L.rtcp_decode_full_batch_dev.argtypes = [vp, sz, vp, vp, sz, vp,
                                             ctypes.c_uint32, vp, vp,
                                             ctypes.c_uint32, vp, vp, vp, vp]
    L.rtcp_encode_batch_dev.argtypes = [ctypes.POINTER(RtcpEncBatch)]
    L.srtp_udp_alloc.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp, vp,
                                 sz, sz, UDP_RECV_H, vp]
    L.srtp_udp_recv.argtypes = [vp, ctypes.c_int]
    L.srtp_udp_send.argtypes = [vp, vp, ctypes.c_uint32,
                                ctypes.POINTER(ctypes.POINTER(Mbuf)),
                                ctypes.POINTER(ctypes.c_int), sz]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.srtp_udp_stats.argtypes = [vp, u64p, u64p, u64p]
    L.srtp_udp_pipeline.argtypes = [vp, ctypes.c_int]
    L.srtp_udp_times.argtypes = [vp, u64p]
    L.srtp_dtls_key_size.argtypes = [ctypes.c_int]
    L.srtp_dtls_key_size.restype = sz
    L.srtp_keyinfo_split.argtypes = [ctypes.c_int, ctypes.c_char_p,
                                     ctypes.c_char_p, sz, ctypes.c_char_p,
                                     sz]
    L.srtp_dtls_keying_many.argtypes = [ctypes.POINTER(DtlsSecret), sz,
                                        ctypes.c_int, ctypes.c_char_p,
                                        ctypes.c_char_p]
    L.srtp_alloc_dtls_many.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                       sz, ctypes.c_int,
                                       ctypes.POINTER(DtlsSecret),
                                       ctypes.c_int, ctypes.c_int]
    L.mbuf_alloc.restype = ctypes.POINTER(Mbuf)
    L.mbuf_alloc.argtypes = [sz]
    L.mbuf_resize.argtypes = [ctypes.POINTER(Mbuf), sz]
    L.mbuf_write_mem.argtypes = [ctypes.POINTER(Mbuf), ctypes.c_char_p, sz]
    L.mem_deref.restype = vp
    L.mem_deref.argtypes = [vp]
    _lib = L
    return L


def lib():
    return load()


def suite_name(suite):
    return lib().srtp_suite_name(suite).decode()


class Srtp:
    """Owning handle around `struct srtp *` (freed with mem_deref)."""

    def __init__(self, suite, key, flags=0):
        L = lib()
        self.ptr = ctypes.c_void_p()
        self.err = L.srtp_alloc(ctypes.byref(self.ptr), suite, key, len(key),
                                flags)
        self.suite = suite

    @classmethod
    def wrap(cls, ptr, suite):
        o = cls.__new__(cls)
        o.ptr = ctypes.c_void_p(ptr)
        o.err = 0
        o.suite = suite
        return o

    def close(self):
        if self.ptr:
            lib().mem_deref(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _op(self, name, mb):
        return getattr(lib(), name)(self.ptr, mb)

    def encrypt(self, mb):
        return self._op("srtp_encrypt", mb)

    def decrypt(self, mb):
        return self._op("srtp_decrypt", mb)

    def rtcp_encrypt(self, mb):
        return self._op("srtcp_encrypt", mb)

    def rtcp_decrypt(self, mb):
        return self._op("srtcp_decrypt", mb)

    def export(self, ssrc):
        st = StreamState()
        e = lib().srtp_stream_export(self.ptr, ssrc, ctypes.byref(st))
        return e, st

    def import_(self, st):
        return lib().srtp_stream_import(self.ptr, ctypes.byref(st))


def alloc_many(n, suite, keys, flags=0):
    """srtp_alloc_many: n sessions in one GPU setup launch."""
    arr = (ctypes.c_void_p * n)()
    klen = key_len(suite) + salt_len(suite)
    e = lib().srtp_alloc_many(arr, n, suite, keys, klen, flags)
    if e:
        return e, []
    return 0, [Srtp.wrap(arr[i], suite) for i in range(n)]


class SrtpUdp:
    """struct srtp_udp (include/re_srtp_udp.h): GPU SRTP between a UDP
    socket and the RTP layer.  handler(src_bytes, mbuf, err) per datagram;
    the mbuf views the receive arena only during the call."""

    STAGES = ("rx_syscall", "rx_gpu", "rx_deliver", "tx_stage", "tx_gpu",
              "tx_syscall")

    def __init__(self, fd, rx=None, tx=None, batch=256, slot=1536,
                 handler=None, pipeline=False):
        # no Python handler: no per-datagram callback at all (the helper
        # still counts received / authentic datagrams, srtp_udp_stats)
        self._cb = UDP_RECV_H(self._recv) if handler else UDP_RECV_H()
        self.handler = handler
        self.ptr = ctypes.c_void_p()
        self.err = lib().srtp_udp_alloc(
            ctypes.byref(self.ptr), fd, rx.ptr if rx else None,
            tx.ptr if tx else None, batch, slot, self._cb, None)
        if not self.err and pipeline:
            self.err = lib().srtp_udp_pipeline(self.ptr, 1)

    def times(self):
        """seconds per stage (srtp_udp_times)"""
        ns = (ctypes.c_uint64 * len(self.STAGES))()
        lib().srtp_udp_times(self.ptr, ns)
        return {k: ns[i] * 1e-9 for i, k in enumerate(self.STAGES)}

    def _recv(self, src, srclen, mb, err, arg):
        if self.handler:
            self.handler(ctypes.string_at(src, srclen), mb, err)

    def recv(self, timeout_ms=100):
        return lib().srtp_udp_recv(self.ptr, timeout_ms)

    def send(self, addr, mbufs):
        """addr: bytes of a struct sockaddr; returns (sent, errs)"""
        n = len(mbufs)
        arr = (ctypes.POINTER(Mbuf) * n)(*mbufs)
        errs = (ctypes.c_int * n)()
        r = lib().srtp_udp_send(self.ptr, addr, len(addr), arr, errs, n)
        return r, list(errs)

    def stats(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lib().srtp_udp_stats(self.ptr, ctypes.byref(a), ctypes.byref(b),
                             ctypes.byref(c))
        return a.value, b.value, c.value

    def close(self):
        if self.ptr:
            lib().mem_deref(self.ptr)
            self.ptr = ctypes.c_void_p()


def sockaddr_in(host, port):
    """struct sockaddr_in bytes (AF_INET) for srtp_udp_send"""
    import socket
    import struct
    return struct.pack("<H", socket.AF_INET) + struct.pack(">H", port) + \
        socket.inet_aton(host) + bytes(8)


def dtls_secrets(items):
    """[(master 48 B, client_random 32 B, server_random 32 B[, prf])] ->
    array (prf: PRF_SHA256 (default) or PRF_SHA384)"""
    arr = (DtlsSecret * max(1, len(items)))()
    for i, it in enumerate(items):
        m, c, r = it[:3]
        ctypes.memmove(arr[i].master, m, 48)
        ctypes.memmove(arr[i].client_random, c, 32)
        ctypes.memmove(arr[i].server_random, r, 32)
        arr[i].prf = it[3] if len(it) > 3 else PRF_SHA256
    return arr


def keyinfo_split(suite, keymat):
    """srtp_keyinfo_split -> (err, cli_key, srv_key)"""
    n = lib().srtp_dtls_key_size(suite)
    cli, srv = ctypes.create_string_buffer(64), ctypes.create_string_buffer(64)
    e = lib().srtp_keyinfo_split(suite, keymat, cli, 64, srv, 64)
    return e, cli.raw[:n], srv.raw[:n]


def dtls_keying_many(suite, items):
    """srtp_dtls_keying_many -> (err, [cli_key], [srv_key])"""
    n, size = len(items), lib().srtp_dtls_key_size(suite)
    cli = ctypes.create_string_buffer(max(1, n * size))
    srv = ctypes.create_string_buffer(max(1, n * size))
    e = lib().srtp_dtls_keying_many(dtls_secrets(items), n, suite, cli, srv)
    return e, [cli.raw[i * size:(i + 1) * size] for i in range(n)], \
        [srv.raw[i * size:(i + 1) * size] for i in range(n)]


def alloc_dtls_many(suite, items, is_client, flags=0):
    """srtp_alloc_dtls_many -> (err, [tx Srtp], [rx Srtp])"""
    n = len(items)
    tx, rx = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
    e = lib().srtp_alloc_dtls_many(tx, rx, n, suite, dtls_secrets(items),
                                   1 if is_client else 0, flags)
    if e:
        return e, [], []
    return 0, [Srtp.wrap(tx[i], suite) for i in range(n)], \
        [Srtp.wrap(rx[i], suite) for i in range(n)]


def new_mbuf(data, size, pos=0):
    """mbuf with buf[0:len(data)] = data, bytes [len, size) zero."""
    L = lib()
    mb = L.mbuf_alloc(size)
    ctypes.memset(mb.contents.buf, 0, mb.contents.size)
    if data:
        ctypes.memmove(mb.contents.buf, data, len(data))
    mb.contents.pos = pos
    mb.contents.end = len(data)
    return mb


def mbuf_bytes(mb, n=None):
    m = mb.contents
    return ctypes.string_at(m.buf, m.end if n is None else n)


def free_mbuf(mb):
    lib().mem_deref(ctypes.cast(mb, ctypes.c_void_p))


_OPS = {"srtp_encrypt": "srtp_encrypt", "srtp_decrypt": "srtp_decrypt",
        "srtcp_encrypt": "srtcp_encrypt", "srtcp_decrypt": "srtcp_decrypt"}


def batch_run(ctx, opname, mbufs):
    """srtp_*_mbufs over a list of mbuf pointers; returns (rc, errs)."""
    n = len(mbufs)
    arr = (ctypes.POINTER(Mbuf) * n)(*mbufs)
    errs = (ctypes.c_int * n)()
    rc = getattr(lib(), opname + "_mbufs")(ctx.ptr, arr, errs, n)
    return rc, list(errs)


def device_batch(opname, sessions, arena_ptr, arena_size, pos, end, cap,
                 sess_idx=None, stream=None, err=None):
    """srtp_*_batch on a device arena.  pos/end/cap: numpy uint32 arrays
    (pos/end updated in place); err: optional int32 output array.
    Returns (rc, err numpy int32)."""
    import numpy as np
    n = len(pos)
    assert pos.dtype == np.uint32 and end.dtype == np.uint32
    cap = np.ascontiguousarray(cap, dtype=np.uint32)
    if err is None:
        err = np.zeros(n, dtype=np.int32)
    assert err.dtype == np.int32 and len(err) == n
    b = SrtpBatch()
    b.arena = arena_ptr
    b.arena_size = arena_size
    b.pos = pos.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    b.end = end.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    b.cap = cap.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    b.err = err.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    if sess_idx is not None:
        sess_idx = np.ascontiguousarray(sess_idx, dtype=np.uint32)
        b.sess = sess_idx.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    b.n = n
    b.stream = stream
    sv = session_array(sessions)
    rc = getattr(lib(), opname + "_batch")(sv, len(sv), ctypes.byref(b))
    return rc, err


def session_array(sessions):
    """`struct srtp *sessv[]` for the batch calls.  Build it once per
    session set (O(sessions) Python work) and pass it back in."""
    if isinstance(sessions, ctypes.Array):
        return sessions
    return (ctypes.c_void_p * len(sessions))(*[s.ptr.value for s in sessions])


def device_batch_dev(opname, sessions, arena_ptr, arena_size, pos_ptr,
                     end_ptr, cap_ptr, err_ptr, n, sess_ptr=None,
                     stream=None):
    """srtp_*_batch_dev: arena and every per-packet array (uint32 pos/end/
    cap, int32 err, optional uint32 sess) are device pointers; pos/end/err
    are updated on the device.  Returns rc."""
    b = SrtpBatchDev()
    b.arena = arena_ptr
    b.arena_size = arena_size
    b.pos, b.end, b.cap, b.err = pos_ptr, end_ptr, cap_ptr, err_ptr
    b.sess = sess_ptr
    b.n = n
    b.stream = stream
    sv = session_array(sessions)
    return getattr(lib(), opname + "_batch_dev")(sv, len(sv),
                                                 ctypes.byref(b))


class RtcpEncBatch(ctypes.Structure):
    """struct rtcp_enc_batch (include/re_rtcp_batch.h); every pointer is
    device memory"""
    _fields_ = [("arena", ctypes.c_void_p), ("arena_size", ctypes.c_size_t),
                ("pos", ctypes.c_void_p), ("end", ctypes.c_void_p),
                ("cap", ctypes.c_void_p), ("mfirst", ctypes.c_void_p),
                ("msgv", ctypes.c_void_p), ("rbv", ctypes.c_void_p),
                ("chunkv", ctypes.c_void_p), ("sdesv", ctypes.c_void_p),
                ("srcv", ctypes.c_void_p), ("pool", ctypes.c_void_p),
                ("nmsg", ctypes.c_uint32), ("nrb", ctypes.c_uint32),
                ("nchunk", ctypes.c_uint32), ("nsdes", ctypes.c_uint32),
                ("nsrc", ctypes.c_uint32), ("pool_size", ctypes.c_uint32),
                ("err", ctypes.c_void_p), ("n", ctypes.c_size_t),
                ("stream", ctypes.c_void_p)]


# numpy layouts of the encode inputs (include/re_rtcp_batch.h)
def rtcp_enc_dtypes():
    import numpy as np
    msg = np.dtype([("pt", "u1"), ("count", "u1"), ("flags", "<u2"),
                    ("w", "<u4", (6,)), ("first", "<u4"), ("num", "<u4"),
                    ("off", "<u4"), ("len", "<u4")])
    rb = np.dtype([("ssrc", "<u4"), ("fraction", "<u4"), ("lost", "<u4"),
                   ("last_seq", "<u4"), ("jitter", "<u4"), ("lsr", "<u4"),
                   ("dlsr", "<u4")])
    chunk = np.dtype([("src", "<u4"), ("first", "<u4"), ("num", "<u4")])
    sdes = np.dtype([("type", "u1"), ("pad", "u1"), ("len", "<u2"),
                     ("off", "<u4")])
    assert msg.itemsize == 44 and rb.itemsize == 28 and sdes.itemsize == 8
    return msg, rb, chunk, sdes


def rtcp_encode_dev(arena_ptr, arena_size, pos_ptr, end_ptr, cap_ptr, n,
                    mfirst_ptr, msg_ptr, nmsg, rb_ptr=None, nrb=0,
                    chunk_ptr=None, nchunk=0, sdes_ptr=None, nsdes=0,
                    src_ptr=None, nsrc=0, pool_ptr=None, pool_size=0,
                    err_ptr=None, stream=None):
    """rtcp_encode_batch_dev over device arrays; returns rc"""
    b = RtcpEncBatch(arena_ptr, arena_size, pos_ptr, end_ptr, cap_ptr,
                     mfirst_ptr, msg_ptr, rb_ptr, chunk_ptr, sdes_ptr,
                     src_ptr, pool_ptr, nmsg, nrb, nchunk, nsdes, nsrc,
                     pool_size, err_ptr, n, stream)
    return lib().rtcp_encode_batch_dev(ctypes.byref(b))


def rtcp_decode_full_dev(arena_ptr, arena_size, pos_ptr, end_ptr, n,
                         desc_ptr, maxmsg, nmsg_ptr, item_ptr, maxitem,
                         nitem_ptr, err_ptr, stop_ptr, stream=None):
    """rtcp_decode_full_batch_dev: descriptors plus every message's items
    (struct rtcp_item: 8 x uint32, word 0 = msg | kind << 16 | sub << 24)"""
    return lib().rtcp_decode_full_batch_dev(
        arena_ptr, arena_size, pos_ptr, end_ptr, n, desc_ptr, maxmsg,
        nmsg_ptr, item_ptr, maxitem, nitem_ptr, err_ptr, stop_ptr, stream)


def rtcp_decode_dev(arena_ptr, arena_size, pos_ptr, end_ptr, n, desc_ptr,
                    maxmsg, nmsg_ptr, err_ptr, stop_ptr, stream=None):
    """rtcp_decode_batch_dev (include/re_rtcp_batch.h): every pointer is
    device memory; desc holds n * maxmsg struct rtcp_desc (5 x uint32:
    off, size, pt | count << 8 | length << 16, ssrc, aux).  Returns rc."""
    return lib().rtcp_decode_batch_dev(arena_ptr, arena_size, pos_ptr,
                                       end_ptr, n, desc_ptr, maxmsg,
                                       nmsg_ptr, err_ptr, stop_ptr, stream)


def device_batch_dev_async(opname, sessions, arena_ptr, arena_size,
                           pos_ptr, end_ptr, cap_ptr, err_ptr, n,
                           sess_ptr=None, stream=None):
    """srtp_*_batch_dev_async: returns (rc, ticket, keepalive); pass the
    ticket to batch_wait() (the session array must outlive it: keep the
    returned keepalive until then)."""
    b = SrtpBatchDev()
    b.arena = arena_ptr
    b.arena_size = arena_size
    b.pos, b.end, b.cap, b.err = pos_ptr, end_ptr, cap_ptr, err_ptr
    b.sess = sess_ptr
    b.n = n
    b.stream = stream
    sv = session_array(sessions)
    t = ctypes.c_void_p()
    rc = getattr(lib(), opname + "_batch_dev_async")(sv, len(sv),
                                                     ctypes.byref(b),
                                                     ctypes.byref(t))
    return rc, t, sv


def batch_wait(ticket):
    """srtp_batch_wait: the asynchronous call's result"""
    return lib().srtp_batch_wait(ticket)


def counter(name):
    """srtp_gpu_counter: "misses", "folds", "rejects" since load"""
    return int(lib().srtp_gpu_counter(name.encode()))


class tune:
    """srtp_gpu_tune as a context manager: with tune(general=1): ...
    (knobs restored to their defaults on exit)"""

    def __init__(self, **knobs):
        self.knobs = knobs

    def __enter__(self):
        for k, v in self.knobs.items():
            if v is not None:
                assert lib().srtp_gpu_tune(k.encode(), int(v)) == 0, k
        return self

    def __exit__(self, *exc):
        for k in self.knobs:
            lib().srtp_gpu_tune(k.encode(), 0)
        return False


def prof_enable(on=True):
    lib().srtp_gpu_prof(1 if on else 0)


def prof_read():
    """{slot: (ms, launches, jobs)} for kernel classes that ran.
    slot = protect*16 + gcm*8 + aes256*4 + shift"""
    return {k: v[:3] for k, v in prof_read_named().items()}


def prof_read_named():
    """{slot: (ms, launches, jobs, kernel name)} (srtp_gpu_prof_read_named)"""
    ms = (ctypes.c_double * 32)()
    la = (ctypes.c_uint64 * 32)()
    jb = (ctypes.c_uint64 * 32)()
    nm = ((ctypes.c_char * 48) * 32)()
    lib().srtp_gpu_prof_read_named(ms, la, jb, nm)
    return {k: (ms[k], la[k], jb[k], nm[k].value.decode())
            for k in range(32) if la[k]}


__all__ = ["errno"]
