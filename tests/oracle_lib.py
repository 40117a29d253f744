"""ctypes binding of the C restatement oracle (oracle/srtp_oracle.c).

Test infrastructure only -- the product never imports this module.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


class OMbuf(ctypes.Structure):
    _fields_ = [("buf", ctypes.POINTER(ctypes.c_uint8)),
                ("size", ctypes.c_size_t),
                ("pos", ctypes.c_size_t),
                ("end", ctypes.c_size_t)]


def _load():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    lib.oracle_srtp_alloc.argtypes = [ctypes.POINTER(vp), ctypes.c_int,
                                      ctypes.c_char_p, ctypes.c_size_t,
                                      ctypes.c_int]
    lib.oracle_srtp_free.argtypes = [vp]
    for n in ("encrypt", "decrypt"):
        for p in ("srtp", "srtcp"):
            f = getattr(lib, "oracle_%s_%s" % (p, n))
            f.argtypes = [vp, ctypes.POINTER(OMbuf)]
    lib.oracle_buf_alloc.restype = ctypes.POINTER(ctypes.c_uint8)
    lib.oracle_buf_alloc.argtypes = [ctypes.c_size_t]
    lib.oracle_buf_free.argtypes = [ctypes.POINTER(ctypes.c_uint8)]
    lib.oracle_srtp_suite_name.restype = ctypes.c_char_p
    lib.oracle_aes_ctr.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                   ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_aes_gcm_encrypt.argtypes = [
        ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p,
        ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
        ctypes.c_char_p]
    lib.oracle_sha1.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                ctypes.c_char_p]
    lib.oracle_hmac_sha1.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                     ctypes.c_char_p, ctypes.c_size_t,
                                     ctypes.c_char_p]
    lib.oracle_srtp_derive.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.c_uint8, ctypes.c_char_p,
                                       ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.c_size_t]
    lib.oracle_bench_pairs.restype = ctypes.c_long
    lib.oracle_bench_pairs.argtypes = [ctypes.c_int, ctypes.c_size_t,
                                       ctypes.c_long]
    u32p = ctypes.POINTER(ctypes.c_uint32)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    lib.oracle_stream_state.argtypes = [vp, ctypes.c_uint32, u32p, u32p,
                                        u64p, u64p]
    lib.oracle_stream_set.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint64, ctypes.c_uint64]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


class OracleBackend:
    """re_srtp.h-shaped backend over the C restatement."""

    def __init__(self):
        self.l = lib()

    def alloc(self, suite, key, flags):
        p = ctypes.c_void_p()
        err = self.l.oracle_srtp_alloc(ctypes.byref(p), suite, key, len(key),
                                       flags)
        return p, err

    def free(self, ctx):
        self.l.oracle_srtp_free(ctx)

    def export(self, ctx, ssrc):
        """(roc, s_l, replay lix, replay bitmap) of ssrc, zeros if none"""
        r, s = ctypes.c_uint32(), ctypes.c_uint32()
        x, b = ctypes.c_uint64(), ctypes.c_uint64()
        if self.l.oracle_stream_state(ctx, ssrc, ctypes.byref(r),
                                      ctypes.byref(s), ctypes.byref(x),
                                      ctypes.byref(b)):
            return (0, 0, 0, 0)
        return (r.value, s.value, x.value, b.value)

    def call(self, ctx, opname, size, pos, end, inb, nout):
        mb = OMbuf()
        mb.buf = self.l.oracle_buf_alloc(size)
        ctypes.memmove(mb.buf, inb, len(inb))
        mb.size, mb.pos, mb.end = size, pos, end
        err = getattr(self.l, "oracle_" + opname)(ctx, ctypes.byref(mb))
        n = max(nout, mb.end)
        buf = ctypes.string_at(mb.buf, min(n, mb.size))
        res = (err, mb.pos, mb.end, mb.size, buf)
        self.l.oracle_buf_free(mb.buf)
        return res


def aes_ctr(key, iv, data):
    out = ctypes.create_string_buffer(len(data))
    lib().oracle_aes_ctr(key, len(key) * 8, iv, out, data, len(data))
    return out.raw


def aes_gcm(key, iv, aad, pt):
    out = ctypes.create_string_buffer(max(1, len(pt)))
    tag = ctypes.create_string_buffer(16)
    lib().oracle_aes_gcm_encrypt(key, len(key) * 8, iv, aad, len(aad), pt,
                                 out, len(pt), tag)
    return out.raw[:len(pt)], tag.raw


def sha1(data):
    out = ctypes.create_string_buffer(20)
    lib().oracle_sha1(data, len(data), out)
    return out.raw


def hmac_sha1(key, data):
    out = ctypes.create_string_buffer(20)
    lib().oracle_hmac_sha1(key, len(key), data, len(data), out)
    return out.raw


def derive(key, salt, label, n):
    out = ctypes.create_string_buffer(32)
    err = lib().oracle_srtp_derive(out, n, label, key, len(key), salt,
                                   len(salt))
    assert err == 0
    return out.raw[:n]
