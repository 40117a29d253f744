"""Golden-replay backend over the product C-ABI (re_amd/lib), per-call
srtp_encrypt/decrypt exactly like the reference tests call libre."""
import ctypes

import re_amd.srtp as P


class ProductBackend:
    def alloc(self, suite, key, flags):
        s = P.Srtp(suite, key, flags)
        return s, s.err

    def free(self, ctx):
        ctx.close()

    def call(self, ctx, opname, size, pos, end, inb, nout):
        mb = P.new_mbuf(inb, size, pos)
        assert mb.contents.end == end
        err = getattr(P.lib(), opname)(ctx.ptr, mb)
        m = mb.contents
        n = max(nout, m.end)
        buf = ctypes.string_at(m.buf, min(n, m.size))
        res = (err, m.pos, m.end, m.size, buf)
        P.free_mbuf(mb)
        return res
