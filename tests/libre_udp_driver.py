"""Driver for tests/test_gpu_libre.py (run in a fresh process: libre keeps
process-global state).  libre's own event loop and UDP socket layer --
src/main, src/udp, src/net, src/sa, src/tmr compiled from the reference
sources WITHOUT src/srtp (oracle/_ref/libre_net.so, oracle/Makefile) --
hosts the LIBRE=1 product library (re_amd/lib/libre_srtp_amd_libre.so,
which takes mem_* / mbuf_* / udp_* / tmr_* from it, as it would when linked
into libre) with its SRTP helper registered on a udp_sock
(srtp_udp_helper_alloc, include/re_srtp_libre.h).

  send:    1024 config-1 packets through udp_send() (the helper protects
           them on the GPU in batches, udp_send_helper() -> sendto());
  receive: the protected datagrams from a plain socket through udp_read()
           -> the helper (GPU unprotect in batches, udp_recv_helper()) ->
           the socket's receive handler;
  errors:  a forged and a replayed datagram among them are dropped;
  rtcp-mux: RTP and RTCP datagrams interleaved on one socket (fresh
           contexts, a second helper): RTCP takes the SRTCP transform both
           ways, in datagram order.

Prints one JSON line with what the handler and the plain socket saw.
"""
import ctypes
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from re_amd import workload as W  # noqa: E402

c_p = ctypes.c_void_p


class Mbuf(ctypes.Structure):
    """struct mbuf (include/re_mbuf.h:43-48)"""
    _fields_ = [("buf", ctypes.POINTER(ctypes.c_uint8)),
                ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t),
                ("end", ctypes.c_size_t)]


class StreamState(ctypes.Structure):
    _fields_ = [("replay_rtp_bitmap", ctypes.c_uint64),
                ("replay_rtp_lix", ctypes.c_uint64),
                ("replay_rtcp_bitmap", ctypes.c_uint64),
                ("replay_rtcp_lix", ctypes.c_uint64),
                ("ssrc", ctypes.c_uint32), ("roc", ctypes.c_uint32),
                ("s_l", ctypes.c_uint16), ("s_l_set", ctypes.c_uint8),
                ("pad", ctypes.c_uint8), ("rtcp_index", ctypes.c_uint32)]


RECV_H = ctypes.CFUNCTYPE(None, c_p, ctypes.POINTER(Mbuf), c_p)
TMR_H = ctypes.CFUNCTYPE(None, c_p)


def main():
    net = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libre_net.so"),
                      ctypes.RTLD_GLOBAL)
    lib = ctypes.CDLL(os.path.join(ROOT, "re_amd", "lib",
                                   "libre_srtp_amd_libre.so"))
    net.mbuf_alloc.restype = ctypes.POINTER(Mbuf)
    net.mbuf_alloc.argtypes = [ctypes.c_size_t]
    net.mbuf_write_mem.argtypes = [ctypes.POINTER(Mbuf), ctypes.c_char_p,
                                   ctypes.c_size_t]
    net.mem_deref.argtypes = [c_p]
    net.mem_deref.restype = c_p
    net.udp_send.argtypes = [c_p, c_p, ctypes.POINTER(Mbuf)]
    net.udp_listen.argtypes = [ctypes.POINTER(c_p), c_p, RECV_H, c_p]
    net.sa_set_str.argtypes = [c_p, ctypes.c_char_p, ctypes.c_uint16]
    net.sa_port.restype = ctypes.c_uint16
    net.sa_port.argtypes = [c_p]
    net.udp_local_get.argtypes = [c_p, c_p]
    net.re_main.argtypes = [c_p]
    net.tmr_init.argtypes = [c_p]
    net.tmr_start_dbg.argtypes = [c_p, ctypes.c_uint64, TMR_H, c_p,
                                  ctypes.c_char_p, ctypes.c_int]
    net.tmr_cancel.argtypes = [c_p]
    lib.srtp_alloc.argtypes = [ctypes.POINTER(c_p), ctypes.c_int,
                               ctypes.c_char_p, ctypes.c_size_t,
                               ctypes.c_int]
    lib.srtp_udp_helper_alloc.argtypes = [
        ctypes.POINTER(c_p), c_p, ctypes.c_int, c_p, c_p, ctypes.c_size_t,
        ctypes.c_size_t, ctypes.c_uint]
    u64 = ctypes.POINTER(ctypes.c_uint64)
    lib.srtp_udp_helper_stats.argtypes = [c_p, u64, u64, u64, u64]
    lib.srtp_stream_export.argtypes = [c_p, ctypes.c_uint32,
                                       ctypes.POINTER(StreamState)]
    lib.srtp_gpu_error.restype = ctypes.c_char_p

    assert net.libre_init() == 0
    out = {}
    got = []

    @RECV_H
    def rh(src, mb, arg):
        m = mb.contents
        got.append((m.pos, m.end, ctypes.string_at(
            ctypes.addressof(m.buf.contents) + m.pos, m.end - m.pos)))
        if len(got) >= want[0]:
            net.re_cancel()

    @TMR_H
    def stop(arg):
        net.re_cancel()

    tmr = ctypes.create_string_buffer(256)
    net.tmr_init(tmr)

    def run(ms):
        net.tmr_start_dbg(tmr, ms, stop, None, b"driver", 0)
        net.re_main(None)
        net.tmr_cancel(tmr)

    sa = ctypes.create_string_buffer(128)
    assert net.sa_set_str(sa, b"127.0.0.1", 0) == 0
    us = c_p()
    assert net.udp_listen(ctypes.byref(us), sa, rh, None) == 0
    local = ctypes.create_string_buffer(128)
    assert net.udp_local_get(us, local) == 0
    port = net.sa_port(local)

    arena, pos, end, cap, _, keys = W.build_config(1)
    n = len(pos)
    key = keys[0].tobytes()
    tx, rx = c_p(), c_p()
    assert lib.srtp_alloc(ctypes.byref(tx), 1, key, 30, 0) == 0, \
        lib.srtp_gpu_error()
    assert lib.srtp_alloc(ctypes.byref(rx), 1, key, 30, 0) == 0
    h = c_p()
    assert lib.srtp_udp_helper_alloc(ctypes.byref(h), us, 0, rx, tx, 64,
                                     256, 1) == 0, lib.srtp_gpu_error()

    # ---- send: udp_send() -> helper (GPU protect) -> sendto ----
    peer = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    peer.bind(("127.0.0.1", 0))
    peer.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
    dst = ctypes.create_string_buffer(128)
    assert net.sa_set_str(dst, b"127.0.0.1", peer.getsockname()[1]) == 0
    want = [1 << 30]
    for i in range(n):
        mb = net.mbuf_alloc(256)
        pkt = arena[pos[i]:end[i]].tobytes()
        net.mbuf_write_mem(mb, pkt, len(pkt))
        mb.contents.pos = 0
        assert net.udp_send(us, dst, mb) == 0
        net.mem_deref(mb)
    run(50)                             # the timer flushes the rest
    peer.settimeout(2.0)
    wire = [peer.recv(2048) for _ in range(n)]
    st = StreamState()
    assert lib.srtp_stream_export(tx, W.SSRC_BASE, ctypes.byref(st)) == 0
    out["wire"] = [w.hex() for w in wire]
    out["tx_state"] = [st.roc, st.s_l, st.replay_rtp_lix,
                       st.replay_rtp_bitmap]

    # ---- receive: plain socket -> udp_read -> helper (GPU unprotect) ->
    # the socket's handler; a forged and a replayed datagram dropped ----
    send = list(wire)
    send.insert(700, wire[500])                     # replay
    q = bytearray(wire[900])
    q[-1] ^= 1
    send[901] = bytes(q)                            # forgery (shifted by 1)
    want[0] = len(send) - 2
    addr = ("127.0.0.1", port)
    for c0 in range(0, len(send), 128):
        for d in send[c0:c0 + 128]:
            peer.sendto(d, addr)
        run(2000)
    st = StreamState()
    assert lib.srtp_stream_export(rx, W.SSRC_BASE, ctypes.byref(st)) == 0
    out["rx_state"] = [st.roc, st.s_l, st.replay_rtp_lix,
                       st.replay_rtp_bitmap]
    out["got"] = [(p, e, b.hex()) for p, e, b in got]
    r, ok, t, dr = (ctypes.c_uint64() for _ in range(4))
    lib.srtp_udp_helper_stats(h, ctypes.byref(r), ctypes.byref(ok),
                              ctypes.byref(t), ctypes.byref(dr))
    out["stats"] = [r.value, ok.value, t.value, dr.value]
    net.mem_deref(h)

    # ---- rtcp-mux: every 10th datagram an RTCP receiver report ----
    mux = mux_packets(arena, pos, end)
    tx2, rx2, h2 = c_p(), c_p(), c_p()
    assert lib.srtp_alloc(ctypes.byref(tx2), 1, key, 30, 0) == 0
    assert lib.srtp_alloc(ctypes.byref(rx2), 1, key, 30, 0) == 0
    got.clear()
    want[0] = 1 << 30
    assert lib.srtp_udp_helper_alloc(ctypes.byref(h2), us, 0, rx2, tx2, 64,
                                     256, 1) == 0
    for pkt in mux:
        mb = net.mbuf_alloc(256)
        net.mbuf_write_mem(mb, pkt, len(pkt))
        mb.contents.pos = 0
        assert net.udp_send(us, dst, mb) == 0
        net.mem_deref(mb)
    run(50)
    wire2 = [peer.recv(2048) for _ in range(len(mux))]
    out["mux_wire"] = [w.hex() for w in wire2]
    want[0] = len(mux)
    for d in wire2:
        peer.sendto(d, addr)
    run(2000)
    out["mux_got"] = [(p, e, b.hex()) for p, e, b in got]
    net.mem_deref(h2)
    net.mem_deref(us)
    print(json.dumps(out))


def mux_packets(arena, pos, end, n=200):
    """n datagrams of one rtcp-mux socket: config-1 RTP packets with an
    RTCP receiver report (PT 201, SSRC 0x01020304, one report block) as
    every 10th (tests/test_gpu_libre.py rebuilds the same list)"""
    out = []
    k = 0
    for i in range(n):
        if i % 10 == 9:
            rr = bytes([0x81, 201, 0, 7]) + (0x01020304).to_bytes(4, "big") \
                + bytes((i * 7 + j) & 0xff for j in range(24))
            out.append(rr)
        else:
            out.append(arena[pos[k]:end[k]].tobytes())
            k += 1
    return out


if __name__ == "__main__":
    main()
