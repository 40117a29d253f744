#!/usr/bin/env python3
"""bench.py -- SRTP protect+unprotect throughput on MI355X (BASELINE.json).

A "step" = one srtp_encrypt_batch + one srtp_decrypt_batch over the whole
device-resident packet arena (config 2 by default: 1M x 1200-B RTP packets,
AES_CM_128_HMAC_SHA1_80, one session).  Every step uses a fresh tx/rx
session pair (a receiver must not see the same indices twice: replay
protection, src/srtp/replay.c:32-62), created outside the timed region.

value = RTP bytes per step over all ranks / step time, in GiB/s
        (N*L / (t_protect + t_unprotect)).
roofline: the dominant kernel's algorithmic bytes per launch (packets x
        (2L + T): read L, write L + T, or read L + T, write L) over its
        average launch time, timed with HIP events on the launch stream.

Multi-GPU (config 5): one process per GPU, rank r protects/unprotects its
contiguous 1M-packet shard of one 8M-packet stream, continuing the
stream state exactly where rank r-1's shard ends (srtp_stream_import).
Packets are independent once their index is known, so there is no data
collective; RCCL all-reduces the per-rank counters and the max time.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
METRIC = ("GiB/s + Mpkt/s SRTP protect+unprotect, 1200B RTP pkts, "
          "device-resident")

CONFIGS = {
    2: dict(suite=1, n=1 << 20, length=1200, nsess=1,
            name="AES_CM_128_HMAC_SHA1_80 1Mx1200B 1 session"),
    3: dict(suite=5, n=1 << 20, length=1200, nsess=1,
            name="AEAD_AES_256_GCM 1Mx1200B 1 session"),
    4: dict(suite=1, n=1 << 20, length=None, nsess=1 << 16,
            name="AES_CM_128_HMAC_SHA1_80 64K sessions mixed 200/1400B"),
    5: dict(suite=1, n=1 << 20, length=1200, nsess=1,
            name="AES_CM_128_HMAC_SHA1_80 8Mx1200B sharded (1M/GPU)"),
}


def cpu_info():
    """(nproc, usable cores, CPU model) of this host"""
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = nproc
    return nproc, usable, model


def cpu_quota():
    """(cores, source) this process may use: the cgroup CPU quota (v2
    cpu.max, v1 cpu.cfs_quota_us / cfs_period_us), else the OMP_NUM_THREADS
    share the box sets for a job, else the affinity mask"""
    _, usable, _ = cpu_info()
    for path, parse in (
            ("/sys/fs/cgroup/cpu.max",
             lambda t: (t.split()[0], t.split()[1])),
            ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
        except OSError:
            continue
        if parse:
            q, p = parse(txt)
        else:
            q = txt
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    p = f.read().strip()
            except OSError:
                continue
        if q not in ("max", "-1"):
            cores = max(1, int(int(q) / int(p)))
            return min(usable, cores), "%s=%s/%s" % (path, q, p)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        return min(usable, int(omp)), "OMP_NUM_THREADS=%s (no cgroup " \
            "quota visible)" % omp
    return usable, "sched_getaffinity"


def cpu_baseline(cfg, rtcp=False):
    """Reference src/srtp (oracle/_ref/ref_bench: the reference sources
    compiled with the box's libcrypto) on the host cores, bounded sample,
    on 1 core and on every core this job may use (cpu_quota(): the cgroup
    quota, or the box's per-job share), one struct srtp pair per thread;
    falls back to the portable restatement (kind "port").  A run with
    errors fails loudly."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    nproc, usable, model = cpu_info()
    threads, limit = cpu_quota()
    length = cfg["length"] or 0          # 0 = mixed 200/1400 in ref_bench
    if os.path.exists(ref) and not rtcp:
        runs = {}
        for t in sorted({1, threads}):
            # ~1-4 s of CPU per run: CTR/HMAC ~0.2 Mpairs/s/core, GCM ~1
            per = (60000 if cfg["suite"] < 4 else 150000) // (1 if t > 1
                                                               else 2)
            out = subprocess.run(
                [ref, str(cfg["suite"]), str(length), str(per), str(t),
                 str(cfg["nsess"])], capture_output=True, text=True,
                timeout=600, check=True).stdout
            r = json.loads(out.strip().splitlines()[-1])
            if r["errors"]:
                raise RuntimeError("ref_bench: %d errors (%s)" %
                                   (r["errors"], out.strip()))
            runs[t] = r
        r, r1 = runs[threads], runs[1]
        procs = None
        if threads > 1:
            # the same work as one single-threaded process per core: the
            # threaded run contends on OpenSSL 3.0's shared HMAC state
            # (SURVEY §6), separate processes do not -- the reference's
            # best all-core figure on this host
            per = 60000 if cfg["suite"] < 4 else 150000
            ps = [subprocess.Popen(
                [ref, str(cfg["suite"]), str(length), str(per), "1",
                 str(cfg["nsess"])], stdout=subprocess.PIPE, text=True)
                for _ in range(threads)]
            rs = []
            for q in ps:
                out, _ = q.communicate(timeout=600)
                if q.returncode:
                    raise RuntimeError("ref_bench process: rc %d" %
                                       q.returncode)
                rs.append(json.loads(out.strip().splitlines()[-1]))
            if any(x["errors"] for x in rs):
                raise RuntimeError("ref_bench processes: errors")
            sec = max(x["seconds"] for x in rs)
            pairs = sum(x["pairs"] for x in rs)
            gib = sum(x["gib_s"] * x["seconds"] for x in rs) / sec
            procs = {"gib_s": gib, "mpairs_s": pairs / sec / 1e6,
                     "pairs": pairs, "seconds": sec}
        best = procs if procs and procs["gib_s"] > r["gib_s"] else None
        return {"value": round((best or r)["gib_s"], 4), "unit": "GiB/s",
                "mpkt_s": round((best or r)["mpairs_s"], 4),
                "cores": threads,
                "value_threads": round(r["gib_s"], 4),
                "value_processes": (round(procs["gib_s"], 4) if procs
                                    else None),
                "value_1core": round(r1["gib_s"], 4),
                "mpkt_s_1core": round(r1["mpairs_s"], 4),
                "kind": "reference", "nproc": nproc, "usable_cores": usable,
                "cores_limit": limit,
                "cpu_model": model, "openssl": r.get("openssl"),
                "sample": "%d protect+unprotect pairs of %s-B RTP packets "
                          "on %d threads of one process, and %s pairs on %d "
                          "single-threaded processes (value: the faster of "
                          "the two), %d pairs on 1 core; %d session(s) per "
                          "thread, reference src/srtp" % (
                              r["pairs"], length or "200/1400", threads,
                              procs["pairs"] if procs else 0,
                              threads if procs else 0, r1["pairs"],
                              cfg["nsess"]),
                "seconds": round(r["seconds"] + r1["seconds"] +
                                 (procs["seconds"] if procs else 0), 3)}
    from tests import oracle_lib as O
    n = 3000
    t0 = time.perf_counter()
    ok = O.lib().oracle_bench_pairs(cfg["suite"], cfg["length"] or 800, n)
    dt = time.perf_counter() - t0
    L = cfg["length"] or 800
    return {"value": round(ok * L / dt / 2**30, 5), "unit": "GiB/s",
            "mpkt_s": round(ok / dt / 1e6, 5), "cores": 1, "kind": "port",
            "nproc": nproc, "cpu_model": model,
            "sample": "%d pairs through the portable C restatement" % n}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nranks):
    """`bench.py --gpus N` with no launcher: start the N ranks ourselves,
    one child process per GPU, each with RANK/LOCAL_RANK/WORLD_SIZE/
    MASTER_ADDR/MASTER_PORT set exactly as torch.distributed.run would.
    The parent never touches the GPU (no torch import here): every child
    initialises HIP itself.  Children inherit stdout, so rank 0's JSON line
    is this command's output.  If any rank fails the others are stopped and
    the parent exits non-zero."""
    env0 = dict(os.environ)
    env0.setdefault("MASTER_ADDR", "127.0.0.1")
    env0.setdefault("MASTER_PORT", str(_free_port()))
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(nranks):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(nranks), LOCAL_WORLD_SIZE=str(nranks),
                   GROUP_RANK="0", ROLE_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 1
                print("bench.py: rank %d exited with %d; stopping the "
                      "others" % (procs.index(p), r), file=sys.stderr,
                      flush=True)
                for q in live:
                    q.terminate()
                stop_at = time.monotonic() + 30
        if live:
            if rc and time.monotonic() > stop_at:
                for q in live:
                    q.kill()
            time.sleep(0.05)
    return rc


SHARD_GOLDEN = os.path.join(ROOT, "tests", "golden", "config5_shards.json")


def shard_golden():
    """the reference's config-5 shards (a committed fixture), or None"""
    if not os.path.exists(SHARD_GOLDEN):
        return None
    with open(SHARD_GOLDEN) as f:
        return json.load(f)


def shard_check(args, cfg_id, rank, n, K, use_dev, plain, make_sessions,
                arena, pos_d, end_d, cap_d, OPS, sptr, log):
    """config 5: True / False (this rank's shard equal to the reference's
    or not), None when the golden file does not cover this run (another
    config or shard size, SRTCP, several SSRCs, host windows)"""
    import hashlib
    import torch
    import re_amd.srtp as P
    from re_amd import workload as W
    ref = shard_golden() if cfg_id == 5 else None
    if (ref is None or not use_dev or args.rtcp or K != 1 or
            n != ref["per"] or rank >= ref["world"]):
        return None
    sh = ref["shards"][rank]
    assert sh["rank"] == rank

    def sha(t):
        return hashlib.sha256(memoryview(np.ascontiguousarray(
            t.cpu().numpy())).cast("B")).hexdigest()

    tx, rx = make_sessions()
    arena.copy_(plain)
    pw, ew = pos_d.clone(), end_d.clone()
    er = torch.full((n,), -1, dtype=torch.int32, device=arena.device)
    ok = sha(arena) == sh["plain"]
    bad = [] if ok else ["plain"]
    for op, ctxs, direction in ((OPS[0], tx, "protect"),
                                (OPS[1], rx, "unprotect")):
        rc = P.device_batch_dev(op, ctxs, arena.data_ptr(), arena.numel(),
                                pw.data_ptr(), ew.data_ptr(),
                                cap_d.data_ptr(), er.data_ptr(), n, None,
                                sptr)
        torch.cuda.synchronize()
        want = sh[direction]
        if rc:
            bad.append((direction, "rc", rc))
            continue
        for name, t in (("arena", arena), ("end", ew), ("err", er)):
            if sha(t) != want[name]:
                bad.append((direction, name))
        e, st = ctxs[0].export(W.SSRC_BASE)
        got = (st.roc, st.s_l, st.s_l_set, st.replay_rtp_lix,
               st.replay_rtp_bitmap) if not e else None
        w = want["state"]
        if got != (w["roc"], w["s_l"], w["s_l_set"], w["lix"], w["bitmap"]):
            bad.append((direction, "state", got, w))
    for s in tx + rx:
        s.close()
    log("shard %d vs reference (%s): %s" % (rank, SHARD_GOLDEN,
                                            "equal" if not bad else bad))
    return not bad


def dry_run(args, world, rank):
    """--dry-run (CPU, testing the launcher): the rank plumbing of the
    sharded run without a GPU -- gloo rendezvous, this rank's shard of the
    config-5 stream (first seq and imported state, re_amd/shard.py) and
    the counter / max-time reduction.  Prints a line that says so; it
    measures nothing."""
    import torch
    import torch.distributed as dist
    from re_amd import shard as S
    from re_amd import workload as W
    if world > 1:
        dist.init_process_group("gloo")
    n = args.packets or 4096
    s0 = S.shard_seq0(rank, n, 65000)
    arena, pos, end, cap = W.make_arena(n, 1200, s0=s0)
    st = S.shard_state(rank, n, 65000, W.SSRC_BASE, True)
    seq = int.from_bytes(arena[pos[0] + 2:pos[0] + 4].tobytes(), "big")
    assert seq == s0, (seq, s0)
    # the boundary states rank r's contexts import at the real shard size,
    # against the reference's over the whole 8M-packet stream
    # (tests/golden/config5_shards.json tx_in / rx_in): no arena needed
    ref = shard_golden()
    st_ok = 0.0
    if ref is not None and rank < ref["world"]:
        sh = ref["shards"][rank]
        good = True
        for key, recv in (("tx_in", False), ("rx_in", True)):
            got = S.shard_state(rank, ref["per"], ref["s0"], W.SSRC_BASE,
                                recv)
            w = sh[key]
            if w is None:
                good &= rank == 0 and got["s_l_set"] == 0
            else:
                good &= (got["roc"], got["s_l"], got["s_l_set"],
                         got["replay_rtp_lix"], got["replay_rtp_bitmap"]) == \
                    (w["roc"], w["s_l"], w["s_l_set"], w["lix"], w["bitmap"])
        st_ok = 1.0 if good else 0.0
    counters = torch.tensor([n, float((end - pos).sum()), 0.0, st_ok],
                            dtype=torch.float64)
    tmax = torch.tensor([0.001 * (rank + 1)], dtype=torch.float64)
    S.reduce_results(dist if world > 1 else None, counters, tmax)
    seen = dist.get_world_size() if world > 1 else 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s",
                          "n_gpus": world, "dist_world": seen,
                          "dist_backend": "gloo" if world > 1 else None,
                          "dry_run": True,
                          "packets_total": int(counters[0].item()),
                          "bytes_total": int(counters[1].item()),
                          "tmax": float(tmax.item()),
                          "rank0_state": st,
                          # ranks whose boundary states equal the
                          # reference's (config5_shards.json)
                          "boundary_states_ok": int(counters[3].item())}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=None,
                    help="BASELINE.json config (2,3,4,5); default 2, or 5 "
                         "when --gpus > 1")
    ap.add_argument("--packets", type=int, default=None,
                    help="override packets per GPU (testing only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--e2e", action="store_true",
                    help="end-to-end: packets start and end in pinned host "
                         "memory (H2D + protect + D2H, H2D + unprotect + "
                         "D2H per step, chunk-pipelined); reported, not "
                         "the headline value")
    ap.add_argument("--e2e-chunks", type=int, default=8)
    ap.add_argument("--rtcp", action="store_true",
                    help="SRTCP: the same arena as RTCP packets through "
                         "srtcp_*_batch_dev (device-planned SRTCP)")
    ap.add_argument("--udp", action="store_true",
                    help="socket to socket: GPU protect + sendmmsg on one "
                         "loopback UDP socket, recvmmsg + GPU unprotect on "
                         "another (include/re_srtp_udp.h); reported in "
                         "DESIGN.md, not the headline value")
    ap.add_argument("--udp-seconds", type=float, default=3.0)
    ap.add_argument("--udp-batch", type=int, default=1024)
    ap.add_argument("--udp-pairs", type=int, default=4,
                    help="--udp: socket pairs, each with a sender and a "
                         "receiver thread")
    ap.add_argument("--udp-sync", action="store_true",
                    help="--udp: synchronous helpers (no pipelining)")
    ap.add_argument("--same-device", action="store_true",
                    help="testing only: all ranks on cuda:0, gloo counters")
    ap.add_argument("--sync", action="store_true",
                    help="synchronous srtp_*_batch_dev calls instead of the "
                         "asynchronous srtp_*_batch_dev_async + "
                         "srtp_batch_wait pair (protect and unprotect "
                         "queued back to back on the stream)")
    ap.add_argument("--async", dest="async_", action="store_true",
                    help="the asynchronous pair with two steps in flight "
                         "for every config (default: for multi-session "
                         "configs and sharded runs; one-session configs on "
                         "one GPU default to the synchronous calls, 1.5-2 "
                         "%% faster there: profiles/r04_sync_async_ab.txt)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="asynchronous pairs: wait for each step before "
                         "issuing the next (default: two steps in flight)")
    ap.add_argument("--host-arrays", action="store_true",
                    help="srtp_*_batch with host pos/end/err arrays instead "
                         "of the device-resident srtp_*_batch_dev")
    ap.add_argument("--tune", action="append", default=[],
                    help="name=value: srtp_gpu_tune knob (A/B runs)")
    ap.add_argument("--forge", type=float, default=0,
                    help="adversarial receive: forge this many packets per "
                         "batch (a fraction if < 1) between protect and "
                         "unprotect, spread evenly (EAUTH expected for "
                         "exactly those)")
    ap.add_argument("--ssrcs", type=int, default=1,
                    help="one session, packets interleaved over this many "
                         "SSRCs (packet i -> stream i mod K, per-stream seq "
                         "from 65000): the per-stream device planner")
    ap.add_argument("--fresh-streams", action="store_true",
                    help="--ssrcs: the session's streams are created by the "
                         "timed batch (default: announced before it, like "
                         "SDP a=ssrc, by srtp_stream_import of a fresh "
                         "stream state)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (traffic, integer roofline) to "
                         "attach; default profiles/r06_pmc.json")
    ap.add_argument("--room", type=int, default=None,
                    help="A/B: bytes of slack per packet slot (default 16: "
                         "1216-B slots for 1200-B packets; 80: 1280-B, "
                         "128-B aligned slots)")
    ap.add_argument("--libre-helper", action="store_true",
                    help="one libre re_main thread receiving config-2 SRTP "
                         "over loopback (oracle/libre_helper_bench.c): no "
                         "helper / the reference srtp_decrypt per datagram "
                         "/ the batched GPU helper at several batch sizes; "
                         "delivered rate, added latency, loop CPU per "
                         "packet; reported in DESIGN.md, not the headline")
    ap.add_argument("--percall", action="store_true",
                    help="the unchanged per-packet API: srtp_encrypt + "
                         "srtp_decrypt of one 1200-B mbuf per call "
                         "(re_amd/bench/percall.c), latency percentiles "
                         "and rates, beside the reference on 1 core")
    ap.add_argument("--percall-calls", type=int, default=20000)
    ap.add_argument("--percall-suite", type=int, default=1,
                    help="--percall: enum srtp_suite (1 AES_CM_128_HMAC_"
                         "SHA1_80, 4 AES_128_GCM, 5 AES_256_GCM)")
    ap.add_argument("--rtcp-report", action="store_true",
                    help="the RTCP report path on the device (SURVEY 8(f)4): "
                         "1M SR + report block + SDES CNAME compounds "
                         "encoded (rtcp_encode_batch_dev), SRTCP-protected, "
                         "-unprotected and decoded with their contents "
                         "(rtcp_decode_full_batch_dev), per stage and end "
                         "to end")
    ap.add_argument("--dry-run", action="store_true",
                    help="testing only (CPU): rank plumbing, no GPU work")
    args = ap.parse_args()

    # ranks: under torch.distributed.run WORLD_SIZE is set and must equal
    # --gpus; without a launcher, --gpus N > 1 starts the N ranks itself
    # (before anything here touches the GPU)
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return spawn_ranks(args.gpus)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" %
              (os.environ["WORLD_SIZE"], args.gpus), file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args, int(os.environ.get("WORLD_SIZE", "1")),
                       int(os.environ.get("RANK", "0")))
    if args.percall:
        return percall_bench(args)
    if args.libre_helper:
        return libre_helper_bench(args)
    if args.rtcp_report:
        return rtcp_report_bench(args)

    import torch
    import torch.distributed as dist
    import re_amd.srtp as P
    from re_amd import shard as S
    from re_amd import workload as W

    if args.udp:
        return udp_bench(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg_id = args.config or (5 if args.gpus > 1 else 2)
    cfg = dict(CONFIGS[cfg_id])
    if args.packets:
        cfg["n"] = args.packets
    # --same-device (testing only): every rank on cuda:0, counters over
    # gloo -- rehearses the sharded path on a one-GPU box
    gpu = 0 if args.same_device else local
    torch.cuda.set_device(gpu)
    if world > 1:
        if args.same_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl",
                                    device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu)
    P.load()
    for kv in args.tune:
        k, v = kv.split("=")
        assert P.lib().srtp_gpu_tune(k.encode(), int(v)) == 0, kv
    tstart = time.perf_counter()

    def log(msg):
        # phase progress on stderr (the JSON line stays alone on stdout)
        print("[bench rank %d/%d %.1fs] %s" % (rank, world,
                                              time.perf_counter() - tstart,
                                              msg),
              file=sys.stderr, flush=True)

    n, suite, nsess = cfg["n"], cfg["suite"], cfg["nsess"]
    s0 = 65000
    if cfg_id == 5:
        s0 = S.shard_seq0(rank, n, 65000)   # this shard's first seq
    lengths = cfg["length"] if cfg["length"] else W.mixed_lengths(n)
    sess = W.random_sessions(n, nsess) if nsess > 1 else None
    gidx = gsess = None
    key_ids = None
    if nsess > 1 and world > 1:
        # a multi-session load shards by session id -- one
        # workload of world x n packets over world x nsess sessions, each
        # rank the packets of the sessions it owns (re_amd/shard.py), so
        # every stream's state stays on its rank (weak scaling: ~n each)
        g_sess = W.random_sessions(n * world, nsess * world)
        gidx, sess = S.shard_sessions(g_sess, world, rank)
        gsess = g_sess[gidx]
        lengths = W.mixed_lengths(n * world)[gidx]
        n = len(gidx)
        key_ids = np.arange(nsess, dtype=np.uint64) * world + rank
        cfg["name"] += ", sessions hashed over %d ranks" % world
    K = max(1, args.ssrcs)
    if K > 1:
        assert nsess == 1 and cfg_id in (2, 3) and not args.rtcp, \
            "--ssrcs: configs 2 and 3"
        cfg["name"] += " x %d SSRCs" % K
    if args.rtcp:
        assert nsess == 1 and cfg["length"], "--rtcp: configs 2 and 3"
        arena_h, pos, end, cap = W.make_rtcp_arena(n, lengths)
    else:
        # config 5: rank r holds packets r*n .. (r+1)*n-1 of the one 8M
        # stream (payload generators and timestamps continue it), exactly
        # the shard the reference digests pin (config5_shards.json)
        arena_h, pos, end, cap = W.make_arena(
            n, lengths, s0=s0 & 0xffff,
            sess=(gsess if gsess is not None else sess) if K == 1 else
            np.arange(n, dtype=np.uint32) % K, idx=gidx,
            first=rank * n if cfg_id == 5 else 0,
            room=args.room or 16)
    OPS = ("srtcp_encrypt", "srtcp_decrypt") if args.rtcp else \
        ("srtp_encrypt", "srtp_decrypt")
    log("workload built (%d packets)" % n)
    arena = torch.from_numpy(arena_h).to(dev)
    plain = arena.clone() if not args.no_verify else None
    klen = P.key_len(suite) + P.salt_len(suite)
    keys = W.make_keys(nsess, klen, ids=key_ids)
    # one explicit stream for the whole run (torch copies and the library
    # calls), so ordering is explicit rather than via the null stream
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = ctypes_stream(stream)
    L = cfg["length"] or 800
    tag = P.tag_len(suite) + (4 if args.rtcp else 0)   # + E||index
    rtp_bytes = int(np.asarray(end - pos, dtype=np.int64).sum())

    def make_sessions():
        e1, tx = P.alloc_many(nsess, suite, keys.tobytes())
        e2, rx = P.alloc_many(nsess, suite, keys.tobytes())
        assert not e1 and not e2, (e1, e2, P.lib().srtp_gpu_error())
        if cfg_id == 5 and rank > 0:
            assert tx[0].import_(S.shard_state(
                rank, n, 65000, W.SSRC_BASE, False, P.StreamState)) == 0
            assert rx[0].import_(S.shard_state(
                rank, n, 65000, W.SSRC_BASE, True, P.StreamState)) == 0
        if K > 1 and not args.fresh_streams:
            for s in tx + rx:
                for k in range(K):
                    st = P.StreamState()
                    st.ssrc = W.SSRC_BASE + k
                    assert s.import_(st) == 0
        return tx, rx

    # per-call descriptor arrays (the API updates pos/end in place).
    # Default: srtp_*_batch_dev -- windows and results resident in HBM like
    # the packets; --host-arrays: srtp_*_batch with host windows.
    use_dev = not args.host_arrays
    # asynchronous pair (srtp_*_batch_dev_async) for the RTP device path
    # one session: the synchronous pair measured faster (the crypto
    # kernel itself: config 3 unprotect 1.570 vs 1.617 ms); many sessions:
    # the pipelined asynchronous pair (its host planning overlaps the
    # previous step on the GPU: config 4 292-295 vs 217-269 GiB/s)
    # (sharded runs keep the pipelined pair: on the shared-GPU rehearsal the
    # synchronous one lost 9 %)
    sync = args.sync or (nsess == 1 and world == 1 and not args.async_)
    use_async = use_dev and not sync and not args.e2e and not args.rtcp
    pipelined = use_async and not args.no_pipeline
    sess_d = None
    if use_dev:
        i32 = lambda a: torch.from_numpy(
            np.asarray(a, dtype=np.uint32).view(np.int32)).to(dev)
        pos_d, end_d, cap_d = i32(pos), i32(end), i32(cap)
        if sess is not None:
            sess_d = i32(sess)
        p_d, e_d = torch.empty_like(pos_d), torch.empty_like(end_d)
        # every step its own input windows (the API moves pos/end in place;
        # an asynchronous call keeps its arrays until it is waited for,
        # re_srtp_batch.h), written before the timed region like the arena
        nwin = max(1, args.steps, args.warmup)
        winp = pos_d.repeat(nwin, 1)
        wine = end_d.repeat(nwin, 1)

        def reset_windows():
            winp.copy_(pos_d.expand(nwin, -1))
            wine.copy_(end_d.expand(nwin, -1))
        # per-step result arrays: the API fills them inside the timed
        # region; the bench tallies them after it (verification, not path)
        errbuf = torch.zeros((2, max(1, args.steps, args.warmup), n), dtype=torch.int32,
                             device=dev)
    else:
        p, e = np.empty_like(pos), np.empty_like(end)
        err_e = np.zeros(n, dtype=np.int32)
        err_d = np.zeros(n, dtype=np.int32)

    if args.e2e:
        assert use_dev, "--e2e uses the device-resident batch API"
        host = torch.from_numpy(arena_h).pin_memory()
        s_up = torch.cuda.Stream(dev)
        s_dn = torch.cuda.Stream(dev)
        K = max(1, args.e2e_chunks)
        per = (n + K - 1) // K
        slot = int(cap[0] - pos[0])
        cuts = [(a, min(n, a + per)) for a in range(0, n, per)]

        def e2e_pass(opname, ss, er):
            ev_up = []
            # host bytes of the previous pass must have landed
            s_up.wait_stream(s_dn)
            s_up.wait_stream(stream)
            with torch.cuda.stream(s_up):
                for a, b in cuts:
                    arena[a * slot:b * slot].copy_(
                        host[a * slot:b * slot], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(s_up)
                    ev_up.append(ev)
            for (a, b), ev in zip(cuts, ev_up):
                stream.wait_event(ev)
                rc = P.device_batch_dev(
                    opname, ss, arena.data_ptr(), arena.numel(),
                    p_d[a:].data_ptr(), e_d[a:].data_ptr(),
                    cap_d[a:].data_ptr(), er[a:].data_ptr(), b - a,
                    None, sptr)
                assert rc == 0, (rc, P.lib().srtp_gpu_error())
                done = torch.cuda.Event()
                done.record(stream)
                s_dn.wait_event(done)
                with torch.cuda.stream(s_dn):
                    host[a * slot:b * slot].copy_(
                        arena[a * slot:b * slot], non_blocking=True)
            stream.wait_stream(s_dn)

    nforge = int(args.forge * n) if 0 < args.forge < 1 else int(args.forge)
    forge_idx = forge_pk = None
    if nforge:
        assert use_dev and not args.e2e and not args.rtcp
        forge_pk = np.linspace(0, n - 1, nforge).astype(np.int64)
        # one payload byte of each forged packet (past any header)
        forge_idx = torch.from_numpy(pos[forge_pk].astype(np.int64) +
                                     12 + 20).to(dev)

    # synchronous device calls: each step's two calls prepared before the
    # timed region (their argument structs, the C entry points), so the
    # timed loop is the library's calls and not Python argument marshalling
    prepared = {}

    def prepare(sets, k0=0):
        prepared.clear()
        if not (use_dev and not use_async and not args.e2e and
                forge_idx is None):
            return
        for k, (tx, rx) in enumerate(sets):
            calls = []
            for d, (opname, ss) in enumerate(((OPS[0], tx), (OPS[1], rx))):
                b = P.SrtpBatchDev()
                b.arena, b.arena_size = arena.data_ptr(), arena.numel()
                b.pos, b.end = winp[k0 + k].data_ptr(), wine[k0 + k].data_ptr()
                b.cap, b.err = cap_d.data_ptr(), errbuf[d, k0 + k].data_ptr()
                b.sess = sess_d.data_ptr() if sess_d is not None else None
                b.n, b.stream = n, sptr
                sv = P.session_array(ss)
                calls.append((getattr(P.lib(), opname + "_batch_dev"), sv,
                              len(sv), ctypes.byref(b), b))
            prepared[(id(tx), k0 + k)] = calls

    def step(tx, rx, k=0, inflight=None):
        pc = prepared.get((id(tx), k))
        if pc is not None:
            for fn, sv, ns, bref, _ in pc:
                rc = fn(sv, ns, bref)
                assert rc == 0, (rc, P.lib().srtp_gpu_error())
            return 0
        if use_dev:
            err_ed, err_dd = errbuf[0, k], errbuf[1, k]
        if args.e2e:
            p_d.copy_(pos_d)
            e_d.copy_(end_d)
            e2e_pass(OPS[0], tx, err_ed)
            e2e_pass(OPS[1], rx, err_dd)
            return 0
        if use_dev:
            pw, ew = winp[k], wine[k]
            pend = []
            for opname, ss, er in ((OPS[0], tx, err_ed),
                                   (OPS[1], rx, err_dd)):
                if forge_idx is not None and opname == OPS[1]:
                    # the forgery flips one byte of protect's output on the
                    # call stream, between protect and unprotect.  An
                    # asynchronous call's arena is the library's until it is
                    # waited for because a call the device could not complete
                    # is re-run from it on the host (re_srtp_batch.h): the
                    # line is only valid if no call was (checked below)
                    with torch.cuda.stream(stream):
                        if use_async and not pipelined:
                            assert P.batch_wait(pend.pop()[0]) == 0
                        arena.index_put_((forge_idx,),
                                         arena[forge_idx] ^ 0x40)
                a = (opname, ss, arena.data_ptr(), arena.numel(),
                     pw.data_ptr(), ew.data_ptr(), cap_d.data_ptr(),
                     er.data_ptr(), n,
                     sess_d.data_ptr() if sess_d is not None else None, sptr)
                if use_async:
                    rc, t, keep = P.device_batch_dev_async(*a)
                    pend.append((t, keep))
                else:
                    rc = P.device_batch_dev(*a)
                assert rc == 0, (rc, P.lib().srtp_gpu_error())
            if inflight is not None:
                inflight.extend(pend)   # the caller waits, a step later
                return 0
            for t, _ in pend:
                rc = P.batch_wait(t)
                assert rc == 0, (rc, P.lib().srtp_gpu_error())
            return 0
        np.copyto(p, pos)
        np.copyto(e, end)
        rc, _ = P.device_batch(OPS[0], tx, arena.data_ptr(),
                               arena.numel(), p, e, cap, sess, sptr, err_e)
        assert rc == 0, (rc, P.lib().srtp_gpu_error())
        rc, _ = P.device_batch(OPS[1], rx, arena.data_ptr(),
                               arena.numel(), p, e, cap, sess, sptr, err_d)
        assert rc == 0, (rc, P.lib().srtp_gpu_error())
        return np.count_nonzero(err_e) + np.count_nonzero(err_d)

    def run_steps(sets, k0=0):
        """one step per session set; asynchronous pairs run two steps in
        flight: step k's calls are issued (their host planning overlaps
        step k-1 on the GPU, which shares the stream), then step k-1's are
        waited for"""
        errs = 0
        inflight = [] if pipelined else None
        for k, (tx, rx) in enumerate(sets):
            mark = len(inflight) if inflight is not None else 0
            errs += step(tx, rx, k0 + k, inflight)
            if inflight is not None:
                done, inflight[:] = inflight[:mark], inflight[mark:]
                for t, _ in done:
                    rc = P.batch_wait(t)
                    assert rc == 0, (rc, P.lib().srtp_gpu_error())
        for t, _ in inflight or []:
            rc = P.batch_wait(t)
            assert rc == 0, (rc, P.lib().srtp_gpu_error())
        return errs

    log("arena resident, warmup")
    # ---- warmup (untimed; as many steps in flight as the timed loop, so
    # the library's per-call workspaces exist before timing) ----
    if args.warmup:
        warm = [make_sessions() for _ in range(args.warmup)]
        if use_dev:
            reset_windows()
        run_steps([(P.session_array(tx), P.session_array(rx))
                   for tx, rx in warm])
        torch.cuda.synchronize()
        for tx, rx in warm:
            for s in tx + rx:
                s.close()
    torch.cuda.synchronize()
    # the C session pointer arrays are built once per set (not timed);
    # the Srtp handles stay alive until the end (they own the sessions)
    sess_objs = [make_sessions() for _ in range(args.steps)]
    log("warmup done, timed steps")
    sess_sets = [(P.session_array(tx), P.session_array(rx))
                 for tx, rx in sess_objs]
    # RE_SRTP_BENCH_NOPROF: no in-run kernel events (A/B of their cost)
    P.prof_enable(not os.environ.get("RE_SRTP_BENCH_NOPROF"))
    P.prof_read()
    if use_dev:
        errbuf.fill_(-1)        # every call must write every result
        reset_windows()
    prepare(sess_sets)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    c_rerun0 = (P.counter("rejects"), P.counter("folds"), P.counter("gated"))
    voided0 = P.counter("prof_voided")
    SPLIT = ("sync_calls", "sync_ns_issue", "sync_ns_wait", "sync_ns_finish")
    split0 = [P.counter(c) for c in SPLIT]
    t0 = time.perf_counter()
    errors = run_steps(sess_sets)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    split = [P.counter(c) - v for c, v in zip(SPLIT, split0)]
    if world > 1:
        dist.barrier()
    prof = P.prof_read_named()
    # launches behind a rejected device plan exit at once: the profiler
    # leaves them out of every slot (srtp_kernels.hip launch/prof_drain)
    voided = P.counter("prof_voided") - voided0
    P.prof_enable(False)
    elapsed = t1 - t0
    if forge_pk is not None and pipelined:
        # the forgery rode the stream between protect and unprotect: valid
        # only if no call was completed on the host (a host re-run reads
        # the arena as the stream left it)
        assert (P.counter("rejects"), P.counter("folds"),
                P.counter("gated")) == c_rerun0, \
            "a call was re-run on the host: forged-packet line invalid"
    if use_dev:
        if forge_pk is not None:
            # exactly the forged packets fail, with EAUTH
            fp = torch.from_numpy(forge_pk).to(dev)
            got = errbuf[1, :args.steps, fp]
            assert bool((got == P.EAUTH).all()), "forged packets not EAUTH"
            errbuf[1, :args.steps, fp] = 0
        errors += int(torch.count_nonzero(errbuf[:, :args.steps]).item())
    counters = torch.tensor([n * args.steps, rtp_bytes * args.steps, errors],
                            dtype=torch.float64, device=dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    log("timed steps done")
    if os.environ.get("BENCH_WATCHDOG"):
        import faulthandler
        faulthandler.dump_traceback_later(
            float(os.environ["BENCH_WATCHDOG"]), exit=False)
    S.reduce_results(dist if world > 1 else None, counters, tmax)
    tot_pkts, tot_bytes, tot_err = [float(x) for x in counters.tolist()]
    T = float(tmax.item())
    verified = None
    if plain is not None:
        # packet windows [pos, end) are restored by protect+unprotect; the
        # bytes past end keep the tag (and the ROC written over it,
        # srtp.c:342-344) exactly like the reference mbuf
        slot = int(cap[0] - pos[0])
        lens = torch.from_numpy((end - pos).astype(np.int64)).to(dev)
        win = torch.arange(slot, device=dev)[None, :] < lens[:, None]
        a2, p2 = arena.view(n, slot), plain.view(n, slot)
        # elementwise compare + count: no boolean-mask gather (its
        # index tensor is ~10 GB at 1M packets and slow to build)
        if forge_pk is not None:
            # a forged packet keeps its ciphertext (srtp.c:358-359)
            win[torch.from_numpy(forge_pk).to(dev)] = False
        bad = int(torch.count_nonzero((a2 != p2) & win).item())
        verified = bad == 0 and tot_err == 0
        del win, a2, p2

    log("verified")
    for tx, rx in sess_objs:
        for s in tx + rx:
            s.close()
    # config 5: this rank's shard against the reference over the whole
    # 8M-packet stream (tests/golden/config5_shards.json, one reference
    # sender and receiver over all shards in order -- ref_digest.c shards):
    # fresh contexts importing the closed-form boundary state, one protect
    # and one unprotect of the plain shard, then the arena, end and errno
    # digests and the exported final state of each direction
    shard_chk = shard_check(args, cfg_id, rank, n, K, use_dev, plain,
                            make_sessions, arena, pos_d, end_d, cap_d, OPS,
                            sptr, log) if plain is not None else None
    del plain
    # ranks checked / ranks equal to the reference, summed over ranks
    chk = torch.tensor([0.0 if shard_chk is None else 1.0,
                        1.0 if shard_chk is True else 0.0],
                       dtype=torch.float64, device=dev)
    S.reduce_results(dist if world > 1 else None, chk,
                     torch.zeros(1, dtype=torch.float64, device=dev))
    shards_checked, shards_ok = [int(x) for x in chk.tolist()]

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel ----
    kern = []
    for slot, (ms, launches, jobs, kname) in prof.items():
        prot = slot >= 16
        pkt = jobs / launches
        nbytes = pkt * (2 * L + tag)
        avg_ms = ms / launches
        kern.append({"slot": slot, "kernel": kname,
                     "dir": "protect" if prot else "unprotect",
                     "avg_ms": avg_ms, "launches": launches,
                     "pkts_per_launch": pkt, "bytes_per_launch": nbytes,
                     "gbs": nbytes / (avg_ms * 1e-3) / 1e9})
    kern.sort(key=lambda d: -d["avg_ms"] * d["launches"])
    dom = kern[0] if kern else None
    if dom:
        # a roofline no launch could reach means the profiler counted work
        # that did not run: fail loudly rather than print it
        per_step = dom["avg_ms"] * dom["launches"] / args.steps
        assert dom["gbs"] <= HBM_PEAK_GBS, ("impossible roofline", dom)
        assert per_step <= T / args.steps * 1e3 * 1.001 or world > 1, \
            ("dominant kernel longer than the step", dom, T)
    # HBM traffic and the integer roofline of the SAME kernel on the SAME
    # workload, from the committed rocprofv3 PMC passes (scripts/
    # gpu_pmc_r03.sh -> scripts/pmc_r03.py); omitted when no pass matches
    # the dominant kernel's name and this workload
    wl = "config%d%s%s%s" % (cfg_id, "_rtcp" if args.rtcp else "",
                             "_ssrc%d" % K if K > 1 else "",
                             "_room%d" % args.room if args.room else "")
    pj = args.traffic_json or os.path.join(ROOT, "profiles", "r06_pmc.json")
    ent = None
    if dom and os.path.exists(pj):
        for e in json.load(open(pj)).get("entries", []):
            if e["kernel"] == dom["kernel"] and e["workload"] == wl:
                ent = e
    scale = dom["pkts_per_launch"] / ent["pkts_per_launch"] if ent else 0
    roof = None
    if dom:
        roof = {"bound": "hbm", "achieved": round(dom["gbs"], 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dom["gbs"] / HBM_PEAK_GBS, 4),
                "traffic": round(ent["traffic_bytes_per_launch"] * scale)
                if ent and ent.get("traffic_bytes_per_launch") else None,
                "int_frac": round(ent["int_frac"], 4)
                if ent and ent.get("int_frac") is not None else None,
                "lds_frac": round(ent["lds_frac"], 4)
                if ent and ent.get("lds_frac") is not None else None,
                "lds_floor_frac": round(ent["lds_floor_frac"], 4)
                if ent and ent.get("lds_floor_frac") is not None else None,
                # the integer issue-time ESTIMATE, co-issue corrected
                # (scripts/pmc_r05.py): max(VALU, LDS) + c x min(VALU, LDS)
                # of the launch, c measured (profiles/r04_ubench_coissue.txt);
                # an estimate, not a hard floor: the GCM kernels run up to
                # ~4 % under it (tests/test_pmc_cpu.py)
                "issue_frac": round(ent["issue_floor_frac"], 4)
                if ent and ent.get("issue_floor_frac") is not None else None,
                "coissue_c": ent.get("coissue_c") if ent else None,
                "issue_sum_frac": round(ent["issue_sum_frac"], 4)
                if ent and ent.get("issue_sum_frac") is not None else None,
                "pmc_src": os.path.basename(pj) + ":" + wl if ent else None,
                "kernel": dom["kernel"],
                "dir": dom["dir"],
                "avg_launch_ms": round(dom["avg_ms"], 4),
                "pkts_per_launch": dom["pkts_per_launch"],
                "bytes_per_launch": dom["bytes_per_launch"],
                "kernels": [{k: (round(v, 4) if isinstance(v, float) else v)
                             for k, v in d.items()} for d in kern]}
    gib = tot_bytes / T / 2**30
    line = {
        "metric": (METRIC.replace("SRTP", "SRTCP").replace("RTP", "RTCP")
                   if args.rtcp else METRIC) +
        (" [end-to-end: host pinned memory, incl. PCIe H2D/D2H]"
         if args.e2e else ""),
        "value": round(gib, 4),
        "unit": "GiB/s",
        "mpkt_s": round(tot_pkts / T / 1e6, 4),
        "n_gpus": world,
        "dist_world": dist.get_world_size() if world > 1 else 1,
        "dist_backend": dist.get_backend() if world > 1 else None,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(T / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "config%d: %s" % (cfg_id, cfg["name"]),
                   "packets_per_gpu": n, "pkt_len": cfg["length"] or
                   "200/1400", "suite": P.suite_name(suite),
                   "sessions": nsess, "ssrcs_per_session": K,
                   "slot_bytes": int(cap[0] - pos[0]),
                   "streams_announced": K > 1 and not args.fresh_streams,
                   "steps_in_flight": 2 if pipelined else 1,
                   "parallelism": "shard%d" % world,
                   "api": ("srtp_*_batch_dev_async" if use_async else
                           "srtp_*_batch_dev") if use_dev else
                   "srtp_*_batch"},
        "hbm_frac_e2e": round(tot_pkts / world * (4 * L + 2 * tag) /
                              (T / 1) / 1e9 / HBM_PEAK_GBS, 4),
        "errors": int(tot_err),
        "forged_per_batch": nforge,
        # where a synchronous one-stream call's host time goes (DESIGN
        # §10.6): issue (plan-out bookkeeping + launches), the stream
        # wait, completion; "outside" = the rest of the call's share of
        # the step (the Python loop, the ctypes call, the entry point)
        "sync_split_us": ({
            "calls_per_step": round(split[0] / args.steps, 2),
            "issue": round(split[1] / split[0] / 1e3, 2),
            "wait": round(split[2] / split[0] / 1e3, 2),
            "finish": round(split[3] / split[0] / 1e3, 2),
            "outside": round(elapsed / split[0] * 1e6 -
                             sum(split[1:]) / split[0] / 1e3, 2),
        } if split[0] else None),
        "folds": {"device": P.counter("devfolds"),
                  "host": P.counter("folds")},
        "plans": {"rejected": P.counter("rejects"),
                  "per_stream": P.counter("splans"),
                  "voided_launches": voided},
        "verified_roundtrip": verified,
        # config 5: ranks whose shard was checked against the reference's
        # digests and boundary states (tests/golden/config5_shards.json),
        # and how many matched
        "shards_vs_reference": {"checked": shards_checked, "ok": shards_ok}
        if shards_checked else None,
        "roofline": roof,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(cfg, args.rtcp)
    print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def udp_bench(args):
    """Socket-to-socket rate of the batched UDP helper: --udp-pairs socket
    pairs, each with a sender thread that protects config-2 packets (1200
    B, AES_CM_128_HMAC_SHA1_80, its own session) on the GPU and
    sendmmsg()s them over loopback, and a receiving thread that
    recvmmsg()s, unprotects on the GPU and counts the authentic packets
    (pipelined helpers by default: batch k+1 on the socket while batch k
    is on the GPU).  Loopback drops what a receiver cannot absorb, so the
    rate is the receivers'.  Per-stage times come from srtp_udp_times."""
    import ctypes
    import socket
    import threading
    import torch
    import re_amd.srtp as P
    from re_amd import workload as W

    torch.cuda.set_device(0)
    P.load()
    n = args.packets or (1 << 18)
    T = max(1, args.udp_pairs)
    pipe = not args.udp_sync
    arena, pos, end, cap = W.make_arena(n, 1200, s0=65000)
    keys = W.make_keys(T, 30)
    B = args.udp_batch
    pairs = []
    for t in range(T):
        a = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        b = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        a.bind(("127.0.0.1", 0))
        b.bind(("127.0.0.1", 0))
        for sk in (a, b):
            for opt in (socket.SO_RCVBUF, socket.SO_SNDBUF):
                sk.setsockopt(socket.SOL_SOCKET, opt, 1 << 26)
        key = keys[t].tobytes()
        tx, rx = P.Srtp(1, key), P.Srtp(1, key)
        st = P.SrtpUdp(a.fileno(), tx=tx, batch=B, slot=1280, pipeline=pipe)
        sr = P.SrtpUdp(b.fileno(), rx=rx, batch=B, slot=1280, pipeline=pipe)
        assert st.err == 0 and sr.err == 0, P.lib().srtp_gpu_error()
        pairs.append(dict(a=a, b=b, tx=tx, rx=rx, st=st, sr=sr,
                          addr=P.sockaddr_in(*b.getsockname()), sent=0,
                          t_end=0.0, last=None))
    base = arena.ctypes.data
    mbs = []
    for i in range(n):                  # mbuf views into the arena
        m = P.Mbuf()
        m.buf = ctypes.cast(base, ctypes.POINTER(ctypes.c_uint8))
        m.size, m.pos, m.end = int(cap[i]), int(pos[i]), int(end[i])
        mbs.append(ctypes.pointer(m))
    chunks = [(ctypes.POINTER(P.Mbuf) * len(mbs[k:k + B]))(*mbs[k:k + B])
              for k in range(0, n, B)]

    def sender(pr, deadline):
        L = P.lib()
        errs = (ctypes.c_int * B)()
        for ch in chunks:
            if time.perf_counter() >= deadline:
                break
            r = L.srtp_udp_send(pr["st"].ptr, pr["addr"], len(pr["addr"]),
                                ch, errs, len(ch))
            pr["sent"] += max(r, 0)
        pr["t_end"] = time.perf_counter()

    def receiver(pr, done):
        sr = pr["sr"]
        while True:
            got = sr.recv(200)
            if got > 0:
                pr["last"] = time.perf_counter()
            elif done.is_set() and got == 0:
                break

    done = threading.Event()
    t0 = time.perf_counter()
    deadline = t0 + args.udp_seconds
    ths = [threading.Thread(target=sender, args=(pr, deadline))
           for pr in pairs]
    rth = [threading.Thread(target=receiver, args=(pr, done))
           for pr in pairs]
    for th in rth + ths:
        th.start()
    for th in ths:
        th.join()
    time.sleep(0.3)
    done.set()
    for th in rth:
        th.join()
    ok = rcv = sent = 0
    stages = {}
    for pr in pairs:
        r, o, _ = pr["sr"].stats()
        rcv += r
        ok += o
        sent += pr["sent"]
        for k, v in list(pr["sr"].times().items()) + \
                list(pr["st"].times().items()):
            stages[k] = stages.get(k, 0.0) + v
    last = max([pr["last"] or t0 for pr in pairs])
    T_s = last - t0
    send_T = max(pr["t_end"] for pr in pairs) - t0
    line = {"metric": "socket-to-socket SRTP protect+send / recv+unprotect "
                      "over loopback UDP, 1200B RTP pkts (batched UDP helper)",
            "value": round(ok * 1200 / T_s / 2**30, 4) if T_s > 0 else 0.0,
            "unit": "GiB/s", "mpkt_s": round(ok / T_s / 1e6, 4) if T_s else
            0.0, "sent": sent, "received": rcv, "authentic": ok,
            "seconds": round(T_s, 3), "batch": B, "pairs": T,
            "pipelined": pipe,
            "send_side_mpkt_s": round(sent / send_T / 1e6, 4),
            "stage_seconds_summed_over_threads":
                {k: round(v, 3) for k, v in stages.items()},
            "data": "synthetic", "dtype": "u8",
            "config": {"workload": "config2 packets over loopback",
                       "suite": "AES_CM_128_HMAC_SHA1_80"}}
    print(json.dumps(line))
    for pr in pairs:
        pr["st"].close()
        pr["sr"].close()


def libre_helper_bench(args):
    """a single-threaded libre application (re_main,
    libre's udp_read per datagram) receiving config-2 SRTP over loopback,
    its transform on libre's UDP helper chain (/root/reference/src/udp/
    udp.c:830-928).  oracle/_ref/helper_bench_{ref,gpu} (built by
    oracle/Makefile, libre's loop from oracle/_ref/libre_net.so): flat out
    and paced runs, 200K datagrams each"""
    refx = os.path.join(ROOT, "oracle", "_ref", "helper_bench_ref")
    gpux = os.path.join(ROOT, "oracle", "_ref", "helper_bench_gpu")
    n = 200000
    runs = [(refx, "none", 0, 0, 0), (refx, "none", 600000, 0, 0)]
    for rate in (0, 100000, 300000, 400000):
        runs.append((refx, "ref", rate, 0, 0))
    for rate, batch in ((0, 1024), (0, 256), (100000, 64), (100000, 256),
                        (200000, 64), (200000, 256), (400000, 256),
                        (400000, 1024), (500000, 1024), (600000, 1024)):
        runs.append((gpux, "gpu", rate, batch, 1))
    res = []
    for exe, mode, rate, batch, flush in runs:
        cmd = [exe, mode, str(n), str(rate)] + \
            ([str(batch), str(flush)] if mode == "gpu" else [])
        out = subprocess.run(cmd, capture_output=True, text=True,
                             timeout=120, check=True, cwd=ROOT).stdout
        r = json.loads(out.strip().splitlines()[-1])
        print("bench.py: %s rate %s batch %s: %s pkt/s, lost %s, p50 %s us"
              % (mode, rate, batch, r["pkt_s"], r["lost"],
                 r["lat_us"]["p50"]), file=sys.stderr, flush=True)
        res.append(r)
    best = max((r for r in res if r["mode"] == "gpu"),
               key=lambda r: r["pkt_s"] * (r["lost"] == 0))
    line = {"metric": "SRTP unprotect on libre's UDP helper chain, one "
                      "re_main thread, 1200-B RTP over loopback",
            "value": best["pkt_s"], "unit": "pkt/s",
            "higher_is_better": True, "n_gpus": 1, "data": "synthetic",
            "dtype": "u8", "runs": res,
            "config": {"workload": "config2 datagrams, libre re_main + "
                                   "udp_read, srtp_udp_helper_alloc"}}
    print(json.dumps(line))
    return 0


def percall_bench(args):
    """per-packet drop-in path (one mbuf per srtp_encrypt / srtp_decrypt
    call, what every libre caller does): re_amd/lib/percall, a C driver of
    libre_srtp_amd.so, then the reference src/srtp on 1 core and on the
    job's cores for the same packet size"""
    exe = os.path.join(ROOT, "re_amd", "lib", "percall")
    threads = sorted({4, 16, 64})
    # --tune knobs reach the driver's library as srtp_gpu_tune calls
    env = dict(os.environ)
    env["PERCALL_SUITE"] = str(args.percall_suite)
    if args.tune:
        env["PERCALL_TUNE"] = ",".join(args.tune)
    out = subprocess.run([exe, str(args.percall_calls)] +
                         [str(t) for t in threads], capture_output=True,
                         text=True, timeout=900, check=True, env=env).stdout
    r = json.loads(out.strip().splitlines()[-1])
    line = {"metric": "per-call srtp_encrypt + srtp_decrypt of one 1200-B "
                      "RTP packet (unchanged re_srtp.h API)",
            "value": r["pairs_per_s_1thread"], "unit": "pairs/s",
            "higher_is_better": True, "n_gpus": 1, "data": "synthetic",
            "dtype": "u8", "percall": r,
            "config": {"workload": "per-call, %s, 1200 B" % r["suite"]}}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(CONFIGS[2])
    print(json.dumps(line))
    return 0


def rtcp_report_bench(args):
    """RTCP report path on one GPU: a step encodes n
    compounds (SR with one report block + SDES CNAME, libre's rtcp_sess
    report shape, one sender SSRC), SRTCP-protects and -unprotects them in
    place (AES_CM_128_HMAC_SHA1_80) and decodes them with their contents.
    value = compounds per second end to end; per-stage device times from
    stages run one at a time; the decoded fields of every 4099th compound
    are checked against the encode inputs after the timed steps."""
    import numpy as np
    import torch
    import re_amd.srtp as P

    torch.cuda.set_device(0)
    P.load()
    n = args.packets or (1 << 20)
    rng = np.random.default_rng(314)
    dm, drb, dch, dsd = P.rtcp_enc_dtypes()
    msg = np.zeros(2 * n, dtype=dm)
    msg["pt"][0::2], msg["pt"][1::2] = 200, 202
    msg["count"][:] = 1
    w = rng.integers(0, 2**32, (n, 6), dtype=np.uint64).astype(np.uint32)
    w[:, 0] = 0x5EED0001
    msg["w"][0::2] = w
    msg["first"][0::2] = msg["first"][1::2] = np.arange(n)
    msg["num"][:] = 1
    rb = np.zeros(n, dtype=drb)
    for f in drb.names:
        rb[f] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    clen = np.full(n, 20, dtype=np.uint32)          # "user@host.example"
    pool = rng.integers(33, 127, int(clen.sum()), dtype=np.uint8)
    chunk = np.zeros(n, dtype=dch)
    chunk["src"], chunk["first"], chunk["num"] = w[:, 0], np.arange(n), 1
    sdes = np.zeros(n, dtype=dsd)
    sdes["type"], sdes["len"] = 1, clen
    sdes["off"] = np.arange(n, dtype=np.uint32) * 20
    A = dict(msg=msg, rb=rb, chunk=chunk, sdes=sdes,
             src=np.zeros(1, dtype=np.uint32), pool=pool,
             mfirst=np.arange(0, 2 * n + 1, 2, dtype=np.uint32))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(
        np.uint8)).cuda()
    dA = {k: dev(v) for k, v in A.items()}
    slot = 192
    pos = np.arange(n, dtype=np.uint32) * slot
    arena = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(
        np.int32)).cuda()
    p_d, c_d = i32(pos), i32(pos + slot)
    e_d = torch.zeros(n, dtype=torch.int32, device="cuda")
    err = torch.zeros(n, dtype=torch.int32, device="cuda")
    maxmsg, maxitem = 2, 4
    desc = torch.zeros(n * maxmsg * 5, dtype=torch.int32, device="cuda")
    item = torch.zeros(n * maxitem * 8, dtype=torch.int32, device="cuda")
    nm, ni, ee, st = (torch.zeros(n, dtype=torch.int32, device="cuda")
                      for _ in range(4))
    key = bytes(range(30))
    tx, rx = P.Srtp(1, key), P.Srtp(1, key)

    def enc():
        assert P.rtcp_encode_dev(
            arena.data_ptr(), arena.numel(), p_d.data_ptr(), e_d.data_ptr(),
            c_d.data_ptr(), n, dA["mfirst"].data_ptr(), dA["msg"].data_ptr(),
            2 * n, dA["rb"].data_ptr(), n, dA["chunk"].data_ptr(), n,
            dA["sdes"].data_ptr(), n, dA["src"].data_ptr(), 1,
            dA["pool"].data_ptr(), len(pool), err.data_ptr()) == 0

    def srtcp(op, ctx):
        assert P.device_batch_dev(op, [ctx], arena.data_ptr(), arena.numel(),
                                  p_d.data_ptr(), e_d.data_ptr(),
                                  c_d.data_ptr(), err.data_ptr(), n) == 0

    def dec():
        assert P.rtcp_decode_full_dev(
            arena.data_ptr(), arena.numel(), p_d.data_ptr(), e_d.data_ptr(),
            n, desc.data_ptr(), maxmsg, nm.data_ptr(), item.data_ptr(),
            maxitem, ni.data_ptr(), ee.data_ptr(), st.data_ptr()) == 0

    stages = [("encode", enc), ("srtcp_protect",
                                lambda: srtcp("srtcp_encrypt", tx)),
              ("srtcp_unprotect", lambda: srtcp("srtcp_decrypt", rx)),
              ("decode_full", dec)]
    for _ in range(max(1, args.warmup)):
        for _, f in stages:
            f()
    torch.cuda.synchronize()
    steps = args.steps
    t0 = time.perf_counter()
    for _ in range(steps):
        for _, f in stages:
            f()
    torch.cuda.synchronize()
    T = (time.perf_counter() - t0) / steps
    # per stage (each idempotent on a plaintext arena; protect and
    # unprotect as a pair)
    per = {}
    for name, fs in (("encode", [enc]),
                     ("srtcp_protect_unprotect", [stages[1][1],
                                                  stages[2][1]]),
                     ("decode_full", [dec])):
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(steps):
            for f in fs:
                f()
        torch.cuda.synchronize()
        per[name] = (time.perf_counter() - a) / steps * 1e3
    # the last stage run was decode_full of a valid arena: check a sample
    it = item.cpu().numpy().view(np.uint32).reshape(n, maxitem, 8)
    ok = bool((ni.cpu().numpy() == 4).all() and not err.cpu().numpy().any())
    for i in range(0, n, 4099):
        ok &= bool((it[i, 0, 1:6] == w[i, 1:6]).all() and
                   it[i, 1, 1] == rb["ssrc"][i] and it[i, 2, 1] == w[i, 0]
                   and it[i, 3, 1] == 20)
    line = {"metric": "RTCP report path: compound encode + SRTCP protect + "
                      "unprotect + decode with contents, per compound",
            "value": round(n / T, 1), "unit": "compounds/s",
            "higher_is_better": True, "n_gpus": 1, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(T * 1e3, 3),
            "stage_ms": {k: round(v, 3) for k, v in per.items()},
            "bytes_per_compound": int((e_d.cpu().numpy().view(np.uint32) -
                                       pos)[0]),
            "verified_roundtrip": ok, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "rtcp-report: %d x (SR + 1 RB + SDES "
                                   "CNAME 20 B), AES_CM_128_HMAC_SHA1_80 "
                                   "SRTCP" % n}}
    print(json.dumps(line))
    tx.close()
    rx.close()
    return 0


def ctypes_stream(stream):
    """raw hipStream_t of a torch stream (None for the null stream)"""
    h = stream.cuda_stream
    return h if h else None


if __name__ == "__main__":
    sys.exit(main() or 0)
