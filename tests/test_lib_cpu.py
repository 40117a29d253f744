"""CPU-side checks of the product C-ABI library (no GPU needed):
it loads, exports every symbol include/*.h declares, validates arguments
like the reference (srtp.c:98-158), and fails loudly (ENOSYS, like the
reference's stub backend src/aes/stub.c) when no HIP device exists."""
import ctypes
import errno
import os
import re
import subprocess

import pytest

import re_amd.srtp as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(headers=None):
    names = set()
    for h in headers or ("re_srtp.h", "re_srtp_batch.h", "re_srtp_udp.h",
              "re_srtp_keying.h", "re_rtcp_batch.h", "re_mbuf.h",
              "re_mem.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"static inline[^{]*\{[^}]*\}", "", src, flags=re.S)
        src = re.sub(r"^typedef.*$", "", src, flags=re.M)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, re.M):
            if m.group(1) not in ("if", "return", "sizeof"):
                names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    L = P.load()
    names = declared_functions()
    assert "srtp_alloc" in names and "srtp_decrypt_batch" in names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def dynsyms(path, defined):
    out = subprocess.run(["nm", "-D", "--defined-only" if defined else
                          "--undefined-only", path], check=True,
                         capture_output=True, text=True).stdout
    return sorted(ln.split()[-1].split("@")[0] for ln in out.splitlines()
                  if ln.strip())


def test_library_exports_nothing_else():
    """the version script (re_amd/exports.map) keeps the shim, the host
    pool and every other internal out of the caller's namespace"""
    got = [s for s in dynsyms(P.LIB_PATH, True)]
    assert got == declared_functions(), set(got) ^ set(declared_functions())


def test_libre_build_links_against_libre_only():
    """LIBRE=1: the build linked into libre itself
    exports only include/re_srtp*.h and takes mem_* / mbuf_* from libre:
    its undefined non-system symbols are exactly libre's own exports
    (declared in include/re_mem.h / re_mbuf.h, which mirror
    /root/reference/include/re_mem.h, re_mbuf.h)"""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "re_amd"),
                    "LIBRE=1"], check=True)
    lib = os.path.join(ROOT, "re_amd", "lib", "libre_srtp_amd_libre.so")
    srtp_only = [n for n in declared_functions()
                 if not n.startswith(("mem_", "mbuf_"))]
    # + the libre UDP helper (include/re_srtp_libre.h): LIBRE=1 only
    helper = declared_functions(("re_srtp_libre.h",))
    assert helper == ["srtp_udp_helper_alloc", "srtp_udp_helper_flush",
                      "srtp_udp_helper_stats"]
    assert dynsyms(lib, True) == sorted(srtp_only + helper)
    assert not set(helper) & set(dynsyms(P.LIB_PATH, True))
    undef = [u for u in dynsyms(lib, False) if u.startswith(("mem_", "mbuf_"))]
    assert undef, "expected libre's mem_/mbuf_ imports"
    assert set(undef) <= set(declared_functions()), undef
    ref = "/root/reference/include"
    if os.path.isdir(ref):
        decl = open(os.path.join(ref, "re_mem.h")).read() + \
            open(os.path.join(ref, "re_mbuf.h")).read()
        for u in undef:
            assert re.search(r"\b%s\s*\(" % u, decl), u


def test_suite_names_match_reference(golden):
    assert [P.lib().srtp_suite_name(s).decode() for s in range(-1, 8)] == \
        golden["names"]


def gpu_present():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(gpu_present(), reason="CPU-only expectation")
def test_alloc_argument_errors_without_gpu(golden):
    """Argument validation precedes any device work, so EINVAL/ENOTSUP are
    reference-exact even here; valid arguments give ENOSYS (no device)."""
    L = P.lib()
    for suite, klen, want in golden["alloc"]:
        p = ctypes.c_void_p()
        e = L.srtp_alloc(ctypes.byref(p), suite, bytes(64), klen, 0)
        if want == 0:
            assert e == errno.ENOSYS
        else:
            assert e == want, (suite, klen)
    assert L.srtp_alloc(None, 1, bytes(30), 30, 0) == errno.EINVAL


def test_mbuf_growth_policy():
    L = P.lib()
    mb = P.new_mbuf(b"\x01" * 10, 10)
    L.mbuf_write_mem  # noqa
    mb.contents.pos = 10
    assert L.mbuf_write_mem(mb, b"\x02" * 4, 4) == 0
    assert mb.contents.size == 20          # MAX(14, 2*10)
    mb.contents.pos = 20
    assert L.mbuf_write_mem(mb, b"\x03" * 30, 30) == 0
    assert mb.contents.size == 50          # MAX(50, 40)
    P.free_mbuf(mb)


def test_host_pool_covers_every_range_once(tmp_path):
    """par_for (re_amd/csrc/host/pool.c, the worker pool of the
    multi-session gather/apply passes; internal to the product library,
    built here on its own): over many back-to-back jobs of varying size
    every index is visited exactly once"""
    import numpy as np
    so = str(tmp_path / "libpool.so")
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", so,
                    os.path.join(ROOT, "re_amd", "csrc", "host", "pool.c"),
                    "-lpthread"], check=True)
    L = ctypes.CDLL(so)
    FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_size_t,
                          ctypes.c_size_t)
    L.par_for.argtypes = [ctypes.c_size_t, ctypes.c_size_t, FN,
                          ctypes.c_void_p]
    L.par_for.restype = None
    for n, min_per in ((1, 1), (7, 1), (100, 3), (5000, 64), (40000, 4096),
                       (3, 0), (64, 8)):
        seen = np.zeros(n, dtype=np.int64)

        def part(_arg, a, b, seen=seen):
            seen[a:b] += 1

        cb = FN(part)
        L.par_for(n, min_per, cb, None)
        assert (seen == 1).all(), (n, min_per)


def test_tune_knobs_and_counters():
    """srtp_gpu_tune accepts every A/B knob the library documents and
    rejects unknown ones; srtp_gpu_counter names every diagnostic counter
    (no GPU needed: neither touches the device)"""
    L = P.load()
    for k in ("noplan", "general", "perclass", "nolean", "nodevfold",
              "splan", "nomk", "freshmulti", "trace", "times",
              # round 6: the one-launch planner for AES-CM, the counting
              # grouping, the copy instead of the post launch, the
              # completion-word wait, the bucket target, the linger
              "lplan", "nobucket", "nopost", "syncspin"):
        assert L.srtp_gpu_tune(k.encode(), 1) == 0, k
        assert L.srtp_gpu_tune(k.encode(), 0) == 0, k
    for k, v in (("bpexp", 2100), ("pclinger", 100)):
        assert L.srtp_gpu_tune(k.encode(), v) == 0, k
        assert L.srtp_gpu_tune(k.encode(), 0) == 0, k
    assert L.srtp_gpu_tune(b"no-such-knob", 1) != 0
    for c in ("misses", "folds", "rejects", "devfolds", "splans",
              "freshmulti", "fused", "lplans", "dplans", "mplans", "rplans",
              "lbtimeouts", "sync_calls", "sync_ns_issue", "sync_ns_wait",
              "sync_ns_finish"):
        assert P.counter(c) >= 0, c


def test_cpu_baseline_threads_and_processes():
    """bench.py's cpu_baseline: the reference src/srtp (oracle/_ref/ref_bench,
    built from the reference's own sources) on 1 core, as threads of one
    process and as single-threaded processes; value is the faster all-core
    leg, every leg error-free (a run with reference errors fails loudly)"""
    import bench
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_bench")):
        pytest.skip("oracle/_ref/ref_bench not built")
    cb = bench.cpu_baseline({"suite": 4, "length": 160, "nsess": 1})
    assert cb["kind"] == "reference"
    assert cb["value_1core"] > 0 and cb["value_threads"] > 0
    if cb["cores"] > 1:
        assert cb["value_processes"] > 0
        assert cb["value"] == max(cb["value_threads"],
                                  cb["value_processes"])
