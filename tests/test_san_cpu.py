"""Host C under gcc's sanitizers (the reference runs ASan,
UBSan and TSan in CI, cmake/sanitizer.cmake, .github/workflows/
sanitizers.yml).

  * the worker pool (re_amd/csrc/host/pool.c) driven by concurrent callers
    (tests/c/pool_stress.c) under ThreadSanitizer and under
    AddressSanitizer + UBSan: no report, every result right;
  * the library's sanitizer builds (make -C re_amd SAN=address,undefined /
    SAN=thread) link and export the same symbols; scripts/san_check.sh
    runs the whole CPU suite (and on a GPU box the GPU suite) against the
    ASan + UBSan build.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "re_amd", "csrc", "host")


def build_run(tmp_path, san):
    exe = str(tmp_path / ("pool_stress_" + san.replace(",", "_")))
    subprocess.check_call(["gcc", "-O1", "-g", "-fsanitize=" + san,
                           "-fno-omit-frame-pointer",
                           "-fno-sanitize-recover=all", "-I" + HOST, "-o",
                           exe, os.path.join(ROOT, "tests", "c",
                                             "pool_stress.c"),
                           os.path.join(HOST, "pool.c"), "-lpthread"])
    env = dict(os.environ, RE_SRTP_THREADS="6", RE_SRTP_SPIN="50",
               TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=env)
    return r


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_pool_under_sanitizer(tmp_path, san):
    r = build_run(tmp_path, san)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        r.stderr[-4000:]
    assert "0 wrong" in r.stdout


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_library_sanitizer_build(san):
    subprocess.check_call(["make", "-s", "-j8", "-C",
                           os.path.join(ROOT, "re_amd"), "SAN=" + san])
    lib = os.path.join(ROOT, "re_amd", "lib", "libre_srtp_amd_san-%s.so" %
                       san.replace(",", "-"))
    plain = os.path.join(ROOT, "re_amd", "lib", "libre_srtp_amd.so")
    syms = lambda p: sorted(ln.split()[-1] for ln in subprocess.run(
        ["nm", "-D", "--defined-only", p], capture_output=True,
        text=True).stdout.splitlines() if " T " in ln)
    assert syms(lib) == syms(plain)
