"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5:
"ASan/UBSan on the CPU oracle"): the product's .nnue parser / writer /
generator and board code, and both CPU restatements (scalar oracle, SIMD
baseline), built with gcc -fsanitize=address,undefined and driven by
tests/sanitize/san_main.cpp on valid and corrupt inputs.  CPU only."""
import os
import shutil
import subprocess

import pytest

from tests.conftest import ROOT

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
       "-march=x86-64-v3"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_code_under_asan_ubsan(tmp_path):
    out = tmp_path / "san_main"
    objs = []
    for src in ("oracle/nnue_oracle.c", "oracle/nnue_cpu_simd.c", "oracle/variant_oracle.c"):
        o = tmp_path / (os.path.basename(src) + ".o")
        subprocess.run(["gcc", "-std=c11", *SAN, "-c", os.path.join(ROOT, src), "-o", str(o)], check=True)
        objs.append(str(o))
    subprocess.run(["g++", "-std=c++17", *SAN, os.path.join(ROOT, "tests/sanitize/san_main.cpp"),
                    os.path.join(ROOT, "fishnet_amd/csrc/net.cpp"), os.path.join(ROOT, "fishnet_amd/csrc/board.cpp"),
                    *objs, "-lpthread", "-o", str(out)], check=True)
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(out)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitized host checks ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_backend_thread_pool_under_tsan(tmp_path):
    """The engine actor's host thread pool (fishnet_amd/csrc/workers.h: tickets
    for as many workers as a loop has chunks) under ThreadSanitizer: 40k runs of
    every size against the grain, each index exactly once, no race, no lost
    wake-up (a hang fails the timeout)."""
    out = tmp_path / "workers_stress"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                    os.path.join(ROOT, "tests/sanitize/workers_stress.cpp"), "-o", str(out)], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(out)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "workers stress ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("mode", ["asan", "ubsan"])
def test_move_text_scan_sanitized(tmp_path, mode):
    """The engine actor's scan of server-supplied move text
    (fishnet_amd/csrc/text_scan.h): under ASan + UBSan (the scalar
    form, every read inside the caller's allocation) and under UBSan alone
    (the 16-byte form against the scalar one, strings at every alignment and
    ending on a page whose successor is inaccessible)."""
    out = tmp_path / f"text_scan_{mode}"
    flags = SAN if mode == "asan" else ["-fsanitize=undefined", "-fno-sanitize-recover=all", "-g", "-O2",
                                          "-march=x86-64-v3"]
    subprocess.run(["g++", "-std=c++17", *flags, os.path.join(ROOT, "tests/sanitize/text_scan_check.cpp"),
                    "-o", str(out)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(out)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "text scan ok" in r.stdout
