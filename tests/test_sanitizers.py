"""Host-side sanitizer runs: the native Prometheus matrix decoder
(``ingest/csrc/prom_parse.cpp``) built with AddressSanitizer + UBSan and driven
by a deterministic mutation harness (``prom_parse_fuzz.cpp``: seed bodies,
byte flips, truncation, duplication, punctuation insertion) through every
entry point, each input in an exactly-sized heap buffer.  GPU sanitizers are
not available on the target pool, so this covers the host parser only."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "foremast_amd", "ingest", "csrc")


def _build(tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "prom_fuzz")
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I", CSRC, "-o", exe, os.path.join(CSRC, "prom_parse_fuzz.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[:200]}")
    assert r.returncode == 0, r.stderr
    return exe


def test_prom_parser_asan_ubsan_fuzz(tmp_path):
    exe = _build(tmp_path)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "30000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "fuzz OK" in r.stdout
