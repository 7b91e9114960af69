"""The C++ host mirror (ipls-java-api_amd/host/ipls_host.hpp: IPLS, Updater,
Light_IPLS_Daemon, MyIPFSClass, Middleware with Java names and exceptions)
driven by tests/cpp/test_host_parity.cpp against the C oracle."""
import subprocess

import pytest

from conftest import GOLDEN, ROOT

BIN = ROOT / "tests" / "cpp" / "build" / "test_host_parity"


def _build():
    subprocess.run(["make", "-s", "-C", str(ROOT / "ipls-java-api_amd"), "host_test"], check=True)
    assert BIN.exists()


def test_host_mirror_host_only():
    _build()
    r = subprocess.run([str(BIN), "--no-gpu", str(GOLDEN)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "2 passed, 0 failed" in r.stdout


@pytest.mark.gpu
def test_host_mirror_on_gpu():
    _build()
    r = subprocess.run([str(BIN), "--gpu", str(GOLDEN)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "8 passed, 0 failed" in r.stdout, r.stdout


def test_partial_update_parser_under_asan():
    """Fuzz the Java-serialisation parser (csrc/javaser.cpp) built for the
    host with AddressSanitizer + UBSan (no GPU code involved)."""
    out = ROOT / "tests" / "cpp" / "build" / "fuzz_javaser"
    out.parent.mkdir(parents=True, exist_ok=True)
    csrc = ROOT / "ipls-java-api_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", f"-I{csrc}", str(ROOT / "tests" / "cpp" / "fuzz_javaser.cpp"),
                    str(csrc / "javaser.cpp"), "-o", str(out)], check=True)
    r = subprocess.run([str(out), str(GOLDEN / "ref_scheduler.ser")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fuzz ok" in r.stdout
