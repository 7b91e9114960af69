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
    n_pass = r.stdout.count("PASS ")
    assert n_pass >= 10 and f"{n_pass} passed, 0 failed" in r.stdout, r.stdout


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


def _pubsub_corpus(path, seed=7, n=6000):
    """Mutated pubsub texts (1 and 2 base64url layers around Marshall_Packet
    frames) with the status and frame Java would produce: oracle/oracle.py's
    restatement of Base64.getUrlDecoder and the GET_GRADIENTS header rules."""
    import struct

    import numpy as np
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    alphabet = b"ABCXYZabcxyz0189-_"
    bad = b"+/=*\n.\x80 \x00"
    out = bytearray()

    def expect(text, layers):
        try:
            fr = O.java_b64url_decode(text)
            if layers == 2:
                fr = O.java_b64url_decode(fr)
        except O.JavaIllegalArgument:
            return -6, b""
        if len(fr) < 14:
            return -6, b""
        nd = int.from_bytes(fr[2:6], "big", signed=True)
        if nd < 0 or 14 + 8 * nd > len(fr):
            return -6, b""
        return 0, fr

    for t in range(n):
        layers = 1 + (t & 1)
        nd = int(rng.integers(0, 6))
        fr = bytearray(O.frame_encode(rng.standard_normal(nd), int(rng.integers(-2, 9)), 3, 3,
                                      bytes(rng.integers(65, 90, size=int(rng.integers(0, 5)), dtype=np.uint8))))
        if t % 13 == 0:
            fr[2:6] = int(rng.integers(-3, 9)).to_bytes(4, "big", signed=True)
        if t % 17 == 0:
            fr = fr[:int(rng.integers(0, len(fr) + 1))]
        m = bytearray(O.java_b64url_encode(bytes(fr)))
        if layers == 2:
            if t % 5 == 1 and len(m):
                m[int(rng.integers(0, len(m)))] = bad[int(rng.integers(0, len(bad)))]
            if t % 9 == 3:
                m = m.rstrip(b"=")
            m = bytearray(O.java_b64url_encode(bytes(m)))
        kind = int(rng.integers(0, 8))
        if kind == 1 and len(m):                        # bad char anywhere
            m[int(rng.integers(0, len(m)))] = bad[int(rng.integers(0, len(bad)))]
        elif kind == 2:                                 # '=' endings of every length
            m = m.rstrip(b"=") + b"=" * int(rng.integers(0, 4))
        elif kind == 3 and len(m):                      # truncation
            m = m[:int(rng.integers(0, len(m)))]
        elif kind == 4:                                 # '=' inside
            if len(m):
                m[int(rng.integers(0, len(m)))] = ord("=")
        elif kind == 5:                                 # random text
            m = bytearray(rng.choice(list(alphabet + b"="), size=int(rng.integers(0, 60))).astype(np.uint8).tobytes())
        elif kind == 6:                                 # extra chars at the end
            m += bytes(rng.choice(list(alphabet), size=int(rng.integers(1, 4))).astype(np.uint8).tobytes())
        st, frame = expect(bytes(m), layers)
        out += struct.pack("<BI", layers, len(m)) + bytes(m) + struct.pack("<iI", st, len(frame)) + frame
    path.write_bytes(bytes(out))


def test_pubsub_host_parser_under_asan(tmp_path):
    """the host half of the pubsub ingest (the '=' rules
    of both base64url layers, the 14-byte header read from the text's ends;
    csrc/pubsub_host.cpp, no HIP in it) built with AddressSanitizer + UBSan
    and fed mutated texts, each checked against the oracle's Java decoder."""
    out = ROOT / "tests" / "cpp" / "build" / "fuzz_pubsub"
    out.parent.mkdir(parents=True, exist_ok=True)
    csrc = ROOT / "ipls-java-api_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", f"-I{csrc}", str(ROOT / "tests" / "cpp" / "fuzz_pubsub.cpp"),
                    str(csrc / "pubsub_host.cpp"), "-o", str(out)], check=True)
    corpus = tmp_path / "pubsub.bin"
    _pubsub_corpus(corpus)
    r = subprocess.run([str(out), str(corpus)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fuzz ok" in r.stdout, r.stdout
