#!/usr/bin/env python3
"""Generate tests/golden/java_pin_cases.txt and java_pin_expected.txt: the
Java-library behaviours the aggregation path depends on, with the answers of
this repository's restatement (oracle/oracle.py, oracle/javaser.py).
tests/java/PinJavaCodecs.java prints the same text from a real JVM (javac +
javatuples 1.2); on a host with a JDK, `diff` pins the restatement.  No JDK
here: parity unpinned.

Cases, one per line (doubles as 16-hex-digit IEEE bit patterns, byte strings
as hex, '-' for an empty list):
  fold ACC G          acc[i] = acc[i] + g[i]   (Updater.java:115-117, IPLS.java:1227)
  divide W SECURE     GetPartitions' divide of one partition (IPLS.java:1159-1174)
  putdouble X         ByteBuffer.putDouble (update_file, MyIPFSClass.java:105-116)
  writedouble X       DataOutputStream.writeDouble (Middleware.java:164-170)
  b64enc BYTES        Base64.getUrlEncoder().encodeToString (MyIPFSClass.java:1016)
  b64dec TEXT         Base64.getUrlDecoder().decode (Utils.java:8-17, IPLS.java:855-859)
  frame PID N_A N_B ORIGIN G   Marshall_Packet(double[],...) bytes (MyIPFSClass.java:990-1016)
  pair WORKERS G      ObjectOutputStream bytes of new Pair<>(workers, double[]) (MyIPFSClass.java:160-166)
Expected: one line per case, `<op> <answer>`; a NaN result prints as NaN
(Java does not specify NaN payloads, JLS 15.18.2); a thrown
IllegalArgumentException prints IAE."""
from __future__ import annotations

import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import javaser as J  # noqa: E402
from oracle import oracle as O  # noqa: E402

HERE = Path(__file__).resolve().parent


def h(x: float) -> str:
    return f"{struct.unpack('>Q', struct.pack('>d', x))[0]:016x}"


def hb(bits: int) -> str:
    return f"{bits:016x}"


def dl(vals) -> str:
    return ",".join(h(float(v)) for v in vals) if len(vals) else "-"


def parse_dl(s: str) -> np.ndarray:
    if s == "-":
        return np.zeros(0)
    return np.array([struct.unpack(">d", bytes.fromhex(t))[0] for t in s.split(",")], dtype=np.float64)


def show(vals) -> str:
    return ",".join("NaN" if v != v else h(float(v)) for v in vals) if len(vals) else "-"


SPECIAL = [0.0, -0.0, 5e-324, -5e-324, 1e16, 1.0, -1e16, 1e308, -1e308, float("inf"), -float("inf"),
           0.1, 0.2, 1.0 / 3.0, 2.5, -7.75]


def cases() -> list[str]:
    rng = np.random.default_rng(4)
    out = []
    for i in range(6):
        a = rng.choice(SPECIAL, 8)
        g = rng.choice(SPECIAL, 8)
        out.append(f"fold {dl(a)} {dl(g)}")
    out.append(f"fold {dl([1e16, 0.0, -0.0])} {dl([1.0, -0.0, -0.0])}")
    for w, sec in (([3.0, -6.0, 0.0], 0), ([1.0, 2.0, 0.0], 0), ([1.0, 2.0, -0.0], 0), ([4.0, 1e-300, 3.0], 0),
                   ([7e12, -1.0, 2.0], 1), ([0.3, 0.6, 3.0], 1), ([5.0, 1.0, float("inf")], 0)):
        out.append(f"divide {dl(w)} {sec}")
    for x in (1.5, -0.0, 5e-324, float("inf")):
        out.append(f"putdouble {h(x)}")
        out.append(f"writedouble {h(x)}")
    out.append(f"putdouble {hb(0x7ff8000000000123)}")   # a NaN payload: putDouble keeps it
    out.append(f"writedouble {hb(0x7ff8000000000123)}")  # writeDouble: doubleToLongBits -> 0x7ff8...
    out.append(f"writedouble {hb(0xfff8000000000000)}")
    for data in (b"", b"\x00", b"\xfb\xff", b"\xfb\xff\xbf", bytes(range(40))):
        out.append(f"b64enc {data.hex() or '-'}")
    for text in ("AAEC", "-_-_", "AA==", "AAA=", "AA=", "A", "AB*C", "QUJD", "QUI", "QUJDRA==="):
        out.append(f"b64dec {text}")
    out.append(f"frame 3 7 42 QmOrigin {dl([1.5, -0.0, 1e300])}")
    out.append("frame 4 0 1 Q -")
    out.append(f"frame -2 -1 2147483647 12D3KooWX {dl(rng.standard_normal(5))}")
    out.append(f"pair 3 {dl([1.5, -0.0, 5e-324])}")
    out.append("pair 0 -")
    out.append(f"pair 2147483647 {dl(rng.standard_normal(4))}")
    return out


def answer(line: str) -> str:
    f = line.split(" ")
    op = f[0]
    if op == "fold":
        acc, g = parse_dl(f[1]), parse_dl(f[2])
        return f"fold {show(O.fold(acc.copy(), g))}"
    if op == "divide":
        return f"divide {show(O.divide(parse_dl(f[1]), bool(int(f[2]))))}"
    if op == "putdouble":
        return f"putdouble {bytes.fromhex(f[1]).hex()}"            # raw bits, big-endian
    if op == "writedouble":
        x = np.frombuffer(bytes.fromhex(f[1]), dtype=">f8").astype(np.float64)
        return f"writedouble {O.be_encode_canonical(x).hex()}"
    if op == "b64enc":
        data = b"" if f[1] == "-" else bytes.fromhex(f[1])
        return f"b64enc {O.java_b64url_encode(data).decode() or '-'}"
    if op == "b64dec":
        try:
            return f"b64dec {O.java_b64url_decode(f[1].encode()).hex() or '-'}"
        except O.JavaIllegalArgument:
            return "b64dec IAE"
    if op == "frame":
        pid, a, b, origin = int(f[1]), int(f[2]), int(f[3]), f[4].encode()
        return f"frame {O.frame_encode(parse_dl(f[5]), a, b, pid, origin).hex()}"
    if op == "pair":
        return f"pair {J.encode_pair(int(f[1]), parse_dl(f[2])).hex()}"
    raise ValueError(line)


def main():
    c = cases()
    (HERE / "java_pin_cases.txt").write_text("\n".join(c) + "\n")
    (HERE / "java_pin_expected.txt").write_text("\n".join(answer(x) for x in c) + "\n")


if __name__ == "__main__":
    main()
