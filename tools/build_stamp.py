#!/usr/bin/env python3
"""Write the provenance record of a freshly linked libipls_agg.so.

Usage: build_stamp.py LIB.so  -> LIB.so.buildinfo.json next to it.

The record ties every bench / PMC number to the code it measured: the .so's
own sha256, the git revision the tree was at when it was linked (plus whether
the library's sources differed from that revision), and a sha256 over the
kernel sources (ipls_kernels.hpp + engine.hip, the kernels and their
dispatch).  The GPU box receives the tree without .git, so the revision is
recorded here, at build time; bench.py re-hashes the .so at run time and
reports whether it is still the library this stamp describes.
"""
import hashlib
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "ipls-java-api_amd" / "csrc"
KERNEL_SOURCES = ("ipls_kernels.hpp", "engine.hip")
LIB_SOURCES = ("ipls-java-api_amd/csrc", "include/ipls_agg.h", "ipls-java-api_amd/Makefile")


def sha256_file(p: Path) -> str:
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def kernel_src_sha256(csrc: Path = CSRC) -> str:
    h = hashlib.sha256()
    for n in KERNEL_SOURCES:
        h.update(n.encode() + b"\0" + (csrc / n).read_bytes())
    return h.hexdigest()


def lib_src_sha256(root: Path = ROOT) -> str:
    """sha256 over every source the library is linked from (csrc/*, the
    header, the Makefile), in name order.  The sources travel to the GPU box
    with the tree, so the box can recompute it and check that the shipped
    .so was built from exactly the sources beside it (ipls.build_info)."""
    h = hashlib.sha256()
    files = sorted(p for p in (root / "ipls-java-api_amd" / "csrc").iterdir() if p.is_file())
    files += [root / "include" / "ipls_agg.h", root / "ipls-java-api_amd" / "Makefile"]
    for p in files:
        h.update(str(p.relative_to(root)).encode() + b"\0" + p.read_bytes())
    return h.hexdigest()


def device_code_sha256(lib: Path):
    """sha256 of the .hip_fatbin section of the .so: the gfx950 code objects of
    every kernel, nothing of the host code.  Two builds with the same value
    run the same kernel ISA, so a PMC count taken on one applies to the other
    (for the same launch).  Pure-Python ELF64 section walk (no binutils
    needed on the GPU box); None if the section is missing."""
    import struct
    data = Path(lib).read_bytes()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        return None
    e_shoff, = struct.unpack_from("<Q", data, 0x28)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sh(i):
        o = e_shoff + i * e_shentsize
        name, _typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", data, o)
        return name, off, size
    _, str_off, _ = sh(e_shstrndx)
    for i in range(e_shnum):
        name, off, size = sh(i)
        end = data.index(b"\0", str_off + name)
        if data[str_off + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()
    return None


def _git(*args):
    try:
        r = subprocess.run(["git", "-C", str(ROOT), *args], capture_output=True, text=True, timeout=30)
        return r.stdout.strip() if r.returncode == 0 else None
    except (OSError, subprocess.SubprocessError):
        return None


def main():
    lib = Path(sys.argv[1]).resolve()
    rev = _git("rev-parse", "HEAD")
    dirty = _git("status", "--porcelain", "--", *LIB_SOURCES)
    rec = {
        "so": lib.name,
        "so_sha256": sha256_file(lib),
        "kernel_src_sha256": kernel_src_sha256(),
        "lib_src_sha256": lib_src_sha256(),
        "device_code_sha256": device_code_sha256(lib),
        "git_rev": rev,
        "sources_dirty": None if dirty is None else bool(dirty),
        "built_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
    }
    out = lib.with_name(lib.name + ".buildinfo.json")
    out.write_text(json.dumps(rec, indent=1) + "\n")
    print(f"build stamp: {out.name} rev {rev} dirty={rec['sources_dirty']} so {rec['so_sha256'][:12]}")


if __name__ == "__main__":
    main()
