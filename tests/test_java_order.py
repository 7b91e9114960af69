"""The Collect_Replicas order (IPLS.java:1218-1227): the key order of the JDK
HashMap<Pair<Integer,String>, double[]> Other_Replica_Gradients
(PeerData.java:140).  CPU only.

- String / javatuples Pair hash codes: the oracle's restatement against
  published Java values, and the library's ipls_java_pair_hash against the
  oracle (UTF-8 including supplementary characters; malformed bytes refused).
- The library front's order model (csrc/java_hashmap.hpp) against the
  oracle's simulation (oracle.JavaHashMap), two separate transliterations of
  JDK 8's HashMap and TreeNode code, over random put/remove/clear streams
  built to collide, resize, trigger treeifyBin's resize below 64 bins and
  build, split and shrink red-black tree bins; the oracle's own structure is
  checked after every step (TreeNode.checkInvariants plus the red-black
  rules).
Parity unpinned: no JDK here; the restatements follow the published JDK 8 and
javatuples 1.2 sources."""
import ctypes
import subprocess

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def O():
    from oracle import oracle
    return oracle

CSRC = ROOT / "ipls-java-api_amd" / "csrc"
DRIVER = ROOT / "tests" / "cpp" / "build" / "java_order_driver"


def test_java_string_hash_known_values(O):
    # values any JDK prints for "...".hashCode()
    assert O.java_string_hash("") == 0
    assert O.java_string_hash("hello") == 99162322
    assert O.java_string_hash("Aa") == O.java_string_hash("BB") == 2112
    assert O.java_string_hash("polygenelubricants") == -2147483648
    assert O.java_string_hash("a") == 97


def test_pair_hash_formula(O):
    # Arrays.asList(p, s).hashCode() = 31*(31*1 + p) + s.hashCode(); Tuple adds 31*1
    for p, s in ((0, ""), (3, "hello"), (-7, "QmXyz"), (2**31 - 1, "polygenelubricants")):
        lst = (31 * (31 + p) + O.java_string_hash(s)) & 0xFFFFFFFF
        want = (31 + lst) & 0xFFFFFFFF
        want = want - (1 << 32) if want >= 1 << 31 else want
        assert O.java_pair_hash(p, s) == want


def test_library_pair_hash_matches_oracle(O):
    import ipls
    from ipls import _native as N
    rng = np.random.default_rng(3)
    alphabet = "abcXYZ0189-_Qm" + "é€" + "\U0001F600"     # 1-, 2-, 3- and 4-byte UTF-8 (a surrogate pair in Java)
    for i in range(300):
        s = "".join(alphabet[j] for j in rng.integers(0, len(alphabet), int(rng.integers(0, 60))))
        p = int(rng.integers(-1000, 1 << 20))
        assert ipls.java_pair_hash(p, s) == O.java_pair_hash(p, s), (p, s)
    lib = ipls.lib()
    out = ctypes.c_int32()
    for bad in (b"\xff", b"\xc0\x80", b"a\xe2\x82", b"\xed\xa0\x80"):   # invalid, overlong, truncated, surrogate
        buf = (ctypes.c_uint8 * len(bad)).from_buffer_copy(bad)
        assert lib.ipls_java_pair_hash(0, ctypes.addressof(buf), len(bad), ctypes.byref(out)) == N.IPLS_E_FORMAT


def test_integer_keyed_hashmap_facts(O):
    """Well-known JDK 8 iteration facts, with Integer keys (hashCode = value):
    small keys iterate ascending whatever the insertion order; 16 and 0 share
    bin 0 of a 16-bin table and iterate in insertion order; the 13th key
    doubles the table, after which 16 and 0 separate."""
    m = O.JavaHashMap()
    for k in (9, 3, 12, 0, 5):
        m.put(k, k, None)
    assert m.keys() == [0, 3, 5, 9, 12]
    m = O.JavaHashMap()
    m.put(16, 16, None)
    m.put(0, 0, None)
    assert m.keys() == [16, 0]
    for k in range(1, 11):                      # 12 keys: still 16 bins
        m.put(k, k, None)
    assert len(m.table) == 16 and m.keys()[:2] == [16, 0]
    m.put(11, 11, None)                         # 13 > 12: resize to 32
    assert len(m.table) == 32 and m.keys() == list(range(12)) + [16]


def _build_driver():
    DRIVER.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    f"-I{CSRC}", str(ROOT / "tests" / "cpp" / "java_order_driver.cpp"), "-o", str(DRIVER)],
                   check=True)


@pytest.mark.parametrize("seed,mode", [(1, "java"), (2, "bits6"), (3, "bits5"), (4, "bits9"), (5, "java"),
                                       (6, "collide"), (7, "collide"), (8, "collide"), (9, "collide_big"),
                                       (10, "collide_big")])
def test_front_model_matches_jdk_table_simulation(O, seed, mode):
    """Random streams of put / remove / collect over (p, aggregator) keys,
    replayed on the library's model (csrc/java_hashmap.hpp, through
    tests/cpp/java_order_driver.cpp) and on the oracle's JavaHashMap -- two
    independent transliterations of JDK 8's HashMap / TreeNode.  After every
    'o' the capacities, tree flags and key orders must agree.  "java": real
    Pair hashCodes; "bitsN": N-bit hashes (many equal full hashes: chains,
    treeifyBin resizes below 64 bins, and trees whose equal-hash ties Java
    breaks by identity -- compared until that flag is raised); "collide":
    distinct full hashes with equal low 10 bits, so bins of >= 64-bin tables
    turn into red-black trees (treeify, putTreeVal, removeTreeNode with its
    rebalancing, split and untreeify on resize) whose chain order is exact."""
    _build_driver()
    rng = np.random.default_rng(seed)
    cmds, expect = [], []
    m, hashes, used = O.JavaHashMap(), {}, set()

    def draw_hash(p, a):
        if mode == "java":
            return O.java_pair_hash(p, f"12D3KooW{a}")
        if mode.startswith("bits"):
            return int(rng.integers(0, 1 << int(mode[4:])))
        base = int(rng.choice([7, 300, 1000]))
        while True:   # distinct full hashes whose spread h ^ (h >>> 16) keeps the low 10 bits = base
            h = base + (1 << 10) * int(rng.integers(0, 64)) + (1 << 26) * int(rng.integers(0, 32))
            if h not in used:
                used.add(h)
                return h

    n_keys = 25 if mode != "collide_big" else 60
    for step in range(3000):
        r = rng.integers(0, 20)
        p, a = int(rng.integers(0, 40)), int(rng.integers(0, n_keys))
        if r < 12:
            h = hashes[(p, a)] if (p, a) in hashes else draw_hash(p, a)
            cmds.append(f"p {p} {a} {h}")
            if (p, a) not in hashes:
                hashes[(p, a)] = h
                m.put((p, a), h, None)
        elif r < 17:
            cmds.append(f"r {p} {a}")
            if (p, a) in hashes:
                m.remove((p, a), hashes.pop((p, a)))
        else:
            cmds.append("o")
            m.check_invariants()                     # the oracle's own structure, JDK's checkInvariants and more
            expect.append((len(m.table) if m.table else 0, int(m.tree_bin), int(m.nondeterministic), m.keys()))
            if r == 19 and rng.random() < 0.15:
                cmds.append("c")
                m, hashes = O.JavaHashMap(), {}
    out = subprocess.run([str(DRIVER)], input="\n".join(cmds) + "\n", capture_output=True, text=True, timeout=120,
                         check=True).stdout.splitlines()
    assert len(out) == len(expect)
    compared = trees = 0
    for line, (cap, tree, nondet, keys) in zip(out, expect):
        f = line.split()
        assert int(f[2]) == nondet, (line[:80], nondet)
        if nondet:                                   # Java's own order is not reproducible from here on
            continue
        assert (int(f[0]), int(f[1])) == (cap, tree), (line[:80], cap, tree)
        got = [tuple(int(x) for x in kv.split(":")) for kv in f[3:]]
        assert got == keys
        compared += 1
        trees += tree
    assert compared > 30
    if mode.startswith("collide"):
        assert trees > 5, trees                      # the tree code really ran


def test_golden_java_order_cases(O):
    """tests/golden/java_order_expected.txt is the oracle's answer to
    java_order_cases.txt (tests/golden/make_java_order.py); the same text is
    what tests/java/PinJavaOrder.java prints from a real JVM, so on a host
    with a JDK a diff pins the restatement.  Here: the oracle still gives the
    committed answer, and so does the library's own model (the C++ driver fed
    the same keys and hashes)."""
    import sys
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_java_order as G
    cases = (ROOT / "tests" / "golden" / "java_order_cases.txt").read_text(encoding="utf-8").splitlines()
    want = (ROOT / "tests" / "golden" / "java_order_expected.txt").read_text(encoding="utf-8").splitlines()
    assert G.expected(cases) == want
    # the library's model: keys as (p, int index of the ID), hashes from the library itself
    import ipls
    _build_driver()
    ids, cmds, present = {}, [], set()
    for ln in cases:
        f = ln.split(" ")
        if f[0] == "put":
            k = (int(f[1]), ids.setdefault(f[2], len(ids)))
            cmds.append(f"p {k[0]} {k[1]} {ipls.java_pair_hash(int(f[1]), f[2])}")
        elif f[0] == "remove":
            cmds.append(f"r {f[1]} {ids.setdefault(f[2], len(ids))}")
        elif f[0] == "order":
            cmds.append("o")
        elif f[0] == "clear":
            cmds.append("c")
    out = subprocess.run([str(DRIVER)], input="\n".join(cmds) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout.splitlines()
    name = {v: k for k, v in ids.items()}
    got = [" ".join(["order"] + [f"{p}:{name[int(a)]}" for p, a in (kv.split(":") for kv in ln.split()[3:])])
           for ln in out]
    assert got == [w for w in want if w.startswith("order")]


def test_golden_java_pin_cases():
    """tests/golden/java_pin_expected.txt is this repository's restatement's
    answer (tests/golden/make_java_pins.py) to java_pin_cases.txt: folds,
    divides, putDouble / writeDouble, Base64 URL encode / decode (with the
    decoder's exceptions), Marshall_Packet frames and the ObjectOutputStream
    bytes of a Pair<Integer,double[]>.  tests/java/PinJavaCodecs.java prints
    the same text from a real JVM, so on a host with a JDK a diff pins them."""
    import sys
    import warnings
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_java_pins as G
    cases = (ROOT / "tests" / "golden" / "java_pin_cases.txt").read_text().splitlines()
    want = (ROOT / "tests" / "golden" / "java_pin_expected.txt").read_text().splitlines()
    assert G.cases() == cases
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)   # inf - inf in the fold cases
        assert [G.answer(c) for c in cases] == want


def test_library_codecs_match_java_pins():
    """The library's own host codecs (ipls_frame_encode, ipls_pair_encode;
    no GPU involved) give the pinned bytes of java_pin_expected.txt."""
    import sys
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_java_pins as G
    import ipls
    cases = (ROOT / "tests" / "golden" / "java_pin_cases.txt").read_text().splitlines()
    want = dict(zip(cases, (ROOT / "tests" / "golden" / "java_pin_expected.txt").read_text().splitlines()))
    n = 0
    for c in cases:
        f = c.split(" ")
        if f[0] == "frame":
            got = ipls.frame_encode(G.parse_dl(f[5]), int(f[2]), int(f[3]), int(f[1]), f[4].encode())
        elif f[0] == "pair":
            got = ipls.pair_encode(int(f[1]), G.parse_dl(f[2]))
        else:
            continue
        assert f"{f[0]} {bytes(got).hex()}" == want[c], c
        n += 1
    assert n == 6


def test_oracle_tree_invariants_hold_and_catch_damage(O):
    """The oracle's JavaHashMap after every operation of a colliding-hash
    stream (trees built, grown, split, shrunk, untreeified) passes
    check_invariants; and the checker is not vacuous: a recoloured node, a
    swapped child and a stale prev link are each reported."""
    rng = np.random.default_rng(11)
    m, hs, trees = O.JavaHashMap(), {}, 0
    for step in range(4000):
        k = (int(rng.integers(0, 8)), int(rng.integers(0, 40)))
        if rng.integers(0, 3) and k not in hs:
            while True:   # distinct hashes with spread low 10 bits = 7: one bin up to 1024 bins
                h = 7 + (1 << 10) * int(rng.integers(0, 64)) + (1 << 26) * int(rng.integers(0, 32))
                if h not in hs.values():
                    break
            hs[k] = h
            m.put(k, h, None)
        elif k in hs:
            m.remove(k, hs.pop(k))
        m.check_invariants()
        trees += m.tree_bin
    assert trees > 1000 and not m.nondeterministic

    def tree_head(mm):
        return next(e for e in mm.table if e is not None and e.tree)

    def damaged(hurt):
        mm = O.JavaHashMap()
        for j in range(20):
            mm.put((0, j), 7 + (1 << 10) * (j + 1), None)
        mm.check_invariants()
        hurt(tree_head(mm))
        with pytest.raises(AssertionError):
            mm.check_invariants()

    damaged(lambda r: setattr(r, "red", True))                                     # red root
    damaged(lambda r: (setattr(r, "left", r.right), setattr(r, "right", r.left)))  # order broken
    damaged(lambda r: setattr(r.next, "prev", None))                               # chain link broken
