"""The Java-serialised partial update, org.javatuples.Pair<Integer, double[]>
(MyIPFSClass.java:160-166 writes it, :326-338 reads it), on the CPU: the
oracle (oracle/javaser.py) pinned against object streams the reference wrote
itself, and the C-ABI codec (ipls_pair_parse / ipls_pair_encode) against the
oracle.  No GPU needed."""
import random

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import javaser as J

SCHED = (GOLDEN / "ref_scheduler.ser").read_bytes()     # the reference's Scheduler file (a Pair)
ETH_HEAD = (GOLDEN / "ref_ethmodel_head.bin").read_bytes()   # first 136 bytes of its ETHModel


@pytest.fixture(scope="module")
def ipls():
    import ipls as _ipls
    try:
        _ipls.lib()
    except ImportError as e:
        pytest.skip(f"libipls_agg.so not built: {e}")
    return _ipls


def test_oracle_reads_reference_stream():
    """A Java-written Pair<ArrayList<Integer>, String> parses completely."""
    o, end = J.read_object(SCHED)
    assert end == len(SCHED) and o["class"] == "org.javatuples.Pair"
    v0 = o["fields"][("org.javatuples.Pair", "val0")]
    v1 = o["fields"][("org.javatuples.Pair", "val1")]
    assert v0["class"] == "java.util.ArrayList" and v0["fields"][("java.util.ArrayList", "size")] == 5
    ints = [x["fields"][("java.lang.Integer", "value")] for x in v0["annotations"]["java.util.ArrayList"][1:]]
    assert ints[-1] == 1 and len(ints) == 5
    assert v1.startswith("Qm") and len(v1) == 46
    tup = o["fields"][("org.javatuples.Tuple", "valueArray")]
    assert tup["values"][0] is v0 and tup["values"][1] == v1


def _desc_bytes(stream: bytes, name: bytes, extra: int) -> bytes:
    i = stream.index(name) - 3                     # TC_CLASSDESC, u16 length
    return stream[i:i + 3 + len(name) + extra]


def test_oracle_encoder_matches_reference_bytes():
    """Every class descriptor of the encoded Pair<Integer,double[]> is
    byte-identical to the one the reference's own streams hold."""
    enc = J.encode_pair(3, np.array([1.0, 2.0]))
    n = 0
    while enc[n] == SCHED[n]:
        n += 1
    assert n >= 224            # magic .. Pair/Tuple descs .. Object[] desc .. array length 2
    for name, extra in ((b"java.lang.Integer", 8 + 1 + 2 + 1 + 2 + 5 + 1), (b"java.lang.Number", 8 + 1 + 2 + 1 + 1),
                        (b"java.util.Arrays$ArrayList", 8 + 1 + 2 + 1 + 3 + 5 + 1 + 1)):
        assert _desc_bytes(enc, name, extra) == _desc_bytes(SCHED, name, extra), name
    d = bytes([0x75, 0x72, 0x00, 0x02]) + b"[D"
    assert enc[enc.index(d):enc.index(d) + 19] == ETH_HEAD[ETH_HEAD.index(d):ETH_HEAD.index(d) + 19]


@pytest.mark.parametrize("n", [0, 1, 3, 1000])
def test_c_codec_matches_oracle(ipls, n):
    rng = np.random.default_rng(n)
    g = rng.standard_normal(n)
    if n >= 3:
        g[:3] = [-0.0, np.inf, 5e-324]
    b = ipls.pair_encode(n * 7 + 1, g)
    assert b == J.encode_pair(n * 7 + 1, g)
    got, w, off = ipls.pair_parse(b)
    ow, og, ooff = J.parse_pair(b)
    assert (w, off) == (ow, ooff) == (n * 7 + 1, ooff)
    assert got.view(np.uint64).tolist() == g.view(np.uint64).tolist() == og.view(np.uint64).tolist()


def test_c_parser_walks_reference_stream(ipls):
    """The reference's Pair<ArrayList,String> is well-formed but not a partial update."""
    with pytest.raises(ipls.IplsError, match="val0 is not an Integer"):
        ipls.pair_parse(SCHED)


def test_c_parser_rejects_truncated_and_mutated(ipls):
    good = J.encode_pair(5, np.arange(40, dtype=np.float64))
    for cut in range(len(good)):
        with pytest.raises(ipls.IplsError):
            ipls.pair_parse(good[:cut])
    rnd = random.Random(7)
    ok = bad = 0
    for _ in range(3000):
        b = bytearray(good if rnd.random() < 0.5 else SCHED)
        for _ in range(rnd.randint(1, 4)):
            b[rnd.randrange(len(b))] = rnd.randrange(256)
        try:
            ipls.pair_parse(bytes(b))
            ok += 1
        except ipls.IplsError:
            bad += 1
    assert ok + bad == 3000 and bad > 0
