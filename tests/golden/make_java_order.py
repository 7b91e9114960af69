#!/usr/bin/env python3
"""Generate tests/golden/java_order_cases.txt and java_order_expected.txt:
operation streams on PeerData.Other_Replica_Gradients (PeerData.java:140) --
the puts of Download_Scheduler.java:254-266, the removes of :215-217 /
:329-332, and Collect_Replicas' `new ArrayList<>(keySet())` (IPLS.java:1218)
followed by `new HashMap<>()` -- and what JDK 8's HashMap gives for them,
as restated by oracle/oracle.py (JavaHashMap, java_pair_hash).

The expected file is the oracle's answer.  tests/java/PinJavaOrder.java
prints the same text from a real JVM (javac + javatuples 1.2, the
reference's pom.xml:66-68): where a JDK exists, `diff` of the two pins the
restatement.  No JDK here: parity unpinned.

Cases file, one command per line:
  case NAME | put P ID | remove P ID | order | clear
Expected file: for every put of an absent key `hash P ID <Pair.hashCode()>`,
for every order `order P:ID P:ID ...`."""
from __future__ import annotations

import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402

HERE = Path(__file__).resolve().parent


def cases() -> list[str]:
    rnd = random.Random(20261017)
    out = []
    # 1: three IPFS-like peer IDs on one partition, then two more partitions
    out.append("case three_aggregators")
    for p in (0, 1, 2):
        for i in range(3):
            out.append(f"put {p} 12D3KooWPeer{chr(65 + i)}{p}")
    out.append("order")
    out.append("clear")
    # 2: growth past 12 and 24 keys (resizes to 32 and 64), removes between
    out.append("case resize_and_remove")
    keys = []
    for j in range(40):
        p, idx = rnd.randrange(16), rnd.randrange(6)
        pid = f"QmAggregator{idx}x{'y' * idx}"
        out.append(f"put {p} {pid}")
        keys.append((p, pid))
        if j % 7 == 6:
            q, qid = rnd.choice(keys)
            out.append(f"remove {q} {qid}")
        if j % 10 == 9:
            out.append("order")
    out.append("clear")
    # 3: a removed key put again goes to the tail of its bin
    out.append("case reinsert_to_tail")
    for pid in ("QmPeer0006", "QmPeer0011", "QmPeer0030", "QmPeerZ"):
        out.append(f"put 0 {pid}")
    out.append("remove 0 QmPeer0006")
    out.append("put 0 QmPeer0006")
    out.append("order")
    out.append("clear")
    # 4: non-ASCII IDs (UTF-16 units, a surrogate pair)
    out.append("case non_ascii")
    for pid in ("Qmété", "Qm€", "Qm\U0001F600", "Qm"):
        out.append(f"put 5 {pid}")
    out.append("order")
    out.append("clear")
    # 5: a red-black tree bin: 14 IDs whose Pair(0, id) hashes agree in the low 8
    # bits after h ^ (h >>> 16) (found by search) share one bin up to 256 bins,
    # so the 9th of them turns the bin into a TreeNode tree at 64 bins; then
    # removals (removeTreeNode), more keys (resizes: split / untreeify)
    out.append("case tree_bin")
    coll, i, want = [], 0, None
    while len(coll) < 14:
        pid = f"QmTree{i}"
        i += 1
        b = O.JavaHashMap.spread(O.java_pair_hash(0, pid)) & 255
        if want is None:
            want = b
        if b == want and O.java_pair_hash(0, pid) not in {O.java_pair_hash(0, c) for c in coll}:
            coll.append(pid)
    for pid in coll:
        out.append(f"put 0 {pid}")
    out.append("order")
    for pid in (coll[3], coll[0], coll[9]):
        out.append(f"remove 0 {pid}")
    out.append("order")
    for j in range(60):
        out.append(f"put {1 + j % 7} 12D3KooWFill{j}")
        if j % 20 == 19:
            out.append("order")
    for pid in coll[4:9]:
        out.append(f"remove 0 {pid}")
    out.append("order")
    out.append("clear")
    # 6: many keys of one aggregator over many partitions (the hashes 992 + 31p + h)
    out.append("case one_aggregator_many_partitions")
    for p in range(0, 200, 3):
        out.append(f"put {p} 12D3KooWSame")
    out.append("order")
    out.append("clear")
    return out


def expected(lines: list[str]) -> list[str]:
    out = []
    m, hashes = O.JavaHashMap(), {}
    for ln in lines:
        f = ln.split(" ")
        if f[0] == "case":
            out.append(ln)
        elif f[0] == "put":
            p, pid = int(f[1]), f[2]
            if (p, pid) not in hashes:
                h = O.java_pair_hash(p, pid)
                hashes[(p, pid)] = h
                m.put((p, pid), h, None)
                out.append(f"hash {p} {pid} {h}")
        elif f[0] == "remove":
            p, pid = int(f[1]), f[2]
            if (p, pid) in hashes:
                m.remove((p, pid), hashes.pop((p, pid)))
        elif f[0] == "order":
            assert not m.nondeterministic
            out.append("order " + " ".join(f"{p}:{pid}" for p, pid in m.keys()))
        elif f[0] == "clear":
            m, hashes = O.JavaHashMap(), {}
    return out


def main():
    c = cases()
    (HERE / "java_order_cases.txt").write_text("\n".join(c) + "\n", encoding="utf-8")
    (HERE / "java_order_expected.txt").write_text("\n".join(expected(c)) + "\n", encoding="utf-8")


if __name__ == "__main__":
    main()
