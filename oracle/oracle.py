"""Python/numpy restatement of the IPLS aggregation path -- TEST INFRASTRUCTURE ONLY.

A second, independent restatement next to ipls_oracle.c (the C one is the
fast checker; this one is the readable spec and cross-checks the C one).
Each function cites the reference Java it follows (paths relative to the
reference root, src/main/java/).  Parity status: see oracle/__init__.py.

numpy elementwise ``+`` and ``/`` on float64 are IEEE-754 round-to-nearest,
identical to Java ``double``.  Peer folds are explicit loops over peers,
never ``np.sum`` (pairwise summation would change the association).
"""
from __future__ import annotations

import ctypes
import os
import struct
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SEED = 0x1B5_2026
GOLDEN_GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1

START_ACCUM, START_ZERO, START_FIRST = 0, 1, 2


# --------------------------------------------------------------------------
# partition geometry
# --------------------------------------------------------------------------
def chunk_size(model_size: int, n_partitions: int) -> int:
    """IPLS.java:1019 -- ``(int)(_MODEL_SIZE/_PARTITIONS) + 1``."""
    return int(model_size // n_partitions) + 1


def partition_len(model_size: int, n_partitions: int, i: int) -> int:
    """IPLS.java:1023-1028 (InitializeWeights 1862-1868 uses the same rule)."""
    c = chunk_size(model_size, n_partitions)
    if (i + 1) * c > model_size:
        return model_size - i * c + 1
    return c + 1


def organize_gradients(flat, model_size: int, n_partitions: int) -> dict[int, np.ndarray]:
    """OrganizeGradients, IPLS.java:1018-1040.

    Raises ValueError where Java throws (negative array size / index out of
    bounds)."""
    flat = np.asarray(flat, dtype=np.float64)
    c = chunk_size(model_size, n_partitions)
    out = {}
    for i in range(n_partitions):
        L = partition_len(model_size, n_partitions, i)
        if L < 0:
            raise ValueError("NegativeArraySizeException (IPLS.java:1024)")
        part = np.zeros(L, dtype=np.float64)
        lo = i * c
        hi = min((i + 1) * c, len(flat))
        j = lo
        if hi > lo:
            if hi - lo > L:
                raise ValueError("ArrayIndexOutOfBoundsException (IPLS.java:1030)")
            part[: hi - lo] = flat[lo:hi]
            j = hi
        if j - lo >= L:
            raise ValueError("ArrayIndexOutOfBoundsException (IPLS.java:1033)")
        part[j - lo] = 1.0
        out[i] = part
    return out


# --------------------------------------------------------------------------
# arithmetic
# --------------------------------------------------------------------------
def fold(acc: np.ndarray, g: np.ndarray) -> np.ndarray:
    """Updater.java:115-117: ``Agg[i] = Agg[i] + Gradient[i]`` for i < len(Agg)."""
    L = len(acc)
    acc[:] = acc + np.asarray(g[:L], dtype=np.float64)
    return acc


def reduce(bufs, L: int, start_mode: int = START_ZERO, acc=None) -> np.ndarray:
    """Fixed-order fold of buckets (peer index ascending).

    ZERO : fresh accumulator +0.0 (IPLS.java:1888,1896; reset 1268)
    ACCUM: fold into ``acc`` (Updater arrival order)
    FIRST: start from bucket 0 (Decentralized_Storage_Receiver.java:240-246)
    """
    if start_mode == START_ACCUM:
        out = np.array(acc, dtype=np.float64, copy=True)
        first = 0
    elif start_mode == START_ZERO:
        out = np.zeros(L, dtype=np.float64)
        first = 0
    else:
        out = np.array(bufs[0][:L], dtype=np.float64, copy=True)
        first = 1
    for b in bufs[first:]:
        fold(out, b)
    return out


def aggregate_partition(agg, rep, w, wa):
    """AggregatePartition, IPLS.java:1255-1270 (non-secure): W = AGG + REP;
    WA = W; AGG = REP = 0.0 (in place)."""
    w[:] = agg + rep
    wa[:] = w
    agg[:] = 0.0
    rep[:] = 0.0


def get_parameters_into(arr: np.ndarray, data: bytes) -> None:
    """MyIPFSClass.GetParameters(hash, double[] arr), MyIPFSClass.java:444-455:
    arr[i] = getDouble() for i < data.length/8; at i == arr.length Java throws
    ArrayIndexOutOfBoundsException after the in-range stores (IndexError here)."""
    n = len(data) // 8
    m = min(n, len(arr))
    arr[:m] = np.frombuffer(bytes(data[:8 * m]), dtype=">f8").astype(np.float64)
    if n > len(arr):
        raise IndexError("ArrayIndexOutOfBoundsException (MyIPFSClass.java:451)")


def gradient_buff_len(model_size: int, n_partitions: int) -> int:
    """new double[(int)_MODEL_SIZE/_PARTITIONS + 2], Updater.java:162."""
    return int(np.int32(np.int64(model_size).astype(np.int32) // np.int32(n_partitions))) + 2


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode(): s[0]*31^(n-1) + ... + s[n-1] over the
    UTF-16 code units, wrapping int32 arithmetic (the JDK's published rule)."""
    h = 0
    units = s.encode("utf-16-be")
    for i in range(0, len(units), 2):
        h = (31 * h + ((units[i] << 8) | units[i + 1])) & 0xFFFFFFFF
    return _i32(h)


def java_pair_hash(p: int, peer_id: str) -> int:
    """new org.javatuples.Pair<Integer,String>(p, peer_id).hashCode(): javatuples
    1.2 (pom.xml:66-68) Tuple.hashCode = 31 * 1 + valueList.hashCode(), with
    valueList = Arrays.asList(p, peer_id) and List.hashCode = fold of
    31 * h + e.hashCode() from 1; Integer.hashCode(p) = p."""
    lst = 1
    for e in (p & 0xFFFFFFFF, java_string_hash(peer_id) & 0xFFFFFFFF):
        lst = (31 * lst + e) & 0xFFFFFFFF
    return _i32(31 * 1 + lst)


class _Node:
    """HashMap.Node: hash (the spread hash, a Java int), key, value, next."""
    __slots__ = ("hash", "key", "value", "next", "parent", "left", "right", "prev", "red", "tree")

    def __init__(self, h, key, value, nxt, tree=False):
        self.hash, self.key, self.value, self.next = h, key, value, nxt
        self.parent = self.left = self.right = self.prev = None
        self.red = False
        self.tree = tree                 # a HashMap.TreeNode


class JavaHashMap:
    """java.util.HashMap as JDK 8 keeps it (the pom compiles for 1.8,
    pom.xml:118-122), restated from the published source, node for node:
    the table of bins (each a chain linked by `next`), hash = h ^ (h >>> 16)
    (a Java int), bin = hash & (n - 1); the table is made with 16 bins at the
    first put after construction and doubled (resize) when ++size > 0.75 n,
    or when a put makes a chain 9 long while n < 64 (treeifyBin); a resize
    splits every chain into its lo (hash & oldCap == 0) and hi halves, each
    in chain order, at j and j + oldCap; a new key is appended at its chain's
    tail; remove unlinks.  A chain that reaches 9 at n >= 64 becomes a
    red-black tree of TreeNodes (treeify, putTreeVal, removeTreeNode,
    balanceInsertion / balanceDeletion, rotations, moveRootToFront, split
    and untreeify below): its iteration order is still the `next` chain,
    which those methods rearrange.  Keys whose spread hashes are equal are
    ordered in a tree by System.identityHashCode (javatuples' Pair is not
    Comparable<Pair>, so HashMap.comparableClassFor is null and tieBreakOrder
    decides) -- not reproducible even by Java; ``nondeterministic`` flags it.
    Iteration walks the bins in index order and each chain in link order.

    This simulates the table itself; the library's model (java_hashmap.hpp)
    is a second transliteration of the same JDK source, and the two are
    checked against each other (tests/test_java_order.py)."""
    TREEIFY, UNTREEIFY, MIN_TREEIFY = 8, 6, 64

    def __init__(self):
        self.table = None            # list of bin heads (_Node or None)
        self.size = 0
        self.threshold = 0
        self.nondeterministic = False
        self._nodes = {}             # key -> node (lookup only; never decides an order)

    @staticmethod
    def spread(h: int) -> int:
        h &= 0xFFFFFFFF
        return h ^ (h >> 16)

    @staticmethod
    def _jint(h: int) -> int:
        h = JavaHashMap.spread(h)
        return h - (1 << 32) if h & 0x80000000 else h

    @property
    def tree_bin(self) -> bool:
        return self.table is not None and any(e is not None and e.tree for e in self.table)

    # ---- HashMap ----
    def _resize(self):
        old = self.table
        old_cap = len(old) if old else 0
        if old_cap > 0:
            new_cap, self.threshold = old_cap << 1, self.threshold << 1
        else:
            new_cap, self.threshold = 16, 12
        tab = [None] * new_cap
        self.table = tab
        for j in range(old_cap):
            e = old[j]
            if e is None:
                continue
            old[j] = None
            if e.next is None:
                tab[e.hash & (new_cap - 1)] = e
            elif e.tree:
                self._split(e, tab, j, old_cap)
            else:
                lo_h = lo_t = hi_h = hi_t = None
                while e is not None:
                    nxt = e.next
                    if e.hash & old_cap == 0:
                        if lo_t is None:
                            lo_h = e
                        else:
                            lo_t.next = e
                        lo_t = e
                    else:
                        if hi_t is None:
                            hi_h = e
                        else:
                            hi_t.next = e
                        hi_t = e
                    e = nxt
                if lo_t is not None:
                    lo_t.next = None
                    tab[j] = lo_h
                if hi_t is not None:
                    hi_t.next = None
                    tab[j + old_cap] = hi_h
        return tab

    def put(self, key, h: int, value) -> None:
        if key in self._nodes:                       # an existing mapping: value replaced, nothing moves
            self._nodes[key].value = value
            return
        hh = self._jint(h)
        tab = self.table
        if tab is None:
            tab = self._resize()
        n = len(tab)
        i = hh & (n - 1)
        p = tab[i]
        if p is None:
            tab[i] = self._nodes[key] = _Node(hh, key, value, None)
        elif p.tree:
            self._nodes[key] = self._put_tree_val(p, tab, hh, key, value)
        else:
            bin_count = 0
            while True:
                if p.next is None:
                    p.next = self._nodes[key] = _Node(hh, key, value, None)
                    if bin_count >= self.TREEIFY - 1:
                        self._treeify_bin(tab, hh)       # replaces the chain's nodes (and their index)
                    break
                p = p.next
                bin_count += 1
        self.size += 1
        if self.size > self.threshold:
            self._resize()

    def get(self, key, h: int):
        e = self._nodes.get(key)
        return None if e is None else e.value

    def remove(self, key, h: int) -> bool:
        node = self._nodes.pop(key, None)
        if node is None:
            return False
        tab = self.table
        i = node.hash & (len(tab) - 1)
        if node.tree:
            self._remove_tree_node(node, tab, True)
        elif tab[i] is node:
            tab[i] = node.next
        else:
            p = tab[i]
            while p.next is not node:
                p = p.next
            p.next = node.next
        self.size -= 1
        return True

    def keys(self) -> list:
        out = []
        for e in (self.table or []):
            while e is not None:
                out.append(e.key)
                e = e.next
        return out

    def __len__(self):
        return self.size

    def check_invariants(self) -> None:
        """Structural checks, independent of how the table got here: every
        node sits in its hash's bin, the lookup index and size agree with the
        chains, and every tree bin is a valid red-black tree over exactly its
        chain's nodes, rooted at the bin's first node, ordered by hash --
        TreeNode.checkInvariants (which moveRootToFront asserts) plus the
        red-black rules (black root, no red node with a red child, one black
        height).  Raises AssertionError."""
        seen = 0
        for j, e in enumerate(self.table or []):
            if e is None:
                continue
            chain, prev = [], None
            while e is not None:
                assert e.hash & (len(self.table) - 1) == j, "node outside its hash's bin"
                assert self._nodes.get(e.key) is e, "lookup index is stale"
                assert e.tree == self.table[j].tree, "tree and plain nodes mixed in one bin"
                if e.tree:
                    assert e.prev is prev, "prev link broken"
                chain.append(e)
                prev, e = e, e.next
            seen += len(chain)
            root = chain[0]
            if not root.tree:
                continue
            assert root.parent is None and not root.red, "bin head is not a black root"
            members = set()

            def walk(t, lo, hi):                     # -> black height; lo/hi bound the hashes
                if t is None:
                    return 1
                assert id(t) not in members, "cycle in tree"
                members.add(id(t))
                assert (lo is None or t.hash >= lo) and (hi is None or t.hash <= hi), "tree not ordered by hash"
                for c in (t.left, t.right):
                    if c is not None:
                        assert c.parent is t, "parent link broken"
                        assert not (t.red and c.red), "red node with a red child"
                bl = walk(t.left, lo, t.hash)
                br = walk(t.right, t.hash, hi)
                assert bl == br, "unequal black heights"
                return bl + (0 if t.red else 1)

            walk(root, None, None)
            assert members == {id(x) for x in chain}, "tree and chain hold different nodes"
        assert seen == self.size == len(self._nodes), "size / index / chains disagree"

    def _treeify_bin(self, tab, hh):
        n = len(tab)
        if n < self.MIN_TREEIFY:
            self._resize()
            return
        index = (n - 1) & hh
        e = tab[index]
        hd = tl = None
        while e is not None:                         # replacementTreeNode, in chain order
            p = _Node(e.hash, e.key, e.value, None, tree=True)
            self._nodes[p.key] = p
            if tl is None:
                hd = p
            else:
                p.prev = tl
                tl.next = p
            tl = p
            e = e.next
        tab[index] = hd
        if hd is not None:
            self._treeify(hd, tab)

    # ---- TreeNode ----
    @staticmethod
    def _root(x):
        while x.parent is not None:
            x = x.parent
        return x

    @staticmethod
    def _move_root_to_front(tab, root):
        if root is None or not tab:
            return
        index = (len(tab) - 1) & root.hash
        first = tab[index]
        if root is not first:
            tab[index] = root
            rp, rn = root.prev, root.next
            if rn is not None:
                rn.prev = rp
            if rp is not None:
                rp.next = rn
            if first is not None:
                first.prev = root
            root.next = first
            root.prev = None

    def _dir(self, h, ph):
        if ph > h:
            return -1
        if ph < h:
            return 1
        self.nondeterministic = True                 # tieBreakOrder: System.identityHashCode
        return -1

    def _treeify(self, head, tab):
        root = None
        x = head
        while x is not None:
            nxt = x.next
            x.left = x.right = None
            if root is None:
                x.parent = None
                x.red = False
                root = x
            else:
                p = root
                while True:
                    d = self._dir(x.hash, p.hash)
                    xp = p
                    p = p.left if d <= 0 else p.right
                    if p is None:
                        x.parent = xp
                        if d <= 0:
                            xp.left = x
                        else:
                            xp.right = x
                        root = self._balance_insertion(root, x)
                        break
            x = nxt
        self._move_root_to_front(tab, root)

    def _untreeify(self, first):
        hd = tl = None
        q = first
        while q is not None:                         # replacementNode, in chain order
            p = _Node(q.hash, q.key, q.value, None)
            self._nodes[p.key] = p
            if tl is None:
                hd = p
            else:
                tl.next = p
            tl = p
            q = q.next
        return hd

    def _put_tree_val(self, first, tab, hh, key, value):
        root = self._root(first) if first.parent is not None else first
        p = root
        while True:
            d = self._dir(hh, p.hash)
            xp = p
            p = p.left if d <= 0 else p.right
            if p is None:
                xpn = xp.next
                x = _Node(hh, key, value, xpn, tree=True)
                if d <= 0:
                    xp.left = x
                else:
                    xp.right = x
                xp.next = x
                x.parent = x.prev = xp
                if xpn is not None:
                    xpn.prev = x
                self._move_root_to_front(tab, self._balance_insertion(root, x))
                return x

    def _remove_tree_node(self, node, tab, movable):
        n = len(tab)
        index = (n - 1) & node.hash
        first = root = tab[index]
        succ, pred = node.next, node.prev
        if pred is None:
            tab[index] = first = succ
        else:
            pred.next = succ
        if succ is not None:
            succ.prev = pred
        if first is None:
            return
        if root.parent is not None:
            root = self._root(root)
        if root is None or (movable and (root.right is None or root.left is None or root.left.left is None)):
            tab[index] = self._untreeify(first)      # too small
            return
        p, pl, pr = node, node.left, node.right
        if pl is not None and pr is not None:
            s = pr
            while s.left is not None:                # successor
                s = s.left
            s.red, p.red = p.red, s.red              # swap colours
            sr, pp = s.right, p.parent
            if s is pr:
                p.parent = s
                s.right = p
            else:
                sp = s.parent
                p.parent = sp
                if sp is not None:
                    if s is sp.left:
                        sp.left = p
                    else:
                        sp.right = p
                s.right = pr
                if pr is not None:
                    pr.parent = s
            p.left = None
            p.right = sr
            if sr is not None:
                sr.parent = p
            s.left = pl
            if pl is not None:
                pl.parent = s
            s.parent = pp
            if pp is None:
                root = s
            elif p is pp.left:
                pp.left = s
            else:
                pp.right = s
            replacement = sr if sr is not None else p
        elif pl is not None:
            replacement = pl
        elif pr is not None:
            replacement = pr
        else:
            replacement = p
        if replacement is not p:
            pp = replacement.parent = p.parent
            if pp is None:
                root = replacement
            elif p is pp.left:
                pp.left = replacement
            else:
                pp.right = replacement
            p.left = p.right = p.parent = None
        r = root if p.red else self._balance_deletion(root, replacement)
        if replacement is p:                         # detach
            pp = p.parent
            p.parent = None
            if pp is not None:
                if p is pp.left:
                    pp.left = None
                elif p is pp.right:
                    pp.right = None
        if movable:
            self._move_root_to_front(tab, r)

    def _split(self, b, tab, index, bit):
        lo_h = lo_t = hi_h = hi_t = None
        lc = hc = 0
        e = b
        while e is not None:
            nxt = e.next
            e.next = None
            if e.hash & bit == 0:
                e.prev = lo_t
                if lo_t is None:
                    lo_h = e
                else:
                    lo_t.next = e
                lo_t = e
                lc += 1
            else:
                e.prev = hi_t
                if hi_t is None:
                    hi_h = e
                else:
                    hi_t.next = e
                hi_t = e
                hc += 1
            e = nxt
        if lo_h is not None:
            if lc <= self.UNTREEIFY:
                tab[index] = self._untreeify(lo_h)
            else:
                tab[index] = lo_h
                if hi_h is not None:
                    self._treeify(lo_h, tab)
        if hi_h is not None:
            if hc <= self.UNTREEIFY:
                tab[index + bit] = self._untreeify(hi_h)
            else:
                tab[index + bit] = hi_h
                if lo_h is not None:
                    self._treeify(hi_h, tab)

    @staticmethod
    def _rotate_left(root, p):
        if p is not None and p.right is not None:
            r = p.right
            rl = p.right = r.left
            if rl is not None:
                rl.parent = p
            pp = r.parent = p.parent
            if pp is None:
                root = r
                r.red = False
            elif pp.left is p:
                pp.left = r
            else:
                pp.right = r
            r.left = p
            p.parent = r
        return root

    @staticmethod
    def _rotate_right(root, p):
        if p is not None and p.left is not None:
            l = p.left
            lr = p.left = l.right
            if lr is not None:
                lr.parent = p
            pp = l.parent = p.parent
            if pp is None:
                root = l
                l.red = False
            elif pp.right is p:
                pp.right = l
            else:
                pp.left = l
            l.right = p
            p.parent = l
        return root

    def _balance_insertion(self, root, x):
        x.red = True
        while True:
            xp = x.parent
            if xp is None:
                x.red = False
                return x
            xpp = xp.parent
            if not xp.red or xpp is None:
                return root
            xppl = xpp.left
            if xp is xppl:
                xppr = xpp.right
                if xppr is not None and xppr.red:
                    xppr.red = False
                    xp.red = False
                    xpp.red = True
                    x = xpp
                else:
                    if x is xp.right:
                        x = xp
                        root = self._rotate_left(root, x)
                        xp = x.parent
                        xpp = None if xp is None else xp.parent
                    if xp is not None:
                        xp.red = False
                        if xpp is not None:
                            xpp.red = True
                            root = self._rotate_right(root, xpp)
            else:
                if xppl is not None and xppl.red:
                    xppl.red = False
                    xp.red = False
                    xpp.red = True
                    x = xpp
                else:
                    if x is xp.left:
                        x = xp
                        root = self._rotate_right(root, x)
                        xp = x.parent
                        xpp = None if xp is None else xp.parent
                    if xp is not None:
                        xp.red = False
                        if xpp is not None:
                            xpp.red = True
                            root = self._rotate_left(root, xpp)

    def _balance_deletion(self, root, x):
        while True:
            if x is None or x is root:
                return root
            xp = x.parent
            if xp is None:
                x.red = False
                return x
            if x.red:
                x.red = False
                return root
            xpl = xp.left
            if xpl is x:
                xpr = xp.right
                if xpr is not None and xpr.red:
                    xpr.red = False
                    xp.red = True
                    root = self._rotate_left(root, xp)
                    xp = x.parent
                    xpr = None if xp is None else xp.right
                if xpr is None:
                    x = xp
                else:
                    sl, sr = xpr.left, xpr.right
                    if (sr is None or not sr.red) and (sl is None or not sl.red):
                        xpr.red = True
                        x = xp
                    else:
                        if sr is None or not sr.red:
                            if sl is not None:
                                sl.red = False
                            xpr.red = True
                            root = self._rotate_right(root, xpr)
                            xp = x.parent
                            xpr = None if xp is None else xp.right
                        if xpr is not None:
                            xpr.red = False if xp is None else xp.red
                            sr = xpr.right
                            if sr is not None:
                                sr.red = False
                        if xp is not None:
                            xp.red = False
                            root = self._rotate_left(root, xp)
                        x = root
            else:
                if xpl is not None and xpl.red:
                    xpl.red = False
                    xp.red = True
                    root = self._rotate_right(root, xp)
                    xp = x.parent
                    xpl = None if xp is None else xp.left
                if xpl is None:
                    x = xp
                else:
                    sl, sr = xpl.left, xpl.right
                    if (sl is None or not sl.red) and (sr is None or not sr.red):
                        xpl.red = True
                        x = xp
                    else:
                        if sl is None or not sl.red:
                            if sr is not None:
                                sr.red = False
                            xpl.red = True
                            root = self._rotate_left(root, xpl)
                            xp = x.parent
                            xpl = None if xp is None else xp.left
                        if xpl is not None:
                            xpl.red = False if xp is None else xp.red
                            sl = xpl.left
                            if sl is not None:
                                sl.red = False
                        if xp is not None:
                            xp.red = False
                            root = self._rotate_right(root, xp)
                        x = root


class ReplicaStore:
    """PeerData.Other_Replica_Gradients + Other_Replica_Gradients_Received
    (PeerData.java:140-141): one JavaHashMap keyed (p, aggregator) with the
    Pair hashCode of (p, peer ID); value [array, received]."""

    def __init__(self):
        self.map = JavaHashMap()
        self.hashes = {}

    def __len__(self):
        return len(self.map)


def index_key_hash(p: int, aggregator: int) -> int:
    """The key hash of an aggregator known only by its index: the peer ID is
    Integer.toString(aggregator) (ipls_agg_other_replica without a hash)."""
    return java_pair_hash(p, str(aggregator))


def other_replica_add(store: ReplicaStore, partition: int, aggregator, g: np.ndarray,
                      key_hash: int | None = None) -> None:
    """Download_Scheduler.java:254-266: the first download of (p, a) becomes the
    stored array (Other_Replica_Gradients.put(key, GetParameters(Hash)) -> new
    double[n]); later ones fold into it for j < len(g) (IndexError where Java
    overruns the stored array) and bump Other_Replica_Gradients_Received."""
    key = (partition, aggregator)
    h = index_key_hash(partition, aggregator) if key_hash is None else key_hash
    cur = store.map.get(key, h)
    if cur is None:
        store.map.put(key, h, [np.array(g, dtype=np.float64, copy=True), 1])
        store.hashes[key] = h
        return
    arr = cur[0]
    if len(g) > len(arr):
        raise IndexError("ArrayIndexOutOfBoundsException (Download_Scheduler.java:257)")
    arr[:len(g)] = arr[:len(g)] + g
    cur[1] += 1


def other_replica_drop(store: ReplicaStore, partition: int, aggregator) -> bool:
    """Other_Replica_Gradients.remove(key) and Other_Replica_Gradients_Received
    .remove(key) (Download_Scheduler.java:215-217, 329-332, 438-440)."""
    key = (partition, aggregator)
    if key not in store.hashes:
        return False
    store.map.remove(key, store.hashes.pop(key))
    return True


def collect_replicas(rep: list, store: ReplicaStore, participants: list | None = None) -> int:
    """IPLS.Collect_Replicas, IPLS.java:1217-1241: for the keys of
    new ArrayList<>(Other_Replica_Gradients.keySet()) in that order,
    REP[p][j] = REP[p][j] + Other[(p, a)][j] for j < len(Other); then the
    store is a new HashMap.  Participants (IPLS.java:1229-1234) is updated
    inside the j loop: put(p, received) if absent, else += received, once per
    ELEMENT -- so each key adds received * len(Other), in Java int
    arithmetic (wrapping at 2^32); an empty array adds nothing."""
    n = 0
    for key in store.map.keys():
        p = key[0]
        arr, received = store.map.get(key, store.hashes[key])
        rep[p][:len(arr)] = rep[p][:len(arr)] + arr
        if participants is not None:
            participants[p] = _i32(participants[p] + received * len(arr))   # received, len(arr) times
        n += 1
    store.map = JavaHashMap()
    store.hashes = {}
    return n


def storage_merge(gradients: list) -> np.ndarray:
    """Decentralized_Storage_Receiver.java:239-256: Aggregation = the first
    file's doubles; Aggregation[j] += g[j] for j < g.length, file by file
    (IndexError where Java overruns the first array)."""
    agg = np.array(gradients[0], dtype=np.float64, copy=True)
    for g in gradients[1:]:
        if len(g) > len(agg):
            raise IndexError("ArrayIndexOutOfBoundsException (Decentralized_Storage_Receiver.java:245)")
        agg[:len(g)] = agg[:len(g)] + g
    return agg


def promote_future(agg: np.ndarray, fut: np.ndarray) -> None:
    """IPLS.java:1557-1562 (Update_Client_WaitAck_List): for j < L,
    Aggregated_Gradients[p][j] = from_future[p].get(j); from_future[p].set(j, 0.0)."""
    agg[:] = fut
    fut[:] = 0.0


def divide(w: np.ndarray, secure: bool = False) -> np.ndarray:
    """GetPartitions, IPLS.java:1159-1174, one partition -> len(w)-1 values."""
    w = np.asarray(w, dtype=np.float64)
    cnt = w[-1]
    body = w[:-1]
    if cnt == 0.0:                       # also true for -0.0, as in Java
        return body.copy()
    if secure:
        return body / (10.0 ** 12 * cnt)  # Math.pow(10,12)*W[last]
    return body / cnt


def get_partitions(weights: list[np.ndarray], secure: bool = False) -> np.ndarray:
    """IPLS.java:1159-1174: concatenate the per-partition divides."""
    return np.concatenate([divide(w, secure) for w in weights]) if weights else np.zeros(0)


def encode_secure(x) -> np.ndarray:
    """Middleware.Encode, Middleware.java:196-210."""
    x = np.asarray(x, dtype=np.float64)
    out = x * 10.0 ** 12
    out = np.where(x > 10.0, 10 * 10.0 ** 12, out)
    out = np.where(x < -10.0, -10 * 10.0 ** 12, out)
    return out


def blend(w, g, a: float, b: float) -> np.ndarray:
    """W[i] = a*W[i] + b*G[i]: Updater.java:58 (a=0.75, b=1) and 67 (a=0.6, b=1-a)."""
    w = np.asarray(w, dtype=np.float64)
    g = np.asarray(g[:len(w)], dtype=np.float64)
    return (a * w) + (b * g)


def scale(w, c: float) -> np.ndarray:
    """Updater.java:198: Aggregated[i] = 0.25*Weights[i]."""
    return c * np.asarray(w, dtype=np.float64)


# --------------------------------------------------------------------------
# byte codecs
# --------------------------------------------------------------------------
def be_decode(data: bytes) -> np.ndarray:
    """GetParameters, MyIPFSClass.java:444-455: ``len/8`` BE doubles."""
    n = len(data) // 8
    return np.frombuffer(bytes(data[: 8 * n]), dtype=">f8").astype(np.float64)


def be_encode(x) -> bytes:
    """update_file(double[]), MyIPFSClass.java:105-116 (putDouble keeps raw NaN bits)."""
    return np.asarray(x, dtype=np.float64).astype(">f8").tobytes()


def be_encode_canonical(x) -> bytes:
    """Middleware.Serialize, Middleware.java:164-170 (writeDouble ->
    doubleToLongBits: every NaN becomes 0x7ff8000000000000)."""
    a = np.asarray(x, dtype=np.float64).copy()
    bits = a.view(np.uint64)
    bits[np.isnan(a)] = np.uint64(0x7FF8000000000000)
    return bits.view(np.float64).astype(">f8").tobytes()


def frame_encode(g, a: int, b: int, pid: int, origin: bytes) -> bytes:
    """Marshall_Packet(double[],origin,partition,iteration,pid) before base64,
    MyIPFSClass.java:990-1017."""
    g = np.zeros(0) if g is None else np.asarray(g, dtype=np.float64)
    head = struct.pack(">hiii", pid, len(g), a, b)
    return head + be_encode(g) + bytes(origin)


def frame_decode(frame: bytes):
    """GET_GRADIENTS / Get_Replica_Model, MyIPFSClass.java:1437-1481 (the pid
    short is read first by ThreadReceiver.process, IPLS.java:405).  Returns
    (pid, n, a, b, gradients-or-None, origin)."""
    if len(frame) < 14:
        raise ValueError("BufferUnderflowException")
    pid, n, a, b = struct.unpack(">hiii", frame[:14])
    if n < 0 or 14 + 8 * n > len(frame):
        raise ValueError("BufferUnderflowException")
    g = be_decode(frame[14:14 + 8 * n]) if n else None   # arr_len == 0 -> null (1449-1451)
    return pid, n, a, b, g, bytes(frame[14 + 8 * n:])


# --------------------------------------------------------------------------
# synthetic workload and checksum
# --------------------------------------------------------------------------
def splitmix64(v: np.ndarray) -> np.ndarray:
    v = np.asarray(v, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = v + np.uint64(GOLDEN_GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_bucket(L: int, p: int, k: int, seed: int = SEED) -> np.ndarray:
    """x_i = (2u-1)*1e-2, u = (splitmix64(seed ^ p<<40 ^ k<<32 ^ i) >> 11) * 2^-53;
    element L-1 is the count slot 1.0."""
    i = np.arange(L, dtype=np.uint64)
    key = np.uint64(seed) ^ np.uint64((p << 40) & M64) ^ np.uint64((k << 32) & M64) ^ i
    u = (splitmix64(key) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    t = 2.0 * u
    t = t - 1.0
    x = t * 1e-2
    if L:
        x[L - 1] = 1.0
    return x


def checksum(x) -> int:
    """sum_i splitmix64(bits(x_i) + i*0x9E3779B97F4A7C15) mod 2^64 (order independent)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    i = np.arange(len(x), dtype=np.uint64)
    with np.errstate(over="ignore"):
        terms = splitmix64(x.view(np.uint64) + i * np.uint64(GOLDEN_GAMMA))
    return int(terms.sum(dtype=np.uint64))


# --------------------------------------------------------------------------
# ETHModel (reference fixture) -- a Java-serialised
# org.nd4j.shade.guava.primitives.Doubles$DoubleArrayAsList.  Parsed by hand;
# nothing in the file is executed.
# --------------------------------------------------------------------------
def parse_ethmodel(data: bytes) -> np.ndarray:
    def u16(o):
        return struct.unpack_from(">H", data, o)[0]

    o = 0
    if data[:4] != b"\xac\xed\x00\x05":
        raise ValueError("not a Java serialization stream")
    o = 4
    if data[o] != 0x73 or data[o + 1] != 0x72:          # TC_OBJECT TC_CLASSDESC
        raise ValueError("unexpected stream layout")
    o += 2
    n = u16(o); o += 2
    cname = data[o:o + n].decode(); o += n
    if not cname.endswith("Doubles$DoubleArrayAsList"):
        raise ValueError(f"unexpected class {cname}")
    o += 8 + 1                                          # serialVersionUID, flags
    nf = u16(o); o += 2
    prims = []
    for _ in range(nf):
        tc = chr(data[o]); o += 1
        ln = u16(o); o += 2
        fname = data[o:o + ln].decode(); o += ln
        if tc in "[L":
            o += 1                                      # TC_STRING
            ln = u16(o); o += 2 + ln
        else:
            prims.append((tc, fname))
    if data[o] != 0x78 or data[o + 1] != 0x70:          # TC_ENDBLOCKDATA, TC_NULL super
        raise ValueError("unexpected class annotation")
    o += 2
    vals = {}
    for tc, fname in prims:
        if tc != "I":
            raise ValueError("unexpected primitive field")
        vals[fname] = struct.unpack_from(">i", data, o)[0]; o += 4
    if data[o] != 0x75 or data[o + 1] != 0x72:          # TC_ARRAY TC_CLASSDESC
        raise ValueError("expected [D array")
    o += 2
    n = u16(o); o += 2
    if data[o:o + n] != b"[D":
        raise ValueError("expected [D")
    o += n + 8 + 1
    if u16(o) != 0 or data[o + 2] != 0x78 or data[o + 3] != 0x70:
        raise ValueError("unexpected [D descriptor")
    o += 4
    count = struct.unpack_from(">i", data, o)[0]; o += 4
    arr = np.frombuffer(data[o:o + 8 * count], dtype=">f8").astype(np.float64)
    start, end = vals.get("start", 0), vals.get("end", count)
    return arr[start:end].copy()


# --------------------------------------------------------------------------
# C oracle (ctypes)
# --------------------------------------------------------------------------
_C = None


def c_oracle():
    """Load oracle/build/libipls_oracle.so (built by oracle/Makefile)."""
    global _C
    if _C is None:
        path = HERE / "build" / "libipls_oracle.so"
        if not path.exists():
            import subprocess
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
        lib = ctypes.CDLL(str(path))
        D = ctypes.POINTER(ctypes.c_double)
        U8 = ctypes.POINTER(ctypes.c_uint8)
        i64, i32, u64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64
        lib.ipls_oracle_chunk.restype = i64
        lib.ipls_oracle_chunk.argtypes = [i64, i32]
        lib.ipls_oracle_partition_len.restype = i64
        lib.ipls_oracle_partition_len.argtypes = [i64, i32, i32]
        lib.ipls_oracle_organize.restype = ctypes.c_int
        lib.ipls_oracle_organize.argtypes = [D, i64, i64, i32, i32, D]
        lib.ipls_oracle_reduce.argtypes = [D, ctypes.POINTER(D), ctypes.c_int, i64, ctypes.c_int]
        lib.ipls_oracle_divide.argtypes = [D, i64, ctypes.c_int, D]
        lib.ipls_oracle_be_decode.argtypes = [U8, i64, D]
        lib.ipls_oracle_be_encode.argtypes = [D, i64, U8]
        lib.ipls_oracle_be_encode_canonical.argtypes = [D, i64, U8]
        lib.ipls_oracle_synth_fill.argtypes = [D, i64, u64, i32, i32]
        lib.ipls_oracle_checksum.restype = u64
        lib.ipls_oracle_checksum.argtypes = [D, i64]
        lib.ipls_oracle_synth_sum_checksum.restype = u64
        lib.ipls_oracle_synth_sum_checksum.argtypes = [u64, i32, i32, i64]
        lib.ipls_oracle_synth_avg_checksum.restype = u64
        lib.ipls_oracle_synth_avg_checksum.argtypes = [u64, i32, i32, i64, i32]
        lib.ipls_oracle_synth_replica_checksum.restype = u64
        lib.ipls_oracle_synth_replica_checksum.argtypes = [u64, i32, i32, i32, i64]
        lib.ipls_oracle_updater_loop.argtypes = [D, ctypes.POINTER(U8), ctypes.c_int, i64, D]
        lib.ipls_oracle_updater_loop_parts.restype = ctypes.c_int
        lib.ipls_oracle_updater_loop_parts.argtypes = [ctypes.c_int, ctypes.POINTER(U8), ctypes.c_int, i64, D]
        lib.ipls_oracle_synth_be_buckets.argtypes = [ctypes.POINTER(U8), ctypes.c_int, ctypes.c_int, i64, u64]
        lib.ipls_oracle_updater_loop_partitions.restype = ctypes.c_int
        lib.ipls_oracle_updater_loop_partitions.argtypes = [ctypes.c_int, ctypes.POINTER(U8), ctypes.c_int, i64,
                                                            ctypes.c_int, ctypes.c_int, D]
        _C = lib
    return _C


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def c_reduce(bufs, L: int, start_mode: int = START_ZERO, acc=None) -> np.ndarray:
    lib = c_oracle()
    out = np.zeros(L) if acc is None else np.array(acc, dtype=np.float64, copy=True)
    bufs = [np.ascontiguousarray(b, dtype=np.float64) for b in bufs]
    arr = (ctypes.POINTER(ctypes.c_double) * max(1, len(bufs)))(*[_dp(b) for b in bufs])
    lib.ipls_oracle_reduce(_dp(out), arr, len(bufs), L, start_mode)
    return out


def c_synth_bucket(L: int, p: int, k: int, seed: int = SEED) -> np.ndarray:
    out = np.empty(L)
    c_oracle().ipls_oracle_synth_fill(_dp(out), L, seed, p, k)
    return out


def c_synth_sum_checksum(L: int, p: int, k: int, seed: int = SEED) -> int:
    return int(c_oracle().ipls_oracle_synth_sum_checksum(seed, p, k, L))


def c_synth_replica_checksum(L: int, p: int, k: int, k_own: int, seed: int = SEED) -> int:
    """W = AGG(peers < k_own) + (+0.0 + partial(peers >= k_own)) (IPLS.java:1256, Updater.java:40-44)."""
    return int(c_oracle().ipls_oracle_synth_replica_checksum(seed, p, k, k_own, L))


def c_synth_avg_checksum(L: int, p: int, k: int, secure: bool = False, seed: int = SEED) -> int:
    return int(c_oracle().ipls_oracle_synth_avg_checksum(seed, p, k, L, int(secure)))


def c_checksum(x) -> int:
    x = np.ascontiguousarray(x, dtype=np.float64)
    return int(c_oracle().ipls_oracle_checksum(_dp(x), len(x)))


def c_divide(w, secure=False) -> np.ndarray:
    w = np.ascontiguousarray(w, dtype=np.float64)
    out = np.empty(max(0, len(w) - 1))
    c_oracle().ipls_oracle_divide(_dp(w), len(w), int(secure), _dp(out))
    return out


def c_updater_loop(be_bufs, L: int) -> np.ndarray:
    """CPU baseline: the reference's single-thread Updater decode+fold loop."""
    lib = c_oracle()
    U8 = ctypes.POINTER(ctypes.c_uint8)
    agg = np.zeros(L)
    scratch = np.empty(L)
    arr = (U8 * len(be_bufs))(*[b.ctypes.data_as(U8) for b in be_bufs])
    lib.ipls_oracle_updater_loop(_dp(agg), arr, len(be_bufs), L, _dp(scratch))
    return agg


def c_updater_loop_parts(be_bufs, L: int, n_parts: int):
    """CPU baseline, N threads: n_parts partitions folded in parallel (each
    one the single-thread Updater loop).  Returns (partition 0 sum, threads)."""
    lib = c_oracle()
    U8 = ctypes.POINTER(ctypes.c_uint8)
    agg0 = np.zeros(L)
    arr = (U8 * len(be_bufs))(*[b.ctypes.data_as(U8) for b in be_bufs])
    t = lib.ipls_oracle_updater_loop_parts(n_parts, arr, len(be_bufs), L, _dp(agg0))
    return agg0, t


def c_synth_be_buckets(n_parts: int, k: int, L: int, seed: int = SEED) -> list[np.ndarray]:
    """BE byte images of the synthetic buckets (p, j), p < n_parts, j < k
    (partition-major), generated in C with OpenMP."""
    U8 = ctypes.POINTER(ctypes.c_uint8)
    bufs = [np.empty(8 * L, dtype=np.uint8) for _ in range(n_parts * k)]
    arr = (U8 * len(bufs))(*[b.ctypes.data_as(U8) for b in bufs])
    c_oracle().ipls_oracle_synth_be_buckets(arr, n_parts, k, L, seed)
    return bufs


def c_updater_loop_partitions(be_bufs, n_parts: int, k: int, L: int, passes: int, threads: int = 0):
    """CPU baseline, N threads: n_parts partitions, each with its own k BE
    buckets (be_bufs partition-major), one thread per partition running the
    single-thread Updater loop, `passes` times.  Returns (partition 0 sum,
    threads used)."""
    lib = c_oracle()
    U8 = ctypes.POINTER(ctypes.c_uint8)
    agg0 = np.zeros(L)
    arr = (U8 * len(be_bufs))(*[b.ctypes.data_as(U8) for b in be_bufs])
    t = lib.ipls_oracle_updater_loop_partitions(n_parts, arr, k, L, passes, threads, _dp(agg0))
    return agg0, t


def ethmodel_path() -> Path | None:
    p = Path(os.environ.get("IPLS_REFERENCE", "/root/reference")) / "MNIST_Partitioned_Dataset" / "ETHModel"
    return p if p.exists() else None


# --------------------------------------------------------------------------
# java.util.Base64 URL decoder (JDK 8+, RFC 4648 §5 alphabet, not MIME).
# The reference decodes every pubsub message twice with
# Base64.getUrlDecoder().decode (IPLS.java:855-859 + 399, Utils.java:14-15);
# the JDK is absent here, so its published decoding rules are restated:
#   * alphabet A-Z a-z 0-9 - _ ; any other byte -> IllegalArgumentException
#   * '=' padding is optional; if present it must complete the 4-char unit
#     ("xx==" or "xxx=") and nothing may follow it
#   * a dangling single char in the last unit is an error
#   * unused low bits of a partial last unit are ignored
# Encoding (Base64.getUrlEncoder(), MyIPFSClass.java:986,1015) pads with '='.
# --------------------------------------------------------------------------
_B64URL = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
_B64VAL = {c: i for i, c in enumerate(_B64URL)}


class JavaIllegalArgument(ValueError):
    pass


def java_b64url_encode(data: bytes) -> bytes:
    import base64
    return base64.urlsafe_b64encode(bytes(data))


def java_b64url_decode(src: bytes) -> bytes:
    src = bytes(src)
    out = bytearray()
    bits = 0
    shiftto = 18
    sp, sl = 0, len(src)
    while sp < sl:
        b = src[sp]
        sp += 1
        if b == ord("="):
            # "=" shiftto==18 unnecessary padding; "x=" shiftto==12; "xx=" needs a 2nd '='
            if (shiftto == 6 and (sp == sl or src[sp] != ord("="))) or shiftto == 18:
                raise JavaIllegalArgument("Input byte array has wrong 4-byte ending unit")
            if shiftto == 6:
                sp += 1
            break
        v = _B64VAL.get(b)
        if v is None:
            raise JavaIllegalArgument(f"Illegal base64 character {b:#x}")
        bits |= v << shiftto
        shiftto -= 6
        if shiftto < 0:
            out += bytes([(bits >> 16) & 0xFF, (bits >> 8) & 0xFF, bits & 0xFF])
            shiftto = 18
            bits = 0
    if shiftto == 6:
        out.append((bits >> 16) & 0xFF)
    elif shiftto == 0:
        out += bytes([(bits >> 16) & 0xFF, (bits >> 8) & 0xFF])
    elif shiftto == 12:
        raise JavaIllegalArgument("Last unit does not have enough valid bits")
    if sp < sl:
        raise JavaIllegalArgument("Input byte array has incorrect ending byte")
    return bytes(out)


def pubsub_message(frame: bytes) -> bytes:
    """The 'data' text a receiver sees for a Marshall_Packet frame: the
    packet is base64url'd by Marshall_Packet and decoded twice on receipt."""
    return java_b64url_encode(java_b64url_encode(frame))


def pubsub_decode(msg: bytes) -> bytes:
    """ThreadReceiver.run + process (IPLS.java:855-859, 399)."""
    return java_b64url_decode(java_b64url_decode(msg))
