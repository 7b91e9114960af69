// java_hashmap.hpp -- the key order of PeerData.Other_Replica_Gradients.
//
// The reference keeps the downloads of other aggregators' buckets in a
// java.util.HashMap<Pair<Integer,String>, double[]> (PeerData.java:140) and
// Collect_Replicas folds them in the order of
// `new ArrayList<>(Other_Replica_Gradients.keySet())` (IPLS.java:1218-1227).
// Floating-point addition does not associate, so that order decides the bits
// of Replicas_Gradients[p] whenever a partition has two or more stored arrays.
// This header restates the order JDK 8's HashMap gives (the pom compiles for
// 1.8, pom.xml:118-122; the algorithm is unchanged in later JDKs), from its
// published source:
//
//   hash(key)  = h ^ (h >>> 16),  h = key.hashCode()
//   bin        = hash & (capacity - 1)
//   capacity   = 16 at the first put after `new HashMap<>()`; doubled when
//                ++size > 0.75 * capacity, and when a put makes one bin's
//                chain 9 long while capacity < 64 (treeifyBin -> resize)
//   a new key is appended at the tail of its bin's chain; a resize splits
//   every chain into its lo / hi halves in chain order; remove unlinks.
//
// Chains only ever append, and resizes keep the relative order of the keys
// that stay together, so while no bin is a tree a key's position in keySet()
// is (bin under the current capacity, insertion order within the bin).  A bin
// that reaches 9 keys at capacity >= 64 becomes a red-black tree whose chain
// order follows the tree's insertions, rotations and removals; the class
// below transliterates all of it (JavaHashOrder), so both cases are exact --
// except keys with equal spread hashes inside a tree, which Java itself
// orders by System.identityHashCode (flagged, see the class comment).
//
// key.hashCode() is javatuples 1.2's Tuple.hashCode (pom.xml:66-68):
// 31 * 1 + Arrays.asList(p, id).hashCode() = 31 + (31 * (31 + p) + id.hashCode()),
// with String.hashCode() = s[0]*31^(n-1) + ... + s[n-1] over UTF-16 units,
// all in wrapping 32-bit arithmetic (java_pair_hash below).
//
// Host-only code, no HIP: the C-ABI front keeps one such model per handle
// (the map is one per JVM across all partitions, so its capacity is too).
#pragma once

#include <algorithm>
#include <cstdint>
#include <map>
#include <utility>
#include <vector>

namespace ipls {

// String.hashCode over the UTF-16 units of a UTF-8 byte string.  Returns
// false for malformed UTF-8 (the caller's bytes are not a Java String's).
inline bool java_string_hash(const uint8_t* s, int64_t n, int32_t* out) {
  uint32_t h = 0;
  auto unit = [&h](uint32_t u) { h = 31u * h + u; };
  for (int64_t i = 0; i < n;) {
    const uint32_t c = s[i];
    uint32_t cp, need;
    if (c < 0x80) { cp = c; need = 0; }
    else if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; need = 1; }
    else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; need = 2; }
    else if ((c & 0xF8) == 0xF0) { cp = c & 0x07; need = 3; }
    else return false;
    if (i + 1 + (int64_t)need > n) return false;
    for (uint32_t k = 1; k <= need; ++k) {
      if ((s[i + k] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (s[i + k] & 0x3F);
    }
    static const uint32_t kMin[4] = {0, 0x80, 0x800, 0x10000};
    if (cp < kMin[need] || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;   // overlong / surrogate
    if (cp >= 0x10000) {   // a supplementary character is two UTF-16 units
      cp -= 0x10000;
      unit(0xD800 + (cp >> 10));
      unit(0xDC00 + (cp & 0x3FF));
    } else {
      unit(cp);
    }
    i += 1 + need;
  }
  *out = (int32_t)h;
  return true;
}

// new org.javatuples.Pair<Integer,String>(p, id).hashCode()
inline int32_t java_pair_hash_of(int32_t p, int32_t id_hash) {
  const uint32_t list = 31u * (31u * 1u + (uint32_t)p) + (uint32_t)id_hash;   // Arrays.asList(p, id).hashCode()
  return (int32_t)(31u * 1u + list);                                          // Tuple.hashCode
}

// The aggregator ID a bare index stands for: Integer.toString(a) (the rule of
// ipls_agg_other_replica without a key hash).
inline int32_t java_index_id_hash(int32_t a) {
  char buf[16];
  int n = 0;
  uint32_t u = a < 0 ? 0u - (uint32_t)a : (uint32_t)a;
  do { buf[n++] = char('0' + u % 10); u /= 10; } while (u);
  if (a < 0) buf[n++] = '-';
  uint32_t h = 0;
  while (n) h = 31u * h + (uint8_t)buf[--n];
  return (int32_t)h;
}

// A transliteration of JDK 8 java.util.HashMap's table and TreeNode code,
// node for node, reduced to what decides the keySet() order (no values).
// Chains are linked by `next`; a bin whose chain reaches 9 at >= 64 bins
// becomes a red-black tree (treeify / putTreeVal / removeTreeNode /
// balanceInsertion / balanceDeletion / rotations / moveRootToFront / split /
// untreeify), whose keySet() order is still the `next` chain those methods
// rearrange.  Keys with equal spread hashes are ordered in a tree by
// System.identityHashCode in Java (javatuples' Pair is not Comparable<Pair>,
// so comparableClassFor is null and tieBreakOrder decides): not reproducible
// even by Java; `nondeterministic()` flags it (the tie goes left here).
class JavaHashOrder {
 public:
  using Key = std::pair<int, int32_t>;   // (partition, aggregator)

  bool contains(const Key& k) const { return index_.count(k) != 0; }
  bool hash_of(const Key& k, int32_t* h) const {
    auto it = index_.find(k);
    if (it == index_.end()) return false;
    *h = it->second.first;
    return true;
  }

  // Other_Replica_Gradients.put(key, array) of an absent key (HashMap.putVal).
  void put_new(const Key& k, int32_t key_hash) {
    const int32_t hh = spread(key_hash);
    if (tab_.empty()) resize();
    const int n = (int)tab_.size();
    const int i = hh & (n - 1);
    int p = tab_[i];
    if (p < 0) {
      const int x = new_node(hh, k, -1, false);
      tab_[i] = x;
      index_[k] = {key_hash, x};
    } else if (nd(p).tree) {
      const int x = put_tree_val(p, hh, k);
      index_[k] = {key_hash, x};
    } else {
      for (int bin_count = 0;; ++bin_count) {
        if (nd(p).next < 0) {
          const int x = new_node(hh, k, -1, false);
          nd(p).next = x;
          index_[k] = {key_hash, x};
          if (bin_count >= kTreeify - 1) treeify_bin(hh);   // replaces the chain's nodes (and their index)
          break;
        }
        p = nd(p).next;
      }
    }
    if (++size_ > threshold_) resize();
  }

  // Other_Replica_Gradients.remove(key) (removeNode): the capacity stays.
  bool remove(const Key& k) {
    auto it = index_.find(k);
    if (it == index_.end()) return false;
    const int node = it->second.second;
    index_.erase(it);
    const int i = nd(node).hash & ((int)tab_.size() - 1);
    if (nd(node).tree) {
      remove_tree_node(node, true);
    } else if (tab_[i] == node) {
      tab_[i] = nd(node).next;
    } else {
      int p = tab_[i];
      while (nd(p).next != node) p = nd(p).next;
      nd(p).next = nd(node).next;
    }
    free_node(node);
    --size_;
    return true;
  }

  // new ArrayList<>(keySet()): bins in index order, each chain in link order.
  std::vector<Key> order() const {
    std::vector<Key> out;
    out.reserve(index_.size());
    for (int head : tab_)
      for (int e = head; e >= 0; e = nd(e).next) out.push_back(nd(e).key);
    return out;
  }

  // Other_Replica_Gradients = new HashMap<>() (IPLS.java:1238)
  void clear() {
    tab_.clear();
    pool_.clear();
    free_.clear();
    index_.clear();
    size_ = threshold_ = 0;
    nondet_ = false;
  }

  int64_t capacity() const { return (int64_t)tab_.size(); }
  size_t size() const { return index_.size(); }
  bool tree_bin() const {
    for (int head : tab_)
      if (head >= 0 && nd(head).tree) return true;
    return false;
  }
  bool nondeterministic() const { return nondet_; }

  // Structural checks (for tests; nullptr = sound): every node in its hash's
  // bin, index / size / chains agree, and every tree bin is a red-black tree
  // over exactly its chain's nodes, rooted at the bin's first node, ordered
  // by hash -- TreeNode.checkInvariants plus the red-black rules.
  const char* check_invariants() const {
    size_t seen = 0;
    const int n = (int)tab_.size();
    for (int j = 0; j < n; ++j) {
      const int head = tab_[(size_t)j];
      if (head < 0) continue;
      std::vector<int> chain;
      for (int e = head, prev = -1; e >= 0; prev = e, e = nd(e).next) {
        if ((nd(e).hash & (n - 1)) != j) return "node outside its hash's bin";
        auto it = index_.find(nd(e).key);
        if (it == index_.end() || it->second.second != e) return "lookup index is stale";
        if (nd(e).tree != nd(head).tree) return "tree and plain nodes mixed in one bin";
        if (nd(e).tree && nd(e).prev != prev) return "prev link broken";
        if (chain.size() > index_.size()) return "cycle in chain";
        chain.push_back(e);
      }
      seen += chain.size();
      if (!nd(head).tree) continue;
      if (nd(head).parent >= 0 || nd(head).red) return "bin head is not a black root";
      std::vector<int> members;
      const char* bad = nullptr;
      // -> black height; lo/hi bound the hashes (inclusive: ties may sit either side after rotations)
      auto walk = [&](auto&& self, int t, int64_t lo, int64_t hi) -> int {
        if (t < 0 || bad) return 1;
        if (members.size() > chain.size()) { bad = "cycle in tree"; return 1; }
        members.push_back(t);
        const Node& x = nd(t);
        if (x.hash < lo || x.hash > hi) { bad = "tree not ordered by hash"; return 1; }
        for (int c : {x.left, x.right})
          if (c >= 0 && (nd(c).parent != t || (x.red && nd(c).red))) { bad = "parent link or red-red"; return 1; }
        const int bl = self(self, x.left, lo, x.hash), br = self(self, x.right, x.hash, hi);
        if (bl != br) bad = "unequal black heights";
        return bl + (x.red ? 0 : 1);
      };
      walk(walk, head, INT64_MIN, INT64_MAX);
      if (bad) return bad;
      std::sort(members.begin(), members.end());
      std::sort(chain.begin(), chain.end());
      if (members != chain) return "tree and chain hold different nodes";
    }
    if (seen != index_.size() || (int64_t)seen != (int64_t)size_) return "size / index / chains disagree";
    return nullptr;
  }

 private:
  static constexpr int kTreeify = 8, kUntreeify = 6, kMinTreeify = 64;
  struct Node {
    int32_t hash = 0;   // the spread hash, a Java int
    Key key{};
    int next = -1, prev = -1, parent = -1, left = -1, right = -1;
    bool red = false, tree = false;
  };
  static int32_t spread(int32_t h) {
    const uint32_t u = (uint32_t)h;
    return (int32_t)(u ^ (u >> 16));
  }
  Node& nd(int i) { return pool_[(size_t)i]; }
  const Node& nd(int i) const { return pool_[(size_t)i]; }
  int new_node(int32_t hh, Key k, int next, bool tree) {   // k by value: the pool may move
    int i;
    if (!free_.empty()) {
      i = free_.back();
      free_.pop_back();
    } else {
      i = (int)pool_.size();
      pool_.emplace_back();
    }
    Node& x = nd(i);
    x = Node{};
    x.hash = hh;
    x.key = k;
    x.next = next;
    x.tree = tree;
    return i;
  }
  void free_node(int i) { free_.push_back(i); }
  void remap(int i) { index_[nd(i).key].second = i; }

  // ---- HashMap ----
  void resize() {
    const int old_cap = (int)tab_.size();
    int new_cap;
    if (old_cap > 0) {
      new_cap = old_cap << 1;
      threshold_ <<= 1;
    } else {
      new_cap = 16;
      threshold_ = 12;
    }
    std::vector<int> old;
    old.swap(tab_);
    tab_.assign((size_t)new_cap, -1);
    for (int j = 0; j < old_cap; ++j) {
      int e = old[(size_t)j];
      if (e < 0) continue;
      if (nd(e).next < 0) {
        tab_[(size_t)(nd(e).hash & (new_cap - 1))] = e;
      } else if (nd(e).tree) {
        split(e, j, old_cap);
      } else {
        int lo_h = -1, lo_t = -1, hi_h = -1, hi_t = -1;
        while (e >= 0) {
          const int nxt = nd(e).next;
          if ((nd(e).hash & old_cap) == 0) {
            if (lo_t < 0) lo_h = e; else nd(lo_t).next = e;
            lo_t = e;
          } else {
            if (hi_t < 0) hi_h = e; else nd(hi_t).next = e;
            hi_t = e;
          }
          e = nxt;
        }
        if (lo_t >= 0) { nd(lo_t).next = -1; tab_[(size_t)j] = lo_h; }
        if (hi_t >= 0) { nd(hi_t).next = -1; tab_[(size_t)(j + old_cap)] = hi_h; }
      }
    }
  }

  void treeify_bin(int32_t hh) {
    const int n = (int)tab_.size();
    if (n < kMinTreeify) {
      resize();
      return;
    }
    const int index = (n - 1) & hh;
    int e = tab_[(size_t)index], hd = -1, tl = -1;
    while (e >= 0) {   // replacementTreeNode, in chain order
      const int nxt = nd(e).next;
      const int p = new_node(nd(e).hash, nd(e).key, -1, true);
      remap(p);
      free_node(e);
      if (tl < 0) hd = p;
      else { nd(p).prev = tl; nd(tl).next = p; }
      tl = p;
      e = nxt;
    }
    tab_[(size_t)index] = hd;
    if (hd >= 0) treeify(hd);
  }

  // ---- TreeNode ----
  int root_of(int x) const {
    while (nd(x).parent >= 0) x = nd(x).parent;
    return x;
  }
  void move_root_to_front(int root) {
    if (root < 0 || tab_.empty()) return;
    const int index = ((int)tab_.size() - 1) & nd(root).hash;
    const int first = tab_[(size_t)index];
    if (root != first) {
      tab_[(size_t)index] = root;
      const int rp = nd(root).prev, rn = nd(root).next;
      if (rn >= 0) nd(rn).prev = rp;
      if (rp >= 0) nd(rp).next = rn;
      if (first >= 0) nd(first).prev = root;
      nd(root).next = first;
      nd(root).prev = -1;
    }
  }
  int dir(int32_t h, int32_t ph) {
    if (ph > h) return -1;
    if (ph < h) return 1;
    nondet_ = true;   // tieBreakOrder: System.identityHashCode
    return -1;
  }
  void treeify(int head) {
    int root = -1;
    for (int x = head, nxt; x >= 0; x = nxt) {
      nxt = nd(x).next;
      nd(x).left = nd(x).right = -1;
      if (root < 0) {
        nd(x).parent = -1;
        nd(x).red = false;
        root = x;
      } else {
        for (int p = root;;) {
          const int d = dir(nd(x).hash, nd(p).hash);
          const int xp = p;
          p = d <= 0 ? nd(p).left : nd(p).right;
          if (p < 0) {
            nd(x).parent = xp;
            if (d <= 0) nd(xp).left = x; else nd(xp).right = x;
            root = balance_insertion(root, x);
            break;
          }
        }
      }
    }
    move_root_to_front(root);
  }
  int untreeify(int first) {
    int hd = -1, tl = -1;
    for (int q = first; q >= 0;) {   // replacementNode, in chain order
      const int nxt = nd(q).next;
      const int p = new_node(nd(q).hash, nd(q).key, -1, false);
      remap(p);
      free_node(q);
      if (tl < 0) hd = p; else nd(tl).next = p;
      tl = p;
      q = nxt;
    }
    return hd;
  }
  int put_tree_val(int first, int32_t hh, const Key& k) {
    const int root = nd(first).parent >= 0 ? root_of(first) : first;
    for (int p = root;;) {
      const int d = dir(hh, nd(p).hash);
      const int xp = p;
      p = d <= 0 ? nd(p).left : nd(p).right;
      if (p < 0) {
        const int xpn = nd(xp).next;
        const int x = new_node(hh, k, xpn, true);
        if (d <= 0) nd(xp).left = x; else nd(xp).right = x;
        nd(xp).next = x;
        nd(x).parent = nd(x).prev = xp;
        if (xpn >= 0) nd(xpn).prev = x;
        move_root_to_front(balance_insertion(root, x));
        return x;
      }
    }
  }
  void remove_tree_node(int node, bool movable) {
    const int n = (int)tab_.size();
    const int index = (n - 1) & nd(node).hash;
    int first = tab_[(size_t)index], root = first;
    const int succ = nd(node).next, pred = nd(node).prev;
    if (pred < 0) tab_[(size_t)index] = first = succ;
    else nd(pred).next = succ;
    if (succ >= 0) nd(succ).prev = pred;
    if (first < 0) return;
    if (nd(root).parent >= 0) root = root_of(root);
    if (root < 0 || (movable && (nd(root).right < 0 || nd(root).left < 0 || nd(nd(root).left).left < 0))) {
      tab_[(size_t)index] = untreeify(first);   // too small
      return;
    }
    const int p = node, pl = nd(node).left, pr = nd(node).right;
    int replacement;
    if (pl >= 0 && pr >= 0) {
      int s = pr;
      while (nd(s).left >= 0) s = nd(s).left;   // successor
      std::swap(nd(s).red, nd(p).red);          // swap colours
      const int sr = nd(s).right, pp = nd(p).parent;
      if (s == pr) {
        nd(p).parent = s;
        nd(s).right = p;
      } else {
        const int sp = nd(s).parent;
        if ((nd(p).parent = sp) >= 0) {
          if (s == nd(sp).left) nd(sp).left = p; else nd(sp).right = p;
        }
        if ((nd(s).right = pr) >= 0) nd(pr).parent = s;
      }
      nd(p).left = -1;
      if ((nd(p).right = sr) >= 0) nd(sr).parent = p;
      if ((nd(s).left = pl) >= 0) nd(pl).parent = s;
      if ((nd(s).parent = pp) < 0) root = s;
      else if (p == nd(pp).left) nd(pp).left = s;
      else nd(pp).right = s;
      replacement = sr >= 0 ? sr : p;
    } else if (pl >= 0) {
      replacement = pl;
    } else if (pr >= 0) {
      replacement = pr;
    } else {
      replacement = p;
    }
    if (replacement != p) {
      const int pp = nd(replacement).parent = nd(p).parent;
      if (pp < 0) root = replacement;
      else if (p == nd(pp).left) nd(pp).left = replacement;
      else nd(pp).right = replacement;
      nd(p).left = nd(p).right = nd(p).parent = -1;
    }
    const int r = nd(p).red ? root : balance_deletion(root, replacement);
    if (replacement == p) {   // detach
      const int pp = nd(p).parent;
      nd(p).parent = -1;
      if (pp >= 0) {
        if (p == nd(pp).left) nd(pp).left = -1;
        else if (p == nd(pp).right) nd(pp).right = -1;
      }
    }
    if (movable) move_root_to_front(r);
  }
  void split(int b, int index, int bit) {
    int lo_h = -1, lo_t = -1, hi_h = -1, hi_t = -1, lc = 0, hc = 0;
    for (int e = b, nxt; e >= 0; e = nxt) {
      nxt = nd(e).next;
      nd(e).next = -1;
      if ((nd(e).hash & bit) == 0) {
        if ((nd(e).prev = lo_t) < 0) lo_h = e; else nd(lo_t).next = e;
        lo_t = e;
        ++lc;
      } else {
        if ((nd(e).prev = hi_t) < 0) hi_h = e; else nd(hi_t).next = e;
        hi_t = e;
        ++hc;
      }
    }
    if (lo_h >= 0) {
      if (lc <= kUntreeify) {
        tab_[(size_t)index] = untreeify(lo_h);
      } else {
        tab_[(size_t)index] = lo_h;
        if (hi_h >= 0) treeify(lo_h);
      }
    }
    if (hi_h >= 0) {
      if (hc <= kUntreeify) {
        tab_[(size_t)(index + bit)] = untreeify(hi_h);
      } else {
        tab_[(size_t)(index + bit)] = hi_h;
        if (lo_h >= 0) treeify(hi_h);
      }
    }
  }
  int rotate_left(int root, int p) {
    int r;
    if (p >= 0 && (r = nd(p).right) >= 0) {
      const int rl = nd(p).right = nd(r).left;
      if (rl >= 0) nd(rl).parent = p;
      const int pp = nd(r).parent = nd(p).parent;
      if (pp < 0) { root = r; nd(r).red = false; }
      else if (nd(pp).left == p) nd(pp).left = r;
      else nd(pp).right = r;
      nd(r).left = p;
      nd(p).parent = r;
    }
    return root;
  }
  int rotate_right(int root, int p) {
    int l;
    if (p >= 0 && (l = nd(p).left) >= 0) {
      const int lr = nd(p).left = nd(l).right;
      if (lr >= 0) nd(lr).parent = p;
      const int pp = nd(l).parent = nd(p).parent;
      if (pp < 0) { root = l; nd(l).red = false; }
      else if (nd(pp).right == p) nd(pp).right = l;
      else nd(pp).left = l;
      nd(l).right = p;
      nd(p).parent = l;
    }
    return root;
  }
  int balance_insertion(int root, int x) {
    nd(x).red = true;
    for (;;) {
      int xp = nd(x).parent, xpp;
      if (xp < 0) {
        nd(x).red = false;
        return x;
      }
      if (!nd(xp).red || (xpp = nd(xp).parent) < 0) return root;
      const int xppl = nd(xpp).left;
      if (xp == xppl) {
        const int xppr = nd(xpp).right;
        if (xppr >= 0 && nd(xppr).red) {
          nd(xppr).red = false;
          nd(xp).red = false;
          nd(xpp).red = true;
          x = xpp;
        } else {
          if (x == nd(xp).right) {
            x = xp;
            root = rotate_left(root, x);
            xp = nd(x).parent;
            xpp = xp < 0 ? -1 : nd(xp).parent;
          }
          if (xp >= 0) {
            nd(xp).red = false;
            if (xpp >= 0) {
              nd(xpp).red = true;
              root = rotate_right(root, xpp);
            }
          }
        }
      } else {
        if (xppl >= 0 && nd(xppl).red) {
          nd(xppl).red = false;
          nd(xp).red = false;
          nd(xpp).red = true;
          x = xpp;
        } else {
          if (x == nd(xp).left) {
            x = xp;
            root = rotate_right(root, x);
            xp = nd(x).parent;
            xpp = xp < 0 ? -1 : nd(xp).parent;
          }
          if (xp >= 0) {
            nd(xp).red = false;
            if (xpp >= 0) {
              nd(xpp).red = true;
              root = rotate_left(root, xpp);
            }
          }
        }
      }
    }
  }
  int balance_deletion(int root, int x) {
    for (;;) {
      if (x < 0 || x == root) return root;
      int xp = nd(x).parent;
      if (xp < 0) {
        nd(x).red = false;
        return x;
      }
      if (nd(x).red) {
        nd(x).red = false;
        return root;
      }
      int xpl = nd(xp).left;
      if (xpl == x) {
        int xpr = nd(xp).right;
        if (xpr >= 0 && nd(xpr).red) {
          nd(xpr).red = false;
          nd(xp).red = true;
          root = rotate_left(root, xp);
          xp = nd(x).parent;
          xpr = xp < 0 ? -1 : nd(xp).right;
        }
        if (xpr < 0) {
          x = xp;
        } else {
          int sl = nd(xpr).left, sr = nd(xpr).right;
          if ((sr < 0 || !nd(sr).red) && (sl < 0 || !nd(sl).red)) {
            nd(xpr).red = true;
            x = xp;
          } else {
            if (sr < 0 || !nd(sr).red) {
              if (sl >= 0) nd(sl).red = false;
              nd(xpr).red = true;
              root = rotate_right(root, xpr);
              xp = nd(x).parent;
              xpr = xp < 0 ? -1 : nd(xp).right;
            }
            if (xpr >= 0) {
              nd(xpr).red = xp < 0 ? false : nd(xp).red;
              if ((sr = nd(xpr).right) >= 0) nd(sr).red = false;
            }
            if (xp >= 0) {
              nd(xp).red = false;
              root = rotate_left(root, xp);
            }
            x = root;
          }
        }
      } else {
        if (xpl >= 0 && nd(xpl).red) {
          nd(xpl).red = false;
          nd(xp).red = true;
          root = rotate_right(root, xp);
          xp = nd(x).parent;
          xpl = xp < 0 ? -1 : nd(xp).left;
        }
        if (xpl < 0) {
          x = xp;
        } else {
          int sl = nd(xpl).left, sr = nd(xpl).right;
          if ((sl < 0 || !nd(sl).red) && (sr < 0 || !nd(sr).red)) {
            nd(xpl).red = true;
            x = xp;
          } else {
            if (sl < 0 || !nd(sl).red) {
              if (sr >= 0) nd(sr).red = false;
              nd(xpl).red = true;
              root = rotate_left(root, xpl);
              xp = nd(x).parent;
              xpl = xp < 0 ? -1 : nd(xp).left;
            }
            if (xpl >= 0) {
              nd(xpl).red = xp < 0 ? false : nd(xp).red;
              if ((sl = nd(xpl).left) >= 0) nd(sl).red = false;
            }
            if (xp >= 0) {
              nd(xp).red = false;
              root = rotate_right(root, xp);
            }
            x = root;
          }
        }
      }
    }
  }

  std::vector<int> tab_;                        // bin heads (node indices, -1 = empty)
  std::vector<Node> pool_;
  std::vector<int> free_;
  std::map<Key, std::pair<int32_t, int>> index_;   // key -> (Pair hashCode, node): lookup only
  int size_ = 0, threshold_ = 0;
  bool nondet_ = false;
};

}  // namespace ipls
