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
// So a key's position in keySet() iteration is (bin under the current
// capacity, then insertion order within the bin): chains only ever append
// and resizes keep the relative order of the keys that stay together.
// Iteration walks bins in ascending index.  One case is not restated: a bin
// that reaches 9 keys at capacity >= 64 becomes a red-black tree whose list
// order follows the tree's rotations (`tree_bin` flags it; the keys of that
// bin then keep insertion order).  With peer IDs as keys that needs nine
// colliding hashes in one of >= 64 bins.
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
#include <unordered_map>
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

class JavaHashOrder {
 public:
  using Key = std::pair<int, int32_t>;   // (partition, aggregator)

  bool contains(const Key& k) const { return keys_.count(k) != 0; }
  bool hash_of(const Key& k, int32_t* h) const {
    auto it = keys_.find(k);
    if (it == keys_.end()) return false;
    *h = it->second.hash;
    return true;
  }

  // Other_Replica_Gradients.put(key, array) of an absent key (HashMap.putVal).
  void put_new(const Key& k, int32_t hash) {
    if (cap_ == 0) set_capacity(16);                // resize() of the empty table
    const uint32_t b = bin(hash, cap_);
    const int64_t chain = bins_[b];                 // keys already in that bin
    keys_[k] = E{hash, seq_++};
    ++bins_[b];
    if (chain >= 8) {                               // binCount >= TREEIFY_THRESHOLD - 1
      if (cap_ < 64) set_capacity(cap_ * 2);        // treeifyBin: resize instead
      else tree_bin_ = true;
    }
    if ((int64_t)keys_.size() > cap_ / 4 * 3) set_capacity(cap_ * 2);   // ++size > threshold
  }

  // Other_Replica_Gradients.remove(key) (removeNode): the capacity stays.
  bool remove(const Key& k) {
    auto it = keys_.find(k);
    if (it == keys_.end()) return false;
    auto b = bins_.find(bin(it->second.hash, cap_));
    if (b != bins_.end() && --b->second == 0) bins_.erase(b);
    keys_.erase(it);
    return true;
  }

  // new ArrayList<>(keySet()): ascending bin, insertion order within a bin.
  std::vector<Key> order() const {
    std::vector<std::pair<std::pair<uint32_t, uint64_t>, Key>> v;
    v.reserve(keys_.size());
    for (const auto& e : keys_) v.push_back({{bin(e.second.hash, cap_), e.second.seq}, e.first});
    std::sort(v.begin(), v.end());
    std::vector<Key> out;
    out.reserve(v.size());
    for (auto& x : v) out.push_back(x.second);
    return out;
  }

  // Other_Replica_Gradients = new HashMap<>() (IPLS.java:1238)
  void clear() {
    keys_.clear();
    bins_.clear();
    cap_ = 0;
    tree_bin_ = false;
  }

  int64_t capacity() const { return cap_; }
  size_t size() const { return keys_.size(); }
  bool tree_bin() const { return tree_bin_; }

 private:
  struct E {
    int32_t hash;
    uint64_t seq;
  };
  // a resize: the per-bin key counts under the new capacity (amortised O(1) per put)
  void set_capacity(int64_t cap) {
    cap_ = cap;
    bins_.clear();
    for (const auto& e : keys_) ++bins_[bin(e.second.hash, cap_)];
  }
  static uint32_t bin(int32_t h, int64_t cap) {
    const uint32_t u = (uint32_t)h;
    return (u ^ (u >> 16)) & (uint32_t)(cap - 1);
  }
  std::map<Key, E> keys_;
  std::unordered_map<uint32_t, int64_t> bins_;   // keys per bin under cap_
  int64_t cap_ = 0;
  uint64_t seq_ = 0;
  bool tree_bin_ = false;
};

}  // namespace ipls
