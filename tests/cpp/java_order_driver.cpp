// Drives ipls::JavaHashOrder (csrc/java_hashmap.hpp, the front's model of
// PeerData.Other_Replica_Gradients' key order) from a command stream, for
// tests/test_java_order.py to compare with oracle.JavaHashMap's simulation of
// the JDK table.  Commands, one per line:
//   p <partition> <aggregator> <hash>   put (if absent)
//   r <partition> <aggregator>          remove
//   o                                   print "<capacity> <tree_bin> <nondeterministic> p:a p:a ..."
//   c                                   clear (new HashMap<>())
// After every command the model's structure is checked (check_invariants);
// a failure is printed to stderr and ends the run with status 3.
#include <cstdio>
#include <cstring>

#include "java_hashmap.hpp"

int main() {
  ipls::JavaHashOrder m;
  char cmd[8];
  while (std::scanf("%7s", cmd) == 1) {
    if (!std::strcmp(cmd, "p")) {
      int p, a, h;
      if (std::scanf("%d %d %d", &p, &a, &h) != 3) return 2;
      if (!m.contains({p, a})) m.put_new({p, a}, h);
    } else if (!std::strcmp(cmd, "r")) {
      int p, a;
      if (std::scanf("%d %d", &p, &a) != 2) return 2;
      m.remove({p, a});
    } else if (!std::strcmp(cmd, "o")) {
      std::printf("%lld %d %d", (long long)m.capacity(), (int)m.tree_bin(), (int)m.nondeterministic());
      for (const auto& k : m.order()) std::printf(" %d:%d", k.first, k.second);
      std::printf("\n");
    } else if (!std::strcmp(cmd, "c")) {
      m.clear();
    } else {
      return 2;
    }
    if (const char* bad = m.check_invariants()) {
      std::fprintf(stderr, "invariant: %s\n", bad);
      return 3;
    }
  }
  return 0;
}
