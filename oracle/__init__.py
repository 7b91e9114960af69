"""CPU oracle for the IPLS aggregation path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline.  The product
(ipls-java-api_amd/) never imports it.

Parity status: "parity unpinned" for the arithmetic (no JDK here and the
reference ships no golden vectors for this path); the
big-endian codec is pinned against MNIST_Partitioned_Dataset/ETHModel.
The JDK 8 HashMap key order and the javatuples Pair hashCode behind
Collect_Replicas (oracle.JavaHashMap, java_pair_hash, including the TreeNode
red-black bins) are restated from the published JDK / javatuples 1.2 sources,
pinned only by published String.hashCode values, JDK iteration facts and the
structural invariants JDK's own TreeNode.checkInvariants asserts
(tests/test_java_order.py);
tests/java/PinJavaOrder.java is the pin for a host with a JDK.
"""
