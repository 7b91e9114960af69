"""CPU oracle for the IPLS aggregation path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline.  The product
(ipls-java-api_amd/) never imports it.

Parity status: "parity unpinned" for the arithmetic (no JDK here and the
reference ships no golden vectors for this path); the
big-endian codec is pinned against MNIST_Partitioned_Dataset/ETHModel.
"""
