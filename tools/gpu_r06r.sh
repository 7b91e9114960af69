#!/bin/bash
# Round 6: the JNI ring -> heap natives' chunk on the two-stream stages:
# 4 MiB vs 8 MiB (IPLS_JNI_RING_CHUNK sets both directions; read the
# finalize / getPartitions columns), alternating processes.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06r
rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  for c in 524288 1048576; do
    IPLS_JNI_RING_CHUNK=$c timeout -k 10 120 python tools/jni_heap_probe.py 4194304 30 > $O/probe_c${c}_$i.json 2> $O/probe_c${c}_$i.err || exit 11
  done
done
echo done > $O/done
