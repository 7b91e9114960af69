#!/bin/bash
# Round 6: JNI heap natives, ring chunk size x copy threads (tools/jni_heap_probe.py).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06d
mkdir -p $O
for c in 262144 524288 1048576 2097152; do
  for t in 3 4 6; do
    IPLS_JNI_RING_CHUNK=$c IPLS_JNI_COPY_THREADS=$t timeout -k 10 120 python tools/jni_heap_probe.py 4194304 20 \
      > $O/probe_c${c}_t$t.json 2> $O/probe_c${c}_t$t.err || exit 11
  done
done
echo done > $O/done
