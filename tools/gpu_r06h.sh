#!/bin/bash
# Round 6: the JNI heap natives with the spinning copy pool -- the JNI GPU
# tests, then tools/jni_heap_probe.py over ring chunk x copy threads.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_jni.py > $O/pytest_jni.log 2>&1 || exit 10
for c in 262144 524288 1048576 2097152; do
  for t in 4 6; do
    IPLS_JNI_RING_CHUNK=$c IPLS_JNI_COPY_THREADS=$t timeout -k 10 120 python tools/jni_heap_probe.py 4194304 20 \
      > $O/probe_c${c}_t$t.json 2> $O/probe_c${c}_t$t.err || exit 11
  done
done
echo done > $O/done
