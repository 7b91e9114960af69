#!/bin/bash
# Round 6: (1) the JNI heap natives with the chunk copies split over helper
# threads: JNI GPU tests, then tools/jni_heap_probe.py at
# 1, 2, 4 and 8 copy threads; (2) config D's BE-vs-native A/B on one fixed
# bucket layout (tools/d_be_probe.py, item 2).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_jni.py > $O/pytest_jni.log 2>&1 || exit 10
for t in 1 2 4 8; do
  IPLS_JNI_COPY_THREADS=$t timeout -k 10 120 python tools/jni_heap_probe.py 4194304 20 > $O/jni_heap_probe_t$t.json 2> $O/jni_heap_probe_t$t.err || exit 11
done
timeout -k 10 300 python tools/d_be_probe.py > $O/d_be_probe.json 2> $O/d_be_probe.err || exit 12
echo done > $O/done
