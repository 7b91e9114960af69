#!/bin/bash
# Round 6: the JNI heap probe at the shim's defaults, three processes.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06g
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python tools/jni_heap_probe.py 4194304 20 > $O/jni_heap_probe_$i.json 2> $O/jni_heap_probe_$i.err || exit 11
done
echo done > $O/done
