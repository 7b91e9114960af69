#!/bin/bash
# Round-5 pass c: JNI heap-array rates on the one-call chunked natives, and
# config B's split with the reduce_batch_out variant.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r05c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/jni_heap_probe.py 4194304 20 > $O/jni_heap_probe.json 2> $O/jni_heap_probe.err || exit 10
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_b -o run -- \
  python3 $R/tools/b_gap_probe.py > $O/b_gap_probe.json 2> $O/b_gap_probe.err || exit 13
echo done > $O/done
