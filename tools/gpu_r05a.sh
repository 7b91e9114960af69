#!/bin/bash
# Round-5 first GPU pass: the new chunked-call / JNI-interleave / middleware
# tests, the default bench line (with the Middleware socket leg), and config
# B's kernel-vs-boundary split (tools/b_gap_probe.py under a kernel trace).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r05a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_jni.py tests/test_gpu_parity.py tests/test_middleware.py \
  -k "chunked or jni or range or loopback or streamed" -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
  > $O/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_new.log
case $rc in 124|134|137|139) exit 10;; esac
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_b -o run -- \
  python3 $R/tools/b_gap_probe.py > $O/b_gap_probe.json 2> $O/b_gap_probe.err || exit 13
echo done > $O/done
