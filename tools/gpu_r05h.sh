#!/bin/bash
# Round-5 pass h: the chunked calls' rings on THP-registered host memory --
# their tests, the JNI heap-array rates and the Middleware leg's native server.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r05h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_jni.py tests/test_gpu_parity.py tests/test_middleware.py tests/test_host_cpp.py \
  -k "chunked or jni or range or loopback or streamed or host_mirror" -v --timeout 300 --timeout-method thread -m gpu \
  -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
case $rc in 124|134|137|139) exit 10;; esac
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/jni_heap_probe.py 4194304 20 > $O/jni_heap_probe_$i.json 2> $O/jni_heap_probe_$i.err || exit 11
done
timeout -k 10 120 ipls-java-api_amd/lib/pinned_read_probe 4194304 200 > $O/pinned_read_probe.txt 2>&1 || exit 12
timeout -k 10 300 ipls-java-api_amd/lib/middleware_e2e 67108848 16 32 4 > $O/middleware_e2e.json 2> $O/middleware_e2e.err || exit 13
echo done > $O/done
