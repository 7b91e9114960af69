#!/bin/bash
# Round-5 pass e: the C++ Middleware server (host test + native harness), the
# JNI updateGradientDirect test, and an N=2 gloo rehearsal of bench.py.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r05e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_host_cpp.py tests/test_jni.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
case $rc in 124|134|137|139) exit 10;; esac
timeout -k 10 300 ipls-java-api_amd/lib/middleware_e2e 67108848 16 32 4 > $O/middleware_e2e.json 2> $O/middleware_e2e.err || exit 11
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || exit 12
echo done > $O/done
