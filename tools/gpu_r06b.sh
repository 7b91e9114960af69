#!/bin/bash
# Round 6: the chunked calls with the shard lock around the fold / snapshot
# only -- the chunked, JNI, Middleware and C++ host GPU
# tests, one process, each step under its own time limit.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "chunked or range or chunked_io" \
  > $O/pytest_chunked.log 2>&1 || exit 10
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_jni.py tests/test_middleware.py tests/test_host_cpp.py \
  > $O/pytest_jni_mw.log 2>&1 || exit 11
echo done > $O/done
