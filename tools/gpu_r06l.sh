#!/bin/bash
# Round 6: two copy streams per stage (chunk k on stream k % 2) against one
# (IPLS_STAGE_STREAMS=1), alternating processes: the JNI heap probe (its
# natives are the chunked calls), then the chunked / JNI / Middleware GPU tests.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06l
mkdir -p $O
for i in 1 2 3; do
  for s in 1 2; do
    IPLS_STAGE_STREAMS=$s timeout -k 10 120 python tools/jni_heap_probe.py 4194304 20 > $O/probe_s${s}_$i.json 2> $O/probe_s${s}_$i.err || exit 11
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_middleware.py tests/test_jni.py tests/test_host_cpp.py \
  -k "stage_pool or stalled or async_many or chunked or jni or loopback or streamed or host_mirror" > $O/pytest.log 2>&1 || exit 10
echo done > $O/done
