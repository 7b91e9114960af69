#!/bin/bash
# Round 6: the chunked calls' pinned ring depth (IPLS_STAGE_SLOTS 2 / 3 / 4),
# A/B in one process per run (tools/jni_heap_probe.py --ab-slots), three
# processes; then the chunked / JNI / Middleware GPU tests on the 3-slot default.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06u
rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python tools/jni_heap_probe.py 4194304 40 --ab-slots=2,3,4 > $O/slots_ab_$i.json 2> $O/slots_ab_$i.err || exit 11
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_middleware.py tests/test_jni.py tests/test_host_cpp.py \
  -k "stage_pool or stalled or async_many or chunked or jni or loopback or streamed or host_mirror or production" > $O/pytest.log 2>&1 || exit 10
echo done > $O/done
