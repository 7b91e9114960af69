#!/bin/bash
# Round 6: the new GPU tests (stage pool under concurrency, a stalled
# Middleware client, UpdateAsyncMany) and the JNI heap probe at the shim's
# defaults (16 MiB in / 4 MiB out chunks, 4 copy threads), three times.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_middleware.py tests/test_jni.py \
  -k "stage_pool or stalled or async_many or chunked or jni or loopback or streamed" > $O/pytest.log 2>&1 || exit 10
for i in 1 2 3; do
  timeout -k 10 120 python tools/jni_heap_probe.py 4194304 20 > $O/jni_heap_probe_$i.json 2> $O/jni_heap_probe_$i.err || exit 11
done
echo done > $O/done
