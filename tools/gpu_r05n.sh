#!/bin/bash
# Round 5: the shipped k_divide with wave-contiguous steps -- the divide and
# round GPU tests, the copy sweep in three processes (with a wave-contiguous
# k_finalize A/B), and the list of PMC counters this box offers.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05n
B=$R/ipls-java-api_amd/lib/copy_sweep
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "divide or partitions or round or chunked or middleware or smoke or stateful or config_a" > $O/pytest.log 2>&1 || exit 10
for i in 1 2 3; do
  timeout -k 10 120 $B 16 4194304 20 > $O/copy_sweep_$i.txt 2>&1 || exit 11
done
cd /tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || exit 12
echo done > $O/done
