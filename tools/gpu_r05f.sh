#!/bin/bash
# Round-5 pass f: k_divide's XCD-contiguous tile order (tools/copy_sweep.hip),
# timed in three processes, then FETCH_SIZE / WRITE_SIZE per variant.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r05f}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 120 ipls-java-api_amd/lib/copy_sweep 16 4194304 20 > $O/copy_sweep_$i.txt 2>&1 || exit 10
done
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run -- \
  $R/ipls-java-api_amd/lib/copy_sweep 16 4194304 2 > $O/pmc_fetch.log 2>&1 || exit 11
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o run -- \
  $R/ipls-java-api_amd/lib/copy_sweep 16 4194304 2 > $O/pmc_write.log 2>&1 || exit 12
echo done > $O/done
