#!/bin/bash
# Round 5: k_divide with wave-contiguous steps (tools/copy_sweep.hip WC),
# three processes, then FETCH_SIZE / WRITE_SIZE passes over one short sweep.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05m
B=$R/ipls-java-api_amd/lib/copy_sweep
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 120 $B 16 4194304 20 > $O/copy_sweep_$i.txt 2>&1 || exit 11
done
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B 16 4194304 3 > $O/pmc_fetch.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B 16 4194304 3 > $O/pmc_write.log 2>&1 || exit 13
echo done > $O/done
