#!/bin/bash
# Round 5: the L2 -> fabric read requests of the copy sweep's kernels by size
# (32 / 64 / 128 B), so that the divide's FETCH_SIZE excess can be read in
# bytes instead of through FETCH_SIZE's 64-B tally.  One pass per pair.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05o
B=$R/ipls-java-api_amd/lib/copy_sweep
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/p1 -o run -- $B 16 4194304 3 > $O/p1.log 2>&1 || exit 11
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $O/p2 -o run -- $B 16 4194304 3 > $O/p2.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum --output-format csv -d $O/p3 -o run -- $B 16 4194304 3 > $O/p3.log 2>&1 || exit 13
echo done > $O/done
