#!/bin/bash
# Round 6: soak of the concurrent paths on the final library, single-shard
# and sharded handles (tools/stress_concurrent.py), each under its own limit.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r06n}
mkdir -p $O
timeout -k 10 400 python -u tools/stress_concurrent.py 60 > $O/stress_single.log 2>&1 || exit 10
timeout -k 10 400 python -u tools/stress_concurrent.py 60 sharded > $O/stress_sharded.log 2>&1 || exit 11
echo done > $O/done
