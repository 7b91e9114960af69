#!/bin/bash
# Round 6: the N>1 path rehearsed on one GPU (two ranks over gloo sharing it):
# the line must carry scaling_check and every leg.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06j
mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || exit 10
echo done > $O/done
