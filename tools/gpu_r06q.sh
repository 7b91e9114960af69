#!/bin/bash
# Round 6: one vs two copy streams per stage, the library's chunk pipeline
# alone (tools/chunk_probe.py: no-op source / sink), alternating processes.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06q
mkdir -p $O
for i in 1 2 3; do
  for s in 1 2; do
    IPLS_STAGE_STREAMS=$s timeout -k 10 200 python tools/chunk_probe.py 4194304 20 > $O/chunk_probe_s${s}_$i.json 2> $O/chunk_probe_s${s}_$i.err || exit 10
  done
done
echo done > $O/done
