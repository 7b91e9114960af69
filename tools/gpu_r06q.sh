#!/bin/bash
# Round 6: one vs two copy streams per stage, the library's chunk pipeline
# alone (tools/chunk_probe.py --ab: no-op source / sink, two handles in one
# process, interleaved rep by rep), three processes.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06q
rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python tools/chunk_probe.py 4194304 60 --ab > $O/chunk_ab_$i.json 2> $O/chunk_ab_$i.err || exit 10
done
echo done > $O/done
