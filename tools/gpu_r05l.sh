#!/bin/bash
# Round 5: does an event packet between config C launches change k_reduce's
# own duration?  tools/b_gap_probe.py at the headline shape, plain and under a
# kernel trace (launch order: 40 warm-up, then per round 20 events_each,
# 20 events_ends, 20 out_ends).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp IPLS_PROBE_CONFIG=C
timeout -k 10 200 python3 -u tools/b_gap_probe.py > $O/probe_plain.json 2> $O/probe_plain.err || exit 11
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/tools/b_gap_probe.py > $O/probe_traced.json 2> $O/probe_traced.err || exit 12
echo done > $O/done
