#!/bin/bash
# Round-6 full pass on one library: the whole GPU suite, smoke, the default
# bench line and a rocprofv3 kernel trace (+ stats) of the headline command.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-r06e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
case $rc in 124|134|137|139) exit 10;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival > $O/bench_trace.json 2> $O/bench_trace.err || exit 13
echo done > $O/done
