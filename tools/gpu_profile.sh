#!/bin/bash
# GPU-box script: parity tests, smoke, bench, rocprofv3 kernel trace and the
# two PMC passes (FETCH_SIZE, WRITE_SIZE) for the bench workload.
# Usage (from the repo root on the box): tools/gpu_profile.sh TAG [bench args]
set -o pipefail
TAG=${1:-r01}; shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
  case $rc in 124|134|137|139) exit 10;; esac
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
fi
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || exit 12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival "$@" > $O/bench_trace.json 2> $O/bench_trace.err || exit 13
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify "$@" --steps 3 --warmup 1 > $O/pmc_fetch.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify "$@" --steps 3 --warmup 1 > $O/pmc_write.log 2>&1 || exit 15
echo done > $O/done
