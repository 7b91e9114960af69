#!/bin/bash
# GPU-box script (round 4): the rocprofv3 kernel trace of config C's bench
# command and the two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, no
# trace domains) for every workload whose traffic the bench line reports:
# C (k_reduce, and the round leg's k_finalize / k_divide / k_round), B, D-be, F.
# Usage (repo root on the box): [CFGS="C B"] [SKIP_TRACE=1] tools/gpu_pmc_all.sh TAG
set -o pipefail
TAG=${1:-r04}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
LEAN="--no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival"
cd /tmp
if [ -z "$SKIP_TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_C -o run -- \
    python3 $R/bench.py $LEAN > $O/bench_trace_C.json 2> $O/bench_trace_C.err || exit 13
  echo "trace done"
fi
for cfg in ${CFGS:-C B D F}; do
  extra=""
  [ $cfg = D ] && extra="--be"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr -T --output-format csv -d $O/pmc_${cfg}_${ctr} -o run -- \
      python3 $R/bench.py $LEAN --no-verify --config $cfg $extra --steps 3 --warmup 1 \
      > $O/pmc_${cfg}_${ctr}.log 2>&1 || exit 14
    echo "pmc $cfg $ctr done"
  done
done
echo done > $O/done
