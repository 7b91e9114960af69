#!/bin/bash
# Round 6, VERDICT r5 item 2: which limit binds config D's big-endian
# k_reduce (84 %) where native config C's runs at 89 %.  One rocprofv3 --pmc
# pass per counter set (SQ <= 8, GRBM <= 2 per pass), each over a short bench
# run of one workload: D-be (64 x 4M x 32, BE in + out) and C (native).
# Counters missing from this box's `rocprofv3 -L` are dropped from a pass
# before it runs (an unknown name is not worth a hang).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || exit 10
have() { grep -qw "$1" $O/counters.txt; }
LEAN="--no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-middleware --no-verify --steps 3 --warmup 1"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAIT_INST_LDS"
n=0
for wl in Dbe C; do
  case $wl in Dbe) args="--config D --be";; C) args="--config C";; esac
  for pass in P1 P2; do
    ctrs=""
    for c in ${!pass}; do have $c && ctrs="$ctrs $c"; done
    echo "$wl $pass:$ctrs" >> $O/passes.txt
    [ -z "$ctrs" ] && continue
    n=$((n+1))
    timeout -s KILL 240 rocprofv3 --pmc $ctrs -T --output-format csv -d $O/${wl}_${pass} -o run -- \
      python3 $R/bench.py $LEAN $args > $O/${wl}_${pass}.log 2>&1 || exit $((10+n))
    echo "$wl $pass done"
  done
done
echo done > $O/done
