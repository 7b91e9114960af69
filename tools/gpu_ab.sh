#!/bin/bash
# GPU-box script for the round-3 A/Bs (from the repo root):
#   shard pool: tools/shard_pool_probe.py on the round-2 library vs the current one
#   D schedule: bench.py --be-schedule-ab in three processes
#   D-be PMC:   FETCH_SIZE / WRITE_SIZE passes of config D (BE in + out) on the current library
#   B sweep:    tools/reduce_sweep.hip over config B's dispatch (lanes x vectors, big vs mid) beside the
#               streaming-read and dwordx4-copy ceilings, three processes
#   B PMC:      FETCH_SIZE / WRITE_SIZE passes of config B
#   fewp:       the same sweep over 1-7 partitions of 4M x 32 (which shape a short batch should get)
#   rehearsal:  bench.py --multi-rehearsal (the single-handle multi-GPU leg over two shards of GPU 0)
#   bench:      the default bench line
#   dprobe:     config D in the default line beside the A/B leg, in one process
#   gloo:       bench.py at N = 2 and 4 over gloo, every rank on GPU 0 (rehearsal of the N>1 legs)
#   tests:      the GPU suite
# Usage: tools/gpu_ab.sh TAG [steps...]   (steps: pool dsched dpmc bsweep bpmc rehearsal bench dprobe tests; default the first 3)
set -o pipefail
TAG=${1:-ab}; shift
STEPS=${*:-pool dsched dpmc}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    pool)
      for lib in ab/libipls_agg_r2.so libipls_agg.so; do
        IPLS_AGG_LIB=$R/ipls-java-api_amd/lib/$lib timeout -k 10 120 python tools/shard_pool_probe.py 2000 8 \
          >> $O/shard_pool_probe.jsonl 2>> $O/shard_pool_probe.err || exit 21
      done
      IPLS_AGG_LIB=$R/ipls-java-api_amd/lib/ab/libipls_agg_r2.so timeout -k 10 120 python tools/shard_pool_probe.py 2000 8 \
        >> $O/shard_pool_probe.jsonl 2>> $O/shard_pool_probe.err || exit 21
      timeout -k 10 120 python tools/shard_pool_probe.py 2000 8 >> $O/shard_pool_probe.jsonl 2>> $O/shard_pool_probe.err || exit 21
      ;;
    dsched)
      for i in 1 2 3; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-other-configs \
          --no-per-arrival --be-schedule-ab >> $O/be_schedule_ab.jsonl 2>> $O/be_schedule_ab.err || exit 22
      done
      ;;
    dpmc)
      cd /tmp
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch_D -o run -- \
        python3 $R/bench.py --config D --be --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify \
        --steps 3 --warmup 1 > $O/pmc_fetch_D.log 2>&1 || exit 23
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write_D -o run -- \
        python3 $R/bench.py --config D --be --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify \
        --steps 3 --warmup 1 > $O/pmc_write_D.log 2>&1 || exit 24
      cd $R
      ;;
    bsweep)
      for i in 1 2 3; do
        SWEEP_QUICK=1 SWEEP_B=1 SWEEP_COPY=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep 16 1048576 8 32 50 \
          >> $O/sweep_B.txt 2>&1 || exit 25
      done
      ;;
    fewp)     # few-partition batches (per-partition flushes, short ranges): lanes x vectors per lane, P = 1..7
      for P in 1 3 5 7 2; do
        SWEEP_QUICK=1 SWEEP_B=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep $P 4194304 32 32 10 \
          >> $O/sweep_fewp.txt 2>&1 || exit 34
      done
      ;;
    s512)     # 1024 vs 512 lanes at R = 16 on B, C, F and D (BE in + out), three processes each
      for i in 1 2 3; do
        SWEEP_QUICK=1 SWEEP_512=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep 16 4194304 32 32 20 >> $O/sweep_512_C.txt 2>&1 || exit 35
        SWEEP_QUICK=1 SWEEP_512=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep 16 1048576 8 32 50 >> $O/sweep_512_B.txt 2>&1 || exit 35
        SWEEP_QUICK=1 SWEEP_512=1 timeout -k 10 200 ipls-java-api_amd/lib/reduce_sweep 16 8388608 64 32 10 >> $O/sweep_512_F.txt 2>&1 || exit 35
        SWEEP_QUICK=1 SWEEP_512=1 SWEEP_BE=1 SWEEP_BE_OUT=1 timeout -k 10 200 ipls-java-api_amd/lib/reduce_sweep 64 4194304 32 32 10 \
          >> $O/sweep_512_D.txt 2>&1 || exit 35
      done
      ;;
    btrace)   # config B under rocprofv3 --kernel-trace --stats: the kernel's own duration
      cd /tmp
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_B -o run -- \
        python3 $R/bench.py --config B --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival \
        > $O/bench_B_trace.json 2> $O/bench_B_trace.err || exit 36
      cd $R
      ;;
    fewp_be)  # few-partition big-endian batches (in + out): 1024/512/256 lanes, R = 16 SEQ vs R = 8
      for P in 1 2 3 5 7; do
        SWEEP_QUICK=1 SWEEP_512=1 SWEEP_BE=1 SWEEP_BE_OUT=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep $P 4194304 32 32 10 \
          >> $O/sweep_fewp_be.txt 2>&1 || exit 37
      done
      ;;
    halfround)  # the fused round on few partitions: shipped big/mid vs the half shape (IPLS_HALF_ROUND=1 build)
      timeout -k 10 300 python tools/half_round_probe.py 5 > $O/half_round_probe.jsonl 2> $O/half_round_probe.err || exit 38
      ;;
    midp)     # 8-15 partitions of 4M (4-7.5 rounds of big tiles): 1024 vs 512 lanes
      for P in 9 10 12 13 8; do
        SWEEP_QUICK=1 SWEEP_512=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep $P 4194304 32 32 10 \
          >> $O/sweep_midp.txt 2>&1 || exit 39
      done
      ;;
    accum)    # ACCUM start (reads the target): R = 8 x 1024 (shipped) vs R = 16 x 512 / 256 on few and many partitions
      for P in 1 2 3 5 16; do
        SWEEP_QUICK=1 SWEEP_ACCUM=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep $P 4194304 32 32 10 \
          >> $O/sweep_accum.txt 2>&1 || exit 40
      done
      ;;
    accum2)   # ACCUM on many partitions, and big-endian ACCUM
      for P in 32 64; do
        SWEEP_QUICK=1 SWEEP_ACCUM=1 timeout -k 10 200 ipls-java-api_amd/lib/reduce_sweep $P 4194304 32 32 6 \
          >> $O/sweep_accum2.txt 2>&1 || exit 41
      done
      for P in 1 3 16; do
        SWEEP_QUICK=1 SWEEP_ACCUM=1 SWEEP_BE=1 timeout -k 10 200 ipls-java-api_amd/lib/reduce_sweep $P 4194304 32 32 8 \
          >> $O/sweep_accum2_be.txt 2>&1 || exit 42
      done
      ;;
    fpmc)     # config F (16 x 8M x 64, one GPU's slice) PMC passes
      cd /tmp
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch_F -o run -- \
        python3 $R/bench.py --config F --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify \
        --steps 3 --warmup 1 > $O/pmc_fetch_F.log 2>&1 || exit 47
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write_F -o run -- \
        python3 $R/bench.py --config F --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify \
        --steps 3 --warmup 1 > $O/pmc_write_F.log 2>&1 || exit 48
      cd $R
      ;;
    cpol)     # cache-policy bits of the bucket loads (buffer loads, sc0/sc1/nt) on C, F and B, three processes
      for i in 1 2 3; do
        SWEEP_QUICK=1 SWEEP_CPOL=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep 16 4194304 32 32 10 >> $O/sweep_cpol_C.txt 2>&1 || exit 54
      done
      SWEEP_QUICK=1 SWEEP_CPOL=1 timeout -k 10 200 ipls-java-api_amd/lib/reduce_sweep 16 8388608 64 32 6 >> $O/sweep_cpol_F.txt 2>&1 || exit 54
      SWEEP_QUICK=1 SWEEP_CPOL=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep 16 1048576 8 32 40 >> $O/sweep_cpol_B.txt 2>&1 || exit 54
      ;;
    cpolbe)   # big-endian in + out through buffer loads (no SEQ fences) vs the shipped SEQF = 3 kernel, D and C shapes
      for i in 1 2; do
        SWEEP_QUICK=1 SWEEP_CPOL_BE=1 SWEEP_BE=1 SWEEP_BE_OUT=1 timeout -k 10 200 ipls-java-api_amd/lib/reduce_sweep 64 4194304 32 32 8 \
          >> $O/sweep_cpol_be_D.txt 2>&1 || exit 55
        SWEEP_QUICK=1 SWEEP_CPOL_BE=1 SWEEP_BE=1 SWEEP_BE_OUT=1 timeout -k 10 120 ipls-java-api_amd/lib/reduce_sweep 16 4194304 32 32 10 \
          >> $O/sweep_cpol_be_C.txt 2>&1 || exit 55
      done
      ;;
    bpmc)
      cd /tmp
      timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch_B -o run -- \
        python3 $R/bench.py --config B --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify \
        --steps 20 --warmup 2 > $O/pmc_fetch_B.log 2>&1 || exit 26
      timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write_B -o run -- \
        python3 $R/bench.py --config B --no-cpu-baseline --no-e2e --no-other-configs --no-per-arrival --no-verify \
        --steps 20 --warmup 2 > $O/pmc_write_B.log 2>&1 || exit 27
      cd $R
      ;;
    rehearsal)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-other-configs \
        --no-per-arrival --multi-rehearsal > $O/bench_multi_rehearsal.json 2> $O/bench_multi_rehearsal.err || exit 28
      ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 29
      ;;
    repeat)   # three default bench runs (no CPU baseline) on one box: the process-to-process spread
      for i in 1 2 3; do
        timeout -k 10 400 python bench.py --no-cpu-baseline >> $O/bench_repeat.jsonl 2>> $O/bench_repeat.err || exit 50
      done
      ;;
    dprobe)   # config D in the default line vs the A/B leg, same process: with and without the other legs
      timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e --no-per-arrival --be-schedule-ab \
        >> $O/dprobe.jsonl 2>> $O/dprobe.err || exit 30
      timeout -k 10 500 python bench.py --be-schedule-ab >> $O/dprobe.jsonl 2>> $O/dprobe.err || exit 31
      ;;
    gloo)     # the N>1 bench legs over gloo with every rank on the one GPU (a code-path rehearsal)
      for n in 2 4; do
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
          --master-port $((29500 + n)) bench.py --gpus $n --dist-backend gloo --steps 20 --warmup 5 \
          > $O/bench_gloo$n.json 2> $O/bench_gloo$n.err || exit 33
      done
      ;;
    halfalways)  # the big shape's remaining grids (C fold / round / ACCUM, F fold) vs the half shape, 3 processes
      for i in 1 2 3; do
        timeout -k 10 300 python tools/variant_probe.py 4 >> $O/half_always_probe.jsonl 2>> $O/half_always_probe.err || exit 46
      done
      ;;
    rot)      # sub-window rotation per tile (IPLS_ROT=1 build) vs shipped, 3 processes
      for i in 1 2 3; do
        timeout -k 10 400 python tools/variant_probe.py 4 libipls_agg_rot.so C,Cround,F,B,D \
          >> $O/rot_probe.jsonl 2>> $O/rot_probe.err || exit 49
      done
      ;;
    soak2)    # longer soaks: 120 production-length seeds, 1000 short ones, ingest mutations
      timeout -k 10 1000 python -u tools/fuzz_stateful.py 5000 120 big > $O/fuzz_stateful_big_120.txt 2>&1 || exit 51
      timeout -k 10 600 python -u tools/fuzz_stateful.py 6000 1000 > $O/fuzz_stateful_1000.txt 2>&1 || exit 52
      timeout -k 10 600 python -u tools/fuzz_ingest.py 7000 200 > $O/fuzz_ingest_200.txt 2>&1 || exit 53
      ;;
    stress)   # the four-thread shared-handle test 200 times, one- and three-shard handles
      timeout -k 10 600 python -u tools/stress_concurrent.py 200 > $O/stress_concurrent_200.txt 2>&1 || exit 56
      timeout -k 10 600 python -u tools/stress_concurrent.py 200 sharded > $O/stress_concurrent_sharded_200.txt 2>&1 || exit 57
      ;;
    fastp)    # per-arrival calls: ipls._fast vs ctypes, interleaved, three processes
      for i in 1 2 3; do
        timeout -k 10 300 python -u tools/fast_probe.py 10 >> $O/fast_probe.jsonl 2>> $O/fast_probe.err || exit 58
      done
      ;;
    gloo8)    # the N = 8 bench over gloo with every rank on GPU 0 (rehearsal of the 8-GPU code path and memory)
      timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29508 bench.py --gpus 8 --dist-backend gloo --steps 10 --warmup 2 \
        > $O/bench_gloo8.json 2> $O/bench_gloo8.err || exit 43
      ;;
    soak)     # random call sequences: 40 seeds at production bucket lengths, 400 short ones
      timeout -k 10 900 python -u tools/fuzz_stateful.py 3000 40 big > $O/fuzz_stateful_big_40.txt 2>&1 || exit 44
      timeout -k 10 600 python -u tools/fuzz_stateful.py 4000 400 > $O/fuzz_stateful_400.txt 2>&1 || exit 45
      ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
      case $rc in 0|1) ;; *) exit 32;; esac
      ;;
  esac
done
echo done > $O/done
