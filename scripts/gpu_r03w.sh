#!/bin/bash
# Round 3 (session 2) measurement of the shipped build: PMC traffic of the dominant kernels
# (FETCH_SIZE / WRITE_SIZE / TCC requests, one rocprofv3 run per pass, calibrated on
# kma_gather_bench) -> profiles/r03_traffic.json, rocprofv3 kernel stats of the c5 and c3 bench
# commands, the bench lines (c5 headline with the CPU baseline, c2, c3, c4), SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03w}; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
GB=kmers.anno_amd/build/kma_gather_bench
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $c | cut -d' ' -f1)
  step pmc_gather_$tag 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_gather_$tag -o run -- $GB 1536 quad 4
  for wl in c5 c2 c3 c4; do
    step pmc_${wl}_$tag 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${wl}_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --workload $wl --no-cpu-baseline --no-extras
  done
done
step traffic 60 python3 scripts/traffic_summary.py $OUT 8388608
cp $OUT/traffic.log profiles/r03_traffic.json
step stats_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
step stats_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c3 -o run -- python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
step bench_c5 600 python3 bench.py
step bench_c2 300 python3 bench.py --workload c2 --no-cpu-baseline
step bench_c3 300 python3 bench.py --workload c3 --no-cpu-baseline
step bench_c4 300 python3 bench.py --workload c4 --no-cpu-baseline
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for wl in c5 c3; do
  step sq_${wl}_p1 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $OUT/sq_${wl}_p1 -o run -- python3 bench.py --steps 3 --warmup 1 --workload $wl --no-cpu-baseline --no-extras
  step sq_${wl}_p2 300 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $OUT/sq_${wl}_p2 -o run -- python3 bench.py --steps 3 --warmup 1 --workload $wl --no-cpu-baseline --no-extras
done
step sq_summary 60 python3 scripts/sq_summary.py $OUT
