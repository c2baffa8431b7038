#!/bin/bash
# Measurement pass of the shipped build on one GPU box (the round-end evidence under profiles/):
#   traffic  PMC traffic of the dominant kernels: FETCH_SIZE / WRITE_SIZE / TCC requests, one
#            rocprofv3 --pmc run per pass (kernel-trace only), calibrated on kma_gather_bench's
#            random 64-B lines -> $TRAFFIC (bench.py's roofline.traffic source)
#   stats    rocprofv3 --kernel-trace --stats of the c5 and c3 bench commands
#   bench    the bench lines: c5 (headline, with the CPU baseline), c2, c3, c4
#   sq       SQ counters of c5 and c3 (VALU / LDS / wait split)
#   lf       c5 bench lines at load factors 0.75 and 0.9 (their PMC requests: WLS="... c5_lf0.75 c5_lf0.9")
# Usage: SECTIONS="traffic stats bench sq" TRAFFIC=profiles/r06_traffic.json \
#          bash scripts/gpu_measure.sh <out-subdir>
# Stops at the first step that does not exit 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:-measure}; mkdir -p $OUT
SECTIONS=${SECTIONS:-traffic stats bench sq}
step() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)" >> $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
GB=kmers.anno_amd/build/kma_gather_bench
SHORT="--steps 3 --warmup 1 --no-cpu-baseline --no-extras"
for s in $SECTIONS; do
  case $s in
    traffic)
      for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
        tag=$(echo $c | cut -d' ' -f1)
        step pmc_gather_$tag 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_gather_$tag -o run -- $GB 1536 quad 4
        for wl in ${WLS:-c5 c2 c3 c4}; do  # c5_lf0.75: c5 at load factor 0.75 (LF sweep lines)
          wa="--workload ${wl%%_lf*}"; [ "$wl" != "${wl#*_lf}" ] && wa="$wa --load-factor ${wl#*_lf}"
          step pmc_${wl}_$tag 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${wl}_$tag -o run -- python3 bench.py $SHORT $wa
        done
      done
      step traffic 60 python3 scripts/traffic_summary.py $OUT 8388608
      cp $OUT/traffic.log ${TRAFFIC:-$OUT/traffic.json} ;;
    stats)
      step stats_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
      step stats_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c3 -o run -- python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras ;;
    bench)
      step bench_c5 600 python3 bench.py
      step bench_c2 300 python3 bench.py --workload c2 --no-cpu-baseline
      step bench_c3 300 python3 bench.py --workload c3 --no-cpu-baseline
      step bench_c4 300 python3 bench.py --workload c4 --no-cpu-baseline ;;
    lf)  # c5 load-factor sweep lines (their PMC requests per window: WLS with c5_lf0.75 c5_lf0.9)
      for lf in 0.75 0.9; do
        step bench_c5_lf$lf 600 python3 bench.py --workload c5 --load-factor $lf --no-cpu-baseline
      done ;;
    sq)
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
      P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
      for wl in ${SQ_WLS:-c5 c3}; do
        step sq_${wl}_p1 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $OUT/sq_${wl}_p1 -o run -- python3 bench.py $SHORT --workload $wl
        step sq_${wl}_p2 300 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $OUT/sq_${wl}_p2 -o run -- python3 bench.py $SHORT --workload $wl
      done
      step sq_summary 60 python3 scripts/sq_summary.py $OUT ;;
  esac
done
