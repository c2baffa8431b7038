#!/bin/bash
# Four-rank rehearsal of the multi-GPU bench path on one GPU (gloo, --same-device, --verify):
# c4 strong-sharded over 4 ranks, c5 reduced (100k proteins per rank) weak-scaled.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1
OUT=gpurun_out/${1:-multirank4}; mkdir -p $OUT
for wl in c4 c5; do
  extra="--workload $wl --steps 3 --warmup 1"
  [ $wl = c5 ] && extra="$extra --n-seq 100000"
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 4 --dist-backend gloo --same-device --verify \
    --no-extras --no-cpu-baseline $extra > $OUT/$wl.json 2> $OUT/$wl.log
  rc=$?; echo "$wl rc=$rc" >> $OUT/steps.log; [ $rc = 0 ] || exit $rc
done
cat $OUT/steps.log
