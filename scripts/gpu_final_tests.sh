#!/bin/bash
# Round-6 final GPU pass: the whole GPU suite + smoke on the final tree, then the replicated
# host fan-out with round 5's oversubscription rehearsed (KMA_OPT_HOST_THREADS = 64: 8
# staging threads per replica for 8 replicas on the box's 16 CPUs) beside the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/gpu_tests.sh ${1:-r06_final}; rc=$?
OUT=gpurun_out/${1:-r06_final}
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/replica_scaling.py --replicas 1,8 --host-threads 64 > $OUT/replicas_t64.jsonl 2> $OUT/replicas_t64.log
r=$?; echo "replicas t64 rc=$r" >> $OUT/steps.log
exit $(( rc != 0 ? rc : r ))
