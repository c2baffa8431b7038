"""The multi-rank product path of bench.py, run on the GPU: 2 ranks as fresh child processes
(torch.distributed.run), both on device 0 with the gloo backend (RCCL takes one rank per GPU and
the box has one), so the code the driver's 8-GPU scaling run executes has already run:
  - the table built on rank 0 and broadcast (host-staged under gloo), its layout broadcast;
  - each rank's timed device calls on its shard / its own batch;
  - the per-function tally reduce inside the timed region and the max-over-ranks timing;
  - then (--verify, on rank 0): the gathered per-rank outputs equal one single-rank call on the
    whole batch, the reduced tally equals steps x the single-rank tallies, both ranks' replicas
    carry the same slot digest and answer a probe batch identically, and the whole batch through
    kma_table_replicate + the host entry point's fan-out over 3 replicas equals the answer.
There is no reference counterpart: the reference has no distributed code; the
partitioning is north_star's (input shards, replicated table, tally gather)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_two_ranks(name, extra, timeout):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--same-device", "--verify", "--no-extras", "--no-cpu-baseline", *extra]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    # the ranks' progress goes to a log as it happens (a long silent test looks hung)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log = os.path.join(ROOT, "gpurun_out", f"multirank_{name}.log")
    with open(log, "w") as err:
        p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=err, text=True,
                           timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (f"rc {p.returncode}\n{p.stdout[-3000:]}\n"
                                         f"{open(log).read()[-5000:]}")
    out = json.loads(lines[-1])
    with open(os.path.join(ROOT, "gpurun_out", f"multirank_{name}.json"), "w") as f:
        f.write(lines[-1] + "\n")  # the rank-0 line, verify record included
    return out


def _check(out, scaling):
    v = out["verify"]
    assert out["n_gpus"] == 2 and v["ranks"] == 2 and out["scaling"] == scaling
    assert v["table_identical_across_ranks"]
    assert v["outputs_equal_single_rank"]
    assert v["tally_equals_single_rank"]
    assert v["replica_fanout_equals"] and len(v["replicas"]) == 3
    assert v["called"] > 0 and v["ok"]
    assert out["value"] > 0 and "gloo" in out["config"]["parallelism"]


@pytest.mark.timeout(900)
def test_two_ranks_c4_full_strong(native_lib):
    """BASELINE configs[3] at full size: ONE 1M-protein batch cut into 2 residue-balanced
    shards against the 10^7-row table broadcast from rank 0 (strong scaling)."""
    _check(_run_two_ranks("c4", ["--workload", "c4", "--steps", "3", "--warmup", "1"], 800), "strong")


@pytest.mark.timeout(900)
def test_two_ranks_c5_reduced_weak(native_lib):
    """BASELINE configs[4] reduced to 100k proteins per rank (each rank its own batch, weak
    scaling) against the full 10^8-row table (1.5 GiB) built on rank 0 and broadcast."""
    _check(_run_two_ranks("c5", ["--workload", "c5", "--n-seq", "100000", "--steps", "3",
                           "--warmup", "1"], 800), "weak")
