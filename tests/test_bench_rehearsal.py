"""bench.py's multi-rank branch end to end on CPU (no GPU): two ranks over gloo through
torch.distributed.run, with tests/bench_rehearsal.py standing in for torch.cuda and
libkmeranno.so. Checks the one JSON line rank 0 prints (contract keys, the joined ranks, the
table broadcast record) and the --verify parity checks (gathered outputs = one single-rank
call, reduced tally, identical replicas), for the strong (c4) and weak (c5) workloads."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("workload,rows", [("c4", 300_000), ("c5", 1_500_000)])
def test_bench_multirank_branch_rehearsal(workload, rows):
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "bench_rehearsal.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--workload", workload, "--n-seq", "300", "--table-rows", str(rows),
           "--dist-backend", "gloo", "--same-device", "--verify", "--no-extras",
           "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline"):
        assert key in out, key
    assert out["n_gpus"] == 2 and out["steps"] == 2
    assert out["scaling"] == ("strong" if workload == "c4" else "weak")
    assert [r["rank"] for r in out["ranks"]] == [0, 1]
    assert out["rank_ms_per_step_min"] <= out["rank_ms_per_step_max"]
    assert out["table_broadcast"]["ms"] is not None and out["table_broadcast"]["bytes"] > 0
    v = out["verify"]
    assert v["ok"] and v["outputs_equal_single_rank"] and v["tally_equals_single_rank"]
    assert v["table_identical_across_ranks"] and v["called"] > 0
