"""CPU tier for bench.py's own rank launcher.

`python bench.py --gpus N` without a launcher starts N rank processes itself
(launch_ranks: fresh interpreters, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
set as torch.distributed.run sets them).  With --stub the ranks do no GPU work:
they rendezvous over gloo, pass a barrier and take the max over ranks of a
stand-in time (0.25 * (rank + 1)), which is exactly the control plane the real
bench uses around its timed region.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_launches_n_ranks(n):
    """N = 8 is the driver's SCALE run (8 ranks, one per GPU of a node)."""
    p = _run(["--gpus", str(n), "--stub"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["stub"] and out["world"] == n
    assert out["max_over_ranks"] == pytest.approx(0.25 * n)  # the slowest rank's time
    assert sorted(r["rank"] for r in out["ranks"]) == list(range(n))
    pids = {r["pid"] for r in out["ranks"]}
    assert len(pids) == n and os.getpid() not in pids  # N separate processes


def test_bench_single_rank_stub_runs_in_process():
    p = _run(["--stub"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["world"] == 1 and out["max_over_ranks"] == pytest.approx(0.25)
