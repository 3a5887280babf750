"""bench.py's own rank launcher (CPU, gloo): ``--gpus N`` without torch.distributed.run
starts N rank processes, each sees WORLD_SIZE == N, rank 0 prints the line, and a
failing rank makes the launcher exit non-zero.  No GPU is touched (--launch-check)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_brings_up_n_ranks(n):
    p = _run(["--gpus", str(n), "--launch-check", "1", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == n
    assert sorted(map(tuple, lines[0]["ranks"])) == [(r, n) for r in range(n)]
    # the per-rank records the N > 1 bench line carries, one per rank in rank order
    pr = lines[0]["per_rank"]
    assert [r["rank"] for r in pr] == list(range(n))
    assert all(set(r) == {"rank", "wall_s", "windows", "tokens", "global_max_s", "gather_s"} for r in pr)
    assert "RCCL all-reduce(max)" in lines[0]["parallelism"]


def test_launcher_single_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--launch-check", "1", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 1 and line["ranks"] == [[0, 1]] and "per_rank" not in line
    assert "no collective" in line["parallelism"]


def test_launcher_balance_tokens_label():
    p = _run(["--gpus", "2", "--launch-check", "1", "--backend", "gloo", "--balance", "tokens"])
    assert p.returncode == 0, p.stderr
    (line,) = _json_lines(p.stdout)
    assert "every 2-th clip" in line["parallelism"]


def test_launcher_fails_when_a_rank_fails():
    p = _run(["--gpus", "2", "--launch-check", "1", "--backend", "no-such-backend"])
    assert p.returncode != 0
    assert "rank(s) failed" in p.stderr


def test_world_must_match_gpus():
    # an external launcher's world size that disagrees with --gpus is refused
    p = _run(["--gpus", "1", "--launch-check", "1", "--backend", "gloo"],
             env_extra=dict(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999"))
    assert p.returncode != 0
    assert "WORLD_SIZE 2" in p.stderr


def test_launcher_ends_survivors_when_a_rank_dies_mid_collective():
    # rank 1 exits 3 after init_process_group while rank 0 waits in an all-gather for it:
    # the launcher must notice, terminate rank 0 and exit non-zero well inside 60 s
    # (the collective's own timeout is set far beyond that, so only the launcher can end it)
    import time
    t0 = time.monotonic()
    p = _run(["--gpus", "2", "--launch-check", "1", "--backend", "gloo", "--launch-check-fail-rank", "1",
              "--dist-timeout", "600"], timeout=120)
    dt = time.monotonic() - t0
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "rank 1 failed with exit code 3" in p.stderr
    assert dt < 60, dt
    assert _json_lines(p.stdout) == []
