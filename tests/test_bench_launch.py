"""bench.py's own multi-rank launcher (`bench.py --gpus N` with no torch.distributed.run around it).

The driver runs `python bench.py --gpus N`; the parent must start N ranks itself without touching
the GPU, relay rank 0's JSON line and fail when any rank fails. AIMET_BENCH_LAUNCH_CHECK makes each
rank form the process group exactly as the bench does and report it, with no GPU work, so this runs
on the CPU over gloo."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(n, check="1", extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(AIMET_BENCH_BACKEND="gloo", AIMET_BENCH_LAUNCH_CHECK=check, CUDA_VISIBLE_DEVICES="")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, BENCH, "--gpus", str(n)], env=env, capture_output=True, text=True,
                          timeout=180)


def test_launcher_forms_two_ranks_over_gloo():
    p = _run(2)
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout      # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec == {"launch_check": True, "n_gpus": 2, "dist_backend": "gloo", "rank_sum": 3}


def test_launcher_forms_four_ranks_over_gloo():
    p = _run(4)
    assert p.returncode == 0, p.stderr
    rec = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert rec["n_gpus"] == 4 and rec["rank_sum"] == 10


def test_launcher_fails_when_a_rank_fails():
    p = _run(2, check="fail1")
    assert p.returncode != 0
    assert "rank 1 exited with 3" in p.stderr


def test_world_size_must_match_gpus():
    env = dict(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    full = {k: v for k, v in os.environ.items()}
    full.update(env)
    full.pop("AIMET_BENCH_LAUNCH_CHECK", None)
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=full, capture_output=True, text=True, timeout=180)
    assert p.returncode != 0
    assert "--gpus 1 but the launcher formed WORLD_SIZE=2" in p.stderr
