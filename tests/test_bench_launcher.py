"""bench.py's multi-rank launcher and argument plumbing on CPU:
`--gpus 2` from a plain `python bench.py` starts two ranks under torch.distributed.run (gloo with
--dry-run), the ranks time the same barrier-bracketed steps, take the max over ranks, and rank 0
prints one JSON line whose n_gpus is the process group's size."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus_2_launches_two_ranks_and_reports_the_group_size():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "3"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout            # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["dry_run"] is True
    assert line["config"]["global_batch"] == 6 and line["config"]["parallelism"] == "dp2"
    assert line["steps"] == 3 and line["value"] > 0


def test_single_rank_default_needs_no_launcher():
    r = _run(["--dry-run", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_lines(r.stdout)[0]["n_gpus"] == 1


def test_gpus_must_match_an_outer_launch():
    r = _run(["--gpus", "2", "--dry-run"], env_extra=dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE 1" in r.stderr
