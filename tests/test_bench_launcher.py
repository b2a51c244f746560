"""bench.py's multi-rank launcher on CPU (gloo): `python bench.py --gpus N` outside torchrun starts the
N ranks itself as a child torch.distributed.run and relays rank 0's JSON line; under torchrun
`--gpus` must equal WORLD_SIZE.  The `--dry-run` step is a CPU stand-in, so no GPU is touched."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          env=e, timeout=timeout, cwd="/tmp")


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "4", "--warmup", "1", "--batch", "3"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 6
    # whole-job value = B * N * steps / elapsed (max over ranks)
    assert abs(d["value"] - 3 * 2 * 4 / d["elapsed_s"]) <= 1e-6 * d["value"]
    assert "launching 2 ranks" in r.stderr


def test_single_rank_runs_in_process():
    r = _run(["--dry-run", "--steps", "2", "--warmup", "0", "--batch", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and "launching" not in r.stderr


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
