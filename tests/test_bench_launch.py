"""bench.py's multi-GPU launch path on CPU: `--gpus 2` without WORLD_SIZE must start two ranks
(torch.distributed.run, rendezvous on 127.0.0.1), report n_gpus == 2, one entry per rank, and a
whole-job time that is the slowest rank's (max over ranks), never rank 0's own.  --dry-run swaps
the replay for a sleep of (rank + 1) ms per step and the RCCL group for gloo."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=e, cwd=ROOT)
    return r


def test_gpus2_spawns_two_ranks_and_reports_slowest():
    r = _bench("--gpus", "2", "--dry-run", "--steps", "20", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                       # rank 0 prints exactly one JSON line
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    ranks = sorted(p["rank"] for p in res["per_rank"])
    assert ranks == [0, 1]
    slowest = max(p["seconds"] for p in res["per_rank"])
    assert abs(res["ms_per_step"] - slowest / 20 * 1e3) < 1e-3 + 1e-6 * res["ms_per_step"]
    # rank 1 sleeps 2 ms a step: the job cannot be faster than that
    assert res["ms_per_step"] >= 2.0


def test_gpus8_spawns_eight_ranks():
    """The driver's widest launch (--gpus 8, one rank per GPU of a node), dry-run on CPU."""
    r = _bench("--gpus", "8", "--dry-run", "--steps", "5", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 8 and sorted(p["rank"] for p in res["per_rank"]) == list(range(8))
    assert res["ms_per_step"] >= 8.0             # rank 7 sleeps 8 ms a step


def test_single_gpu_default_and_world_mismatch():
    r = _bench("--dry-run", "--steps", "3", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
    bad = _bench("--dry-run", "--gpus", "1", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert bad.returncode != 0 and "one rank per GPU" in (bad.stderr + bad.stdout)
