"""bench.py --gpus N outside a torch.distributed launch starts N ranks itself
(VERDICT r03 missing #2): one process per rank through torch.distributed.run,
started before anything touches the GPU, rank 0 printing the one JSON line
with n_gpus = N and every rank's time.  --dry-run runs exactly that rank /
barrier / max-over-ranks path over gloo with a no-op step (no device here)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=240, cwd="/tmp")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return lines


def test_bench_gpus2_launches_two_ranks_one_line():
    lines = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"])
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and len(d["rank_ms_per_step"]) == 2
    ranks = sorted(r for r, _ in d["rank_pids"])
    pids = {p for _, p in d["rank_pids"]}
    assert ranks == [0, 1] and len(pids) == 2
    assert d["ms_per_step"] == max(d["rank_ms_per_step"])


def test_bench_gpus1_stays_in_process():
    d = json.loads(_run(["--dry-run", "--steps", "1", "--warmup", "0"])[0])
    assert d["n_gpus"] == 1 and len(d["rank_pids"]) == 1
