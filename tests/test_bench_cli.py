"""bench.py's argument refusals (CPU: no GPU needed).  A multi-GPU request the machine cannot
serve must exit non-zero with the reason, never run on fewer GPUs and print a line."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True,
                          timeout=300, cwd=str(REPO), env=env)


def test_more_gpus_than_visible_is_refused():
    import torch

    n = torch.cuda.device_count()
    r = _bench(["--gpus", str(n + 1), "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert f"--gpus {n + 1} but only {n} GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE 3" in r.stderr


def test_torch_comm_needs_a_launcher():
    import torch

    if torch.cuda.device_count() >= 2:
        r = _bench(["--gpus", "2", "--comm", "torch", "--steps", "1"])
        assert r.returncode != 0 and "needs one process per GPU" in r.stderr


def test_bench_help_lists_the_paths():
    r = _bench(["--help"])
    assert r.returncode == 0
    for flag in ("--allow-fallback", "--share-gpu", "--gather", "--no-rccl-leg", "c3b"):
        assert flag in r.stdout
