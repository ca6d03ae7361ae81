"""bench.py --gpus N starts N ranks or fails (CPU, gloo; no GPU use).

The driver runs ``python bench.py --gpus N`` under torch.distributed.run; a
plain ``python bench.py --gpus N`` must start the N ranks itself (one child
torch.distributed.run process, rendezvous on 127.0.0.1) and a WORLD_SIZE that
disagrees with --gpus must fail instead of silently measuring another size."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(kw)
    return env


def _lines(out):
    res = []
    for ln in out.splitlines():
        ln = ln.strip()
        while ln.startswith("{"):
            end = ln.index("}") + 1
            res.append(json.loads(ln[:end]))
            ln = ln[end:].strip()
    return res


def test_gpus_2_starts_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    recs = _lines(p.stdout)
    assert sorted(r["rank"] for r in recs) == [0, 1]
    assert all(r["world_size"] == 2 and r["ranks_seen"] == 2 and r["gpus"] == 2 for r in recs)


def test_gpus_1_is_one_process():
    p = subprocess.run([sys.executable, BENCH, "--launch-check"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert _lines(p.stdout) == [{"rank": 0, "world_size": 1, "ranks_seen": 1, "gpus": 1}]


def test_world_size_mismatch_fails():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-check"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in p.stderr
