"""bench.py --gpus N without a launcher starts its own ranks (bench.spawn_ranks): a child
`torch.distributed.run` with the driver's arguments, rank 0's JSON line forwarded, the child's exit
code returned.  Runs on CPU with a stand-in rank script (no GPU is touched by the parent)."""
from __future__ import annotations

import importlib.util
import json
import os
import pathlib
import subprocess
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]

RANK_SCRIPT = r'''
import json, os, sys
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
print(f"progress from rank {rank}", flush=True)
if rank == 0:
    print(json.dumps({"metric": "m", "value": 1.0, "n_gpus": world, "argv": sys.argv[1:]}), flush=True)
sys.exit(int(os.environ.get("FAKE_RC", "0")) if rank == world - 1 else 0)
'''


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_spawn_ranks_forwards_rank0_line(tmp_path, capsys, monkeypatch):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    rc = _bench().spawn_ranks(2, str(script), ["--gpus", "2", "--steps", "3"])
    out = capsys.readouterr().out.strip().splitlines()
    assert rc == 0
    assert len(out) == 1, out  # exactly one JSON line on stdout, progress went to stderr
    line = json.loads(out[0])
    assert line["n_gpus"] == 2 and line["argv"] == ["--gpus", "2", "--steps", "3"]


def test_spawn_ranks_returns_child_rc(tmp_path, capsys, monkeypatch):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    monkeypatch.setenv("FAKE_RC", "2")
    rc = _bench().spawn_ranks(2, str(script), [])
    assert rc != 0


def test_bench_coll_refuses_without_launcher_env():
    """bench_coll.run must not guess a world from --gpus: without WORLD_SIZE / MASTER_ADDR it exits
    before any GPU call."""
    code = ("import sys, types; sys.path.insert(0, %r); import bench_coll; "
            "a = types.SimpleNamespace(gpus=2)\n"
            "try:\n    bench_coll.run(a, None, None)\nexcept SystemExit as e:\n    print('EXIT', e)\n") % str(REPO)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "MASTER_ADDR", "RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert "EXIT bench_coll needs a launcher environment" in r.stdout, r.stdout + r.stderr
