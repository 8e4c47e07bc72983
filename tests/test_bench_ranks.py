"""bench.py starts its own ranks for `--gpus N` when no launcher did (one process
per GPU), and refuses a `--gpus` that disagrees with the launcher's WORLD_SIZE. CPU only: the
spawned ranks join a gloo process group and all-reduce their ids (--spawn-check), which is the
same rank start-up and rendezvous the GPU run goes through before it touches a device."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd="/tmp", env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_starts_its_own_ranks():
    for world in (2, 3):
        p = _run(["--gpus", str(world), "--spawn-check"], {"KPE_DIST_BACKEND": "gloo"})
        assert p.returncode == 0, p.stderr[-2000:]
        line = [l for l in p.stdout.splitlines() if l.startswith("{")]
        assert len(line) == 1, p.stdout  # rank 0 alone prints
        d = json.loads(line[0])
        assert d["n_gpus"] == world and d["rank_sum"] == world * (world - 1) // 2


def test_bench_refuses_gpus_launcher_mismatch():
    p = _run(["--gpus", "3"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0
    assert "--gpus 3" in p.stderr and "WORLD_SIZE=2" in p.stderr


def test_bench_rejects_zero_gpus():
    p = _run(["--gpus", "0"])
    assert p.returncode != 0 and "--gpus" in p.stderr
