"""CPU: ``bench.py --gpus N`` starts N rank processes itself (the driver may run
it without a launcher), each with its RANK/LOCAL_RANK/WORLD_SIZE, and
``--gpus 1`` stays a single process.  ``--dry-launch`` makes every rank print
its environment and exit before importing torch or touching a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=120, env=env)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def test_gpus_n_spawns_n_ranks():
    for n in (2, 4):
        rc, lines, err = _run("--gpus", str(n), "--dry-launch")
        assert rc == 0, err
        assert sorted(x["rank"] for x in lines) == list(range(n))
        assert sorted(x["local_rank"] for x in lines) == list(range(n))
        assert {x["world_size"] for x in lines} == {n}
        assert len({x["master"] for x in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")


def test_gpus_1_is_one_process():
    rc, lines, err = _run("--gpus", "1", "--dry-launch")
    assert rc == 0, err
    assert lines == [{"rank": 0, "local_rank": 0, "world_size": 1, "master": "None:None"}]


def test_launcher_world_must_match_gpus():
    """Under torchrun (WORLD_SIZE set) a mismatched --gpus is an error, not a silent 1-GPU line."""
    rc, lines, err = _run("--gpus", "8", "--dry-launch", env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert rc == 2 and not lines and "WORLD_SIZE=2" in err


def test_failing_rank_fails_the_launch():
    rc, lines, err = _run("--gpus", "2", "--no-such-flag")
    assert rc != 0
