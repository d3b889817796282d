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


def test_report_helpers_cpu():
    """The bench line's compute roofline and the NumPy-subsample and config-2 CPU legs (CPU only)."""
    import importlib.util
    import numpy as np
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r = bench.compute_roofline(100_000_000, 1024, 3, 2.5, 0.2)
    assert r["flop_per_point_candidate"] == 10 and abs(r["achieved"] - 1e8 * 2.5 * 10 / 2e-4 / 1e12) < 1e-9
    assert r["compute_frac"] == r["achieved"] / bench.FP32_PEAK_TFLOPS and r["bruteforce_equivalent"] > r["achieved"]
    assert bench.compute_roofline(10, 4, 3, 1.0, 0.0) is None
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(20_000, 3, 5)
    C = X[R.init_indices(20_000, 16)]
    nb = bench.numpy_baseline(X, C, budget_s=0.02)
    assert nb["value"] > 0 and nb["kind"] == "port" and "NumPy" in nb["sample"]
    cb, ref = bench.cpu_fit_baseline(X, C, 5)
    assert cb["value"] > 0 and ref["n_iter"] <= 5 and ref["labels"].shape == (20_000,)
