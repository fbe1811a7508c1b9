"""bench.py --gpus N and the process layout, on CPU: without a launcher
--gpus 2 starts 2 ranks itself; under a launcher whose WORLD_SIZE differs from --gpus the bench
refuses to run.  --ranks-probe stops after the gloo rendezvous, so no GPU is needed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT", "GSA_BENCH_REHEARSE")}
    env.update(kw)
    return env


def _run(args, **kw):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=_env(**kw),
                          capture_output=True, text=True, timeout=240)


def _line(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_gpus2_without_launcher_starts_two_ranks():
    r = _run(["--gpus", "2", "--ranks-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _line(r.stdout)
    assert j["world"] == 2 and sorted(j["ranks"]) == [0, 1] and j["processes"] == 2
    assert j["n_gpus"] == 2


def test_gpus1_is_one_rank():
    r = _run(["--ranks-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _line(r.stdout)
    assert j["world"] == 1 and j["n_gpus"] == 1 and j["ranks"] == [0]


def test_launcher_world_mismatch_exits_nonzero():
    r = _run(["--gpus", "8", "--ranks-probe"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
    assert not r.stdout.strip()


def test_bad_gpus_count():
    r = _run(["--gpus", "0", "--ranks-probe"])
    assert r.returncode == 2
