"""``python bench.py --gpus 8`` WITHOUT torchrun: bench.main() must start the eight rank processes
itself (bench.launch_ranks), before anything touches a GPU, and print rank 0's one JSON line -- not a 1-GPU line
labelled with whatever WORLD_SIZE happened to be.  The ranks run bench.py's flow on the fake device
(tests/bench_fake_rank.py as the rank script, NVFLARE_AMD_BENCH_WORKER_SCRIPT); the line is checked as the torchrun
rehearsal checks it (tests/test_cpu_bench_world8.py).  A rank that fails or hangs ends the run with a non-zero exit."""

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import bench  # noqa: E402
from test_cpu_bench_world8 import ARGS, WORLD, check_line  # noqa: E402


@pytest.fixture
def no_world(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


@pytest.mark.timeout(600)
def test_gpus_8_without_torchrun_starts_eight_ranks(no_world, capfd):
    no_world.setenv("NVFLARE_AMD_BENCH_WORKER_SCRIPT", os.path.join(ROOT, "tests", "bench_fake_rank.py"))
    bench.main(ARGS)
    out = capfd.readouterr().out
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out  # rank 0's line and nothing else on stdout
    d = json.loads(lines[0])
    check_line(d, WORLD)
    assert d["n_gpus"] == 8 and d["spot_check"]["ranks"] == 8


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text("import os, sys, time\nrank = int(os.environ['RANK'])\n" + body)
    return str(p)


@pytest.mark.timeout(120)
def test_a_failing_rank_fails_the_run(no_world, tmp_path, capfd):
    # rank 2 fails at once; the others would wait forever in a collective: they are killed after the grace period
    no_world.setattr(bench, "RANK_GRACE_S", 2.0)
    no_world.setenv("NVFLARE_AMD_BENCH_WORKER_SCRIPT",
                    _script(tmp_path, "if rank == 2:\n    sys.exit(7)\ntime.sleep(600)\n"))
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4"])
    assert e.value.code == 7


@pytest.mark.timeout(120)
def test_hung_ranks_are_killed_at_the_limit(no_world, tmp_path):
    no_world.setenv("NVFLARE_AMD_BENCH_WORKER_SCRIPT", _script(tmp_path, "time.sleep(600)\n"))
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2", "--rank-timeout-s", "3"])
    assert e.value.code == 124


@pytest.mark.timeout(120)
def test_ranks_see_the_torchrun_environment(no_world, tmp_path, capfd):
    no_world.setenv("NVFLARE_AMD_BENCH_WORKER_SCRIPT", _script(
        tmp_path,
        "import json\n"
        "env = {k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}\n"
        "print(json.dumps(env) if rank == 0 else 'not on stdout')\n"
        "print('rank', rank, 'argv', sys.argv[1:], file=sys.stderr)\n"))
    bench.main(["--gpus", "3", "--steps", "4"])
    cap = capfd.readouterr()
    lines = [ln for ln in cap.out.splitlines() if ln.strip()]
    assert len(lines) == 1
    env = json.loads(lines[0])
    assert env["WORLD_SIZE"] == "3" and env["RANK"] == env["LOCAL_RANK"] == "0" and env["MASTER_ADDR"] == "127.0.0.1"
    assert "[rank 2] not on stdout" in cap.err and "'--steps', '4'" in cap.err


@pytest.mark.timeout(120)
def test_ranks_die_with_the_launcher(no_world, tmp_path):
    """The driver's time limit kills the launcher (SIGTERM, or SIGKILL): no rank may keep running on a GPU after it."""
    import signal
    import subprocess
    import time

    pids = tmp_path / "pids"
    pids.mkdir()
    script = _script(tmp_path, f"open(os.path.join({str(pids)!r}, str(os.getpid())), 'w').close()\ntime.sleep(600)\n")
    env = dict(os.environ, NVFLARE_AMD_BENCH_WORKER_SCRIPT=script)
    for sig in (signal.SIGTERM, signal.SIGKILL):
        for f in pids.iterdir():
            f.unlink()
        launcher = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                                    stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        deadline = time.time() + 60
        while len(list(pids.iterdir())) < 3 and time.time() < deadline:
            time.sleep(0.1)
        ranks = [int(f.name) for f in pids.iterdir()]
        assert len(ranks) == 3
        launcher.send_signal(sig)
        launcher.wait(timeout=30)
        def running(pid):
            try:
                with open(f"/proc/{pid}/status") as f:
                    return "zombie" not in f.read().lower()
            except OSError:
                return False

        deadline = time.time() + 10
        alive = ranks
        while alive and time.time() < deadline:
            alive = [p for p in ranks if running(p)]
            time.sleep(0.1)
        assert not alive, (sig, alive)
