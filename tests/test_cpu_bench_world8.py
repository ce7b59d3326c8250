"""bench.py's default run at N = 8 -- the line the driver's first 8-GPU scaling run prints -- rehearsed on the CPU
(VERDICT r03 item 4): eight gloo ranks run ``bench.main()`` with every default ``also`` entry on the fake device
(tests/bench_fake_rank.py: the kernels restated by the oracle), the BASELINE presets shrunk so the oracle
finishes in seconds.  The line's structure is what is checked: config 3's value counts 4 K P N (weak), configs 5 and
4 split one model into eight buckets (strong), 2h / 2s / 4x are present, spot checks are summed over the ranks, and
every entry's spot check is clean.  Here the test starts the ranks (the torchrun form: WORLD_SIZE set);
tests/test_cpu_bench_spawn.py has bench.py start them itself."""

import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bench_fake_rank import small_presets  # noqa: E402

WORLD = 8
SMALL = small_presets(WORLD)
ARGS = ["--gpus", str(WORLD), "--steps", "2", "--warmup", "1", "--host-resident-params", "10001", "--spot-check", "64",
        "--cpu-baseline-s", "0.2", "--cpu-sample-params", "4096"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD), RANK=str(rank),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import contextlib
    import io

    from bench_fake_rank import install

    bench = install(rank, WORLD)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(ARGS)
    with open(os.path.join(out_dir, f"rank{rank}.out"), "w") as f:
        f.write(buf.getvalue())


def check_line(d, world=WORLD):
    """The default run's line at `world` ranks (shared with tests/test_cpu_bench_spawn.py)."""
    small = small_presets(world)
    K3, P3 = small[3]["clients"], small[3]["params"]
    assert d["n_gpus"] == world and d["scaling"] == "weak" and d["steps"] == 2
    # value = 4 K P N steps / wall: weak scaling counts every rank's own P-param bucket
    wall = d["ms_per_step"] / 1e3
    assert d["value"] == pytest.approx(4.0 * K3 * P3 * world / wall / 2**30, rel=2e-3, abs=0.006)
    assert d["spot_check"]["mismatches"] == 0 and d["spot_check"]["ranks"] == world
    assert d["spot_check"]["sampled"] >= world * 64

    def name(e):
        return e.get("baseline_config") or e["config"]["baseline_config"]

    assert len(d["also"]) == 6, [name(e) for e in d["also"]]
    assert not any("skipped" in e or "error" in e for e in d["also"]), d["also"]
    # the CPU baseline on rank 0 at every N, after the GPU entries
    cb = d["cpu_baseline"]
    assert cb is not None and "error" not in cb, cb
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["n_gpus_in_run"] == world and cb["kind"] == "port"
    # config 2 device-resident (weak): every rank its own 8 x P bucket
    c2 = next(e for e in d["also"] if e["config"].get("clients") == small[2]["clients"] and "roofline" in e)
    assert c2["scaling"] == "weak" and c2["n_gpus"] == world and c2["config"]["params_total"] == small[2]["params"] * world
    assert c2["spot_check"]["mismatches"] == 0 and c2["spot_check"]["ranks"] == world
    c5 = next(e for e in d["also"] if e["config"].get("epilogue") == "adam")
    c4 = next(e for e in d["also"] if e["config"].get("clients") == 256 and "client-sharded" not in name(e))
    for e, cfg in ((c5, small[5]), (c4, small[4])):  # strong: one model split into `world` buckets, counted once
        assert e["scaling"] == "strong" and e["n_gpus"] == world
        assert e["config"]["params_total"] == cfg["params"]
        assert e["spot_check"]["mismatches"] == 0 and e["spot_check"]["ranks"] == world
        assert e["value"] == pytest.approx(4.0 * cfg["clients"] * cfg["params"] / (e["ms_per_step"] / 1e3) / 2**30,
                                           rel=2e-3, abs=0.006)
    # the FedOpt hand-out pull (ShardedServerOptimizer._pull's device work) timed in the config-5 entry
    hp = c5["handout_pull"]
    assert hp["ms"] > 0 and hp["bytes_per_gpu_rank0"] == 4 * c5["config"]["params_per_gpu"]
    h2 = [e for e in d["also"] if "host-resident updates" in name(e)]
    s2 = [e for e in d["also"] if "ONE server process" in name(e)]
    x4 = [e for e in d["also"] if "client-sharded" in name(e)]
    assert len(h2) == len(s2) == len(x4) == 1, [name(e) for e in d["also"]]
    assert h2[0]["scaling"] == "weak" and h2[0]["spot_check"]["mismatches"] == 0 and h2[0]["spot_check"]["ranks"] == world
    assert s2[0]["scaling"] == "strong" and s2[0]["config"]["devices"] == world and s2[0]["spot_check"]["mismatches"] == 0
    assert x4[0]["spot_check"]["ranks"] == world and x4[0]["bits_equal_serial"]


@pytest.mark.timeout(600)
def test_default_run_at_eight_ranks(tmp_path):
    port = _free_port()
    mp.start_processes(_rank, args=(port, str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    outs = [open(tmp_path / f"rank{r}.out").read() for r in range(WORLD)]
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and all(not o.strip() for o in outs[1:]), outs
    check_line(json.loads(lines[0]))
