"""Randomised parity against the REFERENCE helper itself (tests/fuzz_reference_helper.py, in a subprocess with
the reference tree mounted): the drop-in WeightedAggregationHelper on the fake device -- the engine's host logic
with the kernels' per-element sequences restated by the oracle -- gives the reference's keys, key order,
containers, dtypes, shapes and bits on random rounds (client counts, partial keys, 0-d / empty / ragged /
multi-tile / 70001-element shapes, numpy and torch, float32 / float64 / float16 / bfloat16 / integer / bool,
odd weights, weigh_by_local_iter, exclude_vars, HBM budgets that force folds, small slabs, torch threads 1 and
4), and raises the reference's exception type where the reference raises.  The same for the
InTimeAccumulateWeightedAggregator on random accept sequences (single and COLLECTION DXOs, aggregation weights,
exclude_vars, wrong rounds, repeated contributors, wrong kinds, failed return codes, odd NUM_STEPS): accept's
answers, the aggregated DXO and the published stats.  Skipped where the reference tree is absent (the GPU
box)."""

import json
import os
import subprocess
import sys

import pytest

REF = os.environ.get("NVFLARE_REF_ROOT", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "nvflare")), reason="reference tree not mounted")
@pytest.mark.parametrize("mode,seed,threads", [("helper", 11, 1), ("helper", 12, 4), ("intime", 13, 2), ("fedavg", 14, 1)])
def test_random_rounds_match_reference(tmp_path, mode, seed, threads):
    env = dict(os.environ, NVFLARE_REF_ROOT=REF, PYTHONDONTWRITEBYTECODE="1")
    env.pop("NVFLARE_AMD_FORCE_STANDINS", None)
    proc = subprocess.run([sys.executable, os.path.join(HERE, "fuzz_reference_helper.py"), "--cases", "120",
                           "--seed", str(seed), "--threads", str(threads), "--mode", mode], cwd=str(tmp_path), env=env,
                          capture_output=True, text=True, timeout=600)
    line = proc.stdout.strip().splitlines()[-1] if proc.stdout.strip() else "{}"
    stats = json.loads(line)
    assert proc.returncode == 0 and stats.get("n_mismatches") == 0, (stats, proc.stderr[-2000:])
    if mode == "helper":
        assert stats["cases"] == 120 and stats["rounds"] > 150 and stats["keys"] > 400 and stats["launches"] > 0
    elif mode == "intime":
        assert stats["cases"] == 120 and stats["aggregates"] > 150 and stats["rejected"] > 100
    else:
        assert stats["cases"] == 120 and stats["accepted"] > 200


@pytest.mark.parametrize("fixture,family", [("fuzz_fedopt_s31.json", "plain"), ("fuzz_fedopt_sqrt_s41.json", "sqrt")])
def test_recorded_fedopt_cases_regenerate(fixture, family):
    """tests/golden/fuzz_fedopt_s31.json's (and the sqrt family's fuzz_fedopt_sqrt_s41.json) inputs regenerate from
    the seed here: each case's optimizer, container and per-round key sets (the reference's outputs carry every
    state key, the rounds' diffs a subset) come out of fuzz_reference_fedopt.gen_case as recorded."""
    import numpy as np

    import fuzz_reference_fedopt as F

    with open(os.path.join(HERE, "golden", fixture)) as f:
        rec = json.load(f)
    assert rec.get("family", "plain") == family
    rng = np.random.default_rng(rec["seed"])
    n_missing = 0
    for r in rec["records"]:
        spec = F.gen_case(rng, family)
        assert spec["optimizer_args"]["path"] == r["optimizer"] and spec["container"] == r["container"]
        state_keys = list(F.build_model(spec).state_dict())
        for diff, exp in zip(spec["rounds"], r["rounds"]):
            assert list(exp["weights"]) == state_keys
            n_missing += len(state_keys) - len(diff)
    assert n_missing > 10


def test_recorded_reference_rounds_replay_on_the_fake_device(monkeypatch):
    """tests/golden/fuzz_helper_s21.json (the reference's result hashes for 200 random cases) replayed through
    the drop-in on the fake device -- the same check tests/test_gpu_fuzz_replay.py runs on the MI355X; this one
    needs no reference tree."""
    import test_gpu_fuzz_replay as replay
    from fake_device import FakeDeviceContext
    from nvflare_amd.device import DeviceContext

    fake = FakeDeviceContext()
    monkeypatch.setattr(DeviceContext, "get", classmethod(lambda cls, d=None: fake))
    replay.test_fuzz_cases_match_reference_on_the_gpu(monkeypatch)
