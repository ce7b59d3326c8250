"""The randomised reference rounds of tests/fuzz_reference_helper.py replayed on the GPU (the real kernels).

tests/golden/fuzz_helper_s21.json holds, for 200 random helper cases (seed 21, torch at 4 threads), the
REFERENCE helper's result per round -- keys in order, container, dtype, shape and a SHA-256 of the bits (NaNs
canonicalised) -- or the exception type it raised.  Every third case runs the drop-in with deferred results,
every fifth sharded over three parameter buckets (fuzz_reference_helper.dropin_variant).  The inputs are not stored: the same generator regenerates
them from the seed here (numpy's generator is bit-stable for a given version).  The drop-in helper on the
MI355X must give the same keys, containers, dtypes, shapes and bits, and the same exception types."""

import json
import os

import numpy as np
import pytest
import torch

import fuzz_reference_helper as F

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fuzz_cases_match_reference_on_the_gpu(monkeypatch):
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    with open(os.path.join(HERE, "golden", "fuzz_helper_s21.json")) as f:
        rec = json.load(f)
    assert rec["numpy"].split(".")[:2] == np.__version__.split(".")[:2], "the inputs regenerate only on this numpy"
    old = torch.get_num_threads()
    torch.set_num_threads(rec["threads"])
    rng = np.random.default_rng(rec["seed"])
    bad, rounds, keys = [], 0, 0
    try:
        for r in rec["records"]:
            spec = F.gen_helper_case(rng, rec["big"])
            if spec["slots"]:
                monkeypatch.setenv("NVFLARE_AMD_SLAB_SLOTS", spec["slots"])
            else:
                monkeypatch.delenv("NVFLARE_AMD_SLAB_SLOTS", raising=False)
            h = WeightedAggregationHelper(exclude_vars=spec["exclude"], weigh_by_local_iter=spec["weigh"],
                                          max_resident_bytes=spec["budget"], **F.dropin_variant(r["case"]))
            for rnd, exp in enumerate(r["rounds"]):
                res, err = F.play_helper_case(h, spec, rnd)
                if "error" in exp:
                    if err is None or type(err).__name__ != exp["error"]:
                        bad.append(f"case {r['case']} round {rnd}: {err!r}, reference raised {exp['error']}")
                    break
                if err is not None:
                    bad.append(f"case {r['case']} round {rnd}: raised {err!r}")
                    break
                got = F.describe_result(res)
                if got != exp["keys"]:
                    bad.append(f"case {r['case']} round {rnd}: {got} vs {exp['keys']}")
                rounds += 1
                keys += len(got)
    finally:
        torch.set_num_threads(old)
    assert not bad, bad[:10]
    assert rounds > 300 and keys > 800
