"""The randomised reference FedOpt rounds of tests/fuzz_reference_fedopt.py replayed on the GPU.

tests/golden/fuzz_fedopt_s31.json holds, for 60 random cases (seed 31), the REFERENCE
``PTFedOptModelShareableGenerator`` (nvflare/app_opt/pt/fedopt.py:184-270, torch CPU) output per round: the
keys in order, each value's container, dtype, shape and a SHA-256 of its bits, the lr after the step and the
meta.  Cases draw a 1-3 layer Linear model with optional biases and BatchNorm layers (fp32 running stats and
an int64 ``num_batches_tracked`` take the ``base + diff`` branch), numpy or torch containers, keys missing
from later rounds, SGD (momentum, dampening, nesterov, weight decay, maximize), Adamax, Rprop and ASGD, with or
without a StepLR schedule; tests/golden/fuzz_fedopt_sqrt_s41.json (round 3) the same for 60 cases of the
optimizers that take a sqrt (Adam, AdamW, amsgrad, maximize, NAdam, RAdam, RMSprop centered / momentum,
Adagrad).  The drop-in generator steps every parameter with the HIP kernels on cuda:0 and must give the same
bits."""

import copy
import json
import os

import numpy as np
import pytest

import fuzz_reference_fedopt as F

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("fixture,family,n_kinds", [("fuzz_fedopt_s31.json", "plain", 4),
                                                     ("fuzz_fedopt_sqrt_s41.json", "sqrt", 6)])
def test_fuzz_fedopt_cases_match_reference_on_the_gpu(fixture, family, n_kinds, monkeypatch):
    """The sqrt family (Adam, AdamW, amsgrad, NAdam, RAdam, RMSprop, Adagrad) replays with torch CPU's restated
    sqrt, the one the recording container's torch computed (nvflare_amd/torch_sqrt.py)."""
    from nvflare_amd.app_opt.pt import PTFedOptModelShareableGenerator
    from nvflare_amd.compat import (DXO, AppConstants, DataKind, EventType, FLContext, ModelLearnableKey,
                                    make_model_learnable)

    monkeypatch.setenv("NVFLARE_AMD_TORCH_SQRT", "torch_cpu")
    with open(os.path.join(HERE, "golden", fixture)) as f:
        rec = json.load(f)
    assert rec.get("family", "plain") == family
    assert rec["numpy"].split(".")[:2] == np.__version__.split(".")[:2], "the inputs regenerate only on this numpy"
    rng = np.random.default_rng(rec["seed"])
    bad, rounds, keys, kinds = [], 0, 0, set()
    for r in rec["records"]:
        spec = F.gen_case(rng, family)
        assert spec["optimizer_args"]["path"] == r["optimizer"] and spec["container"] == r["container"]
        gen = PTFedOptModelShareableGenerator(optimizer_args=copy.deepcopy(spec["optimizer_args"]),
                                              lr_scheduler_args=copy.deepcopy(spec["lr_scheduler_args"]),
                                              source_model=F.build_model(spec), device="cuda:0")
        gen.handle_event(EventType.START_RUN, FLContext())
        got = F.play(gen, spec, FLContext, AppConstants, make_model_learnable, DXO, DataKind, ModelLearnableKey)
        for rnd, (g, e) in enumerate(zip(got, r["rounds"])):
            if list(g["weights"].items()) != [(k, v) for k, v in e["weights"].items()]:
                wrong = [k for k in e["weights"] if g["weights"].get(k) != e["weights"][k]]
                bad.append(f"case {r['case']} ({r['optimizer']}, {r['container']}) round {rnd}: {wrong[:4]}")
            if g["lr"] != e["lr"] or g["meta"] != e["meta"]:
                bad.append(f"case {r['case']} round {rnd}: lr {g['lr']} vs {e['lr']}, meta {g['meta']} vs {e['meta']}")
            rounds += 1
            keys += len(g["weights"])
        kinds.add(r["optimizer"])
    assert not bad, bad[:10]
    assert rounds == 3 * len(rec["records"]) and keys > 500 and len(kinds) == n_kinds
