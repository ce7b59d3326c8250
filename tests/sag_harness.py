"""Minimal scatter-and-gather round loop (test infrastructure) for the config-1 known-answer test.

It drives an Aggregator exactly the way ScatterAndGather does (nvflare/app_common/workflows/
scatter_and_gather.py:224-349, :393-456): per round, every client's result goes through
``aggregator.accept`` (with the CONTRIBUTION_ROUND cookie and the client's identity as peer prop),
then ``aggregator.aggregate``, then the FullModelShareableGenerator update
(shareablegenerators/full_model_shareable_generator.py:58-75: WEIGHTS replaces, WEIGHT_DIFF adds), then
``aggregator.reset``.  Clients are NPTrainer-like (nvflare/app_common/np/np_trainer.py:114-147):
``weights["numpy_key"] += delta`` and a reply with NUM_STEPS_CURRENT_ROUND = 1.

Not a re-implementation of the workflow: no tasks, no communication, no persistence engine.
"""

from __future__ import annotations

import numpy as np

from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, MetaKey, ReservedKey, Shareable, from_shareable

NUMPY_KEY = "numpy_key"
INITIAL_MODEL = np.array([[1, 2, 3], [4, 5, 6], [7, 8, 9]], dtype=np.float32)  # np_model_persistor.py:76-84


def np_trainer(global_weights: dict, delta: float, kind: str) -> dict:
    data = {k: np.array(v, copy=True) for k, v in global_weights.items()}
    data[NUMPY_KEY] += delta
    if kind == DataKind.WEIGHT_DIFF:
        data = {k: data[k] - global_weights[k] for k in data}
    return data


def run_sag(aggregator, n_clients=2, num_rounds=3, delta=1.0, kind=DataKind.WEIGHTS, client_names=None):
    fl_ctx = FLContext()
    aggregator.handle_event(EventType.START_RUN, fl_ctx)
    model = {NUMPY_KEY: INITIAL_MODEL.copy()}
    names = client_names or [f"site-{i + 1}" for i in range(n_clients)]
    for rnd in range(num_rounds):
        fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=True)
        for name in names:
            data = np_trainer(model, delta, kind)
            s = DXO(kind, data=data, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1}).to_shareable()
            s.set_peer_props({ReservedKey.IDENTITY_NAME: name})
            s.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd)
            if not aggregator.accept(s, fl_ctx):
                raise RuntimeError(f"round {rnd}: result of {name} rejected")
        result = from_shareable(aggregator.aggregate(fl_ctx))
        if result.data_kind == DataKind.WEIGHT_DIFF:
            model = {k: model[k] + result.data[k] for k in model}
        else:
            model = dict(result.data)
        aggregator.reset(fl_ctx)
    return model, fl_ctx
