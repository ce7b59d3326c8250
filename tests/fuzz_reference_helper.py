"""Randomised parity of the drop-in ``WeightedAggregationHelper`` against the REFERENCE helper itself --
TEST INFRASTRUCTURE, run as a subprocess by tests/test_cpu_fuzz_reference.py in the build container (the
reference tree mounted at NVFLARE_REF_ROOT; nothing of it is copied).

The reference helper (weighted_aggregation_helper.py:117-240, imported through the same namespace shim as
tests/ref_suite_plugin.py) and the drop-in helper on tests/fake_device.FakeDeviceContext (the kernels'
per-element sequences restated by the oracle) get the same random contributions: client counts, key subsets
per client, 0-d / empty / ragged / tile-crossing shapes, numpy and torch containers, float32 / float64 /
float16 / bfloat16 / integer / bool values, odd weights, ``weigh_by_local_iter``, ``exclude_vars``, tiny HBM
budgets (folding) and small slabs (chaining), two rounds per helper.  Every result must match the reference's:
keys and their order, container, dtype, shape and bits (NaN payloads aside).

  python tests/fuzz_reference_helper.py --cases 300 --seed 1
"""

import argparse
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def _setup():
    from ref_suite_plugin import _install_shim

    _install_shim(os.environ["NVFLARE_REF_ROOT"])
    import nvflare_amd.compat as compat
    import nvflare_amd.device as device
    from fake_device import FakeDeviceContext

    assert compat.HAVE_NVFLARE
    fake = FakeDeviceContext()
    device.DeviceContext.get = classmethod(lambda cls, d=None: fake)
    from nvflare.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper as Ref

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper as Mine

    return Ref, Mine, fake


SHAPES = [(), (0,), (1,), (3,), (7, 5), (4095,), (4096,), (4097,), (2, 4100), (9000,), (70001,)]
NP_DTYPES = ["float32", "float32", "float32", "float64", "float16", "int32", "int64", "uint8", "bool"]
TORCH_DTYPES = ["float32", "float32", "float32", "float64", "float16", "bfloat16", "int32", "int64", "bool"]


def _value(rng, shape, dt, container):
    import torch

    if dt == "bool":
        a = rng.random(shape) < 0.5
    elif dt in ("int32", "int64", "uint8"):
        lo = 0 if dt == "uint8" else -1000
        a = rng.integers(lo, 1000 if dt != "uint8" else 256, size=shape).astype(dt)
    else:
        a = rng.standard_normal(shape) * float(rng.choice([1.0, 1e-3, 1e3]))
        if rng.random() < 0.2 and a.size:
            flat = a.reshape(-1)
            flat[rng.integers(0, flat.size)] = rng.choice([0.0, -0.0, 1e-40, np.inf, -np.inf, np.nan, 6e4])
        a = a.astype("float32" if dt == "bfloat16" else dt)
    if container == "torch":
        t = torch.from_numpy(np.array(a, copy=True))
        return t.to(torch.bfloat16) if dt == "bfloat16" else t
    return np.array(a, copy=True)


def _weight(rng, wtype=float):
    """One weight; ``wtype`` is the case's weight type: python float, or a numpy scalar type (NEP 50: it then
    sets the result dtype -- a round mixing both changes a key's dtype mid-round, a documented gap)."""
    kind = rng.integers(0, 5)
    if kind == 0:
        w = float(rng.integers(1, 100))
    elif kind == 1:
        w = float(rng.random() * 10)
    elif kind == 2:
        w = float(rng.choice([1e-6, 0.5, 3.0, 1e6, 0.0]))
    else:
        w = float(rng.random()) * float(rng.integers(1, 50))
    return wtype(w)


def _copy(v):
    import torch

    return v.clone() if isinstance(v, torch.Tensor) else np.array(v, copy=True)


def _same(a, b) -> str:
    import torch

    if type(a) is not type(b) and not (isinstance(a, np.generic) or isinstance(b, np.generic)):
        if not (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor)):
            return f"type {type(a).__name__} vs {type(b).__name__}"
    if isinstance(a, torch.Tensor):
        if a.dtype != b.dtype or tuple(a.shape) != tuple(b.shape):
            return f"torch {a.dtype}{tuple(a.shape)} vs {b.dtype}{tuple(b.shape)}"
        if a.dtype == torch.bfloat16:  # bits as int16, NaNs (any payload) from the float values
            an, bn = torch.isnan(a).numpy(), torch.isnan(b).numpy()
            if not np.array_equal(an, bn):
                return "nan positions"
            a, b = a.view(torch.int16).numpy()[~an], b.view(torch.int16).numpy()[~bn]
        else:
            a, b = a.numpy(), b.numpy()
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype != b.dtype or a.shape != b.shape:
        return f"numpy {a.dtype}{a.shape} vs {b.dtype}{b.shape}"
    if a.dtype.kind == "f":
        an, bn = np.isnan(a), np.isnan(b)
        if not np.array_equal(an, bn):
            return "nan positions"
        a, b = a[~an], b[~bn]
    fa, fb = a.reshape(-1), b.reshape(-1)
    if not np.array_equal(fa.view(np.uint8), fb.view(np.uint8)):
        diff = np.nonzero(fa != fb)[0] if fa.dtype.kind != "b" else np.nonzero(fa ^ fb)[0]
        i = int(diff[0]) if diff.size else -1
        return f"bits ({diff.size} of {fa.size} differ; first at {i}: {fa[i]!r} vs {fb[i]!r})"
    return ""


def gen_helper_case(rng, big: bool = True) -> dict:
    """One random helper case, every input drawn up front (replayable from the seed without the reference)."""
    container = "torch" if rng.random() < 0.5 else "numpy"
    shapes = SHAPES if big else SHAPES[:-1]
    keys = {}
    for j in range(int(rng.integers(1, 6))):
        dt = str(rng.choice(TORCH_DTYPES if container == "torch" else NP_DTYPES))
        keys[f"layer{j}.{dt}"] = (shapes[int(rng.integers(0, len(shapes)))], dt)
    weigh = bool(rng.random() < 0.85)
    wtype = [float, np.float64, np.float32][int(rng.integers(0, 3))] if weigh and rng.random() < 0.3 else float
    exclude = str(rng.choice(["", "layer1", "bool|int"])) if rng.random() < 0.3 else None
    budget = int(rng.choice([0, 1, 50_000])) if rng.random() < 0.3 else None
    slots = str(int(rng.choice([2, 3]))) if rng.random() < 0.3 else None
    rounds = []
    for _ in range(2):
        contribs = []
        for k in range(int(rng.integers(1, 13))):
            data = {n: _value(rng, s, dt, container) for n, (s, dt) in keys.items() if rng.random() < 0.8}
            contribs.append((data, _weight(rng, wtype), f"c{k}"))
        rounds.append(contribs)
    return dict(container=container, weigh=weigh, exclude=exclude, budget=budget, slots=slots, rounds=rounds)


def play_helper_case(helper, spec, rnd: int):
    """Feed one round to a helper: (results, None) or (None, exception) -- the first exception ends the case.
    Deferred values (a drop-in helper with defer_result=True) are materialised here, as a consumer would."""
    try:
        for data, w, name in spec["rounds"][rnd]:
            helper.add(data={n: _copy(v) for n, v in data.items()}, weight=w, contributor_name=name,
                       contribution_round=rnd)
        res = helper.get_result()
        return {k: (v.materialize() if hasattr(v, "materialize") and hasattr(v, "container") else v)
                for k, v in res.items()}, None
    except Exception as e:  # e.g. torch refusing alpha=1e6 for a float16 total, div_ on an integer total
        return None, e


def dropin_variant(case: int) -> dict:
    """Drop-in constructor options by case index (no RNG draw, so recorded seeds stay valid): every third case
    defers its fp32 results (DeferredAggregate, materialised by the consumer), every fifth splits every key
    into three parameter buckets (ShardedFedAvg, three engines on one device)."""
    return dict(defer_result=case % 3 == 1, devices=[0, 0, 0] if case % 5 == 2 else None)


def _canonical_bytes(v) -> bytes:
    """A result's bits with every NaN replaced by one canonical NaN (payloads are unspecified)."""
    import torch

    if isinstance(v, torch.Tensor):
        if v.dtype == torch.bfloat16:
            bits = v.view(torch.int16).numpy().copy()
            bits[torch.isnan(v).numpy()] = 0x7FC0
            return bits.tobytes()
        v = v.numpy()
    a = np.array(np.asarray(v), copy=True)
    if a.dtype.kind == "f":
        a[np.isnan(a)] = np.nan
    return a.tobytes()


def describe_result(res) -> list:
    """[(key, container, dtype, shape, sha256 of the canonical bits)] in result order."""
    import hashlib

    import torch

    out = []
    for k, v in res.items():
        if isinstance(v, torch.Tensor):
            cont, dt, shape = "torch", str(v.dtype).replace("torch.", ""), list(v.shape)
        else:
            cont, dt, shape = "numpy", str(np.asarray(v).dtype), list(np.asarray(v).shape)
        out.append([k, cont, dt, shape, hashlib.sha256(_canonical_bytes(v)).hexdigest()])
    return out


def run(cases: int, seed: int, threads: int, record=None, big: bool = True) -> dict:
    import torch

    torch.set_num_threads(threads)  # torch's 16-bit add_ splits tensors of 32768+ elements over the threads
    Ref, Mine, fake = _setup()
    rng = np.random.default_rng(seed)
    stats = {"cases": 0, "rounds": 0, "keys": 0, "errors": 0, "mismatches": [], "launches": 0}
    for case in range(cases):
        spec = gen_helper_case(rng, big)
        if spec["slots"]:
            os.environ["NVFLARE_AMD_SLAB_SLOTS"] = spec["slots"]
        else:
            os.environ.pop("NVFLARE_AMD_SLAB_SLOTS", None)
        ref = Ref(exclude_vars=spec["exclude"], weigh_by_local_iter=spec["weigh"])
        mine = Mine(exclude_vars=spec["exclude"], weigh_by_local_iter=spec["weigh"], max_resident_bytes=spec["budget"],
                    **dropin_variant(case))
        rec = []
        for rnd in range(2):
            tag = (f"case {case} round {rnd} ({spec['container']}, weigh={spec['weigh']}, exclude={spec['exclude']!r}, "
                   f"budget={spec['budget']}, slots={spec['slots']})")
            r_ref, e_ref = play_helper_case(ref, spec, rnd)
            r_mine, e_mine = play_helper_case(mine, spec, rnd)
            if e_ref is not None or e_mine is not None:
                if type(e_ref) is not type(e_mine):
                    stats["mismatches"].append(f"{tag}: drop-in raised {e_mine!r}, reference {e_ref!r}")
                stats["errors"] += 1
                rec.append({"error": type(e_ref).__name__ if e_ref is not None else None})
                break  # the reference fails part-way through a contribution: states differ from here
            rec.append({"keys": describe_result(r_ref)})
            if list(r_ref) != list(r_mine):
                stats["mismatches"].append(f"{tag}: keys {list(r_ref)} vs {list(r_mine)}")
                continue
            for n in r_ref:
                why = _same(r_ref[n], r_mine[n])
                if why:
                    stats["mismatches"].append(f"{tag} key {n}: {why}")
            stats["keys"] += len(r_ref)
            stats["rounds"] += 1
        if record is not None:
            record.append({"case": case, "slots": spec["slots"], "budget": spec["budget"], "rounds": rec})
        stats["cases"] += 1
    stats["launches"] = len(fake.launches)
    return stats


def _intime_classes():
    from nvflare.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator as R

    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import (
        InTimeAccumulateWeightedAggregator as M,
    )

    return R, M


def _same_dxo(a, b, tag, out):
    """Compare two DXOs (data kind, meta, data; COLLECTION recursively)."""
    if a.data_kind != b.data_kind:
        out.append(f"{tag}: kind {a.data_kind} vs {b.data_kind}")
        return
    ma, mb = dict(a.meta or {}), dict(b.meta or {})
    if set(ma) != set(mb) or any(repr(ma[k]) != repr(mb[k]) for k in ma):
        out.append(f"{tag}: meta {ma} vs {mb}")
    if a.data_kind == "COLLECTION":
        if set(a.data) != set(b.data):
            out.append(f"{tag}: collection keys {sorted(a.data)} vs {sorted(b.data)}")
            return
        for k in a.data:
            _same_dxo(a.data[k], b.data[k], f"{tag}/{k}", out)
        return
    if list(a.data) != list(b.data):
        out.append(f"{tag}: keys {list(a.data)} vs {list(b.data)}")
        return
    for k in a.data:
        why = _same(a.data[k], b.data[k])
        if why:
            out.append(f"{tag} key {k}: {why}")


def run_intime(cases: int, seed: int) -> dict:
    """InTimeAccumulateWeightedAggregator (intime_accumulate_model_aggregator.py:47-288 with dxo_aggregator.py:
    71-191) against the reference on random accept sequences: single and COLLECTION DXOs, per-client and
    per-DXO aggregation weights, exclude_vars, weigh_by_local_iter, contributions from a wrong round, repeated
    contributors, wrong data kinds, failed return codes, missing / odd NUM_STEPS, missing sub-DXOs; accept's
    return values, the aggregated DXO and the published AGGREGATION_STATS must match, over two rounds."""
    from nvflare.apis.dxo import DXO, DataKind, MetaKey, from_shareable
    from nvflare.apis.fl_constant import ReservedKey, ReturnCode
    from nvflare.apis.fl_context import FLContext
    from nvflare.apis.shareable import Shareable
    from nvflare.app_common.app_constant import AppConstants

    R, M = _intime_classes()
    rng = np.random.default_rng(seed)
    stats = {"cases": 0, "accepts": 0, "rejected": 0, "aggregates": 0, "mismatches": [], "errors": 0}
    for case in range(cases):
        container = "torch" if rng.random() < 0.4 else "numpy"
        collection = rng.random() < 0.35
        subkeys = ["dxo_a", "dxo_b"] if collection else [""]
        kinds = {k: [DataKind.WEIGHT_DIFF, DataKind.WEIGHTS][int(rng.integers(0, 2))] for k in subkeys}
        edk = kinds if collection else kinds[""]
        names = [f"site-{i}" for i in range(int(rng.integers(1, 7)))]
        aw = None
        if rng.random() < 0.5:
            per = {n: float(rng.random() * 3) for n in names if rng.random() < 0.8}
            aw = {k: dict(per) for k in subkeys} if collection and rng.random() < 0.5 else per
        ex = None
        if rng.random() < 0.3:
            ex = {k: str(rng.choice(["", "bias", "w1"])) for k in subkeys} if collection else "bias"
        weigh = bool(rng.random() < 0.85)
        keys = {"w0": (int(rng.integers(1, 5000)),), "w1": (3, 7), "bias": (5,)}
        vdt = str(rng.choice(["float32", "float32", "float64", "float16"] + (["bfloat16"] if container == "torch" else [])))
        kw = dict(exclude_vars=ex, aggregation_weights=aw, expected_data_kind=edk, weigh_by_local_iter=weigh)
        try:
            ref = R(**kw)
            ref._initialize(ref.aggregation_weights, ref.exclude_vars, ref.expected_data_kind)
        except Exception as e:
            try:
                mine = M(**kw)
                mine._initialize(mine.aggregation_weights, mine.exclude_vars, mine.expected_data_kind)
                stats["mismatches"].append(f"case {case}: reference init raised {e!r}, drop-in did not")
            except Exception as e2:
                if type(e2) is not type(e):
                    stats["mismatches"].append(f"case {case}: init {e2!r} vs {e!r}")
            continue
        mine = M(**kw)
        mine._initialize(mine.aggregation_weights, mine.exclude_vars, mine.expected_data_kind)
        for rnd in range(2):
            ctx_r, ctx_m = FLContext(), FLContext()
            for c in (ctx_r, ctx_m):
                c.set_prop(AppConstants.CURRENT_ROUND, rnd)
            order = list(names) + [str(rng.choice(names)) for _ in range(int(rng.integers(0, 3)))]  # repeats
            rng.shuffle(order)
            for name in order:
                odd = rng.random()
                steps = [1, 3, 7.5, None, 0, -2, 20][int(rng.integers(0, 7))]

                def make():
                    sub = {}
                    for k in subkeys:
                        if collection and odd < 0.05:
                            continue  # a COLLECTION missing a sub-DXO
                        data = {n: _value(rng, s, vdt, container) for n, s in keys.items() if rng.random() < 0.85}
                        kind = kinds[k] if odd >= 0.1 else DataKind.METRICS
                        meta = {} if steps is None else {MetaKey.NUM_STEPS_CURRENT_ROUND: steps}
                        sub[k] = DXO(kind, data=data, meta=meta)
                    return sub

                sub = make()
                pair = []
                for _ in range(2):
                    d = (DXO(DataKind.COLLECTION, data={k: DXO(v.data_kind, data={n: _copy(x) for n, x in v.data.items()},
                                                                 meta=dict(v.meta)) for k, v in sub.items()})
                         if collection else DXO(sub[""].data_kind, data={n: _copy(x) for n, x in sub[""].data.items()},
                                                meta=dict(sub[""].meta)))
                    sh = d.to_shareable()
                    sh.set_peer_props({ReservedKey.IDENTITY_NAME: name})
                    sh.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd if odd < 0.9 else rnd + 1)
                    if 0.15 <= odd < 0.2:
                        sh.set_return_code(ReturnCode.EXECUTION_EXCEPTION)
                    pair.append(sh)
                try:
                    a = ref.accept(pair[0], ctx_r)
                except Exception as e:
                    a = e
                try:
                    b = mine.accept(pair[1], ctx_m)
                except Exception as e:
                    b = e
                stats["accepts"] += 1
                if isinstance(a, Exception) or isinstance(b, Exception):
                    if type(a) is not type(b):
                        stats["mismatches"].append(f"case {case} round {rnd}: accept {b!r} vs {a!r}")
                    stats["errors"] += 1
                elif a != b:
                    stats["mismatches"].append(f"case {case} round {rnd} {name}: accept {b} vs reference {a}")
                elif not a:
                    stats["rejected"] += 1
            try:
                ra = from_shareable(ref.aggregate(ctx_r))
            except Exception as e:
                ra = e
            try:
                ma = from_shareable(mine.aggregate(ctx_m))
            except Exception as e:
                ma = e
            tag = f"case {case} round {rnd} ({container}, collection={collection}, weigh={weigh}, aw={aw is not None}, ex={ex!r})"
            if isinstance(ra, Exception) or isinstance(ma, Exception):
                if type(ra) is not type(ma):
                    stats["mismatches"].append(f"{tag}: aggregate {ma!r} vs {ra!r}")
                stats["errors"] += 1
                break
            _same_dxo(ra, ma, tag, stats["mismatches"])
            sr, sm = ctx_r.get_prop(AppConstants.AGGREGATION_STATS), ctx_m.get_prop(AppConstants.AGGREGATION_STATS)
            if repr(sr) != repr(sm):
                stats["mismatches"].append(f"{tag}: stats {sm} vs {sr}")
            stats["aggregates"] += 1
            ref.reset(ctx_r)
            mine.reset(ctx_m)
        stats["cases"] += 1
    return stats


def _same_flmodel(a, b, tag, out):
    if type(a) is not type(b) or (a is None) != (b is None):
        out.append(f"{tag}: {type(b).__name__} vs {type(a).__name__}")
        return
    if list(a.params or {}) != list(b.params or {}):
        out.append(f"{tag}: params keys {list(b.params or {})} vs {list(a.params or {})}")
    else:
        for k in a.params or {}:
            why = _same(a.params[k], b.params[k])
            if why:
                out.append(f"{tag} param {k}: {why}")
    for field in ("params_type", "current_round", "metrics", "meta"):
        va, vb = getattr(a, field), getattr(b, field)
        if repr(va) != repr(vb):
            out.append(f"{tag} {field}: {vb!r} vs {va!r}")


def run_fedavg(cases: int, seed: int) -> dict:
    """FedAvg-workflow aggregation (base_fedavg.py:93-230, fedavg.py:268-366) against the reference on random
    FLModel lists: ``aggregate_fn`` vs ``BaseFedAvg.aggregate_fn`` and DeviceFedAvgModelAggregator vs FedAvg's
    built-in in-time path (with aggregation_weights) -- odd NUM_STEPS values, missing / empty client names,
    partial params, numpy and torch, metrics of every kind (numbers, bools, strings, nested dicts, NaN, None)."""
    from nvflare.app_common.abstract.fl_model import FLModel
    from nvflare.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper as RefHelper
    from nvflare.app_common.workflows.base_fedavg import BaseFedAvg
    from nvflare.app_common.workflows.fedavg import FedAvg

    from nvflare_amd.app_common.aggregators import DeviceFedAvgModelAggregator
    from nvflare_amd.app_common.workflows import aggregate_fn

    rng = np.random.default_rng(seed)
    stats = {"cases": 0, "mismatches": [], "errors": 0, "accepted": 0}
    odd_steps = [None, True, False, 3, "7", "abc", 0, -1, float("nan"), float("inf"), 2.5, 40, [1]]
    for case in range(cases):
        container = "torch" if rng.random() < 0.5 else "numpy"
        K = int(rng.integers(1, 7))
        keys = {"w": (int(rng.integers(1, 3000)),), "b": (7,), "c": ()}
        names = [f"site-{i}" for i in range(K)]
        models = []
        for i in range(K):
            meta = {}
            r = rng.random()
            if r < 0.8:
                meta["client_name"] = names[i] if r < 0.7 else ""
            st = odd_steps[int(rng.integers(0, len(odd_steps)))]
            if not (container == "torch" and st is not None and not isinstance(st, (bool, list)) and
                    isinstance(st, (int, float)) and abs(float(st)) > 1e30):
                if st is not None:
                    meta["NUM_STEPS_CURRENT_ROUND"] = st
            params = {n: _value(rng, sh, "float32", container) for n, sh in keys.items() if rng.random() < 0.85}
            if not params:
                params = {"w": _value(rng, keys["w"], "float32", container)}
            m = rng.random()
            metrics = None if m < 0.1 else {"acc": float(rng.random()), "n": int(rng.integers(0, 9)),
                                            "flag": bool(m < 0.5), "tag": "x", "nested": {"a": 1},
                                            "bad": float("nan") if m > 0.9 else 0.5}
            models.append(FLModel(params=params, metrics=metrics, current_round=int(rng.integers(0, 3)), meta=meta))

        def clone(ms):
            return [FLModel(params={k: _copy(v) for k, v in x.params.items()}, metrics=None if x.metrics is None else
                            dict(x.metrics), current_round=x.current_round, meta=dict(x.meta)) for x in ms]

        tag = f"case {case} ({container}, K={K})"
        try:
            ra = BaseFedAvg.aggregate_fn(clone(models))
        except Exception as e:
            ra = e
        try:
            ma = aggregate_fn(clone(models))
        except Exception as e:
            ma = e
        if isinstance(ra, Exception) or isinstance(ma, Exception):
            if type(ra) is not type(ma):
                stats["mismatches"].append(f"{tag} aggregate_fn: {ma!r} vs {ra!r}")
            stats["errors"] += 1
        else:
            _same_flmodel(ra, ma, f"{tag} aggregate_fn", stats["mismatches"])
        # FedAvg's built-in in-time path vs the FedAvg(aggregator=...) drop-in
        aw = {n: float(rng.random() * 2) for n in names if rng.random() < 0.6} if rng.random() < 0.5 else None
        wf = FedAvg(num_clients=K, num_rounds=1, aggregation_weights=aw)
        wf.info = wf.warning = wf.debug = lambda *a, **k: None
        wf.fl_ctx = None
        wf.current_round = models[0].current_round
        wf._aggr_helper = RefHelper()
        wf._aggr_metrics_helper = RefHelper()
        wf._expected_count = K
        agg = DeviceFedAvgModelAggregator(aggregation_weights=aw)
        from nvflare.apis.fl_context import FLContext

        agg.handle_event("_start_run", FLContext())
        acc_r, acc_m = [], []
        try:
            for x in clone(models):
                acc_r.append(bool(wf._aggregate_one_result(x)))
            rr = wf._get_aggregated_result()
        except Exception as e:
            rr = e
        try:
            for x in clone(models):
                acc_m.append(bool(agg.accept_model(x)))
            mr = agg.aggregate_model()
        except Exception as e:
            mr = e
        if isinstance(rr, Exception) or isinstance(mr, Exception):
            if type(rr) is not type(mr):
                stats["mismatches"].append(f"{tag} in-time: {mr!r} vs {rr!r}")
            stats["errors"] += 1
        else:
            if acc_r != acc_m:
                stats["mismatches"].append(f"{tag} in-time accepted {acc_m} vs {acc_r}")
            _same_flmodel(rr, mr, f"{tag} in-time", stats["mismatches"])
            stats["accepted"] += sum(acc_r)
        stats["cases"] += 1
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--threads", type=int, default=3)
    ap.add_argument("--mode", choices=["helper", "intime", "fedavg"], default="helper")
    ap.add_argument("--record", default=None, help="helper mode: write the reference's result hashes (GPU replay)")
    ap.add_argument("--small", action="store_true", help="helper mode: no 70001-element shapes")
    a = ap.parse_args()
    if a.mode == "intime":
        _setup()
        stats = run_intime(a.cases, a.seed)
    elif a.mode == "fedavg":
        _setup()
        stats = run_fedavg(a.cases, a.seed)
    else:
        record = [] if a.record else None
        stats = run(a.cases, a.seed, a.threads, record, big=not a.small)
        if a.record:
            with open(a.record, "w") as f:
                json.dump({"generator": "tests/fuzz_reference_helper.py --mode helper --record",
                           "reference": "NVFlare weighted_aggregation_helper.py (/root/reference)", "seed": a.seed,
                           "cases": a.cases, "threads": a.threads, "big": not a.small, "numpy": np.__version__,
                           "torch": __import__("torch").__version__, "records": record}, f, indent=0)
    print(json.dumps({**stats, "mismatches": stats["mismatches"][:20], "n_mismatches": len(stats["mismatches"])}))
    sys.exit(1 if stats["mismatches"] else 0)


if __name__ == "__main__":
    main()
