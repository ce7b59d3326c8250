"""The engine's host logic on the CPU (no GPU): slabs, slots, per-format arenas, folding under a tiny HBM
budget, keys introduced mid-round, slab-geometry chaining, round-to-round reuse and deferred rounds.

The device is ``tests/fake_device.FakeDeviceContext`` (numpy "device memory" poisoned with 0xAB on
allocation and 0xCD on free, synchronous copies, kernels restated with the oracle's numpy sequence).  Every
result must equal the same per-element sequence computed in one shot from the contributions -- i.e. the
bookkeeping (what is staged where, what is folded when, what an accumulator holds) is exact."""

import numpy as np
import pytest
import torch

from fake_device import FakeDeviceContext, fake_engine
from golden_util import as_f32_values, same_bits
from nvflare_amd import _native as N
from oracle import fedavg_oracle as orc


def _one_shot(values, ws, container, fmt=None):
    """The per-element sequence over one key's contributions, computed directly."""
    if fmt is not None:
        rows = [as_f32_values(v, fmt).reshape(-1) for v in values]
        # torch's scalar-loop elements of the add_ (nvflare_amd/torch16.py), as the engine reproduces them
        scalar = orc.torch16_scalar_mask(rows[0].size, torch.get_num_threads())
        res = FakeDeviceContext._agg(rows, ws, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, _count(ws), None, fmt=fmt,
                                     scalar=scalar)
        return res
    op, fin = ((N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV) if container == "torch" else (N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE))
    rows = [np.asarray(v.numpy() if isinstance(v, torch.Tensor) else v, dtype=np.float32).reshape(-1) for v in values]
    return FakeDeviceContext._agg(rows, ws, op, fin, _count(ws), None)


def _count(ws):
    c = None
    for w in ws:
        c = w if c is None else c + w
    return c


def _model(rng, k, drop_emb=False, late_key=False):
    c = {"a.w": torch.from_numpy(rng.standard_normal((64, 129)).astype(np.float32)),
         "a.b": torch.from_numpy(rng.standard_normal(64).astype(np.float32)).to(torch.bfloat16),
         "emb": torch.from_numpy(rng.standard_normal((500, 3)).astype(np.float32)).to(torch.bfloat16),
         "ln": torch.from_numpy(rng.standard_normal(7).astype(np.float16)),
         "steps": torch.tensor(k, dtype=torch.int64)}
    if drop_emb:
        del c["emb"]
    if late_key:
        c["late"] = torch.from_numpy(rng.standard_normal(300).astype(np.float32))
        c["late16"] = torch.from_numpy(rng.standard_normal(40).astype(np.float32)).to(torch.bfloat16)
    return c


@pytest.mark.parametrize("budget", [None, 1, 200_000])
@pytest.mark.parametrize("slab_slots", [None, 3])
def test_mixed_arenas_partial_and_late_keys(budget, slab_slots):
    rng = np.random.default_rng(1)
    K = 12
    clients = [_model(rng, k, drop_emb=(k == 3), late_key=(k >= 5)) for k in range(K)]
    ws = [float(1 + (37 * k) % 11) for k in range(K)]
    e = fake_engine(max_resident_bytes=budget, slab_slots=slab_slots)
    for c, w in zip(clients, ws):
        e.add(list(c.items()), w, True)
    out = e.result()
    for key in ("a.w", "a.b", "emb", "ln", "late", "late16"):
        seq = [(c[key], w) for c, w in zip(clients, ws) if key in c]
        fmt = {torch.bfloat16: "bfloat16", torch.float16: "float16"}.get(seq[0][0].dtype)
        exp = _one_shot([v for v, _ in seq], [w for _, w in seq], "torch", fmt)
        got = as_f32_values(out[key], fmt).reshape(-1) if fmt else out[key].numpy().reshape(-1)
        assert same_bits(got, exp), (key, budget, slab_slots)
    if budget == 1:
        assert e.stats["folds"] > 0


def test_rounds_reuse_slabs_and_consolidate():
    rng = np.random.default_rng(2)
    e = fake_engine()
    for rnd, K in enumerate((20, 20, 7)):
        clients = [{"w": rng.standard_normal(5000).astype(np.float32),
                    "h": rng.standard_normal(33).astype(np.float16)} for _ in range(K)]
        ws = [float(1 + k) for k in range(K)]
        for c, w in zip(clients, ws):
            e.add(list(c.items()), w, True)
        out = e.result()
        assert same_bits(out["w"], _one_shot([c["w"] for c in clients], ws, "numpy"))
        exp_h = clients[0]["h"] * np.float16(ws[0])
        for c, w in zip(clients[1:], ws[1:]):
            exp_h = exp_h + c["h"] * np.float16(w)
        assert same_bits(out["h"], exp_h * np.float16(1.0 / _count(ws)))
        e.reset()
        if rnd == 0:  # round 1 grew 16 + 32 slots; consolidated to one slab of the observed 20 clients
            assert len(e.f32.slabs) == 0
        else:
            assert len(e.f32.slabs) == 1 and e.f32.slabs[0].layout.slots >= 20


def test_deferred_round_settles_before_next_round():
    rng = np.random.default_rng(3)
    e = fake_engine()
    rounds = [[rng.standard_normal(777).astype(np.float32) for _ in range(5)] for _ in range(2)]
    ws = [1.0, 2.0, 3.0, 4.0, 5.0]
    vals = []
    for rows in rounds:
        for r, w in zip(rows, ws):
            e.add([("w", r)], w, True)
        vals.append(e.result_deferred()["w"])
        e.reset()
    for v, rows in zip(vals, rounds):
        assert same_bits(np.asarray(v), _one_shot(rows, ws, "numpy"))


@pytest.mark.parametrize("slab_slots", [None, 4])
def test_pipelined_egress_chunks(monkeypatch, slab_slots):
    """Results above 2 x EGRESS_CHUNK leave through chunked final launches + fedavg_d2h_marked; chunk
    boundaries fall inside keys, between keys and inside multi-slab chains -- results unchanged."""
    import nvflare_amd.engine as E

    monkeypatch.setattr(E, "EGRESS_CHUNK", 64 << 10)  # 16 Ki fp32 elements per chunk
    rng = np.random.default_rng(4)
    sizes = {"k0": 40_000, "k1": 3, "k2": 70_001, "k3": 16_384}
    K = 9
    clients = [{k: rng.standard_normal(n).astype(np.float32) for k, n in sizes.items()} for _ in range(K)]
    clients[2].pop("k1")  # a partial contribution: k1 forms its own run
    ws = [float(1 + 3 * k) for k in range(K)]
    e = fake_engine(slab_slots=slab_slots)
    for c, w in zip(clients, ws):
        e.add(list(c.items()), w, True)
    out = e.result()
    assert getattr(e.ctx, "marked_copies", 0) == 1
    for key in sizes:
        seq = [(c[key], w) for c, w in zip(clients, ws) if key in c]
        assert same_bits(out[key], _one_shot([v for v, _ in seq], [w for _, w in seq], "numpy")), key


def test_plain_numpy_fast_path_keeps_type_checks():
    """Repeat contributions of plain numpy arrays skip type resolution when (dtype, weight type, weighted)
    and shape match an already-checked contribution; any change still takes the full check."""
    eng = fake_engine()
    a = np.arange(10, dtype=np.float32)
    eng.add([("w", a)], 1.0, True)
    eng.add([("w", a + 1)], 2.0, True)  # fast path
    with pytest.raises(TypeError):  # numpy-scalar weight: result dtype float64, not the key's float32
        eng.add([("w", a)], np.float64(3.0), True)
    with pytest.raises(TypeError):
        eng.add([("w", a.astype(np.float64))], 3.0, True)
    with pytest.raises(ValueError):
        eng.add([("w", np.arange(11, dtype=np.float32))], 3.0, True)
    with pytest.raises(TypeError):  # torch tensor for a numpy key
        eng.add([("w", torch.from_numpy(a))], 3.0, True)
    eng.add([("w", np.ascontiguousarray(a[::-1]))], 4.0, True)
    eng.add([("w", a[::-1])], 5.0, True)  # non-contiguous view: staged through a contiguous copy
    res = eng.result()["w"]
    vals = [a, a + 1, a[::-1], a[::-1]]
    assert same_bits(res, _one_shot(vals, [1.0, 2.0, 4.0, 5.0], "numpy"))


@pytest.mark.parametrize("budget,slab_slots", [(None, None), (1, None), (None, 4)])
def test_fp64_arena_with_fp32_keys(budget, slab_slots):
    """numpy float64 keys (numpy's default dtype) in their own arena beside fp32 keys: folding under a tiny
    budget, slab chaining, a key missing from one client -- same bits as the one-shot numpy sequence."""
    rng = np.random.default_rng(8)
    K = 9
    clients = []
    for k in range(K):
        c = {"w64": rng.standard_normal((37, 129)), "w32": rng.standard_normal(5000).astype(np.float32)}
        if k != 4:
            c["b64"] = rng.standard_normal(77)
        clients.append(c)
    ws = [float(1 + (37 * k) % 11) for k in range(K)]
    e = fake_engine(max_resident_bytes=budget, slab_slots=slab_slots)
    for c, w in zip(clients, ws):
        e.add(list(c.items()), w, True)
    out = e.result()
    assert {a.np_dtype for a in e.arenas.values()} >= {np.dtype(np.float64), np.dtype(np.float32)}
    for key in ("w64", "w32", "b64"):
        seq = [(c[key], w) for c, w in zip(clients, ws) if key in c]
        exp = FakeDeviceContext._agg([v.reshape(-1) for v, _ in seq], [w for _, w in seq], N.FEDAVG_OP_NUMPY,
                                     N.FEDAVG_FIN_SCALE, _count([w for _, w in seq]), None)
        assert out[key].dtype == seq[0][0].dtype
        assert same_bits(out[key].reshape(-1), exp), (key, budget, slab_slots)
    if budget == 1:
        assert e.stats["folds"] > 0
