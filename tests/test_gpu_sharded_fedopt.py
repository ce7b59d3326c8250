"""The FedOpt server step sharded by parameter bucket over several devices (sharded_fedopt.py).

``InTimeAccumulateWeightedAggregator(devices=[...], defer_result=True)`` returns ``ShardedDeferredAggregate``
values whose bucket pieces stay on their devices; ``PTFedOptModelShareableGenerator(devices=[...])`` steps each
bucket on its device in the launch that aggregates it and pulls the new weights from every device.  On the
one-GPU test box the "devices" are three engines and three optimizer shards on device 0 (as in
tests/test_gpu_parity.py's sharding test): the bookkeeping -- spans, piece-to-shard matching, group sync,
egress into the host weights, re-uploads -- is the multi-device one.  The bar is bitwise equality, every
round, with the one-device flow (itself pinned to the reference by tests/test_gpu_fedopt_generator.py)."""

import numpy as np
import pytest
import torch

from golden_util import same_bits
from test_gpu_deferred import OPTS, run_fedopt_sag

pytestmark = pytest.mark.gpu

DEVS = [0, 0, 0]


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    return DeviceContext.get(0)


def wide_model():
    """Parameters from one bucket (below 3 x 4096 elements) to all three, BatchNorm buffers, a nested name."""

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin1 = torch.nn.Linear(40, 300)  # 12,000 + 300
            self.bn = torch.nn.BatchNorm1d(300)
            self.body = torch.nn.Sequential(torch.nn.Linear(300, 70), torch.nn.ReLU(), torch.nn.Linear(70, 9))

    return Net()


def _compare(ref, got):
    assert len(ref) == len(got)
    for rnd, ((w_ref, d_ref), (w_got, d_got)) in enumerate(zip(ref, got)):
        assert set(w_ref) == set(w_got)
        for k in w_ref:
            assert w_ref[k].dtype == w_got[k].dtype and w_ref[k].shape == w_got[k].shape, (rnd, k)
            assert same_bits(w_ref[k], w_got[k]), (rnd, k)
        for k in d_ref:
            assert same_bits(d_ref[k], d_got[k]), (rnd, k)


@pytest.mark.parametrize("container", ["numpy", "torch"])
@pytest.mark.parametrize("opt", ["sgd_nesterov", "adam", "adamw", "nadam", "rprop", "asgd"])
def test_sharded_fedopt_matches_one_device(container, opt):
    ref, _, _ = run_fedopt_sag(True, container, opt, 6, rounds=3, model_fn=wide_model)
    got, _, gen = run_fedopt_sag(True, container, opt, 6, rounds=3, model_fn=wide_model, devices=DEVS)
    _compare(ref, got)
    dev = gen._dev_opt
    from nvflare_amd.app_opt.pt.sharded_fedopt import ShardedServerOptimizer

    assert isinstance(dev, ShardedServerOptimizer)
    # lin1.weight spans all three shards; body.2.weight (630 elements, one bucket unit) lives on one shard
    assert all("lin1.weight" in sp for sp in dev.spans) and sum("body.2.weight" in sp for sp in dev.spans) == 1
    # the model's parameters are views of the host weights the generator returned last
    assert dev.is_bound()


def test_sharded_fedopt_eager_aggregates_and_missing_key():
    """Aggregator without defer_result (host differences sliced per shard) and a parameter missing from one
    client's round-1 update: same bits as the one-device flow."""
    ref, _, _ = run_fedopt_sag(False, "numpy", "adam", 5, rounds=3, model_fn=wide_model, drop="lin1.bias")
    got, _, _ = run_fedopt_sag(False, "numpy", "adam", 5, rounds=3, model_fn=wide_model, drop="lin1.bias", devices=DEVS)
    _compare(ref, got)
    got2, _, _ = run_fedopt_sag(True, "numpy", "adam", 5, rounds=3, model_fn=wide_model, drop="lin1.bias", devices=DEVS)
    _compare(ref, got2)


def test_sharded_fedopt_lr_schedule_and_inplace_load():
    """An lr scheduler on the original optimizer reaches every shard; weights loaded into the model in place
    between rounds (load_state_dict) are uploaded to the shards before the next step."""
    args = {"path": "torch.optim.Adam", "args": {"lr": 1e-2}}
    sched = {"path": "torch.optim.lr_scheduler.StepLR", "args": {"step_size": 1, "gamma": 0.5}}
    def reload(rnd, model, gen):
        if rnd == 0:  # a persistor-style reload; in the sharded flow it also rewrites the weights the model
            # parameters view (host weights, like the reference's CPU model), so the test hands both flows the
            # reloaded weights as the next global model
            sd = {k: (v.detach().cpu() * 0.5 if v.dtype == torch.float32 else v.detach().cpu().clone())
                  for k, v in model.state_dict().items()}
            model.load_state_dict(sd)
            return {k: v.clone() for k, v in sd.items()}
        return None

    runs = []
    for devices in (None, DEVS):
        hist, _, gen = run_fedopt_sag(True, "numpy", "adam", 4, rounds=3, model_fn=wide_model, opt_args=args,
                                      sched_args=sched, devices=devices, between_rounds=reload)
        runs.append(hist)
        assert gen.optimizer.param_groups[0]["lr"] == pytest.approx(1e-2 * 0.5 ** 3)
    _compare(runs[0], runs[1])


def test_d2h_multi_pieces(ctx):
    """fedavg_d2h_multi: scattered pieces into page-locked and pageable host arrays."""
    from nvflare_amd.device import HostArenaPool

    rng = np.random.default_rng(3)
    src = rng.standard_normal(100_000).astype(np.float32)
    buf = ctx.alloc(src.nbytes)
    ctx.h2d_ptr(buf.ptr, src.ctypes.data, src.nbytes)
    pieces = [(4 * 10, 4 * 500, 4 * 7), (4 * 20_000, 0, 4 * 40_000), (0, 4 * 99_990, 4 * 10), (4 * 70_000, 4 * 60_000, 0)]
    for host in (np.full(80_000, -1.0, np.float32), HostArenaPool().take(1 << 23, pin=ctx)):
        host[:80_000] = -1.0
        ctx.d2h_multi(host, buf.ptr, pieces)
        exp = np.full(80_000, -1.0, np.float32)
        for ho, do, nb in pieces:
            exp[ho // 4:(ho + nb) // 4] = src[do // 4:(do + nb) // 4]
        assert same_bits(host[:80_000], exp)
    buf.close()


def test_sharded_fedopt_rebind_keeps_state():
    """A re-bind after a few Adam rounds (a parameter re-pointed, so is_bound() is false) starts the new sharded
    image from the shards' moments (ShardedServerOptimizer.export_state), and the original optimizer's
    state_dict() shows them: same bits as the one-device flow, every round and every state entry."""
    def repoint(rnd, model, gen):
        if rnd == 1:
            p = dict(model.named_parameters())["lin1.weight"]
            p.data = p.data.clone()  # same values, new storage: the device image must be re-bound
        return None

    runs = []
    for devices in (None, DEVS):
        hist, _, gen = run_fedopt_sag(True, "numpy", "adam", 4, rounds=4, model_fn=wide_model, devices=devices,
                                      between_rounds=repoint)
        runs.append((hist, gen))
    _compare(runs[0][0], runs[1][0])
    sd_ref = runs[0][1].optimizer.state_dict()["state"]
    sd_got = runs[1][1].optimizer.state_dict()["state"]
    assert set(sd_ref) == set(sd_got) and sd_ref
    for i, st in sd_ref.items():
        assert set(st) == set(sd_got[i]), i
        for k, v in st.items():
            a = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
            b = sd_got[i][k]
            b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
            assert a.shape == b.shape and same_bits(a, b), (i, k)


@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_sharded_fedopt_returned_weights_are_independent(container):
    """The weights a round returns are independent, writable copies (fedopt.py:232-236 hands out
    ``detach().cpu().clone()`` / the ``.numpy()`` of its GPU model): a caller writing into them in place
    changes neither the live parameters nor the next step.  Parameters of the next rounds equal those of a run
    without the edits; every key equals the one-device flow under the same edits."""
    def edit(rnd, weights):
        for v in weights.values():
            if container == "torch":
                assert isinstance(v, torch.Tensor)
                if v.dtype == torch.float32:
                    v.mul_(3.0).add_(1.0)
            else:
                if isinstance(v, np.generic):  # a 0-d key's base + diff is a numpy scalar, as in the reference
                    continue
                assert isinstance(v, np.ndarray) and v.flags.writeable
                if v.dtype == np.float32:
                    v *= 3.0
                    v += 1.0

    plain, _, _ = run_fedopt_sag(True, container, "adam", 4, rounds=3, model_fn=wide_model, devices=DEVS)
    runs = []
    for devices in (None, DEVS):
        hist, _, gen = run_fedopt_sag(True, container, "adam", 4, rounds=3, model_fn=wide_model, devices=devices,
                                      edit_weights=edit)
        runs.append(hist)
    _compare(runs[0], runs[1])
    params = {n for n, _ in wide_model().named_parameters()}
    for (w_plain, _), (w_edit, _) in zip(plain, runs[1]):
        for k in params:
            assert same_bits(w_plain[k], w_edit[k]), k
    assert gen._dev_opt.is_bound()


def test_sharded_to_host_uploads_host_edits_first():
    """ShardedServerOptimizer.to_host pulls the weights it hands out from the device shards; a parameter
    written in place on the host after the last step (load_state_dict, param.copy_) must reach the shards first, or
    the hand-out is the stale shard value.  The hand-out equals the edited host parameters bit for bit, and the
    next step starts from them."""
    _, _, gen = run_fedopt_sag(True, "torch", "adam", 4, rounds=1, model_fn=wide_model, devices=DEVS)
    dev = gen._dev_opt
    assert dev.is_bound()
    with torch.no_grad():
        for p in gen.model.parameters():
            p.mul_(2.0).add_(0.5)
    want = {k: v.detach().clone() for k, v in gen.model.state_dict().items()}
    got = dev.to_host(gen.model.state_dict(), True)
    params = {n for n, _ in gen.model.named_parameters()}
    assert params
    for k in params:
        assert same_bits(got[k].numpy(), want[k].numpy()), k
