"""Host logic of the sharded server optimizer (nvflare_amd/app_opt/pt/sharded_fedopt.py), CPU only: the
per-shard spans match the aggregation's bucket split, shard modules keep the parameter names, shard
optimizers keep the param groups and slice the per-parameter state.  The device steps are checked on the GPU
(tests/test_gpu_sharded_fedopt.py)."""

import numpy as np
import torch

from nvflare_amd.app_opt.pt.sharded_fedopt import shard_module, shard_optimizer, shard_spans
from nvflare_amd.sharding import BUCKET_ALIGN, bucket_ranges


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(50, 400), torch.nn.ReLU(), torch.nn.Linear(400, 3),
                               torch.nn.Sequential(torch.nn.Linear(3, 2)))


def test_spans_cover_every_parameter_as_the_aggregation_splits_it():
    named = list(_model().named_parameters())
    spans = shard_spans(named, 3)
    for name, p in named:
        pieces = sorted(sp[name] for sp in spans if name in sp)
        assert pieces == [(lo, hi) for lo, hi in bucket_ranges(p.numel(), 3) if hi > lo]
        assert pieces[0][0] == 0 and pieces[-1][1] == p.numel()
        assert all(lo % BUCKET_ALIGN == 0 for lo, _ in pieces)


def test_shard_modules_keep_names_and_slices():
    named = list(_model().named_parameters())
    spans = shard_spans(named, 3)
    for b, sp in enumerate(spans):
        mod = shard_module(named, sp)
        got = dict(mod.named_parameters())
        assert set(got) == set(sp)
        for name, (lo, hi) in sp.items():
            src = dict(named)[name].detach().reshape(-1)[lo:hi]
            assert got[name].shape == (hi - lo,) and torch.equal(got[name].detach(), src)
            assert got[name].data_ptr() != src.data_ptr()  # a copy: the shard owns its storage


def test_shard_optimizers_keep_groups_and_slice_state():
    model = _model()
    named = list(model.named_parameters())
    opt = torch.optim.Adam([{"params": list(model[0].parameters()), "lr": 0.01},
                            {"params": list(model[2].parameters()) + list(model[3].parameters()), "lr": 0.2,
                             "betas": (0.5, 0.6)}])
    for p in model.parameters():  # one CPU step: exp_avg / exp_avg_sq / step exist
        p.grad = torch.randn_like(p)
    opt.step()
    spans = shard_spans(named, 3)
    for sp in spans:
        mod = shard_module(named, sp)
        sopt = shard_optimizer(opt, named, mod, sp)
        assert type(sopt) is torch.optim.Adam and len(sopt.param_groups) == 2  # a group may be empty
        for g, sg in zip(opt.param_groups, sopt.param_groups):
            assert {k: v for k, v in g.items() if k != "params"} == {k: v for k, v in sg.items() if k != "params"}
        mine = dict(mod.named_parameters())
        for name, (lo, hi) in sp.items():
            st, sst = opt.state[dict(named)[name]], sopt.state[mine[name]]
            assert float(sst["step"]) == float(st["step"])
            for k in ("exp_avg", "exp_avg_sq"):
                assert np.array_equal(sst[k].numpy(), st[k].reshape(-1)[lo:hi].numpy())
