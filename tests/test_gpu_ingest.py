"""Zero-copy ingest on the GPU path (row f2): contributions staged straight from received bytes (read-only
npy / safetensors views) or from an mmap of disk-offloaded safetensors files aggregate bit-identically to
the same contributions materialised as ordinary arrays / tensors (which tests/test_gpu_parity.py pins to
the reference)."""

import io

import numpy as np
import pytest
import torch

from golden_util import same_bits
from nvflare_amd.ingest import recompose_npy, recompose_safetensors

pytestmark = pytest.mark.gpu


class _LazyRefLike:
    """Same attributes as lazy_tensor_dict.py:60-77's _LazyRef."""

    def __init__(self, file_path, key):
        self.file_path = file_path
        self.key = key

    def materialize(self):
        from safetensors import safe_open

        with safe_open(self.file_path, framework="pt") as f:
            return f.get_tensor(self.key)


def _clients(K, rng):
    out = []
    for _ in range(K):
        out.append({"conv.weight": torch.from_numpy(rng.standard_normal((16, 3, 3, 3)).astype(np.float32)),
                    "fc.weight": torch.from_numpy(rng.standard_normal((100, 1003)).astype(np.float32)),
                    "fc.bias": torch.from_numpy(rng.standard_normal(100).astype(np.float32)),
                    "emb": torch.from_numpy(rng.standard_normal(5000).astype(np.float32)).to(torch.bfloat16),
                    "steps": torch.tensor(7, dtype=torch.int64)})
    return out


def _aggregate(inputs, ws):
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    h = WeightedAggregationHelper()
    for k, (d, w) in enumerate(zip(inputs, ws)):
        h.add(d, w, f"site-{k}", 0)
    return h.get_result()


def _same(a, b):
    assert set(a) == set(b)
    for k in a:
        x, y = a[k], b[k]
        assert type(x) is type(y) and x.dtype == y.dtype, k
        if isinstance(x, torch.Tensor):
            x = x.view(torch.int16).numpy() if x.dtype == torch.bfloat16 else x.numpy()
            y = y.view(torch.int16).numpy() if y.dtype == torch.bfloat16 else y.numpy()
        assert same_bits(np.asarray(x), np.asarray(y)), k


def test_disk_offload_refs_stage_from_mmap(tmp_path):
    from safetensors.torch import save_file

    rng = np.random.default_rng(0)
    clients = _clients(6, rng)
    ws = [float(1 + 3 * k) for k in range(6)]
    refs = []
    for k, c in enumerate(clients):
        path = str(tmp_path / f"client{k}.safetensors")
        save_file(c, path)
        refs.append({name: _LazyRefLike(path, name) for name in c})
    _same(_aggregate(refs, ws), _aggregate(clients, ws))


def test_zero_copy_decoded_payloads():
    from safetensors.torch import save

    rng = np.random.default_rng(1)
    clients = _clients(5, rng)
    ws = [0.5 + k for k in range(5)]
    views = [{k: recompose_safetensors(save({"t": v}))["t"] for k, v in c.items()} for c in clients]
    _same(_aggregate(views, ws), _aggregate(clients, ws))
    np_clients = [{k: v.numpy() for k, v in c.items() if v.dtype != torch.bfloat16} for c in clients]

    def npy(a):
        s = io.BytesIO()
        np.save(s, a, allow_pickle=False)
        return s.getvalue()

    np_views = [{k: recompose_npy(npy(a)) for k, a in c.items()} for c in np_clients]
    _same(_aggregate(np_views, ws), _aggregate(np_clients, ws))
