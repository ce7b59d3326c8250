#!/usr/bin/env python3
"""How far is torch-ROCm's own GPU optimizer from the fused epilogue? (measurement tool, GPU box)

The reference FedOpt generator moves its model to cuda:0 when a GPU is present (app_opt/pt/fedopt.py:97-123),
so on a GPU server the reference's server step is torch's CUDA/ROCm optimizer: multi-tensor (foreach) by
default, single-tensor with foreach=False, or the fused kernel with fused=True.  The drop-in's epilogue
follows torch's CPU single-tensor rounding, which is the reference on a CPU-only server
(tests/test_fedopt_oracle.py: m and v bit-exact; p differs only where torch CPU's vectorised sqrt is off
by 1 ulp).  This tool steps the same state with every implementation and reports the distance per state
tensor, in ulp of the value and (max_rel_to_update) relative to the size of the step's update.

  python tools/fedopt_vs_torch_gpu.py [--n 4194304] > gpurun_out/fedopt_vs_torch_gpu.jsonl
"""

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TILE = 4096


def ordered(a: np.ndarray) -> np.ndarray:
    i = a.view(np.int32).astype(np.int64)
    return np.where(i >= 0, i, -(i & 0x7FFFFFFF))


def ulp_stats(a: np.ndarray, b: np.ndarray, before: np.ndarray = None) -> dict:
    d = np.abs(ordered(a) - ordered(b))
    out = {"max_ulp": int(d.max()), "frac_diff": round(float((d > 0).mean()), 6)}
    if before is not None:  # |difference| relative to the size of this step's update (or 1 ulp of the value)
        a64, b64 = a.astype(np.float64), b.astype(np.float64)
        scale = np.maximum(np.abs(a64 - before.astype(np.float64)), np.spacing(np.abs(a)).astype(np.float64))
        out["max_rel_to_update"] = float((np.abs(a64 - b64) / scale).max())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4 * 1024 * 1024)
    args = ap.parse_args()
    import torch

    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    dev = torch.device("cuda", 0)
    n = args.n // TILE * TILE
    rng = np.random.default_rng(7)
    p0 = rng.standard_normal(n).astype(np.float32)
    d0 = (rng.standard_normal(n) * 0.01).astype(np.float32)
    m0 = (rng.standard_normal(n) * 0.01).astype(np.float32)
    v0 = (rng.random(n) * 1e-4).astype(np.float32)

    cases = [
        ("sgd", dict(lr=0.5, momentum=0.9), 2),
        ("sgd_nesterov_wd", dict(lr=0.5, momentum=0.9, nesterov=True, weight_decay=1e-4), 2),
        ("adam", dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8), 3),
        ("adamw", dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01), 3),
    ]

    def torch_step(name, hp, step, impl, device):
        p = torch.nn.Parameter(torch.from_numpy(p0.copy()).to(device))
        p.grad = torch.from_numpy(-d0).to(device)
        kw = {}
        if impl == "foreach":
            kw["foreach"] = True
        elif impl == "single":
            kw["foreach"] = False
        elif impl == "fused":
            kw["fused"] = True
        if name.startswith("sgd"):
            opt = torch.optim.SGD([p], **hp, **kw)
            opt.state[p] = {"momentum_buffer": torch.from_numpy(m0.copy()).to(device)}
        else:
            cls = torch.optim.AdamW if name == "adamw" else torch.optim.Adam
            opt = cls([p], **hp, **kw)
            st = torch.tensor(float(step - 1), dtype=torch.float32)
            if impl == "fused":
                st = st.to(device)
            opt.state[p] = {"step": st, "exp_avg": torch.from_numpy(m0.copy()).to(device),
                            "exp_avg_sq": torch.from_numpy(v0.copy()).to(device)}
        opt.step()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        s = opt.state[p]
        out = {"p": p.detach().cpu().numpy()}
        if name.startswith("sgd"):
            out["m"] = s["momentum_buffer"].cpu().numpy()
        else:
            out["m"] = s["exp_avg"].cpu().numpy()
            out["v"] = s["exp_avg_sq"].cpu().numpy()
        return out

    def ours(name, hp, step):
        bufs = {k: torch.from_numpy(a.copy()).to(dev) for k, a in (("p", p0), ("m", m0), ("v", v0), ("d", d0))}
        torch.cuda.synchronize(dev)
        e = N.Epilogue()
        e.lr = hp["lr"]
        e.weight_decay = hp.get("weight_decay", 0.0)
        e.param, e.state1 = bufs["p"].data_ptr(), bufs["m"].data_ptr()
        if name.startswith("sgd"):
            e.kind = N.FEDAVG_EPI_SGD
            e.momentum = hp["momentum"]
            e.nesterov = int(hp.get("nesterov", False))
            e.first_step = 0
        else:
            e.kind = N.FEDAVG_EPI_ADAM
            e.beta1, e.beta2 = hp["betas"]
            e.eps = hp["eps"]
            e.step = float(step)
            e.decoupled_weight_decay = int(name == "adamw")
            e.state2 = bufs["v"].data_ptr()
        ctx.accumulate_tiled_epi([], [], TILE, TILE, 0, n, None, 1, 0, 1.0, e, acc_in_ptr=bufs["d"].data_ptr())
        ctx.sync()
        return {k: bufs[k].cpu().numpy() for k in ("p", "m", "v")}

    for name, hp, step in cases:
        mine = ours(name, hp, step)
        impls = [("cpu", "single", torch.device("cpu")), ("cuda", "single", dev), ("cuda", "foreach", dev)]
        if not name.startswith("sgd"):
            impls.append(("cuda", "fused", dev))
        for where, impl, device in impls:
            try:
                ref = torch_step(name, hp, step, impl, device)
            except Exception as exc:  # an implementation this torch build lacks
                print(json.dumps({"optimizer": name, "torch": f"{where}/{impl}", "error": repr(exc)[:200]}), flush=True)
                continue
            row = {"optimizer": name, "torch": f"{where}/{impl}", "n": n}
            for k in ref:
                row[k] = ulp_stats(mine[k], ref[k], {"p": p0, "m": m0, "v": v0}[k])
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
