#!/usr/bin/env python3
"""Which arithmetic torch-ROCm's GPU kernels use for the reference helper's ops on device-resident tensors
(weighted_aggregation_helper.py:181-236 with cuda tensors): mul by a python scalar, add_(v, alpha=w), div_ by a
python scalar -- compared element by element with candidate formulas computed on the host (exact fp64 where
a single rounding is meant).  Prints one JSON line per (dtype, op)."""

import json

import numpy as np
import torch


def r16(x, dt):
    return torch.from_numpy(np.asarray(x, np.float32)).to(dt).float().numpy()


def main():
    rng = np.random.default_rng(0)
    n = 1 << 20
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        t = torch.from_numpy((rng.standard_normal(n) * 30).astype(np.float32)).to(dt)
        v = torch.from_numpy((rng.standard_normal(n) * 30).astype(np.float32)).to(dt)
        w, c = 0.3711, 7.13
        tf, vf = t.float().numpy().astype(np.float64), v.float().numpy().astype(np.float64)
        rnd = (lambda x: np.asarray(x, np.float64).astype(np.float32)) if dt == torch.float32 else (lambda x: r16(np.asarray(x, np.float64).astype(np.float32), dt))
        wr = float(rnd(np.float32(w))) if dt != torch.float32 else float(np.float32(w))
        got = t.cuda().add_(v.cuda(), alpha=w).float().cpu().numpy()
        cand = {"fma_alpha_rounded": rnd(vf * wr + tf), "fma_alpha_float": rnd(vf * float(np.float32(w)) + tf),
                "mul_add_alpha_float": rnd(rnd(vf * float(np.float32(w))).astype(np.float64) + tf) if dt == torch.float32 else
                rnd(np.asarray(vf * float(np.float32(w)), np.float32).astype(np.float64) + tf)}
        print(json.dumps({"dtype": str(dt), "op": "add_(alpha)", **{k: int((got != x).sum()) for k, x in cand.items()}}))
        got = t.cuda().div_(c).float().cpu().numpy()
        cand = {"true_div": rnd(tf / float(np.float32(c))), "mul_reciprocal_f32": rnd(tf * float(np.float32(1.0 / np.float32(c)))),
                "mul_reciprocal_f64": rnd(tf * (1.0 / c))}
        print(json.dumps({"dtype": str(dt), "op": "div_(scalar)", **{k: int((got != x).sum()) for k, x in cand.items()}}))
        got = v.cuda().mul(w).float().cpu().numpy()
        cand = {"mul_float": rnd(vf * float(np.float32(w))), "mul_double": rnd(vf * w)}
        print(json.dumps({"dtype": str(dt), "op": "mul(scalar)", **{k: int((got != x).sum()) for k, x in cand.items()}}))


if __name__ == "__main__":
    main()
