"""Diagnostic: which elements torch-ROCm's float16 add_(v, alpha) rounds once (exact fma -> fp16) and which
twice (fp32, then fp16), by tensor size -- many steps on a growing total make the two visible."""
import sys

import numpy as np
import torch


def step_models(t, v, w):
    exact = v.astype(np.float64) * np.float64(np.float32(w)) + t.astype(np.float64)
    once = exact.astype(np.float16).astype(np.float32)
    twice = exact.astype(np.float32).astype(np.float16).astype(np.float32)
    return once, twice


rng = np.random.default_rng(1)
for n in [int(x) for x in sys.argv[1:]]:
    t = torch.from_numpy(np.asarray(rng.standard_normal(n) * 300, np.float32)).half().cuda()
    once_only = twice_only = both = neither = 0
    idx_once, idx_twice = set(), set()
    for step in range(400):
        v = torch.from_numpy(np.asarray(rng.standard_normal(n) * 3, np.float32)).half().cuda()
        w = float(rng.random() * 3 + 0.1)
        tn, vn = t.float().cpu().numpy(), v.float().cpu().numpy()
        t.add_(v, alpha=w)
        got = t.float().cpu().numpy()
        o, tw = step_models(tn, vn, w)
        mo, mt = got == o, got == tw
        once_only += int((mo & ~mt).sum()); twice_only += int((~mo & mt).sum()); neither += int((~mo & ~mt).sum())
        idx_once |= set(np.nonzero(mo & ~mt)[0].tolist()); idx_twice |= set(np.nonzero(~mo & mt)[0].tolist())
    print(f"n={n} once_only={once_only} twice_only={twice_only} neither={neither} "
          f"once_idx={sorted(idx_once)[:6]}..{sorted(idx_once)[-3:] if idx_once else []} "
          f"twice_idx={sorted(idx_twice)[:6]}..{sorted(idx_twice)[-3:] if idx_twice else []}", flush=True)
