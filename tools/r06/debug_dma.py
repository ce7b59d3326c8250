"""Round 6 debug: where the LDS-DMA fused form's numpy-mode ADD_BASE output differs (against the oracle and the per-tile
form on the same inputs)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import fedavg_oracle as orc  # noqa: E402
import test_gpu_epi_dma as T  # noqa: E402
from nvflare_amd.device import DeviceContext  # noqa: E402

orc.build()
ctx = DeviceContext.get(0)
for K in (1, 2, 3):
    for rng_ix in (1, 2, 3, 4):
        for op, fin in ((0, 1), (1, 2)):
            begin, end = T._ranges(ctx)[rng_ix]
            c = T._Case(ctx, K, begin, end, seed=3000 + 10 * rng_ix + K)
            base = c.rng.standard_normal(c.n).astype(np.float32)
            res = {}
            for variant in (0, 4):
                e = T._epi(1, base=c.buf("base", base))
                outp = c.buf("out", np.zeros(c.n, np.float32))
                T._run(ctx, c, e, op, fin, out_ptr=outp, variant=variant)
                res[variant] = c.get("out")
            want = orc.epilogue_apply(c.d(orc, op), orc.EPI_ADD_BASE, base=base)
            bad0 = np.nonzero(res[0].view(np.uint32) != want.view(np.uint32))[0]
            bad4 = np.nonzero(res[4].view(np.uint32) != want.view(np.uint32))[0]
            print(f"K={K} rng={rng_ix} op={op} begin={begin} n={c.n}: dma {bad0.size} bad, per-tile {bad4.size} bad",
                  (bad0[:8] + begin).tolist(), res[0][bad0[:4]].tolist(), want[bad0[:4]].tolist(), res[4][bad0[:4]].tolist())
            c.close()
