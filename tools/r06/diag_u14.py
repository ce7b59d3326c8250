"""Round 6, session 22: which values the LDS-DMA Adam form (ieee sqrt, 3 clients) wrote into the elements it got wrong
in session 20 (one unit per wave, every wave): compare them with every stream the unit had."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import test_gpu_epi_dma as T  # noqa: E402
from nvflare_amd import _native as N  # noqa: E402
from nvflare_amd.device import DeviceContext  # noqa: E402
from oracle import fedavg_oracle as oracle  # noqa: E402

oracle.build()


def main():
    ctx = DeviceContext.get(0)
    ctx.set_variant(0)
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    begin, end = T._ranges(ctx)[4]
    c = T._Case(ctx, K, begin, end, seed=1000 + 10 * 4 + K)
    n = c.n
    p = c.rng.standard_normal(n).astype(np.float32)
    m = (c.rng.standard_normal(n) * 0.01).astype(np.float32)
    v = (c.rng.random(n) * 1e-4 + 1e-6).astype(np.float32)
    e = T._epi(3, param=c.buf("p", p), state1=c.buf("m", m), state2=c.buf("v", v), step=3.0,
               torch_sqrt=N.FEDAVG_SQRT_IEEE, **T.ADAM)
    T._run(ctx, c, e, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, variant=0)
    gp, gm, gv = (c.get(x) for x in ("p", "m", "v"))
    d = c.d(oracle, 1)
    pw, mw, vw = p.copy(), m.copy(), v.copy()
    oracle.epilogue_apply(d, oracle.EPI_ADAM, p=pw, m=mw, v=vw, step=3.0, torch_cpu_sqrt="ieee", **T.ADAM)
    for nm, g, w in (("p", gp, pw), ("m", gm, mw), ("v", gv, vw)):
        bad = np.flatnonzero(g.view(np.uint32) != w.view(np.uint32))
        print(nm, "mismatches", bad.size, "first", bad[:8].tolist())
        if bad.size:
            tiles = np.unique(bad // 4096)
            print("  tiles", tiles.size, tiles[:16].tolist(), "offsets in tile", np.unique(bad % 4096 // 256).tolist())
            cands = {"p_in": p, "m_in": m, "v_in": v, "d": d, "p_want": pw, "m_want": mw, "v_want": vw}
            for cn, cv in cands.items():
                eq = np.count_nonzero(g[bad].view(np.uint32) == cv[bad].view(np.uint32))
                print("  equal to", cn, eq)
            i = bad[0]
            print("  sample", i, g[i], {cn: float(cv[i]) for cn, cv in cands.items()})
            # shifted candidates: the same stream at another unit (+-256 .. +-4096 elements)
            for sh in (-4096 * 256 * 6, -1024, -256, 256, 1024, 4096):
                idx = bad + sh
                ok = (idx >= 0) & (idx < n)
                for cn, cv in cands.items():
                    eq = np.count_nonzero(g[bad[ok]].view(np.uint32) == cv[idx[ok]].view(np.uint32))
                    if eq > bad.size // 10:
                        print("  shifted", sh, cn, eq)
    c.close()


if __name__ == "__main__":
    main()
