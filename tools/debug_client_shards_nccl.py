"""Debug: the exchange strategy under RCCL at world 1 (one GPU) against the oracle, step by step."""
import os, socket, sys
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group(sys.argv[1] if len(sys.argv) > 1 else "nccl", device_id=torch.device("cuda", 0))
from nvflare_amd.client_shards import ClientShardedFedAvg
from oracle import fedavg_oracle as orc
K, P = 64, int(float(sys.argv[2])) if len(sys.argv) > 2 else 1 << 20
agg = ClientShardedFedAvg(P, [K], device=0, mode="torch")
agg.fill_synthetic(1000, list(range(K)))
order = [(0, g) for g in range(K)]
w = [float(1 + (37 * g) % 100) for g in range(K)]
cols = np.arange(P, dtype=np.uint64)
want = orc.fedavg_c([orc.synth_values(1000, g, cols) for g in range(K)], w, orc.MODE_TORCH, nthreads=16)
def cmp(tag, t):
    g = t.cpu().numpy()
    d = np.nonzero(g.view(np.uint32) != want.view(np.uint32))[0]
    print(tag, d.size, (int(d.min()), int(d.max()), float(np.max(np.abs(g[d] - want[d])))) if d.size else "", flush=True)
cmp("exchange", agg.aggregate(order, w, "exchange"))
torch.cuda.synchronize()
cmp("exchange again", agg.aggregate(order, w, "exchange"))
agg.exchange(); cmp("split", agg.aggregate_exchanged(order, w))
cmp("reduce", agg.aggregate(order, w, "reduce"))
cmp("exchange after reduce", agg.aggregate(order, w, "exchange"))
dist.destroy_process_group()
