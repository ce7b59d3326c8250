"""Client-sharded ingest on the GPU (nvflare_amd/client_shards.py): ranks sharing cuda:0 over gloo (the pool's
boxes have one GPU; RCCL refuses two ranks on one device, so the collectives go through host copies -- the
data path and the kernels are the ones an 8-GPU RCCL run uses).

* exchange strategy: each rank's bucket is BIT-EXACT against the oracle over the whole updates in arrival
  order (unequal clients per rank, interleaved arrival orders, ragged P, torch and numpy modes, more than
  128 clients in one rank's run);
* reduce strategy: within the recursive-summation error bound of an fp64 reference,
  |got - ref| <= (K + 2) * 2^-24 * sum_k |w_k v_k| / count + one result ulp (the reference's own tests
  compare random cases with assert_allclose, in_time_accumulate_weighted_aggregator_test.py:304-385);
* gather_result reassembles the exchange buckets into the whole model on every rank."""

import os
import random
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TILE = 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    try:
        from nvflare_amd.client_shards import ClientShardedFedAvg
        from oracle import fedavg_oracle as orc

        for (P, clients, order, weights, mode) in cases:
            if len(clients) != world:
                continue
            agg = ClientShardedFedAvg(P, clients, device=0, mode=mode)
            if mode == "numpy":  # one tile per all-to-all call: the chunked exchange's every boundary
                agg.max_peer_bytes = 1
            gid = {}
            for s in range(world):
                for j in range(clients[s]):
                    gid[(s, j)] = len(gid)
            agg.fill_synthetic(11, [gid[(rank, j)] for j in range(clients[rank])])
            cols = np.arange(P, dtype=np.uint64)
            full = [orc.synth_values(11, gid[c], cols) for c in order]
            omode = orc.MODE_TORCH if mode == "torch" else orc.MODE_NUMPY
            want = orc.fedavg_c(full, weights, omode)
            b0, b1 = agg.plan.buckets[rank]
            got = agg.aggregate(order, weights, "exchange").cpu().numpy()
            exact = got.view(np.uint32).tolist() == want[b0:b1].view(np.uint32).tolist()
            whole = agg.gather_result().cpu().numpy()
            gathered = whole.view(np.uint32).tolist() == want.view(np.uint32).tolist()
            red = agg.aggregate(order, weights, "reduce").cpu().numpy().astype(np.float64)
            w64 = np.asarray(weights, dtype=np.float64)[:, None]
            v64 = np.stack(full)[:, b0:b1].astype(np.float64)
            count = 0.0
            for i, w in enumerate(weights):
                count = w if i == 0 else count + w
            ref = (w64 * v64).sum(axis=0) / count
            bound = (len(order) + 2) * 2.0 ** -24 * np.abs(w64 * v64).sum(axis=0) / count
            bound += np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
            within = bool(np.all(np.abs(red - ref) <= bound))
            differ = int(np.count_nonzero(red.astype(np.float32).view(np.uint32) != want[b0:b1].view(np.uint32)))
            out.append((P, tuple(clients), mode, exact, gathered, within, differ, b1 - b0))
        q.put((rank, out))
    except Exception as e:  # pragma: no cover - reported through the queue
        import traceback

        q.put((rank, traceback.format_exc() + repr(e)))
    finally:
        dist.destroy_process_group()


def _cases(world, seed):
    rnd = random.Random(seed)
    cases = []
    shapes = {1: [([5], 3 * TILE + 100), ([131], 2 * TILE + 8)],
              2: [([3, 2], 5 * TILE + 1000), ([2, 2], 64 * TILE), ([4, 0], TILE + 4), ([130, 3], 2 * TILE)],
              3: [([2, 1, 3], 9 * TILE + 12), ([1, 1, 1], 3 * TILE)],
              4: [([2, 1, 0, 3], 10 * TILE + 4)]}[world]
    for clients, P in shapes:
        for mode in ("torch", "numpy"):
            order = [(s, j) for s in range(world) for j in range(clients[s])]
            rnd.shuffle(order)
            weights = [float(1 + (37 * k) % 100) if mode == "torch" else rnd.random() * 2 + 0.05 for k in range(len(order))]
            cases.append((P, clients, order, weights, mode))
    return cases


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_client_sharded_exchange_exact_reduce_bounded(world):
    import torch.multiprocessing as mp

    cases = _cases(world, 100 + world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    total = {}
    for rank, out in res:
        assert isinstance(out, list), out
        for P, clients, mode, exact, gathered, within, differ, n in out:
            assert exact, f"rank {rank} {clients} P={P} {mode}: exchange bucket not bit-exact"
            assert gathered, f"rank {rank} {clients} P={P} {mode}: gathered model differs"
            assert within, f"rank {rank} {clients} P={P} {mode}: reduce result outside the summation bound"
            total[(P, clients, mode)] = total.get((P, clients, mode), 0) + n
    for (P, clients, mode), n in total.items():
        assert n == P
