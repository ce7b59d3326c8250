"""Client-sharded ingest (nvflare_amd/client_shards.py) on CPU: the exchange plan, and the all-to-all over
gloo (world sizes 2 and 3) with host tensors standing in for the device slabs.

The HIP kernel cannot run here, so after the exchange each rank rebuilds every client's bucket rows from the
receive buffer through the plan's (offset, tile stride) runs and aggregates them with the C oracle (test
infrastructure), chaining runs through the accumulator exactly as the device launches do.  The result must
equal, bit for bit, the oracle over the original whole updates in arrival order, sliced to the bucket; the
rebuilt rows must equal the originals.  The GPU side is tests/test_gpu_client_shards.py."""

import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nvflare_amd.client_shards import TILE, ExchangePlan, exchange, exchange_chunks


def test_plan_geometry():
    p = ExchangePlan(3 * TILE * 2 + 1000, [3, 1, 0])
    assert p.world == 3 and p.n_tiles == 7
    assert p.buckets[0][0] == 0 and p.buckets[-1][1] == p.P
    for b in range(3):
        t0, t1 = p.tile_range(b)
        b0, b1 = p.buckets[b]
        assert t0 * TILE == b0 and (t1 - 1) * TILE < max(b1, 1) <= t1 * TILE or b1 == b0
    for s in range(3):  # what s sends to b is what b receives from s
        for b in range(3):
            assert p.send_splits(s)[b] == p.recv_splits(b)[s]
        t0, t1 = p.tile_range(s)  # everything but its own bucket leaves the rank
        assert sum(p.send_splits(s)) + (t1 - t0) * TILE * p.clients[s] == (p.slab_elems(s) if p.clients[s] else 0)
        assert p.send_splits(s)[s] == 0 and p.recv_splits(s)[s] == 0
    assert p.recv_offsets(1) == [0, p.recv_splits(1)[0], p.recv_splits(1)[0] + p.recv_splits(1)[1]]
    assert p.bucket_pad() % TILE == 0 and p.bucket_pad() >= max(p.bucket_len(b) for b in range(3))


def test_plan_runs_group_equal_strides():
    p = ExchangePlan(6 * TILE, [2, 2, 1])
    order = [(0, 1), (1, 0), (2, 0), (0, 0), (1, 1)]
    runs = p.exchange_runs(0, order)
    # ranks 0 and 1 share a tile stride (2 clients each): one run until rank 2's client breaks it
    assert [r[0] for r in runs] == [2 * TILE, TILE, 2 * TILE]
    assert [r[2] for r in runs] == [[0, 1], [2], [3, 4]]
    offs = p.recv_offsets(0)
    assert runs[0][1] == [(True, TILE), (False, offs[1])]  # own client 1 from the slab (bucket 0 at tile 0)
    assert p.exchange_runs(1, order)[0][1] == [(False, offs[0] + TILE), (True, p.tile_range(1)[0] * 2 * TILE)]


def test_plan_rejects_bad_orders():
    p = ExchangePlan(TILE, [2, 1])
    with pytest.raises(ValueError):
        p.check_order([(0, 0), (0, 0)])
    with pytest.raises(ValueError):
        p.check_order([(1, 1)])
    with pytest.raises(ValueError):
        ExchangePlan(TILE, [])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _tiled_slab(plan, rows):
    """Host stand-in of a rank's device slab: [tile][slot][TILE] (TiledLayout)."""
    ts = max(len(rows), 1) * TILE  # plan.tstride(rank)
    slab = np.zeros(plan.n_tiles * ts, dtype=np.float32)
    for j, r in enumerate(rows):
        padded = np.zeros(plan.n_tiles * TILE, dtype=np.float32)
        padded[: r.size] = r
        slab.reshape(plan.n_tiles, -1)[:, j * TILE:(j + 1) * TILE] = padded.reshape(plan.n_tiles, TILE)
    return slab


def _worker(rank, world, port, P, clients, order, weights, mode, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import fedavg_oracle as orc

        plan = ExchangePlan(P, clients)
        gid = {}  # (rank, slot) -> global client id (its generator row)
        for s in range(world):
            for j in range(clients[s]):
                gid[(s, j)] = len(gid)
        cols = np.arange(P, dtype=np.uint64)
        mine = [orc.synth_values(7, gid[(rank, j)], cols) for j in range(clients[rank])]
        slab = torch.from_numpy(_tiled_slab(plan, mine))
        recv = torch.full((plan.recv_elems(rank),), float("nan"), dtype=torch.float32)
        exchange(plan, rank, slab, recv, max_peer_bytes=chunk)
        bufs = {False: recv.numpy(), True: slab.numpy()}
        b0, b1 = plan.buckets[rank]
        n = b1 - b0
        omode = orc.MODE_TORCH if mode == "torch" else orc.MODE_NUMPY
        count = None
        for w in weights:
            count = w if count is None else count + w
        acc = None
        got_rows = {}
        runs = plan.exchange_runs(rank, order)
        for i, (ts, offs, pos) in enumerate(runs):
            rows = []
            for (own, o), q_ in zip(offs, pos):
                # logical element e of the bucket lives at o + (e // TILE) * ts + e % TILE
                e = np.arange(n)
                row = bufs[own][o + (e // TILE) * ts + e % TILE] if n else np.zeros(0, np.float32)
                rows.append(row)
                got_rows[order[q_]] = row
            last = i == len(runs) - 1
            fin = None if last else orc.FIN_NONE
            if n:
                acc = orc.fedavg_c(rows, [weights[q_] for q_ in pos], omode, fin=fin, count=count, acc_in=acc)
        full = [orc.synth_values(7, gid[c], cols) for c in order]
        want = orc.fedavg_c(full, weights, omode)[b0:b1] if n else np.zeros(0, np.float32)
        rows_ok = all(np.array_equal(got_rows[c], orc.synth_values(7, gid[c], cols)[b0:b1]) for c in order)
        got = acc if n else np.zeros(0, np.float32)
        q.put((rank, rows_ok, got.view(np.uint32).tolist() == want.view(np.uint32).tolist(), n))
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, repr(e), False, -1))
    finally:
        dist.destroy_process_group()


def test_exchange_chunks_cover_the_splits():
    """Chunked calls move exactly the plan's per-peer splits, in contiguous, non-overlapping pieces."""
    p = ExchangePlan(37 * TILE + 12, [3, 1, 0, 2])
    for rank in range(p.world):
        for limit in (1, 2 * TILE * 4 * 3, 1 << 30):
            chunks = exchange_chunks(p, rank, limit)
            if limit == 1:
                assert len(chunks) == max(t1 - t0 for t0, t1 in (p.tile_range(b) for b in range(p.world)))
            for peer in range(p.world):
                for side, splits in ((0, p.send_splits(rank)), (1, p.recv_splits(rank))):
                    pieces = [c[side][peer] for c in chunks if c[side][peer][1]]
                    assert sum(n for _, n in pieces) == splits[peer]
                    for (o0, n0), (o1, _) in zip(pieces, pieces[1:]):
                        assert o0 + n0 == o1
            # every peer's chunk c carries the same tile sub-range on both ends
            for c in chunks:
                for s in range(p.world):
                    assert c[1][s][1] == exchange_chunks(p, s, limit)[chunks.index(c)][0][rank][1]


@pytest.mark.parametrize("chunk", [1 << 28, 1])
@pytest.mark.parametrize("mode", ["torch", "numpy"])
@pytest.mark.parametrize("clients,P", [([2, 2], 5 * TILE + 1000), ([3, 1], 2 * TILE), ([2, 0, 3], 7 * TILE + 8),
                                       ([1, 1, 1], 2 * TILE + 4),
                                       ([3, 0, 2, 1, 4, 1, 1, 2], 13 * TILE + 52)])  # eight ranks, one empty
def test_exchange_gloo_matches_oracle(clients, P, mode, chunk):
    world = len(clients)
    order = [(s, j) for s in range(world) for j in range(clients[s])]
    random.Random(sum(clients) * 31 + P).shuffle(order)
    rnd = random.Random(P)
    weights = [rnd.random() * 3 + 0.1 for _ in order]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, clients, order, weights, mode, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, rows_ok, bits_ok, n in res:
        assert rows_ok is True, (rank, rows_ok)
        assert bits_ok, f"rank {rank}: bucket of {n} values differs from the oracle"
    assert sum(r[3] for r in res) == P
