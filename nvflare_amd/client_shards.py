"""Client-sharded ingest across ranks (one process per GPU): each rank receives WHOLE updates of its own
clients, and the ranks turn that into the parameter-bucket aggregation of SURVEY.md section 8(e).

The reference aggregates every client on one host (``weighted_aggregation_helper.py:153-240``).  When the
stacked updates overflow one GPU (config 4: 256 clients x 350 M fp32 = 358 GB) and the server's ranks each
terminate a subset of the client connections, the updates land *client-sharded*: rank s holds K_s complete
updates.  Two ways to finish the aggregation over xGMI, both here:

* ``strategy="exchange"`` (default, bit-exact): one RCCL all-to-all moves bucket b of every client to rank
  b (4·P·K_s·(G-1)/G bytes out of rank s; a rank's own clients stay in its slab), then rank b runs the arrival-ordered kernel over ALL K clients
  on its bucket -- the per-element operation sequence of the reference, so the bits equal the one-GPU
  result and the oracle.  The all-to-all needs no repacking on either side: a client's slab is tiled
  ``[tile][slot][4096]`` (``TiledLayout``), so a bucket (a whole-tile range) is ONE contiguous chunk of
  every sender's slab, and on the receiver client (s, j) of the chunk from rank s is an ordinary tiled row
  (base ``off_s + j·4096``, tile stride ``K_s·4096``) that the kernel reads in place.  Consecutive clients
  of the arrival order whose tile strides agree go in one launch; the runs chain through the fp32
  accumulator (``acc_in``), which is the kernel's own running value, so chaining changes no bits.
* ``strategy="reduce"`` (the north_star's "RCCL reduce"; NOT bit-exact): each rank sums its own clients in
  their arrival order (fp32 partial, no finalisation), one RCCL reduce-scatter adds the partials bucket by
  bucket, and each rank finalises its bucket.  It moves only 4·P·(G-1)/G bytes per rank, but it changes
  the association of the sum (about half the elements differ in the last bits), so
  it is tolerance-checked (``tests/test_gpu_client_shards.py``: within the standard recursive-summation
  bound of an fp64 reference) and reported separately, never as the drop-in result.

Either way the result is bucket-sharded (rank b holds ``bucket_ranges(P, G)[b]``); ``gather_result``
all-gathers it when every rank needs the whole model.  The arithmetic is the HIP library's
(``DeviceContext.accumulate_tiled``, launched on the same torch stream as the RCCL calls, so they are
ordered without host synchronisation); there is no CPU path.  With gloo and device tensors (the
one-GPU rehearsal, several ranks sharing ``cuda:0``) the collectives go through host copies.
"""

from __future__ import annotations

from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from .sharding import bucket_ranges

TILE = 4096  # elements per client segment per tile (TiledLayout default, BUCKET_ALIGN)


@dataclass
class ExchangePlan:
    """Geometry of a client-sharded aggregation: P params per client, ``clients[s]`` clients on rank s."""

    P: int
    clients: List[int]
    tile: int = TILE
    buckets: List[Tuple[int, int]] = field(init=False)

    def __post_init__(self):
        if self.P < 0 or any(k < 0 for k in self.clients) or not self.clients:
            raise ValueError("need P >= 0 and a non-negative client count per rank")
        self.buckets = bucket_ranges(self.P, len(self.clients), self.tile)

    @property
    def world(self) -> int:
        return len(self.clients)

    @property
    def n_tiles(self) -> int:
        return (self.P + self.tile - 1) // self.tile

    def tile_range(self, b: int) -> Tuple[int, int]:
        b0, b1 = self.buckets[b]
        return b0 // self.tile, (b1 + self.tile - 1) // self.tile

    def bucket_len(self, b: int) -> int:
        b0, b1 = self.buckets[b]
        return b1 - b0

    def bucket_pad(self) -> int:
        """Largest bucket rounded up to whole tiles: the per-rank chunk of the padded collectives."""
        return max((t1 - t0) for t0, t1 in (self.tile_range(b) for b in range(self.world))) * self.tile

    def tstride(self, s: int) -> int:
        """Tile stride (elements) of rank s's client slab: its clients' segments of one tile, back to back."""
        return max(self.clients[s], 1) * self.tile

    def slab_elems(self, s: int) -> int:
        return self.n_tiles * self.tstride(s)

    def slot_offset(self, j: int) -> int:
        """Element offset of local client j's first segment in its rank's slab."""
        return j * self.tile

    def send_splits(self, s: int) -> List[int]:
        """Elements rank s sends to each rank b: bucket b's tiles of all its clients (one contiguous chunk);
        nothing to itself -- its own clients' bucket rows are read from its slab in place."""
        return [0 if b == s else (t1 - t0) * self.tile * self.clients[s]
                for b, (t0, t1) in enumerate(self.tile_range(b) for b in range(self.world))]

    def recv_splits(self, b: int) -> List[int]:
        t0, t1 = self.tile_range(b)
        return [0 if s == b else (t1 - t0) * self.tile * self.clients[s] for s in range(self.world)]

    def recv_offsets(self, b: int) -> List[int]:
        offs, o = [], 0
        for n in self.recv_splits(b):
            offs.append(o)
            o += n
        return offs

    def recv_elems(self, b: int) -> int:
        return sum(self.recv_splits(b))

    def check_order(self, order: Sequence[Tuple[int, int]]) -> None:
        seen = set()
        for s, j in order:
            if not (0 <= s < self.world and 0 <= j < self.clients[s]):
                raise ValueError(f"client ({s}, {j}) is not on the plan")
            if (s, j) in seen:
                raise ValueError(f"client ({s}, {j}) appears twice in the arrival order")
            seen.add((s, j))

    def exchange_runs(self, b: int, order: Sequence[Tuple[int, int]]):
        """Rank b's launches after the all-to-all: maximal runs of consecutive arrival-order clients whose
        rows share a tile stride -> [(tstride, [(in_slab, element offset) of each row], [position of each
        client in ``order``])].  A row from another rank lies in the receive buffer; rank b's own clients'
        rows are read from its slab (same tile stride), ``in_slab`` True."""
        offs = self.recv_offsets(b)
        own0 = self.tile_range(b)[0] * self.tstride(b)
        runs: List[Tuple[int, List[Tuple[bool, int]], List[int]]] = []
        for pos, (s, j) in enumerate(order):
            ts = self.tstride(s)
            if not runs or runs[-1][0] != ts:
                runs.append((ts, [], []))
            runs[-1][1].append((True, own0 + j * self.tile) if s == b else (False, offs[s] + j * self.tile))
            runs[-1][2].append(pos)
        return runs


def _backend(group) -> str:
    import torch.distributed as dist

    return dist.get_backend(group)


# Largest message per peer per all-to-all call.  Measured on MI355X (torch 2.10 / RCCL 2.26.6): one
# all_to_all_single of 4.1 GB per peer returned with only the first half of the output written, no error
# (tools/debug_client_shards_nccl.py, profiles/r02/client_shards/) -- so the exchange goes in chunks.
MAX_PEER_CHUNK_BYTES = 256 << 20
# Smallest tile range the overlapped exchange hands to the kernel: 2048 tiles (8 Mi params) keep every block of
# a burst launch busy for several tiles; smaller pieces would be launch-ramp bound (fedavg_tiles.h)
MIN_KERNEL_TILES = 2048


def chunk_tiles(plan: ExchangePlan, max_peer_bytes: int = MAX_PEER_CHUNK_BYTES) -> int:
    """Tiles of a bucket per all-to-all call: at most ``max_peer_bytes`` per peer from the rank with the most
    clients (the same count on every rank, so every peer's chunk c is the same tile sub-range)."""
    kmax = max(max(plan.clients), 1)
    return max(1, max_peer_bytes // (plan.tile * 4 * kmax))


def exchange_chunks(plan: ExchangePlan, rank: int, max_peer_bytes: int = MAX_PEER_CHUNK_BYTES):
    """The exchange as a list of all-to-all calls, each moving at most ``max_peer_bytes`` per peer:
    [(send ranges, recv ranges)] with one (element offset, length) per peer, into rank ``rank``'s slab and
    receive buffer.  A sub-range of a bucket's tiles is contiguous on both sides (the slab is tile-major,
    and the chunk from rank s keeps its [tile][K_s][TILE] order), so no call repacks anything.  Call c
    carries tiles [c * chunk_tiles, (c + 1) * chunk_tiles) of every bucket."""
    T, W = plan.tile, plan.world
    ct = chunk_tiles(plan, max_peer_bytes)
    span = [t1 - t0 for t0, t1 in (plan.tile_range(b) for b in range(W))]
    n_chunks = max(1, -(-max(span) // ct))
    roffs = plan.recv_offsets(rank)
    out = []
    for c in range(n_chunks):
        lo = c * ct
        sends, recvs = [], []
        for b in range(W):  # to rank b: tiles [t0_b + lo, ...) of bucket b, all of my clients
            t0, t1 = plan.tile_range(b)
            n = 0 if b == rank else max(0, min(t1, t0 + lo + ct) - (t0 + lo))
            sends.append(((t0 + lo) * plan.tstride(rank), n * T * plan.clients[rank]))
        mine = span[rank]
        n_my = max(0, min(mine, lo + ct) - lo)
        for s in range(W):  # from rank s: the same tiles of my bucket, its clients
            recvs.append((roffs[s] + lo * T * plan.clients[s], 0 if s == rank else n_my * T * plan.clients[s]))
        out.append((sends, recvs))
    return out


def all_to_all(outs, inps, group=None) -> None:
    """List-form all-to-all (``outs[s]`` from rank s, ``inps[b]`` to rank b).  RCCL: grouped send/recv
    straight between the views.  gloo (CPU tests, the one-GPU rehearsal), which has only the single-tensor
    form: packed through one host buffer each way."""
    import torch
    import torch.distributed as dist

    if _backend(group) == "nccl":
        dist.all_to_all(list(outs), list(inps), group=group)
        return
    send = torch.cat([i.reshape(-1).cpu() for i in inps]) if inps else torch.empty(0)
    recv = torch.empty(sum(o.numel() for o in outs), dtype=outs[0].dtype)
    dist.all_to_all_single(recv, send, [o.numel() for o in outs], [i.numel() for i in inps], group=group)
    off = 0
    for o in outs:
        o.copy_(recv[off: off + o.numel()].view(o.shape))
        off += o.numel()


def exchange(plan: ExchangePlan, rank: int, send, recv, group=None, max_peer_bytes: int = MAX_PEER_CHUNK_BYTES):
    """Bucket b of every client to rank b: ``send`` is rank ``rank``'s slab, ``recv`` its receive buffer
    (1-D float32 tensors, ``plan.slab_elems`` / ``plan.recv_elems`` long).  Collective."""
    if plan.world == 1:
        return
    for sends, recvs in exchange_chunks(plan, rank, max_peer_bytes):
        all_to_all([recv[o: o + n] for o, n in recvs], [send[o: o + n] for o, n in sends], group)


def _pieces(n: int, max_peer_bytes: int):
    """[lo, hi) element ranges of an n-element per-peer message, each at most ``max_peer_bytes`` (fp32)."""
    step = max(1, int(max_peer_bytes) // 4)
    return [(lo, min(n, lo + step)) for lo in range(0, max(n, 1), step)] if n else [(0, 0)]


def reduce_scatter(out, inp, group=None, max_peer_bytes: int = MAX_PEER_CHUNK_BYTES) -> None:
    """SUM reduce-scatter of equal chunks (``inp`` = W rank-major chunks of ``out.numel()``), in calls of at
    most ``max_peer_bytes`` per peer (the all-to-all's limit: RCCL was seen to truncate a 4.1 GB message
    silently); gloo with device tensors goes through host copies."""
    import torch
    import torch.distributed as dist

    n = out.numel()
    W = inp.numel() // max(n, 1) if n else 1
    pieces = _pieces(n, max_peer_bytes)
    for lo, hi in pieces:
        if len(pieces) == 1:
            o_v, i_v = out, inp
        else:
            o_v = out[lo:hi]
            i_v = torch.cat([inp[b * n + lo: b * n + hi] for b in range(W)])  # rank-major piece
        if i_v.device.type == "cpu" or _backend(group) == "nccl":
            dist.reduce_scatter_tensor(o_v, i_v, op=dist.ReduceOp.SUM, group=group)
            continue
        o = o_v.new_empty(o_v.shape, device="cpu")
        dist.reduce_scatter_tensor(o, i_v.cpu(), op=dist.ReduceOp.SUM, group=group)
        o_v.copy_(o)


def all_gather(out, inp, group=None, max_peer_bytes: int = MAX_PEER_CHUNK_BYTES) -> None:
    """All-gather of equal chunks (``out`` = W rank-major copies of ``inp``), in calls of at most
    ``max_peer_bytes`` per peer; gloo with device tensors goes through host copies."""
    import torch
    import torch.distributed as dist

    n = inp.numel()
    W = out.numel() // max(n, 1) if n else 1
    pieces = _pieces(n, max_peer_bytes)
    for lo, hi in pieces:
        whole = len(pieces) == 1
        i_v = inp if whole else inp[lo:hi]
        o_v = out if whole else torch.empty(W * (hi - lo), dtype=out.dtype, device=out.device)
        if i_v.device.type == "cpu" or _backend(group) == "nccl":
            dist.all_gather_into_tensor(o_v, i_v, group=group)
        else:
            o = o_v.new_empty(o_v.shape, device="cpu")
            dist.all_gather_into_tensor(o, i_v.cpu(), group=group)
            o_v.copy_(o)
        if not whole:
            for b in range(W):
                out[b * n + lo: b * n + hi].copy_(o_v[b * (hi - lo): (b + 1) * (hi - lo)])


class ClientShardedFedAvg:
    """This rank's side of a client-sharded FedAvg over a process group (one rank per GPU).

    ``clients_per_rank[s]`` clients live on rank s; local client j is staged into slot j of this rank's
    tiled slab (``stage`` from host memory, or written in place through ``slot_ptr``).  ``aggregate(order,
    weights)`` takes the GLOBAL arrival order as (rank, local slot) pairs and the matching per-client
    weights (python floats, as ``DXOAggregator`` computes them), and returns this rank's bucket of the
    result as a device tensor.  ``mode`` "torch" / "numpy" / "unweighted" is the reference branch whose bits
    the exchange strategy reproduces (``weighted_aggregation_helper.py:181-240``).
    """

    def __init__(self, P: int, clients_per_rank: Sequence[int], group=None, device: Optional[int] = None,
                 mode: str = "torch", tile: int = TILE):
        import torch
        import torch.distributed as dist

        from . import _native as N
        from .device import DeviceContext

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if len(clients_per_rank) != self.world:
            raise ValueError(f"clients_per_rank has {len(clients_per_rank)} entries for a world of {self.world}")
        if tile != TILE:
            raise ValueError("tile must be 4096 (the bucket alignment)")
        ops = {"torch": (N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV), "numpy": (N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE),
               "unweighted": (N.FEDAVG_OP_UNWEIGHTED, N.FEDAVG_FIN_SCALE)}
        if mode not in ops:
            raise ValueError(f"mode must be one of {sorted(ops)}")
        self.mode = mode
        self.op, self.fin = ops[mode]
        self._fin_none = N.FEDAVG_FIN_NONE
        self.plan = ExchangePlan(int(P), [int(k) for k in clients_per_rank], tile)
        dev = torch.cuda.current_device() if device is None else int(device)
        self.device = torch.device("cuda", dev)
        self.ctx = DeviceContext.get(dev)
        self._stream = torch.cuda.Stream(self.device)  # collectives + kernels (see _torch_stream)
        self._kstream = torch.cuda.Stream(self.device)  # kernels overlapping the chunked all-to-all
        self.min_kernel_tiles = MIN_KERNEL_TILES
        f32 = torch.float32
        self.slab = torch.empty(max(self.plan.slab_elems(self.rank), 4), dtype=f32, device=self.device)
        self._recv = None  # allocated on the first exchange
        self.max_peer_bytes = MAX_PEER_CHUNK_BYTES  # per peer per all-to-all call (exchange_chunks)
        self._partial = None  # allocated on the first reduce
        pad = self.plan.bucket_pad()
        self.out = torch.empty(max(pad, 4), dtype=f32, device=self.device)

    # -- staging ------------------------------------------------------------------------------------
    def slot_ptr(self, j: int) -> int:
        """Device address of local client j's first segment (its segments repeat every ``plan.tstride``)."""
        if not 0 <= j < self.plan.clients[self.rank]:
            raise IndexError(f"local slot {j} out of range")
        return self.slab.data_ptr() + self.plan.slot_offset(j) * 4

    def stage(self, j: int, host) -> None:
        """Copy local client j's whole update (P fp32 values, C-contiguous host array) into its slot."""
        import numpy as np

        a = np.ascontiguousarray(host, dtype=np.float32).reshape(-1)
        if a.size != self.plan.P:
            raise ValueError(f"update has {a.size} values, the plan has P={self.plan.P}")
        self.ctx.h2d_tiled(self.slot_ptr(j), TILE * 4, self.plan.tstride(self.rank) * 4, 0, a.ctypes.data, a.nbytes)
        self.ctx.sync()

    def fill_synthetic(self, seed: int, client_ids: Sequence[int]) -> None:
        """Bench/test input: local slot j gets the device generator's row ``client_ids[j]`` (host twin:
        ``oracle.fedavg_oracle.synth_values``)."""
        for j, cid in enumerate(client_ids):
            self.ctx.fill_synthetic_f32(self.slot_ptr(j), self.plan.P, seed, int(cid), 0, TILE,
                                        self.plan.tstride(self.rank))
        self.ctx.sync()

    # -- aggregation ---------------------------------------------------------------------------------
    @contextmanager
    def _torch_stream(self):
        """Run the collectives and the library's kernels in order on ONE stream of this object's, fenced
        against the caller's current stream on entry and exit.  (Not the caller's stream itself: torch's
        default stream has the handle 0, which the library reads as "use your own stream".)"""
        import torch

        caller = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(caller)
        prev = self.ctx.stream()
        self.ctx.set_stream(self._stream.cuda_stream)
        try:
            with torch.cuda.stream(self._stream):
                yield
        finally:
            self.ctx.set_stream(prev)
            caller.wait_stream(self._stream)

    @staticmethod
    def _count(weights) -> float:
        c = None
        for w in weights:  # python float sum in arrival order (weighted_aggregation_helper.py:201,216)
            c = w if c is None else c + w
        return float(c)

    def _checked(self, order, weights):
        if len(order) != len(weights) or not order:
            raise ValueError("need one weight per client of a non-empty arrival order")
        self.plan.check_order(order)
        if len(order) != sum(self.plan.clients):
            raise ValueError("the arrival order must name every staged client exactly once")
        if self.mode == "unweighted":
            return list(order), [1.0] * len(order)
        return list(order), [float(w) for w in weights]

    def aggregate(self, order: Sequence[Tuple[int, int]], weights: Sequence[float], strategy: str = "exchange"):
        """This rank's bucket (``plan.buckets[rank]``) of the aggregate, a device tensor view of ``self.out``.
        Collective: every rank of the group calls it with the same order, weights and strategy."""
        if strategy not in ("exchange", "reduce"):
            raise ValueError("strategy must be 'exchange' or 'reduce'")
        order, weights = self._checked(order, weights)
        with self._torch_stream():
            if strategy == "exchange":
                self._exchange_overlapped(order, weights)
            else:
                self._reduce(order, weights)
        return self.out[: self.plan.bucket_len(self.rank)]

    def _exchange_overlapped(self, order, weights) -> None:
        """The exchange strategy with the kernels overlapping the all-to-all: the exchange goes in tile chunks
        (``exchange_chunks``) on the collectives' stream; as soon as the chunks received so far hold at least
        ``min_kernel_tiles`` tiles of this rank's bucket (or the last chunk is in), the arrival-ordered kernels
        over those tiles are launched on a second stream, fenced by an event after the chunk's all-to-all, while
        the next chunks are in flight.  Every element still sees the same launches (the runs chained through the
        accumulator over its tile), so the bits are those of ``exchange()`` + ``aggregate_exchanged``."""
        import torch

        p, r = self.plan, self.rank
        if self._recv is None:
            self._recv = torch.empty(max(p.recv_elems(r), 4), dtype=torch.float32, device=self.device)
        comm = torch.cuda.current_stream(self.device)
        kst = self._kstream
        kst.wait_stream(comm)
        prev = self.ctx.stream()
        self.ctx.set_stream(kst.cuda_stream)
        try:
            t0, t1 = p.tile_range(r)
            my_tiles = t1 - t0
            ct = chunk_tiles(p, self.max_peer_bytes)
            chunks = exchange_chunks(p, r, self.max_peer_bytes) if p.world > 1 else [None]
            end = (p.bucket_len(r) + 3) // 4 * 4
            done = 0
            for c, ch in enumerate(chunks):
                if ch is not None:
                    sends, recvs = ch
                    all_to_all([self._recv[o: o + n] for o, n in recvs], [self.slab[o: o + n] for o, n in sends],
                               self.group)
                arrived = my_tiles if c == len(chunks) - 1 else min(my_tiles, (c + 1) * ct)
                if arrived > done and (arrived - done >= self.min_kernel_tiles or arrived == my_tiles):
                    ev = torch.cuda.Event()
                    ev.record(comm)
                    kst.wait_event(ev)
                    self._launch_runs(order, weights, done * p.tile, min(arrived * p.tile, end))
                    done = arrived
            comm.wait_stream(kst)  # the caller's fence (``_torch_stream``) covers the kernels too
        finally:
            self.ctx.set_stream(prev)

    def _launch_runs(self, order, weights, begin: int, end: int) -> None:
        """The arrival-ordered kernels over bucket elements [begin, end) (after the exchange delivered them)."""
        if end <= begin:
            return
        p, r = self.plan, self.rank
        base = (self._recv.data_ptr(), self.slab.data_ptr())
        out = self.out.data_ptr()
        count = self._count(weights)
        runs = p.exchange_runs(r, order)
        for i, (ts, rows, pos) in enumerate(runs):
            last = i == len(runs) - 1
            self.ctx.accumulate_tiled([base[own] + o * 4 for own, o in rows], [weights[q] for q in pos], TILE, ts, begin,
                                      end, out, self.op, self.fin if last else self._fin_none, count,
                                      acc_in_ptr=out if i else None)

    def aggregate_exchanged(self, order: Sequence[Tuple[int, int]], weights: Sequence[float]):
        """The kernel half of the exchange strategy, after ``exchange()`` (timed apart by the bench)."""
        order, weights = self._checked(order, weights)
        with self._torch_stream():
            self._exchange_and_aggregate(order, weights)
        return self.out[: self.plan.bucket_len(self.rank)]

    def exchange(self) -> None:
        """The all-to-all alone (chunked, ``exchange``): bucket b of every client to rank b (``self._recv``).
        Collective."""
        import torch

        p, r = self.plan, self.rank
        if self._recv is None:
            self._recv = torch.empty(max(p.recv_elems(r), 4), dtype=torch.float32, device=self.device)
        exchange(p, r, self.slab, self._recv, self.group, self.max_peer_bytes)

    def _exchange_and_aggregate(self, order, weights) -> None:
        p, r = self.plan, self.rank
        if self._recv is None:
            raise RuntimeError("exchange() has not run")
        self._launch_runs(order, weights, 0, (p.bucket_len(r) + 3) // 4 * 4)

    def _reduce(self, order, weights) -> None:
        import torch

        p, r = self.plan, self.rank
        pad = p.bucket_pad()
        if self._partial is None:
            self._partial = torch.empty(max(pad * self.world, 4), dtype=torch.float32, device=self.device)
        mine = [(pos, j) for pos, (s, j) in enumerate(order) if s == r]
        part = self._partial.data_ptr()
        if mine:
            ts = p.tstride(r)
            bases = [self.slab.data_ptr() + p.slot_offset(j) * 4 for _, j in mine]
            ws = [weights[pos] for pos, _ in mine]
            for b in range(self.world):  # bucket b's partial at chunk b of the padded buffer
                b0, b1 = p.buckets[b]
                if b1 == b0:
                    continue
                # out + i for global i in [b0, b1) lands at chunk b; b0 is a multiple of 4096 (16 KiB aligned)
                self.ctx.accumulate_tiled(bases, ws, TILE, ts, b0, (b1 + 3) // 4 * 4, part + (b * pad - b0) * 4,
                                          self.op, self._fin_none, 1.0)
        else:
            self._partial.zero_()
        chunk = self.out[:pad]
        # the local kernels ran on torch's stream (set above), so the collective follows them in order
        reduce_scatter(chunk, self._partial[: pad * self.world], self.group, self.max_peer_bytes)
        end = (p.bucket_len(r) + 3) // 4 * 4
        if end:
            # finalise in place: K = 0 clients, acc_in = the reduced partial (fin only)
            self.ctx.accumulate_tiled([], [], TILE, TILE, 0, end, self.out.data_ptr(), self.op, self.fin,
                                      self._count(weights), acc_in_ptr=self.out.data_ptr())

    def gather_result(self):
        """The whole aggregate (P values) on every rank: all-gather of the padded buckets, then unpadded."""
        import torch

        p = self.plan
        pad = p.bucket_pad()
        full = torch.empty(pad * self.world, dtype=torch.float32, device=self.device)
        with self._torch_stream():
            all_gather(full, self.out[:pad], self.group, self.max_peer_bytes)
        return torch.cat([full[b * pad: b * pad + p.bucket_len(b)] for b in range(self.world)])
