"""A host-memory stand-in for ``nvflare_amd.device.DeviceContext`` -- TEST INFRASTRUCTURE ONLY.

It lets the CPU suite drive the engine's host logic (slabs, slots, arenas, folding, chaining, deferred
rounds) without a GPU: "device memory" is numpy byte arrays at fake addresses, copies are synchronous, and
the accumulate entry points restate the kernels' per-element sequence with the oracle's numpy
restatements.  It checks the engine's bookkeeping -- which bytes go where, in which order, into which
launch -- not the kernels (the GPU suite does that against the same oracle).  Never used by the product.
"""

from __future__ import annotations

import bisect
import threading

import numpy as np

from nvflare_amd import _native as N
from oracle import fedavg_oracle as orc

_NP = {N.FEDAVG_F32: np.float32, N.FEDAVG_F64: np.float64, N.FEDAVG_I32: np.int32, N.FEDAVG_I64: np.int64,
       N.FEDAVG_F16: np.float16, N.FEDAVG_BF16: np.uint16, N.FEDAVG_U8: np.uint8, N.FEDAVG_I8: np.int8,
       N.FEDAVG_I16: np.int16, N.FEDAVG_BOOL: np.bool_, N.FEDAVG_U16: np.uint16, N.FEDAVG_U32: np.uint32,
       N.FEDAVG_U64: np.uint64}


class FakeBuffer:
    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        self.ptr = ctx._malloc(self.nbytes)

    def close(self):
        if self.ptr:
            self.ctx._free(self.ptr)
        self.ptr = 0


class FakeDeviceContext:
    def __init__(self, device=0, total_bytes=1 << 34):
        self.device = device
        self.lock = threading.RLock()
        self.total_bytes = total_bytes
        self.num_cus = 256
        self._next = 1 << 40
        self._bases = []  # sorted allocation base addresses
        self._mem = {}  # base -> bytearray-backed numpy uint8 array
        self.launches = []

    # -- memory -------------------------------------------------------------------------------------
    def _malloc(self, nbytes):
        base = self._next
        self._next += (max(nbytes, 1) + 4095) // 4096 * 4096 + 4096
        bisect.insort(self._bases, base)
        self._mem[base] = np.full(max(nbytes, 1), 0xAB, dtype=np.uint8)  # poison: never read unwritten bytes
        return base

    def _free(self, base):
        self._bases.remove(base)
        self._mem[base][:] = 0xCD  # poison freed memory (catches use-after-free)
        del self._mem[base]

    def _view(self, ptr, nbytes):
        i = bisect.bisect_right(self._bases, ptr) - 1
        if i < 0:
            raise ValueError(f"fake device: bad pointer {ptr:#x}")
        base = self._bases[i]
        mem = self._mem[base]
        off = ptr - base
        if off < 0 or off + nbytes > mem.size:
            raise ValueError(f"fake device: access [{off}, {off + nbytes}) outside allocation of {mem.size} bytes")
        return mem[off:off + nbytes]

    def alloc(self, nbytes):
        return FakeBuffer(self, nbytes)

    def mem_info(self):
        return self.total_bytes, self.total_bytes

    def sync(self):
        pass

    # -- copies ---------------------------------------------------------------------------------------
    def h2d_ptr(self, dst, src_ptr, nbytes):
        import ctypes

        if nbytes:
            self._view(dst, nbytes)[:] = np.frombuffer((ctypes.c_char * nbytes).from_address(src_ptr), np.uint8)

    def h2d(self, dst, host):
        a = np.ascontiguousarray(host)
        self._view(dst, a.nbytes)[:] = a.view(np.uint8).reshape(-1)

    def _tiled_write(self, base, tile_b, stride_b, logical_off, data):
        b = logical_off
        pos = 0
        while pos < data.size:
            t, r = divmod(b, tile_b)
            n = min(tile_b - r, data.size - pos)
            self._view(base + t * stride_b + r, n)[:] = data[pos:pos + n]
            b += n
            pos += n

    def h2d_tiled_multi(self, base, tile_b, stride_b, pieces):
        import ctypes

        for off, ptr, nbytes in pieces:
            if nbytes:
                data = np.frombuffer((ctypes.c_char * nbytes).from_address(ptr), np.uint8).copy()
                self._tiled_write(base, tile_b, stride_b, off, data)

    def d2d_tiled(self, base, tile_b, stride_b, logical_off, src, nbytes):
        self._tiled_write(base, tile_b, stride_b, logical_off, self._view(src, nbytes).copy())

    def host_register(self, arr):
        self.registered = getattr(self, "registered", 0) + 1  # page-locking has no effect on the CPU

    def d2h(self, host, src):
        host.reshape(-1).view(np.uint8)[:] = self._view(src, host.nbytes)

    def d2h_multi(self, host, src, pieces):
        assert host.flags.c_contiguous
        flat = host.reshape(-1).view(np.uint8)
        for ho, do, nb in pieces:
            assert 0 <= ho and ho + nb <= flat.size, "d2h_multi piece outside the host array"
            flat[ho:ho + nb] = self._view(src + do, nb)
        self.d2h_multi_calls = getattr(self, "d2h_multi_calls", 0) + 1

    def mark(self, ready_bytes):
        marks = self.__dict__.setdefault("marks", [])
        assert not marks or ready_bytes >= marks[-1], "marks must be non-decreasing"
        marks.append(int(ready_bytes))

    def marks_reset(self):
        self.__dict__.pop("marks", None)

    def d2h_marked(self, host, src):
        marks = self.__dict__.pop("marks", [])
        assert marks and marks[-1] >= host.nbytes, "the last mark must cover the whole copy"
        self.marked_copies = getattr(self, "marked_copies", 0) + 1
        self.d2h(host, src)

    def d2d(self, dst, src, nbytes):
        self._view(dst, nbytes)[:] = self._view(src, nbytes).copy()

    def memset(self, dst, value, nbytes):
        self._view(dst, nbytes)[:] = value

    # -- compute --------------------------------------------------------------------------------------
    @staticmethod
    def _agg(rows, weights, op, fin, count, acc_in, fmt=None, scalar=None):
        """The kernels' per-element sequence (oracle restatements).  rows: fp32 / fp16 / fp64 arrays.
        ``scalar``: bool mask of 16-bit elements that take torch's scalar-loop step (torch mode)."""
        if fmt is not None:  # 16-bit totals (fmt "float16" | "bfloat16"); rows/acc_in are fp32 values
            if op == N.FEDAVG_OP_NUMPY:
                t = None if acc_in is None else acc_in.astype(np.float16)
                for r, w in zip(rows, weights):
                    p = r.astype(np.float16) * np.float16(w)
                    t = p if t is None else t + p
                if fin == N.FEDAVG_FIN_SCALE:
                    t = t * np.float16(1.0 / count)
                return t.astype(np.float32)
            weighted = op == N.FEDAVG_OP_TORCH
            t = acc_in
            for r, w in zip(rows, weights):
                if t is None:
                    t = orc.round16(r * np.float32(w), fmt) if weighted else r.copy()
                elif weighted:
                    a = np.float64(orc.round16(np.float32(w), fmt))
                    vec = orc.round16((r.astype(np.float64) * a + t.astype(np.float64)).astype(np.float32), fmt)
                    if scalar is not None:
                        sc = orc.round16(t + orc.round16(r * np.float32(a), fmt), fmt)
                        vec = np.where(scalar, sc, vec)
                    t = vec
                else:
                    t = orc.round16(t + r, fmt)
            if fin == N.FEDAVG_FIN_DIV:
                t = orc.round16(t / np.float32(count), fmt)
            elif fin == N.FEDAVG_FIN_SCALE:
                t = orc.round16(t * orc.round16(np.float32(1.0 / count), fmt), fmt)
            return t
        mode = orc.MODE_TORCH if op == N.FEDAVG_OP_TORCH else orc.MODE_NUMPY
        acc_t = rows[0].dtype if rows else acc_in.dtype
        if acc_t in (np.float32, np.float64):  # the C restatement: torch steps are one correctly rounded fma
            fin_c = {N.FEDAVG_FIN_SCALE: orc.FIN_NUMPY_SCALE, N.FEDAVG_FIN_DIV: orc.FIN_TORCH_DIV}.get(fin, orc.FIN_NONE)
            if not rows:
                return orc.fedavg_c([], [], mode, fin=fin_c, count=count, acc_in=acc_in)
            return orc.fedavg_c([np.ascontiguousarray(r, dtype=acc_t) for r in rows], weights, mode,
                                weighted=op != N.FEDAVG_OP_UNWEIGHTED, fin=fin_c, count=count, acc_in=acc_in)
        t = None if acc_in is None else acc_in.copy()
        with np.errstate(all="ignore"):
            for r, w in zip(rows, weights):
                wv = acc_t.type(w) if op != N.FEDAVG_OP_UNWEIGHTED else None
                r = r.astype(acc_t)
                if t is None:
                    t = r * wv if op != N.FEDAVG_OP_UNWEIGHTED else r.copy()
                elif op == N.FEDAVG_OP_UNWEIGHTED:
                    t = t + r
                elif mode == orc.MODE_TORCH:
                    t = (r.astype(np.float64) * np.float64(wv) + t.astype(np.float64)).astype(acc_t) \
                        if acc_t == np.float32 else r * wv + t
                else:
                    t = t + r * wv
            if fin == N.FEDAVG_FIN_SCALE:
                t = t * acc_t.type(1.0 / count)
            elif fin == N.FEDAVG_FIN_DIV:
                t = t / acc_t.type(count)
        return t

    def _read_tiled(self, base, tile, stride, begin, end, esize, dtype):
        out = np.empty(end - begin, dtype=dtype)
        flat = out.view(np.uint8)
        i = begin
        while i < end:
            t, r = divmod(i, tile)
            n = min(tile - r, end - i)
            flat[(i - begin) * esize:(i - begin + n) * esize] = self._view(base + (t * stride + r) * esize, n * esize)
            i += n
        return out

    def accumulate_tiled(self, bases, weights, tile, stride, begin, end, out_ptr, op, fin, count=1.0,
                         acc_in_ptr=None):
        self.launches.append(("tiled", len(bases), begin, end))
        rows = [self._read_tiled(b, tile, stride, begin, end, 4, np.float32) for b in bases]
        acc = None if acc_in_ptr is None else self._view(acc_in_ptr + begin * 4, (end - begin) * 4).view(np.float32).copy()
        res = self._agg(rows, weights, op, fin, count, acc)
        self._view(out_ptr + begin * 4, (end - begin) * 4)[:] = res.astype(np.float32).view(np.uint8)

    def accumulate_tiled16(self, fmt, bases, weights, tile, stride, begin, end, out_ptr, op, fin, count=1.0,
                           acc_in_ptr=None, tails=None):
        self.launches.append(("tiled16", len(bases), begin, end))
        name = "bfloat16" if fmt == N.FEDAVG_BF16 else "float16"

        def vals(raw):
            return orc.bf16_bits_to_f32(raw) if name == "bfloat16" else raw.view(np.float16).astype(np.float32)

        rows = [vals(self._read_tiled(b, tile, stride, begin, end, 2, np.uint16)) for b in bases]
        acc = None if acc_in_ptr is None else vals(self._view(acc_in_ptr + begin * 2, (end - begin) * 2).view(np.uint16).copy())
        scalar = None
        if tails is not None and op == N.FEDAVG_OP_TORCH:
            t = np.asarray(tails, dtype=np.int64)
            t = t[(t >= begin) & (t < end)]
            if t.size:
                scalar = np.zeros(end - begin, dtype=bool)
                scalar[t - begin] = True
        res = self._agg(rows, weights, op, fin, count, acc, fmt=name, scalar=scalar)
        bits = orc.f32_to_bf16_bits(res) if name == "bfloat16" else res.astype(np.float16).view(np.uint16)
        self._view(out_ptr + begin * 2, (end - begin) * 2)[:] = bits.view(np.uint8)

    def accumulate_tiled64(self, bases, weights, tile, stride, begin, end, out_ptr, op, fin, count=1.0,
                           acc_in_ptr=None):
        self.launches.append(("tiled64", len(bases), begin, end))
        rows = [self._read_tiled(b, tile, stride, begin, end, 8, np.float64) for b in bases]
        acc = None if acc_in_ptr is None else self._view(acc_in_ptr + begin * 8, (end - begin) * 8).view(np.float64).copy()
        res = self._agg(rows, weights, op, fin, count, acc)
        self._view(out_ptr + begin * 8, (end - begin) * 8)[:] = np.asarray(res, dtype=np.float64).view(np.uint8)

    def accumulate(self, rows, weights, n, out_ptr, in_dt, acc_dt, op, fin, count, acc_in_ptr=None):
        self.launches.append(("rows", len(rows), 0, n))
        tin, tacc = np.dtype(_NP[in_dt]), np.dtype(_NP[acc_dt])
        if acc_dt in (N.FEDAVG_F16, N.FEDAVG_BF16):
            name = "bfloat16" if acc_dt == N.FEDAVG_BF16 else "float16"

            def vals(raw):
                return orc.bf16_bits_to_f32(raw) if name == "bfloat16" else raw.view(np.float16).astype(np.float32)

            rs = [vals(self._view(p, n * 2).view(np.uint16).copy()) for p in rows]
            acc = None if acc_in_ptr is None else vals(self._view(acc_in_ptr, n * 2).view(np.uint16).copy())
            res = self._agg(rs, weights, op, fin, count, acc, fmt=name)
            bits = orc.f32_to_bf16_bits(res) if name == "bfloat16" else res.astype(np.float16).view(np.uint16)
            self._view(out_ptr, n * 2)[:] = bits.view(np.uint8)
            return
        rs = [self._view(p, n * tin.itemsize).view(tin).astype(tacc) for p in rows]
        acc = None if acc_in_ptr is None else self._view(acc_in_ptr, n * tacc.itemsize).view(tacc).copy()
        res = self._agg(rs, weights, op, fin, count, acc)
        self._view(out_ptr, n * tacc.itemsize)[:] = np.asarray(res, dtype=tacc).view(np.uint8)


def fake_engine(max_resident_bytes=None, slab_slots=None):
    """A DeviceFedAvg whose context is a FakeDeviceContext."""
    from nvflare_amd.engine import DeviceFedAvg

    e = DeviceFedAvg(device=0, max_resident_bytes=max_resident_bytes, slab_slots=slab_slots)
    e._ctx = FakeDeviceContext()
    return e


class FakeBenchContext(FakeDeviceContext):
    """FakeDeviceContext with the entry points bench.py drives (launch tuning, synthetic fill, the fused Adam step,
    timing, launch counts, gathers): bench.main() runs on it in the CPU suite (tests/test_cpu_bench_world8.py)."""

    _SQRT = {0: "ieee", 1: "torch_cpu", 2: "torch_cpu_amd"}

    def __init__(self, device=0, total_bytes=1 << 34):
        super().__init__(device, total_bytes)
        self._t0 = None

    def set_launch(self, blocks_per_cu=0, unroll=0):
        pass

    def set_variant(self, variant=0):
        pass

    def launch_count(self):
        return len(self.launches)

    def timing_begin(self):
        import time

        self._t0 = time.perf_counter()

    def timing_end(self):
        import time

        return (time.perf_counter() - self._t0) * 1e3

    def fill_synthetic_f32(self, dst_ptr, n, seed, row, col0=0, tile=0, tile_stride=0):
        vals = orc.synth_values(seed, row, np.arange(col0, col0 + n, dtype=np.uint64)).astype(np.float32)
        if tile:
            self._tiled_write(dst_ptr, tile * 4, tile_stride * 4, 0, vals.view(np.uint8))
        else:
            self._view(dst_ptr, n * 4)[:] = vals.view(np.uint8)

    def gather_f32(self, src_ptr, idx):
        idx = np.asarray(idx, dtype=np.uint64)
        return np.array([self._view(src_ptr + 4 * int(i), 4).view(np.float32)[0] for i in idx], dtype=np.float32)

    def accumulate_tiled_epi(self, bases, weights, tile, stride, begin, end, out_ptr, op, fin, count, epilogue,
                             acc_in_ptr=None):
        """Aggregation + the fused Adam step (the only epilogue bench.py's spot check replays), by the oracle."""
        assert epilogue.kind == N.FEDAVG_EPI_ADAM, "the fake bench context restates the Adam epilogue only"
        self.launches.append(("tiled_epi", len(bases), begin, end))
        rows = [self._read_tiled(b, tile, stride, begin, end, 4, np.float32) for b in bases]
        d = np.asarray(self._agg(rows, weights, op, fin, count, None), dtype=np.float32)
        n = end - begin
        p, m, v = (self._view(ptr + begin * 4, n * 4).view(np.float32)
                   for ptr in (epilogue.param, epilogue.state1, epilogue.state2))
        hp = dict(lr=epilogue.lr, beta1=epilogue.beta1, beta2=epilogue.beta2, eps=epilogue.eps)
        orc.epilogue_apply(d, orc.EPI_ADAM, p=p, m=m, v=v, step=float(epilogue.step),
                           torch_cpu_sqrt=self._SQRT[epilogue.torch_sqrt], **hp)
        if out_ptr:
            self._view(out_ptr + begin * 4, n * 4)[:] = d.view(np.uint8)
