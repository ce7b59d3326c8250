// hbm_pattern_probe.hip -- diagnostic only (not part of the product library): which HBM READ PATTERN
// sustains the most bandwidth on this chip, to tell how far the slab kernel's access pattern (every block
// streams its own 1 MiB tile; tiles dealt round-robin) sits from a chip-wide sequential sweep.
//   mode 0  grid:   grid-stride float4 sweep, U loads in flight per lane (the whole chip reads one window)
//   mode 1  chunk:  block b reads chunks b, b+G, ... of CH bytes sequentially (the slab kernel's pattern)
//   mode 2  chunk_lds: mode 1 through LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction),
//                   16 in flight per wave, nothing read back (the DMA is the consumer)
//   mode 3  chunk_pair: block b reads TWO chunks (b and b + n_chunks/2) alternately, U/2 loads each
//   mode 4  chunk_w: mode 1 plus 4 nontemporal float4 stores per lane per chunk (the slab kernel's
//                   result stream: 16 KiB per 1 MiB chunk) into the buffer's last 1/64
//   mode 6/7/8 chunk_w with buffer stores of cache policy sc1 / sc0 sc1 / plain (instead of nt)
//   mode 9  chunk_wb: results staged in LDS and written as a burst of 8 chunks' results (128 KiB) per block
//   mode 10 chunk_wb_sliced: mode 9 as a sequence of launches of blocks x 8 chunks each, so every launch's
//                   write burst starts chip-wide at about the same time (launch boundaries re-align the blocks)
//   mode 5  chunk_wd: mode 4 with each chunk's stores issued AFTER the next chunk's first load group, so the
//                   wait for those loads (vmcnt counts loads and stores in issue order) never waits on a store
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/hbm_pattern_probe.hip -o tools/build/libhbm_pattern_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(256) p_grid(const f32x4* __restrict__ src, int64_t n4, f32x4* __restrict__ sink) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    sink[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// chunk4 = chunk size in float4 (multiple of 256 * U)
template <int U>
__global__ void __launch_bounds__(256) p_chunk(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                               f32x4* __restrict__ sink) {
    f32x4 acc = {0, 0, 0, 0};
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const f32x4* p = src + c * chunk4 + threadIdx.x;
        for (int64_t j = 0; j < chunk4; j += 256 * U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + j + u * 256);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];
        }
    }
    sink[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int U>
__global__ void __launch_bounds__(256) p_chunk_w(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                                 f32x4* __restrict__ dst) {
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const f32x4* p = src + c * chunk4 + threadIdx.x;
        f32x4 acc[4] = {};
        for (int64_t j = 0; j < chunk4; j += 256 * U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + j + u * 256);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u % 4] += v[u];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(acc[q], dst + c * 1024 + q * 256 + threadIdx.x);
    }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int U, int AUX>
__global__ void __launch_bounds__(256) p_chunk_wp(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                                  f32x4* __restrict__ dst) {
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const f32x4* p = src + c * chunk4 + threadIdx.x;
        f32x4 acc[4] = {};
        for (int64_t j = 0; j < chunk4; j += 256 * U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + j + u * 256);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u % 4] += v[u];
        }
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst + c * 1024, 0, 16384, 0x00020000);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, acc[q]), r, (q * 256 + threadIdx.x) * 16, 0, AUX);
    }
}

template <int U>
__global__ void __launch_bounds__(256) p_chunk_wb(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                                  f32x4* __restrict__ dst) {
    __shared__ f32x4 stage[8][1024];  // 8 chunks x 16 KiB
    int n = 0;
    int64_t first = blockIdx.x;
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const f32x4* p = src + c * chunk4 + threadIdx.x;
        f32x4 acc[4] = {};
        for (int64_t j = 0; j < chunk4; j += 256 * U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + j + u * 256);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u % 4] += v[u];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) stage[n][q * 256 + threadIdx.x] = acc[q];  // own lanes only: no barrier
        if (++n == 8 || c + gridDim.x >= n_chunks) {
            for (int m = 0; m < n; ++m)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    __builtin_nontemporal_store(stage[m][q * 256 + threadIdx.x],
                                                dst + (first + (int64_t)m * gridDim.x) * 1024 + q * 256 + threadIdx.x);
            n = 0;
            first = c + gridDim.x;
        }
    }
}

template <int U>
__global__ void __launch_bounds__(256) p_chunk_wd(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                                  f32x4* __restrict__ dst) {
    f32x4 res[4] = {};
    int64_t prev = -1;
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const f32x4* p = src + c * chunk4 + threadIdx.x;
        f32x4 acc[4] = {};
        for (int64_t j = 0; j < chunk4; j += 256 * U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + j + u * 256);
            if (j == 0) {  // branch-free stores (the first chunk writes its own slot early; rewritten later)
                asm volatile("" ::: "memory");  // keep the stores behind this group's loads
                const int64_t tgt = prev >= 0 ? prev : c;
#pragma unroll
                for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(res[q], dst + tgt * 1024 + q * 256 + threadIdx.x);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u % 4] += v[u];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) res[q] = acc[q];
        prev = c;
    }
    if (prev >= 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(res[q], dst + prev * 1024 + q * 256 + threadIdx.x);
}

template <int U>
__global__ void __launch_bounds__(256) p_chunk_pair(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                                    f32x4* __restrict__ sink) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t half = n_chunks / 2;
    for (int64_t c = blockIdx.x; c < half; c += gridDim.x) {
        const f32x4* p = src + c * chunk4 + threadIdx.x;
        const f32x4* q = src + (c + half) * chunk4 + threadIdx.x;
        for (int64_t j = 0; j < chunk4; j += 256 * (U / 2)) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U / 2; ++u) {
                v[2 * u] = __builtin_nontemporal_load(p + j + u * 256);
                v[2 * u + 1] = __builtin_nontemporal_load(q + j + u * 256);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];
        }
    }
    sink[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// LDS-DMA: each wave owns a 16 KiB ring of 16 x 1 KiB slots; issue 16 DMAs, wait for the oldest 8, repeat.
__global__ void __launch_bounds__(256) p_chunk_lds(const f32x4* __restrict__ src, int64_t n_chunks, int64_t chunk4,
                                                   f32x4* __restrict__ sink) {
    __shared__ f32x4 ring[4][16][64];
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        // wave w reads quarter w of the chunk as a sequential run of 1 KiB pieces
        const int64_t q4 = chunk4 / 4;
        const f32x4* p = src + c * chunk4 + wave * q4 + lane;
        for (int64_t j = 0; j < q4; j += 64 * 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                __builtin_amdgcn_global_load_lds(p + j + u * 64, &ring[wave][((j / 512) & 1) * 8 + u][0], 16, 0, 2);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    sink[(int64_t)blockIdx.x * 256 + threadIdx.x] = ring[wave][lane % 16][lane];
}

// ---------------------------------------------------------------------------------------------------------
// R:1 read/write MIXES (round 3): the shape of a K-client aggregation is K reads per write (config 2: 8:1).
// The buffer is split into a read region of n_chunks chunks of R x 16 KiB and a write region of n_chunks x
// 16 KiB; chunk c's "result" (the sum of its R segments, 16 KiB) goes to write slot c.
//   mix 0  grid:      out[i] = sum_r in_r[i] over R separate arrays, grid-stride (a STREAM-style R-input triad)
//   mix 1  read:      the chunk stream alone (no writes): the read ceiling of this footprint
//   mix 2  tile:      chunk stream, each chunk's 16 KiB stored when it finishes (scattered small writes)
//   mix 3  burst:     REG chunks' results in registers + LDS chunks' results in LDS per block, stored at the end
//                     of a launch of blocks x (REG + LDS) chunks (the burst kernel's pattern, no arithmetic)
//   mix 7  write_aux: mix 4 through buffer stores with cache-policy bits (reg = 0 plain, 2 nt, 16 sc1, 17 sc0 sc1)
//   mix 8 / 9 multi:  G chunks per block per iteration, all their loads in flight, stores immediate / deferred (below)
//   mix 4  write:     the write region alone, 16 KiB per chunk per block (mix 5: grid-stride) -- with mix 1 the
//                     additive bound t_read + t_write of a mix whose reads and writes share the HBM data bus
// ---------------------------------------------------------------------------------------------------------
template <int R>
__global__ void __launch_bounds__(256) m_grid(const f32x4* __restrict__ src, int64_t n4, f32x4* __restrict__ dst) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        f32x4 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = __builtin_nontemporal_load(src + r * n4 + i);
        f32x4 acc = v[0];
#pragma unroll
        for (int r = 1; r < R; ++r) acc += v[r];
        __builtin_nontemporal_store(acc, dst + i);
    }
}

// one chunk of R x 1024 float4: min(R, 4) segments' loads in flight per lane (16 from R = 4 on), 4 float4 of
// result per lane
template <int R>
__device__ inline void m_chunk_sum(const f32x4* __restrict__ p, f32x4 (&acc)[4]) {
    constexpr int GR = R < 4 ? R : 4;
    static_assert(R % GR == 0, "R must be 1, 2, 3 or a multiple of 4");
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f32x4{0, 0, 0, 0};
#pragma unroll 1
    for (int g = 0; g < R; g += GR) {
        f32x4 v[GR * 4];
#pragma unroll
        for (int u = 0; u < GR * 4; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(g + u / 4) * 1024 + (u % 4) * 256);
#pragma unroll
        for (int u = 0; u < GR * 4; ++u) acc[u % 4] += v[u];
    }
}

// mix 8 / 9  multi (few-client shapes, round 4): every block takes G chunks per iteration (chunks base + j * grid,
// round-robin as the slab kernels deal tiles) and issues ALL their R x 4 x G loads per lane before any arithmetic --
// G x R x 64 B in flight per lane -- then stores the G results (mix 8), or holds them and stores them after the NEXT
// iteration's loads are issued (mix 9, DEFER: the stores never sit in front of loads the lane waits for)
template <int R, int G, bool DEFER>
__global__ void __launch_bounds__(256) m_multi(const f32x4* __restrict__ src, int64_t n_chunks, f32x4* __restrict__ dst) {
    f32x4 pend[G][4];
    int64_t pend_base = -1;
    const int64_t step = (int64_t)G * gridDim.x;
    for (int64_t base = blockIdx.x; base < n_chunks; base += step) {
        f32x4 v[G][R][4];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            int64_t c = base + (int64_t)j * gridDim.x;
            c = c < n_chunks ? c : n_chunks - 1;  // clamped: loads unconditional, stores masked
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    v[j][r][q] = __builtin_nontemporal_load(src + (c * R + r) * 1024 + q * 256 + threadIdx.x);
        }
        if constexpr (DEFER) {
            asm volatile("" ::: "memory");  // keep the held stores behind this iteration's loads
            if (pend_base >= 0) {
#pragma unroll
                for (int j = 0; j < G; ++j) {
                    const int64_t c = pend_base + (int64_t)j * gridDim.x;
                    if (c < n_chunks)
#pragma unroll
                        for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(pend[j][q], dst + c * 1024 + q * 256 + threadIdx.x);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            f32x4 acc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc[q] = v[j][0][q];
#pragma unroll
                for (int r = 1; r < R; ++r) acc[q] += v[j][r][q];
            }
            if constexpr (DEFER) {
#pragma unroll
                for (int q = 0; q < 4; ++q) pend[j][q] = acc[q];
            } else {
                const int64_t c = base + (int64_t)j * gridDim.x;
                if (c < n_chunks)
#pragma unroll
                    for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(acc[q], dst + c * 1024 + q * 256 + threadIdx.x);
            }
        }
        if constexpr (DEFER) pend_base = base;
    }
    if constexpr (DEFER) {
        if (pend_base >= 0) {
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const int64_t c = pend_base + (int64_t)j * gridDim.x;
                if (c < n_chunks)
#pragma unroll
                    for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(pend[j][q], dst + c * 1024 + q * 256 + threadIdx.x);
            }
        }
    }
}

template <int R, bool STORE>
__global__ void __launch_bounds__(256) m_tile(const f32x4* __restrict__ src, int64_t n_chunks, f32x4* __restrict__ dst,
                                              f32x4* __restrict__ sink) {
    f32x4 tot = {0, 0, 0, 0};
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        f32x4 acc[4];
        m_chunk_sum<R>(src + c * R * 1024 + threadIdx.x, acc);
        if constexpr (STORE) {
#pragma unroll
            for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(acc[q], dst + c * 1024 + q * 256 + threadIdx.x);
        } else {
            tot += acc[0] + acc[1] + acc[2] + acc[3];
        }
    }
    if constexpr (!STORE) sink[(int64_t)blockIdx.x * 256 + threadIdx.x] = tot;
}

template <int R, int REG, int LDS>
__global__ void __launch_bounds__(256) m_burst(const f32x4* __restrict__ src, int64_t c0, int64_t c_end,
                                               f32x4* __restrict__ dst) {
    f32x4 res[REG > 0 ? REG : 1][4];
    __shared__ f32x4 stage[LDS > 0 ? LDS * 1024 : 1];
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (c < c_end) m_chunk_sum<R>(src + c * R * 1024 + threadIdx.x, res[m]);
    }
#pragma unroll 1
    for (int m = 0; m < LDS; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)(REG + m) * gridDim.x;
        if (c < c_end) {
            f32x4 acc[4];
            m_chunk_sum<R>(src + c * R * 1024 + threadIdx.x, acc);
#pragma unroll
            for (int q = 0; q < 4; ++q) stage[m * 1024 + q * 256 + threadIdx.x] = acc[q];  // own lanes: no barrier
        }
    }
#pragma unroll 1
    for (int m = 0; m < LDS; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)(REG + m) * gridDim.x;
        if (c < c_end)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_nontemporal_store(stage[m * 1024 + q * 256 + threadIdx.x], dst + c * 1024 + q * 256 + threadIdx.x);
    }
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (c < c_end)
#pragma unroll
            for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(res[m][q], dst + c * 1024 + q * 256 + threadIdx.x);
    }
}

// mix 6  burst_dyn: mix 3 with the chunks of a launch handed out DYNAMICALLY (one atomic counter per launch, one
//                     vector atomic per chunk by lane 0): a block takes chunks until the launch's are gone or it
//                     holds REG + LDS results, so blocks that stream faster take more and the launch's blocks
//                     finish closer together (a launch of static round-robin chunks ends with its slowest block)
template <int R, int REG, int LDS>
__global__ void __launch_bounds__(256) m_burst_dyn(const f32x4* __restrict__ src, int64_t c0, int64_t n,
                                                   f32x4* __restrict__ dst, int* __restrict__ ctr) {
    f32x4 res[REG > 0 ? REG : 1][4];
    int64_t held[REG > 0 ? REG : 1];
    __shared__ f32x4 stage[LDS > 0 ? LDS * 1024 : 1];
    __shared__ int64_t lds_tile[LDS > 0 ? LDS : 1];
    __shared__ int grab;
    int nreg = 0, nlds = 0;
    bool more = true;
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        held[m] = -1;
        if (more) {
            if (threadIdx.x == 0) grab = atomicAdd(ctr, 1);
            __syncthreads();
            const int64_t t = grab;
            __syncthreads();
            if (t < n) {
                held[m] = c0 + t;
                m_chunk_sum<R>(src + (c0 + t) * R * 1024 + threadIdx.x, res[m]);
                nreg = m + 1;
            } else {
                more = false;
            }
        }
    }
#pragma unroll 1
    for (int m = 0; m < LDS && more; ++m) {
        if (threadIdx.x == 0) grab = atomicAdd(ctr, 1);
        __syncthreads();
        const int64_t t = grab;
        __syncthreads();
        if (t >= n) break;
        f32x4 acc[4];
        m_chunk_sum<R>(src + (c0 + t) * R * 1024 + threadIdx.x, acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) stage[m * 1024 + q * 256 + threadIdx.x] = acc[q];
        if (threadIdx.x == 0) lds_tile[m] = c0 + t;
        nlds = m + 1;
    }
    __syncthreads();
#pragma unroll 1
    for (int m = 0; m < nlds; ++m) {
        const int64_t c = lds_tile[m];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            __builtin_nontemporal_store(stage[m * 1024 + q * 256 + threadIdx.x], dst + c * 1024 + q * 256 + threadIdx.x);
    }
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        if (m < nreg)
#pragma unroll
            for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(res[m][q], dst + held[m] * 1024 + q * 256 + threadIdx.x);
    }
}

// ---------------------------------------------------------------------------------------------------------
// EPILOGUE-shaped mixes (round 4): the fused server step at few clients.  n chunks; chunk c reads R client
// segments (16 KiB each, contiguous: the slab's tile) and three operand segments (p, m, v: three arrays of n x 16 KiB)
// and writes the three operand segments back IN PLACE -- (R + 3) x 16 KiB read, 3 x 16 KiB written per chunk (Adam at
// R clients; R = 2: 20:12).  The arithmetic is a stand-in (d = sum; p += d; m = 0.9 m + d; v += d d).
//   epi 0  tile2:  per chunk the client loads, then the operand loads (the library's per-tile order), then the stores
//   epi 1  tile1:  per chunk the client and the operand loads together, then the stores
//   epi 2  burst:  REG chunks' new p, m, v held in registers and LDS chunks' in LDS, stored at the end of a launch of
//                  blocks x (REG + LDS) chunks (reads and writes in chip-wide phases)
//   epi 3  burst_d: the library's burst order: the client sums of REG + LDS chunks first (d in registers / LDS), then
//                  per chunk the operand loads, arithmetic and stores (one chunk of operands ahead)
// ---------------------------------------------------------------------------------------------------------
struct EpiBufs {
    const f32x4* cl;
    f32x4* op[3];
};

__device__ inline void e_ops(const f32x4 d, f32x4& p, f32x4& m, f32x4& v) {
    p += d;
    m = m * 0.9f + d;
    v += d * d;
}

template <int R>
__device__ inline void e_sum(const f32x4* __restrict__ cl, int64_t c, f32x4 (&d)[4]) {
    f32x4 x[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) x[r][q] = __builtin_nontemporal_load(cl + (c * R + r) * 1024 + q * 256 + threadIdx.x);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        d[q] = x[0][q];
#pragma unroll
        for (int r = 1; r < R; ++r) d[q] += x[r][q];
    }
}

template <int R, bool TOGETHER>
__global__ void __launch_bounds__(256) e_tile(EpiBufs B, int64_t n) {
    for (int64_t c = blockIdx.x; c < n; c += gridDim.x) {
        f32x4 o[3][4];
        f32x4 d[4];
        if constexpr (TOGETHER) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) o[k][q] = __builtin_nontemporal_load(B.op[k] + c * 1024 + q * 256 + threadIdx.x);
            e_sum<R>(B.cl, c, d);
        } else {
            e_sum<R>(B.cl, c, d);
            asm volatile("" ::: "memory");  // the operand loads after the client sums, as the library orders them
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) o[k][q] = __builtin_nontemporal_load(B.op[k] + c * 1024 + q * 256 + threadIdx.x);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) e_ops(d[q], o[0][q], o[1][q], o[2][q]);
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(o[k][q], B.op[k] + c * 1024 + q * 256 + threadIdx.x);
    }
}

template <int R, int REG, int LDS>
__global__ void __launch_bounds__(256) e_burst(EpiBufs B, int64_t c0, int64_t c_end) {
    f32x4 res[REG > 0 ? REG : 1][3][4];
    __shared__ f32x4 stage[LDS > 0 ? LDS * 3 * 1024 : 1];
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (c < c_end) {
            f32x4 d[4];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) res[m][k][q] = __builtin_nontemporal_load(B.op[k] + c * 1024 + q * 256 + threadIdx.x);
            e_sum<R>(B.cl, c, d);
#pragma unroll
            for (int q = 0; q < 4; ++q) e_ops(d[q], res[m][0][q], res[m][1][q], res[m][2][q]);
        }
    }
#pragma unroll 1
    for (int m = 0; m < LDS; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)(REG + m) * gridDim.x;
        if (c < c_end) {
            f32x4 o[3][4], d[4];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) o[k][q] = __builtin_nontemporal_load(B.op[k] + c * 1024 + q * 256 + threadIdx.x);
            e_sum<R>(B.cl, c, d);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                e_ops(d[q], o[0][q], o[1][q], o[2][q]);
#pragma unroll
                for (int k = 0; k < 3; ++k) stage[(m * 3 + k) * 1024 + q * 256 + threadIdx.x] = o[k][q];
            }
        }
    }
#pragma unroll 1
    for (int m = 0; m < LDS; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)(REG + m) * gridDim.x;
        if (c < c_end)
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    __builtin_nontemporal_store(stage[(m * 3 + k) * 1024 + q * 256 + threadIdx.x], B.op[k] + c * 1024 + q * 256 + threadIdx.x);
    }
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (c < c_end)
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(res[m][k][q], B.op[k] + c * 1024 + q * 256 + threadIdx.x);
    }
}

template <int R, int REG, int LDS>
__global__ void __launch_bounds__(256) e_burst_d(EpiBufs B, int64_t c0, int64_t c_end) {
    f32x4 dd[REG > 0 ? REG : 1][4];
    __shared__ f32x4 stage[LDS > 0 ? LDS * 1024 : 1];
#pragma unroll
    for (int m = 0; m < REG; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (c < c_end) e_sum<R>(B.cl, c, dd[m]);
    }
#pragma unroll 1
    for (int m = 0; m < LDS; ++m) {
        const int64_t c = c0 + blockIdx.x + (int64_t)(REG + m) * gridDim.x;
        if (c < c_end) {
            f32x4 d[4];
            e_sum<R>(B.cl, c, d);
#pragma unroll
            for (int q = 0; q < 4; ++q) stage[m * 1024 + q * 256 + threadIdx.x] = d[q];
        }
    }
    constexpr int NT = REG + LDS;
    auto load_ops = [&](f32x4 (&o)[3][4], int m) __attribute__((always_inline)) {
        int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        c = c < c_end ? c : c_end - 1;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) o[k][q] = __builtin_nontemporal_load(B.op[k] + c * 1024 + q * 256 + threadIdx.x);
    };
    f32x4 cur[3][4], nxt[3][4];
    load_ops(cur, 0);
#pragma unroll
    for (int m = 0; m < NT; ++m) {
        if (m + 1 < NT) load_ops(nxt, m + 1);
        const int64_t c = c0 + blockIdx.x + (int64_t)m * gridDim.x;
        if (c < c_end) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 d = m < REG ? dd[m < REG ? m : 0][q] : stage[(m - REG) * 1024 + q * 256 + threadIdx.x];
                e_ops(d, cur[0][q], cur[1][q], cur[2][q]);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(cur[k][q], B.op[k] + c * 1024 + q * 256 + threadIdx.x);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) cur[k][q] = nxt[k][q];
    }
}

template <int R>
static int epi_launch(int mode, int reg, int lds, EpiBufs B, int64_t n, int blocks, hipStream_t s, int* n_launch) {
    *n_launch = 0;
    if (mode == 0 || mode == 1) {
        if (mode == 0) hipLaunchKernelGGL((e_tile<R, false>), dim3(blocks), dim3(256), 0, s, B, n);
        else hipLaunchKernelGGL((e_tile<R, true>), dim3(blocks), dim3(256), 0, s, B, n);
        *n_launch = 1;
        return 0;
    }
    const int64_t per = (int64_t)blocks * (reg + lds);
    for (int64_t c0 = 0; c0 < n; c0 += per) {
        const int64_t ce = c0 + per < n ? c0 + per : n;
        const int nb = (int)(ce - c0 < blocks ? ce - c0 : blocks);
#define E_B(KERN, RG, LD) \
    if (reg == RG && lds == LD) hipLaunchKernelGGL((KERN<R, RG, LD>), dim3(nb), dim3(256), 0, s, B, c0, ce)
        if (mode == 2) {
            E_B(e_burst, 4, 0);
            else E_B(e_burst, 4, 3);
            else E_B(e_burst, 2, 1);
            else E_B(e_burst, 3, 0);
            else return 4;
        } else {
            E_B(e_burst_d, 8, 4);
            else E_B(e_burst_d, 8, 9);
            else return 4;
        }
#undef E_B
        ++*n_launch;
    }
    return 0;
}

static int g_dyn_avg = 12;  // chunks per block per launch of mix 6 (the blocks' average; capacity REG + LDS)

// write-only streams of the same write region (the other half of an additive read + write bound)
__global__ void __launch_bounds__(256) m_write_chunks(int64_t n_chunks, f32x4* __restrict__ dst) {
    const f32x4 v = {1.0f, 2.0f, 3.0f, (float)blockIdx.x};
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x)
#pragma unroll
        for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(v, dst + c * 1024 + q * 256 + threadIdx.x);
}

// mix 7: the write region through buffer stores with cache-policy bits AUX (0 plain, 2 nt, 16 sc1, 17 sc0 sc1)
template <int AUX>
__global__ void __launch_bounds__(256) m_write_chunks_aux(int64_t n_chunks, f32x4* __restrict__ dst) {
    const f32x4 v = {1.0f, 2.0f, 3.0f, (float)blockIdx.x};
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst + c * 1024, 0, 16384, 0x00020000);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), r, (q * 256 + threadIdx.x) * 16, 0, AUX);
    }
}

__global__ void __launch_bounds__(256) m_write_grid(int64_t n4, f32x4* __restrict__ dst) {
    const f32x4 v = {1.0f, 2.0f, 3.0f, (float)blockIdx.x};
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) __builtin_nontemporal_store(v, dst + i);
}

template <int R>
static int mix_launch(int mode, int reg, int lds, const f32x4* src, int64_t n_chunks, f32x4* dst, f32x4* sink,
                      int blocks, hipStream_t s, int* n_launch) {
    *n_launch = 0;
    if (mode == 0) {
        hipLaunchKernelGGL(m_grid<R>, dim3(blocks), dim3(256), 0, s, src, n_chunks * 1024, dst);
        *n_launch = 1;
    } else if (mode == 4) {
        hipLaunchKernelGGL(m_write_chunks, dim3(blocks), dim3(256), 0, s, n_chunks, dst);
        *n_launch = 1;
    } else if (mode == 5) {
        hipLaunchKernelGGL(m_write_grid, dim3(blocks), dim3(256), 0, s, n_chunks * 1024, dst);
        *n_launch = 1;
    } else if (mode == 7) {  // reg = cache-policy bits of the buffer stores
        if (reg == 0) hipLaunchKernelGGL(m_write_chunks_aux<0>, dim3(blocks), dim3(256), 0, s, n_chunks, dst);
        else if (reg == 2) hipLaunchKernelGGL(m_write_chunks_aux<2>, dim3(blocks), dim3(256), 0, s, n_chunks, dst);
        else if (reg == 16) hipLaunchKernelGGL(m_write_chunks_aux<16>, dim3(blocks), dim3(256), 0, s, n_chunks, dst);
        else if (reg == 17) hipLaunchKernelGGL(m_write_chunks_aux<17>, dim3(blocks), dim3(256), 0, s, n_chunks, dst);
        else return 9;
        *n_launch = 1;
    } else if (mode == 8 || mode == 9) {  // reg = G chunks per iteration
#define M_MULTI(GG)                                                                                                   \
    if (reg == GG) {                                                                                                  \
        if (mode == 8) hipLaunchKernelGGL((m_multi<R, GG, false>), dim3(blocks), dim3(256), 0, s, src, n_chunks, dst); \
        else hipLaunchKernelGGL((m_multi<R, GG, true>), dim3(blocks), dim3(256), 0, s, src, n_chunks, dst);           \
    }
        if constexpr (R <= 4) {
            M_MULTI(1)
            else M_MULTI(2) else M_MULTI(4) else return 11;
        } else {
            M_MULTI(1)
            else return 11;
        }
#undef M_MULTI
        *n_launch = 1;
    } else if (mode == 1 || mode == 2) {
        if (mode == 1) hipLaunchKernelGGL((m_tile<R, false>), dim3(blocks), dim3(256), 0, s, src, n_chunks, dst, sink);
        else hipLaunchKernelGGL((m_tile<R, true>), dim3(blocks), dim3(256), 0, s, src, n_chunks, dst, sink);
        *n_launch = 1;
    } else if (mode == 6) {
        const int64_t per = (int64_t)blocks * g_dyn_avg;
        const int64_t n_l = (n_chunks + per - 1) / per;
        int* ctr = nullptr;
        if (hipMalloc(&ctr, n_l * sizeof(int)) != hipSuccess) return 6;
        if (hipMemsetAsync(ctr, 0, n_l * sizeof(int), s) != hipSuccess) return 7;
        for (int64_t l = 0; l < n_l; ++l) {
            const int64_t c0 = l * per;
            const int64_t n = c0 + per < n_chunks ? per : n_chunks - c0;
            const int nb = (int)(n < blocks ? n : blocks);
#define M_DYN(RG, LD) \
    if (reg == RG && lds == LD) hipLaunchKernelGGL((m_burst_dyn<R, RG, LD>), dim3(nb), dim3(256), 0, s, src, c0, n, dst, ctr + l)
            M_DYN(8, 9);
            else M_DYN(8, 4);
            else return 8;
#undef M_DYN
            ++*n_launch;
        }
        (void)hipStreamSynchronize(s);
        (void)hipFree(ctr);
    } else {
        const int64_t per = (int64_t)blocks * (reg + lds);
        for (int64_t c0 = 0; c0 < n_chunks; c0 += per) {
            const int64_t ce = c0 + per < n_chunks ? c0 + per : n_chunks;
            const int nb = (int)(ce - c0 < blocks ? ce - c0 : blocks);
#define M_BURST(RG, LD) \
    if (reg == RG && lds == LD) hipLaunchKernelGGL((m_burst<R, RG, LD>), dim3(nb), dim3(256), 0, s, src, c0, ce, dst)
            M_BURST(8, 4);
            else M_BURST(8, 5);
            else M_BURST(8, 10);
            else M_BURST(8, 0);
            else M_BURST(0, 8);
            else M_BURST(4, 4);
            else return 4;
#undef M_BURST
            ++*n_launch;
        }
    }
    return 0;
}

extern "C" {
void mix_set_dyn(int avg) { g_dyn_avg = avg > 0 ? avg : 12; }

// R:1 mix over `bytes` of buf (see above); R in {1, 2, 3, 4, 8, 16} (mix 8 / 9: G in {1, 2, 4} up to R = 4, 1 above); returns 0 on success, ms_out = average over reps,
// bytes_out = bytes moved per rep (reads + writes), launches_out = kernel launches per rep
int mix_run(int mode, int R, int reg, int lds, void* buf, size_t bytes, int blocks, int reps, float* ms_out,
            double* bytes_out, int* launches_out) {
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f32x4* sink = nullptr;
    if (hipMalloc(&sink, (size_t)blocks * 256 * sizeof(f32x4)) != hipSuccess) return 2;
    const int64_t unit = (int64_t)(R + 1) * 16384;  // one chunk's reads + its result
    const int64_t n_chunks = (int64_t)bytes / unit;
    const f32x4* src = (const f32x4*)buf;
    f32x4* dst = (f32x4*)buf + n_chunks * R * 1024;
    int rc = 0, nl = 0;
    auto launch = [&]() {
        if (R == 1) rc = mix_launch<1>(mode, reg, lds, src, n_chunks, dst, sink, blocks, s, &nl);
        else if (R == 2) rc = mix_launch<2>(mode, reg, lds, src, n_chunks, dst, sink, blocks, s, &nl);
        else if (R == 3) rc = mix_launch<3>(mode, reg, lds, src, n_chunks, dst, sink, blocks, s, &nl);
        else if (R == 4) rc = mix_launch<4>(mode, reg, lds, src, n_chunks, dst, sink, blocks, s, &nl);
        else if (R == 8) rc = mix_launch<8>(mode, reg, lds, src, n_chunks, dst, sink, blocks, s, &nl);
        else if (R == 16) rc = mix_launch<16>(mode, reg, lds, src, n_chunks, dst, sink, blocks, s, &nl);
        else rc = 5;
    };
    launch();
    hipEventRecord(a, s);
    for (int r = 0; r < reps && rc == 0; ++r) launch();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    *ms_out = ms / reps;
    *bytes_out = (double)n_chunks * (mode == 1 ? R * 16384.0 : (mode == 4 || mode == 5 || mode == 7) ? 16384.0 : (R + 1) * 16384.0);
    *launches_out = nl;
    hipFree(sink);
    hipEventDestroy(a);
    hipEventDestroy(b);
    hipStreamDestroy(s);
    if (rc != 0) return 10 + rc;
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// the epilogue-shaped mixes (above) over `bytes` of buf; R in {1, 2, 3}; bytes_out = bytes moved per rep
int epi_run(int mode, int R, int reg, int lds, void* buf, size_t bytes, int blocks, int reps, float* ms_out,
            double* bytes_out, int* launches_out) {
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int64_t unit = (int64_t)(R + 3) * 16384;
    const int64_t n = (int64_t)bytes / unit;
    EpiBufs B;
    B.cl = (const f32x4*)buf;
    for (int k = 0; k < 3; ++k) B.op[k] = (f32x4*)buf + n * R * 1024 + (int64_t)k * n * 1024;
    int rc = 0, nl = 0;
    auto launch = [&]() {
        if (R == 1) rc = epi_launch<1>(mode, reg, lds, B, n, blocks, s, &nl);
        else if (R == 2) rc = epi_launch<2>(mode, reg, lds, B, n, blocks, s, &nl);
        else if (R == 3) rc = epi_launch<3>(mode, reg, lds, B, n, blocks, s, &nl);
        else rc = 5;
    };
    launch();
    hipEventRecord(a, s);
    for (int r = 0; r < reps && rc == 0; ++r) launch();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    *ms_out = ms / reps;
    *bytes_out = (double)n * (R + 6) * 16384.0;
    *launches_out = nl;
    hipEventDestroy(a);
    hipEventDestroy(b);
    hipStreamDestroy(s);
    if (rc != 0) return 10 + rc;
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// returns 0 on success; ms_out = average over reps
int pattern_run(int mode, int unroll, void* buf, size_t bytes, size_t chunk_bytes, int blocks, int reps, float* ms_out) {
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f32x4* sink = nullptr;
    if (hipMalloc(&sink, (size_t)blocks * 256 * sizeof(f32x4)) != hipSuccess) return 2;
    const int64_t n4 = (int64_t)(bytes / 16);
    const int64_t chunk4 = (int64_t)(chunk_bytes / 16);
    const int64_t n_chunks = n4 / chunk4;
    const f32x4* src = (const f32x4*)buf;
    auto launch = [&]() {
        if (mode == 0) {
            if (unroll == 16) hipLaunchKernelGGL(p_grid<16>, dim3(blocks), dim3(256), 0, s, src, n4, sink);
            else if (unroll == 4) hipLaunchKernelGGL(p_grid<4>, dim3(blocks), dim3(256), 0, s, src, n4, sink);
            else hipLaunchKernelGGL(p_grid<8>, dim3(blocks), dim3(256), 0, s, src, n4, sink);
        } else if (mode == 1) {
            if (unroll == 16) hipLaunchKernelGGL(p_chunk<16>, dim3(blocks), dim3(256), 0, s, src, n_chunks, chunk4, sink);
            else if (unroll == 4) hipLaunchKernelGGL(p_chunk<4>, dim3(blocks), dim3(256), 0, s, src, n_chunks, chunk4, sink);
            else hipLaunchKernelGGL(p_chunk<8>, dim3(blocks), dim3(256), 0, s, src, n_chunks, chunk4, sink);
        } else if (mode == 4) {
            const int64_t nc = n_chunks * 63 / 64;  // the last 1/64 of the buffer takes the results
            hipLaunchKernelGGL(p_chunk_w<16>, dim3(blocks), dim3(256), 0, s, src, nc, chunk4, (f32x4*)buf + nc * chunk4);
        } else if (mode >= 6 && mode <= 9) {
            const int64_t nc = n_chunks * 63 / 64;
            f32x4* d = (f32x4*)buf + nc * chunk4;
            if (mode == 6) hipLaunchKernelGGL((p_chunk_wp<16, 16>), dim3(blocks), dim3(256), 0, s, src, nc, chunk4, d);
            if (mode == 7) hipLaunchKernelGGL((p_chunk_wp<16, 17>), dim3(blocks), dim3(256), 0, s, src, nc, chunk4, d);
            if (mode == 8) hipLaunchKernelGGL((p_chunk_wp<16, 0>), dim3(blocks), dim3(256), 0, s, src, nc, chunk4, d);
            if (mode == 9) hipLaunchKernelGGL(p_chunk_wb<16>, dim3(blocks), dim3(256), 0, s, src, nc, chunk4, d);
        } else if (mode == 10) {
            const int64_t nc = n_chunks * 63 / 64;
            f32x4* d = (f32x4*)buf + nc * chunk4;
            const int64_t per = (int64_t)blocks * 8;
            for (int64_t c0 = 0; c0 < nc; c0 += per) {
                const int64_t m = nc - c0 < per ? nc - c0 : per;
                hipLaunchKernelGGL(p_chunk_wb<16>, dim3(blocks), dim3(256), 0, s, src + c0 * chunk4, m, chunk4,
                                   d + c0 * 1024);
            }
        } else if (mode == 5) {
            const int64_t nc = n_chunks * 63 / 64;
            hipLaunchKernelGGL(p_chunk_wd<16>, dim3(blocks), dim3(256), 0, s, src, nc, chunk4, (f32x4*)buf + nc * chunk4);
        } else if (mode == 2) {
            hipLaunchKernelGGL(p_chunk_lds, dim3(blocks), dim3(256), 0, s, src, n_chunks, chunk4, sink);
        } else {
            if (unroll == 16) hipLaunchKernelGGL(p_chunk_pair<16>, dim3(blocks), dim3(256), 0, s, src, n_chunks, chunk4, sink);
            else hipLaunchKernelGGL(p_chunk_pair<8>, dim3(blocks), dim3(256), 0, s, src, n_chunks, chunk4, sink);
        }
    };
    launch();
    hipEventRecord(a, s);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    *ms_out = ms / reps;
    hipFree(sink);
    hipEventDestroy(a);
    hipEventDestroy(b);
    hipStreamDestroy(s);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
}
