// kmh_matrix.hip -- compact encoding of genomes x k-mers count rows for the multi-GPU
// all-gather.  The reference assembles its organisms x k-mers matrix on one
// CPU (/root/reference/kmerml/ml/features.py:85-117); here every rank owns a block of rows
// and the blocks travel over xGMI.  Rows are sent as saturating u8 (values >= 255 stored as
// 255) plus an exact escape list (row, column, value) of every value >= 255, and widened
// back to u32 after the all-gather: 4x fewer bytes on the links for the same matrix.
#include <algorithm>

#include "kmh_device.h"

namespace kmh {
namespace {

__device__ __forceinline__ uint32_t sat8(uint32_t x) { return x < 255u ? x : 255u; }

// 16 elements per thread per step: four 16-byte loads, one 16-byte store.
__global__ __launch_bounds__(256) void k_encode_u8(const uint32_t* __restrict__ rows,
                                                   uint64_t cols, uint64_t n16,
                                                   uint8_t* __restrict__ out,
                                                   uint32_t* __restrict__ esc, uint32_t cap,
                                                   uint32_t* __restrict__ esc_n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4* src = reinterpret_cast<const uint4*>(rows) + 4 * i;
        uint32_t packed[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = src[q];
            const uint32_t e[4] = {v.x, v.y, v.z, v.w};
            packed[q] = sat8(e[0]) | (sat8(e[1]) << 8) | (sat8(e[2]) << 16) | (sat8(e[3]) << 24);
            if ((v.x | v.y | v.z | v.w) >= 255u) {  // rare: list the escapes
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (e[j] >= 255u) {
                        const uint64_t idx = 16 * i + 4 * q + j;
                        const uint32_t at = atomicAdd(esc_n, 1u);
                        if (at < cap) {
                            esc[3 * (uint64_t)at] = (uint32_t)(idx / cols);
                            esc[3 * (uint64_t)at + 1] = (uint32_t)(idx % cols);
                            esc[3 * (uint64_t)at + 2] = e[j];
                        }
                    }
                }
            }
        }
        reinterpret_cast<uint4*>(out)[i] = make_uint4(packed[0], packed[1], packed[2], packed[3]);
    }
}

__global__ __launch_bounds__(256) void k_apply_escapes(const uint32_t* __restrict__ esc,
                                                       uint32_t cap,
                                                       const uint32_t* __restrict__ esc_n,
                                                       int ranks, uint64_t rows_per_rank,
                                                       uint64_t cols, uint32_t* __restrict__ rows) {
    for (int r = 0; r < ranks; ++r) {
        const uint32_t n = min(esc_n[r], cap);
        const uint32_t* e = esc + (uint64_t)r * cap * 3;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            const uint32_t row = e[3 * i], col = e[3 * i + 1];
            if (row < rows_per_rank && col < cols)   // never trust a slot that came off the wire
                rows[((uint64_t)r * rows_per_rank + row) * cols + col] = e[3 * i + 2];
        }
    }
}

// ---- u4: two counts per byte (element 2i in the low nibble of byte i), values >= 15 stored
// as 15 with an exact (index, value) escape.  Uniform 100 Mbp genomes at k = 12 average ~6
// per bin, so ~0.14 % of the cells escape; 8x fewer bytes than u32 rows on the links.
// Wave-coalesced u8 decode: group g (a u32 of four counts) -> uint4 g of the rows; lanes take
// groups base + 64u + l, so every instruction covers contiguous bytes (256 B loads, 1 KiB
// non-temporal stores).
__global__ __launch_bounds__(256) void k_decode_u8w(const uint32_t* __restrict__ in, uint64_t n4,
                                                    uint32_t* __restrict__ rows) {
    const int lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint4* dst = reinterpret_cast<uint4*>(rows);
    for (uint64_t base = w0 * 512u; base < n4; base += nw * 512u) {
        uint32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
            x[u] = in[e < n4 ? e : n4 - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
            if (e < n4) store_nt(&dst[e], make_uint4(x[u] & 0xFFu, (x[u] >> 8) & 0xFFu, (x[u] >> 16) & 0xFFu, x[u] >> 24));
        }
    }
}

__device__ __forceinline__ uint32_t sat4(uint32_t x) { return x < 15u ? x : 15u; }

// Wave-coalesced u4 encode: a wave takes 512 consecutive 4-count groups (uint4) per step; lane
// l takes groups base + 64u + l, u = 0..7, so every load instruction reads 1 KiB contiguous
// and every store writes 128 B contiguous (group g -> the u16 at index g: the same nibble
// layout: element 2i in the low nibble of byte i).  Escapes are counted per lane, scanned across the wave and appended
// behind one atomic per wave (a single global counter per lane-escape serialises at L2).
__global__ __launch_bounds__(256) void k_encode_u4w(const uint32_t* __restrict__ rows, uint64_t n4,
                                                    uint16_t* __restrict__ out,
                                                    uint32_t* __restrict__ esc, uint32_t cap,
                                                    uint32_t* __restrict__ esc_n) {
    // Per-wave escape staging in LDS: a wave appends its (index, value) pairs here and moves
    // them to the global list behind ONE atomic per kStage entries (uniform genomes: ~3
    // escapes per 512-group step, so ~one global atomic per 170 steps instead of one per
    // step -- a single counter that every wave hits serialises at one L2 channel).
    constexpr uint32_t kStage = 512;
    __shared__ uint32_t stage[4][2 * kStage];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* st = stage[wave];
    uint32_t held = 0u;   // wave-uniform
    auto sync_wave = []() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto flush = [&]() {
        sync_wave();
        uint32_t at0 = 0u;
        if (lane == 0) at0 = atomicAdd(esc_n, held);
        at0 = (uint32_t)__shfl((int)at0, 0);
        for (uint32_t i = (uint32_t)lane; i < held; i += 64u) {
            if (at0 + i < cap) {
                esc[2 * (uint64_t)(at0 + i)] = st[2 * i];
                esc[2 * (uint64_t)(at0 + i) + 1] = st[2 * i + 1];
            }
        }
        sync_wave();
        held = 0u;
    };
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint4* src = reinterpret_cast<const uint4*>(rows);
    for (uint64_t base = w0 * 512u; base < n4; base += nw * 512u) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
            v[u] = src[e < n4 ? e : n4 - 1];   // unconditional load (a guarded one drains vmcnt)
        }
        uint32_t nesc = 0u;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
            const uint4 a = v[u];
            if (e < n4) {
                nesc += (uint32_t)(a.x >= 15u) + (uint32_t)(a.y >= 15u) + (uint32_t)(a.z >= 15u) + (uint32_t)(a.w >= 15u);
                out[e] = (uint16_t)(sat4(a.x) | (sat4(a.y) << 4) | (sat4(a.z) << 8) | (sat4(a.w) << 12));
            }
        }
        if (__ballot(nesc != 0u)) {   // wave-uniform; rare for uniform genomes
            uint32_t incl = nesc;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(incl, d);
                if (lane >= d) incl += t;
            }
            const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
            if (held + tot > kStage) flush();
            const bool direct = tot > kStage;   // a step of mostly escapes: straight to global
            uint32_t at;
            if (direct) {
                uint32_t at0 = 0u;
                if (lane == 63) at0 = atomicAdd(esc_n, incl);
                at = (uint32_t)__shfl((int)at0, 63) + incl - nesc;
            } else {
                at = held + incl - nesc;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
                const uint32_t c[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (e < n4 && c[j] >= 15u) {
                        const uint32_t idx = (uint32_t)(4 * e + (uint64_t)j);
                        if (direct) {
                            if (at < cap) {
                                esc[2 * (uint64_t)at] = idx;
                                esc[2 * (uint64_t)at + 1] = c[j];
                            }
                        } else {
                            st[2 * at] = idx;
                            st[2 * at + 1] = c[j];
                        }
                        ++at;
                    }
                }
            }
            if (!direct) held += tot;
        }
    }
    if (held) flush();
}

// Wave-coalesced u4 decode: group g (a u16 of four nibbles) -> uint4 g of the rows; lanes take
// groups base + 64u + l, so loads read 128 B and non-temporal stores write 1 KiB contiguous per
// instruction.
__global__ __launch_bounds__(256) void k_decode_u4w(const uint16_t* __restrict__ in, uint64_t n4,
                                                    uint32_t* __restrict__ rows) {
    const int lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint4* dst = reinterpret_cast<uint4*>(rows);
    for (uint64_t base = w0 * 512u; base < n4; base += nw * 512u) {
        uint32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
            x[u] = in[e < n4 ? e : n4 - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t e = base + 64u * (uint64_t)u + (uint64_t)lane;
            if (e < n4) store_nt(&dst[e], make_uint4(x[u] & 15u, (x[u] >> 4) & 15u, (x[u] >> 8) & 15u, x[u] >> 12));
        }
    }
}

unsigned grid_waves(uint64_t n4) {   // 256-thread blocks, one 512-group step per wave at least
    const uint64_t b = (n4 + 2047) / 2048;
    return (unsigned)(b < 4096 ? (b ? b : 1) : 4096);
}

__global__ __launch_bounds__(256) void k_apply_escapes_u4(const uint32_t* __restrict__ esc,
                                                          uint32_t cap,
                                                          const uint32_t* __restrict__ esc_n,
                                                          uint64_t lo, uint64_t hi, uint32_t* __restrict__ rows) {
    // escapes whose block index lies in [lo, hi) land at rows[index - lo]; the others (other
    // rows of the block, or garbage in a slot that came off the wire) are ignored
    const uint32_t n = min(*esc_n, cap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t idx = esc[2 * (uint64_t)i];
        if (idx >= lo && idx < hi) rows[idx - lo] = esc[2 * (uint64_t)i + 1];
    }
}

unsigned grid_for(uint64_t n16) {
    const uint64_t b = (n16 + 255) / 256;
    return (unsigned)(b < 8192 ? (b ? b : 1) : 8192);
}

}  // namespace

int rows_encode_u8(Ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols,
                   uint8_t* d_u8, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n,
                   hipStream_t s) {
    if (!d_rows || !d_u8 || !d_esc_n || (cap && !d_esc)) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (cols % 16 != 0) return fail(ctx, KMH_ERR_INVALID, "cols must be a multiple of 16");
    KMH_HIP(ctx, hipMemsetAsync(d_esc_n, 0, sizeof(uint32_t), s));
    const uint64_t n16 = rows * cols / 16;
    if (n16 == 0) return KMH_OK;
    time_begin(ctx, s, "k_encode_u8");
    hipLaunchKernelGGL(k_encode_u8, dim3(grid_for(n16)), dim3(256), 0, s, d_rows, cols, n16, d_u8,
                       d_esc, cap, d_esc_n);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

int rows_decode_u8(Ctx* ctx, const uint8_t* d_u8, uint64_t rows, uint64_t cols,
                   const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n, int ranks,
                   uint64_t rows_per_rank, uint32_t* d_rows, hipStream_t s) {
    if (!d_u8 || !d_rows || (ranks > 0 && (!d_esc_n || (cap && !d_esc))))
        return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (cols % 16 != 0) return fail(ctx, KMH_ERR_INVALID, "cols must be a multiple of 16");
    const uint64_t n16 = rows * cols / 16;
    if (n16) {
        time_begin(ctx, s, "k_decode_u8");
        hipLaunchKernelGGL(k_decode_u8w, dim3((unsigned)std::min<uint64_t>(4096, (4 * n16 + 2047) / 2048)), dim3(256), 0, s,
                           reinterpret_cast<const uint32_t*>(d_u8), 4 * n16, d_rows);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
    }
    if (ranks > 0 && cap > 0) {
        hipLaunchKernelGGL(k_apply_escapes, dim3(64), dim3(256), 0, s, d_esc, cap, d_esc_n, ranks,
                           rows_per_rank, cols, d_rows);
        KMH_HIP(ctx, hipGetLastError());
    }
    return KMH_OK;
}

}  // namespace kmh

namespace kmh {

int rows_encode_u4(Ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols, uint8_t* d_u4,
                   uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n, hipStream_t s) {
    if (!d_rows || !d_u4 || !d_esc_n || (cap && !d_esc)) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (cols % 32 != 0) return fail(ctx, KMH_ERR_INVALID, "cols must be a multiple of 32");
    if (rows * cols >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "u4 blocks must hold fewer than 2^32 - 1 cells");
    KMH_HIP(ctx, hipMemsetAsync(d_esc_n, 0, sizeof(uint32_t), s));
    const uint64_t n32 = rows * cols / 32;
    if (n32 == 0) return KMH_OK;
    time_begin(ctx, s, "k_encode_u4");
    hipLaunchKernelGGL(k_encode_u4w, dim3(grid_waves(8 * n32)), dim3(256), 0, s, d_rows, 8 * n32,
                           reinterpret_cast<uint16_t*>(d_u4), d_esc, cap, d_esc_n);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

int rows_decode_u4(Ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols, const uint32_t* d_esc,
                   uint32_t cap, const uint32_t* d_esc_n, uint32_t* d_rows, hipStream_t s) {
    return rows_decode_u4_range(ctx, d_u4, rows, cols, d_esc, cap, d_esc_n, 0, rows, d_rows, s);
}

int rows_decode_u4_range(Ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols, const uint32_t* d_esc,
                         uint32_t cap, const uint32_t* d_esc_n, uint64_t row0, uint64_t nrows, uint32_t* d_rows,
                         hipStream_t s) {
    if (!d_u4 || !d_rows || !d_esc_n || (cap && !d_esc)) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (cols % 32 != 0) return fail(ctx, KMH_ERR_INVALID, "cols must be a multiple of 32");
    if (rows * cols >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "u4 blocks must hold fewer than 2^32 - 1 cells");
    if (row0 > rows || nrows > rows - row0) return fail(ctx, KMH_ERR_INVALID, "row range outside the block");
    const uint64_t n32 = nrows * cols / 32;
    if (n32 == 0) return KMH_OK;
    time_begin(ctx, s, "k_decode_u4");
    hipLaunchKernelGGL(k_decode_u4w, dim3(grid_waves(8 * n32)), dim3(256), 0, s,
                       reinterpret_cast<const uint16_t*>(d_u4 + row0 * cols / 2), 8 * n32, d_rows);  // 8 four-count groups per 32 counts
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    if (cap > 0) {
        hipLaunchKernelGGL(k_apply_escapes_u4, dim3(64), dim3(256), 0, s, d_esc, cap, d_esc_n, row0 * cols,
                           (row0 + nrows) * cols, d_rows);
        KMH_HIP(ctx, hipGetLastError());
    }
    return KMH_OK;
}

}  // namespace kmh
