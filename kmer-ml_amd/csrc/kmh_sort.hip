// kmh_sort.hip -- device sort, scan and run primitives of the drop-in's sparse path.
//
// The reference keeps k-mers in a dict in first-occurrence order (generate.py:36,58); its
// k{k}.txt lines follow that order (:89-91).  Putting the distinct k-mers of one organism in
// that order, and the exact recount of a hash-table pass that overflowed, need a stable sort
// of (key, value) pairs and run boundaries over up to 2^32 - 2 items (a 3.1 Gbp genome at
// k = 21: more than 2^31 windows, past the int item counts of library sorts).  Hand-written
// for gfx950 with 32-bit offsets and 64-bit item indices:
//
//   radix_sort_pairs  LSD, 8-bit digits; per pass k_rs_count (digit histogram of each
//                     8192-item block, digit-major), scan_exclusive_u32 (block offsets of
//                     every digit), k_rs_scatter (stable ranks: the items of a block are
//                     ranked wave by wave in index order, each wave's 64 keys matched by
//                     digit with eight ballots; one LDS cursor per (wave, digit)).
//   scan_exclusive_u32  three launches: block sums, one workgroup over the sums, block scans.
//   run_starts          heads of equal-key runs of a sorted array, compacted in order.
#include <algorithm>

#include "kmh_device.h"

namespace kmh {
namespace {

constexpr int kRsThreads = 1024;
constexpr int kRsWaves = kRsThreads / 64;
constexpr int kRsSteps = 8;                         // items per lane
constexpr int kRsTile = kRsThreads * kRsSteps;      // 8192 items per block
constexpr int kScanChunk = 8192;                    // values per scan block (1024 x 8)

// Item s of wave w of block b: b * 8192 + w * 512 + s * 64 + lane, so a wave's 8 steps and the
// waves of a block run through the block's items in index order (what makes the ranks stable).
__device__ __forceinline__ uint64_t rs_item(uint64_t blk, int wave, int step, int lane) {
    return blk * (uint64_t)kRsTile + (uint64_t)(wave * 512 + step * 64 + lane);
}

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K key, int shift, uint32_t dmask) {
    return (uint32_t)(key >> shift) & dmask;
}

template <typename K>
__global__ __launch_bounds__(kRsThreads) void k_rs_count(const K* __restrict__ keys, uint64_t n, int shift,
                                                         uint32_t dmask, uint32_t nblk, uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 256) h[tid] = 0u;
    __syncthreads();
    const uint64_t blk = blockIdx.x;
#pragma unroll
    for (int j = 0; j < kRsSteps; ++j) {
        const uint64_t i = rs_item(blk, wave, j, lane);
        if (i < n) atomicAdd(&h[digit_of(keys[i], shift, dmask)], 1u);
    }
    __syncthreads();
    if (tid < 256) counts[(uint64_t)tid * nblk + blk] = h[tid];
}

template <typename K>
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const K* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                           uint64_t n, int shift, uint32_t dmask, uint32_t nblk,
                                                           const uint32_t* __restrict__ offs, K* __restrict__ keys_out,
                                                           uint32_t* __restrict__ vals_out) {
    __shared__ uint32_t cur[kRsWaves][256];   // per-wave digit counts, then cursors
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t blk = blockIdx.x;
    for (int i = tid; i < kRsWaves * 256; i += kRsThreads) (&cur[0][0])[i] = 0u;
    __syncthreads();
    K kr[kRsSteps];
    uint32_t d[kRsSteps];
#pragma unroll
    for (int j = 0; j < kRsSteps; ++j) {
        const uint64_t i = rs_item(blk, wave, j, lane);
        kr[j] = i < n ? keys[i] : (K)0;
        d[j] = digit_of(kr[j], shift, dmask);
        if (i < n) atomicAdd(&cur[wave][d[j]], 1u);
    }
    __syncthreads();
    if (tid < 256) {   // cursor of (wave, digit): the block's digit offset + the earlier waves' counts
        uint32_t run = offs[(uint64_t)tid * nblk + blk];
        for (int w = 0; w < kRsWaves; ++w) {
            const uint32_t c = cur[w][tid];
            cur[w][tid] = run;
            run += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < kRsSteps; ++j) {
        const uint64_t i = rs_item(blk, wave, j, lane);
        const bool ok = i < n;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d[j] >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const int leader = peers ? __ffsll((long long)peers) - 1 : lane;
        uint32_t old = 0u;
        if (ok && lane == leader) old = atomicAdd(&cur[wave][d[j]], (uint32_t)__popcll(peers));
        old = (uint32_t)__shfl((int)old, leader);
        if (ok) {
            const uint32_t pos = old + (uint32_t)__popcll(peers & lt);
            keys_out[pos] = kr[j];
            vals_out[pos] = vals[i];
        }
    }
}

// Exclusive scan helpers: chunks of 8192 values, 8 consecutive per thread.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if (lane >= d) incl += x;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, tot = 0u;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) {
        pre += w < wave ? wsum[w] : 0u;
        tot += wsum[w];
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + incl - v;
}

__global__ __launch_bounds__(1024) void k_scan_reduce(const uint32_t* __restrict__ in, uint64_t n,
                                                      uint32_t* __restrict__ bsum) {
    __shared__ uint32_t wsum[16];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * 8;
    uint32_t s = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += base + j < n ? in[base + j] : 0u;
    uint32_t tot;
    block_excl_scan(s, wsum, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// One workgroup: exclusive scan of the nb block sums in place; *total (nullable) = their sum.
__global__ __launch_bounds__(1024) void k_scan_top(uint32_t* __restrict__ bsum, uint32_t nb,
                                                   uint32_t* __restrict__ total) {
    __shared__ uint32_t wsum[16];
    uint32_t carry = 0u;
    for (uint32_t c0 = 0; c0 < nb; c0 += 1024u) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t v = i < nb ? bsum[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(v, wsum, &tot);
        if (i < nb) bsum[i] = carry + ex;
        carry += tot;
    }
    if (total && threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(1024) void k_scan_down(const uint32_t* __restrict__ in, uint64_t n,
                                                    const uint32_t* __restrict__ bsum, uint32_t* __restrict__ out) {
    __shared__ uint32_t wsum[16];
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * 8;
    uint32_t v[8], s = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        v[j] = base + j < n ? in[base + j] : 0u;
        s += v[j];
    }
    uint32_t run = bsum[blockIdx.x] + block_excl_scan(s, wsum, nullptr);
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (base + j < n) {
            out[base + j] = run;
            run += v[j];
        }
}

template <typename K>
__global__ __launch_bounds__(256) void k_run_flags(const K* __restrict__ keys, uint64_t n, uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_run_emit(const uint32_t* __restrict__ flags, const uint32_t* __restrict__ ex,
                                                  uint64_t n, uint32_t* __restrict__ starts) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && flags[i]) starts[ex[i]] = (uint32_t)i;
}

inline unsigned grid256(uint64_t n) {
    return (unsigned)((n + 255) / 256);
}

}  // namespace

int scan_exclusive_u32(Ctx* ctx, const uint32_t* d_in, uint32_t* d_out, uint64_t n, uint32_t* d_total,
                       hipStream_t s) {
    if (n == 0) {
        if (d_total) KMH_HIP(ctx, hipMemsetAsync(d_total, 0, 4, s));
        return KMH_OK;
    }
    const uint64_t nb = (n + kScanChunk - 1) / kScanChunk;
    if (nb > 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "scan too large");
    int rc = ensure(ctx, ctx->scan_tmp, (size_t)nb * 4 + 256);
    if (rc) return rc;
    uint32_t* bsum = static_cast<uint32_t*>(ctx->scan_tmp.ptr);
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(1024), 0, s, d_in, n, bsum);
    KMH_HIP(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, bsum, (uint32_t)nb, d_total);
    KMH_HIP(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(1024), 0, s, d_in, n, bsum, d_out);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

template <typename K>
int radix_sort_pairs(Ctx* ctx, K* keys, K* keys_alt, uint32_t* vals, uint32_t* vals_alt, uint64_t n, int bit_lo,
                     int bit_hi, bool* result_in_alt, hipStream_t s) {
    *result_in_alt = false;
    if (n <= 1 || bit_hi <= bit_lo) return KMH_OK;
    if (n >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "radix sort: at most 2^32 - 2 items");
    const uint64_t nblk = (n + kRsTile - 1) / kRsTile;
    const uint64_t M = 256 * nblk;
    int rc = ensure(ctx, ctx->sort_tmp, (size_t)M * 8 + 256);
    if (rc) return rc;
    uint32_t* counts = static_cast<uint32_t*>(ctx->sort_tmp.ptr);
    uint32_t* offs = counts + M;
    K *src = keys, *dst = keys_alt;
    uint32_t *vsrc = vals, *vdst = vals_alt;
    for (int sh = bit_lo; sh < bit_hi; sh += 8) {
        const int nbits = std::min(8, bit_hi - sh);
        const uint32_t dmask = (1u << nbits) - 1u;
        hipLaunchKernelGGL(k_rs_count<K>, dim3((unsigned)nblk), dim3(kRsThreads), 0, s, src, n, sh, dmask,
                           (uint32_t)nblk, counts);
        KMH_HIP(ctx, hipGetLastError());
        rc = scan_exclusive_u32(ctx, counts, offs, M, nullptr, s);
        if (rc) return rc;
        hipLaunchKernelGGL(k_rs_scatter<K>, dim3((unsigned)nblk), dim3(kRsThreads), 0, s, src, vsrc, n, sh, dmask,
                           (uint32_t)nblk, offs, dst, vdst);
        KMH_HIP(ctx, hipGetLastError());
        std::swap(src, dst);
        std::swap(vsrc, vdst);
        *result_in_alt = !*result_in_alt;
    }
    return KMH_OK;
}

template int radix_sort_pairs<uint32_t>(Ctx*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint64_t, int, int, bool*,
                                        hipStream_t);
template int radix_sort_pairs<uint64_t>(Ctx*, uint64_t*, uint64_t*, uint32_t*, uint32_t*, uint64_t, int, int, bool*,
                                        hipStream_t);

template <typename K>
int run_starts(Ctx* ctx, const K* d_keys, uint64_t n, uint32_t* d_flags, uint32_t* d_ex, uint32_t* d_starts,
               uint32_t* d_nruns, hipStream_t s) {
    if (n == 0) {
        KMH_HIP(ctx, hipMemsetAsync(d_nruns, 0, 4, s));
        return KMH_OK;
    }
    hipLaunchKernelGGL(k_run_flags<K>, dim3(grid256(n)), dim3(256), 0, s, d_keys, n, d_flags);
    KMH_HIP(ctx, hipGetLastError());
    int rc = scan_exclusive_u32(ctx, d_flags, d_ex, n, d_nruns, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_run_emit, dim3(grid256(n)), dim3(256), 0, s, d_flags, d_ex, n, d_starts);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

template int run_starts<uint32_t>(Ctx*, const uint32_t*, uint64_t, uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                                  hipStream_t);
template int run_starts<uint64_t>(Ctx*, const uint64_t*, uint64_t, uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                                  hipStream_t);

int select_flagged(Ctx* ctx, const uint32_t* d_flags, uint64_t n, uint32_t* d_ex, uint32_t* d_idx, uint32_t* d_count,
                   hipStream_t s) {
    if (n == 0) {
        KMH_HIP(ctx, hipMemsetAsync(d_count, 0, 4, s));
        return KMH_OK;
    }
    int rc = scan_exclusive_u32(ctx, d_flags, d_ex, n, d_count, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_run_emit, dim3(grid256(n)), dim3(256), 0, s, d_flags, d_ex, n, d_idx);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

}  // namespace kmh
