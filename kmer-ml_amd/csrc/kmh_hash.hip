// kmh_hash.hip -- device-resident sparse k-mer counting (13 <= k <= 21, forward or
// canonical) for BASELINE config 5: 250 Mbp genomes at k = 21, where 4^k bins cannot be
// tabulated and almost every k-mer is distinct.  The reference counts into a Python dict
// (a hash table, /root/reference/kmerml/kmers/generate.py:36,58); here the counting is done
// by LDS hash tables after a partition pass, so every hash insert is an LDS operation:
//
//  1. k_sp_partition  one workgroup per 32768-window tile: forward (and reverse-complement)
//                     codes from 2-bit packed registers, bucket = top 11 bits of the code
//                     (2048 buckets), LDS histogram + scan + scatter of the low 2k - 11 bits
//                     (u32 residues), one coalesced store of the tile's entries and an exact
//                     bucket-major offset table toff[bucket][tile] (u16 entry indices; no
//                     padding: entries are consumed one per lane).
//  2. k_sp_sizes      entries per (genome, bucket); the host splits every bucket into
//                     P = ceil(entries / target) passes over equal residue ranges.
//  3. k_sp_count      one workgroup per (genome, bucket, pass): streams the bucket's segments
//                     through a per-wave LDS queue, inserts the pass's residues into a
//                     16384-slot LDS hash table (linear probing, u32 key + u32 count), and
//                     appends the distinct k-mers to the genome's output through one atomic
//                     cursor.  The passes of a bucket are neighbouring work items on one XCD,
//                     so the bucket is read from HBM once and re-read from that XCD's L2.
//  4. fallback        a pass whose distinct keys exceed the table limit emits nothing and is
//                     counted instead by gather + hipCUB radix sort + run-length encode (keys
//                     of different passes are disjoint, so the two never double count).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "kmh_device.h"

namespace kmh {
namespace {

constexpr int kSpThreads = 1024;           // threads of partition and count workgroups
constexpr int kSpBucketBits = 11;
constexpr int kSpBuckets = 1 << kSpBucketBits;
constexpr int kSpTile = kSpThreads * 32;   // 32768 window starts per tile (= kTile)
constexpr int kSlotBits = 14;
constexpr int kSlots = 1 << kSlotBits;     // LDS hash slots: 16384 x (key, count) = 128 KiB
constexpr int kQueue = 256;                // per-wave queue entries (4 load rounds)
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kMaxPasses = 64;

// 2-bit-group reversal of the low 2K bits of ~x: the reverse complement of a K-mer code.
template <int K>
__device__ __forceinline__ uint64_t revcomp(uint64_t x) {
    uint64_t r = __builtin_bitreverse64(~x);
    r = ((r >> 1) & 0x5555555555555555ull) | ((r & 0x5555555555555555ull) << 1);
    return r >> (64 - 2 * K);
}

// Window j (0..31) of the 64 bases held as two 64-bit code words (first base in the top
// bits of hi).  Compile-time j after unrolling.
template <int K>
__device__ __forceinline__ uint64_t window(uint64_t hi, uint64_t lo, int j) {
    constexpr uint64_t M = (1ull << (2 * K)) - 1ull;
    const int e = 2 * (j + K);  // bit end (MSB-first) of the window
    if (e <= 64) return (hi >> (64 - e)) & M;
    return ((hi << (e - 64)) | (lo >> (128 - e))) & M;
}

// The 32 windows starting at tstart + 32 * threadIdx.x: packed codes and invalid masks.
struct Bases {
    uint64_t hi, lo;   // 64 bases, 2 bits each, first base in bit 63..62 of hi
    uint64_t inv;      // bit 63 = base 0 is not ACGT (or lies past the genome end)
};

template <bool FAST>
__device__ __forceinline__ Bases load_bases(const uint8_t* __restrict__ seq, uint64_t base,
                                            uint64_t gend) {
    uint4 v[4];
    if constexpr (FAST) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const uint4*>(seq + base + 16 * q);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = load16(seq, base + 16 * q, gend);
    }
    uint32_t c[4], i[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        enc16(v[q], c[q], i[q]);
        i[q] |= tail_mask(base + 16 * q, gend);
    }
    Bases b;
    b.hi = ((uint64_t)c[0] << 32) | c[1];
    b.lo = ((uint64_t)c[2] << 32) | c[3];
    b.inv = ((uint64_t)i[0] << 48) | ((uint64_t)i[1] << 32) | ((uint64_t)i[2] << 16) | i[3];
    return b;
}

// f(code) for every valid window of this thread (canonical: min(forward, reverse complement)).
template <int K, int CANON, typename F>
__device__ __forceinline__ void each_window(const Bases& b, F&& f) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if (((b.inv << j) >> (64 - K)) == 0ull) {
            uint64_t c = window<K>(b.hi, b.lo, j);
            if (CANON) {
                const uint64_t r = revcomp<K>(c);
                c = r < c ? r : c;
            }
            f(c);
        }
    }
}

template <int K, int CANON>
__global__ __launch_bounds__(kSpThreads) void k_sp_partition(const uint8_t* __restrict__ seq,
                                                             GenomeMap m,
                                                             uint32_t* __restrict__ ent,
                                                             uint16_t* __restrict__ toff,
                                                             uint32_t ldt) {
    constexpr int R = 2 * K - kSpBucketBits;
    constexpr uint64_t RM = (1ull << R) - 1ull;
    __shared__ __attribute__((aligned(16))) uint32_t sorted[kSpTile];
    __shared__ uint32_t cnt[kSpBuckets];
    __shared__ uint32_t cur[kSpBuckets];
    __shared__ uint32_t wsum[kSpThreads / 64];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = xcd_work_id();
    const uint64_t gt = m.tile_lo + lt;
    const int g = find_genome(m, gt);
    const uint64_t tstart = m.goff[g] + (gt - m.tbase[g]) * (uint64_t)kSpTile;
    const uint64_t ge = m.goff[g + 1];

    for (int b = tid; b < kSpBuckets; b += kSpThreads) cnt[b] = 0u;
    __syncthreads();

    const uint64_t base = tstart + 32ull * (uint64_t)tid;
    const Bases bs = (tstart + (uint64_t)kSpTile + 48 <= m.data_end) ? load_bases<true>(seq, base, ge)
                                                                     : load_bases<false>(seq, base, ge);
    each_window<K, CANON>(bs, [&](uint64_t c) { atomicAdd(&cnt[(uint32_t)(c >> R)], 1u); });
    __syncthreads();

    // Exclusive scan of the 2048 bucket counts (two consecutive buckets per thread).
    const uint32_t n0 = cnt[2 * tid], n1 = cnt[2 * tid + 1];
    uint32_t incl = n0 + n1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, total = 0u;
#pragma unroll
    for (int w = 0; w < kSpThreads / 64; ++w) {
        pre += (w < wave) ? wsum[w] : 0u;
        total += wsum[w];
    }
    const uint32_t s0 = pre + incl - n0 - n1;
    cur[2 * tid] = s0;
    cur[2 * tid + 1] = s0 + n0;
    toff[(uint64_t)(2 * tid) * ldt + lt] = (uint16_t)s0;
    toff[(uint64_t)(2 * tid + 1) * ldt + lt] = (uint16_t)(s0 + n0);
    if (tid == 0) toff[(uint64_t)kSpBuckets * ldt + lt] = (uint16_t)total;
    __syncthreads();

    each_window<K, CANON>(bs, [&](uint64_t c) {
        const uint32_t slot = atomicAdd(&cur[(uint32_t)(c >> R)], 1u);
        sorted[slot] = (uint32_t)(c & RM);
    });
    __syncthreads();

    uint32_t* dst = ent + lt * (uint64_t)kSpTile;
    const uint32_t n4 = total / 4;
    for (uint32_t i = tid; i < n4; i += kSpThreads)
        reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(sorted)[i];
    if (tid < (int)(total & 3u)) dst[4 * n4 + tid] = sorted[4 * n4 + tid];
}

// Entries of every (genome, bucket) of a batch: one workgroup per pair.
__global__ __launch_bounds__(256) void k_sp_sizes(const uint16_t* __restrict__ toff, uint32_t ldt,
                                                  const uint64_t* __restrict__ tbase, int g0,
                                                  uint64_t tile_lo, uint32_t* __restrict__ nb) {
    const int gl = blockIdx.x / kSpBuckets, b = blockIdx.x % kSpBuckets;
    const int g = g0 + gl;
    const uint64_t ta = tbase[g] - tile_lo, tb = tbase[g + 1] - tile_lo;
    uint32_t s = 0u;
    for (uint64_t t = ta + threadIdx.x; t < tb; t += 256)
        s += (uint32_t)toff[(uint64_t)(b + 1) * ldt + t] - (uint32_t)toff[(uint64_t)b * ldt + t];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    __shared__ uint32_t ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) nb[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Work item of the count kernel.
struct SpItem {
    uint32_t g;        // genome index (absolute)
    uint32_t b;        // bucket
    uint16_t p, np;    // pass and passes of the bucket
    uint32_t n;        // entries of the bucket
};

__device__ __forceinline__ uint32_t pass_of(uint32_t r, uint32_t np, int R) {
    return (uint32_t)(((uint64_t)r * np) >> R);
}

__global__ __launch_bounds__(kSpThreads) void k_sp_count(
    const uint32_t* __restrict__ ent, const uint16_t* __restrict__ toff, uint32_t ldt,
    const uint64_t* __restrict__ tbase, uint64_t tile_lo, const SpItem* __restrict__ items,
    int R, uint32_t limit, const uint64_t* __restrict__ out_off, uint64_t* __restrict__ codes,
    uint32_t* __restrict__ counts, unsigned long long* __restrict__ nk,
    uint32_t* __restrict__ failed) {
    constexpr int NW = kSpThreads / 64;
    __shared__ uint32_t keys[kSlots];
    __shared__ uint32_t cnts[kSlots];
    __shared__ uint32_t queue[NW][kQueue];
    __shared__ uint32_t used, fail;
    __shared__ uint32_t wsum[NW];
    __shared__ unsigned long long obase;

    const SpItem it = items[xcd_work_id()];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < kSlots; i += kSpThreads) {
        keys[i] = kEmpty;
        cnts[i] = 0u;
    }
    if (tid == 0) {
        used = 0u;
        fail = 0u;
    }
    __syncthreads();

    const uint32_t b = it.b, p = it.p, np = it.np;
    auto insert = [&](uint32_t r) {
        if (*(volatile uint32_t*)&fail) return;
        uint32_t s = (r * 0x9E3779B1u) >> (32 - kSlotBits);
        for (int probe = 0; probe < kSlots; ++probe) {
            const uint32_t k0 = keys[s];
            if (k0 == r) {
                atomicAdd(&cnts[s], 1u);
                return;
            }
            if (k0 == kEmpty) {
                const uint32_t old = atomicCAS(&keys[s], kEmpty, r);
                if (old == kEmpty) {
                    atomicAdd(&cnts[s], 1u);
                    if (atomicAdd(&used, 1u) + 1u > limit) fail = 1u;
                    return;
                }
                if (old == r) {
                    atomicAdd(&cnts[s], 1u);
                    return;
                }
            }
            s = (s + 1u) & (kSlots - 1u);
        }
        fail = 1u;  // unreachable while used <= limit < kSlots - kSpThreads
    };

    const uint64_t ta = tbase[it.g] - tile_lo, tb = tbase[it.g + 1] - tile_lo;
    // tiles per wave batch: expected entries of a batch fill about half the queue
    const uint64_t nt = tb - ta;
    const uint32_t per = nt ? (uint32_t)((it.n + nt - 1) / nt) : 1u;
    uint32_t bt = (uint32_t)kQueue / 2u / (per + 1u);
    bt = bt < 1u ? 1u : (bt > 64u ? 64u : bt);
    uint32_t* q = queue[wave];
    for (uint64_t tw = ta + (uint64_t)wave * bt; tw < tb; tw += (uint64_t)NW * bt) {
        const uint64_t t = tw + (uint64_t)lane;
        const bool in = (uint32_t)lane < bt && t < tb;
        const uint32_t lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
        const uint32_t hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
        const uint32_t nc = hi - lo;
        uint32_t incl = nc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        const uint32_t total = __shfl(incl, 63);
        const uint32_t ebase = (uint32_t)t * (uint32_t)kSpTile + lo;
        if (total <= (uint32_t)kQueue) {
            const uint32_t ex = incl - nc;
            for (uint32_t j = 0; j < nc; ++j) q[ex + j] = ebase + j;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t v[kQueue / 64];
#pragma unroll
            for (int u = 0; u < kQueue / 64; ++u) {
                const uint32_t e = (uint32_t)(u * 64 + lane);
                v[u] = e < total ? ent[q[e]] : kEmpty;
            }
#pragma unroll
            for (int u = 0; u < kQueue / 64; ++u)
                if (v[u] != kEmpty && pass_of(v[u], np, R) == p) insert(v[u]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {  // skewed batch: each lane walks its own segment
            for (uint32_t j = 0; j < nc; ++j) {
                const uint32_t r = ent[(uint64_t)ebase + j];
                if (pass_of(r, np, R) == p) insert(r);
            }
        }
    }
    __syncthreads();
    if (fail) {
        if (tid == 0) {
            const uint32_t at = atomicAdd(&failed[0], 1u);
            failed[1 + at] = xcd_work_id();
        }
        return;
    }

    // Emit the occupied slots: slot i * 1024 + tid for round i; ballot compaction keeps
    // each wave's stores of a round contiguous.
    constexpr int ROUNDS = kSlots / kSpThreads;
    uint32_t mine = 0u;
#pragma unroll
    for (int i = 0; i < ROUNDS; ++i) mine += __popcll(__ballot(keys[i * kSpThreads + tid] != kEmpty));
    if (lane == 0) wsum[wave] = mine;
    __syncthreads();
    if (tid == 0) {
        uint32_t tot = 0u;
        for (int w = 0; w < NW; ++w) {
            const uint32_t x = wsum[w];
            wsum[w] = tot;
            tot += x;
        }
        obase = atomicAdd(&nk[it.g], (unsigned long long)tot);
    }
    __syncthreads();
    uint64_t at = out_off[it.g] + obase + wsum[wave];
    const uint64_t hib = (uint64_t)b << R;
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < ROUNDS; ++i) {
        const uint32_t key = keys[i * kSpThreads + tid];
        const uint64_t mask = __ballot(key != kEmpty);
        if (key != kEmpty) {
            const uint64_t o = at + __popcll(mask & below);
            codes[o] = hib | key;
            counts[o] = cnts[i * kSpThreads + tid];
        }
        at += __popcll(mask);
    }
}

// Fallback, step 1: the residues of bucket b, pass p of genome g, in any order.
__global__ __launch_bounds__(256) void k_sp_gather(const uint32_t* __restrict__ ent,
                                                   const uint16_t* __restrict__ toff, uint32_t ldt,
                                                   uint64_t ta, uint64_t tb, uint32_t b, uint32_t p,
                                                   uint32_t np, int R, uint32_t* __restrict__ out,
                                                   uint32_t* __restrict__ n) {
    const uint64_t t = ta + (uint64_t)blockIdx.x;
    if (t >= tb) return;
    const uint32_t lo = toff[(uint64_t)b * ldt + t], hi = toff[(uint64_t)(b + 1) * ldt + t];
    for (uint32_t j = lo + threadIdx.x; j < hi; j += 256) {
        const uint32_t r = ent[t * (uint64_t)kSpTile + j];
        if (pass_of(r, np, R) == p) out[atomicAdd(n, 1u)] = r;
    }
}

// Fallback, step 3: append the run-length encoded keys to genome g's output.
__global__ __launch_bounds__(256) void k_sp_append(const uint32_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ runs,
                                                   const uint32_t* __restrict__ nruns, uint64_t hib,
                                                   uint64_t off, unsigned long long* __restrict__ nk,
                                                   uint64_t* __restrict__ codes,
                                                   uint32_t* __restrict__ counts) {
    __shared__ unsigned long long base;
    const uint32_t n = *nruns;
    if (threadIdx.x == 0) base = atomicAdd(nk, (unsigned long long)n);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        codes[off + base + i] = hib | keys[i];
        counts[off + base + i] = runs[i];
    }
}

void* carve(char*& p, size_t bytes) {
    void* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return r;
}

template <int K, int CANON>
void launch_partition(unsigned tiles, hipStream_t s, const uint8_t* seq, const GenomeMap& m,
                      uint32_t* ent, uint16_t* toff, uint32_t ldt) {
    hipLaunchKernelGGL((k_sp_partition<K, CANON>), dim3(tiles), dim3(kSpThreads), 0, s, seq, m, ent,
                       toff, ldt);
}

template <int K>
void partition_k(int canonical, unsigned tiles, hipStream_t s, const uint8_t* seq,
                 const GenomeMap& m, uint32_t* ent, uint16_t* toff, uint32_t ldt) {
    if (canonical) launch_partition<K, 1>(tiles, s, seq, m, ent, toff, ldt);
    else launch_partition<K, 0>(tiles, s, seq, m, ent, toff, ldt);
}

void launch_partition_k(int k, int canonical, unsigned tiles, hipStream_t s, const uint8_t* seq,
                        const GenomeMap& m, uint32_t* ent, uint16_t* toff, uint32_t ldt) {
    switch (k) {
    case 13: partition_k<13>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 14: partition_k<14>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 15: partition_k<15>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 16: partition_k<16>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 17: partition_k<17>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 18: partition_k<18>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 19: partition_k<19>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    case 20: partition_k<20>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    default: partition_k<21>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    }
}

// Fallback for one failed work item: gather, radix sort, run-length encode, append.
int fallback_item(Ctx* ctx, const SpItem& it, const uint32_t* ent, const uint16_t* toff,
                  uint32_t ldt, uint64_t ta, uint64_t tb, int R, uint64_t out_off,
                  unsigned long long* nk, uint64_t* codes, uint32_t* counts, hipStream_t s) {
    const int n = (int)it.n;
    size_t t_sort = 0, t_rle = 0;
    uint32_t* nul = nullptr;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortKeys(nullptr, t_sort, nul, nul, n, 0, R, s));
    KMH_HIP(ctx, hipcub::DeviceRunLengthEncode::Encode(nullptr, t_rle, nul, nul, nul, nul, n, s));
    const size_t temp = std::max(t_sort, t_rle);
    const size_t arr = ((size_t)n * 4 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->sparse[5], 4 * arr + temp + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[5].ptr);
    uint32_t* a = static_cast<uint32_t*>(carve(p, (size_t)n * 4));
    uint32_t* bsorted = static_cast<uint32_t*>(carve(p, (size_t)n * 4));
    uint32_t* ukeys = static_cast<uint32_t*>(carve(p, (size_t)n * 4));
    uint32_t* runs = static_cast<uint32_t*>(carve(p, (size_t)n * 4));
    uint32_t* small = static_cast<uint32_t*>(carve(p, 256));
    void* tmp = carve(p, temp);
    KMH_HIP(ctx, hipMemsetAsync(small, 0, 256, s));
    if (tb > ta) {
        hipLaunchKernelGGL(k_sp_gather, dim3((unsigned)(tb - ta)), dim3(256), 0, s, ent, toff, ldt, ta, tb,
                           it.b, (uint32_t)it.p, (uint32_t)it.np, R, a, small);
        KMH_HIP(ctx, hipGetLastError());
    }
    uint32_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, small, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    size_t t = temp;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortKeys(tmp, t, a, bsorted, (int)m, 0, R, s));
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceRunLengthEncode::Encode(tmp, t, bsorted, ukeys, runs, small + 1, (int)m, s));
    hipLaunchKernelGGL(k_sp_append, dim3(1), dim3(256), 0, s, ukeys, runs, small + 1,
                       (uint64_t)it.b << R, out_off, nk + it.g, codes, counts);
    KMH_HIP(ctx, hipGetLastError());
    KMH_HIP(ctx, hipStreamSynchronize(s));
    return KMH_OK;
}

}  // namespace

uint64_t sparse_windows(const uint64_t* offsets, int G, int k, uint64_t* out_off) {
    uint64_t tot = 0;
    for (int g = 0; g < G; ++g) {
        if (out_off) out_off[g] = tot;
        const uint64_t len = offsets[g + 1] - offsets[g];
        tot += len >= (uint64_t)k ? len - (uint64_t)k + 1 : 0;
    }
    if (out_off) out_off[G] = tot;
    return tot;
}

int sparse_count_dev(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                     int canonical, uint64_t* d_codes, uint32_t* d_counts, uint64_t* d_nkmers,
                     hipStream_t s) {
    if (k < 13 || k > 21) return fail(ctx, KMH_ERR_UNSUPPORTED, "device sparse counting needs 13 <= k <= 21");
    if (!d_seq || !d_codes || !d_counts || !d_nkmers) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    Layout L;
    int rc = make_layout(ctx, offsets, G, k, (uint64_t)kSpTile, L);
    if (rc) return rc;
    const int R = 2 * k - kSpBucketBits;
    std::vector<uint64_t> out_off(G + 1);
    sparse_windows(offsets, G, k, out_off.data());

    // Device metadata: goff, tbase (ctx->meta) and out_off (ctx->sparse[1], with the items).
    const uint64_t *d_goff, *d_tbase;
    rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
    if (rc) return rc;
    KMH_HIP(ctx, hipMemsetAsync(d_nkmers, 0, (size_t)G * sizeof(uint64_t), s));
    if (L.ntiles == 0) return KMH_OK;

    const size_t tile_bytes = (size_t)kSpTile * sizeof(uint32_t);
    const size_t budget = env_mb("KMH_SP_BUDGET_MB", 8192) << 20;
    const uint32_t target = (uint32_t)std::max<long>(1, env_long("KMH_SP_TARGET", 8192));
    const uint32_t limit = (uint32_t)std::min<long>(std::max<long>(1, env_long("KMH_SP_LIMIT", 12288)),
                                                    kSlots - kSpThreads - 1);
    // batches of whole genomes whose entries fit the budget
    std::vector<std::pair<int, int>> batches;
    uint64_t max_tiles = 0;
    for (int g = 0; g < G;) {
        int h = g;
        uint64_t tiles = 0;
        do {
            tiles += L.tbase[h + 1] - L.tbase[h];
            ++h;
        } while (h < G && (tiles + (L.tbase[h + 1] - L.tbase[h])) * tile_bytes <= budget);
        batches.emplace_back(g, h);
        max_tiles = std::max(max_tiles, tiles);
        g = h;
    }
    if (max_tiles > 0xFFFFFFFFull / kSpTile) return fail(ctx, KMH_ERR_UNSUPPORTED, "batch too large");
    const uint32_t ldt = (uint32_t)((max_tiles + 63) / 64 * 64);
    rc = ensure(ctx, ctx->sparse[2], std::max<uint64_t>(max_tiles, 1) * tile_bytes);
    if (!rc) rc = ensure(ctx, ctx->sparse[3], (size_t)ldt * (kSpBuckets + 1) * sizeof(uint16_t));
    if (rc) return rc;
    uint32_t* ent = static_cast<uint32_t*>(ctx->sparse[2].ptr);
    uint16_t* toff = static_cast<uint16_t*>(ctx->sparse[3].ptr);

    for (const auto& bt : batches) {
        const int g0 = bt.first, g1 = bt.second, nG = g1 - g0;
        const uint64_t tiles = L.tbase[g1] - L.tbase[g0];
        if (tiles == 0) continue;
        GenomeMap m{d_goff, d_tbase, g0, g1, L.tbase[g0], L.goff[G]};
        time_begin(ctx, s, "k_sp_partition");
        launch_partition_k(k, canonical, (unsigned)tiles, s, d_seq, m, ent, toff, ldt);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());

        // bucket sizes -> work items
        const size_t nb_n = (size_t)nG * kSpBuckets;
        rc = ensure(ctx, ctx->sparse[4], nb_n * 4 + 4096);
        if (rc) return rc;
        uint32_t* d_nb = static_cast<uint32_t*>(ctx->sparse[4].ptr);
        hipLaunchKernelGGL(k_sp_sizes, dim3((unsigned)nb_n), dim3(256), 0, s, toff, ldt, d_tbase, g0,
                           L.tbase[g0], d_nb);
        KMH_HIP(ctx, hipGetLastError());
        std::vector<uint32_t> nb(nb_n);
        KMH_HIP(ctx, hipMemcpyAsync(nb.data(), d_nb, nb_n * 4, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        std::vector<SpItem> items;
        items.reserve(nb_n * 2);
        for (int gl = 0; gl < nG; ++gl)
            for (int b = 0; b < kSpBuckets; ++b) {
                const uint32_t n = nb[(size_t)gl * kSpBuckets + b];
                if (!n) continue;
                const uint32_t np = std::min<uint32_t>(kMaxPasses, (n + target - 1) / target);
                for (uint32_t p = 0; p < np; ++p)
                    items.push_back(SpItem{(uint32_t)(g0 + gl), (uint32_t)b, (uint16_t)p, (uint16_t)np, n});
            }
        if (items.empty()) continue;
        // items + out_off + failed list in ctx->sparse[1]
        const size_t ib = (items.size() * sizeof(SpItem) + 255) & ~(size_t)255;
        const size_t ob = ((size_t)(G + 1) * 8 + 255) & ~(size_t)255;
        const size_t fb = (items.size() + 1) * 4;
        rc = ensure(ctx, ctx->sparse[1], ib + ob + fb);
        if (rc) return rc;
        char* base = static_cast<char*>(ctx->sparse[1].ptr);
        SpItem* d_items = reinterpret_cast<SpItem*>(base);
        uint64_t* d_out_off = reinterpret_cast<uint64_t*>(base + ib);
        uint32_t* d_failed = reinterpret_cast<uint32_t*>(base + ib + ob);
        KMH_HIP(ctx, hipMemcpyAsync(d_items, items.data(), items.size() * sizeof(SpItem), hipMemcpyHostToDevice, s));
        KMH_HIP(ctx, hipMemcpyAsync(d_out_off, out_off.data(), (size_t)(G + 1) * 8, hipMemcpyHostToDevice, s));
        KMH_HIP(ctx, hipMemsetAsync(d_failed, 0, 4, s));
        time_begin(ctx, s, "k_sp_count");
        hipLaunchKernelGGL(k_sp_count, dim3((unsigned)items.size()), dim3(kSpThreads), 0, s, ent, toff, ldt,
                           d_tbase, L.tbase[g0], d_items, R, limit, d_out_off, d_codes, d_counts,
                           reinterpret_cast<unsigned long long*>(d_nkmers), d_failed);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
        uint32_t nfail = 0;
        KMH_HIP(ctx, hipMemcpyAsync(&nfail, d_failed, 4, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        if (nfail) {
            std::vector<uint32_t> ids(nfail);
            KMH_HIP(ctx, hipMemcpyAsync(ids.data(), d_failed + 1, (size_t)nfail * 4, hipMemcpyDeviceToHost, s));
            KMH_HIP(ctx, hipStreamSynchronize(s));
            for (uint32_t id : ids) {
                const SpItem& it = items[id];
                rc = fallback_item(ctx, it, ent, toff, ldt, L.tbase[it.g] - L.tbase[g0],
                                   L.tbase[it.g + 1] - L.tbase[g0], R, out_off[it.g],
                                   reinterpret_cast<unsigned long long*>(d_nkmers), d_codes, d_counts, s);
                if (rc) return rc;
            }
        }
    }
    return KMH_OK;
}

}  // namespace kmh
