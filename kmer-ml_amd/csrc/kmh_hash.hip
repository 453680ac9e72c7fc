// kmh_hash.hip -- device-resident sparse k-mer counting (13 <= k <= 32, forward or
// canonical) for BASELINE config 5: 250 Mbp genomes at k = 21, where 4^k bins cannot be
// tabulated and almost every k-mer is distinct.  The reference counts into a Python dict
// (a hash table, /root/reference/kmerml/kmers/generate.py:36,58); here the counting is done
// by LDS hash tables after two partition passes, so every hash insert is an LDS operation
// and every kernel streams whole 16-byte chunks:
//
//  1. k_sp_partition  one workgroup per 32768-window tile: forward (and reverse-complement)
//                     codes from 2-bit packed registers, bucket = top 10 bits of the code
//                     (1024 buckets), LDS histogram + scan + scatter of the low 2k - 10 bits
//                     (u32 residues for k <= 21, u64 for 22 <= k <= 32 on half-size tiles),
//                     one coalesced store of the tile's entries and an exact
//                     bucket-major offset table toff[bucket][tile] (u16 entry indices).
//  2. k_sp_sizes      entries per (genome, bucket).  The host splits every bucket into
//                     P = ceil(entries / 8192) passes over equal residue ranges (one LDS hash
//                     table each) and into split items of ~12K entries (ranges of tiles).
//  3. k_sp_split      one workgroup per split item: gathers the bucket's segments of its
//                     tiles (16-byte chunk loads, entries outside the segment masked by
//                     position), partitions them by pass (LDS histogram, scan, scatter) and
//                     stores them contiguously with per-pass offsets toff2[item][pass].
//  4. k_sp_count      one workgroup per (genome, bucket, pass): reads that pass's segment of
//                     every split item of the bucket, inserts it into a 16384-slot LDS hash
//                     table (linear probing, 64-bit key|count slots; for u64 residues the count
//                     takes the 64 - (2k - 10) bits the key leaves, and an item whose count
//                     would overflow them goes to the fallback), then scans the table and
//                     appends the distinct k-mers to the genome's output (one atomic cursor).
//  5. fallback        a split item whose entries exceed its staging, or a pass whose distinct
//                     keys exceed the table limit, emits nothing; those passes are counted by
//                     gather + hipCUB radix sort + run-length encode from the step-1 entries
//                     (keys of different passes are disjoint, so nothing is counted twice).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "kmh_device.h"

namespace kmh {
namespace {

constexpr int kSpThreads = 1024;           // threads of every workgroup here
constexpr int kNW = kSpThreads / 64;       // waves per workgroup
constexpr int kSpBucketBits = 10;
constexpr int kSpBuckets = 1 << kSpBucketBits;
constexpr int kTileChunks = 8192;          // 16-byte chunks of a tile's entries (both widths)
constexpr int kQueue = 512;                // per-wave chunk queue of the split kernel
constexpr int kQU = 4;                     // chunk loads in flight per lane

// Entry width: u32 residues (k <= 21) or u64 (22 <= k <= 32).  A u64 tile holds half the windows,
// so a tile's entries (128 KiB) and a split item's staging (80 KiB) keep their LDS size.
template <typename E> struct Sp;
template <> struct Sp<uint32_t> {
    static constexpr int WPT = 32;                 // window starts per thread
    static constexpr int TILE = kSpThreads * WPT;  // 32768 window starts per tile (= kTile)
    static constexpr int CAPS = 20480;             // entries staged by one split item (80 KiB)
    static constexpr int KB = 16;                  // keys a count lane loads per round
};
template <> struct Sp<uint64_t> {
    static constexpr int WPT = 16;
    static constexpr int TILE = kSpThreads * WPT;  // 16384
    static constexpr int CAPS = 10240;             // 80 KiB
    static constexpr int KB = 8;
};
template <typename E> constexpr int epc() { return 16 / (int)sizeof(E); }   // entries per chunk
constexpr int kMaxPasses = 256;
constexpr int kT2 = kMaxPasses + 1;        // toff2 row stride
constexpr uint32_t kEmpty = 0xFFFFFFFFu;   // idle queue entry

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
    constexpr uint64_t M = K == 32 ? ~0ull : (1ull << (2 * K)) - 1ull;
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
template <int K, int CANON, int WPT, typename F>
__device__ __forceinline__ void each_window(const Bases& b, F&& f) {
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
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

template <int K, int CANON, typename E>
__global__ __launch_bounds__(kSpThreads) void k_sp_partition(const uint8_t* __restrict__ seq,
                                                             GenomeMap m,
                                                             E* __restrict__ ent,
                                                             uint16_t* __restrict__ toff,
                                                             uint32_t ldt) {
    constexpr int R = 2 * K - kSpBucketBits;
    constexpr uint64_t RM = (1ull << R) - 1ull;
    constexpr int WPT = Sp<E>::WPT, kSpTile = Sp<E>::TILE, EPC = epc<E>();
    static_assert(kSpBuckets == kSpThreads, "one bucket per thread in the scan");
    static_assert(R <= 8 * (int)sizeof(E), "residues fit the entry");
    __shared__ __attribute__((aligned(16))) E sorted[kSpTile];
    __shared__ uint32_t cnt[kSpBuckets];
    __shared__ uint32_t wsum[kNW];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = xcd_work_id();
    const uint64_t gt = m.tile_lo + lt;
    const int g = find_genome(m, gt);
    const uint64_t tstart = m.goff[g] + (gt - m.tbase[g]) * (uint64_t)kSpTile;
    const uint64_t ge = m.goff[g + 1];

    cnt[tid] = 0u;
    __syncthreads();

    const uint64_t base = tstart + (uint64_t)WPT * (uint64_t)tid;
    const Bases bs = (tstart + (uint64_t)kSpTile + 48 <= m.data_end) ? load_bases<true>(seq, base, ge)
                                                                     : load_bases<false>(seq, base, ge);
    each_window<K, CANON, WPT>(bs, [&](uint64_t c) { atomicAdd(&cnt[(uint32_t)(c >> R)], 1u); });
    __syncthreads();

    // Exclusive scan of the bucket counts; cnt becomes the scatter cursor.
    const uint32_t n0 = cnt[tid];
    uint32_t incl = n0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, total = 0u;
#pragma unroll
    for (int w = 0; w < kNW; ++w) {
        pre += (w < wave) ? wsum[w] : 0u;
        total += wsum[w];
    }
    const uint32_t s0 = pre + incl - n0;
    cnt[tid] = s0;
    toff[(uint64_t)tid * ldt + lt] = (uint16_t)s0;
    if (tid == 0) toff[(uint64_t)kSpBuckets * ldt + lt] = (uint16_t)total;
    __syncthreads();

    each_window<K, CANON, WPT>(bs, [&](uint64_t c) {
        const uint32_t slot = atomicAdd(&cnt[(uint32_t)(c >> R)], 1u);
        sorted[slot] = (E)(c & RM);
    });
    __syncthreads();

    E* dst = ent + lt * (uint64_t)kSpTile;
    const uint32_t n4 = total / EPC;
    for (uint32_t i = tid; i < n4; i += kSpThreads)
        store_nt(reinterpret_cast<uint4*>(dst) + i, reinterpret_cast<const uint4*>(sorted)[i]);
    if (tid < (int)(total % EPC)) __builtin_nontemporal_store(sorted[EPC * n4 + tid], dst + EPC * n4 + tid);
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

// np <= 256 and r < 2^R with R <= 54: the product fits 64 bits
__device__ __forceinline__ uint32_t pass_of(uint64_t r, uint32_t np, int R) {
    return (uint32_t)((r * np) >> R);
}

// Entry i of a 16-byte chunk (4 u32 or 2 u64 entries).
template <typename E>
__device__ __forceinline__ E lane_of(const uint4& v, int i) {
    if constexpr (sizeof(E) == 4) return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
    else return i == 0 ? ((uint64_t)v.y << 32 | v.x) : ((uint64_t)v.w << 32 | v.z);
}

// Split work item: tiles [t0, t1) (batch-relative) of bucket b of one genome.
struct SplitItem {
    uint32_t b, t0, t1, np;
    uint32_t gb;       // (genome, bucket) index within the batch: failure flag slot
    uint32_t per;      // expected entries per tile of this bucket
};

// f(r, true) for every entry of bucket b in tiles [ta, tb) (and f(x, false) for the other
// entries of the chunks read, so the caller can stay branch-free), read as 16-byte chunks through a
// per-wave queue: a wave takes bt tiles at a time (one per lane), lists the chunks that
// cover their segments (tile-in-batch << 13 | chunk-in-tile) and streams them with kQU
// loads in flight per lane; entries outside a segment are masked by position.
template <typename E, typename F>
__device__ __forceinline__ void walk_bucket(const E* __restrict__ ent,
                                            const uint16_t* __restrict__ toff, uint32_t ldt,
                                            uint32_t b, uint64_t ta, uint64_t tb, uint32_t bt,
                                            uint32_t* q, uint32_t* slo, uint32_t* shi, F&& f) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint4* chunks = reinterpret_cast<const uint4*>(ent);
    for (uint64_t tw = ta + (uint64_t)wave * bt; tw < tb; tw += (uint64_t)kNW * bt) {
        const uint64_t t = tw + (uint64_t)lane;
        const bool in = (uint32_t)lane < bt && t < tb;
        const uint32_t lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
        const uint32_t hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
        constexpr uint32_t EPC = (uint32_t)epc<E>();
        const uint32_t c0 = lo / EPC, nc = hi > lo ? (hi + EPC - 1u) / EPC - c0 : 0u;
        uint32_t incl = nc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        const uint32_t total = __shfl(incl, 63);
        if (total == 0u) continue;
        if (total <= (uint32_t)kQueue) {
            slo[lane] = lo;
            shi[lane] = hi;
            const uint32_t ex = incl - nc;
            for (uint32_t j = 0; j < nc; ++j) q[ex + j] = ((uint32_t)lane << 13) | (c0 + j);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t r0 = 0; r0 < total; r0 += 64u * kQU) {
                uint4 v[kQU];
                uint32_t qe[kQU];
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const uint32_t e = r0 + (uint32_t)(u * 64 + lane);
                    qe[u] = q[e < total ? e : 0u];  // idle lanes re-read entry 0 (valid)
                    v[u] = chunks[(tw + (qe[u] >> 13)) * (uint64_t)kTileChunks + (qe[u] & 8191u)];
                    if (e >= total) qe[u] = kEmpty;
                }
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const bool live = qe[u] != kEmpty;   // idle lanes: every entry invalid
                    const uint32_t qv = live ? qe[u] : 0u;
                    const uint32_t tl = qv >> 13, p0 = (qv & 8191u) * EPC;
                    const uint32_t l = slo[tl], h = live ? shi[tl] : 0u;
#pragma unroll
                    for (int i = 0; i < (int)EPC; ++i) f(lane_of<E>(v[u], i), p0 + i >= l && p0 + i < h);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {  // skewed batch: each lane walks its own segment
            for (uint32_t j = lo; j < hi; ++j) f(ent[t * (uint64_t)Sp<E>::TILE + j], true);
        }
    }
}

template <typename E>
__global__ __launch_bounds__(kSpThreads) void k_sp_split(
    const E* __restrict__ ent, const uint16_t* __restrict__ toff, uint32_t ldt,
    const SplitItem* __restrict__ items, int R, E* __restrict__ out,
    uint16_t* __restrict__ toff2, uint32_t* __restrict__ gb_fail) {
    constexpr int kCaps = Sp<E>::CAPS, EPC = epc<E>();
    __shared__ __attribute__((aligned(16))) E sorted[kCaps + 64];   // + scratch tail for out-of-segment lanes
    __shared__ uint32_t hist[kMaxPasses + 32];   // + dummy passes
    __shared__ uint32_t q[kNW][kQueue];
    __shared__ uint32_t slo[kNW][64], shi[kNW][64];
    __shared__ uint32_t wsum[4], total_sh;

    const uint32_t item = xcd_work_id();
    const SplitItem it = items[item];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kMaxPasses) hist[tid] = 0u;
    __syncthreads();
    uint32_t bt = (uint32_t)kQueue / 2u / (it.per / (uint32_t)EPC + 2u);
    bt = bt < 1u ? 1u : (bt > 64u ? 64u : bt);
    const uint32_t np = it.np;
    // Branch-free LDS atomics: an entry outside its segment counts into one of 32 dummy
    // passes (spread over banks by lane) and its scatter store goes to a 64-entry scratch
    // tail of `sorted`, so no exec-mask branch surrounds an atomic.
    const uint32_t dpass = (uint32_t)kMaxPasses + (uint32_t)(lane & 31);
    walk_bucket(ent, toff, ldt, it.b, it.t0, it.t1, bt, q[wave], slo[wave], shi[wave],
                [&](E r, bool ok) { atomicAdd(&hist[ok ? pass_of(r, np, R) : dpass], 1u); });
    __syncthreads();
    // exclusive scan of the pass histogram (threads 0..255)
    uint32_t n0 = 0u, incl = 0u;
    if (tid < kMaxPasses) {
        n0 = hist[tid];
        incl = n0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        if (lane == 63) wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < kMaxPasses) {
        uint32_t pre = 0u;
        for (int w = 0; w < wave; ++w) pre += wsum[w];
        const uint32_t st = pre + incl - n0;
        hist[tid] = st;
        if ((uint32_t)tid < np) toff2[(uint64_t)item * kT2 + tid] = (uint16_t)st;
        if (tid == 0) {
            const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
            total_sh = tot;
            toff2[(uint64_t)item * kT2 + np] = (uint16_t)(tot <= (uint32_t)kCaps ? tot : 0u);
            if (tot > (uint32_t)kCaps) gb_fail[it.gb] = 1u;
        }
    }
    __syncthreads();
    const uint32_t total = total_sh;
    if (total > (uint32_t)kCaps) return;  // staging overflow: the bucket goes to the fallback
    walk_bucket(ent, toff, ldt, it.b, it.t0, it.t1, bt, q[wave], slo[wave], shi[wave], [&](E r, bool ok) {
        const uint32_t slot = atomicAdd(&hist[ok ? pass_of(r, np, R) : dpass], 1u);
        sorted[ok ? slot : (uint32_t)kCaps + (uint32_t)lane] = r;
    });
    __syncthreads();
    E* dst = out + (uint64_t)item * kCaps;
    const uint32_t n4 = total / EPC;
    for (uint32_t i = tid; i < n4; i += kSpThreads)
        store_nt(reinterpret_cast<uint4*>(dst) + i, reinterpret_cast<const uint4*>(sorted)[i]);
    if (tid < (int)(total % EPC)) __builtin_nontemporal_store(sorted[EPC * n4 + tid], dst + EPC * n4 + tid);
}

// Count work item: pass p of bucket b of genome g; its entries are segment p of split items
// [s0, s1).
struct CountItem {
    uint32_t g, b, p, np;
    uint32_t s0, s1;
    uint32_t gb, n;
};

// Work items of one (genome, bucket) with n entries over nt tiles: P = ceil(n / target)
// passes (at most kMaxPasses), split items of ts tiles each (about split_target entries).
struct GbRule {
    uint32_t np, per, ts, nsplit;
    __device__ GbRule(uint32_t n, uint32_t nt, uint32_t target, uint32_t split_target) {
        np = (n + target - 1u) / target;
        np = np < (uint32_t)kMaxPasses ? np : (uint32_t)kMaxPasses;
        per = nt ? (n + nt - 1u) / nt : 0u;
        ts = split_target / (per + 1u);
        ts = ts < 1u ? 1u : ts;
        nsplit = n ? (nt + ts - 1u) / ts : 0u;
        if (!n) np = 0u;
    }
};

__device__ __forceinline__ uint32_t gb_tiles(const uint64_t* tbase, int g0, int gb) {
    const int g = g0 + gb / kSpBuckets;
    return (uint32_t)(tbase[g + 1] - tbase[g]);
}

// Item plan of a batch on the device (one workgroup): split and count items per
// (genome, bucket) pair, exclusive offsets of both in pair order, and the two totals.
__global__ __launch_bounds__(1024) void k_sp_plan(const uint32_t* __restrict__ nb, int ngb,
                                                  const uint64_t* __restrict__ tbase, int g0,
                                                  uint32_t target, uint32_t split_target,
                                                  uint32_t* __restrict__ sofs, uint32_t* __restrict__ cofs,
                                                  uint32_t* __restrict__ totals) {
    __shared__ uint32_t ws[16], wc[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per_t = (ngb + 1023) / 1024;
    const int a = tid * per_t, e = min(ngb, a + per_t);
    uint32_t ns = 0u, nc = 0u;
    for (int gb = a; gb < e; ++gb) {
        const GbRule r(nb[gb], gb_tiles(tbase, g0, gb), target, split_target);
        ns += r.nsplit;
        nc += r.np;
    }
    uint32_t is = ns, ic = nc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(is, d), y = __shfl_up(ic, d);
        if (lane >= d) {
            is += x;
            ic += y;
        }
    }
    if (lane == 63) {
        ws[wave] = is;
        wc[wave] = ic;
    }
    __syncthreads();
    uint32_t bs = 0u, bc = 0u;
    for (int w = 0; w < wave; ++w) {
        bs += ws[w];
        bc += wc[w];
    }
    uint32_t os = bs + is - ns, oc = bc + ic - nc;
    for (int gb = a; gb < e; ++gb) {
        const GbRule r(nb[gb], gb_tiles(tbase, g0, gb), target, split_target);
        sofs[gb] = os;
        cofs[gb] = oc;
        os += r.nsplit;
        oc += r.np;
    }
    if (tid == 1023) {
        totals[0] = os;
        totals[1] = oc;
    }
}

// Writes the items planned by k_sp_plan: one 64-thread workgroup per (genome, bucket).
__global__ __launch_bounds__(64) void k_sp_fill(const uint32_t* __restrict__ nb,
                                                const uint64_t* __restrict__ tbase, int g0,
                                                uint64_t tile_lo, uint32_t target, uint32_t split_target,
                                                const uint32_t* __restrict__ sofs,
                                                const uint32_t* __restrict__ cofs,
                                                SplitItem* __restrict__ sitems, CountItem* __restrict__ citems) {
    const int gb = blockIdx.x;
    const uint32_t n = nb[gb];
    if (!n) return;
    const int g = g0 + gb / kSpBuckets;
    const uint32_t b = (uint32_t)(gb % kSpBuckets);
    const uint32_t ta = (uint32_t)(tbase[g] - tile_lo), tb = (uint32_t)(tbase[g + 1] - tile_lo);
    const GbRule r(n, tb - ta, target, split_target);
    const uint32_t s0 = sofs[gb], s1 = s0 + r.nsplit;
    for (uint32_t i = threadIdx.x; i < r.nsplit; i += 64u) {
        const uint32_t t = ta + i * r.ts;
        sitems[s0 + i] = SplitItem{b, t, min(t + r.ts, tb), r.np, (uint32_t)gb, r.per};
    }
    for (uint32_t p = threadIdx.x; p < r.np; p += 64u)
        citems[cofs[gb] + p] = CountItem{(uint32_t)g, b, p, r.np, s0, s1, (uint32_t)gb, n};
}

template <int SB, int NT, typename E>
__global__ __launch_bounds__(NT) void k_sp_count(
    const E* __restrict__ split, const uint16_t* __restrict__ toff2,
    const CountItem* __restrict__ items, uint32_t nitems, int R, uint32_t limit,
    const uint64_t* __restrict__ out_off, uint64_t* __restrict__ codes,
    uint32_t* __restrict__ counts, unsigned long long* __restrict__ nk,
    const uint32_t* __restrict__ gb_fail, uint32_t* __restrict__ failed,
    unsigned long long* __restrict__ prof) {
    // Slot = key << CB | count (CB = 32 for u32 residues; 64 - R for u64 residues of R bits); a
    // slot is empty iff its count is 0, so every residue (k = 21 uses all 32 bits) is a valid
    // key.  A u64-residue count that would overflow its CB bits fails the item (the fallback
    // recounts it).  Emission scans the table: for each of the
    // kSlots / NT slot rows a wave reads 64 consecutive slots (conflict-free) and compacts
    // the occupied ones to consecutive output positions (ballot + mbcnt), so the stores are
    // coalesced and the insert loop keeps no record of the slots it claimed.
    constexpr int kSlots = 1 << SB, kSlotBits = SB, kNW = NT / 64;
    constexpr int kRows = kSlots / NT;             // slot rows per thread in the scan
    constexpr int kCap = kSlots * 3 / 4;           // distinct keys one table may hold
    __shared__ unsigned long long tbl[kSlots];
    __shared__ unsigned long long dummy[NT];     // CAS target of lanes without a key
    __shared__ uint32_t wtot[kNW], fail[2];
    __shared__ unsigned long long obase;
    constexpr uint32_t kMaxIter = 8u * 1024u;     // probes of one call (8 keys per lane)
    constexpr uint32_t SM = kSlots - 1u;
    constexpr int KB = Sp<E>::KB, kCaps = Sp<E>::CAPS;
    constexpr bool WIDE = sizeof(E) == 8;
    const int CB = WIDE ? 64 - R : 32;
    const unsigned long long CM = (1ull << CB) - 1ull;
    // slot hash: top bits of the low 32 bits of a 24 x 24-bit product (v_mul_u32_u24, full
    // rate; v_mul_lo_u32 is quarter rate) of the key folded to 24 bits (a u64 key first folded
    // to 32 bits)
    auto slot_of = [](E key) -> uint32_t {
        uint32_t x;
        if constexpr (WIDE) x = (uint32_t)key ^ (uint32_t)(key >> 29) * 0x9E3779B1u;
        else x = key;
        return (uint32_t)__umul24(x ^ (x >> 15), 0x9E3779u) >> (32 - kSlotBits);
    };

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t cap = limit < (uint32_t)kCap ? limit : (uint32_t)kCap;
    const uint64_t below = (1ull << lane) - 1ull;   // lanes before this one
    // The table is zero at the top of every item: zeroed once here, then by the emission of
    // each item (every thread clears the slots it has just read).  fail[par] collects the
    // probe-guard failures of the current item; the other flag is cleared for the next one.
    uint4* t4 = reinterpret_cast<uint4*>(tbl);
    for (int i = tid; i < kSlots / 2; i += NT) t4[i] = make_uint4(0u, 0u, 0u, 0u);
    if (tid < 2) fail[tid] = 0u;
    lds_barrier();
    uint32_t par = 0u;

    // Each lane walks its own keys one probe per iteration: CAS(empty -> key|1) claims a
    // slot, a slot holding the key gets +1, anything else sends the key to the next slot,
    // so an iteration waits on a single LDS round trip.  The key list advances by an
    // unconditional select (a conditional shift compiled to phi copies), the slot hash is
    // a full-rate 24-bit multiply, and the runaway guard is a wave-uniform (scalar)
    // iteration count instead of a per-lane probe counter.
    unsigned long long iters = 0, calls = 0;
    auto insert_keys = [&](E (&r)[8], int n) {
        ++calls;
        uint32_t s = slot_of(r[0]);
        for (uint32_t guard = 0; __ballot(n > 0); ++guard) {
            ++iters;
            if (guard == kMaxIter) {  // wave-uniform: a table this full goes to the fallback
                if (n > 0) fail[par] = 1u;
                break;
            }
            // Branch-free body: every lane issues the CAS and the add (a lane without keys
            // works on its own dummy slot, a lane without a match adds 0), and all updates
            // are selects, so the only branches are the uniform guard and the loop edge.
            const bool act = n > 0;
            unsigned long long* slot = act ? &tbl[s] : &dummy[tid];
            const unsigned long long old = atomicCAS(slot, 0ull, ((unsigned long long)r[0] << CB) | 1ull);
            const bool won = old == 0ull;
            const bool match = !won && (E)(old >> CB) == r[0];
            const unsigned long long prev = atomicAdd(slot, match ? 1ull : 0ull);
            if constexpr (WIDE) {   // the add that finds the count field full carried into the key
                if (match && (prev & CM) == CM) fail[par] = 1u;
            }
            const bool done = act && (won || match);
#pragma unroll
            for (int i = 0; i < 7; ++i) r[i] = done ? r[i + 1] : r[i];
            n -= done ? 1 : 0;
            uint32_t h = slot_of(r[0]);
            asm volatile("" : "+v"(h));   // keep the hash unconditional (no branch around it)
            s = done ? h : ((s + 1u) & SM);
        }
    };

    // Persistent: NT-thread workgroups walk the items.
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    const CountItem it = items[item];
    if (gb_fail[it.gb]) continue;  // the split overflowed: the fallback counts this bucket
    const unsigned long long c0 = prof ? clock64() : 0ull;

    // The item's entries are segment p of each split item in [s0, s1).  Per group of up to
    // 64 split items every wave reads the segment bounds (lane j: split item g + j), scans
    // their lengths, and takes an equal share of the group's entries (concatenated in
    // split-item order): entry e lies in the last segment whose exclusive start is <= e.
    // Equal shares matter: the workgroup waits at the barrier for its slowest wave.
    for (uint32_t g = it.s0; g < it.s1; g += 64u) {
        const uint32_t ns = min(64u, it.s1 - g);
        const uint32_t j = g + (uint32_t)lane;
        uint32_t lo = 0u, len = 0u;
        if ((uint32_t)lane < ns) {
            lo = toff2[(uint64_t)j * kT2 + it.p];
            len = (uint32_t)toff2[(uint64_t)j * kT2 + it.p + 1] - lo;
        }
        uint32_t incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        const uint32_t n = __shfl(incl, 63), excl = incl - len;
        // segment base in entries of `split`, minus the segment's exclusive start
        const uint64_t sb = (uint64_t)j * kCaps + lo - excl;   // kCaps: entries per split item
        const uint32_t sb_lo = (uint32_t)sb, sb_hi = (uint32_t)(sb >> 32);
        const uint32_t ea = (uint32_t)((uint64_t)n * (uint32_t)wave / kNW);
        const uint32_t eb = (uint32_t)((uint64_t)n * (uint32_t)(wave + 1) / kNW);
        for (uint32_t c = ea; c < eb; c += 64u * KB) {
            E r[KB];
            int cnt = 0;
#pragma unroll
            for (int u = 0; u < KB; ++u) {
                const uint32_t e0 = c + 64u * (uint32_t)u;        // entry of lane 0
                const uint32_t e = e0 + (uint32_t)lane;
                const bool ok = e < eb;
                // Lanes past the share read a valid entry instead (lane 0's, or entry c)
                // so every load is in bounds; es >= e1 on every lane.
                const uint32_t e1 = e0 < eb ? e0 : c;
                const uint32_t es = ok ? e : e1;
                // segment of e1 (wave-uniform), then step each lane forward to the segment
                // of es; the loop is wave-uniform so every lane takes part in each shuffle
                int sj = __popcll(__ballot((uint32_t)lane < ns && excl <= e1)) - 1;
                for (;;) {
                    const uint32_t nx = __shfl(excl, sj < 63 ? sj + 1 : 63);
                    const bool adv = sj + 1 < (int)ns && nx <= es;
                    if (!__ballot(adv)) break;
                    sj += adv ? 1 : 0;
                }
                const uint64_t base = ((uint64_t)(uint32_t)__shfl((int)sb_hi, sj) << 32) |
                                      (uint32_t)__shfl((int)sb_lo, sj);
                const E v = split[base + es];
                r[u] = ok ? v : (E)0;
                cnt += ok ? 1 : 0;   // valid entries of a lane are a prefix of r
            }
            // calls of 8 keys (a lane's valid keys are a prefix of r)
            E a8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) a8[u] = r[u];
            insert_keys(a8, cnt < 8 ? cnt : 8);
            if constexpr (KB == 16) {
                E b8[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) b8[u] = r[u + 8];
                if (__ballot(cnt > 8)) insert_keys(b8, cnt > 8 ? cnt - 8 : 0);
            }
        }
    }
    lds_barrier();
    const unsigned long long c1 = prof ? clock64() : 0ull;

    // Emission.  Each thread reads its kRows slots (rows q * NT + 64 * wave + lane,
    // conflict-free) into registers once, clears them for the next item, and the wave
    // counts its occupied slots; after the output base is known the registers are stored
    // (occupied slots compacted with ballot + mbcnt, so the stores are coalesced).
    unsigned long long x[kRows];
    uint32_t mine = 0u;
#pragma unroll
    for (int q = 0; q < kRows; ++q) {
        x[q] = tbl[q * NT + tid];
        mine += (uint32_t)__builtin_popcountll(__ballot((x[q] & CM) != 0ull));
    }
#pragma unroll
    for (int q = 0; q < kRows; ++q) tbl[q * NT + tid] = 0ull;
    if (lane == 0) wtot[wave] = mine;
    if (tid == 0) fail[par ^ 1u] = 0u;   // read by the previous item before this one began
    lds_barrier();
    uint32_t before = 0u, used = 0u;
#pragma unroll
    for (int w = 0; w < kNW; ++w) {
        const uint32_t v = wtot[w];
        before += w < wave ? v : 0u;
        used += v;
    }
    const bool bad = fail[par] || used > cap;
    if (tid == 0) {
        if (bad) {
            const uint32_t at = atomicAdd(&failed[0], 1u);
            failed[1 + at] = item;
        } else {
            obase = atomicAdd(&nk[it.g], (unsigned long long)used);
        }
    }
    lds_barrier();
    if (!bad) {
        const uint64_t at = out_off[it.g] + obase + before;
        const uint64_t hib = (uint64_t)it.b << R;
        uint32_t run = 0u;
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
            const bool occ = (x[q] & CM) != 0ull;
            const uint64_t m = __ballot(occ);
            if (occ) {
                const uint64_t i = at + run + (uint32_t)__builtin_popcountll(m & below);
                // plain stores: the wave's rows form one contiguous run, and write-back
                // stores merge the partial lines at row boundaries in L2 (exactly 12 B per
                // distinct k-mer reach HBM); non-temporal stores wrote 32 % more bytes
                codes[i] = hib | (x[q] >> CB);
                counts[i] = (uint32_t)(x[q] & CM);
            }
            run += (uint32_t)__builtin_popcountll(m);
        }
    }
    par ^= 1u;
    if (prof && tid == 0) {
        const unsigned long long c2 = clock64();
        atomicAdd(&prof[0], c1 - c0);
        atomicAdd(&prof[1], c2 - c1);
        atomicAdd(&prof[5], 1ull);
    }
    }
    if (prof && lane == 0) {
        atomicAdd(&prof[3], iters);
        atomicAdd(&prof[4], calls);
    }
}

// Fallback, step 1: the residues of bucket b, pass p of genome g, in any order.
template <typename E>
__global__ __launch_bounds__(256) void k_sp_gather(const E* __restrict__ ent,
                                                   const uint16_t* __restrict__ toff, uint32_t ldt,
                                                   uint64_t ta, uint64_t tb, uint32_t b, uint32_t p,
                                                   uint32_t np, int R, E* __restrict__ out,
                                                   uint32_t* __restrict__ n) {
    const uint64_t t = ta + (uint64_t)blockIdx.x;
    if (t >= tb) return;
    const uint32_t lo = toff[(uint64_t)b * ldt + t], hi = toff[(uint64_t)(b + 1) * ldt + t];
    for (uint32_t j = lo + threadIdx.x; j < hi; j += 256) {
        const E r = ent[t * (uint64_t)Sp<E>::TILE + j];
        if (pass_of(r, np, R) == p) out[atomicAdd(n, 1u)] = r;
    }
}

// Fallback, step 3: append the run-length encoded keys to genome g's output.
template <typename E>
__global__ __launch_bounds__(256) void k_sp_append(const E* __restrict__ keys,
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

template <int K, int CANON, typename E>
void launch_partition(unsigned tiles, hipStream_t s, const uint8_t* seq, const GenomeMap& m,
                      E* ent, uint16_t* toff, uint32_t ldt) {
    hipLaunchKernelGGL((k_sp_partition<K, CANON, E>), dim3(tiles), dim3(kSpThreads), 0, s, seq, m, ent,
                       toff, ldt);
}

template <int K, typename E>
void partition_k(int canonical, unsigned tiles, hipStream_t s, const uint8_t* seq,
                 const GenomeMap& m, E* ent, uint16_t* toff, uint32_t ldt) {
    if (canonical) launch_partition<K, 1, E>(tiles, s, seq, m, ent, toff, ldt);
    else launch_partition<K, 0, E>(tiles, s, seq, m, ent, toff, ldt);
}

template <typename E>
void launch_partition_k(int k, int canonical, unsigned tiles, hipStream_t s, const uint8_t* seq,
                        const GenomeMap& m, E* ent, uint16_t* toff, uint32_t ldt) {
#define KMH_PK(KK) case KK: partition_k<KK, E>(canonical, tiles, s, seq, m, ent, toff, ldt); break;
    if constexpr (sizeof(E) == 4) {
        switch (k) { KMH_PK(13) KMH_PK(14) KMH_PK(15) KMH_PK(16) KMH_PK(17) KMH_PK(18) KMH_PK(19) KMH_PK(20)
                     default: partition_k<21, E>(canonical, tiles, s, seq, m, ent, toff, ldt); break; }
    } else {
        switch (k) { KMH_PK(22) KMH_PK(23) KMH_PK(24) KMH_PK(25) KMH_PK(26) KMH_PK(27) KMH_PK(28) KMH_PK(29)
                     KMH_PK(30) KMH_PK(31)
                     default: partition_k<32, E>(canonical, tiles, s, seq, m, ent, toff, ldt); break; }
    }
#undef KMH_PK
}

// Fallback for pass p of bucket b of genome g: gather, radix sort, run-length encode, append.
template <typename E>
int fallback_pass(Ctx* ctx, uint32_t g, uint32_t b, uint32_t p, uint32_t np, uint32_t n,
                  const E* ent, const uint16_t* toff, uint32_t ldt, uint64_t ta, uint64_t tb,
                  int R, uint64_t out_off, unsigned long long* nk, uint64_t* codes, uint32_t* counts,
                  hipStream_t s) {
    size_t t_sort = 0, t_rle = 0;
    E* nulk = nullptr;
    uint32_t* nul = nullptr;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortKeys(nullptr, t_sort, nulk, nulk, (int)n, 0, R, s));
    KMH_HIP(ctx, hipcub::DeviceRunLengthEncode::Encode(nullptr, t_rle, nulk, nulk, nul, nul, (int)n, s));
    const size_t temp = std::max(t_sort, t_rle);
    const size_t arr = ((size_t)n * sizeof(E) + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->sparse[5], 4 * arr + temp + 1024);
    if (rc) return rc;
    char* p8 = static_cast<char*>(ctx->sparse[5].ptr);
    E* a = static_cast<E*>(carve(p8, (size_t)n * sizeof(E)));
    E* bsorted = static_cast<E*>(carve(p8, (size_t)n * sizeof(E)));
    E* ukeys = static_cast<E*>(carve(p8, (size_t)n * sizeof(E)));
    uint32_t* runs = static_cast<uint32_t*>(carve(p8, (size_t)n * 4));
    uint32_t* small = static_cast<uint32_t*>(carve(p8, 256));
    void* tmp = carve(p8, temp);
    KMH_HIP(ctx, hipMemsetAsync(small, 0, 256, s));
    if (tb > ta) {
        hipLaunchKernelGGL(k_sp_gather<E>, dim3((unsigned)(tb - ta)), dim3(256), 0, s, ent, toff, ldt, ta, tb,
                           b, p, np, R, a, small);
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
    hipLaunchKernelGGL(k_sp_append<E>, dim3(1), dim3(256), 0, s, ukeys, runs, small + 1,
                       (uint64_t)b << R, out_off, nk + g, codes, counts);
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

namespace {

template <typename E>
int sparse_count_dev_impl(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                          int canonical, uint64_t* d_codes, uint32_t* d_counts, uint64_t* d_nkmers,
                          hipStream_t s) {
    constexpr int kSpTile = Sp<E>::TILE, kCaps = Sp<E>::CAPS;
    Layout L;
    int rc = make_layout(ctx, offsets, G, k, (uint64_t)kSpTile, L);
    if (rc) return rc;
    const int R = 2 * k - kSpBucketBits;
    std::vector<uint64_t> out_off(G + 1);
    sparse_windows(offsets, G, k, out_off.data());

    const uint64_t *d_goff, *d_tbase;
    rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
    if (rc) return rc;
    KMH_HIP(ctx, hipMemsetAsync(d_nkmers, 0, (size_t)G * sizeof(uint64_t), s));
    if (L.ntiles == 0) return KMH_OK;

    const size_t tile_bytes = (size_t)kSpTile * sizeof(E);
    const size_t budget = env_mb("KMH_SP_BUDGET_MB", 16384) << 20;
    // LDS hash table of the count kernel: 2^14 slots.  Experiment builds (-DKMH_EXPERIMENTS)
    // also take KMH_SP_TABLE_BITS 12..13: smaller tables, several count workgroups per CU
    // (measured slower).
#ifdef KMH_EXPERIMENTS
    const int table_bits = (int)std::min<long>(14, std::max<long>(12, env_long("KMH_SP_TABLE_BITS", 14)));
#else
    const int table_bits = 14;
#endif
    const unsigned wg_per_cu = 1u << (14 - table_bits);   // LDS-limited residency
    const uint32_t target = (uint32_t)std::max<long>(1, env_long("KMH_SP_TARGET", 1l << (table_bits - 1)));
    const uint32_t split_target = (uint32_t)std::max<long>(1, std::min<long>(env_long("KMH_SP_SPLIT", 12288), kCaps));
    // KMH_SP_LIMIT caps the distinct keys of one table (tests force the fallback with it)
    const uint32_t limit = (uint32_t)std::min<long>(std::max<long>(1, env_long("KMH_SP_LIMIT", 1l << table_bits)),
                                                    1l << table_bits);
    // batches of whole genomes whose step-1 entries fit the budget (at most 2^18 tiles)
    std::vector<std::pair<int, int>> batches;
    uint64_t max_tiles = 0;
    for (int g = 0; g < G;) {
        int h = g;
        uint64_t tiles = 0;
        do {
            tiles += L.tbase[h + 1] - L.tbase[h];
            ++h;
        } while (h < G && (tiles + (L.tbase[h + 1] - L.tbase[h])) * tile_bytes <= budget &&
                 tiles + (L.tbase[h + 1] - L.tbase[h]) <= (1u << 18));
        batches.emplace_back(g, h);
        max_tiles = std::max(max_tiles, tiles);
        g = h;
    }
    if (max_tiles > (1u << 18)) return fail(ctx, KMH_ERR_UNSUPPORTED, "genome too large for the sparse path");
    const uint32_t ldt = (uint32_t)((max_tiles + 63) / 64 * 64);
    rc = ensure(ctx, ctx->sparse[2], std::max<uint64_t>(max_tiles, 1) * tile_bytes);
    if (!rc) rc = ensure(ctx, ctx->sparse[3], (size_t)ldt * (kSpBuckets + 1) * sizeof(uint16_t));
    if (rc) return rc;
    E* ent = static_cast<E*>(ctx->sparse[2].ptr);
    uint16_t* toff = static_cast<uint16_t*>(ctx->sparse[3].ptr);

    // Experiment builds: KMH_SP_PROF=1 or 2 prints the host phases of every batch (2: without
    // the kernel's own cycle counters, which slow it down)
#ifdef KMH_EXPERIMENTS
    const bool hprof = env_long("KMH_SP_PROF", 0) != 0;
#else
    const bool hprof = false;
#endif
    auto now_ms = [] {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    for (const auto& bt : batches) {
        const double h0 = hprof ? now_ms() : 0.0;
        const int g0 = bt.first, g1 = bt.second, nG = g1 - g0;
        const uint64_t tiles = L.tbase[g1] - L.tbase[g0];
        if (tiles == 0) continue;
        GenomeMap m{d_goff, d_tbase, g0, g1, L.tbase[g0], L.goff[G]};
        time_begin(ctx, s, "k_sp_partition");
        launch_partition_k(k, canonical, (unsigned)tiles, s, d_seq, m, ent, toff, ldt);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());

        // bucket sizes -> split and count work items, planned and written on the device;
        // the host reads back only the two item totals to size the buffers
        const size_t ngb = (size_t)nG * kSpBuckets;
        rc = ensure(ctx, ctx->sparse[4], ngb * 16 + 4096);
        if (rc) return rc;
        uint32_t* d_nb = static_cast<uint32_t*>(ctx->sparse[4].ptr);
        uint32_t* d_gbfail = d_nb + ngb;
        uint32_t* d_sofs = d_gbfail + ngb;
        uint32_t* d_cofs = d_sofs + ngb;
        uint32_t* d_totals = d_cofs + ngb;
        KMH_HIP(ctx, hipMemsetAsync(d_gbfail, 0, ngb * 4, s));
        hipLaunchKernelGGL(k_sp_sizes, dim3((unsigned)ngb), dim3(256), 0, s, toff, ldt, d_tbase, g0,
                           L.tbase[g0], d_nb);
        KMH_HIP(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_sp_plan, dim3(1), dim3(1024), 0, s, d_nb, (int)ngb, d_tbase, g0, target,
                           split_target, d_sofs, d_cofs, d_totals);
        KMH_HIP(ctx, hipGetLastError());
        uint32_t totals[2] = {0u, 0u};
        KMH_HIP(ctx, hipMemcpyAsync(totals, d_totals, 8, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        const double h1 = hprof ? now_ms() : 0.0;
        const size_t nsi = totals[0], nci = totals[1];
        if (nci == 0) continue;
        const double h2 = hprof ? now_ms() : 0.0;
        // split output + toff2 (ctx->sparse[6]); items, out_off, failed list (ctx->sparse[1])
        const size_t sbytes = nsi * (size_t)kCaps * sizeof(E);
        const size_t t2bytes = (nsi * kT2 * 2 + 255) & ~(size_t)255;
        rc = ensure(ctx, ctx->sparse[6], sbytes + t2bytes);
        if (rc) return rc;
        E* d_split = static_cast<E*>(ctx->sparse[6].ptr);
        uint16_t* d_toff2 = reinterpret_cast<uint16_t*>(static_cast<char*>(ctx->sparse[6].ptr) + sbytes);
        const size_t sib = (nsi * sizeof(SplitItem) + 255) & ~(size_t)255;
        const size_t cib = (nci * sizeof(CountItem) + 255) & ~(size_t)255;
        const size_t ob = ((size_t)(G + 1) * 8 + 255) & ~(size_t)255;
        const size_t fb = (nci + 1) * 4;
        rc = ensure(ctx, ctx->sparse[1], sib + cib + ob + fb);
        if (rc) return rc;
        char* base = static_cast<char*>(ctx->sparse[1].ptr);
        SplitItem* d_sitems = reinterpret_cast<SplitItem*>(base);
        CountItem* d_citems = reinterpret_cast<CountItem*>(base + sib);
        uint64_t* d_out_off = reinterpret_cast<uint64_t*>(base + sib + cib);
        uint32_t* d_failed = reinterpret_cast<uint32_t*>(base + sib + cib + ob);
        hipLaunchKernelGGL(k_sp_fill, dim3((unsigned)ngb), dim3(64), 0, s, d_nb, d_tbase, g0, L.tbase[g0],
                           target, split_target, d_sofs, d_cofs, d_sitems, d_citems);
        KMH_HIP(ctx, hipGetLastError());
        KMH_HIP(ctx, hipMemcpyAsync(d_out_off, out_off.data(), (size_t)(G + 1) * 8, hipMemcpyHostToDevice, s));
        KMH_HIP(ctx, hipMemsetAsync(d_failed, 0, 4, s));
        time_begin(ctx, s, "k_sp_split");
        hipLaunchKernelGGL(k_sp_split<E>, dim3((unsigned)nsi), dim3(kSpThreads), 0, s, ent, toff, ldt, d_sitems, R,
                           d_split, d_toff2, d_gbfail);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
        time_begin(ctx, s, "k_sp_count");
        const unsigned cgrid = (unsigned)std::min<size_t>(nci, (size_t)std::max(1, ctx->num_cu) * wg_per_cu);
        // KMH_SP_PROF=1 (experiment builds): per-phase cycle counters of k_sp_count on stderr
        unsigned long long* d_prof = nullptr;
#ifdef KMH_EXPERIMENTS
        const bool prof = env_long("KMH_SP_PROF", 0) == 1;
#else
        const bool prof = false;
#endif
        if (prof) {
            rc = ensure(ctx, ctx->sparse[7], 256);
            if (rc) return rc;
            d_prof = static_cast<unsigned long long*>(ctx->sparse[7].ptr);
            KMH_HIP(ctx, hipMemsetAsync(d_prof, 0, 256, s));
        }
#define KMH_SP_COUNT(SB, NT)                                                                         \
    hipLaunchKernelGGL((k_sp_count<SB, NT, E>), dim3(cgrid), dim3(NT), 0, s, d_split, d_toff2, d_citems, \
                       (uint32_t)nci, R, limit, d_out_off, d_codes, d_counts,                               \
                       reinterpret_cast<unsigned long long*>(d_nkmers), d_gbfail, d_failed, d_prof)
#ifdef KMH_EXPERIMENTS
        if (table_bits == 13) KMH_SP_COUNT(13, 1024);
        else if (table_bits == 12) KMH_SP_COUNT(12, 512);
        else
#endif
            KMH_SP_COUNT(14, 1024);
#undef KMH_SP_COUNT
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
        if (prof) {
            unsigned long long h[8];
            KMH_HIP(ctx, hipMemcpyAsync(h, d_prof, 64, hipMemcpyDeviceToHost, s));
            KMH_HIP(ctx, hipStreamSynchronize(s));
            std::fprintf(stderr, "k_sp_count prof: items %llu insert-phase cyc/item %.0f emit cyc/item %.0f "
                         "iterations/call %.2f calls/item %.1f\n", h[5], (double)h[0] / h[5],
                         (double)h[1] / h[5], (double)h[3] / (h[4] ? h[4] : 1), (double)h[4] / h[5]);
        }
        const double h3 = hprof ? now_ms() : 0.0;
        // passes left to the fallback: count items whose table overflowed, and every pass of
        // a bucket whose split overflowed
        uint32_t nfail = 0;
        std::vector<uint32_t> gbf(ngb);
        KMH_HIP(ctx, hipMemcpyAsync(&nfail, d_failed, 4, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipMemcpyAsync(gbf.data(), d_gbfail, ngb * 4, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        std::vector<uint32_t> ids(nfail);
        if (nfail) {
            KMH_HIP(ctx, hipMemcpyAsync(ids.data(), d_failed + 1, (size_t)nfail * 4, hipMemcpyDeviceToHost, s));
            KMH_HIP(ctx, hipStreamSynchronize(s));
        }
        bool any_gbf = false;
        for (uint32_t f : gbf) any_gbf |= f != 0u;
        std::vector<CountItem> citems;
        if (nfail || any_gbf) {  // items are only needed on the host to recount failed passes
            citems.resize(nci);
            KMH_HIP(ctx, hipMemcpyAsync(citems.data(), d_citems, nci * sizeof(CountItem), hipMemcpyDeviceToHost, s));
            KMH_HIP(ctx, hipStreamSynchronize(s));
            for (const CountItem& it : citems)
                if (gbf[it.gb]) ids.push_back((uint32_t)(&it - citems.data()));
        }
        const double h4 = hprof ? now_ms() : 0.0;
        for (uint32_t id : ids) {
            const CountItem& it = citems[id];
            rc = fallback_pass(ctx, it.g, it.b, it.p, it.np, it.n, ent, toff, ldt, L.tbase[it.g] - L.tbase[g0],
                               L.tbase[it.g + 1] - L.tbase[g0], R, out_off[it.g],
                               reinterpret_cast<unsigned long long*>(d_nkmers), d_codes, d_counts, s);
            if (rc) return rc;
        }
        if (hprof)
            std::fprintf(stderr, "sparse batch host phases (ms): partition+sizes wait %.2f, items %.2f (%zu split, "
                         "%zu count), uploads+launches %.2f, split+count wait %.2f, fallback %.2f (%zu passes)\n",
                         h1 - h0, h2 - h1, nsi, nci, h3 - h2, h4 - h3, now_ms() - h4, ids.size());
    }
    return KMH_OK;
}

}  // namespace

int sparse_count_dev(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                     int canonical, uint64_t* d_codes, uint32_t* d_counts, uint64_t* d_nkmers,
                     hipStream_t s) {
    if (k < 13 || k > 32) return fail(ctx, KMH_ERR_UNSUPPORTED, "device sparse counting needs 13 <= k <= 32");
    if (!d_seq || !d_codes || !d_counts || !d_nkmers) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    // residues of 2k - 10 bits: u32 entries up to k = 21, u64 beyond
    if (k <= 21) return sparse_count_dev_impl<uint32_t>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, d_nkmers, s);
    return sparse_count_dev_impl<uint64_t>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, d_nkmers, s);
}

}  // namespace kmh
