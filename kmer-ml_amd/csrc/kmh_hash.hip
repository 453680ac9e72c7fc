// kmh_hash.hip -- device-resident sparse k-mer counting (13 <= k <= 32, forward or
// canonical) for BASELINE config 5: 250 Mbp genomes at k = 21, where 4^k bins cannot be
// tabulated and almost every k-mer is distinct.  The reference counts into a Python dict
// (a hash table, /root/reference/kmerml/kmers/generate.py:36,58); here the keys are
// partitioned twice until one pass of a bucket fits a workgroup's LDS, and then deduplicated
// there by a counting sort; every kernel streams whole 16-byte chunks:
//
//  1. k_sp_partition  one workgroup per 32768-window tile: forward (and reverse-complement)
//                     codes from 2-bit packed registers, bucket = top 10 bits of the code
//                     (1024 buckets), LDS histogram + scan + scatter of the low 2k - 10 bits
//                     (u32 residues for k <= 21, u64 for 22 <= k <= 32 on half-size tiles),
//                     one coalesced store of the tile's entries and an exact
//                     bucket-major offset table toff[bucket][tile] (u16 entry indices).
//  2. k_sp_sizes      entries per (genome, bucket); k_sp_plan (one workgroup, on the device)
//     k_sp_plan       splits every bucket into P = ceil(entries / 7680) passes over equal
//     k_sp_fill       residue ranges (one count item each) and into split items of ~13-16K
//                     entries (ranges of tiles); k_sp_fill writes the items.  The host reads
//                     back only the two item totals.
//  3. k_sp_split      one workgroup per split item: gathers the bucket's segments of its
//                     tiles (16-byte chunk loads, entries outside the segment masked by
//                     position), partitions them by pass (LDS histogram, scan, scatter) and
//                     appends each pass's run to that pass's own region (one count item's
//                     keys, contiguous), at an offset reserved by one atomic per (item, pass).
//  4. k_sp_count      one item per (genome, bucket, pass), two persistent workgroups per CU:
//                     reads its region (contiguous: no segment lookup) into registers and
//                     deduplicates it by an LDS counting sort on the key's position inside the
//                     pass (8192 bins of about one key; equal keys share a bin); each thread
//                     then resolves 16 consecutive sorted positions from registers (neighbours
//                     +-3 compared, +-4 binned) and the rare bins that reach further by their
//                     exact range; bins of repeated keys go through a small LDS hash table.
//  5. fallback        a split item whose entries exceed its staging, or an item the count
//                     kernel cannot hold, emits nothing; those passes are counted by
//                     gather + the hand-written radix sort of kmh_sort.hip + run-length
//                     encode from the step-1 entries (keys of different passes are
//                     disjoint, so nothing is counted twice).
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
constexpr int kQueue = 512;                // per-wave chunk queue of the split kernel
constexpr int kQU = 4;                     // chunk loads in flight per lane (split kernel)

// Entry width: u32 residues (k <= 21) or u64 (22 <= k <= 32).  A u64 tile holds half the windows,
// so a tile's entries (128 KiB) and a split item's staging (80 KiB) keep their LDS size.
// POS (the drop-in's first occurrences): every entry also carries its window position (u32,
// relative to its genome) in a parallel array of the same layout; tiles and stagings are
// halved again so that entries + positions keep the same LDS.
template <typename E, bool POS> struct Sp;
template <> struct Sp<uint32_t, false> {
    static constexpr int WPT = 32;                 // window starts per thread
    static constexpr int TILE = kSpThreads * WPT;  // 32768 window starts per tile (= kTile)
    static constexpr int CAPS = 20480;             // entries staged by one split item (80 KiB)
};
template <> struct Sp<uint64_t, false> {
    static constexpr int WPT = 16;
    static constexpr int TILE = kSpThreads * WPT;  // 16384
    static constexpr int CAPS = 10240;             // 80 KiB
};
template <> struct Sp<uint32_t, true> {
    static constexpr int WPT = 16;
    static constexpr int TILE = kSpThreads * WPT;  // 16384 (entries + positions: 128 KiB)
    static constexpr int CAPS = 10240;             // 80 KiB with positions
};
template <> struct Sp<uint64_t, true> {
    static constexpr int WPT = 8;
    static constexpr int TILE = kSpThreads * WPT;  // 8192 (96 KiB)
    static constexpr int CAPS = 5120;              // 60 KiB
};
// Keys of one count item (one pass of a bucket): the capacity of its region and of the count
// kernel's LDS staging (the bin sort of k_sp_count); half with positions.
template <typename E, bool POS> struct Cnt;
template <> struct Cnt<uint32_t, false> { static constexpr int CAP = 8192; };
template <> struct Cnt<uint64_t, false> { static constexpr int CAP = 4096; };
template <> struct Cnt<uint32_t, true> { static constexpr int CAP = 4096; };    // + positions
template <> struct Cnt<uint64_t, true> { static constexpr int CAP = 2048; };
template <typename E> constexpr int epc() { return 16 / (int)sizeof(E); }   // entries per chunk
// 16-byte chunks of a tile's entries (8192, or 4096 with positions) and the bits of a queue
// entry that hold the chunk (the rest hold the tile within the batch)
template <typename E, bool POS> constexpr int tile_chunks() { return Sp<E, POS>::TILE * (int)sizeof(E) / 16; }
template <typename E, bool POS> constexpr int chunk_bits() { return tile_chunks<E, POS>() == 8192 ? 13 : 12; }
// positions of the entries of one chunk (4 u32 for u32 entries, 2 for u64)
using PosChunk = uint4;

// Tiles a wave of the split kernel takes per queue step, for segments of about `per` entries
// of `epc` per 16-byte chunk: a step fills at most half of the kQueue-chunk queue.
__host__ __device__ __forceinline__ uint32_t split_bt(uint32_t per, uint32_t epc) {
    uint32_t bt = (uint32_t)kQueue / 2u / (per / epc + 2u);
    return bt < 1u ? 1u : (bt > 64u ? 64u : bt);
}

// Passes of one bucket.  With positions (the drop-in) a pass holds 1920-3840 keys, so a bucket of
// a 2^32-window organism needs ~2200 passes; the split keeps each pass's staging start in LDS
// (pst, kMaxPasses + 1 words) and its reserved region offset in registers (one lane per pass).
// A bucket that needs more passes fails them, and they are recounted together (one gather + sort
// per (genome, bucket): fallback_passes).
constexpr int kMaxPasses = 4096;
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
    if (e == 128) return lo & M;  // (a 64-bit shift by 64 is undefined)
    return ((hi << (e - 64)) | (lo >> (128 - e))) & M;
}

// The 32 windows starting at tstart + 32 * threadIdx.x: packed codes and invalid masks.
struct Bases {
    uint64_t hi, lo;   // 64 bases, 2 bits each, first base in bit 63..62 of hi
    uint64_t inv;      // bit 63 = base 0 is not ACGT (or lies past the genome end)
};

// The 64 bytes behind a thread's windows: 16-byte loads inside the data, byte loads (0 past
// gend) in the last tile of the data.
__device__ __forceinline__ void load_raw(const uint8_t* __restrict__ seq, uint64_t base, uint64_t gend, bool fast,
                                         uint4 (&v)[4]) {
    if (fast) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const uint4*>(seq + base + 16 * q);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = load16(seq, base + 16 * q, gend);
    }
}

__device__ __forceinline__ Bases encode_bases(const uint4 (&v)[4], uint64_t base, uint64_t gend) {
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
// The reverse complements come from the reverse complement of the whole 64-base block, taken
// once per thread: window j's is the K bases of that block starting at base 64 - j - K, so it
// costs a constant-shift extract like the forward code instead of a bit reversal per window.
template <int K, int CANON, int WPT, typename F>
__device__ __forceinline__ void each_window(const Bases& b, F&& f) {
    // laundered: each call recomputes its codes rather than keeping the 2 x 32 of the first
    // call alive across the caller's barrier and scan (that spilled)
    uint64_t hi = b.hi, lo = b.lo;
    asm volatile("" : "+v"(hi), "+v"(lo));
    uint64_t rhi = 0ull, rlo = 0ull;
    if constexpr (CANON != 0) {
        rhi = revcomp<32>(lo);
        rlo = revcomp<32>(hi);
    }
    auto code = [&](int j) {
        uint64_t c = window<K>(hi, lo, j);
        if constexpr (CANON != 0) {
            const uint64_t r = window<K>(rhi, rlo, 64 - j - K);
            c = r < c ? r : c;
        }
        return c;
    };
    // a wave whose 64-byte spans hold no non-base byte (every wave of a synthetic genome but the
    // one at its end) takes every window without the per-window validity test and branch
    if (__builtin_amdgcn_ballot_w64(b.inv != 0ull) == 0ull) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) f(code(j), j);
        return;
    }
#pragma unroll
    for (int j = 0; j < WPT; ++j)
        if (((b.inv << j) >> (64 - K)) == 0ull) f(code(j), j);
}

// Persistent, one workgroup per CU (132 KiB of LDS).  XCD x (= blockIdx % 8) takes a contiguous
// run of the tiles, so the u16 offsets its workgroups write side by side share L2 lines, and its
// workgroups stride through that run.  Each tile's 64 bytes per thread are loaded behind the
// previous tile's LDS work, and each tile's entries drain behind the next tile's: the barriers
// wait for LDS operations only (lds_barrier), and the one wait for memory -- the next tile's
// bytes, encoded before this tile's stores are issued -- comes after a tile of LDS work.
template <int K, int CANON, typename E, bool POS>
__global__ __launch_bounds__(kSpThreads) void k_sp_partition(const uint8_t* __restrict__ seq,
                                                             GenomeMap m,
                                                             E* __restrict__ ent,
                                                             uint32_t* __restrict__ epos,
                                                             uint16_t* __restrict__ toff,
                                                             uint32_t ldt, uint32_t ntiles) {
    constexpr int R = 2 * K - kSpBucketBits;
    constexpr uint64_t RM = (1ull << R) - 1ull;
    constexpr int WPT = Sp<E, POS>::WPT, kSpTile = Sp<E, POS>::TILE, EPC = epc<E>();
    static_assert(kSpBuckets == kSpThreads, "one bucket per thread in the scan");
    static_assert(R <= 8 * (int)sizeof(E), "residues fit the entry");
    __shared__ __attribute__((aligned(16))) E sorted[kSpTile];
    __shared__ __attribute__((aligned(16))) uint32_t spos[POS ? kSpTile : 4];
    __shared__ uint32_t cnt[kSpBuckets];
    __shared__ uint32_t wsum[kNW];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t x = blockIdx.x % 8u, nwg = gridDim.x;
    const uint32_t nwx = (nwg - x + 7u) / 8u;                      // workgroups on XCD x
    const uint32_t tq = ntiles / 8u, trem = ntiles % 8u;
    const uint32_t xa = x * tq + (x < trem ? x : trem), xb = xa + tq + (x < trem ? 1u : 0u);
    uint32_t lt = xa + blockIdx.x / 8u;
    if (lt >= xb) return;   // whole workgroup

    // genome cursor (a workgroup's tiles ascend): tiles [tg0, tg1), bytes [gb0, gb1) of genome g
    int g = find_genome(m, m.tile_lo + lt);
    uint64_t tg0 = m.tbase[g], tg1 = m.tbase[g + 1], gb0 = m.goff[g], gb1 = m.goff[g + 1];
    struct Geo {
        uint64_t base, gend;
        uint32_t p0;   // window position of this thread's window 0 within its genome (< 2^32 - 1)
        bool fast;     // 16-byte loads stay inside the data
    };
    auto geo = [&](uint32_t t) {
        const uint64_t gt = m.tile_lo + t;
        if (gt >= tg1) {   // next genome (rare: the cursor's loads may wait for queued stores)
            do {
                ++g;
                tg0 = tg1;
                tg1 = m.tbase[g + 1];
            } while (gt >= tg1);
            gb0 = m.goff[g];
            gb1 = m.goff[g + 1];
        }
        const uint64_t tstart = gb0 + (gt - tg0) * (uint64_t)kSpTile;
        Geo r;
        r.base = tstart + (uint64_t)WPT * (uint64_t)tid;
        r.gend = gb1;
        r.p0 = (uint32_t)(r.base - gb0);
        r.fast = tstart + (uint64_t)kSpTile + 48 <= m.data_end;
        return r;
    };

    Geo cur = geo(lt);
    uint4 v[4];
    load_raw(seq, cur.base, cur.gend, cur.fast, v);
    Bases bs = encode_bases(v, cur.base, cur.gend);
    cnt[tid] = 0u;
    __syncthreads();

    for (;;) {
        const uint32_t nlt = lt + nwx;
        const bool more = nlt < xb;   // uniform
        Geo nxt = cur;
        if (more) {
            nxt = geo(nlt);
            if (nxt.fast) load_raw(seq, nxt.base, nxt.gend, true, v);   // lands during this tile
        }

        each_window<K, CANON, WPT>(bs, [&](uint64_t c, int) { atomicAdd(&cnt[(uint32_t)(c >> R)], 1u); });
        lds_barrier();

        // Exclusive scan of the bucket counts; cnt becomes the scatter cursor.
        const uint32_t n0 = cnt[tid];
        const uint32_t incl = scan64(n0);   // DPP: no LDS-pipe shuffles
        if (lane == 63) wsum[wave] = incl;
        lds_barrier();
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
        lds_barrier();

        const uint32_t p0 = cur.p0;
        each_window<K, CANON, WPT>(bs, [&](uint64_t c, int j) {
            const uint32_t slot = atomicAdd(&cnt[(uint32_t)(c >> R)], 1u);
            sorted[slot] = (E)(c & RM);
            if constexpr (POS) spos[slot] = p0 + (uint32_t)j;
        });
        lds_barrier();

        // the next tile's codes: its loads had this tile's LDS work to land, and waiting for
        // them here (before this tile's stores are queued behind them) costs little
        if (more) {
            if (!nxt.fast) load_raw(seq, nxt.base, nxt.gend, false, v);
            bs = encode_bases(v, nxt.base, nxt.gend);
        }
        cnt[tid] = 0u;   // (the cursors are dead; the next histogram starts after a barrier)

        E* dst = ent + (uint64_t)lt * kSpTile;
#if defined(KMH_EXPERIMENTS) && KMH_SP_PART_EXP == 1
        const uint32_t n4 = total == 0xFFFFFFFFu ? total / EPC : 0u;   // what-if: no entries stored
#else
        const uint32_t n4 = total / EPC;
#endif
        for (uint32_t i = tid; i < n4; i += kSpThreads)
            store_nt(reinterpret_cast<uint4*>(dst) + i, reinterpret_cast<const uint4*>(sorted)[i]);
        if (tid < (int)(total % EPC)) __builtin_nontemporal_store(sorted[EPC * n4 + tid], dst + EPC * n4 + tid);
        if constexpr (POS) {
            uint32_t* pdst = epos + (uint64_t)lt * kSpTile;
            for (uint32_t i = tid; i < total / 4; i += kSpThreads)
                store_nt(reinterpret_cast<uint4*>(pdst) + i, reinterpret_cast<const uint4*>(spos)[i]);
            if (tid < (int)(total % 4)) pdst[4 * (total / 4) + tid] = spos[4 * (total / 4) + tid];
        }
        if (!more) break;
        lds_barrier();   // zeroed counters visible; this tile's LDS reads done before the next scatter
        lt = nlt;
        cur = nxt;
    }
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

// Pass of residue r (R bits) in a bucket of np passes: floor(r * np / 2^R), the high word of
// (r << (W - R)) * np for W-bit residues (one multiply; exact for every np <= kMaxPasses, so a
// pass is a contiguous residue range and passes ascend with the residue).
template <typename E>
__device__ __forceinline__ uint32_t pass_of(E r, uint32_t np, int R) {
    if constexpr (sizeof(E) == 4) return __umulhi((uint32_t)r << (32 - R), np);
    else return (uint32_t)__umul64hi((uint64_t)r << (64 - R), (uint64_t)np);
}

// Entry i of a 16-byte chunk (4 u32 or 2 u64 entries).
template <typename E>
__device__ __forceinline__ E lane_of(const uint4& v, int i) {
    if constexpr (sizeof(E) == 4) return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
    else return i == 0 ? ((uint64_t)v.y << 32 | v.x) : ((uint64_t)v.w << 32 | v.z);
}

// Split work item: tiles [t0, t1) (batch-relative) of bucket b of one genome.
// A value every lane loads from the same address, as a VECTOR load (its address laundered through
// a VGPR).  A scalar load (s_load) counts in lgkmcnt like the LDS operations, and the compiler
// waits for it with lgkmcnt(0) at the next LDS wait (scalar loads return out of order): every
// descriptor prefetched with s_load stalled the following LDS phase for a memory round trip.  A
// vector load counts in vmcnt and is read (readfirstlane) where the wave waits for its vector loads
// anyway.
template <typename T>
__device__ __forceinline__ T vload(const T* p) {
    uint64_t a = reinterpret_cast<uint64_t>(p);
    asm volatile("" : "+v"(a));
    using gT = __attribute__((address_space(1))) const T;
    return *reinterpret_cast<gT*>(a);
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}

struct SplitItem {
    uint32_t b, t0, t1, np;
    uint32_t gb;       // (genome, bucket) index within the batch: failure flag slot
    uint32_t per;      // expected entries per tile of this bucket
    uint32_t cbase;    // count item of pass 0 of this (genome, bucket): pass p's region and
                       // fill counter are those of count item cbase + p
    uint32_t pad;
};

// add + the rank of this lane among the lanes set in ballot m (v_mbcnt_lo / v_mbcnt_hi, which
// add their second operand)
__device__ __forceinline__ uint32_t lane_rank(uint64_t m, uint32_t add = 0u) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, add));
}
// base + a 32-bit byte offset: with a uniform base the compiler addresses it as SGPR base + VGPR
// offset (global_* saddr form)
template <typename T>
__device__ __forceinline__ T* at_byte(T* base, uint32_t bytes) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + bytes);
}
// Positions of entries [4 c, 4 c + 4) (u32 entries) or [2 c, 2 c + 2) (u64) of a tile's layout.
template <typename E>
__device__ __forceinline__ PosChunk load_pos(const uint32_t* __restrict__ epos, uint64_t chunk) {
    if constexpr (sizeof(E) == 4) return reinterpret_cast<const uint4*>(epos)[chunk];
    const uint2 x = reinterpret_cast<const uint2*>(epos)[chunk];
    return make_uint4(x.x, x.y, 0u, 0u);
}

__device__ __forceinline__ uint32_t pos_of(const PosChunk& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// Entries of the chunk starting at entry p0 that lie in the segment [lo, hi): bit i = entry i.
template <uint32_t EPC>
__device__ __forceinline__ uint32_t seg_mask(uint32_t p0, uint32_t lo, uint32_t hi) {
    uint32_t m = 0u;
#pragma unroll
    for (uint32_t i = 0; i < EPC; ++i) m |= (p0 + i >= lo && p0 + i < hi) ? 1u << i : 0u;
    return m;
}

// f(r, pos, true) for every entry of bucket b in tiles [ta, tb) (and f(x, pos, false) for the
// other entries of the chunks read, so the caller can stay branch-free), read from memory as
// 16-byte chunks through a per-wave queue: a wave takes bt tiles at a time (one per lane),
// lists the chunks that cover their segments (tile-in-batch << 13 | chunk-in-tile) and streams
// them with kQU loads in flight per lane; entries outside a segment are masked by position.
// The split kernel's path for a wave whose share of an item does not fit its registers (Held).
template <bool POS, typename E, typename F>
__device__ __forceinline__ void walk_bucket(const E* __restrict__ ent, const uint32_t* __restrict__ epos,
                                            const uint16_t* __restrict__ toff, uint32_t ldt,
                                            uint32_t b, uint64_t ta, uint64_t tb, uint32_t bt,
                                            uint32_t* q, uint32_t* slo, uint32_t* shi, F&& f) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint4* chunks = reinterpret_cast<const uint4*>(ent);
    constexpr uint32_t EPC = (uint32_t)epc<E>();
    constexpr int CB = chunk_bits<E, POS>();
    constexpr uint32_t CM = (1u << CB) - 1u;
    constexpr uint64_t TC = (uint64_t)tile_chunks<E, POS>();
    for (uint64_t tw = ta + (uint64_t)wave * bt; tw < tb; tw += (uint64_t)kNW * bt) {
        const uint64_t t = tw + (uint64_t)lane;
        const bool in = (uint32_t)lane < bt && t < tb;
        const uint32_t lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
        const uint32_t hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
        const uint32_t c0 = lo / EPC, nc = hi > lo ? (hi + EPC - 1u) / EPC - c0 : 0u;
        const uint32_t incl = scan64(nc);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (total == 0u) continue;
        if (total <= (uint32_t)kQueue) {
            slo[lane] = lo;
            shi[lane] = hi;
            const uint32_t ex = incl - nc;
            for (uint32_t j = 0; j < nc; ++j) q[ex + j] = ((uint32_t)lane << CB) | (c0 + j);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t r0 = 0; r0 < total; r0 += 64u * kQU) {
                uint4 v[kQU];
                PosChunk pv[POS ? kQU : 1];
                uint32_t qe[kQU];
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const uint32_t e = r0 + (uint32_t)(u * 64 + lane);
                    qe[u] = q[e < total ? e : 0u];  // idle lanes re-read entry 0 (valid)
                    const uint64_t ci = (tw + (qe[u] >> CB)) * TC + (qe[u] & CM);
                    v[u] = chunks[ci];
                    if constexpr (POS) pv[u] = load_pos<E>(epos, ci);
                    if (e >= total) qe[u] = kEmpty;
                }
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const bool live = qe[u] != kEmpty;   // idle lanes: every entry invalid
                    const uint32_t qv = live ? qe[u] : 0u;
                    const uint32_t tl = qv >> CB, p0 = (qv & CM) * EPC;
                    const uint32_t l = slo[tl], h = live ? shi[tl] : 0u;
#pragma unroll
                    for (int i = 0; i < (int)EPC; ++i)
                        f(lane_of<E>(v[u], i), POS ? pos_of(pv[POS ? u : 0], i) : 0u, p0 + i >= l && p0 + i < h);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {  // skewed batch: each lane walks its own segment
            for (uint32_t j = lo; j < hi; ++j) {
                const uint64_t ix = t * (uint64_t)Sp<E, POS>::TILE + j;
                f(ent[ix], POS ? epos[ix] : 0u, true);
            }
        }
    }
}

// A wave's share of one split item held in registers: kQU chunks per lane and the entries of
// each that lie inside their segment (bit 4u + i: entry i of chunk u).  The split kernel walks
// an item twice (pass histogram, then scatter) and loads the next item's chunks while it works
// on the current one.  kept = false (wave-uniform): the share spans more than one queue step or
// 64 * kQU chunks, and both walks read it from memory (walk_bucket).
template <bool POS>
struct Held {
    uint4 v[kQU];
    PosChunk pv[POS ? kQU : 1];
    uint32_t mask;
    bool kept;
};
static_assert(kQU * 4 <= 32, "chunk masks of a lane fit 32 bits");

// Lists the chunks of the wave's tiles [tw, tw + 64) -- this lane's segment [lo, hi) of tile
// tw + lane -- in the wave's queue with their masks, and issues their loads into h (nobody
// waits for them here).  single: the wave's share of the item is this one step.
template <typename E, bool POS>
__device__ __forceinline__ void hold_chunks(const E* __restrict__ ent, const uint32_t* __restrict__ epos,
                                            uint64_t tw, uint32_t lo, uint32_t hi, bool single, uint32_t* q,
                                            Held<POS>& h) {
    const int lane = threadIdx.x & 63;
    const uint4* chunks = reinterpret_cast<const uint4*>(ent);
    constexpr uint32_t EPC = (uint32_t)epc<E>();
    constexpr int CB = chunk_bits<E, POS>();
    constexpr uint32_t CM = (1u << CB) - 1u;
    constexpr uint64_t TC = (uint64_t)tile_chunks<E, POS>();
    const uint32_t c0 = lo / EPC, nc = hi > lo ? (hi + EPC - 1u) / EPC - c0 : 0u;
    const uint32_t incl = scan64(nc);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    h.mask = 0u;
    h.kept = single && total <= 64u * (uint32_t)kQU;   // wave-uniform
    if (h.kept) {
        // queue entry: mask << 24 | tile-in-step << CB | chunk-in-tile (CB + 6 <= 19 bits); only
        // a segment's first and last chunks hold entries of other segments
        constexpr uint32_t FULL = (1u << EPC) - 1u;
        const uint32_t mf = seg_mask<EPC>(c0 * EPC, lo, hi), ml = seg_mask<EPC>((c0 + nc - 1u) * EPC, lo, hi);
        const uint32_t ex = incl - nc, lt = (uint32_t)lane << CB;
        for (uint32_t j = 0; j < nc; ++j)
            q[ex + j] = (((j == 0 ? mf : FULL) & (j + 1 == nc ? ml : FULL)) << 24) | lt | (c0 + j);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // The loads are issued on every path (a wave that does not keep its share loads chunk 0 of
    // the batch and masks it out), so that the compiler sees them complete at landed() on
    // every path and does not wait for them again behind the item's stores.
#pragma unroll
    for (int u = 0; u < kQU; ++u) {
        // idle lanes (and a wave with no tiles in this item, whose tw may lie past the batch)
        // load chunk 0 of the batch, with no entries
        const uint32_t e = (uint32_t)(u * 64 + lane);
        const bool live = h.kept && e < total;
        const uint32_t qe = live ? q[e] : 0u;
        const uint64_t ci = live ? (tw + ((qe >> CB) & 63u)) * TC + (qe & CM) : 0u;
        h.v[u] = chunks[ci];
        if constexpr (POS) h.pv[u] = load_pos<E>(epos, ci);
        h.mask |= (qe >> 24) << (4 * u);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename E, bool POS, typename F>
__device__ __forceinline__ void each_held(const Held<POS>& h, F&& f) {
    constexpr int EPC = epc<E>();
#pragma unroll
    for (int u = 0; u < kQU; ++u)
#pragma unroll
        for (int i = 0; i < EPC; ++i)
            f(lane_of<E>(h.v[u], i), POS ? pos_of(h.pv[POS ? u : 0], i) : 0u, ((h.mask >> (4 * u + i)) & 1u) != 0u);
}

// Makes the wave wait here for the loads into h (the compiler waits before an asm statement
// that reads a register whose load is still in flight).
template <bool POS>
__device__ __forceinline__ void landed(const Held<POS>& h) {
#pragma unroll
    for (int u = 0; u < kQU; ++u) {
        asm volatile("" ::"v"(h.v[u].x), "v"(h.v[u].y), "v"(h.v[u].z), "v"(h.v[u].w));
        if constexpr (POS) asm volatile("" ::"v"(h.pv[u].x), "v"(h.pv[u].y), "v"(h.pv[u].z), "v"(h.pv[u].w));
    }
}

#ifdef KMH_EXPERIMENTS
// KMH_SP_PROF=1: per-phase clocks of k_sp_split summed over its waves (lane 0 of each); [15] = waves
__device__ unsigned long long g_split_prof[16];
#define KMH_ST(i) if (lane == 0) { const unsigned long long t_ = clock64(); st_[i] += t_ - stl_; stl_ = t_; }
#else
#define KMH_ST(i)
#endif

// Persistent, one workgroup per CU (124 KiB of LDS).  XCD x (= blockIdx % 8) takes a contiguous
// run of the items and its workgroups stride through it.  Per item: (A) the next item's chunks
// are listed and loaded into registers from segment bounds fetched one item earlier, (B) the
// bounds of the item after that are fetched, (C) this item's entries -- already in registers --
// are counted by pass (LDS histogram), scanned and scattered into the LDS staging, then the
// wave waits for A and B, which had C's LDS work to land in, and (D) queues this item's
// stores, which drain behind the next item's work.  Barriers wait for LDS operations only.
template <typename E, bool POS>
__global__ __launch_bounds__(kSpThreads) void k_sp_split(
    const E* __restrict__ ent, const uint32_t* __restrict__ epos, const uint16_t* __restrict__ toff, uint32_t ldt,
    const SplitItem* __restrict__ items, uint32_t nitems, int R, E* __restrict__ out, uint32_t* __restrict__ opos,
    uint32_t* __restrict__ pfill, uint32_t* __restrict__ gb_fail) {
    constexpr int kCaps = Sp<E, POS>::CAPS, EPC = epc<E>(), C = Cnt<E, POS>::CAP;
    static_assert(kCaps < 65536, "staging offsets fit 16 bits");
    __shared__ __attribute__((aligned(16))) E sorted[kCaps + 64];   // + scratch tail for out-of-segment lanes
    __shared__ __attribute__((aligned(16))) uint32_t spos[POS ? kCaps + 64 : 4];
    // pass counters: np <= kRepP passes -- every item of config 5 (~32) -- count in 32 bank
    // replicas each (pass * 32 + lane % 32: the 32 lanes of a lane group never share an
    // address or a bank, where 64 lanes on ~32 plain counters collided); more passes: one
    // counter each.  Out-of-segment entries count into 32 dummies past the replicas.
    constexpr int kRepP = 128;
    static_assert(kRepP * 32 == 4 * kSpThreads && kMaxPasses <= kRepP * 32, "counter layout");
    __shared__ __attribute__((aligned(16))) uint32_t hist[kRepP * 32 + 32];
    __shared__ uint32_t q[kNW][kQueue];
    __shared__ uint32_t slo[kNW][64], shi[kNW][64];
    __shared__ uint32_t wsum[kNW], total_sh;
    __shared__ uint32_t pst[kMaxPasses + 1];   // staging start of every pass (+ the end)
    uint4* hist4 = reinterpret_cast<uint4*>(hist);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t x = blockIdx.x % 8u, nwg = gridDim.x;
    const uint32_t nwx = (nwg - x + 7u) / 8u;                      // workgroups on XCD x
    const uint32_t iq = nitems / 8u, irem = nitems % 8u;
    const uint32_t xa = x * iq + (x < irem ? x : irem), xb = xa + iq + (x < irem ? 1u : 0u);
    uint32_t item = xa + blockIdx.x / 8u;
    if (item >= xb) return;   // whole workgroup

    // this wave's tiles of an item: [t0 + wave * bt, + bt), one per lane; single: no second step
    auto wave_tiles = [&](const SplitItem& it, uint64_t& tw, bool& single) {
        const uint32_t bt = split_bt(it.per, (uint32_t)EPC);
        tw = (uint64_t)it.t0 + (uint64_t)wave * bt;
        single = tw + (uint64_t)kNW * bt >= it.t1;
        return bt;
    };
    auto bounds = [&](const SplitItem& it, uint32_t& lo, uint32_t& hi) {
        uint64_t tw;
        bool single;
        const uint32_t bt = wave_tiles(it, tw, single);
        const uint64_t t = tw + (uint64_t)lane;
        const bool in = (uint32_t)lane < bt && t < it.t1;
        // unconditional loads (see hold_chunks), masked afterwards
        const uint32_t l = toff[in ? (uint64_t)it.b * ldt + t : 0u];
        const uint32_t h = toff[in ? (uint64_t)(it.b + 1) * ldt + t : 0u];
        lo = in ? l : 0u;
        hi = in ? h : 0u;
    };

    hist4[tid] = make_uint4(0u, 0u, 0u, 0u);
    // kPipe: the next item's chunks load during this item (u32 / u64 entries).  With positions
    // two items' chunks do not fit the registers (the compiler spills, and every spill reload
    // waits for all loads and stores in flight), so each item's chunks load when it starts.
    constexpr bool kPipe = !POS;
    SplitItem cur = items[item];
    Held<POS> hc;
    hc.kept = false;
    hc.mask = 0u;
    uint32_t lo_c, hi_c;
    bounds(cur, lo_c, hi_c);
    if constexpr (kPipe) {
        uint64_t tw;
        bool single;
        wave_tiles(cur, tw, single);
        hold_chunks<E, POS>(ent, epos, tw, lo_c, hi_c, single, q[wave], hc);
    }
    uint32_t nitem = item + nwx;
    bool has_n = nitem < xb;
    SplitItem nxt = cur;
    uint32_t lo_n = 0u, hi_n = 0u;
    if (has_n) {
        nxt = items[nitem];
        bounds(nxt, lo_n, hi_n);
    }
    // descriptors are read one item ahead of their bounds (a scalar load's result is first
    // needed an item later)
    SplitItem nn = items[has_n && nitem + nwx < xb ? nitem + nwx : item];
    // complete before the loop on this path too: a wait inside the loop for a load of the
    // prologue would be executed every item, and would drain the previous item's stores
    landed(hc);
    asm volatile("" ::"v"(lo_n), "v"(hi_n), "v"(lo_c), "v"(hi_c));
    __syncthreads();

    // Branch-free LDS atomics: an entry outside its segment counts into one of 32 dummy
    // passes (spread over banks by lane) and its scatter store goes to a 64-entry scratch
    // tail of `sorted`, so no exec-mask branch surrounds an atomic.
    const uint32_t rl = (uint32_t)(lane & 31);
    // pass counter of entry r in an item of np passes (replicated for np <= kRepP)
    auto ctr = [&](uint32_t np, E r, bool ok) {   // branch-free: the dummy is a select
        const bool rep = np <= (uint32_t)kRepP;   // uniform
        const uint32_t c = (pass_of<E>(r, np, R) << (rep ? 5u : 0u)) | (rep ? rl : 0u);
        return ok ? c : (uint32_t)(kRepP * 32) + rl;
    };
    // the pass histogram of an item (its chunks held in h, or walked from memory)
    auto histogram = [&](const SplitItem& it, const Held<POS>& h) {
        auto count_pass = [&](E r, uint32_t, bool ok) { atomicAdd(&hist[ctr(it.np, r, ok)], 1u); };
        if (h.kept) each_held<E, POS>(h, count_pass);   // wave-uniform
        else walk_bucket<POS>(ent, epos, toff, ldt, it.b, it.t0, it.t1, split_bt(it.per, (uint32_t)EPC), q[wave],
                              slo[wave], shi[wave], count_pass);
    };
    // Region offsets of an item's passes, reserved once its pass counts exist (read by readlane
    // in its stores): lane j of wave w reserves pass w + 16 (64 r + j)'s run in that count item's
    // region.  An item whose entries overflow the staging (total > kCaps, its bucket goes to the
    // fallback) reserves too; its count items are skipped, so nothing reads the regions.  These
    // returning adds go to memory (device scope) and take microseconds under the kernel's own
    // traffic; they are issued right after the pass histogram, before the scan.
    constexpr int kRR = (kMaxPasses + 64 * kNW - 1) / (64 * kNW);
    auto reserve = [&](const SplitItem& it, uint32_t (&ao)[kRR]) {
        const bool rep = it.np <= (uint32_t)kRepP;   // uniform
#pragma unroll
        for (int r = 0; r < kRR; ++r) {
            ao[r] = 0u;
            const uint32_t p = (uint32_t)wave + (uint32_t)kNW * (64u * (uint32_t)r + (uint32_t)lane);
            if (p < it.np) {
                uint32_t c = 0u;
                if (rep) {
#pragma unroll
                    for (int qq = 0; qq < 8; ++qq) {
                        const uint4 hv = hist4[8u * p + (uint32_t)qq];
                        c += hv.x + hv.y + hv.z + hv.w;
                    }
                } else {
                    c = hist[p];
                }
#if defined(KMH_EXPERIMENTS) && KMH_SP_SPLIT_EXP == 2
                // what-if: no returning atomic to wait for (every split item writes its run at the
                // region's start: counts wrong; timing only)
                if (c) atomicAdd(&pfill[it.cbase + p], c);
#else
                if (c) ao[r] = atomicAdd(&pfill[it.cbase + p], c);
#endif
            }
        }
    };
    uint32_t aoff[kRR];
#ifdef KMH_EXPERIMENTS
    unsigned long long st_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stl_ = clock64();
#endif
    for (;;) {
        // (A) the next item's chunks, (B) the bounds of the one after
        Held<POS> hn;
        hn.kept = false;
        hn.mask = 0u;
        const uint32_t nnitem = nitem + nwx;
        const bool has_nn = has_n && nnitem < xb;   // uniform
        uint32_t lo_nn = 0u, hi_nn = 0u;
        SplitItem nnn;
        {   // on every path (after the last item: a copy of the current one, never used)
            uint64_t tw;
            bool single;
            if constexpr (kPipe) {
                wave_tiles(nxt, tw, single);
                hold_chunks<E, POS>(ent, epos, tw, lo_n, hi_n, single, q[wave], hn);
            } else {
                wave_tiles(cur, tw, single);
                hold_chunks<E, POS>(ent, epos, tw, lo_c, hi_c, single, q[wave], hc);
            }
            KMH_ST(0)
            bounds(nn, lo_nn, hi_nn);
            KMH_ST(1)
        }

        // (C) this item: pass histogram and reservations, scan, scatter
        const uint32_t np = cur.np;
        const bool rep = np <= (uint32_t)kRepP;   // uniform
        const uint32_t bt = split_bt(cur.per, (uint32_t)EPC);
        histogram(cur, hc);
        KMH_ST(2)
        lds_barrier();
        KMH_ST(3)
        reserve(cur, aoff);
        // exclusive scan of the counters (pass-major): thread t owns counters 4t .. 4t + 3 (pass p's
        // 32 replicas are counters 32p .. 32p + 31, i.e. threads 8p .. 8p + 7; without replicas
        // counter p); counters past the item's passes are zero.  (Its barrier also orders the
        // previous item's reads of pst and of the staging before the writes below.)
        {
            const uint4 cv = hist4[tid];
            const uint32_t sm = cv.x + cv.y + cv.z + cv.w;
            const uint32_t incl = scan64(sm);
            if (lane == 63) wsum[wave] = incl;
            lds_barrier();
            uint32_t pre = 0u, tot = 0u;
#pragma unroll
            for (int w = 0; w < kNW; ++w) {
                const uint32_t x = wsum[w];
                pre += w < wave ? x : 0u;
                tot += x;
            }
            const uint32_t ex = pre + incl - sm;
            const uint32_t e1 = ex + cv.x, e2 = e1 + cv.y, e3 = e2 + cv.z;
            hist4[tid] = make_uint4(ex, e1, e2, e3);
            if (rep) {
                if ((tid & 7) == 0 && (uint32_t)tid / 8u < np) pst[tid / 8] = ex;
            } else {
                const uint32_t p0 = 4u * (uint32_t)tid;
                if (p0 < np) pst[p0] = ex;
                if (p0 + 1u < np) pst[p0 + 1u] = e1;
                if (p0 + 2u < np) pst[p0 + 2u] = e2;
                if (p0 + 3u < np) pst[p0 + 3u] = e3;
            }
            if (tid == 0) {
                total_sh = tot;
                pst[np] = tot;
                if (tot > (uint32_t)kCaps) gb_fail[cur.gb] = 1u;   // staging overflow: the bucket goes to the fallback
            }
        }
        lds_barrier();
        KMH_ST(4)
        const uint32_t total = total_sh;
        const bool fits = total <= (uint32_t)kCaps;   // uniform
        if (fits) {
            auto scatter = [&](E r, uint32_t p, bool ok) {
                const uint32_t slot = atomicAdd(&hist[ctr(np, r, ok)], 1u);
                const uint32_t at = ok ? slot : (uint32_t)kCaps + (uint32_t)lane;
                sorted[at] = r;
                if constexpr (POS) spos[at] = p;
            };
            if (hc.kept) each_held<E, POS>(hc, scatter);
            else walk_bucket<POS>(ent, epos, toff, ldt, cur.b, cur.t0, cur.t1, bt, q[wave], slo[wave], shi[wave], scatter);
        }
        KMH_ST(5)
        lds_barrier();
        KMH_ST(6)

        // the descriptor two items ahead, first used by the next item's bounds: a scalar load counts
        // in lgkmcnt like the LDS operations, so every LDS barrier waits for it -- issued here, after
        // the scatter's barrier, only the end-of-item barrier (behind the wait for A and B and the
        // queued stores) waits for it, instead of the histogram's barrier right after it was issued
        // (round 4: 4.7 Mcyc per wave at that barrier, profiles/r04/r04p/ab/exp0.log)
        nnn = items[has_nn && nnitem + nwx < xb ? nnitem + nwx : item];
        // A and B have landed by now (waited for here, not behind D's stores)
        if constexpr (kPipe) landed(hn);
        asm volatile("" ::"v"(lo_nn), "v"(hi_nn));
        KMH_ST(7)
        hist4[tid] = make_uint4(0u, 0u, 0u, 0u);   // the cursors are dead; the next histogram follows a barrier

        // (D) this item's stores: pass p's run of the staging [pst[p], pst[p + 1]) is appended to
        // count item cbase + p's region at the reserved offset; entries past the region's capacity
        // are dropped (that item's fill counter then exceeds C: it goes to the fallback)
#if defined(KMH_EXPERIMENTS) && KMH_SP_SPLIT_EXP == 1
        if (fits && total == 0xFFFFFFFFu) {   // what-if: no split output (timing of the split only)
#else
        if (fits) {
#endif
            for (uint32_t k = 0; (uint32_t)wave + (uint32_t)kNW * k < np; ++k) {   // (uniform)
                const uint32_t p = (uint32_t)wave + (uint32_t)kNW * k;
                const uint32_t r = k / 64u;   // (uniform; a select chain, not a dynamic register index)
                uint32_t av = aoff[0];
#pragma unroll
                for (int qq = 1; qq < kRR; ++qq) av = r == (uint32_t)qq ? aoff[qq] : av;
                const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)av, (int)(k % 64u));
                const uint32_t s0 = pst[p], n = pst[p + 1] - s0;
                const uint32_t lim = o < (uint32_t)C ? min(n, (uint32_t)C - o) : 0u;
                const uint64_t d = (uint64_t)(cur.cbase + p) * C + o;
                // non-temporal: the runs are read once, by the count kernel (plain stores wrote
                // 16.7 instead of 19.2 GB but ran 11.9 vs 11.2 ms, profiles/r04/r04n)
                for (uint32_t i = (uint32_t)lane; i < lim; i += 64u) {
                    __builtin_nontemporal_store(sorted[s0 + i], out + d + i);
                    if constexpr (POS) __builtin_nontemporal_store(spos[s0 + i], opos + d + i);
                }
            }
        }
        KMH_ST(8)
        if (!has_n) break;
        lds_barrier();   // the zeroed counters visible before the next histogram
        KMH_ST(9)
        item = nitem;
        cur = nxt;
        if constexpr (kPipe) hc = hn;
        nitem = nnitem;
        has_n = has_nn;
        nxt = nn;
        nn = nnn;
        lo_c = lo_n;
        hi_c = hi_n;
        lo_n = lo_nn;
        hi_n = hi_nn;
    }
#ifdef KMH_EXPERIMENTS
    if (lane == 0) {
        for (int i = 0; i < 10; ++i) atomicAdd(&g_split_prof[i], st_[i]);
        atomicAdd(&g_split_prof[15], 1ull);
    }
#endif
}

// Count work item: pass p of bucket b of genome g; its keys are the first pfill[item] entries of
// its region (item * Cnt<E, POS>::CAP), appended by the split items of the bucket.
struct CountItem {
    uint32_t g, b, p, np;
    uint32_t gb, n;    // (genome, bucket) index in the batch; the bucket's entries
};

// Work items of one (genome, bucket) with n entries over nt tiles: P = ceil(n / target)
// passes (at most kMaxPasses), split items of ts tiles each (about split_target entries).
struct GbRule {
    uint32_t np, per, ts, nsplit;
    // ts is also capped at one queue step per wave of the split kernel, so that each wave
    // reads its chunks once (k_sp_split keeps them in registers between its two walks)
    __device__ GbRule(uint32_t n, uint32_t nt, uint32_t target, uint32_t split_target, uint32_t epc) {
        np = (n + target - 1u) / target;
        np = np < (uint32_t)kMaxPasses ? np : (uint32_t)kMaxPasses;
        per = nt ? (n + nt - 1u) / nt : 0u;
        ts = split_target / (per + 1u);
        ts = ts < 1u ? 1u : ts;
        const uint32_t one_step = (uint32_t)kNW * split_bt(per, epc);
        ts = ts < one_step ? ts : one_step;
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
                                                  uint32_t target, uint32_t split_target, uint32_t epc,
                                                  uint32_t* __restrict__ sofs, uint32_t* __restrict__ cofs,
                                                  uint32_t* __restrict__ totals) {
    __shared__ uint32_t ws[16], wc[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per_t = (ngb + 1023) / 1024;
    const int a = tid * per_t, e = min(ngb, a + per_t);
    uint32_t ns = 0u, nc = 0u;
    for (int gb = a; gb < e; ++gb) {
        const GbRule r(nb[gb], gb_tiles(tbase, g0, gb), target, split_target, epc);
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
        const GbRule r(nb[gb], gb_tiles(tbase, g0, gb), target, split_target, epc);
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

// Split items in tile order.  Listed bucket by bucket, the items of one (genome, bucket) would run
// side by side on one XCD (its workgroups take a run of consecutive items) and read one bucket's
// segments from every tile of the genome; the 128-byte line a segment shares with the next
// bucket's segment of the same tile would be read again much later, from HBM (the split read
// 1.6x its entries).  So k_sp_fill writes every genome's split items ordered by (first tile,
// tiles per item ts, bucket): items over the same tiles run together and that line is still in
// the XCD's L2.  The items are the same; only their indices change.  k_sp_order (one workgroup
// per genome, thread = bucket) lists the genome's distinct ts values ascending with the number of
// non-empty buckets using each (tab: ts | count << 16; ts <= 16 * 64, a count <= 1024) and each
// bucket's rank among the buckets of its ts (grank).  Item i of a bucket starts at tile x = i ts;
// the items before it are, for every value v of count c (ns = ceil(tiles / v) items each), c
// min(ns, ceil(x / v)) starting before x, plus c more when v < ts and one of them starts at x,
// plus the bucket's rank.
__global__ __launch_bounds__(kSpBuckets) void k_sp_order(const uint32_t* __restrict__ nb,
                                                         const uint64_t* __restrict__ tbase, int g0,
                                                         uint32_t target, uint32_t split_target, uint32_t epc,
                                                         uint32_t* __restrict__ grank, uint32_t* __restrict__ tab,
                                                         uint32_t* __restrict__ nv) {
    static_assert(kSpBuckets == 1024 && kNW * 64 <= kSpBuckets, "one thread per bucket and per ts value");
    __shared__ uint32_t tss[kSpBuckets], cnt[kSpBuckets], ws[16];
    const uint32_t gl = blockIdx.x, b = threadIdx.x, lane = b & 63u, wave = b >> 6;
    const uint32_t gb = gl * (uint32_t)kSpBuckets + b;
    const GbRule r(nb[gb], gb_tiles(tbase, g0, (int)gb), target, split_target, epc);
    const uint32_t v = r.nsplit ? r.ts : 0u;   // 0: no items
    tss[b] = v;
    cnt[b] = 0u;
    __syncthreads();
    if (v) atomicAdd(&cnt[v - 1u], 1u);
    uint32_t rk = 0u;
    for (uint32_t j = 0; j < b; ++j) rk += tss[j] == v ? 1u : 0u;
    grank[gb] = rk;
    __syncthreads();
    // thread t: value t + 1; the values in use compacted in ascending order
    const uint32_t c = cnt[b], f = c ? 1u : 0u;
    uint32_t incl = f;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if ((int)lane >= d) incl += x;
    }
    if (lane == 63u) ws[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, tot = 0u;
    for (uint32_t w = 0; w < (uint32_t)kNW; ++w) {
        if (w < wave) pre += ws[w];
        tot += ws[w];
    }
    if (c) tab[gb - b + pre + incl - 1u] = (b + 1u) | (c << 16);
    if (b == 0u) nv[gl] = tot;
}

// Writes the items planned by k_sp_plan: one 64-thread workgroup per (genome, bucket); the
// genome's split items in tile order (k_sp_order), its count items in pair order.
__global__ __launch_bounds__(64) void k_sp_fill(const uint32_t* __restrict__ nb,
                                                const uint64_t* __restrict__ tbase, int g0,
                                                uint64_t tile_lo, uint32_t target, uint32_t split_target,
                                                uint32_t epc,
                                                const uint32_t* __restrict__ sofs,
                                                const uint32_t* __restrict__ cofs,
                                                const uint32_t* __restrict__ grank, const uint32_t* __restrict__ tab,
                                                const uint32_t* __restrict__ nv,
                                                SplitItem* __restrict__ sitems, CountItem* __restrict__ citems) {
    __shared__ uint32_t tv[kSpBuckets];
    const int gb = blockIdx.x;
    const uint32_t n = nb[gb];
    if (!n) return;   // (the whole workgroup)
    const int gl = gb / kSpBuckets;
    const int g = g0 + gl;
    const uint32_t V = nv[gl];
    for (uint32_t u = threadIdx.x; u < V; u += 64u) tv[u] = tab[(uint32_t)gl * kSpBuckets + u];
    __syncthreads();
    const uint32_t b = (uint32_t)(gb % kSpBuckets);
    const uint32_t ta = (uint32_t)(tbase[g] - tile_lo), tb = (uint32_t)(tbase[g + 1] - tile_lo), nt = tb - ta;
    const GbRule r(n, nt, target, split_target, epc);
    const uint32_t s0 = sofs[(uint32_t)gl * kSpBuckets] + grank[gb];
    for (uint32_t i = threadIdx.x; i < r.nsplit; i += 64u) {
        const uint32_t x = i * r.ts;
        uint32_t at = s0;
        for (uint32_t u = 0; u < V; ++u) {
            const uint32_t vu = tv[u] & 0xFFFFu, cu = tv[u] >> 16;
            const uint32_t nsu = (nt + vu - 1u) / vu, q = x / vu, rm = x - q * vu;
            at += cu * min(nsu, q + (rm ? 1u : 0u));
            if (vu < r.ts && rm == 0u && q < nsu) at += cu;
        }
        const uint32_t t = ta + x;
        sitems[at] = SplitItem{b, t, min(t + r.ts, tb), r.np, (uint32_t)gb, r.per, cofs[gb], 0u};
    }
    for (uint32_t p = threadIdx.x; p < r.np; p += 64u)
        citems[cofs[gb] + p] = CountItem{(uint32_t)g, b, p, r.np, (uint32_t)gb, n};
}

// Output stores of the count kernel (48 GB per config-5 step, never read back by the kernel): plain
// stores, which the L2 completes into full lines (48.0 GB written).  Non-temporal ones sent each wave
// run's partial 128-byte lines to HBM unmerged: 55.7 GB, count 16.5-16.7 vs 14.6 ms (profiles/r04/r04n).
template <typename T>
__device__ __forceinline__ void out_store(T* p, T v) {
    *p = v;
}

// Count work item: deduplication by a counting sort on 13 bits of the key.  The keys of pass p
// of a bucket are the residues r with floor(r * np / 2^R) = p, a contiguous range; 13 middle
// bits of the residue (bin_of) spread them over 8192 bins of about one key each (8192 keys per
// item).  Equal keys share a bin, so after a counting sort (histogram, scan, scatter: one LDS
// atomic per key per pass over the keys, no
// probing and no per-lane tail) every distinct key is resolved by comparing the few keys of its
// bin.  A bin of more than BIG keys (a repeated k-mer) goes through a small LDS hash table
// instead, so repeats cost what they cost the hash kernel before.
// k_sp_count's `sorted` / `spos` and `hist` are stored with their 16-byte slots XOR-swizzled:
// slot c lives at c ^ ((c >> 4) & 3).  A ds_read_b128 is serviced in lane groups of 16 (e.g.
// lanes 0-3, 12-15, 20-27) whose lane numbers are distinct mod 16; a thread reading slot 4t + q
// (its consecutive keys or bins, t = its thread) then hits 16 distinct slots of a 256-byte bank
// row instead of 4 (a 4-way conflict unswizzled).  An aligned run of 16 slots is permuted within
// itself, so lane-consecutive reads keep one bank per lane.  EPS = elements per slot.
__device__ __forceinline__ uint32_t swz_slot(uint32_t c) { return c ^ ((c >> 4) & 3u); }
template <int EPS>
__device__ __forceinline__ uint32_t swz(uint32_t a) {
    return a ^ ((((a / (uint32_t)EPS) >> 4) & 3u) * (uint32_t)EPS);
}
__device__ __forceinline__ uint32_t swzh_slot(uint32_t c) { return c ^ ((c >> 4) & 3u); }
__device__ __forceinline__ uint32_t swzh(uint32_t a) { return a ^ (((a >> 6) & 3u) << 2); }

constexpr int kBinBits = 13, kBins = 1 << kBinBits;
constexpr int kBig = 32;        // positions: keys of a bin resolved by comparison (byte counts)
constexpr int kBigN = 14;        // no positions: the same, counts kept as nibbles
constexpr int kHSlots = 1024;    // hash table of the big bins
constexpr int kMaxBig = 256;     // big bins of one item (more: the item goes to the fallback)
constexpr int kCntThreads = 512; // two count workgroups per CU (~78 KiB of LDS each) hide each
                                 // other's load latency

#ifdef KMH_EXPERIMENTS
__device__ unsigned long long g_sp_prof[16];   // KMH_SP_PROF: per-phase clocks of k_sp_count
#define KMH_PT(i) if (lane == 0) { const unsigned long long t_ = clock64(); pt[i] += t_ - tl; tl = t_; }
#else
#define KMH_PT(i)
#endif

// Persistent, two workgroups per CU; XCD x (= blockIdx % 8) takes a contiguous run of the
// items and its workgroups stride through it.  Software-pipelined over items, so that no global
// latency is waited for inside an item: the keys of item i + 1 are loaded into registers right
// after item i's scatter (its own keys are dead then) and land during item i's emission; they
// are counted into the histogram (cleared behind the emission) before item i's output stores
// are issued, so the wait for them never queues behind those stores (loads and stores share one
// in-order counter); descriptors (with the item's key count, pfill) are loaded two items ahead;
// the output base (one global atomic per item) returns during the next item's histogram.  Item
// i's keys are re-read from `sorted` for its stores (still intact: item i + 1's scatter comes
// after them), so a lane holds only the next item's keys and its emission results across the
// phases.
//
// Emission.  Without positions (config 5), thread t resolves the KPL consecutive sorted positions
// KPL t .. KPL t + KPL - 1 from registers: it reads them and the 4 positions on each side with
// 16-byte LDS reads; a key is first iff none of the 3 positions before it holds the same key, its
// count is 1 + the equal keys among the 3 after it -- complete whenever its bin lies within those
// +-3 positions, i.e. the keys 4 before and 4 after it fall in other bins (binned from the same
// registers).  The few positions whose bin reaches further (bins of 5+ keys) or that sit within 4
// of the item's ends are resolved by the exact bin range (hist).  Each position's result, 0 (not
// first) or its count (<= kBigN), goes to a 4-bit LDS table that the stores (lane-consecutive
// positions, coalesced) read.  With positions (the drop-in: every k-mer's first position is the
// minimum over its copies), positions are resolved lane-consecutively by four rounds of reads of
// the bin's keys 0..3 (clamped) and a loop for larger bins.
//
// ORD (kmh_count_sparse_sorted_dev, the column-sharded matrix): every genome's rows in code order.
// Item i writes at item_off[i] (the keys of the genome's earlier items, in (bucket, pass) order:
// passes ascend with the residue), so the items of a genome follow each other in code order with
// no atomic; the bin is the top 13 bits of the key's offset in its pass (monotone in the key), a
// bin's keys are sorted in LDS after the scatter (thread t sorts bins 16t .. 16t + 15, ~1 key
// each), and wave w stores the positions [w C / 8, (w + 1) C / 8) in order.  The item's range
// holds its keys; the slots past its distinct k-mers are padding (count 0, code = the pass's last
// code, so the row stays non-decreasing).  An item with a bin of more than kBigN keys fails (the
// sorted fallback recounts it).
template <typename E, bool POS, bool ORD, bool CNT = false>
__global__ __launch_bounds__(kCntThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_sp_count(
    const E* __restrict__ split, const uint32_t* __restrict__ opos, const uint32_t* __restrict__ pfill,
    const CountItem* __restrict__ items, uint32_t nitems, int R, uint32_t limit,
    const uint64_t* __restrict__ out_off, uint64_t* __restrict__ codes,
    uint32_t* __restrict__ counts, uint32_t* __restrict__ firsts, unsigned long long* __restrict__ nk,
    const uint32_t* __restrict__ gb_fail, uint32_t* __restrict__ failed) {
    static_assert(!(POS && ORD), "code order without positions only");
    static_assert(!CNT || ORD, "the distinct-count pass belongs to the ordered count");
    // CNT (the ordered count's first pass): no order, no stores -- each item's distinct k-mers go
    // to firsts[item] (unused without positions), so that the second pass writes compact rows
    // ORD: out_off holds the output base of every item (item_off), not of every genome, and nk
    // receives every genome's distinct k-mers (its row length is written by k_sp_item_offsets)
    constexpr int NT = kCntThreads, kNW = NT / 64, C = Cnt<E, POS>::CAP, BPT = kBins / NT, HPT = kHSlots / NT;
    constexpr int BQ = BPT / 4;   // uint4 words of a thread's bins
    constexpr bool WIDE = sizeof(E) == 8;
    constexpr int KPL = C / NT;          // keys per lane
    constexpr int ECW = (KPL + 3) / 4;   // POS: words of a lane's emission counts, 8 bits each (<= kBig)
    constexpr int BIG = POS ? kBig : kBigN;
    constexpr int EPC = epc<E>();        // keys per 16-byte LDS read
    constexpr int NW = KPL + 8;          // !POS: a thread's keys and the 4 on each side
    static_assert(BPT % 4 == 0 && HPT >= 1 && C % NT == 0 && KPL <= 32 && kBig < 256, "thread layout");
    static_assert(POS || (KPL == 8 || KPL == 16), "nibble layout: 8 or 16 positions per thread");
    static_assert(KPL % EPC == 0 && 4 % EPC == 0, "16-byte reads of a thread's keys");
    // + 32 dummy counters and a 64-entry scratch tail: a lane past its keys adds to a dummy and
    // scatters into the tail, so no exec-mask branch surrounds the atomics of a key
    __shared__ __attribute__((aligned(16))) uint32_t hist[kBins + 32];
    __shared__ __attribute__((aligned(16))) E sorted[C + 64];
    __shared__ uint32_t spos[POS ? C + 64 : 1];     // positions of sorted[] (POS)
    __shared__ uint32_t hmin[POS ? kHSlots : 1];    // first position of each big-bin slot (POS)
    __shared__ unsigned long long htab[kHSlots];
    __shared__ uint32_t bigl[kMaxBig];
    __shared__ uint32_t wtot[kNW];
    __shared__ uint32_t scnt[kNW];                  // !POS: keys each storing wave emits
    __shared__ __attribute__((aligned(16))) uint32_t nib[POS ? 4 : C / 8];   // !POS: 4 bits per position
    __shared__ uint32_t nbig, bad;
    __shared__ unsigned long long obase;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // hash slot = key << CB | count (CB = 32 for u32 residues, 64 - R for u64: a count that
    // would overflow its field fails the item)
    const int CB = WIDE ? 64 - R : 32;
    const unsigned long long CM = (1ull << CB) - 1ull;
    const uint32_t cap = limit < (uint32_t)C ? limit : (uint32_t)C;

    const uint32_t x = blockIdx.x % 8u, nwg = gridDim.x;
    const uint32_t nwx = (nwg - x + 7u) / 8u;                      // workgroups on XCD x
    const uint32_t iq = nitems / 8u, irem = nitems % 8u;
    const uint32_t xa = x * iq + (x < irem ? x : irem), xb = xa + iq + (x < irem ? 1u : 0u);
    uint32_t item = xa + blockIdx.x / 8u;
    if (item >= xb) return;   // whole workgroup

    uint4* h4 = reinterpret_cast<uint4*>(hist);
    auto zero_bins = [&] {
#pragma unroll
        for (int q = 0; q < BQ; ++q) h4[q * NT + tid] = make_uint4(0u, 0u, 0u, 0u);
    };
    zero_bins();
#pragma unroll
    for (int q = 0; q < HPT; ++q) htab[q * NT + tid] = 0ull;
    if constexpr (POS) {
#pragma unroll
        for (int q = 0; q < HPT; ++q) hmin[q * NT + tid] = 0xFFFFFFFFu;
    }
    if (tid == 0) nbig = bad = 0u;
    if (tid < kNW) scnt[tid] = 0u;

    // bin = 13 bits of the residue, bits [s, s + 13) with s = R - ceil(log2 np) - 16 (>= 0): one
    // bit-field extract at a per-item scalar shift.  The counting sort needs only that equal keys
    // share a bin and that a pass's keys spread evenly.  A pass is a contiguous residue range of
    // 2^R / np >= 2^(R - ceil(log2 np)) values, i.e. at least 8 periods of the field (<= 12.5 %
    // uneven), and the field stays clear of the residue's lowest bits: a canonical code is <= its
    // reverse complement, so its last bases are constrained by its first ones (the bucket), and
    // the low 13 bits put ~7x more keys into bins of 5+ (bins >= 5 per item: 122 vs 18 in a 50 Mbp
    // simulation; the lowest-bits version ran config 5's count at 145 ms instead of 16).  The top 13
    // bits of (r * np) mod 2^R (a 32-bit multiply) were no faster, and bimodal run to run (r04k, r04l).
    // ORD: the top 13 bits of r's offset in its pass, (r * np) mod 2^R (monotone within a pass).
    auto bin_of = [&](E r, uint32_t np) -> uint32_t {
        if constexpr (ORD) {
            if constexpr (sizeof(E) == 4) return ((uint32_t)r << (32 - R)) * np >> (32 - kBinBits);
            else return (uint32_t)((((uint64_t)r << (64 - R)) * (uint64_t)np) >> (64 - kBinBits));
        }
        const int lg = np > 1u ? 32 - __builtin_clz(np - 1u) : 0;   // (scalar)
        const int sh = R - lg - 16 > 0 ? R - lg - 16 : 0;
        if constexpr (sizeof(E) == 4) return __builtin_amdgcn_ubfe((uint32_t)r, (uint32_t)sh, (uint32_t)kBinBits);
        else return (uint32_t)((uint64_t)r >> sh) & (uint32_t)(kBins - 1);
    };

    // An item as loaded: its descriptor, the gb_fail flag of its bucket (a pass of a bucket whose
    // split overflowed is left to the fallback: it counts as an item without keys) and its key
    // count (the fill counter the split items appended to).  In the loop, the descriptor of the
    // item three ahead and the flag and count of the item two ahead are VECTOR loads issued behind
    // the next item's keys and read (readfirstlane) after those keys have landed (vload).
    struct Desc {
        CountItem c;
        uint32_t skip, n, idx;
    };
    auto load_desc = [&](uint32_t i) {   // (prologue only: scalar loads)
        Desc d;
        d.c = items[i];
        d.skip = gb_fail[d.c.gb];
        d.n = pfill[i];
        d.idx = i;
        return d;
    };
    static_assert(sizeof(CountItem) == 24, "descriptor as three 8-byte loads");
    struct RawItem {
        uint64_t a, b, c;
    };
    auto vload_item = [&](uint32_t i) {
        const uint64_t* p = reinterpret_cast<const uint64_t*>(items + i);
        return RawItem{vload(p), vload(p + 1), vload(p + 2)};
    };
    auto item_of = [&](const RawItem& r) {
        return CountItem{rfl((uint32_t)r.a), rfl((uint32_t)(r.a >> 32)), rfl((uint32_t)r.b),
                         rfl((uint32_t)(r.b >> 32)), rfl((uint32_t)r.c), rfl((uint32_t)(r.c >> 32))};
    };
    auto keys_of = [&](const Desc& d) -> uint32_t { return d.skip ? 0u : d.n; };

    // Issues the loads of an item's keys into kr / kp (wave w takes the keys [n w / 8, n (w + 1) / 8)
    // of the region, 64 consecutive ones per register: coalesced, all in flight, nobody waits for
    // them here).  Lanes past the share (and an item over capacity, whose keys the fallback counts)
    // load entry 0 of the region, which exists.
    //   The loads are not clamped: a wave's share starts at ea <= 7 C / 8 and its KPL * 64 = C / 8
    //   loads stay inside the item's own region [0, C), so one lane offset + immediate offsets
    //   address them all; a lane's valid keys are the prefix u < kn.
    auto issue_keys = [&](const Desc& d, E (&kr)[KPL], uint32_t (&kp)[POS ? KPL : 1], uint32_t& kn) {
        static_assert(KPL * 64 * kNW == C, "a wave's loads stay in the region");
        const uint32_t n = keys_of(d);
        const uint32_t m = n <= (uint32_t)C ? n : 0u;
        const uint32_t ea = m * (uint32_t)wave / kNW, eb = m * (uint32_t)(wave + 1) / kNW;
        const uint64_t base = (uint64_t)d.idx * C + ea;   // (uniform)
        const E* const kb = split + base;
        const uint32_t span = eb - ea;
        kn = span > (uint32_t)lane ? min((span - (uint32_t)lane + 63u) / 64u, (uint32_t)KPL) : 0u;
#pragma unroll
        for (int u = 0; u < KPL; ++u) {
            const uint32_t e = 64u * (uint32_t)u + (uint32_t)lane;
            kr[u] = kb[e];
            if constexpr (POS) kp[u] = opos[base + e];
        }
    };

    // the histogram of an item, from the registers
    const uint32_t kDummy = (uint32_t)kBins + (uint32_t)(lane & 31);
    E kr[KPL];
    uint32_t kp[POS ? KPL : 1];
    uint32_t kn = 0u;   // valid keys of this lane (a prefix of kr)
    auto count_keys = [&](const Desc& d) {
#pragma unroll
        for (int u = 0; u < KPL; ++u) atomicAdd(&hist[swzh((uint32_t)u < kn ? bin_of(kr[u], d.c.np) : kDummy)], 1u);
    };

    // makes the wave wait for the loads into kr / kp on every path (the compiler waits before
    // an asm statement that reads a register whose load is in flight)
    auto landed_keys = [&] {
#pragma unroll
        for (int u = 0; u < KPL; ++u) {
            asm volatile("" : "+v"(kr[u]));
            if constexpr (POS) asm volatile("" : "+v"(kp[u]));
        }
    };

    // prologue: descriptors of the first three items and the output base of the first, keys and
    // histogram of the first
    Desc cur = load_desc(item);
    uint32_t nitem = item + nwx;
    bool has_n = nitem < xb;
    Desc nxt = load_desc(has_n ? nitem : item);
    uint32_t nnitem = nitem + nwx;
    bool has_nn = has_n && nnitem < xb;
    Desc nn = load_desc(has_nn ? nnitem : item);
    uint64_t obo = ORD ? out_off[item] : out_off[cur.c.g];
    issue_keys(cur, kr, kp, kn);
    lds_barrier();   // cleared state visible
    count_keys(cur);
    landed_keys();
    lds_barrier();
#ifdef KMH_EXPERIMENTS
    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tl = clock64();
#endif

    // Every branch on item data below is workgroup-uniform (descriptor fields, LDS values read
    // after a barrier, or wave totals), so all threads meet the same barriers.
    for (;;) {
        const uint32_t np = cur.c.np;
        const uint32_t ntot = keys_of(cur);
        const bool over = ntot > (uint32_t)C;   // more keys than the staging holds: fallback
        // 1. exclusive scan: thread t owns bins 16t .. 16t + 15; bins of more than BIG keys are
        //    listed; bin b's counter becomes start | start << 16.  2. scatter: the returning add
        //    of 1 << 16 hands each key its slot, so hist[b] ends as start | end << 16 (one read
        //    gives a bin's range; starts and ends <= C < 2^16)
        if (!over) {
            uint32_t v[BPT];
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
                const uint4 a = h4[swzh_slot(BQ * tid + q)];
                v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
            }
            uint32_t tsum = 0u;
#pragma unroll
            for (int i = 0; i < BPT; ++i) tsum += v[i];
            const uint32_t incl = scan64(tsum);
            if (lane == 63) wtot[wave] = incl;
#pragma unroll
            for (int i = 0; i < BPT; ++i) {
                if (v[i] > (uint32_t)BIG) {
                    const uint32_t at = atomicAdd(&nbig, 1u);
                    if (at < (uint32_t)kMaxBig) bigl[at] = (uint32_t)(BPT * tid + i);
                }
            }
            lds_barrier();
            uint32_t st = incl - tsum;
            for (int w = 0; w < wave; ++w) st += wtot[w];
            {
                uint32_t o[BPT];
#pragma unroll
                for (int i = 0; i < BPT; ++i) {
                    o[i] = st;
                    st += v[i];
                }
#pragma unroll
                for (int q = 0; q < BQ; ++q)
                    h4[swzh_slot(BQ * tid + q)] = make_uint4(o[4 * q] * 0x10001u, o[4 * q + 1] * 0x10001u, o[4 * q + 2] * 0x10001u,
                                                  o[4 * q + 3] * 0x10001u);
            }
            lds_barrier();
            KMH_PT(0)
            // all the returning adds first, then the stores (a store right behind its add waited
            // for each add in turn)
            uint32_t slot[KPL];
#pragma unroll
            for (int u = 0; u < KPL; ++u)
                slot[u] = atomicAdd(&hist[swzh((uint32_t)u < kn ? bin_of(kr[u], np) : kDummy)], 0x10000u);
#pragma unroll
            for (int u = 0; u < KPL; ++u) {
                const uint32_t at = swz<EPC>((uint32_t)u < kn ? slot[u] >> 16 : (uint32_t)C + (uint32_t)lane);
                sorted[at] = kr[u];
                if constexpr (POS) spos[at] = kp[u];
            }
            lds_barrier();
            if constexpr (ORD && !CNT) {
                // each bin's keys in ascending order.  ~76 % of the bins hold 0 or 1 key, so each
                // wave lists its threads' bins of 2..BIG keys (~250 of its 1024) in LDS (the hash
                // table's space: ORD never hashes) and its lanes take them 64 at a time: bins of up
                // to 4 keys by a sorting network in registers (four reads clamped into the bin, the
                // missing keys as the largest value), of 5..8 by an 8-key network, larger ones (~1e-5
                // of the bins) by insertion.  (Sorting every bin slot of every thread, empty or not,
                // cost 13.7 of the count's 31.8 Mcyc per wave; an insertion sort per bin before that
                // was a chain of dependent LDS round trips per bin slot, and so was insertion for the
                // ~4 bins of 5..8 keys per wave and item, holding up a whole round of its wave.)  A
                // wave whose list would overflow sorts its bins in place.
                constexpr E kTop = ~(E)0;
                auto cswap = [](E& a, E& b) {
                    const E lo = a < b ? a : b, hi = a < b ? b : a;
                    a = lo;
                    b = hi;
                };
                auto sort_bin = [&](uint32_t bs, uint32_t be) {   // one lane, one bin of 2..BIG keys
                    const uint32_t n = be - bs;
                    if (n <= 4u) {
                        E kv[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const uint32_t y = bs + (uint32_t)t;
                            kv[t] = (uint32_t)t < n ? sorted[swz<EPC>(y < be ? y : bs)] : kTop;
                        }
                        cswap(kv[0], kv[1]);
                        cswap(kv[2], kv[3]);
                        cswap(kv[0], kv[2]);
                        cswap(kv[1], kv[3]);
                        cswap(kv[1], kv[2]);
                        sorted[swz<EPC>(bs)] = kv[0];
                        sorted[swz<EPC>(bs + 1u)] = kv[1];
                        if (n > 2u) sorted[swz<EPC>(bs + 2u)] = kv[2];
                        if (n > 3u) sorted[swz<EPC>(bs + 3u)] = kv[3];
                    } else if (n <= 8u) {   // (Batcher's 19-comparator network: no chain of LDS round trips)
                        E kv[8];
#pragma unroll
                        for (int t = 0; t < 8; ++t) {
                            const uint32_t y = bs + (uint32_t)t;
                            kv[t] = (uint32_t)t < n ? sorted[swz<EPC>(y < be ? y : bs)] : kTop;
                        }
                        constexpr int net[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6},
                                                    {5, 7}, {1, 2}, {5, 6}, {0, 4}, {3, 7}, {1, 5}, {2, 6},
                                                    {1, 4}, {3, 6}, {2, 4}, {3, 5}, {3, 4}};
#pragma unroll
                        for (int c = 0; c < 19; ++c) cswap(kv[net[c][0]], kv[net[c][1]]);
#pragma unroll
                        for (int t = 0; t < 8; ++t)
                            if ((uint32_t)t < n) sorted[swz<EPC>(bs + (uint32_t)t)] = kv[t];
                    } else {
                        for (uint32_t x = bs + 1u; x < be; ++x) {
                            const E key = sorted[swz<EPC>(x)];
                            uint32_t y = x;
                            while (y > bs) {
                                const E o = sorted[swz<EPC>(y - 1u)];
                                if (o <= key) break;
                                sorted[swz<EPC>(y)] = o;
                                --y;
                            }
                            sorted[swz<EPC>(y)] = key;
                        }
                    }
                };
                constexpr uint32_t kList = (uint32_t)(kHSlots * sizeof(unsigned long long) / 2u / kNW);   // u16 per wave
                uint16_t* const lst = reinterpret_cast<uint16_t*>(htab) + (uint32_t)wave * kList;
                // (the bin ranges are read twice rather than held: 16 more registers spilled the
                // u64 variant)
                auto bin_range = [&](int q, int i) {
                    const uint4 rq = h4[swzh_slot(BQ * tid + q)];
                    return i == 0 ? rq.x : (i == 1 ? rq.y : (i == 2 ? rq.z : rq.w));
                };
                uint32_t need = 0u;
#pragma unroll
                for (int q = 0; q < BQ; ++q)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint32_t rg = bin_range(q, i), n = (rg >> 16) - (rg & 0xFFFFu);
                        need += (n >= 2u && n <= (uint32_t)BIG) ? 1u : 0u;
                    }
                const uint32_t incl = scan64(need);
                const uint32_t wtotal = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                if (wtotal <= kList) {   // (wave-uniform)
                    uint32_t at = incl - need;
#pragma unroll
                    for (int q = 0; q < BQ; ++q)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t rg = bin_range(q, i), n = (rg >> 16) - (rg & 0xFFFFu);
                            if (n >= 2u && n <= (uint32_t)BIG) lst[at++] = (uint16_t)(BPT * tid + 4 * q + i);
                        }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    for (uint32_t x = (uint32_t)lane; x < wtotal; x += 64u) {
                        const uint32_t hb = hist[swzh((uint32_t)lst[x])];
                        sort_bin(hb & 0xFFFFu, hb >> 16);
                    }
                } else {
                    for (int q = 0; q < BQ; ++q)
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t rg = bin_range(q, i), bs = rg & 0xFFFFu, be = rg >> 16;
                            if (be - bs >= 2u && be - bs <= (uint32_t)BIG) sort_bin(bs, be);
                        }
                }
                lds_barrier();
            }
        }
        KMH_PT(1)

        // 3. this item's keys are dead: the next item's keys load behind this item's emission,
        //    the descriptor after that behind two items
        if (has_n) issue_keys(nxt, kr, kp, kn);
        const uint32_t nnnitem = nnitem + nwx;
        const bool has_nnn = has_nn && nnnitem < xb;

        KMH_PT(2)

        // 4. big bins: their keys into the hash table (linear probing, CAS(empty -> key|1), +1
        //    on a slot holding the key)
        const uint32_t nb = over ? 0u : nbig;
        if (nb) {
            if (ORD || nb > (uint32_t)kMaxBig) {   // (ORD: a big bin's keys would leave code order)
                if (tid == 0) bad = 1u;
            } else {
                for (uint32_t xb2 = 0; xb2 < nb; ++xb2) {
                    const uint32_t b = bigl[xb2];
                    const uint32_t hb = hist[swzh(b)], s = hb & 0xFFFFu, e = hb >> 16;
                    for (uint32_t i = s + (uint32_t)tid; i < e; i += NT) {
                        const E key = sorted[swz<EPC>(i)];
                        uint32_t h = (uint32_t)key ^ (uint32_t)((uint64_t)key >> 29) * 0x9E3779B1u;
                        h = (uint32_t)__umul24(h ^ (h >> 15), 0x9E3779u) >> (32 - 10);
                        for (uint32_t probe = 0;; ++probe) {
                            if (probe == (uint32_t)kHSlots) {
                                bad = 1u;
                                break;
                            }
                            unsigned long long* slot = &htab[h];
                            const unsigned long long old = atomicCAS(slot, 0ull, ((unsigned long long)key << CB) | 1ull);
                            if (old == 0ull) {
                                if constexpr (POS) atomicMin(&hmin[h], spos[swz<EPC>(i)]);
                                break;
                            }
                            if ((E)(old >> CB) == key) {
                                const unsigned long long prev = atomicAdd(slot, 1ull);
                                if (WIDE && (prev & CM) == CM) bad = 1u;   // count field full
                                if constexpr (POS) atomicMin(&hmin[h], spos[swz<EPC>(i)]);
                                break;
                            }
                            h = (h + 1u) & (uint32_t)(kHSlots - 1);
                        }
                    }
                }
            }
            lds_barrier();
        }

        // 5. emission
        uint32_t fm = 0u;   // POS: bit j: position j * NT + tid is emitted
        uint32_t ecw[ECW];
        uint32_t ef[POS ? KPL : 1];   // first position of the key (POS): the minimum over its bin's copies
#pragma unroll
        for (int q = 0; q < ECW; ++q) ecw[q] = 0u;
        uint32_t wmine = 0u;   // POS: the wave's emitted keys
        if constexpr (!POS) {
            if (!over) {
                // this thread's positions P0 .. P0 + KPL - 1 and the 4 on each side: w[j] = position
                // P0 - 4 + j (thread 0's head and the last threads' tail read real but unrelated
                // entries; the positions they could mislead are resolved by range below)
                const uint32_t P0 = (uint32_t)(KPL * tid);
                const uint4* s4 = reinterpret_cast<const uint4*>(sorted);
                E w[NW];
                {
                    const uint32_t hq = tid ? (P0 - 4u) / EPC : 0u;
#pragma unroll
                    for (int q = 0; q < 4 / EPC; ++q) {
                        const uint4 c = s4[swz_slot(hq + q)];
#pragma unroll
                        for (int i = 0; i < EPC; ++i) w[EPC * q + i] = lane_of<E>(c, i);
                    }
#pragma unroll
                    for (int q = 0; q < KPL / EPC + 4 / EPC; ++q) {
                        const uint4 c = s4[swz_slot(P0 / EPC + q)];
#pragma unroll
                        for (int i = 0; i < EPC; ++i) w[4 + EPC * q + i] = lane_of<E>(c, i);
                    }
                }
                uint32_t bn[NW];
#pragma unroll
                for (int j = 0; j < NW; ++j) bn[j] = bin_of(w[j], np);
                // valid positions u < rem; positions within 4 of either end of the item are resolved
                // by range (their neighbours outside [0, ntot) hold unrelated entries)
                const int rem = (int)ntot - (int)P0;
                uint32_t valid = rem >= KPL ? (KPL == 32 ? 0xFFFFFFFFu : (1u << KPL) - 1u)
                                            : (rem > 0 ? (1u << rem) - 1u : 0u);
                uint32_t slow = tid == 0 ? 0xFu : 0u;
                if (rem < KPL + 4) slow |= valid & ~(rem > 4 ? (1u << (rem - 4)) - 1u : 0u);
                uint64_t nv = 0ull;   // 4 bits per position
#pragma unroll
                for (int u = 0; u < KPL; ++u) {
                    const E k = w[u + 4];
                    const uint32_t bk = bn[u + 4];
                    const bool dup = (w[u + 3] == k) | (w[u + 2] == k) | (w[u + 1] == k);
                    const uint32_t c = 1u + (uint32_t)(w[u + 5] == k) + (uint32_t)(w[u + 6] == k) +
                                       (uint32_t)(w[u + 7] == k);
                    slow |= (uint32_t)((bn[u] == bk) | (bn[u + 8] == bk)) << u;
                    nv |= (uint64_t)(dup ? 0u : c) << (4 * u);
                }
                slow &= valid;
                // positions whose bin reaches past +-3 (bins of 5+ keys), or near the item's ends:
                // the bin's exact range [bs, be) from hist (start | end << 16)
                while (slow) {
                    const uint32_t u = (uint32_t)__builtin_ctz(slow);
                    slow &= slow - 1u;
                    const uint32_t i = P0 + u;
                    E k = w[4];
                    uint32_t bk = bn[4];
#pragma unroll
                    for (int q = 1; q < KPL; ++q) {   // (a select chain, not a dynamic register index)
                        k = u == (uint32_t)q ? w[q + 4] : k;
                        bk = u == (uint32_t)q ? bn[q + 4] : bk;
                    }
                    const uint32_t hb = hist[swzh(bk)], bs = hb & 0xFFFFu, be = hb >> 16;
                    uint32_t c = 0u;
                    if (be - bs <= (uint32_t)BIG) {   // (bigger bins: emitted from the hash table)
                        // the bin's keys, four reads in flight at a time (addresses clamped into the bin)
                        bool first = true;
                        c = 1u;
                        for (uint32_t y0 = bs; y0 < be; y0 += 4u) {
                            E o[4];
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                const uint32_t y = y0 + (uint32_t)t;
                                o[t] = sorted[swz<EPC>(y < be ? y : bs)];
                            }
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                const uint32_t y = y0 + (uint32_t)t;
                                const bool eq = y < be && y != i && o[t] == k;
                                first = first && !(eq && y < i);
                                c += (uint32_t)(eq && y > i);
                            }
                        }
                        c = first ? c : 0u;
                    }
                    nv = (nv & ~(0xFull << (4u * u))) | ((uint64_t)c << (4u * u));
                }
                // nibbles of invalid positions are 0 (dup / c of unrelated entries cleared)
                uint64_t vm = 0ull;
#pragma unroll
                for (int u = 0; u < KPL; ++u) vm |= (uint64_t)((valid >> u) & 1u) * (0xFull << (4 * u));
                nv &= vm;
                if constexpr (KPL == 16) reinterpret_cast<uint2*>(nib)[tid] = make_uint2((uint32_t)nv, (uint32_t)(nv >> 32));
                else nib[tid] = (uint32_t)nv;
                // the storing wave of these positions: position P0 + u is stored by lane
                // (P0 + u) % NT, i.e. wave (P0 % NT) / 64 for every u (KPL divides 64); ORD: wave
                // w stores the positions [w KPL 64, (w + 1) KPL 64) in order, i.e. its own threads'
                uint32_t e = 0u;
#pragma unroll
                for (int u = 0; u < KPL; ++u) e += (uint32_t)(((nv >> (4 * u)) & 0xFull) != 0ull);
                if (e) atomicAdd(&scnt[ORD ? (uint32_t)wave : (P0 % (uint32_t)NT) / 64u], e);
            }
        } else if (!over) {
            // In phases over a group of HB positions, so that every phase's LDS reads are
            // independent and issue back to back: (a) the keys, (b) their bins' ranges, (c) four
            // rounds of one read per position -- the bin's key t, at an address clamped into the
            // bin (most bins hold 1-3 keys), (d) bins of 5..kBig keys, rare, one by one.  Count of
            // position jj (1 + equal keys after it): byte jj % 4 of ecw[jj / 4]; first: bit jj of fm.
            constexpr int HB = KPL < 4 ? KPL : 4;
#pragma unroll
            for (int q = 0; q < ECW; ++q) ecw[q] = 0x01010101u;
#pragma unroll
            for (int h0 = 0; h0 < KPL; h0 += HB) {
                __builtin_amdgcn_sched_barrier(0);
                E key[HB];
                uint32_t rng[HB];   // bs | be << 16
#pragma unroll
                for (int x = 0; x < HB; ++x) {
                    const uint32_t i = (uint32_t)((h0 + x) * NT + tid);
                    key[x] = sorted[swz<EPC>(i < ntot ? i : 0u)];
                }
#pragma unroll
                for (int x = 0; x < HB; ++x) rng[x] = hist[swzh(bin_of(key[x], np))];
#pragma unroll
                for (int x = 0; x < HB; ++x) {
                    const int jj = h0 + x;
                    const uint32_t i = (uint32_t)(jj * NT + tid), bs = rng[x] & 0xFFFFu, be = rng[x] >> 16;
                    fm |= (uint32_t)(i < ntot && be - bs <= (uint32_t)kBig) << jj;
                    ef[jj] = spos[swz<EPC>(i < ntot ? i : 0u)];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    E o[HB];
#pragma unroll
                    for (int x = 0; x < HB; ++x) {
                        const uint32_t bs = rng[x] & 0xFFFFu, be = rng[x] >> 16, y = bs + (uint32_t)t;
                        o[x] = sorted[swz<EPC>(y < be ? y : bs)];
                    }
#pragma unroll
                    for (int x = 0; x < HB; ++x) {
                        const int jj = h0 + x;
                        const uint32_t i = (uint32_t)(jj * NT + tid), be = rng[x] >> 16, y = (rng[x] & 0xFFFFu) + (uint32_t)t;
                        const bool eq = y < be && o[x] == key[x];
                        fm &= ~((uint32_t)(eq && y < i) << jj);
                        ecw[jj / 4] += (uint32_t)(eq && y > i) << (8 * (jj % 4));
                        ef[jj] = (eq && y > i) ? min(ef[jj], spos[swz<EPC>(y)]) : ef[jj];
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int x = 0; x < HB; ++x) {
                    const int jj = h0 + x;
                    const uint32_t i = (uint32_t)(jj * NT + tid), bs = rng[x] & 0xFFFFu, be = rng[x] >> 16;
                    if (((fm >> jj) & 1u) && be - bs > 4u) {
                        bool first = true;
                        for (uint32_t y = bs + 4u; y < be; ++y) {
                            const E o = sorted[swz<EPC>(y)];
                            first = first && !(y < i && o == key[x]);
                            ecw[jj / 4] += (uint32_t)(y > i && o == key[x]) << (8 * (jj % 4));
                            ef[jj] = (y > i && o == key[x]) ? min(ef[jj], spos[swz<EPC>(y)]) : ef[jj];
                        }
                        fm &= ~((uint32_t)!first << jj);
                    }
                }
            }
#pragma unroll
            for (int jj = 0; jj < KPL; ++jj) wmine += (uint32_t)__popcll(__ballot((fm >> jj) & 1u));
        }
        if (!ORD && !over && nb) {   // the hash table's keys are stored by the wave of their slot
            uint32_t hk = 0u;
#pragma unroll
            for (int q = 0; q < HPT; ++q) hk += (uint32_t)__popcll(__ballot((htab[q * NT + tid] & CM) != 0ull));
            if constexpr (POS) wmine += hk;
            else if (lane == 0 && hk) atomicAdd(&scnt[wave], hk);
        }
        KMH_PT(3)
        if (POS && lane == 0) wtot[wave] = wmine;
        lds_barrier();   // (also: every read of hist, and of htab for the totals, is done)
        uint32_t before = 0u, used = 0u;
#pragma unroll
        for (int w = 0; w < kNW; ++w) {
            const uint32_t xw = POS ? wtot[w] : scnt[w];
            before += w < wave ? xw : 0u;
            used += xw;
        }
        const bool fail_item = over || bad != 0u || used > cap;   // uniform
        // (vector loads, read at step 6 once the next item's keys have landed; issued here, after
        // the emission, so that they hold no registers through it): the descriptor three items
        // ahead, the flag and count of the item two ahead, the output offset of the next item
        const RawItem raw_nnn = vload_item(has_nnn ? nnnitem : item);
        const uint32_t v_skip = vload(gb_fail + nn.c.gb), v_n = vload(pfill + nn.idx);
        const uint64_t v_obo = vload(out_off + (ORD ? nitem : nxt.c.g));
        // the output base: one atomic per item, returning during the next item's histogram
        // (its value is first used there: an add here would wait for it)
        unsigned long long ob = 0ull;
        if (tid == 0) {
            if (fail_item) {
                const uint32_t at = atomicAdd(&failed[0], 1u);
                failed[1 + at] = item;
            } else if (CNT) {
                firsts[item] = used;
            } else if (used) {   // (ORD: nk counts the distinct k-mers; the base is item_off)
                // (the address laundered through a VGPR: with a uniform address the compiler
                // rewrites the atomic into a wave reduction whose result is waited for at once)
                uint64_t pa = reinterpret_cast<uint64_t>(nk + cur.c.g);
                asm volatile("" : "+v"(pa));
                using g64 = __attribute__((address_space(1))) unsigned long long;   // global, not flat
                ob = __hip_atomic_fetch_add(reinterpret_cast<g64*>(pa), (unsigned long long)used, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        zero_bins();
        KMH_PT(4)
        lds_barrier();   // cleared bins visible; `bad` read by everybody; scnt read by everybody
        if constexpr (!POS)
            if (tid < kNW) scnt[tid] = 0u;   // (the next item's emission adds after two more barriers)

        // 6. the next item's histogram (the wait for its keys), before this item's stores
        if (has_n) count_keys(nxt);
        // Everything loaded so far has landed here, on every path: the next item's keys (counted
        // above, but only by the lanes that hold keys).  A load still in flight at the stores
        // below would be waited for behind them later (one in-order counter: vmcnt(0) at a
        // register copy or at the scatter).
        landed_keys();
        if (tid == 0) {
            obase = ORD ? obo : ob + obo;
            nbig = bad = 0u;
        }
        Desc nnn;
        nnn.c = item_of(raw_nnn);
        nnn.idx = has_nnn ? nnnitem : item;
        nnn.skip = nnn.n = 0u;   // (loaded one iteration from now, when it is nn)
        nn.skip = rfl(v_skip);
        nn.n = rfl(v_n);
        const uint64_t obo_n = rfl64(v_obo);
        KMH_PT(5)
        lds_barrier();

        // 7. this item's stores, compacted per wave with ballot + mbcnt so that they are
        //    coalesced; keys re-read from `sorted` (the next scatter comes after a barrier)
        if (!CNT && !fail_item && used) {   // uniform
            // the wave's output base, made scalar (readfirstlane): every store below is that base
            // plus a 32-bit byte offset (no 64-bit address arithmetic per key)
            const uint64_t at = rfl64(obase + before);
            uint64_t* const cw = codes + at;
            uint32_t* const nw = counts + at;
            const uint64_t hib = (uint64_t)cur.c.b << R;
            uint32_t run = 0u;
            const uint32_t stid = swz<EPC>((uint32_t)tid);
            constexpr int SB = KPL < 8 ? KPL : 8;   // keys re-read 8 at a time (one round trip)
#pragma unroll
            for (int j0 = 0; j0 < KPL; j0 += SB) {
                __builtin_amdgcn_sched_barrier(0);
                E sk[SB];
                uint32_t nc[SB];   // !POS: the position's nibble (0: not emitted, else its count)
#pragma unroll
                for (int x = 0; x < SB; ++x) {
                    if constexpr (ORD) {   // wave w's positions in order: w KPL 64 + 64 j + lane
                        const uint32_t i = (uint32_t)(wave * KPL * 64 + (j0 + x) * 64 + lane);
                        sk[x] = sorted[swz<EPC>(i)];
                        nc[x] = (nib[i >> 3] >> (4u * (i & 7u))) & 0xFu;
                    } else {
                        const uint32_t i = (uint32_t)((j0 + x) * NT + tid);
                        sk[x] = sorted[(uint32_t)((j0 + x) * NT) + stid];   // (= swz(i): NT is a multiple of 64 slots)
                        if constexpr (!POS) nc[x] = (nib[i >> 3] >> (4u * (i & 7u))) & 0xFu;
                    }
                }
#pragma unroll
                for (int x = 0; x < SB; ++x) {
                    const int jj = j0 + x;
                    bool f;
                    uint32_t cv;
                    if constexpr (POS) {
                        f = (fm >> jj) & 1u;
                        cv = (ecw[jj / 4] >> (8 * (jj % 4))) & 0xFFu;
                    } else {
                        f = nc[x] != 0u;
                        cv = nc[x];
                    }
                    const uint64_t m = __ballot(f);
                    if (f) {
                        const uint32_t ow = lane_rank(m, run);   // < C: offset within the wave's output
                        const uint64_t o = at + ow;
#if defined(KMH_EXPERIMENTS) && KMH_SP_OUT_EXP == 1
                        // what-if: a compact row (u32 residue + u8 count), same positions
                        out_store(reinterpret_cast<uint32_t*>(codes) + o, (uint32_t)sk[x]);
                        out_store(reinterpret_cast<uint8_t*>(counts) + o, (uint8_t)cv);
#elif defined(KMH_EXPERIMENTS) && KMH_SP_OUT_EXP == 2
                        // what-if: no output bytes at all (counts wrong; timing only)
                        if (sk[x] == (E)0x5A5A5A5Au && o == 0ull) codes[0] = hib + cv;
#else
                        out_store(at_byte(cw, 8u * ow), hib | (uint64_t)sk[x]);
                        out_store(at_byte(nw, 4u * ow), cv);
#endif
                        if constexpr (POS) firsts[o] = ef[jj];
                    }
                    run += (uint32_t)__popcll(m);
                }
            }
            if (!ORD && nb) {
#pragma unroll
                for (int q = 0; q < HPT; ++q) {
                    const unsigned long long hs = htab[q * NT + tid];
                    const bool f = (hs & CM) != 0ull;
                    const uint64_t m = __ballot(f);
                    if (f) {
                        const uint64_t o = at + run + lane_rank(m);
                        codes[o] = hib | (hs >> CB);
                        counts[o] = (uint32_t)(hs & CM);
                        if constexpr (POS) firsts[o] = hmin[q * NT + tid];
                    }
                    run += (uint32_t)__popcll(m);
                }
            }
        }
        if (nb) {   // cleared behind its last reads (this thread's); the next inserts follow barriers
#pragma unroll
            for (int q = 0; q < HPT; ++q) htab[q * NT + tid] = 0ull;
            if constexpr (POS) {
#pragma unroll
                for (int q = 0; q < HPT; ++q) hmin[q * NT + tid] = 0xFFFFFFFFu;
            }
        }
        KMH_PT(6)
        if (!has_n) break;
        item = nitem;
        cur = nxt;
        nitem = nnitem;
        has_n = has_nn;
        nxt = nn;
        nnitem = nnnitem;
        has_nn = has_nnn;
        nn = nnn;
        obo = obo_n;
    }
#ifdef KMH_EXPERIMENTS
    if (lane == 0)
        for (int i = 0; i < 8; ++i) atomicAdd(&g_sp_prof[i], pt[i]);
    if (tid == 0) atomicAdd(&g_sp_prof[8], 1ull);
#endif
}

// Fallback, step 1: the residues of bucket b of genome g whose pass is set in the bitmap
// `pmask` (np bits) -- every failed pass of the bucket at once -- and their positions, in any
// order.
template <typename E, bool POS>
__global__ __launch_bounds__(256) void k_sp_gather(const E* __restrict__ ent, const uint32_t* __restrict__ epos,
                                                   const uint16_t* __restrict__ toff, uint32_t ldt,
                                                   uint64_t ta, uint64_t tb, uint32_t b, const uint32_t* __restrict__ pmask,
                                                   uint32_t np, int R, E* __restrict__ out,
                                                   uint32_t* __restrict__ opos, uint32_t* __restrict__ n) {
    const uint64_t t = ta + (uint64_t)blockIdx.x;
    if (t >= tb) return;
    const uint32_t lo = toff[(uint64_t)b * ldt + t], hi = toff[(uint64_t)(b + 1) * ldt + t];
    for (uint32_t j = lo + threadIdx.x; j < hi; j += 256) {
        const uint64_t ix = t * (uint64_t)Sp<E, POS>::TILE + j;
        const E r = ent[ix];
        const uint32_t p = pass_of(r, np, R);
        if ((pmask[p >> 5] >> (p & 31u)) & 1u) {
            const uint32_t at = atomicAdd(n, 1u);
            out[at] = r;
            opos[at] = POS ? epos[ix] : at;   // without positions: any value (the sort needs one)
        }
    }
}

template <typename E>
__global__ __launch_bounds__(256) void k_sp_gather_by(const E* __restrict__ src, const uint32_t* __restrict__ idx,
                                                      uint32_t m, E* __restrict__ dst) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < m) dst[i] = src[idx[i]];
}

__global__ __launch_bounds__(256) void k_sp_iota(uint32_t* __restrict__ out, uint32_t m) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < m) out[i] = i;
}

// Fallback, step 3: append the runs of the sorted keys (count = run length, first position =
// the run's first value: keys were sorted stably after their positions) to genome g's output.
template <typename E, bool POS>
__global__ __launch_bounds__(256) void k_sp_append(const E* __restrict__ keys, const uint32_t* __restrict__ pos,
                                                   uint32_t m, const uint32_t* __restrict__ starts,
                                                   const uint32_t* __restrict__ nruns, uint64_t hib, uint64_t off,
                                                   unsigned long long* __restrict__ nk, uint64_t* __restrict__ codes,
                                                   uint32_t* __restrict__ counts, uint32_t* __restrict__ firsts) {
    __shared__ unsigned long long base;
    const uint32_t n = *nruns;
    if (threadIdx.x == 0) base = atomicAdd(nk, (unsigned long long)n);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < n; r += 256) {
        const uint32_t a = starts[r], e = r + 1 < n ? starts[r + 1] : m;
        codes[off + base + r] = hib | (uint64_t)keys[a];
        counts[off + base + r] = e - a;
        if constexpr (POS) firsts[off + base + r] = pos[a];
    }
}

// ORD: output base of every count item of a batch (items in (genome, bucket, pass) order) = the
// rows written so far (rowbase: earlier batches) + the distinct k-mers of the batch's earlier
// items, so every genome's row follows the previous genome's, and every genome's row length
// nk[g].  Three launches over chunks of kIoChunk items (one workgroup each; a single-workgroup
// version walked 512 items per thread with uncoalesced loads: 5 ms per config-5 batch): (1) chunk
// sums and the genomes' totals (nk, one atomic per wave when its items share a genome), (2) one
// workgroup scans the chunk sums from rowbase and advances rowbase, (3) every item's base.
constexpr int kIoPer = 16, kIoChunk = 256 * kIoPer;

__global__ __launch_bounds__(256) void k_sp_io_sums(const uint32_t* __restrict__ cnt,
                                                    const CountItem* __restrict__ items, uint32_t nci,
                                                    unsigned long long* __restrict__ csum,
                                                    unsigned long long* __restrict__ nk) {
    __shared__ unsigned long long ws[4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t a = blockIdx.x * (uint32_t)kIoChunk + threadIdx.x * (uint32_t)kIoPer;
    unsigned long long tot = 0ull, run = 0ull;
    uint32_t g = a < nci ? items[a].g : 0u;
    bool split = false;   // this thread's items span two genomes or more
    for (uint32_t j = 0; j < (uint32_t)kIoPer && a + j < nci; ++j) {
        const uint32_t i = a + j, gi = items[i].g;
        const unsigned long long v = cnt[i];
        if (gi != g) {
            atomicAdd(&nk[g], run);
            run = 0ull;
            g = gi;
            split = true;
        }
        run += v;
        tot += v;
    }
    // the last genome's run: one atomic per wave when every lane holds the same genome
    const uint32_t g0 = (uint32_t)__shfl(g, 0);
    const bool same = !__any(split || (a < nci && g != g0) || a >= nci);
    if (same) {
        unsigned long long r = run;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) r += __shfl_xor(r, d);
        if (lane == 0u) atomicAdd(&nk[g0], r);
    } else if (a < nci) {
        atomicAdd(&nk[g], run);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d);
    if (lane == 0u) ws[wave] = tot;
    __syncthreads();
    if (threadIdx.x == 0) csum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// One workgroup: csum[c] = *rowbase + the sums of the chunks before c; then *rowbase += all of them.
__global__ __launch_bounds__(1024) void k_sp_io_scan(unsigned long long* __restrict__ csum, uint32_t nch,
                                                     unsigned long long* __restrict__ rowbase) {
    __shared__ unsigned long long ws[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const unsigned long long base = *rowbase;
    const uint32_t per = (nch + 1023u) / 1024u, a = min(nch, tid * per), e = min(nch, a + per);
    unsigned long long s = 0ull;
    for (uint32_t i = a; i < e; ++i) s += csum[i];
    unsigned long long incl = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long x = __shfl_up(incl, d);
        if ((int)lane >= d) incl += x;
    }
    if (lane == 63u) ws[wave] = incl;
    __syncthreads();   // (every thread has read *rowbase)
    unsigned long long p = base + incl - s;
    for (uint32_t w = 0; w < wave; ++w) p += ws[w];
    for (uint32_t i = a; i < e; ++i) {
        const unsigned long long x = csum[i];
        csum[i] = p;
        p += x;
    }
    if (tid == 1023u) *rowbase = p;
}

__global__ __launch_bounds__(256) void k_sp_io_write(const uint32_t* __restrict__ cnt, uint32_t nci,
                                                     const unsigned long long* __restrict__ cpre,
                                                     uint64_t* __restrict__ item_off) {
    __shared__ unsigned long long ws[4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t a = blockIdx.x * (uint32_t)kIoChunk + threadIdx.x * (uint32_t)kIoPer;
    unsigned long long s = 0ull;
    for (uint32_t j = 0; j < (uint32_t)kIoPer && a + j < nci; ++j) s += cnt[a + j];
    unsigned long long incl = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long x = __shfl_up(incl, d);
        if ((int)lane >= d) incl += x;
    }
    if (lane == 63u) ws[wave] = incl;
    __syncthreads();
    unsigned long long p = cpre[blockIdx.x] + incl - s;
    for (uint32_t w = 0; w < wave; ++w) p += ws[w];
    for (uint32_t j = 0; j < (uint32_t)kIoPer && a + j < nci; ++j) {
        item_off[a + j] = p;
        p += cnt[a + j];
    }
}

// ORD fallback, step 3: the runs of the sorted keys of one (genome, bucket)'s failed passes (keys
// ascend, so their passes ascend too) into those passes' item ranges in order (count item of pass
// p: cbase + p).  item_n != nullptr: the count-only first pass -- each failed pass's runs (its
// distinct k-mers) into item_n[cbase + p], nothing written.
template <typename E>
__global__ __launch_bounds__(256) void k_sp_append_ord(const E* __restrict__ keys, uint32_t m,
                                                       const uint32_t* __restrict__ starts,
                                                       const uint32_t* __restrict__ nruns, const uint32_t* __restrict__ pmask,
                                                       uint32_t np, int R, uint64_t hib, uint32_t cbase,
                                                       const uint64_t* __restrict__ item_off, uint32_t* __restrict__ item_n,
                                                       uint64_t* __restrict__ codes, uint32_t* __restrict__ counts,
                                                       unsigned long long* __restrict__ ndist) {
    const uint32_t n = *nruns;
    auto run_pass = [&](uint32_t r) { return pass_of<E>(keys[starts[r]], np, R); };
    auto first_run = [&](uint32_t p) {   // the first run whose pass is >= p
        uint32_t lo = 0u, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2u;
            if (run_pass(mid) < p) lo = mid + 1u;
            else hi = mid;
        }
        return lo;
    };
    if (item_n) {
        for (uint32_t p = threadIdx.x; p < np; p += 256u)
            if ((pmask[p >> 5] >> (p & 31u)) & 1u) item_n[cbase + p] = first_run(p + 1u) - first_run(p);
        return;
    }
    if (threadIdx.x == 0) atomicAdd(ndist, (unsigned long long)n);
    for (uint32_t r = threadIdx.x; r < n; r += 256u) {
        const uint32_t a = starts[r], e = r + 1u < n ? starts[r + 1u] : m;
        const uint32_t p = run_pass(r);
        const uint64_t o = item_off[cbase + p] + (r - first_run(p));
        codes[o] = hib | (uint64_t)keys[a];
        counts[o] = e - a;
    }
}

void* carve(char*& p, size_t bytes) {
    void* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return r;
}

template <int K, int CANON, typename E, bool POS>
void launch_partition(unsigned tiles, unsigned grid, hipStream_t s, const uint8_t* seq, const GenomeMap& m,
                      E* ent, uint32_t* epos, uint16_t* toff, uint32_t ldt) {
    hipLaunchKernelGGL((k_sp_partition<K, CANON, E, POS>), dim3(grid), dim3(kSpThreads), 0, s, seq, m, ent,
                       epos, toff, ldt, (uint32_t)tiles);
}

template <int K, typename E, bool POS>
void partition_k(int canonical, unsigned tiles, unsigned grid, hipStream_t s, const uint8_t* seq,
                 const GenomeMap& m, E* ent, uint32_t* epos, uint16_t* toff, uint32_t ldt) {
    if (canonical) launch_partition<K, 1, E, POS>(tiles, grid, s, seq, m, ent, epos, toff, ldt);
    else launch_partition<K, 0, E, POS>(tiles, grid, s, seq, m, ent, epos, toff, ldt);
}

template <typename E, bool POS>
void launch_partition_k(int k, int canonical, unsigned tiles, unsigned grid, hipStream_t s, const uint8_t* seq,
                        const GenomeMap& m, E* ent, uint32_t* epos, uint16_t* toff, uint32_t ldt) {
#define KMH_PK(KK) case KK: partition_k<KK, E, POS>(canonical, tiles, grid, s, seq, m, ent, epos, toff, ldt); break;
    if constexpr (sizeof(E) == 4) {
        switch (k) { KMH_PK(13) KMH_PK(14) KMH_PK(15) KMH_PK(16) KMH_PK(17) KMH_PK(18) KMH_PK(19) KMH_PK(20)
                     default: partition_k<21, E, POS>(canonical, tiles, grid, s, seq, m, ent, epos, toff, ldt); break; }
    } else {
        switch (k) { KMH_PK(22) KMH_PK(23) KMH_PK(24) KMH_PK(25) KMH_PK(26) KMH_PK(27) KMH_PK(28) KMH_PK(29)
                     KMH_PK(30) KMH_PK(31)
                     default: partition_k<32, E, POS>(canonical, tiles, grid, s, seq, m, ent, epos, toff, ldt); break; }
    }
#undef KMH_PK
}

// Fallback for the failed passes `passes` of bucket b of genome g (n entries in the bucket):
// one gather of all of them (passes hold disjoint keys), sort (radix_sort_pairs: with positions,
// first by position and then stably by key, so a run's first entry holds its first position),
// runs, append.  Hand-written kernels throughout (kmh_sort.hip).
// ORD: item_off / pfill / cbase place the runs in code order (k_sp_append_ord) instead of appending.
template <typename E, bool POS, bool ORD>
int fallback_passes(Ctx* ctx, uint32_t g, uint32_t b, const std::vector<uint32_t>& passes, uint32_t np, uint32_t n,
                    const E* ent, const uint32_t* epos, const uint16_t* toff, uint32_t ldt, uint64_t ta, uint64_t tb,
                    int R, uint64_t out_off, unsigned long long* nk, uint64_t* codes, uint32_t* counts,
                    uint32_t* firsts, const uint64_t* item_off, uint32_t* item_n, uint32_t cbase, hipStream_t s) {
    const size_t ne = ((size_t)n * sizeof(E) + 255) & ~(size_t)255, n4 = ((size_t)n * 4 + 255) & ~(size_t)255;
    const size_t mb = ((size_t)(np + 31) / 32 * 4 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->sparse[5], 2 * ne + 7 * n4 + mb + 1024);
    if (rc) return rc;
    char* p8 = static_cast<char*>(ctx->sparse[5].ptr);
    E* ka = static_cast<E*>(carve(p8, ne));
    E* kb = static_cast<E*>(carve(p8, ne));
    uint32_t* pa = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* pb = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* ia = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* ib = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* flags = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* ex = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* starts = static_cast<uint32_t*>(carve(p8, n4));
    uint32_t* small = static_cast<uint32_t*>(carve(p8, 256));
    uint32_t* d_mask = static_cast<uint32_t*>(carve(p8, mb));
    std::vector<uint32_t> mask((np + 31) / 32, 0u);
    for (uint32_t p : passes) mask[p >> 5] |= 1u << (p & 31u);
    KMH_HIP(ctx, hipMemsetAsync(small, 0, 256, s));
    KMH_HIP(ctx, hipMemcpyAsync(d_mask, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, s));
    if (tb > ta) {
        hipLaunchKernelGGL((k_sp_gather<E, POS>), dim3((unsigned)(tb - ta)), dim3(256), 0, s, ent, epos, toff, ldt,
                           ta, tb, b, d_mask, np, R, ka, pa, small);
        KMH_HIP(ctx, hipGetLastError());
    }
    uint32_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, small, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    const unsigned gm = (m + 255u) / 256u;
    bool alt = false;
    E* keys = ka;
    uint32_t* pos = pa;
    if constexpr (POS) {
        // by position (32 bits, indices as values), then the keys gathered in that order and sorted
        // stably by key with their positions
        hipLaunchKernelGGL(k_sp_iota, dim3(gm), dim3(256), 0, s, ia, m);
        KMH_HIP(ctx, hipGetLastError());
        rc = radix_sort_pairs<uint32_t>(ctx, pa, pb, ia, ib, m, 0, 32, &alt, s);
        if (rc) return rc;
        uint32_t* psorted = alt ? pb : pa;
        uint32_t* isorted = alt ? ib : ia;
        hipLaunchKernelGGL(k_sp_gather_by<E>, dim3(gm), dim3(256), 0, s, ka, isorted, m, kb);
        KMH_HIP(ctx, hipGetLastError());
        uint32_t* pother = alt ? pa : pb;
        rc = radix_sort_pairs<E>(ctx, kb, ka, psorted, pother, m, 0, R, &alt, s);
        if (rc) return rc;
        keys = alt ? ka : kb;
        pos = alt ? pother : psorted;
    } else {
        rc = radix_sort_pairs<E>(ctx, ka, kb, pa, pb, m, 0, R, &alt, s);
        if (rc) return rc;
        keys = alt ? kb : ka;
        pos = alt ? pb : pa;
    }
    rc = run_starts<E>(ctx, keys, m, flags, ex, starts, small + 1, s);
    if (rc) return rc;
    if constexpr (ORD)
        hipLaunchKernelGGL(k_sp_append_ord<E>, dim3(1), dim3(256), 0, s, keys, m, starts, small + 1, d_mask, np, R,
                           (uint64_t)b << R, cbase, item_off, item_n, codes, counts, nk + g);
    else
        hipLaunchKernelGGL((k_sp_append<E, POS>), dim3(1), dim3(256), 0, s, keys, pos, m, starts, small + 1,
                           (uint64_t)b << R, out_off, nk + g, codes, counts, firsts);
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

// ORD: every genome's rows compact, in code order and back to back from entry 0; d_nkmers (the row
// lengths) and d_ndist both receive the distinct k-mers (no padding rows since round 5).
template <typename E, bool POS, bool ORD = false>
int sparse_count_dev_impl(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                          int canonical, uint64_t* d_codes, uint32_t* d_counts, uint32_t* d_firsts,
                          uint64_t* d_nkmers, hipStream_t s, uint64_t* d_ndist = nullptr) {
    constexpr int kSpTile = Sp<E, POS>::TILE, kCaps = Sp<E, POS>::CAPS;
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
    // ORD: the rows written by earlier batches (every genome's row follows the previous one's)
    unsigned long long* d_rowbase = nullptr;
    if (ORD) {
        KMH_HIP(ctx, hipMemsetAsync(d_ndist, 0, (size_t)G * sizeof(uint64_t), s));
        rc = ensure(ctx, ctx->sparse[0], 256);
        if (rc) return rc;
        d_rowbase = static_cast<unsigned long long*>(ctx->sparse[0].ptr);
        KMH_HIP(ctx, hipMemsetAsync(d_rowbase, 0, 8, s));
    }
    if (L.ntiles == 0) return KMH_OK;
    unsigned long long* const d_nk = reinterpret_cast<unsigned long long*>(ORD ? d_ndist : d_nkmers);

    const size_t tile_bytes = (size_t)kSpTile * sizeof(E);
    const size_t budget = env_mb("KMH_SP_BUDGET_MB", 16384) << 20;
    // Keys per count item (one pass of a bucket): the bin sort of k_sp_count stages at most
    // Cnt<E, POS>::CAP keys (8192 u32 / 4096 u64; half with positions); the pass target leaves
    // room for the spread of the pass sizes around it.
    const uint32_t target = (uint32_t)std::max<long>(
        1, env_long("KMH_SP_TARGET", (sizeof(E) == 4 ? 7680 : 3840) / (POS ? 2 : 1)));
    // Entries per split item (capped by the staging, and by ts <= one queue step per wave in GbRule):
    // 16384 against 12288 cut the config-5 split 10.9 -> 10.1 ms (fewer items: fewer reservation
    // round trips and barriers; profiles/r05/r05ah, r05ai); 14336-20480 measured within 0.2 ms.
    const uint32_t split_target = (uint32_t)std::max<long>(1, std::min<long>(env_long("KMH_SP_SPLIT", 16384), kCaps));
    // KMH_SP_LIMIT caps the distinct keys of one item (tests force the fallback with it)
    const uint32_t limit = (uint32_t)std::min<long>(std::max<long>(1, env_long("KMH_SP_LIMIT", Cnt<E, POS>::CAP)),
                                                    Cnt<E, POS>::CAP);
    // batches of whole genomes whose step-1 entries fit the budget (at most 2^20 tiles: toff rows;
    // a genome always forms a batch of its own if it alone passes the budget)
    std::vector<std::pair<int, int>> batches;
    uint64_t max_tiles = 0;
    for (int g = 0; g < G;) {
        int h = g;
        uint64_t tiles = 0;
        do {
            tiles += L.tbase[h + 1] - L.tbase[h];
            ++h;
        } while (h < G && (tiles + (L.tbase[h + 1] - L.tbase[h])) * tile_bytes <= budget &&
                 tiles + (L.tbase[h + 1] - L.tbase[h]) <= (1u << 20));
        batches.emplace_back(g, h);
        max_tiles = std::max(max_tiles, tiles);
        g = h;
    }
    if (max_tiles > (1u << 20)) return fail(ctx, KMH_ERR_UNSUPPORTED, "genome too large for the sparse path");
    const uint32_t ldt = (uint32_t)((max_tiles + 63) / 64 * 64);
    rc = ensure(ctx, ctx->sparse[2], std::max<uint64_t>(max_tiles, 1) * tile_bytes);
    if (!rc) rc = ensure(ctx, ctx->sparse[3], (size_t)ldt * (kSpBuckets + 1) * sizeof(uint16_t));
    if (!rc && POS) rc = ensure(ctx, ctx->sparse[7], std::max<uint64_t>(max_tiles, 1) * (size_t)kSpTile * 4);
    if (rc) return rc;
    E* ent = static_cast<E*>(ctx->sparse[2].ptr);
    uint32_t* epos = POS ? static_cast<uint32_t*>(ctx->sparse[7].ptr) : nullptr;
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
        // persistent partition: one workgroup per CU
        const unsigned pgrid = (unsigned)std::min<uint64_t>(tiles, (uint64_t)std::max(1, ctx->num_cu));
        launch_partition_k<E, POS>(k, canonical, (unsigned)tiles, pgrid, s, d_seq, m, ent, epos, toff, ldt);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());

        // bucket sizes -> split and count work items, planned and written on the device;
        // the host reads back only the two item totals to size the buffers
        const size_t ngb = (size_t)nG * kSpBuckets;
        rc = ensure(ctx, ctx->sparse[4], ngb * 24 + (size_t)nG * 4 + 4096);
        if (rc) return rc;
        uint32_t* d_nb = static_cast<uint32_t*>(ctx->sparse[4].ptr);
        uint32_t* d_gbfail = d_nb + ngb;
        uint32_t* d_sofs = d_gbfail + ngb;
        uint32_t* d_cofs = d_sofs + ngb;
        uint32_t* d_grank = d_cofs + ngb;     // k_sp_order: rank among the genome's buckets of equal ts
        uint32_t* d_tab = d_grank + ngb;      // k_sp_order: distinct ts values per genome
        uint32_t* d_nv = d_tab + ngb;
        uint32_t* d_totals = d_nv + nG;
        KMH_HIP(ctx, hipMemsetAsync(d_gbfail, 0, ngb * 4, s));
        hipLaunchKernelGGL(k_sp_sizes, dim3((unsigned)ngb), dim3(256), 0, s, toff, ldt, d_tbase, g0,
                           L.tbase[g0], d_nb);
        KMH_HIP(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_sp_plan, dim3(1), dim3(1024), 0, s, d_nb, (int)ngb, d_tbase, g0, target,
                           split_target, (uint32_t)epc<E>(), d_sofs, d_cofs, d_totals);
        KMH_HIP(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_sp_order, dim3((unsigned)nG), dim3(kSpBuckets), 0, s, d_nb, d_tbase, g0, target,
                           split_target, (uint32_t)epc<E>(), d_grank, d_tab, d_nv);
        KMH_HIP(ctx, hipGetLastError());
        uint32_t totals[2] = {0u, 0u};
        KMH_HIP(ctx, hipMemcpyAsync(totals, d_totals, 8, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        const double h1 = hprof ? now_ms() : 0.0;
        const size_t nsi = totals[0], nci = totals[1];
        if (nci == 0) continue;
        const double h2 = hprof ? now_ms() : 0.0;
        // count-item regions (+ positions) and their fill counters (ctx->sparse[6]); items, out_off,
        // failed list (ctx->sparse[1])
        constexpr int C = Cnt<E, POS>::CAP;
        const size_t sbytes = nci * (size_t)C * sizeof(E);
        const size_t pbytes = POS ? nci * (size_t)C * 4 : 0;
        const size_t fillb = (nci * 4 + 255) & ~(size_t)255;
        rc = ensure(ctx, ctx->sparse[6], sbytes + pbytes + fillb);
        if (rc) return rc;
        E* d_split = static_cast<E*>(ctx->sparse[6].ptr);
        uint32_t* d_spos = POS ? reinterpret_cast<uint32_t*>(static_cast<char*>(ctx->sparse[6].ptr) + sbytes) : nullptr;
        uint32_t* d_pfill = reinterpret_cast<uint32_t*>(static_cast<char*>(ctx->sparse[6].ptr) + sbytes + pbytes);
        KMH_HIP(ctx, hipMemsetAsync(d_pfill, 0, nci * 4, s));
        const size_t sib = (nsi * sizeof(SplitItem) + 255) & ~(size_t)255;
        const size_t cib = (nci * sizeof(CountItem) + 255) & ~(size_t)255;
        const size_t ob = ((size_t)(G + 1) * 8 + 255) & ~(size_t)255;
        const size_t fb = ((nci + 1) * 4 + 255) & ~(size_t)255;
        // ORD: the items' output bases and a genome-start scratch
        const size_t nch = (nci + kIoChunk - 1) / kIoChunk;
        const size_t iob = ORD ? ((nci * 8 + 255) & ~(size_t)255) + (((size_t)nG * 8 + 255) & ~(size_t)255) +
                                     ((nch * 8 + 255) & ~(size_t)255) + ((nci * 4 + 255) & ~(size_t)255)
                               : 0;
        rc = ensure(ctx, ctx->sparse[1], sib + cib + ob + fb + iob);
        if (rc) return rc;
        char* base = static_cast<char*>(ctx->sparse[1].ptr);
        SplitItem* d_sitems = reinterpret_cast<SplitItem*>(base);
        CountItem* d_citems = reinterpret_cast<CountItem*>(base + sib);
        uint64_t* d_out_off = reinterpret_cast<uint64_t*>(base + sib + cib);
        uint32_t* d_failed = reinterpret_cast<uint32_t*>(base + sib + cib + ob);
        uint64_t* d_item_off = ORD ? reinterpret_cast<uint64_t*>(base + sib + cib + ob + fb) : nullptr;
        unsigned long long* d_gstart =
            ORD ? reinterpret_cast<unsigned long long*>(base + sib + cib + ob + fb + ((nci * 8 + 255) & ~(size_t)255))
                : nullptr;
        hipLaunchKernelGGL(k_sp_fill, dim3((unsigned)ngb), dim3(64), 0, s, d_nb, d_tbase, g0, L.tbase[g0],
                           target, split_target, (uint32_t)epc<E>(), d_sofs, d_cofs, d_grank, d_tab, d_nv, d_sitems,
                           d_citems);
        KMH_HIP(ctx, hipGetLastError());
        KMH_HIP(ctx, hipMemcpyAsync(d_out_off, out_off.data(), (size_t)(G + 1) * 8, hipMemcpyHostToDevice, s));
        KMH_HIP(ctx, hipMemsetAsync(d_failed, 0, 4, s));
        time_begin(ctx, s, "k_sp_split");
        // persistent split: one workgroup per CU
        const unsigned sgrid = (unsigned)std::min<uint64_t>(nsi, (uint64_t)std::max(1, ctx->num_cu));
        hipLaunchKernelGGL((k_sp_split<E, POS>), dim3(sgrid), dim3(kSpThreads), 0, s, ent, epos, toff, ldt,
                           d_sitems, (uint32_t)nsi, R, d_split, d_spos, d_pfill, d_gbfail);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
#ifdef KMH_EXPERIMENTS
        if (env_long("KMH_SP_PROF", 0) == 1) {
            unsigned long long h[16];
            KMH_HIP(ctx, hipStreamSynchronize(s));
            KMH_HIP(ctx, hipMemcpyFromSymbol(h, HIP_SYMBOL(g_split_prof), sizeof(h)));
            const double w = (double)h[15];
            std::fprintf(stderr, "k_sp_split per wave over %zu items on %u WGs (Mcyc): A hold %.2f | B bounds %.2f | "
                         "hist %.2f | bar %.2f | scan %.2f | scatter %.2f | bar %.2f | landed %.2f | stores %.2f | "
                         "bar %.2f\n", nsi, sgrid, h[0] / w / 1e6, h[1] / w / 1e6, h[2] / w / 1e6, h[3] / w / 1e6,
                         h[4] / w / 1e6, h[5] / w / 1e6, h[6] / w / 1e6, h[7] / w / 1e6, h[8] / w / 1e6, h[9] / w / 1e6);
            const unsigned long long z[16] = {};
            KMH_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_split_prof), z, sizeof(z)));
        }
#endif
        // passes left to the fallback: count items whose table overflowed, and every pass of a
        // bucket whose split overflowed; grouped by (genome, bucket): one gather + sort per bucket,
        // however many of its passes failed (a skewed organism's largest buckets can fail every
        // pass).  ORD's first pass (item_n set): each failed pass's distinct k-mers only.
        std::vector<uint32_t> ids;
        auto run_fallback = [&](uint32_t* item_n) -> int {
            uint32_t nfail = 0;
            std::vector<uint32_t> gbf(ngb);
            KMH_HIP(ctx, hipMemcpyAsync(&nfail, d_failed, 4, hipMemcpyDeviceToHost, s));
            KMH_HIP(ctx, hipMemcpyAsync(gbf.data(), d_gbfail, ngb * 4, hipMemcpyDeviceToHost, s));
            KMH_HIP(ctx, hipStreamSynchronize(s));
            ids.assign(nfail, 0u);
            if (nfail) {
                KMH_HIP(ctx, hipMemcpyAsync(ids.data(), d_failed + 1, (size_t)nfail * 4, hipMemcpyDeviceToHost, s));
                KMH_HIP(ctx, hipStreamSynchronize(s));
            }
            bool any_gbf = false;
            for (uint32_t f : gbf) any_gbf |= f != 0u;
#ifdef KMH_EXPERIMENTS
            if (env_long("KMH_SP_NO_FALLBACK", 0)) {   // what-if builds whose counts are wrong by design
                nfail = 0;
                ids.clear();
                any_gbf = false;
            }
#endif
            std::vector<CountItem> citems;
            if (nfail || any_gbf) {  // items are only needed on the host to recount failed passes
                citems.resize(nci);
                KMH_HIP(ctx, hipMemcpyAsync(citems.data(), d_citems, nci * sizeof(CountItem), hipMemcpyDeviceToHost, s));
                KMH_HIP(ctx, hipStreamSynchronize(s));
                for (const CountItem& it : citems)
                    if (gbf[it.gb]) ids.push_back((uint32_t)(&it - citems.data()));
            }
            std::sort(ids.begin(), ids.end(), [&](uint32_t a, uint32_t c) {
                return citems[a].gb != citems[c].gb ? citems[a].gb < citems[c].gb : citems[a].p < citems[c].p;
            });
            ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
            std::vector<uint32_t> passes;
            for (size_t i = 0; i < ids.size();) {
                const CountItem& it = citems[ids[i]];
                passes.clear();
                size_t j = i;
                for (; j < ids.size() && citems[ids[j]].gb == it.gb; ++j) passes.push_back(citems[ids[j]].p);
                if (!item_n) {
                    ctx->fb_passes += passes.size();
                    ctx->fb_groups += 1;
                }
                const int frc = fallback_passes<E, POS, ORD>(
                    ctx, it.g, it.b, passes, it.np, it.n, ent, epos, toff, ldt, L.tbase[it.g] - L.tbase[g0],
                    L.tbase[it.g + 1] - L.tbase[g0], R, out_off[it.g], d_nk, d_codes, d_counts, d_firsts, d_item_off,
                    item_n, ids[i] - it.p, s);
                if (frc) return frc;
                i = j;
            }
            return KMH_OK;
        };
        const unsigned cgrid = (unsigned)std::min<size_t>(nci, (size_t)std::max(1, ctx->num_cu) * 2);
        if constexpr (ORD) {
            // first pass: every item's distinct k-mers (k_sp_count without order or stores, the
            // fallback's runs for its failed passes), then every item's output base (its genome's
            // row offset + the distinct k-mers of its earlier items) and the row lengths: rows come
            // out compact, no padding to drop
            uint32_t* const d_item_n = reinterpret_cast<uint32_t*>(
                reinterpret_cast<char*>(d_gstart) + (((size_t)nG * 8 + 255) & ~(size_t)255) + ((nch * 8 + 255) & ~(size_t)255));
            KMH_HIP(ctx, hipMemsetAsync(d_item_n, 0, nci * 4, s));
            time_begin(ctx, s, "k_sp_count_n");
            hipLaunchKernelGGL((k_sp_count<E, POS, ORD, true>), dim3(cgrid), dim3(kCntThreads), 0, s, d_split, d_spos,
                               d_pfill, d_citems, (uint32_t)nci, R, limit, d_item_off, d_codes, d_counts, d_item_n, d_nk,
                               d_gbfail, d_failed);
            time_end(ctx, s);
            KMH_HIP(ctx, hipGetLastError());
            if ((rc = run_fallback(d_item_n))) return rc;
            unsigned long long* const d_csum = d_gstart + (((size_t)nG * 8 + 255) & ~(size_t)255) / 8;
            unsigned long long* const d_rows = reinterpret_cast<unsigned long long*>(d_nkmers);
            hipLaunchKernelGGL(k_sp_io_sums, dim3((unsigned)nch), dim3(256), 0, s, d_item_n, d_citems, (uint32_t)nci,
                               d_csum, d_rows);
            KMH_HIP(ctx, hipGetLastError());
            hipLaunchKernelGGL(k_sp_io_scan, dim3(1), dim3(1024), 0, s, d_csum, (uint32_t)nch, d_rowbase);
            KMH_HIP(ctx, hipGetLastError());
            hipLaunchKernelGGL(k_sp_io_write, dim3((unsigned)nch), dim3(256), 0, s, d_item_n, (uint32_t)nci, d_csum,
                               d_item_off);
            KMH_HIP(ctx, hipGetLastError());
            KMH_HIP(ctx, hipMemsetAsync(d_failed, 0, 4, s));
        }
        time_begin(ctx, s, "k_sp_count");
        hipLaunchKernelGGL((k_sp_count<E, POS, ORD>), dim3(cgrid), dim3(kCntThreads), 0, s, d_split, d_spos, d_pfill,
                           d_citems, (uint32_t)nci, R, limit, ORD ? d_item_off : d_out_off, d_codes, d_counts, d_firsts,
                           d_nk, d_gbfail, d_failed);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
#ifdef KMH_EXPERIMENTS
        if (env_long("KMH_SP_PROF", 0) == 1) {
            unsigned long long h[16];
            KMH_HIP(ctx, hipStreamSynchronize(s));
            KMH_HIP(ctx, hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sp_prof), sizeof(h)));
            const double w = (double)h[8] * kNW;   // waves
            std::fprintf(stderr, "k_sp_count per wave over %zu items on %u WGs: scan %.2f | scatter %.2f | issue next %.2f | "
                         "big+emission %.2f | totals+clear %.2f | next hist %.2f | stores %.2f | - %.2f Mcyc\n", nci, (unsigned)h[8],
                         h[0] / w / 1e6, h[1] / w / 1e6, h[2] / w / 1e6, h[3] / w / 1e6, h[4] / w / 1e6,
                         h[5] / w / 1e6, h[6] / w / 1e6, h[7] / w / 1e6);
            const unsigned long long z[16] = {};
            KMH_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_sp_prof), z, sizeof(z)));
        }
#endif
        const double h3 = hprof ? now_ms() : 0.0;
        const double h4 = h3;
        if ((rc = run_fallback(nullptr))) return rc;
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
    if (k <= 21)
        return sparse_count_dev_impl<uint32_t, false>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, nullptr,
                                                      d_nkmers, s);
    return sparse_count_dev_impl<uint64_t, false>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, nullptr,
                                                  d_nkmers, s);
}

int sparse_count_dev_sorted(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                            int canonical, uint64_t* d_codes, uint32_t* d_counts, uint64_t* d_nrows,
                            uint64_t* d_ndist, hipStream_t s) {
    if (k < 13 || k > 32) return fail(ctx, KMH_ERR_UNSUPPORTED, "device sparse counting needs 13 <= k <= 32");
    if (!d_seq || !d_codes || !d_counts || !d_nrows || !d_ndist)
        return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (k <= 21)
        return sparse_count_dev_impl<uint32_t, false, true>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts,
                                                            nullptr, d_nrows, s, d_ndist);
    return sparse_count_dev_impl<uint64_t, false, true>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts,
                                                        nullptr, d_nrows, s, d_ndist);
}

int sparse_count_dev_first(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k, int canonical,
                           uint64_t* d_codes, uint32_t* d_counts, uint32_t* d_firsts, uint64_t* d_nkmers,
                           hipStream_t s) {
    if (k < 13 || k > 32) return fail(ctx, KMH_ERR_UNSUPPORTED, "device sparse counting needs 13 <= k <= 32");
    if (!d_seq || !d_codes || !d_counts || !d_firsts || !d_nkmers) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (k <= 21)
        return sparse_count_dev_impl<uint32_t, true>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, d_firsts,
                                                     d_nkmers, s);
    return sparse_count_dev_impl<uint64_t, true>(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, d_firsts,
                                                 d_nkmers, s);
}

}  // namespace kmh
