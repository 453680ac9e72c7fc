// kmh_dense.hip -- dense k-mer counting on MI355X (gfx950): 1 <= k <= 12.
//
// Replaces the window loop of /root/reference/kmerml/kmers/generate.py:49-58 (slide a
// k-window over each record, drop windows with a non-ACGT byte, count) for a batch of
// genomes resident in HBM.  Design and rooflines: DESIGN.md, "Kernels".
//
//   k <= 9   k_direct:     each workgroup counts a span of one genome into an LDS table
//                          (4^k bins, or 32768-bin slices in 4^k/32768 passes for k = 8, 9)
//                          and adds it into the genome's row.
//   k >= 10  k_partition:  one 32768-window tile per workgroup; k-mers are bucketed by
//                          their top 2k-15 bits with an LDS counting sort and each tile
//                          writes its bucket-ordered 15-bit suffixes + bucket offsets.
//            k_bucket_count: one workgroup per (genome, bucket) gathers that bucket's
//                          segments from every tile of the genome into a 32768-bin LDS
//                          histogram and stores the row slice once.
//
// Bases: A/C/G/T in either case (generate.py:41 upper()s the record; :55 keeps windows of
// "ACGT" only).  Any other byte -- including the '\n' the host puts between records and
// bytes past a genome's end -- breaks windows, so windows never span records or genomes.
#include <algorithm>
#include <cstdlib>

#include "kmh_device.h"

namespace kmh {

int make_layout(Ctx* ctx, const uint64_t* offsets, int G, int k, uint64_t tile, Layout& L) {
    if (G < 1) return fail(ctx, KMH_ERR_INVALID, "G must be >= 1");
    if (!offsets) return fail(ctx, KMH_ERR_INVALID, "offsets is NULL");
    L.goff.assign(offsets, offsets + G + 1);
    L.tbase.assign(G + 1, 0);
    for (int g = 0; g < G; ++g) {
        const uint64_t a = offsets[g], b = offsets[g + 1];
        if (b < a) return fail(ctx, KMH_ERR_INVALID, "offsets must be non-decreasing");
        if (a % 16 != 0) return fail(ctx, KMH_ERR_INVALID, "genome start offsets must be multiples of 16");
        if (b - a >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "a genome must be shorter than 2^32 - 1 bytes");
        const uint64_t nwin = (b - a >= (uint64_t)k) ? (b - a - (uint64_t)k + 1) : 0;
        L.tbase[g + 1] = L.tbase[g] + (nwin + tile - 1) / tile;
    }
    L.ntiles = L.tbase[G];
    return KMH_OK;
}

int upload_layout(Ctx* ctx, const Layout& L, hipStream_t s, const uint64_t** d_goff,
                  const uint64_t** d_tbase) {
    const size_t n = L.goff.size();
    int rc = ensure(ctx, ctx->meta, 2 * n * sizeof(uint64_t));
    if (rc) return rc;
    std::vector<uint64_t> both(2 * n);
    std::copy(L.goff.begin(), L.goff.end(), both.begin());
    std::copy(L.tbase.begin(), L.tbase.end(), both.begin() + n);
    rc = upload(ctx, ctx->meta.ptr, both.data(), both.size() * sizeof(uint64_t), s);
    if (rc) return rc;
    *d_goff = static_cast<const uint64_t*>(ctx->meta.ptr);
    *d_tbase = *d_goff + n;
    return KMH_OK;
}

long env_long(const char* name, long dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atol(v) : dflt;
}

size_t env_mb(const char* name, size_t dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    const long x = std::atol(v);
    return x > 0 ? (size_t)x : dflt;
}

namespace {

constexpr int kDirectThreads = kTileThreads;
constexpr int kTargetWorkgroups = 512;

template <int K>
constexpr int num_buckets() { return 1 << (2 * K - kSubBits); }


// Entries per tile in the suffix buffer: every bucket segment is padded to whole 16-byte
// chunks (8 entries) so the count kernel reads aligned chunks with no masking.  Padding
// entries hold kPadBase + ((8 * bucket + slot) & 63): 64 dummy LDS bins past the real
// 32768, spread so that padding lanes of one instruction rarely share an address.
template <int K>
constexpr int tile_cap(int tile) { return tile + num_buckets<K>() * 7; }
constexpr uint32_t kPadBase = (uint32_t)kSubBins;

// Tiles per wave batch of the count kernels: the expected chunks of a batch must fit the
// per-wave queue of qmax entries (a batch that overflows it is walked lane by lane).
template <int K>
constexpr int batch_tiles(int tile, int qmax) {
    const int per = tile / num_buckets<K>() / 8 + 1;       // expected chunks per segment
    int bt = qmax / per;
    bt = bt < 1 ? 1 : (bt > 64 ? 64 : bt);
    int p2 = 1;
    while (p2 * 2 <= bt) p2 *= 2;
    return p2;
}
constexpr uint32_t kPadBins = 64;

// Visit the 32 windows that start at tstart + 32 * threadIdx.x + j, j = 0..31:
// f(j, code, is_valid).  Each thread loads its 32 bytes plus the next 16 (the k - 1 <= 15
// bases its last windows need).  FAST: the three 16-byte loads are issued back to back
// with no guard (the caller checked that every byte read lies before data_end) and bytes
// past the genome end are masked arithmetically; otherwise byte-wise guarded loads.
template <int K, bool FAST, typename F>
__device__ __forceinline__ void walk_tile(const uint8_t* __restrict__ seq, uint64_t tstart,
                                          uint64_t gend, F&& f) {
    static_assert(K >= 1 && K <= 16, "dense windows need k <= 16");
    const uint64_t base = tstart + (uint64_t)threadIdx.x * kTileBpt;
    uint32_t cA, iA, cB, iB, cN, iN;
    if constexpr (FAST) {
        const uint4 a = *reinterpret_cast<const uint4*>(seq + base);
        const uint4 b = *reinterpret_cast<const uint4*>(seq + base + 16);
        const uint4 n = *reinterpret_cast<const uint4*>(seq + base + 32);
        enc16(a, cA, iA);
        enc16(b, cB, iB);
        enc16(n, cN, iN);
        iA |= tail_mask(base, gend);
        iB |= tail_mask(base + 16, gend);
        iN |= tail_mask(base + 32, gend);
    } else {
        enc16(load16(seq, base, gend), cA, iA);
        enc16(load16(seq, base + 16, gend), cB, iB);
        enc16(load16(seq, base + 32, gend), cN, iN);
    }
    constexpr uint32_t KM = (K == 16) ? 0xFFFFFFFFu : ((1u << (2 * K)) - 1u);
    constexpr uint32_t VM = (1u << K) - 1u;
    const uint64_t wAB = ((uint64_t)cA << 32) | cB;
    const uint32_t vAB = (iA << 16) | iB;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t code = (uint32_t)(wAB >> (64 - 2 * (j + K))) & KM;
        f(j, code, ((vAB >> (32 - (j + K))) & VM) == 0u);
    }
    const uint64_t wBN = ((uint64_t)cB << 32) | cN;
    const uint32_t vBN = (iB << 16) | iN;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t code = (uint32_t)(wBN >> (64 - 2 * (j + K))) & KM;
        f(16 + j, code, ((vBN >> (32 - (j + K))) & VM) == 0u);
    }
}

// Dispatch a tile walk of `tpb` threads to the fast or the guarded loads (uniform per
// workgroup: only tiles within 48 bytes of the end of the whole buffer take the slow path).
template <int K, typename F>
__device__ __forceinline__ void walk(const uint8_t* __restrict__ seq, const GenomeMap& m,
                                     uint64_t tstart, uint64_t gend, int tpb, F&& f) {
    if (tstart + (uint64_t)tpb * kTileBpt + 16 <= m.data_end) walk_tile<K, true>(seq, tstart, gend, f);
    else walk_tile<K, false>(seq, tstart, gend, f);
}

// ---------------------------------------------------------------- k <= 9: direct
template <int K>
__global__ __launch_bounds__(kDirectThreads) void k_direct(const uint8_t* __restrict__ seq,
                                                           GenomeMap m, int S,
                                                           uint32_t* __restrict__ out) {
    constexpr uint32_t BINS = 1u << (2 * K);
    constexpr uint32_t SLICE = BINS < (uint32_t)kSubBins ? BINS : (uint32_t)kSubBins;
    constexpr int NPASS = (int)(BINS / SLICE);
    constexpr int REP0 = (int)(16384u / SLICE);  // replicas that fit in 64 KiB
    constexpr int REP = REP0 < 1 ? 1 : (REP0 > 8 ? 8 : REP0);
    __shared__ __attribute__((aligned(16))) uint32_t tbl[REP * SLICE];

    const uint32_t w = xcd_work_id();
    const int gl = (int)(w / (uint32_t)S), s = (int)(w % (uint32_t)S);
    const int g = m.g0 + gl;
    const uint64_t gs = m.goff[g], ge = m.goff[g + 1];
    const uint64_t nt = m.tbase[g + 1] - m.tbase[g];
    const uint64_t ta = nt * (uint64_t)s / (uint64_t)S, tb = nt * (uint64_t)(s + 1) / (uint64_t)S;
    uint32_t* tab = tbl + ((threadIdx.x >> 6) % REP) * SLICE;
    uint32_t* orow = out + (uint64_t)g * BINS;

    for (int p = 0; p < NPASS; ++p) {
        for (uint32_t i = threadIdx.x; i < REP * SLICE; i += kDirectThreads) tbl[i] = 0u;
        __syncthreads();
        for (uint64_t t = ta; t < tb; ++t) {
            walk<K>(seq, m, gs + t * (uint64_t)kTile, ge, kDirectThreads, [&](int, uint32_t code, bool ok) {
                if (NPASS == 1) {
                    if (ok) atomicAdd(&tab[code], 1u);
                } else if (ok && (code / SLICE) == (uint32_t)p) {
                    atomicAdd(&tab[code % SLICE], 1u);
                }
            });
        }
        __syncthreads();
        if (ta < tb) {
            for (uint32_t i = threadIdx.x; i < SLICE; i += kDirectThreads) {
                uint32_t v = 0u;
#pragma unroll
                for (int r = 0; r < REP; ++r) v += tbl[r * SLICE + i];
                if (v) atomicAdd(&orow[(uint64_t)p * SLICE + i], v);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- k >= 10: partition
// Ablation bits (experiments only; outputs are wrong when set): 1 = no histogram atomics
// (synthetic uniform bucket starts), 2 = no scatter, 4 = no write-out.
// SUBT sub-tiles of TPB * 32 windows form one tile (longer bucket segments).
template <int K, int TPB, int ABL, int SUBT = 1>
__global__ __launch_bounds__(TPB) void k_partition(const uint8_t* __restrict__ seq,
                                                   GenomeMap m, uint16_t* __restrict__ suf,
                                                   uint16_t* __restrict__ toff, uint32_t ldt) {
    constexpr int NBK = num_buckets<K>();
    constexpr int TILE = TPB * kTileBpt * SUBT;
    static_assert(NBK <= TPB, "one scan element per thread");
    constexpr int CAP = tile_cap<K>(TILE);
    __shared__ __attribute__((aligned(16))) uint16_t sorted[CAP];
    __shared__ uint32_t cnt[NBK];
    __shared__ uint32_t cur[NBK];
    __shared__ uint32_t wsum[TPB / 64];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = xcd_work_id();  // neighbouring tiles on one XCD: their toff
    const uint64_t gt = m.tile_lo + lt; // stores combine in that XCD's L2
    const int g = find_genome(m, gt);
    const uint64_t tstart = m.goff[g] + (gt - m.tbase[g]) * (uint64_t)TILE;
    const uint64_t ge = m.goff[g + 1];

    for (int b = tid; b < NBK; b += TPB) cnt[b] = (ABL & 1) ? (uint32_t)(TILE / NBK) : 0u;
    __syncthreads();

    uint32_t km[kTileBpt * SUBT];
#pragma unroll
    for (int sub = 0; sub < SUBT; ++sub) {
        walk<K>(seq, m, tstart + (uint64_t)sub * TPB * kTileBpt, ge, TPB, [&](int j, uint32_t code, bool ok) {
            km[sub * kTileBpt + j] = ok ? code : 0xFFFFFFFFu;
            if (!(ABL & 1) && ok) atomicAdd(&cnt[code >> kSubBits], 1u);
        });
    }
    __syncthreads();

    // Exclusive scan of the bucket histogram -> bucket starts.
    const uint32_t nb = tid < NBK ? cnt[tid] : 0u;  // entries of bucket tid
    const uint32_t v = (nb + 7u) & ~7u;              // padded to whole chunks
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, total = 0u;
#pragma unroll
    for (int w = 0; w < TPB / 64; ++w) {
        pre += (w < wave) ? wsum[w] : 0u;
        total += wsum[w];
    }
    // toff, bucket-major [NBK + 1][ldt]: chunk index of every bucket's segment in this
    // tile, then the tile's total chunk count (a count workgroup reads one row).
    const uint32_t start = pre + incl - v;
    if (tid < NBK) {
        cur[tid] = start;
        toff[(uint64_t)tid * ldt + lt] = (uint16_t)(start >> 3);
    }
    if (tid == 0) toff[(uint64_t)NBK * ldt + lt] = (uint16_t)(total >> 3);
    __syncthreads();

    // Scatter 15-bit suffixes into bucket order.
    if (!(ABL & 2)) {
#pragma unroll
        for (int j = 0; j < kTileBpt * SUBT; ++j) {
            const uint32_t c = km[j];
            if (c != 0xFFFFFFFFu) {
                uint32_t slot = atomicAdd(&cur[c >> kSubBits], 1u);
                if (ABL & 1) slot %= (uint32_t)CAP;  // synthetic starts may overrun
                sorted[slot] = (uint16_t)(c & (kSubBins - 1));
            }
        }
        if (tid < NBK)  // pad the bucket's segment to its chunk boundary
            for (uint32_t q = start + nb; q < start + v; ++q)
                sorted[q] = (uint16_t)(kPadBase + ((8u * (uint32_t)tid + q) & (kPadBins - 1)));
    } else {
#pragma unroll
        for (int j = 0; j < kTileBpt * SUBT; ++j) asm volatile("" ::"v"(km[j]));
    }
    __syncthreads();

    if (!(ABL & 4)) {
        uint4* dst = reinterpret_cast<uint4*>(suf + lt * (uint64_t)CAP);
        const uint4* src = reinterpret_cast<const uint4*>(sorted);
        const uint32_t nchunk = total >> 3;
        for (uint32_t c = tid; c < nchunk; c += TPB) store_nt(&dst[c], src[c]);
    }
}

// ---------------------------------------------------------------- k >= 10: persistent partition
// Same output as k_partition (bucket-ordered, chunk-padded 15-bit suffixes + bucket-major
// offsets, one 32768-window tile at a time), with fewer and cheaper LDS operations:
//
//  * Bank-replicated counters.  Lane l of every wave counts into replica (l & 31) of its
//    bucket, rep[bucket][replica] at word 32 * bucket + replica, so the 32 lanes of a lane
//    group always hit 32 different banks (MI355X_MICROARCH.md §LDS: random 4-byte LDS
//    operations run at ~9 lanes/clk/CU, conflict-free atomics at ~15).
//  * One returning add per k-mer.  ds_add_rtn gives the k-mer its rank inside (bucket,
//    replica); a scan turns the counters into segment starts (bucket start + replica
//    prefix), and the scatter reads its start (conflict-free) and writes the suffix (the
//    one random LDS operation left).  k_partition needs three random operations per k-mer.
//  * Persistent with prefetch.  One 1024-thread workgroup per CU walks a contiguous run of
//    tiles; the next tile's 48 bytes per thread are loaded while this tile is scanned,
//    scattered and written out, so the LDS phases of one workgroup overlap its HBM reads.
//
// Experiment (KMH_PART=1), not the default: measured 134 us per 100 Mbp genome against 79 us
// for k_partition at 18 genomes per launch (profiles/r01_rep_bench.txt).  The 140 KiB of LDS
// leave one workgroup per CU, so its seven barriers per tile serialise the phases, and vmcnt
// counts stores as well as loads: waiting for the prefetched bytes also waits for the
// previous tile's 72 KiB of output to drain.  Two co-resident k_partition workgroups hide
// both for free.
template <int K>
__device__ __forceinline__ void visit_raw(uint4 a, uint4 b, uint4 n, uint32_t tm_a, uint32_t tm_b,
                                          uint32_t tm_n, uint32_t (&km)[kTileBpt]) {
    uint32_t cA, iA, cB, iB, cN, iN;
    enc16(a, cA, iA);
    enc16(b, cB, iB);
    enc16(n, cN, iN);
    iA |= tm_a;
    iB |= tm_b;
    iN |= tm_n;
    constexpr uint32_t KM = (1u << (2 * K)) - 1u;
    constexpr uint32_t VM = (1u << K) - 1u;
    const uint64_t wAB = ((uint64_t)cA << 32) | cB;
    const uint32_t vAB = (iA << 16) | iB;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t code = (uint32_t)(wAB >> (64 - 2 * (j + K))) & KM;
        km[j] = (((vAB >> (32 - (j + K))) & VM) == 0u) ? code : 0xFFFFFFFFu;
    }
    const uint64_t wBN = ((uint64_t)cB << 32) | cN;
    const uint32_t vBN = (iB << 16) | iN;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t code = (uint32_t)(wBN >> (64 - 2 * (j + K))) & KM;
        km[16 + j] = (((vBN >> (32 - (j + K))) & VM) == 0u) ? code : 0xFFFFFFFFu;
    }
}

constexpr int kRepThreads = 1024;
constexpr int kRepTile = kRepThreads * kTileBpt;   // 32768 windows, as k_partition<12, 512, ., 2>
constexpr int kRep = 32;                            // counter replicas = banks per lane group

template <int K>
__global__ __launch_bounds__(kRepThreads) void k_partition_rep(const uint8_t* __restrict__ seq,
                                                               GenomeMap m, uint16_t* __restrict__ suf,
                                                               uint16_t* __restrict__ toff, uint32_t ldt,
                                                               uint32_t ntiles) {
    constexpr int NBK = num_buckets<K>();
    constexpr int CAP = tile_cap<K>(kRepTile);
    constexpr int NW = kRepThreads / 64;
    static_assert(NBK >= 2 * NW && NBK <= kRepThreads, "scan layout needs 32 <= buckets <= 1024");
    __shared__ __attribute__((aligned(16))) uint16_t sorted[CAP + 64];    // + dummy slots
    __shared__ __attribute__((aligned(16))) uint32_t rep[(NBK + 1) * kRep];  // + dummy row
    __shared__ uint32_t bst[NBK];
    __shared__ uint32_t wsum[NW];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31;
    const uint32_t w = xcd_work_id();
    const uint64_t tlo = (uint64_t)ntiles * w / gridDim.x, thi = (uint64_t)ntiles * (w + 1) / gridDim.x;

    uint4* rep4 = reinterpret_cast<uint4*>(rep);
    for (int i = tid; i < (NBK + 1) * kRep / 4; i += kRepThreads) rep4[i] = make_uint4(0u, 0u, 0u, 0u);

    // Where the current tile lies: genome g spans batch tiles [tf, tn) and bytes [gs, ge).
    // Advanced tile by tile; the genome table is read only when the run crosses a genome (a
    // per-tile lookup would be a vector load, and waiting for it would also wait for the
    // previous tile's output stores: vmcnt counts both).
    // (readfirstlane: the values are uniform; keep them in scalar registers)
    auto uni = [](uint64_t x) -> uint64_t {
        // (the builtin returns int: zero-extend through uint32_t, never sign-extend)
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
               (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
    };
    int g = __builtin_amdgcn_readfirstlane(find_genome(m, m.tile_lo + tlo));
    uint64_t tf = uni(m.tbase[g] - m.tile_lo), tn = uni(m.tbase[g + 1] - m.tile_lo);
    uint64_t gs = uni(m.goff[g]), ge = uni(m.goff[g + 1]);
    auto advance = [&](uint64_t t) {
        while (t >= tn) {
            ++g;
            tf = tn;
            tn = uni(m.tbase[g + 1] - m.tile_lo);
            gs = uni(m.goff[g]);
            ge = uni(m.goff[g + 1]);
        }
    };

    uint4 ra = make_uint4(0u, 0u, 0u, 0u), rb = ra, rn = ra;   // this tile's 48 bytes
    uint4 pa = ra, pb = ra, pn = ra;                            // the next tile's (prefetch)
    bool have = false;   // pa/pb/pn hold the current tile
    for (uint64_t lt = tlo; lt < thi; ++lt) {
        const uint64_t tstart = gs + (lt - tf) * (uint64_t)kRepTile, gend = ge;
        const uint64_t base = tstart + (uint64_t)tid * kTileBpt;
        if (have) {
            ra = pa;
            rb = pb;
            rn = pn;
        } else if (tstart + (uint64_t)kRepTile + 16 <= m.data_end) {
            ra = *reinterpret_cast<const uint4*>(seq + base);
            rb = *reinterpret_cast<const uint4*>(seq + base + 16);
            rn = *reinterpret_cast<const uint4*>(seq + base + 32);
        } else {
            ra = load16(seq, base, gend);
            rb = load16(seq, base + 16, gend);
            rn = load16(seq, base + 32, gend);
        }
        const uint32_t tma = tail_mask(base, gend), tmb = tail_mask(base + 16, gend),
                       tmn = tail_mask(base + 32, gend);
        lds_barrier();   // rep zeroed, previous tile's copy-out done with `sorted`

        // 1. rank every k-mer inside (bucket, replica).  Branch-free: a window with a
        //    non-ACGT byte (code ~0) counts in the dummy row NBK and is scattered into the
        //    dummy slots past CAP.  The codes are recomputed from the 48 bytes in the scatter
        //    instead of being kept (register pressure).
        uint32_t rk[kTileBpt / 2];   // ranks (< 1024), two per register
        {
            uint32_t km[kTileBpt];
            visit_raw<K>(ra, rb, rn, tma, tmb, tmn, km);
#pragma unroll
            for (int j = 0; j < kTileBpt; j += 2) {
                const uint32_t b0 = min(km[j] >> kSubBits, (uint32_t)NBK);
                const uint32_t b1 = min(km[j + 1] >> kSubBits, (uint32_t)NBK);
                const uint32_t x0 = atomicAdd(&rep[b0 * kRep + r], 1u);
                const uint32_t x1 = atomicAdd(&rep[b1 * kRep + r], 1u);
                rk[j >> 1] = x0 | (x1 << 16);
            }
        }
        // opaque to the compiler: the scatter recomputes the codes instead of keeping 32
        // registers alive across the scan
        __asm__ __volatile__("" : "+v"(ra.x), "+v"(ra.y), "+v"(ra.z), "+v"(ra.w), "+v"(rb.x), "+v"(rb.y),
                             "+v"(rb.z), "+v"(rb.w), "+v"(rn.x), "+v"(rn.y), "+v"(rn.z), "+v"(rn.w));
        // prefetch the next tile behind this tile's LDS phases
        have = false;
        if (lt + 1 < thi) {
            advance(lt + 1);
            const uint64_t ns = gs + (lt + 1 - tf) * (uint64_t)kRepTile;
            if (ns + (uint64_t)kRepTile + 16 <= m.data_end) {
                const uint64_t nb = ns + (uint64_t)tid * kTileBpt;
                pa = *reinterpret_cast<const uint4*>(seq + nb);
                pb = *reinterpret_cast<const uint4*>(seq + nb + 16);
                pn = *reinterpret_cast<const uint4*>(seq + nb + 32);
                have = true;
            }
        }
        lds_barrier();

        // 2a. per bucket: exclusive replica prefixes in place, bucket sizes to bst.  Thread
        //     t owns replicas 16 (t & 1) .. + 15 of bucket t >> 1 (four 16-byte reads).
        constexpr int HALF = kRep / 2;
        uint4* mine = rep4 + (size_t)tid * (HALF / 4);
        if (tid < 2 * NBK) {
            uint4 q[HALF / 4];
            uint32_t run = 0u;
#pragma unroll
            for (int c = 0; c < HALF / 4; ++c) {
                q[c] = mine[c];
                const uint32_t x0 = q[c].x, x1 = q[c].y, x2 = q[c].z, x3 = q[c].w;
                q[c] = make_uint4(run, run + x0, run + x0 + x1, run + x0 + x1 + x2);
                run += x0 + x1 + x2 + x3;
            }
            const uint32_t other = __shfl_xor(run, 1);          // the partner half's total
            const uint32_t add = (tid & 1) ? other : 0u;
#pragma unroll
            for (int c = 0; c < HALF / 4; ++c)
                mine[c] = make_uint4(q[c].x + add, q[c].y + add, q[c].z + add, q[c].w + add);
            if (!(tid & 1)) bst[tid >> 1] = run + other;
        }
        lds_barrier();

        // 2b. bucket starts: exclusive scan of the chunk-padded bucket sizes
        const uint32_t nbk = tid < NBK ? bst[tid] : 0u;
        const uint32_t v = (nbk + 7u) & ~7u;
        uint32_t incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        if (lane == 63) wsum[wave] = incl;
        lds_barrier();
        uint32_t pre = 0u, total = 0u;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            pre += (q < wave) ? wsum[q] : 0u;
            total += wsum[q];
        }
        const uint32_t start = pre + incl - v;
        if (tid < NBK) {
            bst[tid] = start;
            toff[(uint64_t)tid * ldt + lt] = (uint16_t)(start >> 3);
        }
        if (tid == 0) toff[(uint64_t)NBK * ldt + lt] = (uint16_t)(total >> 3);
        lds_barrier();

        // 2c. segment start of every (bucket, replica)
        if (tid < 2 * NBK) {
            const uint32_t add = bst[tid >> 1];
#pragma unroll
            for (int c = 0; c < HALF / 4; ++c) {
                const uint4 x = mine[c];
                mine[c] = make_uint4(x.x + add, x.y + add, x.z + add, x.w + add);
            }
        }
        lds_barrier();

        // 3. scatter the suffixes; pad every bucket's segment to its chunk boundary
        //    (groups of 8: eight start reads in flight, then eight stores -- the compiler
        //    would otherwise wait for every read, stores included, one k-mer at a time)
        uint32_t km[kTileBpt];
        visit_raw<K>(ra, rb, rn, tma, tmb, tmn, km);
#pragma unroll
        for (int j0 = 0; j0 < kTileBpt; j0 += 8) {
            uint32_t pos[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t b = min(km[j0 + j] >> kSubBits, (uint32_t)NBK);
                pos[j] = rep[b * kRep + r];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t c = km[j0 + j];
                const uint32_t rank = (rk[(j0 + j) >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                sorted[(c >> kSubBits) < (uint32_t)NBK ? pos[j] + rank : (uint32_t)CAP + (uint32_t)lane] =
                    (uint16_t)(c & (kSubBins - 1));
            }
        }
        if (tid < NBK) {
#pragma unroll
            for (uint32_t q = 0; q < 7u; ++q) {
                const uint32_t at = start + nbk + q;
                if (nbk + q < v) sorted[at] = (uint16_t)(kPadBase + ((8u * (uint32_t)tid + at) & (kPadBins - 1)));
            }
        }
        lds_barrier();

        // 4. write the tile out; zero the counters for the next tile
        uint4* dst = reinterpret_cast<uint4*>(suf + lt * (uint64_t)CAP);
        const uint4* src = reinterpret_cast<const uint4*>(sorted);
        const uint32_t nchunk = total >> 3;
#pragma unroll 1
        for (uint32_t c = tid; c < nchunk; c += kRepThreads) store_nt(&dst[c], src[c]);
        for (int i = tid; i < (NBK + 1) * kRep / 4; i += kRepThreads) rep4[i] = make_uint4(0u, 0u, 0u, 0u);
    }
}

// Fixed-capacity variant (k = 12 default): every bucket owns a row of FC suffix slots in
// LDS, so one returning LDS add per k-mer yields both the bucket count and the k-mer's
// rank, and the suffix is stored at row[bucket][rank] -- two LDS operations per k-mer
// instead of three (histogram add, rank add, store).  The rows are then copied out as the
// same padded, bucket-ordered segments k_partition writes (one thread per bucket, 16-byte
// chunks).  If any bucket of the tile exceeds FC entries (uniform data: ~1e-8 per bucket;
// repeats make it likelier) the tile is redone in place with the exact three-pass scheme.
// Measured (experiment, KMH_FC=1): 126 us per 100 Mbp genome vs 97 us for k_partition --
// the 117 KiB of rows leave one workgroup per CU, and the phase overlap of two co-resident
// k_partition workgroups is worth more than the saved LDS operation.  Not the default.
template <int K, int TPB, int FC>
__global__ __launch_bounds__(TPB) void k_partition_fc(const uint8_t* __restrict__ seq,
                                                      GenomeMap m, uint16_t* __restrict__ suf,
                                                      uint16_t* __restrict__ toff, uint32_t ldt) {
    constexpr int NBK = num_buckets<K>();
    constexpr int TILE = TPB * kTileBpt;
    constexpr int CAP = tile_cap<K>(TILE);
    static_assert(FC % 8 == 0 && NBK * FC >= CAP, "rows hold whole chunks; the exact path reuses them");
    static_assert(NBK <= TPB, "one bucket per thread");
    __shared__ __attribute__((aligned(16))) uint16_t rows[NBK * FC];
    __shared__ uint32_t cnt[NBK];
    __shared__ uint32_t wsum[TPB / 64];
    __shared__ uint32_t over;
    __shared__ uint16_t cmap[CAP / 8];   // output chunk -> bucket

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = xcd_work_id();
    const uint64_t gt = m.tile_lo + lt;
    const int g = find_genome(m, gt);
    const uint64_t tstart = m.goff[g] + (gt - m.tbase[g]) * (uint64_t)TILE;
    const uint64_t ge = m.goff[g + 1];

    if (tid < NBK) cnt[tid] = 0u;
    if (tid == 0) over = 0u;
    __syncthreads();

    uint32_t km[kTileBpt];
    walk<K>(seq, m, tstart, ge, TPB, [&](int j, uint32_t code, bool ok) {
        km[j] = ok ? code : 0xFFFFFFFFu;
        if (ok) {
            const uint32_t b = code >> kSubBits;
            const uint32_t r = atomicAdd(&cnt[b], 1u);
            if (r < (uint32_t)FC) rows[b * FC + r] = (uint16_t)(code & (kSubBins - 1));
            else over = 1u;
        }
    });
    __syncthreads();
    const bool exact = over != 0u;   // cnt holds the exact histogram either way

    // Exclusive scan of the padded bucket sizes -> segment starts (entries).
    const uint32_t nb = tid < NBK ? cnt[tid] : 0u;
    const uint32_t v = (nb + 7u) & ~7u;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, total = 0u;
#pragma unroll
    for (int w = 0; w < TPB / 64; ++w) {
        pre += (w < wave) ? wsum[w] : 0u;
        total += wsum[w];
    }
    const uint32_t start = pre + incl - v;
    if (tid < NBK) toff[(uint64_t)tid * ldt + lt] = (uint16_t)(start >> 3);
    if (tid == 0) toff[(uint64_t)NBK * ldt + lt] = (uint16_t)(total >> 3);

    uint4* dst = reinterpret_cast<uint4*>(suf + lt * (uint64_t)CAP);
    if (!exact) {
        // Each bucket pads its own row up to a whole chunk and marks its chunks in cmap; then
        // every thread copies chunks c = tid, tid + TPB, ... so a wave's stores are contiguous.
        if (tid < NBK) {
            for (uint32_t q = nb; q < v; ++q)
                rows[tid * FC + q] = (uint16_t)(kPadBase + ((8u * (uint32_t)tid + start + q) & (kPadBins - 1)));
            for (uint32_t c = start >> 3; c < (start + v) >> 3; ++c) cmap[c] = (uint16_t)tid;
            cnt[tid] = start >> 3;    // cnt now holds each bucket's first output chunk
        }
        __syncthreads();
        for (uint32_t c = tid; c < (total >> 3); c += TPB) {
            const uint32_t b = cmap[c];
            dst[c] = reinterpret_cast<const uint4*>(rows + b * FC)[c - cnt[b]];
        }
        return;
    }
    // Exact path: scatter into the packed layout (rows reused as the tile buffer), pad,
    // then one coalesced store of the tile.
    uint16_t* sorted = rows;
    if (tid < NBK) cnt[tid] = start;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kTileBpt; ++j) {
        const uint32_t c = km[j];
        if (c != 0xFFFFFFFFu) sorted[atomicAdd(&cnt[c >> kSubBits], 1u)] = (uint16_t)(c & (kSubBins - 1));
    }
    if (tid < NBK)
        for (uint32_t q = start + nb; q < start + v; ++q)
            sorted[q] = (uint16_t)(kPadBase + ((8u * (uint32_t)tid + q) & (kPadBins - 1)));
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(sorted);
    for (uint32_t c = tid; c < (total >> 3); c += TPB) dst[c] = src[c];
}

// Add one 16-byte chunk (8 suffixes) into the LDS table; padding entries land in the
// dummy bins past kSubBins.
__device__ __forceinline__ void count8(uint32_t* tbl, uint4 q) {
    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) atomicAdd(&tbl[(wd[i >> 1] >> (16 * (i & 1))) & 0xFFFFu], 1u);
}

// One workgroup per (genome, bucket[, split]): gathers the bucket's segment from every
// tile of the genome into a 32768-bin LDS histogram, then writes the row slice once.
// Each wave takes 64 tiles at a time (one per lane; their segment bounds are consecutive
// u16s of the bucket-major offset table), prefix-sums their chunk counts and lists every
// chunk in a per-wave LDS queue; the queue is then streamed with all 64 lanes active:
// U coalesced 16-byte loads in flight per lane, 8 LDS atomics per load.  A batch whose
// chunks overflow the queue (skewed input) is walked lane by lane instead.
// Ablation bits (experiments only): 1 = no LDS atomics, 2 = no suffix loads, 4 = no main
// loop (table zeroing, offset reads and the row store only).
template <int K, int GS, int U, int TILE, int ABL, int PIPE>
__global__ __launch_bounds__(kCountThreads) void k_bucket_count(
    const uint16_t* __restrict__ suf, const uint16_t* __restrict__ toff, uint32_t ldt,
    GenomeMap m, int S, uint32_t* __restrict__ out) {
    constexpr int NBK = num_buckets<K>();
    constexpr int CAP = tile_cap<K>(TILE);
    constexpr uint32_t CPT = CAP / 8;            // chunks per tile in the suffix buffer
    constexpr int NW = kCountThreads / 64;
    constexpr int QMAX = U * 64;                 // queue entries per wave: one load round
    __shared__ __attribute__((aligned(16))) uint32_t tbl[kSubBins + kPadBins];
    __shared__ uint32_t queue[NW][QMAX];

    const uint32_t w = xcd_work_id();
    const int s = (int)(w % (uint32_t)S);
    const uint32_t b = (w / (uint32_t)S) % NBK;
    const int g = m.g0 + (int)(w / ((uint32_t)S * NBK));
    const uint64_t t0 = m.tbase[g] - m.tile_lo, nt = m.tbase[g + 1] - m.tbase[g];
    const uint64_t ta = t0 + nt * (uint64_t)s / (uint64_t)S;
    const uint64_t tb = t0 + nt * (uint64_t)(s + 1) / (uint64_t)S;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint4* chunks = reinterpret_cast<const uint4*>(suf);

    uint4* tbl4 = reinterpret_cast<uint4*>(tbl);
    for (int i = threadIdx.x; i < (kSubBins + (int)kPadBins) / 4; i += kCountThreads) tbl4[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();

    if constexpr (PIPE) {
        // Two-stage software pipeline over 32-tile batches: while batch i's loads are in
        // flight, batch i+1's queue is built and its loads issued; then batch i's atomics.
        constexpr int BT = 32;                    // tiles per wave batch
        constexpr int QH = QMAX / 2;              // queue entries per stage (U/2 rounds)
        constexpr int UH = QH / 64;
        const uint64_t stride = (uint64_t)NW * BT;
        auto bounds = [&](uint64_t tw, uint32_t& lo, uint32_t& hi) {
            const uint64_t t = tw + (uint64_t)lane;
            const bool in = lane < BT && t < tb;
            lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
            hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
        };
        // list the chunks of batch tw in queue slot `slot`; returns the chunk count
        auto build = [&](uint64_t tw, uint32_t lo, uint32_t hi, uint32_t* qs, uint32_t& cb,
                         uint32_t& nc) -> uint32_t {
            nc = hi - lo;
            uint32_t incl = nc;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t x = __shfl_up(incl, d);
                if (lane >= d) incl += x;
            }
            const uint32_t total = __shfl(incl, 63);
            cb = (uint32_t)(tw + (uint64_t)lane) * CPT + lo;
            if (total <= (uint32_t)QH) {
                const uint32_t ex = incl - nc;
                for (uint32_t j = 0; j < nc; ++j) qs[ex + j] = cb + j;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            return total;
        };
        auto issue = [&](const uint32_t* qs, uint32_t total, uint4 (&v)[UH]) {
#pragma unroll
            for (int u = 0; u < UH; ++u) {
                const uint32_t e = (uint32_t)(u * 64 + lane);
                const uint32_t ci = (total <= (uint32_t)QH && e < total) ? qs[e] : 0u;
                v[u] = chunks[ci];
            }
        };
        auto consume = [&](const uint4 (&v)[UH], uint32_t total, uint32_t cb, uint32_t nc) {
            if (total <= (uint32_t)QH) {
#pragma unroll
                for (int u = 0; u < UH; ++u)
                    if ((uint32_t)(u * 64 + lane) < total) count8(tbl, v[u]);
            } else {
                for (uint32_t j = 0; j < nc; ++j) count8(tbl, chunks[cb + j]);
            }
        };
        uint32_t* qbase = queue[wave];
        uint64_t tw = ta + (uint64_t)wave * BT;
        if (tw < tb) {
            uint32_t lo, hi, lo_n = 0, hi_n = 0;
            bounds(tw, lo, hi);
            if (tw + stride < tb) bounds(tw + stride, lo_n, hi_n);
            uint32_t cb, nc;
            int slot = 0;
            uint32_t tot = build(tw, lo, hi, qbase, cb, nc);
            uint4 v[UH];
            issue(qbase, tot, v);
            for (; tw < tb; tw += stride) {
                const uint64_t twn = tw + stride;
                uint4 vn[UH];
                uint32_t tot_n = 0, cb_n = 0, nc_n = 0;
                uint32_t* qn = qbase + (slot ^ 1) * QH;
                if (twn < tb) {
                    tot_n = build(twn, lo_n, hi_n, qn, cb_n, nc_n);
                    issue(qn, tot_n, vn);
                    if (twn + stride < tb) bounds(twn + stride, lo_n, hi_n);
                }
                consume(v, tot, cb, nc);
#pragma unroll
                for (int u = 0; u < UH; ++u) v[u] = vn[u];
                tot = tot_n;
                cb = cb_n;
                nc = nc_n;
                slot ^= 1;
            }
        }
    } else {
        constexpr int BT = batch_tiles<K>(TILE, QMAX);
        uint32_t* q = queue[wave];
        // segment bounds of this lane's tile in batch tw (prefetched one batch ahead)
        auto bounds = [&](uint64_t tw, uint32_t& lo, uint32_t& hi) {
            const uint64_t t = tw + (uint64_t)lane;
            const bool in = lane < BT && t < tb;
            lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
            hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
        };
        uint32_t lo_n = 0, hi_n = 0;
        uint64_t tw = ta + (uint64_t)wave * BT;
        if (tw < tb) bounds(tw, lo_n, hi_n);
        for (; tw < tb; tw += (uint64_t)NW * BT) {
            const uint32_t lo = lo_n, nc = hi_n - lo_n;
            if (ABL & 4) {
                asm volatile("" ::"v"(nc));
                if (tw + (uint64_t)NW * BT < tb) bounds(tw + (uint64_t)NW * BT, lo_n, hi_n);
                continue;
            }
            uint32_t incl = nc;
    #pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t x = __shfl_up(incl, d);
                if (lane >= d) incl += x;
            }
            const uint32_t total = __shfl(incl, 63);
            const uint32_t cbase = (uint32_t)(tw + (uint64_t)lane) * CPT + lo;  // segment's first chunk
            if (total <= (uint32_t)QMAX) {
                const uint32_t ex = incl - nc;
                for (uint32_t j = 0; j < nc; ++j) q[ex + j] = cbase + j;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                uint4 v[U];
    #pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t e = (uint32_t)(u * 64 + lane);
                    const uint32_t ci = e < total ? q[e] : 0u;  // idle lanes re-read chunk 0
                    if (ABL & 2) {
                        const uint32_t x = ci * 2654435761u;
                        v[u] = make_uint4(x & 0x7FFF7FFFu, (x * 3u) & 0x7FFF7FFFu, (x * 5u) & 0x7FFF7FFFu, (x * 7u) & 0x7FFF7FFFu);
                    } else {
                        v[u] = chunks[ci];
                    }
                }
                // next batch's bounds load behind this batch's data loads
                if (tw + (uint64_t)NW * BT < tb) bounds(tw + (uint64_t)NW * BT, lo_n, hi_n);
    #pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (ABL & 1) asm volatile("" ::"v"(v[u].x ^ v[u].y ^ v[u].z ^ v[u].w));
                    else if ((uint32_t)(u * 64 + lane) < total) count8(tbl, v[u]);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            } else {
                if (tw + (uint64_t)NW * BT < tb) bounds(tw + (uint64_t)NW * BT, lo_n, hi_n);
                for (uint32_t j = 0; j < nc; ++j) count8(tbl, chunks[cbase + j]);
            }
        }
    }
    __syncthreads();

    uint32_t* orow = out + (uint64_t)g * (1ull << (2 * K)) + (uint64_t)b * kSubBins;
    if (S == 1) {
        uint4* o4 = reinterpret_cast<uint4*>(orow);
        for (int i = threadIdx.x; i < kSubBins / 4; i += kCountThreads) store_nt(&o4[i], tbl4[i]);
    } else if (ta < tb) {
        for (int i = threadIdx.x; i < kSubBins; i += kCountThreads) {
            const uint32_t x = tbl[i];
            if (x) atomicAdd(&orow[i], x);
        }
    }
}

// ---------------------------------------------------------------- u16 count tables
// Bins are packed two per 32-bit LDS word (bin v in half v & 1 of word v >> 1), halving
// the table so that two count workgroups -- or a count and a partition workgroup -- fit on
// one CU.  Exactness: every wrap of a 16-bit half is seen by exactly one ds_add_rtn (the
// adds to a word are serialised), which appends a correction to a global log:
//   low add, old low == 0xFFFF:  bin v += 65536, and its partner v ^ 1 got a carry: -= 1;
//                                if old high == 0xFFFF too, the carry wrapped it: += 65536
//   high add, old high == 0xFFFF: bin v += 65536
// so for every bin: count = stored half + sum of its logged corrections (mod 2^32), applied
// by k_fixup after the count kernel.  Random genomes never wrap; the log stays empty.
struct FixLog {
    unsigned long long* entries;  // (row index << 1) | (1 = "-1", 0 = "+65536")
    uint32_t* cursor;
    uint32_t cap;
};

__device__ __forceinline__ void log_fix(const FixLog& L, uint64_t idx, uint32_t minus_one) {
    const uint32_t at = atomicAdd(L.cursor, 1u);
    if (at < L.cap) L.entries[at] = (idx << 1) | minus_one;
}

__device__ __forceinline__ void count8_u16(uint32_t* tbl, uint4 q, const FixLog& L,
                                           uint64_t row0) {
    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t v = (wd[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        const uint32_t hi = v & 1u;
        const uint32_t old = atomicAdd(&tbl[v >> 1], hi ? 0x10000u : 1u);
        const bool wrap = hi ? (old >> 16) == 0xFFFFu : (old & 0xFFFFu) == 0xFFFFu;
        if (wrap && v < kPadBase) {  // rare: log the corrections
            log_fix(L, row0 + v, 0u);
            if (!hi) {
                log_fix(L, row0 + (v ^ 1u), 1u);
                if ((old >> 16) == 0xFFFFu) log_fix(L, row0 + (v ^ 1u), 0u);
            }
        }
    }
}

// Same work decomposition as k_bucket_count (per-wave chunk queue), NT threads, u16 table.
template <int K, int U, int TILE, int NT>
__global__ __launch_bounds__(NT) void k_bucket_count16(
    const uint16_t* __restrict__ suf, const uint16_t* __restrict__ toff, uint32_t ldt,
    GenomeMap m, int S, uint32_t* __restrict__ out, FixLog L) {
    constexpr int NBK = num_buckets<K>();
    constexpr int CAP = tile_cap<K>(TILE);
    constexpr uint32_t CPT = CAP / 8;
    constexpr int NW = NT / 64;
    constexpr int QMAX = U * 64;
    constexpr int WORDS = (kSubBins + (int)kPadBins) / 2;
    __shared__ __attribute__((aligned(16))) uint32_t tbl[WORDS];
    __shared__ uint32_t queue[NW][QMAX];

    const uint32_t w = xcd_work_id();
    const int s = (int)(w % (uint32_t)S);
    const uint32_t b = (w / (uint32_t)S) % NBK;
    const int g = m.g0 + (int)(w / ((uint32_t)S * NBK));
    const uint64_t t0 = m.tbase[g] - m.tile_lo, nt = m.tbase[g + 1] - m.tbase[g];
    const uint64_t ta = t0 + nt * (uint64_t)s / (uint64_t)S;
    const uint64_t tb = t0 + nt * (uint64_t)(s + 1) / (uint64_t)S;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint4* chunks = reinterpret_cast<const uint4*>(suf);
    const uint64_t row0 = (uint64_t)g * (1ull << (2 * K)) + (uint64_t)b * kSubBins;

    uint4* tbl4 = reinterpret_cast<uint4*>(tbl);
    for (int i = threadIdx.x; i < WORDS / 4; i += NT) tbl4[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();

    constexpr int BT = batch_tiles<K>(TILE, QMAX);
    uint32_t* q = queue[wave];
    auto bounds = [&](uint64_t tw, uint32_t& lo, uint32_t& hi) {
        const uint64_t t = tw + (uint64_t)lane;
        const bool in = lane < BT && t < tb;
        lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
        hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
    };
    uint32_t lo_n = 0, hi_n = 0;
    uint64_t tw = ta + (uint64_t)wave * BT;
    if (tw < tb) bounds(tw, lo_n, hi_n);
    for (; tw < tb; tw += (uint64_t)NW * BT) {
        const uint32_t lo = lo_n, nc = hi_n - lo_n;
        uint32_t incl = nc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        const uint32_t total = __shfl(incl, 63);
        const uint32_t cbase = (uint32_t)(tw + (uint64_t)lane) * CPT + lo;
        if (total <= (uint32_t)QMAX) {
            const uint32_t ex = incl - nc;
            for (uint32_t j = 0; j < nc; ++j) q[ex + j] = cbase + j;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t e = (uint32_t)(u * 64 + lane);
                v[u] = chunks[e < total ? q[e] : 0u];
            }
            if (tw + (uint64_t)NW * BT < tb) bounds(tw + (uint64_t)NW * BT, lo_n, hi_n);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if ((uint32_t)(u * 64 + lane) < total) count8_u16(tbl, v[u], L, row0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            if (tw + (uint64_t)NW * BT < tb) bounds(tw + (uint64_t)NW * BT, lo_n, hi_n);
            for (uint32_t j = 0; j < nc; ++j) count8_u16(tbl, chunks[cbase + j], L, row0);
        }
    }
    __syncthreads();

    // Expand u16 pairs to the u32 row (plain stores, or adds when split).
    uint32_t* orow = out + row0;
    for (int i = threadIdx.x; i < kSubBins / 8; i += NT) {
        const uint4 x = tbl4[i];
        const uint4 lo4 = make_uint4(x.x & 0xFFFFu, x.x >> 16, x.y & 0xFFFFu, x.y >> 16);
        const uint4 hi4 = make_uint4(x.z & 0xFFFFu, x.z >> 16, x.w & 0xFFFFu, x.w >> 16);
        if (S == 1) {
            reinterpret_cast<uint4*>(orow)[2 * i] = lo4;
            reinterpret_cast<uint4*>(orow)[2 * i + 1] = hi4;
        } else if (ta < tb) {
            const uint32_t e[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (e[j]) atomicAdd(&orow[8 * i + j], e[j]);
        }
    }
}

// Apply the logged u16-wrap corrections (usually none).
__global__ __launch_bounds__(256) void k_fixup(FixLog L, uint32_t* __restrict__ out) {
    const uint32_t n = min(*L.cursor, L.cap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned long long e = L.entries[i];
        atomicAdd(&out[e >> 1], (e & 1ull) ? 0xFFFFFFFFu : 65536u);
    }
}

// ---------------------------------------------------------------- first occurrence
template <int K>
__global__ __launch_bounds__(kTileThreads) void k_first(const uint8_t* __restrict__ seq,
                                                        GenomeMap m,
                                                        uint32_t* __restrict__ first) {
    const uint64_t gt = m.tile_lo + blockIdx.x;
    const int g = find_genome(m, gt);
    const uint64_t gs = m.goff[g];
    const uint64_t rel = (gt - m.tbase[g]) * (uint64_t)kTile + (uint64_t)threadIdx.x * kTileBpt;
    uint32_t* frow = first + (uint64_t)g * (1ull << (2 * K));
    walk<K>(seq, m, gs + (gt - m.tbase[g]) * (uint64_t)kTile, m.goff[g + 1], kTileThreads,
            [&](int j, uint32_t code, bool ok) {
                if (ok) atomicMin(&frow[code], (uint32_t)(rel + (uint64_t)j));
            });
}

// ---------------------------------------------------------------- synthetic genomes
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ out, uint64_t len,
                                               uint64_t stride, uint64_t seed0, int G) {
    const uint64_t wpg = (len + 31) / 32;
    const uint64_t total = wpg * (uint64_t)G;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = idx / wpg, wi = idx % wpg;
        const uint64_t r = splitmix64(splitmix64(seed0 + g) + wi);
        uint8_t* dst = out + g * stride + wi * 32;
        if (wi * 32 + 32 <= len && ((uintptr_t)dst & 15u) == 0u) {
            uint32_t q[8];
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                const uint32_t x = (uint32_t)(r >> (8 * d)) & 0xFFu;
                const uint32_t sel = (x | (x << 6) | (x << 12) | (x << 18)) & 0x03030303u;
                q[d] = __builtin_amdgcn_perm(0u, 0x54474341u, sel);
            }
            reinterpret_cast<uint4*>(dst)[0] = make_uint4(q[0], q[1], q[2], q[3]);
            reinterpret_cast<uint4*>(dst)[1] = make_uint4(q[4], q[5], q[6], q[7]);
        } else {
            for (int i = 0; i < 32 && wi * 32 + i < len; ++i)
                dst[i] = "ACGT"[(r >> (2 * i)) & 3u];
        }
    }
}

// ---------------------------------------------------------------- host side
template <int K>
int run_direct(Ctx* ctx, const uint8_t* d_seq, const Layout& L, const uint64_t* d_goff,
               const uint64_t* d_tbase, int G, uint32_t* d_out, hipStream_t s) {
    const size_t row = (size_t)1 << (2 * K);
    KMH_HIP(ctx, hipMemsetAsync(d_out, 0, row * (size_t)G * sizeof(uint32_t), s));
    // Spans per genome: fill ~kTargetWorkgroups*2 workgroups, at most one per tile.
    uint64_t maxt = 0;
    for (int g = 0; g < G; ++g) maxt = std::max<uint64_t>(maxt, L.tbase[g + 1] - L.tbase[g]);
    if (maxt == 0) return KMH_OK;
    const uint64_t want = (2 * (uint64_t)kTargetWorkgroups + G - 1) / G;
    const int S = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, maxt));
    GenomeMap m{d_goff, d_tbase, 0, G, 0, L.goff[G]};
    time_begin(ctx, s, "k_direct");
    hipLaunchKernelGGL(k_direct<K>, dim3((unsigned)(G * S)), dim3(kDirectThreads), 0, s, d_seq,
                       m, S, d_out);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

template <int K, int TPB, int PABL, int CABL, int GSX = 0, int UX = 0, int PIPE = 0, int SUBT = 1,
          int FCAP = 0, int REP = 0>
int run_partitioned(Ctx* ctx, const uint8_t* d_seq, const Layout& L, const uint64_t* d_goff,
                    const uint64_t* d_tbase, int G, uint32_t* d_out, hipStream_t s) {
    constexpr int NBK = num_buckets<K>();
    constexpr int TILE = REP ? kRepTile : TPB * kTileBpt * SUBT;
    constexpr int CAP = tile_cap<K>(TILE);
    constexpr int GS0 = TILE / NBK / 8;   // lanes per segment: one 16-B chunk each
    constexpr int GS1 = GS0 < 1 ? 1 : (GS0 > 64 ? 64 : GS0);
    constexpr int GS = GSX ? GSX : GS1;
    constexpr int U = UX ? UX : 6;        // chunk loads in flight per lane (queue = 64 U)
    const size_t row = (size_t)1 << (2 * K);
    // Genomes per batch: keep the suffix buffer of one batch within the budget.  Measured
    // (profiles/r01_batch.txt): batches larger than the 256 MiB Infinity Cache are faster --
    // the exchange re-read from HBM costs less than the launch tails and kernel boundaries
    // of one-genome launches (config 3: 11.0 ms per step at 256 MiB, 9.2 ms at 4 GiB = 18
    // genomes per launch).  KMH_SUF_BUDGET_MB overrides.
    const size_t budget = env_mb("KMH_SUF_BUDGET_MB", 4096) << 20;
    const size_t tile_bytes = (size_t)CAP * sizeof(uint16_t);
    // Two suffix/offset buffers when KMH_OVERLAP=1 (experiment): the partition of batch i+1
    // (side stream) overlaps the count of batch i (caller's stream).
    const bool overlap = env_long("KMH_OVERLAP", 0) != 0;
    uint64_t max_batch_tiles = 0;
    {
        int g = 0;
        while (g < G) {
            int h = g;
            uint64_t tiles = 0;
            do {
                tiles += L.tbase[h + 1] - L.tbase[h];
                ++h;
            } while (h < G && (tiles + (L.tbase[h + 1] - L.tbase[h])) * tile_bytes <= budget);
            max_batch_tiles = std::max(max_batch_tiles, tiles);
            g = h;
        }
    }
    const size_t slot_tiles = std::max<uint64_t>(max_batch_tiles, 1);
    const size_t nslots = overlap ? 2 : 1;
    int rc = ensure(ctx, ctx->suf, nslots * slot_tiles * tile_bytes);
    if (rc) return rc;
    const uint32_t ldt = (uint32_t)((slot_tiles + 63) / 64 * 64);
    const size_t toff_slot = (size_t)ldt * (NBK + 1);
    rc = ensure(ctx, ctx->toff, nslots * toff_slot * sizeof(uint16_t));
    if (rc) return rc;
    // u16-packed count tables (KMH_COUNT16=1; KMH_COUNT16_NT=512|1024): half the LDS, same
    // speed here; kept for co-residency experiments.  Default: the u32 kernel.
    const bool c16 = env_long("KMH_COUNT16", 0) != 0;
    const int c16nt = env_long("KMH_COUNT16_NT", 512) == 1024 ? 1024 : 512;
    FixLog fl{nullptr, nullptr, 0};
    if (c16) {
        const uint64_t windows = (uint64_t)L.ntiles * (uint64_t)TILE;
        const uint64_t cap = 3 * (windows / 65536 + 1) + 64;  // >= every possible wrap event
        rc = ensure(ctx, ctx->fix, 256 + cap * sizeof(unsigned long long));
        if (rc) return rc;
        fl.cursor = static_cast<uint32_t*>(ctx->fix.ptr);
        fl.entries = reinterpret_cast<unsigned long long*>(static_cast<char*>(ctx->fix.ptr) + 256);
        fl.cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFF0ull);
        KMH_HIP(ctx, hipMemsetAsync(fl.cursor, 0, 256, s));
    }
    hipStream_t sp = s;
    if (overlap) {
        if (!ctx->side) KMH_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
        for (auto& e : ctx->pipe_ev)
            if (!e) KMH_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        sp = ctx->side;
        KMH_HIP(ctx, hipEventRecord(ctx->pipe_ev[0], s));  // inputs ready
        KMH_HIP(ctx, hipStreamWaitEvent(sp, ctx->pipe_ev[0], 0));
    }

    int g = 0, batch = 0;
    while (g < G) {
        int h = g;
        uint64_t tiles = 0;
        do {
            tiles += L.tbase[h + 1] - L.tbase[h];
            ++h;
        } while (h < G && (tiles + (L.tbase[h + 1] - L.tbase[h])) * tile_bytes <= budget);
        const int nG = h - g;
        const int slot = overlap ? (batch & 1) : 0;
        uint16_t* suf = static_cast<uint16_t*>(ctx->suf.ptr) + (size_t)slot * slot_tiles * CAP;
        uint16_t* toff = static_cast<uint16_t*>(ctx->toff.ptr) + (size_t)slot * toff_slot;
        GenomeMap m{d_goff, d_tbase, g, h, L.tbase[g], L.goff[G]};
        uint64_t maxt = 0;
        for (int q = g; q < h; ++q) maxt = std::max<uint64_t>(maxt, L.tbase[q + 1] - L.tbase[q]);
        const uint64_t want = ((uint64_t)kTargetWorkgroups + (uint64_t)nG * NBK - 1) / ((uint64_t)nG * NBK);
        const int S = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, std::max<uint64_t>(maxt, 1)));
        if (S > 1) KMH_HIP(ctx, hipMemsetAsync(d_out + (size_t)g * row, 0, (size_t)nG * row * sizeof(uint32_t), s));
        if (overlap && batch >= 2) KMH_HIP(ctx, hipStreamWaitEvent(sp, ctx->pipe_ev[3 + slot], 0));
        if (tiles) {
            if constexpr (REP) {
                const unsigned pgrid = (unsigned)std::min<uint64_t>(tiles, (uint64_t)std::max(1, ctx->num_cu));
                time_begin(ctx, sp, "k_partition_rep");
                hipLaunchKernelGGL((k_partition_rep<K>), dim3(pgrid), dim3(kRepThreads), 0, sp,
                                   d_seq, m, suf, toff, ldt, (uint32_t)tiles);
            } else if constexpr (FCAP > 0) {
                time_begin(ctx, sp, "k_partition");
                hipLaunchKernelGGL((k_partition_fc<K, TPB, FCAP>), dim3((unsigned)tiles), dim3(TPB), 0, sp,
                                   d_seq, m, suf, toff, ldt);
            } else {
                time_begin(ctx, sp, "k_partition");
                hipLaunchKernelGGL((k_partition<K, TPB, PABL, SUBT>), dim3((unsigned)tiles), dim3(TPB), 0, sp,
                                   d_seq, m, suf, toff, ldt);
            }
            time_end(ctx, sp);
            KMH_HIP(ctx, hipGetLastError());
        }
        if (overlap) {
            KMH_HIP(ctx, hipEventRecord(ctx->pipe_ev[1 + slot], sp));
            KMH_HIP(ctx, hipStreamWaitEvent(s, ctx->pipe_ev[1 + slot], 0));
        }
        time_begin(ctx, s, "k_bucket_count");
        if (c16 && c16nt == 1024)
            hipLaunchKernelGGL((k_bucket_count16<K, U, TILE, 1024>), dim3((unsigned)(nG * NBK * S)),
                               dim3(1024), 0, s, suf, toff, ldt, m, S, d_out, fl);
        else if (c16)
            hipLaunchKernelGGL((k_bucket_count16<K, U, TILE, 512>), dim3((unsigned)(nG * NBK * S)),
                               dim3(512), 0, s, suf, toff, ldt, m, S, d_out, fl);
        else
            hipLaunchKernelGGL((k_bucket_count<K, GS, U, TILE, CABL, PIPE>), dim3((unsigned)(nG * NBK * S)),
                               dim3(kCountThreads), 0, s, suf, toff, ldt, m, S, d_out);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
        if (overlap) KMH_HIP(ctx, hipEventRecord(ctx->pipe_ev[3 + slot], s));
        g = h;
        ++batch;
    }
    if (c16) {
        time_begin(ctx, s, "k_fixup");
        hipLaunchKernelGGL(k_fixup, dim3(64), dim3(256), 0, s, fl, d_out);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
    }
    return KMH_OK;
}

template <int K>
int count_k(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, uint32_t* d_out,
            hipStream_t s) {
    Layout L;
    const uint64_t *d_goff, *d_tbase;
    if constexpr (K <= 9) {
        int rc = make_layout(ctx, offsets, G, K, kTile, L);
        if (!rc) rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
        if (rc) return rc;
        return run_direct<K>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
    } else {
        // Tile workgroup size (512 or 1024 threads); KMH_TPB overrides.  For k = 12,
        // KMH_ABLATE_P / KMH_ABLATE_C select ablation builds (experiments only: wrong
        // counts) -- see the ablation bits of k_partition / k_bucket_count.
        const int tpb = (int)env_mb("KMH_TPB", 512) == 1024 ? 1024 : 512;
        // k = 12: two 16384-window sub-tiles per partition tile (64-entry segments) unless
        // KMH_SUBT=1.
        const int subt = (K == 12 && tpb == 512 && env_long("KMH_SUBT", 2) == 2) ? 2 : 1;
        // KMH_PART=1 (experiment): the persistent replica-counter partition k_partition_rep.
        // Parity-tested, measured slower (134 vs 79 us per 100 Mbp genome).
        if (env_long("KMH_PART", 0) != 0) {
            int rc = make_layout(ctx, offsets, G, K, (uint64_t)kRepTile, L);
            if (!rc) rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
            if (rc) return rc;
            return run_partitioned<K, 1024, 0, 0, 0, 0, 0, 1, 0, 1>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
        }
        int rc = make_layout(ctx, offsets, G, K, (uint64_t)tpb * kTileBpt * subt, L);
        if (!rc) rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
        if (rc) return rc;
        if constexpr (K == 12) {
            const int pa = (int)env_mb("KMH_ABLATE_P", 0), ca = (int)env_mb("KMH_ABLATE_C", 0);
            if (pa || ca) {
                if (tpb != 512) return fail(ctx, KMH_ERR_INVALID, "ablations use KMH_TPB=512");
                if (pa == 1) return run_partitioned<K, 512, 1, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                if (pa == 2) return run_partitioned<K, 512, 2, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                if (pa == 4) return run_partitioned<K, 512, 4, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                if (ca == 1) return run_partitioned<K, 512, 0, 1, 0, 0, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                if (ca == 2) return run_partitioned<K, 512, 0, 2, 0, 0, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                if (ca == 4) return run_partitioned<K, 512, 0, 4, 0, 0, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                if (ca == 3) return run_partitioned<K, 512, 0, 3, 0, 0, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
                return fail(ctx, KMH_ERR_INVALID, "unknown ablation");
            }
        }
        if constexpr (K == 12) {
            // KMH_FC=1: fixed-capacity partition (1024-thread tiles of the same 32768 windows)
            if (env_long("KMH_FC", 0) == 1) {
                int rc2 = make_layout(ctx, offsets, G, K, (uint64_t)1024 * kTileBpt, L);
                if (!rc2) rc2 = upload_layout(ctx, L, s, &d_goff, &d_tbase);
                if (rc2) return rc2;
                return run_partitioned<K, 1024, 0, 0, 0, 0, 0, 1, 112>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
            }
            // KMH_FC=2: fixed-capacity partition on 512-thread, 16384-window tiles (64-entry
            // rows, 71 KiB of LDS: two workgroups per CU)
            if (env_long("KMH_FC", 0) == 2) {
                int rc2 = make_layout(ctx, offsets, G, K, (uint64_t)512 * kTileBpt, L);
                if (!rc2) rc2 = upload_layout(ctx, L, s, &d_goff, &d_tbase);
                if (rc2) return rc2;
                return run_partitioned<K, 512, 0, 0, 0, 0, 0, 1, 64>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
            }
            if (subt == 2) return run_partitioned<K, 512, 0, 0, 0, 0, 0, 2>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
        }
        if constexpr (K == 12) {  // sweep (experiments): KMH_GSU=6 unpipelined, 4 = U 4 pipelined
            const int gsu = (int)env_mb("KMH_GSU", 0);
            if (tpb == 512 && gsu == 6) return run_partitioned<K, 512, 0, 0, 0, 6, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
            if (tpb == 512 && gsu == 4) return run_partitioned<K, 512, 0, 0, 0, 4, 1>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
        }
        if (tpb == 1024) return run_partitioned<K, 1024, 0, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
        return run_partitioned<K, 512, 0, 0>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
    }
}

template <int K>
int first_k(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, uint32_t* d_first,
            hipStream_t s) {
    Layout L;
    const uint64_t *d_goff, *d_tbase;
    int rc = make_layout(ctx, offsets, G, K, kTile, L);
    if (!rc) rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
    if (rc) return rc;
    const size_t row = (size_t)1 << (2 * K);
    KMH_HIP(ctx, hipMemsetAsync(d_first, 0xFF, row * (size_t)G * sizeof(uint32_t), s));
    if (L.ntiles == 0) return KMH_OK;
    GenomeMap m{d_goff, d_tbase, 0, G, 0, L.goff[G]};
    time_begin(ctx, s, "k_first");
    hipLaunchKernelGGL(k_first<K>, dim3((unsigned)L.ntiles), dim3(kTileThreads), 0, s, d_seq, m,
                       d_first);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

#define KMH_DISPATCH_K(fn, k, ...)                      \
    switch (k) {                                        \
    case 1: return fn<1>(__VA_ARGS__);                  \
    case 2: return fn<2>(__VA_ARGS__);                  \
    case 3: return fn<3>(__VA_ARGS__);                  \
    case 4: return fn<4>(__VA_ARGS__);                  \
    case 5: return fn<5>(__VA_ARGS__);                  \
    case 6: return fn<6>(__VA_ARGS__);                  \
    case 7: return fn<7>(__VA_ARGS__);                  \
    case 8: return fn<8>(__VA_ARGS__);                  \
    case 9: return fn<9>(__VA_ARGS__);                  \
    case 10: return fn<10>(__VA_ARGS__);                \
    case 11: return fn<11>(__VA_ARGS__);                \
    case 12: return fn<12>(__VA_ARGS__);                \
    default: break;                                     \
    }

}  // namespace

int dense_count(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                uint32_t* d_out, hipStream_t s) {
    if (k < 1 || k > KMH_MAX_DENSE_K) return fail(ctx, KMH_ERR_UNSUPPORTED, "dense counting needs 1 <= k <= 12");
    if (!d_seq || !d_out) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    KMH_DISPATCH_K(count_k, k, ctx, d_seq, offsets, G, d_out, s);
    return fail(ctx, KMH_ERR_UNSUPPORTED, "unsupported k");
}

int dense_first(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                uint32_t* d_first, hipStream_t s) {
    if (k < 1 || k > KMH_MAX_DENSE_K) return fail(ctx, KMH_ERR_UNSUPPORTED, "dense counting needs 1 <= k <= 12");
    if (!d_seq || !d_first) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    KMH_DISPATCH_K(first_k, k, ctx, d_seq, offsets, G, d_first, s);
    return fail(ctx, KMH_ERR_UNSUPPORTED, "unsupported k");
}

int synth(Ctx* ctx, uint8_t* d_seq, uint64_t len, uint64_t stride, int G, uint64_t seed0,
          hipStream_t s) {
    if (!d_seq || G < 1 || stride < len) return fail(ctx, KMH_ERR_INVALID, "bad synth arguments");
    const uint64_t words = (len + 31) / 32 * (uint64_t)G;
    const unsigned blocks = (unsigned)std::min<uint64_t>((words + 255) / 256, 65536);
    if (blocks == 0) return KMH_OK;
    time_begin(ctx, s, "k_synth");
    hipLaunchKernelGGL(k_synth, dim3(blocks), dim3(256), 0, s, d_seq, len, stride, seed0, G);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

}  // namespace kmh
