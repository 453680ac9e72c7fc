// kmh_dense.hip -- dense k-mer counting on MI355X (gfx950): 1 <= k <= 12.
//
// Replaces the window loop of /root/reference/kmerml/kmers/generate.py:49-58 (slide a
// k-window over each record, drop windows with a non-ACGT byte, count) for a batch of
// genomes resident in HBM.  Design and rooflines: DESIGN.md, "Kernels".
//
//   k <= 9   k_direct:     each workgroup counts a span of one genome into an LDS table
//                          (4^k bins, or 32768-bin slices in 4^k/32768 passes for k = 8, 9)
//                          and adds it into the genome's row.
//   k >= 10  k_partition:  one 16384-window tile per workgroup (three per CU); k-mers are
//                          bucketed by their top 2k-16 bits with an LDS counting sort and
//                          each tile writes its bucket-ordered 16-bit suffixes + offsets.
//            k_bucket_count: one workgroup per (genome, bucket) gathers that bucket's
//                          segments from every tile of the genome into a 65536-bin u16 LDS
//                          histogram and stores the row slice once.
//
// Bases: A/C/G/T in either case (generate.py:41 upper()s the record; :55 keeps windows of
// "ACGT" only).  Any other byte -- including the '\n' the host puts between records and
// bytes past a genome's end -- breaks windows, so windows never span records or genomes.
#include <algorithm>
#include <cstdio>
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
    void* const before = ctx->meta.ptr;
    int rc = ensure(ctx, ctx->meta, 2 * n * sizeof(uint64_t));
    if (rc) return rc;
    if (ctx->meta.ptr != before) ctx->meta_cache.clear();
    std::vector<uint64_t> both(2 * n);
    std::copy(L.goff.begin(), L.goff.end(), both.begin());
    std::copy(L.tbase.begin(), L.tbase.end(), both.begin() + n);
    // the same layout as the previous call (a bench step, a repeated batch): the device copy is
    // still there (only this function writes ctx->meta, and the calls are stream-ordered), so
    // the host-to-device copy -- ~10 us on the stream before the first kernel -- is skipped
    if (both != ctx->meta_cache) {
        rc = upload(ctx, ctx->meta.ptr, both.data(), both.size() * sizeof(uint64_t), s);
        if (rc) return rc;
        ctx->meta_cache = std::move(both);
    }
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
// Buckets are the top 2k - 16 bits of the code (256 at k = 12); a bucket's 65536 bins are
// counted by one k_bucket_count workgroup in a u16 LDS table (128 KiB).  Tiles of kPTile
// window starts (512 threads x 32) are partitioned by bucket with an LDS counting sort whose
// counters are replicated per LDS bank:
//
//   the u16 half b & 1 of rep word (b >> 1) * 32 + (lane & 31) counts the k-mers of bucket b
//   seen by replica lane & 31, so the 32 lanes of a lane group always hit 32 different banks.
//   A histogram pass adds 1 per k-mer (no returned value), a scan turns the counters into
//   segment starts (bucket start + replica prefix) in place, and the scatter's returning add
//   on the same conflict-free word hands each k-mer its slot, where it stores the 16-bit
//   suffix: the one random LDS access of a k-mer.  No per-k-mer rank is kept in registers and
//   the counters take half the LDS, so three workgroups fit a CU (52.5 KiB, 68 VGPRs).
//   Windows with a non-base byte count in an extra row that the scan places after every
//   bucket, so they need no branch and are never copied out.
//
// Output per tile: the suffixes in bucket order at suf[tile * tile_cap ...], every bucket's
// segment starting at a 16-byte chunk, and toff[b][tile] = first chunk of bucket b's segment
// | (unused slots of its last chunk) << 12; toff[NBK][tile] = chunks written.  The unused slots
// hold stale values: the count kernel adds 0 there.
constexpr int kPThreads = 512;
constexpr int kPTile = kPThreads * kTileBpt;     // 16384 window starts
constexpr int kRep = 32;                         // counter replicas = LDS banks of a lane group
constexpr int kCBits = 16;                       // bins of one count table: 2^16 (u16 in LDS)
constexpr uint32_t kCBins = 1u << kCBits;

template <int K>
constexpr int num_buckets() { return 1 << (2 * K - kCBits); }
// entries per tile in the suffix buffer: every window + the chunk padding of every bucket
template <int K>
constexpr int tile_cap() { return kPTile + 7 * num_buckets<K>(); }

// The 32 window codes of this thread from its 48 loaded bytes (invalid windows: INV, which
// k_partition makes bucket NBK, suffix 0).
template <int K, uint32_t INV>
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
    const uint64_t wBN = ((uint64_t)cB << 32) | cN;
#pragma unroll
    for (int j = 0; j < 16; ++j) km[j] = (uint32_t)(wAB >> (64 - 2 * (j + K))) & KM;
#pragma unroll
    for (int j = 0; j < 16; ++j) km[16 + j] = (uint32_t)(wBN >> (64 - 2 * (j + K))) & KM;
    // only a wave whose 48-byte spans hold a non-base byte (in a synthetic genome: the wave at
    // its end) applies the per-window validity selects: 3 of the ~18 VALU instructions per k-mer
    if (__builtin_amdgcn_ballot_w64((iA | iB | iN) != 0u) != 0ull) {
        const uint32_t vAB = (iA << 16) | iB, vBN = (iB << 16) | iN;
#pragma unroll
        for (int j = 0; j < 16; ++j) km[j] = ((vAB >> (32 - (j + K))) & VM) == 0u ? km[j] : INV;
#pragma unroll
        for (int j = 0; j < 16; ++j) km[16 + j] = ((vBN >> (32 - (j + K))) & VM) == 0u ? km[16 + j] : INV;
    }
}

// Counters the first launch of a count clears on its way (instead of one memset launch each:
// the wrap log's cursor, the escape count, the re-encode list), nullable.
struct Zero3 {
    uint32_t* p[4];
};

template <int K>
__global__ __launch_bounds__(kPThreads, 6) void k_partition(const uint8_t* __restrict__ seq,
                                                            GenomeMap m, uint16_t* __restrict__ suf,
                                                            uint16_t* __restrict__ toff, uint32_t ldt, Zero3 z) {
    constexpr int NBK = num_buckets<K>();
    constexpr int NROW = NBK + 16;                 // + invalid-window row, padded to 16 rows
    constexpr int NW = kPThreads / 64;
    constexpr int CAP = tile_cap<K>();
    static_assert(NBK + 1 <= kPThreads && CAP / 8 < 4096, "scan layout / 12-bit chunk offsets");
    static_assert(NROW + NW <= CAP / 2 && 2 * CAP <= 65535, "starts alias the stage; u16 byte counters");
    constexpr uint32_t kInv = (uint32_t)NBK << kCBits;   // invalid windows: bucket NBK, suffix 0
    static_assert(kCBits == 16, "counter word = code >> 17, half = bit 16 of the code");
    // counters as u16 halves: bucket b, replica r in half b & 1 of word (b >> 1) * 32 + r
    // (52 KiB of LDS per workgroup: three workgroups per CU)
    __shared__ __attribute__((aligned(16))) uint32_t rep[NROW / 2 * kRep];
    __shared__ __attribute__((aligned(16))) uint16_t stage[CAP];
    uint32_t* start = reinterpret_cast<uint32_t*>(stage);   // bucket starts until the scatter
    uint32_t* wsum = start + NROW;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t r4 = ((uint32_t)lane & 31u) << 2;   // byte offset of this lane's replica
    const uint64_t lt = xcd_work_id();
    if (blockIdx.x == 0 && threadIdx.x < 4 && z.p[threadIdx.x]) *z.p[threadIdx.x] = 0u;
    const uint64_t gt = m.tile_lo + lt;
    const int g = find_genome(m, gt);
    const uint64_t tstart = m.goff[g] + (gt - m.tbase[g]) * (uint64_t)kPTile;
    const uint64_t ge = m.goff[g + 1];
    const uint64_t base = tstart + (uint64_t)tid * kTileBpt;
    // counter of code c (bucket c >> 16 <= NBK): byte (c >> 17) * 128 + r4 of rep, half c bit 16
    char* repb = reinterpret_cast<char*>(rep);
    auto ctr = [&](uint32_t c) { return reinterpret_cast<uint32_t*>(repb + (((c >> 17) << 7) | r4)); };
    auto half = [](uint32_t c) { return (c >> 12) & 16u; };

    uint4* rep4 = reinterpret_cast<uint4*>(rep);
    for (int i = tid; i < NROW / 2 * kRep / 4; i += kPThreads) rep4[i] = make_uint4(0u, 0u, 0u, 0u);

    uint32_t km[kTileBpt];
    {
        uint4 ra, rb, rn;
        if (tstart + (uint64_t)kPTile + 16 <= m.data_end) {
            ra = *reinterpret_cast<const uint4*>(seq + base);
            rb = *reinterpret_cast<const uint4*>(seq + base + 16);
            rn = *reinterpret_cast<const uint4*>(seq + base + 32);
        } else {
            ra = load16(seq, base, ge);
            rb = load16(seq, base + 16, ge);
            rn = load16(seq, base + 32, ge);
        }
        // tiles whose bytes all lie inside the genome (all but its last) need no tail masks
        if (tstart + (uint64_t)kPTile + 16 <= ge)   // uniform per workgroup
            visit_raw<K, kInv>(ra, rb, rn, 0u, 0u, 0u, km);
        else
            visit_raw<K, kInv>(ra, rb, rn, tail_mask(base, ge), tail_mask(base + 16, ge), tail_mask(base + 32, ge), km);
    }
    lds_barrier();

    // 1. histogram of (bucket, replica): adds whose results nobody waits for.  Counters,
    //    starts and slots are kept in bytes (2 per k-mer, every value below 2 * CAP < 65536),
    //    so the scatter's returned start is the stage address itself.
#pragma unroll
    for (int j = 0; j < kTileBpt; ++j) {
        __hip_atomic_fetch_add(ctr(km[j]), 2u << half(km[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    lds_barrier();

    // 2a. row totals: one 16-byte read per lane, 8 lanes per word row (two buckets, summed as
    //     packed halves: a bucket holds at most 2 * kPTile < 65536 bytes), 8 word rows per wave
    //     instruction
    for (int i = wave; i < NROW / 16; i += NW) {
        const int wr = i * 8 + (lane >> 3);
        const uint4 v = rep4[wr * (kRep / 4) + (lane & 7)];
        const uint32_t sm = scan8(v.x + v.y + v.z + v.w, lane);
        if ((lane & 7) == 7) {
            start[2 * wr] = sm & 0xFFFFu;
            start[2 * wr + 1] = sm >> 16;
        }
    }
    lds_barrier();

    // 2b. bucket starts: exclusive scan of the chunk-padded bucket sizes, the invalid-window
    //     row last (unpadded)
#if defined(KMH_EXPERIMENTS) && defined(KMH_EXCH_COMPACT)
    uint32_t pad_lo = 0u, pad_hi = 0u;   // this bucket's padding slots, filled with spread values
#endif
    {
        const uint32_t n = tid <= NBK ? start[tid] : 0u;          // bytes: 2 per k-mer
        const uint32_t p = tid < NBK ? (n + 15u) & ~15u : n;       // padded to a 16-byte chunk
        const uint32_t incl = scan64(p);
        if (lane == 63) wsum[wave] = incl;
        lds_barrier();
        uint32_t pre = 0u;
#pragma unroll
        for (int q = 0; q < NW; ++q) pre += q < wave ? wsum[q] : 0u;
        const uint32_t ex = pre + incl - p;
        if (tid <= NBK) start[tid] = ex;
#if defined(KMH_EXPERIMENTS) && defined(KMH_EXCH_COMPACT)
        // A/B only (counts wrong): segments listed at KMH_EXCH_COMPACT / 4 of their chunks,
        // contiguous -- the bytes and the access pattern of a denser exchange code
        if (tid <= NBK) toff[(uint64_t)tid * ldt + lt] = (uint16_t)(((ex >> 4) * KMH_EXCH_COMPACT) >> 2);
        if (tid < NBK) { pad_lo = ex + n; pad_hi = ex + p; }
#else
        if (tid < NBK) toff[(uint64_t)tid * ldt + lt] = (uint16_t)((ex >> 4) | ((p - n) << 11));
        if (tid == NBK) toff[(uint64_t)NBK * ldt + lt] = (uint16_t)(ex >> 4);
#endif
    }
    lds_barrier();
    const uint32_t total = start[NBK];   // bytes to write: the padded buckets

    // 2c. segment start of every (bucket, replica), in place
    //     (packed halves: every start stays below 2 * CAP < 65536)
    for (int i = wave; i < NROW / 16; i += NW) {
        const int wr = i * 8 + (lane >> 3);
        uint4* pr = &rep4[wr * (kRep / 4) + (lane & 7)];
        const uint4 v = *pr;
        const uint32_t sm = v.x + v.y + v.z + v.w;
        const uint32_t ex = scan8(sm, lane) - sm;
        const uint32_t st = (start[2 * wr] + (ex & 0xFFFFu)) | ((start[2 * wr + 1] + (ex >> 16)) << 16);
        *pr = make_uint4(st, st + v.x, st + v.x + v.y, st + v.x + v.y + v.z);
    }
    lds_barrier();

#if defined(KMH_EXPERIMENTS) && defined(KMH_EXCH_COMPACT)
    for (uint32_t i = pad_lo; i < pad_hi; i += 2) stage[i >> 1] = (uint16_t)(i * 40503u);   // no hot bin
#endif
    // 3. scatter the suffixes: a returning add on the (bucket, replica) start gives each k-mer
    //    its slot (groups of 8: eight adds in flight, then eight stores); the order inside a
    //    segment is arbitrary, the count kernel only adds.  The codes are laundered so that the
    //    compiler derives the counter addresses again instead of keeping step 1's 64 live.
#pragma unroll
    for (int j = 0; j < kTileBpt; ++j) __asm__ volatile("" : "+v"(km[j]));
#pragma unroll
    for (int j0 = 0; j0 < kTileBpt; j0 += 8) {
        uint32_t pos[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t h = half(km[j0 + j]);
            pos[j] = __builtin_amdgcn_ubfe(atomicAdd(ctr(km[j0 + j]), 2u << h), h, 16);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(stage) + pos[j]) = (uint16_t)km[j0 + j];
    }
    lds_barrier();

    // 4. write the tile out
    uint4* dst = reinterpret_cast<uint4*>(suf + lt * (uint64_t)CAP);
    const uint4* src = reinterpret_cast<const uint4*>(stage);
#if defined(KMH_EXPERIMENTS) && defined(KMH_EXCH_PLAIN)
    // A/B only: plain stores (the lines may stay in the Infinity Cache for the count kernel)
    for (uint32_t c = tid; c < (total >> 4); c += kPThreads) dst[c] = src[c];
#elif defined(KMH_EXPERIMENTS) && defined(KMH_EXCH_COMPACT)
    for (uint32_t c = tid; c < (((total >> 4) * KMH_EXCH_COMPACT) >> 2); c += kPThreads) store_nt(&dst[c], src[c]);
#else
    for (uint32_t c = tid; c < (total >> 4); c += kPThreads) store_nt(&dst[c], src[c]);
#endif
}

// ---------------------------------------------------------------- k >= 10: count
// u16 count table: bin v in half v & 1 of word v >> 1.  Every wrap of a 16-bit half is seen
// by exactly one ds_add_rtn (the adds to a word are serialised), which logs the correction:
//   low add,  old low  == 0xFFFF: bin v += 65536; its partner v ^ 1 received the carry: -= 1,
//                                 and if old high == 0xFFFF too the carry wrapped it: += 65536
//   high add, old high == 0xFFFF: bin v += 65536 (the carry leaves the word)
// so every bin = stored half + its logged corrections (mod 2^32), applied by k_fixup.  Bins
// below 65536 (every uniform genome) never log.
struct FixLog {
    unsigned long long* entries;  // (row index << 1) | (1 = "-1", 0 = "+65536")
    uint32_t* cursor;
    uint32_t cap;
};

__device__ __forceinline__ void log_wrap(const FixLog& L, uint64_t row0, uint32_t v, uint32_t old) {
    auto put = [&](uint64_t idx, uint32_t minus_one) {
        const uint32_t at = atomicAdd(L.cursor, 1u);
        if (at < L.cap) L.entries[at] = (idx << 1) | minus_one;
    };
    put(row0 + v, 0u);
    if (!(v & 1u)) {
        put(row0 + (v ^ 1u), 1u);
        if ((old >> 16) == 0xFFFFu) put(row0 + (v ^ 1u), 0u);
    }
}

// Fused u4 encoding of the count rows (kmh_count_dense_u4_dev): the same block layout as
// rows_encode_u4 -- nibbles of row g at byte g * 4^k / 2 (element 2i in the low nibble of
// byte i), every count >= 15 as an exact (g * 4^k + column, value) pair behind *esc_n.  A
// bucket whose u16 table wrapped is listed in redo and re-encoded from the corrected u32 row by
// the last workgroup of the last launch (after it applied the wrap log).  rows = 0
// (kmh_count_dense_u4only_dev, the multi-GPU step): the u32 row slices are written only for the
// buckets re-encoded from rows
// (a wrapped table, or escapes past the LDS staging), 67 MB less per 100 Mbp genome at k = 12.
struct U4Out {
    uint32_t* nib;       // u4 block as u32 words (8 counts each)
    uint32_t* esc;       // (index, value) pairs
    uint32_t cap;
    uint32_t* esc_n;
    uint32_t* redo;      // redo[0] = buckets listed; redo[1 + i] = g * NBK + b
    int rows;            // 1: every row slice written; 0: only those of listed buckets
    uint32_t* done;      // workgroups of the last launch that finished (cleared by the partition)
    int tail;            // 1 on the last batch's launch: its last workgroup applies the wrap log
                         // and re-encodes the listed buckets (no k_fixup / k_reencode launches)
};

__device__ __forceinline__ uint32_t sat4(uint32_t x) { return x < 15u ? x : 15u; }

// The first nv entries of one 16-byte chunk (8 suffixes) into the table; the other slots add 0
// (branch-free).  EXACT = false (the first pass over a bucket): plain adds, whose returned
// values nobody waits for.  EXACT = true (the recount of a bucket in which some bin passed
// 65535): the eight returning adds go out back to back; a wrap (an added-to half that held
// 0xFFFF) is looked for once per chunk through the maximum of the returned halves (an add-0
// slot at 0xFFFF is a false alarm that the rare path sorts out).
template <bool EXACT>
__device__ __forceinline__ void count_chunk(uint32_t* tbl, uint4 q, uint32_t nv, const FixLog& L,
                                            uint64_t row0, uint32_t* wrapped) {
    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
    const uint32_t used = (1u << nv) - 1u;   // slots 0 .. nv - 1 add 1 (one bfe per slot)
    uint32_t old[8], off[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t w = wd[i >> 1];
        // entry v = the low / high half of w: word (v >> 1) * 4 bytes, half (v & 1) * 16 bits
        const uint32_t addr = (i & 1) ? (w >> 15) & 0x1FFFCu : (w << 1) & 0x1FFFCu;
        off[i] = (i & 1) ? (w >> 12) & 16u : (w << 4) & 16u;
        const uint32_t add = __builtin_amdgcn_ubfe(used, (uint32_t)i, 1);
        old[i] = __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(tbl) + addr),
                                        add << off[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if constexpr (!EXACT) return;
    uint32_t mx = 0u;
#pragma unroll
    for (int i = 0; i < 8; i += 2)
        mx = max(mx, max(__builtin_amdgcn_ubfe(old[i], off[i], 16), __builtin_amdgcn_ubfe(old[i + 1], off[i + 1], 16)));
    if (__builtin_expect(mx == 0xFFFFu, 0)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t v = (wd[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            if ((uint32_t)i < nv && __builtin_amdgcn_ubfe(old[i], off[i], 16) == 0xFFFFu) {
                log_wrap(L, row0, v, old[i]);
                *wrapped = 1u;   // this bucket's table no longer holds exact counts
            }
        }
    }
}

// Tiles per wave batch: the expected chunks of a batch must fit the wave's queue of qmax
// entries (a batch that overflows it is walked lane by lane).
template <int K>
constexpr int batch_tiles(int qmax) {
    const int per = kPTile / num_buckets<K>() / 8 + 1;   // expected chunks of a segment
    int bt = qmax / per;
    bt = bt < 1 ? 1 : (bt > 64 ? 64 : bt);
    int p2 = 1;
    while (p2 * 2 <= bt) p2 *= 2;
    return p2;
}

// One workgroup per (genome, bucket[, split]): gathers the bucket's segment from every tile of
// the genome into the LDS table, then widens it into the row slice (65536 u32) once.  Each
// wave takes BT tiles at a time (one per lane; their segment bounds are consecutive u16s of the
// bucket-major offset table), lists every 16-byte chunk of their segments in a per-wave LDS
// queue (chunk index relative to the batch, entries used in the chunk) and streams the queue
// with all 64 lanes active: U loads in flight per lane, 8 LDS adds per load.  A batch whose
// chunks overflow the queue (skewed input) is walked lane by lane instead.
#if defined(KMH_EXPERIMENTS) && defined(KMH_DP_CLOCKS)
// KMH_DENSE_PROF: per-phase clocks (a clocks build: its same-address atomics slow the kernel) of k_bucket_count summed over its waves (lane 0 of each)
__device__ unsigned long long g_dense_prof[8];
#define KMH_DP(i) if ((threadIdx.x & 63) == 0) { const unsigned long long t_ = clock64(); atomicAdd(&g_dense_prof[i], t_ - tl_); tl_ = t_; }
#else
#define KMH_DP(i)
#endif

template <int K, int U, bool ENC>
__global__ __launch_bounds__(kCountThreads) void k_bucket_count(
    const uint16_t* __restrict__ suf, const uint16_t* __restrict__ toff, uint32_t ldt, GenomeMap m,
    int S, uint32_t* __restrict__ out, FixLog L, U4Out E) {
    constexpr int NBK = num_buckets<K>();
    constexpr uint32_t CPT = tile_cap<K>() / 8;   // chunks per tile
    constexpr int NW = kCountThreads / 64;
    constexpr int QMAX = U * 64;
    constexpr int BT = batch_tiles<K>(QMAX);
    static_assert((uint32_t)BT * CPT <= (1u << 20), "queue entries hold 20-bit chunk indices");
    constexpr int WORDS = (int)kCBins / 2;
    __shared__ __attribute__((aligned(16))) uint32_t tbl[WORDS];
    __shared__ uint32_t queue[NW][QMAX];     // chunk queues; escape staging of the epilogue
    __shared__ uint32_t wrapped, ecnt, ebase, nent;
    __shared__ unsigned long long hsum;
    __shared__ unsigned long long nextb;     // the next unclaimed tile batch

    const uint32_t w = xcd_work_id();
    const int s = (int)(w % (uint32_t)S);
    const uint32_t b = (w / (uint32_t)S) % NBK;
    const int g = m.g0 + (int)(w / ((uint32_t)S * NBK));
    const uint64_t t0 = m.tbase[g] - m.tile_lo, nt = m.tbase[g + 1] - m.tbase[g];
    const uint64_t ta = t0 + nt * (uint64_t)s / (uint64_t)S;
    const uint64_t tb = t0 + nt * (uint64_t)(s + 1) / (uint64_t)S;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint4* chunks = reinterpret_cast<const uint4*>(suf);
    const uint64_t row0 = (uint64_t)g * (1ull << (2 * K)) + (uint64_t)b * kCBins;

#if defined(KMH_EXPERIMENTS) && defined(KMH_DP_CLOCKS)
    unsigned long long tl_ = clock64();
#endif
    uint4* tbl4 = reinterpret_cast<uint4*>(tbl);
    for (int i = threadIdx.x; i < WORDS / 4; i += kCountThreads) tbl4[i] = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x == 0) {
        wrapped = 0u;
        ecnt = 0u;
        nent = 0u;
        hsum = 0ull;
        nextb = ta;
    }
    __syncthreads();
    KMH_DP(0)

    uint32_t* q = queue[wave];
    // segment of this lane's tile in batch tw: first chunk, chunks, entries in the last chunk
    // (prefetched one batch ahead)
    auto bounds = [&](uint64_t tw, uint32_t g, uint32_t& lo, uint32_t& hi) {
        const uint64_t t = tw + (uint64_t)lane;
        const bool in = (uint32_t)lane < g && t < tb;
        lo = in ? toff[(uint64_t)b * ldt + t] : 0u;
        hi = in ? toff[(uint64_t)(b + 1) * ldt + t] : 0u;
    };
    // One pass over the bucket's segments into the table; returns this lane's share of the
    // bucket's entries.
    auto walk = [&](auto exact) -> uint32_t {
        constexpr bool EX = decltype(exact)::value;
        uint32_t ent = 0u;
        uint32_t lo_n = 0, hi_n = 0;
        // batches claimed from an LDS cursor as the waves get to them, so that the waves of the
        // workgroup finish together (a static round robin left them waiting at the barrier: 1.90
        // -> 1.76 ms per config-3 count launch, profiles/r03/ab/r03o_*)
        auto grab = [&]() -> uint64_t {
            unsigned long long t = 0;
            if (lane == 0) t = atomicAdd(&nextb, (unsigned long long)BT);
            return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)t) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(t >> 32)) << 32);
        };
        const uint32_t gcur = BT, gnext = BT;
        uint64_t tw = grab();
        if (tw < tb) bounds(tw, gcur, lo_n, hi_n);
        for (uint64_t tnext; tw < tb; tw = tnext) {
            tnext = grab();
#if defined(KMH_EXPERIMENTS) && defined(KMH_EXCH_CUT)
            // A/B only (counts wrong): read only the first (KMH_EXCH_CUT - 1) / KMH_EXCH_CUT of
            // every segment's chunks -- fewer bytes AND fewer LDS adds: an upper bound on what a
            // denser exchange code could save in this kernel
            const uint32_t c0 = lo_n & 0xFFFu, nc0 = (hi_n & 0xFFFu) - c0, nc = nc0 - nc0 / KMH_EXCH_CUT;
#else
            const uint32_t c0 = lo_n & 0xFFFu, nc = (hi_n & 0xFFFu) - c0;
#endif
            const uint32_t nlast = 8u - (lo_n >> 12);
            ent += nc ? 8u * nc - (lo_n >> 12) : 0u;
            const uint32_t incl = scan64(nc);
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            const uint64_t cbat = tw * (uint64_t)CPT;                  // the batch's first chunk
            const uint32_t crel = (uint32_t)lane * CPT + c0;           // this segment's, relative
            if (total <= (uint32_t)QMAX) {
                const uint32_t ex = incl - nc;
                for (uint32_t j = 0; j < nc; ++j) q[ex + j] = (crel + j) | ((j + 1 == nc ? nlast - 1u : 7u) << 20);

                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                uint32_t qe[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t e = (uint32_t)(u * 64 + lane);
                    qe[u] = e < total ? q[e] : 0u;                       // idle lanes re-read chunk 0
                }
                uint4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = chunks[cbat + (qe[u] & 0xFFFFFu)];
                // next batch's bounds load behind this batch's data loads
                if (tnext < tb) bounds(tnext, gnext, lo_n, hi_n);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if ((uint32_t)(u * 64 + lane) < total)
                        count_chunk<EX>(tbl, v[u], (qe[u] >> 20) + 1u, L, row0, &wrapped);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            } else {
                if (tnext < tb) bounds(tnext, gnext, lo_n, hi_n);
                for (uint32_t j = 0; j < nc; ++j)
                    count_chunk<EX>(tbl, chunks[cbat + crel + j], j + 1 == nc ? nlast : 8u, L, row0, &wrapped);
            }
        }
        return ent;
    };
    // First pass with plain adds.  A bin that passes 65535 wraps its u16 half (a low half also
    // carries into its partner), and every such event lowers the sum of the table's halves
    // (by 65536, or 65535 for a low half), so the table is exact iff that sum equals the
    // bucket's entries; otherwise the bucket is counted again with returning adds, which log
    // every wrap (skewed genomes only: uniform 100 Mbp genomes stay below 65536 per bin).
    const uint32_t ent = walk(std::false_type{});
    KMH_DP(1)
    {
        uint32_t e = ent;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) e += __shfl_xor(e, d);
        if (lane == 0) atomicAdd(&nent, e);
    }
    // the halves' sum of this thread's table words (64 halves of at most 65535: fits 32 bits),
    // added into hsum
    auto add_hsum = [&](uint32_t hs) {
        unsigned long long h = hs;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d);
        if (lane == 0) atomicAdd(&hsum, h);
    };
    auto halves = [](uint4 x) {
        return (x.x & 0xFFFFu) + (x.x >> 16) + (x.y & 0xFFFFu) + (x.y >> 16) +
               (x.z & 0xFFFFu) + (x.z >> 16) + (x.w & 0xFFFFu) + (x.w >> 16);
    };
    // With one workgroup per bucket (S = 1) the row slice and its nibbles can be rewritten, so
    // the check rides on the widening's own read of the table: the first widening keeps its
    // escapes in LDS (a bucket past the staging is left to the re-encode, which encodes it from
    // the rows), and a failed check drops them, counts the bucket again exactly (the wraps
    // make it a re-encoded bucket) and widens again.  With split rows (S > 1, added with
    // atomics) the table is checked before it is widened.  One call site of each walk (a
    // third inlined copy made the compiler spill to scratch).
#if defined(KMH_EXPERIMENTS) && (defined(KMH_EXCH_CUT) || defined(KMH_EXCH_COMPACT))
    constexpr bool kCheck = false;   // A/B only: no exactness check (the cut exchange counts garbage)
#else
    constexpr bool kCheck = true;
#endif
    const bool post = S == 1;   // uniform
    bool exact = false, enc = false;
#if defined(KMH_EXPERIMENTS) && defined(KMH_DP_CLOCKS)
    __syncthreads();
    KMH_DP(2)
#endif
    constexpr uint32_t kStage = (uint32_t)(NW * QMAX) / 2;   // (index, value) pairs
    uint32_t* stage = &queue[0][0];
    for (;;) {
        if (exact) {
            __syncthreads();
            if (threadIdx.x == 0) {
                ecnt = 0u;   // the first widening's staged escapes are dropped
                nextb = ta;
            }
            for (int i = threadIdx.x; i < WORDS / 4; i += kCountThreads) tbl4[i] = make_uint4(0u, 0u, 0u, 0u);
            __syncthreads();
            walk(std::true_type{});
        }
        __syncthreads();
        if (kCheck && !post && !exact) {
            uint32_t hs0 = 0u;
            for (int i = threadIdx.x; i < WORDS / 4; i += kCountThreads) hs0 += halves(tbl4[i]);
            add_hsum(hs0);
            __syncthreads();
            if (hsum != (unsigned long long)nent) {   // uniform
                exact = true;
                continue;
            }
        }
        // Widen the u16 pairs into the u32 row slice (plain stores, or adds when split).  ENC (S = 1
        // only): also the slice's u4 nibbles (one u32 of 8 counts per thread and step) and its
        // escapes, staged in the LDS of the queues and appended behind one global atomic.
        enc = ENC && wrapped == 0u;                                // uniform
        // the u32 slice: always without ENC; with ENC unless rows = 0 (then only a wrapped
        // table's, which the re-encode reads after the wrap log has corrected it)
        const bool wrows = !ENC || E.rows != 0 || exact;           // uniform
        uint32_t* orow = out + row0;
        uint32_t hs = 0u;
        for (int i = threadIdx.x; i < (int)kCBins / 8; i += kCountThreads) {
            const uint4 x = tbl4[i];
            const uint4 lo4 = make_uint4(x.x & 0xFFFFu, x.x >> 16, x.y & 0xFFFFu, x.y >> 16);
            const uint4 hi4 = make_uint4(x.z & 0xFFFFu, x.z >> 16, x.w & 0xFFFFu, x.w >> 16);
            if (S == 1) {
                if (wrows) {
                    store_nt(reinterpret_cast<uint4*>(orow) + 2 * i, lo4);
                    store_nt(reinterpret_cast<uint4*>(orow) + 2 * i + 1, hi4);
                }
                if (post && !exact) hs += halves(x);
                if (enc) {
                    const uint32_t e[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
                    uint32_t w = 0u, ne = 0u;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        w |= sat4(e[j]) << (4 * j);
                        ne += e[j] >= 15u ? 1u : 0u;
                    }
                    E.nib[row0 / 8 + (uint64_t)i] = w;
                    if (ne) {   // ~1 in 100 threads for uniform 100 Mbp genomes at k = 12
                        uint32_t at = atomicAdd(&ecnt, ne);
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (e[j] >= 15u) {
                                const uint32_t idx = (uint32_t)(row0 + 8 * (uint64_t)i + j);
                                if (at < kStage) {
                                    stage[2 * at] = idx;
                                    stage[2 * at + 1] = e[j];
                                }   // past the staging: this bucket is re-encoded from its row
                                ++at;
                            }
                        }
                    }
                }
            } else if (ta < tb) {
                const uint32_t e[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (e[j]) atomicAdd(&orow[8 * i + j], e[j]);
            }
        }
        KMH_DP(3)
        if (kCheck && post && !exact) {   // uniform
            add_hsum(hs);
            lds_barrier();   // not __syncthreads(): the slice's stores drain behind it
            if (hsum != (unsigned long long)nent) {
                exact = true;
                continue;
            }
        }
        break;
    }
    KMH_DP(4)
    if (ENC) {
        __syncthreads();
        if (ecnt > kStage) enc = false;                            // uniform
        if (!enc && threadIdx.x == 0) {                            // re-encoded from its row (tail)
            const uint32_t at = atomicAdd(E.redo, 1u);
            E.redo[1 + at] = (uint32_t)g * NBK + b;
        }
        if (!enc && !E.rows && !exact) {   // escapes past the staging: the re-encode reads the row slice,
            uint32_t* orow = out + row0;   // which the widening skipped (the table is still exact)
            for (int i = threadIdx.x; i < (int)kCBins / 8; i += kCountThreads) {
                const uint4 x = tbl4[i];
                store_nt(reinterpret_cast<uint4*>(orow) + 2 * i, make_uint4(x.x & 0xFFFFu, x.x >> 16, x.y & 0xFFFFu, x.y >> 16));
                store_nt(reinterpret_cast<uint4*>(orow) + 2 * i + 1, make_uint4(x.z & 0xFFFFu, x.z >> 16, x.w & 0xFFFFu, x.w >> 16));
            }
        }
        const uint32_t n = min(ecnt, kStage);
        if (enc && threadIdx.x == 0) ebase = n ? atomicAdd(E.esc_n, n) : 0u;
        __syncthreads();
        if (enc)
            for (uint32_t i = threadIdx.x; i < n; i += kCountThreads)
                if (ebase + i < E.cap) {
                    E.esc[2 * (uint64_t)(ebase + i)] = stage[2 * i];
                    E.esc[2 * (uint64_t)(ebase + i) + 1] = stage[2 * i + 1];
                }
        if (E.tail) {   // (uniform) the last workgroup to finish applies the wrap log and re-encodes
            // a listed bucket's row slice and wrap-log entries are released before it counts in
            // (the other workgroups wrote nothing the last one reads)
            if (!enc) __threadfence();
            __syncthreads();
            if (threadIdx.x == 0) wrapped = atomicAdd(E.done, 1u) == gridDim.x - 1u ? 2u : 0u;
            __syncthreads();
            if (wrapped == 2u) {   // (uniform)
                __threadfence();
                const uint32_t nf = min(__hip_atomic_load(L.cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), L.cap);
                for (uint32_t i = threadIdx.x; i < nf; i += kCountThreads) {
                    const unsigned long long e = L.entries[i];
                    atomicAdd(&out[e >> 1], (e & 1ull) ? 0xFFFFFFFFu : 65536u);
                }
                __threadfence();
                __syncthreads();
                const uint32_t nr = __hip_atomic_load(E.redo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (uint32_t it = 0; it < nr; ++it) {
                    const uint32_t gb = E.redo[1 + it];
                    const uint64_t r0 = (uint64_t)(gb / NBK) * (1ull << (2 * K)) + (uint64_t)(gb % NBK) * kCBins;
                    for (uint32_t i = threadIdx.x; i < kCBins / 8; i += kCountThreads) {
                        uint32_t w = 0u;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const uint32_t v = out[r0 + 8 * i + j];
                            w |= sat4(v) << (4 * j);
                            if (v >= 15u) {
                                const uint32_t at = atomicAdd(E.esc_n, 1u);
                                if (at < E.cap) {
                                    E.esc[2 * (uint64_t)at] = (uint32_t)(r0 + 8 * i + j);
                                    E.esc[2 * (uint64_t)at + 1] = v;
                                }
                            }
                        }
                        E.nib[r0 / 8 + i] = w;
                    }
                }
            }
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

template <int K>
int run_partitioned(Ctx* ctx, const uint8_t* d_seq, const Layout& L, const uint64_t* d_goff,
                    const uint64_t* d_tbase, int G, uint32_t* d_out, hipStream_t s, const U4Out* enc) {
    constexpr int NBK = num_buckets<K>();
    constexpr int U = 6;                  // chunk loads in flight per lane (queue = 64 U; 7: no gain, r03ab_u7)
    const size_t row = (size_t)1 << (2 * K);
    // Genomes per batch: the suffix buffer of one batch stays within the budget (8 GiB: 36
    // genomes of 100 Mbp at k = 12).  Measured (profiles/ab2_r02.sh, config 3): 2 / 4 / 8 GiB
    // budgets 10.1 / 9.3 / 9.2 ms per step; the partition of batch i + 1 on a side stream beside
    // the count of batch i was no faster (10.3 / 10.3 / 9.3 ms): both kernels move ~5 TB/s of
    // mixed HBM traffic.  KMH_SUF_BUDGET_MB changes only the batching, never the counts (tests
    // force one genome per batch with it).
    const size_t budget = env_mb("KMH_SUF_BUDGET_MB", 8192) << 20;
    const size_t tile_bytes = (size_t)tile_cap<K>() * sizeof(uint16_t);
    auto batch_end = [&](int g) {
        int h = g;
        uint64_t tiles = 0;
        do {
            tiles += L.tbase[h + 1] - L.tbase[h];
            ++h;
        } while (h < G && (tiles + (L.tbase[h + 1] - L.tbase[h])) * tile_bytes <= budget);
        return std::make_pair(h, tiles);
    };
    uint64_t max_batch_tiles = 0;
    for (int g = 0; g < G;) {
        const auto e = batch_end(g);
        max_batch_tiles = std::max(max_batch_tiles, e.second);
        g = e.first;
    }
    const size_t slot_tiles = std::max<uint64_t>(max_batch_tiles, 1);
    int rc = ensure(ctx, ctx->suf, slot_tiles * tile_bytes);
    if (rc) return rc;
    const uint32_t ldt = (uint32_t)((slot_tiles + 63) / 64 * 64);
    rc = ensure(ctx, ctx->toff, (size_t)ldt * (NBK + 1) * sizeof(uint16_t));
    if (rc) return rc;
    // u16-wrap log: every wrap of a bin takes 65536 windows and logs at most 3 entries
    const uint64_t windows = (uint64_t)L.ntiles * (uint64_t)tile_cap<K>();
    const uint64_t cap = 3 * (windows / 65536 + 1) + 64;
    rc = ensure(ctx, ctx->fix, 256 + cap * sizeof(unsigned long long));
    if (rc) return rc;
    FixLog fl;
    fl.cursor = static_cast<uint32_t*>(ctx->fix.ptr);
    fl.entries = reinterpret_cast<unsigned long long*>(static_cast<char*>(ctx->fix.ptr) + 256);
    fl.cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFF0ull);
    // the counters every later kernel adds to: cleared by the first partition launch (a batch
    // without tiles comes first only if every genome of it is too short for one window)
    // (ENC: the last launch's done counter, in the wrap log's header: fl.cursor + 1)
    uint32_t* done = fl.cursor + 1;
    Zero3 z{{fl.cursor, enc ? enc->esc_n : nullptr, enc ? enc->redo : nullptr, done}};
    if (L.tbase[G] == L.tbase[0] || L.tbase[batch_end(0).first] == L.tbase[0]) {
        KMH_HIP(ctx, hipMemsetAsync(fl.cursor, 0, 8, s));
        if (enc) {
            KMH_HIP(ctx, hipMemsetAsync(enc->esc_n, 0, 4, s));
            KMH_HIP(ctx, hipMemsetAsync(enc->redo, 0, 4, s));
        }
        z = Zero3{{nullptr, nullptr, nullptr, nullptr}};
    }

    for (int g = 0; g < G;) {
        const auto e = batch_end(g);
        const int h = e.first;
        const uint64_t tiles = e.second;
        const int nG = h - g;
        uint16_t* suf = static_cast<uint16_t*>(ctx->suf.ptr);
        uint16_t* toff = static_cast<uint16_t*>(ctx->toff.ptr);
        GenomeMap m{d_goff, d_tbase, g, h, L.tbase[g], L.goff[G]};
        uint64_t maxt = 0;
        for (int q = g; q < h; ++q) maxt = std::max<uint64_t>(maxt, L.tbase[q + 1] - L.tbase[q]);
        // splits per (genome, bucket): at least kTargetWorkgroups count workgroups
        const uint64_t want = ((uint64_t)kTargetWorkgroups + (uint64_t)nG * NBK - 1) / ((uint64_t)nG * NBK);
        // (the fused u4 encoding needs each bucket in one workgroup: S = 1)
        int S = enc ? 1 : (int)std::max<uint64_t>(1, std::min<uint64_t>(want, std::max<uint64_t>(maxt, 1)));
#ifdef KMH_EXPERIMENTS
        // A/B only; the fused u4 encode needs one workgroup per bucket, so never with enc
        if (!enc && env_long("KMH_COUNT_S", 0) > 0) S = (int)env_long("KMH_COUNT_S", 1);
#endif
        if (S > 1) KMH_HIP(ctx, hipMemsetAsync(d_out + (size_t)g * row, 0, (size_t)nG * row * sizeof(uint32_t), s));
        if (tiles) {
            time_begin(ctx, s, "k_partition");
            hipLaunchKernelGGL(k_partition<K>, dim3((unsigned)tiles), dim3(kPThreads), 0, s, d_seq, m, suf,
                               toff, ldt, z);
            z = Zero3{{nullptr, nullptr, nullptr, nullptr}};
            time_end(ctx, s);
            KMH_HIP(ctx, hipGetLastError());
        }
        time_begin(ctx, s, "k_bucket_count");
        if (enc) {
            U4Out e = *enc;
            e.done = done;
            e.tail = h == G;   // the last batch's launch does the wrap fixes and re-encodes (only it
                               // counts into `done`, which the first partition launch cleared)
            hipLaunchKernelGGL((k_bucket_count<K, U, true>), dim3((unsigned)(nG * NBK * S)), dim3(kCountThreads), 0,
                               s, suf, toff, ldt, m, S, d_out, fl, e);
        }
        else
            hipLaunchKernelGGL((k_bucket_count<K, U, false>), dim3((unsigned)(nG * NBK * S)), dim3(kCountThreads), 0,
                               s, suf, toff, ldt, m, S, d_out, fl, U4Out{});
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
#if defined(KMH_EXPERIMENTS) && defined(KMH_DP_CLOCKS)
        if (env_long("KMH_DENSE_PROF", 0)) {
            unsigned long long hp[8];
            KMH_HIP(ctx, hipStreamSynchronize(s));
            KMH_HIP(ctx, hipMemcpyFromSymbol(hp, HIP_SYMBOL(g_dense_prof), sizeof(hp)));
            const double waves = (double)nG * NBK * S * (kCountThreads / 64);
            std::fprintf(stderr, "k_bucket_count per wave (kcycles): zero %.1f | walk %.1f | sum+barrier %.1f | "
                         "widen+stores %.1f | check+barrier %.1f  (%d genomes)\n", hp[0] / waves / 1e3,
                         hp[1] / waves / 1e3, hp[2] / waves / 1e3, hp[3] / waves / 1e3, hp[4] / waves / 1e3, nG);
            const unsigned long long z[8] = {};
            KMH_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_dense_prof), z, sizeof(z)));
        }
#endif
        g = h;
    }
    if (!enc) {   // (the fused encode's last count workgroup applies the log and re-encodes)
        time_begin(ctx, s, "k_fixup");
        hipLaunchKernelGGL(k_fixup, dim3(64), dim3(256), 0, s, fl, d_out);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
    }
    return KMH_OK;
}

template <int K>
int count_k(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, uint32_t* d_out,
            hipStream_t s, const U4Out* enc) {
    Layout L;
    const uint64_t *d_goff, *d_tbase;
    int rc = make_layout(ctx, offsets, G, K, K <= 9 ? (uint64_t)kTile : (uint64_t)kPTile, L);
    if (!rc) rc = upload_layout(ctx, L, s, &d_goff, &d_tbase);
    if (rc) return rc;
    if constexpr (K <= 9) return run_direct<K>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s);
    else return run_partitioned<K>(ctx, d_seq, L, d_goff, d_tbase, G, d_out, s, enc);
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
    KMH_DISPATCH_K(count_k, k, ctx, d_seq, offsets, G, d_out, s, nullptr);
    return fail(ctx, KMH_ERR_UNSUPPORTED, "unsupported k");
}

int dense_count_u4(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k, uint32_t* d_out,
                   uint8_t* d_u4, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n, int rows, hipStream_t s) {
    if (k < 3 || k > KMH_MAX_DENSE_K) return fail(ctx, KMH_ERR_UNSUPPORTED, "the fused u4 count needs 3 <= k <= 12");
    if (!d_seq || !d_out || !d_u4 || !d_esc_n || (cap && !d_esc)) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    const uint64_t cols = 1ull << (2 * k);
    if (G < 1 || (uint64_t)G * cols >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "u4 blocks must hold fewer than 2^32 - 1 cells");
    if (k <= 9) {   // k_direct has no per-bucket epilogue: count, then the encoder
        int rc = dense_count(ctx, d_seq, offsets, G, k, d_out, s);
        return rc ? rc : rows_encode_u4(ctx, d_out, (uint64_t)G, cols, d_u4, d_esc, cap, d_esc_n, s);
    }
    const size_t redo_bytes = (1 + (size_t)G * (cols >> kCBits)) * sizeof(uint32_t);
    int rc = ensure(ctx, ctx->redo, redo_bytes);
    if (rc) return rc;
    // (*d_esc_n and the re-encode list are cleared by the count's first partition launch)
    U4Out E{reinterpret_cast<uint32_t*>(d_u4), d_esc, cap, d_esc_n, static_cast<uint32_t*>(ctx->redo.ptr), rows};
    switch (k) {
    case 10: return count_k<10>(ctx, d_seq, offsets, G, d_out, s, &E);
    case 11: return count_k<11>(ctx, d_seq, offsets, G, d_out, s, &E);
    default: return count_k<12>(ctx, d_seq, offsets, G, d_out, s, &E);
    }
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
