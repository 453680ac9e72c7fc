// kmh_shard.hip -- one rank's column shard of the organisms x k-mers matrix for sparse k
// (BASELINE config 5; /root/reference/kmerml/ml/features.py:96-111, _build_matrix: the columns
// are the sorted union of every organism's labels, a missing label is 0).  Input: the rank's
// organism rows restricted to its code range [lo, hi), each row sorted by code (the rows of
// kmh_count_sparse_sorted_dev after the all-to-all), back to back in organism order.  Output:
// the sorted union of their codes (`columns`) and, for every row entry, its column index
// (`indices`): with the rows' offsets as indptr and their counts as values, the shard's CSR.
//
// The code range is cut into units of ~3/4 CAP entries (all rows together), sized by the
// entries' density: a coarse grid of 2^16 power-of-two cells (k_shard_coarse: every row's start
// in every cell, by binary search), each cell cut into ceil(entries / target) equal code spans
// (k_shard_cells, k_shard_units: the units' first and end codes), and every row's start in every
// unit by a search inside its cell (k_shard_ustarts: an interpolated guess, then galloping).  Then
// a persistent grid (two or four workgroups per CU, by shape) takes the units in turn: a workgroup
// gathers a unit's row pieces into registers, sorts them in LDS by a counting sort on 11-12 bits
// of the code (~0.75 entries per bin), puts each bin in order by rank, and equal codes are then
// adjacent: run heads are the union.  k_shard_union runs twice -- the union's size per unit (with
// u32 code offsets: inserts into an LDS hash set, no sort), then (after a scan) the columns and
// the indices -- so no entry moves through memory other than its code being read.  A unit that
// overflows the LDS (more than CAP entries, or a bin of more than kShBin: codes shared by many
// organisms, low-complexity data) is left to an exact fallback: its entries are gathered,
// radix-sorted (kmh_sort.hip) and written the same way.
// (Round 5: until then the units were uniform code spans of ~2048 entries on average and their
// starts came from a pass over every code; the workgroups were latency-bound per unit, and a
// uniform span must stay small enough for the densest part of the range.)
#include <algorithm>
#include <cstdio>
#include <vector>

#include "kmh_device.h"

namespace kmh {
namespace {

constexpr int kShScanThreads = 1024;
constexpr int kShBin = 64;          // entries of one bin sorted in place (more: fallback)
constexpr int kShMaxRows = 4096;    // organisms of one shard (LDS piece table)
constexpr int kShRoffCache = 1024;  // row offsets kept in LDS
constexpr int kShCoarseBits = 16;   // coarse cells: at most 2^16
// Two union shapes (k_shard_union<NT, CAP, ..>): units of up to CAP entries in LDS, ~3/4 CAP on
// average.  Up to kShSmallRows rows, 256 threads and CAP 2048 (four workgroups per CU, ~29 KiB of
// LDS each): a unit's barriers span 4 waves, not 8 (config 5 at N = 1, 16 rows: union passes
// 59.5 -> 55.4 ms); with more rows a unit's row pieces would shrink to a few entries each, so 512
// threads and CAP 4096 (two workgroups per CU, ~58 KiB of LDS each for up to ~500 rows).
constexpr int kShSmallRows = 32;
constexpr int kShSlotRows = 256;    // up to this many rows, an entry's row comes from the 64-entry slot
                                    // table (a u8 row per slot, then a few steps over row starts); beyond,
                                    // by binary search (R = 128, config 5's shard at N = 8: 3 vs 7 LDS
                                    // round trips per entry)

// First entry of row[a, b) that is >= c (row ascending).
__device__ __forceinline__ uint32_t lower_in(const uint64_t* __restrict__ row, uint32_t a, uint32_t b, uint64_t c) {
    while (a < b) {
        const uint32_t m = a + (b - a) / 2u;
        if (row[m] < c) a = m + 1u;
        else b = m;
    }
    return a;
}

// lower_in for a row piece [a, b) whose codes lie in [c0, c0 + w1]: starts at the entry where c
// would sit if the piece's codes were spread evenly over that span and gallops from there (the
// unit starts of k_shard_ustarts: sorted k-mer codes are close to uniform inside a coarse cell, so
// the guess is a few entries off -- one or two cache lines, where a binary search over a piece of
// ~500 entries touched ~6)
__device__ __forceinline__ uint32_t lower_guess(const uint64_t* __restrict__ row, uint32_t a, uint32_t b, uint64_t c,
                                                uint64_t c0, uint64_t w1) {
    if (a >= b) return a;
    const uint32_t n = b - a;
    const double f = (double)(c - c0) / ((double)w1 + 1.0);   // in [0, 1)
    const uint32_t g = a + min(n - 1u, (uint32_t)(f * (double)n));
    uint32_t lo, hi;   // the answer lies in [lo, hi]
    uint32_t step = 1u;
    if (row[g] < c) {
        lo = g + 1u;
        hi = b;
        while (lo + step - 1u < b) {
            const uint32_t p = lo + step - 1u;
            if (row[p] < c) {
                lo = p + 1u;
                step <<= 1;
            } else {
                hi = p;
                break;
            }
        }
    } else {
        lo = a;
        hi = g;
        while (hi - a >= step) {
            const uint32_t p = hi - step;
            if (row[p] >= c) {
                hi = p;
                step <<= 1;
            } else {
                lo = p + 1u;
                break;
            }
        }
    }
    return lower_in(row, lo, hi, c);
}

// cs[r * (Q + 1) + q] = the first entry of row r (relative to the row) whose code is >= the
// start of coarse cell q, lo + q 2^CSH (q = Q: the row's length).  One thread per (q, r).
__global__ __launch_bounds__(256) void k_shard_coarse(const uint64_t* __restrict__ codes,
                                                      const uint64_t* __restrict__ roff, int R, uint64_t lo,
                                                      int CSH, uint32_t Q, uint32_t* __restrict__ cs) {
    const uint64_t x = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (x >= (uint64_t)(Q + 1u) * (uint64_t)R) return;
    const uint32_t r = (uint32_t)(x / (Q + 1u)), q = (uint32_t)(x % (Q + 1u));
    const uint64_t a = roff[r];
    const uint32_t n = (uint32_t)(roff[r + 1] - a);
    cs[x] = q == Q ? n : lower_in(codes + a, 0u, n, lo + ((uint64_t)q << CSH));
}

// Units of coarse cell q: nu[q] = ceil(its entries (all rows) / target).
__global__ __launch_bounds__(256) void k_shard_cells(const uint32_t* __restrict__ cs, int R, uint32_t Q,
                                                     uint64_t lo, uint64_t hi_incl, int CSH, uint32_t target,
                                                     uint32_t* __restrict__ nu) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= Q) return;
    uint64_t e = 0;
    for (int r = 0; r < R; ++r) e += cs[(uint64_t)r * (Q + 1u) + q + 1u] - cs[(uint64_t)r * (Q + 1u) + q];
    // at most one unit per code (a unit of one code holds R entries at most: past the union's
    // LDS it goes to the fallback)
    const uint64_t c0 = lo + ((uint64_t)q << CSH);
    const uint64_t w1 = (q + 1u == Q ? hi_incl : c0 + ((1ull << CSH) - 1u)) - c0;   // width - 1
    const uint64_t n = (e + target - 1) / target;
    nu[q] = (uint32_t)(n == 0u ? 0u : (n - 1u > w1 ? w1 + 1u : n));
}

// The units of cell q (ubase[q] .. + nu[q]): equal code spans [ub, ue] of the cell [lo + q 2^CSH,
// + 2^CSH) (the last cell ends at hi): of its W codes, part j starts at j (W / n) + min(j, W % n).
// One thread per cell.
__global__ __launch_bounds__(256) void k_shard_units(const uint32_t* __restrict__ nu,
                                                     const unsigned long long* __restrict__ ubase, uint32_t Q,
                                                     uint64_t lo, uint64_t hi_incl, int CSH,
                                                     uint64_t* __restrict__ ub, uint64_t* __restrict__ ue,
                                                     uint32_t* __restrict__ ucell) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= Q) return;
    const uint32_t n = nu[q];
    if (!n) return;
    const uint64_t c0 = lo + ((uint64_t)q << CSH);
    const uint64_t last = q + 1u == Q ? hi_incl : c0 + ((1ull << CSH) - 1u);   // the cell's last code
    const uint64_t W = last - c0 + 1u;   // <= 2^63 (CSH <= 63); n <= W (k_shard_cells)
    const uint64_t qw = W / n, rw = W % n;
    const uint64_t u0 = ubase[q];
    for (uint32_t j = 0; j < n; ++j) {
        ub[u0 + j] = c0 + (uint64_t)j * qw + (j < rw ? j : rw);
        ue[u0 + j] = j + 1u == n ? last : c0 + (uint64_t)(j + 1u) * qw + (j + 1u < rw ? j + 1u : rw) - 1u;   // (inclusive)
        ucell[u0 + j] = q;
    }
}

// st[u * R + r] = the first entry of row r whose code is >= unit u's first code, found inside the
// unit's coarse cell; st[U * R + r] = the row's length.  Unit-major, so that a union workgroup reads
// one unit's R row starts as one contiguous run (row-major, each unit read R cache lines: at R = 128
// rows that was most of the union's memory traffic).  One workgroup per 64 units, rows in chunks of
// 64: the searches run units-fastest (a wave searches 64 neighbouring units of ONE row, so its
// loads share lines), then an LDS transpose writes every unit's row starts as one run (searching
// rows-fastest was 2.4x slower at R = 128).
constexpr int kUsU = 64, kUsR = 64;

__global__ __launch_bounds__(256) void k_shard_ustarts(const uint64_t* __restrict__ codes,
                                                       const uint64_t* __restrict__ roff, int R,
                                                       const uint32_t* __restrict__ cs, uint32_t Q,
                                                       uint64_t lo, uint64_t hi_incl, int CSH,
                                                       const uint64_t* __restrict__ ub,
                                                       const uint32_t* __restrict__ ucell, uint32_t U,
                                                       uint32_t* __restrict__ st) {
    __shared__ uint32_t tile[kUsU][kUsR + 1];
    const uint32_t u0 = blockIdx.x * (uint32_t)kUsU;
    const uint32_t nu = min((uint32_t)kUsU, U + 1u - u0);
    for (int r0 = 0; r0 < R; r0 += kUsR) {
        const int nr = min(kUsR, R - r0);
        for (int idx = threadIdx.x; idx < kUsU * nr; idx += 256) {   // (only the chunk's rows: R = 16 uses 16 of 64)
            const uint32_t uu = (uint32_t)(idx % kUsU);
            const int rr = idx / kUsU;
            if (uu < nu) {
                const uint32_t u = u0 + uu;
                const int r = r0 + rr;
                const uint64_t a = roff[r];
                uint32_t v;
                if (u == U) {
                    v = (uint32_t)(roff[r + 1] - a);
                } else {
                    const uint32_t q = ucell[u];
                    const uint32_t* c = cs + (uint64_t)r * (Q + 1u);
                    const uint64_t c0 = lo + ((uint64_t)q << CSH);
                    const uint64_t w1 = (q + 1u == Q ? hi_incl : c0 + ((1ull << CSH) - 1u)) - c0;
                    v = lower_guess(codes + a, c[q], c[q + 1u], ub[u], c0, w1);
                }
                tile[uu][rr] = v;
            }
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < (int)nu * nr; idx += 256) {
            const int rr = idx % nr;
            const uint32_t uu = (uint32_t)(idx / nr);
            st[(uint64_t)(u0 + uu) * (uint64_t)R + (uint64_t)(r0 + rr)] = tile[uu][rr];
        }
        __syncthreads();
    }
}

// Unit of code c (fallback only): the last unit whose first code is <= c.
__device__ __forceinline__ uint32_t unit_of(const uint64_t* __restrict__ ub, uint32_t U, uint64_t c) {
    uint32_t a = 0u, b = U - 1u;
    while (a < b) {
        const uint32_t m = (a + b + 1u) / 2u;
        if (ub[m] <= c) a = m;
        else b = m - 1u;
    }
    return a;
}

// Block-wide exclusive scan of one u32 per thread (NT); returns the thread's prefix,
// *total = the sum.  ws: NT / 64 words of LDS.
//
// Every barrier of the union is lds_barrier() (kmh_device.h): the kernel never reads back what it
// stores, and __syncthreads() -- a workgroup release, s_waitcnt vmcnt(0) -- made each of a unit's
// ~10 barriers wait for the stores of the previous unit and for the loads prefetched for the next
// one (round 6: the software pipelining over units only works with LDS-only barriers).
template <int NT>
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = scan64(v);
    if (lane == 63) ws[wave] = incl;
    lds_barrier();
    uint32_t pre = 0u, tot = 0u;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const uint32_t x = ws[w];
        pre += w < wave ? x : 0u;
        tot += x;
    }
    lds_barrier();   // ws reusable
    *total = tot;
    return pre + incl - v;
}

// One workgroup per unit (persistent: s = blockIdx.x, += gridDim.x; unit s = codes [ub[s], ue[s]],
// row r's piece = entries st[r][s] .. st[r][s + 1]).  WRITE = false: the number of distinct codes of
// every unit into ucount (0 for a unit left to the fallback, which is listed in big).  WRITE =
// true: the columns [colbase[s], colbase[s + 1]) and the column index of every entry.
// Software-pipelined over units: the next unit's row starts are loaded when a unit begins, its
// pieces are scanned (into the other of two LDS tables) and its codes loaded right after this
// unit's scatter, so they land during this unit's sort, heads and stores (one unit at a time per
// workgroup waited for two global round trips per unit: latency-bound).
#ifdef KMH_EXPERIMENTS
// KMH_EXPERIMENTS builds only: clocks of the union's phases, summed over workgroups (thread 0)
__device__ unsigned long long g_shard_pt[2][16];
#define KMH_SPT(i) if (tid == 0) { const unsigned long long t_ = clock64(); pt_[i] += t_ - tl_; tl_ = t_; }
#else
#define KMH_SPT(i)
#endif

template <int NT, int CAP, bool WRITE, typename K, typename IX>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 && sizeof(K) == 4 && !WRITE ? 5 : 4))) void k_shard_union(const uint64_t* __restrict__ codes,
                                                            const uint64_t* __restrict__ roff, int R,
                                                            const uint32_t* __restrict__ st, uint32_t S,
                                                            const uint64_t* __restrict__ ub,
                                                            const uint64_t* __restrict__ ue, uint32_t* __restrict__ ucount,
                                                            uint32_t* __restrict__ big,
                                                            const unsigned long long* __restrict__ colbase,
                                                            uint64_t* __restrict__ columns,
                                                            IX* __restrict__ indices) {
    // NT threads, units of up to CAP entries in LDS, NB = CAP bins of a unit's codes (kBB bits;
    // 2 CAP bins in the write pass, fewer entries sharing a bin, measured slower: 30.9 -> 33.2 ms
    // at 16 rows, the larger histogram's clearing and scan outweigh the rank reads saved), and the
    // sizes pass's hash set of 2 CAP slots
    static_assert(CAP == 2048 || CAP == 4096, "CAP is 2048 or 4096");
    constexpr int NB = CAP;
    constexpr int kBB = CAP == 2048 ? 11 : 12;
    constexpr int kHS = 2 * CAP, kHB = (CAP == 2048 ? 12 : 13);
    // sizes pass with u32 offsets: the union's size by LDS hash-set inserts, no sort (HASH)
    constexpr bool HASH = !WRITE && sizeof(K) == 4;
    // the unit's codes as offsets from its first code: u32 whenever every unit spans < 2^32 codes
    __shared__ __attribute__((aligned(16))) K scode[HASH ? 1 : CAP];
    __shared__ __attribute__((aligned(16))) uint16_t sidx[HASH ? 1 : CAP];
    __shared__ __attribute__((aligned(16))) uint32_t htab[HASH ? kHS : 1];   // HASH: offset + 1, 0 = empty
    __shared__ uint32_t htop;   // HASH: the offset 2^32 - 1 (no room for + 1) occurs
    __shared__ __attribute__((aligned(16))) uint32_t hist[NB];
    __shared__ uint32_t colrel[WRITE ? CAP : 1];   // WRITE: column of gathered entry i - the unit's first
    // dynamic: the rows' offsets (the first kShRoffCache; the rest read from memory), and two
    // piece tables (this unit's, the next unit's): the pieces' exclusive prefix of their sizes
    // (R + 1) and their first entries (relative to their rows)
    extern __shared__ __attribute__((aligned(16))) uint64_t sdyn[];
    uint64_t* const sroff = sdyn;
    uint32_t* const ptab = reinterpret_cast<uint32_t*>(sdyn + (R < kShRoffCache ? R : kShRoffCache));
    auto pfx_of = [&](int k) { return ptab + (uint32_t)k * (2u * (uint32_t)R + 1u); };
    auto pa_of = [&](int k) { return ptab + (uint32_t)k * (2u * (uint32_t)R + 1u) + (uint32_t)R + 1u; };
    // up to kShSlotRows rows, two more tables: row r's piece as one offset, dl[r] = the row's base +
    // its piece's first entry - the entries gathered before it, so gathered entry i of row r is at
    // dl[r] + i in the rows' arrays (codes and indices alike): one LDS read per address, not three
    uint64_t* const dtab = reinterpret_cast<uint64_t*>(
        reinterpret_cast<char*>(ptab) + ((2u * (2u * (uint32_t)R + 1u)) * 4u + 15u) / 16u * 16u);
    auto dl_of = [&](int k) { return dtab + (uint32_t)k * (uint32_t)R; };
    __shared__ uint32_t ws[NT / 64];
    __shared__ uint32_t flag;
    // up to kShSlotRows rows: the row holding gathered entry 64 m of piece table k (rtab[k][m])
    __shared__ uint8_t rtab[2][CAP / 64];
    constexpr int PER = CAP / NT;   // entries per thread
    constexpr int BPT = NB / NT;   // bins per thread
    static_assert(BPT % 4 == 0, "a thread's bins are cleared and checked as 16-byte words");
    const int tid = threadIdx.x;
    for (int r = tid; r < R && r < kShRoffCache; r += NT) sroff[r] = roff[r];
    // (made visible by the first barriers)
    auto row_base = [&](int r) { return r < kShRoffCache ? sroff[r] : roff[r]; };

    // the rows of PER gathered entries at once (table k): up to kShSlotRows rows, the row of the entry's
    // 64-entry slot (rtab, written by build) and then over the row starts up to the entry (a
    // 64-entry window crosses about 64 R / T of them; counting all R row starts per entry cost
    // 2 (R - 1) VALU operations); beyond kShSlotRows rows by binary search
    auto rows_of = [&](const uint32_t* pfx, const uint8_t* rt, const uint32_t (&iv)[PER], int (&rv)[PER]) {
        if (R <= kShSlotRows) {   // (uniform)
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                int r = rt[iv[u] >> 6];
                while (r + 1 < R && pfx[r + 1] <= iv[u]) ++r;
                rv[u] = r;
            }
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                int a = 0, b = R - 1;
                while (a < b) {
                    const int m = (a + b + 1) >> 1;
                    if (pfx[m] <= iv[u]) a = m;
                    else b = m - 1;
                }
                rv[u] = a;
            }
        }
    };
    // next unit's row starts: prefetched into registers when there is one row per thread
    const bool pipe_st = R <= NT;   // (uniform)
    uint32_t sta = 0u, stb = 0u;
    auto issue_st = [&](uint32_t u) {
        if (pipe_st && tid < R) {
            const uint64_t o = (uint64_t)u * (uint64_t)R + tid;
            sta = st[o];
            stb = st[o + (uint64_t)R];
        }
    };
    // the pieces of unit u into table k (block scan: every thread calls it); returns the entries
    auto build = [&](uint32_t u, int k) -> uint32_t {
        uint32_t* const pfx = pfx_of(k);
        uint32_t* const pa = pa_of(k);
        // (R > NT: a contiguous run of rows per thread, so that the block scan of the
        // threads' sums is the rows' prefix in row order)
        const int rq = (R + NT - 1) / NT, r0 = min(R, tid * rq), r1 = min(R, r0 + rq);
        uint32_t mine = 0u;
        if (pipe_st) {
            if (tid < R) {
                pa[tid] = sta;
                mine = stb - sta;
            }
        } else {
            for (int r = r0; r < r1; ++r) {
                const uint64_t o = (uint64_t)u * (uint64_t)R + r;
                pa[r] = st[o];
                mine += st[o + (uint64_t)R] - st[o];
            }
        }
        uint32_t T;
        uint32_t pre = block_scan<NT>(mine, ws, &T);
        if (pipe_st) {
            if (tid < R) pfx[tid] = pre;
        } else {
            for (int r = r0; r < r1; ++r) {
                const uint64_t o = (uint64_t)u * (uint64_t)R + r;
                pfx[r] = pre;
                pre += st[o + (uint64_t)R] - st[o];
            }
        }
        if (tid == 0) pfx[R] = T;
        if (R <= kShSlotRows && tid < R) dl_of(k)[tid] = row_base(tid) + pa[tid] - pre;   // (pipe_st: one row per thread)
        if (R <= kShSlotRows && tid < R && mine) {   // (one row per thread) the 64-entry slots starting in this row
            // (a unit over CAP entries is not gathered: its slots past the table are skipped)
            for (uint32_t m = (pre + 63u) >> 6; (m << 6) < pre + mine && m < (uint32_t)(CAP / 64); ++m)
                rtab[k][m] = (uint8_t)tid;
        }
        return T;
    };
    // the codes of a unit of T (1 .. CAP) entries, table k (visible), all loads in flight;
    // WRITE with up to kShSlotRows rows: the entries' rows packed a byte each into rk, for the index stores
    auto gather = [&](uint32_t T, int k, K (&cv)[PER], uint32_t (&rk)[2]) {
        const uint32_t* const pfx = pfx_of(k);
        const uint32_t* const pa = pa_of(k);
        uint32_t iv[PER];
        int rv[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = (uint32_t)(u * NT + tid);
            iv[u] = i < T ? i : T - 1u;
        }
        rows_of(pfx, rtab[k], iv, rv);
        if (WRITE && R <= kShSlotRows) {
            rk[0] = (uint32_t)rv[0] | (uint32_t)rv[1] << 8 | (uint32_t)rv[2] << 16 | (uint32_t)rv[3] << 24;
            rk[1] = (uint32_t)rv[4] | (uint32_t)rv[5] << 8 | (uint32_t)rv[6] << 16 | (uint32_t)rv[7] << 24;
        }
        uint64_t at[PER];
        if (R <= kShSlotRows) {   // (uniform)
            const uint64_t* const dl = dl_of(k);
#pragma unroll
            for (int u = 0; u < PER; ++u) at[u] = dl[rv[u]] + iv[u];
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) at[u] = row_base(rv[u]) + pa[rv[u]] + (iv[u] - pfx[rv[u]]);
        }
        // (u32 offsets: only the codes' low words are loaded -- a u64 load whose high half the
        // compiler knew to be dead had that half's register reused while the load was in flight,
        // and the wait for it (vmcnt) drained the prefetch at the start of the sort)
        if constexpr (sizeof(K) == 4) {
#pragma unroll
            for (int u = 0; u < PER; ++u) cv[u] = reinterpret_cast<const uint32_t*>(codes)[2 * at[u]];
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) cv[u] = codes[at[u]];
        }
    };

    uint32_t s = blockIdx.x;
    if (s >= S) return;   // (whole workgroup)
    issue_st(s);
    uint32_t Tc = build(s, 0);
    lds_barrier();
    K cv[PER];   // a unit's codes (u32 offsets: their low words; the offsets wrap correctly)
#pragma unroll
    for (int u = 0; u < PER; ++u) cv[u] = (K)0;
    uint32_t rk[2] = {0u, 0u}, rk2[2] = {0u, 0u};   // (this unit's rows, the next unit's)
    if (Tc >= 1u && Tc <= (uint32_t)CAP) gather(Tc, 0, cv, rk);
    unsigned long long cb = WRITE ? colbase[s] : 0ull;
    int k = 0;
#ifdef KMH_EXPERIMENTS
    unsigned long long pt_[16] = {}, tl_ = clock64();
#endif
    for (;;) {
        const uint32_t s2 = s + gridDim.x;
        const bool has2 = s2 < S;   // (uniform)
        if (has2) issue_st(s2);
        const unsigned long long cb2 = WRITE && has2 ? colbase[s2] : 0ull;
        {
            uint4* const hz = reinterpret_cast<uint4*>(hist);
#pragma unroll
            for (int q = 0; q < BPT / 4; ++q) hz[q * NT + tid] = make_uint4(0u, 0u, 0u, 0u);
        }
        if constexpr (HASH) {
            uint4* const h4 = reinterpret_cast<uint4*>(htab);
#pragma unroll
            for (int q = 0; q < kHS / 4 / NT; ++q) h4[q * NT + tid] = make_uint4(0u, 0u, 0u, 0u);
        }
        if (tid == 0) {
            flag = 0u;
            htop = 0u;
        }
        lds_barrier();
        KMH_SPT(0)
        const uint32_t T = Tc;
        const bool ok = T >= 1u && T <= (uint32_t)CAP;   // (uniform)
        if (!ok && !WRITE && tid == 0) {   // empty (a part of a coarse cell with no entries) or too big
            ucount[s] = 0u;
            if (T > (uint32_t)CAP) big[1 + atomicAdd(big, 1u)] = s;
        }
        bool sorted_ok = false;
        uint64_t base = 0ull;
        int bsh = 0;
        uint32_t nf = 0u;   // HASH: this thread's first occurrences
        // the unit's codes have landed here on every path (an empty unit included): otherwise the
        // next gather, writing the same registers, waited for them (vmcnt) behind this unit's
        // stores -- the loads and stores share one in-order counter
#pragma unroll
        for (int u = 0; u < PER; ++u) asm volatile("" : "+v"(cv[u]));
        if (ok) {
            // 2. bins: 12 bits over the unit's span, counted
            base = ub[s];
            const uint64_t span1 = ue[s] - base;   // span - 1
            const int sbits = span1 ? 64 - __builtin_clzll(span1) : 0;
            bsh = sbits > kBB ? sbits - kBB : 0;
            uint32_t bv[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const uint32_t i = (uint32_t)(u * NT + tid);
                bv[u] = (uint32_t)min((K)(cv[u] - (K)base) >> bsh, (K)(NB - 1));
                if (i < T) atomicAdd(&hist[bv[u]], 1u);
            }
            if constexpr (HASH) {
                // the union's size: inserts into an LDS hash set (linear probing, load <= 1/2); an
                // entry counts iff its insert finds an empty slot -- no scan, scatter or sort.  An
                // entry alone in its bin (~40 %) has no equal and counts without an insert.
                lds_barrier();   // (the histogram complete)
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const uint32_t i = (uint32_t)(u * NT + tid);
                    if (i < T) {
                        const uint32_t off = (uint32_t)(cv[u] - (K)base);
                        if (hist[bv[u]] == 1u) {
                            ++nf;
                        } else if (off == 0xFFFFFFFFu) {
                            htop = 1u;
                        } else {
                            const uint32_t key = off + 1u;
                            uint32_t h = (key * 0x9E3779B1u) >> (32 - kHB);
                            for (;;) {
                                const uint32_t old = atomicCAS(&htab[h], 0u, key);
                                if (old == 0u) {
                                    ++nf;
                                    break;
                                }
                                if (old == key) break;
                                h = (h + 1u) & (uint32_t)(kHS - 1);
                            }
                        }
                    }
                }
            }
            lds_barrier();
            KMH_SPT(1)
            // 3. bin starts (start | start << 16); a bin over kShBin entries sends s to the fallback
            //    (HASH: only the check -- the write pass's sort holds the same bins)
            if constexpr (HASH) {
                const uint4* const hv = reinterpret_cast<const uint4*>(hist + BPT * tid);
                uint32_t mx = 0u;
#pragma unroll
                for (int q = 0; q < BPT / 4; ++q) {
                    const uint4 v = hv[q];
                    mx = max(max(mx, max(v.x, v.y)), max(v.z, v.w));
                }
                if (mx > (uint32_t)kShBin) flag = 1u;
            } else {
                uint32_t v[BPT], sum = 0u;
#pragma unroll
                for (int q = 0; q < BPT; ++q) {
                    v[q] = hist[BPT * tid + q];
                    sum += v[q];
                    if (v[q] > (uint32_t)kShBin) flag = 1u;
                }
                uint32_t tot;
                uint32_t o = block_scan<NT>(sum, ws, &tot);
#pragma unroll
                for (int q = 0; q < BPT; ++q) {
                    hist[BPT * tid + q] = o * 0x10001u;
                    o += v[q];
                }
            }
            lds_barrier();
            KMH_SPT(2)
            sorted_ok = flag == 0u;   // (uniform)
            if (!sorted_ok && !WRITE && tid == 0) {
                ucount[s] = 0u;
                big[1 + atomicAdd(big, 1u)] = s;
            }
            if (!HASH && sorted_ok) {
                // 4. scatter by bin (hist ends as start | end << 16)
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const uint32_t i = (uint32_t)(u * NT + tid);
                    if (i < T) {
                        const uint32_t at = atomicAdd(&hist[bv[u]], 0x10000u) >> 16;
                        scode[at] = (K)(cv[u] - (K)base);
                        sidx[at] = (uint16_t)i;
                    }
                }
            }
        }
        // this unit's codes are dead: the next unit's pieces, then its loads (landing during
        // this unit's sort, heads and stores)
        KMH_SPT(3)
        uint32_t T2 = 0u;
        if (has2) T2 = build(s2, k ^ 1);   // (its barriers also order the scatter before the sort)
        lds_barrier();
        KMH_SPT(4)
        if (has2 && T2 >= 1u && T2 <= (uint32_t)CAP) gather(T2, k ^ 1, cv, rk2);
        KMH_SPT(5)
        if (HASH && sorted_ok) {
            uint32_t U;
            block_scan<NT>(nf + (tid == 0 ? htop : 0u), ws, &U);
            if (tid == 0) ucount[s] = U;
        }
        if (!HASH && !WRITE && sorted_ok) {
            // the union's size needs no order: position p counts iff no earlier position of its
            // bin holds its code (bins of up to 4 entries: 4 reads clamped into the bin)
            uint32_t nf = 0u;
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const uint32_t p = (uint32_t)(u * NT + tid), pc = p < T ? p : 0u;
                const K key = scode[pc];
                const uint32_t b = (uint32_t)min(key >> bsh, (K)(NB - 1));
                const uint32_t h = hist[b], bs = h & 0xFFFFu, be = h >> 16;
                bool first = true;
                if (be - bs <= 4u) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const uint32_t y = bs + (uint32_t)t;
                        const K o = scode[y < be ? y : bs];
                        first = first && !(y < pc && o == key);
                    }
                } else {
                    for (uint32_t y = bs; y < pc; ++y) first = first && scode[y] != key;
                }
                nf += (p < T && first) ? 1u : 0u;
            }
            uint32_t U;
            block_scan<NT>(nf, ws, &U);
            if (tid == 0) ucount[s] = U;
        }
        if (WRITE && sorted_ok) {
            const uint32_t* const pfx = pfx_of(k);
            const uint32_t* const pa = pa_of(k);
            // 5. each bin in code order, by rank: position p of a bin [bs, be) moves to bs + the
            //    number of the bin's entries ordered before it (smaller code, or the same code at
            //    an earlier position).  Bins of up to 4 entries (~0.75 per bin; nearly all) read
            //    those 4 slots at addresses clamped into the bin, all of a thread's positions
            //    together and branch-free; larger bins (at most kShBin) loop.  Reads, barrier,
            //    writes.  (An insertion sort per bin was a chain of dependent LDS round trips that
            //    the whole wave took for every bin slot in which one of its lanes had a bin to sort.)
            {
                // (a position's destination and its gathered index packed in one register, dst |
                // index << 16, 0xFFFF = stays: fewer live registers through the sort)
                K key[PER];
                uint32_t dk[PER];
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const uint32_t p = (uint32_t)(u * NT + tid), pc = p < T ? p : 0u;
                    key[u] = scode[pc];
                    dk[u] = (uint32_t)sidx[pc] << 16;
                }
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const uint32_t p = (uint32_t)(u * NT + tid), pc = p < T ? p : 0u;
                    const uint32_t b = (uint32_t)min(key[u] >> bsh, (K)(NB - 1));
                    const uint32_t h = hist[b], bs = h & 0xFFFFu, be = h >> 16;
                    uint32_t rk = 0u;
                    if (be - bs <= 1u) {
                        // a bin of one entry stays in place (~40 % of the entries): no reads
                    } else if (be - bs <= 4u) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const uint32_t y = bs + (uint32_t)t;
                            const K o = scode[y < be ? y : bs];
                            rk += (y < be && (o < key[u] || (o == key[u] && y < pc))) ? 1u : 0u;
                        }
                    } else {
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
                        for (uint32_t y = bs; y < be; ++y) {   // (rare: kept small, no spills)
                            const K o = scode[y];
                            rk += (o < key[u] || (o == key[u] && y < pc)) ? 1u : 0u;
                        }
                    }
                    dk[u] |= p < T && be - bs > 1u ? bs + rk : 0xFFFFu;   // (single entries stay)
                }
                lds_barrier();
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const uint32_t d = dk[u] & 0xFFFFu;
                    if (d != 0xFFFFu) {
                        scode[d] = key[u];
                        sidx[d] = (uint16_t)(dk[u] >> 16);
                    }
                }
            }
            lds_barrier();
            KMH_SPT(6)
            // 6. run heads = the distinct codes; thread t owns positions PER t .. PER t + PER - 1,
            //    read as 16-byte vectors (PER single reads at a stride of PER words were 8-way bank
            //    conflicts); positions past T hold stale codes and are masked
            static_assert(PER == 8, "a thread's positions are two (u32) or four (u64) 16-byte reads");
            K kv[PER];
            {
                const uint4* const sv = reinterpret_cast<const uint4*>(scode + PER * tid);
                if constexpr (sizeof(K) == 4) {
                    const uint4 a = sv[0], b = sv[1];
                    kv[0] = a.x; kv[1] = a.y; kv[2] = a.z; kv[3] = a.w;
                    kv[4] = b.x; kv[5] = b.y; kv[6] = b.z; kv[7] = b.w;
                } else {
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const uint4 a = sv[w];
                        kv[2 * w] = (K)a.x | ((K)a.y << 32);
                        kv[2 * w + 1] = (K)a.z | ((K)a.w << 32);
                    }
                }
            }
            const K prev = tid ? scode[PER * tid - 1] : (K)0;
            uint32_t hm = 0u, nh = 0u;
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const uint32_t p = (uint32_t)(PER * tid + u);
                const bool h = p < T && (p == 0u || kv[u] != (u ? kv[u - 1] : prev));
                hm |= (uint32_t)h << u;
                nh += (uint32_t)h;
            }
            uint32_t U;
            const uint32_t hp = block_scan<NT>(nh, ws, &U);
            KMH_SPT(7)
            {
                // the columns from the heads; every entry's column (relative to the unit's
                // first) into LDS by its gathered index, then stored in gathered order:
                // consecutive threads write consecutive entries of a row's piece (stored by
                // sorted position they scattered over the rows' pieces)
                uint32_t run = hp;   // heads before this thread's positions
                const uint4 ix = *reinterpret_cast<const uint4*>(sidx + PER * tid);
                const uint32_t ixw[4] = {ix.x, ix.y, ix.z, ix.w};
                // the heads compacted into scode[0, U) (every thread read its positions before the
                // scan's barriers, and a head moves down only), then stored lane-consecutively:
                // a thread's own heads, PER words apart across the lanes, made each store a
                // separate 64-byte request per lane
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const uint32_t p = (uint32_t)(PER * tid + u);
                    if (p < T) {
                        if ((hm >> u) & 1u) {
                            scode[run] = kv[u];
                            ++run;
                        }
                        colrel[(ixw[u >> 1] >> (16 * (u & 1))) & 0xFFFFu] = run - 1u;
                    }
                }
                lds_barrier();
                for (uint32_t j = (uint32_t)tid; j < U; j += NT) columns[cb + j] = base + (uint64_t)scode[j];
                KMH_SPT(8)
                if (R <= kShSlotRows) {   // (uniform) the rows found by the gather; all LDS reads, then the stores
                    const uint64_t* const dl = dl_of(k);
                    uint64_t ad[PER];
                    uint32_t cr[PER];
#pragma unroll
                    for (int u = 0; u < PER; ++u) {
                        const uint32_t i = (uint32_t)(u * NT + tid), ic = i < T ? i : 0u;
                        ad[u] = dl[(rk[u >> 2] >> (8 * (u & 3))) & 0xFFu] + ic;
                        cr[u] = colrel[ic];
                    }
#pragma unroll
                    for (int u = 0; u < PER; ++u)
                        if ((uint32_t)(u * NT + tid) < T) indices[ad[u]] = (IX)(cb + cr[u]);
                } else {
                    int rv[PER];
                    uint32_t iv[PER];
#pragma unroll
                    for (int u = 0; u < PER; ++u) {
                        const uint32_t i = (uint32_t)(u * NT + tid);
                        iv[u] = i < T ? i : 0u;
                    }
                    rows_of(pfx, rtab[k], iv, rv);
#pragma unroll
                    for (int u = 0; u < PER; ++u) {
                        const uint32_t i = (uint32_t)(u * NT + tid);
                        if (i < T) indices[row_base(rv[u]) + pa[rv[u]] + (i - pfx[rv[u]])] = (IX)(cb + colrel[i]);
                    }
                }
                KMH_SPT(9)
            }
        }
        if (!has2) break;
        lds_barrier();   // the LDS tables are rewritten by the next unit
        KMH_SPT(10)
        s = s2;
        Tc = T2;
        k ^= 1;
        cb = cb2;
        rk[0] = rk2[0];
        rk[1] = rk2[1];
    }
#ifdef KMH_EXPERIMENTS
    if (tid == 0) {
        pt_[11] = 1u;
        for (int i = 0; i < 12; ++i) atomicAdd(&g_shard_pt[WRITE ? 1 : 0][i], pt_[i]);
    }
#endif
}

// Exclusive u64 scan of n u32: out[i] = sum of in[0 .. i), out[n] = the total.  Blocks of 4096
// (256 threads x 16): block sums, one workgroup scans them, then every block scans itself from its
// base.  (A single workgroup walking 1/1024 of the input per thread took 1.45 ms for the 1.3 M
// units of config 5.)
constexpr int kScPer = 16, kScBlock = 256 * kScPer;

__global__ __launch_bounds__(256) void k_shard_scan_sums(const uint32_t* __restrict__ in, uint32_t n,
                                                         unsigned long long* __restrict__ bsum) {
    __shared__ unsigned long long ws[4];
    const uint32_t base = blockIdx.x * (uint32_t)kScBlock;
    unsigned long long t = 0ull;
#pragma unroll
    for (int j = 0; j < kScPer; ++j) {
        const uint32_t i = base + (uint32_t)j * 256u + threadIdx.x;
        t += i < n ? in[i] : 0u;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d);
    if ((threadIdx.x & 63u) == 0u) ws[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// In place: bsum[b] = the sum of the blocks before b; bsum[nb] = the total (one workgroup).
__global__ __launch_bounds__(kShScanThreads) void k_shard_scan_top(unsigned long long* __restrict__ bsum, uint32_t nb) {
    __shared__ unsigned long long ws[kShScanThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t per = (nb + kShScanThreads - 1u) / kShScanThreads, a = min(nb, tid * per), e = min(nb, a + per);
    unsigned long long s = 0ull;
    for (uint32_t i = a; i < e; ++i) s += bsum[i];
    unsigned long long incl = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long x = __shfl_up(incl, d);
        if ((int)lane >= d) incl += x;
    }
    if (lane == 63u) ws[wave] = incl;
    __syncthreads();
    unsigned long long p = incl - s;
    for (uint32_t w = 0; w < wave; ++w) p += ws[w];
    for (uint32_t i = a; i < e; ++i) {
        const unsigned long long x = bsum[i];
        bsum[i] = p;
        p += x;
    }
    if (tid == kShScanThreads - 1u) bsum[nb] = p;
}

__global__ __launch_bounds__(256) void k_shard_scan_down(const uint32_t* __restrict__ in, uint32_t n,
                                                         const unsigned long long* __restrict__ bsum, uint32_t nb,
                                                         unsigned long long* __restrict__ out) {
    __shared__ unsigned long long ws[4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t a = blockIdx.x * (uint32_t)kScBlock + threadIdx.x * (uint32_t)kScPer;
    uint32_t v[kScPer];
    unsigned long long t = 0ull;
#pragma unroll
    for (int j = 0; j < kScPer; ++j) {
        v[j] = a + (uint32_t)j < n ? in[a + j] : 0u;
        t += v[j];
    }
    unsigned long long incl = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long x = __shfl_up(incl, d);
        if ((int)lane >= d) incl += x;
    }
    if (lane == 63u) ws[wave] = incl;
    __syncthreads();
    unsigned long long p = bsum[blockIdx.x] + incl - t;
    for (uint32_t w = 0; w < wave; ++w) p += ws[w];
#pragma unroll
    for (int j = 0; j < kScPer; ++j) {
        if (a + (uint32_t)j < n) out[a + j] = p;
        p += v[j];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = bsum[nb];
}

// Fallback, sizes: entries of every listed sub-range (big[1 .. nbig]).
__global__ __launch_bounds__(256) void k_shard_big_sizes(const uint32_t* __restrict__ st, int R, uint32_t S,
                                                         const uint32_t* __restrict__ bigs, uint32_t nbig,
                                                         uint32_t* __restrict__ sizes) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= nbig) return;
    const uint32_t s = bigs[j];
    uint32_t t = 0u;
    for (int r = 0; r < R; ++r) t += st[(uint64_t)(s + 1u) * R + r] - st[(uint64_t)s * R + r];
    sizes[j] = t;
}

// Fallback, gather: the entries of listed sub-range j (block j) to goff[j] ..: their codes and
// their positions in the rows' array.
__global__ __launch_bounds__(256) void k_shard_big_gather(const uint64_t* __restrict__ codes,
                                                          const uint64_t* __restrict__ roff, int R,
                                                          const uint32_t* __restrict__ st, uint32_t S,
                                                          const uint32_t* __restrict__ bigs,
                                                          const unsigned long long* __restrict__ goff,
                                                          uint64_t* __restrict__ gcode, uint64_t* __restrict__ gpos,
                                                          uint32_t* __restrict__ gval) {
    const uint32_t j = blockIdx.x, s = bigs[j];
    unsigned long long o = goff[j];
    for (int r = 0; r < R; ++r) {
        const uint32_t a = st[(uint64_t)s * R + r], b = st[(uint64_t)(s + 1u) * R + r];
        for (uint32_t i = a + threadIdx.x; i < b; i += 256u) {
            const unsigned long long t = o + (i - a);
            gcode[t] = codes[roff[r] + i];
            gpos[t] = roff[r] + i;
            gval[t] = (uint32_t)t;
        }
        o += b - a;
    }
}

// Fallback, runs: every run of the sorted gathered codes adds one to its sub-range's count.
__global__ __launch_bounds__(256) void k_shard_big_count(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ starts,
                                                         const uint32_t* __restrict__ nruns,
                                                         const uint64_t* __restrict__ ub, uint32_t U,
                                                         uint32_t* __restrict__ ucount) {
    const uint32_t n = *nruns;
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < n; r += gridDim.x * 256u)
        atomicAdd(&ucount[unit_of(ub, U, keys[starts[r]])], 1u);
}

// Fallback, write: run r's column = colbase[its sub-range] + (r - the sub-range's first run);
// every entry of the run gets it.
template <typename IX>
__global__ __launch_bounds__(256) void k_shard_big_write(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, uint64_t m,
                                                         const uint32_t* __restrict__ starts,
                                                         const uint32_t* __restrict__ nruns,
                                                         const uint64_t* __restrict__ ub, uint32_t U,
                                                         const unsigned long long* __restrict__ colbase,
                                                         const uint64_t* __restrict__ gpos,
                                                         uint64_t* __restrict__ columns, IX* __restrict__ indices) {
    const uint32_t n = *nruns;
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < n; r += gridDim.x * 256u) {
        const uint64_t c = keys[starts[r]];
        const uint32_t s = unit_of(ub, U, c);
        uint32_t a = 0u, b = r;   // the first run of unit s
        while (a < b) {
            const uint32_t mid = (a + b) / 2u;
            if (unit_of(ub, U, keys[starts[mid]]) < s) a = mid + 1u;
            else b = mid;
        }
        const unsigned long long col = colbase[s] + (r - a);
        columns[col] = c;
        const uint64_t e = r + 1u < n ? starts[r + 1u] : m;
        for (uint64_t t = starts[r]; t < e; ++t) indices[gpos[vals[t]]] = (IX)col;
    }
}

}  // namespace

// out[0 .. n] = the exclusive u64 scan of in[0 .. n) and its total (k_shard_scan_*; ctx->scan_tmp).
int scan_u32_u64(Ctx* ctx, const uint32_t* in, uint32_t n, unsigned long long* out, hipStream_t s) {
    const uint32_t nb = std::max<uint32_t>(1u, (n + kScBlock - 1) / kScBlock);
    int rc = ensure(ctx, ctx->scan_tmp, ((size_t)nb + 1) * 8 + 256);
    if (rc) return rc;
    unsigned long long* bsum = static_cast<unsigned long long*>(ctx->scan_tmp.ptr);
    hipLaunchKernelGGL(k_shard_scan_sums, dim3(nb), dim3(256), 0, s, in, n, bsum);
    KMH_HIP(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_shard_scan_top, dim3(1), dim3(kShScanThreads), 0, s, bsum, nb);
    KMH_HIP(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_shard_scan_down, dim3(nb), dim3(256), 0, s, in, n, bsum, nb, out);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

// The union's arguments and its two launches (sizes pass, write pass) in one of the two shapes.
struct UnionArgs {
    const uint64_t* codes;
    const uint64_t* roff;
    int R;
    const uint32_t* st;
    uint32_t S;
    const uint64_t *ub, *ue;
    uint32_t *ucount, *big;
    const unsigned long long* colbase;
    uint64_t* columns;
    uint32_t* ix32;
    int64_t* ix64;
    bool narrow;
    unsigned grid, grid_sizes;
    size_t dyn;
};
template <int NT, int CAP>
void launch_union(const UnionArgs& a, bool write, hipStream_t s) {
    const dim3 g(write ? a.grid : a.grid_sizes), b(NT);
    if (!write) {
        if (a.narrow)
            hipLaunchKernelGGL((k_shard_union<NT, CAP, false, uint32_t, uint32_t>), g, b, a.dyn, s, a.codes, a.roff, a.R,
                               a.st, a.S, a.ub, a.ue, a.ucount, a.big, nullptr, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_shard_union<NT, CAP, false, uint64_t, uint32_t>), g, b, a.dyn, s, a.codes, a.roff, a.R,
                               a.st, a.S, a.ub, a.ue, a.ucount, a.big, nullptr, nullptr, nullptr);
    } else if (a.narrow && a.ix32) {
        hipLaunchKernelGGL((k_shard_union<NT, CAP, true, uint32_t, uint32_t>), g, b, a.dyn, s, a.codes, a.roff, a.R, a.st,
                           a.S, a.ub, a.ue, a.ucount, a.big, a.colbase, a.columns, a.ix32);
    } else if (a.narrow) {
        hipLaunchKernelGGL((k_shard_union<NT, CAP, true, uint32_t, int64_t>), g, b, a.dyn, s, a.codes, a.roff, a.R, a.st,
                           a.S, a.ub, a.ue, a.ucount, a.big, a.colbase, a.columns, a.ix64);
    } else if (a.ix32) {
        hipLaunchKernelGGL((k_shard_union<NT, CAP, true, uint64_t, uint32_t>), g, b, a.dyn, s, a.codes, a.roff, a.R, a.st,
                           a.S, a.ub, a.ue, a.ucount, a.big, a.colbase, a.columns, a.ix32);
    } else {
        hipLaunchKernelGGL((k_shard_union<NT, CAP, true, uint64_t, int64_t>), g, b, a.dyn, s, a.codes, a.roff, a.R, a.st,
                           a.S, a.ub, a.ue, a.ucount, a.big, a.colbase, a.columns, a.ix64);
    }
}

int shard_union(Ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, uint64_t lo,
                uint64_t hi_incl, uint64_t* d_columns, void* d_indices, bool idx32, uint64_t* ncols, hipStream_t s) {
    if (R < 1 || R > kShMaxRows) return fail(ctx, KMH_ERR_UNSUPPORTED, "a shard holds 1 to 4096 organism rows");
    if (!d_codes || !row_off || !ncols || hi_incl < lo) return fail(ctx, KMH_ERR_INVALID, "bad shard arguments");
    const uint64_t T = row_off[R] - row_off[0];
    for (int r = 0; r < R; ++r)
        if (row_off[r + 1] < row_off[r] || row_off[r + 1] - row_off[r] >= 0xFFFFFFFFull)
            return fail(ctx, KMH_ERR_INVALID, "row offsets must ascend, rows below 2^32 - 1 entries");
    *ncols = 0;
    if (T == 0) return KMH_OK;
    if (idx32 && T >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "u32 column indices need fewer than 2^32 - 1 entries");
    if (!d_columns || !d_indices) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    // coarse cells of 2^CSH codes: span <= 2^nbits, at most 2^kShCoarseBits cells
    const uint64_t span1 = hi_incl - lo;   // span - 1
    const int nbits = span1 ? 64 - __builtin_clzll(span1) : 0;
    // (at most 2^25 coarse starts: 2^16 cells up to 512 rows, fewer beyond)
    int rbits = 0;
    while ((1 << rbits) < R) ++rbits;
    const int qb = std::min(std::min(kShCoarseBits, 25 - rbits), nbits), CSH = nbits - qb;
    const uint32_t Q = (uint32_t)((span1 >> CSH) + 1u);

    const size_t csb = (((size_t)R * (Q + 1) * 4) + 255) & ~(size_t)255;
    const size_t rb = (((size_t)R + 1) * 8 + 255) & ~(size_t)255;
    const size_t qb4 = (((size_t)Q + 1) * 4 + 255) & ~(size_t)255, qb8 = (((size_t)Q + 1) * 8 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->sparse[0], csb + rb + qb4 + qb8 + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint32_t* d_cs = reinterpret_cast<uint32_t*>(p);
    uint64_t* d_roff = reinterpret_cast<uint64_t*>(p + csb);
    uint32_t* d_nu = reinterpret_cast<uint32_t*>(p + csb + rb);
    unsigned long long* d_ubase = reinterpret_cast<unsigned long long*>(p + csb + rb + qb4);
    std::vector<uint64_t> rel(R + 1);
    for (int r = 0; r <= R; ++r) rel[r] = row_off[r] - row_off[0];
    const uint64_t* codes = d_codes + row_off[0];
    KMH_HIP(ctx, hipMemcpyAsync(d_roff, rel.data(), (R + 1) * 8, hipMemcpyHostToDevice, s));
    time_begin(ctx, s, "k_shard_plan");
    const uint64_t ncs = (uint64_t)(Q + 1) * (uint64_t)R;
    hipLaunchKernelGGL(k_shard_coarse, dim3((unsigned)((ncs + 255) / 256)), dim3(256), 0, s, codes, d_roff, R, lo, CSH, Q,
                       d_cs);
    KMH_HIP(ctx, hipGetLastError());
    const bool small = R <= kShSmallRows;   // the union's shape
    const uint32_t target = small ? 1792u : 3584u;
    hipLaunchKernelGGL(k_shard_cells, dim3((Q + 255) / 256), dim3(256), 0, s, d_cs, R, Q, lo, hi_incl, CSH, target, d_nu);
    KMH_HIP(ctx, hipGetLastError());
    if ((rc = scan_u32_u64(ctx, d_nu, Q, d_ubase, s))) return rc;
    unsigned long long U64 = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&U64, d_ubase + Q, 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (U64 == 0 || U64 >= (1ull << 31)) return fail(ctx, KMH_ERR_UNSUPPORTED, "shard: unit count out of range");
    const uint32_t S = (uint32_t)U64;

    // units: first / last codes, cells; the rows' starts; union sizes, fallback list, column bases
    const size_t stb = (((size_t)R * (S + 1) * 4) + 255) & ~(size_t)255;
    const size_t u8 = (((size_t)S + 1) * 8 + 255) & ~(size_t)255, u4 = (((size_t)S + 1) * 4 + 255) & ~(size_t)255;
    if ((rc = ensure(ctx, ctx->sparse[1], stb + 2 * u8 + 5 * u4 + 2 * u8 + 1024))) return rc;
    char* p1 = static_cast<char*>(ctx->sparse[1].ptr);
    uint32_t* d_st = reinterpret_cast<uint32_t*>(p1);
    uint64_t* d_ub = reinterpret_cast<uint64_t*>(p1 + stb);
    uint64_t* d_ue = reinterpret_cast<uint64_t*>(p1 + stb + u8);
    uint32_t* d_ucell = reinterpret_cast<uint32_t*>(p1 + stb + 2 * u8);
    uint32_t* d_ucount = reinterpret_cast<uint32_t*>(p1 + stb + 2 * u8 + u4);
    uint32_t* d_big = reinterpret_cast<uint32_t*>(p1 + stb + 2 * u8 + 2 * u4);   // [0] = count, then units
    uint32_t* d_bigs = reinterpret_cast<uint32_t*>(p1 + stb + 2 * u8 + 3 * u4);
    uint32_t* d_sizes = reinterpret_cast<uint32_t*>(p1 + stb + 2 * u8 + 4 * u4);
    unsigned long long* d_colbase = reinterpret_cast<unsigned long long*>(p1 + stb + 2 * u8 + 5 * u4);
    unsigned long long* d_goff = reinterpret_cast<unsigned long long*>(p1 + stb + 3 * u8 + 5 * u4);
    hipLaunchKernelGGL(k_shard_units, dim3((Q + 255) / 256), dim3(256), 0, s, d_nu, d_ubase, Q, lo, hi_incl, CSH, d_ub,
                       d_ue, d_ucell);
    KMH_HIP(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_shard_ustarts, dim3((unsigned)(((uint64_t)S + 1 + kUsU - 1) / kUsU)), dim3(256), 0, s, codes, d_roff, R, d_cs, Q,
                       lo, hi_incl, CSH, d_ub, d_ucell, S, d_st);
    KMH_HIP(ctx, hipGetLastError());
    KMH_HIP(ctx, hipMemsetAsync(d_big, 0, 4, s));
    time_end(ctx, s);
    const unsigned ug = (unsigned)std::min<uint64_t>(S, (uint64_t)std::max(1, ctx->num_cu) * (small ? 4 : 2));
    const size_t dyn = (size_t)std::min(R, kShRoffCache) * 8 + ((2 * ((size_t)2 * R + 1)) * 4 + 15) / 16 * 16 +
                       (R <= kShSlotRows ? (size_t)2 * R * 8 : 0);
    // every unit lies inside one coarse cell of 2^CSH codes: u32 offsets when CSH <= 32
    // (indices at the rows' own offsets: row_off[0] may be past the start of d_indices)
    UnionArgs ua{codes, d_roff, R, d_st, S, d_ub, d_ue, d_ucount, d_big, d_colbase, d_columns,
                 idx32 ? static_cast<uint32_t*>(d_indices) + row_off[0] : nullptr,
                 idx32 ? nullptr : static_cast<int64_t*>(d_indices) + row_off[0], CSH <= 32, ug,
                 (unsigned)std::min<uint64_t>(S, (uint64_t)std::max(1, ctx->num_cu) * (small ? 5 : 2)), dyn};
    uint32_t* const ix32 = ua.ix32;
    int64_t* const ix64 = ua.ix64;
#ifdef KMH_EXPERIMENTS
    {
        unsigned long long z[2][16] = {};
        KMH_HIP(ctx, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_shard_pt), z, sizeof(z), 0, hipMemcpyHostToDevice, s));
    }
#endif
    time_begin(ctx, s, "k_shard_union");
    if (small) launch_union<256, 2048>(ua, false, s);
    else launch_union<512, 4096>(ua, false, s);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    uint32_t nbig = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&nbig, d_big, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));

    // the fallback's entries: sizes, gather, radix sort, runs (their union sizes go into ucount)
    uint64_t m = 0;
    uint64_t *gcode = nullptr, *gpos = nullptr;
    uint32_t *gval = nullptr, *starts = nullptr, *nruns = nullptr;
    bool alt = false;
    if (nbig) {
        std::vector<uint32_t> bigs(nbig), sizes(nbig);
        KMH_HIP(ctx, hipMemcpyAsync(bigs.data(), d_big + 1, (size_t)nbig * 4, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        std::sort(bigs.begin(), bigs.end());
        KMH_HIP(ctx, hipMemcpyAsync(d_bigs, bigs.data(), (size_t)nbig * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_shard_big_sizes, dim3((nbig + 255) / 256), dim3(256), 0, s, d_st, R, S, d_bigs, nbig, d_sizes);
        KMH_HIP(ctx, hipGetLastError());
        KMH_HIP(ctx, hipMemcpyAsync(sizes.data(), d_sizes, (size_t)nbig * 4, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        std::vector<unsigned long long> goff(nbig + 1, 0ull);
        for (uint32_t j = 0; j < nbig; ++j) goff[j + 1] = goff[j] + sizes[j];
        m = goff[nbig];
        if (m >= 0xFFFFFFFFull)
            return fail(ctx, KMH_ERR_UNSUPPORTED, "shard: 2^32 or more entries in units the LDS cannot hold");
        KMH_HIP(ctx, hipMemcpyAsync(d_goff, goff.data(), (nbig + 1) * 8, hipMemcpyHostToDevice, s));
        const size_t m8 = ((size_t)m * 8 + 255) & ~(size_t)255, m4 = ((size_t)m * 4 + 255) & ~(size_t)255;
        if ((rc = ensure(ctx, ctx->order, 3 * m8 + 6 * m4 + 1024))) return rc;
        char* q = static_cast<char*>(ctx->order.ptr);
        gcode = reinterpret_cast<uint64_t*>(q);
        uint64_t* gcode2 = reinterpret_cast<uint64_t*>(q + m8);
        gpos = reinterpret_cast<uint64_t*>(q + 2 * m8);
        gval = reinterpret_cast<uint32_t*>(q + 3 * m8);
        uint32_t* gval2 = reinterpret_cast<uint32_t*>(q + 3 * m8 + m4);
        uint32_t* flags = reinterpret_cast<uint32_t*>(q + 3 * m8 + 2 * m4);
        uint32_t* ex = reinterpret_cast<uint32_t*>(q + 3 * m8 + 3 * m4);
        starts = reinterpret_cast<uint32_t*>(q + 3 * m8 + 4 * m4);
        nruns = reinterpret_cast<uint32_t*>(q + 3 * m8 + 5 * m4);
        hipLaunchKernelGGL(k_shard_big_gather, dim3(nbig), dim3(256), 0, s, codes, d_roff, R, d_st, S, d_bigs, d_goff,
                           gcode, gpos, gval);
        KMH_HIP(ctx, hipGetLastError());
        // the codes of [lo, hi] agree above the highest bit where lo and hi differ: sort below it
        const uint64_t diff = lo ^ hi_incl;
        int hb_bit = 64;
        while (hb_bit > 1 && !((diff >> (hb_bit - 1)) & 1u)) --hb_bit;
        rc = radix_sort_pairs<uint64_t>(ctx, gcode, gcode2, gval, gval2, m, 0, hb_bit, &alt, s);
        if (rc) return rc;
        if (alt) {
            gcode = gcode2;
            gval = gval2;
        }
        rc = run_starts<uint64_t>(ctx, gcode, m, flags, ex, starts, nruns, s);
        if (rc) return rc;
        hipLaunchKernelGGL(k_shard_big_count, dim3(1024), dim3(256), 0, s, gcode, starts, nruns, d_ub, S, d_ucount);
        KMH_HIP(ctx, hipGetLastError());
    }
    if ((rc = scan_u32_u64(ctx, d_ucount, S, d_colbase, s))) return rc;
    unsigned long long total = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&total, d_colbase + S, 8, hipMemcpyDeviceToHost, s));
    time_begin(ctx, s, "k_shard_union");
    if (small) launch_union<256, 2048>(ua, true, s);
    else launch_union<512, 4096>(ua, true, s);
#ifdef KMH_EXPERIMENTS
    {
        unsigned long long z[2][16];
        KMH_HIP(ctx, hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_shard_pt), sizeof(z), 0, hipMemcpyDeviceToHost, s));
        KMH_HIP(ctx, hipStreamSynchronize(s));
        const double wg = (double)std::max(1ull, z[1][11]);
        std::fprintf(stderr, "[union write phases, Mcyc per workgroup]");
        for (int i = 0; i < 11; ++i) std::fprintf(stderr, " %d:%.2f", i, z[1][i] / wg / 1e6);
        std::fprintf(stderr, " (workgroups %.0f)\n", wg);
        const double wg0 = (double)std::max(1ull, z[0][11]);
        std::fprintf(stderr, "[union sizes phases, Mcyc per workgroup]");
        for (int i = 0; i < 11; ++i) std::fprintf(stderr, " %d:%.2f", i, z[0][i] / wg0 / 1e6);
        std::fprintf(stderr, " (workgroups %.0f)\n", wg0);
    }
#endif
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    if (nbig) {
        if (idx32)
            hipLaunchKernelGGL((k_shard_big_write<uint32_t>), dim3(1024), dim3(256), 0, s, gcode, gval, m, starts, nruns, d_ub,
                               S, d_colbase, gpos, d_columns, ix32);
        else
            hipLaunchKernelGGL((k_shard_big_write<int64_t>), dim3(1024), dim3(256), 0, s, gcode, gval, m, starts, nruns, d_ub,
                               S, d_colbase, gpos, d_columns, ix64);
        KMH_HIP(ctx, hipGetLastError());
    }
    KMH_HIP(ctx, hipStreamSynchronize(s));
    *ncols = total;
    return KMH_OK;
}

}  // namespace kmh
