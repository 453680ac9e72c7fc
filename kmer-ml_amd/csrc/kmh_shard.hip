// kmh_shard.hip -- one rank's column shard of the organisms x k-mers matrix for sparse k
// (BASELINE config 5; /root/reference/kmerml/ml/features.py:96-111, _build_matrix: the columns
// are the sorted union of every organism's labels, a missing label is 0).  Input: the rank's
// organism rows restricted to its code range [lo, hi), each row sorted by code (the rows of
// kmh_count_sparse_sorted_dev after the all-to-all), back to back in organism order.  Output:
// the sorted union of their codes (`columns`) and, for every row entry, its column index
// (`indices`): with the rows' offsets as indptr and their counts as values, the shard's CSR.
//
// The code range is cut into S sub-ranges of 2^SH codes (~2048 entries each, all rows
// together).  k_shard_starts finds where every row enters every sub-range (one pass over the
// codes, no search); then one workgroup per sub-range gathers the rows' pieces into LDS and
// sorts them by a counting sort on 13 bits of the code (~0.5 entries per bin) followed by an
// insertion sort of each bin, after which equal codes are adjacent: run heads are the union.
// k_shard_union runs twice -- the union's size per sub-range, then (after a scan) the columns
// and the indices -- so no entry moves through memory other than its code being read.  A
// sub-range that overflows the LDS (more than kShCap entries, or a bin of more than kShBin:
// codes shared by many organisms, low-complexity data) is left to an exact fallback: its
// entries are gathered, radix-sorted (kmh_sort.hip) and written the same way.
#include <algorithm>
#include <vector>

#include "kmh_device.h"

namespace kmh {
namespace {

constexpr int kShThreads = 1024;
constexpr int kShCap = 8192;        // entries of one sub-range in LDS
constexpr int kShBinBits = 13;
constexpr int kShBins = 1 << kShBinBits;
constexpr int kShBin = 32;          // entries of one bin sorted in place (more: fallback)
constexpr int kShMaxRows = 4096;    // organisms of one shard (LDS piece table)
constexpr int kShTarget = 2048;     // expected entries per sub-range

// Sub-range of code c: (c - lo) >> SH.
__device__ __forceinline__ uint64_t sub_of(uint64_t c, uint64_t lo, int SH) { return (c - lo) >> SH; }

// st[r * (S + 1) + s] = the first entry of row r (relative to the row) whose sub-range is >= s,
// for s = 0 .. S (st[.. S] = the row's length).  Entry i writes the sub-ranges (sub(i - 1),
// sub(i)]; the last entry also (sub(n - 1), S].  One grid row per organism row.
__global__ __launch_bounds__(256) void k_shard_starts(const uint64_t* __restrict__ codes,
                                                      const uint64_t* __restrict__ roff, uint64_t lo, int SH,
                                                      uint32_t S, uint32_t* __restrict__ st) {
    const uint32_t r = blockIdx.y;
    const uint64_t a = roff[r], n = roff[r + 1] - a;
    uint32_t* row = st + (uint64_t)r * (S + 1u);
    if (n == 0) {
        for (uint64_t s = (uint64_t)blockIdx.x * 256u + threadIdx.x; s <= S; s += (uint64_t)gridDim.x * 256u)
            row[s] = 0u;
        return;
    }
    // (codes outside [lo, hi] -- not a valid input -- are clamped into the last sub-range: wrong
    // columns, never a write outside the table)
    const uint64_t smax = (uint64_t)S - 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const uint64_t si = min(sub_of(codes[a + i], lo, SH), smax);
        const uint64_t sp = i ? min(sub_of(codes[a + i - 1], lo, SH), smax) + 1u : 0u;
        for (uint64_t s = sp; s <= si; ++s) row[s] = (uint32_t)i;
        if (i + 1 == n)
            for (uint64_t s = si + 1u; s <= S; ++s) row[s] = (uint32_t)n;
    }
}

// Block-wide exclusive scan of one u32 per thread (kShThreads); returns the thread's prefix,
// *total = the sum.  ws: kShThreads / 64 words of LDS.
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = scan64(v);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    uint32_t pre = 0u, tot = 0u;
#pragma unroll
    for (int w = 0; w < kShThreads / 64; ++w) {
        const uint32_t x = ws[w];
        pre += w < wave ? x : 0u;
        tot += x;
    }
    __syncthreads();   // ws reusable
    *total = tot;
    return pre + incl - v;
}

// One workgroup per sub-range (persistent: s = blockIdx.x, += gridDim.x).  WRITE = false: the
// number of distinct codes of every sub-range into ucount (0 for a sub-range left to the
// fallback, which is listed in big).  WRITE = true: the columns [colbase[s], colbase[s + 1]) and
// the column index of every entry.
template <bool WRITE>
__global__ __launch_bounds__(kShThreads) void k_shard_union(const uint64_t* __restrict__ codes,
                                                            const uint64_t* __restrict__ roff, int R,
                                                            const uint32_t* __restrict__ st, uint32_t S, uint64_t lo,
                                                            int SH, uint32_t* __restrict__ ucount,
                                                            uint32_t* __restrict__ big,
                                                            const unsigned long long* __restrict__ colbase,
                                                            uint64_t* __restrict__ columns,
                                                            int64_t* __restrict__ indices) {
    __shared__ __attribute__((aligned(16))) uint64_t scode[kShCap];
    __shared__ uint16_t sidx[kShCap];
    __shared__ uint32_t hist[kShBins];
    __shared__ uint32_t pfx[kShMaxRows + 1];   // the rows' pieces: exclusive prefix of their sizes
    __shared__ uint32_t pa[kShMaxRows];        // the pieces' first entries (relative to their rows)
    __shared__ uint32_t ws[kShThreads / 64];
    __shared__ uint32_t flag;
    constexpr int PER = kShCap / kShThreads;   // entries per thread
    constexpr int BPT = kShBins / kShThreads;  // bins per thread
    const int tid = threadIdx.x;
    const int bsh = SH > kShBinBits ? SH - kShBinBits : 0;

    // row of gathered entry i: the last row whose prefix is <= i
    auto row_of = [&](uint32_t i) {
        int a = 0, b = R - 1;
        while (a < b) {
            const int m = (a + b + 1) >> 1;
            if (pfx[m] <= i) a = m;
            else b = m - 1;
        }
        return a;
    };

    for (uint32_t s = blockIdx.x; s < S; s += gridDim.x) {
        // 1. the pieces of the rows in sub-range s
        // this thread's rows: a contiguous run of at most 4 (R <= kShMaxRows), so that the
        // block scan of the threads' sums is the rows' prefix in row order
        const int rq = (R + kShThreads - 1) / kShThreads, r0 = min(R, tid * rq), r1 = min(R, r0 + rq);
        uint32_t mine = 0u;
        for (int r = r0; r < r1; ++r) {
            const uint64_t o = (uint64_t)r * (S + 1u) + s;
            pa[r] = st[o];
            mine += st[o + 1] - st[o];
        }
        uint32_t T;
        uint32_t pre = block_scan(mine, ws, &T);
        for (int r = r0; r < r1; ++r) {
            const uint64_t o = (uint64_t)r * (S + 1u) + s;
            pfx[r] = pre;
            pre += st[o + 1] - st[o];
        }
        if (tid == 0) {
            pfx[R] = T;
            flag = 0u;
        }
        for (int q = 0; q < BPT; ++q) hist[q * kShThreads + tid] = 0u;
        if (T > (uint32_t)kShCap) {   // (uniform) too many entries: the fallback's
            if (!WRITE && tid == 0) {
                ucount[s] = 0u;
                big[1 + atomicAdd(big, 1u)] = s;
            }
            __syncthreads();
            continue;
        }
        __syncthreads();
        // 2. the codes into registers, their bins counted
        const uint64_t base = lo + ((uint64_t)s << SH);
        uint64_t cv[PER];
        uint32_t bv[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = (uint32_t)(u * kShThreads + tid);
            cv[u] = 0ull;
            bv[u] = 0u;
            if (i < T) {
                const int r = row_of(i);
                cv[u] = codes[roff[r] + pa[r] + (i - pfx[r])];
                bv[u] = (uint32_t)min((cv[u] - base) >> bsh, (uint64_t)(kShBins - 1));
                atomicAdd(&hist[bv[u]], 1u);
            }
        }
        __syncthreads();
        // 3. bin starts (start | start << 16); a bin over kShBin entries sends s to the fallback
        {
            uint32_t v[BPT], sum = 0u;
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                v[q] = hist[BPT * tid + q];
                sum += v[q];
                if (v[q] > (uint32_t)kShBin) flag = 1u;
            }
            uint32_t tot;
            uint32_t o = block_scan(sum, ws, &tot);
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                hist[BPT * tid + q] = o * 0x10001u;
                o += v[q];
            }
        }
        __syncthreads();
        if (flag) {   // (uniform)
            if (!WRITE && tid == 0) {
                ucount[s] = 0u;
                big[1 + atomicAdd(big, 1u)] = s;
            }
            __syncthreads();
            continue;
        }
        // 4. scatter by bin (hist ends as start | end << 16)
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = (uint32_t)(u * kShThreads + tid);
            if (i < T) {
                const uint32_t at = atomicAdd(&hist[bv[u]], 0x10000u) >> 16;
                scode[at] = cv[u];
                sidx[at] = (uint16_t)i;
            }
        }
        __syncthreads();
        // 5. each bin in code order (insertion sort; ~0.5 entries per bin, at most kShBin)
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const uint32_t h = hist[BPT * tid + q], bs = h & 0xFFFFu, be = h >> 16;
            for (uint32_t x = bs + 1u; x < be; ++x) {
                const uint64_t key = scode[x];
                const uint16_t ix = sidx[x];
                uint32_t y = x;
                while (y > bs && scode[y - 1u] > key) {
                    scode[y] = scode[y - 1u];
                    sidx[y] = sidx[y - 1u];
                    --y;
                }
                scode[y] = key;
                sidx[y] = ix;
            }
        }
        __syncthreads();
        // 6. run heads = the distinct codes; thread t owns positions PER t .. PER t + PER - 1
        uint32_t hm = 0u, nh = 0u;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t p = (uint32_t)(PER * tid + u);
            const bool h = p < T && (p == 0u || scode[p] != scode[p - 1u]);
            hm |= (uint32_t)h << u;
            nh += (uint32_t)h;
        }
        uint32_t U;
        const uint32_t hp = block_scan(nh, ws, &U);
        if constexpr (!WRITE) {
            if (tid == 0) ucount[s] = U;
        } else {
            const unsigned long long cb = colbase[s];
            uint32_t run = hp;   // heads before this thread's positions
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const uint32_t p = (uint32_t)(PER * tid + u);
                if (p < T) {
                    if ((hm >> u) & 1u) {
                        columns[cb + run] = scode[p];
                        ++run;
                    }
                    const uint32_t i = sidx[p];
                    const int r = row_of(i);
                    indices[roff[r] + pa[r] + (i - pfx[r])] = (int64_t)(cb + run - 1u);
                }
            }
        }
        __syncthreads();   // the LDS tables are rewritten by the next sub-range
    }
}

// Exclusive u64 scan of n u32 (one workgroup): out[i] = sum of in[0 .. i), out[n] = the total.
__global__ __launch_bounds__(kShThreads) void k_shard_scan(const uint32_t* __restrict__ in, uint32_t n,
                                                           unsigned long long* __restrict__ out) {
    __shared__ unsigned long long ws[kShThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t per = (n + kShThreads - 1u) / kShThreads, a = min(n, tid * per), e = min(n, a + per);
    unsigned long long s = 0ull;
    for (uint32_t i = a; i < e; ++i) s += in[i];
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
        out[i] = p;
        p += in[i];
    }
    if (tid == kShThreads - 1u) out[n] = p;
}

// Fallback, sizes: entries of every listed sub-range (big[1 .. nbig]).
__global__ __launch_bounds__(256) void k_shard_big_sizes(const uint32_t* __restrict__ st, int R, uint32_t S,
                                                         const uint32_t* __restrict__ bigs, uint32_t nbig,
                                                         uint32_t* __restrict__ sizes) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= nbig) return;
    const uint32_t s = bigs[j];
    uint32_t t = 0u;
    for (int r = 0; r < R; ++r) t += st[(uint64_t)r * (S + 1u) + s + 1u] - st[(uint64_t)r * (S + 1u) + s];
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
        const uint32_t a = st[(uint64_t)r * (S + 1u) + s], b = st[(uint64_t)r * (S + 1u) + s + 1u];
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
                                                         const uint32_t* __restrict__ nruns, uint64_t lo, int SH,
                                                         uint32_t* __restrict__ ucount) {
    const uint32_t n = *nruns;
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < n; r += gridDim.x * 256u)
        atomicAdd(&ucount[sub_of(keys[starts[r]], lo, SH)], 1u);
}

// Fallback, write: run r's column = colbase[its sub-range] + (r - the sub-range's first run);
// every entry of the run gets it.
__global__ __launch_bounds__(256) void k_shard_big_write(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, uint64_t m,
                                                         const uint32_t* __restrict__ starts,
                                                         const uint32_t* __restrict__ nruns, uint64_t lo, int SH,
                                                         const unsigned long long* __restrict__ colbase,
                                                         const uint64_t* __restrict__ gpos,
                                                         uint64_t* __restrict__ columns, int64_t* __restrict__ indices) {
    const uint32_t n = *nruns;
    for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < n; r += gridDim.x * 256u) {
        const uint64_t c = keys[starts[r]];
        const uint64_t s = sub_of(c, lo, SH);
        uint32_t a = 0u, b = r;   // the first run of sub-range s
        while (a < b) {
            const uint32_t mid = (a + b) / 2u;
            if (sub_of(keys[starts[mid]], lo, SH) < s) a = mid + 1u;
            else b = mid;
        }
        const unsigned long long col = colbase[s] + (r - a);
        columns[col] = c;
        const uint64_t e = r + 1u < n ? starts[r + 1u] : m;
        for (uint64_t t = starts[r]; t < e; ++t) indices[gpos[vals[t]]] = (int64_t)col;
    }
}

// Padding out of sorted rows (kmh_count_sparse_sorted_dev's rows hold count-0 padding for the
// k-mers that occur more than once): 4096 entries per block, kept entries in order.
constexpr int kCmpBlock = 4096;
constexpr int kCmpPer = kCmpBlock / 256;

__global__ __launch_bounds__(256) void k_cmp_count(const uint32_t* __restrict__ counts, uint64_t n,
                                                   uint32_t* __restrict__ bc) {
    const uint64_t base = (uint64_t)blockIdx.x * kCmpBlock;
    uint32_t c = 0u;
#pragma unroll
    for (int i = 0; i < kCmpPer; ++i) {
        const uint64_t p = base + (uint64_t)i * 256u + threadIdx.x;
        c += (uint32_t)(p < n && counts[p] != 0u);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    __shared__ uint32_t ws[4];
    if ((threadIdx.x & 63u) == 0u) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Entry p = base + 256 i + t (lane-consecutive, coalesced) goes to boff[block] + (kept entries
// before it in position order: rows i, then waves, then lanes).
__global__ __launch_bounds__(256) void k_cmp_scatter(const uint64_t* __restrict__ codes,
                                                     const uint32_t* __restrict__ counts, uint64_t n,
                                                     const uint32_t* __restrict__ boff, uint64_t* __restrict__ oc,
                                                     uint32_t* __restrict__ on) {
    __shared__ uint32_t cw[kCmpPer * 4], pw[kCmpPer * 4];
    const uint64_t base = (uint64_t)blockIdx.x * kCmpBlock;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t cv[kCmpPer];
    uint64_t mk[kCmpPer];
#pragma unroll
    for (int i = 0; i < kCmpPer; ++i) {
        const uint64_t p = base + (uint64_t)i * 256u + threadIdx.x;
        cv[i] = p < n ? counts[p] : 0u;
        mk[i] = __ballot(cv[i] != 0u);
        if (lane == 0u) cw[i * 4 + wave] = (uint32_t)__popcll(mk[i]);
    }
    __syncthreads();
    if (threadIdx.x < 64u) {   // exclusive scan of the 64 (row, wave) counts in position order
        const uint32_t v = cw[threadIdx.x];
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if ((int)lane >= d) x += y;
        }
        pw[threadIdx.x] = x - v;
    }
    __syncthreads();
    const uint32_t b0 = boff[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kCmpPer; ++i) {
        if (cv[i] != 0u) {
            const uint64_t p = base + (uint64_t)i * 256u + threadIdx.x;
            const uint64_t o = (uint64_t)b0 + pw[i * 4 + wave] +
                               __builtin_amdgcn_mbcnt_hi((uint32_t)(mk[i] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk[i], 0u));
            oc[o] = codes[p];
            on[o] = cv[i];
        }
    }
}

}  // namespace

int rows_compact(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* src_off,
                 const uint64_t* src_len, int R, uint64_t* d_out_codes, uint32_t* d_out_counts,
                 const uint64_t* dst_off, hipStream_t s) {
    if (R < 0 || (R && (!src_off || !src_len || !dst_off))) return fail(ctx, KMH_ERR_INVALID, "bad row arguments");
    uint64_t maxb = 1;
    for (int r = 0; r < R; ++r) {
        if (src_len[r] >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "rows below 2^32 - 1 entries");
        maxb = std::max<uint64_t>(maxb, (src_len[r] + kCmpBlock - 1) / kCmpBlock);
    }
    const size_t bb = ((size_t)maxb * 4 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->out2, 2 * bb);
    if (rc) return rc;
    uint32_t* bc = static_cast<uint32_t*>(ctx->out2.ptr);
    uint32_t* boff = reinterpret_cast<uint32_t*>(static_cast<char*>(ctx->out2.ptr) + bb);
    for (int r = 0; r < R; ++r) {
        const uint64_t n = src_len[r];
        if (!n) continue;
        if (!d_codes || !d_counts || !d_out_codes || !d_out_counts) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
        const unsigned nb = (unsigned)((n + kCmpBlock - 1) / kCmpBlock);
        hipLaunchKernelGGL(k_cmp_count, dim3(nb), dim3(256), 0, s, d_counts + src_off[r], n, bc);
        KMH_HIP(ctx, hipGetLastError());
        if ((rc = scan_exclusive_u32(ctx, bc, boff, nb, nullptr, s))) return rc;
        hipLaunchKernelGGL(k_cmp_scatter, dim3(nb), dim3(256), 0, s, d_codes + src_off[r], d_counts + src_off[r], n, boff,
                           d_out_codes + dst_off[r], d_out_counts + dst_off[r]);
        KMH_HIP(ctx, hipGetLastError());
    }
    return KMH_OK;
}

int shard_union(Ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, uint64_t lo,
                uint64_t hi_incl, uint64_t* d_columns, int64_t* d_indices, uint64_t* ncols, hipStream_t s) {
    if (R < 1 || R > kShMaxRows) return fail(ctx, KMH_ERR_UNSUPPORTED, "a shard holds 1 to 4096 organism rows");
    if (!d_codes || !row_off || !ncols || hi_incl < lo) return fail(ctx, KMH_ERR_INVALID, "bad shard arguments");
    const uint64_t T = row_off[R] - row_off[0];
    for (int r = 0; r < R; ++r)
        if (row_off[r + 1] < row_off[r] || row_off[r + 1] - row_off[r] >= 0xFFFFFFFFull)
            return fail(ctx, KMH_ERR_INVALID, "row offsets must ascend, rows below 2^32 - 1 entries");
    *ncols = 0;
    if (T == 0) return KMH_OK;
    if (!d_columns || !d_indices) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    // sub-ranges of 2^SH codes: ~kShTarget entries each, at most 2^24 of them
    const unsigned __int128 span = (unsigned __int128)(hi_incl - lo) + 1u;
    uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(T / kShTarget, 1ull << 24));
    int SH = 0;
    while (SH < 64 && (span >> SH) > (unsigned __int128)want) ++SH;
    const uint32_t S = (uint32_t)((span + ((unsigned __int128)1 << SH) - 1) >> SH);

    const size_t stb = (((size_t)R * (S + 1) * 4) + 255) & ~(size_t)255;
    const size_t rb = (((size_t)R + 1) * 8 + 255) & ~(size_t)255;
    const size_t ub = (((size_t)S + 1) * 4 + 255) & ~(size_t)255;
    const size_t cb = (((size_t)S + 1) * 8 + 255) & ~(size_t)255;
    // + the fallback's list of sub-ranges, their sizes and gather offsets
    int rc = ensure(ctx, ctx->sparse[0], stb + rb + 4 * ub + 2 * cb + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint32_t* d_st = reinterpret_cast<uint32_t*>(p);
    uint64_t* d_roff = reinterpret_cast<uint64_t*>(p + stb);
    uint32_t* d_ucount = reinterpret_cast<uint32_t*>(p + stb + rb);
    uint32_t* d_big = reinterpret_cast<uint32_t*>(p + stb + rb + ub);   // [0] = count, then sub-ranges
    unsigned long long* d_colbase = reinterpret_cast<unsigned long long*>(p + stb + rb + 2 * ub);
    uint32_t* d_bigs = reinterpret_cast<uint32_t*>(p + stb + rb + 2 * ub + cb);
    uint32_t* d_sizes = reinterpret_cast<uint32_t*>(p + stb + rb + 3 * ub + cb);
    unsigned long long* d_goff = reinterpret_cast<unsigned long long*>(p + stb + rb + 4 * ub + cb);
    std::vector<uint64_t> rel(R + 1);
    for (int r = 0; r <= R; ++r) rel[r] = row_off[r] - row_off[0];
    const uint64_t* codes = d_codes + row_off[0];
    KMH_HIP(ctx, hipMemcpyAsync(d_roff, rel.data(), (R + 1) * 8, hipMemcpyHostToDevice, s));
    KMH_HIP(ctx, hipMemsetAsync(d_big, 0, 4, s));
    uint64_t maxlen = 0;
    for (int r = 0; r < R; ++r) maxlen = std::max(maxlen, rel[r + 1] - rel[r]);
    const unsigned gx = (unsigned)std::min<uint64_t>(std::max<uint64_t>((maxlen + 2047) / 2048, 1), 65535);
    time_begin(ctx, s, "k_shard_starts");
    hipLaunchKernelGGL(k_shard_starts, dim3(gx, (unsigned)R), dim3(256), 0, s, codes, d_roff, lo, SH, S, d_st);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    const unsigned ug = (unsigned)std::min<uint64_t>(S, (uint64_t)std::max(1, ctx->num_cu) * 2);
    time_begin(ctx, s, "k_shard_union");
    hipLaunchKernelGGL(k_shard_union<false>, dim3(ug), dim3(kShThreads), 0, s, codes, d_roff, R, d_st, S, lo, SH,
                       d_ucount, d_big, nullptr, nullptr, nullptr);
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
            return fail(ctx, KMH_ERR_UNSUPPORTED, "shard: 2^32 or more entries in sub-ranges the LDS cannot hold");
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
        hipLaunchKernelGGL(k_shard_big_count, dim3(1024), dim3(256), 0, s, gcode, starts, nruns, lo, SH, d_ucount);
        KMH_HIP(ctx, hipGetLastError());
    }
    hipLaunchKernelGGL(k_shard_scan, dim3(1), dim3(kShThreads), 0, s, d_ucount, S, d_colbase);
    KMH_HIP(ctx, hipGetLastError());
    unsigned long long total = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&total, d_colbase + S, 8, hipMemcpyDeviceToHost, s));
    time_begin(ctx, s, "k_shard_union");
    hipLaunchKernelGGL(k_shard_union<true>, dim3(ug), dim3(kShThreads), 0, s, codes, d_roff, R, d_st, S, lo, SH,
                       d_ucount, d_big, d_colbase, d_columns, d_indices + row_off[0]);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    if (nbig) {
        hipLaunchKernelGGL(k_shard_big_write, dim3(1024), dim3(256), 0, s, gcode, gval, m, starts, nruns, lo, SH,
                           d_colbase, gpos, d_columns, d_indices + row_off[0]);
        KMH_HIP(ctx, hipGetLastError());
    }
    KMH_HIP(ctx, hipStreamSynchronize(s));
    *ncols = total;
    return KMH_OK;
}

}  // namespace kmh
