// kmh_sparse.hip -- the drop-in's sparse counting paths (one organism per call, k > 12 or
// canonical) and the first-occurrence order of every result.
//
// Replaces generate.py:49-58 for k where a dense 4^k table is impractical (the reference's dict
// is a hash table, generate.py:36,58).  Its k{k}.txt lines follow the dict's insertion order =
// first occurrence (:89-91), so every path here also yields each distinct k-mer's first window
// start and returns the k-mers sorted by it.  All kernels are hand-written (kmh_sort.hip's
// radix sort, scan and selection; kmh_hash.hip's hash pipeline): item counts are 64-bit and
// positions 32-bit, so any organism below 2^32 - 1 bytes is counted, 2^31 windows and more
// included (a 3.1 Gbp human genome at k = 21).
//
//   13 <= k <= 32         sparse_count_first: the device hash-table pipeline of kmh_hash.hip
//                         with every entry's window position carried along (the count kernel
//                         keeps the minimum per distinct k-mer), then a radix sort by first start.
//   canonical, k <= 12    sparse_count: every valid window's (code, start) selected in start
//                         order, stably radix-sorted by code, runs (count, first = the run's
//                         first start), sorted by first start.
//   33 <= k <= 1024       sparse_count_long: the same over ceil(k / 32) code words (LSD over
//                         the words), forward strand.
//   k <= 12 (dense)       dense_order: the nonzero bins of the dense count row sorted by the
//                         first-start table of k_first.
#include <algorithm>

#include "kmh_internal.h"

namespace kmh {
namespace {

__device__ __forceinline__ int base_code(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

inline unsigned grid256(uint64_t n) {
    return (unsigned)((n + 255) / 256);
}

void* carve(char*& p, size_t bytes) {
    void* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return r;
}

// Bits of a first-start key: starts are < n.
int start_bits(uint64_t n) {
    int bits = 1;
    while (bits < 32 && (1ull << bits) < n) ++bits;
    return bits;
}

// One thread per window start.  The k <= 32 bytes of a window are read byte-wise; the
// vector L1 serves the 32x overlap between neighbouring threads.
__global__ __launch_bounds__(256) void k_window_codes(const uint8_t* __restrict__ seq,
                                                      uint64_t nwin, int k, int canonical,
                                                      uint64_t* __restrict__ codes,
                                                      uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nwin) return;
    uint64_t fwd = 0, rc = 0;
    bool ok = true;
    for (int j = 0; j < k; ++j) {
        const int b = base_code(seq[i + j]);
        ok &= b >= 0;
        const uint64_t bb = (uint64_t)(b & 3);
        fwd = (fwd << 2) | bb;
        rc |= (3ull - bb) << (2 * j);
    }
    codes[i] = (canonical && rc < fwd) ? rc : fwd;
    flags[i] = ok ? 1u : 0u;
}

// Selected windows: (code, start) in start order.
__global__ __launch_bounds__(256) void k_pick_windows(const uint64_t* __restrict__ codes,
                                                      const uint32_t* __restrict__ idx, uint32_t m,
                                                      uint64_t* __restrict__ keys, uint32_t* __restrict__ pos) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < m) {
        const uint32_t w = idx[i];
        keys[i] = codes[w];
        pos[i] = w;
    }
}

// Run r of sorted (key, start) pairs: code, count, first start (the run's first element).
__global__ __launch_bounds__(256) void k_runs_emit(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ pos,
                                                   uint32_t m, const uint32_t* __restrict__ starts,
                                                   const uint32_t* __restrict__ nruns, uint64_t* __restrict__ codes,
                                                   uint32_t* __restrict__ counts, uint32_t* __restrict__ first) {
    const uint32_t r = blockIdx.x * 256u + threadIdx.x, n = *nruns;
    if (r < n) {
        const uint32_t a = starts[r], e = r + 1 < n ? starts[r + 1] : m;
        codes[r] = keys[a];
        counts[r] = e - a;
        first[r] = pos[a];
    }
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* __restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_gather_runs(const uint32_t* __restrict__ idx,
                                                     const uint64_t* __restrict__ codes,
                                                     const uint32_t* __restrict__ counts, uint64_t n,
                                                     uint64_t* __restrict__ codes_out,
                                                     uint32_t* __restrict__ counts_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        codes_out[i] = codes[idx[i]];
        counts_out[i] = counts[idx[i]];
    }
}

__global__ __launch_bounds__(256) void k_nonzero(const uint32_t* __restrict__ counts, uint64_t bins,
                                                 uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < bins) flags[i] = counts[i] ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_gather_first(const uint32_t* __restrict__ codes,
                                                      const uint32_t* __restrict__ first, uint32_t m,
                                                      uint32_t* __restrict__ keys) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < m) keys[i] = first[codes[i]];
}

__global__ __launch_bounds__(256) void k_gather_counts(const uint32_t* __restrict__ codes,
                                                       const uint32_t* __restrict__ counts,
                                                       uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = counts[codes[i]];
}

// ---- long k-mers (33 <= k <= KMH_MAX_LONG_K), forward strand ----
// Word w of window i holds bases [32 w, 32 w + 32) of the window, 2 bits each, first base
// most significant, the last word left-aligned: comparing the words in order compares the
// k-mer strings.  words is word-major (words[w * stride + i], stride >= nwin).
__global__ __launch_bounds__(256) void k_window_words(const uint8_t* __restrict__ seq, uint64_t nwin,
                                                      uint64_t stride, int k, int W,
                                                      uint64_t* __restrict__ words,
                                                      uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nwin) return;
    bool ok = true;
    for (int w = 0; w < W; ++w) {
        const int b0 = 32 * w, len = min(32, k - b0);
        uint64_t v = 0;
        for (int j = 0; j < len; ++j) {
            const int b = base_code(seq[i + b0 + j]);
            ok &= b >= 0;
            v = (v << 2) | (uint64_t)(b & 3);
        }
        if (len < 32) v <<= 2 * (32 - len);
        words[(uint64_t)w * stride + i] = v;
    }
    flags[i] = ok ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_gather_word(const uint64_t* __restrict__ word,
                                                     const uint32_t* __restrict__ perm, uint64_t m,
                                                     uint64_t* __restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) keys[i] = word[perm[i]];
}

// 1 where sorted window i starts a run (its k-mer differs from window i - 1's).
__global__ __launch_bounds__(256) void k_run_heads(const uint64_t* __restrict__ words, uint64_t stride,
                                                   int W, const uint32_t* __restrict__ perm, uint64_t m,
                                                   uint32_t* __restrict__ head) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    bool h = i == 0;
    if (!h) {
        const uint32_t a = perm[i], b = perm[i - 1];
        for (int w = 0; w < W && !h; ++w) h = words[(uint64_t)w * stride + a] != words[(uint64_t)w * stride + b];
    }
    head[i] = h ? 1u : 0u;
}

// Run r: count, first window start (the smallest: the sorts are stable and start from
// ascending positions), and the code of its first 32 bases.
__global__ __launch_bounds__(256) void k_long_runs(const uint32_t* __restrict__ run_start,
                                                   const uint32_t* __restrict__ nruns, uint64_t m,
                                                   const uint32_t* __restrict__ perm,
                                                   const uint64_t* __restrict__ word0,
                                                   uint32_t* __restrict__ counts, uint32_t* __restrict__ first,
                                                   uint64_t* __restrict__ prefix) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nr = *nruns;
    if (r >= nr) return;
    const uint32_t s0 = run_start[r];
    const uint64_t e = r + 1 < nr ? run_start[r + 1] : m;
    counts[r] = (uint32_t)(e - s0);
    first[r] = perm[s0];
    prefix[r] = word0[perm[s0]];
}

// (u64 code, u32 count, u32 first start) results -> first-occurrence order on the host:
// radix sort of the first starts (unique) with the result index, gather, copy out.
int order_by_first(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, uint32_t* d_first, uint64_t m,
                   uint64_t n, std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                   std::vector<uint64_t>& first, hipStream_t s) {
    if (m == 0) return KMH_OK;
    const size_t a4 = ((size_t)m * 4 + 255) & ~(size_t)255, a8 = ((size_t)m * 8 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->order, 4 * a4 + a8 + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->order.ptr);
    uint32_t* f_alt = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* idx = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* idx_alt = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* cnt_o = static_cast<uint32_t*>(carve(p, a4));
    uint64_t* codes_o = static_cast<uint64_t*>(carve(p, a8));
    hipLaunchKernelGGL(k_iota, dim3(grid256(m)), dim3(256), 0, s, idx, m);
    KMH_HIP(ctx, hipGetLastError());
    bool alt = false;
    rc = radix_sort_pairs<uint32_t>(ctx, d_first, f_alt, idx, idx_alt, m, 0, start_bits(n), &alt, s);
    if (rc) return rc;
    const uint32_t* fs = alt ? f_alt : d_first;
    const uint32_t* perm = alt ? idx_alt : idx;
    hipLaunchKernelGGL(k_gather_runs, dim3(grid256(m)), dim3(256), 0, s, perm, d_codes, d_counts, m, codes_o, cnt_o);
    KMH_HIP(ctx, hipGetLastError());
    codes.resize(m);
    counts.resize(m);
    first.resize(m);
    // the u32 starts land in the upper half of the u64 array and are widened in place, front to
    // back (element i's 8 bytes end at or before the 4-byte source of element i + 1)
    uint32_t* f32 = reinterpret_cast<uint32_t*>(first.data()) + m;
    KMH_HIP(ctx, hipMemcpyAsync(codes.data(), codes_o, m * 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(counts.data(), cnt_o, m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(f32, fs, m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    for (uint64_t i = 0; i < m; ++i) first[i] = f32[i];
    return KMH_OK;
}

}  // namespace

// generate.py:36,58 keeps k-mers in first-occurrence order (the dict's insertion order, which
// fixes the line order of k{k}.txt, :89-91).  Each k-mer's first start is unique, so sorting
// the nonzero bins by it gives that order: select, radix sort by start, gather the counts.
int dense_order(Ctx* ctx, const uint32_t* d_counts, const uint32_t* d_first, size_t bins,
                uint64_t n, std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                std::vector<uint64_t>& first, hipStream_t s) {
    codes.clear();
    counts.clear();
    first.clear();
    const size_t a4 = ((bins * 4) + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->sparse[0], 7 * a4 + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint32_t* flags = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* ex = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* sel = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* sel2 = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* keys = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* keys2 = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* cnt2 = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* nsel = static_cast<uint32_t*>(carve(p, 64));
    hipLaunchKernelGGL(k_nonzero, dim3(grid256(bins)), dim3(256), 0, s, d_counts, (uint64_t)bins, flags);
    KMH_HIP(ctx, hipGetLastError());
    if ((rc = select_flagged(ctx, flags, bins, ex, sel, nsel, s))) return rc;
    uint32_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, nsel, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    hipLaunchKernelGGL(k_gather_first, dim3(grid256(m)), dim3(256), 0, s, sel, d_first, m, keys);
    KMH_HIP(ctx, hipGetLastError());
    bool alt = false;
    if ((rc = radix_sort_pairs<uint32_t>(ctx, keys, keys2, sel, sel2, m, 0, start_bits(n), &alt, s))) return rc;
    const uint32_t* ks = alt ? keys2 : keys;
    const uint32_t* vs = alt ? sel2 : sel;
    hipLaunchKernelGGL(k_gather_counts, dim3(grid256(m)), dim3(256), 0, s, vs, d_counts, (uint64_t)m, cnt2);
    KMH_HIP(ctx, hipGetLastError());
    // The u32 codes and first starts land in the upper half of their u64 arrays and are
    // widened in place, front to back (element i's 8 bytes end at or before the 4-byte
    // source of element i + 1), so no u32 staging arrays are allocated.
    codes.resize(m);
    first.resize(m);
    counts.resize(m);
    uint32_t* c32 = reinterpret_cast<uint32_t*>(codes.data()) + m;
    uint32_t* f32 = reinterpret_cast<uint32_t*>(first.data()) + m;
    KMH_HIP(ctx, hipMemcpyAsync(c32, vs, (size_t)m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(f32, ks, (size_t)m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(counts.data(), cnt2, (size_t)m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    for (uint64_t i = 0; i < m; ++i) {
        const uint32_t c = c32[i], f = f32[i];
        codes[i] = c;
        first[i] = f;
    }
    return KMH_OK;
}

// 13 <= k <= 32: the device hash-table pipeline with positions (kmh_hash.hip), then the
// first-occurrence order.
int sparse_count_first(Ctx* ctx, const uint8_t* d_seq, uint64_t n, int k, int canonical,
                       std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                       std::vector<uint64_t>& first, hipStream_t s) {
    codes.clear();
    counts.clear();
    first.clear();
    if (n >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "sequence must be shorter than 2^32 - 1 bytes");
    if (n < (uint64_t)k) return KMH_OK;
    const uint64_t nwin = n - (uint64_t)k + 1;
    const size_t a8 = ((size_t)nwin * 8 + 255) & ~(size_t)255, a4 = ((size_t)nwin * 4 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->first, a8 + 2 * a4 + 256);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->first.ptr);
    uint64_t* d_codes = static_cast<uint64_t*>(carve(p, a8));
    uint32_t* d_counts = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* d_first = static_cast<uint32_t*>(carve(p, a4));
    uint64_t* d_nk = static_cast<uint64_t*>(carve(p, 64));
    const uint64_t off[2] = {0, n};
    if ((rc = sparse_count_dev_first(ctx, d_seq, off, 1, k, canonical, d_codes, d_counts, d_first, d_nk, s)))
        return rc;
    uint64_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, d_nk, 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m > nwin) return fail(ctx, KMH_ERR_HIP, "sparse count: more distinct k-mers than windows");
    // The hash pipeline's entries, positions and pass staging (12-16 B per window) are dead:
    // free them before order_by_first allocates, when they are large (a 3 Gbp organism at
    // k >= 22 would otherwise peak near 200 GB of device memory).
    if (ctx->sparse[2].bytes + ctx->sparse[6].bytes + ctx->sparse[7].bytes > ((size_t)4 << 30))
        for (int i : {2, 6, 7})
            if ((rc = drop(ctx, ctx->sparse[i]))) return rc;
    return order_by_first(ctx, d_codes, d_counts, d_first, m, n, codes, counts, first, s);
}

// Any 1 <= k <= 32 (the drop-in uses it for canonical k <= 12): select the valid windows in
// start order, stable radix sort by code, runs, first-occurrence order.
int sparse_count(Ctx* ctx, const uint8_t* d_seq, uint64_t n, int k, int canonical,
                 std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                 std::vector<uint64_t>& first, hipStream_t s) {
    codes.clear();
    counts.clear();
    first.clear();
    if (k < 1 || k > KMH_MAX_SPARSE_K) return fail(ctx, KMH_ERR_UNSUPPORTED, "sparse counting needs 1 <= k <= 32");
    if (n >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "sequence must be shorter than 2^32 - 1 bytes");
    if (n < (uint64_t)k) return KMH_OK;
    const uint64_t nwin = n - (uint64_t)k + 1;
    const size_t a8 = ((size_t)nwin * 8 + 255) & ~(size_t)255, a4 = ((size_t)nwin * 4 + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->sparse[0], 3 * a8 + 5 * a4 + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint64_t* wcodes = static_cast<uint64_t*>(carve(p, a8));
    uint64_t* keys_a = static_cast<uint64_t*>(carve(p, a8));
    uint64_t* keys_b = static_cast<uint64_t*>(carve(p, a8));
    uint32_t* flags = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* ex = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* idx = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* pos_a = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* pos_b = static_cast<uint32_t*>(carve(p, a4));
    uint32_t* small = static_cast<uint32_t*>(carve(p, 64));

    time_begin(ctx, s, "k_window_codes");
    hipLaunchKernelGGL(k_window_codes, dim3(grid256(nwin)), dim3(256), 0, s, d_seq, nwin, k, canonical, wcodes, flags);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    if ((rc = select_flagged(ctx, flags, nwin, ex, idx, small, s))) return rc;
    uint32_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, small, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    hipLaunchKernelGGL(k_pick_windows, dim3(grid256(m)), dim3(256), 0, s, wcodes, idx, m, keys_a, pos_a);
    KMH_HIP(ctx, hipGetLastError());
    bool alt = false;
    if ((rc = radix_sort_pairs<uint64_t>(ctx, keys_a, keys_b, pos_a, pos_b, m, 0, 2 * k, &alt, s))) return rc;
    const uint64_t* ks = alt ? keys_b : keys_a;
    const uint32_t* ps = alt ? pos_b : pos_a;
    // runs -> (code, count, first) into the spare arrays: wcodes, flags (counts), idx (firsts)
    if ((rc = run_starts<uint64_t>(ctx, ks, m, flags, ex, alt ? pos_a : pos_b, small + 1, s))) return rc;
    const uint32_t* starts = alt ? pos_a : pos_b;
    hipLaunchKernelGGL(k_runs_emit, dim3(grid256(m)), dim3(256), 0, s, ks, ps, m, starts, small + 1, wcodes, flags, idx);
    KMH_HIP(ctx, hipGetLastError());
    uint32_t nruns = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&nruns, small + 1, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    return order_by_first(ctx, wcodes, flags, idx, nruns, n, codes, counts, first, s);
}

// Long k-mers: every valid window's k-mer as W = ceil(k / 32) code words; an LSD sequence of
// W stable radix sorts (least significant word first) carrying the window positions orders
// the windows by k-mer string, runs of equal words give the distinct k-mers with their
// counts and first starts, and the runs are put in first-occurrence order as in
// sparse_count (generate.py:36,58).
int sparse_count_long(Ctx* ctx, const uint8_t* d_seq, uint64_t n, int k, std::vector<uint64_t>& codes,
                      std::vector<uint32_t>& counts, std::vector<uint64_t>& first, hipStream_t s) {
    codes.clear();
    counts.clear();
    first.clear();
    if (k <= KMH_MAX_SPARSE_K || k > KMH_MAX_LONG_K)
        return fail(ctx, KMH_ERR_UNSUPPORTED, "long k-mer counting needs 33 <= k <= 1024");
    if (n >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "sequence must be shorter than 2^32 - 1 bytes");
    if (n < (uint64_t)k) return KMH_OK;
    const uint64_t nwin = n - (uint64_t)k + 1;
    const int W = (k + 31) / 32;
    auto rup = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bytes = (size_t)W * rup(nwin * 8) + 3 * rup(nwin * 8) + 6 * rup(nwin * 4) + 4096;
    int rc = ensure(ctx, ctx->sparse[0], bytes);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint64_t* words = static_cast<uint64_t*>(carve(p, (size_t)W * rup(nwin * 8)));
    const uint64_t wstride = rup(nwin * 8) / 8;   // words of one code word row
    uint64_t* keys_a = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* keys_b = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* prefix_d = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint32_t* perm_a = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* perm_b = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* runs = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* cnt_d = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* flags = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* ex = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* small = static_cast<uint32_t*>(carve(p, 64));

    time_begin(ctx, s, "k_window_words");
    hipLaunchKernelGGL(k_window_words, dim3(grid256(nwin)), dim3(256), 0, s, d_seq, nwin, wstride, k, W, words, flags);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    if ((rc = select_flagged(ctx, flags, nwin, ex, perm_a, small, s))) return rc;
    uint32_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, small, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    for (int w = W - 1; w >= 0; --w) {   // least significant word first; stable sorts
        hipLaunchKernelGGL(k_gather_word, dim3(grid256(m)), dim3(256), 0, s, words + (uint64_t)w * wstride, perm_a,
                           (uint64_t)m, keys_a);
        KMH_HIP(ctx, hipGetLastError());
        bool alt = false;
        if ((rc = radix_sort_pairs<uint64_t>(ctx, keys_a, keys_b, perm_a, perm_b, m, 0, 64, &alt, s))) return rc;
        if (alt) std::swap(perm_a, perm_b);
    }
    hipLaunchKernelGGL(k_run_heads, dim3(grid256(m)), dim3(256), 0, s, words, wstride, W, perm_a, (uint64_t)m, flags);
    KMH_HIP(ctx, hipGetLastError());
    if ((rc = select_flagged(ctx, flags, m, ex, runs, small + 1, s))) return rc;
    // counts, first starts (into perm_b) and first-32-base prefixes of the runs
    hipLaunchKernelGGL(k_long_runs, dim3(grid256(m)), dim3(256), 0, s, runs, small + 1, (uint64_t)m, perm_a, words,
                       cnt_d, perm_b, prefix_d);
    KMH_HIP(ctx, hipGetLastError());
    uint32_t nruns = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&nruns, small + 1, 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    return order_by_first(ctx, prefix_d, cnt_d, perm_b, nruns, n, codes, counts, first, s);
}

}  // namespace kmh
