// kmh_sparse.hip -- sorted sparse k-mer counting for 13 <= k <= 32 on MI355X.
//
// Replaces generate.py:49-58 for k where a dense 4^k table is impractical (the
// reference's dict is a hash table, generate.py:36,58).  Every valid window emits its
// 2k-bit code and start position; the pairs are compacted, radix-sorted by code (stable,
// so equal codes keep ascending positions), and run-length encoded: each run gives one
// distinct k-mer, its count and its first position.  canonical != 0 emits
// min(forward, reverse complement) (BASELINE config 5; not a reference feature).
#include <hipcub/hipcub.hpp>

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

// One thread per window start.  The k <= 32 bytes of a window are read byte-wise; the
// vector L1 serves the 32x overlap between neighbouring threads.
__global__ __launch_bounds__(256) void k_window_codes(const uint8_t* __restrict__ seq,
                                                      uint64_t nwin, int k, int canonical,
                                                      uint64_t* __restrict__ codes,
                                                      uint8_t* __restrict__ flags) {
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
    flags[i] = ok ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_run_first(const uint32_t* __restrict__ pos_sorted,
                                                   const uint32_t* __restrict__ run_start,
                                                   const uint64_t* __restrict__ nruns,
                                                   uint64_t* __restrict__ first) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < *nruns) first[r] = pos_sorted[run_start[r]];
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
                                                 uint8_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < bins) flags[i] = counts[i] ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_gather_first(const uint32_t* __restrict__ codes,
                                                      const uint32_t* __restrict__ first,
                                                      const uint64_t* __restrict__ n,
                                                      uint32_t* __restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < *n) keys[i] = first[codes[i]];
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
                                                      uint8_t* __restrict__ flags) {
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
    flags[i] = ok ? 1 : 0;
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
                                                   uint8_t* __restrict__ head) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    bool h = i == 0;
    if (!h) {
        const uint32_t a = perm[i], b = perm[i - 1];
        for (int w = 0; w < W && !h; ++w) h = words[(uint64_t)w * stride + a] != words[(uint64_t)w * stride + b];
    }
    head[i] = h ? 1 : 0;
}

// Run r: count, first window start (the smallest: the sorts are stable and start from
// ascending positions), and the code of its first 32 bases.
__global__ __launch_bounds__(256) void k_long_runs(const uint32_t* __restrict__ run_start,
                                                   const uint64_t* __restrict__ nruns, uint64_t m,
                                                   const uint32_t* __restrict__ perm,
                                                   const uint64_t* __restrict__ word0,
                                                   uint32_t* __restrict__ counts, uint64_t* __restrict__ first,
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

__global__ __launch_bounds__(256) void k_gather_long(const uint32_t* __restrict__ idx,
                                                     const uint64_t* __restrict__ prefix,
                                                     const uint32_t* __restrict__ counts, uint64_t n,
                                                     uint64_t* __restrict__ prefix_out,
                                                     uint32_t* __restrict__ counts_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        prefix_out[i] = prefix[idx[i]];
        counts_out[i] = counts[idx[i]];
    }
}

void* carve(char*& p, size_t bytes) {
    void* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return r;
}

}  // namespace

// generate.py:36,58 keeps k-mers in first-occurrence order (the dict's insertion order, which
// fixes the line order of k{k}.txt, :89-91).  Each k-mer's first start is unique, so sorting
// the nonzero bins by it gives that order: compact, radix sort by start, gather the counts.
int dense_order(Ctx* ctx, const uint32_t* d_counts, const uint32_t* d_first, size_t bins,
                uint64_t n, std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                std::vector<uint64_t>& first, hipStream_t s) {
    codes.clear();
    counts.clear();
    first.clear();
    const int N = (int)bins;
    int bits = 1;
    while (bits < 32 && (1ull << bits) < n) ++bits;   // first starts are < n
    size_t t_sel = 0, t_sort = 0;
    uint32_t* nul = nullptr;
    uint8_t* nulf = nullptr;
    uint64_t* nuln = nullptr;
    hipcub::CountingInputIterator<uint32_t> iota(0u);
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(nullptr, t_sel, iota, nulf, nul, nuln, N, s));
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, nul, nul, nul, nul, N, 0, bits, s));
    const size_t temp = std::max(t_sel, t_sort);
    const size_t a4 = ((bins * 4) + 255) & ~(size_t)255;
    int rc = ensure(ctx, ctx->order, 5 * a4 + (((bins) + 255) & ~(size_t)255) + temp + 1024);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->order.ptr);
    uint32_t* sel = static_cast<uint32_t*>(carve(p, bins * 4));
    uint32_t* keys = static_cast<uint32_t*>(carve(p, bins * 4));
    uint32_t* keys2 = static_cast<uint32_t*>(carve(p, bins * 4));
    uint32_t* vals2 = static_cast<uint32_t*>(carve(p, bins * 4));
    uint32_t* cnt2 = static_cast<uint32_t*>(carve(p, bins * 4));
    uint8_t* flags = static_cast<uint8_t*>(carve(p, bins));
    uint64_t* nsel = static_cast<uint64_t*>(carve(p, 64));
    void* tmp = carve(p, temp);
    const unsigned g = (unsigned)((bins + 255) / 256);
    hipLaunchKernelGGL(k_nonzero, dim3(g), dim3(256), 0, s, d_counts, (uint64_t)bins, flags);
    KMH_HIP(ctx, hipGetLastError());
    size_t t = temp;
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(tmp, t, iota, flags, sel, nsel, N, s));
    hipLaunchKernelGGL(k_gather_first, dim3(g), dim3(256), 0, s, sel, d_first, nsel, keys);
    KMH_HIP(ctx, hipGetLastError());
    uint64_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, nsel, 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t, keys, keys2, sel, vals2, (int)m, 0, bits, s));
    hipLaunchKernelGGL(k_gather_counts, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, vals2, d_counts, m, cnt2);
    KMH_HIP(ctx, hipGetLastError());
    // The u32 codes and first starts land in the upper half of their u64 arrays and are
    // widened in place, front to back (element i's 8 bytes end at or before the 4-byte
    // source of element i + 1), so no u32 staging arrays are allocated.
    codes.resize(m);
    first.resize(m);
    counts.resize(m);
    uint32_t* c32 = reinterpret_cast<uint32_t*>(codes.data()) + m;
    uint32_t* f32 = reinterpret_cast<uint32_t*>(first.data()) + m;
    KMH_HIP(ctx, hipMemcpyAsync(c32, vals2, m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(f32, keys2, m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(counts.data(), cnt2, m * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    for (uint64_t i = 0; i < m; ++i) {
        const uint32_t c = c32[i], f = f32[i];
        codes[i] = c;
        first[i] = f;
    }
    return KMH_OK;
}

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
    const int N = (int)nwin;  // hipcub item counts are int here; n < 2^31 enforced below
    if (nwin > 0x7FFFFFFFull) return fail(ctx, KMH_ERR_UNSUPPORTED, "sparse path supports < 2^31 windows per call");

    // Scratch sizes of the hipcub passes.
    size_t t_sel = 0, t_sort = 0, t_rle = 0, t_scan = 0;
    uint64_t *kin = nullptr, *kout = nullptr, *nsel = nullptr;
    uint32_t *vin = nullptr, *vout = nullptr;
    uint8_t* flags = nullptr;
    hipcub::CountingInputIterator<uint32_t> iota(0u);
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(nullptr, t_sel, kin, flags, kout, nsel, N, s));
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, kin, kout, vin, vout, N, 0, 2 * k, s));
    KMH_HIP(ctx, hipcub::DeviceRunLengthEncode::Encode(nullptr, t_rle, kin, kout, vin, nsel, N, s));
    KMH_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, vin, vout, N, s));
    const size_t temp = std::max(std::max(t_sel, t_sort), std::max(t_rle, t_scan));

    const size_t bytes = 4 * (((size_t)nwin * 8 + 255) & ~(size_t)255) +
                         3 * (((size_t)nwin * 4 + 255) & ~(size_t)255) +
                         (((size_t)nwin + 255) & ~(size_t)255) + temp + 4096;
    int rc = ensure(ctx, ctx->sparse[0], bytes);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint64_t* codes_all = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* keys_a = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* keys_b = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* first_d = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint32_t* pos_a = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* pos_b = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* cnt_d = static_cast<uint32_t*>(carve(p, nwin * 4));
    flags = static_cast<uint8_t*>(carve(p, nwin));
    uint64_t* small = static_cast<uint64_t*>(carve(p, 64));
    void* tmp = carve(p, temp);
    uint64_t* nvalid_d = small;
    uint64_t* nruns_d = small + 1;

    time_begin(ctx, s, "k_window_codes");
    hipLaunchKernelGGL(k_window_codes, dim3((unsigned)((nwin + 255) / 256)), dim3(256), 0, s,
                       d_seq, nwin, k, canonical, codes_all, flags);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    size_t t = temp;
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(tmp, t, codes_all, flags, keys_a, nvalid_d, N, s));
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(tmp, t, iota, flags, pos_a, nvalid_d, N, s));
    uint64_t nvalid = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&nvalid, nvalid_d, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (nvalid == 0) return KMH_OK;
    const int M = (int)nvalid;
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t, keys_a, keys_b, pos_a, pos_b, M, 0, 2 * k, s));
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceRunLengthEncode::Encode(tmp, t, keys_b, keys_a, cnt_d, nruns_d, M, s));
    uint64_t nruns = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&nruns, nruns_d, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, t, cnt_d, pos_a, (int)nruns, s));
    hipLaunchKernelGGL(k_run_first, dim3((unsigned)((nruns + 255) / 256)), dim3(256), 0, s,
                       pos_b, pos_a, nruns_d, first_d);
    KMH_HIP(ctx, hipGetLastError());
    // First-occurrence order (the reference dict's order, generate.py:36,58): sort the runs
    // by their first start on the device, then gather codes and counts.
    int bits = 1;
    while (bits < 64 && (1ull << bits) < n) ++bits;
    const unsigned gr = (unsigned)((nruns + 255) / 256);
    hipLaunchKernelGGL(k_iota, dim3(gr), dim3(256), 0, s, pos_a, nruns);
    KMH_HIP(ctx, hipGetLastError());
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t, first_d, keys_b, pos_a, pos_b, (int)nruns, 0, bits, s));
    hipLaunchKernelGGL(k_gather_runs, dim3(gr), dim3(256), 0, s, pos_b, keys_a, cnt_d, nruns, codes_all, pos_a);
    KMH_HIP(ctx, hipGetLastError());
    codes.resize(nruns);
    counts.resize(nruns);
    first.resize(nruns);
    KMH_HIP(ctx, hipMemcpyAsync(codes.data(), codes_all, nruns * 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(counts.data(), pos_a, nruns * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(first.data(), keys_b, nruns * 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    return KMH_OK;
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
    if (nwin > 0x7FFFFFFFull) return fail(ctx, KMH_ERR_UNSUPPORTED, "sparse path supports < 2^31 windows per call");
    const int N = (int)nwin, W = (k + 31) / 32;

    size_t t_sel = 0, t_sort = 0;
    uint64_t *k64 = nullptr, *nsel = nullptr;
    uint32_t* v32 = nullptr;
    uint8_t* fl = nullptr;
    hipcub::CountingInputIterator<uint32_t> iota(0u);
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(nullptr, t_sel, iota, fl, v32, nsel, N, s));
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, k64, k64, v32, v32, N, 0, 64, s));
    const size_t temp = std::max(t_sel, t_sort);
    auto rup = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bytes = (size_t)W * rup(nwin * 8) + 5 * rup(nwin * 8) + 4 * rup(nwin * 4) + rup(nwin) +
                         temp + 4096;
    int rc = ensure(ctx, ctx->sparse[0], bytes);
    if (rc) return rc;
    char* p = static_cast<char*>(ctx->sparse[0].ptr);
    uint64_t* words = static_cast<uint64_t*>(carve(p, (size_t)W * rup(nwin * 8)));
    const uint64_t wstride = rup(nwin * 8) / 8;   // words of one code word row
    uint64_t* keys_a = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* keys_b = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* first_d = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* prefix_d = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint64_t* prefix_o = static_cast<uint64_t*>(carve(p, nwin * 8));
    uint32_t* perm_a = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* perm_b = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* runs = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint32_t* cnt_d = static_cast<uint32_t*>(carve(p, nwin * 4));
    uint8_t* flags = static_cast<uint8_t*>(carve(p, nwin));
    uint64_t* small = static_cast<uint64_t*>(carve(p, 64));
    void* tmp = carve(p, temp);
    const unsigned gw = (unsigned)((nwin + 255) / 256);

    time_begin(ctx, s, "k_window_words");
    hipLaunchKernelGGL(k_window_words, dim3(gw), dim3(256), 0, s, d_seq, nwin, wstride, k, W, words, flags);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    size_t t = temp;
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(tmp, t, iota, flags, perm_a, small, N, s));
    uint64_t m = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&m, small, 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    if (m == 0) return KMH_OK;
    const int M = (int)m;
    const unsigned gm = (unsigned)((m + 255) / 256);
    for (int w = W - 1; w >= 0; --w) {   // least significant word first; stable sorts
        hipLaunchKernelGGL(k_gather_word, dim3(gm), dim3(256), 0, s, words + (uint64_t)w * wstride, perm_a, m, keys_a);
        KMH_HIP(ctx, hipGetLastError());
        t = temp;
        KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t, keys_a, keys_b, perm_a, perm_b, M, 0, 64, s));
        std::swap(perm_a, perm_b);
    }
    hipLaunchKernelGGL(k_run_heads, dim3(gm), dim3(256), 0, s, words, wstride, W, perm_a, m, flags);
    KMH_HIP(ctx, hipGetLastError());
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceSelect::Flagged(tmp, t, iota, flags, runs, small + 1, M, s));
    hipLaunchKernelGGL(k_long_runs, dim3(gm), dim3(256), 0, s, runs, small + 1, m, perm_a, words, cnt_d,
                       first_d, prefix_d);
    KMH_HIP(ctx, hipGetLastError());
    uint64_t nruns = 0;
    KMH_HIP(ctx, hipMemcpyAsync(&nruns, small + 1, 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    // first-occurrence order: sort the runs by first start, gather prefix codes and counts
    int bits = 1;
    while (bits < 64 && (1ull << bits) < n) ++bits;
    const unsigned gr = (unsigned)((nruns + 255) / 256);
    hipLaunchKernelGGL(k_iota, dim3(gr), dim3(256), 0, s, perm_b, nruns);
    KMH_HIP(ctx, hipGetLastError());
    t = temp;
    KMH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t, first_d, keys_b, perm_b, runs, (int)nruns, 0, bits, s));
    hipLaunchKernelGGL(k_gather_long, dim3(gr), dim3(256), 0, s, runs, prefix_d, cnt_d, nruns, prefix_o, perm_b);
    KMH_HIP(ctx, hipGetLastError());
    codes.resize(nruns);
    counts.resize(nruns);
    first.resize(nruns);
    KMH_HIP(ctx, hipMemcpyAsync(codes.data(), prefix_o, nruns * 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(counts.data(), perm_b, nruns * 4, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipMemcpyAsync(first.data(), keys_b, nruns * 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    return KMH_OK;
}

}  // namespace kmh

