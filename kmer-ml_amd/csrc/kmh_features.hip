// kmh_features.hip -- per-k-mer feature columns of the feature CSV (row f4) on the device.
//
// The reference computes, per k-mer row, base counts, GC percent, CpG count and observed /
// expected ratio, Shannon entropy and a dinucleotide-repeat flag (statistics.py:188-238), on the
// label it parsed from k{k}.txt -- for integer-parsed files the k-mer with its leading A's
// stripped (statistics.py:157, 248-273).  Every feature is a function of that label, so one
// thread per k-mer code computes them all; the float64 columns use the reference's operations
// in its order, each rounded once (fused multiply-adds are switched off), and the entropy sums
// its terms in the order Python's set() iterates the label's distinct bases: that order
// depends only on which bases appear, in first-appearance order, and the caller passes it as a
// table (computed by the interpreter itself) together with math.log2(n / L) for 1 <= n <= L <= k.
#include "kmh_device.h"

namespace kmh {
namespace {

// Plain operators under this pragma (not the __d*_rn helpers of the HIP headers, whose
// inlined multiply and subtract the default contraction may still fuse into one FMA).
#pragma clang fp contract(off)

__global__ __launch_bounds__(256) void k_features(const uint64_t* __restrict__ codes, uint64_t n, int k,
                                                  const int32_t* __restrict__ order, const double* __restrict__ lg,
                                                  int64_t* __restrict__ cnt_out, int64_t* __restrict__ cpg_out,
                                                  int64_t* __restrict__ rep_out, double* __restrict__ gc_out,
                                                  double* __restrict__ oe_out, double* __restrict__ ent_out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t c = codes ? codes[i] : i;
    auto dig = [&](int p) { return (int)((c >> (2 * (k - 1 - p))) & 3u); };
    // stripped label: positions k - m .. k - 1 (leading A's dropped, at least one base kept)
    int s = 0;
    while (s < k - 1 && dig(s) == 0) ++s;
    const int m = k - s;
    int cnt[4] = {0, 0, 0, 0}, first[4] = {1 << 20, 1 << 20, 1 << 20, 1 << 20};
    int cpg = 0, rep = 0;
    for (int p = s; p < k; ++p) {
        const int d = dig(p);
        ++cnt[d];
        if (first[d] > p) first[d] = p;
        if (p + 1 < k && d == 1 && dig(p + 1) == 2) ++cpg;                       // "CG"
        if (p + 3 < k && d == dig(p + 2) && dig(p + 1) == dig(p + 3)) rep = 1;   // kmer[i:i+2] == kmer[i+2:i+4]
    }
    const double L = (double)m;
    // statistics.py:196: (gc_count / len(kmer)) * 100
    gc_out[i] = ((double)(cnt[2] + cnt[1]) / L) * 100.0;
    // statistics.py:205-212: c_freq * g_freq * (len - 1), 0.001 when the product is 0
    const double prod = ((double)cnt[1] / L) * ((double)cnt[2] / L);
    const double expected = prod > 0.0 ? prod * (L - 1.0) : 0.001;
    oe_out[i] = expected > 0.0 ? (double)cpg / expected : 0.0;
    // first-appearance pattern of the present bases -> set() iteration order (table row)
    int rank[4] = {0, 1, 2, 3};
    for (int a = 1; a < 4; ++a)   // stable sort of the bases by first position
        for (int b = a; b > 0 && first[rank[b]] < first[rank[b - 1]]; --b) {
            const int t = rank[b];
            rank[b] = rank[b - 1];
            rank[b - 1] = t;
        }
    int key = 0;
    for (int r = 0; r < 4; ++r) key = key * 5 + (first[rank[r]] < (1 << 20) ? rank[r] + 1 : 0);
    double ent = 0.0;
    for (int r = 0; r < 4; ++r) {
        const int b = order[key * 4 + r];
        if (b < 0) break;
        const int nb = cnt[b];
        const double p = (double)nb / L;
        const double term = p * lg[nb * (k + 1) + m];
        ent = ent - term;                                             // entropy -= prob * log2(prob)
    }
    ent_out[i] = ent;
    for (int b = 0; b < 4; ++b) cnt_out[(uint64_t)b * n + i] = cnt[b];
    cpg_out[i] = cpg;
    rep_out[i] = rep;
}

}  // namespace

int feature_columns(Ctx* ctx, const uint64_t* d_codes, uint64_t n, int k, const int32_t* d_order, const double* d_lg,
                    int64_t* d_cnt, int64_t* d_cpg, int64_t* d_rep, double* d_gc, double* d_oe, double* d_ent,
                    hipStream_t s) {
    if (k < 1 || k > 32) return fail(ctx, KMH_ERR_UNSUPPORTED, "feature columns need 1 <= k <= 32");
    if (!d_order || !d_lg || !d_cnt || !d_cpg || !d_rep || !d_gc || !d_oe || !d_ent)
        return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if (n == 0) return KMH_OK;
    time_begin(ctx, s, "k_features");
    hipLaunchKernelGGL(k_features, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_codes, n, k, d_order, d_lg,
                       d_cnt, d_cpg, d_rep, d_gc, d_oe, d_ent);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

}  // namespace kmh
