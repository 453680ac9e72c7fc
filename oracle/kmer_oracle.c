/*
 * oracle/kmer_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference's k-mer counting loop, used as the
 * checker for the HIP path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  It is never linked into, called by, or shipped
 * with the product library (kmer-ml_amd/csrc).
 *
 * Restated from /root/reference/kmerml/kmers/generate.py:
 *   :41      sequence = str(record.seq).upper()     -> a/c/g/t count as A/C/G/T
 *   :49-52   for k: for i in range(len(seq)-k+1): kmer = seq[i:i+k]
 *   :55-56   skip the window if any char is not in "ACGT"
 *   :58      all_kmers[k][kmer] += 1                 -> counts per distinct k-mer,
 *            dict insertion order = first occurrence -> we also return the first
 *            window position of every k-mer so the caller can rebuild that order.
 * The input here is ONE record's bytes, or several records joined by a byte that
 * is not a base (windows never span records, generate.py:39-58 loops per record).
 *
 * Pinning: checked against golden vectors produced by the reference's own
 * generate.py (tests/golden/, see tests/golden/make_golden.py).
 *
 * Code convention: 2 bits per base, A=0 C=1 G=2 T=3, first base most significant,
 * so the integer order of codes is the lexicographic order of the k-mer strings.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline int orc_base(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

/* splitmix64 finaliser applied to (x + golden gamma): the synthetic-genome PRNG
 * of SURVEY.md section 8(d).  Host and device generate identical bytes. */
uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* base[i] = "ACGT"[(splitmix64(seed + (i >> 5)) >> (2 * (i & 31))) & 3],
 * for i in [i0, i0 + len). */
void orc_synth(uint8_t* out, uint64_t i0, uint64_t len, uint64_t seed) {
    static const uint8_t acgt[4] = {'A', 'C', 'G', 'T'};
    uint64_t i = i0, end = i0 + len;
    while (i < end) {
        uint64_t r = orc_splitmix64(seed + (i >> 5));
        uint64_t stop = ((i >> 5) + 1) << 5;
        if (stop > end) stop = end;
        for (; i < stop; ++i) *out++ = acgt[(r >> (2 * (i & 31))) & 3];
    }
}

/* Dense count for k <= 16.  counts: 4^k u32 (zeroed here).  first: 4^k u32 or
 * NULL, set to the first window start of each k-mer (0xFFFFFFFF if absent).
 * Returns the number of valid windows, or -1 on bad arguments. */
int64_t orc_count_dense(const uint8_t* seq, uint64_t n, int k, uint32_t* counts,
                        uint32_t* first) {
    if (k < 1 || k > 16) return -1;
    uint64_t bins = 1ull << (2 * k);
    uint64_t mask = bins - 1;
    memset(counts, 0, bins * sizeof(uint32_t));
    if (first) memset(first, 0xFF, bins * sizeof(uint32_t));
    uint64_t code = 0;
    int run = 0;
    int64_t nvalid = 0;
    for (uint64_t i = 0; i < n; ++i) {
        int b = orc_base(seq[i]);
        if (b < 0) { run = 0; code = 0; continue; }
        code = ((code << 2) | (uint64_t)b) & mask;
        if (++run >= k) {
            uint64_t start = i + 1 - (uint64_t)k;
            counts[code]++;
            if (first && first[code] == 0xFFFFFFFFu) first[code] = (uint32_t)start;
            nvalid++;
        }
    }
    return nvalid;
}

typedef struct { uint64_t code; uint64_t pos; } orc_pair;

static int orc_pair_cmp(const void* a, const void* b) {
    const orc_pair* x = (const orc_pair*)a;
    const orc_pair* y = (const orc_pair*)b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    if (x->pos != y->pos) return x->pos < y->pos ? -1 : 1;
    return 0;
}

/* Sparse count for 1 <= k <= 32, optionally canonical (min of the forward code and
 * the reverse-complement code; complement of A0 C1 G2 T3 is 3 - b).  Outputs the
 * distinct k-mers in ascending code order with counts and first window start.
 * codes/counts/first must hold at least max(n - k + 1, 0) entries.
 * Returns the number of distinct k-mers, or -1 on error. */
int64_t orc_count_sparse(const uint8_t* seq, uint64_t n, int k, int canonical,
                         uint64_t* codes, uint32_t* counts, uint64_t* first) {
    if (k < 1 || k > 32) return -1;
    if (n < (uint64_t)k) return 0;
    uint64_t nwin = n - (uint64_t)k + 1;
    orc_pair* v = (orc_pair*)malloc(nwin * sizeof(orc_pair));
    if (!v) return -1;
    uint64_t mask = (k == 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    uint64_t fwd = 0, rc = 0, m = 0;
    int run = 0;
    int top = 2 * (k - 1);
    for (uint64_t i = 0; i < n; ++i) {
        int b = orc_base(seq[i]);
        if (b < 0) { run = 0; fwd = rc = 0; continue; }
        fwd = ((fwd << 2) | (uint64_t)b) & mask;
        rc = (rc >> 2) | ((uint64_t)(3 - b) << top);
        if (++run >= k) {
            uint64_t c = fwd;
            if (canonical && rc < c) c = rc;
            v[m].code = c;
            v[m].pos = i + 1 - (uint64_t)k;
            m++;
        }
    }
    qsort(v, m, sizeof(orc_pair), orc_pair_cmp);
    int64_t d = 0;
    for (uint64_t i = 0; i < m;) {
        uint64_t j = i;
        while (j < m && v[j].code == v[i].code) ++j;
        codes[d] = v[i].code;
        counts[d] = (uint32_t)(j - i);
        first[d] = v[i].pos;
        d++;
        i = j;
    }
    free(v);
    return d;
}
