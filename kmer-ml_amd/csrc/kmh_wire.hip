// kmh_wire.hip -- the exchange step of the column-sharded config-5 matrix
// (/root/reference/kmerml/ml/features.py:96-111: the matrix's columns are the sorted union of every
// organism's labels; here every rank owns a contiguous code range, so every organism row must reach
// the rank of each of its codes).  Rows are sorted by code (kmh_count_sparse_sorted_dev), so what a
// rank sends another is one contiguous slice per row: its start and end come from binary searches of
// the range bounds (k_rows_cuts), which also give the global code histogram that places the bounds.
//
// The compact wire.  A sorted row slice is mostly small gaps between codes
// (k = 21 canonical, 250 Mbp genomes: ~9e3 codes in the dense low end of the canonical code space,
// more towards its top) and counts of 1, so it travels as chunk records of 1024 entries:
//
//   [u64 anchor = the chunk's first code][u32 first escape word of the chunk, slice-relative]
//   [u32 escape words of the chunk | wide << 31]
//   [u16 x 1024: the low 16 bits of each gap, code - previous code (0 for the first entry, and past
//    the slice's end)]
//   [u64 x 16: bit i set = entry i's gap has high bits (gap >> 16 != 0)]
//   [u64 x 16: bit i set = entry i's count is not 1]
//
// (2320 bytes, 2.27 B per entry), and after a slice's records its escape words (u32), in entry
// order: for an entry with high bits, gap >> 16 in one word (two, low word first, in a "wide" chunk,
// one with a gap of 2^48 or more: k >= 25 codes), then for a count that is not 1, the count.  The
// position of an entry's words is the prefix sum of the words of the entries before it, so the
// flags carry no index: an escape costs 4 bytes (8 in a wide chunk).  Exact for any codes and
// counts (k = 32 codes use all 64 bits; the sums wrap like the codes).  A slice is sized first
// (k_wire_count: words per chunk, a scan, the slice's bytes), then packed (k_wire_pack), and the
// receiver rebuilds codes and counts with two scans per chunk (escape positions, then codes;
// k_wire_unpack) straight into its shard's row layout.  Every kernel is one streaming pass: the
// reads and writes are the algorithmic bytes (12 B per entry raw, ~2.4 B packed for config 5).
#include <algorithm>
#include <vector>

#include "kmh_device.h"

namespace kmh {
namespace {

constexpr int kWThreads = 256;
constexpr int kWPer = 4;                               // entries per thread: j * 256 + tid
constexpr int kWChunk = kWThreads * kWPer;             // entries per chunk record
constexpr int kWHead = 16;
constexpr int kWHi = kWHead + 2 * kWChunk;             // offset of the high-bits bitmap
constexpr int kWCnt = kWHi + kWChunk / 8;              // offset of the count bitmap
constexpr int kWRec = kWCnt + kWChunk / 8;             // 2320 bytes
constexpr int kWMaxWords = 3 * kWChunk;                // escape words of one chunk, at most
static_assert(kWRec % 16 == 0, "records keep 16-byte alignment");

// cuts[r * nb + b] = the first entry of row r (relative to the row) whose code is >= bounds[b].
__global__ __launch_bounds__(256) void k_rows_cuts(const uint64_t* __restrict__ codes, const uint64_t* __restrict__ roff,
                                                   uint32_t R, const uint64_t* __restrict__ bounds, uint32_t nb,
                                                   uint64_t* __restrict__ cuts) {
    const uint64_t x = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (x >= (uint64_t)R * nb) return;
    const uint32_t r = (uint32_t)(x / nb), b = (uint32_t)(x % nb);
    const uint64_t a = roff[r], e = roff[r + 1];
    const uint64_t c = bounds[b];
    uint64_t lo = a, hi = e;
    while (lo < hi) {
        const uint64_t m = lo + (hi - lo) / 2u;
        if (codes[m] < c) lo = m + 1u;
        else hi = m;
    }
    cuts[x] = lo - a;
}

// The slice of chunk c: the last s with cbase[s] <= c (cbase: S + 1 non-decreasing chunk starts;
// empty slices own no chunk).
__device__ __forceinline__ uint32_t slice_of(const uint64_t* __restrict__ cbase, uint32_t S, uint64_t c) {
    uint32_t a = 0u, b = S - 1u;
    while (a < b) {
        const uint32_t m = (a + b + 1u) / 2u;
        if (cbase[m] <= c) a = m;
        else b = m - 1u;
    }
    return a;
}

// Sum over the workgroup (kWThreads) of a u64; ws: kWThreads / 64 words.
__device__ __forceinline__ uint64_t block_sum64(uint64_t v, uint64_t* ws) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63u) == 0u) ws[threadIdx.x >> 6] = v;
    lds_barrier();
    uint64_t t = 0u;
#pragma unroll
    for (int w = 0; w < kWThreads / 64; ++w) t += ws[w];
    lds_barrier();
    return t;
}

__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    return v;
}

// Per-entry flags packed for one block reduction: high bits (1 << 0), a high part of 32 bits or
// more (1 << 21), a count that is not 1 (1 << 42).
__device__ __forceinline__ uint64_t flag_bits(uint64_t gap, uint32_t cnt, bool v) {
    if (!v) return 0ull;
    const uint64_t hi = gap >> 16;
    return (hi ? 1ull : 0ull) | ((hi >> 32) ? (1ull << 21) : 0ull) | (cnt != 1u ? (1ull << 42) : 0ull);
}

// Bits 0..15 of x to bits 0, 4, 8, .., 60 (the bitmap words of 16 threads' 4 entries each).
__device__ __forceinline__ uint64_t spread16(uint64_t x) {
    x &= 0xFFFFull;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}

// Escape words of a chunk from its summed flags.
__device__ __forceinline__ uint32_t chunk_words(uint64_t f, bool* wide) {
    const uint32_t nh = (uint32_t)(f & 0x1FFFFFu), nw = (uint32_t)((f >> 21) & 0x1FFFFFu), nc = (uint32_t)(f >> 42);
    *wide = nw != 0u;
    return nh * (nw ? 2u : 1u) + nc;
}

// A chunk's place: slice s, chunk index within it, first entry (input index), entries.
struct Chunk {
    uint32_t s;
    uint64_t cl, base;
    uint32_t n;
};

__device__ __forceinline__ Chunk chunk_at(const uint64_t* __restrict__ sstart, const uint64_t* __restrict__ sn,
                                          const uint64_t* __restrict__ cbase, uint32_t S, uint64_t c) {
    Chunk k;
    k.s = slice_of(cbase, S, c);
    k.cl = c - cbase[k.s];
    k.base = sstart[k.s] + k.cl * kWChunk;
    const uint64_t rem = sn[k.s] - k.cl * kWChunk;
    k.n = (uint32_t)(rem < (uint64_t)kWChunk ? rem : (uint64_t)kWChunk);
    return k;
}

// Escape words of every chunk.
__global__ __launch_bounds__(kWThreads) void k_wire_count(const uint64_t* __restrict__ codes,
                                                          const uint32_t* __restrict__ counts,
                                                          const uint64_t* __restrict__ sstart,
                                                          const uint64_t* __restrict__ sn,
                                                          const uint64_t* __restrict__ cbase, uint32_t S, uint64_t NC,
                                                          uint32_t* __restrict__ esc) {
    __shared__ uint64_t ws[kWThreads / 64];
    const uint32_t tid = threadIdx.x;
    for (uint64_t c = blockIdx.x; c < NC; c += gridDim.x) {
        const Chunk ch = chunk_at(sstart, sn, cbase, S, c);
        // (entries j * 256 + tid: every load instruction reads 512 contiguous bytes; the flags do
        // not depend on which thread holds an entry -- 7.9 vs 11.5 ms at N = 8 with 4 consecutive
        // entries per thread, whose loads stride 32 bytes)
        uint64_t f = 0ull;
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const uint32_t i = (uint32_t)j * kWThreads + tid;
            const bool v = i < ch.n;
            const uint64_t code = v ? codes[ch.base + i] : 0ull;
            const uint64_t prev = v && i ? codes[ch.base + i - 1u] : code;
            f += flag_bits(code - prev, v ? counts[ch.base + i] : 1u, v);
        }
        bool wide;
        const uint32_t t = chunk_words(block_sum64(f, ws), &wide);
        if (tid == 0) esc[c] = t;
    }
}

// Bytes of every slice: its records + its escape words, padded to 16 bytes (esc_off: exclusive scan
// of the chunks' words).
__global__ __launch_bounds__(256) void k_wire_slice_bytes(const uint64_t* __restrict__ cbase,
                                                          const unsigned long long* __restrict__ esc_off, uint32_t S,
                                                          uint64_t* __restrict__ sbytes) {
    const uint32_t s = blockIdx.x * 256u + threadIdx.x;
    if (s >= S) return;
    const uint64_t c0 = cbase[s], c1 = cbase[s + 1];
    sbytes[s] = (c1 - c0) * (uint64_t)kWRec + ((uint64_t)(esc_off[c1] - esc_off[c0]) * 4u + 15u) / 16u * 16u;
}

// Workgroup exclusive scan of a u32 (kWThreads); returns the prefix, *total the sum.
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* ws, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t incl = scan64(v);
    if (lane == 63u) ws[wave] = incl;
    lds_barrier();
    uint32_t pre = incl - v, tot = 0u;
#pragma unroll
    for (int w = 0; w < kWThreads / 64; ++w) {
        pre += (uint32_t)w < wave ? ws[w] : 0u;
        tot += ws[w];
    }
    lds_barrier();
    *total = tot;
    return pre;
}

// Pack every chunk: record at sboff[s] + cl * kWRec, escape words in the slice's table.  Thread t
// packs entries 4t .. 4t + 3: one 8-byte store of their low gap bits, a nibble of each bitmap
// (paired into bytes with the next thread's), and their escape words from one workgroup scan.
__global__ __launch_bounds__(kWThreads) void k_wire_pack(const uint64_t* __restrict__ codes,
                                                         const uint32_t* __restrict__ counts,
                                                         const uint64_t* __restrict__ sstart,
                                                         const uint64_t* __restrict__ sn,
                                                         const uint64_t* __restrict__ cbase, uint32_t S, uint64_t NC,
                                                         const unsigned long long* __restrict__ esc_off,
                                                         const uint64_t* __restrict__ sboff, uint8_t* __restrict__ out) {
    __shared__ uint64_t ws64[kWThreads / 64];
    __shared__ uint64_t scode[kWChunk];
    __shared__ uint32_t scnt[kWChunk];
    const uint32_t tid = threadIdx.x;
    // the chunk's entries by coalesced loads (entry j * 256 + tid), software-pipelined: the next
    // chunk's loads are issued before this chunk's work, then staged in LDS for 4 consecutive
    // entries per thread (their previous entry too: no second global load)
    uint64_t lc[kWPer];
    uint32_t ln[kWPer];
    auto load_chunk = [&](const Chunk& k) {
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const uint32_t i = (uint32_t)j * kWThreads + tid;
            const bool v = i < k.n;
            lc[j] = v ? codes[k.base + i] : 0ull;
            ln[j] = v ? counts[k.base + i] : 1u;
        }
    };
    uint64_t c = blockIdx.x;
    if (c >= NC) return;
    Chunk ch = chunk_at(sstart, sn, cbase, S, c);
    load_chunk(ch);
    for (;;) {
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            scode[(uint32_t)j * kWThreads + tid] = lc[j];
            scnt[(uint32_t)j * kWThreads + tid] = ln[j];
        }
        const uint64_t c2 = c + gridDim.x;
        Chunk ch2 = ch;
        if (c2 < NC) {
            ch2 = chunk_at(sstart, sn, cbase, S, c2);
            load_chunk(ch2);
        }
        const uint64_t c0 = cbase[ch.s];
        uint8_t* const rec = out + sboff[ch.s] + ch.cl * (uint64_t)kWRec;
        const unsigned long long w0 = esc_off[c] - esc_off[c0];   // the chunk's first escape word in the slice
        uint32_t* const etab = reinterpret_cast<uint32_t*>(out + sboff[ch.s] + (cbase[ch.s + 1] - c0) * (uint64_t)kWRec) + w0;
        lds_barrier();
        uint64_t code[kWPer], gap[kWPer];
        uint32_t cnt[kWPer];
        {
            const uint32_t i0 = kWPer * tid;
            const uint64_t p0 = (i0 && i0 < ch.n) ? scode[i0 - 1u] : scode[i0];
#pragma unroll
            for (int j = 0; j < kWPer; ++j) {
                const bool v = i0 + j < ch.n;
                code[j] = scode[i0 + j];
                cnt[j] = v ? scnt[i0 + j] : 1u;
                gap[j] = v ? code[j] - (j ? code[j - 1] : p0) : 0ull;
            }
        }
        // one workgroup scan gives both layouts' word positions and whether the chunk is wide:
        // (words if narrow | words if wide << 21 | wide gaps << 42) per thread
        uint32_t nh = 0u, nc = 0u, nw = 0u;
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const uint64_t hi = gap[j] >> 16;
            nh |= (hi ? 1u : 0u) << j;
            nc |= (cnt[j] != 1u ? 1u : 0u) << j;
            nw += (hi >> 32) ? 1u : 0u;
        }
        const uint32_t ph = (uint32_t)__builtin_popcount(nh), pc = (uint32_t)__builtin_popcount(nc);
        const uint64_t mine = (uint64_t)(ph + pc) | (uint64_t)(2u * ph + pc) << 21 | (uint64_t)nw << 42;
        const uint32_t lane = tid & 63u, wave = tid >> 6;
        const uint64_t incl = wave_incl_u64(mine);
        if (lane == 63u) ws64[wave] = incl;
        const uint64_t hb[4] = {__ballot(nh & 1u), __ballot(nh & 2u), __ballot(nh & 4u), __ballot(nh & 8u)};
        const uint64_t cb[4] = {__ballot(nc & 1u), __ballot(nc & 2u), __ballot(nc & 4u), __ballot(nc & 8u)};
        lds_barrier();   // (also frees scode for the next chunk)
        uint64_t pre = incl - mine, tot = 0ull;
#pragma unroll
        for (int w = 0; w < kWThreads / 64; ++w) {
            pre += (uint32_t)w < wave ? ws64[w] : 0ull;
            tot += ws64[w];
        }
        const bool wide = (tot >> 42) != 0ull;
        const uint32_t words = wide ? (uint32_t)((tot >> 21) & 0x1FFFFFu) : (uint32_t)(tot & 0x1FFFFFu);
        uint32_t pos = wide ? (uint32_t)((pre >> 21) & 0x1FFFFFu) : (uint32_t)(pre & 0x1FFFFFu);
        if (tid == 0) {
            *reinterpret_cast<uint64_t*>(rec) = code[0];
            *reinterpret_cast<uint2*>(rec + 8) = make_uint2((uint32_t)w0, words | (wide ? 0x80000000u : 0u));
        }
        *reinterpret_cast<uint64_t*>(rec + kWHead + 8u * tid) =
            (gap[0] & 0xFFFFull) | (gap[1] & 0xFFFFull) << 16 | (gap[2] & 0xFFFFull) << 32 | (gap[3] & 0xFFFFull) << 48;
        if (lane < 4u) {   // the wave's 256 bits of each bitmap: entry 4 t + j is ballot j's bit t
            const uint32_t sh = 16u * lane;
            const uint64_t h = spread16(hb[0] >> sh) | spread16(hb[1] >> sh) << 1 | spread16(hb[2] >> sh) << 2 |
                               spread16(hb[3] >> sh) << 3;
            const uint64_t q = spread16(cb[0] >> sh) | spread16(cb[1] >> sh) << 1 | spread16(cb[2] >> sh) << 2 |
                               spread16(cb[3] >> sh) << 3;
            *reinterpret_cast<uint64_t*>(rec + kWHi + wave * 32u + 8u * lane) = h;
            *reinterpret_cast<uint64_t*>(rec + kWCnt + wave * 32u + 8u * lane) = q;
        }
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const uint64_t hi = gap[j] >> 16;
            if (hi) {
                etab[pos++] = (uint32_t)hi;
                if (wide) etab[pos++] = (uint32_t)(hi >> 32);
            }
            if (cnt[j] != 1u) etab[pos++] = cnt[j];
        }
        if (c + 1u == cbase[ch.s + 1] && tid < 4u) {   // the slice's last chunk zeroes the table's padding
            const unsigned long long sw = esc_off[c + 1u] - esc_off[c0];
            if (tid < ((4u - (uint32_t)(sw & 3u)) & 3u)) etab[sw - w0 + tid] = 0u;
        }
        if (c2 >= NC) break;
        c = c2;
        ch = ch2;
    }
}

// Unpack every chunk of the received slices: slice s (entries sn[s]) at byte sboff[s] of `in`, its
// entries to sdst[s] .. of the output.  Thread t rebuilds entries 4t .. 4t + 3: two workgroup scans
// per chunk (its escape words' position, then its codes' prefix).  Escape positions are clamped to
// the chunk's words and those to the slice's table, so a damaged buffer cannot make a read or write
// leave the slice.
__global__ __launch_bounds__(kWThreads) void k_wire_unpack(const uint8_t* __restrict__ in,
                                                           const uint64_t* __restrict__ sboff,
                                                           const uint64_t* __restrict__ sn,
                                                           const uint64_t* __restrict__ sesc,
                                                           const uint64_t* __restrict__ sdst,
                                                           const uint64_t* __restrict__ cbase, uint32_t S, uint64_t NC,
                                                           uint64_t* __restrict__ out_codes,
                                                           uint32_t* __restrict__ out_counts) {
    __shared__ uint32_t wbuf[kWMaxWords];
    __shared__ uint64_t ws64[kWThreads / 64];
    __shared__ uint32_t ws[kWThreads / 64];
    __shared__ uint64_t ocode[kWChunk];
    __shared__ uint32_t ocnt[kWChunk];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, i0 = kWPer * tid;
    for (uint64_t c = blockIdx.x; c < NC; c += gridDim.x) {
        const uint32_t s = slice_of(cbase, S, c);
        const uint64_t c0 = cbase[s], cl = c - c0;
        const uint64_t rem = sn[s] - cl * kWChunk;
        const uint32_t n = (uint32_t)(rem < (uint64_t)kWChunk ? rem : (uint64_t)kWChunk);
        const uint8_t* const rec = in + sboff[s] + cl * (uint64_t)kWRec;
        const uint32_t* const etab = reinterpret_cast<const uint32_t*>(in + sboff[s] + (cbase[s + 1] - c0) * (uint64_t)kWRec);
        const uint64_t anchor = *reinterpret_cast<const uint64_t*>(rec);
        const uint2 eh = *reinterpret_cast<const uint2*>(rec + 8);
        const uint64_t lowv = *reinterpret_cast<const uint64_t*>(rec + kWHead + 8u * tid);
        const uint32_t sh = 4u * (tid & 1u);
        const uint32_t hb = (rec[kWHi + tid / 2u] >> sh) & 0xFu, cb = (rec[kWCnt + tid / 2u] >> sh) & 0xFu;
        const bool wide = (eh.y >> 31) != 0u;
        const uint64_t etot = sesc[s];
        const uint64_t wlo = eh.x < etot ? eh.x : etot;
        uint32_t wn = eh.y & 0x7FFFFFFFu;
        wn = (uint32_t)((uint64_t)wn < etot - wlo ? (uint64_t)wn : etot - wlo);
        wn = wn < (uint32_t)kWMaxWords ? wn : (uint32_t)kWMaxWords;
        for (uint32_t w = tid; w < wn; w += kWThreads) wbuf[w] = etab[wlo + w];
        uint32_t tw = 0u;
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const bool v = i0 + j < n;
            tw += (v && ((hb >> j) & 1u) ? (wide ? 2u : 1u) : 0u) + (v && ((cb >> j) & 1u) ? 1u : 0u);
        }
        uint32_t tot;
        uint32_t p = block_excl(tw, ws, &tot);   // (its barriers also publish wbuf)
        uint64_t gap[kWPer];
        uint32_t cnt[kWPer];
        uint64_t sum = 0ull;
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const bool v = i0 + j < n;
            uint64_t hi = 0ull;
            if (v && ((hb >> j) & 1u)) {
                hi = p < wn ? wbuf[p] : 0u;
                ++p;
                if (wide) {
                    hi |= (uint64_t)(p < wn ? wbuf[p] : 0u) << 32;
                    ++p;
                }
            }
            cnt[j] = 1u;
            if (v && ((cb >> j) & 1u)) {
                cnt[j] = p < wn ? wbuf[p] : 0u;
                ++p;
            }
            gap[j] = v ? (((lowv >> (16 * j)) & 0xFFFFull) | (hi << 16)) : 0ull;
            sum += gap[j];
        }
        const uint64_t incl = wave_incl_u64(sum);
        if (lane == 63u) ws64[wave] = incl;
        lds_barrier();
        uint64_t code = anchor + incl - sum;
#pragma unroll
        for (int w = 0; w < kWThreads / 64; ++w) code += (uint32_t)w < wave ? ws64[w] : 0ull;
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            code += gap[j];
            ocode[i0 + j] = code;
            ocnt[i0 + j] = cnt[j];
        }
        lds_barrier();
        // stored from LDS by entry j * 256 + tid: every store instruction writes contiguous bytes
        uint64_t* const oc = out_codes + sdst[s] + cl * kWChunk;
        uint32_t* const on = out_counts + sdst[s] + cl * kWChunk;
#pragma unroll
        for (int j = 0; j < kWPer; ++j) {
            const uint32_t i = (uint32_t)j * kWThreads + tid;
            if (i < n) {
                oc[i] = ocode[i];
                on[i] = ocnt[i];
            }
        }
        lds_barrier();   // wbuf, ws64 and the staging are rewritten by the next chunk
    }
}

unsigned grid_for(Ctx* ctx, uint64_t NC) {
    return (unsigned)std::min<uint64_t>(std::max<uint64_t>(NC, 1), (uint64_t)std::max(1, ctx->num_cu) * 16);
}

uint64_t fnv(uint64_t h, const uint64_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001B3ull;
    }
    return h;
}

}  // namespace

int rows_cuts(Ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, const uint64_t* bounds, int nb,
              uint64_t* d_cuts, hipStream_t s) {
    if (R < 0 || nb < 0 || (R && !row_off) || (nb && !bounds)) return fail(ctx, KMH_ERR_INVALID, "bad cuts arguments");
    if (!R || !nb) return KMH_OK;
    if (!d_codes || !d_cuts) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    for (int r = 0; r < R; ++r)
        if (row_off[r + 1] < row_off[r]) return fail(ctx, KMH_ERR_INVALID, "row offsets must ascend");
    std::vector<uint64_t> h((size_t)R + 1 + nb);
    std::copy(row_off, row_off + R + 1, h.begin());
    std::copy(bounds, bounds + nb, h.begin() + R + 1);
    int rc = ensure(ctx, ctx->wire[0], h.size() * 8 + 256);
    if (rc) return rc;
    uint64_t* d = static_cast<uint64_t*>(ctx->wire[0].ptr);
    if ((rc = upload(ctx, d, h.data(), h.size() * 8, s))) return rc;
    const uint64_t n = (uint64_t)R * (uint64_t)nb;
    time_begin(ctx, s, "k_rows_cuts");
    hipLaunchKernelGGL(k_rows_cuts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_codes, d, (uint32_t)R,
                       d + R + 1, (uint32_t)nb, d_cuts);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

// The plan of S slices (host): chunk starts, chunks; uploads [sstart | sn | cbase] to wire[0].
static int wire_layout(Ctx* ctx, const uint64_t* sstart, const uint64_t* sn, int S, std::vector<uint64_t>& cbase,
                       uint64_t** d_plan, hipStream_t s) {
    cbase.assign((size_t)S + 1, 0);
    for (int i = 0; i < S; ++i) {
        if (sn[i] >= (1ull << 40)) return fail(ctx, KMH_ERR_INVALID, "wire: slice too large");
        cbase[i + 1] = cbase[i] + (sn[i] + kWChunk - 1) / kWChunk;
    }
    std::vector<uint64_t> h(3 * (size_t)S + 1 + S);
    std::copy(sstart, sstart + S, h.begin());
    std::copy(sn, sn + S, h.begin() + S);
    std::copy(cbase.begin(), cbase.end(), h.begin() + 2 * S);
    int rc = ensure(ctx, ctx->wire[0], h.size() * 8 + 256);
    if (rc) return rc;
    *d_plan = static_cast<uint64_t*>(ctx->wire[0].ptr);
    return upload(ctx, *d_plan, h.data(), (3 * (size_t)S + 1) * 8, s);
}

// Count + scan + slice bytes of a plan.  use_cache: take the result of the last sizing if it was
// made on the same inputs and slices and not used yet (the encode right after a size call); every
// use consumes it, and a size call always recomputes, so a stale sizing is never reused.
static int wire_sizes(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* sstart,
                      const uint64_t* sn, int S, std::vector<uint64_t>& cbase, uint64_t** d_plan,
                      std::vector<uint64_t>& sbytes, bool use_cache, hipStream_t s) {
    int rc = wire_layout(ctx, sstart, sn, S, cbase, d_plan, s);
    if (rc) return rc;
    const uint64_t NC = cbase[S];
    uint64_t key = fnv(0xCBF29CE484222325ull, sstart, S);
    key = fnv(key, sn, S);
    const uint64_t ptrs[3] = {(uint64_t)(uintptr_t)d_codes, (uint64_t)(uintptr_t)d_counts, (uint64_t)S};
    key = fnv(key, ptrs, 3);
    if (use_cache && ctx->wire_valid && ctx->wire_key == key && ctx->wire_sbytes.size() == (size_t)S) {
        sbytes = ctx->wire_sbytes;
        ctx->wire_valid = false;   // (one use)
        return KMH_OK;
    }
    ctx->wire_valid = false;
    if ((rc = ensure(ctx, ctx->wire[1], (NC + 1) * 4 + 256))) return rc;
    if ((rc = ensure(ctx, ctx->wire[2], (NC + 2) * 8 + 256))) return rc;
    uint32_t* d_esc = static_cast<uint32_t*>(ctx->wire[1].ptr);
    unsigned long long* d_eoff = static_cast<unsigned long long*>(ctx->wire[2].ptr);
    uint64_t* d_sb = *d_plan + 3 * (size_t)S + 1;
    if (NC) {
        time_begin(ctx, s, "k_wire_count");
        hipLaunchKernelGGL(k_wire_count, dim3(grid_for(ctx, NC)), dim3(kWThreads), 0, s, d_codes, d_counts, *d_plan,
                           *d_plan + S, *d_plan + 2 * S, (uint32_t)S, NC, d_esc);
        time_end(ctx, s);
        KMH_HIP(ctx, hipGetLastError());
    }
    if ((rc = scan_u32_u64(ctx, d_esc, (uint32_t)NC, d_eoff, s))) return rc;
    hipLaunchKernelGGL(k_wire_slice_bytes, dim3((S + 255) / 256), dim3(256), 0, s, *d_plan + 2 * S, d_eoff, (uint32_t)S,
                       d_sb);
    KMH_HIP(ctx, hipGetLastError());
    sbytes.assign(S, 0);
    KMH_HIP(ctx, hipMemcpyAsync(sbytes.data(), d_sb, (size_t)S * 8, hipMemcpyDeviceToHost, s));
    KMH_HIP(ctx, hipStreamSynchronize(s));
    ctx->wire_key = key;
    ctx->wire_sbytes = sbytes;
    ctx->wire_valid = true;
    return KMH_OK;
}

int wire_size(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* sstart, const uint64_t* sn,
              int S, uint64_t* slice_bytes, hipStream_t s) {
    if (S < 0 || (S && (!sstart || !sn || !slice_bytes))) return fail(ctx, KMH_ERR_INVALID, "bad wire arguments");
    if (!S) return KMH_OK;
    uint64_t NE = 0;
    for (int i = 0; i < S; ++i) NE += sn[i];
    if (NE && (!d_codes || !d_counts)) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    if ((uint64_t)S > (1ull << 24) || (NE + kWChunk) / kWChunk >= 0xFFFFFFFFull)
        return fail(ctx, KMH_ERR_UNSUPPORTED, "wire: too many slices or chunks");
    std::vector<uint64_t> cbase, sb;
    uint64_t* d_plan = nullptr;
    int rc = wire_sizes(ctx, d_codes, d_counts, sstart, sn, S, cbase, &d_plan, sb, false, s);
    if (rc) return rc;
    for (int i = 0; i < S; ++i) {
        const uint64_t nch = cbase[i + 1] - cbase[i];
        if ((sb[i] - nch * kWRec) / 4u >= 0xFFFFFFFFull) {
            ctx->wire_valid = false;
            return fail(ctx, KMH_ERR_UNSUPPORTED, "wire: 2^32 or more escape words in one slice");
        }
        slice_bytes[i] = sb[i];
    }
    return KMH_OK;
}

int wire_encode(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* sstart, const uint64_t* sn,
                int S, uint8_t* d_out, uint64_t out_bytes, hipStream_t s) {
    if (S < 0 || (S && (!sstart || !sn))) return fail(ctx, KMH_ERR_INVALID, "bad wire arguments");
    if (!S) return KMH_OK;
    std::vector<uint64_t> sb((size_t)S), cbase, h((size_t)S);
    uint64_t* d_plan = nullptr;
    int rc = wire_sizes(ctx, d_codes, d_counts, sstart, sn, S, cbase, &d_plan, sb, true, s);   // (the size call's)
    if (rc) return rc;
    for (int i = 0; i < S; ++i)
        if ((sb[i] - (cbase[i + 1] - cbase[i]) * kWRec) / 4u >= 0xFFFFFFFFull)
            return fail(ctx, KMH_ERR_UNSUPPORTED, "wire: 2^32 or more escape words in one slice");
    uint64_t total = 0;
    for (int i = 0; i < S; ++i) {
        h[i] = total;
        total += sb[i];
    }
    if (total > out_bytes) return fail(ctx, KMH_ERR_INVALID, "wire: output buffer too small");
    if (total && !d_out) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    const uint64_t NC = cbase[S];
    if (!NC) return KMH_OK;
    uint64_t* d_sboff = d_plan + 3 * (size_t)S + 1;
    if ((rc = upload(ctx, d_sboff, h.data(), (size_t)S * 8, s))) return rc;
    time_begin(ctx, s, "k_wire_pack");
    hipLaunchKernelGGL(k_wire_pack, dim3(grid_for(ctx, NC)), dim3(kWThreads), 0, s, d_codes, d_counts, d_plan, d_plan + S,
                       d_plan + 2 * S, (uint32_t)S, NC, static_cast<const unsigned long long*>(ctx->wire[2].ptr),
                       d_sboff, d_out);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

int wire_decode(Ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const uint64_t* sn, const uint64_t* sbytes,
                const uint64_t* sdst, int S, uint64_t* d_codes, uint32_t* d_counts, hipStream_t s) {
    if (S < 0 || (S && (!sn || !sbytes || !sdst))) return fail(ctx, KMH_ERR_INVALID, "bad wire arguments");
    if (!S) return KMH_OK;
    // plan: [sboff | sn | cbase | sesc | sdst]
    std::vector<uint64_t> h(5 * (size_t)S + 1);
    uint64_t* const sboff = h.data();
    uint64_t* const hsn = sboff + S;
    uint64_t* const cb = hsn + S;
    uint64_t* const sesc = cb + S + 1;
    uint64_t* const hdst = sesc + S;
    uint64_t off = 0;
    cb[0] = 0;
    for (int i = 0; i < S; ++i) {
        const uint64_t nch = (sn[i] + kWChunk - 1) / kWChunk;
        if (sn[i] >= (1ull << 40) || sbytes[i] < nch * kWRec || (sbytes[i] - nch * kWRec) % 16u)
            return fail(ctx, KMH_ERR_INVALID, "wire: slice bytes do not match its entries");
        sboff[i] = off;
        off += sbytes[i];
        hsn[i] = sn[i];
        cb[i + 1] = cb[i] + nch;
        sesc[i] = (sbytes[i] - nch * kWRec) / 4u;   // escape words (with the padding)
        hdst[i] = sdst[i];
    }
    if (off > in_bytes) return fail(ctx, KMH_ERR_INVALID, "wire: input shorter than its slices");
    const uint64_t NC = cb[S];
    if (!NC) return KMH_OK;
    if (!d_in || !d_codes || !d_counts) return fail(ctx, KMH_ERR_INVALID, "NULL device pointer");
    int rc = ensure(ctx, ctx->wire[0], h.size() * 8 + 256);
    if (rc) return rc;
    uint64_t* d = static_cast<uint64_t*>(ctx->wire[0].ptr);
    if ((rc = upload(ctx, d, h.data(), h.size() * 8, s))) return rc;
    time_begin(ctx, s, "k_wire_unpack");
    hipLaunchKernelGGL(k_wire_unpack, dim3(grid_for(ctx, NC)), dim3(kWThreads), 0, s, d_in, d, d + S, d + 3 * S + 1,
                       d + 4 * S + 1, d + 2 * S, (uint32_t)S, NC, d_codes, d_counts);
    time_end(ctx, s);
    KMH_HIP(ctx, hipGetLastError());
    return KMH_OK;
}

}  // namespace kmh
