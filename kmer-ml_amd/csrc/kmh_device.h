// kmh_device.h -- device helpers shared by the HIP translation units (dense and sparse
// counting): the genome/tile map of a launch, 16-byte base loads, the ASCII -> 2-bit
// encoder and the XCD-aware work order.
#pragma once

#include "kmh_internal.h"

namespace kmh {

struct GenomeMap {
    const uint64_t* goff;   // genome byte offsets, G + 1 (device)
    const uint64_t* tbase;  // cumulative tile counts, G + 1 (device), tbase[0] = 0
    int g0, g1;             // genomes covered by this launch
    uint64_t tile_lo;       // tbase[g0]
    uint64_t data_end;      // offsets[G]: bytes at or past it may not be readable
};

// Largest g in [g0, g1) with tbase[g] <= gt (genomes without tiles are skipped).
__device__ __forceinline__ int find_genome(const GenomeMap& m, uint64_t gt) {
    int lo = m.g0, hi = m.g1 - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (m.tbase[mid] <= gt) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// 16 bytes at pos; bytes at or past `end` read as 0 (not a base).
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ seq, uint64_t pos,
                                        uint64_t end) {
    if (pos + 16 <= end) return *reinterpret_cast<const uint4*>(seq + pos);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (pos + i < end) w[i >> 2] |= (uint32_t)seq[pos + i] << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Four ASCII bytes (byte 0 first) -> 8 bits of 2-bit codes (byte 0 in bits 7:6) and a
// 4-bit invalid mask (byte 0 in bit 3).  code = ((c >> 1) ^ (c >> 2)) & 3 maps A/a->0,
// C/c->1, G/g->2, T/t->3; a byte is a base iff (c & 0xDF) == "ACGT"[code].
__device__ __forceinline__ void enc4(uint32_t w, uint32_t& c8, uint32_t& i4) {
    const uint32_t cb = ((w >> 1) ^ (w >> 2)) & 0x03030303u;
    const uint32_t expect = __builtin_amdgcn_perm(0u, 0x54474341u, cb);  // "ACGT"[cb]
    const uint32_t e = (w & 0xDFDFDFDFu) ^ expect;                       // 0 byte = base
    const uint32_t nz = (((e & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | e) & 0x80808080u;
    // byte-weighted sums on the full-rate dot-product unit (v_dot4_u32_u8) instead of
    // quarter-rate 32-bit multiplies: byte 0 gets the top bits
    i4 = __builtin_amdgcn_udot4(nz >> 7, 0x01020408u, 0u, false);
    c8 = __builtin_amdgcn_udot4(cb, 0x01041040u, 0u, false);
}

// 16 bytes -> 32-bit code word (first base in bits 31:30) + 16-bit invalid mask (first
// base in bit 15).
__device__ __forceinline__ void enc16(uint4 v, uint32_t& code, uint32_t& inv) {
    uint32_t c0, c1, c2, c3, i0, i1, i2, i3;
    enc4(v.x, c0, i0);
    enc4(v.y, c1, i1);
    enc4(v.z, c2, i2);
    enc4(v.w, c3, i3);
    code = (c0 << 24) | (c1 << 16) | (c2 << 8) | c3;
    inv = (i0 << 12) | (i1 << 8) | (i2 << 4) | i3;
}

// Invalid-mask bits for the bytes of a 16-byte chunk at pos that lie at or past `end`
// (bit 15 = byte 0).
__device__ __forceinline__ uint32_t tail_mask(uint64_t pos, uint64_t end) {
    if (end >= pos + 16) return 0u;
    if (end <= pos) return 0xFFFFu;
    return 0xFFFFu >> (uint32_t)(end - pos);
}

// XCD-aware work order: blocks b and b+8 share an XCD under the observed round-robin
// placement, so hand each XCD a contiguous range of work items (speed only).
// Bijective for any grid size: XCD group x = b % 8 owns a contiguous run of work items.
__device__ __forceinline__ uint32_t xcd_work_id() {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t q = nb / 8u, rem = nb % 8u, x = b % 8u;
    return x * q + (x < rem ? x : rem) + b / 8u;
}

// DPP: v of lane (lane - D) in the same 16-lane row, 0 where that lane lies outside it.
template <int D>
__device__ __forceinline__ uint32_t dpp_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + D, 0xF, 0xF, true);
}
// Inclusive scan inside each group of 8 lanes (lanes 8i .. 8i+7).
__device__ __forceinline__ uint32_t scan8(uint32_t s, int lane) {
    const int q = lane & 7;
    uint32_t t = dpp_shr<1>(s);
    s += q >= 1 ? t : 0u;
    t = dpp_shr<2>(s);
    s += q >= 2 ? t : 0u;
    t = dpp_shr<4>(s);
    s += q >= 4 ? t : 0u;
    return s;
}
// Inclusive scan over the 64 lanes of a wave.
__device__ __forceinline__ uint32_t scan64(uint32_t s) {
    s += dpp_shr<1>(s);
    s += dpp_shr<2>(s);
    s += dpp_shr<4>(s);
    s += dpp_shr<8>(s);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x142, 0xA, 0xF, false);  // row_bcast:15
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return s;
}

// Workgroup barrier for LDS only.  __syncthreads() is also a release fence for global
// memory, i.e. it waits for every store the wave has in flight (s_waitcnt vmcnt(0)); the
// persistent kernels never read back what they store, so their barriers need only the LDS
// operations to be complete: one item's stores drain, and the next item's prefetched loads
// stay in flight, across the barrier.
__device__ __forceinline__ void lds_barrier() {
    __asm__ __volatile__("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 16-byte store with the non-temporal policy: streamed output that this XCD never reads back
// leaves no dirty lines in L2, so the write-back at the next kernel boundary (which stalls the
// dependent kernel, MI355X_MICROARCH.md "boundary") stays small.
typedef unsigned int kmh_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_nt(uint4* dst, const uint4& v) {
    kmh_u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<kmh_u32x4*>(dst));
}

}  // namespace kmh
