// Microbenchmark: the floor of a CONSUMER-RESIDENT exchange for the dense
// k = 12 count (/root/reference/kmerml/kmers/generate.py:49-58 over 64 x 100 Mbp genomes), memory and
// LDS traffic only.  Today's path writes every window's 16-bit suffix to HBM in bucket order
// (k_partition) and reads it back per bucket (k_bucket_count): DESIGN §4 measured that pattern's
// floor at ~108 us per genome.  Here every CU keeps ONE bucket's 2^16-bin u16 table in LDS for the
// whole run and the suffixes only pass through a ring small enough for the 256 MiB Infinity Cache:
//
//   one workgroup per CU (grid = 256, 1024 threads): waves 0-3 are the consumer of bucket
//   blockIdx.x, waves 4-15 are producers.  A producer WAVE takes tiles t = id, id + 3072, ...
//   (16384 windows = 16 KB of bases each): waits until every consumer has finished tile t - RT
//   (back-pressure: per-wave progress words, polled with sc1 loads, min cached), reads the tile's
//   bases (plain loads), writes the tile's 32 KB of suffixes into ring slot t % RT in 256 segments
//   of 128 B (write-through sc1 stores), drains its stores (vmcnt(0)) and sets ready[slot] = t + 1
//   (sc1 store, one lane).  A consumer wave takes groups of 64 consecutive tiles (wave w: groups
//   w, w + 4, ...): lane i polls ready[] of tile T0 + i (sc1, bounded spin), then loads its tile's
//   segment of this bucket (128 B, sc1) and adds its 64 suffixes into the LDS table (optional),
//   then publishes its progress.  After each genome the 4 consumer waves meet (LDS counter), write
//   the bucket's 65536-bin row slice (256 KB of u32) and clear the table.
//
// Per genome: 100.7 MB of bases read, 201 MB through the ring each way, 67 MB of rows written (the
// same bytes as the real pattern, synthetic segment sizes: 64 entries per (tile, bucket)).  Every
// spin is bounded (a timeout word is set and the kernel exits; the host reports it).
//   ring_bench [genomes=8] [ring_MiB=64] [mode=1] [reps=3] [shape=4x1|4x2|8x1|8x2|12x2]
// mode bit 0: the consumers' LDS adds; bit 1: no hand-off protocol (producers never wait, consumers
// never poll: the data movement alone, results meaningless -- the floor of the bytes).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

constexpr int kB = 256;                      // buckets = workgroups = CUs
constexpr int kTileWin = 16384;              // windows per tile
constexpr int kSegBytes = kTileWin * 2 / kB;  // 128 B per (tile, bucket)
constexpr int kSlotBytes = kTileWin * 2;     // 32 KiB per ring slot
constexpr int kTilesPerGenome = 6144;        // 100.66 Mbp per genome (a multiple of 64 x 4 x ... tiles)
constexpr int kWaves = 16;
constexpr int kGroup = 64;                   // tiles per consumer group (one per lane)
constexpr unsigned kSpinMax = 1u << 22;      // bounded spins (s_sleep 2-16 each: seconds at most)
constexpr int kRep = 8;                      // flag replicas (one per XCD)

typedef __attribute__((address_space(1))) unsigned gu32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
    return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// NC consumer waves (bucket blockIdx.x) and 16 - NC producer waves per workgroup; a consumer wave
// takes GPI of its groups per round (GPI x 8 loads of 16 B per lane in flight).
template <int NC, int GPI>
__global__ __launch_bounds__(1024) void k_ring(const uint8_t* __restrict__ bases, uint8_t* ring, unsigned RT,
                                               unsigned ntiles, unsigned* ready, unsigned* progress,
                                               unsigned* timeout, uint32_t* rows, int lds_adds) {
    __shared__ uint32_t table[32768];   // 2^16 u16 bins, two per word (128 KiB)
    __shared__ unsigned meet;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned b = blockIdx.x;
    for (int i = tid; i < 32768; i += 1024) table[i] = 0u;
    if (tid == 0) meet = 0u;
    __syncthreads();
    constexpr int kCons = NC, kProd = kWaves - NC;
    const auto ring_rsrc = __builtin_amdgcn_make_buffer_rsrc(ring, (short)0, 0x7FFFFFFF, 0x00020000);
    if (wave >= kCons) {
        // ---------------------------------------------------------------- producer wave
        const unsigned pid = b * kProd + (unsigned)(wave - kCons), np = kB * kProd;
        unsigned minprog = 0u;   // all consumers are past tiles < minprog
        for (unsigned t = pid; t < ntiles; t += np) {
            unsigned spins = 0;
            while (!(lds_adds & 2) && t >= minprog + RT) {   // slot t % RT still holds tile t - RT for some consumer
                unsigned m = 0xFFFFFFFFu;
                for (int q = lane; q < kB * kCons; q += 64) m = min(m, ld_agent(progress + q));
                for (int d = 32; d >= 1; d >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, d));
                minprog = m;
                if (t < minprog + RT) break;
                if (++spins > kSpinMax || ld_agent(timeout)) {
                    if (lane == 0) st_agent(timeout, 1u);
                    return;
                }
                __builtin_amdgcn_s_sleep(16);   // (back-pressure polls: 1024 words, not too often)
            }
            // the tile's bases: 16 KB, 256 B per lane, in two halves; 32 KB of suffixes written
            // through (sc1): 512 B per lane
            const unsigned slot = t % RT;
            const int off0 = (int)(slot * (unsigned)kSlotBytes);
            const uint4* src = reinterpret_cast<const uint4*>(bases + (size_t)t * kTileWin);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint4 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = src[(h * 8 + k) * 64 + lane];
                uint32_t acc = 0u;
#pragma unroll
                for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const u32x4 w = {v[k & 7].x ^ acc, v[k & 7].y + (uint32_t)k, v[k & 7].z, t};
                    __builtin_amdgcn_raw_buffer_store_b128(w, ring_rsrc, off0 + ((h * 16 + k) * 64 + lane) * 16, 0, 16);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // one flag replica per XCD (each on lines of its own): the 256 consumers poll every tile's
            // flag, and one replica polled by all of them serialised at its memory channel
            if (lane < kRep) st_agent(ready + (unsigned)lane * RT + slot, t + 1u);
        }
        return;
    }
    // -------------------------------------------------------------------- consumer wave
    const unsigned ngroups = ntiles / kGroup, gpg = kTilesPerGenome / kGroup;   // groups per genome
    unsigned genome = 0;
    for (unsigned gi = (unsigned)wave;; gi += kCons * GPI) {
        // genome boundary for this wave: the waves meet, write the row slice, clear the table
        const unsigned gnext = gi < ngroups ? gi / gpg : ntiles / kTilesPerGenome;
        while (genome < gnext) {
            unsigned spins = 0;
            if (lane == 0) atomicAdd(&meet, 1u);   // (two meets per genome: 2 kCons arrivals)
            while (__hip_atomic_load(&meet, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (2u * genome + 1u) * kCons) {
                if (++spins > kSpinMax || ld_agent(timeout)) {
                    if (lane == 0) st_agent(timeout, 2u);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            // row slice: bins of bucket b of this genome, 256 KB; this wave's share
            uint4* row = reinterpret_cast<uint4*>(rows + ((size_t)genome * kB + b) * 65536u);
            for (int i = wave * 64 + lane; i < 16384; i += kCons * 64) {
                const uint32_t w0 = table[2 * i], w1 = table[2 * i + 1];
                row[i] = make_uint4(w0 & 0xFFFFu, w0 >> 16, w1 & 0xFFFFu, w1 >> 16);
            }
            // every wave has read the whole table before anyone clears it: meet again
            if (lane == 0) atomicAdd(&meet, 1u);
            spins = 0;
            while (__hip_atomic_load(&meet, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (2u * genome + 2u) * kCons) {
                if (++spins > kSpinMax || ld_agent(timeout)) {
                    if (lane == 0) st_agent(timeout, 3u);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            for (int i = wave * 64 + lane; i < 32768; i += kCons * 64) table[i] = 0u;
            ++genome;
        }
        if (gi >= ngroups) break;
        // GPI groups gi, gi + NC, ...: lane i polls tile i of each, then loads their segments
        unsigned slot[GPI], tl[GPI];
#pragma unroll
        for (int q = 0; q < GPI; ++q) {
            tl[q] = (gi + (unsigned)(q * kCons)) * kGroup + (unsigned)lane;
            slot[q] = tl[q] % RT;
        }
        unsigned spins = 0;
        for (;;) {
            if (lds_adds & 2) break;   // mode 2: no hand-off protocol at all (the data movement alone)
            bool ok = true;
#pragma unroll
            for (int q = 0; q < GPI; ++q) ok = ok && ld_agent(ready + (b % kRep) * RT + slot[q]) == tl[q] + 1u;
            if (__all(ok)) break;
            if (++spins > kSpinMax || ld_agent(timeout)) {
                if (lane == 0) st_agent(timeout, 4u);
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        u32x4 sv[GPI][8];
#pragma unroll
        for (int q = 0; q < GPI; ++q) {
            const int off = (int)(slot[q] * (unsigned)kSlotBytes + b * (unsigned)kSegBytes);
#pragma unroll
            for (int k = 0; k < 8; ++k) sv[q][k] = __builtin_amdgcn_raw_buffer_load_b128(ring_rsrc, off + 16 * k, 0, 16);
        }
#pragma unroll
        for (int q = 0; q < GPI; ++q) {
            if (lds_adds & 1) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t w[4] = {sv[q][k].x, sv[q][k].y, sv[q][k].z, sv[q][k].w};
#pragma unroll
                    for (int h = 0; h < 8; ++h) {
                        const uint32_t x = (w[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
                        atomicAdd(&table[x >> 1], 1u << (16 * (x & 1u)));
                    }
                }
            } else {
                uint32_t acc = 0u;
#pragma unroll
                for (int k = 0; k < 8; ++k) acc ^= sv[q][k].x ^ sv[q][k].w;
                if (acc == 0x9E3779B9u) table[lane] = acc;
            }
        }
        // progress: this wave is done with every tile before its next round
        if (lane == 0) st_agent(progress + b * kCons + wave, (gi + kCons * GPI) * kGroup);
    }
    if (lane == 0) st_agent(progress + b * kCons + wave, 0xFFFFFFFFu);
}

int main(int argc, char** argv) {
    const int G = argc > 1 ? atoi(argv[1]) : 8;
    const int ring_mib = argc > 2 ? atoi(argv[2]) : 64;
    const int lds_adds = argc > 3 ? atoi(argv[3]) : 1;
    const int reps = argc > 4 ? atoi(argv[4]) : 3;
    const char* shape = argc > 5 ? argv[5] : "4x1";   // consumer waves x groups per round
    const unsigned RT = (unsigned)((size_t)ring_mib * 1024 * 1024 / kSlotBytes);
    const unsigned ntiles = (unsigned)G * kTilesPerGenome;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    if (ncu != kB) {
        printf("{\"error\": \"needs %d CUs (one bucket per CU), device has %d\"}\n", kB, ncu);
        return 2;
    }
    uint8_t *bases, *ring;
    unsigned *ready, *progress, *timeout;
    uint32_t* rows;
    if (hipMalloc(&bases, (size_t)ntiles * kTileWin) || hipMalloc(&ring, (size_t)RT * kSlotBytes) ||
        hipMalloc(&ready, (size_t)RT * 4 * kRep) || hipMalloc(&progress, kB * 16 * 4) || hipMalloc(&timeout, 256) ||
        hipMalloc(&rows, (size_t)G * kB * 65536 * 4)) {
        printf("{\"error\": \"alloc failed\"}\n");
        return 1;
    }
    (void)hipMemset(bases, 0x41, (size_t)ntiles * kTileWin);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ms;
    unsigned tmo = 0;
    for (int r = 0; r < reps + 1 && !tmo; ++r) {
        (void)hipMemset(ready, 0, (size_t)RT * 4 * kRep);
        (void)hipMemset(progress, 0, kB * 16 * 4);
        (void)hipMemset(timeout, 0, 256);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, 0);
        auto k = &k_ring<4, 1>;
        if (!strcmp(shape, "4x2")) k = &k_ring<4, 2>;
        if (!strcmp(shape, "8x1")) k = &k_ring<8, 1>;
        if (!strcmp(shape, "8x2")) k = &k_ring<8, 2>;
        if (!strcmp(shape, "12x2")) k = &k_ring<12, 2>;
        hipLaunchKernelGGL(k, dim3(kB), dim3(1024), 0, 0, bases, ring, RT, ntiles, ready, progress, timeout, rows,
                           lds_adds);
        (void)hipEventRecord(e1, 0);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("{\"error\": \"kernel failed\"}\n");
            return 3;
        }
        (void)hipMemcpy(&tmo, timeout, 4, hipMemcpyDeviceToHost);
        float f = 0.f;
        (void)hipEventElapsedTime(&f, e0, e1);
        if (r) ms.push_back(f);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms.empty() ? 0.0 : ms[ms.size() / 2];
    printf("{\"shape\": \"%s\", \"genomes\": %d, \"ring_MiB\": %d, \"ring_tiles\": %u, \"lds_adds\": %d, \"timeout\": %u, "
           "\"ms\": %.4f, \"us_per_genome\": %.2f, \"bases_per_genome\": %d, "
           "\"hbm_algorithmic_MB_per_genome\": %.1f, \"ring_MB_each_way_per_genome\": %.1f}\n",
           shape, G, ring_mib, RT, lds_adds, tmo, med, med * 1000.0 / G, kTilesPerGenome * kTileWin,
           (kTilesPerGenome * (double)kTileWin + kB * 65536.0 * 4) / 1e6, kTilesPerGenome * (double)kSlotBytes / 1e6);
    return tmo ? 4 : 0;
}
