// Fabric / Infinity-Cache microbenchmark for the k = 12 exchange (partition -> count).
// Question: does an exchange buffer that stays resident in the 256 MiB Infinity Cache
// (written, then read back soon after, overwritten in place) cost HBM bandwidth, and what do
// reads and writes reach when they run concurrently?  Every number is GB/s of bytes moved
// by the kernel (sum of reads and writes), HIP events, best of 5.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Role split inside one launch: blocks with (blockIdx % 8) < nr8 read, the others write
// (every XCD gets the same mix).  Reads: src[0, nr) streamed.  Writes: dst[(i) % ring].
__global__ __launch_bounds__(256) void k_mix(const uint4* __restrict__ src, size_t nr,
                                             uint4* __restrict__ dst, size_t nw, size_t ring,
                                             int nr8, int nt, uint32_t* sink) {
    const int x = blockIdx.x % 8;
    const bool reader = x < nr8;
    const size_t nblk = gridDim.x / 8;             // blocks per XCD slot
    const size_t rblk = nblk * (size_t)nr8, wblk = nblk * (size_t)(8 - nr8);
    const size_t myb = (blockIdx.x / 8) * (size_t)(reader ? nr8 : (8 - nr8)) + (reader ? x : x - nr8);
    if (reader) {
        uint32_t acc = 0;
        const size_t stride = rblk * 256;
        size_t i = myb * 256 + threadIdx.x;
        for (; i + 3 * stride < nr; i += 4 * stride) {
            const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
            acc ^= a.x ^ b.y ^ c.z ^ d.w;
        }
        for (; i < nr; i += stride) acc ^= src[i].x;
        if (acc == 0x9E3779B9u) *sink = acc;
    } else {
        const size_t stride = wblk * 256;
        for (size_t i = myb * 256 + threadIdx.x; i < nw; i += stride) {
            size_t j = i;
            if (j >= ring) j %= ring;
            const uint4 v = make_uint4((uint32_t)i, (uint32_t)(i >> 32), 7u, 9u);
            if (nt == 1) {
                u32x4 q = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(dst + j));
            } else if (nt == 2) {
                u32x4 q = {v.x, v.y, v.z, v.w};
                asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst + j), "v"(q) : "memory");
            } else {
                dst[j] = v;
            }
        }
    }
}

static hipEvent_t e0, e1;

static float timeit(const uint4* src, size_t nr, uint4* dst, size_t nw, size_t ring, int nr8, int nt,
                    uint32_t* sink, int grid = 256 * 8 * 2) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, src, nr, dst, nw, ring, nr8, nt, sink);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
    }
    return best;
}

int main() {
    const size_t GB = (size_t)1 << 30, MB = (size_t)1 << 20;
    uint4 *big, *big2, *ring;
    uint32_t* sink;
    if (hipMalloc(&big, 4 * GB) || hipMalloc(&big2, 4 * GB) || hipMalloc(&ring, 512 * MB) ||
        hipMalloc(&sink, 64)) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(big, 1, 4 * GB);
    (void)hipMemset(big2, 2, 4 * GB);
    (void)hipMemset(ring, 3, 512 * MB);
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipDeviceSynchronize();
    const size_t n2g = 2 * GB / 16;

    // 1. pure streams
    float t = timeit(big, n2g, nullptr, 0, 1, 8, 0, sink);
    printf("read 2 GB (HBM)                         %7.3f ms %7.0f GB/s\n", t, 2.0 * GB / (t * 1e-3) / 1e9);
    for (int nt = 0; nt < 2; ++nt) {
        t = timeit(nullptr, 0, big2, n2g, (size_t)-1, 0, nt, sink);
        printf("write 2 GB fresh (HBM) nt=%d              %7.3f ms %7.0f GB/s\n", nt, t, 2.0 * GB / (t * 1e-3) / 1e9);
    }
    // 2. writes into a ring of S MB (resident?), steady state
    for (size_t S : {16, 64, 128, 192, 256, 512}) {
        for (int nt = 0; nt < 2; ++nt) {
            t = timeit(nullptr, 0, ring, n2g, S * MB / 16, 0, nt, sink);
            printf("write 2 GB into %3zu MB ring nt=%d         %7.3f ms %7.0f GB/s\n", S, nt, t, 2.0 * GB / (t * 1e-3) / 1e9);
        }
    }
    // 2b. plain writes into larger rings (HBM write rate vs footprint)
    for (size_t S : {768, 1024, 1536, 2048, 3072, 4096}) {
        t = timeit(nullptr, 0, big2, n2g, S * MB / 16, 0, 0, sink);
        printf("write 2 GB into %4zu MB ring             %7.3f ms %7.0f GB/s\n", S, t, 2.0 * GB / (t * 1e-3) / 1e9);
    }
    // 2c. reads of 2 GB at different offsets / from the second buffer
    t = timeit(big + n2g, n2g, nullptr, 0, 1, 8, 0, sink);
    printf("read 2 GB (HBM, upper half)             %7.3f ms %7.0f GB/s\n", t, 2.0 * GB / (t * 1e-3) / 1e9);
    t = timeit(big, 2 * n2g, nullptr, 0, 1, 8, 0, sink);
    printf("read 4 GB (HBM)                         %7.3f ms %7.0f GB/s\n", t, 4.0 * GB / (t * 1e-3) / 1e9);
    // 2d. sc1 (write-through) stores into small rings
    for (size_t S : {16, 64, 128}) {
        t = timeit(nullptr, 0, ring, n2g, S * MB / 16, 0, 2, sink);
        printf("write 2 GB into %3zu MB ring sc1          %7.3f ms %7.0f GB/s\n", S, t, 2.0 * GB / (t * 1e-3) / 1e9);
    }
    // 3. read back a just-written S MB region (repeated write S / read S)
    for (size_t S : {64, 128, 192, 256, 512}) {
        const size_t n = S * MB / 16;
        float tw = 1e30f, tr = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_mix, dim3(4096), dim3(256), 0, 0, nullptr, 0, ring, n, n, 0, 0, sink);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float a;
            (void)hipEventElapsedTime(&a, e0, e1);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_mix, dim3(4096), dim3(256), 0, 0, ring, n, nullptr, 0, 1, 8, 0, sink);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float b;
            (void)hipEventElapsedTime(&b, e0, e1);
            if (rep) { tw = std::min(tw, a); tr = std::min(tr, b); }
        }
        printf("ring %3zu MB: write %7.0f GB/s, read-back %7.0f GB/s\n", S, S * MB / (tw * 1e-3) / 1e9,
               S * MB / (tr * 1e-3) / 1e9);
    }
    // 4. concurrent read (HBM stream) + write: fresh HBM vs a 64 / 128 MB ring; mixes of
    //    reader:writer blocks 2:6, 4:4, 6:2 with the bytes in the same ratio
    for (int nr8 : {2, 4, 6}) {
        const size_t nr = n2g * nr8 / 8, nw = n2g * (8 - nr8) / 8;
        const double bytes = 2.0 * GB;
        t = timeit(big, nr, big2, nw, (size_t)-1, nr8, 0, sink);
        printf("mix r%d:w%d fresh HBM                     %7.3f ms %7.0f GB/s\n", nr8, 8 - nr8, t, bytes / (t * 1e-3) / 1e9);
        t = timeit(big, nr, big2, nw, (size_t)-1, nr8, 1, sink);
        printf("mix r%d:w%d fresh HBM nt                  %7.3f ms %7.0f GB/s\n", nr8, 8 - nr8, t, bytes / (t * 1e-3) / 1e9);
        for (size_t S : {32, 64, 128}) {
            t = timeit(big, nr, ring, nw, S * MB / 16, nr8, 0, sink);
            printf("mix r%d:w%d ring %3zu MB                  %7.3f ms %7.0f GB/s\n", nr8, 8 - nr8, S, t, bytes / (t * 1e-3) / 1e9);
        }
    }
    return 0;
}
