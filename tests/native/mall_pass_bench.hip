// Microbenchmark of the k = 12 exchange pattern, memory traffic only (no LDS work): per genome,
// a "partition" kernel streams the genome's 100 MB of bases and writes X MB of exchange, then
// a "count" kernel reads the X MB back and writes the genome's row bytes.  Compared:
//   A  one pass per genome, the exchange in a fresh 4 GB region per batch of 18 genomes
//      (round 1's layout: HBM round trip);
//   B  two passes per genome over bucket halves: each pass re-reads the genome (the second
//      time from the Infinity Cache) and writes / reads half the exchange into ONE reused
//      buffer (resident in the 256 MiB Infinity Cache).
// Prints ms per genome for each phase and in total.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>

__global__ __launch_bounds__(256) void k_part(const uint4* __restrict__ g, size_t ng, uint4* __restrict__ x,
                                              size_t nx, uint32_t* sink) {
    // read ng chunks, write nx chunks (nx ~ 2 ng or ng): each thread interleaves its share
    const size_t stride = (size_t)gridDim.x * blockDim.x, t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (size_t i = t; i < ng; i += stride) {
        const uint4 v = g[i];
        acc ^= v.x ^ v.w;
    }
    for (size_t i = t; i < nx; i += stride) x[i] = make_uint4((uint32_t)i, acc, 1u, 2u);
    if (acc == 0x9E3779B9u) *sink = acc;
}

__global__ __launch_bounds__(256) void k_count(const uint4* __restrict__ x, size_t nx, uint4* __restrict__ row,
                                               size_t nrow, uint32_t* sink) {
    const size_t stride = (size_t)gridDim.x * blockDim.x, t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (size_t i = t; i < nx; i += stride) {
        const uint4 v = x[i];
        acc ^= v.x ^ v.w;
    }
    for (size_t i = t; i < nrow; i += stride) row[i] = make_uint4((uint32_t)i, acc, 3u, 4u);
    if (acc == 0x9E3779B9u) *sink = acc;
}

int main() {
    const size_t MB = (size_t)1 << 20;
    const int G = 36;
    const size_t L = 100'000'000, X = 211'000'000, ROW = 64 * MB;
    uint4 *gen, *xa, *xb, *rows;
    uint32_t* sink;
    if (hipMalloc(&gen, (size_t)G * L) || hipMalloc(&xa, 18 * X) || hipMalloc(&xb, X) ||
        hipMalloc(&rows, (size_t)G * ROW) || hipMalloc(&sink, 64)) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(gen, 1, (size_t)G * L);
    (void)hipMemset(xa, 2, 18 * X);
    (void)hipMemset(rows, 3, (size_t)G * ROW);
    hipEvent_t e[5];
    for (auto& q : e) (void)hipEventCreate(&q);
    const int grid = 256 * 8;
    auto ms = [&](hipEvent_t a, hipEvent_t b) {
        float f;
        (void)hipEventElapsedTime(&f, a, b);
        return f;
    };
    for (int rep = 0; rep < 3; ++rep) {
        // A: batches of 18 genomes, exchange per batch in xa (18 x 211 MB)
        float pa = 0, ca = 0;
        for (int b0 = 0; b0 < G; b0 += 18) {
            (void)hipEventRecord(e[0]);
            for (int g = b0; g < b0 + 18; ++g)
                hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, gen + (size_t)g * L / 16, L / 16,
                                   xa + (size_t)(g - b0) * X / 16, X / 16, sink);
            (void)hipEventRecord(e[1]);
            for (int g = b0; g < b0 + 18; ++g)
                hipLaunchKernelGGL(k_count, dim3(grid), dim3(256), 0, 0, xa + (size_t)(g - b0) * X / 16, X / 16,
                                   rows + (size_t)g * ROW / 16, ROW / 16, sink);
            (void)hipEventRecord(e[2]);
            (void)hipEventSynchronize(e[2]);
            pa += ms(e[0], e[1]);
            ca += ms(e[1], e[2]);
        }
        // B: per genome two passes of half the exchange through one resident buffer
        float pb = 0, cb = 0;
        for (int g = 0; g < G; ++g) {
            for (int h = 0; h < 2; ++h) {
                (void)hipEventRecord(e[0]);
                hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, gen + (size_t)g * L / 16, L / 16, xb,
                                   X / 32, sink);
                (void)hipEventRecord(e[1]);
                hipLaunchKernelGGL(k_count, dim3(grid), dim3(256), 0, 0, xb, X / 32,
                                   rows + ((size_t)g * ROW + h * ROW / 2) / 16, ROW / 32, sink);
                (void)hipEventRecord(e[2]);
                (void)hipEventSynchronize(e[2]);
                pb += ms(e[0], e[1]);
                cb += ms(e[1], e[2]);
            }
        }
        // B without events between the launches (launch gaps included, as in a real step)
        (void)hipEventRecord(e[3]);
        for (int g = 0; g < G; ++g)
            for (int h = 0; h < 2; ++h) {
                hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, gen + (size_t)g * L / 16, L / 16, xb,
                                   X / 32, sink);
                hipLaunchKernelGGL(k_count, dim3(grid), dim3(256), 0, 0, xb, X / 32,
                                   rows + ((size_t)g * ROW + h * ROW / 2) / 16, ROW / 32, sink);
            }
        (void)hipEventRecord(e[4]);
        (void)hipEventSynchronize(e[4]);
        const float bb = ms(e[3], e[4]);
        // C: one pass per genome, the whole exchange through ONE reused buffer (211 MB: resident
        // in the Infinity Cache between the partition and the count of the same genome)
        (void)hipEventRecord(e[3]);
        for (int g = 0; g < G; ++g) {
            hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, gen + (size_t)g * L / 16, L / 16, xb,
                               X / 16, sink);
            hipLaunchKernelGGL(k_count, dim3(grid), dim3(256), 0, 0, xb, X / 16, rows + (size_t)g * ROW / 16,
                               ROW / 16, sink);
        }
        (void)hipEventRecord(e[4]);
        (void)hipEventSynchronize(e[4]);
        const float cc = ms(e[3], e[4]);
        // D: as A but without events between the launches
        (void)hipEventRecord(e[3]);
        for (int b0 = 0; b0 < G; b0 += 18) {
            for (int g = b0; g < b0 + 18; ++g)
                hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, gen + (size_t)g * L / 16, L / 16,
                                   xa + (size_t)(g - b0) * X / 16, X / 16, sink);
            for (int g = b0; g < b0 + 18; ++g)
                hipLaunchKernelGGL(k_count, dim3(grid), dim3(256), 0, 0, xa + (size_t)(g - b0) * X / 16, X / 16,
                                   rows + (size_t)g * ROW / 16, ROW / 16, sink);
        }
        (void)hipEventRecord(e[4]);
        (void)hipEventSynchronize(e[4]);
        const float dd = ms(e[3], e[4]);
        // E: batches of gb genomes through an exchange region of gb x 211 MB that every batch
        //    reuses (a small address footprint for the exchange writes)
        for (int gb : {1, 2, 4, 8}) {
            (void)hipEventRecord(e[3]);
            for (int b0 = 0; b0 < G; b0 += gb) {
                for (int g = b0; g < b0 + gb && g < G; ++g)
                    hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, gen + (size_t)g * L / 16, L / 16,
                                       xa + (size_t)(g - b0) * X / 16, X / 16, sink);
                for (int g = b0; g < b0 + gb && g < G; ++g)
                    hipLaunchKernelGGL(k_count, dim3(grid), dim3(256), 0, 0, xa + (size_t)(g - b0) * X / 16,
                                       X / 16, rows + (size_t)g * ROW / 16, ROW / 16, sink);
            }
            (void)hipEventRecord(e[4]);
            (void)hipEventSynchronize(e[4]);
            printf("rep %d  E(batch %d, exchange region %d MB): %.1f us/genome\n", rep, gb, (int)(gb * X >> 20),
                   ms(e[3], e[4]) * 1e3 / G);
        }
        printf("rep %d  A: part %.1f + count %.1f us/genome = %.1f   B: part %.1f + count %.1f = %.1f us/genome"
               "   B back-to-back %.1f   C (one resident buffer) back-to-back %.1f   A back-to-back %.1f us/genome\n",
               rep, pa * 1e3 / G, ca * 1e3 / G, (pa + ca) * 1e3 / G, pb * 1e3 / G, cb * 1e3 / G,
               (pb + cb) * 1e3 / G, bb * 1e3 / G, cc * 1e3 / G, dd * 1e3 / G);
    }
    return 0;
}
