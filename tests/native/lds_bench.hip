// LDS throughput microbenchmark for the histogram regime of kmh_dense.hip: one 1024-thread
// workgroup per CU (128 KiB table), 16 operations per thread per iteration.
// Prints LDS lane-operations per second per CU for each access pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int T = 1024, BINS = 32768, ITERS = 256;

template <int MODE>
__global__ __launch_bounds__(T) void k_lds(uint32_t* out, uint32_t seed) {
    __shared__ uint32_t tbl[BINS];
    for (int i = threadIdx.x; i < BINS; i += T) tbl[i] = 0;
    __syncthreads();
    uint32_t r[16];
    uint32_t x = (threadIdx.x + 1) * 2654435761u ^ seed ^ blockIdx.x * 97u;
#pragma unroll
    for (int j = 0; j < 16; ++j) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; r[j] = x; }
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t a;
            if (MODE == 2) a = (threadIdx.x + (uint32_t)(it * 16 + j) * T) & (BINS - 1);           // conflict-free
            else if (MODE == 4 || MODE == 11) a = (((r[j] + it * 7919u) >> 5) << 5 | (lane & 31)) & (BINS - 1);  // one bank per lane
            else a = (r[j] + it * 7919u) & (BINS - 1);                                             // random
            if (MODE == 0 || MODE == 2 || MODE == 4) atomicAdd(&tbl[a], 1u);
            else if (MODE == 1 || MODE == 11) acc += atomicAdd(&tbl[a], 1u);
            else if (MODE == 3) reinterpret_cast<uint16_t*>(tbl)[a * 2 + (j & 1)] = (uint16_t)it;
            else if (MODE == 5) acc += tbl[a];
            else if (MODE == 6) acc += atomicCAS(&tbl[a], 0u, r[j]);                     // cas b32, mostly fails
            else if (MODE == 7) acc += atomicCAS(&tbl[a], tbl[a], r[j]);                 // cas b32, mostly succeeds
            else if (MODE == 8) {
                unsigned long long* t64 = reinterpret_cast<unsigned long long*>(tbl);
                acc += (uint32_t)atomicCAS(&t64[a >> 1], 0ull, (unsigned long long)r[j]);  // cas b64
            } else if (MODE == 9) {
                unsigned long long* t64 = reinterpret_cast<unsigned long long*>(tbl);
                atomicAdd(&t64[a >> 1], 1ull);                                           // add u64, no return
            } else if (MODE == 10) {
                unsigned long long* t64 = reinterpret_cast<unsigned long long*>(tbl);
                acc += (uint32_t)t64[a >> 1];                                            // read b64
            }
        }
    }
    __syncthreads();
    uint32_t s = acc;
    for (int i = threadIdx.x; i < BINS; i += T) s += tbl[i];
    atomicAdd(out, s);
}

template <int MODE>
double run(const char* name, int nblocks) {
    uint32_t* d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_lds<MODE>, dim3(nblocks), dim3(T), 0, 0, d, 1u);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_lds<MODE>, dim3(nblocks), dim3(T), 0, 0, d, 7u + rep);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    const double ops = (double)nblocks * T * ITERS * 16;
    const double per_cu = ops / (best * 1e-3) / 256.0;
    printf("%-28s %8.3f ms  %7.2f Gop/s/CU  (%.2f lane-ops/clk/CU at 2.1 GHz)\n", name, best,
           per_cu / 1e9, per_cu / 2.1e9);
    (void)hipFree(d);
    return per_cu;
}

int main() {
    const int nb = 256 * 4;
    run<0>("ds_add random", nb);
    run<1>("ds_add_rtn random", nb);
    run<2>("ds_add conflict-free", nb);
    run<4>("ds_add bank-per-lane", nb);
    run<3>("ds_write_b16 random", nb);
    run<5>("ds_read_b32 random", nb);
    run<6>("ds_cmpst_rtn_b32 (fail)", nb);
    run<7>("ds_cmpst_rtn_b32 (success)", nb);
    run<8>("ds_cmpst_rtn_b64", nb);
    run<9>("ds_add_u64", nb);
    run<10>("ds_read_b64 random", nb);
    run<11>("ds_add_rtn bank-per-lane", nb);
    return 0;
}
