// cas_chain.hip -- latency of a dependent chain of LDS operations per wave, the shape of the
// k_sp_count insert loop (kmh_hash.hip): every lane issues one operation on a pseudo-random
// slot of a 16384-slot u64 table, waits for its result and derives the next slot from it.
// Prints cycles per iteration (s_memtime, shader clock) for T threads per workgroup, one
// workgroup per CU.  Not part of the product; DESIGN.md 2b cites its output.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kSlots = 16384;
constexpr int kIter = 4096;

// MODE 0: ds_cmpst_rtn_b64 (CAS(0 -> v): the table fills, so most probes fail as in a
//         half-full hash table); 1: ds_read_b64; 2: ds_add_rtn_u64; 3: ds_cmpst_rtn_b32.
template <int MODE, int T>
__global__ __launch_bounds__(T) void k_chain(unsigned long long* out, uint32_t seed) {
    __shared__ unsigned long long tbl[kSlots];
    for (int i = threadIdx.x; i < kSlots; i += T) tbl[i] = 0ull;
    __syncthreads();
    uint32_t s = (threadIdx.x * 2654435761u + seed) & (kSlots - 1);
    unsigned long long acc = 0;
    const unsigned long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
        unsigned long long v;
        const unsigned long long mine = ((unsigned long long)(s ^ i) << 32) | 1ull;
        if (MODE == 0) v = atomicCAS(&tbl[s], 0ull, mine);
        else if (MODE == 1) v = tbl[s];
        else if (MODE == 2) v = atomicAdd(&tbl[s], 1ull);
        else v = atomicCAS(reinterpret_cast<unsigned int*>(tbl) + s, 0u, (unsigned)mine);
        acc += v;
        s = ((uint32_t)v * 0x9E3779B1u + (uint32_t)(v >> 32) + s * 2654435761u + (uint32_t)i) >> 18;
    }
    const unsigned long long t1 = clock64();
    if ((threadIdx.x & 63) == 0) atomicAdd(&out[0], t1 - t0);
    if (acc == 0x1234567ull) out[1] = acc;
}

template <int MODE, int T>
void run(const char* name, int nblocks) {
    unsigned long long* d;
    hipMalloc(&d, 16);
    hipMemset(d, 0, 16);
    hipLaunchKernelGGL((k_chain<MODE, T>), dim3(nblocks), dim3(T), 0, 0, d, 1u);
    hipDeviceSynchronize();
    hipMemset(d, 0, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_chain<MODE, T>), dim3(nblocks), dim3(T), 0, 0, d, 7u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    const double waves = (double)nblocks * (T / 64);
    const double cyc = (double)h[0] / waves / kIter;
    const double lane_ops = (double)nblocks * T * kIter / (ms * 1e-3) / nblocks;
    std::printf("%-22s %4d waves/CU  %8.1f cycles/iteration/wave  %6.2f Gop/s/CU  (%.3f ms)\n", name, T / 64,
                cyc, lane_ops / 1e9, ms);
    hipFree(d);
}

int main() {
    int cu = 0;
    hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    run<0, 256>("cas_b64 chain", cu);
    run<0, 512>("cas_b64 chain", cu);
    run<0, 1024>("cas_b64 chain", cu);
    run<1, 1024>("read_b64 chain", cu);
    run<2, 1024>("add_rtn_u64 chain", cu);
    run<3, 1024>("cas_b32 chain", cu);
    return 0;
}
