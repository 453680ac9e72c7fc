// Issue rate of the 32-bit integer multiplies on gfx950 (which form bin_of / pass_of should use):
// 8 independent chains per lane of 4096 dependent ops each, 1024 workgroups of 256 threads;
// prints ns per wave-instruction-per-SIMD for v_mul_lo_u32, v_mul_hi_u32, v_mul_u32_u24,
// v_mul_hi_u32_u24 and v_add_u32.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t m) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 2654435761u + i;
    for (int it = 0; it < 4096; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            else if constexpr (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            else if constexpr (OP == 2) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            else asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
float run(uint32_t* d) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<OP><<<1024, 256>>>(d, 0x9E3779B1u);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<OP><<<1024, 256>>>(d, 0x9E3779B1u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    uint32_t* d;
    if (hipMalloc(&d, 1024 * 256 * 4) != hipSuccess) return 1;
    // wave-instructions per SIMD: 1024 WGs * 4 waves / 1024 SIMDs * 4096 * 8
    const double wi = 1024.0 * 4 / 1024 * 4096 * 8;
    const char* names[] = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "-", "v_add_u32"};
    float t[5];
    t[0] = run<0>(d);
    t[1] = run<1>(d);
    t[2] = run<2>(d);
    t[4] = run<4>(d);
    for (int i : {0, 1, 2, 4}) printf("%-20s %8.3f ms  %6.3f ns per wave-instruction per SIMD\n", names[i], t[i], t[i] * 1e6 / wi);
    (void)hipFree(d);
    return 0;
}
