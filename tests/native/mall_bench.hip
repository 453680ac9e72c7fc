// Infinity-Cache round-trip microbenchmark: write X MB with dwordx4 stores, then read it
// back, for X from 32 MB to 1 GB, plus read-only and write-only passes over the same buffer.
// Prints effective GB/s of each phase (the k=12 partition->count exchange pattern).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_write(uint4* p, size_t n, uint32_t salt) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i ^ salt, salt, (uint32_t)(i >> 7), 3u);
}
__global__ __launch_bounds__(256) void k_read(const uint4* p, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) *sink = acc;
}

int main() {
    const size_t maxb = (size_t)1 << 30;
    uint4* buf;
    uint32_t* sink;
    uint4* scrub;
    (void)hipMalloc(&buf, maxb);
    (void)hipMalloc(&sink, 4);
    (void)hipMalloc(&scrub, maxb);
    hipEvent_t e0, e1, e2;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventCreate(&e2);
    const int grid = 256 * 8;
    printf("%8s %12s %12s\n", "MB", "write GB/s", "read-after-write GB/s");
    for (size_t mb : {32, 64, 128, 192, 256, 384, 512, 1024}) {
        const size_t n = (mb << 20) / 16;
        float bw = 0, br = 0;
        for (int rep = 0; rep < 4; ++rep) {
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, scrub, maxb / 16, 7u);  // evict
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, buf, n, (uint32_t)rep);
            (void)hipEventRecord(e1);
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, buf, n, sink);
            (void)hipEventRecord(e2);
            (void)hipEventSynchronize(e2);
            float tw, tr;
            (void)hipEventElapsedTime(&tw, e0, e1);
            (void)hipEventElapsedTime(&tr, e1, e2);
            if (rep) { bw += (mb << 20) / (tw * 1e-3) / 1e9 / 3; br += (mb << 20) / (tr * 1e-3) / 1e9 / 3; }
        }
        printf("%8zu %12.0f %12.0f\n", mb, bw, br);
    }
    return 0;
}
