// Native self-test of libkmerhip.so through the C ABI only (no torch, no Python):
// synthetic genomes on the device, dense counts for several k, row sums checked.
// Build: make selftest   Run: kmer-ml_amd/csrc/build/kmh_selftest
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../include/kmerhip.h"

#define CHECK(x)                                                                  \
    do {                                                                          \
        int rc_ = (x);                                                            \
        if (rc_ != 0) {                                                           \
            fprintf(stderr, "FAIL %s -> %d: %s\n", #x, rc_, kmh_last_error(ctx)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main(int argc, char** argv) {
    const uint64_t L = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000;
    const int G = argc > 2 ? atoi(argv[2]) : 2;
    kmh_ctx* ctx = nullptr;
    printf("version %s\n", kmh_version());
    fflush(stdout);
    CHECK(kmh_ctx_create(0, &ctx));
    printf("ctx ok\n");
    fflush(stdout);
    uint8_t* d_seq = nullptr;
    if (hipMalloc(&d_seq, L * G) != hipSuccess) return 2;
    CHECK(kmh_synth_dev(ctx, d_seq, L, L, G, 0x6B6D65724D4C0000ull, nullptr));
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    printf("synth ok\n");
    fflush(stdout);
    std::vector<uint64_t> off(G + 1);
    for (int g = 0; g <= G; ++g) off[g] = (uint64_t)g * L;
    for (int k : {1, 4, 8, 9, 10, 12}) {
        const size_t bins = (size_t)1 << (2 * k);
        uint32_t* d_out = nullptr;
        if (hipMalloc(&d_out, bins * G * 4) != hipSuccess) return 4;
        CHECK(kmh_count_dense_dev(ctx, d_seq, off.data(), G, k, d_out, nullptr));
        std::vector<uint32_t> h(bins * G);
        if (hipMemcpy(h.data(), d_out, bins * G * 4, hipMemcpyDeviceToHost) != hipSuccess) return 5;
        for (int g = 0; g < G; ++g) {
            uint64_t s = 0;
            for (size_t i = 0; i < bins; ++i) s += h[g * bins + i];
            printf("k=%d genome=%d sum=%llu expect=%llu %s\n", k, g, (unsigned long long)s,
                   (unsigned long long)(L - k + 1), s == L - k + 1 ? "OK" : "BAD");
        }
        fflush(stdout);
        (void)hipFree(d_out);
    }
    kmh_kmers* r = nullptr;
    std::vector<uint8_t> hseq(L);
    if (hipMemcpy(hseq.data(), d_seq, L, hipMemcpyDeviceToHost) != hipSuccess) return 6;
    CHECK(kmh_count_host(ctx, hseq.data(), L, 21, 0, &r));
    printf("k=21 distinct=%llu\n", (unsigned long long)kmh_kmers_size(r));
    kmh_kmers_free(r);
    CHECK(kmh_count_host(ctx, hseq.data(), L, 12, 0, &r));
    printf("k=12 host distinct=%llu\n", (unsigned long long)kmh_kmers_size(r));
    kmh_kmers_free(r);
    kmh_ctx_destroy(ctx);
    printf("selftest done\n");
    return 0;
}
