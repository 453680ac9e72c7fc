// kmh_api.cpp -- the C ABI of libkmerhip.so (include/kmerhip.h): contexts, device
// workspace, kernel timing, and the host-buffer counting entry points that replace the
// counting loop of /root/reference/kmerml/kmers/generate.py:36-58.
#include <string.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "kmh_internal.h"

struct kmh_ctx : kmh::Ctx {};

struct kmh_kmers {
    std::vector<uint64_t> codes;   // first-occurrence order
    std::vector<uint32_t> counts;
    std::vector<uint64_t> first;
};

namespace kmh {

namespace {
thread_local std::string t_err;
}

void set_thread_error(const std::string& msg) { t_err = msg; }

int fail(Ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    else t_err = msg;
    return code;
}

int hip_fail(Ctx* ctx, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(ctx, e == hipErrorOutOfMemory ? KMH_ERR_NOMEM : KMH_ERR_HIP, m);
}

int ensure(Ctx* ctx, DevBuf& b, size_t bytes) {
    if (bytes <= b.bytes) return KMH_OK;
    if (b.ptr) {
        // the buffer may still be read by queued work on the context stream
        KMH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        KMH_HIP(ctx, hipDeviceSynchronize());
        KMH_HIP(ctx, hipFree(b.ptr));
        b.ptr = nullptr;
        b.bytes = 0;
    }
    const size_t sz = std::max<size_t>(bytes, 4096);
    KMH_HIP(ctx, hipMalloc(&b.ptr, sz));
    b.bytes = sz;
    return KMH_OK;
}

int drop(Ctx* ctx, DevBuf& b) {
    if (!b.ptr) return KMH_OK;
    KMH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    KMH_HIP(ctx, hipDeviceSynchronize());
    KMH_HIP(ctx, hipFree(b.ptr));
    if (&b == &ctx->seq) ctx->staged_ok = false;
    if (&b == &ctx->meta) ctx->meta_cache.clear();
    b.ptr = nullptr;
    b.bytes = 0;
    return KMH_OK;
}

int upload(Ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (ctx->pinned_ready) KMH_HIP(ctx, hipEventSynchronize(ctx->pinned_ready));
    if (bytes > ctx->pinned_bytes) {
        if (ctx->pinned) KMH_HIP(ctx, hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        const size_t sz = std::max<size_t>(bytes, 1 << 16);
        KMH_HIP(ctx, hipHostMalloc(&ctx->pinned, sz, hipHostMallocDefault));
        ctx->pinned_bytes = sz;
    }
    memcpy(ctx->pinned, src, bytes);
    KMH_HIP(ctx, hipMemcpyAsync(dst, ctx->pinned, bytes, hipMemcpyHostToDevice, s));
    if (!ctx->pinned_ready) KMH_HIP(ctx, hipEventCreateWithFlags(&ctx->pinned_ready, hipEventDisableTiming));
    KMH_HIP(ctx, hipEventRecord(ctx->pinned_ready, s));
    return KMH_OK;
}

static hipEvent_t take_event(Ctx* ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void time_begin(Ctx* ctx, hipStream_t s, const char* name) {
    if (!ctx->timing) return;
    // KMH_TIMING_ONLY=name,name: event pairs only around those kernels (each pair costs a few
    // microseconds of stream time; the bench times only the kernels its roofline names)
    ctx->timing_skip = !ctx->timing_only.empty() &&
                       ctx->timing_only.find("," + std::string(name) + ",") == std::string::npos;
    if (ctx->timing_skip) return;
    TimedLaunch t{name, take_event(ctx), take_event(ctx)};
    if (t.start) (void)hipEventRecord(t.start, s);
    ctx->launches.push_back(t);
}

void time_end(Ctx* ctx, hipStream_t s) {
    if (!ctx->timing || ctx->timing_skip || ctx->launches.empty()) return;
    TimedLaunch& t = ctx->launches.back();
    if (t.stop) (void)hipEventRecord(t.stop, s);
}

}  // namespace kmh

using kmh::fail;

// NULL means the HIP null stream (the convention of every HIP API, and the handle of
// torch's default stream); the context's own stream serves the host-buffer calls only.
static hipStream_t pick_stream(kmh_ctx*, void* stream) { return static_cast<hipStream_t>(stream); }

// Stream order of the context's workspace (one context shared by threads on different streams).
// The _dev entry points return before their kernels finish and every call reuses the context's
// cached device workspace, so a call on stream s first makes s wait for the work the previous
// call queued on another stream, then records ctx->ws_done on s once its own work is queued.
// Calls on one stream are ordered by the stream; calls on different streams run one after the
// other on the device and never share the workspace in flight (tests/test_gpu_parity.py,
// test_context_shared_by_two_streams).  Buffer growth and release synchronise the device.
template <typename F>
static int on_stream(kmh_ctx* ctx, hipStream_t s, F&& body) {
    if (ctx->ws_pending && ctx->ws_stream != s) KMH_HIP(ctx, hipStreamWaitEvent(s, ctx->ws_done, 0));
    const int rc = body(s);
    if (!ctx->ws_done) KMH_HIP(ctx, hipEventCreateWithFlags(&ctx->ws_done, hipEventDisableTiming));
    KMH_HIP(ctx, hipEventRecord(ctx->ws_done, s));
    ctx->ws_stream = s;
    ctx->ws_pending = true;
    return rc;
}

extern "C" {

const char* kmh_version(void) { return "kmerhip 0.2.0 gfx950"; }

#ifndef KMH_BUILD_ID
#define KMH_BUILD_ID "unknown"
#endif
const char* kmh_build_id(void) { return KMH_BUILD_ID; }

int kmh_ctx_create(int device, kmh_ctx** out) {
    if (!out) {
        kmh::set_thread_error("kmh_ctx_create: out is NULL");
        return KMH_ERR_INVALID;
    }
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) {
        kmh::set_thread_error(std::string("no HIP device available: ") + hipGetErrorString(e));
        return KMH_ERR_HIP;
    }
    if (device < 0 || device >= ndev) {
        kmh::set_thread_error("kmh_ctx_create: device index out of range");
        return KMH_ERR_INVALID;
    }
    std::unique_ptr<kmh_ctx> c(new (std::nothrow) kmh_ctx);
    if (!c) return KMH_ERR_NOMEM;
    c->device = device;
    if ((e = hipSetDevice(device)) != hipSuccess || (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) {
        kmh::set_thread_error(std::string("kmh_ctx_create: ") + hipGetErrorString(e));
        return KMH_ERR_HIP;
    }
    *out = c.release();
    return KMH_OK;
}

// Every cached device buffer and the pinned staging (after the queued work that may read them).
static void free_workspace(kmh_ctx* ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipDeviceSynchronize();
    auto drop = [](kmh::DevBuf& b) {
        if (b.ptr) (void)hipFree(b.ptr);
        b.ptr = nullptr;
        b.bytes = 0;
    };
    for (kmh::DevBuf* b : {&ctx->seq, &ctx->suf, &ctx->toff, &ctx->meta, &ctx->out, &ctx->out2, &ctx->fix,
                           &ctx->redo, &ctx->order, &ctx->sort_tmp, &ctx->scan_tmp, &ctx->first})
        drop(*b);
    for (auto& b : ctx->sparse) drop(b);
    for (auto& b : ctx->wire) drop(b);
    ctx->wire_valid = false;
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_bytes = 0;
    ctx->staged_ok = false;
    ctx->meta_cache.clear();
}

static uint64_t workspace_bytes(const kmh_ctx* ctx) {
    uint64_t t = ctx->pinned_bytes;
    for (const kmh::DevBuf* b : {&ctx->seq, &ctx->suf, &ctx->toff, &ctx->meta, &ctx->out, &ctx->out2, &ctx->fix,
                                 &ctx->redo, &ctx->order, &ctx->sort_tmp, &ctx->scan_tmp, &ctx->first})
        t += b->bytes;
    for (const auto& b : ctx->sparse) t += b.bytes;
    for (const auto& b : ctx->wire) t += b.bytes;
    return t;
}

int kmh_ctx_release(kmh_ctx* ctx) {
    if (!ctx) {
        kmh::set_thread_error("kmh_ctx_release: ctx is NULL");
        return KMH_ERR_INVALID;
    }
    KMH_HIP(ctx, hipSetDevice(ctx->device));
    free_workspace(ctx);
    return KMH_OK;
}

uint64_t kmh_ctx_workspace_bytes(const kmh_ctx* ctx) { return ctx ? workspace_bytes(ctx) : 0; }

int kmh_ctx_stats(const kmh_ctx* ctx, uint64_t* stats, int n) {
    if (!ctx || (n > 0 && !stats)) return KMH_ERR_INVALID;
    const uint64_t v[3] = {ctx->fb_passes, ctx->fb_groups, workspace_bytes(ctx)};
    for (int i = 0; i < n && i < 3; ++i) stats[i] = v[i];
    return 3;
}

int kmh_ctx_trim(kmh_ctx* ctx, uint64_t keep_bytes) {
    if (!ctx) {
        kmh::set_thread_error("kmh_ctx_trim: ctx is NULL");
        return KMH_ERR_INVALID;
    }
    ctx->err.clear();
    if (workspace_bytes(ctx) <= keep_bytes) return KMH_OK;
    KMH_HIP(ctx, hipSetDevice(ctx->device));
    free_workspace(ctx);
    return KMH_OK;
}

void kmh_ctx_destroy(kmh_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    free_workspace(ctx);
    if (ctx->pinned_ready) (void)hipEventDestroy(ctx->pinned_ready);
    for (auto& t : ctx->launches) {
        if (t.start) (void)hipEventDestroy(t.start);
        if (t.stop) (void)hipEventDestroy(t.stop);
    }
    for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->ws_done) (void)hipEventDestroy(ctx->ws_done);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* kmh_last_error(const kmh_ctx* ctx) {
    return ctx ? ctx->err.c_str() : kmh::t_err.c_str();
}

int kmh_timing_enable(kmh_ctx* ctx, int enable) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->timing = enable != 0;
    ctx->timing_skip = false;
    const char* only = std::getenv("KMH_TIMING_ONLY");
    ctx->timing_only = (only && *only) ? "," + std::string(only) + "," : std::string();
    for (auto& t : ctx->launches) {
        if (t.start) ctx->event_pool.push_back(t.start);
        if (t.stop) ctx->event_pool.push_back(t.stop);
    }
    ctx->launches.clear();
    return KMH_OK;
}

int kmh_timing_report(kmh_ctx* ctx, const char** names, uint64_t* launches, double* total_ms,
                      int cap) {
    if (!ctx) return KMH_ERR_INVALID;
    (void)hipSetDevice(ctx->device);
    std::map<std::string, std::pair<uint64_t, double>> acc;
    std::vector<std::string> order;
    for (auto& t : ctx->launches) {
        float ms = 0.f;
        if (t.start && t.stop) {
            if (hipEventSynchronize(t.stop) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "timing: event sync failed");
            (void)hipEventElapsedTime(&ms, t.start, t.stop);
        }
        auto it = acc.find(t.name);
        if (it == acc.end()) {
            order.push_back(t.name);
            acc[t.name] = {1, (double)ms};
        } else {
            it->second.first += 1;
            it->second.second += ms;
        }
    }
    ctx->report_names = order;
    const int n = (int)order.size();
    for (int i = 0; i < n && i < cap; ++i) {
        if (names) names[i] = ctx->report_names[i].c_str();
        if (launches) launches[i] = acc[order[i]].first;
        if (total_ms) total_ms[i] = acc[order[i]].second;
    }
    return n;
}

int kmh_count_dense_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G,
                        int k, uint32_t* d_matrix, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::dense_count(ctx, d_seq, offsets, G, k, d_matrix, s);
    });
}

int kmh_first_dense_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G,
                        int k, uint32_t* d_first, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::dense_first(ctx, d_seq, offsets, G, k, d_first, s);
    });
}

int kmh_synth_dev(kmh_ctx* ctx, uint8_t* d_seq, uint64_t len, uint64_t stride, int G,
                  uint64_t seed0, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::synth(ctx, d_seq, len, stride, G, seed0, s);
    });
}

int kmh_count_sparse_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G,
                         int k, int canonical, uint64_t* d_codes, uint32_t* d_counts,
                         uint64_t* d_nkmers, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::sparse_count_dev(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, d_nkmers,
                                 s);
    });
}

int kmh_count_sparse_sorted_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G,
                                int k, int canonical, uint64_t* d_codes, uint32_t* d_counts,
                                uint64_t* d_nrows, uint64_t* d_ndistinct, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::sparse_count_dev_sorted(ctx, d_seq, offsets, G, k, canonical, d_codes, d_counts, d_nrows,
                                            d_ndistinct, s);
    });
}

int kmh_shard_union_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R,
                        uint64_t lo_code, uint64_t hi_code_incl, uint64_t* d_columns, int64_t* d_indices,
                        uint64_t* ncols, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::shard_union(ctx, d_codes, row_off, R, lo_code, hi_code_incl, d_columns, d_indices, false, ncols, s);
    });
}

int kmh_shard_union_u32_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R,
                            uint64_t lo_code, uint64_t hi_code_incl, uint64_t* d_columns, uint32_t* d_indices,
                            uint64_t* ncols, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::shard_union(ctx, d_codes, row_off, R, lo_code, hi_code_incl, d_columns, d_indices, true, ncols, s);
    });
}

int kmh_rows_cuts_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, const uint64_t* bounds,
                      int nb, uint64_t* d_cuts, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::rows_cuts(ctx, d_codes, row_off, R, bounds, nb, d_cuts, s);
    });
}

int kmh_wire_size_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* slice_start,
                      const uint64_t* slice_n, int S, uint64_t* slice_bytes, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::wire_size(ctx, d_codes, d_counts, slice_start, slice_n, S, slice_bytes, s);
    });
}

int kmh_wire_encode_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* slice_start,
                        const uint64_t* slice_n, int S, uint8_t* d_out, uint64_t out_bytes, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::wire_encode(ctx, d_codes, d_counts, slice_start, slice_n, S, d_out, out_bytes, s);
    });
}

int kmh_wire_decode_dev(kmh_ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const uint64_t* slice_n,
                        const uint64_t* slice_bytes, const uint64_t* slice_dst, int S, uint64_t* d_codes,
                        uint32_t* d_counts, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::wire_decode(ctx, d_in, in_bytes, slice_n, slice_bytes, slice_dst, S, d_codes, d_counts, s);
    });
}

uint64_t kmh_sparse_out_offsets(const uint64_t* offsets, int G, int k, uint64_t* out_off) {
    if (!offsets || G < 0) return 0;
    return kmh::sparse_windows(offsets, G, k, out_off);
}

int kmh_rows_encode_u8_dev(kmh_ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols,
                           uint8_t* d_u8, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n,
                           void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::rows_encode_u8(ctx, d_rows, rows, cols, d_u8, d_esc, cap, d_esc_n, s);
    });
}

int kmh_rows_decode_u8_dev(kmh_ctx* ctx, const uint8_t* d_u8, uint64_t rows, uint64_t cols,
                           const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n,
                           int ranks, uint64_t rows_per_rank, uint32_t* d_rows, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::rows_decode_u8(ctx, d_u8, rows, cols, d_esc, cap, d_esc_n, ranks, rows_per_rank,
                               d_rows, s);
    });
}

int kmh_rows_encode_u4_dev(kmh_ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols,
                           uint8_t* d_u4, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n,
                           void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::rows_encode_u4(ctx, d_rows, rows, cols, d_u4, d_esc, cap, d_esc_n, s);
    });
}

int kmh_rows_decode_u4_dev(kmh_ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols,
                           const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n,
                           uint32_t* d_rows, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::rows_decode_u4(ctx, d_u4, rows, cols, d_esc, cap, d_esc_n, d_rows, s);
    });
}

int kmh_count_dense_u4_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                           uint32_t* d_matrix, uint8_t* d_u4, uint32_t* d_esc, uint32_t cap,
                           uint32_t* d_esc_n, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::dense_count_u4(ctx, d_seq, offsets, G, k, d_matrix, d_u4, d_esc, cap, d_esc_n, 1, s);
    });
}

int kmh_count_dense_u4only_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                               uint32_t* d_scratch, uint8_t* d_u4, uint32_t* d_esc, uint32_t cap,
                               uint32_t* d_esc_n, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::dense_count_u4(ctx, d_seq, offsets, G, k, d_scratch, d_u4, d_esc, cap, d_esc_n, 0, s);
    });
}

int kmh_rows_decode_u4_range_dev(kmh_ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols,
                                 const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n,
                                 uint64_t row0, uint64_t nrows, uint32_t* d_rows, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::rows_decode_u4_range(ctx, d_u4, rows, cols, d_esc, cap, d_esc_n, row0, nrows, d_rows,
                                     s);
    });
}

int kmh_feature_columns_dev(kmh_ctx* ctx, const uint64_t* d_codes, uint64_t n, int k, const int32_t* d_order,
                            const double* d_lg, int64_t* d_cnt, int64_t* d_cpg, int64_t* d_rep, double* d_gc,
                            double* d_oe, double* d_ent, void* stream) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, pick_stream(ctx, stream), [&](hipStream_t s) {
        return kmh::feature_columns(ctx, d_codes, n, k, d_order, d_lg, d_cnt, d_cpg, d_rep, d_gc, d_oe, d_ent,
                                s);
    });
}

// Host sequence -> device (padded with one non-base byte so loads past the end are safe).
static int stage_sequence(kmh_ctx* ctx, const uint8_t* seq, uint64_t n, uint8_t** d_seq) {
    ctx->staged_ok = false;
    int rc = kmh::ensure(ctx, ctx->seq, (size_t)n + 64);
    if (rc) return rc;
    uint8_t* d = static_cast<uint8_t*>(ctx->seq.ptr);
    if (n) KMH_HIP(ctx, hipMemcpyAsync(d, seq, n, hipMemcpyHostToDevice, ctx->stream));
    KMH_HIP(ctx, hipMemsetAsync(d + n, 0, 64, ctx->stream));
    *d_seq = d;
    return KMH_OK;
}

// The counting dispatch of kmh_count_host / kmh_count_staged on a sequence already in
// ctx->seq (n bytes + 64 zero bytes).
static int count_staged_impl(kmh_ctx* ctx, uint8_t* d_seq, uint64_t n, int k, int canonical, kmh_kmers** out);

int kmh_count_dense_host(kmh_ctx* ctx, const uint8_t* seq, uint64_t n, int k, uint32_t* counts) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (!counts || (n && !seq)) return fail(ctx, KMH_ERR_INVALID, "NULL argument");
    if (k < 1 || k > KMH_MAX_DENSE_K) return fail(ctx, KMH_ERR_UNSUPPORTED, "dense counting needs 1 <= k <= 12");
    if (n >= 0xFFFFFFFFull) return fail(ctx, KMH_ERR_INVALID, "sequence must be shorter than 2^32 - 1 bytes");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    const size_t bins = (size_t)1 << (2 * k);
    return on_stream(ctx, ctx->stream, [&](hipStream_t) {
        uint8_t* d_seq = nullptr;
        int rc = stage_sequence(ctx, seq, n, &d_seq);
        if (rc) return rc;
        if ((rc = kmh::ensure(ctx, ctx->out, bins * sizeof(uint32_t)))) return rc;
        const uint64_t off[2] = {0, n};
        uint32_t* d_counts = static_cast<uint32_t*>(ctx->out.ptr);
        if ((rc = kmh::dense_count(ctx, d_seq, off, 1, k, d_counts, ctx->stream))) return rc;
        KMH_HIP(ctx, hipMemcpyAsync(counts, d_counts, bins * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
        KMH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        return KMH_OK;
    });
}

// Checks of every host-buffer count call, before any byte is read or staged.
static int check_count_args(kmh_ctx* ctx, uint64_t n, int k, int canonical) {
    if (k < 1 || k > KMH_MAX_LONG_K)
        return fail(ctx, KMH_ERR_UNSUPPORTED, "k must be in [1, 1024] (k = " + std::to_string(k) + ")");
    if (canonical && k > KMH_MAX_SPARSE_K)
        return fail(ctx, KMH_ERR_UNSUPPORTED, "canonical counting needs k <= 32 (k = " + std::to_string(k) + ")");
    // Size limit ("Limits"): every path takes sequences below 2^32 - 1 bytes (u32
    // positions and counts; item counts are 64-bit).
    if (n >= 0xFFFFFFFFull)
        return fail(ctx, KMH_ERR_UNSUPPORTED, "sequence must be shorter than 2^32 - 1 bytes (one call)");
    return KMH_OK;
}

int kmh_count_host(kmh_ctx* ctx, const uint8_t* seq, uint64_t n, int k, int canonical,
                   kmh_kmers** out) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (!out || (n && !seq)) return fail(ctx, KMH_ERR_INVALID, "NULL argument");
    *out = nullptr;
    int rc = check_count_args(ctx, n, k, canonical);
    if (rc) return rc;
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, ctx->stream, [&](hipStream_t) {
        uint8_t* d_seq = nullptr;
        int rc2 = stage_sequence(ctx, seq, n, &d_seq);
        return rc2 ? rc2 : count_staged_impl(ctx, d_seq, n, k, canonical, out);
    });
}

int kmh_stage_host(kmh_ctx* ctx, const uint8_t* seq, uint64_t n) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (n && !seq) return fail(ctx, KMH_ERR_INVALID, "NULL argument");
    if (n >= 0xFFFFFFFFull)
        return fail(ctx, KMH_ERR_UNSUPPORTED, "sequence must be shorter than 2^32 - 1 bytes (one call)");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    uint8_t* d_seq = nullptr;
    int rc = on_stream(ctx, ctx->stream, [&](hipStream_t) { return stage_sequence(ctx, seq, n, &d_seq); });
    if (rc) return rc;
    // the host buffer may change after return: the copy from pageable memory completes first
    KMH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->staged_n = n;
    ctx->staged_ok = true;
    return KMH_OK;
}

int kmh_count_staged(kmh_ctx* ctx, int k, int canonical, kmh_kmers** out) {
    if (!ctx) return KMH_ERR_INVALID;
    ctx->err.clear();
    if (!out) return fail(ctx, KMH_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (!ctx->staged_ok || !ctx->seq.ptr)
        return fail(ctx, KMH_ERR_INVALID, "kmh_count_staged: no staged sequence (kmh_stage_host first; another "
                                          "host-buffer call or kmh_ctx_release/trim replaces or frees it)");
    int rc = check_count_args(ctx, ctx->staged_n, k, canonical);
    if (rc) return rc;
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, KMH_ERR_HIP, "hipSetDevice failed");
    return on_stream(ctx, ctx->stream, [&](hipStream_t) {
        return count_staged_impl(ctx, static_cast<uint8_t*>(ctx->seq.ptr), ctx->staged_n, k, canonical, out);
    });
}

static int count_staged_impl(kmh_ctx* ctx, uint8_t* d_seq, uint64_t n, int k, int canonical, kmh_kmers** out) {
    std::unique_ptr<kmh_kmers> r(new (std::nothrow) kmh_kmers);
    if (!r) return fail(ctx, KMH_ERR_NOMEM, "out of host memory");
    int rc = KMH_OK;
    try {
        if (k <= KMH_MAX_DENSE_K && !canonical) {
            const size_t bins = (size_t)1 << (2 * k);
            if ((rc = kmh::ensure(ctx, ctx->out, bins * sizeof(uint32_t)))) return rc;
            if ((rc = kmh::ensure(ctx, ctx->out2, bins * sizeof(uint32_t)))) return rc;
            uint32_t* d_counts = static_cast<uint32_t*>(ctx->out.ptr);
            uint32_t* d_first = static_cast<uint32_t*>(ctx->out2.ptr);
            const uint64_t off[2] = {0, n};
            if ((rc = kmh::dense_count(ctx, d_seq, off, 1, k, d_counts, ctx->stream))) return rc;
            if ((rc = kmh::dense_first(ctx, d_seq, off, 1, k, d_first, ctx->stream))) return rc;
            if ((rc = kmh::dense_order(ctx, d_counts, d_first, bins, n, r->codes, r->counts, r->first,
                                       ctx->stream)))
                return rc;

        } else if (k <= KMH_MAX_DENSE_K) {   // canonical, k <= 12: sort path
            if ((rc = kmh::sparse_count(ctx, d_seq, n, k, canonical, r->codes, r->counts, r->first,
                                        ctx->stream)))
                return rc;
        } else if (k <= KMH_MAX_SPARSE_K) {  // 13 <= k <= 32: hash-table path with first positions
            if ((rc = kmh::sparse_count_first(ctx, d_seq, n, k, canonical, r->codes, r->counts, r->first,
                                              ctx->stream)))
                return rc;
        } else {
            if ((rc = kmh::sparse_count_long(ctx, d_seq, n, k, r->codes, r->counts, r->first, ctx->stream)))
                return rc;
        }
    } catch (const std::bad_alloc&) {
        return fail(ctx, KMH_ERR_NOMEM, "out of host memory");
    }
    *out = r.release();
    return KMH_OK;
}

uint64_t kmh_kmers_size(const kmh_kmers* r) { return r ? r->codes.size() : 0; }

int kmh_kmers_export(const kmh_kmers* r, uint64_t* codes, uint32_t* counts, uint64_t* first) {
    if (!r) return KMH_ERR_INVALID;
    const size_t n = r->codes.size();
    if (codes && n) memcpy(codes, r->codes.data(), n * sizeof(uint64_t));
    if (counts && n) memcpy(counts, r->counts.data(), n * sizeof(uint32_t));
    if (first && n) memcpy(first, r->first.data(), n * sizeof(uint64_t));
    return KMH_OK;
}

int kmh_kmers_data(const kmh_kmers* r, const uint64_t** codes, const uint32_t** counts,
                   const uint64_t** first) {
    if (!r) return KMH_ERR_INVALID;
    if (codes) *codes = r->codes.data();
    if (counts) *counts = r->counts.data();
    if (first) *first = r->first.data();
    return KMH_OK;
}

void kmh_kmers_free(kmh_kmers* r) { delete r; }

}  // extern "C"
