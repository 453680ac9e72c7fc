// Internal declarations shared by the host runtime (kmh_api.cpp, kmh_fasta.cpp) and the
// HIP translation units (kmh_dense.hip, kmh_sparse.hip).  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/kmerhip.h"

namespace kmh {

// Geometry of the dense path ("Kernels").
constexpr int kTileThreads = 1024;                     // threads of a tile workgroup
constexpr int kTileBpt = 32;                           // window starts per thread
constexpr int kTile = kTileThreads * kTileBpt;         // 32768 window starts per tile
constexpr int kSubBits = 15;                           // k_direct: LDS slice of 32768 u32 bins
constexpr int kSubBins = 1 << kSubBits;                // = 128 KiB of LDS
constexpr int kCountThreads = 1024;                    // threads of a bucket-count workgroup
constexpr int kDirectMaxK = 7;                         // k <= 7: whole table in LDS

// A growable device allocation owned by a context.
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
};

struct TimedLaunch {
    const char* name;
    hipEvent_t start;
    hipEvent_t stop;
};

struct Ctx {
    int device = 0;
    int num_cu = 256;                  // compute units of the device (persistent grids)
    hipStream_t stream = nullptr;
    std::string err;
    // device workspace
    DevBuf seq, suf, toff, meta, out, out2, fix, redo, sparse[8], order, sort_tmp, scan_tmp, first;
    // the config-5 exchange (kmh_wire.hip): [0] slice plan, [1] escapes per chunk, [2] their scan;
    // the scan and the slices' bytes are kept for the encode call that follows a size call on the
    // same slices (wire_key: a hash of the device pointers and the slice arrays)
    DevBuf wire[3];
    uint64_t wire_key = 0;
    bool wire_valid = false;
    std::vector<uint64_t> wire_sbytes;
    // the (goff, tbase) layout last copied to `meta` (upload_layout skips an identical copy)
    std::vector<uint64_t> meta_cache;
    // kmh_stage_host: bytes of the host sequence staged in `seq` (valid while staged_ok)
    uint64_t staged_n = 0;
    bool staged_ok = false;
    // kmh_ctx_stats: sparse passes recounted by the exact fallback, and the (genome, bucket)
    // groups they were recounted in (one gather + sort each), since the context was created
    uint64_t fb_passes = 0, fb_groups = 0;
    // pinned staging for small host->device tables
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    hipEvent_t pinned_ready = nullptr;
    // workspace stream order (kmh_api.cpp, on_stream): the stream of the last call that queued
    // work on the workspace, and an event recorded on it after that work
    hipEvent_t ws_done = nullptr;
    hipStream_t ws_stream = nullptr;
    bool ws_pending = false;
    // per-kernel timing
    bool timing = false;
    bool timing_skip = false;        // the launch in flight is not timed (KMH_TIMING_ONLY)
    std::string timing_only;         // ",name,name," -- empty: time every launch
    std::vector<TimedLaunch> launches;
    std::vector<hipEvent_t> event_pool;
    std::vector<std::string> report_names;
};

// Error helpers: set ctx->err (or the thread-local message when ctx == nullptr).
int fail(Ctx* ctx, int code, const std::string& msg);
int hip_fail(Ctx* ctx, hipError_t e, const char* what);
void set_thread_error(const std::string& msg);

#define KMH_HIP(ctx, call)                                   \
    do {                                                     \
        hipError_t e_ = (call);                              \
        if (e_ != hipSuccess) return hip_fail((ctx), e_, #call); \
    } while (0)

// Grow-only device buffer.
int ensure(Ctx* ctx, DevBuf& b, size_t bytes);
// Free one cached buffer after the queued work that may read it (workspace policy).
int drop(Ctx* ctx, DevBuf& b);
// Copy a small host table to device through the pinned staging buffer (async on s).
int upload(Ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t s);

// Kernel timing brackets (no-ops unless ctx->timing).
void time_begin(Ctx* ctx, hipStream_t s, const char* name);
void time_end(Ctx* ctx, hipStream_t s);

// Genome/tile layout of a batch launch: goff = genome byte offsets (G + 1), tbase =
// cumulative tile counts (G + 1) for tiles of `tile` window starts.
struct Layout {
    std::vector<uint64_t> goff, tbase;
    uint64_t ntiles = 0;
};
int make_layout(Ctx* ctx, const uint64_t* offsets, int G, int k, uint64_t tile, Layout& L);
// Copies goff and tbase to ctx->meta; returns their device addresses.
int upload_layout(Ctx* ctx, const Layout& L, hipStream_t s, const uint64_t** d_goff,
                  const uint64_t** d_tbase);
// Integer environment knobs (experiments): env_mb treats values <= 0 as unset.
long env_long(const char* name, long dflt);
size_t env_mb(const char* name, size_t dflt);

// ---- dense path (kmh_dense.hip) ----
// offsets: host, G+1 entries.  d_out: G x 4^k u32.
// dense_count plus the u4 encoding of the rows (rows_encode_u4's layout), fused into the
// count kernel's epilogue for k >= 10.  rows = 0: d_out is scratch, written only where the
// encoding needs the u32 rows (k >= 10; k <= 9 counts every row, then encodes them).
int dense_count_u4(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k, uint32_t* d_out,
                   uint8_t* d_u4, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n, int rows, hipStream_t s);
int dense_count(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                uint32_t* d_out, hipStream_t s);
int dense_first(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                uint32_t* d_first, hipStream_t s);
int synth(Ctx* ctx, uint8_t* d_seq, uint64_t len, uint64_t stride, int G, uint64_t seed0,
          hipStream_t s);

// ---- matrix assembly encoding (kmh_matrix.hip) ----
int rows_encode_u8(Ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols,
                   uint8_t* d_u8, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n,
                   hipStream_t s);
int rows_decode_u8(Ctx* ctx, const uint8_t* d_u8, uint64_t rows, uint64_t cols,
                   const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n, int ranks,
                   uint64_t rows_per_rank, uint32_t* d_rows, hipStream_t s);

int rows_encode_u4(Ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols, uint8_t* d_u4,
                   uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n, hipStream_t s);
int rows_decode_u4(Ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols, const uint32_t* d_esc,
                   uint32_t cap, const uint32_t* d_esc_n, uint32_t* d_rows, hipStream_t s);
int rows_decode_u4_range(Ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols, const uint32_t* d_esc,
                         uint32_t cap, const uint32_t* d_esc_n, uint64_t row0, uint64_t nrows, uint32_t* d_rows,
                         hipStream_t s);

// ---- sparse path (kmh_sparse.hip) ----
// Counts the windows of d_seq[0, n) for 13 <= k <= 32 (works for any 1 <= k <= 32).
// On return the host vectors hold the distinct codes in first-occurrence order (sorted by
// first window start on the device), their counts and their first window start.
int sparse_count(Ctx* ctx, const uint8_t* d_seq, uint64_t n, int k, int canonical,
                 std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                 std::vector<uint64_t>& first, hipStream_t s);
// 13 <= k <= 32: the same result through the device hash pipeline with positions (kmh_hash.hip).
int sparse_count_first(Ctx* ctx, const uint8_t* d_seq, uint64_t n, int k, int canonical,
                       std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                       std::vector<uint64_t>& first, hipStream_t s);
// 33 <= k <= KMH_MAX_LONG_K, forward strand: sort by ceil(k / 32) code words (kmh_sparse.hip).
int sparse_count_long(Ctx* ctx, const uint8_t* d_seq, uint64_t n, int k, std::vector<uint64_t>& codes,
                      std::vector<uint32_t>& counts, std::vector<uint64_t>& first, hipStream_t s);

// First-occurrence order of a dense count row on the device (kmh_sparse.hip): the codes with
// a nonzero count, sorted by their first window start, with counts and starts, to the host.
int dense_order(Ctx* ctx, const uint32_t* d_counts, const uint32_t* d_first, size_t bins,
                uint64_t n, std::vector<uint64_t>& codes, std::vector<uint32_t>& counts,
                std::vector<uint64_t>& first, hipStream_t s);

// ---- device-resident sparse path (kmh_hash.hip) ----
// Windows per genome -> cumulative output offsets (out_off: G + 1 entries, nullable).
uint64_t sparse_windows(const uint64_t* offsets, int G, int k, uint64_t* out_off);
int sparse_count_dev(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                     int canonical, uint64_t* d_codes, uint32_t* d_counts, uint64_t* d_nkmers,
                     hipStream_t s);
// The same counts with every genome's rows in ascending code order, compact and back to back from
// entry 0: genome g's rows follow those of genomes 0 .. g - 1, codes strictly ascending, every count
// nonzero; d_nrows[g] = d_ndist[g] = its distinct k-mers (no padding since round 5).
int sparse_count_dev_sorted(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                            int canonical, uint64_t* d_codes, uint32_t* d_counts, uint64_t* d_nrows,
                            uint64_t* d_ndist, hipStream_t s);
// The same pipeline with every entry's window position carried along: d_firsts[i] (u32, relative
// to the genome) = the first window start of k-mer i (the drop-in's first-occurrence order).
int sparse_count_dev_first(Ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k, int canonical,
                           uint64_t* d_codes, uint32_t* d_counts, uint32_t* d_firsts, uint64_t* d_nkmers,
                           hipStream_t s);

// ---- column shard of the sparse matrix (kmh_shard.hip) ----
// R sorted organism rows of codes in [lo, hi_incl], rows back to back: row r is d_codes[row_off[r],
// row_off[r + 1]) (host offsets).  d_columns (>= the entries) receives the sorted union of the
// codes, d_indices[e] (for every entry e of the rows) its column; *ncols the union's size.
// idx32: d_indices is uint32_t[] (the rows hold fewer than 2^32 entries), else int64_t[].
int shard_union(Ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, uint64_t lo,
                uint64_t hi_incl, uint64_t* d_columns, void* d_indices, bool idx32, uint64_t* ncols, hipStream_t s);
// out[0 .. n] = the exclusive u64 scan of in[0 .. n) and its total (ctx->scan_tmp).
int scan_u32_u64(Ctx* ctx, const uint32_t* in, uint32_t n, unsigned long long* out, hipStream_t s);

// ---- the config-5 exchange (kmh_wire.hip) ----
// d_cuts[r * nb + b] = first entry of row r (relative) with code >= bounds[b] (host row_off, bounds).
int rows_cuts(Ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, const uint64_t* bounds, int nb,
              uint64_t* d_cuts, hipStream_t s);
// Compact wire of S row slices (slice i = entries [sstart[i], + sn[i]) of d_codes / d_counts, host
// arrays): wire_size -> bytes per slice (synchronises); wire_encode -> the slices back to back.
int wire_size(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* sstart, const uint64_t* sn,
              int S, uint64_t* slice_bytes, hipStream_t s);
int wire_encode(Ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* sstart, const uint64_t* sn,
                int S, uint8_t* d_out, uint64_t out_bytes, hipStream_t s);
// Slices back to back in d_in (sn entries, sbytes bytes each) -> entries sdst[i] .. of the output.
int wire_decode(Ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const uint64_t* sn, const uint64_t* sbytes,
                const uint64_t* sdst, int S, uint64_t* d_codes, uint32_t* d_counts, hipStream_t s);


// ---- feature columns of the feature CSV (kmh_features.hip) ----
int feature_columns(Ctx* ctx, const uint64_t* d_codes, uint64_t n, int k, const int32_t* d_order, const double* d_lg,
                    int64_t* d_cnt, int64_t* d_cpg, int64_t* d_rep, double* d_gc, double* d_oe, double* d_ent,
                    hipStream_t s);

// ---- sort / scan / runs (kmh_sort.hip), n < 2^32 - 1 items ----
// Stable LSD radix sort of (key, value) pairs on key bits [bit_lo, bit_hi), 8 bits per pass;
// *result_in_alt: the sorted pairs ended in keys_alt / vals_alt (odd number of passes).
template <typename K>
int radix_sort_pairs(Ctx* ctx, K* keys, K* keys_alt, uint32_t* vals, uint32_t* vals_alt, uint64_t n, int bit_lo,
                     int bit_hi, bool* result_in_alt, hipStream_t s);
// out[i] = sum of in[0 .. i); *d_total (device, nullable) = the sum of all n (must fit 32 bits).
int scan_exclusive_u32(Ctx* ctx, const uint32_t* d_in, uint32_t* d_out, uint64_t n, uint32_t* d_total,
                       hipStream_t s);
// Start index of every run of equal keys of a sorted array, in order; *d_nruns (device).
// d_flags / d_ex: scratch of n u32 each.
template <typename K>
int run_starts(Ctx* ctx, const K* d_keys, uint64_t n, uint32_t* d_flags, uint32_t* d_ex, uint32_t* d_starts,
               uint32_t* d_nruns, hipStream_t s);
// Indices i with d_flags[i] != 0 (flags are 0 / 1), in order; *d_count (device).  d_ex: n u32 scratch.
int select_flagged(Ctx* ctx, const uint32_t* d_flags, uint64_t n, uint32_t* d_ex, uint32_t* d_idx, uint32_t* d_count,
                   hipStream_t s);

}  // namespace kmh
