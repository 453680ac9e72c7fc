/*
 * kmerhip.h -- C ABI of libkmerhip.so, the MI355X (gfx950) k-mer counting library
 * that replaces the hot path of Masthetheus/kmer-ml.
 *
 * The reference has no FFI: its boundary is the Python class API.  Each entry point
 * below replaces one piece of /root/reference/kmerml/kmers/generate.py; the Python
 * host mirror (kmer-ml_amd/kmerml/kmers/generate.py) binds them with ctypes so that
 * scripts/extract_kmers.py runs unchanged.  See INTEGRATION.md for the binding.
 *
 * Conventions
 *   - Plain C types only; every int-returning call returns KMH_OK (0) or a negative
 *     KMH_ERR_* code; the message is available from kmh_last_error(ctx) (or
 *     kmh_last_error(NULL) for calls without a context).  No C++ exception crosses
 *     this boundary.
 *   - The caller owns every host buffer; the library owns the device buffers of a
 *     context.  Functions with a _dev suffix take DEVICE pointers (hipMalloc /
 *     torch tensors on the context's device) and a hipStream_t passed as void*
 *     (NULL = the HIP null stream, as everywhere in HIP; torch's default stream);
 *     they only enqueue work.
 *   - The caller serialises the calls on one context (the Python mirror holds a lock);
 *     different contexts may be used concurrently.  Threads may share a context with
 *     different streams: a call's device work waits for the work the previous call
 *     queued on another stream (the cached workspace is never used by two calls in
 *     flight), so such calls run one after the other on the device.
 *   - Base alphabet: A/C/G/T in either case are bases (generate.py:41 upper()s the
 *     record, :55 keeps windows whose characters are all in "ACGT"); every other
 *     byte breaks windows.  k-mer codes are 2 bits per base, A=0 C=1 G=2 T=3, first
 *     base most significant, so code order = lexicographic order of the strings.
 *   - Counts are exact 32-bit integers: a sequence handed to a count call must be
 *     shorter than 2^32 - 1 bytes (KMH_ERR_INVALID otherwise).
 */
#ifndef KMERHIP_H
#define KMERHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMH_OK               0
#define KMH_ERR_INVALID     -1  /* bad argument                        */
#define KMH_ERR_HIP         -2  /* HIP runtime error                    */
#define KMH_ERR_NOMEM       -3  /* host or device allocation failed     */
#define KMH_ERR_UNSUPPORTED -4  /* k outside the supported range        */
#define KMH_ERR_IO          -5  /* file could not be read               */

#define KMH_MAX_DENSE_K  12     /* dense 4^k tables: 1 <= k <= 12        */
#define KMH_MAX_SPARSE_K 32     /* device hash pipeline: 13 <= k <= 32   */
#define KMH_MAX_LONG_K   1024   /* long k-mers (forward strand): 33 <= k <= 1024, sorted by
                                   ceil(k / 32) code words                      */

typedef struct kmh_ctx kmh_ctx;
typedef struct kmh_fasta kmh_fasta;
typedef struct kmh_kmers kmh_kmers;

/* ---- library / context ------------------------------------------------------ */

/* Version string, e.g. "kmerhip 0.1.0 gfx950". */
const char* kmh_version(void);

/* Build id: the first 16 hex digits of a SHA-256 over the library's sources (set by the
 * Makefile; "unknown" for other builds).  bench.py matches it against the build id stamped
 * into profiles/pmc_traffic.json before it reports a PMC traffic figure. */
const char* kmh_build_id(void);

/* Create a context on HIP device `device`: selects the device, creates a stream and
 * an empty device workspace.  Replaces nothing in the reference (it has no device). */
int kmh_ctx_create(int device, kmh_ctx** out);
void kmh_ctx_destroy(kmh_ctx* ctx);
/* Free the context's cached device workspace and pinned staging (they grow to the largest
 * call: tens of GB after a config-5 batch) after waiting for the work queued on the null
 * stream and the context stream; the next call allocates again.  For long-lived processes
 * that hand the device to other work.  Replaces nothing in the reference. */
int kmh_ctx_release(kmh_ctx* ctx);
/* Bytes the context holds now (cached device workspace + pinned staging). */
uint64_t kmh_ctx_workspace_bytes(const kmh_ctx* ctx);
/* Workspace policy of a long-lived process: kmh_ctx_release if the context holds more than
 * keep_bytes, else nothing.  The drop-in calls it after every organism, so the serial loop of
 * /root/reference/kmerml/kmers/generate.py:116-126 (extract_from_genome_list) does not keep a
 * config-5-sized workspace (tens of GB) between genomes. */
int kmh_ctx_trim(kmh_ctx* ctx, uint64_t keep_bytes);
/* Counters of the context since its creation, into stats[0 .. n): [0] sparse passes recounted by
 * the exact sort fallback, [1] the (genome, bucket) groups they were recounted in (one gather +
 * radix sort per group, however many of the bucket's passes failed), [2] workspace bytes.
 * Returns the number of counters the library keeps (3). */
int kmh_ctx_stats(const kmh_ctx* ctx, uint64_t* stats, int n);

/* Last error message of `ctx`, or of the calling thread's context-free calls when
 * ctx == NULL.  Never NULL; "" when there was no error. */
const char* kmh_last_error(const kmh_ctx* ctx);

/* Per-kernel timing with HIP events on the launch stream (bench / profiling).
 * enable != 0 starts recording; kmh_timing_report fills up to `cap` entries of
 * name/launches/total_ms and returns the number of distinct kernels. */
int kmh_timing_enable(kmh_ctx* ctx, int enable);
int kmh_timing_report(kmh_ctx* ctx, const char** names, uint64_t* launches,
                      double* total_ms, int cap);

/* ---- FASTA ingest (host) ----------------------------------------------------- */
/* Replaces `for record in SeqIO.parse(fasta_file, "fasta")` + `str(record.seq)`
 * (generate.py:39-41; Biopython 1.85 SimpleFastaParser semantics): universal newlines,
 * text before the first '>' skipped, id = first whitespace token of the title,
 * sequence lines rstrip()-ed and joined with every ' ' and '\r' removed. */
int kmh_fasta_read(const char* path, kmh_fasta** out);
uint64_t kmh_fasta_count(const kmh_fasta* f);
/* Record i: id bytes, sequence bytes (case preserved) and the sequence length in
 * characters (UTF-8 code points; equals the byte length for ASCII input), the value
 * generate.py:44 compares with max(k_values). */
int kmh_fasta_record(const kmh_fasta* f, uint64_t i, const char** id, uint64_t* id_len,
                     const uint8_t** seq, uint64_t* seq_len, uint64_t* char_len);
/* Concatenate the sequences of the records whose char_len >= min_len (the record
 * filter of generate.py:44-46), each followed by one '\n' separator byte, into `out`
 * (capacity `cap`).  kept (nullable, kmh_fasta_count bytes) receives 1/0 per record.
 * With out == NULL only *out_len is computed. */
int kmh_fasta_pack(const kmh_fasta* f, uint64_t min_len, uint8_t* out, uint64_t cap,
                   uint64_t* out_len, uint8_t* kept);
void kmh_fasta_free(kmh_fasta* f);

/* ---- counting, host buffers (the drop-in path) -------------------------------- */
/* Replaces the counting loop generate.py:36-58 for one k: counts every window of
 * `seq` whose k bytes are all bases.  Result = distinct k-mers in FIRST-OCCURRENCE
 * order (the insertion order of the reference's dict, which fixes the line order of
 * k{k}.txt, generate.py:89-91), with exact counts and the first window start.
 * 1 <= k <= 12: dense 4^k table on the GPU; 13 <= k <= 32: the device hash pipeline of
 * kmh_count_sparse_dev with every window's position carried (the minimum per k-mer), then a
 * radix sort of the first positions;
 * 33 <= k <= KMH_MAX_LONG_K: GPU sort of ceil(k / 32) code words per window + run-length,
 * and codes[i] then holds only the k-mer's first 32 bases (the whole k-mer is
 * seq[first[i] .. first[i] + k); kmh_format_lines_seq writes its text).
 * canonical != 0 counts min(forward, reverse complement) codes (not in the reference,
 * which is forward-strand only; used for BASELINE config 5; k <= 32 only). */
int kmh_count_host(kmh_ctx* ctx, const uint8_t* seq, uint64_t n, int k, int canonical,
                   kmh_kmers** out);
/* kmh_count_host in two steps, so that an organism crosses PCIe once for all its k (the
 * reference loops `for k in k_values` over the same record, generate.py:49): kmh_stage_host
 * copies seq to the context's device staging (it returns once the host buffer may change);
 * kmh_count_staged counts it at k like kmh_count_host.  The staging stays valid until the next
 * host-buffer call of any kind on the context or kmh_ctx_release / kmh_ctx_trim
 * (KMH_ERR_INVALID then). */
int kmh_stage_host(kmh_ctx* ctx, const uint8_t* seq, uint64_t n);
int kmh_count_staged(kmh_ctx* ctx, int k, int canonical, kmh_kmers** out);
uint64_t kmh_kmers_size(const kmh_kmers* r);
/* Copy the result out; any pointer may be NULL.  codes/counts/first: size() entries. */
int kmh_kmers_export(const kmh_kmers* r, uint64_t* codes, uint32_t* counts, uint64_t* first);
/* Borrow the result arrays without a copy (valid until kmh_kmers_free); any pointer may be
 * NULL.  The Python mirror wraps them as numpy views that keep the result alive. */
int kmh_kmers_data(const kmh_kmers* r, const uint64_t** codes, const uint32_t** counts,
                   const uint64_t** first);
void kmh_kmers_free(kmh_kmers* r);

/* Dense 4^k count vector of one host sequence (1 <= k <= 12), counts[4^k]
 * caller-owned.  Same counting rule as kmh_count_host. */
int kmh_count_dense_host(kmh_ctx* ctx, const uint8_t* seq, uint64_t n, int k,
                         uint32_t* counts);

/* ---- counting, device-resident batch (feature matrix; bench; multi-GPU) ------- */
/* G genomes in one device buffer: genome g = d_seq[offsets[g] .. offsets[g+1]),
 * offsets (HOST array, G+1 entries, non-decreasing) must be multiples of 16 bytes.
 * Writes the G x 4^k u32 count matrix (row g = genome g, column = k-mer code) to
 * d_matrix.  This is the per-rank block of the genomes x k-mers feature matrix that
 * the reference assembles in features.py:85-117 (kmerml.ml.features.KmerFeatureBuilder)
 * from the per-organism files; rows are all-gathered across ranks by the host. */
int kmh_count_dense_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets,
                        int G, int k, uint32_t* d_matrix, void* stream);

/* First window start of every k-mer per genome (0xFFFFFFFF = absent), G x 4^k u32,
 * same layout and arguments as kmh_count_dense_dev.  Used to rebuild the
 * first-occurrence line order of k{k}.txt. */
int kmh_first_dense_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets,
                        int G, int k, uint32_t* d_first, void* stream);

/* Synthetic genomes on the device: G genomes of `len` bases written
 * at d_seq + g * stride; base i of genome g is
 * "ACGT"[(splitmix64(s_g + (i >> 5)) >> (2 * (i & 31))) & 3] with
 * s_g = splitmix64(seed0 + g) (seed0 = 0x6B6D65724D4C0000 for the bench genomes). */
int kmh_synth_dev(kmh_ctx* ctx, uint8_t* d_seq, uint64_t len, uint64_t stride, int G,
                  uint64_t seed0, void* stream);

/* ---- sparse counting, device-resident batch (BASELINE config 5) --------------- */
/* The reference counts every k in a Python dict, a hash table (generate.py:36,58); for
 * 13 <= k <= 32 this counts G device-resident genomes (layout as kmh_count_dense_dev):
 * two partition passes bring one pass of a bucket into a workgroup's LDS, where a counting
 * sort deduplicates it (u32 residues up to k = 21, u64 beyond; what the LDS cannot hold
 * goes to the exact sort-based fallback).  canonical != 0 counts min(forward, reverse
 * complement) codes.  Genome g's distinct k-mers (2-bit codes, A0 C1 G2 T3, first base
 * most significant) and their exact counts are written to d_codes / d_counts starting at
 * entry out_off[g] (kmh_sparse_out_offsets: the number of windows of the genomes before
 * g, so a genome never needs more room than its windows); d_nkmers[g] (device) receives
 * the number of distinct k-mers.  Order within a genome is unspecified (grouped by bucket,
 * the top 10 bits of the code, and pass).  Synchronises `stream` (the work list depends on the bucket
 * sizes). */
int kmh_count_sparse_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G,
                         int k, int canonical, uint64_t* d_codes, uint32_t* d_counts,
                         uint64_t* d_nkmers, void* stream);
/* kmh_count_sparse_dev with every genome's rows in ascending code order (the organism rows of
 * the column-sharded matrix, /root/reference/kmerml/ml/features.py:96-111: its columns are the
 * sorted union of labels).  The genomes' rows are back to back from entry 0: genome g's are
 * d_codes / d_counts [sum of d_nrows[0 .. g), + d_nrows[g]), codes strictly ascending, every
 * count nonzero; d_nrows[g] and d_ndistinct[g] (device) both receive its distinct k-mers (since
 * round 5 a distinct-count pass places every item first: no padding, no compaction).  The
 * buffers need kmh_sparse_out_offsets' total, as for kmh_count_sparse_dev.  Same arguments and
 * limits otherwise. */
int kmh_count_sparse_sorted_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G,
                                int k, int canonical, uint64_t* d_codes, uint32_t* d_counts,
                                uint64_t* d_nrows, uint64_t* d_ndistinct, void* stream);
/* One rank's column shard of the organisms x k-mers matrix for sparse k (features.py:96-111:
 * columns = the sorted union of the organisms' labels).  d_codes holds R organism rows back to
 * back, row r = d_codes[row_off[r], row_off[r + 1]) (row_off: host, R + 1 entries), each sorted
 * by code, every code in [lo_code, hi_code_incl] (the rows of kmh_count_sparse_sorted_dev, cut to
 * the rank's code range).  Writes the sorted union of the codes to
 * d_columns (room for row_off[R] - row_off[0] entries), the column index of every row entry to
 * d_indices[row_off[0] ..] (so row_off, these indices and the rows' counts form the shard's CSR),
 * and the union's size to *ncols (host).  1 <= R <= 4096.  Synchronises `stream`. */
int kmh_shard_union_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R,
                        uint64_t lo_code, uint64_t hi_code_incl, uint64_t* d_columns, int64_t* d_indices,
                        uint64_t* ncols, void* stream);
/* kmh_shard_union_dev with u32 column indices (half the index bytes): the rows must hold fewer than
 * 2^32 - 1 entries (KMH_ERR_INVALID otherwise), so every column index fits.  The shard's default
 * (kmerml.kmers.matrix.shard_from_rows). */
int kmh_shard_union_u32_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R,
                            uint64_t lo_code, uint64_t hi_code_incl, uint64_t* d_columns, uint32_t* d_indices,
                            uint64_t* ncols, void* stream);

/* ---- the exchange of the column-sharded sparse matrix (multi-GPU, config 5) ---- */
/* Each rank owns a contiguous code range of the matrix's columns (features.py:96-111's sorted union
 * of labels); a rank's organism rows are sorted by code, so what it sends a peer is one slice per
 * row, between two cuts.  d_cuts[r * nb + b] (device, R x nb u64) = the first entry of row r
 * (relative to the row) whose code is >= bounds[b]: rows as for kmh_shard_union_dev (host row_off,
 * R + 1 entries), bounds a host array of nb codes.  Also gives a code histogram (cuts at the
 * histogram's edges) without a pass over the entries. */
int kmh_rows_cuts_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint64_t* row_off, int R, const uint64_t* bounds,
                      int nb, uint64_t* d_cuts, void* stream);
/* Compact wire format of S row slices for the all-to-all: slice i = entries [slice_start[i],
 * slice_start[i] + slice_n[i]) of d_codes / d_counts (device; host slice arrays), codes ascending
 * within a slice.  Per 1024 entries one 2320-byte record (the first code, the low 16 bits of every
 * gap, a bit per gap with higher bits and per count that is not 1) and, per slice, the escape words
 * (u32, in entry order: gap >> 16, then the count) at positions implied by the bits: exact for any
 * codes and counts, ~2.4 bytes per entry for config 5's rows against 12 raw.  kmh_wire_size_dev
 * writes every slice's byte size to slice_bytes (host; synchronises the stream); kmh_wire_encode_dev
 * writes the slices back to back to d_out (out_bytes >= the sum), reusing the sizing of a
 * kmh_wire_size_dev call with the same arguments just before it (the data must not change in
 * between).  KMH_ERR_UNSUPPORTED past 2^24 slices, 2^32 chunks or 2^32 escape words in one slice. */
int kmh_wire_size_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* slice_start,
                      const uint64_t* slice_n, int S, uint64_t* slice_bytes, void* stream);
int kmh_wire_encode_dev(kmh_ctx* ctx, const uint64_t* d_codes, const uint32_t* d_counts, const uint64_t* slice_start,
                        const uint64_t* slice_n, int S, uint8_t* d_out, uint64_t out_bytes, void* stream);
/* Decode S slices back to back in d_in (slice i: slice_n[i] entries in slice_bytes[i] bytes, as the
 * sender's kmh_wire_size_dev reported; host arrays) into d_codes / d_counts at entry slice_dst[i]
 * (the caller's output must hold them).  A slice whose bytes do not match its entries is
 * KMH_ERR_INVALID; escape positions are clamped to their chunk and slice, so damaged bytes cannot
 * move a read or write outside it. */
int kmh_wire_decode_dev(kmh_ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const uint64_t* slice_n,
                        const uint64_t* slice_bytes, const uint64_t* slice_dst, int S, uint64_t* d_codes,
                        uint32_t* d_counts, void* stream);
/* Output offsets of kmh_count_sparse_dev: out_off[g] for g = 0..G (out_off nullable);
 * returns out_off[G], the total capacity in entries. */
uint64_t kmh_sparse_out_offsets(const uint64_t* offsets, int G, int k, uint64_t* out_off);

/* ---- feature-matrix assembly (multi-GPU) ------------------------------------- */
/* The reference assembles its organisms x k-mers matrix on one CPU (features.py:85-117).
 * Here each rank owns a block of count rows; blocks are all-gathered over xGMI as
 * saturating u8 rows plus an exact escape list, 4x fewer bytes than u32 rows.
 *
 * Encode rows x cols u32 counts (cols % 16 == 0) into d_u8 (values >= 255 stored as 255) and
 * append every value >= 255 as a (row, col, value) u32 triple to d_esc (capacity `cap`
 * triples).  *d_esc_n (device) receives the number of escapes; if it exceeds cap the
 * encoding is incomplete and the caller must send u32 rows instead. */
int kmh_rows_encode_u8_dev(kmh_ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols,
                           uint8_t* d_u8, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n,
                           void* stream);
/* Widen gathered u8 rows (rows x cols) to u32 and apply the escapes of `ranks` ranks:
 * rank r's escape triples are d_esc[r * cap * 3 ...], its count d_esc_n[r], its rows start
 * at row r * rows_per_rank. */
int kmh_rows_decode_u8_dev(kmh_ctx* ctx, const uint8_t* d_u8, uint64_t rows, uint64_t cols,
                           const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n,
                           int ranks, uint64_t rows_per_rank, uint32_t* d_rows, void* stream);

/* u4 wire format (the multi-GPU default, 8x fewer bytes than u32 rows): two counts per byte,
 * element 2i in the low nibble of byte i; values >= 15 are stored as 15 and appended to
 * d_esc as an exact (index, value) u32 pair, index = row * cols + col within the block.
 * Needs cols % 32 == 0 and rows * cols < 2^32 - 1.  *d_esc_n (device) receives the number of
 * escapes; if it exceeds cap the encoding is incomplete (send u32 rows instead). */
int kmh_rows_encode_u4_dev(kmh_ctx* ctx, const uint32_t* d_rows, uint64_t rows, uint64_t cols,
                           uint8_t* d_u4, uint32_t* d_esc, uint32_t cap, uint32_t* d_esc_n,
                           void* stream);
/* kmh_count_dense_dev into d_matrix (G x 4^k u32) and, in the same pass, the u4 encoding of
 * those rows exactly as kmh_rows_encode_u4_dev(d_matrix, G, 4^k, ...) would write it: for
 * k >= 10 the count kernel writes each bucket's nibbles and escapes straight from its LDS
 * table (no second pass over the rows).  3 <= k <= 12, G * 4^k < 2^32 - 1.  The multi-GPU
 * step's count + encode (each rank's slot of the all-gather that assembles the matrix of
 * /root/reference/kmerml/ml/features.py:85-117). */
int kmh_count_dense_u4_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                           uint32_t* d_matrix, uint8_t* d_u4, uint32_t* d_esc, uint32_t cap,
                           uint32_t* d_esc_n, void* stream);
/* The same u4 slot without the u32 rows: d_scratch (G x 4^k u32, device) is working memory
 * for the rare buckets whose encoding is redone from rows (a count past 65535, or more escapes
 * than the kernel stages), and its contents are unspecified afterwards.  For k >= 10 this is
 * the multi-GPU step's count (bench.py, kmerml.kmers.matrix): 4^k x 4 bytes less written per
 * genome.  Replaces the same reference code as kmh_count_dense_u4_dev. */
int kmh_count_dense_u4only_dev(kmh_ctx* ctx, const uint8_t* d_seq, const uint64_t* offsets, int G, int k,
                               uint32_t* d_scratch, uint8_t* d_u4, uint32_t* d_esc, uint32_t cap,
                               uint32_t* d_esc_n, void* stream);
/* Widen one block of u4 rows (rows x cols) to u32 at d_rows and apply its escapes (pairs with an
 * index outside the block are ignored: a slot that came off the wire never writes elsewhere). */
int kmh_rows_decode_u4_dev(kmh_ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols,
                           const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n,
                           uint32_t* d_rows, void* stream);
/* Widen rows [row0, row0 + nrows) of one u4 block (rows x cols) to u32 at d_rows (nrows x cols)
 * with exactly their escapes: the row accessor of a matrix kept in the compact u4 + escape
 * form after the all-gather (the organisms x k-mers matrix of
 * /root/reference/kmerml/ml/features.py:85-117, one row per organism). */
int kmh_rows_decode_u4_range_dev(kmh_ctx* ctx, const uint8_t* d_u4, uint64_t rows, uint64_t cols,
                                 const uint32_t* d_esc, uint32_t cap, const uint32_t* d_esc_n,
                                 uint64_t row0, uint64_t nrows, uint32_t* d_rows, void* stream);

/* ---- file output (host) -------------------------------------------------------- */
/* Write n bytes to `path`: plain when gzip_level < 0, else gzip at that level (0..9; the
 * reference uses 9 via gzip.open, generate.py:82-85) as independently deflated 8 MiB members
 * on up to `threads` threads (0 = all cores, at most 16); any gzip reader returns the same
 * bytes.  KMH_ERR_IO if the file cannot be written. */
int kmh_write_file(const char* path, const void* data, uint64_t n, int gzip_level, int threads);

/* ---- k{k}.txt text (host) ----------------------------------------------------- */
/* Replaces the writer loop of _save_kmers_to_file (generate.py:89-91): one line
 * "<digits>\t<count>\n" per k-mer, digits A=0 T=1 C=2 G=3 (generate.py:71).
 * Writes at most `cap` bytes; returns the number of bytes the full text needs (so a
 * call with out == NULL sizes the buffer), or a negative error code. */
int64_t kmh_format_lines(int k, const uint64_t* codes, const uint64_t* counts, uint64_t n,
                         char* out, uint64_t cap);

/* Same text for any k, with the digits taken from the sequence the k-mers were counted in:
 * line i is seq[first[i] .. first[i] + k) in digits, a tab, counts[i] (the form used for
 * k > 32, where a code no longer fits 64 bits; seq = the buffer given to kmh_count_host and
 * first = its kmh_kmers_export first positions).  KMH_ERR_INVALID if a k-mer lies outside
 * seq[0, seq_len). */
int64_t kmh_format_lines_seq(int k, const uint8_t* seq, uint64_t seq_len, const uint64_t* first,
                             const uint64_t* counts, uint64_t n, char* out, uint64_t cap);

/* ---- feature columns (device) ------------------------------------------------- */
/* Replaces the per-row feature functions of /root/reference/kmerml/kmers/statistics.py:188-238
 * (base counts, GC percent, CpG count and observed/expected ratio, Shannon entropy, dinucleotide
 * repeat) for the labels of integer-parsed k{k}.txt lines: code i's label is the k-mer with its
 * leading A's stripped ("A" for A...A; statistics.py:157, 248-273).  n codes (d_codes, or NULL for
 * all codes 0 .. n - 1); all arrays are DEVICE arrays of n entries except d_cnt (4 x n: the A, C,
 * G, T counts, base-major), d_order (625 x 4 int32: for the first-appearance pattern key of a
 * label, the bases in the order Python's set() iterates them, -1-padded; computed by the caller's
 * interpreter) and d_lg ((k + 1) x (k + 1) doubles: math.log2(n / L) at [n][L]).  Every float64 is
 * the reference's operation sequence, rounded once per operation (no fused multiply-add). */
int kmh_feature_columns_dev(kmh_ctx* ctx, const uint64_t* d_codes, uint64_t n, int k, const int32_t* d_order,
                            const double* d_lg, int64_t* d_cnt, int64_t* d_cpg, int64_t* d_rep, double* d_gc,
                            double* d_oe, double* d_ent, void* stream);

/* ---- feature CSV text (host) --------------------------------------------------- */
/* Replaces pandas' DataFrame.to_csv(index=False) of the per-organism feature table
 * (/root/reference/kmerml/kmers/statistics.py:136-144): the rows of a block of columns as CSV
 * text, no header, '\n' after every row, exactly as pandas writes them -- int64 / uint64 as
 * decimal integers, float64 as Python's float repr (shortest round trip; fixed notation for
 * decimal exponents -4 < e <= 16, else d.ddde+XX).  Column j has kinds[j] and data[j] / aux[j]:
 *   KMH_CSV_I64   data: const int64_t[nrows]                       aux: unused
 *   KMH_CSV_F64   data: const double[nrows]                        aux: unused
 *   KMH_CSV_STR   data: UTF-8 bytes of every field back to back    aux: const uint64_t[nrows + 1]
 *                 field offsets
 *   KMH_CSV_LABEL data: const uint64_t[nrows] k-mer codes (A0 C1 G2 T3) aux: const int64_t* k
 *                 (1..32): the reference's label of an integer-parsed k-mer file line, the k-mer
 *                 with its leading A's stripped ("A" for A...A; statistics.py:157, 248-273)
 *   KMH_CSV_U64   data: const uint64_t[nrows]                      aux: unused
 * Formatted on up to `threads` host threads (0 = all cores, at most 16).  KMH_ERR_UNSUPPORTED
 * when pandas would write a value differently (NaN or inf, an empty text field, a field with
 * ',', '"', '\n' or '\r': pandas quotes it): the caller then writes that block with pandas. */
#define KMH_CSV_I64   0
#define KMH_CSV_F64   1
#define KMH_CSV_STR   2
#define KMH_CSV_LABEL 3
#define KMH_CSV_U64   4
typedef struct kmh_text kmh_text;
int kmh_csv_format(int ncols, const int32_t* kinds, const void* const* data, const void* const* aux,
                   uint64_t nrows, int threads, kmh_text** out);
/* Borrow the text (valid until kmh_text_free). */
int kmh_text_data(const kmh_text* t, const char** data, uint64_t* len);
void kmh_text_free(kmh_text* t);

#ifdef __cplusplus
}
#endif

#endif /* KMERHIP_H */
