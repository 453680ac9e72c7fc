// kmh_fasta.cpp -- host FASTA ingest and k{k}.txt text formatting.
//
// kmh_fasta_read replaces `for record in SeqIO.parse(fasta_file, "fasta")` followed by
// `str(record.seq)` (/root/reference/kmerml/kmers/generate.py:39-41).  The parser rules
// are those of Biopython 1.85's SimpleFastaParser/FastaIterator (third-party, not in the
// reference; requirements.txt:1) as read through Python's text mode:
//   * universal newlines: "\r\n", "\r" and "\n" each end a line;
//   * lines before the first line starting with '>' are skipped;
//   * title = line[1:].rstrip(); id = first whitespace-separated word of the title;
//   * sequence lines are rstrip()-ed, joined, and every ' ' is removed.
// rstrip()/split() whitespace is Python's str.isspace() set, decoded from UTF-8.
//
// kmh_format_lines replaces the writer loop of _save_kmers_to_file (generate.py:86-91).
#include <errno.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <memory>
#include <new>
#include <string>
#include <vector>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <system_error>
#include <thread>
#include "kmh_internal.h"

struct kmh_fasta {
    struct Rec {
        uint64_t id_off, id_len, seq_off, seq_len, char_len;
    };
    struct Free {
        void operator()(uint8_t* q) const { free(q); }
    };
    std::string ids;
    std::unique_ptr<uint8_t[], Free> seqs;   // every record's bytes, back to back
    uint64_t nseq = 0;
    std::vector<Rec> recs;
};

namespace {

// Length of the Python-whitespace character ending at p[n-1] (0 if none).
size_t trailing_space(const uint8_t* p, size_t n) {
    if (n == 0) return 0;
    const uint8_t c = p[n - 1];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F)) return 1;
    if (n >= 2 && p[n - 2] == 0xC2 && (c == 0x85 || c == 0xA0)) return 2;  // U+0085, U+00A0
    if (n >= 3) {
        const uint8_t a = p[n - 3], b = p[n - 2];
        if (a == 0xE1 && b == 0x9A && c == 0x80) return 3;                    // U+1680
        if (a == 0xE2 && b == 0x80 && ((c >= 0x80 && c <= 0x8A) || c == 0xA8 || c == 0xA9 || c == 0xAF))
            return 3;                                                         // U+2000-200A, 2028, 2029, 202F
        if (a == 0xE2 && b == 0x81 && c == 0x9F) return 3;                    // U+205F
        if (a == 0xE3 && b == 0x80 && c == 0x80) return 3;                    // U+3000
    }
    return 0;
}

// Length of the Python-whitespace character starting at p[0] (0 if none).
size_t leading_space(const uint8_t* p, size_t n) {
    if (n == 0) return 0;
    const uint8_t c = p[0];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F)) return 1;
    if (n >= 2 && c == 0xC2 && (p[1] == 0x85 || p[1] == 0xA0)) return 2;
    if (n >= 3) {
        const uint8_t b = p[1], d = p[2];
        if (c == 0xE1 && b == 0x9A && d == 0x80) return 3;
        if (c == 0xE2 && b == 0x80 && ((d >= 0x80 && d <= 0x8A) || d == 0xA8 || d == 0xA9 || d == 0xAF))
            return 3;
        if (c == 0xE2 && b == 0x81 && d == 0x9F) return 3;
        if (c == 0xE3 && b == 0x80 && d == 0x80) return 3;
    }
    return 0;
}

size_t rstrip_len(const uint8_t* p, size_t n) {
    for (size_t t; (t = trailing_space(p, n)) != 0;) n -= t;
    return n;
}


// n bytes (at least 1) for a whole file: 2 MiB aligned with transparent huge pages requested,
// so that first-touching a genome-sized buffer takes a few hundred page faults, not ~25 000
// per 100 MB.  Throws std::bad_alloc.
uint8_t* alloc_bytes(size_t n) {
    constexpr size_t kHuge = 2u << 20;
    void* q = nullptr;
    const size_t sz = (std::max<size_t>(n, 1) + kHuge - 1) / kHuge * kHuge;
    if (posix_memalign(&q, kHuge, sz) != 0 || !q) throw std::bad_alloc();
    madvise(q, sz, MADV_HUGEPAGE);   // advisory: ignored where THP is off
    return static_cast<uint8_t*>(q);
}

// One piece of a FASTA buffer, parsed in place: its sequence bytes (lines before its first
// header included -- whether they belong to a record is decided when the pieces are stitched)
// are compacted to the front of the piece's own byte range, which they never outgrow, so
// parsing allocates nothing.  Each header keeps the output offset where its record's bases
// start and the continuation-byte count before it.
struct Piece {
    struct Hdr {
        uint64_t at, cont_before;
        std::string id;
    };
    uint64_t len = 0, cont = 0;
    std::vector<Hdr> hdrs;
};

uint64_t count_continuation(const uint8_t* p, size_t n);

// The lines of p[a, b): a is a line start, b a line start or the end of the buffer.
void parse_lines(uint8_t* p, size_t a, size_t b, Piece& out) {
    size_t i = a, w = a;   // read and write positions, w <= i
    while (i < b) {
        // line end: the first '\n' or '\r' (memchr: vectorised scans of ~80-byte lines)
        const void* nl = memchr(p + i, '\n', b - i);
        size_t j = nl ? (size_t)(static_cast<const uint8_t*>(nl) - p) : b;
        if (const void* cr = memchr(p + i, '\r', j - i)) j = (size_t)(static_cast<const uint8_t*>(cr) - p);
        const uint8_t* line = p + i;
        const size_t len = j - i;
        // advance past the line terminator (\r\n counts once)
        if (j < b && p[j] == '\r' && j + 1 < b && p[j + 1] == '\n') i = j + 2;
        else i = j + 1;
        if (len > 0 && line[0] == '>') {
            const size_t tl = rstrip_len(line + 1, len - 1);
            const uint8_t* t = line + 1;
            size_t c = 0;
            for (size_t x; c < tl && (x = leading_space(t + c, tl - c)) != 0;) c += x;
            size_t d = c;
            while (d < tl && leading_space(t + d, tl - d) == 0) ++d;
            out.hdrs.push_back(Piece::Hdr{w - a, out.cont, std::string(reinterpret_cast<const char*>(t + c), d - c)});
            continue;
        }
        const size_t sl = rstrip_len(line, len);
        const size_t w0 = w;
        if (!memchr(line, ' ', sl)) {
            memmove(p + w, line, sl);
            w += sl;
        } else {
            for (size_t q = 0; q < sl; ++q)
                if (line[q] != ' ') p[w++] = line[q];
        }
        out.cont += count_continuation(p + w0, w - w0);
    }
    out.len = w - a;
}

// Run f(t) for t in [0, n) on up to `threads` threads (the caller's thread included).
template <typename F>
void run_pool(size_t n, unsigned threads, F&& f) {
    if (n == 0) return;
    std::atomic<size_t> next{0};
    std::atomic<bool> oom{false};
    auto work = [&]() {
        try {
            for (size_t t; (t = next.fetch_add(1)) < n;) f(t);
        } catch (const std::bad_alloc&) {
            oom = true;
        }
    };
    std::vector<std::thread> pool;
    const unsigned nt = (unsigned)std::min<size_t>(n, std::max(1u, threads));
    for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    if (oom) throw std::bad_alloc();
}

// UTF-8 continuation bytes (10xxxxxx) of p[0, n): a record's character count, the length
// Python's len(str) reports for generate.py:44's short-record rule, is bytes minus these.
uint64_t count_continuation(const uint8_t* p, size_t n) {
    uint64_t c = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        c += (uint64_t)__builtin_popcountll(w & ~(w << 1) & 0x8080808080808080ull);
    }
    for (; i < n; ++i) c += (p[i] & 0xC0u) == 0x80u;
    return c;
}

// Records from the pieces in order: a piece's bytes before its first header continue the
// record open at its start (text before the file's first header belongs to none).  The
// pieces' outputs are moved down over the gaps (header lines, line ends) left between them,
// in order, inside the same buffer, which then holds every record back to back.
void stitch(std::vector<Piece>& pieces, const std::vector<size_t>& cut, uint8_t* buf, kmh_fasta& f) {
    uint64_t pos = 0, cont = 0;   // output end; continuation bytes of the open record
    bool in_record = false;
    auto move = [&](uint64_t from, uint64_t len) {
        if (from != pos && len) memmove(buf + pos, buf + from, len);
        pos += len;
    };
    auto close = [&]() {
        kmh_fasta::Rec& r = f.recs.back();
        r.seq_len = pos - r.seq_off;
        r.char_len = r.seq_len - cont;
    };
    for (size_t t = 0; t < pieces.size(); ++t) {
        const Piece& pc = pieces[t];
        const uint64_t base = cut[t];
        const uint64_t first = pc.hdrs.empty() ? pc.len : pc.hdrs[0].at;
        if (in_record) {
            move(base, first);
            cont += pc.hdrs.empty() ? pc.cont : pc.hdrs[0].cont_before;
        }
        for (size_t h = 0; h < pc.hdrs.size(); ++h) {
            if (in_record) close();
            in_record = true;
            kmh_fasta::Rec r{};
            r.id_off = f.ids.size();
            r.id_len = pc.hdrs[h].id.size();
            f.ids += pc.hdrs[h].id;
            r.seq_off = pos;
            f.recs.push_back(r);
            const bool last = h + 1 == pc.hdrs.size();
            const uint64_t end = last ? pc.len : pc.hdrs[h + 1].at;
            move(base + pc.hdrs[h].at, end - pc.hdrs[h].at);
            cont = (last ? pc.cont : pc.hdrs[h + 1].cont_before) - pc.hdrs[h].cont_before;
        }
    }
    if (in_record) close();
    f.nseq = pos;
}

}  // namespace

namespace {

// One line of k{k}.txt (generate.py:86-91): digits A=0 T=1 C=2 G=3, a tab, the count, a
// newline.  Writes it at o (when not null) and returns its length.
inline uint64_t format_line(int k, uint64_t code, uint64_t count, char* o) {
    static const char digit[4] = {'0', '2', '3', '1'};  // codes A C G T
    char num[24];
    int nd = 0;
    do {
        num[nd++] = (char)('0' + count % 10);
        count /= 10;
    } while (count);
    if (o) {
        for (int j = 0; j < k; ++j) o[j] = digit[(code >> (2 * (k - 1 - j))) & 3];
        o[k] = '\t';
        for (int d = 0; d < nd; ++d) o[k + 1 + d] = num[nd - 1 - d];
        o[k + 1 + nd] = '\n';
    }
    return (uint64_t)k + 2 + (uint64_t)nd;
}

}  // namespace

extern "C" {

int kmh_fasta_read(const char* path, kmh_fasta** out) {
    if (!path || !out) {
        kmh::set_thread_error("kmh_fasta_read: NULL argument");
        return KMH_ERR_INVALID;
    }
    *out = nullptr;
    FILE* fp = fopen(path, "rb");
    if (!fp) {
        kmh::set_thread_error(std::string("cannot open ") + path + ": " + strerror(errno));
        return KMH_ERR_IO;
    }
    // The file is read straight into one buffer of its size, by up to 16 threads with pread
    // (a page-cache copy); anything past that size (a file that grew, a pipe) is appended
    // from a chunked read.
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned max_threads = std::min(16u, hw);
    const bool prof = kmh::env_long("KMH_FASTA_PROF", 0) != 0;   // phase times on stderr
    auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = prof ? now() : 0.0;
    std::unique_ptr<uint8_t[], kmh_fasta::Free> whole;
    std::vector<uint8_t> more;
    size_t n = 0;
    try {
        long sz = -1;
        if (fseek(fp, 0, SEEK_END) == 0) {
            sz = ftell(fp);
            fseek(fp, 0, SEEK_SET);
        }
        if (sz > 0) {
            whole.reset(alloc_bytes((size_t)sz));
            const int fd = fileno(fp);
            const size_t blk = std::max<size_t>(1u << 22, ((size_t)sz + max_threads - 1) / max_threads);
            const size_t nblk = ((size_t)sz + blk - 1) / blk;
            std::vector<size_t> got(nblk, 0);
            run_pool(nblk, max_threads, [&](size_t b) {
                const size_t a0 = b * blk, e = std::min((size_t)sz, a0 + blk);
                size_t q = a0;
                while (q < e) {
                    const ssize_t r = pread(fd, whole.get() + q, e - q, (off_t)q);
                    if (r <= 0) break;
                    q += (size_t)r;
                }
                got[b] = q - a0;
            });
            bool full = true;
            for (size_t b = 0; b < nblk; ++b) full = full && got[b] == std::min((size_t)sz, (b + 1) * blk) - b * blk;
            n = full ? (size_t)sz : 0;   // a short read: read the whole file sequentially below
            if (fseek(fp, (long)n, SEEK_SET) != 0) n = 0;
        }
        uint8_t chunk[1 << 16];
        size_t got;
        while ((got = fread(chunk, 1, sizeof chunk, fp)) > 0) more.insert(more.end(), chunk, chunk + got);
        if (!more.empty() && n) more.insert(more.begin(), whole.get(), whole.get() + n);
    } catch (const std::bad_alloc&) {
        fclose(fp);
        kmh::set_thread_error("out of host memory reading FASTA");
        return KMH_ERR_NOMEM;
    }
    const bool read_error = ferror(fp) != 0;
    fclose(fp);
    if (read_error) {
        kmh::set_thread_error(std::string("read error on ") + path);
        return KMH_ERR_IO;
    }
    if (!more.empty()) {   // the parse works in place: the bytes go to one owned buffer
        n = more.size();
        whole.reset(alloc_bytes(n));
        memcpy(whole.get(), more.data(), n);
        more = std::vector<uint8_t>();
    }
    if (!whole) whole.reset(alloc_bytes(1));   // an empty file: records point into a valid buffer
    uint8_t* p = whole.get();

    std::unique_ptr<kmh_fasta> f(new (std::nothrow) kmh_fasta);
    if (!f) return KMH_ERR_NOMEM;
    try {
        // Pieces of max(4 MiB, n / threads) bytes (KMH_FASTA_CHUNK overrides: tests use tiny pieces), each
        // ending just after a '\n' -- always a line end, never inside "\r\n" -- parsed on up
        // to 16 threads, then stitched in order.
        const long env_chunk = kmh::env_long("KMH_FASTA_CHUNK", 0);
        const size_t cs = env_chunk > 0 ? (size_t)env_chunk
                                        : std::max<size_t>(4u << 20, (n + max_threads - 1) / max_threads);
        std::vector<size_t> cut{0};
        while (cut.back() < n) {
            size_t at = cut.back() + cs;
            if (at >= n) {
                cut.push_back(n);
                break;
            }
            const void* nl = memchr(p + at, '\n', n - at);
            cut.push_back(nl ? (size_t)(static_cast<const uint8_t*>(nl) - p) + 1 : n);
        }
        const size_t np = cut.size() - 1;
        std::vector<Piece> pieces(np);
        const double t1 = prof ? now() : 0.0;
        run_pool(np, max_threads, [&](size_t t) { parse_lines(p, cut[t], cut[t + 1], pieces[t]); });
        const double t2 = prof ? now() : 0.0;
        stitch(pieces, cut, p, *f);
        f->seqs = std::move(whole);
        if (prof)
            fprintf(stderr, "kmh_fasta_read: read %.4f s, parse %.4f s (%zu pieces), stitch %.4f s\n", t1 - t0,
                    t2 - t1, np, now() - t2);
    } catch (const std::bad_alloc&) {
        kmh::set_thread_error("out of host memory parsing FASTA");
        return KMH_ERR_NOMEM;
    }
    *out = f.release();
    return KMH_OK;
}

uint64_t kmh_fasta_count(const kmh_fasta* f) { return f ? f->recs.size() : 0; }

int kmh_fasta_record(const kmh_fasta* f, uint64_t i, const char** id, uint64_t* id_len,
                     const uint8_t** seq, uint64_t* seq_len, uint64_t* char_len) {
    if (!f || i >= f->recs.size()) {
        kmh::set_thread_error("kmh_fasta_record: bad handle or index");
        return KMH_ERR_INVALID;
    }
    const kmh_fasta::Rec& r = f->recs[i];
    if (id) *id = f->ids.data() + r.id_off;
    if (id_len) *id_len = r.id_len;
    if (seq) *seq = f->seqs.get() + r.seq_off;
    if (seq_len) *seq_len = r.seq_len;
    if (char_len) *char_len = r.char_len;
    return KMH_OK;
}

int kmh_fasta_pack(const kmh_fasta* f, uint64_t min_len, uint8_t* out, uint64_t cap,
                   uint64_t* out_len, uint8_t* kept) {
    if (!f || !out_len) {
        kmh::set_thread_error("kmh_fasta_pack: NULL argument");
        return KMH_ERR_INVALID;
    }
    uint64_t need = 0;
    for (size_t i = 0; i < f->recs.size(); ++i) {
        const bool keep = f->recs[i].char_len >= min_len;
        if (kept) kept[i] = keep ? 1 : 0;
        if (keep) need += f->recs[i].seq_len + 1;
    }
    *out_len = need;
    if (!out) return KMH_OK;
    if (cap < need) {
        kmh::set_thread_error("kmh_fasta_pack: output buffer too small");
        return KMH_ERR_INVALID;
    }
    uint8_t* o = out;
    for (const auto& r : f->recs) {
        if (r.char_len < min_len) continue;
        memcpy(o, f->seqs.get() + r.seq_off, r.seq_len);
        o += r.seq_len;
        *o++ = '\n';
    }
    return KMH_OK;
}

void kmh_fasta_free(kmh_fasta* f) { delete f; }

}  // extern "C"

namespace {

// Writes n lines with line(i, out) (out == NULL: return the length only) into out: blocks
// of lines are sized, prefix-summed and written on up to 16 threads (a k = 12 file is
// ~16.7 M lines, ~250 MB).  Returns the bytes the full text needs.
template <typename Line>
int64_t format_blocks(uint64_t n, char* out, uint64_t cap, Line&& line) {
    const uint64_t per = 1u << 18;
    const uint64_t nblk = n ? (n + per - 1) / per : 0;
    std::vector<uint64_t> start(nblk + 1, 0);
    const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({nblk, 16, std::max(1u, std::thread::hardware_concurrency())}));
    auto parallel = [&](auto&& body) {   // the line functions allocate nothing
        std::atomic<uint64_t> next{0};
        auto work = [&]() {
            for (uint64_t b = next++; b < nblk; b = next++) body(b);
        };
        std::vector<std::thread> pool;
        try {
            for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
        } catch (const std::system_error&) {   // fewer threads: the ones started finish the work
        }
        work();
        for (auto& t : pool) t.join();
    };
    parallel([&](uint64_t b) {
        uint64_t bytes = 0;
        for (uint64_t i = b * per, e = std::min(n, (b + 1) * per); i < e; ++i) bytes += line(i, nullptr);
        start[b + 1] = bytes;
    });
    for (uint64_t b = 0; b < nblk; ++b) start[b + 1] += start[b];
    const uint64_t total = start[nblk];
    if (out && total <= cap) {
        parallel([&](uint64_t b) {
            char* o = out + start[b];
            for (uint64_t i = b * per, e = std::min(n, (b + 1) * per); i < e; ++i) o += line(i, o);
        });
    } else if (out) {   // partial buffer: whole lines that fit, in order
        uint64_t pos = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t len = line(i, nullptr);
            if (pos + len <= cap) line(i, out + pos);
            pos += len;
        }
    }
    return (int64_t)total;
}

}  // namespace

extern "C" {

int64_t kmh_format_lines(int k, const uint64_t* codes, const uint64_t* counts, uint64_t n,
                         char* out, uint64_t cap) {
    if (k < 1 || k > 32 || (n && (!codes || !counts))) {
        kmh::set_thread_error("kmh_format_lines: bad arguments");
        return KMH_ERR_INVALID;
    }
    try {
        return format_blocks(n, out, cap, [&](uint64_t i, char* o) { return format_line(k, codes[i], counts[i], o); });
    } catch (const std::bad_alloc&) {
        kmh::set_thread_error("kmh_format_lines: out of host memory");
        return KMH_ERR_NOMEM;
    }
}

int64_t kmh_format_lines_seq(int k, const uint8_t* seq, uint64_t seq_len, const uint64_t* first,
                             const uint64_t* counts, uint64_t n, char* out, uint64_t cap) {
    if (k < 1 || (n && (!seq || !first || !counts))) {
        kmh::set_thread_error("kmh_format_lines_seq: bad arguments");
        return KMH_ERR_INVALID;
    }
    for (uint64_t i = 0; i < n; ++i)
        if (first[i] > seq_len || seq_len - first[i] < (uint64_t)k) {
            kmh::set_thread_error("kmh_format_lines_seq: a k-mer lies outside the sequence");
            return KMH_ERR_INVALID;
        }
    // digit of every byte that can start a counted window (either case); others never occur
    static const struct Tab {
        char d[256];
        Tab() {
            memset(d, '?', sizeof d);
            d['A'] = d['a'] = '0';
            d['T'] = d['t'] = '1';
            d['C'] = d['c'] = '2';
            d['G'] = d['g'] = '3';
        }
    } tab;
    try {
        return format_blocks(n, out, cap, [&](uint64_t i, char* o) -> uint64_t {
        uint64_t count = counts[i];
        char num[24];
        int nd = 0;
        do {
            num[nd++] = (char)('0' + count % 10);
            count /= 10;
        } while (count);
        if (o) {
            const uint8_t* w = seq + first[i];
            for (int j = 0; j < k; ++j) o[j] = tab.d[w[j]];
            o[k] = '\t';
            for (int d = 0; d < nd; ++d) o[k + 1 + d] = num[nd - 1 - d];
            o[k + 1 + nd] = '\n';
        }
        return (uint64_t)k + 2 + (uint64_t)nd;
        });
    } catch (const std::bad_alloc&) {
        kmh::set_thread_error("kmh_format_lines_seq: out of host memory");
        return KMH_ERR_NOMEM;
    }
}

}  // extern "C"
