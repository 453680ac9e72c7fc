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
#include <stdio.h>
#include <string.h>

#include <memory>
#include <new>
#include <string>
#include <vector>

#include <algorithm>
#include <atomic>
#include <thread>
#include "kmh_internal.h"

struct kmh_fasta {
    struct Rec {
        uint64_t id_off, id_len, seq_off, seq_len, char_len;
    };
    std::string ids;
    std::vector<uint8_t> seqs;
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
    std::vector<uint8_t> buf;
    try {
        if (fseek(fp, 0, SEEK_END) == 0) {
            const long sz = ftell(fp);
            if (sz > 0) buf.reserve((size_t)sz);
            fseek(fp, 0, SEEK_SET);
        }
        uint8_t chunk[1 << 16];
        size_t got;
        while ((got = fread(chunk, 1, sizeof chunk, fp)) > 0) buf.insert(buf.end(), chunk, chunk + got);
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

    std::unique_ptr<kmh_fasta> f(new (std::nothrow) kmh_fasta);
    if (!f) return KMH_ERR_NOMEM;
    try {
        f->seqs.reserve(buf.size());
        const uint8_t* p = buf.data();
        const size_t n = buf.size();
        size_t i = 0;
        bool in_record = false;
        kmh_fasta::Rec cur{};
        auto close_record = [&]() {
            cur.seq_len = f->seqs.size() - cur.seq_off;
            // characters = bytes that are not UTF-8 continuation bytes (a vectorised count)
            const uint8_t* sp = f->seqs.data() + cur.seq_off;
            uint64_t cont = 0;
            for (uint64_t q = 0, e = cur.seq_len; q < e; ++q) cont += (sp[q] & 0xC0u) == 0x80u;
            cur.char_len = cur.seq_len - cont;
            f->recs.push_back(cur);
        };
        while (i < n) {
            // line end: the first '\n' or '\r' (memchr: vectorised scans of ~80-byte lines)
            const void* nl = memchr(p + i, '\n', n - i);
            size_t j = nl ? (size_t)(static_cast<const uint8_t*>(nl) - p) : n;
            if (const void* cr = memchr(p + i, '\r', j - i)) j = (size_t)(static_cast<const uint8_t*>(cr) - p);
            const uint8_t* line = p + i;
            const size_t len = j - i;
            // advance past the line terminator (\r\n counts once)
            if (j < n && p[j] == '\r' && j + 1 < n && p[j + 1] == '\n') i = j + 2;
            else i = j + 1;
            if (len > 0 && line[0] == '>') {
                if (in_record) close_record();
                in_record = true;
                const size_t tl = rstrip_len(line + 1, len - 1);
                const uint8_t* t = line + 1;
                size_t a = 0;
                for (size_t w; a < tl && (w = leading_space(t + a, tl - a)) != 0;) a += w;
                size_t b = a;
                while (b < tl && leading_space(t + b, tl - b) == 0) ++b;
                cur = kmh_fasta::Rec{};
                cur.id_off = f->ids.size();
                cur.id_len = b - a;
                f->ids.append(reinterpret_cast<const char*>(t + a), b - a);
                cur.seq_off = f->seqs.size();
                continue;
            }
            if (!in_record) continue;  // text before the first record
            const size_t sl = rstrip_len(line, len);
            if (!memchr(line, ' ', sl)) {
                f->seqs.insert(f->seqs.end(), line, line + sl);
            } else {
                for (size_t q = 0; q < sl; ++q)
                    if (line[q] != ' ') f->seqs.push_back(line[q]);
            }
        }
        if (in_record) close_record();
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
    if (seq) *seq = f->seqs.data() + r.seq_off;
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
        memcpy(o, f->seqs.data() + r.seq_off, r.seq_len);
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
    auto parallel = [&](auto&& body) {
        std::atomic<uint64_t> next{0};
        auto work = [&]() {
            for (uint64_t b = next++; b < nblk; b = next++) body(b);
        };
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
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
    return format_blocks(n, out, cap, [&](uint64_t i, char* o) { return format_line(k, codes[i], counts[i], o); });
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
}

}  // extern "C"
