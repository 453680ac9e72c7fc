// kmh_csv.cpp -- the per-organism feature CSV text (row f4).
//
// The reference writes <organism>_kmer_features.csv with pandas (statistics.py:136-144:
// pd.DataFrame(all_features).to_csv(output_file, index=False)).  pandas prints an int64 column
// with str() and a float64 column with the shortest round-trip repr (numpy's, which follows
// Python's float repr: the shortest digits that read back to the same double; fixed notation
// for decimal exponents -4 < e <= 16, else d.ddde+XX).  Python repr costs ~2-4 us per value,
// ~18 s for the 4 M rows x 4 float columns of one dense k = 12 file.  Here the columns of a
// block of rows are formatted on up to 16 threads, each float by std::to_chars (shortest
// round trip, ties to the value nearest the double) re-laid in Python's notation.  Anything
// pandas would write differently (NaN / inf, a text field that needs quoting) is refused with
// KMH_ERR_UNSUPPORTED, and the caller writes that block with pandas itself.
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "kmh_internal.h"

struct kmh_text {
    std::unique_ptr<char[]> buf;
    size_t n = 0;
};

namespace {

// Python repr of a finite double (float_repr_style 'short'): the digits and exponent of the
// shortest round-trip scientific form, laid out the way Python's format_float_short does.
inline char* put_f64(char* o, double v) {
    char buf[48];
    auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
    const char* p = buf;
    if (*p == '-') {
        *o++ = '-';
        ++p;
    }
    char dig[24];
    int nd = 0;
    while (p < r.ptr && *p != 'e') {
        if (*p != '.') dig[nd++] = *p;
        ++p;
    }
    int e = 0;
    std::from_chars(p + 1 + (p[1] == '+'), r.ptr, e);
    const int decpt = e + 1;   // value = 0.d1d2... x 10^decpt
    if (decpt <= -4 || decpt > 16) {
        *o++ = dig[0];
        if (nd > 1) {
            *o++ = '.';
            std::memcpy(o, dig + 1, nd - 1);
            o += nd - 1;
        }
        *o++ = 'e';
        *o++ = e < 0 ? '-' : '+';
        int ae = e < 0 ? -e : e;
        if (ae >= 100) {
            *o++ = char('0' + ae / 100);
            ae %= 100;
        }
        *o++ = char('0' + ae / 10);
        *o++ = char('0' + ae % 10);
    } else if (decpt <= 0) {
        *o++ = '0';
        *o++ = '.';
        for (int i = 0; i < -decpt; ++i) *o++ = '0';
        std::memcpy(o, dig, nd);
        o += nd;
    } else if (decpt < nd) {
        std::memcpy(o, dig, decpt);
        o += decpt;
        *o++ = '.';
        std::memcpy(o, dig + decpt, nd - decpt);
        o += nd - decpt;
    } else {
        std::memcpy(o, dig, nd);
        o += nd;
        for (int i = nd; i < decpt; ++i) *o++ = '0';
        *o++ = '.';
        *o++ = '0';
    }
    return o;
}

inline char* put_i64(char* o, int64_t v) {
    return std::to_chars(o, o + 24, v).ptr;
}

inline char* put_u64(char* o, uint64_t v) {
    return std::to_chars(o, o + 24, v).ptr;
}

// The label the reference's statistics.py sees for an integer-parsed k-mer (statistics.py:
// 253-273 reads the digit column as int64, which drops leading zeros = A's; :157 / :248-251
// decode 0->A 1->T 2->C 3->G): the k-mer with its leading A's stripped, "A" for A...A.
inline char* put_label(char* o, uint64_t code, int k) {
    static const char kBase[4] = {'A', 'C', 'G', 'T'};
    int i = 0;
    while (i < k - 1 && ((code >> (2 * (k - 1 - i))) & 3) == 0) ++i;
    for (; i < k; ++i) *o++ = kBase[(code >> (2 * (k - 1 - i))) & 3];
    return o;
}

struct Col {
    int kind;
    const void* data;
    const void* aux;
};

// Upper bound of one row's text (KMH_CSV_STR: its field length).
size_t row_bound(const std::vector<Col>& cols, uint64_t r) {
    size_t n = 1;
    for (const Col& c : cols) {
        if (c.kind == KMH_CSV_STR) {
            const uint64_t* off = static_cast<const uint64_t*>(c.aux);
            n += off[r + 1] - off[r] + 1;
        } else if (c.kind == KMH_CSV_LABEL) {
            n += (size_t)*static_cast<const int64_t*>(c.aux) + 1;
        } else {
            n += 32;
        }
    }
    return n;
}

// Formats rows [lo, hi) into `out`; false if a value needs pandas' own writer.
bool format_rows(const std::vector<Col>& cols, uint64_t lo, uint64_t hi, std::string& out) {
    size_t bound = 0;
    bool var = false;
    for (const Col& c : cols) var |= c.kind == KMH_CSV_STR;
    if (var) {
        for (uint64_t r = lo; r < hi; ++r) bound += row_bound(cols, r);
    } else {
        bound = (hi - lo) * row_bound(cols, lo);
    }
    out.resize(bound);
    char* o = out.data();
    for (uint64_t r = lo; r < hi; ++r) {
        for (size_t j = 0; j < cols.size(); ++j) {
            const Col& c = cols[j];
            if (j) *o++ = ',';
            switch (c.kind) {
            case KMH_CSV_I64:
                o = put_i64(o, static_cast<const int64_t*>(c.data)[r]);
                break;
            case KMH_CSV_U64:
                o = put_u64(o, static_cast<const uint64_t*>(c.data)[r]);
                break;
            case KMH_CSV_F64: {
                const double v = static_cast<const double*>(c.data)[r];
                if (!(v - v == 0.0)) return false;   // NaN / inf: pandas writes "" / "inf"
                o = put_f64(o, v);
                break;
            }
            case KMH_CSV_STR: {
                const uint64_t* off = static_cast<const uint64_t*>(c.aux);
                const char* s = static_cast<const char*>(c.data) + off[r];
                const size_t len = off[r + 1] - off[r];
                // pandas (csv.QUOTE_MINIMAL) quotes a field holding the delimiter, a quote or a
                // line break, and an empty field of a text column is written as ""
                if (len == 0) return false;
                for (size_t i = 0; i < len; ++i)
                    if (s[i] == ',' || s[i] == '"' || s[i] == '\n' || s[i] == '\r') return false;
                std::memcpy(o, s, len);
                o += len;
                break;
            }
            case KMH_CSV_LABEL:
                o = put_label(o, static_cast<const uint64_t*>(c.data)[r],
                              (int)*static_cast<const int64_t*>(c.aux));
                break;
            }
        }
        *o++ = '\n';
    }
    out.resize(o - out.data());
    return true;
}

}  // namespace

extern "C" int kmh_csv_format(int ncols, const int32_t* kinds, const void* const* data,
                              const void* const* aux, uint64_t nrows, int threads, kmh_text** out) {
    if (!out || ncols < 0 || (ncols && (!kinds || !data || !aux))) {
        kmh::set_thread_error("kmh_csv_format: bad arguments");
        return KMH_ERR_INVALID;
    }
    *out = nullptr;
    std::vector<Col> cols;
    for (int j = 0; j < ncols; ++j) {
        const int kind = kinds[j];
        if (kind < KMH_CSV_I64 || kind > KMH_CSV_U64 || (nrows && !data[j]) ||
            ((kind == KMH_CSV_STR || kind == KMH_CSV_LABEL) && !aux[j])) {
            kmh::set_thread_error("kmh_csv_format: bad column " + std::to_string(j));
            return KMH_ERR_INVALID;
        }
        if (kind == KMH_CSV_LABEL) {
            const int64_t k = *static_cast<const int64_t*>(aux[j]);
            if (k < 1 || k > 32) {
                kmh::set_thread_error("kmh_csv_format: label column needs 1 <= k <= 32");
                return KMH_ERR_INVALID;
            }
        }
        cols.push_back({kind, data[j], aux[j]});
    }
    try {
        constexpr uint64_t kRows = 1u << 16;   // rows per piece
        const uint64_t npiece = nrows ? (nrows + kRows - 1) / kRows : 0;
        unsigned nt = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
        nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({nt ? nt : 1u, 16u, npiece ? npiece : 1}));
        std::vector<std::string> piece(npiece);
        std::atomic<uint64_t> next{0};
        std::atomic<bool> ok{true}, oom{false};
        auto work = [&]() {
            try {
                for (uint64_t p = next++; p < npiece && ok; p = next++)
                    if (!format_rows(cols, p * kRows, std::min(nrows, (p + 1) * kRows), piece[p])) ok = false;
            } catch (const std::bad_alloc&) {
                oom = true;
                ok = false;
            }
        };
        std::vector<std::thread> pool;
        try {
            for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
        } catch (const std::system_error&) {   // fewer threads: the ones started finish the work
        }
        work();
        for (auto& t : pool) t.join();
        if (oom) {
            kmh::set_thread_error("kmh_csv_format: out of host memory");
            return KMH_ERR_NOMEM;
        }
        if (!ok) {
            kmh::set_thread_error("kmh_csv_format: a value pandas writes differently (NaN, inf, or text that "
                                  "needs quoting)");
            return KMH_ERR_UNSUPPORTED;
        }
        // one contiguous text: every piece copied to its offset, in parallel
        std::vector<size_t> at(npiece + 1, 0);
        for (uint64_t p = 0; p < npiece; ++p) at[p + 1] = at[p] + piece[p].size();
        std::unique_ptr<kmh_text> t(new kmh_text);
        t->n = at[npiece];
        t->buf.reset(new char[std::max<size_t>(t->n, 1)]);
        next = 0;
        auto copy = [&]() {
            for (uint64_t p = next++; p < npiece; p = next++) {
                std::memcpy(t->buf.get() + at[p], piece[p].data(), piece[p].size());
                std::string().swap(piece[p]);
            }
        };
        pool.clear();
        try {
            for (unsigned q = 1; q < nt; ++q) pool.emplace_back(copy);
        } catch (const std::system_error&) {
        }
        copy();
        for (auto& q : pool) q.join();
        *out = t.release();
        return KMH_OK;
    } catch (const std::bad_alloc&) {
        kmh::set_thread_error("kmh_csv_format: out of host memory");
        return KMH_ERR_NOMEM;
    }
}

extern "C" int kmh_text_data(const kmh_text* t, const char** data, uint64_t* len) {
    if (!t) {
        kmh::set_thread_error("kmh_text_data: NULL text");
        return KMH_ERR_INVALID;
    }
    if (data) *data = t->buf.get();
    if (len) *len = t->n;
    return KMH_OK;
}

extern "C" void kmh_text_free(kmh_text* t) {
    delete t;
}
