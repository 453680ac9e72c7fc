// kmh_io.cpp -- file output of the k{k}.txt text (generate.py:68-91).
//
// The reference writes gzip with Python's gzip module at level 9 (generate.py:82-85) on one
// core, the slowest stage of its pipeline at k = 12.  Here the text is
// cut into blocks that are deflated concurrently, each as a complete gzip member; the members
// are written in order.  A gzip file may hold several members and decompresses to their
// concatenation (RFC 1952 section 2.2), so every reader sees the same text.  The compressed
// bytes differ from the reference's, which embed a timestamp and are not reproducible anyway.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "kmh_internal.h"

namespace {

bool deflate_member(const uint8_t* src, size_t n, int level, std::vector<uint8_t>& out) {
    z_stream z{};
    // windowBits 15 + 16: gzip wrapper (header with mtime 0, CRC-32 and length trailer)
    if (deflateInit2(&z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    // Level 9 with a short match chain (good 4, lazy 16, nice 64, chain 32 instead of 32 / 258 /
    // 258 / 4096): on k-mer text -- sorted, highly repetitive lines -- zlib's level-9 chains search
    // long and find nothing better; these settings compress an 8 MiB k = 12 block to 21.7 % of the
    // text instead of 22.1 %, 14x faster (1.9 -> 26 MB/s per thread, round 5), so the class
    // default compress=True stops being the drop-in's slowest stage.
    if (level == 9 && deflateTune(&z, 4, 16, 64, 32) != Z_OK) {
        deflateEnd(&z);
        return false;
    }
    out.resize(deflateBound(&z, (uLong)n) + 64);
    z.next_in = const_cast<Bytef*>(src);
    z.avail_in = (uInt)n;
    z.next_out = out.data();
    z.avail_out = (uInt)out.size();
    const int r = deflate(&z, Z_FINISH);
    out.resize(out.size() - z.avail_out);
    deflateEnd(&z);
    return r == Z_STREAM_END;
}

}  // namespace

extern "C" int kmh_write_file(const char* path, const void* data, uint64_t n, int gzip_level,
                              int threads) {
    if (!path || (n && !data)) {
        kmh::set_thread_error("kmh_write_file: NULL argument");
        return KMH_ERR_INVALID;
    }
    if (gzip_level > 9) {
        kmh::set_thread_error("kmh_write_file: gzip level must be <= 9");
        return KMH_ERR_INVALID;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        kmh::set_thread_error(std::string("cannot open ") + path + " for writing");
        return KMH_ERR_IO;
    }
    const uint8_t* src = static_cast<const uint8_t*>(data);
    bool ok = true;
    if (gzip_level < 0) {
        ok = n == 0 || std::fwrite(src, 1, n, f) == n;
    } else {
        constexpr size_t kBlock = 2u << 20;   // 2 MiB of text per member (k = 9..11 files keep the threads busy too)
        const size_t nblk = n ? (n + kBlock - 1) / kBlock : 1;
        unsigned nt = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
        nt = std::max(1u, std::min<unsigned>({nt, 16u, (unsigned)nblk}));
        std::atomic<bool> good{true}, oom{false};
        try {
            std::vector<std::vector<uint8_t>> out(nblk);
            std::atomic<size_t> next{0};
            auto work = [&]() {   // a worker never lets an exception escape its thread
                try {
                    for (size_t b = next++; b < nblk; b = next++) {
                        const size_t lo = b * kBlock, len = std::min(kBlock, (size_t)n - lo);
                        if (!deflate_member(src + lo, n ? len : 0, gzip_level, out[b])) good = false;
                    }
                } catch (const std::bad_alloc&) {
                    oom = true;
                    good = false;
                }
            };
            std::vector<std::thread> pool;
            try {
                for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
            } catch (const std::system_error&) {   // fewer threads: the ones started finish the work
            }
            work();
            for (auto& t : pool) t.join();
            ok = good;
            for (size_t b = 0; ok && b < nblk; ++b)
                ok = out[b].empty() || std::fwrite(out[b].data(), 1, out[b].size(), f) == out[b].size();
        } catch (const std::bad_alloc&) {
            oom = true;
            ok = false;
        }
        if (oom) {
            std::fclose(f);
            kmh::set_thread_error(std::string("out of host memory writing ") + path);
            return KMH_ERR_NOMEM;
        }
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        kmh::set_thread_error(std::string("error writing ") + path);
        return KMH_ERR_IO;
    }
    return KMH_OK;
}
