// cc_n5.cpp -- native N5 chunk codec (host C++, zlib): libcc_n5.so, include/cc_n5.h.  Host only,
// no HIP: it is built and loaded apart from the device library, so reading a dataset never
// brings up a GPU runtime (one HIP runtime per process: torch's, which libcc_mi355x binds to).
//
// The reference reads and writes every dataset of the path through elf.io.open_file -> z5py
// (C++): cluster_tools/utils/volume_utils.py:21-22 (file_reader), ds_in[bb] / ds_out[bb] in
// block_components.py:151,180, the uint64 output created with chunks = block_shape // 2 and gzip
// (block_components.py:99-106), the assignments LUT (merge_assignments.py:136-139) and the
// in-place write (write.py:84-91,185-202).  z5py is not vendored in /root/reference; this follows
// the N5 specification (byte-layout parity unpinned):
//   chunk file <dataset>/<i_fastest>/.../<i_slowest>; header big-endian u16 mode (0 default,
//   1 varlength: + u32 element count), u16 ndim, u32 dims[ndim] fastest first; payload the
//   big-endian C-order elements, raw or gzip (zlib windowBits 31 on write, 47 = gzip or zlib
//   auto-detected on read); a missing chunk reads as the fill value 0.
//
// A region read / write fans the chunks it touches out over n_threads host threads (each
// chunk: file read, inflate, byte swap into the caller's C-order box -- or the reverse), the
// work the Python reference did one chunk at a time under z5py.
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <stdint.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cc_n5.h"

static thread_local std::string g_err;

namespace cc_n5 {

struct Spec {
    int ndim = 0;
    int64_t shape[4] = {0, 0, 0, 0}, chunks[4] = {0, 0, 0, 0};
    int64_t begin[4] = {0, 0, 0, 0}, end[4] = {0, 0, 0, 0};
    int esize = 0;           // element size in bytes (1, 2, 4, 8)
    int compression = 0;     // 0 raw, 1 gzip
    int level = 5;
};

struct Errors {
    std::mutex m;
    std::string first;
    std::atomic<bool> any{false};
    void set(const std::string& e) {
        std::lock_guard<std::mutex> g(m);
        if (first.empty()) first = e;
        any = true;
    }
};

static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static inline void put16(std::vector<uint8_t>& v, uint16_t x) { v.push_back(x >> 8); v.push_back(x & 0xFF); }
static inline void put32(std::vector<uint8_t>& v, uint32_t x) {
    for (int s = 24; s >= 0; s -= 8) v.push_back((x >> s) & 0xFF);
}

// copy n elements swapping their byte order (big-endian file <-> little-endian host)
static inline void swap_copy(uint8_t* dst, const uint8_t* src, int64_t n, int es) {
    switch (es) {
        case 1: std::memcpy(dst, src, n); break;
        case 2: for (int64_t i = 0; i < n; ++i) { uint16_t v; std::memcpy(&v, src + 2 * i, 2); v = __builtin_bswap16(v); std::memcpy(dst + 2 * i, &v, 2); } break;
        case 4: for (int64_t i = 0; i < n; ++i) { uint32_t v; std::memcpy(&v, src + 4 * i, 4); v = __builtin_bswap32(v); std::memcpy(dst + 4 * i, &v, 4); } break;
        default: for (int64_t i = 0; i < n; ++i) { uint64_t v; std::memcpy(&v, src + 8 * i, 8); v = __builtin_bswap64(v); std::memcpy(dst + 8 * i, &v, 8); } break;
    }
}

static std::string chunk_path(const std::string& ds, const Spec& s, const int64_t* cid) {
    std::string p = ds;
    for (int a = s.ndim - 1; a >= 0; --a) p += "/" + std::to_string(cid[a]);
    return p;
}

static void mkdirs(const std::string& dir) {
    if (dir.empty()) return;
    struct stat st;
    if (::stat(dir.c_str(), &st) == 0) return;
    const size_t k = dir.find_last_of('/');
    if (k != std::string::npos && k > 0) mkdirs(dir.substr(0, k));
    if (::mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST) throw std::runtime_error("mkdir " + dir + ": " + std::strerror(errno));
}

static bool read_file(const std::string& p, std::vector<uint8_t>& buf) {
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) {
        if (errno == ENOENT) return false;
        throw std::runtime_error("open " + p + ": " + std::strerror(errno));
    }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.resize(n > 0 ? (size_t)n : 0);
    const size_t got = n > 0 ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
    std::fclose(f);
    if ((long)got != n) throw std::runtime_error("short read " + p);
    return true;
}

static void inflate_all(const uint8_t* src, size_t n, uint8_t* dst, size_t want, const std::string& p) {
    z_stream z;
    std::memset(&z, 0, sizeof(z));
    if (inflateInit2(&z, 47) != Z_OK) throw std::runtime_error("inflateInit2 failed");
    z.next_in = const_cast<uint8_t*>(src);
    z.avail_in = (uInt)n;
    z.next_out = dst;
    z.avail_out = (uInt)want;
    const int rc = inflate(&z, Z_FINISH);
    const size_t got = want - z.avail_out;
    inflateEnd(&z);
    if (rc != Z_STREAM_END || got != want) throw std::runtime_error("corrupt gzip chunk " + p);
}

// chunk box of chunk id cid: [cb, ce)
static void chunk_box(const Spec& s, const int64_t* cid, int64_t* cb, int64_t* ce) {
    for (int a = 0; a < s.ndim; ++a) {
        cb[a] = cid[a] * s.chunks[a];
        ce[a] = std::min(cb[a] + s.chunks[a], s.shape[a]);
    }
}

// visit every row (contiguous run along the last axis) of the intersection of the region with
// the chunk box: f(offset of the row in the region, offset in the chunk array of dims cd, length)
template <class F>
static void for_rows(const Spec& s, const int64_t* cb, const int64_t* ce, const int64_t* cd, F&& f) {
    int64_t lo[4], hi[4];
    for (int a = 0; a < s.ndim; ++a) {
        lo[a] = std::max(s.begin[a], cb[a]);
        hi[a] = std::min(s.end[a], ce[a]);
        if (hi[a] <= lo[a]) return;
    }
    const int L = s.ndim - 1;
    int64_t idx[4] = {0, 0, 0, 0};
    for (int a = 0; a < L; ++a) idx[a] = lo[a];
    while (true) {
        int64_t ro = 0, co = 0;
        for (int a = 0; a < s.ndim; ++a) {
            const int64_t i = a == L ? lo[a] : idx[a];
            ro = ro * (s.end[a] - s.begin[a]) + (i - s.begin[a]);
            co = co * cd[a] + (i - cb[a]);
        }
        f(ro, co, hi[L] - lo[L]);
        int a = L - 1;
        for (; a >= 0; --a) {
            if (++idx[a] < hi[a]) break;
            idx[a] = lo[a];
        }
        if (a < 0) break;
    }
}

// ids of the chunks the region touches, C order
static std::vector<std::array<int64_t, 4>> region_chunks(const Spec& s) {
    int64_t c0[4] = {0, 0, 0, 0}, c1[4] = {1, 1, 1, 1};
    for (int a = 0; a < s.ndim; ++a) {
        if (s.end[a] <= s.begin[a]) return {};
        c0[a] = s.begin[a] / s.chunks[a];
        c1[a] = (s.end[a] - 1) / s.chunks[a] + 1;
    }
    std::vector<std::array<int64_t, 4>> ids;
    std::array<int64_t, 4> c = {c0[0], c0[1], c0[2], c0[3]};
    while (true) {
        ids.push_back(c);
        int a = s.ndim - 1;
        for (; a >= 0; --a) {
            if (++c[a] < c1[a]) break;
            c[a] = c0[a];
        }
        if (a < 0) break;
    }
    return ids;
}

// decode one chunk file into `arr` (C order, dims cd); returns false if the chunk is missing
static bool decode_chunk(const std::string& p, const Spec& s, std::vector<uint8_t>& file, std::vector<uint8_t>& arr,
                         int64_t* cd) {
    if (!read_file(p, file)) return false;
    if (file.size() < 4) throw std::runtime_error("truncated chunk header " + p);
    const uint16_t mode = be16(file.data()), nd = be16(file.data() + 2);
    if (mode > 1) throw std::runtime_error("unsupported chunk mode " + std::to_string(mode) + " " + p);
    if (nd != s.ndim) throw std::runtime_error("chunk ndim mismatch " + p);
    size_t off = 4 + 4 * (size_t)nd + (mode == 1 ? 4 : 0);
    if (file.size() < off) throw std::runtime_error("truncated chunk header " + p);
    // the header is untrusted: every dim bounded by the dataset's chunk size (so the product
    // cannot overflow), and a varlength (mode 1) element count must equal that product -- the
    // caller indexes the decoded array with these dims
    int64_t n = 1;
    for (int a = 0; a < nd; ++a) {
        const int64_t d = be32(file.data() + 4 + 4 * a);     // header dims fastest first
        if (d > s.chunks[nd - 1 - a]) throw std::runtime_error("chunk dims exceed the dataset's chunk size " + p);
        cd[nd - 1 - a] = d;
        n *= d;
    }
    if (mode == 1 && (int64_t)be32(file.data() + 4 + 4 * nd) != n)
        throw std::runtime_error("varlength chunk element count differs from its dims " + p);
    const size_t bytes = (size_t)n * s.esize;
    std::vector<uint8_t> raw;
    const uint8_t* payload = file.data() + off;
    if (s.compression == 1) {
        raw.resize(bytes);
        inflate_all(payload, file.size() - off, raw.data(), bytes, p);
        payload = raw.data();
    } else if (file.size() - off < bytes) {
        throw std::runtime_error("truncated raw chunk " + p);
    }
    arr.resize(bytes);
    swap_copy(arr.data(), payload, n, s.esize);
    return true;
}

static void encode_chunk(const std::string& p, const Spec& s, const uint8_t* arr, const int64_t* cd) {
    int64_t n = 1;
    for (int a = 0; a < s.ndim; ++a) n *= cd[a];
    std::vector<uint8_t> be((size_t)n * s.esize);
    swap_copy(be.data(), arr, n, s.esize);
    std::vector<uint8_t> out;
    out.reserve(64);
    put16(out, 0);
    put16(out, (uint16_t)s.ndim);
    for (int a = s.ndim - 1; a >= 0; --a) put32(out, (uint32_t)cd[a]);
    const size_t head = out.size();
    if (s.compression == 1) {
        z_stream z;
        std::memset(&z, 0, sizeof(z));
        if (deflateInit2(&z, s.level, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY) != Z_OK)
            throw std::runtime_error("deflateInit2 failed");
        const uLong bound = deflateBound(&z, (uLong)be.size());
        out.resize(head + bound);
        z.next_in = be.data();
        z.avail_in = (uInt)be.size();
        z.next_out = out.data() + head;
        z.avail_out = (uInt)bound;
        const int rc = deflate(&z, Z_FINISH);
        const size_t got = bound - z.avail_out;
        deflateEnd(&z);
        if (rc != Z_STREAM_END) throw std::runtime_error("deflate failed " + p);
        out.resize(head + got);
    } else {
        out.insert(out.end(), be.begin(), be.end());
    }
    const size_t k = p.find_last_of('/');
    mkdirs(p.substr(0, k));
    // unique per process AND thread: thread ids repeat across processes (ranks of the sharded
    // job, concurrent local jobs writing one dataset)
    const std::string tmp = p + ".tmp" + std::to_string((long long)::getpid()) + "_" +
                            std::to_string((unsigned long long)std::hash<std::thread::id>()(std::this_thread::get_id()));
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw std::runtime_error("open " + tmp + ": " + std::strerror(errno));
    const size_t w = std::fwrite(out.data(), 1, out.size(), f);
    const int cl = std::fclose(f);
    if (w != out.size() || cl != 0) throw std::runtime_error("write " + tmp + " failed");
    if (std::rename(tmp.c_str(), p.c_str()) != 0) throw std::runtime_error("rename " + tmp + ": " + std::strerror(errno));
}

template <class F>
static void parallel_chunks(size_t n, int n_threads, Errors& err, F&& f) {
    std::atomic<size_t> next{0};
    auto worker = [&] {
        std::vector<uint8_t> file, arr;
        for (size_t i; !err.any && (i = next.fetch_add(1)) < n;) {
            try {
                f(i, file, arr);
            } catch (const std::exception& e) {
                err.set(e.what());
            }
        }
    };
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, n_threads), n));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(worker);
    worker();
    for (auto& t : pool) t.join();
}

// region read: out is the C-order region [begin, end) (missing chunks read as 0)
static void read_region(const std::string& ds, const Spec& s, uint8_t* out, int n_threads) {
    const auto ids = region_chunks(s);
    Errors err;
    parallel_chunks(ids.size(), n_threads, err, [&](size_t i, std::vector<uint8_t>& file, std::vector<uint8_t>& arr) {
        int64_t cb[4], ce[4], cd[4];
        chunk_box(s, ids[i].data(), cb, ce);
        const int L = s.ndim - 1;
        if (!decode_chunk(chunk_path(ds, s, ids[i].data()), s, file, arr, cd)) {
            for_rows(s, cb, ce, cd, [&](int64_t ro, int64_t, int64_t n) { std::memset(out + ro * s.esize, 0, n * s.esize); });
            return;
        }
        // an edge chunk may be stored full size (dims >= the truncated box): read its top corner
        for (int a = 0; a < s.ndim; ++a)
            if (cd[a] < ce[a] - cb[a]) throw std::runtime_error("chunk smaller than its box");
        (void)L;
        for_rows(s, cb, ce, cd, [&](int64_t ro, int64_t co, int64_t n) {
            std::memcpy(out + ro * s.esize, arr.data() + co * s.esize, n * s.esize);
        });
    });
    if (err.any) throw std::runtime_error(err.first);
}

// region write: chunks the region covers completely are encoded from `in`; partially covered
// ones are read, merged and rewritten.  skip_zero: an all-zero chunk with no file on disk is
// not written (the reference never writes empty blocks: block_components.py:175-177,
// write.py:194-197, so those chunks stay absent and read as the fill value).
static void write_region(const std::string& ds, const Spec& s, const uint8_t* in, int n_threads, bool skip_zero) {
    const auto ids = region_chunks(s);
    Errors err;
    parallel_chunks(ids.size(), n_threads, err, [&](size_t i, std::vector<uint8_t>& file, std::vector<uint8_t>& arr) {
        int64_t cb[4], ce[4], cd[4];
        chunk_box(s, ids[i].data(), cb, ce);
        bool full = true;
        int64_t n = 1;
        for (int a = 0; a < s.ndim; ++a) {
            full &= s.begin[a] <= cb[a] && s.end[a] >= ce[a];
            cd[a] = ce[a] - cb[a];
            n *= cd[a];
        }
        const std::string p = chunk_path(ds, s, ids[i].data());
        bool exists = true;
        if (full) {
            arr.resize((size_t)n * s.esize);
        } else {
            int64_t od[4];
            exists = decode_chunk(p, s, file, arr, od);
            bool same = exists;
            for (int a = 0; a < s.ndim && same; ++a) same = od[a] == cd[a];
            // an edge chunk may be stored full size (dims >= the truncated box), never smaller
            for (int a = 0; a < s.ndim && exists; ++a)
                if (od[a] < cd[a]) throw std::runtime_error("chunk smaller than its box " + p);
            if (!same) {     // absent, or stored full size at an edge: rebuild in the truncated shape
                std::vector<uint8_t> t((size_t)n * s.esize, 0);
                if (exists) {
                    Spec q = s;
                    for (int a = 0; a < s.ndim; ++a) { q.begin[a] = cb[a]; q.end[a] = ce[a]; }
                    for_rows(q, cb, ce, od, [&](int64_t ro, int64_t co, int64_t m) {
                        std::memcpy(t.data() + ro * s.esize, arr.data() + co * s.esize, m * s.esize);
                    });
                }
                arr.swap(t);
            }
        }
        for_rows(s, cb, ce, cd, [&](int64_t ro, int64_t co, int64_t m) {
            std::memcpy(arr.data() + co * s.esize, in + ro * s.esize, m * s.esize);
        });
        if (skip_zero) {
            bool zero = true;
            for (size_t k = 0; k < arr.size() && zero; ++k) zero = arr[k] == 0;
            if (zero) {
                struct stat st;
                if (full) exists = ::stat(p.c_str(), &st) == 0;
                if (!exists) return;
            }
        }
        encode_chunk(p, s, arr.data(), cd);
    });
    if (err.any) throw std::runtime_error(err.first);
}

static Spec make_spec(int ndim, const int64_t* shape, const int64_t* chunks, int esize, int compression, int level,
                      const int64_t* begin, const int64_t* end) {
    if (ndim < 1 || ndim > 4) throw std::runtime_error("n5: ndim must be 1..4");
    if (esize != 1 && esize != 2 && esize != 4 && esize != 8) throw std::runtime_error("n5: element size must be 1, 2, 4 or 8");
    if (compression != 0 && compression != 1) throw std::runtime_error("n5: compression must be 0 (raw) or 1 (gzip)");
    Spec s;
    s.ndim = ndim;
    s.esize = esize;
    s.compression = compression;
    s.level = level;
    for (int a = 0; a < ndim; ++a) {
        s.shape[a] = shape[a];
        s.chunks[a] = chunks[a];
        s.begin[a] = begin ? begin[a] : 0;
        s.end[a] = end ? end[a] : shape[a];
        if (chunks[a] <= 0 || shape[a] < 0 || s.begin[a] < 0 || s.end[a] > shape[a] || s.begin[a] > s.end[a])
            throw std::runtime_error("n5: bad shape / chunks / region");
    }
    return s;
}

}  // namespace cc_n5

extern "C" {

#ifndef CC_SRC_HASH
#define CC_SRC_HASH "unknown"
#endif
const char* cc_n5_version(void) { return "cc_n5 0.2 src=" CC_SRC_HASH; }

const char* cc_n5_last_error(void) { return g_err.c_str(); }

int cc_n5_read(const char* dataset_path, int ndim, const int64_t* shape, const int64_t* chunks, int elem_size,
               int compression, const int64_t* begin, const int64_t* end, void* out, int n_threads) {
    try {
        if (!dataset_path || !shape || !chunks || !out) throw std::runtime_error("NULL argument");
        const cc_n5::Spec s = cc_n5::make_spec(ndim, shape, chunks, elem_size, compression, 5, begin, end);
        cc_n5::read_region(dataset_path, s, (uint8_t*)out, n_threads);
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int cc_n5_write(const char* dataset_path, int ndim, const int64_t* shape, const int64_t* chunks, int elem_size,
                int compression, int level, const int64_t* begin, const int64_t* end, const void* in, int n_threads,
                int skip_zero_chunks) {
    try {
        if (!dataset_path || !shape || !chunks || !in) throw std::runtime_error("NULL argument");
        const cc_n5::Spec s = cc_n5::make_spec(ndim, shape, chunks, elem_size, compression, level, begin, end);
        cc_n5::write_region(dataset_path, s, (const uint8_t*)in, n_threads, skip_zero_chunks != 0);
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

}  // extern "C"
