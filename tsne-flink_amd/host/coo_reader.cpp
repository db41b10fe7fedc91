// coo_reader.cpp -- parallel mmap reader of the reference's COO CSV input
// (Tsne.scala:138-159); see coo_reader.hpp.
#include "coo_reader.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <unordered_map>

namespace tsne_flink {
namespace {

struct Chunk {
    CooTriples t;
    std::string err;
};

// "[-+]digits" -> int64, advances p; false if no digits
bool parseInt(const char *&p, const char *end, long long &out) {
    bool neg = false;
    if (p < end && (*p == '-' || *p == '+')) { neg = *p == '-'; ++p; }
    const char *s = p;
    long long v = 0;
    while (p < end && *p >= '0' && *p <= '9') {
        v = v * 10 + (*p - '0');
        if (v > (1ll << 40)) return false;
        ++p;
    }
    if (p == s) return false;
    out = neg ? -v : v;
    return true;
}

void parseRange(const char *b, const char *e, Chunk &c) {
    // rough reservation: ~24 bytes per line
    const size_t guess = (size_t)(e - b) / 24 + 16;
    c.t.i.reserve(guess); c.t.j.reserve(guess); c.t.v.reserve(guess);
    char num[128];
    const char *p = b;
    while (p < e) {
        const char *eol = static_cast<const char *>(std::memchr(p, '\n', (size_t)(e - p)));
        if (!eol) eol = e;
        const char *le = eol;
        if (le > p && le[-1] == '\r') --le;
        if (le > p) {
            const char *q = p;
            long long i = 0, j = 0;
            bool ok = parseInt(q, le, i) && q < le && *q == ',';
            if (ok) { ++q; ok = parseInt(q, le, j) && q < le && *q == ','; }
            double v = 0.0;
            if (ok) {
                ++q;
                // std::from_chars (correctly rounded, ~3x faster than strtod
                // here); strtod for what it does not take whole ('+', hex,
                // inf / nan, out-of-range values): the same doubles either way
                const std::from_chars_result fr = std::from_chars(q, le, v);
                if (!(fr.ec == std::errc() && fr.ptr == le)) {
                    const size_t n = (size_t)(le - q);
                    ok = n > 0 && n < sizeof(num);
                    if (ok) {
                        std::memcpy(num, q, n);
                        num[n] = 0;
                        char *ep = nullptr;
                        v = std::strtod(num, &ep);
                        ok = ep != num && *ep == 0;
                    }
                }
            }
            if (!ok || i < INT32_MIN || i > INT32_MAX || j < INT32_MIN || j > INT32_MAX) {
                c.err = "bad line: " + std::string(p, le);
                return;
            }
            c.t.i.push_back((int32_t)i);
            c.t.j.push_back((int32_t)j);
            c.t.v.push_back(v);
        }
        p = eol + 1;
    }
}


// buf[0..len) parsed by `threads` threads into per-thread chunks (file order)
std::vector<Chunk> parseChunks(const char *buf, size_t len, int threads) {
    if (threads <= 0) threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (len < (1u << 20)) threads = 1;
    std::vector<size_t> cut(threads + 1, len);
    cut[0] = 0;
    for (int t = 1; t < threads; ++t) {   // advance each cut to just past a newline
        size_t c = len * (size_t)t / (size_t)threads;
        c = std::max(c, cut[t - 1]);
        const void *nl = c < len ? std::memchr(buf + c, '\n', len - c) : nullptr;
        cut[t] = nl ? (size_t)(static_cast<const char *>(nl) - buf) + 1 : len;
    }
    std::vector<Chunk> ch(threads);
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t)
        pool.emplace_back([&, t] { parseRange(buf + cut[t], buf + cut[t + 1], ch[t]); });
    parseRange(buf + cut[0], buf + cut[1], ch[0]);
    for (auto &th : pool) th.join();
    for (auto &c : ch)
        if (!c.err.empty()) throw std::runtime_error(c.err);
    return ch;
}

// the file mapped read-only for the duration of f(buf, len)
template <class F> void withMappedFile(const std::string &path, F &&f) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd, &st) != 0) { ::close(fd); throw std::runtime_error("cannot stat " + path); }
    const size_t len = (size_t)st.st_size;
    if (len == 0) { ::close(fd); f(static_cast<const char *>(nullptr), (size_t)0); return; }
    void *m = ::mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) throw std::runtime_error("cannot mmap " + path);
    (void)::madvise(m, len, MADV_SEQUENTIAL);
    try {
        f(static_cast<const char *>(m), len);
    } catch (...) {
        ::munmap(m, len);
        throw;
    }
    ::munmap(m, len);
}

}  // namespace

CooTriples parseCoo(const char *buf, size_t len, int threads) {
    std::vector<Chunk> ch = parseChunks(buf, len, threads);
    CooTriples out;
    size_t total = 0;
    for (auto &c : ch) total += c.t.i.size();
    out.i.reserve(total); out.j.reserve(total); out.v.reserve(total);
    for (auto &c : ch) {   // file order
        out.i.insert(out.i.end(), c.t.i.begin(), c.t.i.end());
        out.j.insert(out.j.end(), c.t.j.begin(), c.t.j.end());
        out.v.insert(out.v.end(), c.t.v.begin(), c.t.v.end());
    }
    return out;
}

CooTriples readCooFile(const std::string &path, int threads) {
    CooTriples t;
    withMappedFile(path, [&](const char *buf, size_t len) {
        if (len) t = parseCoo(buf, len, threads);
    });
    return t;
}

void readInputDense(const std::string &path, int dimension, std::vector<int32_t> &ids, std::vector<double> &X,
                    int threads) {
    std::vector<Chunk> ch;
    withMappedFile(path, [&](const char *buf, size_t len) {
        if (len) ch = parseChunks(buf, len, threads);
    });
    const int T = (int)ch.size();
    size_t m = 0;
    int64_t lo = 0, hi = -1;
    for (auto &c : ch) {
        m += c.t.i.size();
        for (size_t e = 0; e < c.t.i.size(); ++e) {
            lo = std::min<int64_t>(lo, c.t.i[e]);
            hi = std::max<int64_t>(hi, c.t.i[e]);
            if (c.t.j[e] < 0 || c.t.j[e] >= dimension)
                throw std::out_of_range("index " + std::to_string(c.t.j[e]) + " out of dimension");
        }
    }
    ids.clear();
    X.clear();
    if (m == 0) return;
    if (!(lo >= 0 && hi < 4 * (int64_t)m + 1024)) {   // sparse ids: the general path
        CooTriples t;
        for (auto &c : ch) {
            t.i.insert(t.i.end(), c.t.i.begin(), c.t.i.end());
            t.j.insert(t.j.end(), c.t.j.begin(), c.t.j.end());
            t.v.insert(t.v.end(), c.t.v.begin(), c.t.v.end());
        }
        auto rows = cooToVectors(t, dimension);
        std::sort(rows.begin(), rows.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        X.resize(rows.size() * (size_t)dimension);
        for (size_t r = 0; r < rows.size(); ++r) {
            ids.push_back(rows[r].first);
            std::memcpy(&X[r * (size_t)dimension], rows[r].second.data(), sizeof(double) * dimension);
        }
        return;
    }
    // ids present -> row slots in id order
    std::vector<uint8_t> present((size_t)hi + 1, 0);
    auto par = [&](auto &&body) {
        std::vector<std::thread> pool;
        for (int t = 1; t < T; ++t) pool.emplace_back([&, t] { body(t); });
        body(0);
        for (auto &th : pool) th.join();
    };
    // (each thread marks the ids of its own chunk; several threads may store
    // the same 1 to one byte, so the marks go through relaxed atomics)
    par([&](int t) {
        for (int32_t i : ch[t].t.i) __atomic_store_n(&present[(size_t)i], (uint8_t)1, __ATOMIC_RELAXED);
    });
    std::vector<int32_t> slot((size_t)hi + 1, -1);
    for (int64_t i = 0; i <= hi; ++i)
        if (present[(size_t)i]) { slot[(size_t)i] = (int32_t)ids.size(); ids.push_back((int32_t)i); }
    const size_t n = ids.size(), d = (size_t)dimension;
    X.assign(n * d, 0.0);
    // scatter: the first value of a cell is stored (0 + v, as VectorBuilder's
    // zero start); a cell met again is only noted, and re-summed below
    std::vector<uint64_t> seen((n * d + 63) / 64, 0);
    std::vector<std::vector<size_t>> again(T);
    par([&](int t) {
        const CooTriples &c = ch[t].t;
        for (size_t e = 0; e < c.i.size(); ++e) {
            const size_t cell = (size_t)slot[(size_t)c.i[e]] * d + (size_t)c.j[e];
            const uint64_t bit = 1ull << (cell & 63);
            if (__atomic_fetch_or(&seen[cell >> 6], bit, __ATOMIC_RELAXED) & bit) again[t].push_back(cell);
            else X[cell] = 0.0 + c.v[e];
        }
    });
    size_t ndup = 0;
    for (auto &a : again) ndup += a.size();
    if (ndup == 0) return;
    // cells with several values: zero, then every value in file order
    std::vector<uint64_t> dup((n * d + 63) / 64, 0);
    for (auto &a : again)
        for (size_t cell : a) dup[cell >> 6] |= 1ull << (cell & 63);
    for (size_t w = 0; w < dup.size(); ++w)
        for (uint64_t b = dup[w]; b; b &= b - 1) X[w * 64 + (size_t)__builtin_ctzll(b)] = 0.0;
    for (auto &c : ch)
        for (size_t e = 0; e < c.t.i.size(); ++e) {
            const size_t cell = (size_t)slot[(size_t)c.t.i[e]] * d + (size_t)c.t.j[e];
            if ((dup[cell >> 6] >> (cell & 63)) & 1ull) X[cell] += c.t.v[e];
        }
}

std::vector<std::pair<int32_t, std::vector<double>>> cooToVectors(const CooTriples &t, int dimension) {
    std::vector<std::pair<int32_t, std::vector<double>>> out;
    const size_t m = t.i.size();
    // slot of each id in order of first appearance: dense table when ids are
    // small non-negative ints, hash map otherwise
    int32_t lo = 0, hi = -1;
    for (size_t e = 0; e < m; ++e) { lo = std::min(lo, t.i[e]); hi = std::max(hi, t.i[e]); }
    const bool dense = lo >= 0 && (int64_t)hi < (int64_t)4 * (int64_t)m + 1024;
    std::vector<int32_t> table(dense ? (size_t)hi + 1 : 0, -1);
    std::unordered_map<int32_t, int32_t> map;
    for (size_t e = 0; e < m; ++e) {
        const int32_t j = t.j[e];
        if (j < 0 || j >= dimension) throw std::out_of_range("index " + std::to_string(j) + " out of dimension");
        int32_t s;
        if (dense) {
            s = table[t.i[e]];
            if (s < 0) { s = table[t.i[e]] = (int32_t)out.size(); out.push_back({t.i[e], std::vector<double>(dimension, 0.0)}); }
        } else {
            auto it = map.find(t.i[e]);
            if (it == map.end()) {
                it = map.emplace(t.i[e], (int32_t)out.size()).first;
                out.push_back({t.i[e], std::vector<double>(dimension, 0.0)});
            }
            s = it->second;
        }
        out[s].second[j] += t.v[e];   // VectorBuilder.add accumulates, in file order
    }
    return out;
}

}  // namespace tsne_flink
