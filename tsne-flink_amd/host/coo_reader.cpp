// coo_reader.cpp -- parallel mmap reader of the reference's COO CSV input
// (Tsne.scala:138-159); see coo_reader.hpp.
#include "coo_reader.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
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

}  // namespace

CooTriples parseCoo(const char *buf, size_t len, int threads) {
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
    CooTriples out;
    size_t total = 0;
    for (auto &c : ch) {
        if (!c.err.empty()) throw std::runtime_error(c.err);
        total += c.t.i.size();
    }
    out.i.reserve(total); out.j.reserve(total); out.v.reserve(total);
    for (auto &c : ch) {   // file order
        out.i.insert(out.i.end(), c.t.i.begin(), c.t.i.end());
        out.j.insert(out.j.end(), c.t.j.begin(), c.t.j.end());
        out.v.insert(out.v.end(), c.t.v.begin(), c.t.v.end());
    }
    return out;
}

CooTriples readCooFile(const std::string &path, int threads) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd, &st) != 0) { ::close(fd); throw std::runtime_error("cannot stat " + path); }
    const size_t len = (size_t)st.st_size;
    if (len == 0) { ::close(fd); return CooTriples(); }
    void *m = ::mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) throw std::runtime_error("cannot mmap " + path);
    (void)::madvise(m, len, MADV_SEQUENTIAL);
    CooTriples t;
    try {
        t = parseCoo(static_cast<const char *>(m), len, threads);
    } catch (...) {
        ::munmap(m, len);
        throw;
    }
    ::munmap(m, len);
    return t;
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
