// tsne_helpers.cpp -- C++ host mirror of TsneHelpers over libtsne_hip.
#include "tsne_helpers.hpp"

#include <algorithm>
#include <random>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace tsne_flink {

void check(int status) {
    if (status == TSNE_OK) return;
    std::string msg = tsne_last_error();
    if (status == TSNE_ERR_ARG) throw std::invalid_argument(msg);
    throw std::runtime_error("libtsne_hip status " + std::to_string(status) + ": " + msg);
}

int32_t getMetric(const std::string &name) {
    int32_t m = 0;
    check(tsne_metric_from_name(name.c_str(), &m));
    return m;
}

TsneHelpers::TsneHelpers(int device) { check(tsne_ctx_create(device, &ctx_)); }
TsneHelpers::~TsneHelpers() { tsne_ctx_destroy(ctx_); }

// Triples -> CSR over the sorted distinct ids (rows in id order, a row's
// entries in input order).  O(nnz): ids map to rows through a table when they
// are dense enough (the usual 0..n-1), else by binary search; rows by a
// stable counting sort.  (A comparison sort plus a binary search per entry
// took ~10 s per call for the 161M entries of P at C3.)
Csr toCsr(const std::vector<Triple> &t, const std::vector<int32_t> *idsIn) {
    Csr c;
    if (idsIn) {
        c.ids = *idsIn;
    } else {
        c.ids.reserve(2 * t.size());
        for (const auto &e : t) { c.ids.push_back(e.i); c.ids.push_back(e.j); }
        std::sort(c.ids.begin(), c.ids.end());
        c.ids.erase(std::unique(c.ids.begin(), c.ids.end()), c.ids.end());
    }
    const size_t n = c.ids.size();
    std::vector<int32_t> table;   // id - lo -> row, -1 for an id not in ids
    int64_t lo = 0;
    if (n > 0) {
        lo = c.ids.front();
        const int64_t span = (int64_t)c.ids.back() - lo + 1;
        if (span <= 4 * (int64_t)n + 1024) {
            table.assign((size_t)span, -1);
            for (size_t r = 0; r < n; ++r) table[(size_t)(c.ids[r] - lo)] = (int32_t)r;
        }
    }
    auto dense = [&](int32_t id) -> int32_t {
        if (!table.empty()) {
            const int64_t o = (int64_t)id - lo;
            if (o >= 0 && o < (int64_t)table.size() && table[(size_t)o] >= 0) return table[(size_t)o];
        } else {
            auto it = std::lower_bound(c.ids.begin(), c.ids.end(), id);
            if (it != c.ids.end() && *it == id) return (int32_t)(it - c.ids.begin());
        }
        throw std::invalid_argument("unknown point id " + std::to_string(id));
    };
    std::vector<int32_t> row(t.size());
    c.row_ptr.assign(n + 1, 0);
    for (size_t e = 0; e < t.size(); ++e) {
        row[e] = dense(t[e].i);
        c.row_ptr[(size_t)row[e] + 1]++;
    }
    for (size_t i = 0; i < n; ++i) c.row_ptr[i + 1] += c.row_ptr[i];
    c.col.resize(t.size());
    c.val.resize(t.size());
    std::vector<int64_t> fill(c.row_ptr.begin(), c.row_ptr.end() - (n > 0 ? 1 : 0));
    for (size_t e = 0; e < t.size(); ++e) {   // stable: input order within a row
        const int64_t k = fill[(size_t)row[e]]++;
        c.col[(size_t)k] = dense(t[e].j);
        c.val[(size_t)k] = t[e].v;
    }
    return c;
}

std::vector<Triple> fromCsr(const Csr &c) {
    std::vector<Triple> out;
    out.reserve(c.val.size());
    for (size_t i = 0; i + 1 < c.row_ptr.size(); ++i)
        for (int64_t e = c.row_ptr[i]; e < c.row_ptr[i + 1]; ++e) out.push_back({c.ids[i], c.ids[c.col[e]], c.val[e]});
    return out;
}

// The input's dense rows sorted by id (the kNN row order), as one n x d array.
static void denseInput(const Vectors &input, std::vector<int32_t> &ids, std::vector<double> &X, int32_t &d) {
    const size_t n = input.size();
    d = (int32_t)input[0].second.size();
    std::vector<size_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return input[a].first < input[b].first; });
    X.resize(n * (size_t)d);
    ids.resize(n);
    for (size_t r = 0; r < n; ++r) {
        const auto &v = input[order[r]];
        if ((int32_t)v.second.size() != d) throw std::invalid_argument("vectors of different lengths");
        ids[r] = v.first;
        std::memcpy(&X[r * (size_t)d], v.second.data(), sizeof(double) * d);
    }
}

// kNearestNeighbors (TsneHelpers.scala:41-59, also partitionKnn :61-91: the
// same exact result) or projectKnn (:93-160: the iterations-1 shift vectors
// are uniform [0,1)^dimension draws -- DenseVector.rand, unseeded in the
// reference -- from a 64-bit Mersenne twister seeded with randomState).
Csr TsneHelpers::kNearestNeighborsCsr(const Vectors &input, int32_t k, int32_t metric, const std::string &method,
                                      int32_t iterations, int64_t randomState) {
    Csr c;
    if (input.size() < 2) {
        c.row_ptr.assign(1, 0);
        return c;
    }
    std::vector<double> X;
    std::vector<int32_t> ids;
    int32_t d = 0;
    denseInput(input, ids, X, d);
    return kNearestNeighborsCsr(std::move(ids), X, d, k, metric, method, iterations, randomState);
}

Csr TsneHelpers::kNearestNeighborsCsr(std::vector<int32_t> ids, const std::vector<double> &X, int32_t d, int32_t k,
                                      int32_t metric, const std::string &method, int32_t iterations,
                                      int64_t randomState) {
    Csr c;
    c.ids = std::move(ids);
    const int64_t n = (int64_t)c.ids.size();
    if (n < 2) {
        c.row_ptr.assign(1, 0);
        c.ids.clear();
        return c;
    }
    const int64_t kk = std::min<int64_t>(k, n - 1);
    c.col.resize((size_t)(n * kk));
    c.val.resize((size_t)(n * kk));
    if (method == "project") {
        std::mt19937_64 rng((uint64_t)randomState);
        std::vector<double> shifts((size_t)std::max(iterations - 1, 0) * d);
        for (double &v : shifts) v = (double)(rng() >> 11) * 0x1.0p-53;
        check(tsne_project_knn(ctx_, X.data(), n, d, metric, k, iterations, shifts.empty() ? nullptr : shifts.data(),
                               c.col.data(), c.val.data()));
    } else {
        check(tsne_knn(ctx_, X.data(), n, d, metric, k, 0, n, c.col.data(), c.val.data()));
    }
    c.row_ptr.resize((size_t)n + 1);
    for (int64_t r = 0; r <= n; ++r) c.row_ptr[(size_t)r] = r * kk;
    return c;
}

std::vector<Triple> TsneHelpers::kNearestNeighbors(const Vectors &input, int32_t k, int32_t metric) {
    return fromCsr(kNearestNeighborsCsr(input, k, metric));
}

std::vector<Triple> TsneHelpers::projectKnn(const Vectors &input, int32_t k, int32_t metric, int32_t iterations,
                                            int64_t randomState) {
    return fromCsr(kNearestNeighborsCsr(input, k, metric, "project", iterations, randomState));
}

std::vector<Triple> TsneHelpers::partitionKnn(const Vectors &input, int32_t k, int32_t metric, int32_t) {
    return kNearestNeighbors(input, k, metric);
}

Csr TsneHelpers::pairwiseAffinitiesCsr(const Csr &knn, double perplexity) {
    Csr c;
    c.ids = knn.ids;
    c.row_ptr = knn.row_ptr;
    c.col = knn.col;
    c.val.resize(knn.val.size());
    check(tsne_pairwise_affinities(ctx_, knn.row_ptr.data(), knn.val.data(), (int64_t)knn.ids.size(), perplexity,
                                   c.val.data()));
    return c;
}

std::vector<Triple> TsneHelpers::pairwiseAffinities(const std::vector<Triple> &knn, double perplexity) {
    return fromCsr(pairwiseAffinitiesCsr(toCsr(knn), perplexity));
}

Csr TsneHelpers::jointDistributionCsr(const Csr &aff) {
    const int64_t n = (int64_t)aff.ids.size();
    const int64_t cap = 2 * (int64_t)aff.val.size() + 1;
    Csr c;
    c.ids = aff.ids;
    c.row_ptr.resize((size_t)n + 1);
    c.col.resize((size_t)cap);
    c.val.resize((size_t)cap);
    int64_t nnz = 0;
    check(tsne_joint_distribution(ctx_, aff.row_ptr.data(), aff.col.data(), aff.val.data(), n, cap,
                                  c.row_ptr.data(), c.col.data(), c.val.data(), &nnz));
    c.col.resize((size_t)nnz);
    c.val.resize((size_t)nnz);
    return c;
}

std::vector<Triple> TsneHelpers::jointDistribution(const std::vector<Triple> &aff) {
    return fromCsr(jointDistributionCsr(toCsr(aff)));
}

WorkingSet TsneHelpers::initWorkingSet(const std::vector<int32_t> &ids, int32_t nComponents,
                                       int64_t randomState) {
    WorkingSet w;
    w.ids = ids;
    std::sort(w.ids.begin(), w.ids.end());
    w.n_components = nComponents;
    const size_t ne = w.ids.size() * (size_t)nComponents;
    w.y.resize(ne);
    w.upd.resize(ne);
    w.gains.resize(ne);
    check(tsne_init_working_set(ctx_, (int64_t)w.ids.size(), nComponents, (uint64_t)randomState, w.y.data(),
                                w.upd.data(), w.gains.data()));
    return w;
}

std::vector<std::pair<int32_t, std::vector<double>>> TsneHelpers::gradient(const std::vector<Triple> &P,
                                                                         const WorkingSet &ws, int32_t metric,
                                                                         double theta, double exaggeration) {
    Csr c = toCsr(P, &ws.ids);
    const int64_t n = (int64_t)ws.ids.size();
    const int32_t nc = ws.n_components;   // 2, or 3 for the octree extension
    std::vector<double> g((size_t)n * (size_t)std::max(nc, 1));
    check(tsne_gradient_c(ctx_, c.row_ptr.data(), c.col.data(), c.val.data(), n, nc, ws.y.data(), metric, theta,
                          exaggeration, g.data(), nullptr, nullptr));
    std::vector<std::pair<int32_t, std::vector<double>>> out;
    for (int64_t i = 0; i < n; ++i) out.push_back({ws.ids[i], std::vector<double>(g.begin() + nc * i, g.begin() + nc * (i + 1))});
    return out;
}

void TsneHelpers::updateEmbedding(const std::vector<double> &grad, WorkingSet &ws, double minGain, double momentum,
                                  double learningRate) {
    check(tsne_update_embedding(ctx_, (int64_t)ws.ids.size(), ws.n_components, grad.data(), ws.y.data(),
                                ws.upd.data(), ws.gains.data(), minGain, momentum, learningRate));
}

void TsneHelpers::centerEmbedding(WorkingSet &ws) {
    check(tsne_center_embedding(ctx_, (int64_t)ws.ids.size(), ws.n_components, ws.y.data()));
}

void TsneHelpers::optimizeCsr(const Csr &c, WorkingSet &ws, double learningRate, int32_t iterations, int32_t metric,
                              double earlyExaggeration, double initialMomentum, double finalMomentum, double theta,
                              std::map<int32_t, double> *loss) {
    if (c.ids != ws.ids) throw std::invalid_argument("P's rows are not the working set's ids");
    tsne_params p;
    tsne_params_default(&p);
    p.n_components = ws.n_components;
    p.metric = metric;
    p.learning_rate = learningRate;
    p.iterations = iterations;
    p.early_exaggeration = earlyExaggeration;
    p.initial_momentum = initialMomentum;
    p.final_momentum = finalMomentum;
    p.theta = theta;
    const int32_t cap = iterations / 10 + 1;
    std::vector<int32_t> keys(cap);
    std::vector<double> vals(cap);
    int32_t nl = 0;
    check(tsne_optimize(ctx_, &p, c.row_ptr.data(), c.col.data(), c.val.data(), (int64_t)ws.ids.size(),
                        ws.y.data(), ws.upd.data(), ws.gains.data(), keys.data(), vals.data(), cap, &nl));
    if (loss)
        for (int32_t k = 0; k < std::min(nl, cap); ++k) (*loss)[keys[k]] += vals[k];
}

void TsneHelpers::optimize(const std::vector<Triple> &P, WorkingSet &ws, double learningRate, int32_t iterations,
                           int32_t metric, double earlyExaggeration, double initialMomentum, double finalMomentum,
                           double theta, std::map<int32_t, double> *loss) {
    optimizeCsr(toCsr(P, &ws.ids), ws, learningRate, iterations, metric, earlyExaggeration, initialMomentum,
                finalMomentum, theta, loss);
}

// java.lang.Double.toString: shortest round-trip digits; plain notation for
// 1e-3 <= |v| < 1e7 (at least one fractional digit), else d.dddE<exp>.
std::string javaDouble(double v) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
    if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
    std::string s(buf, r.ptr);
    // s = [-]d[.ddd]e[+-]XX
    bool neg = s[0] == '-';
    if (neg) s.erase(0, 1);
    size_t epos = s.find('e');
    int exp = std::stoi(s.substr(epos + 1));
    std::string mant = s.substr(0, epos);
    std::string digits;
    for (char ch : mant)
        if (ch != '.') digits.push_back(ch);
    std::string out;
    const double a = std::fabs(v);
    if (a >= 1e-3 && a < 1e7) {
        int point = exp + 1;  // digits before the decimal point
        if (point <= 0) {
            out = "0." + std::string(-point, '0') + digits;
        } else if (point >= (int)digits.size()) {
            out = digits + std::string(point - digits.size(), '0') + ".0";
        } else {
            out = digits.substr(0, point) + "." + digits.substr(point);
        }
    } else {
        out = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(exp);
    }
    return (neg ? "-" : "") + out;
}

// java.util.HashMap<Integer, Double>.toString: "{k=v, k=v}" in bucket order
// (capacity 16 doubling at load factor 0.75; Integer hash h ^ (h >>> 16)).
std::string javaHashMapString(const std::map<int32_t, double> &m) {
    size_t cap = 16;
    while ((double)m.size() > 0.75 * (double)cap) cap <<= 1;
    std::vector<std::pair<uint32_t, int32_t>> order;
    size_t ins = 0;
    std::vector<std::pair<std::pair<uint32_t, size_t>, int32_t>> keyed;
    for (const auto &kv : m) {  // insertion order = ascending iteration (keys accumulate in order)
        uint32_t h = (uint32_t)kv.first;
        h ^= (h >> 16);
        keyed.push_back({{h & (uint32_t)(cap - 1), ins++}, kv.first});
    }
    std::sort(keyed.begin(), keyed.end());
    std::string s = "{";
    for (size_t i = 0; i < keyed.size(); ++i) {
        if (i) s += ", ";
        s += std::to_string(keyed[i].second) + "=" + javaDouble(m.at(keyed[i].second));
    }
    return s + "}";
}

}  // namespace tsne_flink
