// cutsim.cpp -- offline estimate (CPU) of how many BH cell pops per query the
// traversal needs on a real embedding snapshot (bench.py --dump-y), with the
// current fast paths (all-open box test, near-exact test) and with a
// candidate "uniform cut" shortcut: an opened subtree S whose every cell above
// level L is opened and every level-L cell is summarised by the query
// (decided from the point-box distance bounds of S) is evaluated from the
// moments of its level-L cell masses in one step.
// Build: g++ -O2 -fopenmp -std=c++17 scripts/cutsim.cpp -o /tmp/cutsim
// Run:   /tmp/cutsim gpurun_out/Y_t200.npy [queries]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

struct Cell {
    double cx, cy, h;             // centre of mass, half width
    double bx0, bx1, by0, by1;    // bbox of points
    double hmin;                  // min h of branching cells in subtree
    int first, last, cnt;
    int ch[4], nch;               // branching children (collapsed chains)
    int level;
};

static std::vector<double> X, Yv;
static std::vector<Cell> cells;
static std::vector<uint64_t> key;

static std::vector<double> load_npy(const char *path, long &n) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    char magic[10];
    fread(magic, 1, 10, f);
    uint16_t hl = (uint8_t)magic[8] | ((uint8_t)magic[9] << 8);
    std::vector<char> hdr(hl);
    fread(hdr.data(), 1, hl, f);
    std::string hs(hdr.begin(), hdr.end());
    size_t p = hs.find("'shape': (");
    n = atol(hs.c_str() + p + 10);
    std::vector<double> v(2 * n);
    fread(v.data(), 8, 2 * n, f);
    fclose(f);
    return v;
}

// build over sorted points [a, b] sharing the top 2*lev key bits; returns cell id or -1-point for a leaf
static int build(int a, int b, int lev, double h) {
    if (a == b) return -1 - a;
    // descend single-child chains
    while (lev < 31) {
        int sh = 60 - 2 * lev;
        uint64_t d0 = (key[a] >> sh) & 3, d1 = (key[b] >> sh) & 3;
        if (d0 != d1) break;
        ++lev;
        h *= 0.5;
    }
    Cell c{};
    c.first = a; c.last = b; c.cnt = b - a + 1; c.h = h; c.level = lev;
    double sx = 0, sy = 0;
    c.bx0 = c.by0 = 1e300; c.bx1 = c.by1 = -1e300;
    for (int i = a; i <= b; ++i) {
        sx += X[2 * i]; sy += X[2 * i + 1];
        c.bx0 = std::min(c.bx0, X[2 * i]); c.bx1 = std::max(c.bx1, X[2 * i]);
        c.by0 = std::min(c.by0, X[2 * i + 1]); c.by1 = std::max(c.by1, X[2 * i + 1]);
    }
    c.cx = sx / c.cnt; c.cy = sy / c.cnt;
    int id = (int)cells.size();
    cells.push_back(c);
    if (lev >= 31) { cells[id].nch = 0; cells[id].hmin = h; return id; }   // tie group: all leaves
    int sh = 60 - 2 * lev;
    int s = a, nch = 0;
    double hmin = h;
    int chs[4];
    while (s <= b) {
        uint64_t dg = (key[s] >> sh) & 3;
        int e = s;
        while (e + 1 <= b && ((key[e + 1] >> sh) & 3) == dg) ++e;
        int r = build(s, e, lev + 1, h * 0.5);
        chs[nch++] = r;
        if (r >= 0) hmin = std::min(hmin, cells[r].hmin);
        s = e + 1;
    }
    for (int k = 0; k < nch; ++k) cells[id].ch[k] = chs[k];
    cells[id].nch = nch;
    cells[id].hmin = hmin;
    return id;
}

static inline void box_d(double qx, double qy, const Cell &c, double &dmin, double &dmax) {
    double ax = std::max({c.bx0 - qx, 0.0, qx - c.bx1}), ay = std::max({c.by0 - qy, 0.0, qy - c.by1});
    dmin = ax * ax + ay * ay;
    double mx = std::max(std::fabs(qx - c.bx0), std::fabs(qx - c.bx1));
    double my = std::max(std::fabs(qy - c.by0), std::fabs(qy - c.by1));
    dmax = mx * mx + my * my;
}

struct Count { double pops = 0, tiles = 0, cuts = 0, cutk = 0, leafsum = 0, summ = 0; };

// count pops for one query; mode 0 = current fast paths, 1 = + uniform cuts (k >= kmin)
static void walk(int root, double qx, double qy, double theta, double near_dmax, int mode, int kmin, Count &cnt) {
    std::vector<int> st;
    st.push_back(root);
    while (!st.empty()) {
        int id = st.back(); st.pop_back();
        const Cell &c = cells[id];
        cnt.pops += 1;
        double dmin, dmax;
        box_d(qx, qy, c, dmin, dmax);
        if (c.nch == 0 || dmax <= c.hmin / theta || dmax <= near_dmax) { cnt.tiles += 1; cnt.leafsum += c.cnt; continue; }
        if (mode == 1 && dmin > 0) {
            // smallest k >= 1 with h/2^k < theta*dmin; need h/2^(k-1) >= theta*dmax
            int k = 1;
            double hk = c.h * 0.5;
            while (!(hk < theta * dmin * (1 - 1e-12)) && k < 40) { hk *= 0.5; ++k; }
            if (k >= kmin && 2 * hk >= theta * dmax * (1 + 1e-12)) { cnt.cuts += 1; cnt.cutk += k; continue; }
        }
        for (int k = 0; k < c.nch; ++k) {
            int r = c.ch[k];
            if (r < 0) { cnt.summ += 1; continue; }
            const Cell &d = cells[r];
            double dx = qx - d.cx, dy = qy - d.cy, D = dx * dx + dy * dy;
            if (d.h / D < theta) cnt.summ += 1;
            else st.push_back(r);
        }
    }
}

int main(int argc, char **argv) {
    long n;
    std::vector<double> Y = load_npy(argv[1], n);
    int nq = argc > 2 ? atoi(argv[2]) : 2048;
    double theta = 0.5;
    double tol = argc > 3 ? atof(argv[3]) : 1e-6;
    double near_dmax = std::sqrt(tol / (48 * theta * theta));
    double x0 = 1e300, x1 = -1e300, y0 = 1e300, y1 = -1e300;
    for (long i = 0; i < n; ++i) {
        x0 = std::min(x0, Y[2 * i]); x1 = std::max(x1, Y[2 * i]);
        y0 = std::min(y0, Y[2 * i + 1]); y1 = std::max(y1, Y[2 * i + 1]);
    }
    double W = std::max(x1 - x0, y1 - y0) * 0.5 * (1 + 1e-9), cx = (x0 + x1) / 2, cy = (y0 + y1) / 2;
    std::vector<std::pair<uint64_t, int>> kv(n);
    for (long i = 0; i < n; ++i) {
        double u = (Y[2 * i] - (cx - W)) / (2 * W), v = (Y[2 * i + 1] - (cy - W)) / (2 * W);
        uint64_t a = (uint64_t)std::min(std::ldexp(u, 31), std::ldexp(1.0, 31) - 1);
        uint64_t b = (uint64_t)std::min(std::ldexp(v, 31), std::ldexp(1.0, 31) - 1);
        uint64_t k = 0;
        for (int l = 30; l >= 0; --l) k = (k << 2) | (((b >> l) & 1) << 1) | ((a >> l) & 1);
        kv[i] = {k, (int)i};
    }
    std::sort(kv.begin(), kv.end());
    X.resize(2 * n); key.resize(n);
    for (long i = 0; i < n; ++i) { key[i] = kv[i].first; X[2 * i] = Y[2 * kv[i].second]; X[2 * i + 1] = Y[2 * kv[i].second + 1]; }
    cells.reserve(2 * n);
    int root = build(0, (int)n - 1, 0, W);
    printf("n=%ld extent=%.4g cells=%zu near_dmax=%.3g\n", n, 2 * W, cells.size(), near_dmax);
    std::mt19937_64 rng(1);
    std::vector<int> qs(nq);
    for (int i = 0; i < nq; ++i) qs[i] = (int)(rng() % n);
    for (int mode = 0; mode <= 1; ++mode) {
        for (int kmin : {2, 3}) {
            if (mode == 0 && kmin == 3) continue;
            Count tot;
#pragma omp parallel
            {
                Count loc;
#pragma omp for schedule(dynamic, 16)
                for (int i = 0; i < nq; ++i) walk(root, X[2 * qs[i]], X[2 * qs[i] + 1], theta, near_dmax, mode, kmin, loc);
#pragma omp critical
                {
                    tot.pops += loc.pops; tot.tiles += loc.tiles; tot.cuts += loc.cuts; tot.cutk += loc.cutk;
                    tot.leafsum += loc.leafsum; tot.summ += loc.summ;
                }
            }
            printf("mode %d kmin %d: pops/q %.1f tiles/q %.1f tilepts/q %.1f cuts/q %.1f (mean k %.2f) summarised/q %.1f\n",
                   mode, kmin, tot.pops / nq, tot.tiles / nq, tot.leafsum / nq, tot.cuts / nq,
                   tot.cuts > 0 ? tot.cutk / tot.cuts : 0.0, tot.summ / nq);
        }
    }
}
