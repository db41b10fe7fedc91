/*
 * tsne_oracle.c -- CPU fp64 restatement of the tsne-flink hot path.
 * TEST INFRASTRUCTURE ONLY (see tsne_oracle.h).  Compiled with
 * -ffp-contract=off so that every a*b+c rounds twice, as on the JVM.
 */
#include "tsne_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ metrics */

/* breeze squaredDistance: sequential sum of (a_i - b_i)^2 in index order. */
/* Neumaier-compensated running sum for the KL loss: a sequential sum over
 * ~1e8 terms drifts by up to n*eps relative (1e-8 at C3's size), more than
 * the 1e-9 the loss is checked at; the reference's reduce order is Flink's
 * anyway (TsneHelpers.scala:297-299), so the exact sum is the oracle. */
static void kahan_add(double *s, double *c, double x) {
    const double t = *s + x;
    *c += fabs(*s) >= fabs(x) ? (*s - t) + x : (x - t) + *s;
    *s = t;
}

static double sqdist(const double *a, const double *b, int32_t d) {
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) {
        double t = a[i] - b[i];
        s += t * t;
    }
    return s;
}

static double dot(const double *a, const double *b, int32_t d) {
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) s += a[i] * b[i];
    return s;
}

/* Tsne.scala:161-168.  euclidean = sqrt(squaredDistance);
 * cosine = 1 - (a.b) / (|a| |b|)  (breeze cosineDistance; parity unpinned). */
double oracle_metric(const double *a, const double *b, int32_t d, int metric) {
    switch (metric) {
    case ORACLE_SQEUCLIDEAN: return sqdist(a, b, d);
    case ORACLE_EUCLIDEAN: return sqrt(sqdist(a, b, d));
    case ORACLE_COSINE: {
        double na = sqrt(dot(a, a, d)), nb = sqrt(dot(b, b, d));
        return 1.0 - dot(a, b, d) / (na * nb);
    }
    default: return NAN;
    }
}

/* ---------------------------------------------------------------------- kNN */

/* (d, j) order; NaN sorts after every number. */
static int less_dj(double da, int32_t ja, double db, int32_t jb) {
    int na = isnan(da), nb = isnan(db);
    if (na != nb) return nb;            /* number < NaN */
    if (!na && da != db) return da < db;
    return ja < jb;
}

typedef struct { double d; int32_t j; } dj_t;

static void heap_sift_down(dj_t *h, int32_t n, int32_t i) {
    /* max-heap under less_dj */
    for (;;) {
        int32_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < n && less_dj(h[m].d, h[m].j, h[l].d, h[l].j)) m = l;
        if (r < n && less_dj(h[m].d, h[m].j, h[r].d, h[r].j)) m = r;
        if (m == i) return;
        dj_t t = h[i]; h[i] = h[m]; h[m] = t; i = m;
    }
}

static int cmp_dj(const void *a, const void *b) {
    const dj_t *x = (const dj_t *)a, *y = (const dj_t *)b;
    if (less_dj(x->d, x->j, y->d, y->j)) return -1;
    if (less_dj(y->d, y->j, x->d, x->j)) return 1;
    return 0;
}

/* TsneHelpers.scala:41-59: cross, filter i != j (by index, so duplicates at
 * distance 0 stay), group by i, sort by d ascending, first(k). */
int oracle_knn(const double *X, int64_t n, int32_t d, int metric, int32_t k,
               int64_t q0, int64_t q1, int32_t *idx, double *dist, int threads) {
    if (!X || n < 1 || d < 1 || k < 1 || q0 < 0 || q1 > n || q0 > q1) return -1;
    int32_t kk = (int32_t)((int64_t)k < n - 1 ? k : n - 1);
    if (kk <= 0) return 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel num_threads(threads)
#endif
    {
        dj_t *h = (dj_t *)malloc(sizeof(dj_t) * (size_t)kk);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int64_t i = q0; i < q1; ++i) {
            int32_t cnt = 0;
            const double *xi = X + i * d;
            for (int64_t j = 0; j < n; ++j) {
                if (j == i) continue;
                double dv = oracle_metric(xi, X + j * d, d, metric);
                if (cnt < kk) {
                    h[cnt].d = dv; h[cnt].j = (int32_t)j; ++cnt;
                    if (cnt == kk)
                        for (int32_t s = kk / 2 - 1; s >= 0; --s) heap_sift_down(h, kk, s);
                } else if (less_dj(dv, (int32_t)j, h[0].d, h[0].j)) {
                    h[0].d = dv; h[0].j = (int32_t)j;
                    heap_sift_down(h, kk, 0);
                }
            }
            qsort(h, (size_t)kk, sizeof(dj_t), cmp_dj);
            int64_t o = (i - q0) * kk;
            for (int32_t t = 0; t < kk; ++t) { idx[o + t] = h[t].j; dist[o + t] = h[t].d; }
        }
        free(h);
    }
    return 0;
}

/* ----------------------------------------------------------- affinities */

/* computeH (TsneHelpers.scala:490-495) */
static double compute_h(const double *d, int64_t len, double beta) {
    double s = 0.0, sdp = 0.0;
    for (int64_t t = 0; t < len; ++t) s += exp(-d[t] * beta);
    for (int64_t t = 0; t < len; ++t) sdp += d[t] * exp(-d[t] * beta);
    double sp = (s == 0.0) ? 1e-7 : s;
    return log(sp) + beta * sdp / sp;
}

/* computeP (TsneHelpers.scala:497-504) */
static void compute_p(const double *d, int64_t len, double beta, double *p) {
    double s = 0.0;
    for (int64_t t = 0; t < len; ++t) s += exp(-d[t] * beta);
    double sp = (s == 0.0) ? 1e-7 : s;
    for (int64_t t = 0; t < len; ++t) p[t] = exp(-d[t] * beta) / sp;
}

/* binarySearch / approximateBeta (TsneHelpers.scala:434-484) */
int oracle_affinities(const int64_t *row_ptr, const double *dist, int64_t nrows,
                      double perplexity, double *p_out, int32_t *iters_out) {
    if (!row_ptr || nrows < 0) return -1;
    const double target = log(perplexity);
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t b = row_ptr[i], len = row_ptr[i + 1] - row_ptr[i];
        const double *d = dist + b;
        double beta = 1.0, mn = -INFINITY, mx = INFINITY;
        int32_t budget = 50, used = 0;
        for (;;) {
            double h = compute_h(d, len, beta);
            if (fabs(h - target) < 1e-5 || budget == 0) { compute_p(d, len, beta, p_out + b); break; }
            double nb;
            if (h - target > 0) {
                nb = isinf(mx) ? beta * 2 : (beta + mx) / 2;
                mn = beta;
            } else {
                nb = isinf(mn) ? beta / 2 : (beta + mn) / 2;
                mx = beta;
            }
            beta = nb; --budget; ++used;
        }
        if (iters_out) iters_out[i] = used;
    }
    return 0;
}

/* ----------------------------------------------------------------- joint */

typedef struct { int32_t r, c; double v; } rcv_t;

static int cmp_rcv(const void *a, const void *b) {
    const rcv_t *x = (const rcv_t *)a, *y = (const rcv_t *)b;
    if (x->r != y->r) return x->r < y->r ? -1 : 1;
    if (x->c != y->c) return x->c < y->c ? -1 : 1;
    return 0;
}

/* TsneHelpers.scala:182-196 */
int oracle_joint(const int64_t *row_ptr, const int32_t *col, const double *p,
                 int64_t n, int64_t *out_row_ptr, int32_t *out_col, double *out_val,
                 int64_t cap, int64_t *nnz_out) {
    if (!row_ptr || n < 0) return -1;
    int64_t nnz = row_ptr[n];
    rcv_t *e = (rcv_t *)malloc(sizeof(rcv_t) * (size_t)(2 * nnz + 1));
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t t = row_ptr[i]; t < row_ptr[i + 1]; ++t) {
            e[m].r = (int32_t)i; e[m].c = col[t]; e[m].v = p[t]; ++m;      /* input      */
            e[m].r = col[t]; e[m].c = (int32_t)i; e[m].v = p[t]; ++m;      /* transposed */
        }
    qsort(e, (size_t)m, sizeof(rcv_t), cmp_rcv);
    int64_t u = 0;
    for (int64_t t = 0; t < m; ++t) {
        if (u > 0 && e[u - 1].r == e[t].r && e[u - 1].c == e[t].c) e[u - 1].v += e[t].v;
        else e[u++] = e[t];
    }
    *nnz_out = u;
    if (u > cap) { free(e); return -2; }
    double sum = 0.0;
    for (int64_t t = 0; t < u; ++t) sum += e[t].v;
    for (int64_t i = 0; i <= n; ++i) out_row_ptr[i] = 0;
    for (int64_t t = 0; t < u; ++t) out_row_ptr[e[t].r + 1]++;
    for (int64_t i = 0; i < n; ++i) out_row_ptr[i + 1] += out_row_ptr[i];
    for (int64_t t = 0; t < u; ++t) { out_col[t] = e[t].c; out_val[t] = e[t].v / sum; }
    free(e);
    return 0;
}

/* -------------------------------------------------------------- quadtree */

/* QuadTree.scala:28-36 / Cell.scala:24-36: pointer quadtree, capacity 1. */
typedef struct {
    double x, y, hw, hh;                 /* Cell: centre, half width, half height */
    double sumx, sumy, comx, comy;
    double px, py;
    int32_t cum, leaf, has_point;
    int32_t child[4];                    /* NW, NE, SW, SE */
} qnode_t;

typedef struct { qnode_t *v; int64_t n, cap; } qtree_t;

static int32_t qt_new(qtree_t *t, double x, double y, double hw, double hh) {
    if (t->n == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 1024;
        t->v = (qnode_t *)realloc(t->v, sizeof(qnode_t) * (size_t)t->cap);
    }
    qnode_t *q = &t->v[t->n];
    memset(q, 0, sizeof(*q));
    q->x = x; q->y = y; q->hw = hw; q->hh = hh; q->leaf = 1;
    q->child[0] = q->child[1] = q->child[2] = q->child[3] = -1;
    return (int32_t)t->n++;
}

/* Cell.contains (Cell.scala:31-36), closed intervals */
static int cell_contains(const qnode_t *q, double px, double py) {
    return (q->x - q->hw <= px) && (q->x + q->hw >= px) && (q->y - q->hh <= py) && (q->y + q->hh >= py);
}

static int qt_insert(qtree_t *t, int32_t ni, double px, double py);

/* insertIntoSubTree / checkAndInsert (QuadTree.scala:87-114) */
static int qt_insert_sub(qtree_t *t, int32_t ni, double px, double py) {
    for (int c = 0; c < 4; ++c) {
        int32_t ch = t->v[ni].child[c];
        if (ch >= 0 && cell_contains(&t->v[ch], px, py)) {
            if (qt_insert(t, ch, px, py)) return 1;
        }
    }
    return 0;
}

/* subDivide (QuadTree.scala:72-85): both new extents from hWidth */
static void qt_subdivide(qtree_t *t, int32_t ni) {
    double x = t->v[ni].x, y = t->v[ni].y, hw = t->v[ni].hw;
    double nw = 0.5 * hw, nh = 0.5 * hw;
    int32_t a = qt_new(t, x - nw, y + nh, nw, nh);
    int32_t b = qt_new(t, x + nw, y + nh, nw, nh);
    int32_t c = qt_new(t, x - nw, y - nh, nw, nh);
    int32_t d = qt_new(t, x + nw, y - nh, nw, nh);
    qnode_t *q = &t->v[ni];
    q->child[0] = a; q->child[1] = b; q->child[2] = c; q->child[3] = d;
}

/* insert (QuadTree.scala:38-70) */
static int qt_insert(qtree_t *t, int32_t ni, double px, double py) {
    qnode_t *q = &t->v[ni];
    if (!cell_contains(q, px, py)) return 0;
    q->sumx += px; q->sumy += py;
    q->cum += 1;
    q->comx = q->sumx / (double)q->cum;
    q->comy = q->sumy / (double)q->cum;
    if (q->leaf) {
        if (q->has_point) {
            if (q->px == px && q->py == py) return 1;    /* same point: keep */
            double lx = q->px, ly = q->py;
            qt_subdivide(t, ni);
            q = &t->v[ni];
            q->leaf = 0;
            qt_insert_sub(t, ni, lx, ly);                /* the leaf's point, once */
            qt_insert_sub(t, ni, px, py);
            t->v[ni].has_point = 0;
            return 1;
        }
        q->has_point = 1; q->px = px; q->py = py;
        return 1;
    }
    return qt_insert_sub(t, ni, px, py);
}

/* computeRepulsiveForce (QuadTree.scala:123-152) */
static void qt_repulsive(const qtree_t *t, int32_t ni, double px, double py, double theta,
                         double *fx, double *fy, double *sq, int64_t *visits) {
    const qnode_t *q = &t->v[ni];
    ++*visits;
    if ((q->leaf && q->cum == 0) || (q->leaf && q->px == px && q->py == py)) {
        *fx = 0.0; *fy = 0.0; *sq = 0.0;
        return;
    }
    double dx = px - q->comx, dy = py - q->comy;
    double D = dx * dx + dy * dy;              /* squaredDistance(point, centerOfMass) */
    double h = q->hh > q->hw ? q->hh : q->hw;  /* max(hHeigth, hWidth) */
    if (q->leaf || (h / D < theta)) {
        double Q = 1.0 / (1.0 + D);
        double mult = (double)q->cum * Q;
        double s = mult * Q;
        *sq = 0.0 + mult;
        *fx = s * (px - q->comx);
        *fy = s * (py - q->comy);
        return;
    }
    double ax = 0, ay = 0, as = 0;
    for (int c = 0; c < 4; ++c) {
        double cx, cy, cs;
        qt_repulsive(t, q->child[c], px, py, theta, &cx, &cy, &cs, visits);
        if (c == 0) { ax = cx; ay = cy; as = cs; }
        else { ax = ax + cx; ay = ay + cy; as = as + cs; }
    }
    *fx = ax; *fy = ay; *sq = as;
}

/* Tree of all points, root Cell(0, 0, max(dX, dY)) (TsneHelpers.scala:228-256) */
static void build_tree(qtree_t *t, const double *Y, int64_t n) {
    double mnx = Y[0], mxx = Y[0], mny = Y[1], mxy = Y[1];
    for (int64_t i = 1; i < n; ++i) {
        double x = Y[2 * i], y = Y[2 * i + 1];
        mnx = fmin(mnx, x); mxx = fmax(mxx, x);
        mny = fmin(mny, y); mxy = fmax(mxy, y);
    }
    double W = fmax(mxx - mnx, mxy - mny);   /* scala.math.max */
    /* mean = (sum of zero vectors) / count = (0, 0) */
    t->v = NULL; t->n = t->cap = 0;
    qt_new(t, 0.0, 0.0, W, W);
    for (int64_t i = 0; i < n; ++i) qt_insert(t, 0, Y[2 * i], Y[2 * i + 1]);
}

int oracle_repulsion(const double *Y, int64_t n, double theta, int64_t q0, int64_t q1,
                     double *rep, double *zi, int threads) {
    if (!Y || n < 1 || q0 < 0 || q1 > n || q0 > q1) return -1;
    qtree_t t;
    build_tree(&t, Y, n);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
#endif
    for (int64_t i = q0; i < q1; ++i) {
        double fx, fy, s;
        int64_t v = 0;
        qt_repulsive(&t, 0, Y[2 * i], Y[2 * i + 1], theta, &fx, &fy, &s, &v);
        rep[2 * (i - q0)] = fx; rep[2 * (i - q0) + 1] = fy;
        zi[i - q0] = s;
    }
    free(t.v);
    return 0;
}

/* -------------------------------------------------------------- gradient */

/* TsneHelpers.scala:221-318 */
int oracle_gradient(const int64_t *row_ptr, const int32_t *col, const double *val,
                    int64_t n, const double *Y, int metric, double theta,
                    double exaggeration, double *grad, double *sumq_out, double *loss_out,
                    double *rep_out, double *zi_out, double *attr_out, int64_t *visits_out,
                    int threads) {
    if (!row_ptr || !Y || n < 1) return -1;
    qtree_t t;
    build_tree(&t, Y, n);
    double *rep = (double *)malloc(sizeof(double) * 2 * (size_t)n);
    double *zi = (double *)malloc(sizeof(double) * (size_t)n);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
#endif
    for (int64_t i = 0; i < n; ++i) {
        double fx, fy, s;
        int64_t v = 0;
        qt_repulsive(&t, 0, Y[2 * i], Y[2 * i + 1], theta, &fx, &fy, &s, &v);
        rep[2 * i] = fx; rep[2 * i + 1] = fy; zi[i] = s;
        if (visits_out) visits_out[i] = v;
    }
    free(t.v);
    double Z = 0.0;                                  /* sumQ reduce (TsneHelpers.scala:266) */
    for (int64_t i = 0; i < n; ++i) Z = Z + zi[i];
    double loss = 0.0, loss_c = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double gx = 0.0, gy = 0.0;
        const double *yi = Y + 2 * i;
        for (int64_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            const double *yj = Y + 2 * (int64_t)col[e];
            double pij = val[e] * exaggeration;      /* x._2 * earlyExaggeration */
            double qij = 1.0 / (1.0 + oracle_metric(yi, yj, 2, metric));
            double s = pij * qij;
            gx = gx + s * (yi[0] - yj[0]);
            gy = gy + s * (yi[1] - yj[1]);
            if (loss_out) kahan_add(&loss, &loss_c, pij * log(pij / (qij / Z)));
        }
        if (attr_out) { attr_out[2 * i] = gx; attr_out[2 * i + 1] = gy; }
        grad[2 * i] = gx - rep[2 * i] / Z;           /* attrForce - repForce / sumQ */
        grad[2 * i + 1] = gy - rep[2 * i + 1] / Z;
    }
    if (sumq_out) *sumq_out = Z;
    if (loss_out) *loss_out = loss + loss_c;
    if (rep_out) memcpy(rep_out, rep, sizeof(double) * 2 * (size_t)n);
    if (zi_out) memcpy(zi_out, zi, sizeof(double) * (size_t)n);
    free(rep); free(zi);
    return 0;
}

/* ------------------------------------------------------------- optimizer */

/* updateEmbedding (TsneHelpers.scala:341-369) */
int oracle_update(int64_t n, int32_t c, const double *grad, double *Y, double *upd,
                  double *gains, double min_gain, double momentum, double lr) {
    for (int64_t i = 0; i < n * c; ++i) {
        double g = grad[i], u = upd[i], gn;
        if ((g > 0.0) == (u > 0.0)) gn = fmax(gains[i] * 0.8, min_gain);
        else gn = fmax(gains[i] + 0.2, min_gain);
        double un = momentum * u - lr * gn * g;
        gains[i] = gn;
        upd[i] = un;
        Y[i] = un + Y[i];
    }
    return 0;
}

/* centerEmbedding (TsneHelpers.scala:320-329) */
int oracle_center(int64_t n, int32_t c, double *Y) {
    double s[8] = {0};
    if (c > 8) return -1;
    for (int64_t i = 0; i < n; ++i)
        for (int32_t k = 0; k < c; ++k) s[k] = s[k] + Y[i * c + k];
    for (int32_t k = 0; k < c; ++k) s[k] = s[k] / (double)n;
    for (int64_t i = 0; i < n; ++i)
        for (int32_t k = 0; k < c; ++k) Y[i * c + k] = Y[i * c + k] - s[k];
    return 0;
}

/* optimize (TsneHelpers.scala:396-430) + iterationComputation (371-394) */
int oracle_optimize(const int64_t *row_ptr, const int32_t *col, const double *val,
                    int64_t n, double *Y, double *upd, double *gains, int metric,
                    double learning_rate, int32_t iterations, double early_exaggeration,
                    double initial_momentum, double final_momentum, double theta,
                    int32_t *loss_keys, double *loss_vals, int32_t *n_loss, int threads) {
    int32_t n1 = iterations < 20 ? iterations : 20;
    int32_t n2 = (iterations - n1) < 81 ? (iterations - n1) : 81;
    int32_t nl = 0;
    double *grad = (double *)malloc(sizeof(double) * 2 * (size_t)n);
    for (int32_t t = 1; t <= iterations; ++t) {
        double ex = (t <= n1 + n2) ? early_exaggeration : 1.0;
        double mom = (t <= n1) ? initial_momentum : final_momentum;
        int want_loss = (t % 10 == 0);
        double loss = 0.0, Z = 0.0;
        oracle_gradient(row_ptr, col, val, n, Y, metric, theta, ex, grad, &Z,
                        want_loss ? &loss : NULL, NULL, NULL, NULL, NULL, threads);
        if (want_loss && loss_keys) { loss_keys[nl] = t; loss_vals[nl] = loss; ++nl; }
        oracle_update(n, 2, grad, Y, upd, gains, 0.01, mom, learning_rate);
        oracle_center(n, 2, Y);
    }
    if (n_loss) *n_loss = nl;
    free(grad);
    return 0;
}

/* ------------------------------------------------ sharded-path helpers */

/* Repulsion of an arbitrary query list against the tree of all n points. */
int oracle_repulsion_queries(const double *Y, int64_t n, double theta, const double *Q, int64_t nq,
                             double *rep, double *zi, int threads) {
    if (!Y || n < 1 || nq < 0) return -1;
    qtree_t t;
    build_tree(&t, Y, n);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
#endif
    for (int64_t i = 0; i < nq; ++i) {
        double fx, fy, s;
        int64_t v = 0;
        qt_repulsive(&t, 0, Q[2 * i], Q[2 * i + 1], theta, &fx, &fy, &s, &v);
        rep[2 * i] = fx; rep[2 * i + 1] = fy; zi[i] = s;
    }
    free(t.v);
    return 0;
}

/* The CPU baseline's two legs timed apart (bench.py cpu_baseline): the serial
 * tree build of all n points (TsneHelpers.scala:234-256, one Flink task) once,
 * then query batches against that tree (TsneHelpers.scala:258-264, the
 * parallel map over points).  The handle is an opaque qtree_t. */
void *oracle_tree_build(const double *Y, int64_t n) {
    if (!Y || n < 1) return NULL;
    qtree_t *t = (qtree_t *)malloc(sizeof(qtree_t));
    build_tree(t, Y, n);
    return t;
}

int oracle_tree_query(const void *handle, double theta, const double *Q, int64_t nq, double *rep, double *zi,
                      int64_t *visits, int threads) {
    const qtree_t *t = (const qtree_t *)handle;
    if (!t || nq < 0) return -1;
    int64_t vsum = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : vsum)
#endif
    for (int64_t i = 0; i < nq; ++i) {
        double fx, fy, s;
        int64_t v = 0;
        qt_repulsive(t, 0, Q[2 * i], Q[2 * i + 1], theta, &fx, &fy, &s, &v);
        rep[2 * i] = fx; rep[2 * i + 1] = fy; zi[i] = s;
        vsum += v;
    }
    if (visits) *visits = vsum;
    return 0;
}

void oracle_tree_free(void *handle) {
    qtree_t *t = (qtree_t *)handle;
    if (!t) return;
    free(t->v);
    free(t);
}

/* Attraction + combine for rows [r0, r1) given the full repulsion and Z
 * (TsneHelpers.scala:269-317).  grad is (r1-r0) x 2; loss (nullable) is the
 * partial KL sum of these rows. */
int oracle_attraction_rows(const int64_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                           const double *Y, int metric, double exaggeration, const double *rep,
                           double Z, int64_t r0, int64_t r1, double *grad, double *loss) {
    if (!row_ptr || !Y || r0 < 0 || r1 > n || r0 > r1) return -1;
    double l = 0.0, l_c = 0.0;
    for (int64_t i = r0; i < r1; ++i) {
        double gx = 0.0, gy = 0.0;
        const double *yi = Y + 2 * i;
        for (int64_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            const double *yj = Y + 2 * (int64_t)col[e];
            double pij = val[e] * exaggeration;
            double qij = 1.0 / (1.0 + oracle_metric(yi, yj, 2, metric));
            double s = pij * qij;
            gx = gx + s * (yi[0] - yj[0]);
            gy = gy + s * (yi[1] - yj[1]);
            if (loss) kahan_add(&l, &l_c, pij * log(pij / (qij / Z)));
        }
        grad[2 * (i - r0)] = gx - rep[2 * i] / Z;
        grad[2 * (i - r0) + 1] = gy - rep[2 * i + 1] / Z;
    }
    if (loss) *loss = l + l_c;
    return 0;
}

/* ---------------------------------------------------- 3-D octree (extension)
 * The reference supports only 2-D embeddings (Cell.scala:32 requires
 * len == 2; nComponents = 3 crashes).  SURVEY.md section 8f defines the 3-D
 * extension as the natural generalisation, restated here and documented in
 * root Cell(0, 0, 0, W) with W = max(dX, dY, dZ); capacity 1;
 * subDivide halves hWidth for all three extents; children tried and summed
 * in the order upper (z >= cz) NW, NE, SW, SE, then lower NW, NE, SW, SE
 * (closed intervals: west iff x <= cx, north iff y >= cy, upper iff z >= cz);
 * criterion max(h) / D < theta with D the squared 3-D distance.
 * No reference output exists for this path: parity unpinned (self-consistency
 * of this restatement: theta = 0 equals the exact O(N^2) sums, tested). */
typedef struct {
    double x, y, z, hw;
    double sumx, sumy, sumz, comx, comy, comz;
    double px, py, pz;
    int32_t cum, leaf, has_point;
    int32_t child[8];
} onode_t;

typedef struct { onode_t *v; int64_t n, cap; } otree_t;

static int32_t ot_new(otree_t *t, double x, double y, double z, double hw) {
    if (t->n == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 1024;
        t->v = (onode_t *)realloc(t->v, sizeof(onode_t) * (size_t)t->cap);
    }
    onode_t *q = &t->v[t->n];
    memset(q, 0, sizeof(*q));
    q->x = x; q->y = y; q->z = z; q->hw = hw; q->leaf = 1;
    for (int c = 0; c < 8; ++c) q->child[c] = -1;
    return (int32_t)t->n++;
}

static int ocell_contains(const onode_t *q, double px, double py, double pz) {
    return (q->x - q->hw <= px) && (q->x + q->hw >= px) && (q->y - q->hw <= py) && (q->y + q->hw >= py) &&
           (q->z - q->hw <= pz) && (q->z + q->hw >= pz);
}

static int ot_insert(otree_t *t, int32_t ni, double px, double py, double pz);

static int ot_insert_sub(otree_t *t, int32_t ni, double px, double py, double pz) {
    for (int c = 0; c < 8; ++c) {
        int32_t ch = t->v[ni].child[c];
        if (ch >= 0 && ocell_contains(&t->v[ch], px, py, pz)) {
            if (ot_insert(t, ch, px, py, pz)) return 1;
        }
    }
    return 0;
}

static void ot_subdivide(otree_t *t, int32_t ni) {
    double x = t->v[ni].x, y = t->v[ni].y, z = t->v[ni].z, h = 0.5 * t->v[ni].hw;
    int32_t ch[8];
    for (int c = 0; c < 8; ++c) {
        double cx = (c & 1) ? x + h : x - h;     /* east : west */
        double cy = (c & 2) ? y - h : y + h;     /* south : north */
        double cz = (c & 4) ? z - h : z + h;     /* lower : upper */
        ch[c] = ot_new(t, cx, cy, cz, h);
    }
    for (int c = 0; c < 8; ++c) t->v[ni].child[c] = ch[c];
}

static int ot_insert(otree_t *t, int32_t ni, double px, double py, double pz) {
    onode_t *q = &t->v[ni];
    if (!ocell_contains(q, px, py, pz)) return 0;
    q->sumx += px; q->sumy += py; q->sumz += pz;
    q->cum += 1;
    q->comx = q->sumx / (double)q->cum;
    q->comy = q->sumy / (double)q->cum;
    q->comz = q->sumz / (double)q->cum;
    if (q->leaf) {
        if (q->has_point) {
            if (q->px == px && q->py == py && q->pz == pz) return 1;
            double lx = q->px, ly = q->py, lz = q->pz;
            ot_subdivide(t, ni);
            t->v[ni].leaf = 0;
            ot_insert_sub(t, ni, lx, ly, lz);
            ot_insert_sub(t, ni, px, py, pz);
            t->v[ni].has_point = 0;
            return 1;
        }
        q->has_point = 1; q->px = px; q->py = py; q->pz = pz;
        return 1;
    }
    return ot_insert_sub(t, ni, px, py, pz);
}

static void ot_repulsive(const otree_t *t, int32_t ni, double px, double py, double pz, double theta,
                         double *f, double *sq) {
    const onode_t *q = &t->v[ni];
    if ((q->leaf && q->cum == 0) || (q->leaf && q->px == px && q->py == py && q->pz == pz)) {
        f[0] = f[1] = f[2] = 0.0; *sq = 0.0;
        return;
    }
    double dx = px - q->comx, dy = py - q->comy, dz = pz - q->comz;
    double D = dx * dx + dy * dy + dz * dz;
    if (q->leaf || (q->hw / D < theta)) {
        double Q = 1.0 / (1.0 + D);
        double mult = (double)q->cum * Q;
        double s = mult * Q;
        *sq = 0.0 + mult;
        f[0] = s * dx; f[1] = s * dy; f[2] = s * dz;
        return;
    }
    double a[3] = {0, 0, 0}, as = 0;
    for (int c = 0; c < 8; ++c) {
        double cf[3], cs;
        ot_repulsive(t, q->child[c], px, py, pz, theta, cf, &cs);
        if (c == 0) { a[0] = cf[0]; a[1] = cf[1]; a[2] = cf[2]; as = cs; }
        else { a[0] = a[0] + cf[0]; a[1] = a[1] + cf[1]; a[2] = a[2] + cf[2]; as = as + cs; }
    }
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; *sq = as;
}

static void build_otree(otree_t *t, const double *Y, int64_t n) {
    double mn[3], mx[3];
    for (int k = 0; k < 3; ++k) mn[k] = mx[k] = Y[k];
    for (int64_t i = 1; i < n; ++i)
        for (int k = 0; k < 3; ++k) { mn[k] = fmin(mn[k], Y[3 * i + k]); mx[k] = fmax(mx[k], Y[3 * i + k]); }
    double W = fmax(fmax(mx[0] - mn[0], mx[1] - mn[1]), mx[2] - mn[2]);
    t->v = NULL; t->n = t->cap = 0;
    ot_new(t, 0.0, 0.0, 0.0, W);
    for (int64_t i = 0; i < n; ++i) ot_insert(t, 0, Y[3 * i], Y[3 * i + 1], Y[3 * i + 2]);
}

int oracle_gradient3(const int64_t *row_ptr, const int32_t *col, const double *val,
                     int64_t n, const double *Y, int metric, double theta,
                     double exaggeration, double *grad, double *sumq_out, double *loss_out,
                     double *rep_out, double *zi_out, int threads) {
    if (!row_ptr || !Y || n < 1) return -1;
    otree_t t;
    build_otree(&t, Y, n);
    double *rep = (double *)malloc(sizeof(double) * 3 * (size_t)n);
    double *zi = (double *)malloc(sizeof(double) * (size_t)n);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
#endif
    for (int64_t i = 0; i < n; ++i)
        ot_repulsive(&t, 0, Y[3 * i], Y[3 * i + 1], Y[3 * i + 2], theta, rep + 3 * i, zi + i);
    free(t.v);
    double Z = 0.0;
    for (int64_t i = 0; i < n; ++i) Z = Z + zi[i];
    double loss = 0.0, loss_c = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double g[3] = {0, 0, 0};
        const double *yi = Y + 3 * i;
        for (int64_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            const double *yj = Y + 3 * (int64_t)col[e];
            double pij = val[e] * exaggeration;
            double qij = 1.0 / (1.0 + oracle_metric(yi, yj, 3, metric));
            double s = pij * qij;
            for (int k = 0; k < 3; ++k) g[k] = g[k] + s * (yi[k] - yj[k]);
            if (loss_out) kahan_add(&loss, &loss_c, pij * log(pij / (qij / Z)));
        }
        for (int k = 0; k < 3; ++k) grad[3 * i + k] = g[k] - rep[3 * i + k] / Z;
    }
    if (sumq_out) *sumq_out = Z;
    if (loss_out) *loss_out = loss + loss_c;
    if (rep_out) memcpy(rep_out, rep, sizeof(double) * 3 * (size_t)n);
    if (zi_out) memcpy(zi_out, zi, sizeof(double) * (size_t)n);
    free(rep); free(zi);
    return 0;
}

int oracle_optimize3(const int64_t *row_ptr, const int32_t *col, const double *val,
                     int64_t n, double *Y, double *upd, double *gains, int metric,
                     double learning_rate, int32_t iterations, double early_exaggeration,
                     double initial_momentum, double final_momentum, double theta,
                     int32_t *loss_keys, double *loss_vals, int32_t *n_loss, int threads) {
    int32_t n1 = iterations < 20 ? iterations : 20;
    int32_t n2 = (iterations - n1) < 81 ? (iterations - n1) : 81;
    int32_t nl = 0;
    double *grad = (double *)malloc(sizeof(double) * 3 * (size_t)n);
    for (int32_t t = 1; t <= iterations; ++t) {
        double ex = (t <= n1 + n2) ? early_exaggeration : 1.0;
        double mom = (t <= n1) ? initial_momentum : final_momentum;
        int want_loss = (t % 10 == 0);
        double loss = 0.0, Z = 0.0;
        oracle_gradient3(row_ptr, col, val, n, Y, metric, theta, ex, grad, &Z,
                         want_loss ? &loss : NULL, NULL, NULL, threads);
        if (want_loss && loss_keys) { loss_keys[nl] = t; loss_vals[nl] = loss; ++nl; }
        oracle_update(n, 3, grad, Y, upd, gains, 0.01, mom, learning_rate);
        oracle_center(n, 3, Y);
    }
    if (n_loss) *n_loss = nl;
    free(grad);
    return 0;
}

/* 3-D sharded-path helpers (the 2-D ones above, one more component). */
int oracle_repulsion3_queries(const double *Y, int64_t n, double theta, const double *Q, int64_t nq,
                              double *rep, double *zi, int threads) {
    if (!Y || n < 1 || nq < 0) return -1;
    otree_t t;
    build_otree(&t, Y, n);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
#endif
    for (int64_t i = 0; i < nq; ++i)
        ot_repulsive(&t, 0, Q[3 * i], Q[3 * i + 1], Q[3 * i + 2], theta, rep + 3 * i, zi + i);
    free(t.v);
    return 0;
}

int oracle_attraction3_rows(const int64_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                            const double *Y, int metric, double exaggeration, const double *rep,
                            double Z, int64_t r0, int64_t r1, double *grad, double *loss) {
    if (!row_ptr || !Y || r0 < 0 || r1 > n || r0 > r1) return -1;
    double l = 0.0, l_c = 0.0;
    for (int64_t i = r0; i < r1; ++i) {
        double g[3] = {0, 0, 0};
        const double *yi = Y + 3 * i;
        for (int64_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            const double *yj = Y + 3 * (int64_t)col[e];
            double pij = val[e] * exaggeration;
            double qij = 1.0 / (1.0 + oracle_metric(yi, yj, 3, metric));
            double s = pij * qij;
            for (int k = 0; k < 3; ++k) g[k] = g[k] + s * (yi[k] - yj[k]);
            if (loss) kahan_add(&l, &l_c, pij * log(pij / (qij / Z)));
        }
        for (int k = 0; k < 3; ++k) grad[3 * (i - r0) + k] = g[k] - rep[3 * i + k] / Z;
    }
    if (loss) *loss = l + l_c;
    return 0;
}

/* ------------------------------------------------------------ projectKnn
 * Approximate kNN of TsneHelpers.scala:93-160 with ZOrder.scala:25-42:
 * for the input and for each shifted copy x + r_s (r_s = the caller's
 * uniform [0,1)^d vectors, `iterations - 1` of them; the reference draws them
 * unseeded), sort the points by the Z-order comparator and take the k
 * points on either side of each point as candidates; the union of candidates
 * is ranked by the exact metric on the ORIGINAL vectors and the k nearest
 * kept, ordered by (distance, j).  compareByZorder XORs the raw IEEE bit
 * patterns as SIGNED Java longs (less_msb); it is a total order for
 * nonnegative inputs, the only case with a defined result (the parity tests
 * use such data); exact duplicate vectors are ordered by index here. */
static int z_greater(const double *a, const double *b, int32_t d) {
    int32_t j = 0;
    int64_t x = 0;
    for (int32_t i = 0; i < d; ++i) {
        int64_t ai, bi;
        memcpy(&ai, a + i, 8);
        memcpy(&bi, b + i, 8);
        int64_t y = ai ^ bi;
        if ((x < y) && (x < (x ^ y))) { j = i; x = y; }
    }
    return a[j] > b[j];
}

static const double *g_zx;
static int32_t g_zd;
static int z_cmp(const void *pa, const void *pb) {
    int32_t i = *(const int32_t *)pa, j = *(const int32_t *)pb;
    const double *a = g_zx + (int64_t)i * g_zd, *b = g_zx + (int64_t)j * g_zd;
    if (z_greater(b, a, g_zd)) return -1;
    if (z_greater(a, b, g_zd)) return 1;
    return (i > j) - (i < j);
}

int oracle_project_knn(const double *X, int64_t n, int32_t d, int metric, int32_t k, int32_t iterations,
                       const double *shifts, int32_t *idx, double *dist) {
    if (!X || n < 2 || d < 1 || k < 1 || iterations < 1) return -1;
    const int32_t kk = (int32_t)(k < n - 1 ? k : n - 1);
    int32_t S = iterations;
    int32_t **order = (int32_t **)malloc(sizeof(int32_t *) * S);
    int32_t **rank = (int32_t **)malloc(sizeof(int32_t *) * S);
    double *Xs = (double *)malloc(sizeof(double) * (size_t)(n * d));
    for (int32_t s = 0; s < S; ++s) {
        for (int64_t i = 0; i < n; ++i)
            for (int32_t c = 0; c < d; ++c)
                Xs[i * d + c] = s == 0 ? X[i * d + c] : X[i * d + c] + shifts[(int64_t)(s - 1) * d + c];
        order[s] = (int32_t *)malloc(sizeof(int32_t) * n);
        rank[s] = (int32_t *)malloc(sizeof(int32_t) * n);
        for (int64_t i = 0; i < n; ++i) order[s][i] = (int32_t)i;
        g_zx = Xs; g_zd = d;
        qsort(order[s], (size_t)n, sizeof(int32_t), z_cmp);
        for (int64_t p = 0; p < n; ++p) rank[s][order[s][p]] = (int32_t)p;
    }
    free(Xs);
    int64_t cap = (int64_t)2 * k * S;
    dj_t *c = (dj_t *)malloc(sizeof(dj_t) * (size_t)cap);
    for (int64_t i = 0; i < n; ++i) {
        int64_t m = 0;
        for (int32_t s = 0; s < S; ++s) {
            int64_t p = rank[s][i];
            for (int64_t q = p - k; q <= p + k; ++q) {
                if (q < 0 || q >= n || q == p) continue;
                int32_t j = order[s][q];
                int dup = 0;
                for (int64_t t = 0; t < m; ++t) if (c[t].j == j) { dup = 1; break; }
                if (dup) continue;
                c[m].j = j;
                c[m].d = oracle_metric(X + i * d, X + (int64_t)j * d, d, metric);
                ++m;
            }
        }
        qsort(c, (size_t)m, sizeof(dj_t), cmp_dj);
        for (int32_t t = 0; t < kk; ++t) { idx[i * kk + t] = c[t].j; dist[i * kk + t] = c[t].d; }
    }
    free(c);
    for (int32_t s = 0; s < S; ++s) { free(order[s]); free(rank[s]); }
    free(order); free(rank);
    return 0;
}
