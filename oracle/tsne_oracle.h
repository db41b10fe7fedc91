/*
 * tsne_oracle.h -- CPU fp64 restatement of the tsne-flink hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libtsne_hip / the
 * tsne-flink_amd package) links, loads or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Every function restates one piece of the reference (ChristophAl/tsne-flink,
 * Scala/Flink) exactly as the reference computes it, in fp64, in the same
 * evaluation order where the order is defined by the reference code:
 *   kNearestNeighbors        TsneHelpers.scala:41-59
 *   pairwiseAffinities       TsneHelpers.scala:162-180, 434-504
 *   jointDistribution        TsneHelpers.scala:182-196
 *   gradient (quadtree BH)   TsneHelpers.scala:221-318, QuadTree.scala:38-152, Cell.scala:31-36
 *   updateEmbedding          TsneHelpers.scala:341-369
 *   centerEmbedding          TsneHelpers.scala:320-329
 *   optimize / iteration     TsneHelpers.scala:371-430
 *   metrics                  Tsne.scala:161-168 (breeze squaredDistance /
 *                            euclideanDistance / cosineDistance)
 *
 * Parity pinning: checked against every golden vector of
 * TsneHelpersTestSuite.scala (tests/golden/reference_goldens.json).
 * Not pinned by any reference golden (restatement-only, "parity unpinned"):
 * theta > 0, euclidean / cosine metrics, multi-iteration trajectories, loss
 * values, tie order (the reference leaves it to Flink's sort; we order by
 * (distance, index)).
 */
#ifndef TSNE_ORACLE_H
#define TSNE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_SQEUCLIDEAN = 0, ORACLE_EUCLIDEAN = 1, ORACLE_COSINE = 2 };

/* breeze metric on two fp64 vectors of length d (Tsne.scala:161-168). */
double oracle_metric(const double *a, const double *b, int32_t d, int metric);

/* Brute-force kNN (TsneHelpers.scala:41-59): for every row i the
 * kk = min(k, n-1) smallest metric(x_i, x_j) over j != i, ascending by
 * (d, j).  X is row-major n x d.  idx/dist are n x kk.  `threads` > 1 uses
 * OpenMP over query rows (CPU baseline only).  Rows [q0, q1) only. */
int oracle_knn(const double *X, int64_t n, int32_t d, int metric, int32_t k,
               int64_t q0, int64_t q1, int32_t *idx, double *dist, int threads);

/* Perplexity binary search per CSR row (TsneHelpers.scala:434-504).
 * iters_out (nullable) receives the number of beta updates per row. */
int oracle_affinities(const int64_t *row_ptr, const double *dist, int64_t nrows,
                      double perplexity, double *p_out, int32_t *iters_out);

/* Symmetrisation (TsneHelpers.scala:182-196): J = P + P^T over the union of
 * the pattern and its transpose (explicit zeros kept), then J / sum(J).
 * Output CSR rows sorted by column.  Returns -2 if cap < nnz (nnz_out set). */
int oracle_joint(const int64_t *row_ptr, const int32_t *col, const double *p,
                 int64_t n, int64_t *out_row_ptr, int32_t *out_col, double *out_val,
                 int64_t cap, int64_t *nnz_out);

/* One gradient evaluation (TsneHelpers.scala:221-318) with the reference
 * pointer quadtree (QuadTree.scala) built in row order.  P values are
 * multiplied by `exaggeration` first (TsneHelpers.scala:410).  Y is n x 2.
 * grad (n x 2) = attr - rep / Z.  Optional outputs (nullable): sumq (Z),
 * loss (sum of p*ln(p/(q/Z)), TsneHelpers.scala:297-299), rep (n x 2 raw
 * repulsive force), zi (n, per-point sum of Q), attr (n x 2),
 * visits (n, nodes touched per query). */
int oracle_gradient(const int64_t *row_ptr, const int32_t *col, const double *val,
                    int64_t n, const double *Y, int metric, double theta,
                    double exaggeration, double *grad, double *sumq, double *loss,
                    double *rep, double *zi, double *attr, int64_t *visits, int threads);

/* BH repulsion only, for queries [q0, q1) against the tree of all n points
 * (used by the CPU baseline sample). */
int oracle_repulsion(const double *Y, int64_t n, double theta, int64_t q0, int64_t q1,
                     double *rep, double *zi, int threads);

/* Repulsion of an arbitrary query list Q (nq x 2) against the tree of Y. */
int oracle_repulsion_queries(const double *Y, int64_t n, double theta, const double *Q, int64_t nq,
                             double *rep, double *zi, int threads);

/* The reference tree of all n points built once (serial, row order), then
 * queried in batches: the CPU baseline times the build and the queries apart.
 * visits (nullable) = nodes touched over the batch.  Free with
 * oracle_tree_free. */
void *oracle_tree_build(const double *Y, int64_t n);
int oracle_tree_query(const void *tree, double theta, const double *Q, int64_t nq, double *rep, double *zi,
                      int64_t *visits, int threads);
void oracle_tree_free(void *tree);

/* Attraction + combine for rows [r0, r1) given full rep (n x 2) and Z. */
int oracle_attraction_rows(const int64_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                           const double *Y, int metric, double exaggeration, const double *rep,
                           double Z, int64_t r0, int64_t r1, double *grad, double *loss);

/* updateEmbedding (TsneHelpers.scala:341-369), in place. */
int oracle_update(int64_t n, int32_t c, const double *grad, double *Y, double *upd,
                  double *gains, double min_gain, double momentum, double lr);

/* centerEmbedding (TsneHelpers.scala:320-329), in place. */
int oracle_center(int64_t n, int32_t c, double *Y);

/* optimize (TsneHelpers.scala:396-430) from an injected working set
 * (Y, upd, gains), all n x 2, updated in place.  loss_keys/loss_vals get
 * one entry per iteration t with t % 10 == 0 (capacity iterations/10). */
int oracle_optimize(const int64_t *row_ptr, const int32_t *col, const double *val,
                    int64_t n, double *Y, double *upd, double *gains, int metric,
                    double learning_rate, int32_t iterations, double early_exaggeration,
                    double initial_momentum, double final_momentum, double theta,
                    int32_t *loss_keys, double *loss_vals, int32_t *n_loss, int threads);

/* 3-D extension (octree): the natural generalisation of the
 * quadtree path, defined in tsne_oracle.c; Y, grad, rep are n x 3.
 * Parity unpinned (no reference output exists for nComponents = 3). */
int oracle_gradient3(const int64_t *row_ptr, const int32_t *col, const double *val,
                     int64_t n, const double *Y, int metric, double theta,
                     double exaggeration, double *grad, double *sumq, double *loss,
                     double *rep, double *zi, int threads);
/* projectKnn (TsneHelpers.scala:93-160, ZOrder.scala:25-42): Z-order
 * neighbours of the input and of `iterations - 1` shifted copies (shifts:
 * (iterations-1) x d, caller-supplied), ranked by the exact metric; idx/dist
 * n x min(k, n-1), ascending by (d, j).  Defined for nonnegative inputs. */
int oracle_project_knn(const double *X, int64_t n, int32_t d, int metric, int32_t k, int32_t iterations,
                       const double *shifts, int32_t *idx, double *dist);
int oracle_repulsion3_queries(const double *Y, int64_t n, double theta, const double *Q, int64_t nq,
                              double *rep, double *zi, int threads);
int oracle_attraction3_rows(const int64_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                            const double *Y, int metric, double exaggeration, const double *rep,
                            double Z, int64_t r0, int64_t r1, double *grad, double *loss);
int oracle_optimize3(const int64_t *row_ptr, const int32_t *col, const double *val,
                     int64_t n, double *Y, double *upd, double *gains, int metric,
                     double learning_rate, int32_t iterations, double early_exaggeration,
                     double initial_momentum, double final_momentum, double theta,
                     int32_t *loss_keys, double *loss_vals, int32_t *n_loss, int threads);

#ifdef __cplusplus
}
#endif
#endif
