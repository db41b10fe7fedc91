/*
 * tsne_hip_jni.c -- the JNI shim between TsneHip.java and the C ABI of
 * libtsne_hip (include/tsne_hip.h).  One C call per Java method: off-heap
 * addresses (jlong, from sun.misc.Unsafe.allocateMemory) and 64-bit sizes in,
 * tsne_status out; a non-zero status becomes IllegalArgumentException
 * (TSNE_ERR_ARG, the reference's exception for an unknown metric / method:
 * Tsne.scala:78,166) or RuntimeException.
 *
 * Build (where a JDK exists; there is none in this image):
 *   make -C jni JAVA_HOME=/usr/lib/jvm/java-8-openjdk-amd64
 * The header and shim compile without a JDK against jni/jni_stub for the
 * signature check in tests/test_jni_shim.py (never linked or run).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "tsne_hip.h"

#define CTX(x) ((tsne_ctx *)(intptr_t)(x))
#define PTR(T, a) ((T *)(intptr_t)(a))
#define JNI_FN(name) JNICALL Java_de_tu_1berlin_dima_impro3_TsneHip_##name

static jint chk(JNIEnv *e, int rc) {
    if (rc != TSNE_OK) {
        const char *cls = rc == TSNE_ERR_ARG ? "java/lang/IllegalArgumentException" : "java/lang/RuntimeException";
        jclass k = (*e)->FindClass(e, cls);
        if (k) (*e)->ThrowNew(e, k, tsne_last_error());
    }
    return rc;
}

JNIEXPORT jlong JNI_FN(ctxCreate)(JNIEnv *e, jclass c, jint dev) {
    tsne_ctx *ctx = NULL;
    (void)c;
    chk(e, tsne_ctx_create(dev, &ctx));
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT jlong JNI_FN(ctxCreateMulti)(JNIEnv *e, jclass c, jintArray devs) {
    tsne_ctx *ctx = NULL;
    (void)c;
    const jsize n = (*e)->GetArrayLength(e, devs);
    jint *d = (*e)->GetIntArrayElements(e, devs, NULL);
    int32_t *dv = (int32_t *)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    for (jsize i = 0; i < n; ++i) dv[i] = d[i];
    (*e)->ReleaseIntArrayElements(e, devs, d, JNI_ABORT);
    chk(e, tsne_ctx_create_multi(dv, n, &ctx));
    free(dv);
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNI_FN(ctxDestroy)(JNIEnv *e, jclass c, jlong ctx) {
    (void)e; (void)c;
    tsne_ctx_destroy(CTX(ctx));
}

/* Per-handle tunables (tsne_ctx_set_option); unknown keys / bad values throw
 * IllegalArgumentException. */
JNIEXPORT void JNI_FN(ctxSetOption)(JNIEnv *e, jclass c, jlong ctx, jstring key, jdouble value) {
    (void)c;
    const char *k = (*e)->GetStringUTFChars(e, key, NULL);
    const int rc = tsne_ctx_set_option(CTX(ctx), k, value);
    (*e)->ReleaseStringUTFChars(e, key, k);
    chk(e, rc);
}

JNIEXPORT jint JNI_FN(metricFromName)(JNIEnv *e, jclass c, jstring name) {
    (void)c;
    const char *s = (*e)->GetStringUTFChars(e, name, NULL);
    int32_t m = -1;
    const int rc = tsne_metric_from_name(s, &m);
    (*e)->ReleaseStringUTFChars(e, name, s);
    chk(e, rc);
    return m;
}

JNIEXPORT void JNI_FN(cooToCsr)(JNIEnv *e, jclass c, jlong row, jlong col, jlong val, jlong nnz, jlong n,
                                jlong rp, jlong oc, jlong ov) {
    (void)c;
    chk(e, tsne_coo_to_csr(PTR(const int32_t, row), PTR(const int32_t, col), PTR(const double, val), nnz, n,
                           PTR(int64_t, rp), PTR(int32_t, oc), PTR(double, ov)));
}

JNIEXPORT jint JNI_FN(knn)(JNIEnv *e, jclass c, jlong ctx, jlong X, jlong n, jint d, jint metric, jint k,
                           jlong q0, jlong q1, jlong idx, jlong dist) {
    (void)c;
    return chk(e, tsne_knn(CTX(ctx), PTR(const double, X), n, d, metric, k, q0, q1, PTR(int32_t, idx),
                           PTR(double, dist)));
}

JNIEXPORT jint JNI_FN(projectKnn)(JNIEnv *e, jclass c, jlong ctx, jlong X, jlong n, jint d, jint metric, jint k,
                                  jint it, jlong shifts, jlong idx, jlong dist) {
    (void)c;
    return chk(e, tsne_project_knn(CTX(ctx), PTR(const double, X), n, d, metric, k, it, PTR(const double, shifts),
                                   PTR(int32_t, idx), PTR(double, dist)));
}

JNIEXPORT jint JNI_FN(pairwiseAffinities)(JNIEnv *e, jclass c, jlong ctx, jlong rp, jlong dist, jlong nrows,
                                          jdouble perp, jlong p) {
    (void)c;
    return chk(e, tsne_pairwise_affinities(CTX(ctx), PTR(const int64_t, rp), PTR(const double, dist), nrows, perp,
                                           PTR(double, p)));
}

JNIEXPORT jlong JNI_FN(jointDistribution)(JNIEnv *e, jclass c, jlong ctx, jlong rp, jlong col, jlong p, jlong n,
                                          jlong cap, jlong orp, jlong oc, jlong ov) {
    (void)c;
    int64_t nnz = 0;
    const int rc = tsne_joint_distribution(CTX(ctx), PTR(const int64_t, rp), PTR(const int32_t, col),
                                           PTR(const double, p), n, cap, PTR(int64_t, orp), PTR(int32_t, oc),
                                           PTR(double, ov), &nnz);
    if (rc != TSNE_ERR_CAPACITY) chk(e, rc);   /* capacity: the caller re-allocates nnz entries */
    return nnz;
}

JNIEXPORT jint JNI_FN(optimize)(JNIEnv *e, jclass c, jlong ctx, jint nc, jdouble lr, jint it, jint metric,
                                jdouble ex, jdouble m0, jdouble m1, jdouble theta, jlong rp, jlong col, jlong P,
                                jlong n, jlong Y, jlong upd, jlong gains, jlong lk, jlong lv) {
    (void)c;
    tsne_params p;
    tsne_params_default(&p);
    p.n_components = nc;   /* 2, or 3 for the octree extension (Y, upd, gains: n x nc) */
    p.learning_rate = lr;
    p.iterations = it;
    p.metric = metric;
    p.early_exaggeration = ex;
    p.initial_momentum = m0;
    p.final_momentum = m1;
    p.theta = theta;
    int32_t nl = 0;
    chk(e, tsne_optimize(CTX(ctx), &p, PTR(const int64_t, rp), PTR(const int32_t, col), PTR(const double, P), n,
                         PTR(double, Y), PTR(double, upd), PTR(double, gains), PTR(int32_t, lk), PTR(double, lv),
                         it / 10 + 1, &nl));
    return nl;
}

JNIEXPORT jint JNI_FN(initWorkingSet)(JNIEnv *e, jclass c, jlong ctx, jlong n, jint nc, jlong seed, jlong Y,
                                      jlong upd, jlong gains) {
    (void)c;
    return chk(e, tsne_init_working_set(CTX(ctx), n, nc, (uint64_t)seed, PTR(double, Y), PTR(double, upd),
                                        PTR(double, gains)));
}

JNIEXPORT jstring JNI_FN(lastError)(JNIEnv *e, jclass c) {
    (void)c;
    return (*e)->NewStringUTF(e, tsne_last_error());
}
