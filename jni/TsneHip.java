/*
 * TsneHip.java -- JNI declarations of libtsne_hip for the Flink job
 * (the drop-in for TsneHelpers.scala's hot path; see INTEGRATION.md).
 * Buffers are direct ByteBuffers in native byte order; int returns are
 * tsne_status values (the shim already threw on error).  Compiled where a JDK
 * 6-8 exists (Flink 0.9 / Scala 2.10, pom.xml:216-217); none in this image.
 */
package de.tu_berlin.dima.impro3;

import java.nio.ByteBuffer;

public final class TsneHip {
    static { System.loadLibrary("tsne_hip_jni"); }   // links libtsne_hip.so

    private TsneHip() {}

    /** tsne_ctx_create: one GPU. */
    public static native long ctxCreate(int device);
    /** tsne_ctx_create_multi: one handle over several GPUs (RCCL over xGMI); knn and
     *  optimize fan out over them from this one call (SURVEY.md 8b "Threading"). */
    public static native long ctxCreateMulti(int[] devices);
    public static native void ctxDestroy(long ctx);

    /** Tsne.getMetric (Tsne.scala:161-168): unknown name -> IllegalArgumentException. */
    public static native int metricFromName(String name);

    /** kNearestNeighbors / partitionKnn (TsneHelpers.scala:41-91), query rows [q0, q1). */
    public static native int knn(long ctx, ByteBuffer X, long n, int d, int metric, int k, long q0, long q1,
                                 ByteBuffer idxOut, ByteBuffer distOut);
    /** projectKnn (TsneHelpers.scala:93-160): shifts = (iterations-1) x d doubles. */
    public static native int projectKnn(long ctx, ByteBuffer X, long n, int d, int metric, int k, int iterations,
                                        ByteBuffer shifts, ByteBuffer idxOut, ByteBuffer distOut);
    /** pairwiseAffinities (TsneHelpers.scala:162-180) over CSR rows. */
    public static native int pairwiseAffinities(long ctx, ByteBuffer rowPtr, ByteBuffer dist, long nrows,
                                                double perplexity, ByteBuffer pOut);
    /** jointDistribution (TsneHelpers.scala:182-196); returns nnz (> cap: buffers too small, nothing written). */
    public static native long jointDistribution(long ctx, ByteBuffer rowPtr, ByteBuffer col, ByteBuffer p, long n,
                                                long cap, ByteBuffer outRowPtr, ByteBuffer outCol,
                                                ByteBuffer outVal);
    /** optimize (TsneHelpers.scala:396-430): all iterations on the GPU(s); Y, upd, gains in place;
     *  returns the number of (iteration, KL) pairs written to lossKeys / lossVals. */
    public static native int optimize(long ctx, int nComponents, double learningRate, int iterations, int metric,
                                      double earlyExaggeration, double initialMomentum, double finalMomentum,
                                      double theta, ByteBuffer rowPtr, ByteBuffer col, ByteBuffer P, long n,
                                      ByteBuffer Y, ByteBuffer upd, ByteBuffer gains, ByteBuffer lossKeys,
                                      ByteBuffer lossVals);
    /** initWorkingSet (TsneHelpers.scala:198-219), seeded by --randomState. */
    public static native int initWorkingSet(long ctx, long n, int nComponents, long seed, ByteBuffer Y,
                                            ByteBuffer upd, ByteBuffer gains);

    public static native String lastError();
}
