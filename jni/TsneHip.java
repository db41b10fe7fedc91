/*
 * TsneHip.java -- JNI declarations of libtsne_hip for the Flink job
 * (the drop-in for TsneHelpers.scala's hot path; see INTEGRATION.md).
 * Every buffer is an off-heap address (sun.misc.Unsafe.allocateMemory, the
 * same memory Flink's own MemorySegments use) with 64-bit element counts, so
 * no argument is bounded by a 2 GiB ByteBuffer: C5's 2.5e9-entry distance
 * matrix crosses as it is.  int returns are tsne_status values (the shim
 * already threw on error).  Compiled where a JDK 6-8 exists (Flink 0.9 /
 * Scala 2.10, pom.xml:216-217); none in this image.
 */
package de.tu_berlin.dima.impro3;

public final class TsneHip {
    static { System.loadLibrary("tsne_hip_jni"); }   // links libtsne_hip.so

    private TsneHip() {}

    /** tsne_ctx_create: one GPU. */
    public static native long ctxCreate(int device);
    /** tsne_ctx_create_multi: one handle over several GPUs (RCCL over xGMI); knn and
     *  optimize fan out over them from this one call (SURVEY.md 8b "Threading"). */
    public static native long ctxCreateMulti(int[] devices);
    public static native void ctxDestroy(long ctx);
    /** tsne_ctx_set_option: per-handle tunables (include/tsne_hip.h; the defaults are the library's choices). */
    public static native void ctxSetOption(long ctx, String key, double value);

    /** Tsne.getMetric (Tsne.scala:161-168): unknown name -> IllegalArgumentException. */
    public static native int metricFromName(String name);

    /** tsne_coo_to_csr: the groupBy(0) of a triple DataSet (stable, rows in index order). */
    public static native void cooToCsr(long row, long col, long val, long nnz, long n, long rowPtrOut,
                                       long colOut, long valOut);

    /** kNearestNeighbors / partitionKnn (TsneHelpers.scala:41-91), query rows [q0, q1);
     *  X: n x d doubles, idxOut: (q1-q0) x min(k, n-1) ints, distOut the same in doubles. */
    public static native int knn(long ctx, long X, long n, int d, int metric, int k, long q0, long q1,
                                 long idxOut, long distOut);
    /** projectKnn (TsneHelpers.scala:93-160): shifts = (iterations-1) x d doubles. */
    public static native int projectKnn(long ctx, long X, long n, int d, int metric, int k, int iterations,
                                        long shifts, long idxOut, long distOut);
    /** pairwiseAffinities (TsneHelpers.scala:162-180) over CSR rows (rowPtr: nrows + 1 longs). */
    public static native int pairwiseAffinities(long ctx, long rowPtr, long dist, long nrows, double perplexity,
                                                long pOut);
    /** jointDistribution (TsneHelpers.scala:182-196); returns nnz (> cap: buffers too small, nothing written). */
    public static native long jointDistribution(long ctx, long rowPtr, long col, long p, long n, long cap,
                                                long outRowPtr, long outCol, long outVal);
    /** optimize (TsneHelpers.scala:396-430): all iterations on the GPU(s); Y, upd, gains in place;
     *  returns the number of (iteration, KL) pairs written to lossKeys (ints) / lossVals (doubles). */
    public static native int optimize(long ctx, int nComponents, double learningRate, int iterations, int metric,
                                      double earlyExaggeration, double initialMomentum, double finalMomentum,
                                      double theta, long rowPtr, long col, long P, long n, long Y, long upd,
                                      long gains, long lossKeys, long lossVals);
    /** initWorkingSet (TsneHelpers.scala:198-219), seeded by --randomState. */
    public static native int initWorkingSet(long ctx, long n, int nComponents, long seed, long Y, long upd,
                                            long gains);

    public static native String lastError();
}
