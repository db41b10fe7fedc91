/*
 * TsneHipOperators.scala -- bodies for the hot-path methods of TsneHelpers
 * (TsneHelpers.scala:41-59, 61-91, 162-196, 396-430) that call libtsne_hip
 * through TsneHip (JNI).  Same DataSet types and argument meaning as the
 * reference; each body is one operator at parallelism 1 on the GPU node that
 * collects its input into direct buffers (the reference already builds the
 * quadtree at parallelism 1, TsneHelpers.scala:234) and makes ONE library
 * call -- the optimizer runs every iteration on the GPU(s) with the embedding
 * resident in HBM, and its (iteration, KL) pairs are fed into the same "loss"
 * MapAccumulator the reference fills (TsneHelpers.scala:281,297-300), so
 * Tsne.scala:97-101 writes the same loss file.
 *
 * The metric is passed by NAME (Tsne.getMetric's names, Tsne.scala:161-168)
 * instead of as a breeze function: computeEmbedding passes `metricName`
 * alongside.  GPU list: TsneHipOperators.devices (all GPUs of the node).
 * Source only in this image (no scalac / JDK).
 */
package de.tu_berlin.dima.impro3

import java.nio.{ByteBuffer, ByteOrder}

import breeze.linalg.{DenseVector, SparseVector, Vector}
import org.apache.flink.api.common.functions.RichGroupReduceFunction
import org.apache.flink.api.scala._
import org.apache.flink.configuration.Configuration
import org.apache.flink.util.Collector

import scala.collection.JavaConverters._

object TsneHipOperators {

  /** GPUs driven by one call (tsne_ctx_create_multi); one entry = one GPU. */
  @volatile var devices: Array[Int] = Array(0)

  private def direct(bytes: Long): ByteBuffer = {
    require(bytes <= Int.MaxValue, "a single direct buffer holds at most 2 GiB")
    ByteBuffer.allocateDirect(math.max(1L, bytes).toInt).order(ByteOrder.nativeOrder())
  }

  private def withCtx[T](f: Long => T): T = {
    val ctx = if (devices.length == 1) TsneHip.ctxCreate(devices(0)) else TsneHip.ctxCreateMulti(devices)
    try f(ctx) finally TsneHip.ctxDestroy(ctx)
  }

  /** CSR over triples grouped by row id: (row ids, row_ptr, col indices, values), ids dense-remapped. */
  private final case class Csr(ids: Array[Int], rowPtr: ByteBuffer, col: ByteBuffer, value: ByteBuffer, nnz: Long)

  private def toCsr(triples: Array[(Int, Int, Double)], ids: Array[Int]): Csr = {
    val index = ids.zipWithIndex.toMap
    val byRow = triples.groupBy(_._1)
    val n = ids.length
    val rp = direct(8L * (n + 1)); val col = direct(4L * triples.length); val v = direct(8L * triples.length)
    var e = 0L
    rp.putLong(0, 0L)
    for (r <- 0 until n) {
      for (t <- byRow.getOrElse(ids(r), Array.empty[(Int, Int, Double)])) {   // file / group order kept
        col.putInt((4 * e).toInt, index(t._2)); v.putDouble((8 * e).toInt, t._3); e += 1
      }
      rp.putLong(8 * (r + 1), e)
    }
    Csr(ids, rp, col, v, e)
  }

  // ---------------------------------------------------------------- kNN
  /** kNearestNeighbors (TsneHelpers.scala:41-59). */
  def kNearestNeighbors(input: DataSet[(Int, Vector[Double])], k: Int, metricName: String)
      : DataSet[(Int, Int, Double)] =
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val rows = it.toArray.sortBy(_._1)
      val n = rows.length
      if (n >= 2) {
        val d = rows(0)._2.length
        val X = direct(8L * n * d)
        rows.foreach(r => r._2.foreach(x => X.putDouble(x)))
        val kk = math.min(k, n - 1)
        val idx = direct(4L * n * kk); val dist = direct(8L * n * kk)
        withCtx { ctx =>
          TsneHip.knn(ctx, X, n, d, TsneHip.metricFromName(metricName), k, 0, n, idx, dist)
        }
        for (i <- 0 until n; t <- 0 until kk) {
          val o = i * kk + t
          out.collect((rows(i)._1, rows(idx.getInt(4 * o))._1, dist.getDouble(8 * o)))
        }
      }
    }.setParallelism(1)

  /** partitionKnn (TsneHelpers.scala:61-91): the same exact kNN; blocks are a tiling detail. */
  def partitionKnn(input: DataSet[(Int, Vector[Double])], k: Int, metricName: String, blocks: Int)
      : DataSet[(Int, Int, Double)] = kNearestNeighbors(input, k, metricName)

  // --------------------------------------------------------- affinities
  /** pairwiseAffinities (TsneHelpers.scala:162-180): beta search per row i. */
  def pairwiseAffinities(input: DataSet[(Int, Int, Double)], perplexity: Double): DataSet[(Int, Int, Double)] =
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val rows = it.toArray.groupBy(_._1).toArray.sortBy(_._1)     // (i, its triples in group order)
      val nnz = rows.map(_._2.length.toLong).sum
      val rp = direct(8L * (rows.length + 1)); val dist = direct(8L * nnz); val p = direct(8L * nnz)
      var e = 0
      for ((r, k) <- rows.zipWithIndex) {
        for (t <- r._2) { dist.putDouble(8 * e, t._3); e += 1 }
        rp.putLong(8 * (k + 1), e)
      }
      withCtx(ctx => TsneHip.pairwiseAffinities(ctx, rp, dist, rows.length, perplexity, p))
      e = 0
      for (r <- rows; t <- r._2) { out.collect((t._1, t._2, p.getDouble(8 * e))); e += 1 }
    }.setParallelism(1)

  /** jointDistribution (TsneHelpers.scala:182-196): P = (C + C^T) / sum over the union pattern. */
  def jointDistribution(input: DataSet[(Int, Int, Double)]): DataSet[(Int, Int, Double)] =
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val t = it.toArray
      val ids = (t.map(_._1) ++ t.map(_._2)).distinct.sorted
      val csr = toCsr(t, ids)
      val n = ids.length
      val cap = 2 * csr.nnz
      val orp = direct(8L * (n + 1)); val oc = direct(4L * cap); val ov = direct(8L * cap)
      val nnz = withCtx(ctx => TsneHip.jointDistribution(ctx, csr.rowPtr, csr.col, csr.value, n, cap, orp, oc, ov))
      for (r <- 0 until n; e <- orp.getLong(8 * r) until orp.getLong(8 * (r + 1)))
        out.collect((ids(r), ids(oc.getInt((4 * e).toInt)), ov.getDouble((8 * e).toInt)))
      require(nnz <= cap)
    }.setParallelism(1)

  // ---------------------------------------------------------- optimizer
  /** optimize (TsneHelpers.scala:396-430): the three phases and every iteration of
   *  iterationComputation (:371-394) in one call; the embedding never leaves the GPU. */
  def optimize(highDimAffinities: DataSet[(Int, SparseVector[Double])],
               initialWorkingSet: DataSet[(Int, Vector[Double], Vector[Double], Vector[Double])],
               learningRate: Double, iterations: Int, metricName: String, earlyExaggeration: Double,
               initialMomentum: Double, finalMomentum: Double, theta: Double, dimension: Int)
      : DataSet[(Int, Vector[Double])] =
    highDimAffinities.map(x => (0, x)).groupBy(0).reduceGroup(
      new RichGroupReduceFunction[(Int, (Int, SparseVector[Double])), (Int, Vector[Double])] {
        private val lossAccumulator = new MapAccumulator()
        private var workingSet: Seq[(Int, Vector[Double], Vector[Double], Vector[Double])] = null

        override def open(parameters: Configuration): Unit = {
          getRuntimeContext.addAccumulator("loss", lossAccumulator)   // TsneHelpers.scala:281
          workingSet = getRuntimeContext
            .getBroadcastVariable[(Int, Vector[Double], Vector[Double], Vector[Double])]("workingSet").asScala
        }

        override def reduce(it: java.lang.Iterable[(Int, (Int, SparseVector[Double]))],
                            out: Collector[(Int, Vector[Double])]): Unit = {
          val rows = it.asScala.map(_._2).toArray.sortBy(_._1)
          val ws = workingSet.sortBy(_._1).toArray
          val ids = ws.map(_._1)
          val index = ids.zipWithIndex.toMap
          val n = ids.length
          val c = dimension
          val nnz = rows.map(_._2.activeSize.toLong).sum
          val rp = direct(8L * (n + 1)); val col = direct(4L * nnz); val P = direct(8L * nnz)
          val byId = rows.map(r => r._1 -> r._2).toMap
          var e = 0L
          for (r <- 0 until n) {
            byId.get(ids(r)).foreach { sv =>
              for (o <- 0 until sv.activeSize) {
                col.putInt((4 * e).toInt, index(sv.indexAt(o))); P.putDouble((8 * e).toInt, sv.valueAt(o)); e += 1
              }
            }
            rp.putLong(8 * (r + 1), e)
          }
          val Y = direct(8L * n * c); val upd = direct(8L * n * c); val gains = direct(8L * n * c)
          for (r <- 0 until n; k <- 0 until c) {
            Y.putDouble(8 * (r * c + k), ws(r)._2(k))
            upd.putDouble(8 * (r * c + k), ws(r)._3(k))
            gains.putDouble(8 * (r * c + k), ws(r)._4(k))
          }
          val slots = iterations / 10 + 1
          val lk = direct(4L * slots); val lv = direct(8L * slots)
          val nl = withCtx { ctx =>
            TsneHip.optimize(ctx, c, learningRate, iterations, TsneHip.metricFromName(metricName),
              earlyExaggeration, initialMomentum, finalMomentum, theta, rp, col, P, n, Y, upd, gains, lk, lv)
          }
          for (s <- 0 until math.min(nl, slots))                        // the "loss" channel
            lossAccumulator.add((lk.getInt(4 * s), lv.getDouble(8 * s)))
          for (r <- 0 until n)
            out.collect((ids(r), DenseVector.tabulate(c)(k => Y.getDouble(8 * (r * c + k)))))
        }
      }).withBroadcastSet(initialWorkingSet, "workingSet").setParallelism(1)
}
