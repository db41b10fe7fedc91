/*
 * TsneHipOperators.scala -- drop-in bodies of the hot-path methods of
 * TsneHelpers (TsneHelpers.scala:41-59, 61-91, 93-160, 162-196, 396-430) that
 * call libtsne_hip through TsneHip (JNI), with the reference's exact
 * signatures: the metric is the same `(Vector[Double], Vector[Double]) =>
 * Double` that Tsne.getMetric returns (Tsne.scala:161-168), so
 * computeEmbedding (Tsne.scala:115-134) and Tsne.main (:74-84) change only in
 * the object they import (INTEGRATION.md §1).
 *
 * Each body is one operator at parallelism 1 on the GPU node (the reference
 * already builds the quadtree at parallelism 1, TsneHelpers.scala:234): it
 * streams its input iterator into off-heap arrays addressed by Long index
 * (sun.misc.Unsafe, as Flink's MemorySegments) and makes ONE library call;
 * nothing is bounded by JVM array or ByteBuffer sizes (C5's 2.5e9-entry
 * distance matrix crosses as it is, host memory permitting).  The optimizer
 * runs every iteration on the GPU(s) with the embedding resident in HBM, and
 * its (iteration, KL) pairs are fed into the same "loss" MapAccumulator the
 * reference fills (TsneHelpers.scala:281,297-300), so Tsne.scala:97-101 writes
 * the same loss file.  GPU list: TsneHipOperators.devices.
 * Source only in this image (no scalac / JDK).
 */
package de.tu_berlin.dima.impro3

import breeze.linalg.{DenseVector, SparseVector, Vector, cosineDistance, euclideanDistance, squaredDistance}
import org.apache.flink.api.common.functions.RichGroupReduceFunction
import org.apache.flink.api.scala._
import org.apache.flink.configuration.Configuration
import org.apache.flink.util.Collector

import scala.collection.JavaConverters._

/** Off-heap arrays with 64-bit indexes (freed explicitly; every body frees what it allocates). */
private[impro3] object OffHeap {
  val U: sun.misc.Unsafe = {
    val f = classOf[sun.misc.Unsafe].getDeclaredField("theUnsafe")
    f.setAccessible(true)
    f.get(null).asInstanceOf[sun.misc.Unsafe]
  }

  /** A growable off-heap array of `width`-byte elements (for an iterator of unknown length). */
  final class Buf(width: Int, initial: Long = 1L << 16) {
    private var cap = math.max(1L, initial)
    var addr: Long = U.allocateMemory(cap * width)
    var length = 0L
    def reserve(n: Long): Unit = if (n > cap) {
      while (cap < n) cap *= 2
      addr = U.reallocateMemory(addr, cap * width)
    }
    def free(): Unit = if (addr != 0L) { U.freeMemory(addr); addr = 0L }
  }
  final class Ints(n: Long = 0L) {
    val b = new Buf(4, math.max(n, 1L)); b.length = n
    def apply(i: Long): Int = U.getInt(b.addr + 4 * i)
    def update(i: Long, v: Int): Unit = U.putInt(b.addr + 4 * i, v)
    def +=(v: Int): Unit = { b.reserve(b.length + 1); U.putInt(b.addr + 4 * b.length, v); b.length += 1 }
    def addr: Long = b.addr
    def length: Long = b.length
    def free(): Unit = b.free()
  }
  final class Longs(n: Long) {
    val b = new Buf(8, math.max(n, 1L)); b.length = n
    def apply(i: Long): Long = U.getLong(b.addr + 8 * i)
    def update(i: Long, v: Long): Unit = U.putLong(b.addr + 8 * i, v)
    def addr: Long = b.addr
    def free(): Unit = b.free()
  }
  final class Doubles(n: Long = 0L) {
    val b = new Buf(8, math.max(n, 1L)); b.length = n
    def apply(i: Long): Double = U.getDouble(b.addr + 8 * i)
    def update(i: Long, v: Double): Unit = U.putDouble(b.addr + 8 * i, v)
    def +=(v: Double): Unit = { b.reserve(b.length + 1); U.putDouble(b.addr + 8 * b.length, v); b.length += 1 }
    def addr: Long = b.addr
    def length: Long = b.length
    def free(): Unit = b.free()
  }
}

object TsneHipOperators {
  import OffHeap._

  /** GPUs driven by one call (tsne_ctx_create_multi); one entry = one GPU. */
  @volatile var devices: Array[Int] = Array(0)

  private def withCtx[T](f: Long => T): T = {
    val ctx = if (devices.length == 1) TsneHip.ctxCreate(devices(0)) else TsneHip.ctxCreateMulti(devices)
    try f(ctx) finally TsneHip.ctxDestroy(ctx)
  }

  // ------------------------------------------------------------- metric
  // Tsne.getMetric (Tsne.scala:161-168) hands out breeze's squaredDistance /
  // euclideanDistance / cosineDistance as fresh function values, so they are
  // recognised by what they compute: the function is evaluated on fixed probe
  // pairs and compared with the three breeze functions themselves (exact
  // equality: the same JVM code).  Anything else is not a metric the GPU
  // path implements: IllegalArgumentException, as Tsne.scala:166.
  private val probes: Seq[(Vector[Double], Vector[Double])] = Seq(
    (DenseVector(1.0, 2.0, 0.0), DenseVector(0.0, 2.0, 3.0)),
    (DenseVector(0.5, -1.25, 2.0, 7.0), DenseVector(3.0, 1.0, -1.5, 0.25)))
  private lazy val known: Seq[(String, Seq[Double])] = Seq(
    "sqeuclidean" -> probes.map { case (a, b) => squaredDistance(a, b) },
    "euclidean" -> probes.map { case (a, b) => euclideanDistance(a, b) },
    "cosine" -> probes.map { case (a, b) => cosineDistance(a, b) })

  /** The name (Tsne.getMetric's) of a metric function, by probe evaluation. */
  def metricName(metric: (Vector[Double], Vector[Double]) => Double): String = {
    val got = probes.map { case (a, b) => metric(a, b) }
    known.find(_._2 == got).map(_._1).getOrElse(throw new IllegalArgumentException(
      "metric is not one of Tsne.getMetric's breeze functions (sqeuclidean, euclidean, cosine)"))
  }

  // ---------------------------------------------------------------- kNN
  /** The rows of `input` sorted by id into an off-heap n x d matrix (ids ascending). */
  private def rowsByIdOffHeap(it: Iterator[(Int, Vector[Double])]): (Array[Int], Doubles, Int) = {
    val ids = new Ints()
    val x = new Doubles()
    var d = -1
    it.foreach { case (id, v) =>
      if (d < 0) d = v.length
      require(v.length == d, "rows of different dimension")
      ids += id
      var k = 0
      while (k < d) { x += v(k); k += 1 }
    }
    val n = ids.length.toInt   // rows (points) are < 2^31; entries are Long throughout
    val order = (0 until n).sortBy(i => ids(i)).toArray
    val X = new Doubles(n.toLong * math.max(d, 0))
    for (r <- 0 until n; k <- 0 until d) X(r.toLong * d + k) = x(order(r).toLong * d + k)
    val sortedIds = order.map(i => ids(i))
    ids.free(); x.free()
    (sortedIds, X, math.max(d, 0))
  }

  /** kNearestNeighbors (TsneHelpers.scala:41-59): the k smallest metric values per
   *  point over all others, ascending by (distance, id). */
  def kNearestNeighbors(input: DataSet[(Int, Vector[Double])], k: Int,
                        metric: (Vector[Double], Vector[Double]) => Double): DataSet[(Int, Int, Double)] = {
    val m = metricName(metric)
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val (ids, X, d) = rowsByIdOffHeap(it)
      val n = ids.length
      if (n >= 2) {
        val kk = math.min(k, n - 1)
        val idx = new Ints(n.toLong * kk); val dist = new Doubles(n.toLong * kk)
        withCtx(ctx => TsneHip.knn(ctx, X.addr, n, d, TsneHip.metricFromName(m), k, 0, n, idx.addr, dist.addr))
        for (i <- 0 until n; t <- 0 until kk) {
          val o = i.toLong * kk + t
          out.collect((ids(i), ids(idx(o)), dist(o)))
        }
        idx.free(); dist.free()
      }
      X.free()
    }.setParallelism(1)
  }

  /** partitionKnn (TsneHelpers.scala:61-91): the same exact kNN; `blocks` is a CPU tiling detail. */
  def partitionKnn(input: DataSet[(Int, Vector[Double])], k: Int,
                   metric: (Vector[Double], Vector[Double]) => Double, blocks: Int): DataSet[(Int, Int, Double)] =
    kNearestNeighbors(input, k, metric)

  /** projectKnn (TsneHelpers.scala:93-160): Z-order neighbours of the input and of
   *  iterations - 1 shifted copies (uniform [0,1)^d shifts, unseeded as the reference). */
  def projectKnn(input: DataSet[(Int, Vector[Double])], k: Int,
                 metric: (Vector[Double], Vector[Double]) => Double, dimension: Int,
                 iterations: Int): DataSet[(Int, Int, Double)] = {
    val m = metricName(metric)
    val shifts: Seq[DenseVector[Double]] = for (_ <- 1 until iterations) yield DenseVector.rand[Double](dimension)
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val (ids, X, d) = rowsByIdOffHeap(it)
      val n = ids.length
      if (n >= 2) {
        require(d == dimension, "rows must have --dimension entries")
        val sh = new Doubles(math.max(1L, (iterations - 1).toLong * d))
        for ((v, s) <- shifts.zipWithIndex; c <- 0 until d) sh(s.toLong * d + c) = v(c)
        val kk = math.min(k, n - 1)
        val idx = new Ints(n.toLong * kk); val dist = new Doubles(n.toLong * kk)
        withCtx(ctx => TsneHip.projectKnn(ctx, X.addr, n, d, TsneHip.metricFromName(m), k, iterations,
          if (iterations > 1) sh.addr else 0L, idx.addr, dist.addr))
        for (i <- 0 until n; t <- 0 until kk) {
          val o = i.toLong * kk + t
          out.collect((ids(i), ids(idx(o)), dist(o)))
        }
        idx.free(); dist.free(); sh.free()
      }
      X.free()
    }.setParallelism(1)
  }

  // --------------------------------------------------------- affinities
  /** Triples streamed into off-heap COO, grouped by row (tsne_coo_to_csr: row index
   *  = the triple's id, rows in id order, each row's triples in input order). */
  private final class Csr(val n: Long, val rp: Longs, val col: Ints, val value: Doubles, val nnz: Long) {
    def free(): Unit = { rp.free(); col.free(); value.free() }
  }
  private def csrOf(it: Iterator[(Int, Int, Double)], colsAreRows: Boolean): Csr = {
    val ri = new Ints(); val ci = new Ints(); val v = new Doubles()
    var maxId = -1
    it.foreach { case (i, j, x) =>
      require(i >= 0 && j >= 0, "point ids must be non-negative")
      ri += i; ci += j; v += x
      maxId = math.max(maxId, if (colsAreRows) math.max(i, j) else i)
    }
    val n = maxId + 1L
    val nnz = ri.length
    val rp = new Longs(n + 1); val col = new Ints(nnz); val value = new Doubles(nnz)
    TsneHip.cooToCsr(ri.addr, ci.addr, v.addr, nnz, n, rp.addr, col.addr, value.addr)
    ri.free(); ci.free(); v.free()
    new Csr(n, rp, col, value, nnz)
  }

  /** pairwiseAffinities (TsneHelpers.scala:162-180): the beta search per row i; the
   *  distance-matrix mode (Tsne.scala:69-70) feeds N-1- or N-long rows through here. */
  def pairwiseAffinities(input: DataSet[(Int, Int, Double)], perplexity: Double): DataSet[(Int, Int, Double)] =
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val c = csrOf(it, colsAreRows = false)
      val p = new Doubles(c.nnz)
      withCtx(ctx => TsneHip.pairwiseAffinities(ctx, c.rp.addr, c.value.addr, c.n, perplexity, p.addr))
      var r = 0L
      while (r < c.n) {
        var e = c.rp(r)
        while (e < c.rp(r + 1)) { out.collect((r.toInt, c.col(e), p(e))); e += 1 }
        r += 1
      }
      p.free(); c.free()
    }.setParallelism(1)

  /** jointDistribution (TsneHelpers.scala:182-196): P = (C + C^T) / sum over the union pattern. */
  def jointDistribution(input: DataSet[(Int, Int, Double)]): DataSet[(Int, Int, Double)] =
    input.reduceGroup { (it, out: Collector[(Int, Int, Double)]) =>
      val c = csrOf(it, colsAreRows = true)
      val cap = 2 * c.nnz
      val orp = new Longs(c.n + 1); val oc = new Ints(cap); val ov = new Doubles(cap)
      val nnz = withCtx(ctx => TsneHip.jointDistribution(ctx, c.rp.addr, c.col.addr, c.value.addr, c.n, cap,
        orp.addr, oc.addr, ov.addr))
      require(nnz <= cap)
      var r = 0L
      while (r < c.n) {
        var e = orp(r)
        while (e < orp(r + 1)) { out.collect((r.toInt, oc(e), ov(e))); e += 1 }
        r += 1
      }
      orp.free(); oc.free(); ov.free(); c.free()
    }.setParallelism(1)

  // ---------------------------------------------------------- optimizer
  /** optimize (TsneHelpers.scala:396-430): the three phases and every iteration of
   *  iterationComputation (:371-394) in one call; the embedding never leaves the GPU. */
  def optimize(highDimAffinities: DataSet[(Int, SparseVector[Double])],
               initialWorkingSet: DataSet[(Int, Vector[Double], Vector[Double], Vector[Double])],
               learningRate: Double, iterations: Int, metric: (Vector[Double], Vector[Double]) => Double,
               earlyExaggeration: Double, initialMomentum: Double, finalMomentum: Double, theta: Double,
               dimension: Int): DataSet[(Int, Vector[Double])] = {
    val m = metricName(metric)
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
          val ws = workingSet.sortBy(_._1).toArray
          val ids = ws.map(_._1)
          val n = ids.length
          val c = dimension
          // point id -> row of the working set: identity for the usual dense ids,
          // else a table (ids < 4n) or a hash map
          val maxId = if (n == 0) -1 else ids(n - 1)
          val dense = ids.zipWithIndex.forall { case (id, r) => id == r }
          val table: Array[Int] = if (!dense && maxId >= 0 && maxId < 4L * n) {
            val a = Array.fill(maxId + 1)(-1); for (r <- 0 until n) a(ids(r)) = r; a
          } else null
          val hash = if (!dense && table == null) ids.zipWithIndex.toMap else null
          def index(id: Int): Int = {
            val r = if (dense) id else if (table != null) (if (id >= 0 && id < table.length) table(id) else -1)
                    else hash.getOrElse(id, -1)
            require(r >= 0 && r < n, s"point $id of P is not in the working set")
            r
          }
          // P streamed into off-heap COO (row = the row's point, col = its entries' points)
          val ri = new Ints(); val ci = new Ints(); val pv = new Doubles()
          it.asScala.foreach { case (_, (id, sv)) =>
            val r = index(id)
            // a row is indexed by point ids: Tsne.scala:121 sizes it inputDimension^2,
            // which is shorter than the ids whenever N > D^2 (INTEGRATION.md section 1)
            if (sv.length <= maxId)
              throw new IllegalArgumentException(
                s"row $id of P is a SparseVector of length ${sv.length}, but the point ids reach $maxId: " +
                "build the rows with VectorBuilder(number of points), not inputDimension * inputDimension " +
                "(Tsne.scala:121; INTEGRATION.md section 1)")
            var o = 0
            while (o < sv.activeSize) { ri += r; ci += index(sv.indexAt(o)); pv += sv.valueAt(o); o += 1 }
          }
          val nnz = ri.length
          val rp = new Longs(n + 1L); val col = new Ints(nnz); val P = new Doubles(nnz)
          TsneHip.cooToCsr(ri.addr, ci.addr, pv.addr, nnz, n, rp.addr, col.addr, P.addr)
          ri.free(); ci.free(); pv.free()
          val Y = new Doubles(n.toLong * c); val upd = new Doubles(n.toLong * c); val gains = new Doubles(n.toLong * c)
          for (r <- 0 until n; k <- 0 until c) {
            val o = r.toLong * c + k
            Y(o) = ws(r)._2(k); upd(o) = ws(r)._3(k); gains(o) = ws(r)._4(k)
          }
          val slots = iterations / 10 + 1
          val lk = new Ints(slots); val lv = new Doubles(slots)
          val nl = withCtx { ctx =>
            TsneHip.optimize(ctx, c, learningRate, iterations, TsneHip.metricFromName(m), earlyExaggeration,
              initialMomentum, finalMomentum, theta, rp.addr, col.addr, P.addr, n, Y.addr, upd.addr, gains.addr,
              lk.addr, lv.addr)
          }
          for (s <- 0 until math.min(nl, slots))                        // the "loss" channel
            lossAccumulator.add((lk(s), lv(s)))
          for (r <- 0 until n)
            out.collect((ids(r), DenseVector.tabulate(c)(k => Y(r.toLong * c + k))))
          rp.free(); col.free(); P.free(); Y.free(); upd.free(); gains.free(); lk.free(); lv.free()
        }
      }).withBroadcastSet(initialWorkingSet, "workingSet").setParallelism(1)
  }
}
