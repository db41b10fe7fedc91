// comm.cpp -- the collectives of the row-sharded multi-GPU path, behind one
// interface with three backends:
//   * RCCL over xGMI: one rank per GPU (one process per GPU, the unique id
//     shipped out of band by the caller, or one thread per GPU of a
//     tsne_ctx_create_multi group, communicators from ncclCommInitAll);
//   * loopback: several ranks on ONE device, one host thread each, inside one
//     process (tsne_ctx_create_multi with a repeated device id).  Collectives
//     meet at a host barrier and copy through the shared device memory in a
//     fixed rank order.  It executes the library's own world > 1 code path
//     on a single GPU, which is how the multi-GPU optimizer is tested;
//   * callbacks: collectives on host buffers supplied by the caller
//     (tsne_ctx_init_comm_callbacks): the host dataflow's own exchange.
// Per optimizer iteration the traffic is the all-gather of the owned slices
// of the updated embedding (16 B per point, ragged slices) and an all-reduce
// of the Z normaliser (one double); every 10th iteration one more double (the
// loss); every relabel (25 iterations) an all-reduce of the 256-query bucket
// costs and an all-gather of the momentum / gains slices.
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <functional>
#include <map>
#include <mutex>
#include <thread>

#include "comm_guard.hpp"
#include "common.hpp"

namespace tsne {

struct Comm {
    virtual ~Comm() = default;
    // in place: every rank's buf becomes the element-wise sum over ranks
    virtual void allreduce_f64(tsne_ctx *ctx, double *buf, size_t count) = 0;
    virtual void allreduce_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count) = 0;
    // in place: rank r's bytes [off[r], off[r+1]) of buf are copied to every rank
    virtual void allgatherv(tsne_ctx *ctx, void *buf, const int64_t *off) = 0;
    // in place: on rank r, elements [off[r], off[r+1]) of buf become their sum
    // over the ranks (the rest of buf is unspecified afterwards).  Default: an
    // all-reduce of the whole buffer (the caller-callback transport).
    virtual void reduce_scatterv_f64(tsne_ctx *ctx, double *buf, const int64_t *off) {
        allreduce_f64(ctx, buf, (size_t)off[ctx->world]);
    }
    // a rank failed: make every pending and later collective of this rank
    // fail (TSNE_ERR_COMM) instead of waiting for it; callable from another thread
    virtual void abort() {}
    // the calling rank's work in a group call has ended (loopback serial mode:
    // hand the device turn on); called on the rank's own thread
    virtual void release(tsne_ctx *) {}
    // a phase boundary inside a rank's work (loopback serial mode: timed)
    virtual void mark(tsne_ctx *, const char *) {}
    virtual int kind() const = 0;   // 1 RCCL, 2 loopback, 3 caller callbacks
    virtual std::string loop_profile() { return std::string(); }   // loopback serial-mode summary
    int64_t calls = 0;              // collectives this rank has issued
};

namespace {

void nccl_check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) fail(TSNE_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

// RCCL under the CommGuard protocol (comm_guard.hpp): communicators are
// created non-blocking, so no RCCL call holds the rank's thread while a peer
// is missing, and abort() from a failing peer's thread never waits for one.
struct RcclBackend {
    using Handle = ncclComm_t;
    static int code(ncclResult_t r) { return r == ncclSuccess ? 0 : r == ncclInProgress ? 1 : -(int)r; }
    template <class F> static int call(Handle h, F &&f) { return code(f(h)); }
    static int poll(Handle h) {
        ncclResult_t a = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(h, &a);
        return r != ncclSuccess ? -(int)r : code(a);
    }
    static void abort(Handle h) {
        if (h) (void)ncclCommAbort(h);
    }
    static void destroy(Handle h) {
        if (!h) return;
        if (ncclCommFinalize(h) == ncclInProgress || poll(h) == 1)
            while (poll(h) == 1) std::this_thread::yield();
        (void)ncclCommDestroy(h);
    }
};

// wait for a non-blocking communicator's initialisation
void nccl_wait_init(ncclComm_t c, const char *what) {
    for (;;) {
        const int p = RcclBackend::poll(c);
        if (p == 0) return;
        if (p < 0) fail(TSNE_ERR_COMM, std::string(what) + ": " + ncclGetErrorString((ncclResult_t)-p));
        std::this_thread::yield();
    }
}

ncclConfig_t nonblocking_config() {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    return cfg;
}

struct RcclComm : Comm {
    CommGuard<RcclBackend> g;
    int kind() const override { return 1; }
    ~RcclComm() override { g.destroy(); }
    // ncclCommAbort stops this rank's in-flight collective kernels and frees
    // the communicator: a peer blocked in a collective with it then fails
    // instead of hanging (run_group aborts every rank of a group once one
    // rank has thrown).  Later calls report TSNE_ERR_COMM.
    void abort() override { g.abort(); }
    void run(const char *what, const std::function<ncclResult_t(ncclComm_t)> &op) {
        const int rc = g.run([&](ncclComm_t c) { return op(c); });
        if (rc == -1) fail(TSNE_ERR_COMM, "RCCL communicator aborted (another rank failed)");
        if (rc == -2) {   // the failing call's or the async poll's own code
            const int e = g.error();
            fail(TSNE_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(e > 0 ? (ncclResult_t)e : ncclInternalError));
        }
    }
    void allreduce_f64(tsne_ctx *ctx, double *buf, size_t count) override {
        run("ncclAllReduce", [&](ncclComm_t c) { return ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, c, ctx->stream); });
    }
    void allreduce_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count) override {
        run("ncclAllReduce", [&](ncclComm_t c) { return ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, c, ctx->stream); });
    }
    // ragged reduce-scatter: one in-place reduce per root, fused into one group
    void reduce_scatterv_f64(tsne_ctx *ctx, double *buf, const int64_t *off) override {
        run("ncclReduce group", [&](ncclComm_t c) {
            ncclResult_t r = ncclGroupStart();
            for (int q = 0; q < ctx->world && r == ncclSuccess; ++q) {
                const size_t cnt = (size_t)(off[q + 1] - off[q]);
                if (cnt == 0) continue;
                r = ncclReduce(buf + off[q], buf + off[q], cnt, ncclFloat64, ncclSum, q, c, ctx->stream);
            }
            const ncclResult_t e = ncclGroupEnd();
            return r != ncclSuccess ? r : e;
        });
    }
    // ragged all-gather: one in-place broadcast per root, fused into one group
    void allgatherv(tsne_ctx *ctx, void *buf, const int64_t *off) override {
        uint8_t *b = static_cast<uint8_t *>(buf);
        run("ncclBroadcast group", [&](ncclComm_t c) {
            ncclResult_t r = ncclGroupStart();
            for (int q = 0; q < ctx->world && r == ncclSuccess; ++q) {
                const size_t bytes = (size_t)(off[q + 1] - off[q]);
                if (bytes == 0) continue;
                r = ncclBroadcast(b + off[q], b + off[q], bytes, ncclUint8, q, c, ctx->stream);
            }
            const ncclResult_t e = ncclGroupEnd();
            return r != ncclSuccess ? r : e;
        });
    }
};

// Shared state of the ranks of one loopback group (one device).
//
// Options::loop_serial (set on the group handle before tsne_optimize): the
// ranks take turns on the device.  A rank holds the turn from the end of one
// collective to the start of the next, drains the device before it lets go,
// and logs the wall time of that segment of its own work.  With the segments
// of one collective aligned across ranks, the sum over collectives of the
// slowest rank's segment is the compute span a world-size group of devices
// would take (collectives excluded: they are the loopback's host copies
// here).  tsne_ctx_loop_profile returns the summary (JSON): a projection tool
// for N GPUs measured on one (scripts/loop_projection.py).
struct LoopGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    bool aborted = false;
    std::vector<void *> ptr;
    // serial timing mode
    std::mutex turn;
    std::vector<char> holding;
    std::vector<std::chrono::steady_clock::time_point> t_acq;
    std::vector<std::vector<std::pair<std::string, double>>> segs;   // per rank: (collective, ms)
    explicit LoopGroup(int w) : world(w), ptr(w, nullptr), holding(w, 0), t_acq(w), segs(w) {}
    static bool serial(const tsne_ctx *ctx) { return ctx->opts.loop_serial != 0; }
    // the summary of the segments logged so far (then cleared)
    std::string summary() {
        std::string out;
        char b[256];
        // collectives are issued in the same sequence on every rank
        size_t m = segs[0].size();
        for (int r = 1; r < world; ++r) m = std::min(m, segs[r].size());
        std::map<std::string, std::vector<double>> lab;   // [sum of max, sum of mean, count]
        std::map<std::string, std::vector<double>> ser;   // per 100 occurrences of a label: sum of max
        double span = 0.0;
        std::vector<double> tot(world, 0.0);
        for (size_t i = 0; i < m; ++i) {
            double mx = 0.0, sm = 0.0;
            for (int r = 0; r < world; ++r) {
                mx = std::max(mx, segs[r][i].second);
                sm += segs[r][i].second;
                tot[r] += segs[r][i].second;
            }
            auto &v = lab[segs[0][i].first];
            if (v.empty()) v.assign(3, 0.0);
            const size_t occ = (size_t)v[2];
            v[0] += mx; v[1] += sm / world; v[2] += 1.0;
            auto &sv = ser[segs[0][i].first];
            if (sv.size() <= occ / 100) sv.resize(occ / 100 + 1, 0.0);
            sv[occ / 100] += mx;
            span += mx;
        }
        snprintf(b, sizeof(b), "{\"world\": %d, \"segments\": %zu, \"span_ms\": %.6f, \"rank_total_ms\": [", world, m, span);
        out += b;
        for (int r = 0; r < world; ++r) { snprintf(b, sizeof(b), "%s%.6f", r ? ", " : "", tot[r]); out += b; }
        out += "], \"by_collective\": {";
        bool first = true;
        for (auto &kv : lab) {
            snprintf(b, sizeof(b), "%s\"%s\": {\"max_ms\": %.6f, \"mean_ms\": %.6f, \"count\": %.0f}", first ? "" : ", ",
                     kv.first.c_str(), kv.second[0], kv.second[1], kv.second[2]);
            out += b;
            first = false;
        }
        out += "}, \"max_ms_per_100\": {";
        first = true;
        for (auto &kv : ser) {
            snprintf(b, sizeof(b), "%s\"%s\": [", first ? "" : ", ", kv.first.c_str());
            out += b;
            for (size_t k = 0; k < kv.second.size(); ++k) { snprintf(b, sizeof(b), "%s%.3f", k ? ", " : "", kv.second[k]); out += b; }
            out += "]";
            first = false;
        }
        out += "}}";
        for (auto &sg : segs) sg.clear();
        return out;
    }
    // serial mode: the end of a segment of this rank's work (before a collective)
    void seg_end(tsne_ctx *ctx, const char *what) {
        if (!serial(ctx)) return;
        TSNE_HIP(hipDeviceSynchronize());   // the side stream too
        const int r = ctx->rank;
        if (holding[r]) {
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_acq[r]).count();
            segs[r].emplace_back(what, ms);
            holding[r] = 0;
            turn.unlock();
        }
    }
    // serial mode: a phase boundary -- the stretch so far is logged as `what`
    // and the next one starts (the turn is kept)
    void seg_mark(tsne_ctx *ctx, const char *what) {
        if (!serial(ctx) || !holding[ctx->rank]) return;
        TSNE_HIP(hipDeviceSynchronize());
        const int r = ctx->rank;
        const auto now = std::chrono::steady_clock::now();
        segs[r].emplace_back(what, std::chrono::duration<double, std::milli>(now - t_acq[r]).count());
        t_acq[r] = now;
    }
    void seg_release(tsne_ctx *ctx) {
        if (!holding[ctx->rank]) return;
        holding[ctx->rank] = 0;
        turn.unlock();
    }
    // serial mode: the start of the next segment (after a collective)
    void seg_begin(tsne_ctx *ctx) {
        if (!serial(ctx)) return;
        const int r = ctx->rank;
        turn.lock();
        holding[r] = 1;
        t_acq[r] = std::chrono::steady_clock::now();
    }
    // all ranks meet; throws on every rank once one rank has aborted
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) fail(TSNE_ERR_COMM, "loopback group aborted by another rank");
        const uint64_t gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen || aborted; });
            if (generation == gen) fail(TSNE_ERR_COMM, "loopback group aborted by another rank");
        }
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

struct LoopComm : Comm {
    std::shared_ptr<LoopGroup> g;
    int kind() const override { return 2; }
    explicit LoopComm(std::shared_ptr<LoopGroup> grp) : g(std::move(grp)) {}

    // publish this rank's pointer once its stream has produced the data
    void publish(tsne_ctx *ctx, void *p, const char *what) {
        TSNE_HIP(hipStreamSynchronize(ctx->stream));
        g->seg_end(ctx, what);
        g->ptr[ctx->rank] = p;
        g->barrier();
    }
    template <class T> void allreduce(tsne_ctx *ctx, T *buf, size_t count) {
        if (count == 0) return;
        const std::string what = std::string(sizeof(T) == 8 && T(0.5) != T(0) ? "allreduce_f64[" : "allreduce_u64[") +
                                 std::to_string(count) + "]";
        publish(ctx, buf, what.c_str());
        std::vector<T> acc(count, T(0)), tmp(count);
        for (int r = 0; r < g->world; ++r) {   // fixed rank order: identical sums on every rank
            TSNE_HIP(hipMemcpy(tmp.data(), g->ptr[r], sizeof(T) * count, hipMemcpyDeviceToHost));
            for (size_t e = 0; e < count; ++e) acc[e] += tmp[e];
        }
        g->barrier();   // every rank has read every buffer before any is overwritten
        TSNE_HIP(hipMemcpy(buf, acc.data(), sizeof(T) * count, hipMemcpyHostToDevice));
        g->seg_begin(ctx);
    }
    void allreduce_f64(tsne_ctx *ctx, double *buf, size_t count) override { allreduce(ctx, buf, count); }
    void allreduce_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count) override { allreduce(ctx, buf, count); }
    // this rank's slice summed over the ranks in fixed rank order
    void reduce_scatterv_f64(tsne_ctx *ctx, double *buf, const int64_t *off) override {
        publish(ctx, buf, "reduce_scatterv");
        const int64_t a = off[ctx->rank], cnt = off[ctx->rank + 1] - a;
        std::vector<double> acc(cnt, 0.0), tmp(cnt);
        for (int r = 0; r < g->world && cnt > 0; ++r) {
            TSNE_HIP(hipMemcpy(tmp.data(), static_cast<const double *>(g->ptr[r]) + a, sizeof(double) * cnt,
                               hipMemcpyDeviceToHost));
            for (int64_t e = 0; e < cnt; ++e) acc[e] += tmp[e];
        }
        g->barrier();   // every rank has read its slice of every buffer before any is overwritten
        if (cnt > 0) TSNE_HIP(hipMemcpy(buf + a, acc.data(), sizeof(double) * cnt, hipMemcpyHostToDevice));
        g->seg_begin(ctx);
    }
    void abort() override { g->abort(); }
    std::string loop_profile() override { return g->summary(); }
    void release(tsne_ctx *ctx) override { g->seg_release(ctx); }
    void mark(tsne_ctx *ctx, const char *what) override { g->seg_mark(ctx, what); }
    void allgatherv(tsne_ctx *ctx, void *buf, const int64_t *off) override {
        publish(ctx, buf, "allgatherv");
        uint8_t *b = static_cast<uint8_t *>(buf);
        for (int r = 0; r < g->world; ++r) {
            if (r == ctx->rank || off[r + 1] == off[r]) continue;
            const uint8_t *src = static_cast<const uint8_t *>(g->ptr[r]);
            TSNE_HIP(hipMemcpy(b + off[r], src + off[r], (size_t)(off[r + 1] - off[r]), hipMemcpyDeviceToDevice));
        }
        g->barrier();
        g->seg_begin(ctx);
    }
};

// Caller-supplied collectives on host buffers (tsne_ctx_init_comm_callbacks):
// the host dataflow's own exchange (e.g. Flink's network stack, MPI, or
// torch.distributed/gloo in the tests) carries the library's messages.  The
// library stages each message through host memory.
struct CallbackComm : Comm {
    int kind() const override { return 3; }
    tsne_comm_ops ops{};
    void *user = nullptr;
    std::vector<uint8_t> host;
    void check(int rc, const char *what) {
        if (rc != 0) fail(TSNE_ERR_COMM, std::string(what) + " callback returned " + std::to_string(rc));
    }
    template <class T> T *stage_in(tsne_ctx *ctx, const T *dev, size_t bytes) {
        if (host.size() < bytes) host.resize(bytes);
        if (bytes) TSNE_HIP(hipMemcpyAsync(host.data(), dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
        TSNE_HIP(hipStreamSynchronize(ctx->stream));
        return reinterpret_cast<T *>(host.data());
    }
    void stage_out(tsne_ctx *ctx, void *dev, size_t bytes) {
        if (bytes) TSNE_HIP(hipMemcpyAsync(dev, host.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
        TSNE_HIP(hipStreamSynchronize(ctx->stream));
    }
    void allreduce_f64(tsne_ctx *ctx, double *buf, size_t count) override {
        double *h = stage_in(ctx, buf, count * sizeof(double));
        check(ops.allreduce_sum_f64(user, h, (int64_t)count), "allreduce_sum_f64");
        stage_out(ctx, buf, count * sizeof(double));
    }
    void allreduce_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count) override {
        uint64_t *h = reinterpret_cast<uint64_t *>(stage_in(ctx, buf, count * sizeof(uint64_t)));
        check(ops.allreduce_sum_u64(user, h, (int64_t)count), "allreduce_sum_u64");
        stage_out(ctx, buf, count * sizeof(uint64_t));
    }
    void allgatherv(tsne_ctx *ctx, void *buf, const int64_t *off) override {
        const size_t bytes = (size_t)off[ctx->world];
        uint8_t *h = stage_in(ctx, static_cast<uint8_t *>(buf), bytes);
        check(ops.allgatherv(user, h, off), "allgatherv");
        stage_out(ctx, buf, bytes);
    }
};

}  // namespace

void comm_init_callbacks(tsne_ctx *ctx, int rank, int world, const tsne_comm_ops *ops, void *user) {
    TSNE_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    TSNE_REQUIRE(ops && ops->allreduce_sum_f64 && ops->allreduce_sum_u64 && ops->allgatherv, "incomplete comm ops");
    comm_destroy(ctx);
    if (world == 1 && !ctx->opts.comm_world1) return;
    CallbackComm *c = new CallbackComm();
    c->ops = *ops;
    c->user = user;
    ctx->comm = c;
    ctx->rank = rank;
    ctx->world = world;
}

void comm_unique_id(uint8_t *out) {
    static_assert(sizeof(ncclUniqueId) == TSNE_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::memcpy(out, &id, sizeof(id));
}

void comm_init(tsne_ctx *ctx, int rank, int world, const uint8_t *id) {
    TSNE_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    comm_destroy(ctx);
    if (world == 1 && !ctx->opts.comm_world1) { ctx->rank = 0; ctx->world = 1; return; }
    ncclUniqueId uid;
    if (id) std::memcpy(&uid, id, sizeof(uid));
    else nccl_check(ncclGetUniqueId(&uid), "ncclGetUniqueId");   // world 1: our own id
    std::unique_ptr<RcclComm> c(new RcclComm());
    ncclConfig_t cfg = nonblocking_config();
    const ncclResult_t r = ncclCommInitRankConfig(&c->g.h, world, uid, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) nccl_check(r, "ncclCommInitRankConfig");
    nccl_wait_init(c->g.h, "ncclCommInitRankConfig");
    ctx->comm = c.release();
    ctx->rank = rank;
    ctx->world = world;
}

// Communicators for the contexts of one tsne_ctx_create_multi group: RCCL
// (ncclCommInitAll) when every device is distinct, loopback when all are the
// same device.
void comm_init_group(const std::vector<tsne_ctx *> &subs, bool loopback) {
    const int world = (int)subs.size();
    if (world == 1) return;
    if (loopback) {
        auto g = std::make_shared<LoopGroup>(world);
        for (int r = 0; r < world; ++r) {
            comm_destroy(subs[r]);
            subs[r]->comm = new LoopComm(g);
            subs[r]->rank = r;
            subs[r]->world = world;
        }
        return;
    }
    // one thread initialises every device's rank: a group of non-blocking
    // ncclCommInitRankConfig calls (ncclCommInitAll has no config)
    std::vector<ncclComm_t> comms(world, nullptr);
    ncclUniqueId uid;
    nccl_check(ncclGetUniqueId(&uid), "ncclGetUniqueId");
    ncclConfig_t cfg = nonblocking_config();
    int dev0 = 0;
    TSNE_HIP(hipGetDevice(&dev0));
    // on any failure below: the caller's device back (the guard) and the
    // communicators created so far aborted, not leaked
    struct InitCleanup {
        std::vector<ncclComm_t> &c;
        bool done = false;
        ~InitCleanup() {
            if (done) return;
            for (ncclComm_t x : c)
                if (x) (void)ncclCommAbort(x);
        }
    } cleanup{comms};
    {
        DeviceGuard dg(dev0);
        bool in_group = false;
        try {
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            in_group = true;
            for (int r = 0; r < world; ++r) {
                TSNE_HIP(hipSetDevice(subs[r]->device));
                const ncclResult_t e = ncclCommInitRankConfig(&comms[r], world, uid, r, &cfg);
                if (e != ncclSuccess && e != ncclInProgress) nccl_check(e, "ncclCommInitRankConfig");
            }
            in_group = false;
            const ncclResult_t ge = ncclGroupEnd();
            if (ge != ncclSuccess && ge != ncclInProgress) nccl_check(ge, "ncclGroupEnd");
        } catch (...) {
            if (in_group) (void)ncclGroupEnd();   // close the group before the aborts
            throw;
        }
    }
    for (int r = 0; r < world; ++r) nccl_wait_init(comms[r], "ncclCommInitRankConfig");
    cleanup.done = true;
    for (int r = 0; r < world; ++r) {
        comm_destroy(subs[r]);
        RcclComm *c = new RcclComm();
        c->g.h = comms[r];
        subs[r]->comm = c;
        subs[r]->rank = r;
        subs[r]->world = world;
    }
}

// A rank failed: its collectives (and, for a loopback group, every rank's
// barrier) fail from now on instead of waiting.
void comm_abort(tsne_ctx *ctx) {
    if (ctx->comm) ctx->comm->abort();
}

void comm_mark(tsne_ctx *ctx, const char *what) {
    if (ctx->comm) ctx->comm->mark(ctx, what);
}

void comm_release(tsne_ctx *ctx) {
    if (ctx->comm) ctx->comm->release(ctx);
}

std::string comm_loop_profile(tsne_ctx *ctx) { return ctx->comm ? ctx->comm->loop_profile() : std::string(); }

int64_t comm_counter(const tsne_ctx *ctx, bool calls) {
    if (!ctx->comm) return 0;
    return calls ? ctx->comm->calls : ctx->comm->kind();
}

void comm_destroy(tsne_ctx *ctx) {
    delete ctx->comm;
    ctx->comm = nullptr;
    ctx->rank = 0;
    ctx->world = 1;
}

void comm_allgatherv(tsne_ctx *ctx, void *buf, const int64_t *off_bytes) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    ++ctx->comm->calls;
    ctx->comm->allgatherv(ctx, buf, off_bytes);
}

void comm_allreduce_sum_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    ++ctx->comm->calls;
    ctx->comm->allreduce_u64(ctx, buf, count);
}

void comm_reduce_scatterv_f64(tsne_ctx *ctx, double *buf, const int64_t *off_elems) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    ++ctx->comm->calls;
    ctx->comm->reduce_scatterv_f64(ctx, buf, off_elems);
}

void comm_allreduce_sum_f64(tsne_ctx *ctx, double *buf, size_t count) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    ++ctx->comm->calls;
    ctx->comm->allreduce_f64(ctx, buf, count);
}

}  // namespace tsne
