// capi.cpp -- the extern "C" boundary of libtsne_hip (include/tsne_hip.h).
// Every entry point converts internal tsne::Error exceptions into a status
// code plus a thread-local message; nothing throws across the ABI.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <new>
#include <algorithm>
#include <thread>

#include "bhtree.hpp"
#include "common.hpp"

namespace tsne {

static thread_local std::string g_last_error;

[[noreturn]] void fail(int status, const std::string &msg) { throw Error(status, msg); }

template <class Fn> static int guard(Fn &&fn) {
    try {
        fn();
        return TSNE_OK;
    } catch (const Error &e) {
        g_last_error = e.what();
        return e.status;
    } catch (const std::bad_alloc &) {
        g_last_error = "host allocation failed";
        return TSNE_ERR_NOMEM;
    } catch (const std::exception &e) {
        g_last_error = e.what();
        return TSNE_ERR_HIP;
    } catch (...) {
        g_last_error = "unknown error";
        return TSNE_ERR_HIP;
    }
}

static void check_ctx(tsne_ctx *ctx) {
    if (!ctx) fail(TSNE_ERR_ARG, "context is NULL");
}

// Single-device operators on a group handle run on its first rank.
static tsne_ctx *primary(tsne_ctx *ctx) { return ctx->group.empty() ? ctx : ctx->group[0]; }

// The device-resident optimizer (tsne_dev_opt_*) is one rank's state: on a
// tsne_ctx_create_multi handle of several ranks its first context is rank 0 of
// a world > 1 communicator, whose collectives would wait for ranks that never
// call in.  Such handles run the optimizer through tsne_optimize (every rank
// on its own thread); the device form is refused.
static tsne_ctx *opt_ctx(tsne_ctx *ctx) {
    if (ctx->group.size() > 1)
        fail(TSNE_ERR_UNSUPPORTED, "tsne_dev_opt_* on a multi-rank handle: use tsne_optimize, or one context per rank");
    return primary(ctx);
}

// Run fn(rank context, rank) on every rank of a group, one host thread each
// (device made current per thread); the first failure is rethrown here after
// the other ranks were released (loopback barrier abort) and joined.
template <class Fn> static void run_group(tsne_ctx *g, Fn &&fn) {
    const int world = (int)g->group.size();
    std::vector<std::exception_ptr> err(world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            try {
                DeviceGuard dg(g->group[r]->device);
                fn(g->group[r], r);
                comm_release(g->group[r]);
            } catch (...) {
                err[r] = std::current_exception();
                comm_release(g->group[r]);
                // release every rank: a loopback barrier, or the peers' RCCL
                // collectives still waiting for this rank (ncclCommAbort)
                for (tsne_ctx *c : g->group) comm_abort(c);
            }
        });
    for (auto &t : th) t.join();
    // report the root cause: a rank's own failure before the others' "aborted"
    for (int pass = 0; pass < 2; ++pass)
        for (int r = 0; r < world; ++r) {
            if (!err[r]) continue;
            try {
                std::rethrow_exception(err[r]);
            } catch (const Error &e) {
                if (pass == 0 && e.status == TSNE_ERR_COMM) continue;
                throw;
            }
        }
}

template <class T> static T *upload(tsne_ctx *ctx, const std::string &name, const T *h, size_t count) {
    T *d = ctx->ws.get<T>(name, count ? count : 1);
    if (count) TSNE_HIP(hipMemcpyAsync(d, h, sizeof(T) * count, hipMemcpyHostToDevice, ctx->stream));
    return d;
}

template <class T> static void download(tsne_ctx *ctx, T *h, const T *d, size_t count) {
    if (count) TSNE_HIP(hipMemcpyAsync(h, d, sizeof(T) * count, hipMemcpyDeviceToHost, ctx->stream));
}

static void sync(tsne_ctx *ctx) { TSNE_HIP(hipStreamSynchronize(ctx->stream)); }

// The Options fields by key (tsne_ctx_set_option); values range-checked.
struct OptionField {
    const char *key;
    double Options::*d;
    int Options::*i;
    double lo, hi;
};
static const OptionField k_options[] = {
    {"near_tol_early", &Options::near_tol_early, nullptr, 0.0, 1e-2},
    {"near_tol_late", &Options::near_tol_late, nullptr, 0.0, 1e-2},
    {"mom_tol", &Options::mom_tol, nullptr, 0.0, 1e-4},
    {"near_tol3_early", &Options::near_tol3_early, nullptr, 0.0, 1e-2},
    {"near_tol3_late", &Options::near_tol3_late, nullptr, 0.0, 1e-2},
    {"mom3_tol", &Options::mom3_tol, nullptr, 0.0, 1e-4},
    {"oct_moments", nullptr, &Options::oct_moments, 0, 1},
    {"oct_records", nullptr, &Options::oct_records, 0, 2},
    {"coherent_sort", nullptr, &Options::coherent_sort, 0, 1},
    {"oct_layout_switch", &Options::oct_layout_switch, nullptr, 0, 1e6},
    {"root_tile", nullptr, &Options::root_tile, 0, 1},
    {"attract_tiles", nullptr, &Options::attract_tiles, 0, 1},
    {"attract_tiles3", nullptr, &Options::attract_tiles3, 0, 1},
    {"attract_cfg", nullptr, &Options::attract_cfg, -1, 3},
    {"attract_pipe", nullptr, &Options::attract_pipe, 0, 5},
    {"attract_dyn", nullptr, &Options::attract_dyn, 0, 1},
    {"graph_order", nullptr, &Options::graph_order, 0, 1},
    {"relabel", nullptr, &Options::relabel, -1, 2},
    {"recut", nullptr, &Options::recut, 0, 1},
    {"knn_bf16", nullptr, &Options::knn_bf16, 0, 1},
    {"narrow", &Options::narrow, nullptr, 0.0, 1e6},
    {"reuse_costs", nullptr, &Options::reuse_costs, 0, 1},
    {"spill", &Options::spill, nullptr, 0.0, 1e6},
    {"spill_task", &Options::spill_task, nullptr, 0.0, 1e6},
    {"spill_min", nullptr, &Options::spill_min, 1, 1 << 30},
    {"spill_force", nullptr, &Options::spill_force, 0, 1 << 30},
    {"spill_drains", nullptr, &Options::spill_drains, 1, 8},
    {"tile_stream", nullptr, &Options::tile_stream, 0, 8},
    {"tile_stream_max", nullptr, &Options::tile_stream_max, -1, 1 << 30},
    {"tile_stream_frac", &Options::tile_stream_frac, nullptr, 0.0, 64.0},
    {"tile_stream_gate", nullptr, &Options::tile_stream_gate, 0, 1},
    {"trav_prio", nullptr, &Options::trav_prio, 0, 3},
    {"trav_front", &Options::trav_front, nullptr, 0.0, 1e6},
    {"trav_front_cur", &Options::trav_front_cur, nullptr, 0.0, 1e6},
    {"wave_log", nullptr, &Options::wave_log, 0, 1},
    {"attract_serial_t0", nullptr, &Options::attract_serial_t0, 0, 1 << 30},
    {"attract_serial_t1", nullptr, &Options::attract_serial_t1, -1, 1 << 30},
    {"tile_stream_wait", nullptr, &Options::tile_stream_wait, 1, 1 << 20},
    {"comm_world1", nullptr, &Options::comm_world1, 0, 1},
    {"rep_stats", nullptr, &Options::rep_stats, 0, 1},
    {"loop_serial", nullptr, &Options::loop_serial, 0, 1},
    {"bu_acqrel", nullptr, &Options::bu_acqrel, 0, 1},
    {"bh_split", nullptr, &Options::bh_split, 0, 1},
};
static const OptionField &option_field(const char *key) {
    for (const OptionField &f : k_options)
        if (std::strcmp(f.key, key) == 0) return f;
    fail(TSNE_ERR_ARG, std::string("unknown option '") + key + "'");
}
static void set_option(Options &o, const char *key, double v) {
    const OptionField &f = option_field(key);
    TSNE_REQUIRE(v >= f.lo && v <= f.hi, std::string("option '") + key + "' out of range");
    if (f.d) o.*f.d = v;
    else {
        TSNE_REQUIRE(v == std::floor(v), std::string("option '") + key + "' takes an integer");
        o.*f.i = (int)v;
    }
}
static double get_option(const Options &o, const char *key) {
    const OptionField &f = option_field(key);
    return f.d ? o.*f.d : (double)(o.*f.i);
}

}  // namespace tsne

using namespace tsne;

extern "C" {

int tsne_abi_version(void) { return TSNE_HIP_ABI_VERSION; }

const char *tsne_last_error(void) { return g_last_error.c_str(); }

void tsne_params_default(tsne_params *p) {
    if (!p) return;
    p->n_components = 2;
    p->metric = TSNE_METRIC_SQEUCLIDEAN;
    p->learning_rate = 1000.0;
    p->iterations = 300;
    p->early_exaggeration = 4.0;
    p->initial_momentum = 0.5;
    p->final_momentum = 0.8;
    p->theta = 0.25;
    p->min_gain = 0.01;
}

int tsne_metric_from_name(const char *name, int32_t *metric_out) {
    return guard([&] {
        std::string m = name ? name : "";
        int32_t v;
        if (m == "sqeuclidean") v = TSNE_METRIC_SQEUCLIDEAN;
        else if (m == "euclidean") v = TSNE_METRIC_EUCLIDEAN;
        else if (m == "cosine") v = TSNE_METRIC_COSINE;
        else fail(TSNE_ERR_ARG, "Metric '" + m + "' not defined");  // Tsne.scala:166
        if (metric_out) *metric_out = v;
    });
}

int tsne_coo_to_csr(const int32_t *row, const int32_t *col, const double *val, int64_t nnz, int64_t n,
                    int64_t *row_ptr_out, int32_t *col_out, double *val_out) {
    return guard([&] {
        TSNE_REQUIRE(nnz >= 0 && n >= 0 && row_ptr_out != nullptr, "bad arguments");
        TSNE_REQUIRE(nnz == 0 || (row && col && col_out), "NULL buffer");
        TSNE_REQUIRE((val == nullptr) == (val_out == nullptr), "val and val_out go together");
        std::fill(row_ptr_out, row_ptr_out + n + 1, (int64_t)0);
        for (int64_t e = 0; e < nnz; ++e) {
            const int32_t r = row[e];
            if (r < 0 || r >= n) fail(TSNE_ERR_ARG, "row index " + std::to_string(r) + " out of [0, n)");
            ++row_ptr_out[r + 1];
        }
        for (int64_t r = 0; r < n; ++r) row_ptr_out[r + 1] += row_ptr_out[r];
        std::vector<int64_t> next(row_ptr_out, row_ptr_out + n);   // stable: input order within a row
        for (int64_t e = 0; e < nnz; ++e) {
            const int64_t o = next[row[e]]++;
            col_out[o] = col[e];
            if (val_out) val_out[o] = val[e];
        }
    });
}

int tsne_shard_rows(int64_t n, int32_t world, int32_t rank, int64_t *r0, int64_t *r1) {
    return guard([&] {
        TSNE_REQUIRE(n >= 0 && world >= 1 && rank >= 0 && rank < world, "bad shard arguments");
        const int64_t chunk = ceil_div(n, world);
        const int64_t a = std::min<int64_t>(n, chunk * rank);
        if (r0) *r0 = a;
        if (r1) *r1 = std::min<int64_t>(n, a + chunk);
    });
}

int tsne_balance_cuts(const uint64_t *bcost, int64_t nb, int64_t n, int32_t world, int32_t bucket,
                      int64_t *bounds) {
    return guard([&] {
        TSNE_REQUIRE(bounds != nullptr && (bcost != nullptr || nb == 0) && nb >= 0 && n >= 0 && world >= 1 &&
                         bucket >= 1,
                     "bad balance arguments");
        uint64_t total = 0;
        for (int64_t b = 0; b < nb; ++b) total += bcost[b];
        bounds[0] = 0;
        bounds[world] = n;
        for (int r = 1; r < world; ++r) {
            const uint64_t target = total / world * r + (total % world) * r / world;
            bounds[r] = target == 0 ? 0 : n;
            uint64_t run = 0;
            for (int64_t b = 0; b < nb; ++b) {
                const uint64_t nxt = run + bcost[b];
                if (run < target && nxt >= target) { bounds[r] = std::min<int64_t>(n, (b + 1) * bucket); break; }
                run = nxt;
            }
        }
        for (int r = 1; r < world; ++r) {
            if (total == 0) bounds[r] = n * r / world;
            if (bounds[r] < bounds[r - 1]) bounds[r] = bounds[r - 1];
        }
    });
}

int tsne_dev_balance_cuts(tsne_ctx *ctx, const uint64_t *d_bcost, int64_t n, int32_t world, int64_t *d_bounds) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(d_bcost != nullptr && d_bounds != nullptr && n >= 0 && world >= 1, "bad balance arguments");
        bh_balance(ctx, reinterpret_cast<const unsigned long long *>(d_bcost), n, world, d_bounds);
    });
}

int tsne_ctx_create(int32_t device, tsne_ctx **out) {
    return guard([&] {
        TSNE_REQUIRE(out != nullptr, "out is NULL");
        *out = nullptr;
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
            fail(TSNE_ERR_NO_DEVICE, "no HIP device visible");
        TSNE_REQUIRE(device >= 0 && device < count, "device index out of range");
        TSNE_HIP(hipSetDevice(device));
        hipDeviceProp_t prop;
        TSNE_HIP(hipGetDeviceProperties(&prop, device));
        std::unique_ptr<tsne_ctx> c(new tsne_ctx());
        c->device = device;
        c->cu_count = prop.multiProcessorCount;
        TSNE_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
        TSNE_HIP(hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
        for (auto &e : c->aux_ev) TSNE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        TSNE_HIP(hipHostMalloc(reinterpret_cast<void **>(&c->pinned), 64 * sizeof(int32_t)));
        *out = c.release();
    });
}

int tsne_ctx_create_multi(const int32_t *devices, int32_t ndev, tsne_ctx **out) {
    return guard([&] {
        TSNE_REQUIRE(out != nullptr, "out is NULL");
        *out = nullptr;
        TSNE_REQUIRE(devices != nullptr && ndev >= 1 && ndev <= 64, "bad device list");
        bool same = true, distinct = true;
        for (int a = 0; a < ndev; ++a)
            for (int b = a + 1; b < ndev; ++b) {
                if (devices[a] == devices[b]) distinct = false;
                else same = false;
            }
        TSNE_REQUIRE(same || distinct, "devices must be all distinct (RCCL) or all the same (loopback ranks)");
        std::unique_ptr<tsne_ctx> g(new tsne_ctx());
        struct Undo {
            tsne_ctx *g;
            ~Undo() { if (g) for (tsne_ctx *c : g->group) tsne_ctx_destroy(c); }
        } undo{g.get()};
        for (int r = 0; r < ndev; ++r) {
            tsne_ctx *c = nullptr;
            const int rc = tsne_ctx_create(devices[r], &c);
            if (rc != TSNE_OK) throw Error(rc, g_last_error);
            g->group.push_back(c);
        }
        g->device = devices[0];
        g->cu_count = g->group[0]->cu_count;
        comm_init_group(g->group, same && ndev > 1);
        g->world = ndev;
        undo.g = nullptr;
        *out = g.release();
    });
}

int tsne_ctx_destroy(tsne_ctx *ctx) {
    if (!ctx) return TSNE_OK;
    if (!ctx->group.empty()) {
        int rc = TSNE_OK;
        for (tsne_ctx *c : ctx->group) {
            const int r = tsne_ctx_destroy(c);
            if (rc == TSNE_OK) rc = r;
        }
        delete ctx;
        return rc;
    }
    int rc = guard([&] {
        DeviceGuard g(ctx->device);
        (void)hipStreamSynchronize(ctx->stream);
        opt_destroy(ctx);
        delete ctx->single_tree;
        ctx->single_tree = nullptr;
        comm_destroy(ctx);
        ctx->timers.clear();
        ctx->ws.clear();
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
        if (ctx->aux_stream) (void)hipStreamSynchronize(ctx->aux_stream);
        if (ctx->aux_stream) (void)hipStreamDestroy(ctx->aux_stream);
        for (auto &e : ctx->aux_ev)
            if (e) (void)hipEventDestroy(e);
        if (ctx->st_stream) (void)hipStreamSynchronize(ctx->st_stream);
        if (ctx->st_stream) (void)hipStreamDestroy(ctx->st_stream);
        for (auto &e : ctx->st_ev)
            if (e) (void)hipEventDestroy(e);
    });
    delete ctx;
    return rc;
}

int tsne_ctx_set_stream(tsne_ctx *ctx, void *hip_stream) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        if (ctx->own_stream && ctx->stream) {
            TSNE_HIP(hipStreamSynchronize(ctx->stream));
            TSNE_HIP(hipStreamDestroy(ctx->stream));
        }
        if (hip_stream) {
            ctx->stream = static_cast<hipStream_t>(hip_stream);
            ctx->own_stream = false;
        } else {
            TSNE_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
            ctx->own_stream = true;
        }
    });
}

void *tsne_ctx_stream(tsne_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int tsne_ctx_set_option(tsne_ctx *ctx, const char *key, double value) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(key != nullptr, "option key is NULL");
        TSNE_REQUIRE(value == value, "option value is NaN");
        Options o = ctx->opts;
        set_option(o, key, value);
        ctx->opts = o;
        for (tsne_ctx *c : ctx->group) c->opts = o;
    });
}

int tsne_debug_wave_log(tsne_ctx *ctx, uint64_t *out, int64_t cap, int64_t *count) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(count != nullptr && (out != nullptr || cap == 0) && cap >= 0, "bad output buffer");
        DeviceGuard g(ctx->device);
        *count = 0;
        if (!ctx->ws.has("rep.wavelog")) return;
        const unsigned long long *d = ctx->ws.get<unsigned long long>("rep.wavelog", 1);
        uint64_t n = 0;
        TSNE_HIP(hipMemcpyAsync(&n, d, 8, hipMemcpyDeviceToHost, ctx->stream));
        TSNE_HIP(hipStreamSynchronize(ctx->stream));
        n = std::min<uint64_t>(n, (uint64_t)(1 << 17));
        *count = (int64_t)n;
        const uint64_t m = std::min<uint64_t>(n, (uint64_t)cap);
        if (m) {
            TSNE_HIP(hipMemcpyAsync(out, d + 1, 16 * m, hipMemcpyDeviceToHost, ctx->stream));
            TSNE_HIP(hipStreamSynchronize(ctx->stream));
        }
    });
}

int tsne_ctx_counter(tsne_ctx *ctx, const char *name, int64_t *value_out) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(name != nullptr && value_out != nullptr, "NULL argument");
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        const std::string k = name;
        if (k == "bh.narrow_groups") *value_out = ctx->single_tree ? bh_narrow_groups(ctx, *ctx->single_tree) : 0;
        else if (k == "opt.narrow_groups") *value_out = opt_tree(ctx) ? bh_narrow_groups(ctx, *opt_tree(ctx)) : 0;
        else if (k == "opt.wave_mhz") *value_out = opt_wave_mhz(ctx);
        else if (k == "bh.csort_oversized") *value_out = ctx->single_tree ? csort_oversized(ctx, ctx->single_tree->cs) : 0;
        else if (k == "opt.attract_kernel") *value_out = opt_attract_kernel(ctx);
        else if (k == "bh.spill_tasks" || k == "bh.spill_flags")
            *value_out = ctx->single_tree ? bh_spill_counter(ctx, *ctx->single_tree, k == "bh.spill_flags") : 0;
        else if (k == "opt.spill_tasks" || k == "opt.spill_flags")
            *value_out = opt_tree(ctx) ? bh_spill_counter(ctx, *opt_tree(ctx), k == "opt.spill_flags") : 0;
        else if (k == "bh.stream_lists")
            *value_out = ctx->single_tree ? bh_stream_counter(ctx, *ctx->single_tree) : 0;
        else if (k == "opt.stream_lists")
            *value_out = opt_tree(ctx) ? bh_stream_counter(ctx, *opt_tree(ctx)) : 0;
        else if (k.rfind("bh.", 0) == 0 && repulsion_stat(ctx, k, value_out)) {}
        else if (k == "comm.kind") *value_out = comm_counter(ctx, false);
        else if (k == "comm.calls") *value_out = comm_counter(ctx, true);
        else if (k == "opt.csort_oversized") *value_out = opt_tree(ctx) ? csort_oversized(ctx, opt_tree(ctx)->cs) : 0;
        else if (k == "opt.csort_oversized_total")
            *value_out = opt_tree(ctx) ? csort_oversized(ctx, opt_tree(ctx)->cs, true) : 0;
        else fail(TSNE_ERR_ARG, "unknown counter '" + k + "'");
    });
}

int tsne_ctx_loop_profile(tsne_ctx *ctx, char *buf, int64_t cap, int64_t *len_out) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(len_out != nullptr, "NULL argument");
        // the summary is taken (and the log cleared) once; a length query
        // (buf NULL) keeps it pending for the call that copies it out
        tsne_ctx *p = primary(ctx);
        if (p->loop_profile_pending.empty()) p->loop_profile_pending = comm_loop_profile(p);
        const std::string &js = p->loop_profile_pending;
        *len_out = (int64_t)js.size();
        if (buf && cap > 0) {
            const size_t k = std::min<size_t>(js.size(), (size_t)cap - 1);
            std::memcpy(buf, js.data(), k);
            buf[k] = 0;
            p->loop_profile_pending.clear();
        }
    });
}

int tsne_hip_versions(int32_t *built_out, int32_t *runtime_out) {
    return guard([&] {
        int rt = 0;
        TSNE_HIP(hipRuntimeGetVersion(&rt));
        if (built_out) *built_out = HIP_VERSION;
        if (runtime_out) *runtime_out = rt;
    });
}

int tsne_ctx_get_option(tsne_ctx *ctx, const char *key, double *value_out) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(key != nullptr && value_out != nullptr, "NULL argument");
        *value_out = get_option(primary(ctx)->opts, key);
    });
}

int tsne_ctx_synchronize(tsne_ctx *ctx) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        sync(ctx);
    });
}

int tsne_comm_unique_id(uint8_t id_out[TSNE_UNIQUE_ID_BYTES]) {
    return guard([&] {
        TSNE_REQUIRE(id_out != nullptr, "id_out is NULL");
        comm_unique_id(id_out);
    });
}

int tsne_ctx_init_comm(tsne_ctx *ctx, int32_t rank, int32_t world, const uint8_t id[TSNE_UNIQUE_ID_BYTES]) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(ctx->group.empty(), "a tsne_ctx_create_multi group has its communicator already");
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(world == 1 || id != nullptr, "unique id is NULL");
        comm_init(ctx, rank, world, id);
    });
}

int tsne_ctx_init_comm_callbacks(tsne_ctx *ctx, int32_t rank, int32_t world, const tsne_comm_ops *ops,
                                 void *user) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(ctx->group.empty(), "a tsne_ctx_create_multi group has its communicator already");
        DeviceGuard g(ctx->device);
        comm_init_callbacks(ctx, rank, world, ops, user);
    });
}

int tsne_ctx_rank(tsne_ctx *ctx, int32_t *rank, int32_t *world) {
    return guard([&] {
        check_ctx(ctx);
        if (rank) *rank = ctx->rank;
        if (world) *world = ctx->world;
    });
}

// ------------------------------------------------------------ device API

int tsne_dev_knn(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t k,
                 int64_t q0, int64_t q1, int32_t *d_idx, double *d_dist) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        knn_device(ctx, dX, n, d, metric, k, q0, q1, d_idx, d_dist);
    });
}

int tsne_dev_pairwise_affinities(tsne_ctx *ctx, const int64_t *d_row_ptr, const double *d_dist,
                                 int64_t nrows, double perplexity, double *d_p) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        affinities_device(ctx, d_row_ptr, d_dist, nrows, perplexity, d_p);
    });
}

int tsne_dev_joint_distribution(tsne_ctx *ctx, const int64_t *d_row_ptr, const int32_t *d_col,
                                const double *d_p, int64_t n, int64_t cap, int64_t *d_out_row_ptr,
                                int32_t *d_out_col, double *d_out_val, int64_t *nnz_out) {
    int64_t nnz = -1;
    int rc = guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(n >= 1, "empty matrix");
        nnz = joint_device(ctx, d_row_ptr, d_col, d_p, n, cap, d_out_row_ptr, d_out_col, d_out_val);
    });
    if (nnz_out) *nnz_out = nnz;
    if (rc == TSNE_OK && nnz > cap) {
        g_last_error = "joint distribution needs " + std::to_string(nnz) + " entries, cap is " + std::to_string(cap);
        return TSNE_ERR_CAPACITY;
    }
    return rc;
}

int tsne_dev_opt_setup(tsne_ctx *ctx, const tsne_params *params, const int64_t *d_row_ptr,
                       const int32_t *d_col, const double *d_P, int64_t n, double *d_Y,
                       double *d_upd, double *d_gains) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        opt_setup(ctx, params, d_row_ptr, d_col, d_P, n, d_Y, d_upd, d_gains);
    });
}

int tsne_dev_opt_step(tsne_ctx *ctx, int32_t t) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        opt_step(ctx, t);
    });
}

int tsne_dev_opt_losses(tsne_ctx *ctx, int32_t *loss_keys, double *loss_vals, int32_t cap, int32_t *n_loss) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        int32_t k = opt_losses(ctx, loss_keys, loss_vals, cap);
        if (n_loss) *n_loss = k;
    });
}

int tsne_ctx_stage_ms(tsne_ctx *ctx, const char *stage, double *ms_out, int32_t cap, int32_t *count) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(stage != nullptr, "stage is NULL");
        const std::vector<double> v = ctx->timers.ms(stage);
        for (size_t k = 0; k < v.size() && (int64_t)k < cap; ++k) ms_out[k] = v[k];
        if (count) *count = (int32_t)v.size();
    });
}

int tsne_dev_opt_attract_log(tsne_ctx *ctx, int32_t *iters, int32_t *standalone, double *ms, int32_t cap,
                             int32_t *count) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        int32_t k = opt_attract_log(ctx, iters, standalone, ms, cap);
        if (count) *count = k;
    });
}

int tsne_dev_opt_last_z(tsne_ctx *ctx, double *z_out) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(z_out != nullptr, "z_out is NULL");
        *z_out = opt_last_z(ctx);
    });
}

int tsne_dev_opt_profile(tsne_ctx *ctx, int32_t enable, double *ms_out5, int64_t *counters_out10) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        opt_profile(ctx, enable, ms_out5, counters_out10);
    });
}

// ------------------------------------------------------------ host API

int tsne_knn(tsne_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t metric, int32_t k,
             int64_t q0, int64_t q1, int32_t *idx_out, double *dist_out) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(X && idx_out && dist_out, "NULL buffer");
        TSNE_REQUIRE(n >= 2 && d >= 1 && k >= 1, "bad sizes");
        TSNE_REQUIRE(q0 >= 0 && q1 <= n && q0 <= q1, "query range out of bounds");
        const int64_t kk = std::min<int64_t>(k, n - 1);
        if (!ctx->group.empty()) {   // query rows split evenly over the group's devices
            const int world = (int)ctx->group.size();
            run_group(ctx, [&](tsne_ctx *c, int r) {
                const int64_t a = q0 + (q1 - q0) * r / world, b = q0 + (q1 - q0) * (r + 1) / world;
                if (b == a) return;
                double *dX = upload(c, "h.X", X, (size_t)(n * d));
                int32_t *di = c->ws.get<int32_t>("h.knn_idx", (size_t)((b - a) * kk));
                double *dd = c->ws.get<double>("h.knn_dist", (size_t)((b - a) * kk));
                knn_device(c, dX, n, d, metric, k, a, b, di, dd);
                download(c, idx_out + (a - q0) * kk, di, (size_t)((b - a) * kk));
                download(c, dist_out + (a - q0) * kk, dd, (size_t)((b - a) * kk));
                sync(c);
            });
            return;
        }
        DeviceGuard g(ctx->device);
        double *dX = upload(ctx, "h.X", X, (size_t)(n * d));
        int32_t *di = ctx->ws.get<int32_t>("h.knn_idx", (size_t)std::max<int64_t>(1, (q1 - q0) * kk));
        double *dd = ctx->ws.get<double>("h.knn_dist", (size_t)std::max<int64_t>(1, (q1 - q0) * kk));
        knn_device(ctx, dX, n, d, metric, k, q0, q1, di, dd);
        download(ctx, idx_out, di, (size_t)((q1 - q0) * kk));
        download(ctx, dist_out, dd, (size_t)((q1 - q0) * kk));
        sync(ctx);
    });
}

int tsne_project_knn(tsne_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t metric, int32_t k,
                     int32_t iterations, const double *shifts, int32_t *idx_out, double *dist_out) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(X && idx_out && dist_out && n >= 2 && d >= 1 && iterations >= 1, "bad arguments");
        TSNE_REQUIRE(iterations == 1 || shifts, "NULL shifts");
        const int64_t kk = std::min<int64_t>(k, n - 1);
        double *dX = upload(ctx, "h.X", X, (size_t)(n * d));
        double *dr = iterations > 1 ? upload(ctx, "h.shifts", shifts, (size_t)(iterations - 1) * d) : nullptr;
        int32_t *di = ctx->ws.get<int32_t>("h.pidx", (size_t)(n * kk));
        double *dd = ctx->ws.get<double>("h.pdist", (size_t)(n * kk));
        project_knn_device(ctx, dX, n, d, metric, k, iterations, dr, di, dd);
        download(ctx, idx_out, di, (size_t)(n * kk));
        download(ctx, dist_out, dd, (size_t)(n * kk));
        sync(ctx);
    });
}

int tsne_dev_project_knn(tsne_ctx *ctx, const double *dX, int64_t n, int32_t d, int32_t metric, int32_t k,
                         int32_t iterations, const double *d_shifts, int32_t *d_idx, double *d_dist) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        project_knn_device(ctx, dX, n, d, metric, k, iterations, d_shifts, d_idx, d_dist);
    });
}

int tsne_pairwise_affinities(tsne_ctx *ctx, const int64_t *row_ptr, const double *dist, int64_t nrows,
                             double perplexity, double *p_out) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(row_ptr && nrows >= 0, "bad CSR");
        const int64_t nnz = row_ptr[nrows] - row_ptr[0];
        TSNE_REQUIRE(row_ptr[0] == 0, "row_ptr[0] must be 0");
        TSNE_REQUIRE(nnz == 0 || (dist && p_out), "NULL buffer");
        int64_t *drp = upload(ctx, "h.rp", row_ptr, (size_t)nrows + 1);
        double *dd = upload(ctx, "h.dist", dist, (size_t)nnz);
        double *dp = ctx->ws.get<double>("h.p", (size_t)nnz + 1);
        affinities_device(ctx, drp, dd, nrows, perplexity, dp);
        download(ctx, p_out, dp, (size_t)nnz);
        sync(ctx);
    });
}

int tsne_joint_distribution(tsne_ctx *ctx, const int64_t *row_ptr, const int32_t *col, const double *p,
                            int64_t n, int64_t cap, int64_t *out_row_ptr, int32_t *out_col,
                            double *out_val, int64_t *nnz_out) {
    int64_t nnz = -1;
    int rc = guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(row_ptr && n >= 1 && row_ptr[0] == 0, "bad CSR");
        const int64_t nin = row_ptr[n];
        for (int64_t e = 0; e < nin; ++e)
            if (col[e] < 0 || col[e] >= n) fail(TSNE_ERR_ARG, "column index out of range");
        int64_t *drp = upload(ctx, "h.rp", row_ptr, (size_t)n + 1);
        int32_t *dc = upload(ctx, "h.col", col, (size_t)nin);
        double *dp = upload(ctx, "h.p", p, (size_t)nin);
        const int64_t dcap = 2 * nin + 1;
        int64_t *orp = ctx->ws.get<int64_t>("h.orp", (size_t)n + 1);
        int32_t *oc = ctx->ws.get<int32_t>("h.ocol", (size_t)dcap);
        double *ov = ctx->ws.get<double>("h.oval", (size_t)dcap);
        nnz = joint_device(ctx, drp, dc, dp, n, dcap, orp, oc, ov);
        if (nnz <= cap) {
            download(ctx, out_row_ptr, orp, (size_t)n + 1);
            download(ctx, out_col, oc, (size_t)nnz);
            download(ctx, out_val, ov, (size_t)nnz);
            sync(ctx);
        }
    });
    if (nnz_out) *nnz_out = nnz;
    if (rc == TSNE_OK && nnz > cap) {
        g_last_error = "joint distribution needs " + std::to_string(nnz) + " entries, cap is " + std::to_string(cap);
        return TSNE_ERR_CAPACITY;
    }
    return rc;
}

int tsne_gradient(tsne_ctx *ctx, const int64_t *row_ptr, const int32_t *col, const double *P, int64_t n,
                  const double *Y, int32_t metric, double theta, double exaggeration, double *grad_out,
                  double *sumq_out, double *loss_out) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(row_ptr && Y && grad_out && n >= 1 && row_ptr[0] == 0, "bad arguments");
        TSNE_REQUIRE(metric >= 0 && metric <= 2, "unknown metric");
        const int64_t nnz = row_ptr[n];
        int64_t *drp = upload(ctx, "h.rp", row_ptr, (size_t)n + 1);
        int32_t *dc = upload(ctx, "h.col", col, (size_t)nnz);
        double *dp = upload(ctx, "h.p", P, (size_t)nnz);
        double *dY = upload(ctx, "h.Y", Y, (size_t)n * 2);
        double *dg = ctx->ws.get<double>("h.grad", (size_t)n * 2);
        gradient_device(ctx, drp, dc, dp, n, dY, metric, theta, exaggeration, dg, sumq_out, loss_out);
        download(ctx, grad_out, dg, (size_t)n * 2);
        sync(ctx);
    });
}

int tsne_gradient_c(tsne_ctx *ctx, const int64_t *row_ptr, const int32_t *col, const double *P, int64_t n,
                    int32_t c, const double *Y, int32_t metric, double theta, double exaggeration,
                    double *grad_out, double *sumq_out, double *loss_out) {
    if (c == 2) return tsne_gradient(ctx, row_ptr, col, P, n, Y, metric, theta, exaggeration, grad_out, sumq_out,
                                     loss_out);
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        if (c != 3) fail(TSNE_ERR_UNSUPPORTED, "n_components must be 2 (quadtree) or 3 (octree extension)");
        TSNE_REQUIRE(row_ptr && Y && grad_out && n >= 1 && row_ptr[0] == 0, "bad arguments");
        TSNE_REQUIRE(metric >= 0 && metric <= 2, "unknown metric");
        const int64_t nnz = row_ptr[n];
        int64_t *drp = upload(ctx, "h.rp", row_ptr, (size_t)n + 1);
        int32_t *dc = upload(ctx, "h.col", col, (size_t)nnz);
        double *dp = upload(ctx, "h.p", P, (size_t)nnz);
        double *dY = upload(ctx, "h.Y", Y, (size_t)n * 3);
        double *dg = ctx->ws.get<double>("h.grad", (size_t)n * 3);
        gradient3_device(ctx, drp, dc, dp, n, dY, metric, theta, exaggeration, dg, sumq_out, loss_out);
        download(ctx, grad_out, dg, (size_t)n * 3);
        sync(ctx);
    });
}

int tsne_repulsion(tsne_ctx *ctx, const double *Y, int64_t n, int32_t c, double theta, double *F_out,
                   double *z_out) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        if (c != 2 && c != 3) fail(TSNE_ERR_UNSUPPORTED, "n_components must be 2 (quadtree) or 3 (octree extension)");
        TSNE_REQUIRE(Y && F_out && z_out && n >= 1, "bad arguments");
        double *dY = upload(ctx, "h.Y", Y, (size_t)n * c);
        double *dF = ctx->ws.get<double>("h.repF", (size_t)n * c);
        double *dz = ctx->ws.get<double>("h.repz", (size_t)n);
        repulsion_device(ctx, dY, n, c, theta, dF, dz);
        download(ctx, F_out, dF, (size_t)n * c);
        download(ctx, z_out, dz, (size_t)n);
        sync(ctx);
    });
}

int tsne_dev_repulsion(tsne_ctx *ctx, const double *dY, int64_t n, int32_t c, double theta, double *d_F,
                       double *d_z) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        if (c != 2 && c != 3) fail(TSNE_ERR_UNSUPPORTED, "n_components must be 2 (quadtree) or 3 (octree extension)");
        TSNE_REQUIRE(dY && d_F && d_z && n >= 1, "bad arguments");
        repulsion_device(ctx, dY, n, c, theta, d_F, d_z);
    });
}

int tsne_update_embedding(tsne_ctx *ctx, int64_t n, int32_t c, const double *grad, double *Y, double *upd,
                          double *gains, double min_gain, double momentum, double learning_rate) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(grad && Y && upd && gains && n >= 0 && c >= 1, "bad arguments");
        const size_t ne = (size_t)(n * c);
        double *dg = upload(ctx, "h.grad", grad, ne);
        double *dY = upload(ctx, "h.Y", Y, ne);
        double *du = upload(ctx, "h.upd", upd, ne);
        double *dn = upload(ctx, "h.gains", gains, ne);
        update_device(ctx, n, c, dg, dY, du, dn, min_gain, momentum, learning_rate);
        download(ctx, Y, dY, ne);
        download(ctx, upd, du, ne);
        download(ctx, gains, dn, ne);
        sync(ctx);
    });
}

int tsne_center_embedding(tsne_ctx *ctx, int64_t n, int32_t c, double *Y) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(Y && n >= 1 && c >= 1 && c <= 8, "bad arguments");
        double *dY = upload(ctx, "h.Y", Y, (size_t)(n * c));
        center_device(ctx, n, c, dY);
        download(ctx, Y, dY, (size_t)(n * c));
        sync(ctx);
    });
}

int tsne_init_working_set(tsne_ctx *ctx, int64_t n, int32_t c, uint64_t seed, double *Y, double *upd,
                          double *gains) {
    return guard([&] {
        check_ctx(ctx);
        ctx = primary(ctx);
        DeviceGuard g(ctx->device);
        TSNE_REQUIRE(Y && upd && gains && n >= 0 && c >= 1, "bad arguments");
        const size_t ne = (size_t)(n * c);
        double *dY = ctx->ws.get<double>("h.Y", ne + 1);
        double *du = ctx->ws.get<double>("h.upd", ne + 1);
        double *dn = ctx->ws.get<double>("h.gains", ne + 1);
        init_working_set_device(ctx, n, c, seed, dY, du, dn);
        download(ctx, Y, dY, ne);
        download(ctx, upd, du, ne);
        download(ctx, gains, dn, ne);
        sync(ctx);
    });
}

int tsne_optimize(tsne_ctx *ctx, const tsne_params *params, const int64_t *row_ptr, const int32_t *col,
                  const double *P, int64_t n, double *Y, double *upd, double *gains, int32_t *loss_keys,
                  double *loss_vals, int32_t loss_cap, int32_t *n_loss) {
    return guard([&] {
        check_ctx(ctx);
        TSNE_REQUIRE(params && row_ptr && Y && upd && gains && n >= 1 && row_ptr[0] == 0, "bad arguments");
        if (params->n_components != 2 && params->n_components != 3)
            fail(TSNE_ERR_UNSUPPORTED, "n_components must be 2 (quadtree) or 3 (octree extension)");
        const size_t C = (size_t)params->n_components;
        const int64_t nnz = row_ptr[n];
        TSNE_REQUIRE(nnz == 0 || (col && P), "NULL buffer");
        for (int64_t e = 0; e < nnz; ++e)
            if (col[e] < 0 || col[e] >= n) fail(TSNE_ERR_ARG, "column index out of range");
        // every rank gets the full P and working set and runs the same
        // iterations on its own rows; in a group (one thread per rank, shared
        // host buffers) rank 0 writes the results back
        auto run = [&](tsne_ctx *c, int rank) {
            int64_t *drp = upload(c, "h.rp", row_ptr, (size_t)n + 1);
            int32_t *dc = upload(c, "h.col", col, (size_t)nnz);
            double *dp = upload(c, "h.p", P, (size_t)nnz);
            double *dY = upload(c, "h.Yopt", Y, (size_t)n * C);
            double *du = upload(c, "h.updopt", upd, (size_t)n * C);
            double *dn = upload(c, "h.gainsopt", gains, (size_t)n * C);
            opt_setup(c, params, drp, dc, dp, n, dY, du, dn);
            for (int32_t t = 1; t <= params->iterations; ++t) opt_step(c, t);
            opt_sync(c);
            if (rank != 0) {
                sync(c);
                return;
            }
            download(c, Y, dY, (size_t)n * C);
            download(c, upd, du, (size_t)n * C);
            download(c, gains, dn, (size_t)n * C);
            sync(c);
            int32_t k = opt_losses(c, loss_keys, loss_vals, loss_cap);
            if (n_loss) *n_loss = k;
        };
        if (!ctx->group.empty()) {
            run_group(ctx, run);
            return;
        }
        DeviceGuard g(ctx->device);
        run(ctx, 0);   // one process per rank: every process writes its own host buffers
    });
}

int tsne_dev_opt_sync(tsne_ctx *ctx) {
    return guard([&] {
        check_ctx(ctx);
        ctx = opt_ctx(ctx);
        DeviceGuard g(ctx->device);
        opt_sync(ctx);
    });
}

}  // extern "C"
