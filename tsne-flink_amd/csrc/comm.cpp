// comm.cpp -- RCCL (over xGMI) for the row-sharded multi-GPU path: one
// process per GPU, the unique id shipped out of band by the caller.
// Per optimizer iteration the traffic is an all-reduce of the zero-filled
// (F, z) buffers holding each rank's cost-balanced BH slice, an all-reduce of
// the 256-query bucket costs (n/256 integers), the all-gather of the updated
// embedding slices, and every 10th iteration a one-double all-reduce of the
// loss.
#include <rccl/rccl.h>

#include "common.hpp"

namespace tsne {

struct Comm {
    ncclComm_t comm = nullptr;
};

static void nccl_check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) fail(TSNE_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
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
    if (world == 1) { ctx->rank = 0; ctx->world = 1; return; }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    Comm *c = new Comm();
    ncclResult_t r = ncclCommInitRank(&c->comm, world, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        nccl_check(r, "ncclCommInitRank");
    }
    ctx->comm = c;
    ctx->rank = rank;
    ctx->world = world;
}

void comm_destroy(tsne_ctx *ctx) {
    if (ctx->comm) {
        if (ctx->comm->comm) (void)ncclCommDestroy(ctx->comm->comm);
        delete ctx->comm;
        ctx->comm = nullptr;
    }
    ctx->rank = 0;
    ctx->world = 1;
}

void comm_allgather_bytes(tsne_ctx *ctx, const void *send, void *recv, size_t bytes_per_rank) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    nccl_check(ncclAllGather(send, recv, bytes_per_rank, ncclUint8, ctx->comm->comm, ctx->stream),
               "ncclAllGather");
}

void comm_allreduce_sum_u64(tsne_ctx *ctx, unsigned long long *buf, size_t count) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    nccl_check(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, ctx->comm->comm, ctx->stream),
               "ncclAllReduce");
}

void comm_allreduce_sum_f64(tsne_ctx *ctx, double *buf, size_t count) {
    TSNE_REQUIRE(ctx->comm != nullptr, "communicator not initialised");
    nccl_check(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, ctx->comm->comm, ctx->stream),
               "ncclAllReduce");
}

}  // namespace tsne
