// comm_guard.hpp -- abort protocol of a non-blocking collective communicator.
//
// The optimizer's collectives run on the rank's own thread; abort() runs on a
// failing peer's thread (capi.cpp run_group).  The communicator is created
// non-blocking (RCCL config.blocking = 0), so every library call returns at
// once (success, an error, or "in progress"); the owner then polls the
// communicator's async state.  Rules:
//   * `api` is held only around one non-blocking library call (never across
//     a wait), so abort() always gets it promptly: no deadlock with an owner
//     waiting for a peer that has died (the round-4 advisor's finding);
//   * abort() sets `aborted` first, then aborts the communicator under `api`
//     exactly once; the owner checks `aborted` under `api` before every call,
//     so no call ever reaches the library after the communicator was freed;
//   * a poll that sees `aborted` fails with the caller's error instead of
//     waiting on;
//   * a call or poll that reports a library error records it (`err`, under
//     `api`): the communicator is then in an error state, so destroy() takes
//     the abort path (NCCL's rule for an errored communicator) instead of the
//     orderly finalize + destroy, and the caller's message names the async
//     error itself rather than the enqueue's "in progress".
// The backend B supplies the library calls; the header has no RCCL dependency
// so that the protocol is tested on the CPU with a fake backend
// (tests/test_comm_guard.py).
#pragma once

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

namespace tsne {

// B: struct with
//   using Handle = ...;
//   static int call(Handle, F&&)   -- run one non-blocking op: 0 ok, 1 in progress, <0 error
//   static int poll(Handle)        -- async state: 0 done, 1 in progress, <0 error
//   static void abort(Handle)      -- free the communicator (stops its in-flight work)
//   static void destroy(Handle)    -- orderly teardown
template <class B>
struct CommGuard {
    typename B::Handle h{};
    std::mutex api;
    std::atomic<bool> aborted{false};
    bool freed = false;   // under api
    int err = 0;          // under api: the backend's error (-code) once a call or poll failed

    // 0 ok; -1 aborted (by another thread); -2 library error (error() names it)
    template <class F> int run(F &&op) {
        int rc;
        {
            std::lock_guard<std::mutex> lk(api);
            if (aborted.load()) return -1;
            rc = B::call(h, op);
            if (rc < 0) err = -rc;
        }
        while (rc == 1) {
            std::this_thread::yield();
            std::lock_guard<std::mutex> lk(api);
            if (aborted.load()) return -1;
            rc = B::poll(h);
            if (rc < 0) err = -rc;
        }
        return rc < 0 ? -2 : 0;
    }
    // the backend's error code of the last failed call or poll (0: none)
    int error() {
        std::lock_guard<std::mutex> lk(api);
        return err;
    }
    // callable from any thread, any number of times
    void abort() {
        aborted.store(true);
        std::lock_guard<std::mutex> lk(api);
        if (!freed) {
            freed = true;
            B::abort(h);
        }
    }
    void destroy() {
        std::lock_guard<std::mutex> lk(api);
        if (!freed) {
            freed = true;
            if (err) B::abort(h);   // an errored communicator is aborted, not finalized
            else B::destroy(h);
        }
    }
};

}  // namespace tsne
