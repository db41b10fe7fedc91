// Failure injection for the collective abort protocol (csrc/comm_guard.hpp)
// with a fake backend on the CPU: a rank inside a collective whose peer never
// arrives must be released by abort() from another thread, and no library
// call may reach the communicator after abort freed it.  Prints "ok".
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>

#include "comm_guard.hpp"

struct Fake {
    std::atomic<bool> peer{false};      // the collective's peer has arrived
    std::atomic<int> async_err{0};      // > 0: the next poll reports this library error
    std::atomic<bool> freed{false};
    std::atomic<int> aborts{0}, destroys{0};
    std::atomic<int> after_free{0};     // library calls on a freed communicator (must stay 0)
    std::atomic<int> calls{0};
};
struct FakeBackend {
    using Handle = Fake *;
    template <class F> static int call(Handle h, F &&f) {
        if (h->freed) ++h->after_free;
        ++h->calls;
        return f(h);
    }
    static int poll(Handle h) {
        if (h->freed) ++h->after_free;
        if (h->async_err) return -h->async_err;
        return h->peer ? 0 : 1;
    }
    static void abort(Handle h) { h->freed = true; ++h->aborts; }
    static void destroy(Handle h) { h->freed = true; ++h->destroys; }
};

static int fail(const char *m) {
    std::printf("FAIL %s\n", m);
    return 1;
}

int main() {
    using namespace std::chrono;
    {   // the peer died: the owner waits in the poll loop until abort() releases it
        Fake f;
        tsne::CommGuard<FakeBackend> g;
        g.h = &f;
        std::atomic<int> rc{99};
        std::thread owner([&] { rc = g.run([](Fake *h) { return h->peer ? 0 : 1; }); });
        std::this_thread::sleep_for(milliseconds(50));
        if (rc != 99) return fail("returned before the peer or an abort");
        const auto t0 = steady_clock::now();
        std::thread peer([&] { g.abort(); });   // the failing peer's thread
        peer.join();
        owner.join();
        if (duration_cast<milliseconds>(steady_clock::now() - t0).count() > 1000) return fail("abort blocked");
        if (rc != -1) return fail("owner not released with 'aborted'");
        if (f.after_free != 0) return fail("library call after abort");
        // later collectives fail at once, without touching the communicator
        const int c0 = f.calls;
        if (g.run([](Fake *) { return 0; }) != -1 || f.calls != c0) return fail("call after abort");
        g.abort();   // idempotent
        g.destroy();
    }
    {   // the peer arrives: the collective completes
        Fake f;
        tsne::CommGuard<FakeBackend> g;
        g.h = &f;
        std::atomic<int> rc{99};
        std::thread owner([&] { rc = g.run([](Fake *h) { return h->peer ? 0 : 1; }); });
        std::this_thread::sleep_for(milliseconds(20));
        f.peer = true;
        owner.join();
        if (rc != 0) return fail("completed collective reported an error");
        g.destroy();
        if (!f.freed) return fail("destroy");
    }
    {   // the library reports an async error while the collective is in flight:
        // run() fails with it, and destroy() then aborts the errored communicator
        Fake f;
        tsne::CommGuard<FakeBackend> g;
        g.h = &f;
        std::atomic<int> rc{99};
        std::thread owner([&] { rc = g.run([](Fake *h) { return h->peer ? 0 : 1; }); });
        std::this_thread::sleep_for(milliseconds(20));
        f.async_err = 7;
        owner.join();
        if (rc != -2) return fail("async error not reported");
        if (g.error() != 7) return fail("the async error's own code not kept");
        g.destroy();
        if (f.aborts != 1 || f.destroys != 0) return fail("errored communicator not aborted at destroy");
        if (f.after_free != 0) return fail("library call after free");
    }
    {   // a clean run is destroyed in order (finalize + destroy), not aborted
        Fake f;
        f.peer = true;
        tsne::CommGuard<FakeBackend> g;
        g.h = &f;
        if (g.run([](Fake *) { return 0; }) != 0 || g.error() != 0) return fail("clean run");
        g.destroy();
        if (f.aborts != 0 || f.destroys != 1) return fail("clean communicator not destroyed in order");
    }
    {   // many concurrent aborts against a rank issuing collectives in a loop
        for (int rep = 0; rep < 200; ++rep) {
            Fake f;
            f.peer = true;
            tsne::CommGuard<FakeBackend> g;
            g.h = &f;
            std::thread owner([&] {
                for (int i = 0; i < 1000; ++i)
                    if (g.run([](Fake *) { return 0; }) == -1) break;
            });
            std::thread a([&] { g.abort(); }), b([&] { g.abort(); });
            a.join(); b.join(); owner.join();
            if (f.after_free != 0) return fail("race: call after abort");
        }
    }
    std::printf("ok\n");
    return 0;
}
