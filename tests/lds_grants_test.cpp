// CPU test of the dynamic-LDS opt-in bookkeeping (csrc/lds_grants.h), built
// and run by tests/test_lds_grants.py with g++.  A fake `set` stands in for
// hipFuncSetAttribute and counts its calls per (device, kernel).
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "../distributed_processor_amd/csrc/lds_grants.h"

static int failures = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); failures++; } \
    } while (0)

int main()
{
    using dpemu::LdsGrants;
    static const char k1 = 0, k2 = 0;        // two "kernels"
    const void *f1 = &k1, *f2 = &k2;
    {
        LdsGrants g;
        int calls = 0;
        auto set_ok = [&] { calls++; return 0; };
        CHECK(g.ensure(0, f1, 32 * 1024, set_ok) == 0 && calls == 0);       // under the default: no opt-in
        CHECK(g.ensure(0, f1, 80 * 1024, set_ok) == 0 && calls == 1);
        CHECK(g.ensure(0, f1, 72 * 1024, set_ok) == 0 && calls == 1);       // covered by the grant
        CHECK(g.ensure(0, f1, 96 * 1024, set_ok) == 0 && calls == 2);       // grows
        CHECK(g.granted(0, f1) == 96 * 1024);
        // another device, same kernel: its own opt-in (the round-3 static skipped it)
        CHECK(g.ensure(1, f1, 80 * 1024, set_ok) == 0 && calls == 3);
        CHECK(g.granted(1, f1) == 80 * 1024 && g.granted(0, f1) == 96 * 1024);
        // another kernel, same device
        CHECK(g.ensure(0, f2, 80 * 1024, set_ok) == 0 && calls == 4);
        // a failed opt-in records nothing and returns the error
        auto set_bad = [&] { calls++; return 7; };
        CHECK(g.ensure(2, f1, 80 * 1024, set_bad) == 7 && calls == 5);
        CHECK(g.granted(2, f1) == 0);
        CHECK(g.ensure(2, f1, 80 * 1024, set_ok) == 0 && calls == 6);
    }
    {
        // many threads, two devices, growing requests: every request is
        // covered when ensure() returns, and each (device, size step) is set
        // at most once per thread that saw it uncovered
        LdsGrants g;
        std::atomic<int> calls{0};
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        for (int t = 0; t < 8; t++) {
            th.emplace_back([&, t] {
                for (int i = 0; i < 2000; i++) {
                    const int dev = (t + i) & 1;
                    const size_t bytes = (65 + (i % 64)) * 1024;
                    if (g.ensure(dev, f1, bytes, [&] { calls++; return 0; }) != 0) bad++;
                    if (g.granted(dev, f1) < bytes) bad++;
                }
            });
        }
        for (auto &x : th) x.join();
        CHECK(bad == 0);
        CHECK(g.granted(0, f1) == 128 * 1024 && g.granted(1, f1) == 128 * 1024);
        CHECK(calls <= 2 * 64 * 8);
    }
    std::printf(failures ? "FAILED %d\n" : "OK\n", failures);
    return failures ? 1 : 0;
}
