// lds_grants.h -- bookkeeping of the dynamic-LDS opt-in (host code only).
//
// A launch with more than 64 KiB of dynamic LDS needs
// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) first, and the
// attribute belongs to (device, kernel): a process driving two devices, or
// two threads launching on one, must each see their own grant.  LdsGrants
// records the largest size granted per (device, kernel) under a mutex and
// asks the caller's `set` only when a request grows past it.  Header-only and
// free of HIP types so the CPU test suite can exercise it with a fake `set`
// (tests/test_lds_grants.py).
#pragma once

#include <cstddef>
#include <map>
#include <mutex>
#include <utility>

namespace dpemu {

class LdsGrants {
public:
    static constexpr size_t DEFAULT_LIMIT = 64 * 1024;   // no opt-in needed up to here

    // ensure `bytes` of dynamic LDS may be launched for `fn` on `device`;
    // `set()` performs the opt-in on the current device and returns 0 on
    // success (an error code otherwise, returned as is, nothing recorded)
    template <typename Set>
    int ensure(int device, const void *fn, size_t bytes, Set &&set)
    {
        if (bytes <= DEFAULT_LIMIT) return 0;
        std::lock_guard<std::mutex> lock(mu_);
        size_t &g = granted_[std::make_pair(device, fn)];
        if (bytes <= g) return 0;
        const int e = set();
        if (e == 0) g = bytes;
        return e;
    }

    size_t granted(int device, const void *fn)
    {
        std::lock_guard<std::mutex> lock(mu_);
        auto it = granted_.find(std::make_pair(device, fn));
        return it == granted_.end() ? 0 : it->second;
    }

private:
    std::mutex mu_;
    std::map<std::pair<int, const void *>, size_t> granted_;
};

}  // namespace dpemu
