// covt_scratch.h -- per (device, stream) device scratch of the small-batch split passes (geometry assembly,
// property materialization; covt_assemble.hip, covt_props.hip).
//
// Launches on one stream are ordered, so they share one scratch block; the block's look-back records carry
// an epoch that the launch's own prep kernel advances in device memory (so a captured HIP graph replays
// with a fresh epoch every time).  A block is allocated and zeroed on a stream's first use; at most
// kMaxSlots blocks are kept per kind, the least recently used one is freed beyond that (hipFree waits for
// the device), and covt_release_scratch (include/covt.h) frees them on request.
#ifndef COVT_SCRATCH_H
#define COVT_SCRATCH_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

namespace covt {

class StreamScratch {
   public:
    static constexpr size_t kMaxSlots = 16;
    explicit StreamScratch(size_t bytes) : bytes_(bytes) {}

    // the block of (current device, s), or nullptr on an allocation / device error (nothing is kept then)
    void* get(hipStream_t s) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return nullptr;
        std::lock_guard<std::mutex> g(mu_);
        const auto key = std::make_pair(dev, s);
        auto it = slots_.find(key);
        if (it != slots_.end()) {
            it->second.used = ++clock_;
            return it->second.p;
        }
        if (slots_.size() >= kMaxSlots) {  // evict the least recently used block
            auto lru = slots_.begin();
            for (auto j = slots_.begin(); j != slots_.end(); ++j)
                if (j->second.used < lru->second.used) lru = j;
            free_slot(lru->first.first, lru->second.p);
            slots_.erase(lru);
        }
        void* p = nullptr;
        if (hipMalloc(&p, bytes_) != hipSuccess) return nullptr;
        // zero: epoch 0 is never a launch's, so no record reads as current before it is written.  On `s`
        // itself: a non-blocking stream (PyTorch's) is not ordered after the null stream's hipMemset
        if (hipMemsetAsync(p, 0, bytes_, s) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        slots_[key] = Slot{p, ++clock_};
        return p;
    }

    // frees the block of (current device, s), or every block when `all`; returns the number freed
    int release(hipStream_t s, bool all) {
        int dev = 0;
        if (!all && hipGetDevice(&dev) != hipSuccess) return 0;
        std::lock_guard<std::mutex> g(mu_);
        int n = 0;
        for (auto it = slots_.begin(); it != slots_.end();) {
            if (all || it->first == std::make_pair(dev, s)) {
                free_slot(it->first.first, it->second.p);
                it = slots_.erase(it);
                ++n;
            } else {
                ++it;
            }
        }
        return n;
    }

    size_t size() {
        std::lock_guard<std::mutex> g(mu_);
        return slots_.size();
    }

   private:
    struct Slot {
        void* p;
        uint64_t used;
    };
    static void free_slot(int dev, void* p) {
        int cur = 0;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        if (have && cur != dev) (void)hipSetDevice(dev);
        (void)hipFree(p);  // waits for the device: no launch still uses the block
        if (have && cur != dev) (void)hipSetDevice(cur);
    }
    size_t bytes_;
    std::mutex mu_;
    std::map<std::pair<int, hipStream_t>, Slot> slots_;
    uint64_t clock_ = 0;
};

// the two kinds' managers (covt_assemble.hip, covt_props.hip)
StreamScratch& assembly_scratch();
StreamScratch& property_scratch();

}  // namespace covt

#endif
