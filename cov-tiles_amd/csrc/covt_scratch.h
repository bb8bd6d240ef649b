// covt_scratch.h -- per (device, stream) device scratch of the small-batch split passes (geometry assembly,
// property materialization; covt_assemble.hip, covt_props.hip).
//
// Launches on one stream are ordered, so they share one scratch block; the block's look-back records carry
// an epoch that the launch's own prep kernel advances in device memory (so a captured HIP graph replays
// with a fresh epoch every time).  A block is allocated and zeroed on a stream's first use; at most
// kMaxSlots blocks are kept per kind, the least recently used one is freed beyond that (hipFree waits for
// the device), and covt_release_scratch (include/covt.h) frees them on request.
// A block handed out while its stream is capturing a HIP graph is pinned: the graph holds its address, so
// the block is never evicted and covt_release_scratch frees it only when asked to with
// COVT_RELEASE_PINNED (the caller then promises that no graph captured on that stream replays again).
// A block cannot be allocated during a capture (hipMemsetAsync would be captured and re-zero the epoch
// records on every replay): the stream must have run one launch before its capture.
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
        hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cst) != hipSuccess) return nullptr;
        const bool capturing = cst != hipStreamCaptureStatusNone;
        std::lock_guard<std::mutex> g(mu_);
        const auto key = std::make_pair(dev, s);
        auto it = slots_.find(key);
        if (it != slots_.end()) {
            it->second.used = ++clock_;
            it->second.pinned |= capturing;  // a captured graph now points at this block
            return it->second.p;
        }
        if (capturing) return nullptr;  // (see the header comment)
        if (slots_.size() >= kMaxSlots) {  // evict the least recently used unpinned block (if any)
            auto lru = slots_.end();
            for (auto j = slots_.begin(); j != slots_.end(); ++j)
                if (!j->second.pinned && (lru == slots_.end() || j->second.used < lru->second.used)) lru = j;
            if (lru != slots_.end()) {
                free_slot(lru->first.first, lru->second.p);
                slots_.erase(lru);
            }
        }
        void* p = nullptr;
        if (hipMalloc(&p, bytes_) != hipSuccess) return nullptr;
        // zero: epoch 0 is never a launch's, so no record reads as current before it is written.  On `s`
        // itself: a non-blocking stream (PyTorch's) is not ordered after the null stream's hipMemset
        if (hipMemsetAsync(p, 0, bytes_, s) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        slots_[key] = Slot{p, ++clock_, false};
        return p;
    }

    // frees the block of (current device, s), or every block when `all`; pinned blocks only with
    // `pinned_too`; returns the number freed
    int release(hipStream_t s, bool all, bool pinned_too) {
        int dev = 0;
        if (!all && hipGetDevice(&dev) != hipSuccess) return 0;
        std::lock_guard<std::mutex> g(mu_);
        int n = 0;
        for (auto it = slots_.begin(); it != slots_.end();) {
            if ((all || it->first == std::make_pair(dev, s)) && (pinned_too || !it->second.pinned)) {
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
        bool pinned;  // first used or reused under a graph capture
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
