// evam_rings.h — host-side bookkeeping of libevam_pp.so's two per-handle descriptor rings, written against
// a small backend interface: evam_pp.hip instantiates it with HIP events, streams and pinned memory, and
// tests/native/ring_check.cpp drives the same code under AddressSanitizer / UBSan with a simulated device
// timeline (every host write into a slot and every copy out of it is checked against the kernels that
// may still read that slot).
//
// Backend B provides (all return 0 or a negative evam_pp status):
//   typename B::Event, typename B::Stream       (value types; a default-constructed Event is "none")
//   event_create(Event*), event_destroy(Event), event_record(Event, Stream), event_sync(Event)
//   stream_create(Stream*), stream_destroy(Stream), stream_wait(Stream, Event), stream_sync(Stream)
//   pinned_alloc(uint8_t** host, const uint8_t** dev, size_t, bool* wc)   (kernels read it in place; wc: the host
//       writes it through a write-combined mapping of device memory: stream whole lines, fence after)
//   pinned_free(uint8_t*, bool wc), host_alloc(uint8_t**, size_t), host_free(uint8_t*)
//   dev_alloc(uint8_t**, size_t), dev_free(uint8_t*), copy_h2d(uint8_t* dst, const uint8_t* src, size_t, Stream)
#ifndef EVAM_RINGS_H
#define EVAM_RINGS_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

namespace evam {

// Per-call ROI records ([RoiRec x n], launch order) change with every detection result. They are written
// into a slot that the ROI kernel reads in place — fine-grained device memory the host writes through its
// BAR mapping where the platform maps it, else pinned, coherent host memory read over PCIe: one pass of
// host stores per call and no copy command. Slots are used in order and fenced in runs of kFence: one
// event, recorded after the call that used the run's last slot, covers the run (an event record per call
// adds a packet the command processor serves between every two ROI launches).
template <class B>
struct PinRingT {
    static constexpr int N = 16;
    static constexpr int kFence = 4;
    uint8_t* host[N] = {};
    const uint8_t* dev[N] = {};  // device address of host[k]
    size_t cap[N] = {};
    bool wc[N] = {};             // host[k] is a write-combined mapping of device memory
    typename B::Event used[N] = {};
    bool used_rec[N] = {};
    int cur = -1;

    // Next slot with at least n bytes. Blocks only while a kernel of up to N calls ago may still read it:
    // the fence of the slot's run was recorded after the run's last call of the previous lap. One wait per run,
    // on entering it: the run's fence is not recorded again before the run's last slot is used, so it still
    // covers the run's other slots (a synchronize per call cost ~1 us of host time even on a passed event).
    int acquire(B& b, size_t n, uint8_t** h, const uint8_t** d, bool* is_wc = nullptr) {
        const int k = (cur + 1) % N;
        const int fk = k | (kFence - 1);
        if (!used[fk]) {
            if (int rc = b.event_create(&used[fk])) return rc;
        }
        if (used_rec[fk] && (k & (kFence - 1)) == 0) {
            if (int rc = b.event_sync(used[fk])) return rc;
        }
        if (cap[k] < n) {
            if (host[k]) {
                if (int rc = b.pinned_free(host[k], wc[k])) return rc;
            }
            host[k] = nullptr;
            dev[k] = nullptr;
            cap[k] = 0;
            wc[k] = false;
            const size_t c = std::max<size_t>(n * 2, 64 * 1024);
            if (int rc = b.pinned_alloc(&host[k], &dev[k], c, &wc[k])) return rc;
            cap[k] = c;
        }
        cur = k;
        *h = host[k];
        *d = dev[k];
        if (is_wc) *is_wc = wc[k];
        return 0;
    }

    // After a call's launches on stream s: the run's fence when the call used the run's last slot.
    int fence(B& b, typename B::Stream s) {
        if (cur < 0 || (cur & (kFence - 1)) != kFence - 1) return 0;
        if (int rc = b.event_record(used[cur], s)) return rc;
        used_rec[cur] = true;
        return 0;
    }

    // A call that failed after acquire() may have launched kernels that read its slot, and (when it held
    // a run's last slot) recorded no fence: drain the stream so no slot is still read, whatever the fences say.
    int abandon(B& b, typename B::Stream s) { return b.stream_sync(s); }

    void release(B& b) {
        for (int k = 0; k < N; k++) {
            if (host[k]) (void)b.pinned_free(host[k], wc[k]);
            if (used[k]) (void)b.event_destroy(used[k]);
            host[k] = nullptr;
            dev[k] = nullptr;
            wc[k] = false;
            used[k] = typename B::Event{};
            used_rec[k] = false;
            cap[k] = 0;
        }
        cur = -1;
    }
};

// The per-call descriptor block ([LUT][ItemDesc x n][tables]) changes with the configuration and geometry
// (not with the frames). It is written into a pinned host slot and copied on a private copy stream into a
// device slot of the same index, so the host never blocks on the copy and the copy of call k+1 can overlap
// the kernel of call k. Slot reuse is fenced by two events: `copied` (the copy out of the host slot
// finished) and `used` (the last kernel that read the device slot finished). A call whose block equals the
// resident one reuses it and records nothing.
template <class B>
struct DescRingT {
    static constexpr int N = 3;
    uint8_t* host[N] = {};
    uint8_t* dev[N] = {};
    size_t cap[N] = {};
    typename B::Event copied[N] = {};
    typename B::Event used[N] = {};
    bool copied_rec[N] = {};
    bool used_rec[N] = {};
    typename B::Stream copy = {};
    bool have_copy = false;
    int cur = -1;
    std::vector<uint8_t> last;  // bytes currently held by dev[cur]

    // Make bytes[0, n) visible to kernels launched next on stream s; *out = its device copy.
    int upload(B& b, typename B::Stream s, const uint8_t* bytes, size_t n, const uint8_t** out) {
        if (cur >= 0 && last.size() == n && memcmp(last.data(), bytes, n) == 0) {
            *out = dev[cur];
            return 0;
        }
        if (!have_copy) {
            if (int rc = b.stream_create(&copy)) return rc;
            have_copy = true;
            for (int k = 0; k < N; k++) {
                if (int rc = b.event_create(&copied[k])) return rc;
                if (int rc = b.event_create(&used[k])) return rc;
            }
        }
        // Fence the slot being retired: every kernel that read it is already on s (a stream switch
        // orders the new stream behind the old one), so one event recorded now covers them all.
        if (cur >= 0) {
            if (int rc = b.event_record(used[cur], s)) return rc;
            used_rec[cur] = true;
        }
        const int k = (cur + 1) % N;
        if (copied_rec[k]) {
            if (int rc = b.event_sync(copied[k])) return rc;  // the host slot is free
        }
        if (cap[k] < n) {
            if (used_rec[k]) {
                if (int rc = b.event_sync(used[k])) return rc;  // the device slot is no longer read
            }
            if (host[k]) {
                if (int rc = b.host_free(host[k])) return rc;
            }
            if (dev[k]) {
                if (int rc = b.dev_free(dev[k])) return rc;
            }
            host[k] = dev[k] = nullptr;
            cap[k] = 0;
            const size_t c = std::max<size_t>(n * 2, 64 * 1024);
            if (int rc = b.host_alloc(&host[k], c)) return rc;
            if (int rc = b.dev_alloc(&dev[k], c)) return rc;
            cap[k] = c;
        }
        memcpy(host[k], bytes, n);
        if (used_rec[k]) {
            if (int rc = b.stream_wait(copy, used[k])) return rc;  // the copy waits for the slot's last reader
        }
        if (int rc = b.copy_h2d(dev[k], host[k], n, copy)) return rc;
        if (int rc = b.event_record(copied[k], copy)) return rc;
        copied_rec[k] = true;
        if (int rc = b.stream_wait(s, copied[k])) return rc;  // kernels on s see the new block
        cur = k;
        last.assign(bytes, bytes + n);
        *out = dev[k];
        return 0;
    }

    void release(B& b) {
        for (int k = 0; k < N; k++) {
            if (host[k]) (void)b.host_free(host[k]);
            if (dev[k]) (void)b.dev_free(dev[k]);
            if (copied[k]) (void)b.event_destroy(copied[k]);
            if (used[k]) (void)b.event_destroy(used[k]);
            host[k] = dev[k] = nullptr;
            copied[k] = used[k] = typename B::Event{};
            copied_rec[k] = used_rec[k] = false;
            cap[k] = 0;
        }
        if (have_copy) (void)b.stream_destroy(copy);
        have_copy = false;
        cur = -1;
        last.clear();
    }
};

}  // namespace evam

#endif  // EVAM_RINGS_H
