// ring_check.cpp — host-only check of libevam_pp.so's descriptor-ring bookkeeping (csrc/evam_rings.h), built
// and run under AddressSanitizer + UBSan by tests/test_native_asan.py.
//
// The rings run against a simulated device: streams execute enqueued kernels and copies in order on a
// timeline, events carry the time of the work before them, host synchronisation advances the host clock.
// Every host write into a slot, every copy into a device slot and every free is checked against the
// intervals during which enqueued kernels (or copies) read that buffer: a write or free while a reader
// may still run is a violation. The driver issues random calls the way evam_pp_run does — ROI records
// into the pinned ring (run-of-4 fences), descriptor blocks that change now and then and grow past the
// slot capacity, kernels of random length, failed calls (PinRingT::abandon), stream switches. A second
// pass with event waits disabled must report violations (the checker has teeth).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <random>
#include <vector>

#include "../../edge-video-analytics-microservice_amd/csrc/evam_rings.h"

using namespace evam;

static std::mt19937_64 rng(20261017);
static double unif(double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); }
static int uni(int a, int b) { return std::uniform_int_distribution<int>(a, b)(rng); }

struct Sim {
    struct Event { int id = 0; explicit operator bool() const { return id != 0; } };
    using Stream = int;
    double host_t = 0;
    std::map<int, double> tail;    // stream -> time its last enqueued op ends
    std::map<int, double> ev_t;    // event -> time of the work recorded before it
    std::map<const uint8_t*, std::vector<std::pair<double, double>>> readers;  // buffer -> read intervals
    std::map<const uint8_t*, size_t> live;  // allocations
    int next_id = 1, violations = 0;
    bool sabotage = false;  // negative control: event / stream synchronisation does nothing
    double t(Stream s) { return tail.count(s) ? tail[s] : 0.0; }

    void check_free_of_readers(const uint8_t* p, double at, const char* what) {
        for (auto& iv : readers[p])
            if (iv.second > at + 1e-12) {
                if (violations < 5) fprintf(stderr, "violation: %s at t=%.3f while a reader runs [%.3f, %.3f]\n", what, at, iv.first, iv.second);
                violations++;
                break;
            }
    }
    // -- backend interface (evam_rings.h) --
    int event_create(Event* e) { e->id = next_id++; return 0; }
    int event_destroy(Event) { return 0; }
    int event_record(Event e, Stream s) { ev_t[e.id] = std::max(t(s), host_t); return 0; }
    int event_sync(Event e) { if (!sabotage) host_t = std::max(host_t, ev_t[e.id]); return 0; }
    int stream_create(Stream* s) { *s = next_id++; return 0; }
    int stream_destroy(Stream) { return 0; }
    int stream_wait(Stream s, Event e) { if (!sabotage) tail[s] = std::max(t(s), ev_t[e.id]); return 0; }
    int stream_sync(Stream s) { if (!sabotage) host_t = std::max(host_t, t(s)); return 0; }
    int alloc(uint8_t** p, size_t n) {
        *p = static_cast<uint8_t*>(malloc(n));
        if (!*p) return -1;
        live[*p] = n;
        readers[*p].clear();
        return 0;
    }
    int release(uint8_t* p, double at, const char* what) {
        check_free_of_readers(p, at, what);
        live.erase(p);
        readers.erase(p);
        free(p);
        return 0;
    }
    int pinned_alloc(uint8_t** h, const uint8_t** d, size_t n, bool* wc) {
        int rc = alloc(h, n);
        *d = *h;
        *wc = (++pinned_allocs & 1) != 0;  // both slot kinds, alternating
        return rc;
    }
    int pinned_free(uint8_t* h, bool) { return release(h, host_t, "pinned slot freed"); }
    int pinned_allocs = 0;
    int host_alloc(uint8_t** h, size_t n) { return alloc(h, n); }
    int host_free(uint8_t* h) { return release(h, host_t, "host staging slot freed"); }
    int dev_alloc(uint8_t** d, size_t n) { return alloc(d, n); }
    int dev_free(uint8_t* d) { return release(d, host_t, "device slot freed"); }
    int copy_h2d(uint8_t* dst, const uint8_t* src, size_t n, Stream s) {
        const double start = std::max(t(s), host_t), end = start + 0.5 + n * 1e-5;
        check_free_of_readers(dst, start, "device slot overwritten by a copy");
        memcpy(dst, src, n);  // ASan: both slots hold n bytes
        readers[src].push_back({start, end});
        tail[s] = end;
        return 0;
    }
    // -- what evam_pp_run does besides the rings --
    void host_write(uint8_t* p, size_t n, const char* what) {
        check_free_of_readers(p, host_t, what);
        memset(p, uni(0, 255), n);  // ASan: the slot holds n bytes
    }
    void kernel(Stream s, std::vector<const uint8_t*> reads) {
        const double start = std::max(t(s), host_t), end = start + unif(2, 120);
        for (const uint8_t* p : reads) readers[p].push_back({start, end});
        tail[s] = end;
    }
    void prune() {  // forget reads that ended before the host clock (they can no longer conflict)
        for (auto& kv : readers) {
            auto& v = kv.second;
            v.erase(std::remove_if(v.begin(), v.end(), [&](auto& iv) { return iv.second <= host_t; }), v.end());
        }
    }
};

static int run(bool sabotage, int calls, bool abandon = true) {
    Sim sim;
    sim.sabotage = sabotage;
    PinRingT<Sim> pin;
    DescRingT<Sim> desc;
    int stream = 1000;
    std::vector<uint8_t> block(4096);
    size_t roi_bytes = 6400;
    int failed = 0, grown = 0, uploads = 0, switches = 0;
    for (int c = 0; c < calls; c++) {
        sim.host_t += unif(0.3, 4.0);  // host work of a call
        if (uni(0, 99) < 8) {  // a new geometry / configuration: a new block, sometimes past the slot size
            const size_t n = uni(0, 9) == 0 ? block.size() * 2 + uni(0, 4096) : std::max<size_t>(512, block.size() + uni(-1024, 1024));
            block.resize(std::min<size_t>(n, 1 << 20));
            for (auto& x : block) x = (uint8_t)uni(0, 255);
            uploads++;
        }
        if (uni(0, 199) == 0) {  // evam_pp_set_stream: the new stream waits for the old one's work
            Sim::Event e;
            sim.event_create(&e);
            sim.event_record(e, stream);
            const int ns = stream + 1;
            sim.stream_wait(ns, e);
            stream = ns;
            switches++;
        }
        const bool roi = uni(0, 99) < 70;
        uint8_t* hslot = nullptr;
        const uint8_t* dslot = nullptr;
        if (roi) {
            if (uni(0, 499) == 0 && roi_bytes < (256u << 10)) { roi_bytes = roi_bytes * 3 / 2 + 64; grown++; }
            const size_t n = std::max<size_t>(64, roi_bytes - uni(0, 63) * 64);
            if (pin.acquire(sim, n, &hslot, &dslot)) return -1;
            sim.host_write(hslot, n, "pinned ROI records written while a kernel reads them");
        }
        const uint8_t* dblock = nullptr;
        if (desc.upload(sim, stream, block.data(), block.size(), &dblock)) return -1;
        std::vector<const uint8_t*> reads = {dblock};
        if (roi) reads.push_back(dslot);
        const int nk = uni(1, 3);
        const bool fail = roi && uni(0, 99) < 4;
        for (int k = 0; k < nk; k++) {
            sim.kernel(stream, reads);
            if (fail && k == 0) break;  // a later launch of the call failed
        }
        if (roi) {
            if (fail) {  // evam_pp_run's PinGuard (abandon=false: the round-2 code, which recorded nothing)
                if (abandon) pin.abandon(sim, stream);
                failed++;
            }
            else if (pin.fence(sim, stream)) return -1;
        }
        if (uni(0, 99) == 0) sim.stream_sync(stream);  // the caller synchronises now and then
        if (c % 64 == 0) sim.prune();
    }
    sim.stream_sync(stream);  // evam_pp_destroy: drain the launch stream and the copy stream first
    if (desc.have_copy) sim.stream_sync(desc.copy);
    pin.release(sim);
    desc.release(sim);
    printf("%s: %d calls, %d failed calls, %d ROI capacity growths, %d new blocks, %d stream switches, "
           "%d violations\n", sabotage ? "sabotaged waits" : (abandon ? "rings" : "rings, failed calls not drained"), calls, failed, grown, uploads, switches,
           sim.violations);
    return sim.violations;
}

int main() {
    const int v = run(false, 8000);
    const int neg = run(true, 2000);
    // a call that fails after taking a run's last pinned slot records no fence; without the
    // drain the next lap reuses the run's slots while this lap's kernels may still read them
    const int noab = run(false, 8000, false);
    if (noab == 0) {
        printf("FAIL: failed calls left undrained produced no violation: the failure path is not exercised\n");
        return 1;
    }
    if (v != 0) {
        printf("FAIL: %d violations with the rings' own fences\n", v);
        return 1;
    }
    if (neg == 0) {
        printf("FAIL: the negative control (no event waits) found no violation: the checker has no teeth\n");
        return 1;
    }
    printf("all checks passed\n");
    return 0;
}
