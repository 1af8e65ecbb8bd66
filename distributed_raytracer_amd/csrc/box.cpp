// box.cpp — one worker process driving the GPUs of a box behind the BulkTrace contract
// (SURVEY.md §8(b) mirt_create(n_devices), §8(e); include/mirt.h mirt_box_*).
//
// The reference's master cuts every frame into one rectangle per registered worker
// (master/main.go:54-91) and each worker serves its rectangle with a per-pixel loop
// (worker/distributed/main.go:46-91).  A box worker registers ONCE and serves each order on
// all of its GPUs: the rectangle is cut into `strip`-pixel-wide column strips dealt round
// robin (strip k to device k % n), every device traces its strips back to back (each strip
// column-major, so a strip is one contiguous range of the order's i*h + j layout), and the
// strips are assembled on device 0 from the devices' planes — over RCCL send/recv (the
// communicator of ncclCommInitAll over the box's devices: xGMI), or by device copies when
// devices repeat (one GPU standing in for several: the same assembly without RCCL, which
// refuses two ranks on one GPU) — then copied once into the caller's host buffers.  The
// "host" transport instead copies every device's strips straight into a pinned host buffer
// over each device's own PCIe link.  Every transport gives the same bytes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "host_internal.hpp"

using namespace mirt;

namespace {

#define BOX_HIP(expr)                                                                                \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess) return set_error(MIRT_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)
#define BOX_RCCL(expr)                                                                               \
    do {                                                                                             \
        ncclResult_t _r = (expr);                                                                    \
        if (_r != ncclSuccess) return set_error(MIRT_E_DEVICE, std::string(#expr) + ": " + rccl().error_string(_r)); \
    } while (0)

// the output planes of mirt_outputs, in this order, and their bytes per pixel
constexpr int kPlanes = 6;
constexpr size_t kElem[kPlanes] = {24, 3, 1, 4, 4, 4};  // rgb, rgb8, valid, face, object, rgbv

void* host_plane(const mirt_outputs* o, int p) {
    switch (p) {
        case 0: return o->rgb;
        case 1: return o->rgb8;
        case 2: return o->valid;
        case 3: return o->face;
        case 4: return o->object;
        default: return o->rgbv;
    }
}

// Byte offset of plane p in a buffer holding the requested planes of px pixels back to back
// (16-byte aligned starts).
size_t plane_offset(const bool want[kPlanes], uint64_t px, int p) {
    size_t off = 0;
    for (int q = 0; q < p; ++q)
        if (want[q]) off += (px * kElem[q] + 15) & ~(size_t)15;
    return off;
}

OutPlanes planes_at(uint8_t* base, const bool want[kPlanes], uint64_t px) {
    uint8_t* p[kPlanes];
    for (int q = 0; q < kPlanes; ++q) p[q] = want[q] ? base + plane_offset(want, px, q) : nullptr;
    return OutPlanes{(double*)p[0], p[1], p[2], (int32_t*)p[3], (int32_t*)p[4], (uint32_t*)p[5]};
}

template <class T>
int grow_on(int dev, T*& p, size_t& cap, size_t need, bool pinned = false) {
    if (need <= cap) return MIRT_OK;
    BOX_HIP(hipSetDevice(dev));
    if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
    p = nullptr;
    cap = 0;
    const size_t n = std::max<size_t>(need, 256);
    hipError_t e = pinned ? hipHostMalloc((void**)&p, n) : hipMalloc((void**)&p, n);
    if (e != hipSuccess) return set_error(MIRT_E_NOMEM, std::string("box allocation: ") + hipGetErrorString(e));
    cap = n;
    return MIRT_OK;
}

// The workspace of one in-flight order (orders are served concurrently: gRPC runs each
// BulkTrace in its own goroutine).
struct BoxCall {
    std::vector<hipStream_t> s;    // per entry, on its device
    std::vector<hipEvent_t> ev;    // per entry: its trace (and summary copy) enqueued
    std::vector<uint8_t*> buf;     // per entry, on its device: the planes of its strips
    std::vector<size_t> buf_cap;
    uint8_t* recv = nullptr;       // device 0: the other entries' planes back to back
    size_t recv_cap = 0;
    uint8_t* tile = nullptr;       // device 0: the assembled order, i*h + j per plane
    size_t tile_cap = 0;
    uint8_t* host = nullptr;       // pinned: the assembled order (host transport)
    size_t host_cap = 0;
    cnt_t* sum = nullptr;          // pinned: kStatN statistics per entry
};

}  // namespace

// MIRT_BOX_TIMERS=1: host time per phase of the box's orders, summed over calls and printed by
// mirt_box_destroy (diagnostic).
struct BoxTimers {
    bool on = false;
    std::atomic<uint64_t> ns[6] = {};  // hit rect, enqueue, host fill + GPU wait, host fill + copy, whole call, calls
};
inline uint64_t box_now() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct mirt_box {
    BoxTimers tm;
    std::vector<int> dev;              // per entry
    std::vector<mirt_ctx*> ctx;        // per entry
    std::vector<ncclComm_t> comm;      // per entry (RCCL transport)
    int transport = MIRT_BOX_RCCL;
    uint32_t strip = 8;
    std::mutex mu;                     // the call pool and the settings
    std::mutex rccl_mu;                // the order of RCCL groups on the comms (issue only)
    std::vector<std::unique_ptr<BoxCall>> calls;
    std::vector<BoxCall*> free_calls;
};

namespace {

void call_free(mirt_box* b, BoxCall* k) {
    for (size_t d = 0; d < k->s.size(); ++d) {
        (void)hipSetDevice(b->dev[d]);
        if (k->s[d]) (void)hipStreamSynchronize(k->s[d]);
        if (k->buf[d]) (void)hipFree(k->buf[d]);
        if (k->ev[d]) (void)hipEventDestroy(k->ev[d]);
        if (k->s[d]) (void)hipStreamDestroy(k->s[d]);
    }
    (void)hipSetDevice(b->dev[0]);
    if (k->recv) (void)hipFree(k->recv);
    if (k->tile) (void)hipFree(k->tile);
    if (k->host) (void)hipHostFree(k->host);
    if (k->sum) (void)hipHostFree(k->sum);
}

// A free workspace, or a new one (a workspace whose set-up failed stays out of the pool; the
// box frees it at destroy).
int call_acquire(mirt_box* b, BoxCall*& out) {
    out = nullptr;
    BoxCall* k = nullptr;
    {
        std::lock_guard<std::mutex> g(b->mu);
        if (!b->free_calls.empty()) {
            out = b->free_calls.back();
            b->free_calls.pop_back();
            return MIRT_OK;
        }
        b->calls.emplace_back(new BoxCall());
        k = b->calls.back().get();
    }
    const size_t n = b->dev.size();
    k->s.assign(n, nullptr);
    k->ev.assign(n, nullptr);
    k->buf.assign(n, nullptr);
    k->buf_cap.assign(n, 0);
    for (size_t d = 0; d < n; ++d) {
        BOX_HIP(hipSetDevice(b->dev[d]));
        BOX_HIP(hipStreamCreateWithFlags(&k->s[d], hipStreamNonBlocking));
        BOX_HIP(hipEventCreateWithFlags(&k->ev[d], hipEventDisableTiming));
    }
    BOX_HIP(hipSetDevice(b->dev[0]));
    BOX_HIP(hipHostMalloc((void**)&k->sum, n * kStatN * sizeof(cnt_t)));
    out = k;
    return MIRT_OK;
}

void call_release(mirt_box* b, BoxCall* k) {
    std::lock_guard<std::mutex> g(b->mu);
    b->free_calls.push_back(k);
}

// Every stream of the call is idle (an error path leaves nothing running on its buffers).
void call_drain(mirt_box* b, BoxCall* k) {
    for (size_t d = 0; d < k->s.size(); ++d) {
        (void)hipSetDevice(b->dev[d]);
        if (k->s[d]) (void)hipStreamSynchronize(k->s[d]);
    }
}

// The strips of entry d among `active` entries: strip k = d, d + active, ...
struct Deal {
    uint32_t sw = 8, nst = 0, active = 0;
    uint32_t strips_of(uint32_t d) const { return d < active ? (nst - d + active - 1) / active : 0; }
};

// Miss value of plane p, byte-wise (tracer.go:88-90: colour zero and Trace false; face and
// object -1, i.e. 0xff bytes).
uint8_t miss_byte(int p) { return (p == 3 || p == 4) ? 0xff : 0; }

// The order's planes in the caller's buffers, in two steps.  fill_misses: every pixel outside I
// (the order's part of the frame's hit rectangle) gets its miss value — no GPU work or transfer
// for them, their rays cannot meet the object; it needs no GPU result, so it runs while the GPU
// traces I.  copy_hits: I's pixels from the pinned staging buffer, which holds I's planes
// column-major over I's height, once they are there.
void fill_misses(const bool want[kPlanes], const mirt_outputs* hout, uint32_t x, uint32_t y, uint32_t w, uint32_t h,
                 const uint32_t I[4]) {
    const bool empty = I[2] <= I[0] || I[3] <= I[1];
    for (int p = 0; p < kPlanes; ++p) {
        if (!want[p]) continue;
        const size_t e = kElem[p], col = (size_t)h * e;
        uint8_t* dst = (uint8_t*)host_plane(hout, p);
        const uint8_t mb = miss_byte(p);
        if (empty) {
            memset(dst, mb, (size_t)w * col);
            continue;
        }
        const uint32_t c0 = I[0] - x, c1 = I[2] - x, r0 = I[1] - y, r1 = I[3] - y;
        memset(dst, mb, (size_t)c0 * col);
        for (uint32_t c = c0; c < c1; ++c) {
            uint8_t* d = dst + (size_t)c * col;
            memset(d, mb, (size_t)r0 * e);
            memset(d + (size_t)r1 * e, mb, (size_t)(h - r1) * e);
        }
        memset(dst + (size_t)c1 * col, mb, (size_t)(w - c1) * col);
    }
}
void copy_hits(const bool want[kPlanes], const mirt_outputs* hout, const uint8_t* stage, uint32_t x, uint32_t y,
               uint32_t h, const uint32_t I[4]) {
    const uint32_t iw = I[2] - I[0], ih = I[3] - I[1];
    const uint64_t ipx = (uint64_t)iw * ih;
    if (ipx == 0) return;
    for (int p = 0; p < kPlanes; ++p) {
        if (!want[p]) continue;
        const size_t e = kElem[p], col = (size_t)h * e;
        uint8_t* dst = (uint8_t*)host_plane(hout, p);
        const uint8_t* src = stage + plane_offset(want, ipx, p);
        const uint32_t c0 = I[0] - x, r0 = I[1] - y;
        for (uint32_t c = 0; c < iw; ++c)
            memcpy(dst + (size_t)(c0 + c) * col + (size_t)r0 * e, src + (size_t)c * ih * e, (size_t)ih * e);
    }
}

// Trace the rectangle (x, y, w, h) of frame f on the box's entries and land its requested
// planes (column-major over h, back to back at plane_offset) in the call's pinned staging
// buffer k->host; returns once they are there.  One entry traces the rectangle as one tile;
// several deal it in `strip`-px column strips (strip s to entry s % active) and the strips are
// assembled on device 0 (RCCL send/recv or device copies) or copied by every entry straight
// into the staging buffer (host transport).
template <class HostWork>
int box_trace_rect(mirt_box* b, const mirt_frame* f, uint32_t x, uint32_t y, uint32_t w, uint32_t h, uint32_t W,
                   uint32_t H, const bool want[kPlanes], const volatile int* cancel, BoxCall* k, uint32_t& active_out,
                   HostWork&& while_tracing) {
    Deal dl;
    int tr;
    {
        std::lock_guard<std::mutex> g(b->mu);
        tr = b->transport;
        dl.sw = b->strip;
    }
    dl.nst = (w + dl.sw - 1) / dl.sw;
    dl.active = std::min<uint32_t>((uint32_t)b->dev.size(), dl.nst);
    active_out = dl.active;
    const uint64_t npx = (uint64_t)w * h;
    const size_t total = plane_offset(want, npx, kPlanes);
    const int dev0 = b->dev[0];
    int r;
    if ((r = grow_on(dev0, k->host, k->host_cap, std::max<size_t>(total, 16), true)) != MIRT_OK) return r;
    const uint64_t te0 = b->tm.on ? box_now() : 0;
    if (dl.active == 1) {
        // one entry: the rectangle is one tile, already the order's i*h + j layout
        if ((r = grow_on(dev0, k->buf[0], k->buf_cap[0], std::max<size_t>(total, 16))) != MIRT_OK) return r;
        const mirt_tile t{x, y, w, h};
        uint64_t pixels = 0;
        if ((r = trace_tiles_enqueue(b->ctx[0], f, W, H, &t, 1, planes_at(k->buf[0], want, npx), k->s[0], cancel,
                                     k->sum, &pixels)) != MIRT_OK)
            return r;
        BOX_HIP(hipSetDevice(dev0));
        BOX_HIP(hipMemcpyAsync(k->host, k->buf[0], total, hipMemcpyDeviceToHost, k->s[0]));
        const uint64_t te1 = b->tm.on ? box_now() : 0;
        while_tracing();
        BOX_HIP(hipStreamSynchronize(k->s[0]));
        if (b->tm.on) {
            b->tm.ns[1] += te1 - te0;
            b->tm.ns[2] += box_now() - te1;
        }
        return MIRT_OK;
    }
    std::vector<uint64_t> px(dl.active), roff(dl.active, 0);
    std::vector<size_t> bytes(dl.active);
    uint64_t rtotal = 0;
    for (uint32_t d = 0; d < dl.active; ++d) {
        px[d] = 0;
        for (uint32_t s = d; s < dl.nst; s += dl.active) px[d] += (uint64_t)std::min(dl.sw, w - s * dl.sw) * h;
        bytes[d] = plane_offset(want, px[d], kPlanes);
        if (d > 0) {
            roff[d] = rtotal;
            rtotal += bytes[d];
        }
    }
    // 1. every entry traces its strips (each strip column-major, back to back)
    std::vector<mirt_tile> tiles;
    for (uint32_t d = 0; d < dl.active; ++d) {
        if ((r = grow_on(b->dev[d], k->buf[d], k->buf_cap[d], std::max<size_t>(bytes[d], 16))) != MIRT_OK) return r;
        tiles.clear();
        for (uint32_t s = d; s < dl.nst; s += dl.active)
            tiles.push_back(mirt_tile{x + s * dl.sw, y, std::min(dl.sw, w - s * dl.sw), h});
        uint64_t pixels = 0;
        if ((r = trace_tiles_enqueue(b->ctx[d], f, W, H, tiles.data(), (uint32_t)tiles.size(),
                                     planes_at(k->buf[d], want, px[d]), k->s[d], cancel, k->sum + (size_t)d * kStatN,
                                     &pixels)) != MIRT_OK)
            return r;
        BOX_HIP(hipEventRecord(k->ev[d], k->s[d]));
    }
    if (cancel && *cancel) return set_error(MIRT_E_CANCELLED, "cancelled");
    // 2. the strips into the staging buffer in the order's layout
    auto place = [&](uint32_t d, const uint8_t* src, uint8_t* base, hipMemcpyKind kind, hipStream_t s) -> int {
        const uint32_t m = dl.strips_of(d);
        const bool last_partial = (w % dl.sw) != 0 && (dl.nst - 1) % dl.active == d;
        const uint32_t full = last_partial ? m - 1 : m;
        for (int p = 0; p < kPlanes; ++p) {
            if (!want[p]) continue;
            const size_t e = kElem[p], col = (size_t)dl.sw * h * e;
            const uint8_t* sp = src + plane_offset(want, px[d], p);
            uint8_t* dp = base + plane_offset(want, npx, p);
            if (full) BOX_HIP(hipMemcpy2DAsync(dp + d * col, (size_t)dl.active * col, sp, col, col, full, kind, s));
            if (last_partial) {
                const size_t sl = dl.nst - 1;
                BOX_HIP(hipMemcpyAsync(dp + sl * col, sp + (size_t)full * col, (size_t)(w - sl * dl.sw) * h * e, kind, s));
            }
        }
        return MIRT_OK;
    };
    if (tr != MIRT_BOX_HOST) {
        if ((r = grow_on(dev0, k->recv, k->recv_cap, std::max<uint64_t>(rtotal, 16))) != MIRT_OK) return r;
        if ((r = grow_on(dev0, k->tile, k->tile_cap, std::max<size_t>(total, 16))) != MIRT_OK) return r;
        if (tr == MIRT_BOX_RCCL) {
            const Rccl& R = rccl();
            // every comm sees the groups in one order; the lock covers the issue only (the
            // group runs asynchronously on the call's streams)
            std::lock_guard<std::mutex> g(b->rccl_mu);
            BOX_RCCL(R.group_start());
            ncclResult_t rr = ncclSuccess;
            for (uint32_t d = 1; d < dl.active && rr == ncclSuccess; ++d) {
                rr = R.send(k->buf[d], bytes[d], ncclUint8, 0, b->comm[d], k->s[d]);
                if (rr == ncclSuccess) rr = R.recv(k->recv + roff[d], bytes[d], ncclUint8, (int)d, b->comm[0], k->s[0]);
            }
            const ncclResult_t re = R.group_end();  // always closed, also after a failed send/recv
            if (rr == ncclSuccess) rr = re;
            if (rr != ncclSuccess) return set_error(MIRT_E_DEVICE, std::string("box RCCL gather: ") + R.error_string(rr));
        } else {
            BOX_HIP(hipSetDevice(dev0));
            for (uint32_t d = 1; d < dl.active; ++d) {
                BOX_HIP(hipStreamWaitEvent(k->s[0], k->ev[d], 0));
                BOX_HIP(hipMemcpyPeerAsync(k->recv + roff[d], dev0, k->buf[d], b->dev[d], bytes[d], k->s[0]));
            }
        }
        BOX_HIP(hipSetDevice(dev0));
        for (uint32_t d = 0; d < dl.active; ++d)
            if ((r = place(d, d == 0 ? k->buf[0] : k->recv + roff[d], k->tile, hipMemcpyDeviceToDevice, k->s[0])) !=
                MIRT_OK)
                return r;
        BOX_HIP(hipMemcpyAsync(k->host, k->tile, total, hipMemcpyDeviceToHost, k->s[0]));
    } else {
        // host transport: each entry's strips over its own link into the pinned staging buffer
        for (uint32_t d = 0; d < dl.active; ++d) {
            BOX_HIP(hipSetDevice(b->dev[d]));
            if ((r = place(d, k->buf[d], k->host, hipMemcpyDeviceToHost, k->s[d])) != MIRT_OK) return r;
        }
    }
    const uint64_t te1 = b->tm.on ? box_now() : 0;
    while_tracing();
    for (uint32_t d = 0; d < dl.active; ++d) {
        BOX_HIP(hipSetDevice(b->dev[d]));
        BOX_HIP(hipStreamSynchronize(k->s[d]));
    }
    if (b->tm.on) {
        b->tm.ns[1] += te1 - te0;
        b->tm.ns[2] += box_now() - te1;
    }
    return MIRT_OK;
}

// One order: only its part inside the frame's hit rectangle is traced and crosses PCIe; the
// rest of the caller's planes is filled with miss values on the host.
int box_trace(mirt_box* b, const mirt_frame* f, uint32_t x, uint32_t y, uint32_t w, uint32_t h, uint32_t W, uint32_t H,
              const mirt_outputs* hout, const volatile int* cancel, mirt_stats* st, BoxCall* k) {
    bool want[kPlanes];
    for (int p = 0; p < kPlanes; ++p) want[p] = host_plane(hout, p) != nullptr;
    const uint64_t t0 = b->tm.on ? box_now() : 0;
    uint32_t R[4];
    int r = frame_hit_rect(b->ctx[0], f, W, H, R);
    if (r != MIRT_OK) return r;
    if (b->tm.on) b->tm.ns[0] += box_now() - t0;
    uint32_t I[4] = {std::max(x, R[0]), std::max(y, R[1]), std::min(x + w, R[2]), std::min(y + h, R[3])};
    if (I[0] >= I[2] || I[1] >= I[3]) I[0] = I[2] = x, I[1] = I[3] = y;  // no pixel of the order can hit
    uint32_t active = 0;
    // the misses are written while the GPU traces I (the wait below then overlaps that host work)
    uint64_t fill_ns = 0;
    auto fill = [&] {
        const uint64_t tf = b->tm.on ? box_now() : 0;
        fill_misses(want, hout, x, y, w, h, I);
        if (b->tm.on) fill_ns = box_now() - tf;
    };
    if (I[2] > I[0]) {
        r = box_trace_rect(b, f, I[0], I[1], I[2] - I[0], I[3] - I[1], W, H, want, cancel, k, active, fill);
        if (r != MIRT_OK) return r;
    } else {
        fill();
    }
    if (cancel && *cancel) return set_error(MIRT_E_CANCELLED, "cancelled");
    const uint64_t tx = b->tm.on ? box_now() : 0;
    copy_hits(want, hout, k->host, x, y, h, I);
    if (b->tm.on) {
        const uint64_t t1 = box_now();
        b->tm.ns[3] += t1 - tx + fill_ns;
        b->tm.ns[4] += t1 - t0;
        b->tm.ns[5] += 1;
    }
    if (st) {
        memset(st, 0, sizeof(*st));
        st->primary_rays = (uint64_t)w * h;
        for (uint32_t d = 0; d < active; ++d) {
            const cnt_t* s = k->sum + (size_t)d * kStatN;
            st->hits += s[kStatHits];
            st->shadow_rays += s[kStatShadowRays];
            st->tri_tests += s[kStatPrimTests] + s[kStatShadowTests];
            st->reflection_rays += s[kStatReflRays];
        }
    }
    return MIRT_OK;
}

}  // namespace

extern "C" {

int mirt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void mirt_box_destroy(mirt_box* b) {
    if (!b) return;
    if (b->tm.on && b->tm.ns[5]) {
        const double n = (double)b->tm.ns[5];
        fprintf(stderr, "box_timers_us_per_order hit_rect %.2f enqueue %.2f fill_and_wait %.2f fill_and_copy %.2f call %.2f (%llu orders)\n",
                b->tm.ns[0] / n / 1e3, b->tm.ns[1] / n / 1e3, b->tm.ns[2] / n / 1e3, b->tm.ns[3] / n / 1e3,
                b->tm.ns[4] / n / 1e3, (unsigned long long)b->tm.ns[5]);
    }
    for (auto& k : b->calls) call_free(b, k.get());
    if (!b->comm.empty() && rccl().ok)
        for (ncclComm_t c : b->comm)
            if (c) (void)rccl().comm_destroy(c);
    for (mirt_ctx* c : b->ctx) mirt_destroy(c);
    delete b;
}

int mirt_box_create(const int* devices, uint32_t n, mirt_box** out) {
    if (!out) return set_error(MIRT_E_INVALID, "out is NULL");
    *out = nullptr;
    if (n < 1 || n > 64) return set_error(MIRT_E_INVALID, "a box drives 1..64 device entries");
    std::unique_ptr<mirt_box, void (*)(mirt_box*)> b(new mirt_box(), mirt_box_destroy);
    {
        const char* e = getenv("MIRT_BOX_TIMERS");
        b->tm.on = e && *e && strcmp(e, "0") != 0;
    }
    const int count = mirt_device_count();
    for (uint32_t i = 0; i < n; ++i) {
        const int d = devices ? devices[i] : (int)i;
        if (d < 0 || d >= count) return set_error(MIRT_E_INVALID, "no HIP device " + std::to_string(d));
        b->dev.push_back(d);
    }
    for (uint32_t i = 0; i < n; ++i) {
        mirt_ctx* c = nullptr;
        int r = mirt_create(b->dev[i], &c);
        if (r != MIRT_OK) return r;
        b->ctx.push_back(c);
    }
    std::vector<int> sorted(b->dev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    b->transport = (n > 1 && distinct) ? MIRT_BOX_RCCL : MIRT_BOX_COPY;
    if (b->transport == MIRT_BOX_RCCL) {
        const Rccl& R = rccl();
        if (!R.ok || !R.comm_init_all) {
            b->transport = MIRT_BOX_COPY;  // device copies give the same bytes without RCCL
        } else {
            b->comm.assign(n, nullptr);
            BOX_RCCL(R.comm_init_all(b->comm.data(), (int)n, b->dev.data()));
        }
    }
    *out = b.release();
    return MIRT_OK;
}

int mirt_box_size(const mirt_box* b) { return b ? (int)b->dev.size() : 0; }

mirt_ctx* mirt_box_ctx(mirt_box* b, uint32_t i) { return b && i < b->ctx.size() ? b->ctx[i] : nullptr; }

int mirt_box_set_transport(mirt_box* b, int transport) {
    if (!b) return set_error(MIRT_E_INVALID, "NULL box");
    if (transport != MIRT_BOX_RCCL && transport != MIRT_BOX_COPY && transport != MIRT_BOX_HOST)
        return set_error(MIRT_E_INVALID, "transport must be MIRT_BOX_RCCL, MIRT_BOX_COPY or MIRT_BOX_HOST");
    if (transport == MIRT_BOX_RCCL && b->dev.size() > 1 && b->comm.empty())
        return set_error(MIRT_E_INVALID, "no RCCL communicator (devices repeat, or librccl lacks ncclCommInitAll)");
    std::lock_guard<std::mutex> g(b->mu);
    b->transport = transport;
    return MIRT_OK;
}

int mirt_box_transport(const mirt_box* b) { return b ? b->transport : -1; }

int mirt_box_set_strip(mirt_box* b, uint32_t strip) {
    if (!b) return set_error(MIRT_E_INVALID, "NULL box");
    if (strip < 1 || strip > 4096) return set_error(MIRT_E_INVALID, "strip width must be 1..4096 pixels");
    std::lock_guard<std::mutex> g(b->mu);
    b->strip = strip;
    return MIRT_OK;
}

int mirt_box_set_options(mirt_box* b, uint32_t flags) {
    if (!b) return set_error(MIRT_E_INVALID, "NULL box");
    for (mirt_ctx* c : b->ctx) {
        int r = mirt_set_options(c, flags);
        if (r != MIRT_OK) return r;
    }
    return MIRT_OK;
}

int mirt_box_mesh_upload(mirt_box* b, const double* v, uint32_t nv, const double* vn, uint32_t nn, const uint32_t* fv,
                         const uint32_t* fn, const uint32_t* fmat, uint32_t nf, const mirt_material* mats, uint32_t nm,
                         uint32_t* mesh_id) {
    if (!b || !mesh_id) return set_error(MIRT_E_INVALID, "NULL box or mesh_id");
    uint32_t id0 = 0;
    for (size_t i = 0; i < b->ctx.size(); ++i) {
        uint32_t id = 0;
        int r = mirt_mesh_upload(b->ctx[i], v, nv, vn, nn, fv, fn, fmat, nf, mats, nm, &id);
        if (r == MIRT_OK && i > 0 && id != id0) {
            (void)mirt_mesh_release(b->ctx[i], id);
            r = set_error(MIRT_E_INVALID, "the box's devices disagree on the mesh id (meshes uploaded outside the box?)");
        }
        if (r != MIRT_OK) {
            for (size_t j = 0; j < i; ++j) (void)mirt_mesh_release(b->ctx[j], id0);
            return r;
        }
        if (i == 0) id0 = id;
    }
    *mesh_id = id0;
    return MIRT_OK;
}

int mirt_box_mesh_release(mirt_box* b, uint32_t mesh_id) {
    if (!b) return set_error(MIRT_E_INVALID, "NULL box");
    int rc = MIRT_OK;
    for (mirt_ctx* c : b->ctx) {
        int r = mirt_mesh_release(c, mesh_id);
        if (r != MIRT_OK) rc = r;
    }
    return rc;
}

int mirt_box_trace_tile(mirt_box* b, const mirt_frame* f, uint32_t x, uint32_t y, uint32_t w, uint32_t h, uint32_t W,
                        uint32_t H, const mirt_outputs* hout, const volatile int* cancel, mirt_stats* st) {
    if (!b || !hout || !f) return set_error(MIRT_E_INVALID, "NULL box, frame or outputs");
    if (!w || !h || (uint64_t)x + w > W || (uint64_t)y + h > H)
        return set_error(MIRT_E_INVALID, "the order is empty or exceeds the screen");
    BoxCall* k = nullptr;
    int r = call_acquire(b, k);
    if (r != MIRT_OK) return r;
    r = box_trace(b, f, x, y, w, h, W, H, hout, cancel, st, k);
    if (r != MIRT_OK) call_drain(b, k);  // nothing of this call may still run on its buffers
    call_release(b, k);
    return r;
}

}  // extern "C"
