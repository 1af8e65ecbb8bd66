// host_internal.hpp — host-only internals shared by the translation units of libmirt
// (mirt.cpp: contexts, launches, frame groups; box.cpp: one process driving several GPUs).
// Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>

#include "../../include/mirt.h"
#include "mirt_internal.hpp"

namespace mirt {

// Sets the thread-local mirt_last_error() text; returns code.
int set_error(int code, const std::string& msg);

// RCCL entry points, resolved at first use with dlopen("librccl.so.1") (the copy torch
// loaded, else /opt/rocm's): the library loads without RCCL and single-GPU callers never
// touch it.
struct Rccl {
    bool ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;  // optional (mirt_box: one process, several GPUs)
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;    // optional (peer exclusion)
    decltype(&ncclCommShrink) comm_shrink = nullptr;  // optional (peer exclusion without a new id)
};
const Rccl& rccl();

// Enqueue the trace of a tile list of one frame on stream s of context c (the body of
// mirt_trace_tiles_async) and, after it, a copy of the frame's statistic totals (kStatN
// counters) into h_summary (pinned host memory, read after s has been synchronised).
// *pixels receives the pixel count of the list.
int trace_tiles_enqueue(mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, const mirt_tile* tiles,
                        uint32_t n, const OutPlanes& out, hipStream_t s, const volatile int* cancel,
                        cnt_t* h_summary, uint64_t* pixels);

// The frame's conservative hit rectangle {x0, y0, x1, y1} (half-open) on a W x H screen: every
// pixel outside it misses (mirt.cpp hit_rect; the whole screen without the block pre-test).
int frame_hit_rect(mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, uint32_t out[4]);

}  // namespace mirt
