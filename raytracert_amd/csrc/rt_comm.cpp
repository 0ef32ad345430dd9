// rt_comm.cpp — the multi-GPU form of the 'r' loop for C/C++ hosts: one process
// (or host thread) per GPU, screen tiles dealt round-robin over the ranks, one RCCL gather of the
// quantised tile shards to rank 0 over xGMI, a device un-permute there. No other collective touches
// the data path, and the bytes equal the one-GPU render's (quantisation is per pixel, main.cpp:117).
//
// RCCL is loaded on first use (dlopen of librccl.so.1, RTLD_LOCAL): a process that never makes a
// communicator never loads it, and a process that already holds one (e.g. PyTorch's) shares it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "rt_internal.h"
#include "rt_kernels.h"

namespace rt {
namespace {

struct Rccl {
    bool loaded = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t *) = nullptr;
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) { r.why = std::string("cannot load librccl.so.1: ") + dlerror(); return; }
        bool ok = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) { ok = false; r.why = std::string("librccl.so.1 lacks ") + name; }
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.comm_init_rank, "ncclCommInitRank");
        sym(r.comm_destroy, "ncclCommDestroy");
        sym(r.comm_abort, "ncclCommAbort");
        sym(r.get_async_error, "ncclCommGetAsyncError");
        sym(r.gather, "ncclGather");   // RCCL's gather (rccl.h); NCCL proper has none
        sym(r.error_string, "ncclGetErrorString");
        r.loaded = ok;
    });
    return r;
}

int rccl_fail(const char *what, ncclResult_t e) {
    return set_error(RT_E_RCCL, std::string(what) + ": " + (rccl().error_string ? rccl().error_string(e) : "error"));
}

#define RT_HIP(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return set_error(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

}  // namespace
}  // namespace rt

struct rt_comm {
    int device = 0, rank = 0, nranks = 1;
    ncclComm_t nccl = nullptr;
    uint8_t *shard = nullptr, *gathered = nullptr;   // device: this rank's tiles; rank 0: all ranks' tiles
    size_t shard_bytes = 0;
    // Pipelined calls (rt_comm_set_pipeline 2): call i renders on rstream[i % 2] into shard i % 2,
    // the gather and the un-permute run on xstream in call order; the caller's stream waits only for
    // its own call's un-permute, so call i+1's render runs while call i's gather and un-permute do
    // (and beside call i's render too when the scene keeps frames in flight, RT_TUNE_FRAMES_IN_FLIGHT).
    int depth = 1, next = 0;
    hipStream_t rstream[2] = {}, xstream = nullptr;
    uint8_t *shard2 = nullptr;
    hipEvent_t rendered[2] = {}, gathered_ev[2] = {}, done = nullptr, entered = nullptr;
    bool pending[2] = {false, false};
};

using namespace rt;

extern "C" {

int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]) {
    try {
        static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES is NCCL_UNIQUE_ID_BYTES");
        if (!id) return set_error(RT_E_ARG, "id is NULL");
        Rccl &r = rccl();
        if (!r.loaded) return set_error(RT_E_RCCL, r.why);
        ncclUniqueId u;
        const ncclResult_t e = r.get_unique_id(&u);
        if (e != ncclSuccess) return rccl_fail("ncclGetUniqueId", e);
        std::memcpy(id, &u, sizeof(u));
        return RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

int rt_comm_init(int32_t device, int32_t rank, int32_t nranks, const uint8_t id[RT_COMM_ID_BYTES], rt_comm **out) {
    try {
        if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return set_error(RT_E_ARG, "invalid communicator arguments");
        *out = nullptr;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return set_error(RT_E_NODEV, "no such HIP device");
        Rccl &r = rccl();
        if (!r.loaded) return set_error(RT_E_RCCL, r.why);
        RT_HIP(hipSetDevice(device));
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        rt_comm *c = new rt_comm();
        c->device = device;
        c->rank = rank;
        c->nranks = nranks;
        const ncclResult_t e = r.comm_init_rank(&c->nccl, nranks, u, rank);   // collective over the nranks ranks
        if (e != ncclSuccess) { delete c; return rccl_fail("ncclCommInitRank", e); }
        *out = c;
        return RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

void rt_comm_destroy(rt_comm *c) {
    try {
        if (!c) return;
        hipSetDevice(c->device);
        hipDeviceSynchronize();
        if (c->nccl) rccl().comm_destroy(c->nccl);
        hipFree(c->shard);
        hipFree(c->shard2);
        hipFree(c->gathered);
        for (int b = 0; b < 2; ++b) {
            if (c->rendered[b]) hipEventDestroy(c->rendered[b]);
            if (c->gathered_ev[b]) hipEventDestroy(c->gathered_ev[b]);
        }
        if (c->done) hipEventDestroy(c->done);
        if (c->entered) hipEventDestroy(c->entered);
        for (int b = 0; b < 2; ++b)
            if (c->rstream[b]) hipStreamDestroy(c->rstream[b]);
        if (c->xstream) hipStreamDestroy(c->xstream);
        delete c;
    } catch (...) {
    }
}

int rt_comm_set_pipeline(rt_comm *c, int32_t depth) {
    try {
        if (!c) return set_error(RT_E_ARG, "comm is NULL");
        if (depth != 1 && depth != 2) return set_error(RT_E_ARG, "pipeline depth must be 1 or 2");
        RT_HIP(hipSetDevice(c->device));
        RT_HIP(hipDeviceSynchronize());   // (no call of the old depth is still in flight)
        if (depth == 2 && !c->xstream) {   // streams and events made here, never inside the frame loop
            for (int b = 0; b < 2; ++b) RT_HIP(hipStreamCreateWithFlags(&c->rstream[b], hipStreamNonBlocking));
            RT_HIP(hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking));
            for (int b = 0; b < 2; ++b) {
                RT_HIP(hipEventCreateWithFlags(&c->rendered[b], hipEventDisableTiming));
                RT_HIP(hipEventCreateWithFlags(&c->gathered_ev[b], hipEventDisableTiming));
            }
            RT_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
            RT_HIP(hipEventCreateWithFlags(&c->entered, hipEventDisableTiming));
        }
        c->depth = depth;
        c->next = 0;
        c->pending[0] = c->pending[1] = false;
        return RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

int rt_comm_info(const rt_comm *c, int32_t *rank, int32_t *nranks, int32_t *device) {
    try {
        if (!c) return set_error(RT_E_ARG, "comm is NULL");
        if (rank) *rank = c->rank;
        if (nranks) *nranks = c->nranks;
        if (device) *device = c->device;
        return RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

int rt_comm_check(rt_comm *c) {
    try {
        if (!c || !c->nccl) return set_error(RT_E_ARG, "comm is NULL");
        ncclResult_t async = ncclSuccess;
        const ncclResult_t e = rccl().get_async_error(c->nccl, &async);
        if (e != ncclSuccess) return rccl_fail("ncclCommGetAsyncError", e);
        if (async != ncclSuccess && async != ncclInProgress) return rccl_fail("communicator asynchronous error", async);
        return RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

int rt_assemble_tiles_device(int32_t device, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h, int32_t frames,
                             int32_t nranks, const void *d_gathered, size_t gathered_bytes, void *d_frames_out,
                             size_t out_capacity, void *stream) {
    try {
        if (width <= 0 || height <= 0 || tile_w <= 0 || tile_h <= 0 || frames < 1 || nranks < 1 || !d_gathered || !d_frames_out)
            return set_error(RT_E_ARG, "invalid assemble arguments");
        const int64_t T = static_cast<int64_t>((width + tile_w - 1) / tile_w) * ((height + tile_h - 1) / tile_h);
        // tile ids g = f * T + t index the kernel's int arithmetic: the bound rt_render_tiles_device keeps
        if (frames * T > (int64_t(1) << 30)) return set_error(RT_E_ARG, "frames x tiles exceeds 2^30");
        const int64_t slots = (frames * T + nranks - 1) / nranks;
        if (static_cast<uint64_t>(nranks) * slots * tile_w * tile_h * 3 > gathered_bytes)
            return set_error(RT_E_ARG, "gathered buffer smaller than nranks x slots tiles");
        if (static_cast<uint64_t>(frames) * width * height * 3 > out_capacity) return set_error(RT_E_ARG, "output buffer too small");
        RT_HIP(hipSetDevice(device));
        launch_assemble_tiles(static_cast<const uint8_t *>(d_gathered), width, height, tile_w, tile_h, frames, nranks,
                              static_cast<uint8_t *>(d_frames_out), static_cast<hipStream_t>(stream));
        RT_HIP(hipGetLastError());
        return RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

int rt_render_frames_sharded(rt_scene *scene, const rt_params *params, rt_comm *c, int32_t tile_w, int32_t tile_h,
                             int32_t frames, void *d_frames_out, size_t out_capacity, void *stream, uint64_t counts[3]) {
    try {
        if (!scene || !params || !c) return set_error(RT_E_ARG, "scene/params/comm is NULL");
        if (scene_device(scene) != c->device) return set_error(RT_E_ARG, "scene and communicator are on different devices");
        if (tile_w <= 0 || tile_h <= 0 || frames < 1 || params->width <= 0 || params->height <= 0)
            return set_error(RT_E_ARG, "invalid tiling");
        if (c->rank == 0 && (!d_frames_out || static_cast<uint64_t>(frames) * params->width * params->height * 3 > out_capacity))
            return set_error(RT_E_ARG, "rank 0 needs an output buffer of frames x height x width x 3 bytes");
        const int64_t T = static_cast<int64_t>((params->width + tile_w - 1) / tile_w) * ((params->height + tile_h - 1) / tile_h);
        const int64_t slots = (frames * T + c->nranks - 1) / c->nranks;
        const size_t shard = static_cast<size_t>(slots) * tile_w * tile_h * 3;
        hipStream_t st = static_cast<hipStream_t>(stream);
        RT_HIP(hipSetDevice(c->device));
        if (shard > c->shard_bytes) {   // equal-sized shards (padded): one gather of fixed counts
            RT_HIP(hipDeviceSynchronize());
            hipFree(c->shard);
            hipFree(c->shard2);
            hipFree(c->gathered);
            c->shard = c->shard2 = c->gathered = nullptr;
            c->shard_bytes = 0;
            RT_HIP(hipMalloc(&c->shard, shard));
            RT_HIP(hipMalloc(&c->shard2, shard));
            if (c->rank == 0) RT_HIP(hipMalloc(&c->gathered, shard * static_cast<size_t>(c->nranks)));
            RT_HIP(hipMemset(c->shard, 0, shard));
            RT_HIP(hipMemset(c->shard2, 0, shard));
            c->shard_bytes = shard;
            c->pending[0] = c->pending[1] = false;
        }
        if (c->depth == 2 && !counts) {
            // render on rstream[b] into shard b once the gather that last read it is done, then
            // gather + un-permute on xstream; the caller's stream waits for this call's un-permute only.
            // The render reads no caller-stream data (the scene and its device arrays are the library's,
            // the parameters travel as kernel arguments), so it does not wait for the caller's stream.
            const int b = c->next;
            c->next ^= 1;
            uint8_t *buf = b ? c->shard2 : c->shard;
            hipStream_t rs = c->rstream[b];
            if (c->pending[b]) RT_HIP(hipStreamWaitEvent(rs, c->gathered_ev[b], 0));
            int32_t n = 0;
            int rc = rt_render_tiles_device(scene, params, tile_w, tile_h, frames, c->rank, c->nranks, buf, c->shard_bytes,
                                            rs, &n, nullptr);
            if (rc) return rc;
            RT_HIP(hipEventRecord(c->rendered[b], rs));
            RT_HIP(hipStreamWaitEvent(c->xstream, c->rendered[b], 0));
            // the caller's earlier work (e.g. on d_frames_out) comes before this call's un-permute writes
            RT_HIP(hipEventRecord(c->entered, st));
            RT_HIP(hipStreamWaitEvent(c->xstream, c->entered, 0));
            const ncclResult_t e = rccl().gather(buf, c->gathered, shard, ncclUint8, 0, c->nccl, c->xstream);
            if (e != ncclSuccess) return rccl_fail("ncclGather", e);
            RT_HIP(hipEventRecord(c->gathered_ev[b], c->xstream));
            c->pending[b] = true;
            if (c->rank == 0) {
                rc = rt_assemble_tiles_device(c->device, params->width, params->height, tile_w, tile_h, frames, c->nranks,
                                              c->gathered, shard * static_cast<size_t>(c->nranks), d_frames_out, out_capacity,
                                              c->xstream);
                if (rc) return rc;
            }
            RT_HIP(hipEventRecord(c->done, c->xstream));
            RT_HIP(hipStreamWaitEvent(st, c->done, 0));
            return RT_OK;
        }
        if (c->depth == 2) {   // a call with counts synchronises anyway: drain the pipeline first
            for (int b = 0; b < 2; ++b) RT_HIP(hipStreamSynchronize(c->rstream[b]));
            RT_HIP(hipStreamSynchronize(c->xstream));
        }
        int32_t n = 0;
        int rc = rt_render_tiles_device(scene, params, tile_w, tile_h, frames, c->rank, c->nranks, c->shard, c->shard_bytes,
                                        stream, &n, counts);
        if (rc) return rc;
        const ncclResult_t e = rccl().gather(c->shard, c->gathered, shard, ncclUint8, 0, c->nccl, st);
        if (e != ncclSuccess) return rccl_fail("ncclGather", e);
        if (c->rank == 0) {
            rc = rt_assemble_tiles_device(c->device, params->width, params->height, tile_w, tile_h, frames, c->nranks, c->gathered,
                                          shard * static_cast<size_t>(c->nranks), d_frames_out, out_capacity, stream);
            if (rc) return rc;
        }
        // (depth 2: the next call renders into a shard and gathers into `gathered` from its own streams,
        // which do not wait for the caller's: this call's gather and un-permute finish first)
        if (c->depth == 2) RT_HIP(hipStreamSynchronize(st));
        return counts ? rt_comm_check(c) : RT_OK;
    } catch (...) {
        return rt::guard_failure();
    }
}

}  // extern "C"
