// och_group.cpp -- multi-GPU frames from ONE host process:
// a reference host in C++ (ORT/test_och_h_octree.cpp:437-457 renders one
// frame per OnUserUpdate) drives every GPU of the node from one thread.
//
//   * each device holds a replica of the read-only node pool (one H2D upload);
//   * rows are dealt in chunks of row_chunk rows round-robin over the devices
//     (och_shard_rows), each device renders its slice -- raygen, traversal and
//     shading fused, as 1-byte colour codes (or RGBA8 words for palettes of
//     more than OCH_CODE_MAX_VOXELS ids);
//   * one RCCL all-gather over xGMI (ncclCommInitAll over the devices, one
//     ncclAllGather per device inside ncclGroupStart/End) gives every device
//     all slices, and one kernel per device shades + unshards them into the
//     [views][H][W] RGBA8 frames (olc::Pixel layout).
// All work is enqueued asynchronously on the pools' streams; the host thread
// never waits unless it downloads a frame or synchronises.
//
// RCCL is loaded on first use with dlopen (an RCCL already in the process,
// e.g. PyTorch's, is reused), so the library has no link-time dependency on
// it and single-GPU users never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "och_internal.h"

namespace {

struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;
    bool ok = false;
};

const Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);         // already in the process
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            r.error = std::string("cannot load RCCL: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            all &= fn != nullptr;
        };
        sym(r.comm_init_all, "ncclCommInitAll");
        sym(r.comm_destroy, "ncclCommDestroy");
        sym(r.all_gather, "ncclAllGather");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
        if (!all) {
            r.error = "RCCL lacks an nccl* entry point";
            return;
        }
        r.ok = true;
    });
    return r;
}

std::string hip_err(const char *what, hipError_t e) { return std::string(what) + ": " + hipGetErrorString(e); }

}  // namespace

struct och_frame_group {
    int n = 0;
    std::vector<int> devices;
    std::vector<och_gpu_pool *> pools;
    std::vector<ncclComm_t> comms;
    // per device: slice (this device's rows), gathered (all slices), frames
    std::vector<void *> slice, gathered;
    std::vector<uint32_t *> frames;
    size_t slice_bytes = 0, frame_bytes = 0;
    int width = 0, height = 0, n_views = 0, row_chunk = 0;
    bool rendered = false;
    bool codes = true;       // exchange format of the last render
};

namespace {

int group_fail(int status, const std::string &msg) { return och::report(status, msg.c_str()); }

void free_buffers(och_frame_group *g)
{
    for (int r = 0; r < g->n; ++r) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(g->devices[r]);
        if (r < (int)g->slice.size() && g->slice[r]) (void)hipFree(g->slice[r]);
        if (r < (int)g->gathered.size() && g->gathered[r]) (void)hipFree(g->gathered[r]);
        if (r < (int)g->frames.size() && g->frames[r]) (void)hipFree(g->frames[r]);
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    g->slice.assign(g->n, nullptr);
    g->gathered.assign(g->n, nullptr);
    g->frames.assign(g->n, nullptr);
    g->slice_bytes = g->frame_bytes = 0;
}

// Buffers for n_views frames of W x H, slices of rows x W in `elem`-byte pixels.
int ensure_buffers(och_frame_group *g, int W, int H, int n_views, int row_chunk, size_t elem)
{
    int slice_rows = 0;
    if (och_gpu_slice_rows(g->pools[0], H, row_chunk, g->n, &slice_rows) != OCH_OK) return OCH_E_INVALID;
    const size_t rows = (size_t)slice_rows;
    const size_t slice = (size_t)n_views * rows * W * elem;
    const size_t frame = (size_t)n_views * H * W * 4;
    if (slice <= g->slice_bytes && frame <= g->frame_bytes) return OCH_OK;
    for (int r = 0; r < g->n; ++r) (void)och_gpu_synchronize(g->pools[r]);
    free_buffers(g);
    int prev = -1;
    (void)hipGetDevice(&prev);
    int st = OCH_OK;
    for (int r = 0; r < g->n && st == OCH_OK; ++r) {
        hipError_t e = hipSetDevice(g->devices[r]);
        if (e == hipSuccess) e = hipMalloc(&g->slice[r], slice);
        if (e == hipSuccess) e = hipMalloc(&g->gathered[r], slice * g->n);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&g->frames[r]), frame);
        if (e != hipSuccess) st = group_fail(OCH_E_NOMEM, hip_err("frame group buffers", e));
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    if (st != OCH_OK) {
        free_buffers(g);
        return st;
    }
    g->slice_bytes = slice;
    g->frame_bytes = frame;
    return OCH_OK;
}

}  // namespace

extern "C" {

OCH_API int och_frame_group_create(const int *devices, int n_devices, const uint32_t *nodes, uint32_t n_nodes,
                                   uint32_t root, int depth, int index_base, float miss_t, och_frame_group **out)
{
    if (!out || !nodes || n_devices < 1 || n_devices > 64) return group_fail(OCH_E_INVALID, "bad frame group arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return group_fail(OCH_E_NODEV, "no HIP device visible");
    std::vector<int> devs(n_devices);
    if (!devices) {                          // the first n_devices gfx950 devices, in HIP order
        std::vector<int> all(ndev);
        int n950 = 0;
        if (och_device_list(all.data(), ndev, &n950) != OCH_OK || n950 < n_devices)
            return group_fail(OCH_E_NODEV, std::to_string(n_devices) + " gfx950 devices asked, " +
                                               std::to_string(n950) + " visible");
        for (int r = 0; r < n_devices; ++r) devs[r] = all[r];
    }
    for (int r = 0; r < n_devices; ++r) {
        if (devices) devs[r] = devices[r];
        if (devs[r] < 0 || devs[r] >= ndev) return group_fail(OCH_E_NODEV, "device " + std::to_string(devs[r]) + " not visible");
        for (int q = 0; q < r; ++q)
            if (devs[q] == devs[r]) return group_fail(OCH_E_INVALID, "a device appears twice in the group");
    }
    const Rccl &R = rccl();
    if (!R.ok) return group_fail(OCH_E_NODEV, R.error);
    auto *g = new och_frame_group;
    g->n = n_devices;
    g->devices = devs;
    g->pools.assign(n_devices, nullptr);
    g->slice.assign(n_devices, nullptr);
    g->gathered.assign(n_devices, nullptr);
    g->frames.assign(n_devices, nullptr);
    for (int r = 0; r < n_devices; ++r) {
        const int st = och_gpu_pool_create(nodes, n_nodes, root, depth, index_base, miss_t, devs[r], &g->pools[r]);
        if (st != OCH_OK) {
            const std::string msg = och_last_error();
            och_frame_group_destroy(g);
            return group_fail(st, "device " + std::to_string(devs[r]) + ": " + msg);
        }
    }
    g->comms.assign(n_devices, nullptr);
    const ncclResult_t nr = R.comm_init_all(g->comms.data(), n_devices, devs.data());
    if (nr != ncclSuccess) {
        g->comms.clear();
        och_frame_group_destroy(g);
        return group_fail(OCH_E_HIP, std::string("ncclCommInitAll: ") + R.error_string(nr));
    }
    *out = g;
    return OCH_OK;
}

OCH_API int och_frame_group_destroy(och_frame_group *g)
{
    if (!g) return OCH_OK;
    for (och_gpu_pool *p : g->pools)
        if (p) (void)och_gpu_synchronize(p);
    const Rccl &R = rccl();
    for (ncclComm_t c : g->comms)
        if (c && R.ok) (void)R.comm_destroy(c);
    free_buffers(g);
    for (och_gpu_pool *p : g->pools)
        if (p) och_gpu_pool_destroy(p);
    delete g;
    return OCH_OK;
}

OCH_API int och_frame_group_size(const och_frame_group *g, int *n_devices)
{
    if (!g || !n_devices) return group_fail(OCH_E_INVALID, "NULL argument");
    *n_devices = g->n;
    return OCH_OK;
}

OCH_API int och_frame_group_pool(och_frame_group *g, int rank, och_gpu_pool **pool)
{
    if (!g || !pool || rank < 0 || rank >= g->n) return group_fail(OCH_E_INVALID, "bad rank");
    *pool = g->pools[rank];
    return OCH_OK;
}

OCH_API int och_frame_group_set_palette(och_frame_group *g, const uint32_t *rgba, uint32_t n_voxels)
{
    if (!g) return group_fail(OCH_E_INVALID, "NULL group");
    for (och_gpu_pool *p : g->pools) {
        const int st = och_gpu_set_palette(p, rgba, n_voxels);
        if (st != OCH_OK) return st;
    }
    return OCH_OK;
}

OCH_API int och_frame_group_set_option(och_frame_group *g, int option, int value)
{
    if (!g) return group_fail(OCH_E_INVALID, "NULL group");
    for (och_gpu_pool *p : g->pools) {
        const int st = och_gpu_set_option(p, option, value);
        if (st != OCH_OK) return st;
    }
    return OCH_OK;
}

OCH_API int och_frame_group_plan(och_frame_group *g, const och_camera *cams, int n_views, int row_chunk)
{
    if (!g || !cams || row_chunk < 1 || n_views < 1) return group_fail(OCH_E_INVALID, "bad plan arguments");
    if (g->n > 1) {
        // deal the row chunks by their cost in one timed render of these views
        // (device 0), instead of round-robin, so every device gets an equal share
        const int H = cams[0].height, n_chunks = (H + row_chunk - 1) / row_chunk;
        std::vector<float> costs(n_chunks);
        std::vector<int32_t> deal(n_chunks);
        int st = och_gpu_chunk_costs(g->pools[0], cams, n_views, row_chunk, costs.data());
        if (st == OCH_OK) st = och_deal_chunks(costs.data(), n_chunks, g->n, nullptr, deal.data());
        for (int r = 0; r < g->n && st == OCH_OK; ++r)
            st = och_gpu_set_row_deal(g->pools[r], H, row_chunk, g->n, deal.data());
        if (st != OCH_OK) return st;
    }
    for (int r = 0; r < g->n; ++r) {
        int st = och_gpu_plan_views(g->pools[r], cams, n_views, row_chunk, r, g->n);
        if (st == OCH_OK) st = och_gpu_set_option(g->pools[r], OCH_OPT_TILE_ORDER, 2);
        if (st != OCH_OK) return st;
    }
    return OCH_OK;
}

OCH_API int och_frame_group_render(och_frame_group *g, const och_camera *cams, int n_views, int row_chunk, int bounce)
{
    if (!g || !cams || n_views < 1 || n_views > OCH_MAX_VIEWS || row_chunk < 1)
        return group_fail(OCH_E_INVALID, "bad frame group render arguments");
    const int W = cams[0].width, H = cams[0].height;
    // Indexed colour when the palette allows it (a quarter of the RGBA8 bytes on xGMI).
    int n_vox = 0;
    int st = och::pool_palette_size(g->pools[0], &n_vox);
    if (st != OCH_OK) return st;
    const bool codes = n_vox <= OCH_CODE_MAX_VOXELS;
    st = ensure_buffers(g, W, H, n_views, row_chunk, codes ? 1 : 4);
    if (st != OCH_OK) return st;
    int slice_rows = 0;
    st = och_gpu_slice_rows(g->pools[0], H, row_chunk, g->n, &slice_rows);
    if (st != OCH_OK) return st;
    const size_t count = (size_t)n_views * slice_rows * W;
    for (int r = 0; r < g->n && st == OCH_OK; ++r)
        st = codes ? och_gpu_render_codes_views_dev(g->pools[r], cams, n_views, static_cast<uint8_t *>(g->slice[r]),
                                                    row_chunk, r, g->n, bounce)
                   : (bounce ? och_gpu_render_bounce_views_dev(g->pools[r], cams, n_views,
                                                               static_cast<uint32_t *>(g->slice[r]), row_chunk, r, g->n)
                             : och_gpu_render_views_dev(g->pools[r], cams, n_views, static_cast<uint32_t *>(g->slice[r]),
                                                        row_chunk, r, g->n));
    if (st != OCH_OK) return st;
    // The exchange: every device receives every slice, on its pool's stream.
    const Rccl &R = rccl();
    ncclResult_t nr = R.group_start();
    for (int r = 0; r < g->n && nr == ncclSuccess; ++r)
        nr = R.all_gather(g->slice[r], g->gathered[r], count, codes ? ncclUint8 : ncclUint32,
                          g->comms[r], static_cast<hipStream_t>(och::pool_stream(g->pools[r])));
    const ncclResult_t ne = R.group_end();
    if (nr == ncclSuccess) nr = ne;
    if (nr != ncclSuccess) return group_fail(OCH_E_HIP, std::string("ncclAllGather: ") + R.error_string(nr));
    for (int r = 0; r < g->n && st == OCH_OK; ++r)
        st = codes ? och_gpu_shade_unshard_views_dev(g->pools[r], static_cast<const uint8_t *>(g->gathered[r]),
                                                     g->frames[r], W, H, row_chunk, g->n, n_views)
                   : och_gpu_unshard_views_dev(g->pools[r], static_cast<const uint32_t *>(g->gathered[r]), g->frames[r],
                                               W, H, row_chunk, g->n, n_views);
    if (st != OCH_OK) return st;
    g->width = W;
    g->height = H;
    g->n_views = n_views;
    g->row_chunk = row_chunk;
    g->codes = codes;
    g->rendered = true;
    return OCH_OK;
}

OCH_API int och_frame_group_frames_dev(och_frame_group *g, int rank, uint32_t **frames)
{
    if (!g || !frames || rank < 0 || rank >= g->n) return group_fail(OCH_E_INVALID, "bad rank");
    if (!g->rendered) return group_fail(OCH_E_INVALID, "nothing rendered yet");
    *frames = g->frames[rank];
    return OCH_OK;
}

OCH_API int och_frame_group_download(och_frame_group *g, int rank, uint32_t *rgba)
{
    if (!g || !rgba || rank < 0 || rank >= g->n) return group_fail(OCH_E_INVALID, "bad rank");
    if (!g->rendered) return group_fail(OCH_E_INVALID, "nothing rendered yet");
    int prev = -1;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(g->devices[rank]);
    const hipStream_t s = static_cast<hipStream_t>(och::pool_stream(g->pools[rank]));
    const size_t bytes = (size_t)g->n_views * g->height * g->width * 4;
    if (e == hipSuccess) e = hipMemcpyAsync(rgba, g->frames[rank], bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) return group_fail(OCH_E_HIP, hip_err("frame download", e));
    return OCH_OK;
}

OCH_API int och_frame_group_synchronize(och_frame_group *g)
{
    if (!g) return group_fail(OCH_E_INVALID, "NULL group");
    for (och_gpu_pool *p : g->pools) {
        const int st = och_gpu_synchronize(p);
        if (st != OCH_OK) return st;
    }
    return OCH_OK;
}

}  // extern "C"
