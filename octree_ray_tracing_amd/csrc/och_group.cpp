// och_group.cpp -- multi-GPU frames from ONE host process:
// a reference host in C++ (ORT/test_och_h_octree.cpp:437-457 renders one
// frame per OnUserUpdate) drives every GPU of the node.
//
//   * each device holds a replica of the read-only node pool (one H2D upload);
//   * rows are dealt in chunks of row_chunk rows over the devices
//     (och_shard_rows, or och_frame_group_plan's cost deal); each device
//     renders its slice -- raygen, traversal and shading fused -- as 1-byte
//     colour codes (or RGBA8 words for palettes of more than
//     OCH_CODE_MAX_VOXELS ids);
//   * one RCCL all-gather over xGMI (ncclCommInitAll over the devices) gives
//     every device all slices, and one kernel per device shades + unshards
//     them into the [views][H][W] RGBA8 frames (olc::Pixel layout).
// Each device has its own issuing thread (one thread per GPU),
// which enqueues its device's render, its ncclAllGather on its own
// communicator and its shade; the calling thread posts the frame to every
// worker and returns once all of them have enqueued it, so the devices'
// launch costs overlap instead of adding up.  Frames rotate over up to
// kMaxSets buffer sets, each with its own stream per device, so several
// frames can be in flight (och_frame_group_render_steps).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "och_internal.h"
#include "och_rccl.h"

namespace {

constexpr int kMaxSets = 8;

std::string hip_err(const char *what, hipError_t e) { return std::string(what) + ": " + hipGetErrorString(e); }

// One host thread bound to one device: runs the jobs posted to it, one at a
// time, and reports each job's status (and its thread-local error text).
class DeviceWorker {
  public:
    explicit DeviceWorker(int device) : device_(device), thread_([this] { loop(); }) {}
    ~DeviceWorker()
    {
        {
            std::lock_guard<std::mutex> l(m_);
            quit_ = true;
        }
        cv_.notify_all();
        thread_.join();
    }
    void post(std::function<int()> job)
    {
        {
            std::lock_guard<std::mutex> l(m_);
            job_ = std::move(job);
            busy_ = true;
        }
        cv_.notify_all();
    }
    // Wait for the posted job; its status, and its error text on failure.
    int wait(std::string &error)
    {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [this] { return !busy_; });
        error = error_;
        return status_;
    }

  private:
    void loop()
    {
        const bool dev_ok = hipSetDevice(device_) == hipSuccess;
        std::unique_lock<std::mutex> l(m_);
        for (;;) {
            cv_.wait(l, [this] { return busy_ || quit_; });
            if (quit_) return;
            std::function<int()> job = std::move(job_);
            l.unlock();
            int st = dev_ok ? job() : och::report(OCH_E_HIP, "worker thread could not select its device");
            std::string err = st == OCH_OK ? std::string() : std::string(och_last_error());
            l.lock();
            status_ = st;
            error_ = std::move(err);
            busy_ = false;
            cv_.notify_all();
        }
    }

    int device_;
    std::mutex m_;
    std::condition_variable cv_;
    std::function<int()> job_;
    bool busy_ = false, quit_ = false;
    int status_ = OCH_OK;
    std::string error_;
    std::thread thread_;   // last: starts after the members it reads
};

}  // namespace

struct och_frame_group {
    int n = 0;
    std::vector<int> devices;
    std::vector<och_gpu_pool *> pools;
    std::vector<ncclComm_t> comms;
    std::vector<std::unique_ptr<DeviceWorker>> workers;
    // per device r, per buffer set b: stream, slice (this device's rows),
    // gathered (all slices), frames
    int n_sets = 0;
    std::vector<std::vector<hipStream_t>> streams;
    std::vector<std::vector<void *>> slice, gathered;
    std::vector<std::vector<uint32_t *>> frames;
    size_t slice_bytes = 0, frame_bytes = 0;
    int width = 0, height = 0, n_views = 0, row_chunk = 0;
    int last_set = 0;        // the buffer set of the last frame
    bool rendered = false;
    bool codes = true;       // exchange format of the last render
    // a device's frame failed after others may have queued their all-gathers:
    // the communicators were aborted and the group refuses further frames
    bool broken = false;
};

namespace {

int group_fail(int status, const std::string &msg) { return och::report(status, msg.c_str()); }

// Run job(r) on every device's worker thread; the first failure is reported
// (with its device) on the calling thread.
int run_on_devices(och_frame_group *g, const std::function<int(int)> &job)
{
    for (int r = 0; r < g->n; ++r) g->workers[r]->post([&job, r] { return job(r); });
    int st = OCH_OK;
    std::string first;
    for (int r = 0; r < g->n; ++r) {
        std::string err;
        const int s = g->workers[r]->wait(err);
        if (s != OCH_OK && st == OCH_OK) {
            st = s;
            first = "device " + std::to_string(g->devices[r]) + ": " + err;
        }
    }
    return st == OCH_OK ? OCH_OK : group_fail(st, first);
}

int sync_all(och_frame_group *g)
{
    for (int r = 0; r < g->n; ++r) {
        if (int st = och_gpu_synchronize(g->pools[r])) return st;
        for (hipStream_t s : g->streams[r]) {
            int prev = -1;
            (void)hipGetDevice(&prev);
            (void)hipSetDevice(g->devices[r]);
            const hipError_t e = hipStreamSynchronize(s);
            if (prev >= 0) (void)hipSetDevice(prev);
            if (e != hipSuccess) return group_fail(OCH_E_HIP, hip_err("frame group synchronize", e));
        }
    }
    return OCH_OK;
}

void free_buffers(och_frame_group *g)
{
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (int r = 0; r < g->n; ++r) {
        (void)hipSetDevice(g->devices[r]);
        for (int b = 0; b < g->n_sets; ++b) {
            if (g->slice[r][b]) (void)hipFree(g->slice[r][b]);
            if (g->gathered[r][b]) (void)hipFree(g->gathered[r][b]);
            if (g->frames[r][b]) (void)hipFree(g->frames[r][b]);
        }
        g->slice[r].assign(g->n_sets, nullptr);
        g->gathered[r].assign(g->n_sets, nullptr);
        g->frames[r].assign(g->n_sets, nullptr);
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    g->slice_bytes = g->frame_bytes = 0;
}

void free_streams(och_frame_group *g)
{
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (int r = 0; r < g->n; ++r) {
        (void)hipSetDevice(g->devices[r]);
        for (hipStream_t s : g->streams[r])
            if (s) (void)hipStreamDestroy(s);
        g->streams[r].clear();
    }
    if (prev >= 0) (void)hipSetDevice(prev);
}

// n_sets buffer sets for n_views frames of W x H, slices of rows x W in
// `elem`-byte pixels, and one stream per set and device.
int ensure_buffers(och_frame_group *g, int W, int H, int n_views, int row_chunk, size_t elem, int n_sets)
{
    int slice_rows = 0;
    if (och_gpu_slice_rows(g->pools[0], H, row_chunk, g->n, &slice_rows) != OCH_OK) return OCH_E_INVALID;
    const size_t slice = (size_t)n_views * (size_t)slice_rows * W * elem;
    const size_t frame = (size_t)n_views * H * W * 4;
    if (n_sets <= g->n_sets && slice <= g->slice_bytes && frame <= g->frame_bytes) return OCH_OK;
    if (int st = sync_all(g)) return st;
    free_buffers(g);
    const int sets = std::max(n_sets, g->n_sets);
    int prev = -1;
    (void)hipGetDevice(&prev);
    int st = OCH_OK;
    for (int r = 0; r < g->n && st == OCH_OK; ++r) {
        hipError_t e = hipSetDevice(g->devices[r]);
        while (e == hipSuccess && (int)g->streams[r].size() < sets) {
            hipStream_t s = nullptr;
            e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            if (e == hipSuccess) g->streams[r].push_back(s);
        }
        g->slice[r].assign(sets, nullptr);
        g->gathered[r].assign(sets, nullptr);
        g->frames[r].assign(sets, nullptr);
        for (int b = 0; b < sets && e == hipSuccess; ++b) {
            e = hipMalloc(&g->slice[r][b], slice);
            if (e == hipSuccess) e = hipMalloc(&g->gathered[r][b], slice * g->n);
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&g->frames[r][b]), frame);
        }
        if (e != hipSuccess) st = group_fail(OCH_E_NOMEM, hip_err("frame group buffers", e));
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    g->n_sets = sets;
    if (st != OCH_OK) {
        free_buffers(g);
        return st;
    }
    g->slice_bytes = slice;
    g->frame_bytes = frame;
    return OCH_OK;
}

// One frame on device r, buffer set b, issued by r's worker: render this
// device's slice, all-gather on r's communicator, shade + unshard -- all on
// set b's stream of device r.
int device_frame(och_frame_group *g, int r, int b, const och_camera *cams, int n_views, int row_chunk, int bounce,
                 bool codes, size_t count)
{
    och_gpu_pool *p = g->pools[r];
    const hipStream_t s = g->streams[r][b];
    const int W = cams[0].width, H = cams[0].height;
    int st = och_gpu_set_stream(p, s);
    if (st != OCH_OK) return st;
    st = codes ? och_gpu_render_codes_views_dev(p, cams, n_views, static_cast<uint8_t *>(g->slice[r][b]), row_chunk,
                                                r, g->n, bounce)
               : (bounce ? och_gpu_render_bounce_views_dev(p, cams, n_views, static_cast<uint32_t *>(g->slice[r][b]),
                                                           row_chunk, r, g->n)
                         : och_gpu_render_views_dev(p, cams, n_views, static_cast<uint32_t *>(g->slice[r][b]),
                                                    row_chunk, r, g->n));
    if (st != OCH_OK) return st;
    // one thread per communicator: no RCCL group call is needed
    const ncclResult_t nr = och::rccl().all_gather(g->slice[r][b], g->gathered[r][b], codes ? count : count * 4,
                                                   ncclUint8, g->comms[r], s);
    if (nr != ncclSuccess)
        return group_fail(OCH_E_HIP, std::string("ncclAllGather: ") + och::rccl().error_string(nr));
    return codes ? och_gpu_shade_unshard_views_dev(p, static_cast<const uint8_t *>(g->gathered[r][b]),
                                                   g->frames[r][b], W, H, row_chunk, g->n, n_views)
                 : och_gpu_unshard_views_dev(p, static_cast<const uint32_t *>(g->gathered[r][b]), g->frames[r][b], W,
                                             H, row_chunk, g->n, n_views);
}

// Abort every device's communicator (ncclCommAbort): after one device's
// frame failed, the others' all-gathers of that frame have no partner and
// would hold their streams forever.
void abort_comms(och_frame_group *g)
{
    const och::Rccl &R = och::rccl();
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (int r = 0; r < (int)g->comms.size(); ++r)
        if (g->comms[r] && R.ok) {
            (void)hipSetDevice(g->devices[r]);
            (void)R.comm_abort(g->comms[r]);
            g->comms[r] = nullptr;
        }
    if (prev >= 0) (void)hipSetDevice(prev);
    g->broken = true;
}

int render_steps(och_frame_group *g, const och_camera *cams, int n_views, int n_steps, int n_sets, int row_chunk,
                 int bounce)
{
    if (!g || !cams || n_views < 1 || n_views > OCH_MAX_VIEWS || row_chunk < 1 || n_steps < 0 || n_sets < 1 ||
        n_sets > kMaxSets)
        return group_fail(OCH_E_INVALID, "bad frame group render arguments");
    if (g->broken) return group_fail(OCH_E_HIP, "frame group unusable after a failed frame (communicators aborted)");
    const int W = cams[0].width, H = cams[0].height;
    for (int v = 0; v < n_views; ++v)
        if (cams[v].width != W || cams[v].height != H || W <= 0 || H <= 0)
            return group_fail(OCH_E_INVALID, "views must share one positive width and height");
    // Indexed colour when the palette allows it (a quarter of the RGBA8 bytes on xGMI).
    int n_vox = 0;
    int st = och::pool_palette_size(g->pools[0], &n_vox);
    if (st != OCH_OK) return st;
    const bool codes = n_vox <= OCH_CODE_MAX_VOXELS;
    st = ensure_buffers(g, W, H, n_views, row_chunk, codes ? 1 : 4, n_sets);
    if (st != OCH_OK) return st;
    int slice_rows = 0;
    st = och_gpu_slice_rows(g->pools[0], H, row_chunk, g->n, &slice_rows);
    if (st != OCH_OK) return st;
    const size_t count = (size_t)n_views * slice_rows * W;
    if (n_steps == 0) return OCH_OK;
    // the shade of every device needs its code table (checked before any frame is queued)
    if (codes)
        for (int r = 0; r < g->n; ++r) {
            int nv = 0;
            if (och::pool_palette_size(g->pools[r], &nv) != OCH_OK || nv < 1)
                return group_fail(OCH_E_INVALID, "device " + std::to_string(g->devices[r]) + " has no palette");
        }
    st = run_on_devices(g, [&](int r) {
        int s = OCH_OK;
        for (int k = 0; k < n_steps && s == OCH_OK; ++k)
            s = device_frame(g, r, k % n_sets, cams, n_views, row_chunk, bounce, codes, count);
        return s;
    });
    if (st != OCH_OK) {
        const std::string msg = och_last_error();
        abort_comms(g);
        return group_fail(st, msg + " (communicators aborted; destroy the group)");
    }
    g->width = W;
    g->height = H;
    g->n_views = n_views;
    g->row_chunk = row_chunk;
    g->codes = codes;
    g->last_set = (n_steps - 1) % n_sets;
    g->rendered = true;
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
    const och::Rccl &R = och::rccl();
    if (!R.ok) return group_fail(OCH_E_NODEV, R.error);
    auto *g = new och_frame_group;
    g->n = n_devices;
    g->devices = devs;
    g->pools.assign(n_devices, nullptr);
    g->slice.assign(n_devices, {});
    g->gathered.assign(n_devices, {});
    g->frames.assign(n_devices, {});
    g->streams.assign(n_devices, {});
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
    for (int r = 0; r < n_devices; ++r) g->workers.emplace_back(new DeviceWorker(devs[r]));
    *out = g;
    return OCH_OK;
}

OCH_API int och_frame_group_destroy(och_frame_group *g)
{
    if (!g) return OCH_OK;
    (void)sync_all(g);
    g->workers.clear();                      // joins the issuing threads
    const och::Rccl &R = och::rccl();
    for (ncclComm_t c : g->comms)
        if (c && R.ok) (void)R.comm_destroy(c);
    // the pools first: each may still point at one of the group's streams
    // (device_frame sets it), which pool destroy synchronises
    for (och_gpu_pool *p : g->pools)
        if (p) och_gpu_pool_destroy(p);
    free_buffers(g);
    free_streams(g);
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
    OCH_ENTRY();
    if (!g || !cams || row_chunk < 1 || n_views < 1) return group_fail(OCH_E_INVALID, "bad plan arguments");
    if (g->broken) return group_fail(OCH_E_HIP, "frame group unusable after a failed frame (communicators aborted)");
    if (int st = sync_all(g)) return st;     // frames in flight may read the deal and the plans
    if (g->n > 1) {
        // deal the row chunks by their cost in one timed render of these views
        // (device 0), instead of round-robin, so every device gets an equal
        // share.  The deal is set on every pool or on none: a group whose
        // pools disagree would unshard slices into the wrong rows.
        const int H = cams[0].height, n_chunks = (H + row_chunk - 1) / row_chunk;
        std::vector<float> costs(n_chunks);
        std::vector<int32_t> deal(n_chunks);
        int st = och_gpu_chunk_costs(g->pools[0], cams, n_views, row_chunk, costs.data());
        if (st == OCH_OK) st = och_deal_chunks(costs.data(), n_chunks, g->n, nullptr, deal.data());
        for (int r = 0; r < g->n && st == OCH_OK; ++r)
            st = och_gpu_set_row_deal(g->pools[r], H, row_chunk, g->n, deal.data());
        if (st != OCH_OK) {
            const std::string msg = och_last_error();
            for (int r = 0; r < g->n; ++r) (void)och_gpu_set_row_deal(g->pools[r], H, row_chunk, g->n, nullptr);
            return group_fail(st, msg + " (every device back to round-robin chunks)");
        }
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
    OCH_ENTRY();
    return render_steps(g, cams, n_views, 1, 1, row_chunk, bounce);
}

OCH_API int och_frame_group_render_steps(och_frame_group *g, const och_camera *cams, int n_views, int n_steps,
                                         int n_buffers, int row_chunk, int bounce)
{
    OCH_ENTRY();
    return render_steps(g, cams, n_views, n_steps, n_buffers, row_chunk, bounce);
}

OCH_API int och_frame_group_frames_dev(och_frame_group *g, int rank, uint32_t **frames)
{
    if (!g || !frames || rank < 0 || rank >= g->n) return group_fail(OCH_E_INVALID, "bad rank");
    if (!g->rendered) return group_fail(OCH_E_INVALID, "nothing rendered yet");
    *frames = g->frames[rank][g->last_set];
    return OCH_OK;
}

OCH_API int och_frame_group_download(och_frame_group *g, int rank, uint32_t *rgba)
{
    if (!g || !rgba || rank < 0 || rank >= g->n) return group_fail(OCH_E_INVALID, "bad rank");
    if (!g->rendered) return group_fail(OCH_E_INVALID, "nothing rendered yet");
    int prev = -1;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(g->devices[rank]);
    const hipStream_t s = g->streams[rank][g->last_set];
    const size_t bytes = (size_t)g->n_views * g->height * g->width * 4;
    if (e == hipSuccess) e = hipMemcpyAsync(rgba, g->frames[rank][g->last_set], bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) return group_fail(OCH_E_HIP, hip_err("frame download", e));
    return OCH_OK;
}

OCH_API int och_frame_group_synchronize(och_frame_group *g)
{
    if (!g) return group_fail(OCH_E_INVALID, "NULL group");
    return sync_all(g);
}

}  // extern "C"
