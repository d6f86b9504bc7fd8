// och_gpu.hpp -- header-only C++ host mirror over the C ABI (och_gpu.h).
//
// Gives a reference user the same call shapes they had:
//   tree.sse_trace(ox, oy, oz, dx, dy, dz, hit_direction, hit_voxel, hit_time)
//                                               ORT/och_h_octree.h:292, :449-452
//   camera.update_position() + window.update_image()
//                                               ORT/test_och_h_octree.cpp:87-138, :437-457
// with the work done by the gfx950 kernels.  Errors throw och::gpu::error.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <array>
#include <vector>

#include "och_gpu.h"

namespace och {
namespace gpu {

// och::direction (ORT/och_tree_helper.h:7-18).
enum class direction : int32_t {
    x_pos = 0, y_pos = 1, z_pos = 2, x_neg = 3, y_neg = 4, z_neg = 5, exit = 6, inside = 7, error = 8
};

struct error : std::runtime_error {
    int status;
    error(int s, const std::string &what) : std::runtime_error(what), status(s) {}
};

inline void check(int status, const char *what)
{
    if (status != OCH_OK) throw error(status, std::string(what) + ": " + och_last_error());
}

// HIP indices of the visible gfx950 devices (och_device_list).
inline std::vector<int> devices()
{
    int n = 0;
    check(och_device_list(nullptr, 0, &n), "och_device_list");
    std::vector<int> d(n);
    if (n) check(och_device_list(d.data(), n, &n), "och_device_list");
    return d;
}

struct float3 {
    float x, y, z;
};

// A node pool resident on one GPU.  Construct from the reference's own table
// (h_octree: table->nodes, capacity, root_idx, Depth) or from och_build_terrain.
class tree {
public:
    tree(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int index_base = 1,
         float miss_t = __builtin_inff(), int device = -1)
    {
        check(och_gpu_pool_create(nodes, n_nodes, root, depth, index_base, miss_t, device, &pool_), "och_gpu_pool_create");
    }
    tree(const tree &) = delete;
    tree &operator=(const tree &) = delete;
    ~tree() { och_gpu_pool_destroy(pool_); }

    // h_octree::sse_trace, one ray (synchronous; fine for the pick ray of :536).
    void sse_trace(float ox, float oy, float oz, float dx, float dy, float dz, direction &hit_direction,
                   uint32_t &hit_voxel, float &hit_time) const
    {
        int32_t d = 0;
        check(och_gpu_trace(pool_, ox, oy, oz, dx, dy, dz, &d, &hit_voxel, &hit_time), "och_gpu_trace");
        hit_direction = static_cast<direction>(d);
    }
    void sse_trace(float3 o, float3 d, direction &hit_direction, uint32_t &hit_voxel, float &hit_time) const
    {
        sse_trace(o.x, o.y, o.z, d.x, d.y, d.z, hit_direction, hit_voxel, hit_time);
    }

    // Many rays at once (the per-pixel loop's calls, batched).  width > 0: the
    // rays are a camera's, a row-major image that many rays wide (x + y * W,
    // ORT/test_och_h_octree.cpp:135), traced 8x8 tiles per wave
    // (och_gpu_trace_batch_image); same records either way.
    void trace_batch(float3 origin, const std::vector<float3> &dirs, std::vector<direction> &dir_out,
                     std::vector<uint32_t> &voxel_out, std::vector<float> &t_out, uint32_t width = 0) const
    {
        const uint32_t n = static_cast<uint32_t>(dirs.size());
        std::vector<int32_t> d(n);
        voxel_out.resize(n);
        t_out.resize(n);
        if (width)
            check(och_gpu_trace_batch_image(pool_, &origin.x, 0, &dirs[0].x, n, width, d.data(), voxel_out.data(),
                                            t_out.data()),
                  "och_gpu_trace_batch_image");
        else
            check(och_gpu_trace_batch(pool_, &origin.x, 0, &dirs[0].x, n, d.data(), voxel_out.data(), t_out.data()),
                  "och_gpu_trace_batch");
        dir_out.resize(n);
        for (uint32_t i = 0; i < n; ++i) dir_out[i] = static_cast<direction>(d[i]);
    }

    void set_palette(const std::vector<uint32_t> &rgba)
    {
        check(och_gpu_set_palette(pool_, rgba.data(), static_cast<uint32_t>(rgba.size() / 6)), "och_gpu_set_palette");
    }

    // update_position + update_image into an olc::Sprite-compatible RGBA8 buffer
    // (memcpy it into GetDrawTarget()->GetData(), olcPixelGameEngine.h:945).
    void render(const och_camera &cam, uint32_t *rgba) const { check(och_gpu_render(pool_, &cam, rgba), "och_gpu_render"); }

    och_gpu_pool *handle() const { return pool_; }

private:
    och_gpu_pool *pool_ = nullptr;
};

// h_octree::set / at (ORT/och_h_octree.h:176-258) with a device mirror that is
// refreshed by uploading only the slots the edits wrote.
class editor {
public:
    editor(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, uint32_t capacity)
        : depth_(depth)
    {
        check(och_editor_create(nodes, n_nodes, root, depth, capacity, &ed_), "och_editor_create");
    }
    editor(const editor &) = delete;
    editor &operator=(const editor &) = delete;
    ~editor() { och_editor_destroy(ed_); }

    void set(int x, int y, int z, uint32_t v) { check(och_editor_set(ed_, x, y, z, v), "och_editor_set"); }
    uint32_t at(int x, int y, int z) const { return och_editor_at(ed_, x, y, z); }
    uint32_t get_root() const
    {
        och_editor_stats st;
        och_editor_info(ed_, &st);
        return st.root;
    }

    // The device pool that mirrors this editor; refresh it with flush().
    tree make_tree(int device = -1) const
    {
        const uint32_t *words = nullptr;
        uint32_t slots = 0, root = 0;
        check(och_editor_nodes(ed_, &words, &slots, &root), "och_editor_nodes");
        return tree(words, slots, root, depth_, 1, __builtin_inff(), device);
    }
    void flush(tree &t) { check(och_editor_flush(ed_, t.handle()), "och_editor_flush"); }

    och_editor *handle() const { return ed_; }

private:
    och_editor *ed_ = nullptr;
    int depth_;
};

// Every GPU of the node from one host thread: a pool replica
// per device, row chunks dealt round-robin, one RCCL all-gather, shading on
// every device.  frames(rank) is device rank's [views][H][W] RGBA8 copy.
class frame_group {
public:
    frame_group(const std::vector<int> &devices, const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth,
                int index_base = 1, float miss_t = __builtin_inff())
    {
        check(och_frame_group_create(devices.data(), static_cast<int>(devices.size()), nodes, n_nodes, root, depth,
                                     index_base, miss_t, &g_),
              "och_frame_group_create");
    }
    frame_group(const frame_group &) = delete;
    frame_group &operator=(const frame_group &) = delete;
    ~frame_group() { och_frame_group_destroy(g_); }

    int size() const
    {
        int n = 0;
        check(och_frame_group_size(g_, &n), "och_frame_group_size");
        return n;
    }
    void set_palette(const std::vector<uint32_t> &rgba)
    {
        check(och_frame_group_set_palette(g_, rgba.data(), static_cast<uint32_t>(rgba.size() / 6)),
              "och_frame_group_set_palette");
    }
    void set_option(och_option option, int value)
    {
        check(och_frame_group_set_option(g_, option, value), "och_frame_group_set_option");
    }
    // Cost-planned launch order for frames of these cameras' geometry.
    void plan(const std::vector<och_camera> &cams, int row_chunk = 8)
    {
        check(och_frame_group_plan(g_, cams.data(), static_cast<int>(cams.size()), row_chunk), "och_frame_group_plan");
    }
    // One frame of every view, asynchronous on all devices.
    void render(const std::vector<och_camera> &cams, int row_chunk = 8, bool bounce = false)
    {
        check(och_frame_group_render(g_, cams.data(), static_cast<int>(cams.size()), row_chunk, bounce ? 1 : 0),
              "och_frame_group_render");
    }
    // n_steps frames, up to n_buffers in flight, each device's issued by its own
    // thread; frames() / download() then give the last one.
    void render_steps(const std::vector<och_camera> &cams, int n_steps, int n_buffers = 3, int row_chunk = 8,
                      bool bounce = false)
    {
        check(och_frame_group_render_steps(g_, cams.data(), static_cast<int>(cams.size()), n_steps, n_buffers,
                                           row_chunk, bounce ? 1 : 0),
              "och_frame_group_render_steps");
    }
    uint32_t *frames(int rank) const
    {
        uint32_t *p = nullptr;
        check(och_frame_group_frames_dev(g_, rank, &p), "och_frame_group_frames_dev");
        return p;
    }
    void download(int rank, uint32_t *rgba) const { check(och_frame_group_download(g_, rank, rgba), "och_frame_group_download"); }
    void synchronize() const { check(och_frame_group_synchronize(g_), "och_frame_group_synchronize"); }

private:
    och_frame_group *g_ = nullptr;
};

// The library's RCCL communicator for one process per GPU: rank 0 makes the
// id (unique_id()), the launcher hands it to every rank (MPI_Bcast, a file,
// torch.distributed), every rank constructs comm(id, n_ranks, rank, device).
class comm {
public:
    using id_t = std::array<uint8_t, OCH_COMM_ID_BYTES>;
    static id_t unique_id()
    {
        id_t id{};
        check(och_comm_unique_id(id.data()), "och_comm_unique_id");
        return id;
    }
    comm(const id_t &id, int n_ranks, int rank, int device)
    {
        check(och_comm_create(id.data(), n_ranks, rank, device, &c_), "och_comm_create");
    }
    comm(const comm &) = delete;
    comm &operator=(const comm &) = delete;
    ~comm() { och_comm_destroy(c_); }
    och_comm *handle() const { return c_; }

private:
    och_comm *c_ = nullptr;
};

// tree_camera's per-frame state (pos :55, dir :53, fov :95).
struct camera {
    float3 pos{1.5F, 1.5F, 1.5F};
    float yaw = 0.0F, pitch = 0.0F, fov = 1.25F;
    int width = 640, height = 360;

    och_camera update_position() const
    {
        och_camera c;
        check(och_camera_setup(pos.x, pos.y, pos.z, yaw, pitch, fov, width, height, &c), "och_camera_setup");
        return c;
    }
};

}  // namespace gpu
}  // namespace och
