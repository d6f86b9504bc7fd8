// examples/render_frame.cpp -- headless C++ host over the C ABI: builds the
// demo terrain, renders one frame on the GPU into an RGBA8 buffer (the
// olc::Pixel layout the reference's window blits) and writes it as a PPM.
// Also traces the reference's per-frame pick ray (ORT/test_och_h_octree.cpp:527-536)
// through the reference signature, tree.sse_trace(o, d, dir&, voxel&, t&).
//
//   make -C examples && ./examples/render_frame 10 out.ppm [width height yaw pitch]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "och_gpu.hpp"
#include "palette.hpp"

int main(int argc, char **argv)
{
    const int depth = argc > 1 ? std::atoi(argv[1]) : 10;
    const char *path = argc > 2 ? argv[2] : "frame.ppm";
    och::gpu::camera cam;
    cam.width = argc > 4 ? std::atoi(argv[3]) : 1280;
    cam.height = argc > 4 ? std::atoi(argv[4]) : 720;
    cam.yaw = argc > 6 ? std::strtof(argv[5], nullptr) : 0.3F;
    cam.pitch = argc > 6 ? std::strtof(argv[6], nullptr) : -0.6F;
    och_terrain_params tp = {depth, 1, 1, 0, 0, 1};   // voxelised on the GPU
    och_host_pool hp;
    och::gpu::check(och_build_terrain(&tp, &hp), "och_build_terrain");
    std::printf("terrain depth %d: %u nodes (%.2f s)\n", depth, hp.n_nodes, hp.build_seconds);
    try {
        och::gpu::tree tree(hp.nodes, hp.n_nodes, hp.root, hp.depth);
        tree.set_palette(examples::reference_palette());
        const och_camera c = cam.update_position();
        std::vector<uint32_t> rgba((size_t)cam.width * cam.height);
        tree.render(c, rgba.data());
        // pick ray along the view direction (the demo traces camera.pos along its look vector)
        const float dx = cosf(cam.yaw) * cosf(cam.pitch), dy = sinf(cam.yaw) * cosf(cam.pitch), dz = sinf(cam.pitch);
        och::gpu::direction dir;
        uint32_t vox;
        float t;
        tree.sse_trace(cam.pos, {dx, dy, dz}, dir, vox, t);
        std::printf("pick ray: d %a %a %a direction %d voxel %u t %a\n", dx, dy, dz, (int)dir, vox, t);
        if (!examples::write_ppm(path, rgba.data(), cam.width, cam.height)) return 1;
        std::printf("wrote %s\n", path);
    } catch (const och::gpu::error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        och_host_pool_free(&hp);
        return 1;
    }
    och_host_pool_free(&hp);
    return 0;
}
