// examples/render_frame.cpp -- headless C++ host over the C ABI: builds the
// demo terrain, renders one frame on the GPU into an RGBA8 buffer (the
// olc::Pixel layout the reference's window blits) and writes it as a PPM.
// Also traces the reference's per-frame pick ray (ORT/test_och_h_octree.cpp:527-536).
//
//   make -C examples && ./examples/render_frame 10 out.ppm
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "och_gpu.hpp"

static std::vector<uint32_t> reference_palette()
{
    // voxels.txt (ORT/voxels.txt): Stone, Grass, Dark Grass, Dirt; x_pos..z_neg.
    const uint32_t rgb[4][6] = {
        {0x44445D, 0x4E4E5B, 0x4E6155, 0x2B352F, 0x33333A, 0x232328},
        {0x5D2917, 0x3D260F, 0x4F2E14, 0x603718, 0x6D2E0D, 0x3F8527},
        {0x5D2917, 0x3D260F, 0x4F2E14, 0x603718, 0x6D2E0D, 0x317D1A},
        {0x5D2917, 0x3D260F, 0x4F2E14, 0x603718, 0x6D2E0D, 0x56220F}};
    std::vector<uint32_t> out;
    for (auto &v : rgb)
        for (uint32_t c : v) out.push_back(0xFF000000u | ((c & 0xFF) << 16) | (c & 0xFF00) | (c >> 16));
    return out;
}

int main(int argc, char **argv)
{
    const int depth = argc > 1 ? std::atoi(argv[1]) : 10;
    const char *path = argc > 2 ? argv[2] : "frame.ppm";
    och_terrain_params tp = {depth, 1, 1, 0, 0, 1};
    och_host_pool hp;
    och::gpu::check(och_build_terrain(&tp, &hp), "och_build_terrain");
    std::printf("terrain depth %d: %u nodes (%.2f s)\n", depth, hp.n_nodes, hp.build_seconds);
    try {
        och::gpu::tree tree(hp.nodes, hp.n_nodes, hp.root, hp.depth);
        tree.set_palette(reference_palette());
        och::gpu::camera cam;
        cam.yaw = 0.3F;
        cam.pitch = -0.6F;
        cam.width = 1280;
        cam.height = 720;
        const och_camera c = cam.update_position();
        std::vector<uint32_t> rgba((size_t)cam.width * cam.height);
        tree.render(c, rgba.data());
        // pick ray along the view direction
        const float dx = cosf(cam.yaw) * cosf(cam.pitch), dy = sinf(cam.yaw) * cosf(cam.pitch), dz = sinf(cam.pitch);
        och::gpu::direction dir;
        uint32_t vox;
        float t;
        tree.sse_trace(cam.pos, {dx, dy, dz}, dir, vox, t);
        std::printf("pick ray: direction %d voxel %u t %.6f\n", (int)dir, vox, t);
        FILE *f = std::fopen(path, "wb");
        std::fprintf(f, "P6\n%d %d\n255\n", cam.width, cam.height);
        for (uint32_t p : rgba) {
            const unsigned char px[3] = {(unsigned char)(p & 0xFF), (unsigned char)((p >> 8) & 0xFF),
                                         (unsigned char)((p >> 16) & 0xFF)};
            std::fwrite(px, 1, 3, f);
        }
        std::fclose(f);
        std::printf("wrote %s\n", path);
    } catch (const och::gpu::error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        och_host_pool_free(&hp);
        return 1;
    }
    och_host_pool_free(&hp);
    return 0;
}
