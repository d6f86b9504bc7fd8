// examples/multi_gpu_frame.cpp -- the reference's frame loop
// (ORT/test_och_h_octree.cpp:437-457) across every GPU of the node from one
// host thread: och::gpu::frame_group deals row chunks over the devices, one
// RCCL all-gather assembles the frame on every device.  Renders `frames`
// frames of two views (pitch 0 and -0.6), reports the frame time, writes
// view `view` of the last device's copy as a PPM.
//
//   ./examples/multi_gpu_frame 12 3840 2160 out.ppm [n_devices] [frames] [view]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "och_gpu.hpp"
#include "palette.hpp"

int main(int argc, char **argv)
{
    const int depth = argc > 1 ? std::atoi(argv[1]) : 12;
    const int W = argc > 2 ? std::atoi(argv[2]) : 3840, H = argc > 3 ? std::atoi(argv[3]) : 2160;
    const char *path = argc > 4 ? argv[4] : "multi_gpu_frame.ppm";
    // the gfx950 devices by HIP index: a node may list other devices too
    const std::vector<int> gfx950 = och::gpu::devices();
    int n = (int)gfx950.size();
    if (argc > 5 && std::atoi(argv[5]) < n) n = std::atoi(argv[5]);
    const int frames = argc > 6 ? std::atoi(argv[6]) : 10;
    const int view = argc > 7 ? std::atoi(argv[7]) : 1;
    if (n < 1) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 1;
    }
    och_terrain_params tp = {depth, 1, 1, 0, 0, 1};   // voxelised on the GPU
    och_host_pool hp;
    och::gpu::check(och_build_terrain(&tp, &hp), "och_build_terrain");
    int rc = 0;
    try {
        const std::vector<int> devices(gfx950.begin(), gfx950.begin() + n);
        och::gpu::frame_group group(devices, hp.nodes, hp.n_nodes, hp.root, hp.depth);
        group.set_palette(examples::reference_palette());
        std::vector<och_camera> cams;
        for (float pitch : {0.0F, -0.6F}) {
            och::gpu::camera cam;
            cam.yaw = 0.3F;
            cam.pitch = pitch;
            cam.width = W;
            cam.height = H;
            cams.push_back(cam.update_position());
        }
        group.plan(cams);                         // costliest tiles first (one timed render per device)
        group.render(cams);                       // warm-up
        group.synchronize();
        const auto t0 = std::chrono::steady_clock::now();
        for (int f = 0; f < frames; ++f) group.render(cams);
        group.synchronize();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%d devices, %dx%d x2 views, depth %d: %.4f ms per frame pair, %.1f Mrays/s\n", n, W, H, depth,
                    s / frames * 1e3, 2.0 * W * H * frames / s / 1e6);
        std::vector<uint32_t> rgba((size_t)2 * W * H);
        group.download(n - 1, rgba.data());
        if (!examples::write_ppm(path, rgba.data() + (size_t)view * W * H, W, H)) rc = 1;
        else std::printf("wrote %s (view %d, device %d's copy)\n", path, view, devices[n - 1]);
    } catch (const och::gpu::error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        rc = 1;
    }
    och_host_pool_free(&hp);
    return rc;
}
