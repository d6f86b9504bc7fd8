// examples/sharded_frame.cpp -- the reference's frame loop
// (ORT/test_och_h_octree.cpp:437-457) as one process per GPU, the layout an MPI
// or torch.distributed launch gives (and the driver's N-GPU bench runs):
//   * rank 0 makes the RCCL id (och_comm_unique_id) and hands it to the other
//     ranks through a file -- any launcher's broadcast does the same -- and
//     every rank joins (och_comm_create: ncclCommInitRank on its device);
//   * the row chunks are dealt with the display rank (rank 0, which shades
//     the whole frame) at a lighter weight (och_deal_chunks, och_gpu_set_row_deal);
//   * one och_gpu_render_sharded_steps_dev call per rank issues `frames`
//     frames of two views, B = 3 in flight on 3 streams: each rank renders its
//     rows as 1-byte colour codes, sends them to rank 0 (OCH_EXCHANGE_GATHER:
//     ncclSend / ncclRecv), and rank 0 shades them into RGBA8 frames.
// Rank 0 reports the frame time and writes view `view` of its last frame as
// a PPM.
//
//   ./examples/sharded_frame depth W H out.ppm rank n_ranks id_file [frames] [view]
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "och_gpu.hpp"
#include "palette.hpp"

namespace {

void hip_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) throw och::gpu::error(OCH_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Rank 0 writes the id to `path` (complete files only: write, then rename);
// the other ranks wait for it.
och::gpu::comm::id_t share_id(int rank, const std::string &path)
{
    och::gpu::comm::id_t id{};
    if (rank == 0) {
        id = och::gpu::comm::unique_id();
        const std::string tmp = path + ".tmp";
        std::ofstream(tmp, std::ios::binary).write(reinterpret_cast<const char *>(id.data()), id.size());
        if (std::rename(tmp.c_str(), path.c_str()) != 0) throw och::gpu::error(OCH_E_INVALID, "cannot publish " + path);
        return id;
    }
    for (int waited = 0; waited < 600; ++waited) {
        std::ifstream in(path, std::ios::binary);
        if (in && in.read(reinterpret_cast<char *>(id.data()), id.size())) return id;
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    throw och::gpu::error(OCH_E_INVALID, "no RCCL id in " + path + " after 60 s");
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 8) {
        std::fprintf(stderr, "usage: sharded_frame depth W H out.ppm rank n_ranks id_file [frames] [view]\n");
        return 2;
    }
    const int depth = std::atoi(argv[1]), W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    const char *path = argv[4];
    const int rank = std::atoi(argv[5]), n_ranks = std::atoi(argv[6]);
    const std::string id_file = argv[7];
    const int frames = argc > 8 ? std::atoi(argv[8]) : 10;
    const int view = argc > 9 ? std::atoi(argv[9]) : 1;
    constexpr int kViews = 2, kChunk = 8, kBuffers = 3;
    const std::vector<int> gfx950 = och::gpu::devices();
    if (gfx950.empty()) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 1;
    }
    const int device = gfx950[rank % gfx950.size()];
    int rc = 0;
    och_host_pool hp{};
    std::vector<void *> owned;
    std::vector<hipStream_t> streams;
    try {
        hip_check(hipSetDevice(device), "hipSetDevice");
        och_terrain_params tp = {depth, 1, 1, 0, 0, 1};    // voxelised on this rank's GPU
        och::gpu::check(och_build_terrain(&tp, &hp), "och_build_terrain");
        och::gpu::tree tree(hp.nodes, hp.n_nodes, hp.root, hp.depth, 1, __builtin_inff(), device);
        tree.set_palette(examples::reference_palette());
        och::gpu::comm comm(share_id(rank, id_file), n_ranks, rank, device);
        std::vector<och_camera> cams;
        for (float pitch : {0.0F, -0.6F}) {
            och::gpu::camera cam;
            cam.yaw = 0.3F;
            cam.pitch = pitch;
            cam.width = W;
            cam.height = H;
            cams.push_back(cam.update_position());
        }
        // the deal: rank 0 shades the whole frame, so it renders fewer rows
        // (octree_ray_tracing_amd.display_weight: 0.9 / 0.7 / 0.5 at 2 / 4 / 8 ranks)
        const int n_chunks = (H + kChunk - 1) / kChunk;
        std::vector<float> costs(n_chunks, 1.0F), weights(n_ranks, 1.0F);
        weights[0] = n_ranks == 2 ? 0.9F : n_ranks == 4 ? 0.7F : n_ranks >= 8 ? 0.5F : 1.0F - 0.0625F * n_ranks;
        std::vector<int32_t> deal(n_chunks);
        och::gpu::check(och_deal_chunks(costs.data(), n_chunks, n_ranks, weights.data(), deal.data()), "och_deal_chunks");
        och::gpu::check(och_gpu_set_row_deal(tree.handle(), H, kChunk, n_ranks, deal.data()), "och_gpu_set_row_deal");
        // launch order: costliest tiles first (one timed planning render)
        och::gpu::check(och_gpu_plan_views(tree.handle(), cams.data(), kViews, kChunk, rank, n_ranks), "och_gpu_plan_views");
        och::gpu::check(och_gpu_set_option(tree.handle(), OCH_OPT_TILE_ORDER, 2), "och_gpu_set_option");
        int rows = 0;
        och::gpu::check(och_gpu_slice_rows(tree.handle(), H, kChunk, n_ranks, &rows), "och_gpu_slice_rows");
        const size_t slice = (size_t)kViews * rows * W;
        std::vector<void *> st(kBuffers);
        std::vector<uint8_t *> slices(kBuffers), gathered(kBuffers, nullptr);
        std::vector<uint32_t *> frames_dev(kBuffers, nullptr);
        auto alloc = [&](size_t bytes) {
            void *p = nullptr;
            hip_check(hipMalloc(&p, bytes), "hipMalloc");
            owned.push_back(p);
            return p;
        };
        for (int b = 0; b < kBuffers; ++b) {
            hipStream_t s = nullptr;
            hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
            streams.push_back(s);
            st[b] = s;
            slices[b] = static_cast<uint8_t *>(alloc(slice));
            if (rank == 0) {                                     // the gather's root receives and shades
                gathered[b] = static_cast<uint8_t *>(alloc(slice * n_ranks));
                frames_dev[b] = static_cast<uint32_t *>(alloc((size_t)kViews * H * W * 4));
            }
        }
        auto run = [&](int n) {
            och::gpu::check(och_gpu_render_sharded_steps_dev(tree.handle(), comm.handle(), cams.data(), kViews, n,
                                                             st.data(), slices.data(), gathered.data(),
                                                             frames_dev.data(), kBuffers, nullptr, nullptr, kChunk,
                                                             /*bounce*/ 0, OCH_EXCHANGE_GATHER),
                            "och_gpu_render_sharded_steps_dev");
            for (hipStream_t s : streams) hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
        };
        run(kBuffers);                                           // warm-up
        const auto t0 = std::chrono::steady_clock::now();
        run(frames);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("rank %d of %d (device %d): %dx%d x2 views, depth %d, rows %d: %.4f ms per frame pair, "
                    "%.1f Mrays/s for the job\n", rank, n_ranks, device, W, H, depth, rows, s / frames * 1e3,
                    2.0 * W * H * frames / s / 1e6);
        if (rank == 0) {
            std::vector<uint32_t> rgba((size_t)W * H);
            const uint32_t *last = frames_dev[(frames - 1) % kBuffers] + (size_t)view * W * H;
            hip_check(hipMemcpy(rgba.data(), last, rgba.size() * 4, hipMemcpyDeviceToHost), "hipMemcpy");
            if (!examples::write_ppm(path, rgba.data(), W, H)) rc = 1;
            else std::printf("wrote %s (view %d)\n", path, view);
        }
    } catch (const och::gpu::error &e) {
        std::fprintf(stderr, "rank %d: %s\n", rank, e.what());
        rc = 1;
    }
    // A HIP error some earlier call left pending (RCCL's init, say) is cleared
    // by the next launch and kept: say so once, with where it was found.
    int stale = 0, n_stale = 0;
    char where[320] = "";
    if (och_discarded_error(&stale, &n_stale, where, sizeof where, 1) == OCH_OK && n_stale)
        std::fprintf(stderr, "rank %d: %d pending HIP error(s) cleared before launches; the first: %s\n", rank,
                     n_stale, where);
    for (void *p : owned) (void)hipFree(p);
    for (hipStream_t s : streams) (void)hipStreamDestroy(s);
    if (hp.nodes) och_host_pool_free(&hp);
    return rc;
}
