// och_comm.cpp -- the library's own RCCL communicator for one process per GPU
// (the driver's N > 1 bench runs one rank per GPU).
//
// The reference renders a frame on one core (ORT/test_och_h_octree.cpp:
// 437-457).  Sharded, every rank renders its row chunks and one all-gather
// over xGMI hands the slices round; och_gpu_render_sharded_steps_dev
// (och_api.cpp) issues a window of such frames -- render, all-gather, shade --
// from one library call per rank, so no interpreter sits between a frame's
// launch and its collective.  The communicator is RCCL's own: rank 0 makes
// the id (och_comm_unique_id), the caller's launcher hands it to every rank
// (torch.distributed broadcast, MPI, a file), and every rank joins with
// och_comm_create (ncclCommInitRank).  This file also owns the RCCL loader
// that the one-process device group (och_group.cpp) uses.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>

#include "och_internal.h"
#include "och_rccl.h"

namespace och {

const Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // An RCCL already in the process first: torch's is loaded as
        // "librccl.so" (no soname), ROCm's as librccl.so.1.
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
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
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.comm_init_rank, "ncclCommInitRank");
        sym(r.comm_init_all, "ncclCommInitAll");
        sym(r.comm_destroy, "ncclCommDestroy");
        sym(r.comm_abort, "ncclCommAbort");
        sym(r.all_gather, "ncclAllGather");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
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

}  // namespace och

struct och_comm {
    ncclComm_t comm = nullptr;
    int n_ranks = 0;
    int rank = 0;
    int device = -1;
};

namespace {

static_assert(sizeof(ncclUniqueId) == OCH_COMM_ID_BYTES, "OCH_COMM_ID_BYTES must match ncclUniqueId");

int comm_fail(int status, const std::string &msg) { return och::report(status, msg.c_str()); }

int rccl_fail(const char *what, ncclResult_t r)
{
    return comm_fail(OCH_E_HIP, std::string(what) + ": " + och::rccl().error_string(r));
}

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DevGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

namespace och {

int comm_ranks(const och_comm *c, int *n_ranks, int *rank, int *device)
{
    if (!c || !c->comm) return comm_fail(OCH_E_INVALID, "communicator is NULL or destroyed");
    if (n_ranks) *n_ranks = c->n_ranks;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return OCH_OK;
}

int comm_all_gather(och_comm *c, const void *send, void *recv, size_t bytes, hipStream_t stream)
{
    if (!c || !c->comm) return comm_fail(OCH_E_INVALID, "communicator is NULL or destroyed");
    const ncclResult_t r = rccl().all_gather(send, recv, bytes, ncclUint8, c->comm, stream);
    return r == ncclSuccess ? OCH_OK : rccl_fail("ncclAllGather", r);
}

// Rank `root` receives every rank's `bytes` into recv[r * bytes]; the other
// ranks only send.  One RCCL group of point-to-point calls on the root: no rank
// but the root spends HBM or CUs on receiving.
int comm_gather(och_comm *c, const void *send, void *recv, size_t bytes, int root, hipStream_t stream)
{
    if (!c || !c->comm) return comm_fail(OCH_E_INVALID, "communicator is NULL or destroyed");
    if (root < 0 || root >= c->n_ranks) return comm_fail(OCH_E_INVALID, "gather root outside the communicator");
    const Rccl &R = rccl();
    if (c->rank == root) {
        if (recv == nullptr) return comm_fail(OCH_E_INVALID, "the gather root needs a receive buffer");
        char *dst = static_cast<char *>(recv);
        // One group: a receive from every rank, the root's own slice included
        // (a send to itself), so the same RCCL calls run at every world size --
        // world size 1, the one a one-GPU box can run, exercises them too.
        ncclResult_t r = R.group_start();
        if (r == ncclSuccess && send != dst + (size_t)root * bytes)
            r = R.send(send, bytes, ncclUint8, root, c->comm, stream);
        for (int p = 0; p < c->n_ranks && r == ncclSuccess; ++p)
            if (p != root || send != dst + (size_t)root * bytes)
                r = R.recv(dst + (size_t)p * bytes, bytes, ncclUint8, p, c->comm, stream);
        const ncclResult_t e = R.group_end();
        if (r == ncclSuccess) r = e;
        return r == ncclSuccess ? OCH_OK : rccl_fail("ncclSend / ncclRecv group", r);
    }
    const ncclResult_t r = R.send(send, bytes, ncclUint8, root, c->comm, stream);
    return r == ncclSuccess ? OCH_OK : rccl_fail("ncclSend", r);
}

// After a failure that follows an issued collective (a rank whose window
// stopped part way leaves its peers' collectives without a partner): abort
// the communicator so no stream waits on it forever, and mark it destroyed,
// so every later call on it fails instead of issuing.
void comm_abort(och_comm *c)
{
    if (!c || !c->comm) return;
    DevGuard g(c->device);
    (void)rccl().comm_abort(c->comm);
    c->comm = nullptr;
}

}  // namespace och

extern "C" {

OCH_API int och_comm_unique_id(uint8_t *id)
{
    if (!id) return comm_fail(OCH_E_INVALID, "NULL id buffer");
    const och::Rccl &R = och::rccl();
    if (!R.ok) return comm_fail(OCH_E_NODEV, R.error);
    ncclUniqueId u;
    const ncclResult_t r = R.get_unique_id(&u);
    if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
    std::memcpy(id, &u, sizeof u);
    return OCH_OK;
}

OCH_API int och_comm_create(const uint8_t *id, int n_ranks, int rank, int device, och_comm **out)
{
    if (!id || !out) return comm_fail(OCH_E_INVALID, "NULL argument");
    *out = nullptr;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return comm_fail(OCH_E_INVALID, "rank " + std::to_string(rank) + " of " + std::to_string(n_ranks));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return comm_fail(OCH_E_NODEV, "no HIP device visible");
    if (device < 0 || device >= ndev) return comm_fail(OCH_E_NODEV, "device " + std::to_string(device) + " not visible");
    const och::Rccl &R = och::rccl();
    if (!R.ok) return comm_fail(OCH_E_NODEV, R.error);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    DevGuard g(device);
    ncclComm_t comm = nullptr;
    // Collective over the ranks: returns once every rank has joined.
    const ncclResult_t r = R.comm_init_rank(&comm, n_ranks, u, rank);
    if (r != ncclSuccess) return rccl_fail("ncclCommInitRank", r);
    auto *c = new och_comm;
    c->comm = comm;
    c->n_ranks = n_ranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return OCH_OK;
}

OCH_API int och_comm_available(void)
{
    const och::Rccl &R = och::rccl();
    return R.ok ? OCH_OK : comm_fail(OCH_E_NODEV, R.error);
}

// For a watchdog on another thread: a collective that never completes (a peer
// that died or never issued its side) keeps its stream, and the host waiting
// on it, blocked; ncclCommAbort makes RCCL stop waiting.  The handle stays
// valid for och_comm_destroy; every later call on it fails.
OCH_API int och_comm_abort(och_comm *c)
{
    if (!c) return comm_fail(OCH_E_INVALID, "NULL communicator");
    och::comm_abort(c);
    return OCH_OK;
}

OCH_API int och_comm_destroy(och_comm *c)
{
    if (!c) return OCH_OK;
    if (c->comm) {
        DevGuard g(c->device);
        (void)och::rccl().comm_destroy(c->comm);
    }
    delete c;
    return OCH_OK;
}

OCH_API int och_comm_info(const och_comm *c, int *n_ranks, int *rank, int *device)
{
    return och::comm_ranks(c, n_ranks, rank, device);
}

OCH_API int och_comm_all_gather(och_comm *c, const void *send, void *recv, size_t bytes, void *stream)
{
    if (bytes && (!send || !recv)) return comm_fail(OCH_E_INVALID, "NULL buffer");
    DevGuard g(c ? c->device : -1);
    return och::comm_all_gather(c, send, recv, bytes, static_cast<hipStream_t>(stream));
}

OCH_API int och_comm_gather(och_comm *c, const void *send, void *recv, size_t bytes, int root, void *stream)
{
    if (bytes && !send) return comm_fail(OCH_E_INVALID, "NULL send buffer");
    DevGuard g(c ? c->device : -1);
    return och::comm_gather(c, send, recv, bytes, root, static_cast<hipStream_t>(stream));
}

}  // extern "C"
