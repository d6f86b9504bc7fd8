// och_rccl.h -- RCCL entry points, loaded on first use (dlopen).
//
// The library has no link-time dependency on RCCL: single-GPU users never
// load it, and an RCCL already in the process (PyTorch's) is reused, so the
// library's communicators and torch's share one runtime.  Shared by the
// one-process device group (och_group.cpp) and the one-process-per-GPU
// communicator (och_comm.cpp).  Not part of the public ABI.
#pragma once
#include <rccl/rccl.h>

#include <string>

namespace och {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;      // why loading failed (ok == false)
    bool ok = false;
};

// The process's RCCL, loaded once (thread-safe).
const Rccl &rccl();

}  // namespace och
