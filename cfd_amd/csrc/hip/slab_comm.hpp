// slab_comm.hpp -- collectives of the Z-slab decomposition.
//
// A SlabComm is one rank's endpoint. The projection driver only needs three
// operations, all enqueued on the caller's stream with no host round trip:
//   halo        -- refresh local planes 0 and nz-1 from the neighbours' last /
//                  first owned planes (nothing at a global z face unless the
//                  z boundary is periodic);
//   allreduce   -- sum of n doubles / max of n uint64 over ranks.
// Two backends: RCCL (one process per GPU, send/recv + allreduce over xGMI)
// and an in-process group (ranks = slab contexts of one process, each driven
// by its own host thread; copies and reductions are plain stream work
// ordered with events and a host barrier). The in-process group runs the
// multi-rank driver on one GPU, where RCCL refuses two ranks per device.
#pragma once

#include <hip/hip_runtime.h>

#include "cfd_hip/cfd_abi.h"

namespace cfdhip {
struct Mbox;
}
struct hip_proj_group;

struct SlabComm {
    int rank = 0, size = 1, device = 0;
    virtual ~SlabComm() {}
    // f[q] are local slabs of nz planes with plane pitch ps (doubles).
    // periodic: rank 0's lower neighbour is rank size-1 and vice versa, which
    // is exactly the periodic z boundary copy (plane 0 <- nz-2, nz-1 <- 1).
    virtual cfd_status_t halo(hipStream_t s, double* const* f, int nf, long long ps, int nz,
                              bool periodic) = 0;
    int lower(bool periodic) const { return rank > 0 ? rank - 1 : (periodic ? size - 1 : -1); }
    int upper(bool periodic) const { return rank < size - 1 ? rank + 1 : (periodic ? 0 : -1); }
    virtual cfd_status_t allreduce_sum(hipStream_t s, const double* in, double* out, int n) = 0;
    virtual cfd_status_t allreduce_max_u64(hipStream_t s, const unsigned long long* in,
                                           unsigned long long* out, int n) = 0;
    // Device mailbox for the one-shot CG dot all-reduce fused into the sweeps
    // (kernels.hpp mbox_allreduce); nullptr = all-reduce through allreduce_sum.
    virtual cfdhip::Mbox* device_mailbox() { return nullptr; }
    // the in-process group whose host lock this rank's calls take (ctx.hpp
    // GroupHostLock); nullptr for RCCL
    virtual hip_proj_group* host_group() { return nullptr; }
};

struct hip_proj_comm {
    SlabComm* impl = nullptr;
};
