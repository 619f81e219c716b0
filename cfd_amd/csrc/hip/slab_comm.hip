// slab_comm.hip -- RCCL and in-process backends of SlabComm (slab_comm.hpp)
// and their C-ABI constructors (include/cfd_hip/projection_hip.h).
#include "slab_comm.hpp"

#include "mbox.hpp"

#include "cfd_hip/projection_hip.h"

#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

extern "C" void cfd_set_error(cfd_status_t status, const char* message) __attribute__((weak));

static cfd_status_t fail(cfd_status_t s, const char* what, const char* detail) {
    char buf[256];
    snprintf(buf, sizeof(buf), "slab comm: %s%s%s", what, detail ? ": " : "", detail ? detail : "");
    if (cfd_set_error) cfd_set_error(s, buf);
    return s;
}

#define HIPC(call)                                                                  \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) return fail(CFD_ERROR, #call, hipGetErrorString(e_)); \
    } while (0)

#define NCCLC(call)                                                                    \
    do {                                                                               \
        ncclResult_t r_ = (call);                                                      \
        if (r_ != ncclSuccess) return fail(CFD_ERROR, #call, ncclGetErrorString(r_));  \
    } while (0)

namespace {

// ---------------------------------------------------------------------------
// RCCL: halo planes move with grouped ncclSend/ncclRecv (one plane each way
// per neighbour and field, point-to-point over xGMI), dot products with an
// 8-B ncclAllReduce. Everything is stream-ordered on the caller's stream.
// ---------------------------------------------------------------------------
struct RcclComm final : SlabComm {
    ncclComm_t comm = nullptr;   // all-reduces
    ncclComm_t hcomm = nullptr;  // halo send/recv: its own communicator, so a
                                 // halo on a side stream may overlap an all-reduce
    // opt-in device mailbox (CFD_HIP_DEVICE_ALLREDUCE=1)
    void* mbox = nullptr;                    // own mailbox (uncached device memory)
    std::vector<void*> peer_open;            // peers' mailboxes mapped through IPC
    cfdhip::Mbox* d_mb = nullptr;            // device copy of the Mbox descriptor
    ~RcclComm() override {
        for (void* p : peer_open)
            if (p) hipIpcCloseMemHandle(p);
        if (d_mb) hipFree(d_mb);
        if (mbox) hipFree(mbox);
        if (hcomm) ncclCommDestroy(hcomm);
        if (comm) ncclCommDestroy(comm);
    }
    cfdhip::Mbox* device_mailbox() override { return d_mb; }
    cfd_status_t setup_mailbox();
    // Posting order matters only when both neighbours are the same peer
    // (2 ranks, periodic): sends go to-lower then to-upper, receives come
    // from-upper then from-lower, so the k-th send to a peer always pairs
    // with the k-th receive the peer posts from us.
    cfd_status_t halo(hipStream_t s, double* const* f, int nf, long long ps, int nz,
                      bool periodic) override {
        if (size == 1) return CFD_SUCCESS;
        const int lo = lower(periodic), hi = upper(periodic);
        NCCLC(ncclGroupStart());
        for (int q = 0; q < nf; ++q) {
            if (lo >= 0) NCCLC(ncclSend(f[q] + ps, (size_t)ps, ncclDouble, lo, hcomm, s));
            if (hi >= 0) NCCLC(ncclSend(f[q] + ps * (nz - 2), (size_t)ps, ncclDouble, hi, hcomm, s));
            if (hi >= 0) NCCLC(ncclRecv(f[q] + ps * (nz - 1), (size_t)ps, ncclDouble, hi, hcomm, s));
            if (lo >= 0) NCCLC(ncclRecv(f[q], (size_t)ps, ncclDouble, lo, hcomm, s));
        }
        NCCLC(ncclGroupEnd());
        return CFD_SUCCESS;
    }
    cfd_status_t allreduce_sum(hipStream_t s, const double* in, double* out, int n) override {
        NCCLC(ncclAllReduce(in, out, (size_t)n, ncclDouble, ncclSum, comm, s));
        return CFD_SUCCESS;
    }
    cfd_status_t allreduce_max_u64(hipStream_t s, const unsigned long long* in,
                                   unsigned long long* out, int n) override {
        NCCLC(ncclAllReduce(in, out, (size_t)n, ncclUint64, ncclMax, comm, s));
        return CFD_SUCCESS;
    }
};

// Every rank allocates a small uncached mailbox, exports it through IPC, and
// the handles are all-gathered over RCCL; each rank then maps every peer's
// mailbox (xGMI peer access) into its Mbox descriptor.
cfd_status_t RcclComm::setup_mailbox() {
    constexpr size_t MB_BYTES = 4096;
    static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
    // local part; whatever happens here, every rank still joins the all-gather
    unsigned char hbytes[64] = {0};
    bool local = hipExtMallocWithFlags(&mbox, MB_BYTES, hipDeviceMallocUncached) == hipSuccess &&
                 hipMemset(mbox, 0, MB_BYTES) == hipSuccess;
    if (local) {
        hipIpcMemHandle_t h;
        local = hipIpcGetMemHandle(&h, mbox) == hipSuccess;
        if (local) memcpy(hbytes, &h, sizeof(h));
    }
    (void)hipGetLastError();
    unsigned char *d_send = nullptr, *d_recv = nullptr;
    hipStream_t s = nullptr;
    std::vector<unsigned char> all(64 * (size_t)size, 0);
    HIPC(hipMalloc((void**)&d_send, 64));
    HIPC(hipMalloc((void**)&d_recv, 64 * (size_t)size));
    HIPC(hipMemcpy(d_send, hbytes, 64, hipMemcpyHostToDevice));
    HIPC(hipStreamCreate(&s));
    ncclResult_t r = ncclAllGather(d_send, d_recv, 64, ncclUint8, comm, s);
    hipError_t e = hipStreamSynchronize(s);
    hipStreamDestroy(s);
    hipError_t e2 = hipMemcpy(all.data(), d_recv, all.size(), hipMemcpyDeviceToHost);
    hipFree(d_send);
    hipFree(d_recv);
    if (r != ncclSuccess) return fail(CFD_ERROR, "ncclAllGather (mailbox handles)", ncclGetErrorString(r));
    HIPC(e);
    HIPC(e2);
    if (!local) return fail(CFD_ERROR, "mailbox allocation / IPC export failed", nullptr);
    cfdhip::Mbox hmb{};
    hmb.n = size;
    hmb.rank = rank;
    hmb.count = 0;
    int rate_khz = 0;
    HIPC(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device));
    hmb.timeout_ticks = (long long)std::max(rate_khz, 1000) * 1000LL * 20;  // 20 s
    peer_open.assign(size, nullptr);
    for (int q = 0; q < size; ++q) {
        if (q == rank) {
            hmb.slot[q] = (unsigned long long*)mbox;
            continue;
        }
        hipIpcMemHandle_t ph;
        memcpy(&ph, all.data() + 64 * (size_t)q, sizeof(ph));
        void* p = nullptr;
        HIPC(hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess));
        peer_open[q] = p;
        hmb.slot[q] = (unsigned long long*)p;
    }
    HIPC(hipMalloc((void**)&d_mb, sizeof(hmb)));
    HIPC(hipMemcpy(d_mb, &hmb, sizeof(hmb), hipMemcpyHostToDevice));
    return CFD_SUCCESS;
}

namespace {
__global__ void k_mbox_selftest(cfdhip::Mbox* mb, double v, double* out, int* ok) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double s = 0.0;
        *ok = cfdhip::mbox_allreduce(mb, v, &s) ? 1 : 0;
        *out = s;
    }
}
}  // namespace

// Collective: every rank reports whether its mailbox is set up and a one-shot
// all-reduce of rank+1 over it returns n(n+1)/2 within ~2 s; the mailbox stays
// enabled only if that holds on every rank (else all fall back to RCCL).
static bool mailbox_verified(RcclComm* c, bool local_ok) {
    int ok = 0;
    if (local_ok) {
        cfdhip::Mbox h{};
        hipMemcpy(&h, c->d_mb, sizeof(h), hipMemcpyDeviceToHost);
        const long long full = h.timeout_ticks;
        h.timeout_ticks = full / 10;  // short bound for the probe
        hipMemcpy(c->d_mb, &h, sizeof(h), hipMemcpyHostToDevice);
        double* d_out = nullptr;
        int* d_ok = nullptr;
        if (hipMalloc((void**)&d_out, sizeof(double)) == hipSuccess &&
            hipMalloc((void**)&d_ok, sizeof(int)) == hipSuccess) {
            hipLaunchKernelGGL(k_mbox_selftest, dim3(1), dim3(64), 0, 0, c->d_mb,
                               (double)(c->rank + 1), d_out, d_ok);
            double out = 0.0;
            int kok = 0;
            if (hipDeviceSynchronize() == hipSuccess &&
                hipMemcpy(&out, d_out, sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(&kok, d_ok, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess)
                ok = (kok == 1 && out == 0.5 * c->size * (c->size + 1)) ? 1 : 0;
        }
        if (d_out) hipFree(d_out);
        if (d_ok) hipFree(d_ok);
        hipMemcpy(&h, c->d_mb, sizeof(h), hipMemcpyDeviceToHost);  // keeps count
        h.timeout_ticks = full;
        hipMemcpy(c->d_mb, &h, sizeof(h), hipMemcpyHostToDevice);
    }
    int* d_flag = nullptr;
    int all = 0;
    hipStream_t s = nullptr;
    if (hipMalloc((void**)&d_flag, sizeof(int)) == hipSuccess && hipStreamCreate(&s) == hipSuccess) {
        hipMemcpy(d_flag, &ok, sizeof(int), hipMemcpyHostToDevice);
        if (ncclAllReduce(d_flag, d_flag, 1, ncclInt32, ncclMin, c->comm, s) == ncclSuccess &&
            hipStreamSynchronize(s) == hipSuccess)
            hipMemcpy(&all, d_flag, sizeof(int), hipMemcpyDeviceToHost);
    }
    if (s) hipStreamDestroy(s);
    if (d_flag) hipFree(d_flag);
    return all == 1;
}

// ---------------------------------------------------------------------------
// In-process group: each rank's host thread publishes what it exposes,
// records an event, meets the others at a host barrier, makes its stream wait
// on the peers' events, pulls / reduces, records a second event and meets
// them again so no rank reuses a buffer a peer is still reading.
// ---------------------------------------------------------------------------
constexpr int GROUP_MAX = 16;
struct GroupPtrs {
    const void* p[GROUP_MAX];
    int n;
};

__global__ void k_group_sum(GroupPtrs in, double* out, int count) {
    for (int e = threadIdx.x; e < count; e += blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < in.n; ++r) s += ((const double*)in.p[r])[e];  // rank order
        out[e] = s;
    }
}

__global__ void k_group_max_u64(GroupPtrs in, unsigned long long* out, int count) {
    for (int e = threadIdx.x; e < count; e += blockDim.x) {
        unsigned long long m = 0;
        for (int r = 0; r < in.n; ++r) {
            const unsigned long long v = ((const unsigned long long*)in.p[r])[e];
            m = v > m ? v : m;
        }
        out[e] = m;
    }
}

}  // namespace

struct hip_proj_group;
// the group whose host lock this thread holds, and the entry-point nesting
// depth (an entry point may call another: only the outermost locks)
static thread_local hip_proj_group* t_held = nullptr;
static thread_local int t_depth = 0;

struct hip_proj_group {
    int size = 0;
    std::mutex host;  // serialises the ranks' host work (ctx.hpp GroupHostLock)
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    unsigned long long gen = 0;
    bool broken = false;
    int timeout_s = 300;
    std::vector<hipEvent_t> ev_ready, ev_done;
    std::vector<const void*> pub;
    std::vector<double* const*> pubf;
    std::vector<int> pubnz, joined;

    // false once any rank timed out: a rank that failed before reaching a
    // collective must not leave the others blocked forever.
    // The host lock is given up while waiting (the other ranks must reach
    // the barrier) and taken back before returning.
    bool barrier() {
        const bool held = (t_held == this);
        if (held) host.unlock();
        const bool ok = wait_all_ranks();
        if (held) host.lock();
        return ok;
    }

  private:
    bool wait_all_ranks() {
        std::unique_lock<std::mutex> lk(m);
        if (broken) return false;
        const unsigned long long my = gen;
        if (++arrived == size) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::seconds(timeout_s),
                                    [&] { return gen != my || broken; });
        if (!ok || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

__attribute__((visibility("hidden"))) void group_host_enter(hip_proj_group* g) {
    if (!g) return;
    if (t_depth++ == 0) {
        g->host.lock();
        t_held = g;
    }
}

__attribute__((visibility("hidden"))) void group_host_leave(hip_proj_group* g) {
    if (!g) return;
    if (--t_depth == 0) {
        t_held = nullptr;
        g->host.unlock();
    }
}

namespace {

struct LocalComm final : SlabComm {
    hip_proj_group* G = nullptr;
    hip_proj_group* host_group() override { return G; }

    cfd_status_t meet() {
        if (!G->barrier()) return fail(CFD_ERROR, "in-process group barrier timed out", nullptr);
        return CFD_SUCCESS;
    }
    cfd_status_t wait_all(hipStream_t s, const std::vector<hipEvent_t>& ev) {
        for (int r = 0; r < size; ++r)
            if (r != rank) HIPC(hipStreamWaitEvent(s, ev[r], 0));
        return CFD_SUCCESS;
    }
    cfd_status_t halo(hipStream_t s, double* const* f, int nf, long long ps, int nz,
                      bool periodic) override {
        if (size == 1) return CFD_SUCCESS;
        const int lo = lower(periodic), hi = upper(periodic);
        G->pubf[rank] = f;
        G->pubnz[rank] = nz;
        HIPC(hipEventRecord(G->ev_ready[rank], s));
        cfd_status_t st = meet();
        if (st != CFD_SUCCESS) return st;
        if (lo >= 0) HIPC(hipStreamWaitEvent(s, G->ev_ready[lo], 0));
        if (hi >= 0 && hi != lo) HIPC(hipStreamWaitEvent(s, G->ev_ready[hi], 0));
        const size_t bytes = (size_t)ps * sizeof(double);
        for (int q = 0; q < nf; ++q) {
            if (lo >= 0) {
                const double* src = G->pubf[lo][q] + ps * (G->pubnz[lo] - 2);
                HIPC(hipMemcpyAsync(f[q], src, bytes, hipMemcpyDeviceToDevice, s));
            }
            if (hi >= 0) {
                const double* src = G->pubf[hi][q] + ps;
                HIPC(hipMemcpyAsync(f[q] + ps * (nz - 1), src, bytes, hipMemcpyDeviceToDevice, s));
            }
        }
        HIPC(hipEventRecord(G->ev_done[rank], s));
        if ((st = meet()) != CFD_SUCCESS) return st;
        // peers pulled from our owned planes; do not overwrite them before that
        if (lo >= 0) HIPC(hipStreamWaitEvent(s, G->ev_done[lo], 0));
        if (hi >= 0 && hi != lo) HIPC(hipStreamWaitEvent(s, G->ev_done[hi], 0));
        return CFD_SUCCESS;
    }
    template <typename K>
    cfd_status_t reduce(hipStream_t s, const void* in, K launch) {
        G->pub[rank] = in;
        HIPC(hipEventRecord(G->ev_ready[rank], s));
        cfd_status_t st = meet();
        if (st != CFD_SUCCESS) return st;
        if ((st = wait_all(s, G->ev_ready)) != CFD_SUCCESS) return st;
        GroupPtrs ptrs{};
        ptrs.n = size;
        for (int r = 0; r < size; ++r) ptrs.p[r] = G->pub[r];
        launch(ptrs);
        HIPC(hipGetLastError());
        HIPC(hipEventRecord(G->ev_done[rank], s));
        if ((st = meet()) != CFD_SUCCESS) return st;
        return wait_all(s, G->ev_done);
    }
    cfd_status_t allreduce_sum(hipStream_t s, const double* in, double* out, int n) override {
        return reduce(s, in, [&](const GroupPtrs& p) {
            hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(64), 0, s, p, out, n);
        });
    }
    cfd_status_t allreduce_max_u64(hipStream_t s, const unsigned long long* in,
                                   unsigned long long* out, int n) override {
        return reduce(s, in, [&](const GroupPtrs& p) {
            hipLaunchKernelGGL(k_group_max_u64, dim3(1), dim3(64), 0, s, p, out, n);
        });
    }
};

}  // namespace

extern "C" {

cfd_status_t hip_proj_comm_unique_id(unsigned char id[HIP_PROJ_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == HIP_PROJ_UNIQUE_ID_BYTES, "ncclUniqueId size");
    if (!id) return CFD_ERROR_INVALID;
    ncclUniqueId u;
    NCCLC(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return CFD_SUCCESS;
}

hip_proj_comm_t* hip_proj_comm_create_rccl(const unsigned char id[HIP_PROJ_UNIQUE_ID_BYTES],
                                           int rank, int size, int device) {
    if (!id || size < 1 || rank < 0 || rank >= size) {
        fail(CFD_ERROR_INVALID, "bad rank/size", nullptr);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        fail(CFD_ERROR, "hipSetDevice failed", nullptr);
        return nullptr;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    auto* c = new RcclComm();
    c->rank = rank;
    c->size = size;
    c->device = device;
    ncclResult_t r = ncclCommInitRank(&c->comm, size, u, rank);
    if (r != ncclSuccess) {
        fail(CFD_ERROR, "ncclCommInitRank", ncclGetErrorString(r));
        c->comm = nullptr;
        delete c;
        return nullptr;
    }
    r = ncclCommSplit(c->comm, 0, rank, &c->hcomm, nullptr);
    if (r != ncclSuccess) {
        fail(CFD_ERROR, "ncclCommSplit", ncclGetErrorString(r));
        c->hcomm = nullptr;
        delete c;
        return nullptr;
    }
    // one-shot device all-reduce for the CG dots; default on, CFD_HIP_DEVICE_ALLREDUCE=0
    // keeps every dot on ncclAllReduce
    const char* mb = getenv("CFD_HIP_DEVICE_ALLREDUCE");
    if (size > 1 && size <= cfdhip::MBOX_MAX && !(mb && atoi(mb) == 0)) {
        const bool local_ok = (c->setup_mailbox() == CFD_SUCCESS);
        if (!mailbox_verified(c, local_ok)) {
            for (void* p : c->peer_open)
                if (p) hipIpcCloseMemHandle(p);
            c->peer_open.clear();
            if (c->d_mb) hipFree(c->d_mb);
            c->d_mb = nullptr;
            if (c->mbox) hipFree(c->mbox);
            c->mbox = nullptr;
            (void)hipGetLastError();
        }
    }
    auto* h = new hip_proj_comm();
    h->impl = c;
    return h;
}

hip_proj_group_t* hip_proj_group_create(int size) {
    if (size < 1 || size > GROUP_MAX) {
        fail(CFD_ERROR_INVALID, "group size must be 1..16", nullptr);
        return nullptr;
    }
    auto* g = new hip_proj_group();
    g->size = size;
    if (const char* t = getenv("CFD_HIP_GROUP_TIMEOUT_S")) g->timeout_s = std::max(1, atoi(t));
    g->ev_ready.assign(size, nullptr);
    g->ev_done.assign(size, nullptr);
    g->pub.assign(size, nullptr);
    g->pubf.assign(size, nullptr);
    g->pubnz.assign(size, 0);
    g->joined.assign(size, 0);
    return g;
}

void hip_proj_group_destroy(hip_proj_group_t* g) {
    if (!g) return;
    for (auto e : g->ev_ready)
        if (e) hipEventDestroy(e);
    for (auto e : g->ev_done)
        if (e) hipEventDestroy(e);
    delete g;
}

hip_proj_comm_t* hip_proj_comm_create_local(hip_proj_group_t* g, int rank, int device) {
    if (!g || rank < 0 || rank >= g->size || g->joined[rank]) {
        fail(CFD_ERROR_INVALID, "bad group rank", nullptr);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_ready[rank], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_done[rank], hipEventDisableTiming) != hipSuccess) {
        fail(CFD_ERROR, "event creation failed", nullptr);
        return nullptr;
    }
    // ranks on other devices read this one's buffers directly (best effort;
    // fails harmlessly when already enabled or on the same device)
    int ndev = 0;
    hipGetDeviceCount(&ndev);
    for (int d = 0; d < ndev; ++d) {
        int ok = 0;
        if (d != device && hipDeviceCanAccessPeer(&ok, device, d) == hipSuccess && ok) {
            hipDeviceEnablePeerAccess(d, 0);
            (void)hipGetLastError();
        }
    }
    g->joined[rank] = 1;
    auto* c = new LocalComm();
    c->G = g;
    c->rank = rank;
    c->size = g->size;
    c->device = device;
    auto* h = new hip_proj_comm();
    h->impl = c;
    return h;
}

void hip_proj_comm_destroy(hip_proj_comm_t* c) {
    if (!c) return;
    delete c->impl;
    delete c;
}

int hip_proj_comm_rank(const hip_proj_comm_t* c) { return c && c->impl ? c->impl->rank : -1; }
int hip_proj_comm_device_allreduce(const hip_proj_comm_t* c) {
    return (c && c->impl && c->impl->device_mailbox()) ? 1 : 0;
}
int hip_proj_comm_size(const hip_proj_comm_t* c) { return c && c->impl ? c->impl->size : 0; }

}  // extern "C"

// ---------------------------------------------------------------------------
// All-reduce microbenchmark (hip_proj_comm_mailbox_bench): the per-iteration
// price of the CG dot exchange, the piece of the N-rank budget (DESIGN.md
// section 5) that one GPU cannot time. Rank r contributes (r + 1 + i, 1) in
// all-reduce i; every result is checked against n (n + 1) / 2 + n i and n.
// ---------------------------------------------------------------------------
namespace {
__global__ void k_mbox_bench(cfdhip::Mbox* mb, int iters, int base, int* bad) {
    if (threadIdx.x != 0) return;
    const int n = mb->n, me = mb->rank;
    for (int i = 0; i < iters; ++i) {
        double a = 0.0, b = 0.0;
        if (!cfdhip::mbox_allreduce2(mb, (double)(me + 1 + base + i), 1.0, &a, &b)) {
            *bad = 2;  // a peer did not arrive within the mailbox's bound
            return;
        }
        const double ea = 0.5 * n * (n + 1) + (double)n * (double)(base + i);
        if (a != ea || b != (double)n) *bad = 1;
    }
}

__global__ void k_bench_set(double* v, int rank, int i) {
    if (threadIdx.x == 0) {
        v[0] = (double)(rank + 1 + i);
        v[1] = 1.0;
    }
}

__global__ void k_bench_check(const double* s, int n, int i, int* bad) {
    if (threadIdx.x == 0) {
        const double ea = 0.5 * n * (n + 1) + (double)n * (double)i;
        if (s[0] != ea || s[1] != (double)n) *bad = 1;
    }
}
}  // namespace

extern "C" cfd_status_t hip_proj_comm_mailbox_bench(hip_proj_comm_t* comm, int iters, int mode,
                                                    double* us) {
    if (us) *us = 0.0;
    if (!comm || !comm->impl || iters <= 0 || mode < 0 || mode > 2 || !us)
        return fail(CFD_ERROR_INVALID, "mailbox bench: bad arguments", nullptr);
    SlabComm* c = comm->impl;
    if (c->host_group())
        return fail(CFD_ERROR_UNSUPPORTED, "mailbox bench: RCCL communicators only", nullptr);
    cfdhip::Mbox* mb = c->device_mailbox();
    if (mode < 2 && !mb)
        return fail(CFD_ERROR_UNSUPPORTED, "mailbox bench: no device mailbox", nullptr);
    HIPC(hipSetDevice(c->device));
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    double* d = nullptr;
    int* bad = nullptr;
    cfd_status_t st = CFD_SUCCESS;
    float ms = 0.f;
    int hbad = 0;
    auto run = [&]() -> cfd_status_t {
        HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        HIPC(hipEventCreate(&e0));
        HIPC(hipEventCreate(&e1));
        HIPC(hipMalloc((void**)&d, 8 * sizeof(double)));
        HIPC(hipMalloc((void**)&bad, sizeof(int)));
        HIPC(hipMemsetAsync(bad, 0, sizeof(int), s));
        HIPC(hipMemsetAsync(d, 0, 8 * sizeof(double), s));
        // start together: one all-reduce over RCCL first (ranks meet there)
        cfd_status_t r = c->allreduce_sum(s, d, d + 4, 2);
        if (r != CFD_SUCCESS) return r;
        HIPC(hipStreamSynchronize(s));
        HIPC(hipEventRecord(e0, s));
        if (mode == 0) {
            hipLaunchKernelGGL(k_mbox_bench, dim3(1), dim3(64), 0, s, mb, iters, 0, bad);
        } else if (mode == 1) {
            for (int i = 0; i < iters; ++i)
                hipLaunchKernelGGL(k_mbox_bench, dim3(1), dim3(64), 0, s, mb, 1, i, bad);
        } else {
            for (int i = 0; i < iters; ++i) {
                hipLaunchKernelGGL(k_bench_set, dim3(1), dim3(64), 0, s, d, c->rank, i);
                if ((r = c->allreduce_sum(s, d, d + 2, 2)) != CFD_SUCCESS) return r;
                hipLaunchKernelGGL(k_bench_check, dim3(1), dim3(64), 0, s, d + 2, c->size, i, bad);
            }
        }
        HIPC(hipGetLastError());
        HIPC(hipEventRecord(e1, s));
        HIPC(hipStreamSynchronize(s));
        HIPC(hipEventElapsedTime(&ms, e0, e1));
        HIPC(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
        return CFD_SUCCESS;
    };
    st = run();
    if (bad) hipFree(bad);
    if (d) hipFree(d);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (s) hipStreamDestroy(s);
    if (st != CFD_SUCCESS) return st;
    if (hbad) return fail(CFD_ERROR, "mailbox bench: wrong sums or a lost peer", nullptr);
    *us = 1e3 * (double)ms / (double)iters;
    return CFD_SUCCESS;
}
