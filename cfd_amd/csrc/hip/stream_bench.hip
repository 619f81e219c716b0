// stream_bench.hip -- BabelStream-style copy and triad on the device, in the
// same library as the CG sweeps, so bench.py can report the measured HBM
// roof beside the 8 TB/s spec (SURVEY.md §8d "Run a BabelStream-style triad
// in the same binary and report both").
//
// fp64 arrays of n elements, 16-B lanes (double2, the width the sweeps use),
// flat grids with 1-8 independent 16-B loads per thread (best reported). Bytes counted
// as BabelStream does: copy 2 x 8 B, triad 3 x 8 B per element.
#include "cfd_hip/projection_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace {

__global__ __launch_bounds__(256) void k_stream_init(double2* a, double2* b, double2* c,
                                                     size_t n2) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2;
         i += (size_t)gridDim.x * blockDim.x) {
        a[i] = make_double2(1.0, 1.0);
        b[i] = make_double2(2.0, 2.0);
        c[i] = make_double2(0.0, 0.0);
    }
}

// One block covers 256 * U consecutive double2: U independent 16-B loads per
// thread in flight before the stores (a flat grid, no grid-stride loop).
template <int U>
__global__ __launch_bounds__(256) void k_stream_copy(const double2* __restrict__ a,
                                                     double2* __restrict__ c, size_t n2) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    double2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        v[u] = i < n2 ? a[i] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n2) c[i] = v[u];
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_stream_triad(double2* __restrict__ a,
                                                      const double2* __restrict__ b,
                                                      const double2* __restrict__ c,
                                                      double s, size_t n2) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    double2 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        x[u] = i < n2 ? b[i] : make_double2(0.0, 0.0);
        y[u] = i < n2 ? c[i] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n2) a[i] = make_double2(x[u].x + s * y[u].x, x[u].y + s * y[u].y);
    }
}

template <int U>
void launch_copy(hipStream_t s, const double2* a, double2* c, size_t n2) {
    const unsigned g = (unsigned)((n2 + 256 * U - 1) / (256 * U));
    hipLaunchKernelGGL(k_stream_copy<U>, dim3(g), dim3(256), 0, s, a, c, n2);
}

template <int U>
void launch_triad(hipStream_t s, double2* a, const double2* b, const double2* c, size_t n2) {
    const unsigned g = (unsigned)((n2 + 256 * U - 1) / (256 * U));
    hipLaunchKernelGGL(k_stream_triad<U>, dim3(g), dim3(256), 0, s, a, b, c, 0.4, n2);
}

void copy_u(int u, hipStream_t s, const double2* a, double2* c, size_t n2) {
    switch (u) {
        case 1: return launch_copy<1>(s, a, c, n2);
        case 2: return launch_copy<2>(s, a, c, n2);
        case 4: return launch_copy<4>(s, a, c, n2);
        default: return launch_copy<8>(s, a, c, n2);
    }
}

void triad_u(int u, hipStream_t s, double2* a, const double2* b, const double2* c, size_t n2) {
    switch (u) {
        case 1: return launch_triad<1>(s, a, b, c, n2);
        case 2: return launch_triad<2>(s, a, b, c, n2);
        case 4: return launch_triad<4>(s, a, b, c, n2);
        default: return launch_triad<8>(s, a, b, c, n2);
    }
}

}  // namespace

extern "C" cfd_status_t cfd_hip_stream_bench(int device, size_t n, int reps, double* copy_gbps,
                                             double* triad_gbps) {
    if (!copy_gbps || !triad_gbps || n < 2 || reps < 1) return CFD_ERROR_INVALID;
    *copy_gbps = *triad_gbps = 0.0;
    if (hipSetDevice(device) != hipSuccess) return CFD_ERROR_UNSUPPORTED;
    const size_t n2 = n / 2;
    double2 *a = nullptr, *b = nullptr, *c = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    cfd_status_t st = CFD_ERROR;
    const unsigned grid = 2048;  // init only
    if (hipMalloc(&a, n2 * sizeof(double2)) == hipSuccess &&
        hipMalloc(&b, n2 * sizeof(double2)) == hipSuccess &&
        hipMalloc(&c, n2 * sizeof(double2)) == hipSuccess &&
        hipStreamCreate(&s) == hipSuccess && hipEventCreate(&e0) == hipSuccess &&
        hipEventCreate(&e1) == hipSuccess) {
        hipLaunchKernelGGL(k_stream_init, dim3(grid), dim3(256), 0, s, a, b, c, n2);
        // the roof is the best over unroll depths 1..8 and `reps` rounds each
        double best_copy = 1e30, best_triad = 1e30;
        bool ok = true;
        for (int u = 1; u <= 8 && ok; u *= 2) {
            for (int r = 0; r < reps + 1 && ok; ++r) {  // first round is warm-up
                float ms = 0.f;
                hipEventRecord(e0, s);
                copy_u(u, s, a, c, n2);
                hipEventRecord(e1, s);
                ok = hipEventSynchronize(e1) == hipSuccess &&
                     hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
                if (ok && r > 0) best_copy = std::min(best_copy, (double)ms);
                hipEventRecord(e0, s);
                triad_u(u, s, a, b, c, n2);
                hipEventRecord(e1, s);
                ok = ok && hipEventSynchronize(e1) == hipSuccess &&
                     hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
                if (ok && r > 0) best_triad = std::min(best_triad, (double)ms);
            }
        }
        if (ok) {
            const double bytes = (double)(2 * n2) * sizeof(double);
            *copy_gbps = 2.0 * bytes / (best_copy * 1e-3) / 1e9;
            *triad_gbps = 3.0 * bytes / (best_triad * 1e-3) / 1e9;
            st = CFD_SUCCESS;
        }
    }
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (s) hipStreamDestroy(s);
    hipFree(a);
    hipFree(b);
    hipFree(c);
    return st;
}
