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

// NI streamed inputs, NO streamed outputs (r03): out_o = sum of the inputs
// scaled by (o + 1); the roof of a kernel with that stream mix (the
// predictor: 3 / 3, the corrector: 4 / 3, the CG sweeps: 2 / 1).
constexpr int NM_MAX = 8;
struct Ptrs {
    double2* p[NM_MAX];
};

template <int NI, int NO, int U>
__global__ __launch_bounds__(256) void k_stream_nm(Ptrs in, Ptrs out, size_t n2) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    double2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = make_double2(0.0, 0.0);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            const double2 v = i < n2 ? in.p[q][i] : make_double2(0.0, 0.0);
            acc[u].x += v.x;
            acc[u].y += v.y;
        }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n2) out.p[o][i] = make_double2(acc[u].x * (o + 1), acc[u].y * (o + 1));
        }
    }
}

template <int NI, int NO>
void launch_nm(int u, hipStream_t s, const Ptrs& in, const Ptrs& out, size_t n2) {
    auto go = [&](auto kern, int uu) {
        const unsigned g = (unsigned)((n2 + 256 * uu - 1) / (256 * uu));
        hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, s, in, out, n2);
    };
    if (u == 1) go(k_stream_nm<NI, NO, 1>, 1);
    else if (u == 2) go(k_stream_nm<NI, NO, 2>, 2);
    else go(k_stream_nm<NI, NO, 4>, 4);
}

bool nm_u(int ni, int no, int u, hipStream_t s, const Ptrs& in, const Ptrs& out, size_t n2) {
#define NM_CASE(I, O) \
    if (ni == I && no == O) return launch_nm<I, O>(u, s, in, out, n2), true;
    NM_CASE(1, 1) NM_CASE(2, 1) NM_CASE(3, 1) NM_CASE(2, 2) NM_CASE(3, 3) NM_CASE(4, 3)
    NM_CASE(4, 4) NM_CASE(5, 3)
#undef NM_CASE
    return false;
}

}  // namespace

// Streamed fp64 arrays of n elements each, `ni` read and `no` written per
// element (built pairs: 1/1, 2/1, 3/1, 2/2, 3/3, 4/3, 4/4, 5/3); best of
// `reps` timed rounds over 1-4 loads per lane, bytes (ni + no) x 8 per element.
extern "C" cfd_status_t cfd_hip_stream_bench_nm(int device, size_t n, int ni, int no, int reps,
                                                double* gbps) {
    if (!gbps || n < 2 || reps < 1 || ni < 1 || no < 1 || ni > 5 || no > 4) return CFD_ERROR_INVALID;
    *gbps = 0.0;
    if (hipSetDevice(device) != hipSuccess) return CFD_ERROR_UNSUPPORTED;
    const size_t n2 = n / 2;
    Ptrs in{}, out{};
    double2* bufs[NM_MAX] = {};
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    cfd_status_t st = CFD_ERROR;
    bool ok = hipStreamCreate(&s) == hipSuccess && hipEventCreate(&e0) == hipSuccess &&
              hipEventCreate(&e1) == hipSuccess;
    for (int q = 0; q < ni + no && ok; ++q) {
        ok = hipMalloc(&bufs[q], n2 * sizeof(double2)) == hipSuccess;
        if (ok) hipLaunchKernelGGL(k_stream_init, dim3(2048), dim3(256), 0, s, bufs[q], bufs[q],
                                   bufs[q], n2);
    }
    if (ok) {
        for (int q = 0; q < ni; ++q) in.p[q] = bufs[q];
        for (int o = 0; o < no; ++o) out.p[o] = bufs[ni + o];
        double best = 1e30;
        for (int u = 1; u <= 4 && ok; u *= 2) {
            for (int r = 0; r < reps + 1 && ok; ++r) {
                float ms = 0.f;
                hipEventRecord(e0, s);
                ok = nm_u(ni, no, u, s, in, out, n2);
                hipEventRecord(e1, s);
                ok = ok && hipEventSynchronize(e1) == hipSuccess &&
                     hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
                if (ok && r > 0) best = std::min(best, (double)ms);
            }
        }
        if (ok) {
            *gbps = (double)(ni + no) * (double)(2 * n2) * sizeof(double) / (best * 1e-3) / 1e9;
            st = CFD_SUCCESS;
        } else {
            st = CFD_ERROR_INVALID;
        }
    }
    for (double2* b : bufs)
        if (b) hipFree(b);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (s) hipStreamDestroy(s);
    return st;
}

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
