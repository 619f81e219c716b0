// stencil_mb4.hip -- scratch microbenchmark round 4 (not product code):
// y register blocking (RY rows per thread), 1-wave blocks, XCD-aware tiles,
// for sweep A (two stencil inputs, two outputs) and sweep B.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);               \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

struct G {
    int nx, ny, nz;
    long long px, ps;
    double cx, cy, cz;
};

__device__ __forceinline__ double wsum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}
__device__ __forceinline__ void wave_partial(double acc, double* part, int slot) {
    acc = wsum(acc);
    if ((threadIdx.x & 63) == 0) part[slot] = acc;
}
__device__ __forceinline__ double lap7(const G& g, double c, double xm, double xp, double ym,
                                       double yp, double zm, double zp) {
    return ((xp - 2.0 * c + xm) * g.cx) + ((yp - 2.0 * c + ym) * g.cy) + ((zp + zm - 2.0 * c) * g.cz);
}
__device__ __forceinline__ int tile_of(int b, int nt) {
    int q = nt / 8, rem = nt % 8;
    int x = b % 8, l = b / 8;
    int start = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    return start + l;
}
__device__ __forceinline__ double2 ld2(const double* p, long long i) {
    return *(const double2*)&p[i];
}
__device__ __forceinline__ double2 axpy2(double2 a, double b, double2 c) {
    return make_double2(a.x + b * c.x, a.y + b * c.y);
}

__global__ void s_r3w2(const double2* __restrict__ a, const double2* __restrict__ b,
                       const double2* __restrict__ c, double2* __restrict__ d,
                       double2* __restrict__ e) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    double2 x = a[i], y = b[i], z = c[i];
    d[i] = make_double2(x.x + 0.5 * y.x, x.y + 0.5 * y.y);
    e[i] = make_double2(z.x + 0.25 * y.x, z.y + 0.25 * y.y);
}
__global__ void s_r2w1(const double2* __restrict__ a, double2* __restrict__ b) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    double2 x = a[i], y = b[i];
    b[i] = make_double2(y.x + 0.5 * x.x, y.y + 0.5 * x.y);
}

// B with RY rows per thread; one wave per block; tile = 128 x RY
template <int RY>
__global__ __launch_bounds__(64) void b_ry(G g, int kc, int tx_n, int ty_n, int tz_n,
                                           const double* __restrict__ p, double* __restrict__ r,
                                           double ma, double* part) {
    double acc = 0;
    const int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x;
    const int t = tile_of(blockIdx.x, nt);
    const int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
    const int i0 = tx * 128 + 2 * lane;
    const int j0 = ty * RY;
    const int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
    const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
    const int ic = min(i0, g.nx - 2);
    // rows j0-1 .. j0+RY (RY+2 rows), clamped to the array
    double2 zm[RY], zc[RY];
    long long base = (long long)kb * g.ps + ic;
#pragma unroll
    for (int q = 0; q < RY; ++q) {
        int j = min(j0 + q, g.ny - 1);
        zm[q] = ld2(p, base - g.ps + (long long)j * g.px);
        zc[q] = ld2(p, base + (long long)j * g.px);
    }
    for (int k = kb; k < ke; ++k, base += g.ps) {
        double2 row[RY + 2];
#pragma unroll
        for (int q = 0; q < RY + 2; ++q) {
            int j = min(max(j0 - 1 + q, 0), g.ny - 1);
            row[q] = (q >= 1 && q <= RY) ? zc[q - 1] : ld2(p, base + (long long)j * g.px);
        }
        double2 zp[RY];
#pragma unroll
        for (int q = 0; q < RY; ++q) {
            int j = min(j0 + q, g.ny - 1);
            zp[q] = ld2(p, base + g.ps + (long long)j * g.px);
        }
#pragma unroll
        for (int q = 0; q < RY; ++q) {
            int j = j0 + q;
            double2 pc = zc[q];
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            long long idx = base + (long long)min(j, g.ny - 1) * g.px;
            if (lane == 0) left = (i0 >= 1) ? p[idx - 1] : 0.0;
            if (lane == 63) right = (i0 + 2 < g.nx) ? p[idx + 2] : 0.0;
            if (j >= 1 && j <= g.ny - 2 && i0 < g.nx) {
                double2 rr = ld2(r, idx);
                double Ap0 = -lap7(g, pc.x, left, pc.y, row[q].x, row[q + 2].x, zm[q].x, zp[q].x);
                double Ap1 = -lap7(g, pc.y, pc.x, right, row[q].y, row[q + 2].y, zm[q].y, zp[q].y);
                double2 rn;
                rn.x = in0 ? rr.x + ma * Ap0 : rr.x;
                rn.y = in1 ? rr.y + ma * Ap1 : rr.y;
                *(double2*)&r[idx] = rn;
                if (in0) acc += rn.x * rn.x;
                if (in1) acc += rn.y * rn.y;
            }
            zm[q] = zc[q];
            zc[q] = zp[q];
        }
    }
    wave_partial(acc, part, blockIdx.x);
}

// A with RY rows per thread; p = r + beta pold computed once per loaded point
template <int RY>
__global__ __launch_bounds__(64) void a_ry(G g, int kc, int tx_n, int ty_n, int tz_n,
                                           const double* __restrict__ r,
                                           const double* __restrict__ po,
                                           double* __restrict__ pn, double* __restrict__ x,
                                           double beta, double alpha, double* part) {
    double acc = 0;
    const int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x;
    const int t = tile_of(blockIdx.x, nt);
    const int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
    const int i0 = tx * 128 + 2 * lane;
    const int j0 = ty * RY;
    const int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
    const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
    const int ic = min(i0, g.nx - 2);
    double2 zm[RY], zc[RY], oc[RY];
    long long base = (long long)kb * g.ps + ic;
#pragma unroll
    for (int q = 0; q < RY; ++q) {
        int j = min(j0 + q, g.ny - 1);
        long long o = (long long)j * g.px;
        zm[q] = axpy2(ld2(r, base - g.ps + o), beta, ld2(po, base - g.ps + o));
        oc[q] = ld2(po, base + o);
        zc[q] = axpy2(ld2(r, base + o), beta, oc[q]);
    }
    for (int k = kb; k < ke; ++k, base += g.ps) {
        double2 ylo, yhi;
        {
            int jl = max(j0 - 1, 0), jh = min(j0 + RY, g.ny - 1);
            ylo = axpy2(ld2(r, base + (long long)jl * g.px), beta, ld2(po, base + (long long)jl * g.px));
            yhi = axpy2(ld2(r, base + (long long)jh * g.px), beta, ld2(po, base + (long long)jh * g.px));
        }
        double2 zp[RY], op[RY];
#pragma unroll
        for (int q = 0; q < RY; ++q) {
            long long o = (long long)min(j0 + q, g.ny - 1) * g.px;
            op[q] = ld2(po, base + g.ps + o);
            zp[q] = axpy2(ld2(r, base + g.ps + o), beta, op[q]);
        }
#pragma unroll
        for (int q = 0; q < RY; ++q) {
            int j = j0 + q;
            double2 pc = zc[q];
            double2 ys = (q == 0) ? ylo : zc[q - 1];
            double2 yn = (q == RY - 1) ? yhi : zc[q + 1];
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            long long idx = base + (long long)min(j, g.ny - 1) * g.px;
            if (lane == 0) left = (i0 >= 1) ? r[idx - 1] + beta * po[idx - 1] : 0.0;
            if (lane == 63) right = (i0 + 2 < g.nx) ? r[idx + 2] + beta * po[idx + 2] : 0.0;
            if (j >= 1 && j <= g.ny - 2 && i0 < g.nx) {
                double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, zm[q].x, zp[q].x);
                double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, zm[q].y, zp[q].y);
                double2 xo = ld2(x, idx);
                double2 pw, xw;
                pw.x = in0 ? pc.x : 0.0;
                pw.y = in1 ? pc.y : 0.0;
                xw.x = in0 ? xo.x + alpha * oc[q].x : xo.x;
                xw.y = in1 ? xo.y + alpha * oc[q].y : xo.y;
                *(double2*)&pn[idx] = pw;
                *(double2*)&x[idx] = xw;
                if (in0) acc += pc.x * Ap0;
                if (in1) acc += pc.y * Ap1;
            }
            zm[q] = zc[q];
            zc[q] = zp[q];
            oc[q] = op[q];
        }
    }
    wave_partial(acc, part, blockIdx.x);
}

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 512;
    int reps = argc > 2 ? atoi(argv[2]) : 20;
    G g;
    g.nx = g.ny = g.nz = n;
    g.px = n;
    g.ps = (long long)n * n;
    g.cx = g.cy = g.cz = 1.0;
    long long N = g.ps * n;
    double *p, *r, *r0, *part, *x, *pn;
    CK(hipMalloc(&p, N * 8));
    CK(hipMalloc(&r, N * 8));
    CK(hipMalloc(&r0, N * 8));
    CK(hipMalloc(&x, N * 8));
    CK(hipMalloc(&pn, N * 8));
    CK(hipMalloc(&part, 1 << 22));
    std::vector<double> h(N);
    for (long long q = 0; q < N; ++q) {
        long long i = q % n, j = (q / n) % n, k = q / g.ps;
        h[q] = (i == 0 || j == 0 || k == 0 || i == n - 1 || j == n - 1 || k == n - 1)
                   ? 0.0 : (double)((q * 2654435761ull) % 1000) * 1e-3;
    }
    CK(hipMemcpy(p, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(r0, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(r, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(x, h.data(), N * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double ncell = (double)(n - 2) * (n - 2) * (n - 2);
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int q = 0; q < reps; ++q) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-34s %9.4f ms %8.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    long long N2 = N / 2;
    timeit("stream r2w1", 24.0 * N, [&] { s_r2w1<<<N2 / 256, 256>>>((double2*)p, (double2*)r); });
    timeit("stream r3w2", 40.0 * N, [&] {
        s_r3w2<<<N2 / 256, 256>>>((double2*)p, (double2*)r0, (double2*)x, (double2*)pn, (double2*)r);
    });
    CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(x, r0, N * 8, hipMemcpyDeviceToDevice));
    const double ma = -1e-9;
    int txn = (n + 127) / 128;
#define RB(RY, KC)                                                                           \
    {                                                                                        \
        int tyn = (n + RY - 1) / RY, tzn = (n - 2 + KC - 1) / KC;                           \
        int nt = txn * tyn * tzn;                                                            \
        char name[80];                                                                       \
        snprintf(name, sizeof name, "B ry=%d kc=%d G=%d", RY, KC, nt);                       \
        timeit(name, 24.0 * ncell, [&] { b_ry<RY><<<nt, 64>>>(g, KC, txn, tyn, tzn, p, r, ma, part); }); \
    }
#define RA(RY, KC)                                                                           \
    {                                                                                        \
        int tyn = (n + RY - 1) / RY, tzn = (n - 2 + KC - 1) / KC;                           \
        int nt = txn * tyn * tzn;                                                            \
        char name[80];                                                                       \
        snprintf(name, sizeof name, "A ry=%d kc=%d G=%d", RY, KC, nt);                       \
        timeit(name, 40.0 * ncell, [&] { a_ry<RY><<<nt, 64>>>(g, KC, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); }); \
    }
    RB(1, 510);
    RB(2, 510);
    RB(4, 510);
    RB(8, 510);
    RB(2, 255);
    RB(4, 255);
    RB(4, 128);
    RA(1, 510);
    RA(2, 510);
    RA(4, 510);
    RA(8, 510);
    RA(1, 255);
    RA(2, 255);
    RA(4, 255);
    RA(4, 128);
    RA(8, 255);
    // correctness: A and B results against a scalar host recompute on a sample
    {
        std::vector<double> hp(N), hr(N);
        CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
        int tyn = (n + 3) / 4, tzn = 1;
        b_ry<4><<<txn * tyn * tzn, 64>>>(g, 510, txn, tyn, tzn, p, r, -0.5, part);
        CK(hipMemcpy(hr.data(), r, N * 8, hipMemcpyDeviceToHost));
        double maxd = 0;
        for (long long q = 0; q < N; q += 997) {
            long long i = q % n, j = (q / n) % n, k = q / g.ps;
            if (i == 0 || j == 0 || k == 0 || i == n - 1 || j == n - 1 || k == n - 1) continue;
            double c = h[q];
            double lap = ((h[q + 1] - 2.0 * c + h[q - 1])) + ((h[q + n] - 2.0 * c + h[q - n])) +
                         ((h[q + g.ps] + h[q - g.ps] - 2.0 * c));
            double want = h[q] + (-0.5) * (-lap);
            maxd = std::max(maxd, std::abs(want - hr[q]));
        }
        printf("check B ry4 maxdiff %.3e\n", maxd);
    }
    return 0;
}
