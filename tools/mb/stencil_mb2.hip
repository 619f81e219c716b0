// stencil_mb2.hip -- scratch microbenchmark round 2 (not product code):
// better STREAM references and x-vectorised stencil variants.
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
template <int NT>
__device__ __forceinline__ void block_partial(double acc, double* part) {
    __shared__ double sh[NT / 64];
    acc = wsum(acc);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0;
        for (int w = 0; w < NT / 64; ++w) s += sh[w];
        part[blockIdx.x] = s;
    }
}
__device__ __forceinline__ double lap7(const G& g, double c, double xm, double xp, double ym,
                                       double yp, double zm, double zp) {
    return ((xp - 2.0 * c + xm) * g.cx) + ((yp - 2.0 * c + ym) * g.cy) + ((zp + zm - 2.0 * c) * g.cz);
}

// STREAM: one 16-B element per thread, no loop
__global__ void s_copy16_flat(const double2* __restrict__ a, double2* __restrict__ b) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    b[i] = a[i];
}
// STREAM: U 16-B elements per thread, block-contiguous chunks
template <int U>
__global__ void s_copy16_unroll(const double2* __restrict__ a, double2* __restrict__ b) {
    long long base = (long long)blockIdx.x * blockDim.x * U + threadIdx.x;
    double2 v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = a[base + q * blockDim.x];
#pragma unroll
    for (int q = 0; q < U; ++q) b[base + q * blockDim.x] = v[q];
}
__global__ void s_copy16_nt(const double2* __restrict__ a, double2* __restrict__ b) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    double2 v;
    v.x = __builtin_nontemporal_load(&a[i].x);
    v.y = __builtin_nontemporal_load(&a[i].y);
    __builtin_nontemporal_store(v.x, &b[i].x);
    __builtin_nontemporal_store(v.y, &b[i].y);
}
__global__ void s_read16(const double2* __restrict__ a, double* out) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    double2 v = a[i];
    double s = wsum(v.x + v.y);
    if ((threadIdx.x & 63) == 0 && s == 12345.678) out[0] = s;
}
__global__ void s_triad16(const double2* __restrict__ a, const double2* __restrict__ c,
                          double2* __restrict__ b, double s) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    double2 x = a[i], y = c[i];
    b[i] = make_double2(x.x + s * y.x, x.y + s * y.y);
}

// v2: 2 cells/thread (double2), tile 128 x 4, z-march (from round 1)
template <bool NT_STORE>
__global__ __launch_bounds__(256) void v2(G g, int kc, int tx_n, int ty_n, int tz_n,
                                          const double* __restrict__ p, double* __restrict__ r,
                                          double ma, double* part) {
    double acc = 0;
    int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x & 63;
    for (int t = blockIdx.x; t < nt; t += gridDim.x) {
        int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
        int i0 = tx * 128 + 2 * lane;
        int j = ty * 4 + (threadIdx.x >> 6);
        int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
        if (!((j >= 1 && j <= g.ny - 2) && (i0 < g.nx))) continue;
        long long idx = kb * g.ps + j * g.px + i0;
        double2 pm = *(const double2*)&p[idx - g.ps];
        double2 pc = *(const double2*)&p[idx];
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 pp = *(const double2*)&p[idx + g.ps];
            double2 ys = *(const double2*)&p[idx - g.px];
            double2 yn = *(const double2*)&p[idx + g.px];
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = (i0 >= 1) ? p[idx - 1] : 0.0;
            if (lane == 63) right = (i0 + 2 < g.nx) ? p[idx + 2] : 0.0;
            double2 rr = *(const double2*)&r[idx];
            double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
            double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
            double2 rn;
            bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
            rn.x = in0 ? rr.x + ma * Ap0 : rr.x;
            rn.y = in1 ? rr.y + ma * Ap1 : rr.y;
            if (NT_STORE) {
                __builtin_nontemporal_store(rn.x, &r[idx]);
                __builtin_nontemporal_store(rn.y, &r[idx + 1]);
            } else {
                *(double2*)&r[idx] = rn;
            }
            if (in0) acc += rn.x * rn.x;
            if (in1) acc += rn.y * rn.y;
            pm = pc;
            pc = pp;
        }
    }
    block_partial<256>(acc, part);
}

// v4: 4 cells/thread (two double2 per row), tile 256 x 4
__global__ __launch_bounds__(256) void v4(G g, int kc, int tx_n, int ty_n, int tz_n,
                                          const double* __restrict__ p, double* __restrict__ r,
                                          double ma, double* part) {
    double acc = 0;
    int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x & 63;
    for (int t = blockIdx.x; t < nt; t += gridDim.x) {
        int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
        int i0 = tx * 256 + 2 * lane;   // cells i0, i0+1 and i0+128, i0+129
        int j = ty * 4 + (threadIdx.x >> 6);
        int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
        if (!((j >= 1 && j <= g.ny - 2) && (i0 < g.nx))) continue;
        long long idx = kb * g.ps + j * g.px + i0;
        double2 pm[2], pc[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            pm[h] = *(const double2*)&p[idx + 128 * h - g.ps];
            pc[h] = *(const double2*)&p[idx + 128 * h];
        }
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 pp[2], ys[2], yn[2], rr[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                pp[h] = *(const double2*)&p[idx + 128 * h + g.ps];
                ys[h] = *(const double2*)&p[idx + 128 * h - g.px];
                yn[h] = *(const double2*)&p[idx + 128 * h + g.px];
                rr[h] = *(const double2*)&r[idx + 128 * h];
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int ii = i0 + 128 * h;
                double left = __shfl_up(pc[h].y, 1, 64);
                double right = __shfl_down(pc[h].x, 1, 64);
                if (lane == 0) left = (ii >= 1) ? p[idx + 128 * h - 1] : 0.0;
                if (lane == 63) right = (ii + 2 < g.nx) ? p[idx + 128 * h + 2] : 0.0;
                double Ap0 = -lap7(g, pc[h].x, left, pc[h].y, ys[h].x, yn[h].x, pm[h].x, pp[h].x);
                double Ap1 = -lap7(g, pc[h].y, pc[h].x, right, ys[h].y, yn[h].y, pm[h].y, pp[h].y);
                bool in0 = (ii >= 1 && ii <= g.nx - 2), in1 = (ii + 1 <= g.nx - 2);
                double2 rn;
                rn.x = in0 ? rr[h].x + ma * Ap0 : rr[h].x;
                rn.y = in1 ? rr[h].y + ma * Ap1 : rr[h].y;
                if (ii < g.nx) *(double2*)&r[idx + 128 * h] = rn;
                if (in0) acc += rn.x * rn.x;
                if (in1) acc += rn.y * rn.y;
                pm[h] = pc[h];
                pc[h] = pp[h];
            }
        }
    }
    block_partial<256>(acc, part);
}

// v5: v2 with two planes per loop trip (more loads in flight)
__global__ __launch_bounds__(256) void v5(G g, int kc, int tx_n, int ty_n, int tz_n,
                                          const double* __restrict__ p, double* __restrict__ r,
                                          double ma, double* part) {
    double acc = 0;
    int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x & 63;
    for (int t = blockIdx.x; t < nt; t += gridDim.x) {
        int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
        int i0 = tx * 128 + 2 * lane;
        int j = ty * 4 + (threadIdx.x >> 6);
        int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
        if (!((j >= 1 && j <= g.ny - 2) && (i0 < g.nx))) continue;
        const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
        long long idx = kb * g.ps + j * g.px + i0;
        double2 pm = *(const double2*)&p[idx - g.ps];
        double2 pc = *(const double2*)&p[idx];
        int k = kb;
        for (; k + 1 < ke; k += 2, idx += 2 * g.ps) {
            double2 pp = *(const double2*)&p[idx + g.ps];
            double2 pq = *(const double2*)&p[idx + 2 * g.ps];
            double2 ys0 = *(const double2*)&p[idx - g.px];
            double2 yn0 = *(const double2*)&p[idx + g.px];
            double2 ys1 = *(const double2*)&p[idx + g.ps - g.px];
            double2 yn1 = *(const double2*)&p[idx + g.ps + g.px];
            double2 r0 = *(const double2*)&r[idx];
            double2 r1 = *(const double2*)&r[idx + g.ps];
            double l0 = __shfl_up(pc.y, 1, 64), rt0 = __shfl_down(pc.x, 1, 64);
            double l1 = __shfl_up(pp.y, 1, 64), rt1 = __shfl_down(pp.x, 1, 64);
            if (lane == 0) {
                l0 = (i0 >= 1) ? p[idx - 1] : 0.0;
                l1 = (i0 >= 1) ? p[idx + g.ps - 1] : 0.0;
            }
            if (lane == 63) {
                rt0 = (i0 + 2 < g.nx) ? p[idx + 2] : 0.0;
                rt1 = (i0 + 2 < g.nx) ? p[idx + g.ps + 2] : 0.0;
            }
            double a0 = -lap7(g, pc.x, l0, pc.y, ys0.x, yn0.x, pm.x, pp.x);
            double a1 = -lap7(g, pc.y, pc.x, rt0, ys0.y, yn0.y, pm.y, pp.y);
            double b0 = -lap7(g, pp.x, l1, pp.y, ys1.x, yn1.x, pc.x, pq.x);
            double b1 = -lap7(g, pp.y, pp.x, rt1, ys1.y, yn1.y, pc.y, pq.y);
            double2 n0, n1;
            n0.x = in0 ? r0.x + ma * a0 : r0.x;
            n0.y = in1 ? r0.y + ma * a1 : r0.y;
            n1.x = in0 ? r1.x + ma * b0 : r1.x;
            n1.y = in1 ? r1.y + ma * b1 : r1.y;
            *(double2*)&r[idx] = n0;
            *(double2*)&r[idx + g.ps] = n1;
            if (in0) acc += n0.x * n0.x;
            if (in1) acc += n0.y * n0.y;
            if (in0) acc += n1.x * n1.x;
            if (in1) acc += n1.y * n1.y;
            pm = pp;
            pc = pq;
        }
        for (; k < ke; ++k, idx += g.ps) {
            double2 pp = *(const double2*)&p[idx + g.ps];
            double2 ys = *(const double2*)&p[idx - g.px];
            double2 yn = *(const double2*)&p[idx + g.px];
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = (i0 >= 1) ? p[idx - 1] : 0.0;
            if (lane == 63) right = (i0 + 2 < g.nx) ? p[idx + 2] : 0.0;
            double2 rr = *(const double2*)&r[idx];
            double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
            double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
            double2 rn;
            rn.x = in0 ? rr.x + ma * Ap0 : rr.x;
            rn.y = in1 ? rr.y + ma * Ap1 : rr.y;
            *(double2*)&r[idx] = rn;
            if (in0) acc += rn.x * rn.x;
            if (in1) acc += rn.y * rn.y;
            pm = pc;
            pc = pp;
        }
    }
    block_partial<256>(acc, part);
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
    double *p, *r, *r0, *part;
    CK(hipMalloc(&p, N * 8));
    CK(hipMalloc(&r, N * 8));
    CK(hipMalloc(&r0, N * 8));
    CK(hipMalloc(&part, 1 << 20));
    std::vector<double> h(N);
    for (long long q = 0; q < N; ++q) {
        long long i = q % n, j = (q / n) % n, k = q / g.ps;
        h[q] = (i == 0 || j == 0 || k == 0 || i == n - 1 || j == n - 1 || k == n - 1)
                   ? 0.0 : (double)((q * 2654435761ull) % 1000) * 1e-3;
    }
    CK(hipMemcpy(p, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(r0, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(r, h.data(), N * 8, hipMemcpyHostToDevice));
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
        printf("%-30s %9.4f ms %8.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    long long N2 = N / 2;
    double2 *a2 = (double2*)p, *b2 = (double2*)r, *c2 = (double2*)r0;
    timeit("copy16 flat", 16.0 * N, [&] { s_copy16_flat<<<N2 / 256, 256>>>(a2, b2); });
    timeit("copy16 flat 512thr", 16.0 * N, [&] { s_copy16_flat<<<N2 / 512, 512>>>(a2, b2); });
    timeit("copy16 unroll4", 16.0 * N, [&] { s_copy16_unroll<4><<<N2 / 1024, 256>>>(a2, b2); });
    timeit("copy16 unroll8", 16.0 * N, [&] { s_copy16_unroll<8><<<N2 / 2048, 256>>>(a2, b2); });
    timeit("copy16 nt", 16.0 * N, [&] { s_copy16_nt<<<N2 / 256, 256>>>(a2, b2); });
    timeit("read16", 8.0 * N, [&] { s_read16<<<N2 / 256, 256>>>(a2, part); });
    timeit("triad16 flat", 24.0 * N, [&] { s_triad16<<<N2 / 256, 256>>>(a2, c2, b2, 0.5); });
    CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
    const double ma = -1e-9;
    int tyn = (n + 3) / 4;
    for (int kc : {32, 64, 128, 510}) {
        int tzn = (n - 2 + kc - 1) / kc;
        int txn2 = (n + 127) / 128, txn4 = (n + 255) / 256;
        for (int gcap : {2048, 4096, 8192}) {
            char name[64];
            int grid = std::min(txn2 * tyn * tzn, gcap);
            snprintf(name, sizeof name, "v2 kc=%d G=%d", kc, grid);
            timeit(name, 24.0 * ncell, [&] { v2<false><<<grid, 256>>>(g, kc, txn2, tyn, tzn, p, r, ma, part); });
        }
        char name[64];
        int grid = std::min(txn2 * tyn * tzn, 4096);
        snprintf(name, sizeof name, "v2nt kc=%d", kc);
        timeit(name, 24.0 * ncell, [&] { v2<true><<<grid, 256>>>(g, kc, txn2, tyn, tzn, p, r, ma, part); });
        grid = std::min(txn4 * tyn * tzn, 4096);
        snprintf(name, sizeof name, "v4 kc=%d", kc);
        timeit(name, 24.0 * ncell, [&] { v4<<<grid, 256>>>(g, kc, txn4, tyn, tzn, p, r, ma, part); });
        grid = std::min(txn2 * tyn * tzn, 4096);
        snprintf(name, sizeof name, "v5 kc=%d", kc);
        timeit(name, 24.0 * ncell, [&] { v5<<<grid, 256>>>(g, kc, txn2, tyn, tzn, p, r, ma, part); });
    }
    auto check = [&](const char* name) {
        std::vector<double> out(N);
        CK(hipMemcpy(out.data(), r, N * 8, hipMemcpyDeviceToHost));
        double s = 0;
        for (long long q = 0; q < N; q += 7) s += out[q];
        printf("   check %s %.12e\n", name, s);
    };
    int kc = 64, tzn = (n - 2 + kc - 1) / kc;
    CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
    v2<false><<<4096, 256>>>(g, kc, (n + 127) / 128, tyn, tzn, p, r, -0.5, part);
    check("v2");
    CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
    v4<<<4096, 256>>>(g, kc, (n + 255) / 256, tyn, tzn, p, r, -0.5, part);
    check("v4");
    CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
    v5<<<4096, 256>>>(g, kc, (n + 127) / 128, tyn, tzn, p, r, -0.5, part);
    check("v5");
    return 0;
}
