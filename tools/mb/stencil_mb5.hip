// stencil_mb5.hip -- scratch microbenchmark round 5 (not product code):
// one-wave blocks, 16-B lanes, XCD-aware tiles; z chunk sweep and a
// software-pipelined variant that loads plane k+2 while computing plane k.
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

// Sweep B, one wave per block, tile 128 x 1 x kc. PF: prefetch next plane.
template <bool PF>
__global__ __launch_bounds__(64) void kb_(G g, int kc, int tx_n, int ty_n, int tz_n,
                                          const double* __restrict__ p, double* __restrict__ r,
                                          double ma, double* part) {
    const int nt = tx_n * ty_n * tz_n;
    const int t = tile_of(blockIdx.x, nt);
    const int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
    const int lane = threadIdx.x;
    const int i0 = tx * 128 + 2 * lane;
    const int j = ty;
    const int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
    double acc = 0;
    if (j >= 1 && j <= g.ny - 2 && i0 < g.nx) {
        const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
        long long idx = kb * g.ps + j * g.px + i0;
        double2 pm = ld2(p, idx - g.ps), pc = ld2(p, idx);
        double2 pp = ld2(p, idx + g.ps), ys = ld2(p, idx - g.px), yn = ld2(p, idx + g.px);
        double2 rr = ld2(r, idx);
        double el = (lane == 0 && i0 >= 1) ? p[idx - 1] : 0.0;
        double er = (lane == 63 && i0 + 2 < g.nx) ? p[idx + 2] : 0.0;
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 pp2, ys2, yn2, rr2;
            double el2 = 0, er2 = 0;
            if (PF && k + 1 < ke) {
                long long n = idx + g.ps;
                pp2 = ld2(p, n + g.ps);
                ys2 = ld2(p, n - g.px);
                yn2 = ld2(p, n + g.px);
                rr2 = ld2(r, n);
                if (lane == 0 && i0 >= 1) el2 = p[n - 1];
                if (lane == 63 && i0 + 2 < g.nx) er2 = p[n + 2];
            }
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = el;
            if (lane == 63) right = er;
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
            if (PF) {
                pp = pp2; ys = ys2; yn = yn2; rr = rr2; el = el2; er = er2;
            } else if (k + 1 < ke) {
                long long n = idx + g.ps;
                pp = ld2(p, n + g.ps);
                ys = ld2(p, n - g.px);
                yn = ld2(p, n + g.px);
                rr = ld2(r, n);
                el = (lane == 0 && i0 >= 1) ? p[n - 1] : 0.0;
                er = (lane == 63 && i0 + 2 < g.nx) ? p[n + 2] : 0.0;
            }
        }
    }
    acc = wsum(acc);
    if (lane == 0) part[blockIdx.x] = acc;
}

// Sweep A, one wave per block.
template <bool PF>
__global__ __launch_bounds__(64) void ka_(G g, int kc, int tx_n, int ty_n, int tz_n,
                                          const double* __restrict__ r,
                                          const double* __restrict__ po,
                                          double* __restrict__ pn, double* __restrict__ x,
                                          double beta, double alpha, double* part) {
    const int nt = tx_n * ty_n * tz_n;
    const int t = tile_of(blockIdx.x, nt);
    const int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
    const int lane = threadIdx.x;
    const int i0 = tx * 128 + 2 * lane;
    const int j = ty;
    const int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
    double acc = 0;
    if (j >= 1 && j <= g.ny - 2 && i0 < g.nx) {
        const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
        long long idx = kb * g.ps + j * g.px + i0;
        double2 pm = axpy2(ld2(r, idx - g.ps), beta, ld2(po, idx - g.ps));
        double2 oc = ld2(po, idx);
        double2 pc = axpy2(ld2(r, idx), beta, oc);
        // plane-k operands
        double2 op = ld2(po, idx + g.ps), rp = ld2(r, idx + g.ps);
        double2 ysr = ld2(r, idx - g.px), yso = ld2(po, idx - g.px);
        double2 ynr = ld2(r, idx + g.px), yno = ld2(po, idx + g.px);
        double2 xo = ld2(x, idx);
        double el = (lane == 0 && i0 >= 1) ? r[idx - 1] + beta * po[idx - 1] : 0.0;
        double er = (lane == 63 && i0 + 2 < g.nx) ? r[idx + 2] + beta * po[idx + 2] : 0.0;
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 op2, rp2, ysr2, yso2, ynr2, yno2, xo2;
            double el2 = 0, er2 = 0;
            const bool more = k + 1 < ke;
            if (PF && more) {
                long long n = idx + g.ps;
                op2 = ld2(po, n + g.ps);
                rp2 = ld2(r, n + g.ps);
                ysr2 = ld2(r, n - g.px);
                yso2 = ld2(po, n - g.px);
                ynr2 = ld2(r, n + g.px);
                yno2 = ld2(po, n + g.px);
                xo2 = ld2(x, n);
                if (lane == 0 && i0 >= 1) el2 = r[n - 1] + beta * po[n - 1];
                if (lane == 63 && i0 + 2 < g.nx) er2 = r[n + 2] + beta * po[n + 2];
            }
            double2 pp = axpy2(rp, beta, op);
            double2 ys = axpy2(ysr, beta, yso);
            double2 yn = axpy2(ynr, beta, yno);
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = el;
            if (lane == 63) right = er;
            double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
            double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
            double2 pw, xw;
            pw.x = in0 ? pc.x : 0.0;
            pw.y = in1 ? pc.y : 0.0;
            xw.x = in0 ? xo.x + alpha * oc.x : xo.x;
            xw.y = in1 ? xo.y + alpha * oc.y : xo.y;
            *(double2*)&pn[idx] = pw;
            *(double2*)&x[idx] = xw;
            if (in0) acc += pc.x * Ap0;
            if (in1) acc += pc.y * Ap1;
            pm = pc;
            pc = pp;
            oc = op;
            if (PF) {
                op = op2; rp = rp2; ysr = ysr2; yso = yso2; ynr = ynr2; yno = yno2; xo = xo2;
                el = el2; er = er2;
            } else if (more) {
                long long n = idx + g.ps;
                op = ld2(po, n + g.ps);
                rp = ld2(r, n + g.ps);
                ysr = ld2(r, n - g.px);
                yso = ld2(po, n - g.px);
                ynr = ld2(r, n + g.px);
                yno = ld2(po, n + g.px);
                xo = ld2(x, n);
                el = (lane == 0 && i0 >= 1) ? r[n - 1] + beta * po[n - 1] : 0.0;
                er = (lane == 63 && i0 + 2 < g.nx) ? r[n + 2] + beta * po[n + 2] : 0.0;
            }
        }
    }
    acc = wsum(acc);
    if (lane == 0) part[blockIdx.x] = acc;
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
    const double ma = -1e-9;
    int txn = (n + 127) / 128, tyn = n;
    for (int kc : {510, 255, 128, 64, 32}) {
        int tzn = (n - 2 + kc - 1) / kc, nt = txn * tyn * tzn;
        char name[80];
        snprintf(name, sizeof name, "B kc=%d G=%d", kc, nt);
        timeit(name, 24.0 * ncell, [&] { kb_<false><<<nt, 64>>>(g, kc, txn, tyn, tzn, p, r, ma, part); });
        snprintf(name, sizeof name, "B pf kc=%d G=%d", kc, nt);
        timeit(name, 24.0 * ncell, [&] { kb_<true><<<nt, 64>>>(g, kc, txn, tyn, tzn, p, r, ma, part); });
    }
    for (int kc : {510, 255, 128, 64, 32}) {
        int tzn = (n - 2 + kc - 1) / kc, nt = txn * tyn * tzn;
        char name[80];
        snprintf(name, sizeof name, "A kc=%d G=%d", kc, nt);
        timeit(name, 40.0 * ncell, [&] { ka_<false><<<nt, 64>>>(g, kc, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); });
        snprintf(name, sizeof name, "A pf kc=%d G=%d", kc, nt);
        timeit(name, 40.0 * ncell, [&] { ka_<true><<<nt, 64>>>(g, kc, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); });
    }
    // correctness: B once from r0 vs host
    {
        std::vector<double> hr(N);
        CK(hipMemcpy(r, r0, N * 8, hipMemcpyDeviceToDevice));
        int kc = 64, tzn = (n - 2 + kc - 1) / kc, nt = txn * tyn * tzn;
        kb_<true><<<nt, 64>>>(g, kc, txn, tyn, tzn, p, r, -0.5, part);
        CK(hipMemcpy(hr.data(), r, N * 8, hipMemcpyDeviceToHost));
        double maxd = 0;
        for (long long q = 0; q < N; q += 997) {
            long long i = q % n, j = (q / n) % n, k = q / g.ps;
            if (i == 0 || j == 0 || k == 0 || i == n - 1 || j == n - 1 || k == n - 1) continue;
            double c = h[q];
            double lap = ((h[q + 1] - 2.0 * c + h[q - 1])) + ((h[q + n] - 2.0 * c + h[q - n])) +
                         ((h[q + g.ps] + h[q - g.ps] - 2.0 * c));
            maxd = std::max(maxd, std::abs(h[q] + (-0.5) * (-lap) - hr[q]));
        }
        printf("check B pf maxdiff %.3e\n", maxd);
    }
    return 0;
}
