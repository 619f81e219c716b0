// stencil_mb6.hip -- scratch microbenchmark round 6 (not product code):
// (a) sweep A with y neighbours exchanged through LDS (TY waves per block);
// (b) rebalanced CG sweeps: A' = {r, pold stencils -> pnew} (24 B/cell),
//     B' = {p stencil, r, x -> r, x} (40 B/cell).
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

// (a) A with LDS rows: block = TY waves = TY rows of 128 cells; rows j0-1 and
// j0+TY (halo) computed by waves 0 and TY-1 in addition to their own row.
template <int TY>
__global__ __launch_bounds__(64 * TY) void a_lds(G g, int kc, int tx_n, int ty_n, int tz_n,
                                                 const double* __restrict__ r,
                                                 const double* __restrict__ po,
                                                 double* __restrict__ pn, double* __restrict__ x,
                                                 double beta, double alpha, double* part) {
    __shared__ double2 rows[2][TY + 2][64];
    const int nt = tx_n * ty_n * tz_n;
    const int t = tile_of(blockIdx.x, nt);
    const int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i0 = tx * 128 + 2 * lane;
    const int j = ty * TY + w;
    const int jc = min(j, g.ny - 1);
    const int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
    const bool act = (j >= 1 && j <= g.ny - 2 && i0 < g.nx);
    const bool in0 = act && (i0 >= 1 && i0 <= g.nx - 2), in1 = act && (i0 + 1 <= g.nx - 2);
    const int ic = min(i0, g.nx - 2);
    // halo row for waves 0 (below) and TY-1 (above)
    const bool hal = (w == 0) || (w == TY - 1);
    const int jh = (w == 0) ? max(ty * TY - 1, 0) : min(ty * TY + TY, g.ny - 1);
    const int hslot = (w == 0) ? 0 : TY + 1;
    double acc = 0;
    long long idx = (long long)kb * g.ps + (long long)jc * g.px + ic;
    long long hidx = (long long)kb * g.ps + (long long)jh * g.px + ic;
    double2 pm = axpy2(ld2(r, idx - g.ps), beta, ld2(po, idx - g.ps));
    double2 oc = ld2(po, idx);
    double2 pc = axpy2(ld2(r, idx), beta, oc);
    double2 hc = hal ? axpy2(ld2(r, hidx), beta, ld2(po, hidx)) : make_double2(0, 0);
    int buf = 0;
    for (int k = kb; k < ke; ++k, idx += g.ps, hidx += g.ps) {
        double2 op = ld2(po, idx + g.ps), rp = ld2(r, idx + g.ps);
        double2 hp = hal && (k + 1 < ke) ? axpy2(ld2(r, hidx + g.ps), beta, ld2(po, hidx + g.ps))
                                         : make_double2(0, 0);
        double2 xo = ld2(x, idx);
        double el = (lane == 0 && i0 >= 1) ? r[idx - 1] + beta * po[idx - 1] : 0.0;
        double er = (lane == 63 && i0 + 2 < g.nx) ? r[idx + 2] + beta * po[idx + 2] : 0.0;
        rows[buf][w + 1][lane] = pc;
        if (hal) rows[buf][hslot][lane] = hc;
        __syncthreads();
        double2 ys = rows[buf][w][lane];
        double2 yn = rows[buf][w + 2][lane];
        double2 pp = axpy2(rp, beta, op);
        double left = __shfl_up(pc.y, 1, 64);
        double right = __shfl_down(pc.x, 1, 64);
        if (lane == 0) left = el;
        if (lane == 63) right = er;
        double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
        double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
        if (act) {
            double2 pw, xw;
            pw.x = in0 ? pc.x : 0.0;
            pw.y = in1 ? pc.y : 0.0;
            xw.x = in0 ? xo.x + alpha * oc.x : xo.x;
            xw.y = in1 ? xo.y + alpha * oc.y : xo.y;
            *(double2*)&pn[idx] = pw;
            *(double2*)&x[idx] = xw;
        }
        if (in0) acc += pc.x * Ap0;
        if (in1) acc += pc.y * Ap1;
        pm = pc;
        pc = pp;
        oc = op;
        hc = hp;
        buf ^= 1;
    }
    acc = wsum(acc);
    if (lane == 0) part[blockIdx.x * TY + w] = acc;
}

// (b1) A' : p = r + beta pold at 5 points, Ap, (p,Ap), write pnew only (24 B/cell)
__global__ __launch_bounds__(64) void a_prime(G g, int kc, int tx_n, int ty_n, int tz_n,
                                              const double* __restrict__ r,
                                              const double* __restrict__ po,
                                              double* __restrict__ pn, double beta,
                                              double* part) {
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
        double2 pc = axpy2(ld2(r, idx), beta, ld2(po, idx));
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 op = ld2(po, idx + g.ps), rp = ld2(r, idx + g.ps);
            double2 ysr = ld2(r, idx - g.px), yso = ld2(po, idx - g.px);
            double2 ynr = ld2(r, idx + g.px), yno = ld2(po, idx + g.px);
            double el = (lane == 0 && i0 >= 1) ? r[idx - 1] + beta * po[idx - 1] : 0.0;
            double er = (lane == 63 && i0 + 2 < g.nx) ? r[idx + 2] + beta * po[idx + 2] : 0.0;
            double2 pp = axpy2(rp, beta, op);
            double2 ys = axpy2(ysr, beta, yso), yn = axpy2(ynr, beta, yno);
            double left = __shfl_up(pc.y, 1, 64), right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = el;
            if (lane == 63) right = er;
            double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
            double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
            double2 pw;
            pw.x = in0 ? pc.x : 0.0;
            pw.y = in1 ? pc.y : 0.0;
            *(double2*)&pn[idx] = pw;
            if (in0) acc += pc.x * Ap0;
            if (in1) acc += pc.y * Ap1;
            pm = pc;
            pc = pp;
        }
    }
    acc = wsum(acc);
    if (lane == 0) part[blockIdx.x] = acc;
}

// (b2) B' : Ap from p stencil, r -= a Ap, x += a p, (r,r) (40 B/cell)
__global__ __launch_bounds__(64) void b_prime(G g, int kc, int tx_n, int ty_n, int tz_n,
                                              const double* __restrict__ p, double* __restrict__ r,
                                              double* __restrict__ x, double a, double* part) {
    const int nt = tx_n * ty_n * tz_n;
    const int t = tile_of(blockIdx.x, nt);
    const int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
    const int lane = threadIdx.x;
    const int i0 = tx * 128 + 2 * lane;
    const int j = ty;
    const int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
    double acc = 0;
    const double ma = -a;
    if (j >= 1 && j <= g.ny - 2 && i0 < g.nx) {
        const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
        long long idx = kb * g.ps + j * g.px + i0;
        double2 pm = ld2(p, idx - g.ps), pc = ld2(p, idx);
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 pp = ld2(p, idx + g.ps), ys = ld2(p, idx - g.px), yn = ld2(p, idx + g.px);
            double2 rr = ld2(r, idx), xo = ld2(x, idx);
            double el = (lane == 0 && i0 >= 1) ? p[idx - 1] : 0.0;
            double er = (lane == 63 && i0 + 2 < g.nx) ? p[idx + 2] : 0.0;
            double left = __shfl_up(pc.y, 1, 64), right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = el;
            if (lane == 63) right = er;
            double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
            double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
            double2 rn, xn;
            rn.x = in0 ? rr.x + ma * Ap0 : rr.x;
            rn.y = in1 ? rr.y + ma * Ap1 : rr.y;
            xn.x = in0 ? xo.x + a * pc.x : xo.x;
            xn.y = in1 ? xo.y + a * pc.y : xo.y;
            *(double2*)&r[idx] = rn;
            *(double2*)&x[idx] = xn;
            if (in0) acc += rn.x * rn.x;
            if (in1) acc += rn.y * rn.y;
            pm = pc;
            pc = pp;
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
        return ms;
    };
    int txn = (n + 127) / 128;
    for (int kc : {510, 128, 64}) {
        int tzn = (n - 2 + kc - 1) / kc;
        char name[80];
        {
            int tyn = (n + 3) / 4, nt = txn * tyn * tzn;
            snprintf(name, sizeof name, "A lds ty=4 kc=%d G=%d", kc, nt);
            timeit(name, 40.0 * ncell, [&] { a_lds<4><<<nt, 256>>>(g, kc, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); });
        }
        {
            int tyn = (n + 7) / 8, nt = txn * tyn * tzn;
            snprintf(name, sizeof name, "A lds ty=8 kc=%d G=%d", kc, nt);
            timeit(name, 40.0 * ncell, [&] { a_lds<8><<<nt, 512>>>(g, kc, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); });
        }
        {
            int tyn = (n + 1) / 2, nt = txn * tyn * tzn;
            snprintf(name, sizeof name, "A lds ty=2 kc=%d G=%d", kc, nt);
            timeit(name, 40.0 * ncell, [&] { a_lds<2><<<nt, 128>>>(g, kc, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); });
        }
        int tyn = n, nt = txn * tyn * tzn;
        double ta, tb;
        snprintf(name, sizeof name, "A' kc=%d G=%d", kc, nt);
        ta = timeit(name, 24.0 * ncell, [&] { a_prime<<<nt, 64>>>(g, kc, txn, tyn, tzn, r, p, pn, 0.5, part); });
        snprintf(name, sizeof name, "B' kc=%d G=%d", kc, nt);
        tb = timeit(name, 40.0 * ncell, [&] { b_prime<<<nt, 64>>>(g, kc, txn, tyn, tzn, p, r, x, 1e-9, part); });
        printf("   A'+B' = %.4f ms per CG iteration (%.1f GB/s at 64 B/cell)\n", ta + tb,
               64.0 * ncell / ((ta + tb) * 1e-3) / 1e9);
    }
    return 0;
}
