// stencil_mb3.hip -- scratch microbenchmark round 3 (not product code):
// whole-column z-march with 16-B lanes; tile height, XCD-aware mapping, and
// the same structure for CG sweep A (two stencil inputs).
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

// tile id for block b: XCD-aware remap keeps y-adjacent tiles on one XCD
__device__ __forceinline__ int tile_of(int b, int nt, bool xcd) {
    if (!xcd) return b;
    int q = nt / 8, rem = nt % 8;
    int x = b % 8, l = b / 8;
    int start = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    return start + l;
}

template <int TY, bool XCD>
__global__ __launch_bounds__(64 * TY) void vb(G g, int kc, int tx_n, int ty_n, int tz_n,
                                              const double* __restrict__ p,
                                              double* __restrict__ r, double ma, double* part) {
    double acc = 0;
    int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x & 63;
    for (int b = blockIdx.x; b < nt; b += gridDim.x) {
        int t = tile_of(b, nt, XCD && gridDim.x == nt);
        int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
        int i0 = tx * 128 + 2 * lane;
        int j = ty * TY + (threadIdx.x >> 6);
        int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
        if (!((j >= 1 && j <= g.ny - 2) && (i0 < g.nx))) continue;
        const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
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
            rn.x = in0 ? rr.x + ma * Ap0 : rr.x;
            rn.y = in1 ? rr.y + ma * Ap1 : rr.y;
            *(double2*)&r[idx] = rn;
            if (in0) acc += rn.x * rn.x;
            if (in1) acc += rn.y * rn.y;
            pm = pc;
            pc = pp;
        }
    }
    block_partial<64 * TY>(acc, part);
}

// sweep A: p = r + beta*pold at 5 points, Ap, pAp, write pnew, x += a*pold
template <int TY, bool XCD>
__global__ __launch_bounds__(64 * TY) void va(G g, int kc, int tx_n, int ty_n, int tz_n,
                                              const double* __restrict__ r,
                                              const double* __restrict__ po,
                                              double* __restrict__ pn, double* __restrict__ x,
                                              double beta, double alpha, double* part) {
    double acc = 0;
    int nt = tx_n * ty_n * tz_n;
    const int lane = threadIdx.x & 63;
    for (int b = blockIdx.x; b < nt; b += gridDim.x) {
        int t = tile_of(b, nt, XCD && gridDim.x == nt);
        int tx = t % tx_n, ty = (t / tx_n) % ty_n, tz = t / (tx_n * ty_n);
        int i0 = tx * 128 + 2 * lane;
        int j = ty * TY + (threadIdx.x >> 6);
        int kb = 1 + tz * kc, ke = min(kb + kc, g.nz - 1);
        if (!((j >= 1 && j <= g.ny - 2) && (i0 < g.nx))) continue;
        const bool in0 = (i0 >= 1 && i0 <= g.nx - 2), in1 = (i0 + 1 <= g.nx - 2);
        long long idx = kb * g.ps + j * g.px + i0;
#define PD(ix) ([&] { double2 a_ = *(const double2*)&r[ix]; double2 b_ = *(const double2*)&po[ix]; \
        return make_double2(a_.x + beta * b_.x, a_.y + beta * b_.y); }())
        double2 pm = PD(idx - g.ps);
        double2 poc = *(const double2*)&po[idx];
        double2 rc = *(const double2*)&r[idx];
        double2 pc = make_double2(rc.x + beta * poc.x, rc.y + beta * poc.y);
        for (int k = kb; k < ke; ++k, idx += g.ps) {
            double2 pop = *(const double2*)&po[idx + g.ps];
            double2 rp = *(const double2*)&r[idx + g.ps];
            double2 pp = make_double2(rp.x + beta * pop.x, rp.y + beta * pop.y);
            double2 ys = PD(idx - g.px);
            double2 yn = PD(idx + g.px);
            double left = __shfl_up(pc.y, 1, 64);
            double right = __shfl_down(pc.x, 1, 64);
            if (lane == 0) left = (i0 >= 1) ? r[idx - 1] + beta * po[idx - 1] : 0.0;
            if (lane == 63) right = (i0 + 2 < g.nx) ? r[idx + 2] + beta * po[idx + 2] : 0.0;
            double Ap0 = -lap7(g, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
            double Ap1 = -lap7(g, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
            double2 xo = *(const double2*)&x[idx];
            double2 pw, xw;
            pw.x = in0 ? pc.x : 0.0;
            pw.y = in1 ? pc.y : 0.0;
            xw.x = in0 ? xo.x + alpha * poc.x : xo.x;
            xw.y = in1 ? xo.y + alpha * poc.y : xo.y;
            *(double2*)&pn[idx] = pw;
            *(double2*)&x[idx] = xw;
            if (in0) acc += pc.x * Ap0;
            if (in1) acc += pc.y * Ap1;
            pm = pc;
            pc = pp;
            poc = pop;
        }
#undef PD
    }
    block_partial<64 * TY>(acc, part);
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
    int txn = (n + 127) / 128;
#define RUNB(TY, XCD, KC)                                                                    \
    {                                                                                        \
        int tyn = (n + TY - 1) / TY, tzn = (n - 2 + KC - 1) / KC;                           \
        int nt = txn * tyn * tzn;                                                            \
        char name[80];                                                                       \
        snprintf(name, sizeof name, "B ty=%d xcd=%d kc=%d G=%d", TY, XCD, KC, nt);           \
        timeit(name, 24.0 * ncell, [&] { vb<TY, XCD><<<nt, 64 * TY>>>(g, KC, txn, tyn, tzn, p, r, ma, part); }); \
    }
#define RUNA(TY, XCD, KC)                                                                    \
    {                                                                                        \
        int tyn = (n + TY - 1) / TY, tzn = (n - 2 + KC - 1) / KC;                           \
        int nt = txn * tyn * tzn;                                                            \
        char name[80];                                                                       \
        snprintf(name, sizeof name, "A ty=%d xcd=%d kc=%d G=%d", TY, XCD, KC, nt);           \
        timeit(name, 40.0 * ncell, [&] { va<TY, XCD><<<nt, 64 * TY>>>(g, KC, txn, tyn, tzn, r, p, pn, x, 0.5, 1e-9, part); }); \
    }
    RUNB(4, false, 510);
    RUNB(4, true, 510);
    RUNB(2, false, 510);
    RUNB(2, true, 510);
    RUNB(8, false, 510);
    RUNB(8, true, 510);
    RUNB(4, true, 255);
    RUNB(2, true, 255);
    RUNB(4, true, 170);
    RUNB(1, true, 510);
    RUNA(4, false, 510);
    RUNA(4, true, 510);
    RUNA(2, true, 510);
    RUNA(8, true, 510);
    RUNA(4, true, 255);
    RUNA(2, true, 255);
    return 0;
}
