// shell_io.hip -- boundary-shell transfers of the host-buffer step's resident
// mode (hip_proj_config_t.dirty_faces, SURVEY.md:449-455).
//
// Between two `step` calls a reference driver changes only boundary cells of
// its host flow_field (lid / periodic / Neumann BCs, lid_driven_cavity_common.h:306-308,
// taylor_green_3d_reference.h:297-313), and reads only the boundary layer and
// the layer next to it (what those BC routines read). In the resident mode the
// interior stays in HBM: a step uploads the depth-1 shell of u, v, w, p (T)
// and downloads the depth-2 shell, instead of whole fields.
//
// Shell of depth D, in the packed order both sides use: for each z plane k,
// for each row j, the row's shell cells in x order. A row is whole (nx cells)
// when k < D or k >= nz-D (3-D) or j < D or j >= ny-D; otherwise it holds its
// first D and last D cells. Fields follow each other in the staging buffer.
#include "ctx.hpp"

#include <thread>

namespace {

struct ShellMap {
    long long nx, ny, nz;
    int D;
    long long fp, pp;  // cells of a whole plane / of a plane with only x,y shell rows

    __host__ __device__ bool whole_plane(long long k) const {
        return nz > 1 && (k < D || k >= nz - D);
    }
    __host__ __device__ static long long clampll(long long v, long long lo, long long hi) {
        return v < lo ? lo : (v > hi ? hi : v);
    }
    __host__ __device__ long long plane_off(long long k) const {
        if (nz == 1) return 0;
        const long long whole = (k < D ? k : D) + (k > nz - D ? k - (nz - D) : 0);
        return whole * fp + clampll(k - D, 0, nz - 2 * D) * pp;
    }
    __host__ __device__ long long total() const {
        return nz == 1 ? pp : 2LL * D * fp + (nz - 2LL * D) * pp;
    }
    // packed offset of row (j, k) within one field; *whole = row stored whole
    __host__ __device__ long long row_off(long long j, long long k, bool* whole) const {
        const long long o = plane_off(k);
        if (whole_plane(k)) {
            *whole = true;
            return o + j * nx;
        }
        *whole = (j < D || j >= ny - D);
        const long long wr = (j < D ? j : D) + (j > ny - D ? j - (ny - D) : 0);
        return o + wr * nx + clampll(j - D, 0, ny - 2 * D) * (2LL * D);
    }
};

ShellMap make_map(const hip_proj_ctx* c, int D) {
    ShellMap m;
    m.nx = (long long)c->nx;
    m.ny = (long long)c->ny;
    m.nz = (long long)c->nz;
    m.D = D;
    m.fp = m.nx * m.ny;
    m.pp = 2LL * D * m.nx + (m.ny - 2LL * D) * (2LL * D);
    return m;
}

struct FieldSet {
    double* f[5];
};

// One wavefront per row; PACK: device fields -> staging, else staging -> fields.
template <bool PACK>
__global__ __launch_bounds__(256) void k_shell_io(FieldSet fs, int nf, ShellMap m, long long px,
                                                  long long ps, double* buf) {
    const int lane = threadIdx.x & 63;
    const long long nrows = m.ny * m.nz;
    const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
    const long long total = m.total();
    for (long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
         row < nrows * nf; row += waves) {
        const int fi = (int)(row / nrows);
        const long long r = row - fi * nrows;
        const long long k = r / m.ny, j = r - k * m.ny;
        bool whole;
        double* b = buf + fi * total + m.row_off(j, k, &whole);
        double* d = fs.f[fi] + k * ps + j * px;
        if (whole) {
            for (long long i = lane; i < m.nx; i += 64) {
                if (PACK) b[i] = d[i];
                else d[i] = b[i];
            }
        } else if (lane < 2 * m.D) {
            const long long i = (lane < m.D) ? lane : m.nx - 2 * m.D + lane;
            if (PACK) b[lane] = d[i];
            else d[i] = b[lane];
        }
    }
}

// Host side of the same layout over caller arrays (nx*ny*nz, packed), split
// over threads by rows: the partial rows touch two cache lines each, 4 KB or
// more apart, which one core walks at a fraction of the copy rate.
// CFD_HIP_SHELL_THREADS (experiments), read once per process
static int shell_threads_env() {
    static const int n = [] {
        const char* e = getenv("CFD_HIP_SHELL_THREADS");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    return n;
}

void host_rows(const ShellMap& m, int nf, double* const* host, double* buf, bool gather) {
    const long long nrows = m.ny * m.nz * nf;
    const long long total = m.total();
    auto work = [&](long long r0, long long r1) {
        for (long long row = r0; row < r1; ++row) {
            const int fi = (int)(row / (m.ny * m.nz));
            const long long r = row - fi * m.ny * m.nz;
            const long long k = r / m.ny, j = r - k * m.ny;
            bool whole;
            double* b = buf + fi * total + m.row_off(j, k, &whole);
            double* h = host[fi] + (k * m.ny + j) * m.nx;
            if (whole) {
                if (gather) memcpy(b, h, m.nx * sizeof(double));
                else memcpy(h, b, m.nx * sizeof(double));
            } else {
                const long long tail = m.nx - m.D;
                if (gather) {
                    memcpy(b, h, m.D * sizeof(double));
                    memcpy(b + m.D, h + tail, m.D * sizeof(double));
                } else {
                    memcpy(h, b, m.D * sizeof(double));
                    memcpy(h + tail, b + m.D, m.D * sizeof(double));
                }
            }
        }
    };
    const long long cells = total * nf;
    unsigned hc = std::thread::hardware_concurrency();
    int nt = (int)std::min<unsigned>(hc ? hc : 1, 16);
    if (shell_threads_env() > 0) nt = shell_threads_env();
    if (cells < (1LL << 18)) nt = 1;
    if (nt == 1) {
        work(0, nrows);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; ++t) {
        const long long r0 = nrows * t / nt, r1 = nrows * (t + 1) / nt;
        try {
            th.emplace_back(work, r0, r1);
        } catch (...) {  // no thread: this share on the caller's (C ABI)
            work(r0, r1);
        }
    }
    for (auto& t : th) t.join();
}

cfd_status_t ensure_staging(hip_proj_ctx* c, size_t n) {
    if (c->shell_cap >= n) return CFD_SUCCESS;
    if (c->shell_host) hipHostFree(c->shell_host);
    c->shell_host = nullptr;
    c->shell_cap = 0;
    if (c->shell_dev) hipFree(c->shell_dev);
    c->shell_dev = nullptr;
    HIP_TRY(hipMalloc((void**)&c->shell_dev, n * sizeof(double)));
    HIP_TRY(hipHostMalloc((void**)&c->shell_host, n * sizeof(double), hipHostMallocDefault));
    c->shell_cap = n;
    return CFD_SUCCESS;
}

unsigned io_blocks(const ShellMap& m, int nf) {
    const long long waves = m.ny * m.nz * nf;
    return (unsigned)std::max(1LL, std::min((waves + 3) / 4, 8192LL));
}

}  // namespace

bool ctx_shell_fits(const hip_proj_ctx* c, int depth) {
    return c->nranks == 1 && (long long)c->nx > 2 * depth && (long long)c->ny > 2 * depth &&
           (c->nz == 1 || (long long)c->nz > 2 * depth);
}

cfd_status_t ctx_shell_put(hip_proj_ctx* c, const double* const* host, double* const* dev, int nf,
                           int depth) {
    const ShellMap m = make_map(c, depth);
    const size_t n = (size_t)(m.total() * nf);
    ST_TRY(ensure_staging(c, n));
    HIP_TRY(hipStreamSynchronize(c->stream));  // the staging buffer may still be in flight
    host_rows(m, nf, const_cast<double* const*>(host), c->shell_host, true);
    HIP_TRY(hipMemcpyAsync(c->shell_dev, c->shell_host, n * sizeof(double), hipMemcpyHostToDevice,
                           c->stream));
    FieldSet fs{};
    for (int i = 0; i < nf; ++i) fs.f[i] = dev[i];
    hipLaunchKernelGGL(k_shell_io<false>, dim3(io_blocks(m, nf)), dim3(256), 0, c->stream, fs, nf,
                       m, c->px, c->ps, c->shell_dev);
    HIP_TRY(hipGetLastError());
    return CFD_SUCCESS;
}

cfd_status_t ctx_shell_get(hip_proj_ctx* c, double* const* host, double* const* dev, int nf,
                           int depth) {
    const ShellMap m = make_map(c, depth);
    const size_t n = (size_t)(m.total() * nf);
    ST_TRY(ensure_staging(c, n));
    FieldSet fs{};
    for (int i = 0; i < nf; ++i) fs.f[i] = dev[i];
    hipLaunchKernelGGL(k_shell_io<true>, dim3(io_blocks(m, nf)), dim3(256), 0, c->stream, fs, nf, m,
                       c->px, c->ps, c->shell_dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->shell_host, c->shell_dev, n * sizeof(double), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    host_rows(m, nf, host, c->shell_host, false);
    return CFD_SUCCESS;
}

// compute_max_temperature (solver_registry.c:52-62) over a host array with
// the reference's sequential semantics, m = T[0]; m = T[i] if T[i] > m, split
// over up to 16 threads: each chunk's maximum from -inf with the same strict
// comparison (its first occurrence; NaNs never compare greater), combined in
// chunk order with that comparison, so the result is the sequential loop's
// bit for bit (a NaN T[0] stays; -0.0 / +0.0 keep the earlier one).
double ctx_host_max(const double* T, size_t n) {
    if (n == 0) return 0.0;
    unsigned hc = std::thread::hardware_concurrency();
    int nt = (int)std::min<unsigned>(hc ? hc : 1, 16);
    if (n < (1u << 20)) nt = 1;
    std::vector<double> part(nt, -INFINITY);
    auto work = [&](int t) {
        const size_t a = 1 + (n - 1) * (size_t)t / (size_t)nt;
        const size_t b = 1 + (n - 1) * (size_t)(t + 1) / (size_t)nt;
        double m = -INFINITY;
        for (size_t i = a; i < b; ++i)
            if (T[i] > m) m = T[i];
        part[t] = m;
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(nt);
        for (int t = 0; t < nt; ++t) {
            try {
                th.emplace_back(work, t);
            } catch (...) {  // no thread: this share on the caller's (C ABI)
                work(t);
            }
        }
        for (auto& t : th) t.join();
    }
    double m = T[0];
    for (double v : part)
        if (v > m) m = v;
    return m;
}

// Resident-mode guard (hip_proj_config_t.dirty_verify_interval): hashes of
// the host arrays' cells inside the outer layer (the layer a caller's BC
// routine writes), in two parts: the deep interior (every index in
// [2, n-3]; the resident steps never write it on the host, so its hash holds
// until a full download) and layer 1 (the cells next to the boundary, which
// every step's depth-2 shell download rewrites, so its hash is retaken after
// each step; shell-sized). Each cell contributes mix(bits) * (2 idx + 1), so
// a sum is order-independent (summed per plane range over threads) and
// changes when any value changes or two values swap.
void ctx_host_hash(const hip_proj_ctx* c, const double* const* host, int nf, bool layer1,
                   unsigned long long* out) {
    const long long nx = (long long)c->nx, ny = (long long)c->ny, nz = (long long)c->nz;
    const bool is3d = nz > 1;
    const long long k0 = is3d ? 1 : 0, k1 = is3d ? nz - 1 : 1;
    const long long planes = k1 - k0;
    unsigned hc = std::thread::hardware_concurrency();
    int nt = (int)std::min<unsigned>(hc ? hc : 1, 16);
    if (shell_threads_env() > 0) nt = shell_threads_env();
    if (layer1) nt = std::min(nt, 4);
    nt = (int)std::max(1LL, std::min<long long>(nt, planes));
    auto mix = [](const double* p, long long idx) {
        unsigned long long b;
        memcpy(&b, p, sizeof(b));
        b ^= b >> 31;
        b *= 0x9E3779B97F4A7C15ull;
        return b * (unsigned long long)(2 * idx + 1);
    };
    for (int f = 0; f < nf; ++f) {
        std::vector<unsigned long long> part(nt, 0ull);
        auto work = [&](int t) {
            unsigned long long h = 0;
            for (long long k = k0 + planes * t / nt; k < k0 + planes * (t + 1) / nt; ++k) {
                const bool kedge = is3d && (k == 1 || k == nz - 2);
                for (long long j = 1; j < ny - 1; ++j) {
                    const long long row = (k * ny + j) * nx;
                    const bool edge_row = kedge || j == 1 || j == ny - 2;
                    if (!layer1) {
                        if (edge_row) continue;
                        for (long long i = 2; i < nx - 2; ++i) h += mix(host[f] + row + i, row + i);
                    } else if (edge_row) {
                        for (long long i = 1; i < nx - 1; ++i) h += mix(host[f] + row + i, row + i);
                    } else {
                        h += mix(host[f] + row + 1, row + 1);
                        h += mix(host[f] + row + nx - 2, row + nx - 2);
                    }
                }
            }
            part[t] = h;
        };
        if (nt == 1) {
            work(0);
        } else {
            // reached from extern "C" entry points: a thread that cannot be
            // created (std::system_error) must not cross the C ABI, so its
            // share runs on this thread instead (the sum is order-free)
            std::vector<std::thread> th;
            th.reserve(nt);
            for (int t = 0; t < nt; ++t) {
                try {
                    th.emplace_back(work, t);
                } catch (...) {
                    work(t);
                }
            }
            for (auto& t : th) t.join();
        }
        unsigned long long h = 0;
        for (auto v : part) h += v;
        out[f] = h;
    }
}
