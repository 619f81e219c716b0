// checkpoint_hip.hip -- restart files of the device-resident state
// (SURVEY.md §8f row 4), in the reference's `.cfdchk` format
// (lib/include/cfd/io/checkpoint.h, layout in ../host/chk_format.h).
//
// The fields never take a detour through host flow_field arrays: each field
// streams between HBM and the file through two pinned staging buffers (the
// D2H/H2D copy of one chunk overlaps the fwrite/fread of the other), and its
// CRC-32 is computed on the GPU straight from the padded device layout, in
// the packed k*nx*ny + j*nx + i byte order of the file:
//
//   one wavefront per chunk of C consecutive values; lane l folds values
//   l, l+64, l+128, ... into a register: acc <- upd8(shift504(acc), value)
//   (slicing-by-8 tables + a byte-sliced "skip 504 bytes" operator, 12 KB of
//   LDS), so each register is the CRC of its values spaced 512 B apart; the
//   lanes are moved to the chunk end (GF(2) multiply by x^(8 d)) and XORed,
//   the chunk is moved to the field end and XORed into one word with an
//   atomic (XOR is order-free, so the result is deterministic).
//
// The host joins the field CRCs with the header/parameter bytes it CRCs
// itself: S' = S * x^(8 |field|) ^ raw0(field) (chk_format.h chk_crc_join).
// A read lands in scratch fields first and replaces the state only when the
// trailing CRC matches, so a corrupt file leaves the context untouched; the
// borrowed scratch is zeroed again afterwards.
#include "ctx.hpp"

#include "../host/chk_format.h"

#include <memory>

namespace {

struct DevCrcTab {
    uint32_t t[8][256];  // slicing-by-8
    uint32_t h[4][256];  // register * x^(8*504), byte-sliced
    uint32_t x8[64];     // x^(64 * 2^b): skip 8 * 2^b bytes
};

constexpr long long CRC_CHUNK = 8192;  // values per wavefront
constexpr int CRC_WAVES = 4;           // wavefronts (chunks) per workgroup

__device__ __forceinline__ uint32_t dgf_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll 4
    for (int i = 0; i < 32; i++) {
        if (a & 0x80000000u) r ^= b;
        a <<= 1;
        b = (b & 1u) ? (b >> 1) ^ CHK_POLY : b >> 1;
    }
    return r;
}

// register moved past q * 8 zero bytes
__device__ __forceinline__ uint32_t skip8(const uint32_t* x8, uint32_t v, unsigned long long q) {
    for (int b = 0; q && v; ++b, q >>= 1)
        if (q & 1ull) v = dgf_mul(x8[b], v);
    return v;
}

__global__ __launch_bounds__(64 * CRC_WAVES) void k_crc_raw(const double* __restrict__ f, int nx,
                                                            int ny, long long px, long long ps,
                                                            long long n, const DevCrcTab* tab,
                                                            unsigned* out) {
    __shared__ uint32_t t[8][256];
    __shared__ uint32_t h[4][256];
    for (int e = threadIdx.x; e < 8 * 256; e += blockDim.x) t[e >> 8][e & 255] = tab->t[e >> 8][e & 255];
    for (int e = threadIdx.x; e < 4 * 256; e += blockDim.x) h[e >> 8][e & 255] = tab->h[e >> 8][e & 255];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const long long start = ((long long)blockIdx.x * CRC_WAVES + (threadIdx.x >> 6)) * CRC_CHUNK;
    if (start >= n) return;
    const long long end = min(start + CRC_CHUNK, n);
    long long s = start + lane;
    long long i = s % nx, rest = s / nx;
    long long j = rest % ny, k = rest / ny;
    uint32_t acc = 0;
    long long last = -1;
    for (; s < end; s += 64) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(f[k * ps + j * px + i]);
        acc = h[0][acc & 255u] ^ h[1][(acc >> 8) & 255u] ^ h[2][(acc >> 16) & 255u] ^ h[3][acc >> 24];
        const uint32_t lo = (uint32_t)bits ^ acc, hi = (uint32_t)(bits >> 32);
        acc = t[7][lo & 255u] ^ t[6][(lo >> 8) & 255u] ^ t[5][(lo >> 16) & 255u] ^ t[4][lo >> 24] ^
              t[3][hi & 255u] ^ t[2][(hi >> 8) & 255u] ^ t[1][(hi >> 16) & 255u] ^ t[0][hi >> 24];
        last = s;
        i += 64;
        while (i >= nx) {
            i -= nx;
            if (++j == ny) {
                j = 0;
                ++k;
            }
        }
    }
    uint32_t v = (last >= 0) ? skip8(tab->x8, acc, (unsigned long long)(end - 1 - last)) : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v ^= (uint32_t)__shfl_xor((int)v, off, 64);
    if (lane == 0 && v) atomicXor(out, skip8(tab->x8, v, (unsigned long long)(n - end)));
}

__global__ void k_fill_const(double* f, long long n, double v) {
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x)
        f[e] = v;
}

struct Pinned {
    void* p = nullptr;
    ~Pinned() {
        if (p) hipHostFree(p);
    }
};

struct EventPair {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~EventPair() {
        for (hipEvent_t x : e)
            if (x) hipEventDestroy(x);
    }
};

struct FileCloser {
    FILE* fp = nullptr;
    ~FileCloser() {
        if (fp) fclose(fp);
    }
};

// Scratch fields the checkpoint borrowed go back to the zeros they hold after
// allocation: the CG relies on zero boundary cells in r and p (the lagged-BC
// semantics, SURVEY.md App. A trap 1) and the other scratch arrays are
// rewritten by the step anyway.
void scrub_scratch(hip_proj_ctx* c, double* a, double* b) {
    const size_t bytes = field_elems(c) * sizeof(double);
    for (double* f : {a, b})
        if (f) hipMemsetAsync(f, 0, bytes, c->stream);
    hipStreamSynchronize(c->stream);
}

// staging: whole planes, about 64 MB per buffer
size_t stage_planes(const hip_proj_ctx* c) {
    const size_t plane = c->nx * c->ny * sizeof(double);
    return std::max<size_t>(1, std::min<size_t>(c->nz, (64u << 20) / std::max<size_t>(plane, 1)));
}

cfd_status_t crc_tables(hip_proj_ctx* c, DevCrcTab** out) {
    static_assert(sizeof(DevCrcTab) % 4 == 0, "table layout");
    std::unique_ptr<DevCrcTab> h(new DevCrcTab);
    chk_crc_tables T;
    chk_crc_tables_init(&T);
    memcpy(h->t, T.t, sizeof(h->t));
    const uint32_t x504 = chk_xpow_bytes(504);
    for (int b = 0; b < 4; b++)
        for (uint32_t v = 0; v < 256; v++) h->h[b][v] = chk_gf_mul(x504, v << (8 * b));
    for (int b = 0; b < 64; b++) h->x8[b] = b < 61 ? chk_xpow_bytes(8ull << b) : 0x80000000u;
    DevCrcTab* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, sizeof(DevCrcTab)));
    if (hipMemcpy(d, h.get(), sizeof(DevCrcTab), hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(d);
        set_err(CFD_ERROR, "checkpoint: CRC table upload failed");
        return CFD_ERROR;
    }
    *out = d;
    return CFD_SUCCESS;
}

void launch_crc(hip_proj_ctx* c, const double* f, const DevCrcTab* tab, unsigned* out) {
    const long long n = (long long)(c->nx * c->ny * c->nz);
    const long long chunks = (n + CRC_CHUNK - 1) / CRC_CHUNK;
    const unsigned blocks = (unsigned)((chunks + CRC_WAVES - 1) / CRC_WAVES);
    hipLaunchKernelGGL(k_crc_raw, dim3(blocks), dim3(64 * CRC_WAVES), 0, c->stream, f, (int)c->nx,
                       (int)c->ny, c->px, c->ps, n, tab, out);
}

// zero-register CRCs of `nf` device fields (packed order)
cfd_status_t device_crcs(hip_proj_ctx* c, const double* const* fs, int nf, uint32_t* raw) {
    DevCrcTab* tab = nullptr;
    unsigned* d_out = nullptr;
    ST_TRY(crc_tables(c, &tab));
    cfd_status_t st = CFD_SUCCESS;
    if (hipMalloc((void**)&d_out, sizeof(unsigned) * nf) != hipSuccess ||
        hipMemsetAsync(d_out, 0, sizeof(unsigned) * nf, c->stream) != hipSuccess) {
        st = CFD_ERROR;
    } else {
        for (int q = 0; q < nf; ++q) launch_crc(c, fs[q], tab, d_out + q);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(raw, d_out, sizeof(unsigned) * nf, hipMemcpyDeviceToHost, c->stream) !=
                hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            st = CFD_ERROR;
    }
    if (d_out) hipFree(d_out);
    hipFree(tab);
    if (st != CFD_SUCCESS) set_err(st, "checkpoint: device CRC failed");
    return st;
}

}  // namespace

extern "C" {

cfd_status_t hip_proj_field_crc32(hip_proj_ctx_t* c, int field_id, uint32_t* crc) {
    GroupHostLock hl_(c);
    if (!c || !crc) return CFD_ERROR_INVALID;
    const double* f = field_ptr(c, field_id);
    if (!f) return CFD_ERROR_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    uint32_t raw = 0;
    ST_TRY(device_crcs(c, &f, 1, &raw));
    *crc = chk_crc_join(0xFFFFFFFFu, (uint64_t)c->nx * c->ny * c->nz * 8, raw) ^ 0xFFFFFFFFu;
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_checkpoint_write(hip_proj_ctx_t* c, const char* path, const grid* g,
                                       const ns_solver_params_t* params, double current_time,
                                       const char* solver_name, const char* run_prefix,
                                       const char* output_base_dir) {
    GroupHostLock hl_(c);
    if (!c || !path || !g || !params || !solver_name) {
        set_err(CFD_ERROR_INVALID, "hip_proj_checkpoint_write: NULL argument");
        return CFD_ERROR_INVALID;
    }
    if (g->nx != c->nx || g->ny != c->ny || g->nz != c->nz) {
        set_err(CFD_ERROR_INVALID, "hip_proj_checkpoint_write: grid/context dimension mismatch");
        return CFD_ERROR_INVALID;
    }
    if (dist(c) || !chk_host_little_endian()) {
        set_err(CFD_ERROR_UNSUPPORTED,
                "hip_proj_checkpoint_write: Z-slab contexts / big-endian hosts not supported");
        return CFD_ERROR_UNSUPPORTED;
    }
    HIP_TRY(hipSetDevice(c->device));
    // u, v, w, p, rho, T: a context without a per-cell density or temperature
    // writes rho0 / 0 everywhere (a scratch field holds the constant)
    const double* fs[CHK_NFIELDS] = {c->u, c->v, c->w, c->p, c->rho, c->T};
    const long long ne = (long long)field_elems(c);
    if (!c->rho) {
        hipLaunchKernelGGL(k_fill_const, dim3(4096), dim3(256), 0, c->stream, c->us, ne, c->rho0);
        fs[4] = c->us;
    }
    if (!c->T) {
        hipLaunchKernelGGL(k_fill_const, dim3(4096), dim3(256), 0, c->stream, c->vs, ne, 0.0);
        fs[5] = c->vs;
    }
    uint32_t raw[CHK_NFIELDS];
    ST_TRY(device_crcs(c, fs, CHK_NFIELDS, raw));

    chk_buf pre{}, suf{};
    chk_put_prefix(&pre, g);
    chk_put_suffix(&suf, params, current_time, solver_name, run_prefix, output_base_dir);
    std::unique_ptr<chk_crc_tables> T(new chk_crc_tables);
    chk_crc_tables_init(T.get());
    cfd_status_t st = (pre.oom || suf.oom) ? CFD_ERROR_NOMEM : CFD_SUCCESS;
    const uint64_t fbytes = (uint64_t)c->nx * c->ny * c->nz * sizeof(double);
    uint32_t crc = chk_crc_update(T.get(), 0xFFFFFFFFu, pre.p, pre.n);
    for (int q = 0; q < CHK_NFIELDS; ++q) crc = chk_crc_join(crc, fbytes, raw[q]);
    crc = chk_crc_update(T.get(), crc, suf.p, suf.n);

    FileCloser file;
    Pinned stage[2];
    EventPair ev;
    const size_t kp = stage_planes(c);
    const size_t row = c->nx * sizeof(double);
    const size_t sbytes = kp * c->ny * row;
    if (st == CFD_SUCCESS && !(file.fp = fopen(path, "wb"))) st = CFD_ERROR_IO;
    if (st == CFD_SUCCESS &&
        (hipHostMalloc(&stage[0].p, sbytes, hipHostMallocDefault) != hipSuccess ||
         hipHostMalloc(&stage[1].p, sbytes, hipHostMallocDefault) != hipSuccess ||
         hipEventCreateWithFlags(&ev.e[0], hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&ev.e[1], hipEventDisableTiming) != hipSuccess))
        st = CFD_ERROR_NOMEM;
    if (st == CFD_SUCCESS && fwrite(pre.p, 1, pre.n, file.fp) != pre.n) st = CFD_ERROR_IO;
    // chunk m of the whole stream: field m / nchunk, planes [k0, k0 + kp)
    const size_t nchunk = (c->nz + kp - 1) / kp;
    const size_t total = CHK_NFIELDS * nchunk;
    size_t pend_bytes[2] = {0, 0};
    auto issue = [&](size_t m) -> bool {
        const int q = (int)(m / nchunk);
        const size_t k0 = (m % nchunk) * kp, nk = std::min(kp, c->nz - k0);
        const int b = (int)(m & 1);
        pend_bytes[b] = nk * c->ny * row;
        return hipMemcpy2DAsync(stage[b].p, row, fs[q] + k0 * c->ps, c->px * sizeof(double), row,
                                c->ny * nk, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
               hipEventRecord(ev.e[b], c->stream) == hipSuccess;
    };
    if (st == CFD_SUCCESS && !issue(0)) st = CFD_ERROR;
    for (size_t m = 0; m < total && st == CFD_SUCCESS; ++m) {
        if (m + 1 < total && !issue(m + 1)) st = CFD_ERROR;  // overlaps this chunk's fwrite
        const int b = (int)(m & 1);
        if (st == CFD_SUCCESS && hipEventSynchronize(ev.e[b]) != hipSuccess) st = CFD_ERROR;
        if (st == CFD_SUCCESS && fwrite(stage[b].p, 1, pend_bytes[b], file.fp) != pend_bytes[b])
            st = CFD_ERROR_IO;
        // the next issue into buffer b happens only after this fwrite returned
    }
    hipStreamSynchronize(c->stream);
    scrub_scratch(c, c->rho ? nullptr : c->us, c->T ? nullptr : c->vs);
    if (st == CFD_SUCCESS &&
        (fwrite(suf.p, 1, suf.n, file.fp) != suf.n || !chk_write_trailer(file.fp, crc)))
        st = CFD_ERROR_IO;
    if (file.fp) {
        if (fclose(file.fp) != 0 && st == CFD_SUCCESS) st = CFD_ERROR_IO;
        file.fp = nullptr;
    }
    chk_buf_free(&pre);
    chk_buf_free(&suf);
    if (st != CFD_SUCCESS) set_err(st, "hip_proj_checkpoint_write: write failed");
    return st;
}

cfd_status_t hip_proj_checkpoint_read(hip_proj_ctx_t* c, const char* path, grid** out_grid,
                                      ns_solver_params_t* out_params, double* out_current_time,
                                      char* out_solver_name, size_t solver_name_cap,
                                      char* out_run_prefix, size_t run_prefix_cap,
                                      char* out_output_base_dir, size_t output_base_dir_cap) {
    GroupHostLock hl_(c);
    if (out_grid) *out_grid = nullptr;
    if (!c || !path || !out_params) {
        set_err(CFD_ERROR_INVALID, "hip_proj_checkpoint_read: NULL argument");
        return CFD_ERROR_INVALID;
    }
    memset(out_params, 0, sizeof(*out_params));
    if (dist(c) || !chk_host_little_endian()) {
        set_err(CFD_ERROR_UNSUPPORTED,
                "hip_proj_checkpoint_read: Z-slab contexts / big-endian hosts not supported");
        return CFD_ERROR_UNSUPPORTED;
    }
    HIP_TRY(hipSetDevice(c->device));
    std::unique_ptr<chk_crc_tables> T(new chk_crc_tables);
    chk_crc_tables_init(T.get());
    FileCloser file;
    if (!(file.fp = fopen(path, "rb"))) {
        set_err(CFD_ERROR_IO, "hip_proj_checkpoint_read: failed to open file");
        return CFD_ERROR_IO;
    }
    chk_rd r{file.fp, CFD_SUCCESS, 0xFFFFFFFFu, T.get()};
    grid* g = nullptr;
    uint16_t flags = 0;
    chk_get_prefix(&r, &g, &flags);
    if (r.st == CFD_SUCCESS && (g->nx != c->nx || g->ny != c->ny || g->nz != c->nz))
        r.st = CFD_ERROR_INVALID;  // the context's dimensions are fixed at creation
    // fields land in scratch: u v w p rho T -> us vs ws pn r pa
    double* dst[CHK_NFIELDS] = {c->us, c->vs, c->ws, c->pn, c->r, c->pa};
    Pinned stage[2];
    EventPair ev;
    double rho0 = c->rho0;
    if (r.st == CFD_SUCCESS) {
        const size_t kp = stage_planes(c);
        const size_t row = c->nx * sizeof(double);
        if (hipHostMalloc(&stage[0].p, kp * c->ny * row, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&stage[1].p, kp * c->ny * row, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&ev.e[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ev.e[1], hipEventDisableTiming) != hipSuccess)
            r.st = CFD_ERROR_NOMEM;
        const size_t nchunk = (c->nz + kp - 1) / kp;
        bool used[2] = {false, false};
        for (size_t m = 0; m < CHK_NFIELDS * nchunk && r.st == CFD_SUCCESS; ++m) {
            const int q = (int)(m / nchunk), b = (int)(m & 1);
            const size_t k0 = (m % nchunk) * kp, nk = std::min(kp, c->nz - k0);
            const size_t bytes = nk * c->ny * row;
            // buffer b is free once its previous upload finished
            if (used[b] && hipEventSynchronize(ev.e[b]) != hipSuccess) r.st = CFD_ERROR;
            if (r.st == CFD_SUCCESS && fread(stage[b].p, 1, bytes, file.fp) != bytes)
                r.st = CFD_ERROR_IO;
            if (r.st != CFD_SUCCESS) break;
            if (q == 4 && k0 == 0) memcpy(&rho0, stage[b].p, sizeof(double));
            if (hipMemcpy2DAsync(dst[q] + k0 * c->ps, c->px * sizeof(double), stage[b].p, row, row,
                                 c->ny * nk, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
                hipEventRecord(ev.e[b], c->stream) != hipSuccess)
                r.st = CFD_ERROR;
            used[b] = true;
        }
        hipStreamSynchronize(c->stream);
    }
    if (r.st == CFD_SUCCESS) {
        // the field bytes join the running CRC from the device, then the
        // suffix continues on the host
        uint32_t raw[CHK_NFIELDS];
        const double* fs[CHK_NFIELDS] = {dst[0], dst[1], dst[2], dst[3], dst[4], dst[5]};
        if (device_crcs(c, fs, CHK_NFIELDS, raw) != CFD_SUCCESS) {
            r.st = CFD_ERROR;
        } else {
            const uint64_t fbytes = (uint64_t)c->nx * c->ny * c->nz * sizeof(double);
            for (int q = 0; q < CHK_NFIELDS; ++q) r.crc = chk_crc_join(r.crc, fbytes, raw[q]);
        }
    }
    double tm = 0.0;
    chk_get_suffix(&r, out_params, &tm, out_solver_name, solver_name_cap, out_run_prefix,
                   run_prefix_cap, out_output_base_dir, output_base_dir_cap);
    chk_check_trailer(&r, flags);
    if (fclose(file.fp) != 0 && r.st == CFD_SUCCESS) r.st = CFD_ERROR_IO;
    file.fp = nullptr;
    if (r.st == CFD_SUCCESS && !c->T && dalloc(c, &c->T, field_elems(c)) != CFD_SUCCESS)
        r.st = CFD_ERROR_NOMEM;
    // the file's density may be non-uniform: keep it per cell (RK4 reads rho[idx])
    if (r.st == CFD_SUCCESS && !c->rho && dalloc(c, &c->rho, field_elems(c)) != CFD_SUCCESS)
        r.st = CFD_ERROR_NOMEM;
    if (r.st == CFD_SUCCESS) {
        // verified: the scratch copies become the state
        const size_t bytes = field_elems(c) * sizeof(double);
        double* state[CHK_NFIELDS] = {c->u, c->v, c->w, c->p, c->rho, c->T};
        for (int q = 0; q < CHK_NFIELDS && r.st == CFD_SUCCESS; ++q) {
            if (hipMemcpyAsync(state[q], dst[q], bytes, hipMemcpyDeviceToDevice, c->stream) !=
                hipSuccess)
                r.st = CFD_ERROR;
        }
        if (hipStreamSynchronize(c->stream) != hipSuccess) r.st = CFD_ERROR;
        c->rho0 = rho0;
        c->have_T = c->T_dirty = 1;
        c->resident = 0;
    }
    for (int q = 0; q < CHK_NFIELDS; q += 2) scrub_scratch(c, dst[q], dst[q + 1]);
    if (r.st != CFD_SUCCESS) {
        if (g) {
            free(g->x); free(g->y); free(g->dx); free(g->dy); free(g->z); free(g->dz);
            free(g);
        }
        set_err(r.st, "hip_proj_checkpoint_read: read failed");
        return r.st;
    }
    if (out_grid) {
        *out_grid = g;
    } else {
        free(g->x); free(g->y); free(g->dx); free(g->dy); free(g->z); free(g->dz);
        free(g);
    }
    if (out_current_time) *out_current_time = tm;
    return CFD_SUCCESS;
}

}  // extern "C"
