/*
 * chk_format.h -- the `.cfdchk` restart format of the reference
 * (lib/include/cfd/io/checkpoint.h:16-47, lib/src/io/checkpoint.c), shared by
 * the host mirror (cfd_checkpoint_write/read in libcfd_host.so: host arrays,
 * CRC on the CPU) and the device path (hip_proj_checkpoint_write/read in
 * libcfd_hip.so: field arrays streamed between HBM and the file, CRC computed
 * on the GPU).
 *
 * Stream layout (all little-endian; order of checkpoint.c:249-327,357-364):
 *   prefix  magic "CFDCHK\0\0", u32 format version 1, u32 endian marker
 *           0x01020304, u16 x3 library version 0.3.0, u16 flags (bit 0: CRC
 *           present), u64 reserved 0; grid: u64 nx ny nz, f64 xmin xmax ymin
 *           ymax zmin zmax, f64 x[nx] y[ny] dx[nx-1] dy[ny-1] and, when nz > 1,
 *           z[nz] dz[nz-1] inv_dz2; field dims u64 nx ny nz
 *   fields  f64 u, v, w, p, rho, T (nx*ny*nz each, idx = k*nx*ny + j*nx + i)
 *   suffix  params (f64 dt cfl gamma mu k, i32 max_iter, f64 tolerance
 *           amp_u amp_v decay pressure_coupling alpha beta T_ref g[3], i32
 *           thermal BC types left right bottom top front back, f64 Dirichlet
 *           values left right top bottom front back), f64 time, three
 *           u32-length-prefixed strings (solver name, run prefix, base dir)
 *   trailer u32 CRC-32 (IEEE, reflected 0xEDB88320, init/xorout 0xFFFFFFFF)
 *           of every byte before it
 *
 * CRC arithmetic is kept in "raw register" form: crc_update(state, bytes)
 * with state starting at 0xFFFFFFFF; the final CRC is state ^ 0xFFFFFFFF.
 * The register is linear over GF(2), so a block B computed elsewhere from a
 * zero register (raw0(B), e.g. on the GPU) joins a running state S as
 * S' = shift(S, |B|) ^ raw0(B), shift(S, n) = S * x^(8n) mod P.
 */
#ifndef CFD_HIP_CHK_FORMAT_H
#define CFD_HIP_CHK_FORMAT_H

#include "cfd_hip/cfd_abi.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK_VERSION       1u
#define CHK_ENDIAN        0x01020304u
#define CHK_FLAG_CRC      0x0001u
#define CHK_LIB_MAJOR     0u /* reference cfd_version.h:11-13 */
#define CHK_LIB_MINOR     3u
#define CHK_LIB_PATCH     0u
#define CHK_DIM_LIMIT     (1ull << 24) /* reader sanity caps (checkpoint.c:32-33) */
#define CHK_STR_LIMIT     (1u << 20)
#define CHK_POLY          0xEDB88320u
#define CHK_NFIELDS       6

static const unsigned char chk_magic[8] = {'C', 'F', 'D', 'C', 'H', 'K', 0, 0};

static inline int chk_host_little_endian(void) {
    const uint32_t one = 1u;
    unsigned char b;
    memcpy(&b, &one, 1);
    return b == 1;
}

/* ---- CRC-32: slicing-by-8 tables and GF(2) register arithmetic --------- */
typedef struct {
    uint32_t t[8][256];
} chk_crc_tables;

static inline void chk_crc_tables_init(chk_crc_tables* T) {
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ CHK_POLY : c >> 1;
        T->t[0][b] = c;
    }
    for (int s = 1; s < 8; s++)
        for (uint32_t b = 0; b < 256; b++)
            T->t[s][b] = (T->t[s - 1][b] >> 8) ^ T->t[0][T->t[s - 1][b] & 255u];
}

/* register after appending n bytes (little-endian host: 8 bytes per step) */
static inline uint32_t chk_crc_update(const chk_crc_tables* T, uint32_t s, const void* data,
                                      size_t n) {
    const unsigned char* p = (const unsigned char*)data;
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= s;
        s = T->t[7][lo & 255u] ^ T->t[6][(lo >> 8) & 255u] ^ T->t[5][(lo >> 16) & 255u] ^
            T->t[4][lo >> 24] ^ T->t[3][hi & 255u] ^ T->t[2][(hi >> 8) & 255u] ^
            T->t[1][(hi >> 16) & 255u] ^ T->t[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) s = (s >> 8) ^ T->t[0][(s ^ *p++) & 255u];
    return s;
}

/* a(x) * b(x) mod P in the reflected representation (x^0 = 0x80000000) */
static inline uint32_t chk_gf_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 32; i++) {
        if (a & 0x80000000u) r ^= b;
        a <<= 1;
        b = (b & 1u) ? (b >> 1) ^ CHK_POLY : b >> 1;
    }
    return r;
}

/* x^(8 n) mod P: the operator that moves a register past n zero bytes */
static inline uint32_t chk_xpow_bytes(uint64_t n) {
    uint32_t r = 0x80000000u;   /* x^0 */
    uint32_t sq = 0x00800000u;  /* x^8 */
    while (n) {
        if (n & 1u) r = chk_gf_mul(r, sq);
        sq = chk_gf_mul(sq, sq);
        n >>= 1;
    }
    return r;
}

/* running register S followed by a block of n bytes whose zero-register
 * CRC is raw0 */
static inline uint32_t chk_crc_join(uint32_t s, uint64_t n, uint32_t raw0) {
    return chk_gf_mul(chk_xpow_bytes(n), s) ^ raw0;
}

/* ---- little-endian byte buffer ----------------------------------------- */
typedef struct {
    unsigned char* p;
    size_t n, cap;
    int oom;
} chk_buf;

static inline void chk_buf_free(chk_buf* b) {
    free(b->p);
    b->p = NULL;
    b->n = b->cap = 0;
}

static inline void chk_put_bytes(chk_buf* b, const void* src, size_t n) {
    if (b->oom || n == 0) return;
    if (b->n + n > b->cap) {
        size_t cap = b->cap ? b->cap : 1024;
        while (cap < b->n + n) cap *= 2;
        unsigned char* q = (unsigned char*)realloc(b->p, cap);
        if (!q) {
            b->oom = 1;
            return;
        }
        b->p = q;
        b->cap = cap;
    }
    memcpy(b->p + b->n, src, n);
    b->n += n;
}

static inline void chk_put_le(chk_buf* b, uint64_t v, int nbytes) {
    unsigned char t[8];
    for (int i = 0; i < nbytes; i++) t[i] = (unsigned char)(v >> (8 * i));
    chk_put_bytes(b, t, (size_t)nbytes);
}

static inline void chk_put_f64(chk_buf* b, double v) {
    uint64_t u;
    memcpy(&u, &v, 8);
    chk_put_le(b, u, 8);
}

static inline void chk_put_f64s(chk_buf* b, const double* a, size_t n) {
    for (size_t i = 0; i < n; i++) chk_put_f64(b, a[i]);
}

static inline void chk_put_str(chk_buf* b, const char* s) {
    const size_t len = s ? strlen(s) : 0;
    chk_put_le(b, (uint64_t)len, 4);
    chk_put_bytes(b, s, len);
}

/* header + grid + field dimensions (checkpoint.c:249-286) */
static inline void chk_put_prefix(chk_buf* b, const grid* g) {
    chk_put_bytes(b, chk_magic, 8);
    chk_put_le(b, CHK_VERSION, 4);
    chk_put_le(b, CHK_ENDIAN, 4);
    chk_put_le(b, CHK_LIB_MAJOR, 2);
    chk_put_le(b, CHK_LIB_MINOR, 2);
    chk_put_le(b, CHK_LIB_PATCH, 2);
    chk_put_le(b, CHK_FLAG_CRC, 2);
    chk_put_le(b, 0, 8);
    chk_put_le(b, g->nx, 8);
    chk_put_le(b, g->ny, 8);
    chk_put_le(b, g->nz, 8);
    const double lim[6] = {g->xmin, g->xmax, g->ymin, g->ymax, g->zmin, g->zmax};
    chk_put_f64s(b, lim, 6);
    chk_put_f64s(b, g->x, g->nx);
    chk_put_f64s(b, g->y, g->ny);
    chk_put_f64s(b, g->dx, g->nx - 1);
    chk_put_f64s(b, g->dy, g->ny - 1);
    if (g->nz > 1) {
        chk_put_f64s(b, g->z, g->nz);
        chk_put_f64s(b, g->dz, g->nz - 1);
        chk_put_f64(b, g->inv_dz2);
    }
    chk_put_le(b, g->nx, 8);
    chk_put_le(b, g->ny, 8);
    chk_put_le(b, g->nz, 8);
}

/* scalar parameters, time and the three strings (checkpoint.c:295-327,361-364) */
static inline void chk_put_suffix(chk_buf* b, const ns_solver_params_t* p, double time,
                                  const char* solver, const char* prefix, const char* base) {
    const double a[5] = {p->dt, p->cfl, p->gamma, p->mu, p->k};
    chk_put_f64s(b, a, 5);
    chk_put_le(b, (uint32_t)p->max_iter, 4);
    const double c[11] = {p->tolerance, p->source_amplitude_u, p->source_amplitude_v,
                          p->source_decay_rate, p->pressure_coupling, p->alpha, p->beta,
                          p->T_ref, p->gravity[0], p->gravity[1], p->gravity[2]};
    chk_put_f64s(b, c, 11);
    const ns_thermal_bc_config_t* t = &p->thermal_bc;
    const int32_t ty[6] = {(int32_t)t->left, (int32_t)t->right, (int32_t)t->bottom,
                           (int32_t)t->top, (int32_t)t->front, (int32_t)t->back};
    for (int i = 0; i < 6; i++) chk_put_le(b, (uint32_t)ty[i], 4);
    const bc_dirichlet_values_t* d = &t->dirichlet_values;
    const double dv[6] = {d->left, d->right, d->top, d->bottom, d->front, d->back};
    chk_put_f64s(b, dv, 6);
    chk_put_f64(b, time);
    chk_put_str(b, solver);
    chk_put_str(b, prefix);
    chk_put_str(b, base);
}

/* ---- reader: latching status, running CRC register ---------------------- */
typedef struct {
    FILE* fp;
    cfd_status_t st;
    uint32_t crc;
    const chk_crc_tables* T;
} chk_rd;

static inline void chk_get_bytes(chk_rd* r, void* dst, size_t n) {
    if (r->st != CFD_SUCCESS || n == 0) return;
    if (fread(dst, 1, n, r->fp) != n) {
        r->st = CFD_ERROR_IO;
        memset(dst, 0, n);
        return;
    }
    r->crc = chk_crc_update(r->T, r->crc, dst, n);
}

static inline uint64_t chk_get_le(chk_rd* r, int nbytes) {
    unsigned char t[8] = {0};
    chk_get_bytes(r, t, (size_t)nbytes);
    uint64_t v = 0;
    for (int i = 0; i < nbytes; i++) v |= (uint64_t)t[i] << (8 * i);
    return v;
}

static inline double chk_get_f64(chk_rd* r) {
    uint64_t u = chk_get_le(r, 8);
    double v;
    memcpy(&v, &u, 8);
    return v;
}

static inline void chk_get_f64s(chk_rd* r, double* a, size_t n) {
    for (size_t i = 0; i < n; i++) a[i] = chk_get_f64(r);
}

/* length-prefixed string into buf (NULL: consumed); INVALID when the stored
 * length is implausible or does not fit the caller's buffer */
static inline void chk_get_str(chk_rd* r, char* buf, size_t cap) {
    const uint64_t len = chk_get_le(r, 4);
    if (r->st != CFD_SUCCESS) return;
    if (len > CHK_STR_LIMIT || (buf && (cap == 0 || len + 1 > cap))) {
        r->st = CFD_ERROR_INVALID;
        return;
    }
    unsigned char tmp[512];
    uint64_t left = len;
    size_t at = 0;
    while (left && r->st == CFD_SUCCESS) {
        const size_t k = left < sizeof(tmp) ? (size_t)left : sizeof(tmp);
        chk_get_bytes(r, tmp, k);
        if (buf && r->st == CFD_SUCCESS) memcpy(buf + at, tmp, k);
        at += k;
        left -= k;
    }
    if (buf && r->st == CFD_SUCCESS) buf[len] = '\0';
}

/* Header and grid. Allocates *gout (calloc'd arrays, freed by grid_destroy)
 * on success; leaves it NULL on failure. */
static inline void chk_get_prefix(chk_rd* r, grid** gout, uint16_t* flags) {
    *gout = NULL;
    unsigned char m[8];
    chk_get_bytes(r, m, 8);
    if (r->st == CFD_SUCCESS && memcmp(m, chk_magic, 8) != 0) r->st = CFD_ERROR_INVALID;
    const uint64_t ver = chk_get_le(r, 4), endian = chk_get_le(r, 4);
    (void)chk_get_le(r, 6); /* library version */
    *flags = (uint16_t)chk_get_le(r, 2);
    (void)chk_get_le(r, 8);
    if (r->st == CFD_SUCCESS && (ver != CHK_VERSION || endian != CHK_ENDIAN))
        r->st = CFD_ERROR_UNSUPPORTED;
    const uint64_t nx = chk_get_le(r, 8), ny = chk_get_le(r, 8), nz = chk_get_le(r, 8);
    double lim[6];
    chk_get_f64s(r, lim, 6);
    if (r->st != CFD_SUCCESS) return;
    if (nx < 2 || ny < 2 || nz < 1 || nx > CHK_DIM_LIMIT || ny > CHK_DIM_LIMIT ||
        nz > CHK_DIM_LIMIT) {
        r->st = CFD_ERROR_INVALID;
        return;
    }
    /* the reference rebuilds the grid with grid_create, which refuses empty
     * bounds; its reader reports that as an allocation failure */
    if (!(lim[1] > lim[0]) || !(lim[3] > lim[2]) || (nz > 1 && !(lim[5] > lim[4]))) {
        r->st = CFD_ERROR_NOMEM;
        return;
    }
    grid* g = (grid*)calloc(1, sizeof(grid));
    if (!g) {
        r->st = CFD_ERROR_NOMEM;
        return;
    }
    g->nx = (size_t)nx;
    g->ny = (size_t)ny;
    g->nz = (size_t)nz;
    g->xmin = lim[0];
    g->xmax = lim[1];
    g->ymin = lim[2];
    g->ymax = lim[3];
    g->x = (double*)calloc(g->nx, sizeof(double));
    g->y = (double*)calloc(g->ny, sizeof(double));
    g->dx = (double*)calloc(g->nx - 1, sizeof(double));
    g->dy = (double*)calloc(g->ny - 1, sizeof(double));
    int ok = g->x && g->y && g->dx && g->dy;
    if (g->nz > 1) {
        g->zmin = lim[4];
        g->zmax = lim[5];
        g->z = (double*)calloc(g->nz, sizeof(double));
        g->dz = (double*)calloc(g->nz - 1, sizeof(double));
        ok = ok && g->z && g->dz;
        g->stride_z = g->nx * g->ny;
        g->k_start = 1;
        g->k_end = g->nz - 1;
    } else {
        g->k_start = 0;
        g->k_end = 1;
    }
    if (ok) {
        chk_get_f64s(r, g->x, g->nx);
        chk_get_f64s(r, g->y, g->ny);
        chk_get_f64s(r, g->dx, g->nx - 1);
        chk_get_f64s(r, g->dy, g->ny - 1);
        if (g->nz > 1) {
            chk_get_f64s(r, g->z, g->nz);
            chk_get_f64s(r, g->dz, g->nz - 1);
            g->inv_dz2 = chk_get_f64(r);
        }
        const uint64_t fx = chk_get_le(r, 8), fy = chk_get_le(r, 8), fz = chk_get_le(r, 8);
        if (r->st == CFD_SUCCESS && (fx != nx || fy != ny || fz != nz)) r->st = CFD_ERROR_INVALID;
    } else if (r->st == CFD_SUCCESS) {
        r->st = CFD_ERROR_NOMEM;
    }
    if (r->st != CFD_SUCCESS) {
        free(g->x); free(g->y); free(g->dx); free(g->dy); free(g->z); free(g->dz);
        free(g);
        return;
    }
    *gout = g;
}

/* parameters (callbacks left NULL), time, strings */
static inline void chk_get_suffix(chk_rd* r, ns_solver_params_t* p, double* time, char* solver,
                                  size_t solver_cap, char* prefix, size_t prefix_cap, char* base,
                                  size_t base_cap) {
    memset(p, 0, sizeof(*p));
    p->dt = chk_get_f64(r);
    p->cfl = chk_get_f64(r);
    p->gamma = chk_get_f64(r);
    p->mu = chk_get_f64(r);
    p->k = chk_get_f64(r);
    p->max_iter = (int32_t)(uint32_t)chk_get_le(r, 4);
    p->tolerance = chk_get_f64(r);
    p->source_amplitude_u = chk_get_f64(r);
    p->source_amplitude_v = chk_get_f64(r);
    p->source_decay_rate = chk_get_f64(r);
    p->pressure_coupling = chk_get_f64(r);
    p->alpha = chk_get_f64(r);
    p->beta = chk_get_f64(r);
    p->T_ref = chk_get_f64(r);
    for (int i = 0; i < 3; i++) p->gravity[i] = chk_get_f64(r);
    ns_thermal_bc_config_t* t = &p->thermal_bc;
    t->left = (bc_type_t)(int32_t)(uint32_t)chk_get_le(r, 4);
    t->right = (bc_type_t)(int32_t)(uint32_t)chk_get_le(r, 4);
    t->bottom = (bc_type_t)(int32_t)(uint32_t)chk_get_le(r, 4);
    t->top = (bc_type_t)(int32_t)(uint32_t)chk_get_le(r, 4);
    t->front = (bc_type_t)(int32_t)(uint32_t)chk_get_le(r, 4);
    t->back = (bc_type_t)(int32_t)(uint32_t)chk_get_le(r, 4);
    bc_dirichlet_values_t* d = &t->dirichlet_values;
    d->left = chk_get_f64(r);
    d->right = chk_get_f64(r);
    d->top = chk_get_f64(r);
    d->bottom = chk_get_f64(r);
    d->front = chk_get_f64(r);
    d->back = chk_get_f64(r);
    const double tm = chk_get_f64(r);
    if (time) *time = tm;
    chk_get_str(r, solver, solver_cap);
    chk_get_str(r, prefix, prefix_cap);
    chk_get_str(r, base, base_cap);
}

/* trailing CRC (not part of the register), checked when the flag is set */
static inline void chk_check_trailer(chk_rd* r, uint16_t flags) {
    if (!(flags & CHK_FLAG_CRC) || r->st != CFD_SUCCESS) return;
    unsigned char t[4];
    if (fread(t, 1, 4, r->fp) != 4) {
        r->st = CFD_ERROR_IO;
        return;
    }
    const uint32_t stored = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) |
                            ((uint32_t)t[3] << 24);
    if (stored != (r->crc ^ 0xFFFFFFFFu)) r->st = CFD_ERROR_IO;
}

static inline int chk_write_trailer(FILE* fp, uint32_t state) {
    const uint32_t c = state ^ 0xFFFFFFFFu;
    const unsigned char t[4] = {(unsigned char)c, (unsigned char)(c >> 8),
                                (unsigned char)(c >> 16), (unsigned char)(c >> 24)};
    return fwrite(t, 1, 4, fp) == 4;
}

#endif /* CFD_HIP_CHK_FORMAT_H */
