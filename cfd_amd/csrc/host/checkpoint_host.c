/*
 * checkpoint_host.c -- the reference's restart API on host arrays, for the
 * standalone host mirror (libcfd_host.so):
 *   cfd_checkpoint_write / cfd_checkpoint_read   lib/include/cfd/io/checkpoint.h:49-115
 *   save_simulation_checkpoint,
 *   load_simulation_from_checkpoint,
 *   restore_simulation_checkpoint                lib/include/cfd/api/simulation_api.h:93-111,
 *                                                lib/src/api/simulation_api.c:257-440
 * Same file format, status codes and ownership rules as the reference; the
 * stream is assembled in memory (prefix / fields / suffix) and the CRC is a
 * slicing-by-8 register over it (chk_format.h). The device-resident variant,
 * which streams fields straight from HBM and computes their CRC on the GPU,
 * is hip_proj_checkpoint_write/read in libcfd_hip.so.
 */
#include "cfd_hip/cfd_host.h"

#include "chk_format.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const double* const* field_arrays(const flow_field* f, const double* a[CHK_NFIELDS]) {
    a[0] = f->u;
    a[1] = f->v;
    a[2] = f->w;
    a[3] = f->p;
    a[4] = f->rho;
    a[5] = f->T;
    return a;
}

cfd_status_t cfd_checkpoint_write(const char* path, const grid* g, const flow_field* field,
                                  const ns_solver_params_t* params, double current_time,
                                  const char* solver_name, const char* run_prefix,
                                  const char* output_base_dir) {
    if (!path || !g || !field || !params || !solver_name) {
        cfd_set_error(CFD_ERROR_INVALID, "cfd_checkpoint_write: NULL argument");
        return CFD_ERROR_INVALID;
    }
    if (field->nx != g->nx || field->ny != g->ny || field->nz != g->nz) {
        cfd_set_error(CFD_ERROR_INVALID, "cfd_checkpoint_write: field/grid dimension mismatch");
        return CFD_ERROR_INVALID;
    }
    if (!chk_host_little_endian()) {
        cfd_set_error(CFD_ERROR_UNSUPPORTED, "cfd_checkpoint_write: big-endian host");
        return CFD_ERROR_UNSUPPORTED;
    }
    chk_crc_tables* T = (chk_crc_tables*)malloc(sizeof(chk_crc_tables));
    chk_buf pre = {0}, suf = {0};
    if (!T) return CFD_ERROR_NOMEM;
    chk_crc_tables_init(T);
    chk_put_prefix(&pre, g);
    chk_put_suffix(&suf, params, current_time, solver_name, run_prefix, output_base_dir);
    cfd_status_t st = (pre.oom || suf.oom) ? CFD_ERROR_NOMEM : CFD_SUCCESS;
    FILE* fp = NULL;
    if (st == CFD_SUCCESS && !(fp = fopen(path, "wb"))) st = CFD_ERROR_IO;
    if (st == CFD_SUCCESS) {
        const size_t n = g->nx * g->ny * g->nz;
        const double* a[CHK_NFIELDS];
        field_arrays(field, a);
        uint32_t crc = chk_crc_update(T, 0xFFFFFFFFu, pre.p, pre.n);
        if (fwrite(pre.p, 1, pre.n, fp) != pre.n) st = CFD_ERROR_IO;
        for (int q = 0; q < CHK_NFIELDS && st == CFD_SUCCESS; q++) {
            /* x86 stores IEEE doubles little-endian: the array is the encoding */
            if (fwrite(a[q], sizeof(double), n, fp) != n) st = CFD_ERROR_IO;
            crc = chk_crc_update(T, crc, a[q], n * sizeof(double));
        }
        if (st == CFD_SUCCESS) {
            crc = chk_crc_update(T, crc, suf.p, suf.n);
            if (fwrite(suf.p, 1, suf.n, fp) != suf.n || !chk_write_trailer(fp, crc))
                st = CFD_ERROR_IO;
        }
        if (fclose(fp) != 0 && st == CFD_SUCCESS) st = CFD_ERROR_IO;
    }
    chk_buf_free(&pre);
    chk_buf_free(&suf);
    free(T);
    if (st != CFD_SUCCESS) cfd_set_error(st, "cfd_checkpoint_write: write failed");
    return st;
}

cfd_status_t cfd_checkpoint_read(const char* path, grid** out_grid, flow_field** out_field,
                                 ns_solver_params_t* out_params, double* out_current_time,
                                 char* out_solver_name, size_t solver_name_cap,
                                 char* out_run_prefix, size_t run_prefix_cap,
                                 char* out_output_base_dir, size_t output_base_dir_cap) {
    if (out_grid) *out_grid = NULL;
    if (out_field) *out_field = NULL;
    if (!path || !out_grid || !out_field || !out_params) {
        cfd_set_error(CFD_ERROR_INVALID, "cfd_checkpoint_read: NULL argument");
        return CFD_ERROR_INVALID;
    }
    memset(out_params, 0, sizeof(*out_params));
    if (!chk_host_little_endian()) {
        cfd_set_error(CFD_ERROR_UNSUPPORTED, "cfd_checkpoint_read: big-endian host");
        return CFD_ERROR_UNSUPPORTED;
    }
    chk_crc_tables* T = (chk_crc_tables*)malloc(sizeof(chk_crc_tables));
    if (!T) return CFD_ERROR_NOMEM;
    chk_crc_tables_init(T);
    FILE* fp = fopen(path, "rb");
    if (!fp) {
        free(T);
        cfd_set_error(CFD_ERROR_IO, "cfd_checkpoint_read: failed to open file");
        return CFD_ERROR_IO;
    }
    chk_rd r = {fp, CFD_SUCCESS, 0xFFFFFFFFu, T};
    grid* g = NULL;
    flow_field* f = NULL;
    uint16_t flags = 0;
    double tm = 0.0;
    chk_get_prefix(&r, &g, &flags);
    if (r.st == CFD_SUCCESS) {
        f = flow_field_create(g->nx, g->ny, g->nz);
        if (!f) r.st = CFD_ERROR_NOMEM;
    }
    if (r.st == CFD_SUCCESS) {
        const size_t n = g->nx * g->ny * g->nz;
        double* a[CHK_NFIELDS] = {f->u, f->v, f->w, f->p, f->rho, f->T};
        for (int q = 0; q < CHK_NFIELDS; q++) chk_get_bytes(&r, a[q], n * sizeof(double));
    }
    chk_get_suffix(&r, out_params, &tm, out_solver_name, solver_name_cap, out_run_prefix,
                   run_prefix_cap, out_output_base_dir, output_base_dir_cap);
    chk_check_trailer(&r, flags);
    if (fclose(fp) != 0 && r.st == CFD_SUCCESS) r.st = CFD_ERROR_IO;
    free(T);
    if (r.st != CFD_SUCCESS) {
        grid_destroy(g);
        flow_field_destroy(f);
        cfd_set_error(r.st, "cfd_checkpoint_read: read failed");
        return r.st;
    }
    *out_grid = g;
    *out_field = f;
    if (out_current_time) *out_current_time = tm;
    return CFD_SUCCESS;
}

/* ---- simulation-level wrappers (simulation_api.c:257-440) ---------------- */

cfd_status_t save_simulation_checkpoint(const simulation_data* sim, const char* path) {
    if (!sim || !path) {
        cfd_set_error(CFD_ERROR_INVALID, "save_simulation_checkpoint: NULL argument");
        return CFD_ERROR_INVALID;
    }
    if (!sim->grid || !sim->field || !sim->solver) {
        cfd_set_error(CFD_ERROR_INVALID, "save_simulation_checkpoint: simulation not initialized");
        return CFD_ERROR_INVALID;
    }
    return cfd_checkpoint_write(path, sim->grid, sim->field, &sim->params, sim->current_time,
                                sim->solver->name ? sim->solver->name : "", sim->run_prefix,
                                sim->output_base_dir);
}

typedef struct {
    grid* g;
    flow_field* f;
    ns_solver_params_t params;
    double time;
    char solver[128];
    char prefix[256];
    char base[512];
} chk_state;

static cfd_status_t read_state(const char* path, chk_state* s) {
    memset(s, 0, sizeof(*s));
    return cfd_checkpoint_read(path, &s->g, &s->f, &s->params, &s->time, s->solver,
                               sizeof(s->solver), s->prefix, sizeof(s->prefix), s->base,
                               sizeof(s->base));
}

simulation_data* load_simulation_from_checkpoint(const char* path) {
    if (!path) {
        cfd_set_error(CFD_ERROR_INVALID, "load_simulation_from_checkpoint: NULL path");
        return NULL;
    }
    chk_state s;
    if (read_state(path, &s) != CFD_SUCCESS) return NULL;
    simulation_data* sim = (simulation_data*)calloc(1, sizeof(simulation_data));
    if (!sim) {
        grid_destroy(s.g);
        flow_field_destroy(s.f);
        return NULL;
    }
    sim->grid = s.g;
    sim->field = s.f;
    sim->params = s.params;
    sim->last_stats = ns_solver_stats_default();
    sim->current_time = s.time;
    snprintf(sim->output_base_dir, sizeof(sim->output_base_dir), "%s",
             s.base[0] ? s.base : "../../artifacts");
    sim->registry = cfd_registry_create();
    if (!sim->registry) goto fail;
    cfd_registry_register_defaults(sim->registry);
    sim->solver = cfd_solver_create(sim->registry, s.solver);
    if (!sim->solver) {
        cfd_set_error(CFD_ERROR_NOT_FOUND, "load_simulation_from_checkpoint: solver not registered");
        goto fail;
    }
    if (solver_init(sim->solver, sim->grid, &sim->params) != CFD_SUCCESS) goto fail;
    if (s.prefix[0]) {
        sim->run_prefix = (char*)malloc(strlen(s.prefix) + 1);
        if (!sim->run_prefix) goto fail;
        strcpy(sim->run_prefix, s.prefix);
    }
    return sim;
fail:
    free_simulation(sim);
    return NULL;
}

cfd_status_t restore_simulation_checkpoint(simulation_data* sim, const char* path) {
    if (!sim || !path) {
        cfd_set_error(CFD_ERROR_INVALID, "restore_simulation_checkpoint: NULL argument");
        return CFD_ERROR_INVALID;
    }
    if (!sim->registry) {
        cfd_set_error(CFD_ERROR_INVALID, "restore_simulation_checkpoint: simulation not initialized");
        return CFD_ERROR_INVALID;
    }
    chk_state s;
    cfd_status_t st = read_state(path, &s);
    if (st != CFD_SUCCESS) return st;
    /* build the new solver first: any failure leaves the simulation as it was */
    ns_solver_t* solver = cfd_solver_create(sim->registry, s.solver);
    if (!solver) {
        grid_destroy(s.g);
        flow_field_destroy(s.f);
        cfd_set_error(CFD_ERROR_NOT_FOUND, "restore_simulation_checkpoint: solver not registered");
        return CFD_ERROR_NOT_FOUND;
    }
    s.params.source_func = sim->params.source_func;  /* callbacks are the caller's */
    s.params.source_context = sim->params.source_context;
    s.params.heat_source_func = sim->params.heat_source_func;
    s.params.heat_source_context = sim->params.heat_source_context;
    st = solver_init(solver, s.g, &s.params);
    if (st != CFD_SUCCESS) {
        solver_destroy(solver);
        grid_destroy(s.g);
        flow_field_destroy(s.f);
        return st;
    }
    if (sim->solver) solver_destroy(sim->solver);
    grid_destroy(sim->grid);
    flow_field_destroy(sim->field);
    sim->solver = solver;
    sim->grid = s.g;
    sim->field = s.f;
    sim->params = s.params;
    sim->current_time = s.time;
    if (s.prefix[0]) {  /* an allocation failure keeps the old prefix */
        char* prefix = (char*)malloc(strlen(s.prefix) + 1);
        if (prefix) {
            strcpy(prefix, s.prefix);
            free(sim->run_prefix);
            sim->run_prefix = prefix;
        }
    } else {
        free(sim->run_prefix);
        sim->run_prefix = NULL;
    }
    snprintf(sim->output_base_dir, sizeof(sim->output_base_dir), "%s",
             s.base[0] ? s.base : "../../artifacts");
    return CFD_SUCCESS;
}
