/* reference_driver.c -- a C program against the REAL reference API, linked by
 * tools/reference_link.py with the reference built from its own sources plus
 * the INTEGRATION.md section-1 edits, and with libcfd_hip.so. It reports, as
 * one JSON line:
 *  - which object defines gpu_is_available / solve_projection_method_gpu /
 *    cfd_hip_register_solvers (dladdr; the documented link puts them in
 *    libcfd_hip.so);
 *  - the registry's view: the backend the reference infers for the HIP names
 *    (solver_registry.c:257-279 with edit (b)), cfd_registry_list_by_backend
 *    (CUDA) and simulation_list_solvers (simulation_api.c:454-478, edit (d));
 *  - cfd_backend_is_available(CUDA) and what init_simulation_with_solver(...,
 *    "projection_hip") returns: on a box with no device the factory returns
 *    NULL with CFD_ERROR_UNSUPPORTED (solver_registry.c:1155-1181 pattern).
 * Compiled with the reference's headers only (plus cfd_hip/projection_hip.h
 * for the name macros, in its CFD_HIP_REFERENCE_TYPES mode). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include "cfd/api/simulation_api.h"
#include "cfd/core/cfd_init.h"
#include "cfd/core/cfd_status.h"
#include "cfd/core/gpu_device.h"
#include "cfd/solvers/navier_stokes_solver.h"

#define CFD_HIP_REFERENCE_TYPES 1
#include "cfd_hip/projection_hip.h"

static const char* where(void* fn) {
    Dl_info info;
    if (!fn || !dladdr(fn, &info) || !info.dli_fname) return "?";
    const char* s = strrchr(info.dli_fname, '/');
    return s ? s + 1 : info.dli_fname;
}

static int contains(const char** names, int n, const char* want) {
    for (int i = 0; i < n; ++i)
        if (names[i] && strcmp(names[i], want) == 0) return 1;
    return 0;
}

int main(void) {
    cfd_init();
    const char* hip_names[5] = {NS_SOLVER_TYPE_PROJECTION_HIP, NS_SOLVER_TYPE_PROJECTION_HIP_RBSOR,
                                NS_SOLVER_TYPE_PROJECTION_HIP_JACOBI, NS_SOLVER_TYPE_RK4_HIP,
                                NS_SOLVER_TYPE_PROJECTION_HIP_CG1};
    ns_solver_registry_t* reg = cfd_registry_create();
    cfd_registry_register_defaults(reg);
    const char* by_cuda[64];
    const int n_cuda = cfd_registry_list_by_backend(reg, NS_SOLVER_BACKEND_CUDA, by_cuda, 64);
    const char* listed[64];
    const int n_list = simulation_list_solvers(listed, 64);
    int in_cuda = 0, in_list = 0;
    for (int i = 0; i < 5; ++i) {
        in_cuda += contains(by_cuda, n_cuda, hip_names[i]);
        in_list += contains(listed, n_list, hip_names[i]);
    }
    const int cuda_avail = cfd_backend_is_available(NS_SOLVER_BACKEND_CUDA);
    const int gpu_avail = gpu_is_available();
    /* the registry's checked create: NULL while the backend is unavailable */
    cfd_clear_error();
    ns_solver_t* checked = cfd_solver_create_checked(reg, NS_SOLVER_TYPE_PROJECTION_HIP);
    const int checked_null = checked == NULL;
    if (checked) solver_destroy(checked);
    cfd_clear_error();
    simulation_data* sim = init_simulation_with_solver(17, 17, 17, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0,
                                                       NS_SOLVER_TYPE_PROJECTION_HIP);
    const cfd_status_t st = cfd_get_last_status();
    const char* err = cfd_get_last_error();
    char errbuf[160] = {0};
    if (err) {
        strncpy(errbuf, err, sizeof errbuf - 1);
        for (char* p = errbuf; *p; ++p)
            if (*p == '"' || *p == '\\') *p = '\'';
    }
    printf("{\"gpu_is_available\": \"%s\", \"solve_projection_method_gpu\": \"%s\", "
           "\"cfd_hip_register_solvers\": \"%s\", \"cfd_registry_register\": \"%s\", "
           "\"hip_names_by_cuda_backend\": %d, \"hip_names_in_simulation_list\": %d, "
           "\"n_cuda_backend\": %d, \"n_listed\": %d, \"cuda_backend_available\": %d, "
           "\"gpu_available\": %d, \"create_checked_null\": %d, \"init_sim_null\": %d, "
           "\"init_sim_status\": %d, \"init_sim_error\": \"%s\"}\n",
           where((void*)gpu_is_available), where((void*)solve_projection_method_gpu),
           where((void*)cfd_hip_register_solvers), where((void*)cfd_registry_register), in_cuda,
           in_list, n_cuda, n_list, cuda_avail, gpu_avail, checked_null, sim == NULL, (int)st,
           errbuf);
    if (sim) free_simulation(sim);
    cfd_registry_destroy(reg);
    return 0;
}
