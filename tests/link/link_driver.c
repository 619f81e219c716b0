/*
 * Test fixture: an application linked the way a reference build links
 * (tests/test_reference_link.py varies the order). Prints, for each GPU entry
 * point the registry object references, the file its definition came from.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <libgen.h>
#include <stdio.h>
#include <string.h>

int probe_backend_gpu_available(void);
void* probe_gpu_is_available(void);
void* probe_solve_projection_method_gpu(void);
void* probe_solve_rk4_method_gpu(void);
int probe_config_enable_gpu(void);

static const char* where(void* fn) {
    Dl_info info;
    static char buf[3][256];
    static int slot = 0;
    if (!dladdr(fn, &info) || !info.dli_fname) return "?";
    char* b = buf[slot++ % 3];
    snprintf(b, 256, "%s", info.dli_fname);
    return basename(b);
}

int main(void) {
    (void)probe_backend_gpu_available();
    printf("gpu_is_available %s\n", where(probe_gpu_is_available()));
    printf("solve_projection_method_gpu %s\n", where(probe_solve_projection_method_gpu()));
    printf("solve_rk4_method_gpu %s\n", where(probe_solve_rk4_method_gpu()));
    printf("enable_gpu %d\n", probe_config_enable_gpu());
    return 0;
}
