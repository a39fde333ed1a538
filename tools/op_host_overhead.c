/* op_host_overhead.c -- what op/hip adds to a reduction on HOST buffers.
 *
 * In Open MPI every ompi_op_reduce -- MPI_Reduce_local, and coll/tuned's on its host temporaries --
 * dispatches through the op's slot table (ompi/op/op.h:570-574: one indirect call to the base
 * loop).  With op/hip selected that slot is mca_op_hip_2buff, which classifies its operands before
 * handing host ones to the saved base loop.  This tool times, in one process on the host:
 *   base       the base loop called directly (op_base_functions.c's 2-buff SUM on float,
 *              restated here: inout[i] = inout[i] + in[i])
 *   table      ompi_op_reduce through an op selected WITHOUT op/hip (the reference's dispatch)
 *   op_hip     ompi_op_reduce through an op selected WITH op/hip (mca_op_hip_2buff in the slot)
 *   ptr_query  mi355x_ptr_is_device on the same host pointer, alone
 * at count 1, 16, 1 Ki and 64 Ki floats; one JSON line per (variant, count), nanoseconds per call
 * (median of 7 timed batches).  Needs the HIP runtime (the pointer query), so it runs on the GPU box.
 * build: make -C tools (links libompi_mini + libmi355x_rt; dlopens mca_op_hip.so) */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "../ompi-release_amd/csrc/harness/ompi_mini.h"
#include "mi355x_rt.h"

static void base2_sum_float(void *in, void *inout, int *count, struct ompi_datatype_t **dt,
                            struct ompi_op_base_module_1_0_0_t *m)
{
    (void)dt;
    (void)m;
    const float *a = (const float *)in;
    float *b = (float *)inout;
    for (int i = 0; i < *count; ++i) b[i] = b[i] + a[i];
}

static void base3_sum_float(void *in1, void *in2, void *out, int *count, struct ompi_datatype_t **dt,
                            struct ompi_op_base_module_1_0_0_t *m)
{
    (void)dt;
    (void)m;
    const float *a = (const float *)in1, *b = (const float *)in2;
    float *o = (float *)out;
    for (int i = 0; i < *count; ++i) o[i] = a[i] + b[i];
}

static double now_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e9 + t.tv_nsec;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

enum { V_BASE, V_TABLE, V_OPHIP, V_QUERY };
static const char *vname[] = {"base", "table", "op_hip", "ptr_query"};

int main(int argc, char **argv)
{
    const char *libdir = argc > 1 ? argv[1] : "ompi-release_amd/lib";
    char path[512];
    snprintf(path, sizeof(path), "%s/mca_op_hip.so", libdir);
    void *h = dlopen(path, RTLD_NOW);
    if (!h) {
        fprintf(stderr, "%s\n", dlerror());
        return 1;
    }
    ompi_op_base_component_t *comp = (ompi_op_base_component_t *)dlsym(h, "mca_op_hip_component");
    if (!comp || comp->opc_init_query(false, false) != OMPI_SUCCESS) {
        fprintf(stderr, "op/hip unavailable (no GPU?)\n");
        return 1;
    }
    mini_init();
    mini_set_base_function(MI355X_OP_SUM, MI355X_T_FLOAT, (void *)base2_sum_float, (void *)base3_sum_float);
    ompi_op_t *plain = mini_op_create(MI355X_OP_SUM), *hip = mini_op_create(MI355X_OP_SUM);
    if (mini_op_select(plain, NULL, 0) || mini_op_select(hip, &comp, 1)) {
        fprintf(stderr, "op select failed\n");
        return 1;
    }
    ompi_datatype_t *dt = mini_datatype(mini_datatype_id_for_slot(MI355X_T_FLOAT));
    const int counts[] = {1, 16, 1024, 65536};
    for (int ci = 0; ci < 4; ++ci) {
        const int n = counts[ci];
        /* the buffers a host reduction of this size gets from malloc: the brk heap below glibc's mmap
         * threshold (128 KiB), an anonymous mapping above it */
        float *a = calloc((size_t)n, sizeof(float)), *b = calloc((size_t)n, sizeof(float));
        const long reps = n <= 16 ? 200000 : n <= 1024 ? 50000 : 2000;
        double med[4];
        for (int v = 0; v < 4; ++v) {
            double t[7];
            for (int k = 0; k < 7; ++k) {
                int cnt = n, d = 0;
                ompi_datatype_t *dp = dt;
                const double t0 = now_ns();
                for (long r = 0; r < reps; ++r) {
                    switch (v) {
                    case V_BASE: base2_sum_float(a, b, &cnt, &dp, NULL); break;
                    case V_TABLE: mini_op_reduce(plain, a, b, n, dt); break;
                    case V_OPHIP: mini_op_reduce(hip, a, b, n, dt); break;
                    default: mi355x_ptr_is_device(a, &d); break;
                    }
                }
                t[k] = (now_ns() - t0) / (double)reps;
            }
            qsort(t, 7, sizeof(double), cmp_d);
            med[v] = t[3];
        }
        for (int v = 0; v < 4; ++v)
            printf("{\"variant\": \"%s\", \"count\": %d, \"ns_per_call\": %.1f%s}\n", vname[v], n, med[v],
                   v == V_OPHIP ? "" : "");
        printf("{\"count\": %d, \"op_hip_over_table_ns\": %.1f, \"op_hip_over_table_frac\": %.4f}\n", n,
               med[V_OPHIP] - med[V_TABLE], (med[V_OPHIP] - med[V_TABLE]) / med[V_TABLE]);
        free(a);
        free(b);
    }
    /* the classification of host memory outside the brk heap and the stack: a private anonymous
     * mapping (glibc's allocations above the mmap threshold) and a shared one (shared-memory
     * segments), each with the op_hip reduction at count 16 on it */
    for (int kind = 0; kind < 2; ++kind) {
        const size_t bytes = (size_t)1 << 20;
        float *m = (float *)mmap(NULL, bytes, PROT_READ | PROT_WRITE, (kind ? MAP_SHARED : MAP_PRIVATE) | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) continue;
        memset(m, 0, bytes);
        double tq[7], tr[7];
        for (int k = 0; k < 7; ++k) {
            int d = 0;
            double t0 = now_ns();
            for (long r = 0; r < 100000; ++r) mi355x_ptr_is_device(m + 1024, &d);
            tq[k] = (now_ns() - t0) / 1e5;
            t0 = now_ns();
            for (long r = 0; r < 100000; ++r) mini_op_reduce(hip, m, m + 4096, 16, dt);
            tr[k] = (now_ns() - t0) / 1e5;
        }
        qsort(tq, 7, sizeof(double), cmp_d);
        qsort(tr, 7, sizeof(double), cmp_d);
        printf("{\"variant\": \"ptr_query_%s\", \"ns_per_call\": %.1f}\n", kind ? "mmap_shared" : "mmap_private", tq[3]);
        printf("{\"variant\": \"op_hip_%s\", \"count\": 16, \"ns_per_call\": %.1f}\n", kind ? "mmap_shared" : "mmap_private", tr[3]);
        munmap(m, bytes);
    }
    fflush(stdout);
    mini_op_destroy(plain);
    mini_op_destroy(hip);
    return 0;
}
