/* small_ar_c.c -- small-message MPI_Allreduce latency through the engine's C ABI, no Python in the
 * loop: N processes forked before any HIP call (all on device 0: the one-GPU rehearsal), each times
 * `reps` calls per size, plus mi355x_comm_barrier alone.  Rank 0 prints one JSON line per row.
 * usage: small_ar_c <nranks> <reps> [paths]   paths: comma list of host (per-call launch + host
 *        synchronisation), ll (per-call LL kernels), svc (resident LL service); default host
 *        SMALL_COLL=p2p_host / p2p_dev: MPI_Send / MPI_Recv ping-pong between ranks 0 and 1 through
 *        the engine (host malloc'd or device buffers), one-way microseconds per size
 * build: gcc -O2 -o tools/build/small_ar_c tools/small_ar_c.c -Iinclude -Lompi-release_amd/lib -lmi355x_rt
 *        -Wl,-rpath,'$ORIGIN/../../ompi-release_amd/lib' */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "mi355x_rt.h"

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int run(int rank, int n, int reps, const char *key, const char *paths)
{
    mi355x_comm_t *c = NULL;
    if (mi355x_set_device(0) || mi355x_comm_create(key, rank, n, 0, &c)) {
        fprintf(stderr, "rank %d: %s\n", rank, mi355x_last_error());
        return 1;
    }
    size_t sizes[16] = {8, 1024, 65536, 1 << 20};
    int nsizes = 4;
    const char *ss = getenv("SMALL_SIZES");  /* comma list of byte counts (<= 64 MiB) */
    if (ss) {
        char buf[256];
        snprintf(buf, sizeof(buf), "%s", ss);
        nsizes = 0;
        for (char *p = strtok(buf, ","); p && nsizes < 16; p = strtok(NULL, ",")) sizes[nsizes++] = strtoull(p, NULL, 10);
    }
    /* buffers sized for the largest message (allgather: n blocks of it); refuse what they cannot hold */
    size_t maxb = 0;
    for (int k = 0; k < nsizes; ++k) maxb = sizes[k] > maxb ? sizes[k] : maxb;
    if (maxb == 0 || maxb > ((size_t)64 << 20)) {
        fprintf(stderr, "SMALL_SIZES: sizes must be 1 .. 64 MiB\n");
        return 1;
    }
    void *s = NULL, *r = NULL;
    if (mi355x_malloc(&s, maxb) || mi355x_malloc(&r, (size_t)n * maxb)) {
        fprintf(stderr, "rank %d: %s\n", rank, mi355x_last_error());
        return 1;
    }
    mi355x_memset_async(s, 0, maxb, NULL);
    mi355x_device_sync();
    char pl[128];
    snprintf(pl, sizeof(pl), "%s", paths);
    for (char *path = strtok(pl, ","); path; path = strtok(NULL, ",")) {
    const int svc = strcmp(path, "svc") == 0, ll = strcmp(path, "ll") == 0;
    mi355x_comm_set(c, MI355X_KNOB_SVC_MAX_BYTES, svc ? 1 << 20 : 0);
    mi355x_comm_set(c, MI355X_KNOB_LL_MAX_BYTES, ll ? 1 << 20 : 0);
    long on = 0;
    mi355x_comm_get(c, svc ? MI355X_KNOB_SVC_MAX_BYTES : MI355X_KNOB_LL_MAX_BYTES, &on);
    if ((svc || ll) && !on) {
        if (rank == 0) printf("{\"path\": \"%s\", \"error\": \"not available\"}\n", path);
        continue;
    }
    const char *slp = getenv("SMALL_SLEEP_MS");  /* let an idle resident service leave first */
    if (slp) usleep(atoi(slp) * 1000);
    long resident = -1;
    mi355x_comm_get(c, MI355X_KNOB_SVC_RESIDENT, &resident);
    if (rank == 0) printf("{\"path\": \"%s\", \"svc_resident_before\": %ld}\n", path, resident);
    /* SMALL_TYPE / SMALL_OP: the (type, op) slot (default 14 = MPI_FLOAT, 3 = MPI_SUM), 4-B types */
    const int ty = getenv("SMALL_TYPE") ? atoi(getenv("SMALL_TYPE")) : 14;
    const int op = getenv("SMALL_OP") ? atoi(getenv("SMALL_OP")) : 3;
    /* SMALL_COLL: allreduce (default), allgather (bytes per rank), bcast (from rank 0) or
     * reduce_scatter_block (bytes per rank's block; the input is n blocks) */
    const char *coll = getenv("SMALL_COLL") ? getenv("SMALL_COLL") : "allreduce";
    const int kind = strcmp(coll, "allgather") == 0 ? 1 : strcmp(coll, "bcast") == 0 ? 2
                   : strcmp(coll, "reduce_scatter_block") == 0 ? 3 : strncmp(coll, "p2p_", 4) == 0 ? 4 : 0;
    if (kind == 4) {  /* point-to-point ping-pong: ranks 0 and 1 (the others only take part in barriers) */
        const int host = strcmp(coll, "p2p_host") == 0;
        char *hb = host ? malloc(maxb) : NULL;
        void *buf = host ? (void *)hb : s;
        if (host) memset(hb, rank, maxb);
        for (int k = 0; k < nsizes; ++k) {
            double us = 0;
            for (int phase = 0; phase < 2; ++phase) {
                const int it = phase ? reps : 50;
                mi355x_comm_barrier(c);
                const double t0 = now_us();
                for (int i = 0; i < it && rank < 2; ++i) {
                    int e = 0;
                    if (rank == 0) {
                        e = mi355x_send(c, buf, sizes[k], NULL, 1, 5, NULL) || mi355x_recv(c, buf, sizes[k], NULL, 1, 6, NULL, NULL);
                    } else {
                        e = mi355x_recv(c, buf, sizes[k], NULL, 0, 5, NULL, NULL) || mi355x_send(c, buf, sizes[k], NULL, 0, 6, NULL);
                    }
                    if (e) {
                        fprintf(stderr, "rank %d: %s\n", rank, mi355x_last_error());
                        return 1;
                    }
                }
                us = (now_us() - t0) / it / 2;
            }
            if (rank == 0)
                printf("{\"coll\": \"%s\", \"bytes\": %zu, \"one_way_us\": %.2f, \"n\": %d, \"caller\": \"C\"}\n", coll,
                       sizes[k], us, n);
        }
        free(hb);
        fflush(stdout);
        break;
    }
    for (int k = 0; k < nsizes; ++k) {
        const size_t cnt = sizes[k] / 4;
#define ONE_CALL() (kind == 1 ? mi355x_allgather(c, s, r, sizes[k], NULL) \
                   : kind == 2 ? mi355x_bcast(c, s, sizes[k], 0, NULL) \
                   : kind == 3 ? mi355x_reduce_scatter_block(c, r, s, cnt, ty, op, NULL) : mi355x_allreduce(c, s, r, cnt, ty, op, NULL))
        for (int i = 0; i < 50; ++i) ONE_CALL();
        mi355x_comm_barrier(c);
        const double t0 = now_us();
        for (int i = 0; i < reps; ++i)
            if (ONE_CALL()) {
                fprintf(stderr, "rank %d: %s\n", rank, mi355x_last_error());
                return 1;
            }
        const double us = (now_us() - t0) / reps;
        if (rank == 0)
            printf("{\"coll\": \"%s\", \"path\": \"%s\", \"bytes\": %zu, \"us_per_call\": %.2f, \"alg\": %d, "
                   "\"n\": %d, \"caller\": \"C\"}\n", coll, path, sizes[k], us, mi355x_comm_last_algorithm(c), n);
    }
    }
    mi355x_comm_barrier(c);
    double t0 = now_us();
    for (int i = 0; i < reps; ++i) mi355x_comm_barrier(c);
    if (rank == 0) printf("{\"barrier_us\": %.3f, \"n\": %d}\n", (now_us() - t0) / reps, n);
    fflush(stdout);
    mi355x_free(s);
    mi355x_free(r);
    mi355x_comm_destroy(c);
    return 0;
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2, reps = argc > 2 ? atoi(argv[2]) : 2000;
    const char *paths = argc > 3 ? argv[3] : "host";
    char key[64];
    snprintf(key, sizeof(key), "lat_%d", (int)getpid());
    for (int r = 1; r < n; ++r)
        if (fork() == 0) _exit(run(r, n, reps, key, paths));
    int rc = run(0, n, reps, key, paths);
    for (int r = 1; r < n; ++r) {
        int st = 0;
        wait(&st);
        if (!WIFEXITED(st) || WEXITSTATUS(st)) rc = 1;
    }
    return rc;
}
