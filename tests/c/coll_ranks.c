/*
 * coll_ranks.c -- the C ABI (include/mi355x_rt.h) driven from plain C, the way an MPI library's C
 * code would: N processes (forked before any HIP call, one communicator rank each, all on device
 * 0), every collective of the engine plus device point-to-point, each checked exactly on integer-
 * valued data (so every reduction order gives the same bits).
 *
 * usage: coll_ranks <nranks>     exit 0 and "rank r C-ABI OK" per rank on success
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "../../include/mi355x_rt.h"

#define CHECK(call)                                                                       \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != MI355X_SUCCESS) {                                                      \
            fprintf(stderr, "rank %d: %s failed (%d): %s\n", rank, #call, rc_, mi355x_last_error()); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)
#define EXPECT(cond, what)                                                                \
    do {                                                                                  \
        if (!(cond)) {                                                                    \
            fprintf(stderr, "rank %d: %s\n", rank, what);                                 \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

static int run(int rank, int n, const char *key)
{
    mi355x_comm_t *c = NULL;
    CHECK(mi355x_set_device(0));
    CHECK(mi355x_comm_create(key, rank, n, 0, &c));
    const size_t count = 1 << 20;   /* 4 MiB of MPI_FLOAT per rank */
    float *h = malloc(count * n * sizeof(float));
    float *d_s = NULL, *d_r = NULL;
    CHECK(mi355x_malloc((void **)&d_s, count * n * sizeof(float)));
    CHECK(mi355x_malloc((void **)&d_r, count * n * sizeof(float)));

    /* MPI_Allreduce(MPI_SUM, MPI_FLOAT): x_r[i] = r + (i % 7) -> n(n-1)/2 + n (i % 7) */
    for (size_t i = 0; i < count; ++i) h[i] = (float)(rank + (int)(i % 7));
    CHECK(mi355x_memcpy(d_s, h, count * sizeof(float)));
    CHECK(mi355x_allreduce(c, d_s, d_r, count, MI355X_T_FLOAT, MI355X_OP_SUM, NULL));
    CHECK(mi355x_memcpy(h, d_r, count * sizeof(float)));
    for (size_t i = 0; i < count; i += 4099)
        EXPECT(h[i] == (float)(n * (n - 1) / 2 + n * (int)(i % 7)), "allreduce value");

    /* MPI_Reduce_scatter_block: block r of sum over ranks of (q + j) */
    for (size_t i = 0; i < count * n; ++i) h[i] = (float)(rank + (int)(i % 5));
    CHECK(mi355x_memcpy(d_s, h, count * n * sizeof(float)));
    CHECK(mi355x_reduce_scatter_block(c, d_s, d_r, count, MI355X_T_FLOAT, MI355X_OP_SUM, NULL));
    CHECK(mi355x_memcpy(h, d_r, count * sizeof(float)));
    for (size_t i = 0; i < count; i += 4099) {
        const size_t g = (size_t)rank * count + i;
        EXPECT(h[i] == (float)(n * (n - 1) / 2 + n * (int)(g % 5)), "reduce_scatter_block value");
    }

    /* MPI_Bcast from the last rank, MPI_Allgather */
    for (size_t i = 0; i < count; ++i) h[i] = (float)(rank * 1000 + (int)(i % 11));
    CHECK(mi355x_memcpy(d_r, h, count * sizeof(float)));
    CHECK(mi355x_bcast(c, d_r, count * sizeof(float), n - 1, NULL));
    CHECK(mi355x_memcpy(h, d_r, count * sizeof(float)));
    for (size_t i = 0; i < count; i += 4099) EXPECT(h[i] == (float)((n - 1) * 1000 + (int)(i % 11)), "bcast value");
    for (size_t i = 0; i < count; ++i) h[i] = (float)(rank + 1);
    CHECK(mi355x_memcpy(d_s, h, count * sizeof(float)));
    CHECK(mi355x_allgather(c, d_s, d_r, count * sizeof(float), NULL));
    CHECK(mi355x_memcpy(h, d_r, count * n * sizeof(float)));
    for (int q = 0; q < n; ++q) EXPECT(h[(size_t)q * count + 17] == (float)(q + 1), "allgather value");

    /* MPI_Scan(MPI_SUM, MPI_INT) */
    int32_t *hi = (int32_t *)h;
    for (size_t i = 0; i < 1000; ++i) hi[i] = rank + 1;
    CHECK(mi355x_memcpy(d_s, hi, 1000 * sizeof(int32_t)));
    CHECK(mi355x_scan(c, d_s, d_r, 1000, MI355X_T_INT32, MI355X_OP_SUM, NULL));
    CHECK(mi355x_memcpy(hi, d_r, 1000 * sizeof(int32_t)));
    EXPECT(hi[999] == (rank + 1) * (rank + 2) / 2, "scan value");

    /* MPI_Sendrecv ring on device buffers, then MPI_Irecv(MPI_ANY_SOURCE) from everyone */
    for (size_t i = 0; i < 4096; ++i) hi[i] = rank * 100000 + (int)i;
    CHECK(mi355x_memcpy(d_s, hi, 4096 * sizeof(int32_t)));
    mi355x_status_t st;
    CHECK(mi355x_sendrecv(c, d_s, 4096 * sizeof(int32_t), NULL, (rank + 1) % n, 5, d_r, 4096 * sizeof(int32_t), NULL,
                          (rank + n - 1) % n, 5, NULL, &st));
    EXPECT(st.source == (rank + n - 1) % n && st.tag == 5 && st.bytes == 4096 * sizeof(int32_t), "sendrecv status");
    CHECK(mi355x_memcpy(hi, d_r, 4096 * sizeof(int32_t)));
    EXPECT(hi[4095] == ((rank + n - 1) % n) * 100000 + 4095, "sendrecv value");
    mi355x_request_t *rq[64];
    int nr = 0;
    for (int q = 0; q < n; ++q)
        if (q != rank)
            CHECK(mi355x_irecv(c, (char *)d_r + (size_t)q * 64, 64, NULL, MI355X_ANY_SOURCE, 9, NULL, &rq[nr++]));
    for (int q = 0; q < n; ++q)
        if (q != rank) CHECK(mi355x_isend(c, d_s, 64, NULL, q, 9, NULL, &rq[nr++]));
    int seen = 0;
    for (int k = 0; k < nr; ++k) {
        CHECK(mi355x_request_wait(rq[k]));
        CHECK(mi355x_request_get_status(rq[k], &st));
        if (k < n - 1) seen |= 1 << st.source;
        CHECK(mi355x_request_free(rq[k]));
    }
    EXPECT(seen == (((1 << n) - 1) & ~(1 << rank)), "any-source senders");

    CHECK(mi355x_comm_barrier(c));
    CHECK(mi355x_free(d_s));
    CHECK(mi355x_free(d_r));
    free(h);
    CHECK(mi355x_comm_destroy(c));
    printf("rank %d C-ABI OK\n", rank);
    fflush(stdout);
    return 0;
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2;
    if (n < 2 || n > 8) return 2;
    char key[64];
    snprintf(key, sizeof(key), "cabi_%d", (int)getpid());
    /* fork before any HIP call: every rank initialises its own runtime */
    pid_t pids[8];
    for (int r = 0; r < n; ++r) {
        pids[r] = fork();
        if (pids[r] == 0) _exit(run(r, n, key));
    }
    int bad = 0;
    for (int r = 0; r < n; ++r) {
        int s = 0;
        waitpid(pids[r], &s, 0);
        if (!WIFEXITED(s) || WEXITSTATUS(s) != 0) {
            fprintf(stderr, "rank %d exited with status %d\n", r, s);
            bad = 1;
        }
    }
    return bad;
}
