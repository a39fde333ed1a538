/*
 * cpu_ring.c -- the reference's CPU allreduce path (BASELINE configs[0]: coll/tuned segmented ring
 * over the sm BTL), restated as n ranks running concurrently on n host cores.
 *
 * TEST / BENCH INFRASTRUCTURE ONLY (see oracle.h): the timed CPU baseline next to the GPU
 * allreduce, and a second witness of the ring's element order (its results must equal
 * oracle_allreduce's simulation bit for bit).
 *
 * What is restated:
 *   schedule   ompi_coll_tuned_allreduce_intra_ring_segmented (coll_tuned_allreduce.c:635-873):
 *              sbuf -> rbuf copy (:429 / :707), num_phases reduce-scatter passes over sub-blocks
 *              (:721-831; rank r first sends its own piece, step j reduces piece r-j as
 *              rbuf = rbuf (op) inbuf), then the ring allgather of whole blocks (:834-860).
 *              Falls back to the plain ring (:360-554) when count < n*segcount.
 *   transport  the sm BTL path ob1 takes for these messages (btl_sm.c:756-1000,
 *              btl_sm_component.c:243-253): the sender copies the message into shared-memory
 *              fragments of at most 32 KiB (btl_sm_max_send_size) queued on a per-peer FIFO,
 *              the receiver copies each fragment out into its receive buffer -- two memcpy per
 *              byte, both sides progressing their send and receive concurrently (isend+irecv).
 *   op         oracle_op_2buff (the restated op/base loop).
 * Ranks are threads pinned to distinct cores (the copies and loops cost the same as in separate
 * processes; the reference's processes share nothing else on this path).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define FRAG (32u * 1024u)
#define NSLOT 16

struct slot {
    _Atomic int full;
    uint32_t bytes;
    char data[FRAG];
};

struct fifo { /* rank r -> rank r+1 */
    struct slot s[NSLOT];
};

struct job {
    int n, type, op;
    size_t count;
    uint32_t segsize;
    const void *const *sbufs;
    void *const *rbufs;
    struct fifo *fifos;
    pthread_barrier_t *bar;
    int reps, core0;
    double *elapsed; /* per rank, seconds of the timed reps */
};

struct rank_arg {
    struct job *j;
    int rank;
};

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* send `sb` bytes to the right neighbour and receive `rb` bytes from the left one, concurrently */
static void sendrecv(struct job *j, int r, const char *sp, size_t sb, char *rp, size_t rb)
{
    struct fifo *out = &j->fifos[r], *in = &j->fifos[(r + j->n - 1) % j->n];
    size_t sent = 0, got = 0;
    unsigned tail = 0, head = 0;
    static _Thread_local unsigned out_tail = 0, in_head = 0;
    tail = out_tail;
    head = in_head;
    while (sent < sb || got < rb) {
        int progress = 0;
        if (sent < sb) {
            struct slot *s = &out->s[tail % NSLOT];
            if (!atomic_load_explicit(&s->full, memory_order_acquire)) {
                uint32_t k = (uint32_t)((sb - sent) < FRAG ? (sb - sent) : FRAG);
                memcpy(s->data, sp + sent, k);
                s->bytes = k;
                atomic_store_explicit(&s->full, 1, memory_order_release);
                sent += k;
                tail++;
                progress = 1;
            }
        }
        if (got < rb) {
            struct slot *s = &in->s[head % NSLOT];
            if (atomic_load_explicit(&s->full, memory_order_acquire)) {
                memcpy(rp + got, s->data, s->bytes);
                got += s->bytes;
                atomic_store_explicit(&s->full, 0, memory_order_release);
                head++;
                progress = 1;
            }
        }
        if (!progress) sched_yield();
    }
    out_tail = tail;
    in_head = head;
}

static void blockcount(size_t count, size_t nblocks, size_t *split, size_t *early, size_t *late)
{
    *early = *late = count / nblocks;
    *split = count % nblocks;
    if (*split) *early += 1;
}
static size_t boff(size_t b, size_t split, size_t early, size_t late) { return b < split ? b * early : b * late + split; }
static size_t blen(size_t b, size_t split, size_t early, size_t late) { return b < split ? early : late; }

static size_t segcount_of(uint32_t segsize, size_t esz, size_t count)
{
    if (segsize >= esz && segsize < esz * count) {
        size_t sc = segsize / esz, residual = segsize - sc * esz;
        if (residual > (esz >> 1)) sc++;
        return sc;
    }
    return count;
}

static void one_allreduce(struct job *j, int r, char *inbuf)
{
    const int n = j->n;
    const size_t esz = oracle_type_size(j->type), count = j->count;
    char *rbuf = (char *)j->rbufs[r];
    if (j->sbufs[r]) memcpy(rbuf, j->sbufs[r], count * esz);
    size_t split, early, late;
    blockcount(count, (size_t)n, &split, &early, &late);
    size_t sc = segcount_of(j->segsize, esz, count), phases = 1;
    if (count >= (size_t)n * sc && j->segsize) {
        size_t ns = (size_t)n * sc;
        phases = count / ns;
        if ((count % ns >= (size_t)n) && (count % ns > ns / 2)) phases++;
    }
    for (size_t ph = 0; ph < phases; ++ph) {
        size_t po[64], pl[64];
        for (int b = 0; b < n; ++b) {
            size_t bl = blen((size_t)b, split, early, late), ps, pe, pla;
            blockcount(bl, phases, &ps, &pe, &pla);
            po[b] = boff((size_t)b, split, early, late) + boff(ph, ps, pe, pla);
            pl[b] = blen(ph, ps, pe, pla);
        }
        int sb = r;
        for (int k = 1; k < n; ++k) {
            int b = (r - k + n) % n;
            sendrecv(j, r, rbuf + po[sb] * esz, pl[sb] * esz, inbuf, pl[b] * esz);
            oracle_op_2buff(j->op, j->type, inbuf, rbuf + po[b] * esz, pl[b]);
            sb = b;
        }
    }
    /* rank r owns block r+1; round k sends block r+1-k and receives block r-k */
    for (int k = 0; k < n - 1; ++k) {
        size_t sbk = (size_t)((r + 1 - k + 2 * n) % n), rbk = (size_t)((r - k + 2 * n) % n);
        sendrecv(j, r, rbuf + boff(sbk, split, early, late) * esz, blen(sbk, split, early, late) * esz,
                 rbuf + boff(rbk, split, early, late) * esz, blen(rbk, split, early, late) * esz);
    }
}

static void *rank_main(void *p)
{
    struct rank_arg *a = (struct rank_arg *)p;
    struct job *j = a->j;
    const int r = a->rank;
    if (j->core0 >= 0) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(j->core0 + r, &cs);
        pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
    }
    const size_t esz = oracle_type_size(j->type);
    char *inbuf = malloc((j->count / (size_t)j->n + 1) * esz);
    pthread_barrier_wait(j->bar);
    one_allreduce(j, r, inbuf); /* warm-up (page faults, caches) */
    pthread_barrier_wait(j->bar);
    double t0 = now();
    for (int i = 0; i < j->reps; ++i) one_allreduce(j, r, inbuf);
    double t1 = now();
    j->elapsed[r] = t1 - t0;
    pthread_barrier_wait(j->bar);
    free(inbuf);
    return NULL;
}

/* Run 1 + reps allreduces of `count` elements over n concurrent ranks; *sec_per_call = the
 * slowest rank's time per timed call.  sbufs[r] == NULL means MPI_IN_PLACE. core0 < 0: no
 * pinning, else rank r runs on core core0 + r.  Returns 0, or < 0 on bad arguments. */
int oracle_cpu_allreduce(int n, size_t count, int type, int op, uint32_t segsize, const void *const *sbufs,
                         void *const *rbufs, int reps, int core0, double *sec_per_call)
{
    if (n < 2 || n > 64 || !oracle_has_op(op, type) || count < (size_t)n) return -1;
    struct job j;
    j.n = n;
    j.type = type;
    j.op = op;
    j.count = count;
    j.segsize = segsize;
    j.sbufs = sbufs;
    j.rbufs = rbufs;
    j.reps = reps;
    j.core0 = core0;
    j.fifos = calloc((size_t)n, sizeof(struct fifo));
    double el[64] = {0};
    j.elapsed = el;
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)n);
    j.bar = &bar;
    pthread_t th[64];
    struct rank_arg args[64];
    for (int r = 0; r < n; ++r) {
        args[r].j = &j;
        args[r].rank = r;
        pthread_create(&th[r], NULL, rank_main, &args[r]);
    }
    for (int r = 0; r < n; ++r) pthread_join(th[r], NULL);
    pthread_barrier_destroy(&bar);
    free(j.fifos);
    double mx = 0;
    for (int r = 0; r < n; ++r)
        if (el[r] > mx) mx = el[r];
    if (sec_per_call) *sec_per_call = reps > 0 ? mx / reps : 0.0;
    return 0;
}
