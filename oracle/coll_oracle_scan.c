/* coll_oracle_scan.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * MPI_Scan / MPI_Exscan as coll/basic runs them: a linear chain over the ranks.
 *   scan   (ompi/mca/coll/basic/coll_basic_scan.c:40-120): rank 0 copies sbuf to rbuf; rank r > 0
 *          copies sbuf to rbuf, receives the prior answer from r-1 into a temporary and calls
 *          ompi_op_reduce(op, temp, rbuf) -- rbuf = temp (op) rbuf -- then sends rbuf to r+1.
 *   exscan (coll_basic_exscan.c:40-110): rank 0 sends sbuf to 1; the last rank receives into
 *          rbuf; a middle rank r copies sbuf to a temporary, receives the prior answer into rbuf,
 *          calls ompi_op_reduce(op, rbuf, temp) and sends temp on.  Rank 0's rbuf is untouched.
 * The chain is simulated rank by rank with the restated op loops (op_oracle.c).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

int oracle_scan(int exclusive, int n, size_t count, int type, int op, const void *const *sbufs,
                void *const *rbufs)
{
    const size_t bytes = count * oracle_type_size(type);
    if (n < 1) return -1;
    if (!exclusive) {
        memcpy(rbufs[0], sbufs[0], bytes);
        for (int r = 1; r < n; ++r) {
            memcpy(rbufs[r], sbufs[r], bytes);
            /* the prior answer (rank r-1's rbuf, sent) is `in`, rbuf is `inout` */
            if (oracle_op_2buff(op, type, rbufs[r - 1], rbufs[r], count)) return -1;
        }
        return 0;
    }
    if (n == 1) return 0;
    void *carry = malloc(bytes + 1);   /* what rank r-1 sends to rank r */
    if (!carry) return -1;
    memcpy(carry, sbufs[0], bytes);    /* rank 0 sends its sbuf */
    for (int r = 1; r < n; ++r) {
        memcpy(rbufs[r], carry, bytes); /* receive the prior answer into rbuf */
        if (r == n - 1) break;
        memcpy(carry, sbufs[r], bytes); /* reduce_buffer = sbuf */
        if (oracle_op_2buff(op, type, rbufs[r], carry, count)) {
            free(carry);
            return -1;
        }
    }
    free(carry);
    return 0;
}
