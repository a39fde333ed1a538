/*
 * ddt_oracle.c -- datatype pack/unpack and convertor checksum of Open MPI 1.8.5, restated.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The packed stream of `count` instances of a derived datatype is its type map in order
 * (MPI-3.1 §4.1.11; opal_generic_simple_pack walks the description in that order,
 * opal/datatype/opal_datatype_pack.c:250-374): instance k at base + k*extent, inside it `nblk`
 * blocks at j*stride, inside a block the runs (disp, len) in order.  Constructors restated:
 *   MPI_Type_vector   ompi/datatype/ompi_datatype_create_vector.c:36-65
 *   MPI_Type_indexed  ompi/datatype/ompi_datatype_create_indexed.c:32-66 (merges adjacent blocks)
 *   contiguous / struct-of-predefined (e.g. MPI_LONG_DOUBLE_INT) as run lists.
 * A run is made of basic elements of `elem` bytes; opal_convertor_set_position only stops on
 * element boundaries, which oracle_ddt_round_position restates for the segment tests of
 * test/datatype/position.c / position_noncontig.c.
 * Checksum: opal_uicsum_partial (opal/util/crc.c:921-1060) restated byte for byte, accumulated
 * per copied run as MEMCPY_CSUM does (opal/datatype/opal_datatype_checksum.h:40-46).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define MAXRUNS 4096

struct oracle_ddt {
    int nruns;
    int64_t disp[MAXRUNS];
    int64_t len[MAXRUNS];
    int64_t elem[MAXRUNS];
    int64_t nblk, stride, extent;
    int64_t blk_bytes;
};

static oracle_ddt_t *ddt_new(void)
{
    oracle_ddt_t *d = calloc(1, sizeof(*d));
    d->nblk = 1;
    return d;
}

static void add_run(oracle_ddt_t *d, int64_t disp, int64_t len, int64_t elem)
{
    if (len <= 0) return;
    /* merge with the previous run when contiguous and of the same element size */
    if (d->nruns > 0 && d->disp[d->nruns - 1] + d->len[d->nruns - 1] == disp && d->elem[d->nruns - 1] == elem) {
        d->len[d->nruns - 1] += len;
    } else {
        d->disp[d->nruns] = disp;
        d->len[d->nruns] = len;
        d->elem[d->nruns] = elem;
        d->nruns++;
    }
    d->blk_bytes += len;
}

oracle_ddt_t *oracle_ddt_contiguous(int64_t count, int64_t elem)
{
    oracle_ddt_t *d = ddt_new();
    add_run(d, 0, count * elem, elem);
    d->extent = count * elem;
    return d;
}

oracle_ddt_t *oracle_ddt_vector(int64_t count, int64_t blocklen, int64_t stride, int64_t elem)
{
    oracle_ddt_t *d = ddt_new();
    if (count <= 0) return d;
    if (blocklen == stride || count <= 1) {
        add_run(d, 0, count * blocklen * elem, elem);
    } else {
        add_run(d, 0, blocklen * elem, elem);
        d->nblk = count;
        d->stride = stride * elem;
    }
    d->extent = ((count - 1) * stride + blocklen) * elem;
    return d;
}

oracle_ddt_t *oracle_ddt_indexed(int count, const int *blocklens, const int *disps, int64_t elem)
{
    oracle_ddt_t *d = ddt_new();
    int64_t lo = 0, hi = 0;
    int first = 1;
    for (int i = 0; i < count; ++i) {
        add_run(d, (int64_t)disps[i] * elem, (int64_t)blocklens[i] * elem, elem);
        if (blocklens[i] > 0) {
            int64_t a = (int64_t)disps[i] * elem, b = a + (int64_t)blocklens[i] * elem;
            if (first || a < lo) lo = a;
            if (first || b > hi) hi = b;
            first = 0;
        }
    }
    d->extent = hi - lo;
    return d;
}

/* struct of predefined members: runs (disp, len, elem) and an explicit extent */
oracle_ddt_t *oracle_ddt_struct(int n, const int64_t *disp, const int64_t *len, const int64_t *elem, int64_t extent)
{
    oracle_ddt_t *d = ddt_new();
    for (int i = 0; i < n; ++i) add_run(d, disp[i], len[i], elem[i]);
    d->extent = extent;
    return d;
}

void oracle_ddt_free(oracle_ddt_t *d) { free(d); }
int64_t oracle_ddt_size(const oracle_ddt_t *d) { return d->nblk * d->blk_bytes; }
int64_t oracle_ddt_extent(const oracle_ddt_t *d) { return d->extent; }

/* byte offset in memory of packed byte p, and the element size / offset within its element */
static int64_t map_byte(const oracle_ddt_t *d, int64_t p, int64_t *elem_off)
{
    const int64_t inst = d->nblk * d->blk_bytes;
    const int64_t k = p / inst, rem = p % inst;
    const int64_t j = rem / d->blk_bytes;
    int64_t q = rem % d->blk_bytes;
    int r = 0;
    while (q >= d->len[r]) { q -= d->len[r]; ++r; }
    if (elem_off) *elem_off = q % d->elem[r];
    return k * d->extent + j * d->stride + d->disp[r] + q;
}

/* the largest position <= pos that is a basic-element boundary of the stream */
int64_t oracle_ddt_round_position(const oracle_ddt_t *d, int64_t count, int64_t pos)
{
    const int64_t total = count * oracle_ddt_size(d);
    if (pos >= total) return total;
    int64_t eo = 0;
    map_byte(d, pos, &eo);
    return pos - eo;
}

/* pack packed bytes [pos, pos+bytes) of `count` instances at base into dst */
int oracle_ddt_pack(const oracle_ddt_t *d, int64_t count, const void *base, int64_t pos, void *dst, int64_t bytes)
{
    const int64_t total = count * oracle_ddt_size(d);
    if (pos < 0 || pos + bytes > total) return MI355X_ERR_ARG;
    const char *b = (const char *)base;
    char *o = (char *)dst;
    for (int64_t i = 0; i < bytes; ++i) o[i] = b[map_byte(d, pos + i, NULL)];
    return MI355X_SUCCESS;
}

int oracle_ddt_unpack(const oracle_ddt_t *d, int64_t count, void *base, int64_t pos, const void *src, int64_t bytes)
{
    const int64_t total = count * oracle_ddt_size(d);
    if (pos < 0 || pos + bytes > total) return MI355X_ERR_ARG;
    char *b = (char *)base;
    const char *s = (const char *)src;
    for (int64_t i = 0; i < bytes; ++i) b[map_byte(d, pos + i, NULL)] = s[i];
    return MI355X_SUCCESS;
}

/* ---- opal_uicsum_partial (opal/util/crc.c:921-1060): sum of the stream's native 32-bit words,
 *      carried across calls through (lastPartialInt, lastPartialLength). */
#define INTALIGNED(x) ((((uintptr_t)(x)) & (sizeof(unsigned int) - 1)) == 0)
unsigned long oracle_uicsum_partial(const void *source, size_t csumlen, unsigned int *lastPartialInt,
                                    size_t *lastPartialLength)
{
    const unsigned int *src = (const unsigned int *)source;
    unsigned int csum = 0, temp = *lastPartialInt;
    unsigned long i;
    const size_t W = sizeof(unsigned int);
    if (*lastPartialLength) {
        if (csumlen >= W - *lastPartialLength) {
            memcpy((char *)&temp + *lastPartialLength, src, W - *lastPartialLength);
            src = (const unsigned int *)((const char *)src + W - *lastPartialLength);
            csum += temp - *lastPartialInt;
            csumlen -= W - *lastPartialLength;
            for (i = 0; i < csumlen / W; i++) {
                memcpy(&temp, src, W);
                csum += temp;
                src++;
            }
            csumlen -= i * W;
            *lastPartialInt = 0;
            *lastPartialLength = 0;
        } else {
            memcpy((char *)&temp + *lastPartialLength, src, csumlen);
            src = (const unsigned int *)((const char *)src + csumlen);
            csum += temp - *lastPartialInt;
            *lastPartialInt = temp;
            *lastPartialLength += csumlen;
            csumlen = 0;
        }
    } else {
        for (; csumlen >= W; csumlen -= W) {
            memcpy(&temp, src, W);
            src++;
            csum += temp;
        }
        *lastPartialLength = 0;
        *lastPartialInt = 0;
    }
    if (csumlen != 0) {
        temp = *lastPartialInt;
        if (*lastPartialLength) {
            if (csumlen >= W - *lastPartialLength) {
                memcpy((char *)&temp + *lastPartialLength, src, W - *lastPartialLength);
                csum += temp - *lastPartialInt;
                csumlen -= W - *lastPartialLength;
                src = (const unsigned int *)((const char *)src + W - *lastPartialLength);
                *lastPartialLength = csumlen;
                temp = 0;
                if (csumlen) memcpy(&temp, src, csumlen);
                csum += temp;
                *lastPartialInt = temp;
            } else {
                memcpy((char *)&temp + *lastPartialLength, src, csumlen);
                csum += temp - *lastPartialInt;
                *lastPartialInt = temp;
                *lastPartialLength += csumlen;
            }
        } else {
            memcpy(&temp, src, csumlen);
            csum += temp;
            *lastPartialInt = temp;
            *lastPartialLength = csumlen;
        }
    }
    return csum;
}

/* convertor-style packing with checksum: the stream is produced run by run (one MEMCPY_CSUM per
 * contiguous piece, as pack_predefined_data / pack_contiguous_loop do) and every piece is added
 * to the running checksum.  Returns the 32-bit convertor checksum. */
uint32_t oracle_ddt_pack_checksum(const oracle_ddt_t *d, int64_t count, const void *base, void *dst)
{
    unsigned int ui1 = 0;
    size_t ui2 = 0;
    uint32_t sum = 0;
    char *o = (char *)dst;
    const char *b = (const char *)base;
    for (int64_t k = 0; k < count; ++k)
        for (int64_t j = 0; j < d->nblk; ++j)
            for (int r = 0; r < d->nruns; ++r) {
                const char *s = b + k * d->extent + j * d->stride + d->disp[r];
                memcpy(o, s, (size_t)d->len[r]);
                sum += (uint32_t)oracle_uicsum_partial(o, (size_t)d->len[r], &ui1, &ui2);
                o += d->len[r];
            }
    return sum;
}

/* whole-message pack as the reference's homogeneous engine does it for a GPU-less host: one
 * memcpy per contiguous run (opal_generic_simple_pack -> pack_predefined_data / MEMCPY,
 * opal/datatype/opal_datatype_pack.h:24-76).  Used as the timed CPU baseline. */
void oracle_ddt_pack_runs(const oracle_ddt_t *d, int64_t count, const void *base, void *dst)
{
    char *o = (char *)dst;
    const char *b = (const char *)base;
    for (int64_t k = 0; k < count; ++k)
        for (int64_t j = 0; j < d->nblk; ++j)
            for (int r = 0; r < d->nruns; ++r) {
                memcpy(o, b + k * d->extent + j * d->stride + d->disp[r], (size_t)d->len[r]);
                o += d->len[r];
            }
}
