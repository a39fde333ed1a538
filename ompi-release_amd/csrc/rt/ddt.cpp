// ddt.cpp -- datatype layouts for the GPU convertor (host side).
//
// Builders restate the MPI constructors' type maps (ompi_datatype_create_vector.c:36-65,
// ompi_datatype_create_indexed.c:32-66 incl. the merge of adjacent blocks) and, for drop-in use
// inside Open MPI, compile an optimized opal description (opt_desc: ELEM / LOOP / END_LOOP
// records, opal/datatype/opal_datatype_internal.h:148-188) into the same layout.
#include <algorithm>
#include <cstring>
#include <vector>

#include "ddt_internal.hpp"
#include "rt_internal.hpp"

#include <mutex>

struct mi355x_ddt {
    std::vector<int64_t> disp, len, elem, pfx;
    int64_t nblk = 1, stride = 0, extent = 0;
    uint64_t run_bits = 0;  // OR of every run's displacement and length (their common alignment)
    int64_t max_len = 0;    // longest run
    int64_t *ddisp = nullptr, *dlen = nullptr, *dpfx = nullptr;  // device copies, made on first use
    int dev = -1;
    std::mutex mtx;
};

namespace mi355x {

static void add_run(mi355x_ddt *d, int64_t disp, int64_t len, int64_t elem)
{
    if (len <= 0) return;
    if (!d->disp.empty() && d->disp.back() + d->len.back() == disp && d->elem.back() == elem) {
        d->len.back() += len;
        return;
    }
    d->disp.push_back(disp);
    d->len.push_back(len);
    d->elem.push_back(elem);
}

static int finalize(mi355x_ddt *d, mi355x_ddt_t **out)
{
    if (d->disp.empty()) {  // empty datatype: one zero-length run keeps the tables non-empty
        d->disp.push_back(0);
        d->len.push_back(0);
        d->elem.push_back(1);
    }
    const size_t n = d->disp.size();
    d->pfx.assign(n, 0);
    for (size_t r = 1; r < n; ++r) d->pfx[r] = d->pfx[r - 1] + d->len[r - 1];
    d->run_bits = 0;
    d->max_len = 0;
    for (size_t r = 0; r < n; ++r) {
        d->run_bits |= (uint64_t)d->disp[r] | (uint64_t)d->len[r];
        d->max_len = std::max<int64_t>(d->max_len, d->len[r]);
    }
    *out = d;
    return MI355X_SUCCESS;
}

// device copies of the run tables (uploaded once per datatype)
static int upload(mi355x_ddt *d)
{
    std::lock_guard<std::mutex> g(d->mtx);
    if (d->ddisp) return MI355X_SUCCESS;
    const size_t n = d->disp.size() * 8;
    MI_HIP(hipMalloc(&d->ddisp, n));
    MI_HIP(hipMalloc(&d->dlen, n));
    MI_HIP(hipMalloc(&d->dpfx, n));
    MI_HIP(hipMemcpy(d->ddisp, d->disp.data(), n, hipMemcpyHostToDevice));
    MI_HIP(hipMemcpy(d->dlen, d->len.data(), n, hipMemcpyHostToDevice));
    MI_HIP(hipMemcpy(d->dpfx, d->pfx.data(), n, hipMemcpyHostToDevice));
    return MI355X_SUCCESS;
}

static int64_t blk_bytes(const mi355x_ddt *d)
{
    int64_t b = 0;
    for (int64_t l : d->len) b += l;
    return b;
}

// opal description records (opal_datatype_internal.h:148-188), x86-64 layout: 32 bytes each
struct OElem { uint16_t flags, type; uint32_t count, blocklen; int64_t extent, disp; };
struct OLoop { uint16_t flags, type; uint32_t loops, items; uint64_t unused; int64_t extent; };
struct OEnd { uint16_t flags, type; uint32_t items, unused; uint64_t size; int64_t first_elem_disp; };
static_assert(sizeof(OElem) == 32 && sizeof(OLoop) == 32 && sizeof(OEnd) == 32, "opal dt_elem_desc is 32 B");
constexpr uint16_t kOpalLoop = 0, kOpalEndLoop = 1, kOpalLB = 2, kOpalUB = 3;  // :107-110

// expand records [i, end) at displacement `base` into runs (recursing into loops)
static int expand(mi355x_ddt *d, const unsigned char *desc, uint32_t i, uint32_t end, int64_t base,
                  const uint32_t *basic, size_t budget)
{
    while (i < end) {
        const uint16_t type = ((const OElem *)(desc + 32 * (size_t)i))->type;
        if (type == kOpalLoop) {
            const OLoop *l = (const OLoop *)(desc + 32 * (size_t)i);
            const uint32_t body_end = i + l->items;  // index of the END_LOOP record
            for (uint32_t k = 0; k < l->loops; ++k) {
                int rc = expand(d, desc, i + 1, body_end, base + (int64_t)k * l->extent, basic, budget);
                if (rc) return rc;
                if (d->disp.size() > budget) return set_error(MI355X_ERR_UNSUPPORTED, "datatype too irregular");
            }
            i = body_end + 1;
        } else if (type == kOpalEndLoop || type == kOpalLB || type == kOpalUB) {
            ++i;
        } else {
            const OElem *e = (const OElem *)(desc + 32 * (size_t)i);
            const int64_t sz = basic[type];
            if (sz <= 0) return set_error(MI355X_ERR_ARG, "unknown basic type %u", type);
            if (e->extent == sz) {
                add_run(d, base + e->disp, (int64_t)e->count * sz, sz);
            } else {
                for (uint32_t c = 0; c < e->count; ++c) add_run(d, base + e->disp + (int64_t)c * e->extent, sz, sz);
            }
            if (d->disp.size() > budget) return set_error(MI355X_ERR_UNSUPPORTED, "datatype too irregular");
            ++i;
        }
    }
    return MI355X_SUCCESS;
}

} // namespace mi355x

using namespace mi355x;

extern "C" {

int mi355x_ddt_create(const int64_t *disp, const int64_t *len, size_t nruns, size_t nblk, int64_t stride,
                      int64_t extent, mi355x_ddt_t **out)
{
    if (!out || (nruns && (!disp || !len)) || nblk < 1) return set_error(MI355X_ERR_ARG, "bad ddt arguments");
    auto *d = new mi355x_ddt();
    for (size_t r = 0; r < nruns; ++r) add_run(d, disp[r], len[r], 1);
    d->nblk = (int64_t)nblk;
    d->stride = stride;
    d->extent = extent;
    return finalize(d, out);
}

// MPI_Type_vector(count, blocklen, stride, oldtype) with a gap-free oldtype of elem_size bytes
int mi355x_ddt_create_vector(size_t count, size_t blocklen, int64_t stride, size_t elem_size, mi355x_ddt_t **out)
{
    if (!out || elem_size == 0) return set_error(MI355X_ERR_ARG, "bad vector arguments");
    auto *d = new mi355x_ddt();
    const int64_t e = (int64_t)elem_size;
    if (count > 0) {
        if ((int64_t)blocklen == stride || count <= 1) {
            add_run(d, 0, (int64_t)(count * blocklen) * e, e);
        } else {
            add_run(d, 0, (int64_t)blocklen * e, e);
            d->nblk = (int64_t)count;
            d->stride = stride * e;
        }
        d->extent = ((int64_t)(count - 1) * stride + (int64_t)blocklen) * e;
    }
    return finalize(d, out);
}

// MPI_Type_indexed(count, blocklens, disps, oldtype): adjacent blocks merge, as
// ompi_datatype_create_indexed.c:48-63 does
int mi355x_ddt_create_indexed(size_t count, const int *blocklens, const int *disps, size_t elem_size,
                              mi355x_ddt_t **out)
{
    if (!out || elem_size == 0 || (count && (!blocklens || !disps))) return set_error(MI355X_ERR_ARG, "bad indexed arguments");
    auto *d = new mi355x_ddt();
    const int64_t e = (int64_t)elem_size;
    int64_t lo = 0, hi = 0;
    bool first = true;
    for (size_t i = 0; i < count; ++i) {
        add_run(d, (int64_t)disps[i] * e, (int64_t)blocklens[i] * e, e);
        if (blocklens[i] > 0) {
            const int64_t a = (int64_t)disps[i] * e, b = a + (int64_t)blocklens[i] * e;
            if (first || a < lo) lo = a;
            if (first || b > hi) hi = b;
            first = false;
        }
    }
    d->extent = hi - lo;
    return finalize(d, out);
}

// Compile an opal description (opt_desc.desc, opt_desc.used records) of a datatype whose extent
// is `extent` (ub - lb).  basic_sizes[type] = size of each opal basic type id.
int mi355x_ddt_from_opal(const void *desc, uint32_t used, int64_t extent, const uint32_t *basic_sizes,
                         mi355x_ddt_t **out)
{
    if (!desc || !basic_sizes || !out) return set_error(MI355X_ERR_ARG, "bad opal description arguments");
    auto *d = new mi355x_ddt();
    const unsigned char *p = (const unsigned char *)desc;
    // a top-level LOOP covering the whole description (the vector shape) keeps its loop as
    // the block layer instead of being unrolled into runs
    const OLoop *l0 = (const OLoop *)p;
    int rc;
    if (used >= 2 && l0->type == kOpalLoop && l0->items + 1 == used) {
        rc = expand(d, p, 1, l0->items, 0, basic_sizes, 1u << 20);
        d->nblk = l0->loops;
        d->stride = l0->extent;
    } else {
        rc = expand(d, p, 0, used, 0, basic_sizes, 1u << 20);
    }
    if (rc) {
        delete d;
        return rc;
    }
    d->extent = extent;
    return finalize(d, out);
}

int mi355x_ddt_destroy(mi355x_ddt_t *d)
{
    if (!d) return MI355X_SUCCESS;
    if (d->ddisp) {
        (void)hipFree(d->ddisp);
        (void)hipFree(d->dlen);
        (void)hipFree(d->dpfx);
    }
    delete d;
    return MI355X_SUCCESS;
}

size_t mi355x_ddt_size(const mi355x_ddt_t *d) { return d ? (size_t)(d->nblk * blk_bytes(d)) : 0; }
int64_t mi355x_ddt_extent(const mi355x_ddt_t *d) { return d ? d->extent : 0; }
int mi355x_ddt_nruns(const mi355x_ddt_t *d) { return d ? (int)d->disp.size() : 0; }

static int ddt_move(const mi355x_ddt_t *d, bool pack, size_t count, void *mem, size_t pos, void *packed,
                    size_t bytes, uint32_t *checksum, void *stream)
{
    if (!d || (bytes && (!mem || !packed))) return set_error(MI355X_ERR_ARG, "bad pack arguments");
    const int64_t inst = d->nblk * blk_bytes(d);
    if ((int64_t)(pos + bytes) > (int64_t)count * inst) return set_error(MI355X_ERR_ARG, "window past the message");
    if (checksum) *checksum = 0;
    if (bytes == 0 || inst == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    int rc0 = upload(const_cast<mi355x_ddt *>(d));
    if (rc0) return rc0;
    DdtDev dv;
    dv.disp = d->ddisp;
    dv.len = d->dlen;
    dv.pfx = d->dpfx;
    dv.pfx_host = d->pfx.data();
    dv.len_host = d->len.data();
    dv.nruns = (int)d->disp.size();
    dv.nblk = d->nblk;
    dv.stride = d->stride;
    dv.extent = d->extent;
    dv.blk_bytes = blk_bytes(d);
    dv.inst_bytes = inst;
    dv.run_bits = d->run_bits;
    dv.max_len = d->max_len;
    unsigned h = 0;
    unsigned *sum = checksum ? &h : nullptr;  // the launchers wait for the kernel when asked for one
    int rc = 1;
    if (d->disp.size() == 1)
        rc = launch_ddt_rows(dv, 1, d->disp[0], d->len[0], pack, mem, packed, (int64_t)pos, (int64_t)bytes, sum, s);
    if (rc == 1) rc = launch_ddt(dv, pack, mem, packed, (int64_t)pos, (int64_t)bytes, sum, s);
    if (rc) return rc;
    if (checksum) *checksum = h;
    return MI355X_SUCCESS;
}

} // extern "C"

namespace mi355x {
// true when `count` instances of d occupy one gap-free byte range starting at base + *first
bool ddt_contiguous(const mi355x_ddt *d, size_t count, int64_t *first)
{
    *first = 0;
    if (!d || d->disp.size() != 1) return false;
    const int64_t len = d->len[0];
    *first = d->disp[0];
    if (d->nblk > 1 && d->stride != len) return false;
    return count <= 1 || d->extent == d->nblk * len;
}
} // namespace mi355x

extern "C" {

int mi355x_ddt_tune(int unroll_pack, int unroll_unpack, int threads, int nontemporal)
{
    auto ok_u = [](int u) { return u == 0 || u == 2 || u == 4 || u == 8; };
    if (!ok_u(unroll_pack) || !ok_u(unroll_unpack)) return set_error(MI355X_ERR_ARG, "unroll must be 2, 4 or 8");
    if (threads != 0 && threads != 256 && threads != 512 && threads != 1024)
        return set_error(MI355X_ERR_ARG, "threads must be 256, 512 or 1024");
    if (nontemporal < -2 || nontemporal > 3) return set_error(MI355X_ERR_ARG, "nontemporal must be -2..3");
    DdtTune &t = ddt_tune();
    if (unroll_pack) t.unroll_pack = unroll_pack;
    if (unroll_unpack) t.unroll_unpack = unroll_unpack;
    if (threads) t.threads = threads;
    if (nontemporal != -2) t.nontemporal = nontemporal;
    return MI355X_SUCCESS;
}

int mi355x_ddt_tune_rows(int mode)
{
    if (mode < 0 || mode > 3) return set_error(MI355X_ERR_ARG, "row-kernel mode must be 0..3");
    ddt_tune().rows = mode;
    return MI355X_SUCCESS;
}

int mi355x_pack(const mi355x_ddt_t *d, size_t count, const void *base, size_t pos, void *dst, size_t bytes,
                uint32_t *checksum, void *stream)
{
    return ddt_move(d, true, count, const_cast<void *>(base), pos, dst, bytes, checksum, stream);
}

} // extern "C"

namespace mi355x {
// The type map as memory pieces in packed-stream order, from packed position `pos`: fn(offset of
// the piece from base, its length, its packed position) for pieces covering [pos, pos + bytes).
// Instance k, block j, run r sits at k*extent + j*stride + disp[r]; a run is cut only at the
// window's edges; fn returns false to stop early.  Returns false when the window runs past count
// instances.
template <class F>
static bool walk(const mi355x_ddt *d, size_t count, size_t pos, size_t bytes, F &&fn)
{
    const int64_t blk = blk_bytes(d), inst = d->nblk * blk;
    if ((int64_t)(pos + bytes) > (int64_t)count * inst) return false;
    if (bytes == 0 || inst == 0) return true;
    int64_t k = (int64_t)pos / inst, rem = (int64_t)pos % inst;
    int64_t j = rem / blk, in_blk = rem % blk;
    size_t r = (size_t)(std::upper_bound(d->pfx.begin(), d->pfx.end(), in_blk) - d->pfx.begin()) - 1;
    while (r + 1 < d->len.size() && d->len[r] == 0) ++r;  // zero-length runs hold no bytes
    int64_t within = in_blk - d->pfx[r];
    size_t done = 0;
    while (done < bytes) {
        const int64_t avail = d->len[r] - within;
        const size_t take = (size_t)std::min<int64_t>(avail, (int64_t)(bytes - done));
        if (take && !fn(k * d->extent + j * d->stride + d->disp[r] + within, take, pos + done)) return true;
        done += take;
        within += (int64_t)take;
        if (within == d->len[r]) {
            within = 0;
            if (++r == d->len.size()) {
                r = 0;
                if (++j == d->nblk) {
                    j = 0;
                    ++k;
                }
            }
        }
    }
    return true;
}
} // namespace mi355x

extern "C" {

// the convertor on host memory: what ob1 does for a host buffer with a derived datatype
// (opal_generic_simple_pack / _unpack, opal_datatype_pack.c:250-374, opal_datatype_unpack.c:245-…)
int mi355x_pack_host(const mi355x_ddt_t *d, size_t count, const void *base, size_t pos, void *dst, size_t bytes)
{
    if (!d || (bytes && (!base || !dst))) return set_error(MI355X_ERR_ARG, "bad host pack arguments");
    const char *b = (const char *)base;
    char *o = (char *)dst;
    if (!walk(d, count, pos, bytes, [&](int64_t off, size_t len, size_t p) {
            std::memcpy(o + (p - pos), b + off, len);
            return true;
        }))
        return set_error(MI355X_ERR_ARG, "window past the message");
    return MI355X_SUCCESS;
}

int mi355x_unpack_host(const mi355x_ddt_t *d, size_t count, void *base, size_t pos, const void *src, size_t bytes)
{
    if (!d || (bytes && (!base || !src))) return set_error(MI355X_ERR_ARG, "bad host unpack arguments");
    char *b = (char *)base;
    const char *i = (const char *)src;
    if (!walk(d, count, pos, bytes, [&](int64_t off, size_t len, size_t p) {
            std::memcpy(b + off, i + (p - pos), len);
            return true;
        }))
        return set_error(MI355X_ERR_ARG, "window past the message");
    return MI355X_SUCCESS;
}

// opal_convertor_raw (opal/datatype/opal_convertor_raw.c:37-…): the memory pieces of the type map
// from packed position *pos, at most *iov_count of them; *iov_count = pieces returned, *max_data =
// their bytes, *pos advanced.  Returns 1 once the whole message has been described, else 0 (the
// reference's return convention).  Runs are merged where the layout merges them (adjacent blocks of
// one constructor), so a piece may cover several of the reference's iovecs; the byte sequence is
// the same.
int mi355x_ddt_raw(const mi355x_ddt_t *d, size_t count, size_t *pos, int64_t *disp, size_t *len, uint32_t *iov_count,
                   size_t *max_data)
{
    if (!d || !pos || !iov_count || !max_data || (*iov_count && (!disp || !len)))
        return set_error(MI355X_ERR_ARG, "bad raw arguments");
    const size_t total = count * (size_t)(d->nblk * blk_bytes(d));
    const uint32_t cap = *iov_count;
    uint32_t n = 0;
    size_t got = 0;
    size_t p = *pos;
    while (n < cap && p < total) {
        // one piece: the rest of the current run
        int64_t off0 = 0;
        size_t len0 = 0;
        (void)walk(d, count, p, total - p, [&](int64_t off, size_t l, size_t) {
            off0 = off;
            len0 = l;
            return false;
        });
        disp[n] = off0;
        len[n] = len0;
        ++n;
        got += len0;
        p += len0;
    }
    *iov_count = n;
    *max_data = got;
    *pos = p;
    return p >= total ? 1 : 0;
}

int mi355x_unpack(const mi355x_ddt_t *d, size_t count, void *base, size_t pos, const void *src, size_t bytes,
                  uint32_t *checksum, void *stream)
{
    return ddt_move(d, false, count, base, pos, const_cast<void *>(src), bytes, checksum, stream);
}

} // extern "C"
