// ddt_kernels.hip -- GPU convertor: pack / unpack of derived datatypes on device buffers.
//
// Replaces the reference's per-run synchronous device memcpy (MEMCPY_CSUM -> cbmemcpy ->
// cuMemcpy, opal/datatype/opal_datatype_pack.h:24-76, opal_datatype_cuda.c:93-115; one 256-byte
// copy per vector block) with one kernel per fragment.
//
// Layout (mi355x_ddt): instance k at base + k*extent; inside it nblk blocks at j*stride; inside a
// block the runs (disp, len) in order.  The packed stream is that type map in order (the order
// opal_generic_simple_pack walks the description in).  A launch handles the packed window
// [pos, pos+bytes) -- any byte position, as opal_convertor_set_position + pack does per fragment.
//
// Each lane owns 16-byte packed slots.  A slot that lies inside one run, inside the window, with
// 16-B aligned source and destination moves as one dwordx4 copy; anything else (run edges that
// are not 16-B multiples, window edges) falls back to bytes.  Optional checksum: the sum of the
// stream's native 32-bit words (opal_uicsum_partial, opal/util/crc.c:921) -- additive over
// windows, so per-fragment sums add up to the whole-message convertor checksum.
#include <algorithm>

#include "ddt_internal.hpp"
#include "rt_internal.hpp"

#include <mutex>
#include <vector>

namespace mi355x {

typedef unsigned int u32x4d __attribute__((ext_vector_type(4)));
// the same 16 bytes at an address only 4-B aligned (the memory side of k_ddt_units_wide): the
// type's alignment says so, so the compiler may not assume 16 (the dwordx4 access is legal on any
// 4-B boundary)
typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

struct Where {
    int64_t mem;     // byte offset in memory (relative to base)
    int64_t left;    // bytes left in this run
};

__device__ __forceinline__ Where locate(const DdtDev &d, int64_t p)
{
    const int64_t k = p / d.inst_bytes;
    const int64_t rem = p - k * d.inst_bytes;
    const int64_t j = rem / d.blk_bytes;
    const int64_t q = rem - j * d.blk_bytes;
    // runs: binary search in the packed prefix table (pfx[r] = packed offset of run r in a block)
    int lo = 0, hi = d.nruns - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (d.pfx[mid] <= q) lo = mid;
        else hi = mid - 1;
    }
    const int64_t o = q - d.pfx[lo];
    Where w;
    w.mem = k * d.extent + j * d.stride + d.disp[lo] + o;
    w.left = d.len[lo] - o;
    return w;
}

// checksum: every block stores its partial sum (waves reduced by shuffles, then through LDS);
// k_csum_finish, the next launch on the stream, adds the partials and writes the result straight
// into host-mapped memory -- no device-to-host copy, and no atomics (a one-shot grid has tens of
// thousands of blocks: one counter for them all would serialise, MI355X_MICROARCH.md "fanin")
struct CsumSink {
    unsigned *partial;   // one word per block
    unsigned *out;       // host-mapped result word
    unsigned nblocks;
};

__device__ __forceinline__ unsigned block_reduce(unsigned acc)
{
    __shared__ unsigned ws[16];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
    __syncthreads();
    unsigned t = 0;
    if (threadIdx.x == 0)
        for (unsigned i = 0; i < (blockDim.x + 63) / 64; ++i) t += ws[i];
    return t;  // valid in thread 0
}

__device__ __forceinline__ void block_sum_store(unsigned acc, const CsumSink &k)
{
    const unsigned t = block_reduce(acc);
    if (threadIdx.x == 0) k.partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void k_csum_finish(CsumSink k)
{
    // tens of thousands of partials through one workgroup: 16-B loads, 8 in flight per lane
    unsigned a = 0;
    const unsigned nv = k.nblocks / 4;
    const u32x4d *pv = reinterpret_cast<const u32x4d *>(k.partial);
    for (unsigned base = threadIdx.x; base < nv; base += 8 * blockDim.x) {
        u32x4d v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned i = base + u * blockDim.x;
            v[u] = i < nv ? pv[i] : u32x4d{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (unsigned i = 4 * nv + threadIdx.x; i < k.nblocks; i += blockDim.x) a += k.partial[i];
    const unsigned total = block_reduce(a);
    if (threadIdx.x == 0) __hip_atomic_store(k.out, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool PACK, bool CSUM>
__global__ __launch_bounds__(256) void k_ddt(DdtDev d, char *mem, char *packed, int64_t pos, int64_t bytes,
                                             CsumSink csum)
{
    const int64_t first = pos >> 4, last = (pos + bytes + 15) >> 4;   // 16-B slots touching the window
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (int64_t s = first + tid; s < last; s += nthr) {
        const int64_t p0 = s << 4;
        char *pk = packed + (p0 - pos);                 // packed buffer holds the window only
        Where w = locate(d, p0);
        if (p0 >= pos && p0 + 16 <= pos + bytes && w.left >= 16 && ((w.mem + (int64_t)(uintptr_t)mem) & 15) == 0 &&
            (((uintptr_t)pk) & 15) == 0) {
            u32x4d v;
            if constexpr (PACK) {
                v = *reinterpret_cast<const u32x4d *>(mem + w.mem);
                *reinterpret_cast<u32x4d *>(pk) = v;
            } else {
                v = *reinterpret_cast<const u32x4d *>(pk);
                *reinterpret_cast<u32x4d *>(mem + w.mem) = v;
            }
            if constexpr (CSUM) acc += v.x + v.y + v.z + v.w;
        } else {
            const int64_t a = p0 > pos ? p0 : pos;
            const int64_t e = (p0 + 16 < pos + bytes) ? p0 + 16 : pos + bytes;
            if (a < e) w = locate(d, a);
            for (int64_t p = a; p < e; ++p) {
                if (w.left <= 0) w = locate(d, p);
                unsigned char byte;
                if constexpr (PACK) {
                    byte = (unsigned char)mem[w.mem];
                    packed[p - pos] = (char)byte;
                } else {
                    byte = (unsigned char)packed[p - pos];
                    mem[w.mem] = (char)byte;
                }
                if constexpr (CSUM) acc += (unsigned)byte << (8 * (p & 3));
                w.mem++;
                w.left--;
            }
        }
    }
    if constexpr (CSUM) block_sum_store(acc, csum);
}

// ---------------------------------------------------------------------------------------------
// Row kernel: the layout is one run of L bytes per block (vector, contiguous-with-gaps: what
// MPI_Type_vector and most derived types used for halos/columns compile to).  The packed stream
// is cut into W-byte slots, W the largest power of two (<= 16) dividing the run length, the run's
// address, the stride, the extent, the packed address and the window: 16 for the configs[4]
// shape, 8 for a column of doubles (MPI_Type_vector(n, 1, s, MPI_DOUBLE)), 4 for 3-float blocks,
// down to 1 for odd byte windows.  Row g (over all instances) starts at
// (g / nblk) * extent + (g % nblk) * stride + disp.  One-shot grid: each lane moves U slots,
// lanes of a wave on consecutive slots (one wave-instruction = 64 W contiguous packed bytes), all
// U loads issued before the stores.  The two divisions per slot are 32-bit multiply-high
// (Granlund-Montgomery magic numbers computed on the host), no 64-bit division, no search.
struct FastDiv {
    uint32_t m, l, d;
};

static FastDiv make_fastdiv(uint32_t d)
{
    FastDiv f;
    f.d = d;
    uint32_t l = 0;
    while (l < 32 && ((uint64_t)1 << l) < d) ++l;
    f.l = l;
    f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f)
{
    return (uint32_t)(((uint64_t)__umulhi(f.m, n) + n) >> f.l);
}

struct RowArgs {
    char *mem;
    char *packed;
    int64_t disp, stride, extent;
    FastDiv per_row;   // slots per row
    FastDiv per_inst;  // rows per instance (nblk)
    uint32_t first;    // first slot (pos / W)
    uint32_t nslots;
};

template <int W> struct SlotT;
template <> struct SlotT<16> { typedef u32x4d type; };
template <> struct SlotT<8> { typedef unsigned long long type; };
template <> struct SlotT<4> { typedef unsigned type; };
template <> struct SlotT<2> { typedef unsigned short type; };
template <> struct SlotT<1> { typedef unsigned char type; };

// the slot's share of the checksum (opal_uicsum_partial: the sum of the stream's native 32-bit
// words; q = absolute slot index, so the slot starts at packed byte q * W)
template <int W> __device__ __forceinline__ unsigned slot_csum(const typename SlotT<W>::type &v, uint32_t q)
{
    if constexpr (W == 16) return v.x + v.y + v.z + v.w;
    else if constexpr (W == 8) return (unsigned)v + (unsigned)(v >> 32);
    else if constexpr (W == 4) return v;
    else if constexpr (W == 2) return (unsigned)v << (16 * (q & 1));
    else return (unsigned)v << (8 * (q & 3));
}

template <bool PACK, bool CSUM, int NTM, int U, int W>
__device__ __forceinline__ unsigned rows_pass(const RowArgs &a, uint32_t base, uint32_t tpb)
{
    typedef typename SlotT<W>::type S;
    S v[U];
    char *mp[U];
    unsigned acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + (uint32_t)u * tpb;
        mp[u] = nullptr;
        if (i < a.nslots) {
            const uint32_t q = a.first + i;
            const uint32_t g = fdiv(q, a.per_row);
            const uint32_t w = q - g * a.per_row.d;
            const uint32_t k = fdiv(g, a.per_inst);
            const uint32_t j = g - k * a.per_inst.d;
            mp[u] = a.mem + (int64_t)k * a.extent + (int64_t)j * a.stride + a.disp + (int64_t)w * W;
            const S *src = reinterpret_cast<const S *>(PACK ? mp[u] : a.packed + (size_t)i * W);
            if constexpr ((NTM & 1) != 0) v[u] = __builtin_nontemporal_load(src);
            else v[u] = *src;
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (mp[u]) {
            const uint32_t i = base + (uint32_t)u * tpb;
            S *dst = reinterpret_cast<S *>(PACK ? a.packed + (size_t)i * W : mp[u]);
            if constexpr ((NTM & 2) != 0) __builtin_nontemporal_store(v[u], dst);
            else *dst = v[u];
            if constexpr (CSUM) acc += slot_csum<W>(v[u], a.first + i);
        }
    }
    return acc;
}

// one-shot grid, every lane one pass of U slots (measured fastest); with a checksum every block
// then stores its partial
template <bool PACK, bool CSUM, int NTM, int U, int W>
__global__ __launch_bounds__(1024) void k_ddt_rows(RowArgs a, CsumSink csum)
{
    const uint32_t tpb = blockDim.x;
    const unsigned acc = rows_pass<PACK, CSUM, NTM, U, W>(a, blockIdx.x * (tpb * U) + threadIdx.x, tpb);
    if constexpr (CSUM) block_sum_store(acc, csum);
}

// largest slot index the 32-bit row / unit kernels take: their grid-stride and last-block index
// arithmetic (at most 2^22 slots past the end) must not wrap
constexpr int64_t kSlot32Max = ((int64_t)1 << 32) - ((int64_t)1 << 22);

// the slot width the row kernel can use (0: it does not apply): one run per block, and every
// address, length and window a multiple of W; slot / row counts in 32 bits
static int rows_width(const DdtDev &d, int nruns_host, int64_t run_disp, int64_t run_len, const void *mem,
                      const void *packed, int64_t pos, int64_t bytes)
{
    if (nruns_host != 1 || run_len <= 0) return 0;
    const uint64_t bits = (uint64_t)run_len | ((uintptr_t)mem + (uint64_t)run_disp) | (uint64_t)d.stride |
                          (uint64_t)d.extent | (uintptr_t)packed | (uint64_t)pos | (uint64_t)bytes;
    int w = 16;
    while (w > 1 && (bits & (uint64_t)(w - 1))) w >>= 1;
    const int64_t last_slot = (pos + bytes) / w;
    const int64_t rows = last_slot / (run_len / w) + 1;
    // 32-bit slot arithmetic, with headroom for the last block's (tpb x U)-slot stride
    if (last_slot >= kSlot32Max || rows >= ((int64_t)1 << 32) || d.nblk >= ((int64_t)1 << 32) ||
        (run_len / w) >= ((int64_t)1 << 32))
        return 0;
    return w;
}

DdtTune &ddt_tune()
{
    static DdtTune t;
    return t;
}

// checksum workspaces: partials on the device, the result word in host-mapped memory; pooled per
// device (a call holds one until its stream has finished with it)
struct CsumWs {
    int device = -1;
    unsigned *partial = nullptr;
    size_t cap = 0;
    unsigned *host = nullptr, *host_dev = nullptr;
};
static std::mutex g_csum_mtx;
static std::vector<CsumWs *> g_csum_free;

struct Csum {
    CsumWs *ws = nullptr;
    CsumSink sink{};
    // take a workspace with room for `blocks` partials (nothing when no checksum is wanted)
    int get(unsigned *want, unsigned blocks)
    {
        if (!want) return MI355X_SUCCESS;
        int dev = 0;
        MI_HIP(hipGetDevice(&dev));
        {
            std::lock_guard<std::mutex> g(g_csum_mtx);
            for (size_t i = 0; i < g_csum_free.size(); ++i)
                if (g_csum_free[i]->device == dev) {
                    ws = g_csum_free[i];
                    g_csum_free.erase(g_csum_free.begin() + (long)i);
                    break;
                }
        }
        if (!ws) {
            ws = new CsumWs();
            ws->device = dev;
            MI_HIP(hipHostMalloc((void **)&ws->host, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
            MI_HIP(hipHostGetDevicePointer((void **)&ws->host_dev, ws->host, 0));
        }
        if (ws->cap < blocks) {
            if (ws->partial) MI_HIP(hipFree(ws->partial));
            ws->partial = nullptr;
            ws->cap = 0;
            MI_HIP(hipMalloc((void **)&ws->partial, sizeof(unsigned) * blocks));
            ws->cap = blocks;
        }
        sink.partial = ws->partial;
        sink.out = ws->host_dev;
        sink.nblocks = blocks;
        return MI355X_SUCCESS;
    }
    // add the partials (next launch on the stream), wait, hand the checksum over, return the
    // workspace to the pool
    int finish(unsigned *want, hipStream_t s)
    {
        if (!want) return MI355X_SUCCESS;
        hipLaunchKernelGGL(k_csum_finish, dim3(1), dim3(1024), 0, s, sink);
        MI_HIP(hipGetLastError());
        MI_HIP(hipStreamSynchronize(s));
        *want = __atomic_load_n(ws->host, __ATOMIC_ACQUIRE);
        std::lock_guard<std::mutex> g(g_csum_mtx);
        g_csum_free.push_back(ws);
        ws = nullptr;
        return MI355X_SUCCESS;
    }
    ~Csum()
    {
        // a workspace still held here belongs to a failed launch (a kernel may still use it): it
        // is dropped rather than pooled
        if (ws) {
            (void)hipFree(ws->partial);
            (void)hipHostFree(ws->host);
            delete ws;
        }
    }
};

template <bool PACK, bool CSUM, int NTM>
static void launch_rows_u(const RowArgs &a, int unroll, unsigned tpb, unsigned blocks, const CsumSink &part,
                          hipStream_t s)
{
    switch (unroll) {
    case 2: hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, NTM, 2, 16>), dim3(blocks), dim3(tpb), 0, s, a, part); break;
    case 8: hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, NTM, 8, 16>), dim3(blocks), dim3(tpb), 0, s, a, part); break;
    default: hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, NTM, 4, 16>), dim3(blocks), dim3(tpb), 0, s, a, part); break;
    }
}

template <bool PACK, bool CSUM>
static void launch_rows(const RowArgs &a, int ntm, int unroll, unsigned tpb, unsigned blocks, const CsumSink &part,
                        hipStream_t s)
{
    switch (ntm & 3) {
    case 0: launch_rows_u<PACK, CSUM, 0>(a, unroll, tpb, blocks, part, s); break;
    case 1: launch_rows_u<PACK, CSUM, 1>(a, unroll, tpb, blocks, part, s); break;
    case 2: launch_rows_u<PACK, CSUM, 2>(a, unroll, tpb, blocks, part, s); break;
    default: launch_rows_u<PACK, CSUM, 3>(a, unroll, tpb, blocks, part, s); break;
    }
}

// narrow slots (W < 16): fixed shape, kNarrowUnroll slots per lane, non-temporal or not
constexpr int kNarrowUnroll = 8;
template <bool PACK, bool CSUM, int W>
static void launch_rows_w(const RowArgs &a, bool nt, unsigned tpb, unsigned blocks, const CsumSink &part, hipStream_t s)
{
    if (nt) hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, 3, kNarrowUnroll, W>), dim3(blocks), dim3(tpb), 0, s, a, part);
    else hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, 0, kNarrowUnroll, W>), dim3(blocks), dim3(tpb), 0, s, a, part);
}

template <bool PACK, bool CSUM>
static void launch_rows_narrow(int w, const RowArgs &a, bool nt, unsigned tpb, unsigned blocks, const CsumSink &part,
                               hipStream_t s)
{
    switch (w) {
    case 8: launch_rows_w<PACK, CSUM, 8>(a, nt, tpb, blocks, part, s); break;
    case 4: launch_rows_w<PACK, CSUM, 4>(a, nt, tpb, blocks, part, s); break;
    case 2: launch_rows_w<PACK, CSUM, 2>(a, nt, tpb, blocks, part, s); break;
    default: launch_rows_w<PACK, CSUM, 1>(a, nt, tpb, blocks, part, s); break;
    }
}

int launch_ddt_rows(const DdtDev &d, int nruns_host, int64_t run_disp, int64_t run_len, bool pack, void *mem,
                    void *packed, int64_t pos, int64_t bytes, unsigned *csum, hipStream_t s)
{
    const int mode = ddt_tune().rows;
    const int w = mode > 0 ? rows_width(d, nruns_host, run_disp, run_len, mem, packed, pos, bytes) : 0;
    if (w == 0 || (w < 16 && mode < 2)) return 1;
    RowArgs a;
    a.mem = static_cast<char *>(mem);
    a.packed = static_cast<char *>(packed);
    a.disp = run_disp;
    a.stride = d.stride;
    a.extent = d.extent;
    a.per_row = make_fastdiv((uint32_t)(run_len / w));
    a.per_inst = make_fastdiv((uint32_t)d.nblk);
    a.first = (uint32_t)(pos / w);
    a.nslots = (uint32_t)(bytes / w);
    const DdtTune &t = ddt_tune();
    int unroll = pack ? t.unroll_pack : t.unroll_unpack;
    if (unroll != 2 && unroll != 8) unroll = 4;
    if (w < 16) unroll = kNarrowUnroll;
    const unsigned tpb = (t.threads == 256 || t.threads == 512) ? (unsigned)t.threads : 1024u;
    int ntm = t.nontemporal;
    if (ntm < 0) ntm = (2 * bytes > ((int64_t)256 << 20)) ? kDdtAutoNT : 0;  // streaming sizes
    const uint64_t per = (uint64_t)tpb * (uint64_t)unroll;
    const unsigned blocks = (unsigned)((a.nslots + per - 1) / per);
    Csum part;
    int rc = part.get(csum, blocks);
    if (rc) return rc;
    if (w < 16) {
        if (pack) {
            if (csum) launch_rows_narrow<true, true>(w, a, ntm != 0, tpb, blocks, part.sink, s);
            else launch_rows_narrow<true, false>(w, a, ntm != 0, tpb, blocks, part.sink, s);
        } else {
            if (csum) launch_rows_narrow<false, true>(w, a, ntm != 0, tpb, blocks, part.sink, s);
            else launch_rows_narrow<false, false>(w, a, ntm != 0, tpb, blocks, part.sink, s);
        }
    } else if (pack) {
        if (csum) launch_rows<true, true>(a, ntm, unroll, tpb, blocks, part.sink, s);
        else launch_rows<true, false>(a, ntm, unroll, tpb, blocks, part.sink, s);
    } else {
        if (csum) launch_rows<false, true>(a, ntm, unroll, tpb, blocks, part.sink, s);
        else launch_rows<false, false>(a, ntm, unroll, tpb, blocks, part.sink, s);
    }
    MI_HIP(hipGetLastError());
    return part.finish(csum, s);
}

// ---------------------------------------------------------------------------------------------
// Unit kernel: any run list (indexed, struct, several runs per block) whose runs, strides, the
// buffers and the window are all multiples of a W-byte unit (W = 16, 8, 4, 2 or 1).  The run
// tables are staged into LDS once per workgroup (packed prefix in units as 32-bit words, run
// displacements) -- the "gathered datatype" staging: every unit's run lookup is then a binary
// search in LDS instead of dependent global loads; instance and block come from two 32-bit
// multiply-high divisions.  Lanes of a wave take consecutive units (the packed side coalesces);
// a persistent grid so the table staging is paid once per workgroup, not per unit.
struct UnitArgs {
    char *mem;
    char *packed;
    const int64_t *disp;   // device run tables (bytes)
    const int64_t *pfx;
    int nruns;
    int lw;                // log2(W)
    int64_t stride, extent;
    FastDiv per_inst;      // units per instance
    FastDiv per_blk;       // units per block
    uint32_t first;        // first unit (pos / W)
    uint32_t nunits;
};

constexpr int kUnitMaxRuns = 4096;   // LDS: 12 B per run -> 48 KiB
constexpr int kUnitU = 4;            // units per lane per pass
constexpr int kWideRunUnits = 8;     // wide slots only for runs this long on average

template <bool PACK, bool CSUM, int W>
__global__ __launch_bounds__(256) void k_ddt_units(UnitArgs a, CsumSink csum)
{
    typedef typename SlotT<W>::type S;
    extern __shared__ int64_t unit_lds[];
    int64_t *sdisp = unit_lds;
    uint32_t *spfx = reinterpret_cast<uint32_t *>(unit_lds + a.nruns);
    for (int r = threadIdx.x; r < a.nruns; r += blockDim.x) {
        sdisp[r] = a.disp[r];
        spfx[r] = (uint32_t)(a.pfx[r] >> a.lw);
    }
    __syncthreads();
    const uint32_t tpb = blockDim.x, stride = gridDim.x * tpb * kUnitU;
    unsigned acc = 0;
    for (uint32_t base = blockIdx.x * tpb * kUnitU + threadIdx.x; base < a.nunits; base += stride) {
        S v[kUnitU];
        char *mp[kUnitU];
#pragma unroll
        for (int u = 0; u < kUnitU; ++u) {
            const uint32_t i = base + (uint32_t)u * tpb;
            mp[u] = nullptr;
            if (i < a.nunits) {
                const uint32_t q = a.first + i;
                const uint32_t k = fdiv(q, a.per_inst);
                const uint32_t rem = q - k * a.per_inst.d;
                const uint32_t j = fdiv(rem, a.per_blk);
                const uint32_t o = rem - j * a.per_blk.d;
                int lo = 0, hi = a.nruns - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (spfx[mid] <= o) lo = mid;
                    else hi = mid - 1;
                }
                mp[u] = a.mem + (int64_t)k * a.extent + (int64_t)j * a.stride + sdisp[lo] + (int64_t)(o - spfx[lo]) * W;
                v[u] = *reinterpret_cast<const S *>(PACK ? mp[u] : a.packed + (size_t)i * W);
            }
        }
#pragma unroll
        for (int u = 0; u < kUnitU; ++u) {
            if (mp[u]) {
                const uint32_t i = base + (uint32_t)u * tpb;
                *reinterpret_cast<S *>(PACK ? a.packed + (size_t)i * W : mp[u]) = v[u];
                if constexpr (CSUM) acc += slot_csum<W>(v[u], a.first + i);
            }
        }
    }
    if constexpr (CSUM) block_sum_store(acc, csum);
}

// packed unit o of a block (o < units per block) -> its run, by binary search in the LDS table
__device__ __forceinline__ int unit_run(const uint32_t *spfx, int nruns, uint32_t o)
{
    int lo = 0, hi = nruns - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (spfx[mid] <= o) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Wide slots: the packed side is 16-B aligned but the memory side only W-aligned (W = 8 or 4: a
// triangle of doubles, runs of 3 floats): a lane moves a 16-B packed slot = 16 / W units; when the
// slot lies inside one run the memory side is one 16-B access at a W-aligned address (global
// dwordx4 needs only dword alignment), else the units go one by one.  The run tables are in LDS as
// in k_ddt_units (units of W).
template <bool PACK, bool CSUM, int W>
__global__ __launch_bounds__(256) void k_ddt_units_wide(UnitArgs a, CsumSink csum)
{
    typedef typename SlotT<W>::type S;
    constexpr uint32_t UPS = 16 / W;  // units per slot
    extern __shared__ int64_t unit_lds[];
    int64_t *sdisp = unit_lds;
    uint32_t *spfx = reinterpret_cast<uint32_t *>(unit_lds + a.nruns);
    for (int r = threadIdx.x; r < a.nruns; r += blockDim.x) {
        sdisp[r] = a.disp[r];
        spfx[r] = (uint32_t)(a.pfx[r] >> a.lw);
    }
    __syncthreads();
    const uint32_t blk_u = a.per_blk.d, nblk = a.per_inst.d / a.per_blk.d, nslots = a.nunits / UPS;
    const uint32_t tpb = blockDim.x, stride = gridDim.x * tpb * kUnitU;
    unsigned acc = 0;
    for (uint32_t base = blockIdx.x * tpb * kUnitU + threadIdx.x; base < nslots; base += stride) {
        u32x4d v[kUnitU];
        char *mp[kUnitU];   // the slot's memory address when it lies inside one run, else NULL
        bool live[kUnitU];
#pragma unroll
        for (int u = 0; u < kUnitU; ++u) {
            const uint32_t i = base + (uint32_t)u * tpb;
            live[u] = i < nslots;
            mp[u] = nullptr;
            if (!live[u]) continue;
            uint32_t q = a.first + i * UPS;
            uint32_t k = fdiv(q, a.per_inst);
            const uint32_t rem = q - k * a.per_inst.d;
            uint32_t j = fdiv(rem, a.per_blk);
            uint32_t o = rem - j * blk_u;
            int r = unit_run(spfx, a.nruns, o);
            o -= spfx[r];
            const uint32_t rl = (r + 1 < a.nruns ? spfx[r + 1] : blk_u) - spfx[r];
            char *m0 = a.mem + (int64_t)k * a.extent + (int64_t)j * a.stride + sdisp[r] + (int64_t)o * W;
            if (o + UPS <= rl) {
                mp[u] = m0;
                v[u] = PACK ? *reinterpret_cast<const u32x4a4 *>(m0)
                            : *reinterpret_cast<const u32x4d *>(a.packed + (size_t)i * 16);
                continue;
            }
            // the slot crosses a run boundary: unit by unit
            S part[UPS];
            const S *pk = reinterpret_cast<const S *>(a.packed + (size_t)i * 16);
#pragma unroll
            for (uint32_t t = 0; t < UPS; ++t) {
                char *mt = a.mem + (int64_t)k * a.extent + (int64_t)j * a.stride + sdisp[r] + (int64_t)o * W;
                if (PACK) part[t] = *reinterpret_cast<const S *>(mt);
                else *reinterpret_cast<S *>(mt) = pk[t];
                if (++o == (r + 1 < a.nruns ? spfx[r + 1] : blk_u) - spfx[r]) {
                    o = 0;
                    if (++r == a.nruns) {
                        r = 0;
                        if (++j == nblk) {
                            j = 0;
                            ++k;
                        }
                    }
                }
            }
            if (PACK) __builtin_memcpy(&v[u], part, 16);
            else v[u] = *reinterpret_cast<const u32x4d *>(a.packed + (size_t)i * 16);
        }
#pragma unroll
        for (int u = 0; u < kUnitU; ++u) {
            if (!live[u]) continue;
            const uint32_t i = base + (uint32_t)u * tpb;
            if (PACK) *reinterpret_cast<u32x4d *>(a.packed + (size_t)i * 16) = v[u];
            else if (mp[u]) *reinterpret_cast<u32x4a4 *>(mp[u]) = v[u];
            if constexpr (CSUM) acc += slot_csum<16>(v[u], 0);
        }
    }
    if constexpr (CSUM) block_sum_store(acc, csum);
}

template <bool PACK, bool CSUM>
static void launch_units_wide(int w, const UnitArgs &a, unsigned blocks, size_t lds, const CsumSink &part, hipStream_t s)
{
    if (w == 8) hipLaunchKernelGGL((k_ddt_units_wide<PACK, CSUM, 8>), dim3(blocks), dim3(256), lds, s, a, part);
    else hipLaunchKernelGGL((k_ddt_units_wide<PACK, CSUM, 4>), dim3(blocks), dim3(256), lds, s, a, part);
}

template <bool PACK, bool CSUM>
static void launch_units_w(int w, const UnitArgs &a, unsigned blocks, size_t lds, const CsumSink &part, hipStream_t s)
{
    switch (w) {
    case 16: hipLaunchKernelGGL((k_ddt_units<PACK, CSUM, 16>), dim3(blocks), dim3(256), lds, s, a, part); break;
    case 8: hipLaunchKernelGGL((k_ddt_units<PACK, CSUM, 8>), dim3(blocks), dim3(256), lds, s, a, part); break;
    case 4: hipLaunchKernelGGL((k_ddt_units<PACK, CSUM, 4>), dim3(blocks), dim3(256), lds, s, a, part); break;
    case 2: hipLaunchKernelGGL((k_ddt_units<PACK, CSUM, 2>), dim3(blocks), dim3(256), lds, s, a, part); break;
    default: hipLaunchKernelGGL((k_ddt_units<PACK, CSUM, 1>), dim3(blocks), dim3(256), lds, s, a, part); break;
    }
}

// Unpack of long W-aligned runs (W = 8 or 4, e.g. an upper triangle of doubles): one WAVE per run
// of one block of one instance, one-shot grid, no run search -- the wave's index is the run's
// (instance, block, run) and its table entries are uniform loads.  The lanes store 16-B ALIGNED
// memory slots (the unit kernel stores W bytes, its wide form unaligned 16-B vectors: both slower,
// profiles/r03_unpack_ceiling.jsonl) and read the packed side with 16-B loads at W-aligned
// addresses; the run's unaligned head and tail move as W-byte units.  Needs the base, extent and
// stride 16-B aligned (a run's misalignment is then its displacement's) and runs of balanced length
// (ddt_move checks kRunsMinBytes / kRunsMaxSkew).  Any W-aligned window [pos, pos + bytes) of the
// packed stream (the convertor's set_position fragments, a16): the waves cover the runs from the
// one holding byte pos to the one holding its last byte (found on the host, once per launch), and
// each wave clips its run to the window.
struct RunsArgs {
    char *mem;
    const char *packed;  // the window's bytes (packed stream offset pos)
    const int64_t *disp, *len, *pfx;
    int64_t stride, extent, blk_bytes, inst_bytes;
    int64_t pos, end;    // the window in the packed stream
    FastDiv per_inst;    // runs per instance (nblk * nruns)
    FastDiv nruns;
    uint32_t q0;         // the window's first run (message-wide index)
    uint32_t nwaves;     // runs the window touches
};

constexpr int64_t kRunsMinBytes = 512;   // average run length the wave-per-run unpack needs
constexpr int64_t kRunsMaxSkew = 8;      // longest run at most this many times the average

template <int W>
__global__ __launch_bounds__(256) void k_ddt_runs_unpack(RunsArgs a)
{
    typedef typename SlotT<W>::type S;
    const uint32_t wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wv >= a.nwaves) return;
    const uint32_t q = a.q0 + wv;
    const int lane = threadIdx.x & 63;
    const uint32_t k = fdiv(q, a.per_inst);
    const uint32_t rem = q - k * a.per_inst.d;
    const uint32_t j = fdiv(rem, a.nruns);
    const uint32_t r = rem - j * a.nruns.d;
    // the run in the packed stream, clipped to the window
    const int64_t P = (int64_t)k * a.inst_bytes + (int64_t)j * a.blk_bytes + a.pfx[r];
    const int64_t lo = a.pos > P ? a.pos - P : 0;
    const int64_t hi = a.end - P < a.len[r] ? a.end - P : a.len[r];
    const int64_t len = hi - lo;
    char *m = a.mem + (int64_t)k * a.extent + (int64_t)j * a.stride + a.disp[r] + lo;
    const char *pk = a.packed + (P + lo - a.pos);
    int64_t h = (16 - ((uintptr_t)m & 15)) & 15;
    if (h > len) h = len;
    const int64_t end = h + ((len - h) & ~(int64_t)15);
    if (lane < h / W) *reinterpret_cast<S *>(m + lane * W) = *reinterpret_cast<const S *>(pk + lane * W);
    for (int64_t o = h + (int64_t)lane * 16; o < end; o += 64 * 16)
        *reinterpret_cast<u32x4d *>(m + o) = *reinterpret_cast<const u32x4a4 *>(pk + o);
    if (lane < (len - end) / W)
        *reinterpret_cast<S *>(m + end + lane * W) = *reinterpret_cast<const S *>(pk + end + lane * W);
}

// message-wide index of the run holding packed byte x (x inside the message)
static uint64_t run_at(const DdtDev &d, int64_t x)
{
    const int64_t k = x / d.inst_bytes, in_inst = x - k * d.inst_bytes;
    const int64_t j = in_inst / d.blk_bytes, in_blk = in_inst - j * d.blk_bytes;
    const int64_t r = (int64_t)(std::upper_bound(d.pfx_host, d.pfx_host + d.nruns, in_blk) - d.pfx_host) - 1;
    return ((uint64_t)k * (uint64_t)d.nblk + (uint64_t)j) * (uint64_t)d.nruns + (uint64_t)r;
}

// returns 1 when the wave-per-run unpack does not apply
static int launch_runs_unpack(const DdtDev &d, int w, void *mem, const void *packed, int64_t pos, int64_t bytes,
                              hipStream_t s)
{
    if (d.inst_bytes <= 0 || d.max_len <= 0 || bytes <= 0 || !d.pfx_host || !d.len_host) return 1;
    for (int r = 0; r < d.nruns; ++r)
        if (d.len_host[r] <= 0) return 1;  // (run_at assumes every run holds bytes)
    if ((((uintptr_t)mem) | (uint64_t)d.extent | (uint64_t)d.stride) & 15) return 1;
    if (d.blk_bytes < kRunsMinBytes * d.nruns || d.max_len * d.nruns > kRunsMaxSkew * d.blk_bytes) return 1;
    const uint64_t per_inst = (uint64_t)d.nblk * (uint64_t)d.nruns;
    const uint64_t q0 = run_at(d, pos), q1 = run_at(d, pos + bytes - 1);
    if (per_inst >= ((uint64_t)1 << 32) || q1 >= ((uint64_t)1 << 32) - 4) return 1;
    RunsArgs a;
    a.mem = static_cast<char *>(mem);
    a.packed = static_cast<const char *>(packed);
    a.disp = d.disp;
    a.len = d.len;
    a.pfx = d.pfx;
    a.stride = d.stride;
    a.extent = d.extent;
    a.blk_bytes = d.blk_bytes;
    a.inst_bytes = d.inst_bytes;
    a.pos = pos;
    a.end = pos + bytes;
    a.per_inst = make_fastdiv((uint32_t)per_inst);
    a.nruns = make_fastdiv((uint32_t)d.nruns);
    a.q0 = (uint32_t)q0;
    a.nwaves = (uint32_t)(q1 - q0 + 1);
    const unsigned blocks = (a.nwaves + 3) / 4;
    if (w == 8) hipLaunchKernelGGL((k_ddt_runs_unpack<8>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_ddt_runs_unpack<4>), dim3(blocks), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

// returns 1 when the unit kernel does not apply
static int launch_ddt_units(const DdtDev &d, bool pack, void *mem, void *packed, int64_t pos, int64_t bytes,
                            unsigned *csum, hipStream_t s)
{
    if (ddt_tune().rows < 2 || d.nruns > kUnitMaxRuns || d.nruns < 1 || d.blk_bytes <= 0) return 1;
    const uint64_t bits = d.run_bits | (uint64_t)d.stride | (uint64_t)d.extent | (uintptr_t)mem | (uintptr_t)packed |
                          (uint64_t)pos | (uint64_t)bytes | (uint64_t)d.blk_bytes;
    int w = 16, lw = 4;
    while (w > 1 && (bits & (uint64_t)(w - 1))) {
        w >>= 1;
        --lw;
    }
    const int64_t last = (pos + bytes) / w;
    if (last >= kSlot32Max || d.inst_bytes / w >= ((int64_t)1 << 32) || d.nblk >= ((int64_t)1 << 32)) return 1;
    UnitArgs a;
    a.mem = static_cast<char *>(mem);
    a.packed = static_cast<char *>(packed);
    a.disp = d.disp;
    a.pfx = d.pfx;
    a.nruns = d.nruns;
    a.lw = lw;
    a.stride = d.stride;
    a.extent = d.extent;
    a.per_inst = make_fastdiv((uint32_t)(d.inst_bytes / w));
    a.per_blk = make_fastdiv((uint32_t)(d.blk_bytes / w));
    a.first = (uint32_t)(pos / w);
    a.nunits = (uint32_t)(bytes / w);
    // wide slots: the packed side 16-B aligned, the memory side 4- or 8-B, pack only and runs of at
    // least kWideRunUnits units on average (mode 3 keeps W-byte units).  Measured (256 MiB packed,
    // profiles/r02_legs_ddt_wide.jsonl): triangle of doubles pack 4.70 vs 4.24 TB/s, but its unpack
    // 3.53 vs 3.73 (16-B stores at 8-B alignment) and 7-run floats pack 3.18 vs 3.30 (short runs:
    // most slots cross a run boundary)
    if (ddt_tune().rows == 2 && !pack && !csum && (w == 8 || w == 4)) {
        const int rrc = launch_runs_unpack(d, w, mem, packed, pos, bytes, s);
        if (rrc != 1) return rrc;
    }
    const uint64_t pk_bits = (uintptr_t)packed | (uint64_t)pos | (uint64_t)bytes;
    const bool wide = ddt_tune().rows == 2 && pack && (w == 8 || w == 4) && (pk_bits & 15) == 0 &&
                      (uint64_t)(d.blk_bytes / w) >= (uint64_t)kWideRunUnits * (uint64_t)d.nruns;
    const uint64_t per = 256u * kUnitU * (wide ? 16u / (unsigned)w : 1u);
    uint64_t blocks = (a.nunits + per - 1) / per;
    const uint64_t cap = (uint64_t)8 * (uint64_t)device_cu_count();
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    const size_t lds = (size_t)d.nruns * (sizeof(int64_t) + sizeof(uint32_t));
    Csum part;
    int rc = part.get(csum, (unsigned)blocks);
    if (rc) return rc;
    if (wide) {
        if (pack) {
            if (csum) launch_units_wide<true, true>(w, a, (unsigned)blocks, lds, part.sink, s);
            else launch_units_wide<true, false>(w, a, (unsigned)blocks, lds, part.sink, s);
        } else {
            if (csum) launch_units_wide<false, true>(w, a, (unsigned)blocks, lds, part.sink, s);
            else launch_units_wide<false, false>(w, a, (unsigned)blocks, lds, part.sink, s);
        }
    } else if (pack) {
        if (csum) launch_units_w<true, true>(w, a, (unsigned)blocks, lds, part.sink, s);
        else launch_units_w<true, false>(w, a, (unsigned)blocks, lds, part.sink, s);
    } else {
        if (csum) launch_units_w<false, true>(w, a, (unsigned)blocks, lds, part.sink, s);
        else launch_units_w<false, false>(w, a, (unsigned)blocks, lds, part.sink, s);
    }
    MI_HIP(hipGetLastError());
    return part.finish(csum, s);
}

int launch_ddt(const DdtDev &d, bool pack, void *mem, void *packed, int64_t pos, int64_t bytes, unsigned *csum,
               hipStream_t s)
{
    if (bytes <= 0) return MI355X_SUCCESS;
    const int urc = launch_ddt_units(d, pack, mem, packed, pos, bytes, csum, s);
    if (urc != 1) return urc;
    const int64_t slots = ((pos + bytes + 15) >> 4) - (pos >> 4);
    size_t blocks = (size_t)((slots + 255) / 256);
    const size_t cap = (size_t)8 * (size_t)device_cu_count();
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    char *m = static_cast<char *>(mem), *pk = static_cast<char *>(packed);
    Csum part;
    int rc = part.get(csum, (unsigned)blocks);
    if (rc) return rc;
    const CsumSink &pp = part.sink;
    if (pack) {
        if (csum) hipLaunchKernelGGL((k_ddt<true, true>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, pp);
        else hipLaunchKernelGGL((k_ddt<true, false>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, pp);
    } else {
        if (csum) hipLaunchKernelGGL((k_ddt<false, true>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, pp);
        else hipLaunchKernelGGL((k_ddt<false, false>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, pp);
    }
    MI_HIP(hipGetLastError());
    return part.finish(csum, s);
}

} // namespace mi355x
