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
#include "ddt_internal.hpp"
#include "rt_internal.hpp"

#include <mutex>
#include <vector>

namespace mi355x {

typedef unsigned int u32x4d __attribute__((ext_vector_type(4)));

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
// MPI_Type_vector and most derived types used for halos/columns compile to), everything 16-byte
// aligned.  Row g (over all instances) starts at (g / nblk) * extent + (g % nblk) * stride + disp.
// One-shot grid: each lane moves U 16-byte slots, lanes of a wave on consecutive slots, all U
// loads issued before the stores.  The two divisions per slot are 32-bit multiply-high
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
    uint32_t first;    // first slot (pos / 16)
    uint32_t nslots;
};

template <bool PACK, bool CSUM, int NTM, int U>
__device__ __forceinline__ unsigned rows_pass(const RowArgs &a, uint32_t base, uint32_t tpb)
{
    u32x4d v[U];
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
            mp[u] = a.mem + (int64_t)k * a.extent + (int64_t)j * a.stride + a.disp + ((int64_t)w << 4);
            const u32x4d *src = reinterpret_cast<const u32x4d *>(PACK ? mp[u] : a.packed + ((size_t)i << 4));
            if constexpr ((NTM & 1) != 0) v[u] = __builtin_nontemporal_load(src);
            else v[u] = *src;
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (mp[u]) {
            u32x4d *dst = reinterpret_cast<u32x4d *>(PACK ? a.packed + ((size_t)(base + (uint32_t)u * tpb) << 4) : mp[u]);
            if constexpr ((NTM & 2) != 0) __builtin_nontemporal_store(v[u], dst);
            else *dst = v[u];
            if constexpr (CSUM) acc += v[u].x + v[u].y + v[u].z + v[u].w;
        }
    }
    return acc;
}

// one-shot grid, every lane one pass of U slots (measured fastest); with a checksum every block
// then stores its partial
template <bool PACK, bool CSUM, int NTM, int U>
__global__ __launch_bounds__(1024) void k_ddt_rows(RowArgs a, CsumSink csum)
{
    const uint32_t tpb = blockDim.x;
    const unsigned acc = rows_pass<PACK, CSUM, NTM, U>(a, blockIdx.x * (tpb * U) + threadIdx.x, tpb);
    if constexpr (CSUM) block_sum_store(acc, csum);
}

// the row kernel applies: one run per block, every address and the window 16-B aligned, and
// slot / row counts in 32 bits
static bool rows_apply(const DdtDev &d, int nruns_host, int64_t run_disp, int64_t run_len, const void *mem,
                       const void *packed, int64_t pos, int64_t bytes)
{
    if (nruns_host != 1 || (run_len & 15) || run_len == 0) return false;
    if (((uintptr_t)mem + (uint64_t)run_disp) & 15) return false;
    if ((d.stride & 15) || (d.extent & 15) || ((uintptr_t)packed & 15) || (pos & 15) || (bytes & 15)) return false;
    const int64_t last_slot = (pos + bytes) >> 4;
    const int64_t rows = last_slot / (run_len >> 4) + 1;
    return last_slot < ((int64_t)1 << 32) && rows < ((int64_t)1 << 32) && d.nblk < ((int64_t)1 << 32) &&
           (run_len >> 4) < ((int64_t)1 << 32);
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
    case 2: hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, NTM, 2>), dim3(blocks), dim3(tpb), 0, s, a, part); break;
    case 8: hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, NTM, 8>), dim3(blocks), dim3(tpb), 0, s, a, part); break;
    default: hipLaunchKernelGGL((k_ddt_rows<PACK, CSUM, NTM, 4>), dim3(blocks), dim3(tpb), 0, s, a, part); break;
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

int launch_ddt_rows(const DdtDev &d, int nruns_host, int64_t run_disp, int64_t run_len, bool pack, void *mem,
                    void *packed, int64_t pos, int64_t bytes, unsigned *csum, hipStream_t s)
{
    if (!rows_apply(d, nruns_host, run_disp, run_len, mem, packed, pos, bytes)) return 1;
    RowArgs a;
    a.mem = static_cast<char *>(mem);
    a.packed = static_cast<char *>(packed);
    a.disp = run_disp;
    a.stride = d.stride;
    a.extent = d.extent;
    a.per_row = make_fastdiv((uint32_t)(run_len >> 4));
    a.per_inst = make_fastdiv((uint32_t)d.nblk);
    a.first = (uint32_t)(pos >> 4);
    a.nslots = (uint32_t)(bytes >> 4);
    const DdtTune &t = ddt_tune();
    int unroll = pack ? t.unroll_pack : t.unroll_unpack;
    if (unroll != 2 && unroll != 8) unroll = 4;
    const unsigned tpb = (t.threads == 256 || t.threads == 512) ? (unsigned)t.threads : 1024u;
    int ntm = t.nontemporal;
    if (ntm < 0) ntm = (2 * bytes > ((int64_t)256 << 20)) ? kDdtAutoNT : 0;  // streaming sizes
    const uint64_t per = (uint64_t)tpb * (uint64_t)unroll;
    const unsigned blocks = (unsigned)((a.nslots + per - 1) / per);
    Csum part;
    int rc = part.get(csum, blocks);
    if (rc) return rc;
    if (pack) {
        if (csum) launch_rows<true, true>(a, ntm, unroll, tpb, blocks, part.sink, s);
        else launch_rows<true, false>(a, ntm, unroll, tpb, blocks, part.sink, s);
    } else {
        if (csum) launch_rows<false, true>(a, ntm, unroll, tpb, blocks, part.sink, s);
        else launch_rows<false, false>(a, ntm, unroll, tpb, blocks, part.sink, s);
    }
    MI_HIP(hipGetLastError());
    return part.finish(csum, s);
}

int launch_ddt(const DdtDev &d, bool pack, void *mem, void *packed, int64_t pos, int64_t bytes, unsigned *csum,
               hipStream_t s)
{
    if (bytes <= 0) return MI355X_SUCCESS;
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
