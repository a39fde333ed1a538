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

template <bool PACK, bool CSUM>
__global__ __launch_bounds__(256) void k_ddt(DdtDev d, char *mem, char *packed, int64_t pos, int64_t bytes,
                                             unsigned *csum)
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
    if constexpr (CSUM) {
        // wave reduction then one atomic per wave (sum mod 2^32)
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(csum, acc);
    }
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
    if (pack) {
        if (csum) hipLaunchKernelGGL((k_ddt<true, true>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, csum);
        else hipLaunchKernelGGL((k_ddt<true, false>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, csum);
    } else {
        if (csum) hipLaunchKernelGGL((k_ddt<false, true>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, csum);
        else hipLaunchKernelGGL((k_ddt<false, false>), dim3((unsigned)blocks), dim3(256), 0, s, d, m, pk, pos, bytes, csum);
    }
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

} // namespace mi355x
