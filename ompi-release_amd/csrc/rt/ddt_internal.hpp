// ddt_internal.hpp -- device view of a datatype layout (see ddt_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

struct mi355x_ddt;

namespace mi355x {

// true when `count` instances occupy one gap-free byte range starting at base + *first (ddt.cpp)
bool ddt_contiguous(const mi355x_ddt *d, size_t count, int64_t *first);

struct DdtDev {
    const int64_t *disp;   // run displacement inside a block (device array)
    const int64_t *len;    // run length in bytes
    const int64_t *pfx;    // packed offset of the run inside a block
    const int64_t *pfx_host;  // the packed offsets and lengths in host memory
    const int64_t *len_host;
    int nruns;
    int64_t nblk, stride, extent;
    int64_t blk_bytes, inst_bytes;
    uint64_t run_bits;     // OR of every run's displacement and length (their common alignment)
    int64_t max_len;       // longest run
};

// launch shape of the row kernel: slots per lane (2, 4, 8) and the non-temporal mask
// (-1 auto: kDdtAutoNT above 256 MiB of traffic; else 1 = loads, 2 = stores)
constexpr int kDdtAutoNT = 3;
struct DdtTune {
    int unroll_pack = 4;
    int unroll_unpack = 2;
    int threads = 256;
    int nontemporal = -1;
    // mi355x_ddt_tune_rows: 2 row kernel any slot width + unit kernel (16-B packed slots over 8/4-B
    // aligned runs where the packed side allows), 3 the same with W-byte units only, 1 16-B rows
    // only, 0 neither
    int rows = 2;
};
DdtTune &ddt_tune();

// csum: NULL, or where the window's checksum goes (the launch is then waited for)
int launch_ddt(const DdtDev &d, bool pack, void *mem, void *packed, int64_t pos, int64_t bytes, unsigned *csum,
               hipStream_t s);
// the row kernel (one run per block, slots of the widest power-of-two width <= 16 B every
// address and length allows); returns 1 when it does not apply
int launch_ddt_rows(const DdtDev &d, int nruns_host, int64_t run_disp, int64_t run_len, bool pack, void *mem,
                    void *packed, int64_t pos, int64_t bytes, unsigned *csum, hipStream_t s);

} // namespace mi355x
