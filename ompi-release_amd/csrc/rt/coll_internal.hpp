// coll_internal.hpp -- kernel argument blocks and schedule types of the coll/mi355x engine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace mi355x {

constexpr int kMaxRanks = 64;   // ranks per communicator handled by the engine
constexpr int kFoldChunk = 8;   // ranks whose loads are issued together in k_fold
constexpr int kTreeMax = 16;    // register-program width of k_tree
constexpr int kTreeSteps = 64;

// k_fold: acc = x[order[0]]; acc = role_j ? op2(acc, x[order[j]]) : op2(x[order[j]], acc)
struct FoldArgs {
    const void *src[kMaxRanks];  // rank inputs, already offset to this launch's first element
    void *dst[kMaxRanks];        // destinations, same offset
    int order[kMaxRanks];        // fold order (rank indices into src)
    uint64_t role_mask;          // bit j set: step j keeps the accumulator as the `out` operand
    int nr;                      // ranks folded
    int nd;                      // destinations written
    size_t n;                    // elements
    size_t head, nvec;           // filled by the launcher
};

struct TreeStep {
    int8_t dst, out, in;         // R[dst] = op2(out = R[out], in = R[in])
};

// k_tree: register program over nr <= kTreeMax rank inputs
struct TreeArgs {
    const void *src[kTreeMax];
    void *dst[kMaxRanks];
    TreeStep steps[kTreeSteps];
    int nsteps, nr, nd, result;
    size_t n;
};

// k_copy: bytes from one source to nd destinations
struct CopyArgs {
    const void *src;
    void *dst[kMaxRanks];
    int nd;
    size_t n, head, nvec;        // n in bytes
};

// k_multicopy: nseg independent byte segments copied concurrently by one launch (the pull side of
// allgather / the distribution phase of allreduce: one segment per peer, so every xGMI link is
// busy at once).  Blocks are dealt to segments in proportion to their length.
constexpr int kMaxSegs = kMaxRanks;
struct MultiCopyArgs {
    const void *src[kMaxSegs];
    void *dst[kMaxSegs];
    size_t len[kMaxSegs];
    unsigned first_block[kMaxSegs + 1];  // segment s owns blocks [first_block[s], first_block[s+1])
    int nseg;
};

struct CollTune {
    int blocks_per_cu = 4;
    int push = 0;   // 1: allreduce owners write into the peers' rbufs (one phase); 0: pull (two phases)
};
CollTune &coll_tune();

int launch_fold_slot(int op, int type, const FoldArgs &a, hipStream_t s);
int launch_tree_slot(int op, int type, const TreeArgs &a, hipStream_t s);
int launch_copy(CopyArgs a, hipStream_t s);
int launch_multicopy(MultiCopyArgs a, hipStream_t s);

} // namespace mi355x
