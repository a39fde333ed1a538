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

// k_ring_all: the ring allreduce's per-element order over the WHOLE vector in one launch -- element
// i of ring block b folds x_b, x_{b+1}, ..., x_{b+n-1} with the partial as the `in` operand
// (coll_tuned_allreduce.c:470-512); block b = the reference partition (coll_tuned.h:546-552)
struct RingAllArgs {
    const void *src[kMaxRanks];  // every rank's input (vector base)
    void *dst;                   // my rbuf
    int n;
    uint32_t count, early, late, split;  // elements; the first `split` blocks hold `early` elements
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

// Low-latency one-shot path (coll_ll.hip) for small messages (communicators of <= 8 ranks):
// every rank pushes its data into slot (parity, me) of every peer's uncached LL region over xGMI
// as 8-byte granules {4 B payload, 4 B call tag} -- one store each, so the tag vouches for the
// payload and no fence or separate flag is needed -- and the receivers poll their own slots for
// the tag.  Parity double-buffering + a per-call acknowledgement (written by the last block of
// every rank into every peer) make back-to-back calls safe.  No host barrier, no per-call IPC
// exchange.
constexpr size_t kLLChunk = 4096;  // payload bytes per thread block (256 threads x 16 B)
constexpr int kLLMaxRanks = 8;     // sources held in registers per thread
enum { LL_AR = 0, LL_AG = 1, LL_BC = 2, LL_RED = 3,     // allreduce, allgather, bcast, reduce
       LL_PULL = 4,    // (resident service only) one-phase allreduce pulled from the peers' mapped inputs,
       LL_PULL_AG = 5, // allgather and
       LL_PULL_BC = 6, // bcast copied from them,
       LL_PULL_RS = 7 };  // reduce_scatter(_block): this rank's block evaluated from them
enum { LL_FOLD = 0, LL_RING = 1, LL_TREE = 2 };   // per-element program of LL_AR
struct LLArgs {
    const void *src;                   // this rank's data (NULL: nothing to push)
    void *dst;                         // result (rbuf / buf)
    uint64_t *peer_data[kMaxRanks];    // granules of slot (parity, me) in peer q's LL region
    uint64_t *peer_ack[kMaxRanks];     // ack word `me` in peer q's LL region
    const uint64_t *my_data;           // this rank's slots of this parity (slot q at q * slot_gran)
    const uint64_t *my_ack;            // this rank's ack words (word q written by rank q)
    uint64_t *ctr;                     // blocks done, monotonic (device memory)
    uint64_t ctr_target;               // its value once this call's last block is done
    uint32_t *err;                     // host-visible error word (timeout)
    uint64_t push_mask, recv_mask;     // bit q: push to / receive from rank q
    uint64_t seq, slot_gran, nbytes, timeout_ticks;
    uint64_t count, early, late, split;  // elements; ring block partition (coll_tuned.h:546-552)
    uint64_t role_mask;
    int mode, prog, n, me, root, nsteps, result;
    int order[kMaxRanks];
    TreeStep steps[kTreeSteps];
};
int launch_ll_slot(int op, int type, const LLArgs &a, hipStream_t s);  // LL_AR / LL_RED
int launch_ll_copy(const LLArgs &a, hipStream_t s);                   // LL_AG / LL_BC
constexpr size_t kLLAckBytes = 4096;  // LL region: [ack words][2 parities x n slots of granules]

// Resident LL service (coll_svc.hip, svc_queue.cpp): the LL protocol run by a kernel that stays
// resident between calls on a private HSA queue and waits on a doorbell, so a small collective
// costs a host store and a device poll instead of a launch and a completion wait.  The host
// writes the call into the doorbell page (fine-grained device memory, stored through the BAR),
// then the call's number into `door`; every workgroup of the service polls `door`, serves the call
// (chunks wg, wg + nwg, ...), publishes its results and counts itself done; the last one
// acknowledges the call to every peer and stores its number into the host's completion word.
constexpr uint64_t kSvcQuit = ~0ull;  // door value that ends the service
constexpr int kSvcPartBits = 7;       // door = (call number << 7) | workgroups the call needs (<= 64)
constexpr int kSvcThreads = 256;      // threads per workgroup (16 B each: one LL slice per pass)
struct SvcCall {
    uint64_t seq;                     // the call's number (= its LL tag), written with the call
    const void *src;
    void *dst;
    uint64_t nbytes, count, early, late, split, role_mask, push_mask, recv_mask;
    int32_t op, type, mode, prog, root, nsteps, result, pad;
    int32_t order[kLLMaxRanks];
    TreeStep steps[kTreeSteps];
    const void *srcs[kLLMaxRanks];    // LL_PULL: every rank's input, mapped (16-B aligned)
};
// LL_PULL: rank q tells every peer it has read the peer's input for call k by storing k into word
// kSvcPullDoneWord + q of the peer's LL acknowledgement page
constexpr int kSvcPullDoneWord = 256;
struct SvcPage {                      // the doorbell page
    uint64_t door;                    // (number << kSvcPartBits) | participants of the posted call;
                                      // kSvcQuit: leave
    uint64_t pad0[15];
    uint64_t ctr;                     // workgroups done, zeroed by the host before every launch
    uint64_t pad1[15];
    uint64_t go;                      // workgroup 0's verdict on call `want`: want = serve it, kSvcQuit =
                                      // leave (zeroed by the host before every launch)
    uint64_t pad2[15];
    uint64_t shrink;                  // set by workgroup 0 once idle for shrink_ticks: the other
                                      // workgroups leave (zeroed by the host before every launch)
    uint64_t pad3[15];
    SvcCall call;
};
// a shrunk service (workgroup 0 alone) serves calls of up to this many 4-KiB slices by itself (the
// LL form: 32 KiB); a call that wants more workgroups makes the host relaunch the full grid
constexpr uint64_t kSvcShrunkMaxPart = 8;
struct SvcArgs {                      // fixed for one launch
    const SvcPage *page;
    uint64_t *done;                   // host word: number of the last call completed
    uint32_t *err;                    // host word: set on a timeout waiting for a peer
    char *my_ll;                      // my LL region
    char *peer_ll[kLLMaxRanks];       // every rank's LL region, mapped
    uint64_t first;                   // the call number this launch serves first
    uint64_t slot_gran, idle_ticks, timeout_ticks;
    uint64_t shrink_ticks;            // idle time after which the other workgroups leave (0: never)
    uint64_t *shrunk;                 // host word: set when they have been told to
    int32_t n, me, nwg, probe;        // probe: return at once (loads the code object)
    uint64_t *trace;                  // NULL, or kSvcTraceCalls rows of kSvcTraceCols words (MI355X_SVC_TRACE)
};
// MI355X_SVC_TRACE=1: workgroup 0 stamps s_memrealtime (100 MHz) at each stage of a call (in LDS;
// the row is written to device memory once the call is complete) into row
// seq % kSvcTraceCalls: seq, door seen, descriptor in LDS, slices pushed, peers' slices received,
// results stored, completion stored, evaluated; the granule forms also: the first slice's results
// issued, the workgroup joined after it
constexpr int kSvcTraceCalls = 1024, kSvcTraceCols = 12;

// Pipelined allreduce (coll_pipe.hip): fold of my ring block and pulls of the peers' blocks in
// one launch, chunk by chunk, with per-chunk ready flags (uncached region, written by the
// producer into every peer over xGMI) and a device work queue.
struct PipeArgs {
    const void *src[kMaxRanks];        // every rank's input, mapped (vector base)
    const char *peer_rbuf[kMaxRanks];  // every rank's rbuf, mapped (vector base)
    char *dst;                         // my rbuf
    uint64_t *peer_flag[kMaxRanks];    // row `me` of peer q's flag region (q != me)
    const uint64_t *my_flag;           // my flag region: row q = flags raised by rank q
    uint64_t *queue;                   // work-queue counter (device memory, monotonic)
    uint32_t *err;                     // host-visible error word (timeout)
    uint64_t qbase, seq, timeout_ticks, kmax, chunk, count;
    uint64_t boff[kMaxRanks], blen[kMaxRanks];  // ring block partition (elements)
    uint64_t role_mask;                // my block's fold program (ring_block_program)
    uint64_t co_pull;                  // bit q: peer q's rbuf and mine share alignment mod 16
    int order[kMaxRanks];
    int n, me, co_fold;                // co_fold: every input and dst share alignment mod 16
    int wt;                            // publish write-through (sc0 sc1), no per-chunk fences
    uint32_t nchunks;                  // chunks per block (the longest block)
    uint64_t *dbg;                     // NULL, or 4 words per workgroup: item, stage, flag seen, polls
};
int launch_pipe_slot(int op, int type, const PipeArgs &a, unsigned grid, hipStream_t s);
// workgroups of the pipelined kernel for (op, type, count) one CU can hold at once: ranks sharing a
// GPU must fit their persistent grids side by side (a rank's pulls spin until a peer's folds run)
int pipe_blocks_per_cu(int op, int type, size_t count);

struct CollTune {
    // grid cap of k_fold / k_copy / k_multicopy in blocks per CU; 1024 = one-shot grids (every
    // thread one pass), measured fastest for 1 GiB allreduce (one-GPU rehearsal: 0.94 ms vs 1.16 ms
    // at 2 blocks per CU, profiles/r01_bench_n2_rehearsal_1gpu.json); the N > 1 bench re-tunes it
    int blocks_per_cu = 1024;
    // k_multicopy: KiB per block before the grid cap applies; 4 measured best (tools/ab_copy.py:
    // 1 GiB pull 0.35 ms vs 0.39 at 16 KiB, 0.41 at 64 KiB, one GPU)
    int copy_block_kib = 4;
    // 1: allreduce owners write into the peers' rbufs (one phase); 0: pull (two phases, default).
    // Push is correct on one device only: across xGMI a remote write lands in HBM behind the
    // owner's L2, which may still hold old lines of the destination (coarse-grained memory is not
    // probed), so the owner could read stale data afterwards.
    int push = 0;
    // pipelined allreduce: workgroups (256 threads) per CU of its persistent grid, split among the
    // ranks sharing a GPU; chunk size in KiB (0: ~512 chunks per ring block, >= 64 KiB)
    int pipe_wg_per_cu = 2;
    int pipe_chunk_kib = 0;
    // pipelined allreduce: publish chunks write-through instead of L2 write-back + invalidate fences
    // (faster at every n measured: rehearsal n = 8 3.50-3.78 vs 4.69 ms, n = 4 2.03 vs 2.29)
    int pipe_wt = 1;
};
CollTune &coll_tune();          // the calling engine call's communicator's (else the process defaults)
CollTune &coll_tune_default();  // the process defaults new communicators start from
CollTune *coll_tune_use(CollTune *t);  // install t for this thread; returns the previous one

int launch_fold_slot(int op, int type, const FoldArgs &a, hipStream_t s);
int launch_ring_all_slot(int op, int type, const RingAllArgs &a, hipStream_t s);
int launch_tree_slot(int op, int type, const TreeArgs &a, hipStream_t s);
int launch_copy(CopyArgs a, hipStream_t s);
int launch_multicopy(MultiCopyArgs a, hipStream_t s);

} // namespace mi355x
