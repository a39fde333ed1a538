// comm_internal.hpp -- state shared by the engine's translation units (coll_comm.cpp: bootstrap,
// registration cache, collectives; p2p.cpp: device point-to-point).  Not part of the C ABI.
#pragma once

#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "coll_internal.hpp"
#include "coll_sched.hpp"
#include "rt_internal.hpp"
#include "svc_queue.hpp"

namespace mi355x {

// MI355X_DEBUG=1: trace every stage of a collective on stderr (rank, stage, elapsed time)
inline bool debug_on()
{
    static const bool on = getenv("MI355X_DEBUG") && atoi(getenv("MI355X_DEBUG")) > 0;
    return on;
}
#define TRACE(c, ...)                                                                          \
    do {                                                                                       \
        if (debug_on()) {                                                                      \
            fprintf(stderr, "[mi355x r%d seq %llu] ", (c)->rank, (unsigned long long)(c)->seq); \
            fprintf(stderr, __VA_ARGS__);                                                      \
            fputc('\n', stderr);                                                               \
        }                                                                                      \
    } while (0)

constexpr uint64_t kMagic = 0x4d49333535584331ull;  // "MI355XC1"
constexpr int kMaxBufs = 3;
// every wait's bound unless MI355X_TIMEOUT_S / the TIMEOUT_S knob says otherwise: one day.  MPI's
// waits are unbounded -- a rank late by minutes or hours (checkpoint I/O) is not an error -- and a
// dead peer is found by its pid and start time (peer_gone), not by a timeout; the bound only turns a
// hang into an error eventually (tests set seconds)
constexpr double kDefaultTimeoutS = 86400.0;
constexpr int kVoteRing = 64;    // buffer-kind votes a rank keeps (mi355x_comm_vote)
constexpr int kVoteWindow = 32;  // calls per vote window: every rank waits at each window's last call

struct BufDesc {
    hipIpcMemHandle_t h;
    uint64_t off;
    uint64_t raw;      // loopback: the pointer itself
    uint64_t present;  // 0: NULL buffer
    uint64_t base;     // exporter's allocation base (its VA; the peer-map key)
    uint64_t id;       // exporter's allocation id (HIP_POINTER_ATTRIBUTE_BUFFER_ID)
    uint64_t staged;   // 1: the dmabuf route (>= ipc_max, or a bounded cache) or the staged flow;
                       // 2: not exportable at all this call: the staged flow
    uint64_t size;     // dmabuf: the exported allocation's size
    int32_t dmabuf;    // 1: exported as a dmabuf fd (fd is a descriptor of the exporter process)
    int32_t fd;
};

struct alignas(64) RankSlot {
    std::atomic<uint64_t> seq;
    int32_t pid, dev, nbuf;
    int32_t retiring;             // this rank holds retired peer mappings to close in the call's close window
    std::atomic<uint64_t> map_state;  // exchange: (call << 2) | 1 opens done, 2 an open failed, 3 closed (coll_ctl.cpp)
    std::atomic<uint32_t> opening;    // a barrier's progress pass that may open peer mappings runs (barrier_progress)
    std::atomic<uint32_t> closing;    // this rank closes retired peer mappings (close_window)
    uint64_t sig[4];
    BufDesc buf[kMaxBufs];
    int32_t probe_fd, probe_ok;   // dmabuf capability probe
    uint64_t probe_size;
    int64_t varg[2 * kMaxRanks];  // per-peer counts / displacements of v-collectives (bytes)
    int32_t ll_ok, pad_ll;        // LL self-test result at creation (1 ok, 2 failed)
    int32_t svc_claim, svc_ok;    // resident LL service at creation: this process's service is mine
                                  // (1) or taken (2); its self-test passed (1) or failed (2)
    uint64_t dev_uid;             // hash of the device's PCI bus id: ranks sharing one GPU
    uint64_t pid_start;           // the process's start time (/proc/<pid>/stat field 22): a recycled pid differs
    uint64_t pid_ns;              // inode of its PID namespace: a pid from another namespace is not checked
    // mi355x_comm_vote: call v's entry at [v % kVoteRing] = (v << 2) | (window flag << 1) | (this
    // rank's buffers are device memory); a ring because one side of a call publishes and moves on.
    // The window flag (checkpoint calls only): this rank voted device somewhere in the window
    std::atomic<uint64_t> vote[kVoteRing];
    // pipelined allreduce admission for the call whose exchange carries sequence s:
    // (s << 1) | (this rank holds its GPU's pipelined-grid token)
    std::atomic<uint64_t> pipe_adm;
    // finish(): the number of finish points this rank's stream has passed, written by the GPU's
    // command processor behind the rank's kernels (hipStreamWriteValue64 into the host-registered
    // control segment); every rank polls every rank's word instead of a stream sync + barrier
    alignas(64) std::atomic<uint64_t> done;
    // the call gate (coll_comm.cpp, CallGate): 0 between calls, 1 inside an engine collective, 2
    // held by a process that is taking the resident service away from this communicator (it may do
    // so only while every rank is between the same two calls); calls = gated calls completed
    alignas(64) std::atomic<uint32_t> gate;
    uint32_t flow_ok;                 // flow self-test: the MI355X_FLOW_* this rank saw exact
    std::atomic<uint64_t> verdict;    // device setup: hash of the flow verdicts this process holds for
                                      // the communicator's member set (0: none), agreed before reuse
    std::atomic<uint64_t> calls;
    std::atomic<uint64_t> svc_last_ns;  // CLOCK_MONOTONIC time of this rank's last service call
};

struct Ctrl {
    uint64_t magic;
    uint32_t size;
    uint32_t pad0;
    // random bits rank 0 draws at creation: part of the fd-passing sockets' names, so only a
    // process that can read this 0600 segment (the job's user) can compute them -- the segment's
    // name alone (visible in /dev/shm) does not give them away
    uint64_t secret;
    alignas(64) std::atomic<uint32_t> attached;
    alignas(64) std::atomic<uint64_t> bar_count;
    alignas(64) std::atomic<uint64_t> bar_gen;
    alignas(64) std::atomic<uint32_t> abort_flag;
    // the service epoch (claim number) another process took the resident service away at: every
    // rank lets go of it at its next call (CallGate)
    alignas(64) std::atomic<uint64_t> svc_revoked;
    alignas(64) RankSlot slot[1];
};

// Point-to-point mailboxes (p2p.cpp) follow the rank slots: for every ordered pair (src, dst) a
// ring of kP2PSlots envelopes that src fills and dst drains (the ob1 match/RGET header plus the
// FIN the receiver returns, pml_ob1_hdr.h:58-190, carried in shared memory as btl/smcuda's FIFOs
// carry them, btl_smcuda_fifo.h).
constexpr int kP2PSlots = 32;
constexpr size_t kP2PInline = 128;  // payloads up to this size travel inside the envelope (p2p.cpp)
struct alignas(64) Envelope {
    std::atomic<uint64_t> full;   // message number + 1 once posted (sender, release)
    std::atomic<uint64_t> done;   // message number + 1 once the receiver no longer reads it
    int32_t tag, flags;           // flags: kEnvPacked, kEnvHost (p2p.cpp)
    uint64_t bytes;               // packed size of the message
    union {
        BufDesc buf;              // where the (packed) bytes are: the sender's device export, or
                                  // (kEnvHost) its host arena: id = segment generation, off = offset
        unsigned char inl[sizeof(BufDesc)];  // (kEnvInline) the payload itself, <= kP2PInline bytes
    };
    // (kEnvDual: a small device payload offered two ways) the sender's host copy in its arena --
    // generation and offset -- and who reads the payload, as ((message number + 1) << 2) | state
    // (p2p.cpp, claim_word): state 0 undecided, 1 the host copy is complete and the receiver reads
    // it (set by the sender, whose send then completes), 2 the receiver pulls from the sender's
    // device buffer (set by the receiver; the sender waits for the FIN).  The message number makes
    // a late compare-and-swap about an earlier message of the slot fail once the slot is reused.
    uint64_t hoff;
    uint32_t hgen, pad;
    std::atomic<uint64_t> claim;
};
inline size_t p2p_offset(int size)
{
    return (sizeof(Ctrl) + sizeof(RankSlot) * (size_t)(size - 1) + 4095) & ~(size_t)4095;
}
inline size_t ctrl_bytes(int size)
{
    return p2p_offset(size) + sizeof(Envelope) * (size_t)kP2PSlots * (size_t)size * (size_t)size;
}
inline Envelope *p2p_ring(Ctrl *k, int size, int src, int dst)
{
    return (Envelope *)((char *)k + p2p_offset(size)) + ((size_t)src * (size_t)size + (size_t)dst) * kP2PSlots;
}

// A peer allocation is keyed by (peer, its base VA) and remembered with its allocation id: when
// the exporter frees and reallocates at the same address the id changes and the stale mapping
// is closed and replaced (the invalidation mpool/rgpusm does on a buffer-id mismatch,
// ompi/mca/mpool/rgpusm/mpool_rgpusm_module.c:243-281, common_cuda.c:1709-1745).
struct HandleKey {
    int peer;
    uint64_t base;
    bool operator<(const HandleKey &o) const
    {
        if (peer != o.peer) return peer < o.peer;
        return base < o.base;
    }
};

struct PeerMap {
    uint64_t id;
    void *mapped;
    uint64_t last_use;             // LRU stamp (use_clock) of the last collective or point-to-point use
    hipExternalMemory_t ext;       // dmabuf import (NULL: hipIpcOpenMemHandle mapping)
    uint64_t coll_use = ~0ull;     // collective (seq) that last used it (~0: point-to-point only)
    int pins = 0;                  // in-flight point-to-point reads: never closed meanwhile
    bool persistent = false;       // a region the engine keeps mapped for the communicator's
                                   // life (LL and pipeline flag regions): never dropped
    size_t bytes = 0;              // the exporter's allocation size (the rcache byte limit)
};

inline void close_map(PeerMap &m)
{
    if (m.ext) {
        (void)hipFree(m.mapped);
        (void)hipDestroyExternalMemory(m.ext);
    } else {
        (void)hipIpcCloseMemHandle(m.mapped);
    }
}

struct LocalReg {
    uintptr_t base;
    size_t size;
    uint64_t id;
    hipIpcMemHandle_t h;
    bool has_h;       // false: too large for hipIpc* (never passed to hipIpcGetMemHandle)
    int fd;           // dmabuf export of a large allocation (-1: none yet)
    uint64_t sent;    // bit q: the dmabuf fd went to rank q (SCM_RIGHTS, once per peer)
};

inline void drop_reg(LocalReg &r)
{
    if (r.fd >= 0) close(r.fd);
    r.fd = -1;
}

struct LoopShared {
    Ctrl *ctrl = nullptr;
    int refs = 0;
    std::mutex mtx;
};

struct P2P;  // point-to-point state of a communicator (p2p.cpp)

} // namespace mi355x

struct mi355x_request {
    std::atomic<int> done{0};
    int rc = MI355X_SUCCESS;
    std::string err;
    std::function<int(hipStream_t)> run;  // the blocking algorithm, on the progress stream
    hipEvent_t ev = nullptr;              // the caller-stream point the call starts after
    // point-to-point requests (p2p.cpp) complete from mi355x_p2p_progress, not from a thread
    int kind = 0;                         // 0 collective, 1 send, 2 receive
    mi355x_comm *comm = nullptr;
    int peer = 0, tag = 0;
    const mi355x_ddt_t *ddt = nullptr;    // NULL: `count` contiguous bytes
    size_t count = 0;
    void *buf = nullptr;
    size_t bytes = 0;                     // packed bytes: of the message (send), of the buffer (receive)
    uint64_t msg = 0;                     // send: message number to `peer`
    mi355x::BufDesc desc;                 // send: the export announced in the envelope
    mi355x::Envelope *env = nullptr;      // the envelope in flight
    void *packed = nullptr;               // send: copy in the device arena (packed layout / buffered)
    mi355x::PeerMap *pin = nullptr;       // receive: the pinned mapping being read
    void *hpin = nullptr;                 // receive: the peer host-arena segment a copy kernel reads (p2p.cpp)
    int st_source = 0, st_tag = 0, st_error = 0;
    size_t st_bytes = 0;
    int mode = 4;                         // send mode (MI355X_SEND_*; 4 standard)
    bool host = false;                    // the caller's buffer is host memory
    bool internal = false;                // send owned by the engine: the caller's request completed
                                          // when the payload was copied (eager / buffered)
    bool cancelled = false;               // receive cancelled before it matched
    int32_t env_flags = 0;                // send: kEnvPacked / kEnvHost (p2p.cpp)
    void *hslot = nullptr;                // send: payload slot in the host shared-memory arena
    mi355x_request *twin = nullptr;       // send (kEnvDual): the caller's request, completed once the
                                          // payload is safe (host copy taken) or delivered (FIN)
    bool copy_done = false;               // send (kEnvDual): the host copy's kernel has finished
    bool copy_launched = false;           // send (kEnvDual): ... has been launched
    double dual_t0 = 0;                   // send (kEnvDual): when it was posted (steady clock, s)
    const void *dual_src = nullptr;       // send (kEnvDual): the caller's device bytes
    uint64_t hoff = 0;                    // send (kEnvDual): the host copy's arena offset and generation
    uint32_t hgen = 0;
    mi355x::BufDesc hdesc{};              // send (kEnvDual): the host copy's slot as a host-arena send names it
    void *stage = nullptr;                // receive: device staging slot (host destination)
    std::vector<char> htmp;               // receive: host copy awaiting the host convertor
    unsigned char inl[mi355x::kP2PInline]; // send: an inline payload until its envelope is posted
};

struct mi355x_comm {
    int rank = 0, size = 1, device = 0;
    mi355x::Ctrl *ctrl = nullptr;
    bool loopback = false;
    std::shared_ptr<mi355x::LoopShared> loop;
    std::string shm_name;
    uint64_t seq = 0;
    uint64_t vote_seq = 0;                        // mi355x_comm_vote calls made
    bool vote_host_waits = true;                  // this window's mode: host ranks wait (else device ranks)
    bool vote_window_dev = false;                 // this rank voted device in the current window
    std::map<mi355x::HandleKey, mi355x::PeerMap> peer_maps;
    // mappings evicted during a call's mapping phase: closed in the next exchange's close window,
    // never while a peer exports or imports (coll_rcache.cpp: retire_map)
    std::vector<mi355x::PeerMap> retired_maps;
    hipStream_t call_s = nullptr;     // the stream of the collective in progress (CallStream): setup work uses it
    int call_depth = 0;               // collectives in progress on this thread of control (call_s valid when > 0)
    bool export_check = true;         // verify each new dmabuf export of the bounded cache (MI355X_EXPORT_CHECK=0: off)
    uint64_t export_mismatches = 0;   // exports that named another buffer object
    // peer-mapping cache bounds (MI355X_RCACHE_MAX_MAPS / MI355X_RCACHE_SIZE_LIMIT, knobs of the same
    // names; 0 = unlimited, the default, as mpool_rgpusm_rcache_size_limit): LRU eviction
    size_t rcache_max_maps = 0, rcache_limit = 0;
    uint64_t rcache_evictions = 0;
    std::vector<mi355x::LocalReg> local_regs;
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    int dmabuf_state = 0;                         // large allocations via dmabuf: 0 unknown, 1 yes, -1 no
    // dmabuf fds travel between ranks as SCM_RIGHTS ancillary data over one AF_UNIX datagram
    // socket per rank (abstract name derived from the control segment's name); received fds wait
    // here, keyed by (exporting rank, allocation id), until a mapping needs them
    int fd_sock = -1;
    std::map<std::pair<int, uint64_t>, int> fd_stash;
    void *stage = nullptr;                        // staging buffer of the staged data flow
    size_t stage_bytes = (size_t)1 << 30;         // its size (an allocation below ipc_max)
    size_t ipc_max = (size_t)1 << 31;             // allocations >= this are never exported
    // low-latency path (coll_ll.hip): uncached LL region [ack words][2 x n slots of 8-B granules]
    // per-rank message bytes served by the LL path: 0 by default (MI355X_LL_MAX_BYTES) -- on the
    // one-GPU rehearsal it does not beat the host-synchronised path (profiles/r02_ll_probe.txt);
    // the 8-GPU bench legs measure both
    size_t ll_max = 0;
    bool ll_ok = false;                           // creation-time LL self-test passed on every rank
    char *ll_base = nullptr;
    size_t ll_slot = 0;                           // payload bytes per slot
    std::vector<char *> ll_peer;                  // every rank's LL region, mapped
    uint64_t ll_seq = 0;
    uint64_t *ll_ctr = nullptr;                   // blocks done (device), monotonic
    uint64_t ll_ctr_base = 0;                     // its value before the next call
    uint32_t *ll_err = nullptr;                   // host-visible timeout word
    // resident LL service (coll_svc.hip, svc_queue.cpp): small collectives up to svc_max bytes per
    // rank served by a kernel resident on a private HSA queue.  One service per process and GPU; the
    // communicator that finds it free on every rank at creation owns it (svc_ok), every other
    // communicator uses the per-call paths
    // MI355X_SVC_MAX_BYTES / MI355X_KNOB_SVC_MAX_BYTES: 32 KiB by default, where the service beat the
    // host-synchronised path at every size measured (one-GPU rehearsal, np = 2: 9.8-11.7 vs
    // 16.7-17.3 us up to 16 KiB, even at 64 KiB; np = 4: 15-17 vs 22-24 us up to 16 KiB, even at
    // 64 KiB; profiles/r03_svc_latency.jsonl)
    size_t svc_max = (size_t)32 << 10;
    bool svc_ok = false;
    bool svc_owner = false;                       // this process's service is claimed by this communicator
    mi355x::SvcQueue *svcq = nullptr;
    mi355x::SvcPage *svc_page = nullptr;          // doorbell page (host-writable; device address == host address)
    bool svc_page_dev = false;                    // the page is fine-grained device memory (else pinned host)
    uint64_t *svc_host = nullptr;                 // pinned host words: [0] call completed, [1] error word, [2] shrunk
    int svc_nwg = 16;                             // workgroups of the service (16 x 4 KiB slices per pass)
    // the service leaves after this long without a call (MI355X_SVC_IDLE_MS, default 1 ms): a burst
    // of small calls keeps it resident, a call after a longer gap relaunches it
    double svc_idle_s = 0.001;
    // ... and after this long without a call all its workgroups but the first leave
    // (MI355X_SVC_SHRINK_US, default 100 us; 0: never): between bursts the service holds one CU, and
    // serves the small calls alone; a call of more than kSvcShrunkMaxPart slices relaunches the grid
    double svc_shrink_s = 100e-6;
    uint64_t svc_calls = 0, svc_launches = 0, svc_regrows = 0;
    // one-phase ring-ordered allreduce above svc_max and up to svc_pull_max bytes per rank served by
    // the service from the peers' mapped inputs (LL_PULL; MI355X_SVC_PULL_MAX_BYTES); also the
    // largest block of a reduce_scatter(_block) the service evaluates (LL_PULL_RS, any size up to it)
    // (128 KiB by default: one-GPU rehearsal with 16 service workgroups, np = 2: 64 KiB 12.1 vs 17.4 us,
    // 128 KiB 15.2 vs 18.7, 256 KiB 22.1 vs 17.5; np = 4: 17.5 vs 25.9, 22.4 vs 23.7, 33.0 vs 22.9 --
    // the service's 16 workgroups are latency-bound where a one-shot launch has the whole GPU;
    // profiles/r03_svc_pull.log)
    size_t svc_pull_max = (size_t)128 << 10;
    // allgather / bcast above svc_max and up to svc_copy_max bytes per rank copied by the service
    // from the peers' mapped buffers (LL_PULL_AG / LL_PULL_BC; MI355X_SVC_PULL_COPY_MAX_BYTES)
    // (1 MiB by default: the copies are read-bound on every link at once, no fold, so the service's
    // workgroups keep up -- one-GPU rehearsal, allgather np = 2: 256 KiB 8.9 vs 16.1 us, 1 MiB 11.9 vs
    // 16.8; np = 4: 11.9 vs 20.7, 19.2 vs 23.1; bcast np = 2 512 KiB 8.8 vs 15.3;
    // profiles/r03_svc_pull_copy.log).  bcast of 1 MiB and more takes the scatter + allgather shape.
    size_t svc_copy_max = (size_t)1 << 20;
    // reduce_scatter(_block) through the service (LL_PULL_RS): on by default since round 4 (exact on
    // the GPU at 2 and 3 ranks; np = 2 10.2-16.1 vs 17.0-19.4 us, np = 4 12.5-21.1 vs 20.6-22.2 us for
    // the host-synchronised flow, profiles/r04_svc_rs_latency.jsonl); MI355X_SVC_RS=0 turns it off
    bool svc_rs = true;
    bool svc_keep = false;                        // this call's exchange leaves the service resident
    // ownership (coll_comm.cpp, svc_claim): claimed at a communicator's first service-sized call,
    // agreed by every rank in that call; handed over when another communicator of the process wants
    // the service and this one has been idle on every rank for svc_handover_s (svc_revoke)
    bool svc_want = false;                        // may claim (multi-process, <= 8 ranks, LL self-test ok)
    bool svc_attached = false;                    // counted among the users of the process's service resources
    bool svc_flows_tested = false;                // the service flows' self-test has run (first claim)
    int selftest_reused = 0;                      // MI355X_KNOB_SELFTEST_REUSED
    uint64_t svc_epoch = 0;                       // successful claims (same on every rank)
    uint64_t svc_tries = 0;                       // service-sized calls made without the service
    uint64_t svc_retry = 16;                      // a claim is attempted every svc_retry such calls
    uint64_t svc_revocations = 0;                 // times this communicator lost the service to another
    double svc_handover_s = 0.01;                 // MI355X_SVC_HANDOVER_MS: idle time before a handover
    // cross-device flows (MI355X_FLOW_*) this communicator may use, and those that failed their
    // self-test on some rank (creation: the pipelined flow; first claim: the service's flows)
    unsigned flows = 0x1f, flows_failed = 0;
    bool pipe_untested = false;                   // the pipelined flow's self-test was not admitted
    size_t pipe_chunk_override = 0;               // elements per chunk (the self-test's small chunks)
    bool gated = false;                           // multi-process: engine calls pass the call gate
    uint64_t gate_calls = 0;                      // gated calls completed (RankSlot::calls)
    size_t ll_bytes = 0;                          // LL region size (ll_resync)
    double create_us = 0, selftest_us = 0;
    void *gf_buf = nullptr;                       // gather-then-fold slots (coll_gfold.cpp): every rank's input
    size_t gf_bytes = 0;
    double gf_used = 0;                           // last gather-then-fold call (steady clock, s)
    mi355x::CollTune tune = mi355x::coll_tune_default();  // launch-shape knobs of this communicator's calls
    uint64_t use_clock = 0;                       // LRU clock of the peer-mapping cache (every use ticks it)
    // device-side setup (done words, LL region + self-test, the service's resources, the pipelined
    // flow's self-test), deferred from creation to the first device-buffer collective (dev_setup)
    bool dev_ready = false;
    bool selftest = true;                         // MI355X_KNOB_SELFTEST (env MI355X_SELFTEST)
    double setup_us = 0;
    std::vector<std::pair<int, long>> preset;     // knobs set before dev_setup, applied after it
    bool svc_stuck = false;                       // a service kernel never left (its memory is leaked, never reused)
    uint64_t *svc_trace = nullptr;                // MI355X_SVC_TRACE=1: stage stamps (device memory), printed at destroy
    // pipelined allreduce (coll_pipe.hip): per-chunk ready flags in an uncached region that
    // every peer writes into (row q = flags raised by rank q), and the work-queue counter
    char *pipe_base = nullptr;
    size_t pipe_kmax = 0;                         // flags per row (chunks per ring block, max)
    std::vector<char *> pipe_peer;                // every rank's flag region, mapped
    uint64_t *pipe_queue = nullptr;               // device work-queue counter (monotonic)
    uint64_t pipe_qbase = 0;                      // its value when the next launch starts
    uint64_t pipe_seq = 0;                        // calls of the pipelined flow so far
    int pipe_share = 1;                           // ranks of this communicator on my GPU (set at creation)
    // ring-ordered allreduce up to this many bytes per rank in one phase (k_ring_all); beyond it
    // the n-fold reads outweigh the host barrier + stream sync the second phase costs: a rank reads
    // (n-1) S over n-1 links instead of 2 (n-1) S / n, i.e. S (1 - 2/n) more per link, against
    // ~17 us saved (one-GPU rehearsal, n = 2: 64 KiB 18.4 vs 34.7 us, 1 MiB 18.6 vs 35.8 us) --
    // break-even near 1.7 MB at n = 8 with 76.8 GB/s per link and direction
    // (MI355X_KNOB_ONE_PHASE_MAX_BYTES, env MI355X_ONE_PHASE_MAX_BYTES)
    size_t one_phase_max = (size_t)1 << 20;
    bool pipe_on = false;                         // MI355X_KNOB_PIPE (env MI355X_PIPE; default: size >= 4)
    uint64_t pipe_holder = 0;                     // this communicator's id in the GPU token table
    int pipe_token = -1;                          // token table slot of my GPU (-1: not looked up)
    int pipe_entry = -1;                          // my registration in that token's holder list while held
    uint64_t pipe_refused = 0;                    // calls that fell back because a token was taken
    uint64_t pipe_calls = 0;                      // allreduces served by the pipelined flow
    // finish() by device-written completion words (see RankSlot::done): the control segment
    // registered with HIP (hipHostRegister) and its device address; 0 = stream sync + barrier
    // MI355X_LAT_PROFILE=1: host time of the small-message allreduce's steps (entry -> input sync
    // -> exchange -> launch -> finish), averaged and printed at destroy
    std::mutex prog_mtx;                          // compiled size-only programs (recursive doubling,
    std::map<int, mi355x::Program> prog_cache;    // linear), keyed by the coll/tuned algorithm id
    bool lat_on = false;
    double lat_acc[4] = {0, 0, 0, 0};
    uint64_t lat_n = 0;
    char *ctrl_dev = nullptr;
    bool ctrl_registered = false;
    uint64_t done_seq = 0;
    uint64_t *pipe_dbg = nullptr;                 // MI355X_DEBUG: per-workgroup progress words
    // nonblocking collectives: one progress thread per communicator runs the posted calls in
    // order on its own stream; blocking calls first wait until nothing is pending
    std::thread worker;
    std::mutex q_mtx;
    std::condition_variable q_cv;
    std::deque<mi355x_request *> queue;
    bool stop = false;
    int pending = 0;                              // posted, not finished (guarded by q_mtx)
    hipStream_t nb_stream = nullptr;
    int knob_allreduce = 0, knob_reduce = 0, knob_rs = 0;
    int chain_fanout = mi355x::kDefaultChainFanout;
    const mi355x_rules_t *rules = nullptr;        // coll/tuned dynamic rules (not owned)
    int last_alg = -1;
    double timeout_s = mi355x::kDefaultTimeoutS;
    bool time_phases = false;                     // MI355X_KNOB_TIME_PHASES
    hipEvent_t tev[4] = {nullptr, nullptr, nullptr, nullptr};
    float phase_ms[2] = {-1.f, -1.f};
    mi355x::P2P *p2p = nullptr;                   // created on first point-to-point call
    std::recursive_mutex reg_mtx;                 // registration cache: collectives (progress
                                                  // thread) and point-to-point (caller) share it
};

namespace mi355x {
// shared by coll_comm.cpp and p2p.cpp
int barrier(mi355x_comm *c);
int local_handle(mi355x_comm *c, const void *p, BufDesc *d, bool force);
// export the large allocation of `d` as a dmabuf fd and pass it to every rank in `peers` that
// has not received it yet
int export_dmabuf(mi355x_comm *c, BufDesc *d, uint64_t peers);
int fd_drain(mi355x_comm *c, bool wait);  // receive queued dmabuf fds, serve fd requests (caller holds reg_mtx)
// map_peer's "retry after a close window" (an open failed and stale mappings were retired)
constexpr int kOpenRetry = 1;
int map_peer(mi355x_comm *c, int peer, const BufDesc &d, void **out, PeerMap **entry = nullptr, bool coll = true);
size_t peer_map_count(const mi355x_comm *c);  // evictable-kind peer mappings currently open
// publish nbuf buffers, meet every rank, map every rank's buffers: peers[b][r] (coll_comm.cpp)
// persistent: the mappings stay for the communicator's life (never dropped to make room)
int exchange(mi355x_comm *c, int nbuf, const void *const *mine, const uint64_t sig[4],
             std::vector<std::vector<void *>> &peers, bool *staged = nullptr, bool force = false,
             bool persistent = false);
int finish(mi355x_comm *c, hipStream_t s);          // stream sync + barrier
int ensure_scratch(mi355x_comm *c, size_t bytes);   // exportable per-communicator scratch
int run_program(int op, int type, const Program &pr, const std::vector<void *> &in,
                const std::vector<void *> &dst, size_t off, size_t len, hipStream_t s);
int check_common(mi355x_comm *c, int op, int type);
void drain(mi355x_comm *c);                         // wait for every posted nonblocking call
int post(mi355x_comm *c, void *stream, std::function<int(hipStream_t)> run, mi355x_request **out);
void p2p_destroy(mi355x_comm *c);
// the call gate around every engine collective of a multi-process communicator (coll_comm.cpp)
void gate_enter(mi355x_comm *c);
void gate_exit(mi355x_comm *c);
struct CallGate {
    mi355x_comm *c;
    explicit CallGate(mi355x_comm *c_) : c(c_ && c_->gated ? c_ : nullptr)
    {
        if (c) gate_enter(c);
    }
    ~CallGate()
    {
        if (c) gate_exit(c);
    }
    CallGate(const CallGate &) = delete;
    CallGate &operator=(const CallGate &) = delete;
};
int p2p_progress(mi355x_comm *c);
bool p2p_defer_maps(bool on);  // this thread's passes defer reads that open a peer mapping; returns the old value
void run_progress_hook();      // the caller's progress engine (mi355x_set_progress_hook: opal_progress), not re-entered
void progress_hook_off_this_thread();  // an engine thread: never runs the caller's progress engine
void p2p_progress_all(bool defer_maps = false);  // every communicator's point-to-point (the engine's host-side waits)
int p2p_wait(mi355x_request *r);
} // namespace mi355x
