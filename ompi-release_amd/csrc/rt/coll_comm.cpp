// coll_comm.cpp -- host side of the coll/mi355x engine: node-local bootstrap, barrier, IPC
// registration cache, and the device-buffer collectives.
//
// Transport (replaces the PML/BTL path the reference takes for device buffers: coll/cuda host
// staging, coll_cuda_allreduce.c:30-77, and smcuda CUDA-IPC RDMA, btl/smcuda/README:13-113):
//   * ranks on one node share a small control segment (POSIX shm, or process memory for the
//     in-process "loopback" communicator used by tests);
//   * per call each rank publishes the IPC handle + offset of its buffers (hipIpcGetMemHandle on
//     the allocation base, cached per base: the reference's mpool/rgpusm registration cache,
//     common_cuda.c:971-1137); peers map them once (hipIpcOpenMemHandle, cached per handle);
//   * one kernel per rank then reads every rank's input directly over xGMI, folds it in the
//     reference schedule's order (coll_sched.cpp) and pushes the result into every destination.
// A call is: sync caller stream -> publish -> barrier -> kernel(s) -> sync -> barrier.
// Default data flow is PULL: every kernel writes only its own rank's memory and reads peers'
// memory, so coherence rests on kernel-completion release + the host barrier and never on a peer
// GPU's L2 seeing a remote write.  Allreduce: phase 1 the owner folds its ring block locally,
// phase 2 every rank pulls the other blocks (one launch, one segment per peer).  A one-phase
// PUSH variant (owners write into every peer's rbuf) is kept behind MI355X_KNOB_PUSH.
//
// Large allocations: hipIpcOpenMemHandle never returns for an allocation of 2 GiB or more on
// this platform (ROCm 7.2, dmabuf IPC; measured: 2046 MiB maps, 2048 MiB hangs).  A buffer whose
// allocation is at least `ipc_max` bytes is therefore never exported: the call switches, on every
// rank (the decision is taken after the exchange, from every rank's descriptors), to the STAGED
// data flow -- the message moves through each rank's persistent staging buffer (one allocation
// < 2 GiB, mapped once) in block-strided windows, like the segmented ring's phases.

#include <fcntl.h>
#include <immintrin.h>
#include <poll.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "coll_internal.hpp"
#include "coll_sched.hpp"
#include "rt_internal.hpp"

#include "comm_internal.hpp"

#include "coll_comm_int.hpp"

using namespace mi355x;

extern "C" {


int mi355x_comm_create(const char *key, int rank, int size, int device, mi355x_comm_t **out)
{
    if (!key || !out || size < 1 || size > kMaxRanks || rank < 0 || rank >= size)
        return set_error(MI355X_ERR_ARG, "bad comm_create arguments");
    *out = nullptr;
    const auto t_create = std::chrono::steady_clock::now();
    DeviceGuard dg(device);
    char bus[64] = "";
    MI_HIP(hipDeviceGetPCIBusId(bus, (int)sizeof(bus), device));
    auto *c = new mi355x_comm();
    c->rank = rank;
    c->size = size;
    c->device = device;
    c->timeout_s = env_double("MI355X_TIMEOUT_S", kDefaultTimeoutS);
    c->selftest = env_double("MI355X_SELFTEST", 1.0) != 0.0;
    c->export_check = env_double("MI355X_EXPORT_CHECK", 1.0) != 0.0;
    c->shm_name = std::string("/mi355x_") + key;
    for (char &ch : c->shm_name)
        if (ch != '/' && !isalnum((unsigned char)ch) && ch != '_' && ch != '-') ch = '_';
    const size_t bytes = ctrl_bytes(size);
    int fd = -1;
    if (rank == 0) {
        // the key must be node-unique (coll/mi355x: rank 0's pid + a counter + random bits,
        // broadcast at enable time); an existing segment of that name belongs to somebody else
        // and is never unlinked here
        fd = shm_open(c->shm_name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) {
            const int e = errno;
            delete c;
            return set_error(MI355X_ERR_PEER, "control segment %s: %s%s", key, strerror(e),
                             e == EEXIST ? " (the rendezvous key is in use by another communicator)" : "");
        }
        if (ftruncate(fd, (off_t)bytes) != 0) {
            close(fd);
            shm_unlink(c->shm_name.c_str());
            delete c;
            return set_error(MI355X_ERR_PEER, "ftruncate of control segment %s failed", key);
        }
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        for (int tries = 0;; ++tries) {
            fd = shm_open(c->shm_name.c_str(), O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
                close(fd);
                fd = -1;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                delete c;
                return set_error(MI355X_ERR_TIMEOUT, "rank %d: control segment %s never appeared", rank, key);
            }
            // ranks that enter together (an MPI_Comm_dup after a barrier) find rank 0's segment within
            // tens of microseconds: poll finely first, then back off
            usleep(tries < 200 ? 10 : 1000);
        }
    }
    void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        delete c;
        return set_error(MI355X_ERR_PEER, "mmap of the control segment failed");
    }
    c->ctrl = (Ctrl *)m;
    if (rank == 0) {
        // (a fresh O_EXCL object: ftruncate zero-filled it, and touching every page here would
        // only fault the peers' envelope rings in early)
        c->ctrl->size = (uint32_t)size;
        uint64_t secret = 0;
        FILE *ur = fopen("/dev/urandom", "rb");
        if (!ur || fread(&secret, sizeof(secret), 1, ur) != 1)
            secret = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^ ((uint64_t)getpid() << 32);
        if (ur) fclose(ur);
        c->ctrl->secret = secret;
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&c->ctrl->magic, kMagic, __ATOMIC_RELEASE);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        for (int tries = 0; __atomic_load_n(&c->ctrl->magic, __ATOMIC_ACQUIRE) != kMagic; ++tries) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                munmap(m, bytes);
                delete c;
                return set_error(MI355X_ERR_TIMEOUT, "rank %d: control segment never initialised", rank);
            }
            if (tries < 2000) sched_yield();
            else usleep(200);
        }
    }
    c->ctrl->slot[rank].pid_start = proc_start_time(getpid());
    c->ctrl->slot[rank].pid_ns = pid_namespace();
    c->ctrl->slot[rank].pid = (int32_t)getpid();
    c->ctrl->slot[rank].dev = device;
    uint64_t uid = 1469598103934665603ull;
    for (const char *p = bus; *p; ++p) uid = (uid ^ (unsigned char)tolower((unsigned char)*p)) * 1099511628211ull;
    c->ctrl->slot[rank].dev_uid = uid;
    c->ctrl->attached.fetch_add(1);
    int rc = size > 1 ? fd_sock_open(c) : MI355X_SUCCESS;
    if (rc) {
        c->ctrl->abort_flag.store(1);  // the others leave their creation barrier with an error
        if (rank == 0) shm_unlink(c->shm_name.c_str());
        const std::string msg = mi355x_last_error();
        mi355x_comm_destroy(c);
        return set_error(rc, "%s", msg.c_str());
    }
    rc = barrier(c);  // everybody mapped the segment and bound its socket: the name can go
    if (rank == 0) shm_unlink(c->shm_name.c_str());
    // ranks of this communicator on my GPU (a one-GPU rehearsal, or an oversubscribed node): they
    // split the CUs, and a persistent or spinning launch of one must stay co-resident with the others'
    int share = 0;
    for (int q = 0; q < size; ++q) share += c->ctrl->slot[q].dev_uid == uid;
    c->pipe_share = std::max(1, share);
    c->ll_max = (size_t)std::max(0.0, env_double("MI355X_LL_MAX_BYTES", 0.0));
    // pipelined allreduce by default from 4 ranks up: ahead of the two-phase flow at n = 4 and 8,
    // behind at n = 2 in the one-GPU rehearsal (profiles/r02_bench_n{2,4,8}_*); MI355X_PIPE=0/1 decides
    c->pipe_on = env_double("MI355X_PIPE", size >= 4 ? 1.0 : 0.0) != 0.0;
    c->one_phase_max = (size_t)std::max(0.0, env_double("MI355X_ONE_PHASE_MAX_BYTES", (double)c->one_phase_max));
    c->lat_on = env_double("MI355X_LAT_PROFILE", 0.0) != 0.0;
    c->rcache_max_maps = (size_t)std::max(0.0, env_double("MI355X_RCACHE_MAX_MAPS", 0.0));
    c->rcache_limit = (size_t)std::max(0.0, env_double("MI355X_RCACHE_SIZE_LIMIT", 0.0));
    c->gated = size > 1;
    // nothing device-side happens here: the LL region, the service's queue, the flows' self-tests
    // and their allocations wait for the first device-buffer collective (dev_setup), so a
    // host-only communicator costs one barrier and no device memory
    if (rc) {
        mi355x_comm_destroy(c);
        return rc;
    }
    c->create_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_create).count();
    *out = c;
    return MI355X_SUCCESS;
}

int mi355x_comm_create_loopback(int size, int device, mi355x_comm_t **comms)
{
    if (!comms || size < 1 || size > kMaxRanks) return set_error(MI355X_ERR_ARG, "bad loopback arguments");
    auto shared = std::make_shared<LoopShared>();
    shared->ctrl = (Ctrl *)calloc(1, ctrl_bytes(size));
    if (!shared->ctrl) return set_error(MI355X_ERR_NOMEM, "calloc");
    shared->ctrl->magic = kMagic;
    shared->ctrl->size = (uint32_t)size;
    for (int r = 0; r < size; ++r) {
        auto *c = new mi355x_comm();
        c->rank = r;
        c->size = size;
        c->device = device;
        c->ctrl = shared->ctrl;
        c->loopback = true;
        c->loop = shared;
        c->timeout_s = env_double("MI355X_TIMEOUT_S", kDefaultTimeoutS);
        shared->refs++;
        comms[r] = c;
    }
    return MI355X_SUCCESS;
}

int mi355x_comm_destroy(mi355x_comm_t *c)
{
    if (!c) return MI355X_SUCCESS;
    if (c->worker.joinable()) {
        {
            std::lock_guard<std::mutex> g(c->q_mtx);
            c->stop = true;
        }
        c->q_cv.notify_all();
        c->worker.join();
    }
    DeviceGuard dg(c->device);
    if (c->gated) gate_enter(c);  // (never while another process's revoker is taking the service from it)
    svc_release(c);
    p2p_destroy(c);
    for (hipEvent_t e : c->tev)
        if (e) (void)hipEventDestroy(e);
    if (c->nb_stream) (void)hipStreamDestroy(c->nb_stream);
    flush_retired(c);
    for (auto &kv : c->peer_maps) close_map(kv.second);
    for (LocalReg &r : c->local_regs) drop_reg(r);
    for (auto &kv : c->fd_stash) close(kv.second);
    if (c->fd_sock >= 0) close(c->fd_sock);
    if (c->pipe_base) (void)hipFree(c->pipe_base);
    if (c->pipe_queue) (void)hipFree(c->pipe_queue);
    if (c->pipe_dbg) (void)hipHostFree(c->pipe_dbg);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->gf_buf) {  // (stream-ordered allocation, coll_gfold.cpp)
        (void)hipFreeAsync(c->gf_buf, nullptr);
        (void)hipStreamSynchronize(nullptr);
    }
    if (c->stage) (void)hipFree(c->stage);
    if (!c->svc_stuck) {  // (a service kernel that never left may still read and write these)
        if (c->ll_base) (void)hipFree(c->ll_base);
        if (c->ll_ctr) (void)hipFree(c->ll_ctr);
        if (c->ll_err) (void)hipHostFree(c->ll_err);
    }
    if (c->lat_on && c->lat_n)
        fprintf(stderr, "[mi355x r%d] small allreduce steps over %llu calls (us): input sync %.2f, exchange %.2f, "
                "launch %.2f, finish %.2f\n", c->rank, (unsigned long long)c->lat_n, c->lat_acc[0] / c->lat_n,
                c->lat_acc[1] / c->lat_n, c->lat_acc[2] / c->lat_n, c->lat_acc[3] / c->lat_n);
    if (c->ctrl_registered) (void)hipHostUnregister(c->ctrl);
    if (c->loopback) {
        std::lock_guard<std::mutex> g(c->loop->mtx);
        if (--c->loop->refs == 0) free(c->loop->ctrl);
    } else if (c->ctrl) {
        munmap(c->ctrl, ctrl_bytes(c->size));
    }
    delete c;
    return MI355X_SUCCESS;
}

int mi355x_comm_set_rules(mi355x_comm_t *c, const mi355x_rules_t *rules)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    c->rules = rules;
    return MI355X_SUCCESS;
}

int mi355x_comm_rank(const mi355x_comm_t *c) { return c ? c->rank : -1; }
int mi355x_comm_size(const mi355x_comm_t *c) { return c ? c->size : -1; }
int mi355x_comm_barrier(mi355x_comm_t *c)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    return barrier(c);
}
static void (*g_progress_hook)(void) = nullptr;
int mi355x_set_progress_hook(void (*progress)(void))
{
    g_progress_hook = progress;
    return MI355X_SUCCESS;
}

} // extern "C"

// set while the hook runs (its callbacks may wait in the engine again) and for good on the engine's
// own threads (a nonblocking collective's worker): the caller's progress engine runs only on the
// caller's threads, as MPI's thread level allows
static thread_local bool t_hook_blocked = false;

void mi355x::run_progress_hook()
{
    if (!g_progress_hook || t_hook_blocked) return;
    t_hook_blocked = true;
    g_progress_hook();
    t_hook_blocked = false;
}

void mi355x::progress_hook_off_this_thread() { t_hook_blocked = true; }

extern "C" {

// The buffer-kind vote (mi355x_rt.h).  One side of a call waits for every vote: both at a window's
// checkpoint (every kVoteWindow-th call), the host ranks in a window that follows device use (they
// join the engine on device copies when a peer holds device buffers), the device ranks otherwise
// (they stage to the host component when a peer holds host buffers).  The mode of the next window
// is a function of the checkpoint's votes, which every rank reads, so every rank agrees on it.  A
// non-waiting rank may run ahead: a host rank by many host calls (a bcast root), a device rank by
// at most the engine's own slack, since every engine call needs every rank; so a waiter that finds
// a peer's ring entry already reused by a later call knows that peer did not wait in the engine --
// it voted host.  A waiter must not stall other work: the wait drives the caller's progress engine
// (opal_progress through the hook) and this communicator's point-to-point, so a peer that first
// needs an outstanding send of ours to complete still gets there (ob1's blocking waits progress the
// same way, req_wait.c).  The wait is unbounded, like a host collective's receive: a rank that is
// late by minutes (checkpoint I/O) is not an error, and nothing poisons the communicator.
int mi355x_comm_vote(mi355x_comm_t *c, int device, int *engine)
{
    if (!c || !engine) return set_error(MI355X_ERR_ARG, "NULL argument");
    *engine = device ? 1 : 0;
    if (c->size == 1) return MI355X_SUCCESS;
    const uint64_t s = ++c->vote_seq;
    const bool ckpt = (s % kVoteWindow) == 0;
    if (device) c->vote_window_dev = true;
    Ctrl *k = c->ctrl;
    const uint64_t word = (s << 2) | ((ckpt && c->vote_window_dev) ? 2u : 0u) | (device ? 1u : 0u);
    k->slot[c->rank].vote[s % kVoteRing].store(word, std::memory_order_release);
    const bool wait = ckpt || (c->vote_host_waits ? !device : device);
    if (!wait) return MI355X_SUCCESS;  // (*engine = device: a host rank is never in the engine here, nor a device rank out of it)
    bool any_dev = device, all_dev = device, win_dev = c->vote_window_dev;
    for (int r = 0; r < c->size; ++r) {
        if (r == c->rank) continue;
        unsigned spins = 0;
        for (;;) {
            const uint64_t v = k->slot[r].vote[s % kVoteRing].load(std::memory_order_acquire);
            if ((v >> 2) == s) {
                any_dev = any_dev || (v & 1u);
                all_dev = all_dev && (v & 1u);
                win_dev = win_dev || (v & 2u);
                break;
            }
            if ((v >> 2) > s) {
                if (ckpt || c->vote_host_waits)  // (every rank waits at a checkpoint; a device rank in this mode is in the engine)
                    return set_error(MI355X_ERR_PEER, "rank %d is %d or more collectives ahead of rank %d", r,
                                     kVoteRing, c->rank);
                all_dev = false;  // a host rank that ran ahead
                break;
            }
            if (k->abort_flag.load(std::memory_order_relaxed))
                return set_error(MI355X_ERR_PEER, "a peer aborted the communicator");
            if (++spins > 2048) {
                if ((spins & 63) == 0) {
                    p2p_progress_all();
                    run_progress_hook();
                }
                if ((spins & 0xffff) == 0 && peer_gone(c)) return MI355X_ERR_PEER;
                sched_yield();
            }
        }
    }
    if (ckpt) {
        *engine = any_dev ? 1 : 0;  // a mixed checkpoint call runs in the engine
        c->vote_host_waits = win_dev;
        c->vote_window_dev = false;
    } else {
        *engine = c->vote_host_waits ? (any_dev ? 1 : 0) : (all_dev ? 1 : 0);
    }
    return MI355X_SUCCESS;
}

int mi355x_comm_last_algorithm(const mi355x_comm_t *c) { return c ? c->last_alg : -1; }

// test hook without a GPU: the token table's holder protocol for a device uid, as a communicator
// named `name` would use it (op 1: try to take it; 0: give it back).  Returns 1 while held.  The
// CPU tests kill a holder process and check that the next process takes the token back.
int mi355x_debug_token(uint64_t dev_uid, const char *name, int op)
{
    static std::mutex mtx;
    static std::map<std::string, mi355x_comm *> comms;
    if (!name) return set_error(MI355X_ERR_ARG, "name is NULL");
    std::lock_guard<std::mutex> g(mtx);
    mi355x_comm *&c = comms[name];
    if (!c) {
        c = new mi355x_comm();
        c->ctrl = (Ctrl *)calloc(1, ctrl_bytes(1));
        c->ctrl->slot[0].dev_uid = dev_uid;
        c->shm_name = std::string("/mi355x_") + name;
    }
    if (op) return (c->pipe_entry >= 0 || pipe_token_acquire(c)) ? 1 : 0;
    if (c->pipe_entry >= 0) pipe_token_release(c);
    return 0;
}

// test hook: take (1) or give back (0) this communicator's pipelined-grid token of its GPU outside
// any call, as a rank inside a pipelined allreduce holds it (tests kill a holder, then check that
// the next communicator on the GPU is admitted again)
int mi355x_debug_pipe_token(mi355x_comm_t *c, int acquire)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (acquire) return pipe_token_acquire(c) ? 1 : 0;
    if (c->pipe_entry >= 0) pipe_token_release(c);
    return 0;
}
// the service limits a communicator reports: its own once the device setup decided it may have
// the service; before that setup (deferred to the first device-buffer collective) the configured
// ones, which it will have unless that setup finds the service unusable
static bool svc_limit_visible(const mi355x_comm_t *c)
{
    return c->svc_ok || c->svc_want || (!c->dev_ready && !c->loopback && c->size > 1);
}

int mi355x_comm_get(const mi355x_comm_t *c, int knob, long *value)
{
    if (!c || !value) return set_error(MI355X_ERR_ARG, "NULL argument");
    switch (knob) {
    case MI355X_KNOB_ALLREDUCE_ALG: *value = c->knob_allreduce; break;
    case MI355X_KNOB_REDUCE_ALG: *value = c->knob_reduce; break;
    case MI355X_KNOB_REDUCE_SCATTER_ALG: *value = c->knob_rs; break;
    case MI355X_KNOB_BLOCKS_PER_CU: *value = c->tune.blocks_per_cu; break;
    case MI355X_KNOB_TIMEOUT_S: *value = (long)c->timeout_s; break;
    case MI355X_KNOB_PUSH: *value = c->tune.push; break;
    case MI355X_KNOB_IPC_MAX_BYTES: *value = (long)c->ipc_max; break;
    case MI355X_KNOB_STAGE_BYTES: *value = (long)c->stage_bytes; break;
    case MI355X_KNOB_PIPE_REFUSED: *value = (long)c->pipe_refused; break;
    case MI355X_KNOB_LL_MAX_BYTES: *value = (long)c->ll_max; break;
    case MI355X_KNOB_REDUCE_CHAIN_FANOUT: *value = c->chain_fanout; break;
    case MI355X_KNOB_TIME_PHASES: *value = c->time_phases ? 1 : 0; break;
    case MI355X_KNOB_COPY_BLOCK_KIB: *value = c->tune.copy_block_kib; break;
    case MI355X_KNOB_PIPE: *value = c->pipe_on ? 1 : 0; break;
    case MI355X_KNOB_PIPE_WG_PER_CU: *value = c->tune.pipe_wg_per_cu; break;
    case MI355X_KNOB_PIPE_CHUNK_KIB: *value = c->tune.pipe_chunk_kib; break;
    case MI355X_KNOB_PIPE_WT: *value = c->tune.pipe_wt; break;
    case MI355X_KNOB_ONE_PHASE_MAX_BYTES: *value = (long)c->one_phase_max; break;
    case MI355X_KNOB_SVC_MAX_BYTES: *value = svc_limit_visible(c) ? (long)c->svc_max : 0; break;
    case MI355X_KNOB_SVC_CALLS: *value = (long)c->svc_calls; break;
    case MI355X_KNOB_SVC_LAUNCHES: *value = (long)c->svc_launches; break;
    case MI355X_KNOB_SVC_RESIDENT: *value = c->svcq && svc_resident(c->svcq) ? 1 : 0; break;
    case MI355X_KNOB_SVC_PULL_MAX_BYTES: *value = svc_limit_visible(c) ? (long)c->svc_pull_max : 0; break;
    case MI355X_KNOB_SVC_PULL_COPY_MAX_BYTES: *value = svc_limit_visible(c) ? (long)c->svc_copy_max : 0; break;
    case MI355X_KNOB_FLOWS: *value = (long)c->flows; break;
    case MI355X_KNOB_FLOWS_FAILED: *value = (long)c->flows_failed; break;
    case MI355X_KNOB_CREATE_US: *value = (long)c->create_us; break;
    case MI355X_KNOB_SELFTEST_US: *value = (long)c->selftest_us; break;
    case MI355X_KNOB_SELFTEST_REUSED: *value = (long)c->selftest_reused; break;
    case MI355X_KNOB_DEV_SETUP: *value = c->dev_ready ? 1 : 0; break;
    case MI355X_KNOB_SELFTEST: *value = c->selftest ? 1 : 0; break;
    case MI355X_KNOB_PIPE_CALLS: *value = (long)c->pipe_calls; break;
    case MI355X_KNOB_EXPORT_MISMATCHES: *value = (long)c->export_mismatches; break;
    case MI355X_KNOB_SETUP_US: *value = (long)c->setup_us; break;
    case MI355X_KNOB_SVC_OWNER: *value = c->svc_ok ? 1 : 0; break;
    case MI355X_KNOB_SVC_CLAIMS: *value = (long)c->svc_epoch; break;
    case MI355X_KNOB_SVC_IDLE_US: *value = (long)(c->svc_idle_s * 1e6 + 0.5); break;
    case MI355X_KNOB_SVC_SHRINK_US: *value = (long)(c->svc_shrink_s * 1e6 + 0.5); break;
    case MI355X_KNOB_SVC_REGROWS: *value = (long)c->svc_regrows; break;
    case MI355X_KNOB_RCACHE_MAX_MAPS: *value = (long)c->rcache_max_maps; break;
    case MI355X_KNOB_RCACHE_SIZE_LIMIT: *value = (long)c->rcache_limit; break;
    case MI355X_KNOB_PEER_MAPS: {
        std::lock_guard<std::recursive_mutex> g(const_cast<mi355x_comm *>(c)->reg_mtx);
        *value = (long)peer_map_count(c);
        break;
    }
    case MI355X_KNOB_RCACHE_EVICTIONS: *value = (long)c->rcache_evictions; break;
    default: return set_error(MI355X_ERR_ARG, "unknown knob %d", knob);
    }
    return MI355X_SUCCESS;
}

int mi355x_comm_phase_ms(const mi355x_comm_t *c, float *phase1_ms, float *phase2_ms)
{
    if (!c || !phase1_ms || !phase2_ms) return set_error(MI355X_ERR_ARG, "NULL argument");
    *phase1_ms = c->phase_ms[0];
    *phase2_ms = c->phase_ms[1];
    return MI355X_SUCCESS;
}

int mi355x_comm_set(mi355x_comm_t *c, int knob, long value)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (!c->dev_ready && !c->loopback && c->size > 1) {
        // limits that size or depend on the device setup: kept for dev_setup (which sizes the LL
        // region by them) and applied through this function once the self-tests have run
        size_t *field = knob == MI355X_KNOB_LL_MAX_BYTES ? &c->ll_max
                        : knob == MI355X_KNOB_SVC_MAX_BYTES ? &c->svc_max
                        : knob == MI355X_KNOB_SVC_PULL_MAX_BYTES ? &c->svc_pull_max
                        : knob == MI355X_KNOB_SVC_PULL_COPY_MAX_BYTES ? &c->svc_copy_max : nullptr;
        if (field) {
            const long hi = (knob == MI355X_KNOB_LL_MAX_BYTES || knob == MI355X_KNOB_SVC_MAX_BYTES) ? (64l << 20) : (1l << 30);
            if (value < 0 || value > hi) return set_error(MI355X_ERR_ARG, "knob %d out of range", knob);
            *field = (size_t)value;
            c->preset.emplace_back(knob, value);
            return MI355X_SUCCESS;
        }
    }
    switch (knob) {
    case MI355X_KNOB_SELFTEST: c->selftest = value != 0; break;  // (read by the device setup)
    case MI355X_KNOB_ALLREDUCE_ALG: c->knob_allreduce = (int)value; break;
    case MI355X_KNOB_REDUCE_ALG: c->knob_reduce = (int)value; break;
    case MI355X_KNOB_REDUCE_SCATTER_ALG: c->knob_rs = (int)value; break;
    case MI355X_KNOB_BLOCKS_PER_CU:
        // up to 1024: with that many the streaming kernels' grids are one-shot (every thread one pass)
        if (value < 1 || value > 1024) return set_error(MI355X_ERR_ARG, "blocks_per_cu out of range");
        c->tune.blocks_per_cu = (int)value;
        break;
    case MI355X_KNOB_TIMEOUT_S: c->timeout_s = (double)value; break;
    case MI355X_KNOB_PUSH: c->tune.push = value ? 1 : 0; break;
    case MI355X_KNOB_IPC_MAX_BYTES:
        if (value < 0) return set_error(MI355X_ERR_ARG, "ipc_max_bytes < 0");
        c->ipc_max = (size_t)value;
        break;
    case MI355X_KNOB_REDUCE_CHAIN_FANOUT:
        if (value < 1 || value > 32) return set_error(MI355X_ERR_ARG, "chain fan-out out of range");
        c->chain_fanout = (int)value;
        break;
    case MI355X_KNOB_COPY_BLOCK_KIB:
        if (value < 4 || value > 256) return set_error(MI355X_ERR_ARG, "copy_block_kib out of range");
        c->tune.copy_block_kib = (int)value;
        break;
    case MI355X_KNOB_PIPE: c->pipe_on = value != 0 && (c->flows & MI355X_FLOW_PIPE); break;  // (a failed self-test keeps it off)
    case MI355X_KNOB_PIPE_WG_PER_CU:
        if (value < 1 || value > 8) return set_error(MI355X_ERR_ARG, "pipe_wg_per_cu out of range");
        c->tune.pipe_wg_per_cu = (int)value;
        break;
    case MI355X_KNOB_PIPE_CHUNK_KIB:
        if (value < 0 || value > (1l << 20)) return set_error(MI355X_ERR_ARG, "pipe_chunk_kib out of range");
        c->tune.pipe_chunk_kib = (int)value;
        break;
    case MI355X_KNOB_PIPE_WT: c->tune.pipe_wt = value != 0; break;
    case MI355X_KNOB_ONE_PHASE_MAX_BYTES:
        if (value < 0 || value > (1l << 30)) return set_error(MI355X_ERR_ARG, "one_phase_max_bytes out of range");
        c->one_phase_max = (size_t)value;
        break;
    case MI355X_KNOB_TIME_PHASES:
        c->time_phases = value != 0;
        if (c->time_phases && !c->tev[0]) {
            DeviceGuard dg(c->device);
            for (hipEvent_t &e : c->tev) MI_HIP(hipEventCreate(&e));
        }
        break;
    case MI355X_KNOB_LL_MAX_BYTES:
        if (value < 0 || value > (64l << 20)) return set_error(MI355X_ERR_ARG, "ll_max_bytes out of range");
        c->ll_max = c->ll_ok ? (size_t)value : 0;  // a failed (or skipped) self-test keeps it off
        break;
    case MI355X_KNOB_SVC_PULL_MAX_BYTES:
        if (value < 0 || value > (1l << 30)) return set_error(MI355X_ERR_ARG, "svc_pull_max_bytes out of range");
        if (c->svc_ok || c->svc_want) {
            drain(c);
            c->svc_pull_max = (size_t)value;
        }
        break;
    case MI355X_KNOB_SVC_PULL_COPY_MAX_BYTES:
        if (value < 0 || value > (1l << 30)) return set_error(MI355X_ERR_ARG, "svc_pull_copy_max_bytes out of range");
        if (c->svc_ok || c->svc_want) {
            drain(c);
            c->svc_copy_max = (size_t)value;
        }
        break;
    case MI355X_KNOB_SVC_MAX_BYTES:
        if (value < 0 || value > (64l << 20)) return set_error(MI355X_ERR_ARG, "svc_max_bytes out of range");
        if (c->svc_ok || c->svc_want) {  // a communicator that cannot have the service keeps 0
            drain(c);
            c->svc_max = (size_t)value;
        }
        break;
    case MI355X_KNOB_RCACHE_MAX_MAPS:
    case MI355X_KNOB_RCACHE_SIZE_LIMIT: {
        if (value < 0) return set_error(MI355X_ERR_ARG, "rcache bound < 0");
        drain(c);
        std::lock_guard<std::recursive_mutex> g(c->reg_mtx);
        (knob == MI355X_KNOB_RCACHE_MAX_MAPS ? c->rcache_max_maps : c->rcache_limit) = (size_t)value;
        rcache_trim(c, nullptr);
        break;
    }
    case MI355X_KNOB_SVC_SHRINK_US:
    case MI355X_KNOB_SVC_IDLE_US:
        if (knob == MI355X_KNOB_SVC_SHRINK_US ? (value < 0 || value > 60000000) : (value < 100 || value > 60000000))
            return set_error(MI355X_ERR_ARG, "%s out of range", knob == MI355X_KNOB_SVC_SHRINK_US ? "svc_shrink_us" : "svc_idle_us");
        drain(c);
        (knob == MI355X_KNOB_SVC_SHRINK_US ? c->svc_shrink_s : c->svc_idle_s) = (double)value * 1e-6;
        {  // a resident service picks the new limit up at its next launch (g_svc_mtx: not while a
           // revoker detaches this communicator)
            std::lock_guard<std::mutex> g(g_svc_mtx);
            if (c->svc_ok && c->svcq) svc_park(c);
        }
        break;
    case MI355X_KNOB_STAGE_BYTES:
        if (value < 4096 || value >= (1l << 31)) return set_error(MI355X_ERR_ARG, "stage_bytes out of range");
        if (c->stage) (void)hipFree(c->stage);
        c->stage = nullptr;
        c->stage_bytes = (size_t)value & ~(size_t)4095;
        break;
    default: return set_error(MI355X_ERR_ARG, "unknown knob %d", knob);
    }
    return MI355X_SUCCESS;
}

// Describe the per-element program the engine runs (host only, no GPU needed).  Layout:
//   fold: [1, nr, len, order[0..len-1], role[0..len-1]]
//   tree: [0, nr, nsteps, result, (dst, out, in) x nsteps]
// kind 1: allreduce (alg 3 = recursive doubling, 4/5 = ring block `block`,
//                    1/2 = reduce-to-0 with reduce algorithm `block` (1..5) + bcast)
// kind 2: reduce to rank `block` with reduce algorithm `alg`;  kind 3: reduce_scatter ring block;
// kind 4: reduce_scatter recursive halving block; kind 5: reduce chain to 0 with fan-out `block`.
// Returns the number of ints written or < 0.
int mi355x_sched_program(int kind, int n, int alg, int block, int *out, int cap)
{
    if (!out || n < 1 || n > kMaxRanks) return set_error(MI355X_ERR_ARG, "bad arguments");
    Program pr;
    ExprPool ep;
    bool ok = true;
    switch (kind) {
    case 1:
        if (alg == AR_RING || alg == AR_RING_SEGMENTED) pr = ring_block_program(n, block);
        else if (alg == AR_RECDBL) ok = compile_expr(ep, expr_allreduce_recursive_doubling(ep, n), n, &pr);
        else ok = compile_expr(ep, expr_reduce(ep, block, n, 0), n, &pr);
        break;
    case 2: ok = compile_expr(ep, expr_reduce(ep, alg, n, block), n, &pr); break;  // block = root
    case 5: ok = compile_expr(ep, expr_reduce(ep, RED_CHAIN, n, 0, block), n, &pr); break;  // block = fan-out
    case 3: pr = reduce_scatter_ring_block_program(n, block); break;
    case 4: {
        std::vector<int> roots = expr_reduce_scatter_rechalving(ep, n);
        ok = compile_expr(ep, roots[block], n, &pr);
        break;
    }
    default: return set_error(MI355X_ERR_ARG, "unknown kind %d", kind);
    }
    if (!ok) return set_error(MI355X_ERR_UNSUPPORTED, "schedule does not compile");
    std::vector<int> v;
    if (pr.is_fold) {
        v = {1, pr.nr, (int)pr.order.size()};
        for (int r : pr.order) v.push_back(r);
        for (size_t j = 0; j < pr.order.size(); ++j) v.push_back((int)((pr.role_mask >> j) & 1u));
    } else {
        v = {0, pr.nr, (int)pr.steps.size(), pr.result};
        for (const TreeStep &t : pr.steps) {
            v.push_back(t.dst);
            v.push_back(t.out);
            v.push_back(t.in);
        }
    }
    if ((int)v.size() > cap) return set_error(MI355X_ERR_ARG, "cap too small");
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    return (int)v.size();
}


} // extern "C"
