// coll_comm_int.hpp -- declarations shared by the engine's host-side files (coll_ctl.cpp,
// coll_dmabuf.cpp, coll_rcache.cpp, coll_staged.cpp, coll_ll_host.cpp, coll_svc_host.cpp,
// coll_selftest.cpp, coll_pipe_host.cpp, coll_tokens.cpp, coll_decide.cpp, coll_flows.cpp,
// coll_comm.cpp): what one of them defines and another calls.
#pragma once

#include <map>
#include <mutex>
#include <sys/socket.h>
#include <sys/un.h>

#include "comm_internal.hpp"

namespace mi355x {

struct GpuTokens;  // coll_tokens.cpp
// the resident service's owner per device and its lock (coll_svc_host.cpp)
extern std::mutex g_svc_mtx;
extern std::map<int, mi355x_comm *> g_svc_owner;

// The service's resources -- its HSA queue, doorbell page and host words -- exist once per process
// and GPU: created with the first communicator that may use the service (svc_setup; an idle queue
// also keeps the host flows of ranks sharing a GPU fast), shared by the communicators that own the
// service in turn (a handover creates no queue), freed with the last communicator attached.
struct SvcRes {
    SvcQueue *q = nullptr;
    SvcPage *page = nullptr;
    bool page_dev = false;
    uint64_t *host = nullptr;
    int users = 0;       // communicators attached (claimed once at least, not destroyed)
    bool stuck = false;  // a service kernel never left: never freed
};
extern std::map<int, SvcRes> g_svc_res;

bool pid_alive(pid_t pid);
bool peer_gone(mi355x_comm *c);
uint64_t pid_namespace();
int barrier(mi355x_comm *c);
// point-to-point progress from a host wait inside a collective (MPI's progress rule), gated against
// the members' close windows (coll_ctl.cpp)
void barrier_progress(mi355x_comm *c, bool drain_fds = true);
uint64_t buffer_id(const void *p);
int local_handle(mi355x_comm *c, const void *p, BufDesc *d, bool force);
// the stream a collective runs on, for the setup work it triggers (device setup, dmabuf probe, LL
// resync): ordered with the call's own work and never a stream of its own -- a second stream per
// process is a second hardware queue, and eight processes sharing one GPU then time-slice their
// queues: the 8-rank 1 GiB allreduce rehearsal took 22.9 ms per call instead of 3.7 while every
// rank held an idle setup stream (profiles/r05_setup_stream_bisect.txt)
void gfold_idle(mi355x_comm *c, hipStream_t s);  // coll_gfold.cpp
struct CallStream {
    mi355x_comm *c;
    hipStream_t prev;
    CollTune *prev_tune;
    CallStream(mi355x_comm *c_, hipStream_t s) : c(c_), prev(c_->call_s), prev_tune(coll_tune_use(&c_->tune))
    {
        c->call_s = s;  // (NULL is the null stream: call_depth says whether call_s is set)
        c->call_depth++;
        if (c->gf_buf) gfold_idle(c, s);  // (an idle gather-then-fold buffer is dropped on this stream)
    }
    ~CallStream()
    {
        c->call_depth--;
        c->call_s = prev;
        coll_tune_use(prev_tune);
    }
};

void retire_map(mi355x_comm *c, const PeerMap &m);
void flush_retired(mi355x_comm *c);
int exchange(mi355x_comm *c, int nbuf, const void *const *mine, const uint64_t sig[4],
             std::vector<std::vector<void *>> &peers, bool *staged, bool force, bool persistent);
int finish(mi355x_comm *c, hipStream_t s);
int setup_done_words(mi355x_comm *c);
int ensure_scratch(mi355x_comm *c, size_t bytes);
void fd_sock_addr(const mi355x_comm *c, int rank, sockaddr_un *a, socklen_t *len);
int fd_sock_open(mi355x_comm *c);
int fd_drain(mi355x_comm *c, bool wait);
int send_fds(mi355x_comm *c, int peer, const int *fds, const uint64_t *ids, int nfd);
int send_fd(mi355x_comm *c, int peer, int fd, uint64_t id);
int take_fd(mi355x_comm *c, int peer, uint64_t id, int *out);
int serve_fd(mi355x_comm *c, int peer, uint64_t id);
void drop_stash(mi355x_comm *c, int peer, uint64_t id);
int export_dmabufs(mi355x_comm *c, BufDesc *const *ds, int nd, uint64_t peers);
int export_dmabuf(mi355x_comm *c, BufDesc *d, uint64_t peers);
int import_dmabuf(mi355x_comm *c, int peer, uint64_t id, size_t size, void **mapped, hipExternalMemory_t *ext);
int probe_dmabuf(mi355x_comm *c);
bool evictable(const mi355x_comm *c, const PeerMap &m, const PeerMap *keep);
void rcache_trim(mi355x_comm *c, const PeerMap *keep);
size_t peer_map_count(const mi355x_comm *c);
int map_peer(mi355x_comm *c, int peer, const BufDesc &d, void **out, PeerMap **entry, bool coll);
int run_program(int op, int type, const Program &pr, const std::vector<void *> &in,
                       const std::vector<void *> &dst, size_t off, size_t len, hipStream_t s);
int stage_peers(mi355x_comm *c, std::vector<void *> &sp);
int staged_reduce(mi355x_comm *c, int op, int type, const Program &pr, const void *in,
                         const std::vector<size_t> &boff, const std::vector<size_t> &blen, void *mine_dst,
                         bool distribute, void *rbuf, hipStream_t s);
int staged_allgather(mi355x_comm *c, const void *src, void *rbuf, size_t bytes, hipStream_t s);
int staged_bcast(mi355x_comm *c, void *buf, size_t bytes, int root, hipStream_t s);
bool svc_usable(const mi355x_comm *c, size_t bytes);
bool ll_usable(const mi355x_comm *c, size_t bytes);
int ensure_ll(mi355x_comm *c);
void verdict_store(mi355x_comm *c);  // coll_selftest.cpp: flow verdicts for the member set
int ll_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s);
int ll_selftest(mi355x_comm *c);
uint64_t mono_ns();
uint64_t *svc_done_word(mi355x_comm *c);
uint32_t *svc_err_word(mi355x_comm *c);
void svc_ring(mi355x_comm *c, uint64_t v);
int svc_launch(mi355x_comm *c, uint64_t first);
bool svc_stop(mi355x_comm *c);
void svc_park(mi355x_comm *c);
int svc_call(mi355x_comm *c, const SvcCall &call, uint64_t part);
int svc_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s);
bool svc_pull_usable(const mi355x_comm *c, size_t bytes, size_t esz);
bool svc_pull_copy_usable(const mi355x_comm *c, size_t bytes);
int svc_pull_copy_run(mi355x_comm *c, int mode, const std::vector<std::vector<void *>> &P, const void *src,
                             void *dst, size_t bytes, int root);
int svc_pull_run(mi355x_comm *c, int op, int type, const std::vector<std::vector<void *>> &P, const void *in,
                        void *rbuf, size_t count, size_t esz, size_t early, size_t late, size_t split);
void svc_trace_report(mi355x_comm *c);
bool svc_attach(mi355x_comm *c);
void svc_detach(mi355x_comm *c);
void svc_unclaim_locked(mi355x_comm *c);
void svc_let_go(mi355x_comm *c);
void svc_release(mi355x_comm *c);
uint32_t gate_revoker_word();
void gate_enter(mi355x_comm *c);
void gate_exit(mi355x_comm *c);
bool svc_revoke(mi355x_comm *x);
int ll_resync(mi355x_comm *c);
unsigned selftest_injected();
bool selftest_on(const mi355x_comm *c);
uint32_t st_val(uint64_t seed, int q, size_t i);
int agree_flows(mi355x_comm *c, unsigned mine, unsigned *all);
int svc_selftest(mi355x_comm *c);
int pipe_selftest(mi355x_comm *c);
int svc_claim(mi355x_comm *c);
int svc_maybe_claim(mi355x_comm *c, bool sized);
void svc_setup(mi355x_comm *c);
int dev_setup(mi355x_comm *c);
bool coll_slot_supported(int op, int type);  // coll_kernels.hip: the fold families carry (op, type)
// gather-then-fold (coll_gfold.cpp): elements [e0, e0 + ne) evaluated with `pr`, results to dst
struct GfSeg {
    size_t e0 = 0, ne = 0;
    Program pr;
    char *dst = nullptr;  // where element e0's result goes (nullptr: evaluate nothing)
};
int gather_fold(mi355x_comm *c, const void *in, size_t count, int type, int op, const std::vector<GfSeg> &segs,
                hipStream_t s);
void gfold_idle(mi355x_comm *c, hipStream_t s);
int gfold_allreduce(mi355x_comm *c, const void *in, void *rbuf, size_t count, int type, int op, hipStream_t s);
int gfold_reduce(mi355x_comm *c, const void *in, void *rbuf, size_t count, int type, int op, int root, hipStream_t s);
int gfold_reduce_scatter_block(mi355x_comm *c, const void *in, void *rbuf, size_t rcount, int type, int op,
                               hipStream_t s);
int gfold_reduce_scatter(mi355x_comm *c, const void *in, void *rbuf, const size_t *disp, int type, int op,
                         hipStream_t s);
int gfold_scan(mi355x_comm *c, const void *in, void *rbuf, size_t count, int type, int op, int last, hipStream_t s);
hipStream_t setup_stream(mi355x_comm *c);
int ensure_pipe(mi355x_comm *c);
int pipe_allreduce(mi355x_comm *c, int op, int type, const Program &pr,
                          const std::vector<std::vector<void *>> &P, size_t count, hipStream_t s);
void ll_program(LLArgs &a, const Program &pr);
bool svc_rs_usable(const mi355x_comm *c, size_t max_block_bytes, const Program &pr);
int svc_rs_run(mi355x_comm *c, int op, int type, const Program &pr, const std::vector<std::vector<void *>> &P,
                      const void *in, size_t off, void *rbuf, size_t bytes, size_t esz);
uint64_t proc_start_time(pid_t pid);
bool holder_alive(uint64_t who, uint64_t start);
GpuTokens *gpu_tokens();
bool pipe_token_reclaim(GpuTokens *t, int i, uint64_t cur);
bool pipe_token_acquire(mi355x_comm *c);
void pipe_token_release(mi355x_comm *c);
int rule_alg(const mi355x_comm *c, int coll, size_t bytes, int *faninout);
int pick_allreduce(const mi355x_comm *c, size_t count, size_t esz);
int pick_reduce(const mi355x_comm *c, size_t count, size_t esz, int *chain_fanout);
int pick_reduce_scatter(const mi355x_comm *c, size_t total, size_t esz);
bool reduce_program(const mi355x_comm *c, size_t count, size_t esz, int root, Program *pr, int *alg);
bool allreduce_tree_program(mi355x_comm *c, int alg, size_t count, size_t esz, Program *pr);
int check_common(mi355x_comm *c, int op, int type);
double env_double(const char *name, double dflt);
void drain(mi355x_comm *c);
void worker_main(mi355x_comm *c);
int post(mi355x_comm *c, void *stream, std::function<int(hipStream_t)> run, mi355x_request **out);
int allreduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op,
                     void *stream);
int reduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                  void *stream);
int reduce_scatter_block_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t rcount, int type,
                                int op, void *stream);
int reduce_scatter_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, const int *rcounts, int type,
                          int op, void *stream);
int allgather_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream);
int bcast_impl(mi355x_comm_t *c, void *buf, size_t bytes, int root, void *stream);

} // namespace mi355x
