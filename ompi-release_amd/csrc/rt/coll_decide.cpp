// coll_decide.cpp -- algorithm choice (coll/tuned's decision order) and the communicator's
// nonblocking worker (split out of coll_comm.cpp).

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

namespace mi355x {

// ----------------------------------------------------------------- algorithm choice
// The order of coll/tuned's dec_dynamic functions (coll_tuned_decision_dynamic.c:59-99): a file
// rule for this communicator size and message size, else the forced (MCA) algorithm, else the
// fixed decision.
int rule_alg(const mi355x_comm *c, int coll, size_t bytes, int *faninout)
{
    int alg = 0;
    if (c->rules) mi355x_rules_decide(c->rules, coll, c->size, bytes, &alg, faninout, nullptr);
    return alg;
}

int pick_allreduce(const mi355x_comm *c, size_t count, size_t esz)
{
    const int r = rule_alg(c, MI355X_COLL_ALLREDUCE, count * esz, nullptr);
    if (r) return r;
    return c->knob_allreduce ? c->knob_allreduce : allreduce_decision(c->size, count, esz);
}

// what comm->c_coll.coll_reduce would run for `count` elements (ompi_coll_tuned_reduce_intra_
// dec_dynamic): used by MPI_Reduce and by the algorithms that call it (nonoverlapping allreduce,
// coll/basic reduce_scatter_block, nonoverlapping reduce_scatter)
int pick_reduce(const mi355x_comm *c, size_t count, size_t esz, int *chain_fanout)
{
    int fio = 0;
    const int r = rule_alg(c, MI355X_COLL_REDUCE, count * esz, &fio);
    if (r) {
        *chain_fanout = fio;
        return r;
    }
    *chain_fanout = c->chain_fanout;
    return c->knob_reduce ? c->knob_reduce : reduce_decision(c->size, count, esz);
}

int pick_reduce_scatter(const mi355x_comm *c, size_t total, size_t esz)
{
    const int r = rule_alg(c, MI355X_COLL_REDUCESCATTER, total * esz, nullptr);
    if (r) return r;
    return c->knob_rs ? c->knob_rs : reduce_scatter_decision(c->size, total, esz);
}

// per-element program of a reduce to `root` of `count` elements
bool reduce_program(const mi355x_comm *c, size_t count, size_t esz, int root, Program *pr, int *alg)
{
    int fanout = kDefaultChainFanout;
    *alg = pick_reduce(c, count, esz, &fanout);
    ExprPool ep;
    return compile_expr(ep, expr_reduce(ep, *alg, c->size, root, fanout), c->size, pr);
}

// program of the non-ring allreduce algorithms: recursive doubling, or reduce to 0 + bcast
// (nonoverlapping: comm->c_coll.coll_reduce, coll_tuned_allreduce.c:67-100; linear: the linear
// reduce, :897-929)
bool allreduce_tree_program(mi355x_comm *c, int alg, size_t count, size_t esz, Program *pr)
{
    if (alg == AR_RECDBL || alg == AR_LINEAR) {
        // these depend on the communicator size only: compiled once (the symbolic re-execution of
        // the schedule costs about a microsecond, a visible share of a small allreduce)
        std::lock_guard<std::mutex> g(c->prog_mtx);
        auto it = c->prog_cache.find(alg);
        if (it != c->prog_cache.end()) {
            *pr = it->second;
            return true;
        }
        ExprPool ep;
        const bool ok = compile_expr(ep, alg == AR_RECDBL ? expr_allreduce_recursive_doubling(ep, c->size)
                                                          : expr_reduce(ep, RED_LINEAR, c->size, 0),
                                     c->size, pr);
        if (ok) c->prog_cache.emplace(alg, *pr);
        return ok;
    }
    int ra;
    return reduce_program(c, count, esz, 0, pr, &ra);
}

int check_common(mi355x_comm *c, int op, int type)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (!mi355x_op_supported(op, type))
        return set_error(MI355X_ERR_UNSUPPORTED, "no GPU kernel for op %d type %d", op, type);
    return MI355X_SUCCESS;
}

double env_double(const char *name, double dflt)
{
    const char *v = getenv(name);
    return v ? atof(v) : dflt;
}

// ----------------------------------------------------------------- nonblocking
// Wait until every posted nonblocking call of this communicator has finished (MPI orders a
// blocking collective after the nonblocking ones posted before it on every rank).
void drain(mi355x_comm *c)
{
    std::unique_lock<std::mutex> g(c->q_mtx);
    c->q_cv.wait(g, [c] { return c->pending == 0; });
}

void worker_main(mi355x_comm *c)
{
    (void)hipSetDevice(c->device);
    progress_hook_off_this_thread();
    for (;;) {
        mi355x_request *r;
        {
            std::unique_lock<std::mutex> g(c->q_mtx);
            c->q_cv.wait(g, [c] { return c->stop || !c->queue.empty(); });
            if (c->queue.empty()) return;  // stop requested and nothing left
            r = c->queue.front();
            c->queue.pop_front();
        }
        int rc = MI355X_SUCCESS;
        if (hipStreamWaitEvent(c->nb_stream, r->ev, 0) != hipSuccess)
            rc = set_error(MI355X_ERR_HIP, "hipStreamWaitEvent failed");
        if (rc == MI355X_SUCCESS) {
            CallGate gate(c);
            rc = r->run(c->nb_stream);
        }
        r->rc = rc;
        if (rc != MI355X_SUCCESS) r->err = mi355x_last_error();
        r->run = nullptr;
        r->done.store(1, std::memory_order_release);
        {
            std::lock_guard<std::mutex> g(c->q_mtx);
            c->pending--;
        }
        c->q_cv.notify_all();
    }
}

// queue `run` after the caller's work on `stream`; the request completes when it has run
int post(mi355x_comm *c, void *stream, std::function<int(hipStream_t)> run, mi355x_request **out)
{
    if (!out) return set_error(MI355X_ERR_ARG, "request pointer is NULL");
    *out = nullptr;
    if (!c->nb_stream) {
        DeviceGuard dg(c->device);
        MI_HIP(hipStreamCreateWithFlags(&c->nb_stream, hipStreamNonBlocking));
    }
    auto *r = new mi355x_request();
    hipError_t e = hipEventCreateWithFlags(&r->ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(r->ev, resolve_stream(stream));
    if (e != hipSuccess) {
        if (r->ev) (void)hipEventDestroy(r->ev);
        delete r;
        return set_error(MI355X_ERR_HIP, "event on the caller stream: %s", hipGetErrorString(e));
    }
    r->run = std::move(run);
    {
        std::lock_guard<std::mutex> g(c->q_mtx);
        if (!c->worker.joinable()) c->worker = std::thread(worker_main, c);
        c->queue.push_back(r);
        c->pending++;
    }
    c->q_cv.notify_all();
    *out = r;
    return MI355X_SUCCESS;
}


} // namespace mi355x
