// coll_selftest.cpp -- the flows' creation-time self-tests and the service's claim / setup
// (split out of coll_comm.cpp).

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

// ---- the flows' self-test.  Every cross-device flow that is on by default runs one short call on
// data that changes with the communicator (its secret) and the test, into a destination poisoned
// beforehand, and every rank checks its result exactly; the outcome is agreed in the control
// segment (every rank's mask ANDed, as the LL self-test agrees ll_ok) and a flow that failed on
// any rank is turned off on every rank -- its calls take the host-synchronised flows, whose
// coherence rests on kernel completion and a host barrier.  The reference negotiates CUDA IPC per
// peer pair the same way before using it, falling back to host staging (btl/smcuda/README:41-100,
// pml_ob1_cuda.c:183-210).  MI355X_SELFTEST_FAIL=<flow,...> (svc_ll, svc_pull, svc_copy, svc_rs,
// pipe) makes this rank report those flows failed (fault injection for tests); MI355X_SELFTEST=0
// skips the tests.
unsigned selftest_injected()
{
    const char *e = getenv("MI355X_SELFTEST_FAIL");
    if (!e) return 0;
    unsigned m = 0;
    const struct { const char *name; unsigned bit; } names[] = {{"svc_ll", MI355X_FLOW_SVC_LL}, {"svc_pull", MI355X_FLOW_SVC_PULL},
                                                                {"svc_copy", MI355X_FLOW_SVC_COPY}, {"svc_rs", MI355X_FLOW_SVC_RS},
                                                                {"pipe", MI355X_FLOW_PIPE}};
    std::string s(e);
    for (const auto &n : names)
        if (s.find(n.name) != std::string::npos) m |= n.bit;
    return m;
}

bool selftest_on(const mi355x_comm *c) { return c->selftest; }

uint32_t st_val(uint64_t seed, int q, size_t i)
{
    uint64_t x = seed ^ ((uint64_t)(q + 1) << 40) ^ ((uint64_t)i * 0x9e3779b97f4a7c15ull);
    x ^= x >> 31;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 29;
    return (uint32_t)(x & 0xffffff);  // (sums of <= 64 ranks stay below 2^31)
}

// restores the communicator's last_algorithm and pipelined-call count when a self-test that ran
// collectives of its own returns (its calls are not the caller's)
struct LastAlgKeeper {
    mi355x_comm *c;
    int alg;
    uint64_t pipe_calls = c->pipe_calls;
    ~LastAlgKeeper()
    {
        c->last_alg = alg;
        c->pipe_calls = pipe_calls;
    }
};

// device buffers of the self-test: my input (n x count int32 for the reduce_scatter block), output
struct SelfTest {
    mi355x_comm *c;
    uint64_t seed;
    char *in = nullptr, *out = nullptr;
    size_t cap = 0;
    bool ok = true;
    hipStream_t s = nullptr;  // setup_stream: the stream of the collective that runs the self-test
    SelfTest(mi355x_comm *c_, uint64_t salt, size_t bytes) : c(c_), cap(bytes)
    {
        seed = c->ctrl->secret ^ (salt * 0x632be59bd9b4e019ull);
        s = setup_stream(c);
        ok = hipMalloc((void **)&in, cap) == hipSuccess && hipMalloc((void **)&out, cap) == hipSuccess;
    }
    ~SelfTest()
    {
        if (in) (void)hipFree(in);
        if (out) (void)hipFree(out);
        (void)hipGetLastError();
    }
    // my input: `count` int32 of test `t`; the output poisoned
    bool prepare(int t, size_t count)
    {
        std::vector<uint32_t> h(count);
        for (size_t i = 0; i < count; ++i) h[i] = st_val(seed + (uint64_t)t, c->rank, i);
        return ok && count * 4 <= cap && hipMemcpyAsync(in, h.data(), count * 4, hipMemcpyHostToDevice, s) == hipSuccess &&
               hipMemsetAsync(out, 0xa5, cap, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
    }
    bool fetch(std::vector<uint32_t> &h, size_t count)
    {
        h.assign(count, 0);
        return hipMemcpyAsync(h.data(), out, count * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
               hipStreamSynchronize(s) == hipSuccess;
    }
    // element i of the SUM over every rank's input of test t
    uint32_t sum(int t, size_t i) const
    {
        uint32_t a = 0;
        for (int q = 0; q < c->size; ++q) a += st_val(seed + (uint64_t)t, q, i);
        return a;
    }
};

// agree on the masks every rank saw pass; returns the AND (collective)
int agree_flows(mi355x_comm *c, unsigned mine, unsigned *all)
{
    c->ctrl->slot[c->rank].flow_ok = mine;
    int rc = barrier(c);
    if (rc) return rc;
    unsigned a = ~0u;
    for (int q = 0; q < c->size; ++q) a &= c->ctrl->slot[q].flow_ok;
    *all = a;
    return barrier(c);  // nobody rewrites its word before every rank has read it
}


} // namespace mi355x

namespace mi355x {


// The service's flows, at its first claim (the service is claimed on every rank; collective).
int svc_selftest(mi355x_comm *c)
{
    LastAlgKeeper keep_alg{c, c->last_alg};  // (the test's own calls must not show in last_algorithm)
    c->svc_flows_tested = true;
    const unsigned tested = MI355X_FLOW_SVC_LL | MI355X_FLOW_SVC_PULL | MI355X_FLOW_SVC_COPY | MI355X_FLOW_SVC_RS;
    if (!selftest_on(c)) return MI355X_SUCCESS;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = c->size;
    // the flows' mechanisms at fixed sizes, whatever the limits are set to now; nothing forced
    struct Saved {
        size_t svc_max, pull, copy, one;
        bool rs, ok;
        int ar, red, rs_alg;
        const mi355x_rules_t *rules;
        double timeout;
        unsigned flows;
    } sv{c->svc_max, c->svc_pull_max, c->svc_copy_max, c->one_phase_max, c->svc_rs, c->svc_ok, c->knob_allreduce,
         c->knob_reduce, c->knob_rs, c->rules, c->timeout_s, c->flows};
    c->svc_max = 8192;
    c->svc_pull_max = c->svc_copy_max = 65536;
    c->one_phase_max = std::max<size_t>(c->one_phase_max, 65536);
    c->svc_rs = true;
    c->svc_ok = true;
    c->knob_allreduce = c->knob_reduce = c->knob_rs = 0;
    c->rules = nullptr;
    c->timeout_s = env_double("MI355X_LL_PROBE_S", 5.0);
    c->flows |= tested;
    unsigned pass = 0;
    {
        SelfTest st(c, c->svc_epoch, (size_t)n * 65536);
        const int i32 = MI355X_T_INT32, sum = MI355X_OP_SUM;
        std::vector<uint32_t> h;
        // a call of `flow` served by the service: exact, and the service served `calls` of them
        auto served = [&](uint64_t before, uint64_t calls) { return c->svc_calls - before == calls; };
        // LL form: an allgather and a reducing allreduce (granules pushed into every peer)
        {
            bool ok = st.prepare(1, 2048);
            const uint64_t b = c->svc_calls;
            ok = ok && allgather_impl(c, st.in, st.out, 8192, st.s) == MI355X_SUCCESS && st.fetch(h, 2048 * (size_t)n);
            for (int q = 0; q < n && ok; ++q)
                for (size_t i = 0; i < 2048 && ok; ++i) ok = h[(size_t)q * 2048 + i] == st_val(st.seed + 1, q, i);
            ok = ok && st.prepare(2, 2048) && allreduce_impl(c, st.in, st.out, 2048, i32, sum, st.s) == MI355X_SUCCESS &&
                 st.fetch(h, 2048);
            for (size_t i = 0; i < 2048 && ok; ++i) ok = h[i] == st.sum(2, i);
            if (ok && served(b, 2)) pass |= MI355X_FLOW_SVC_LL;
        }
        // pull form: a one-phase ring allreduce folded from the peers' mapped inputs
        if (pass & MI355X_FLOW_SVC_LL) {
            const size_t cnt = 12288;  // 48 KiB
            bool ok = st.prepare(3, cnt);
            const uint64_t b = c->svc_calls;
            ok = ok && allreduce_impl(c, st.in, st.out, cnt, i32, sum, st.s) == MI355X_SUCCESS && st.fetch(h, cnt);
            for (size_t i = 0; i < cnt && ok; ++i) ok = h[i] == st.sum(3, i);
            if (ok && served(b, 1)) pass |= MI355X_FLOW_SVC_PULL;
            // pull copies: allgather of every peer's block, bcast of the last rank's buffer
            ok = st.prepare(4, cnt);
            const uint64_t b2 = c->svc_calls;
            ok = ok && allgather_impl(c, st.in, st.out, cnt * 4, st.s) == MI355X_SUCCESS && st.fetch(h, cnt * (size_t)n);
            for (int q = 0; q < n && ok; ++q)
                for (size_t i = 0; i < cnt && ok; ++i) ok = h[(size_t)q * cnt + i] == st_val(st.seed + 4, q, i);
            ok = ok && st.prepare(5, cnt) && hipMemcpyAsync(st.out, st.in, cnt * 4, hipMemcpyDeviceToDevice, st.s) == hipSuccess &&
                 bcast_impl(c, st.out, cnt * 4, n - 1, st.s) == MI355X_SUCCESS && st.fetch(h, cnt);
            for (size_t i = 0; i < cnt && ok; ++i) ok = h[i] == st_val(st.seed + 5, n - 1, i);
            if (ok && served(b2, 2)) pass |= MI355X_FLOW_SVC_COPY;
            // reduce-scatter form: my 16 KiB block evaluated from the peers' mapped inputs
            const size_t rc_ = 4096;
            ok = st.prepare(6, rc_ * (size_t)n);
            const uint64_t b3 = c->svc_calls;
            ok = ok && reduce_scatter_block_impl(c, st.in, st.out, rc_, i32, sum, st.s) == MI355X_SUCCESS &&
                 st.fetch(h, rc_);
            for (size_t i = 0; i < rc_ && ok; ++i) ok = h[i] == st.sum(6, (size_t)c->rank * rc_ + i);
            if (ok && served(b3, 1)) pass |= MI355X_FLOW_SVC_RS;
        }
        (void)hipGetLastError();
    }
    pass &= ~selftest_injected();
    c->svc_max = sv.svc_max;
    c->svc_pull_max = sv.pull;
    c->svc_copy_max = sv.copy;
    c->one_phase_max = sv.one;
    c->svc_rs = sv.rs;
    c->svc_ok = sv.ok;
    c->knob_allreduce = sv.ar;
    c->knob_reduce = sv.red;
    c->knob_rs = sv.rs_alg;
    c->rules = sv.rules;
    c->timeout_s = sv.timeout;
    c->flows = sv.flows;
    unsigned all = 0;
    int rc = agree_flows(c, pass | ~tested, &all);
    if (rc) return rc;
    const unsigned failed = tested & ~all;
    c->flows &= ~failed;
    c->flows_failed |= failed;
    if (failed) {
        if (c->rank == 0)
            fprintf(stderr, "[mi355x] resident-service flow self-test failed (flows 0x%x): those calls take the "
                    "host-synchronised flows\n", failed);
        rc = ll_resync(c);
        if (rc) return rc;
    }
    c->selftest_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    TRACE(c, "service flow self-test: passed here 0x%x, agreed 0x%x", pass, all & tested);
    verdict_store(c);
    return MI355X_SUCCESS;
}

// The pipelined allreduce's per-chunk flag hand-off, at creation (multi-process, collective): one
// allreduce of 128 KiB blocks in 16 KiB chunks (8 per block), forced onto the pipelined flow.
int pipe_selftest(mi355x_comm *c)
{
    LastAlgKeeper keep_alg{c, c->last_alg};  // (the test's own calls must not show in last_algorithm)
    if (!selftest_on(c)) return MI355X_SUCCESS;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = c->size;
    const size_t count = (size_t)n * 32768;
    struct Saved {
        bool pipe, want;
        size_t one;
        int ar;
        const mi355x_rules_t *rules;
        double timeout;
    } sv{c->pipe_on, c->svc_want, c->one_phase_max, c->knob_allreduce, c->rules, c->timeout_s};
    c->pipe_on = true;
    c->svc_want = false;  // (no claim from inside this call, whatever the service limits are)
    c->one_phase_max = 0;
    c->knob_allreduce = AR_RING;
    c->rules = nullptr;
    c->pipe_chunk_override = 4096;
    c->timeout_s = env_double("MI355X_LL_PROBE_S", 5.0);
    unsigned pass = 0;
    bool admitted = false;
    {
        SelfTest st(c, 0x9e37u, count * 4);
        std::vector<uint32_t> h;
        const uint64_t refused = c->pipe_refused;
        bool ok = st.prepare(7, count) &&
                  allreduce_impl(c, st.in, st.out, count, MI355X_T_INT32, MI355X_OP_SUM, st.s) == MI355X_SUCCESS &&
                  st.fetch(h, count);
        for (size_t i = 0; i < count && ok; ++i) ok = h[i] == st.sum(7, i);
        admitted = c->pipe_refused == refused;
        if (ok) pass |= MI355X_FLOW_PIPE;
        (void)hipGetLastError();
    }
    c->pipe_on = sv.pipe;
    c->svc_want = sv.want;
    c->one_phase_max = sv.one;
    c->knob_allreduce = sv.ar;
    c->rules = sv.rules;
    c->timeout_s = sv.timeout;
    c->pipe_chunk_override = 0;
    pass &= ~selftest_injected();
    // not admitted (another communicator's grid held a GPU): the call ran two phases -- nothing
    // learnt about the flag hand-off, so it counts as untested, not failed (every rank agrees:
    // admission is agreed per call)
    unsigned all = 0;
    int rc = agree_flows(c, (pass | ~(unsigned)MI355X_FLOW_PIPE) | (admitted ? 0u : (unsigned)MI355X_FLOW_PIPE), &all);
    if (rc) return rc;
    c->pipe_untested = !admitted;
    if (!(all & MI355X_FLOW_PIPE)) {
        c->flows &= ~(unsigned)MI355X_FLOW_PIPE;
        c->flows_failed |= MI355X_FLOW_PIPE;
        c->pipe_on = false;
        if (c->rank == 0)
            fprintf(stderr, "[mi355x] pipelined allreduce self-test failed: large allreduces take the two-phase flow\n");
    }
    c->selftest_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    TRACE(c, "pipelined flow self-test: %s", !admitted ? "not admitted (untested)" : (all & MI355X_FLOW_PIPE) ? "ok" : "failed -> off");
    return MI355X_SUCCESS;
}

// Collective: claim the process's service for this communicator on every rank, or on none.  Called
// from a service-sized call on every rank alike (svc_maybe_claim).  A rank whose service another
// communicator owns takes it over if that owner has been idle long enough (svc_revoke).
int svc_claim(mi355x_comm *c)
{
    const auto t0 = std::chrono::steady_clock::now();
    int mine = 2;  // 1 claimed, 2 owned by a busy communicator, 3 the service cannot run here
    {
        std::lock_guard<std::mutex> g(g_svc_mtx);
        auto it = g_svc_owner.find(c->device);
        const bool free_ = it == g_svc_owner.end() || it->second == c;
        if (free_ || svc_revoke(it->second)) {
            if (it != g_svc_owner.end()) g_svc_owner.erase(it);  // (a revoked owner is no owner any more)
            if (!svc_attach(c)) {
                mine = 3;
            } else {
                g_svc_owner[c->device] = c;
                c->svc_owner = true;
                mine = 1;
            }
        }
    }
    c->ctrl->slot[c->rank].svc_claim = mine;
    int rc = barrier(c);
    if (rc) return rc;
    bool all = true, broken = false;
    for (int q = 0; q < c->size; ++q) {
        all = all && c->ctrl->slot[q].svc_claim == 1;
        broken = broken || c->ctrl->slot[q].svc_claim == 3;
    }
    rc = barrier(c);  // every rank has read the claims before they are rewritten
    if (rc) return rc;
    if (!all) {
        if (mine == 1) svc_let_go(c);
        if (broken) {
            c->svc_want = false;  // the service cannot run on some rank: stop trying (every rank saw it)
            if (c->rank == 0) fprintf(stderr, "[mi355x] resident LL service unavailable: small collectives use the per-call paths\n");
        }
        TRACE(c, "service claim: %s", broken ? "unavailable" : "owned by another communicator on some rank");
        return MI355X_SUCCESS;
    }
    c->svc_epoch++;
    c->ctrl->slot[c->rank].svc_last_ns.store(mono_ns(), std::memory_order_relaxed);
    if (!c->svc_flows_tested) {
        rc = svc_selftest(c);
        if (rc) return rc;
    }
    if (!(c->flows & MI355X_FLOW_SVC_LL)) {
        svc_let_go(c);
        c->svc_want = false;
        return MI355X_SUCCESS;
    }
    c->svc_ok = true;
    TRACE(c, "service claimed (epoch %llu) in %.0f us", (unsigned long long)c->svc_epoch,
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return MI355X_SUCCESS;
}

// at a service-sized call: claim the service if this communicator does not have it (every
// svc_retry-th such call; the same decision on every rank: sizes and agreed state only)
int svc_maybe_claim(mi355x_comm *c, bool sized)
{
    if (c->svc_ok || !c->svc_want || !sized) return MI355X_SUCCESS;
    if (c->svc_tries++ % c->svc_retry != 0) return MI355X_SUCCESS;
    return svc_claim(c);
}

// ---- flow verdicts reused across communicators.  The self-tests above check mechanisms between
// processes and GPUs -- IPC-mapped LL regions, flag hand-offs over xGMI, the resident service's
// forms -- not anything of one communicator, so a communicator whose members are the same processes
// on the same GPUs as an earlier one (an MPI_Comm_dup, a split that keeps the group) takes the
// earlier verdicts over instead of running the tests again (31.7 ms at 2 ranks, 71 ms at 8,
// profiles/r05_lazy_setup.txt).  Key: the sorted set of (device uid, pid, process start time) of
// the members; every rank publishes a hash of the verdicts it holds for the key, and they are
// reused only if every rank holds the same ones -- so a flow that failed anywhere stays off for
// the dup as well.
struct FlowVerdict {
    bool ll_ok = false;
    unsigned flows = 0, failed = 0;  // MI355X_FLOW_* agreed on / turned off
    bool pipe_tested = false, svc_tested = false;
};
static std::mutex g_verdict_mtx;
static std::map<std::string, FlowVerdict> g_verdicts;

static std::string member_key(const mi355x_comm *c)
{
    std::vector<std::array<uint64_t, 3>> m;
    for (int q = 0; q < c->size; ++q) {
        const RankSlot &r = c->ctrl->slot[q];
        m.push_back({r.dev_uid, (uint64_t)(uint32_t)r.pid, r.pid_start});
    }
    std::sort(m.begin(), m.end());
    std::string k;
    char b[64];
    for (const auto &e : m) {
        snprintf(b, sizeof(b), "%llx:%llx:%llx;", (unsigned long long)e[0], (unsigned long long)e[1],
                 (unsigned long long)e[2]);
        k += b;
    }
    return k;
}

static uint64_t verdict_hash(const std::string &key, const FlowVerdict &v)
{
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
    for (char ch : key) mix((unsigned char)ch);
    mix(v.ll_ok);
    mix(v.flows);
    mix(v.failed);
    mix(v.pipe_tested);
    mix(v.svc_tested);
    return h | 1;  // (0 means "none")
}

// record this communicator's verdicts (after its tests; every rank of it records the same)
void verdict_store(mi355x_comm *c)
{
    if (c->size < 2 || c->loopback || !selftest_on(c)) return;
    FlowVerdict v;
    v.ll_ok = c->ll_ok;
    v.flows = c->flows;
    v.failed = c->flows_failed;
    v.pipe_tested = !c->pipe_untested;
    v.svc_tested = c->svc_flows_tested;
    std::lock_guard<std::mutex> g(g_verdict_mtx);
    g_verdicts[member_key(c)] = v;
}

// collective: take over verdicts every rank holds for this member set; true if taken
static int verdict_reuse(mi355x_comm *c, FlowVerdict *out, bool *reused)
{
    *reused = false;
    if (!selftest_on(c) || env_double("MI355X_SELFTEST_REUSE", 1.0) == 0.0) return MI355X_SUCCESS;
    const std::string key = member_key(c);
    FlowVerdict v;
    bool have = false;
    {
        std::lock_guard<std::mutex> g(g_verdict_mtx);
        auto it = g_verdicts.find(key);
        if (it != g_verdicts.end()) {
            v = it->second;
            have = true;
        }
    }
    const uint64_t h = have ? verdict_hash(key, v) : 0;
    c->ctrl->slot[c->rank].verdict.store(h, std::memory_order_release);
    int rc = barrier(c);
    if (rc) return rc;
    bool all = h != 0;
    for (int q = 0; q < c->size && all; ++q) all = c->ctrl->slot[q].verdict.load(std::memory_order_acquire) == h;
    rc = barrier(c);  // every rank has read the hashes before they are rewritten
    if (rc) return rc;
    if (all) {
        *out = v;
        *reused = true;
    }
    return MI355X_SUCCESS;
}

// at creation: the service's settings (the claim itself waits for a service-sized call)
// The communicator's device-side setup: the completion words, the LL region and its self-test, the
// service's resources and the pipelined flow's self-test, with their allocations.  Deferred from
// mi355x_comm_create to the first device-buffer collective, as smcuda checks CUDA IPC support
// "lazily, when the first GPU access occurs, rather than during MPI_Init() time"
// (btl/smcuda/README:36-40): a communicator that only ever moves host buffers (a dup for a host
// library, a split used for bookkeeping) costs one barrier and no device memory.  Collective:
// every rank reaches it in the same call, because every collective entry calls it before its
// first step and collectives are called in the same order on every rank.  Knobs set before it
// (preset) are applied once the self-tests have decided what this communicator may use.
int dev_setup(mi355x_comm *c)
{
    if (c->dev_ready) return MI355X_SUCCESS;
    c->dev_ready = true;  // (the self-tests below run collectives themselves)
    if (c->size < 2 || c->loopback) return MI355X_SUCCESS;
    const auto t0 = std::chrono::steady_clock::now();
    int rc = setup_done_words(c);
    FlowVerdict v;
    bool reused = false;
    if (rc == MI355X_SUCCESS) rc = verdict_reuse(c, &v, &reused);
    if (rc == MI355X_SUCCESS && reused) {
        // an earlier communicator of these processes tested the flows: its verdicts, no tests
        c->ll_ok = v.ll_ok;
        if (c->ll_ok) rc = ensure_ll(c);
        else c->ll_max = 0;
        const unsigned tested = MI355X_FLOW_PIPE | (v.svc_tested ? (unsigned)(MI355X_FLOW_SVC_LL | MI355X_FLOW_SVC_PULL |
                                                                              MI355X_FLOW_SVC_COPY | MI355X_FLOW_SVC_RS)
                                                                   : 0u);
        c->flows = (c->flows & ~tested) | (v.flows & tested);
        c->flows_failed |= v.failed & tested;
        c->pipe_untested = !v.pipe_tested;
        if (!(c->flows & MI355X_FLOW_PIPE)) c->pipe_on = false;
        c->svc_flows_tested = v.svc_tested;
        c->selftest_reused = v.svc_tested ? 2 : 1;
        if (rc == MI355X_SUCCESS) svc_setup(c);
        TRACE(c, "device setup: flow verdicts of an earlier communicator of these processes reused (flows 0x%x)", c->flows);
    } else {
        if (rc == MI355X_SUCCESS) rc = ll_selftest(c);
        if (rc == MI355X_SUCCESS) {
            svc_setup(c);
            rc = pipe_selftest(c);
        }
        if (rc == MI355X_SUCCESS) verdict_store(c);
    }
    std::vector<std::pair<int, long>> pre;
    pre.swap(c->preset);
    for (const auto &kv : pre)
        if (rc == MI355X_SUCCESS) rc = mi355x_comm_set(c, kv.first, kv.second);
    c->setup_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    TRACE(c, "device setup: %.0f us, rc %d", c->setup_us, rc);
    return rc;
}

void svc_setup(mi355x_comm *c)
{
    c->svc_max = (size_t)std::max(0.0, env_double("MI355X_SVC_MAX_BYTES", (double)c->svc_max));
    c->svc_idle_s = std::max(0.0001, env_double("MI355X_SVC_IDLE_MS", c->svc_idle_s * 1e3) * 1e-3);
    c->svc_shrink_s = std::max(0.0, env_double("MI355X_SVC_SHRINK_US", c->svc_shrink_s * 1e6) * 1e-6);
    c->svc_nwg = (int)std::min(64.0, std::max(1.0, env_double("MI355X_SVC_WGS", (double)c->svc_nwg)));
    c->svc_pull_max = (size_t)std::max(0.0, env_double("MI355X_SVC_PULL_MAX_BYTES", (double)c->svc_pull_max));
    c->svc_copy_max = (size_t)std::max(0.0, env_double("MI355X_SVC_PULL_COPY_MAX_BYTES", (double)c->svc_copy_max));
    c->svc_rs = env_double("MI355X_SVC_RS", c->svc_rs ? 1.0 : 0.0) != 0.0;
    c->svc_handover_s = std::max(0.0, env_double("MI355X_SVC_HANDOVER_MS", c->svc_handover_s * 1e3) * 1e-3);
    c->svc_retry = (uint64_t)std::max(1.0, env_double("MI355X_SVC_RETRY_CALLS", (double)c->svc_retry));
    const char *env = getenv("MI355X_SVC");
    c->svc_want = c->ll_ok && c->size <= kLLMaxRanks && !c->loopback && !(env && atoi(env) == 0);
    // The service's resources (its HSA queue above all) are created now, not at the first claim:
    // an idle HSA queue in the process changes how the GPU schedules the HIP queues of several
    // processes sharing it -- the host-synchronised small allreduce / allgather of 4 ranks on one
    // GPU takes 20 us with it and 55 us without (profiles/r04_host_flow_idle_queue.jsonl: the
    // queue alone, without any dispatch, makes the difference; hsa_init, a probe launch or a signal
    // alone do not).  MI355X_SVC_EAGER=0 defers them to the first claim; MI355X_SVC_PREP=<mask>
    // repeats the experiment (1 hsa_init, 2 probe launch, 8 a bare queue, 16 a signal).
    if (c->svc_want && env_double("MI355X_SVC_EAGER", 1.0) != 0.0) {
        std::lock_guard<std::mutex> g(g_svc_mtx);
        if (!g_svc_res[c->device].q && svc_attach(c)) svc_detach(c);
    }
    const int prep = (int)env_double("MI355X_SVC_PREP", 0.0);
    if (prep & ~4) (void)svc_prep(c->device, prep);
}

} // namespace mi355x
