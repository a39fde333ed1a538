// ipc_repro.hip -- the peer-mapping churn of tests/ipc_worker.py::rcache without the engine or
// torch: N processes on one GPU, each allocates K buffers per round (hipMalloc, distinct sizes),
// fills each with a word naming (rank, round, k), exports it (hipIpcGetMemHandle); every peer
// opens every handle (hipIpcOpenMemHandle) and reads the first and last word back.  Mappings are
// kept in a per-process LRU list and closed when the list exceeds BOUND (0: never during a round;
// all closed after the exporters freed the round's buffers).  Between rounds every process frees
// its buffers.  A wrong word names whose buffer the mapping really shows.
//   ipc_repro NPROC ROUNDS K BOUND [DEFER]   -> one JSON line; exit 1 on any wrong word or failed call
// DEFER=1: the LRU closes of one call happen at the start of the next, i.e. while the peers export
// their next buffers; DEFER=2: closes stay apart from exports, but a process frees its round's
// buffers while the peers that freed first already export the next round's (as a program that frees
// between collectives does).  UNCACHED=1: before the churn every process also exports an uncached
// region (hipDeviceMallocUncached, as the engine's LL and flag regions) that every peer keeps mapped
// (measurement / diagnosis tool, not part of the product)
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>

namespace {
constexpr int kMaxProc = 8;
struct Shared {
    std::atomic<int> count;
    std::atomic<int> gen;
    hipIpcMemHandle_t h[kMaxProc][2];
    std::atomic<int> wrong, failed;
    char first_error[kMaxProc][160];
};
Shared *g;
int nproc;

void barrier()
{
    const int gen = g->gen.load();
    if (g->count.fetch_add(1) + 1 == nproc) {
        g->count.store(0);
        g->gen.fetch_add(1);
    } else {
        while (g->gen.load() == gen) usleep(5);
    }
}

uint32_t word(int rank, int round, int k) { return 0x5a000000u | ((uint32_t)rank << 16) | ((uint32_t)round << 8) | (uint32_t)k; }

void note(int rank, const char *fmt, ...)
{
    if (g->first_error[rank][0]) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g->first_error[rank], sizeof(g->first_error[rank]), fmt, ap);
    va_end(ap);
}

struct Map {
    int peer, round, k;
    void *p;
};

int defer = 0;
int uncached = 0;

int run(int rank, int rounds, int K, int bound)
{
    if (hipSetDevice(0) != hipSuccess) return 1;
    std::deque<Map> lru;
    std::vector<void *> persistent;
    void *region = nullptr;
    if (uncached) {
        if (hipExtMallocWithFlags(&region, (size_t)4 << 20, hipDeviceMallocUncached) != hipSuccess ||
            hipIpcGetMemHandle(&g->h[rank][0], region) != hipSuccess) {
            note(rank, "uncached region");
            g->failed++;
            return 1;
        }
        barrier();
        for (int q = 0; q < nproc; ++q) {
            void *p = nullptr;
            if (q != rank && hipIpcOpenMemHandle(&p, g->h[q][0], hipIpcMemLazyEnablePeerAccess) == hipSuccess)
                persistent.push_back(p);
        }
        barrier();
    }
    for (int r = 0; r < rounds; ++r) {
        // torch's allocation pattern of tests/ipc_worker.py::rcache: call k allocates x and y of
        // 1 MiB + k * 2 MiB floats' bytes, rounded to 2 MiB segments; at k = 0 both share one
        // 2 MiB segment (the small pool)
        std::vector<void *> mine;
        for (int k = 0; k < K; ++k) {
            const size_t bytes = k == 0 ? ((size_t)2 << 20) : (size_t)(k + 1) * ((size_t)2 << 20);
            const int nb = k == 0 ? 1 : 2;
            while (defer == 1 && bound > 0 && (int)lru.size() > bound) {
                (void)hipIpcCloseMemHandle(lru.front().p);
                lru.pop_front();
            }
            for (int b = 0; b < nb; ++b) {
                void *p = nullptr;
                if (hipMalloc(&p, bytes) != hipSuccess ||
                    hipMemsetD32((hipDeviceptr_t)p, word(rank, r, k) | (uint32_t)b << 7, bytes / 4) != hipSuccess ||
                    hipDeviceSynchronize() != hipSuccess) {
                    note(rank, "alloc/fill r%d k%d", r, k);
                    g->failed++;
                    return 1;
                }
                mine.push_back(p);
                if (hipIpcGetMemHandle(&g->h[rank][b], p) != hipSuccess) {
                    note(rank, "hipIpcGetMemHandle r%d k%d: %s", r, k, hipGetErrorString(hipGetLastError()));
                    g->failed++;
                    memset(&g->h[rank][b], 0, sizeof(g->h[rank][b]));
                }
            }
            barrier();
            for (int q = 0; q < nproc; ++q) {
                if (q == rank) continue;
                for (int b = 0; b < nb; ++b) {
                    hipIpcMemHandle_t h = g->h[q][b];
                    void *p = nullptr;
                    if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                        note(rank, "hipIpcOpenMemHandle r%d k%d peer %d: %s", r, k, q, hipGetErrorString(hipGetLastError()));
                        g->failed++;
                        continue;
                    }
                    uint32_t w[2] = {0, 0};
                    if (hipMemcpy(&w[0], p, 4, hipMemcpyDeviceToHost) != hipSuccess ||
                        hipMemcpy(&w[1], (char *)p + bytes - 4, 4, hipMemcpyDeviceToHost) != hipSuccess) {
                        note(rank, "read r%d k%d peer %d", r, k, q);
                        g->failed++;
                    }
                    const uint32_t want = word(q, r, k) | (uint32_t)b << 7;
                    if (w[0] != want || w[1] != want) {
                        if (g->wrong++ < 1)
                            note(rank, "r%d k%d peer %d buf %d: read %08x/%08x (rank %u round %u k %u), want %08x", r, k, q, b,
                                 w[0], w[1], (w[0] >> 16) & 0xff, (w[0] >> 8) & 0xff, w[0] & 0x7f, want);
                    }
                    lru.push_back(Map{q, r, k, p});
                    while (defer != 1 && bound > 0 && (int)lru.size() > bound) {
                        (void)hipIpcCloseMemHandle(lru.front().p);
                        lru.pop_front();
                    }
                }
            }
            barrier();  // every peer has read my handle slots
        }
        barrier();
        for (void *p : mine) (void)hipFree(p);
        if (defer == 2) continue;  // (no barrier: the next round's exports overlap the peers' frees)
        barrier();  // every exporter freed its round
        if (bound == 0) {
            for (Map &m : lru) (void)hipIpcCloseMemHandle(m.p);
            lru.clear();
        }
        barrier();
    }
    for (Map &m : lru) (void)hipIpcCloseMemHandle(m.p);
    barrier();
    for (void *p : persistent) (void)hipIpcCloseMemHandle(p);
    barrier();
    if (region) (void)hipFree(region);
    return 0;
}
} // namespace

int main(int argc, char **argv)
{
    nproc = argc > 1 ? atoi(argv[1]) : 3;
    const int rounds = argc > 2 ? atoi(argv[2]) : 2;
    const int K = argc > 3 ? atoi(argv[3]) : 64;
    const int bound = argc > 4 ? atoi(argv[4]) : 16;
    defer = argc > 5 ? atoi(argv[5]) : 0;
    uncached = argc > 6 ? atoi(argv[6]) : 0;
    if (nproc < 2 || nproc > kMaxProc) return 2;
    g = (Shared *)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (g == MAP_FAILED) return 2;
    memset((void *)g, 0, sizeof(Shared));
    std::vector<pid_t> kids;
    for (int r = 1; r < nproc; ++r) {  // (forked before any HIP call)
        const pid_t pid = fork();
        if (pid == 0) _exit(run(r, rounds, K, bound));
        kids.push_back(pid);
    }
    int rc = run(0, rounds, K, bound);
    for (pid_t pid : kids) {
        int st = 0;
        waitpid(pid, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
    }
    printf("{\"tool\": \"ipc_repro\", \"nproc\": %d, \"rounds\": %d, \"k\": %d, \"bound\": %d, \"defer\": %d, \"uncached\": %d, \"wrong\": %d, \"failed\": %d",
           nproc, rounds, K, bound, defer, uncached, g->wrong.load(), g->failed.load());
    for (int r = 0; r < nproc; ++r)
        if (g->first_error[r][0]) printf(", \"rank%d\": \"%s\"", r, g->first_error[r]);
    printf("}\n");
    return (rc || g->wrong.load() || g->failed.load()) ? 1 : 0;
}
