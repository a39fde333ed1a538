// coll_rcache.cpp -- the bounded peer-mapping cache (mpool/rgpusm's registration cache):
// mapping peers' allocations and LRU eviction (split out of coll_comm.cpp).

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


// Bounded peer-mapping cache (mpool/rgpusm's rcache_size_limit with LRU eviction,
// mpool_rgpusm_component.c:92-100, mpool_rgpusm_module.c:104-120,396-419): when the hipIpc mappings
// of peers' allocations exceed rcache_max_maps (count) or rcache_limit (bytes), the least recently
// used ones that the current collective does not use, that no point-to-point read has pinned and
// that are not the communicator's own regions are closed.  Recency is a clock every use ticks --
// collective or point-to-point -- so the bounds hold in phases of point-to-point traffic alone
// (a mapping a point-to-point read made is evictable once the read has finished and unpinned it).  A mapping keeps the exporter's allocation
// alive on ROCm, so a long job that churns allocations would otherwise hold every freed block of
// every peer.  Both limits default to 0 = unlimited, as in the reference.  With a bound set, every
// allocation travels as a dmabuf fd (local_handle, via_dmabuf): see retire_map for why hipIpc
// mappings are not closed under churn; an evicted dmabuf import is asked for again (serve_fd).
// hipIpcCloseMemHandle in one process while a peer process exports (hipIpcGetMemHandle) or
// imports can hand that peer the wrong allocation -- a third rank's buffer through one rank's
// handle -- or fail the export / import with "invalid argument" (ROCm 7.2, dmabuf IPC mode;
// tools/ipc_repro.hip reproduces it with plain hipMalloc / hipIpc* calls and no engine:
// profiles/r05_ipc_close_race.jsonl).  So an evicted mapping is only retired in the mapping phase
// and closed in the next exchange's close window (exchange(): after every rank's exports, before
// anybody opens, then one more barrier).  A replaced mapping (same exporter base, new allocation
// id) is still closed at once: an import with the same handle words left open would be handed
// back by hipIpcOpenMemHandle instead of the new allocation.
// A dmabuf import (the route every allocation with a buffer object of its own takes under a bound)
// is released at once: the race is hipIpcCloseMemHandle's.  A hipIpc mapping waits for a close
// window however many accumulate: in a point-to-point-only phase they are closed at the next
// collective's exchange, never eagerly while peers export or import.
void retire_map(mi355x_comm *c, const PeerMap &m)
{
    if (m.ext) {
        PeerMap x = m;
        close_map(x);
        return;
    }
    c->retired_maps.push_back(m);
}

void flush_retired(mi355x_comm *c)
{
    std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);
    for (PeerMap &m : c->retired_maps) close_map(m);
    c->retired_maps.clear();
}

bool evictable(const mi355x_comm *c, const PeerMap &m, const PeerMap *keep)
{
    return &m != keep && !m.persistent && m.pins == 0 && m.coll_use != c->seq;
}

void rcache_trim(mi355x_comm *c, const PeerMap *keep)
{
    if (!c->rcache_max_maps && !c->rcache_limit) return;
    for (;;) {
        size_t nmaps = 0, bytes = 0;
        auto lru = c->peer_maps.end();
        for (auto it = c->peer_maps.begin(); it != c->peer_maps.end(); ++it) {
            if (it->second.persistent) continue;
            nmaps++;
            bytes += it->second.bytes;
            if (evictable(c, it->second, keep) && (lru == c->peer_maps.end() || it->second.last_use < lru->second.last_use))
                lru = it;
        }
        const bool over = (c->rcache_max_maps && nmaps > c->rcache_max_maps) || (c->rcache_limit && bytes > c->rcache_limit);
        if (!over || lru == c->peer_maps.end()) return;
        TRACE(c, "rcache: evict peer %d base %llx (%zu maps, %zu bytes)", lru->first.peer,
              (unsigned long long)lru->first.base, nmaps, bytes);
        retire_map(c, lru->second);
        c->peer_maps.erase(lru);
        c->rcache_evictions++;
    }
}

size_t peer_map_count(const mi355x_comm *c)
{
    size_t n = 0;
    for (const auto &kv : c->peer_maps) n += !kv.second.persistent;
    return n;
}

int map_peer(mi355x_comm *c, int peer, const BufDesc &d, void **out, PeerMap **entry, bool coll)
{
    std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);
    *out = nullptr;
    if (entry) *entry = nullptr;
    if (!d.present) return MI355X_SUCCESS;
    if (c->loopback) {
        *out = (void *)(uintptr_t)d.raw;
        return MI355X_SUCCESS;
    }
    HandleKey key;
    key.peer = peer;
    key.base = d.base;
    auto it = c->peer_maps.find(key);
    if (it != c->peer_maps.end() && (it->second.id != d.id || (d.id == 0 && it->second.pins == 0))) {
        if (it->second.ext) drop_stash(c, peer, it->second.id);  // the peer replaced that allocation
        TRACE(c, "replace peer %d base %llx: id %llu -> %llu (was at %p)", peer, (unsigned long long)d.base,
              (unsigned long long)it->second.id, (unsigned long long)d.id, it->second.mapped);
        close_map(it->second);  // (now: an import with the same handle words still open would be handed back)
        c->peer_maps.erase(it);
        it = c->peer_maps.end();
    }
    if (it == c->peer_maps.end() && d.dmabuf) {
        void *mapped = nullptr;
        hipExternalMemory_t ext = nullptr;
        int rc = import_dmabuf(c, peer, d.id, d.size, &mapped, &ext);
        if (rc) return rc;
        it = c->peer_maps.emplace(key, PeerMap{d.id, mapped, ++c->use_clock, ext}).first;
        it->second.bytes = d.size;
        if (coll) it->second.coll_use = c->seq;
        rcache_trim(c, &it->second);
    }
    void *base;
    if (it != c->peer_maps.end()) {
        base = it->second.mapped;
        it->second.last_use = ++c->use_clock;
        if (coll) it->second.coll_use = c->seq;
    } else {
        if (debug_on()) {
            uint32_t w[16];
            std::memcpy(w, &d.h, sizeof(w));
            TRACE(c, "open peer %d base %llx id %llu handle %08x %08x %08x %08x %08x %08x %08x %08x %08x %08x %08x %08x",
                  peer, (unsigned long long)d.base, (unsigned long long)d.id, w[0], w[1], w[2], w[3], w[4], w[5], w[6],
                  w[7], w[8], w[9], w[10], w[11]);
        }
        hipError_t e = hipIpcOpenMemHandle(&base, d.h, hipIpcMemLazyEnablePeerAccess);
        TRACE(c, "opened peer %d -> %p (%s)", peer, base, hipGetErrorString(e));
        if (e != hipSuccess) {
            // A mapping of an allocation the peer has since freed can still hold the block the new
            // allocation was carved from (small allocations share blocks): the open then fails
            // with "invalid device pointer".  This peer's mappings that the current call does not
            // use must go before one more try -- but closing hipIpc mappings while peers export or
            // import hands them wrong memory (retire_map), so inside a collective they are only
            // retired here and the exchange closes them in a window of its own (kOpenRetry);
            // point-to-point reads have no such window and close them at once.
            (void)hipGetLastError();
            int dropped = (int)c->retired_maps.size();
            for (auto m = c->peer_maps.begin(); m != c->peer_maps.end();) {
                if (m->first.peer == peer && m->second.coll_use != c->seq && m->second.pins == 0 &&
                    !m->second.persistent) {
                    retire_map(c, m->second);
                    m = c->peer_maps.erase(m);
                    dropped++;
                } else {
                    ++m;
                }
            }
            TRACE(c, "open failed; retired %d stale mappings of peer %d", dropped, peer);
            if (dropped && coll) return kOpenRetry;
            if (dropped) {  // (point-to-point: no window to wait for -- closed now, as before)
                flush_retired(c);
                e = hipIpcOpenMemHandle(&base, d.h, hipIpcMemLazyEnablePeerAccess);
            }
            if (e != hipSuccess)
                return set_error(MI355X_ERR_PEER, "hipIpcOpenMemHandle(rank %d): %s", peer, hipGetErrorString(e));
        }
        if (debug_on()) {
            for (const auto &kv : c->peer_maps) {  // a new mapping must not overlap a live one
                const uintptr_t a0 = (uintptr_t)kv.second.mapped, b0 = (uintptr_t)base;
                if (!kv.second.ext && a0 < b0 + d.size && b0 < a0 + kv.second.bytes)
                    TRACE(c, "ALIAS: peer %d base %llx id %llu mapped at %p overlaps peer %d base %llx id %llu at %p",
                          peer, (unsigned long long)d.base, (unsigned long long)d.id, base, kv.first.peer,
                          (unsigned long long)kv.first.base, (unsigned long long)kv.second.id, kv.second.mapped);
            }
        }
        it = c->peer_maps.emplace(key, PeerMap{d.id, base, ++c->use_clock, nullptr}).first;
        it->second.bytes = d.size;
        if (coll) it->second.coll_use = c->seq;
        rcache_trim(c, &it->second);
    }
    if (entry) *entry = &it->second;
    *out = (char *)base + d.off;
    return MI355X_SUCCESS;
}

} // namespace mi355x
