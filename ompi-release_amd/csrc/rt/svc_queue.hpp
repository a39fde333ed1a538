// svc_queue.hpp -- the resident LL service's private HSA queue (svc_queue.cpp).
#pragma once

#include <cstdint>
#include <string>

#include "coll_internal.hpp"

namespace mi355x {

struct SvcQueue {
    void *queue;             // hsa_queue_t *
    uint64_t signal;         // completion signal of the resident launch (1 while resident)
    uint64_t agent;          // hsa_agent_t of the HIP device
    uint64_t kernel_object;  // mi355x_k_svc's kernel descriptor
    uint32_t kernarg_bytes, group_bytes, private_bytes;
    void *kernarg;           // pinned host memory
    bool hsa_inited;
};

// one HIP launch of the service kernel that returns at once (coll_svc.hip): HIP then has the
// code object loaded on `device`
int svc_probe_launch(int device);
int svc_prep(int device, int mask);  // (experiment: parts of the service's creation alone)
// 0 on success; on failure `why` names the step (the service then stays off)
int svc_queue_create(int device, SvcQueue *q, std::string *why);
// dispatch nwg workgroups of the service; -1 if the previous launch is still resident
int svc_dispatch(SvcQueue *q, const SvcArgs &args, int nwg);
bool svc_resident(const SvcQueue *q);
bool svc_wait_exit(const SvcQueue *q, double seconds);  // true once the launch has left
void svc_queue_destroy(SvcQueue *q);
// the doorbell page: fine-grained device memory the host may store into (large-BAR mapping,
// *device = true), else pinned host memory; the same address serves host and kernel
int svc_page_alloc(SvcQueue *q, size_t bytes, void **p, bool *device);
void svc_page_free(void *p, bool device);

} // namespace mi355x
