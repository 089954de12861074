// vx_ctx.cpp — context lifetime, error reporting, stage profiling and the RCCL communicator.
#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cstring>

#include "vx_internal.hpp"

namespace vx {

int set_error(vx_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

int hip_fail(vx_ctx* c, hipError_t e, const char* what) {
    return set_error(c, VX_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

// Cross-context ordering events order work of one device: a device-scope release / acquire is
// all they need ($VX_EVENT_SYSTEM_FENCE=1 restores the default system-scope fences).
static const unsigned kSyncEventFlags = [] {
    const char* e = std::getenv("VX_EVENT_SYSTEM_FENCE");
    return (e && std::atoi(e) != 0) ? 0u : (unsigned)hipEventDisableSystemFence;
}();

static hipEvent_t get_event(vx_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    // timing only: no system-scope fences (nothing here needs host visibility of device memory;
    // the fences made every bracketed dispatch ~2 us longer than rocprofv3 sees it)
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

ProfScope::ProfScope(vx_ctx* c_, int st, hipStream_t on) : c(c_), stage(st), s(on ? on : c_->stream) {
    if (!c->prof || !((c->prof_mask >> st) & 1u)) return;
    a = get_event(c);
    if (a) (void)hipEventRecord(a, s);
}

ProfScope::~ProfScope() {
    if (!c->prof || !a) return;
    hipEvent_t b = get_event(c);
    if (!b) return;
    (void)hipEventRecord(b, s);
    c->pending.push_back({a, b, stage});
}

KTiming prof_kernel_events(vx_ctx* c, int stage) {
    KTiming t;
    if (!c->prof || !((c->prof_mask >> stage) & 1u)) return t;
    t.a = get_event(c);
    t.b = get_event(c);
    if (!t.a || !t.b) t.a = t.b = nullptr;
    return t;
}

void prof_kernel_done(vx_ctx* c, int stage, KTiming t) { c->pending.push_back({t.a, t.b, stage}); }

void prof_collect(vx_ctx* c) {
    for (auto& pe : c->pending) {
        float ms = 0.f;
        if (hipEventSynchronize(pe.b) == hipSuccess && hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            c->prof_ms[pe.stage] += ms;
            c->prof_n[pe.stage] += 1;
        }
        c->event_pool.push_back(pe.a);
        c->event_pool.push_back(pe.b);
    }
    c->pending.clear();
}

uint64_t next_serial() {
    static std::atomic<uint64_t> n{1};
    return n++;
}

// Capture-or-replay of one graph slot: exec == nullptr && !seen -> eager run (and remember);
// seen once -> capture + instantiate + launch; exec set -> launch.
static int graph_slot_run(vx_ctx* c, hipGraphExec_t& exec, bool& seen, int (*enqueue)(vx_ctx*, void*), void* arg) {
    if (exec) {
        ++c->graphs.launched;
        VX_HIP(c, hipGraphLaunch(exec, c->stream));
        return VX_OK;
    }
    if (!seen) {  // first sighting: eager (allocations happen outside any capture)
        seen = true;
        return enqueue(c, arg);
    }
    VX_HIP(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed));
    const int rc = enqueue(c, arg);
    hipGraph_t g = nullptr;
    const hipError_t ce = hipStreamEndCapture(c->stream, &g);
    hipGraphExec_t x = nullptr;
    hipError_t ie = hipErrorUnknown;
    if (rc == VX_OK && ce == hipSuccess && g) ie = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (rc != VX_OK) return rc;
    if (ie != hipSuccess) {  // not capturable here: stay eager from now on
        c->use_graphs = false;
        return enqueue(c, arg);
    }
    exec = x;
    ++c->graphs.captured;
    ++c->graphs.launched;
    VX_HIP(c, hipGraphLaunch(exec, c->stream));
    return VX_OK;
}

int graph_run(vx_ctx* c, const std::vector<uint64_t>& key, int (*enqueue)(vx_ctx*, void*), void* arg) {
    if (!c->use_graphs || c->prof) return enqueue(c, arg);
    GraphCache& gc = c->graphs;
    const uint64_t now = ++gc.tick;
    GraphCache::Entry* e = nullptr;
    for (auto& x : gc.entries)
        if (x.key == key) {
            e = &x;
            break;
        }
    if (!e) {
        constexpr size_t kMaxGraphs = 64;
        if (gc.entries.size() >= kMaxGraphs) {
            auto lru = std::min_element(gc.entries.begin(), gc.entries.end(),
                                        [](const GraphCache::Entry& a, const GraphCache::Entry& b) { return a.last < b.last; });
            if (lru->exec) (void)hipGraphExecDestroy(lru->exec);
            gc.entries.erase(lru);
        }
        gc.entries.push_back({key, nullptr, now});
        e = &gc.entries.back();
        bool seen = false;
        return graph_slot_run(c, e->exec, seen, enqueue, arg);
    }
    e->last = now;
    bool seen = true;
    return graph_slot_run(c, e->exec, seen, enqueue, arg);
}

int graph_run_owned(vx_ctx* c, OwnedGraph& g, int (*enqueue)(vx_ctx*, void*), void* arg) {
    if (!c->use_graphs || c->prof) return enqueue(c, arg);
    return graph_slot_run(c, g.exec, g.seen, enqueue, arg);
}

OwnedGraph::~OwnedGraph() {
    if (exec) (void)hipGraphExecDestroy(exec);
}

void OwnedGraph::reset() {
    if (exec) (void)hipGraphExecDestroy(exec);
    exec = nullptr;
    seen = false;
}

}  // namespace vx

static const char* kStageNames[vx::kStCount] = {
    "orb_gray",       "orb_resize",    "orb_fast_harris", "orb_select",  "orb_blur",
    "orb_describe",   "match_partial", "match_merge",     "ba_reset",    "ba_pose_partial",
    "ba_pose_sum",    "ba_allreduce",  "ba_pose_solve",   "ba_landmark",    "orb_pyramid",
    "sba_landmark",   "sba_blocks",    "sba_solve",       "sba_update",     "sba_allreduce",
    "lm_depth",       "lm_triangulate", "lm_compact",  "pnp_hypotheses", "pnp_refine",
    "em_hypotheses",  "em_select",     "ba_iter",         "ba_prologue",
    "ba_window"};

extern "C" {

int vx_version(void) { return 100; }

int vx_create(int device, vx_ctx** out) { return vx_create_ex(device, 0, nullptr, 0, out); }

int vx_device_cus(int device) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return -1;
    return n;
}

int vx_create_ex(int device, int priority, const uint32_t* cu_mask, int mask_words, vx_ctx** out) {
    if (!out) return VX_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return VX_ERR_HIP;
    if (device < 0 || device >= n) return VX_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return VX_ERR_HIP;
    auto* c = new vx_ctx();
    c->device = device;
    if (const char* f = std::getenv("VX_GRAPHS")) c->use_graphs = std::atoi(f) != 0;
    // one HIP stream per context (HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues, 4 by
    // default: streams beyond that share queues and serialise)
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    const hipError_t se =
        (cu_mask && mask_words > 0)
            ? hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask_words, cu_mask)
            : hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, priority > 0 ? greatest : least);
    if (se != hipSuccess) {
        vx_destroy(c);
        return VX_ERR_HIP;
    }
    *out = c;
    return VX_OK;
}

// (a 64-byte header records how the block was allocated: page-locked, or plain pageable memory when
// the runtime has no device to lock pages for — a host-only build or test still gets working arrays)
void* vx_host_alloc(size_t bytes) {
    constexpr size_t kHdr = 64;
    static const bool pageable = std::getenv("VX_HOST_PAGEABLE") != nullptr;  // (A/B switch)
    void* p = nullptr;
    uint32_t kind = 1;
    if (pageable || hipHostMalloc(&p, bytes + kHdr, hipHostMallocNonCoherent) != hipSuccess) {
        (void)hipGetLastError();
        p = std::aligned_alloc(kHdr, (bytes + 2 * kHdr - 1) / kHdr * kHdr);  // (64-byte aligned either way)
        kind = 2;
        if (!p) return nullptr;
    }
    *static_cast<uint32_t*>(p) = kind;
    return static_cast<uint8_t*>(p) + kHdr;
}

void vx_host_free(void* q) {
    if (!q) return;
    void* p = static_cast<uint8_t*>(q) - 64;
    if (*static_cast<uint32_t*>(p) == 1) (void)hipHostFree(p);
    else std::free(p);
}

void vx_destroy(vx_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->graphs.entries)
        if (e.exec) (void)hipGraphExecDestroy(e.exec);
    vx::prof_collect(c);
    if (c->snap_map) vx_dmap_destroy(c->snap_map);
    vx::plan_pool_release(c);
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    for (auto e : {c->order_event})
        if (e) (void)hipEventDestroy(e);
#ifndef VX_NO_RCCL
    if (c->comm) ncclCommDestroy(c->comm);
#endif
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* vx_last_error(const vx_ctx* c) { return c ? c->err.c_str() : "null context"; }

int vx_graph_enable(vx_ctx* c, int enable) {
    if (!c) return VX_ERR_INVALID;
    c->use_graphs = enable != 0;
    return VX_OK;
}

int vx_set_grid_share(vx_ctx* c, float share) {
    if (!c) return VX_ERR_INVALID;
    if (!(share > 0.0f && share <= 1.0f)) return vx::set_error(c, VX_ERR_INVALID, "grid share must be in (0, 1]");
    if (share == c->grid_share) return VX_OK;
    VX_HIP(c, hipSetDevice(c->device));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    // captured launch sequences bake the old grids in: drop them with the cached geometry
    for (auto& e : c->graphs.entries)
        if (e.exec) (void)hipGraphExecDestroy(e.exec);
    c->graphs.entries.clear();
    c->grid_share = share;
    c->geo_valid = false;
    return VX_OK;
}

int vx_graph_counts(const vx_ctx* c, int* captured, int* launched) {
    if (!c) return VX_ERR_INVALID;
    if (captured) *captured = c->graphs.captured;
    if (launched) *launched = c->graphs.launched;
    return VX_OK;
}

void* vx_stream(vx_ctx* c) { return c ? (void*)c->stream : nullptr; }

int vx_synchronize(vx_ctx* c) {
    if (!c) return VX_ERR_INVALID;
    VX_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) vx::prof_collect(c);
    return VX_OK;
}

int vx_stream_wait_ctx(vx_ctx* c, vx_ctx* after) {
    if (!c || !after) return VX_ERR_INVALID;
    if (c == after) return VX_OK;
    if (c->device != after->device)
        return vx::set_error(c, VX_ERR_INVALID, "vx_stream_wait_ctx: contexts on devices %d and %d", c->device,
                             after->device);
    if (!after->order_event)
        VX_HIP(c, hipEventCreateWithFlags(&after->order_event, hipEventDisableTiming | vx::kSyncEventFlags));
    VX_HIP(c, hipEventRecord(after->order_event, after->stream));
    VX_HIP(c, hipStreamWaitEvent(c->stream, after->order_event, 0));
    return VX_OK;
}

int vx_event_create(vx_ctx* c, vx_event** out) {
    if (!c || !out) return VX_ERR_INVALID;
    *out = nullptr;
    VX_HIP(c, hipSetDevice(c->device));
    auto* e = new vx_event();
    e->device = c->device;
    const hipError_t r = hipEventCreateWithFlags(&e->ev, hipEventDisableTiming | vx::kSyncEventFlags);
    if (r != hipSuccess) {
        delete e;
        return vx::hip_fail(c, r, "hipEventCreateWithFlags");
    }
    *out = e;
    return VX_OK;
}

int vx_event_record(vx_ctx* c, vx_event* e) {
    if (!c || !e) return VX_ERR_INVALID;
    if (e->device != c->device) return vx::set_error(c, VX_ERR_INVALID, "vx_event_record: event of device %d", e->device);
    VX_HIP(c, hipEventRecord(e->ev, c->stream));
    return VX_OK;
}

int vx_event_wait(vx_ctx* c, vx_event* e) {
    if (!c || !e) return VX_ERR_INVALID;
    if (e->device != c->device) return vx::set_error(c, VX_ERR_INVALID, "vx_event_wait: event of device %d", e->device);
    // an event whose work has already finished orders nothing: no barrier packet in the queue
    // (each costs the waiting stream a dependency-resolution bubble)
    if (hipEventQuery(e->ev) == hipSuccess) return VX_OK;
    VX_HIP(c, hipStreamWaitEvent(c->stream, e->ev, 0));
    return VX_OK;
}

void vx_event_destroy(vx_event* e) {
    if (!e) return;
    (void)hipEventDestroy(e->ev);
    delete e;
}

int vx_prof_enable(vx_ctx* c, int mask) {
    if (!c) return VX_ERR_INVALID;
    if (!mask) {
        (void)hipStreamSynchronize(c->stream);
        vx::prof_collect(c);
    }
    c->prof = mask != 0;
    c->prof_mask = (unsigned)mask;
    return VX_OK;
}

int vx_prof_count(void) { return vx::kStCount; }

const char* vx_prof_name(int s) { return (s >= 0 && s < vx::kStCount) ? kStageNames[s] : ""; }

int vx_prof_read(vx_ctx* c, double* ms, int64_t* launches, int reset) {
    if (!c) return VX_ERR_INVALID;
    VX_HIP(c, hipStreamSynchronize(c->stream));
    vx::prof_collect(c);
    for (int i = 0; i < vx::kStCount; ++i) {
        if (ms) ms[i] = c->prof_ms[i];
        if (launches) launches[i] = c->prof_n[i];
        if (reset) {
            c->prof_ms[i] = 0;
            c->prof_n[i] = 0;
        }
    }
    return VX_OK;
}

int vx_comm_unique_id(uint8_t* out) {
#ifndef VX_NO_RCCL
    if (!out) return VX_ERR_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return VX_ERR_COMM;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    std::memcpy(out, &id, 128);
    return VX_OK;
#else
    (void)out;
    return VX_ERR_COMM;
#endif
}

int vx_comm_init(vx_ctx* c, const uint8_t* id128, int nranks, int rank) {
    if (!c || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return VX_ERR_INVALID;
#ifndef VX_NO_RCCL
    VX_HIP(c, hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, id128, 128);
    if (c->comm) {
        ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess)
        return vx::set_error(c, VX_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
    c->nranks = nranks;
    c->rank = rank;
    return VX_OK;
#else
    return VX_ERR_COMM;
#endif
}

int vx_comm_info(vx_ctx* c, int* nranks, int* rank) {
    if (!c || !nranks || !rank) return VX_ERR_INVALID;
#ifndef VX_NO_RCCL
    if (!c->comm) return vx::set_error(c, VX_ERR_STATE, "vx_comm_info: no communicator (vx_comm_init)");
    ncclResult_t r = ncclCommCount(c->comm, nranks);
    if (r == ncclSuccess) r = ncclCommUserRank(c->comm, rank);
    if (r != ncclSuccess) return vx::set_error(c, VX_ERR_COMM, "ncclCommCount/UserRank: %s", ncclGetErrorString(r));
    return VX_OK;
#else
    return VX_ERR_COMM;
#endif
}

}  // extern "C"
