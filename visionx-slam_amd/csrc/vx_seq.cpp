// vx_seq.cpp — recorded enqueue sequences (vx_seq_*, include/vx_slam.h).
//
// A pipelined caller (bench.py's Extract | Match | LocalBA step over several contexts) issues, per
// frame, about eight C-ABI calls: event waits and records between the contexts and the three async
// entry points, each of which replays a captured hipGraph.  Through a language binding every call
// costs microseconds of host time on top of the HIP runtime's own.  A vx_seq records such a call
// list once, with every argument resolved, and vx_seq_run replays it from C: the same calls, in the
// same order, with the same device-side semantics (nothing is fused or reordered), so a whole step of
// F frames is one call from the binding.
//
// With vx_seq_set_threads(seq, n > 1) the replay is split by context: each context's calls run on
// a host thread of their own (contexts are single-threaded, so one context never has two), in their
// recorded order, and every cross-context edge of the recorded order that the device semantics depend
// on is kept on the host: a wait on an event is issued after the record of that event it follows in
// the sequence, and a record is issued only after every wait on the event's previous record (so no
// wait can see a later record than in the sequential replay).  Everything else on different
// contexts may be issued concurrently — which is what the sequential replay's streams see anyway.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "vx_internal.hpp"

struct vx_seq {
    enum Kind { kWait, kRecord, kExtract, kMatch, kBaRun };
    struct Op {
        Kind kind;
        vx_ctx* c;
        vx_event* ev;
        vx_orb_params params;
        const uint8_t* img;
        int w, h, ch, slot;
        int64_t stride;
        const uint8_t *q, *t;
        const int32_t *nq, *nt;
        int capq, capt;
        float ratio;
        vx_ba_plan* plan;
    };
    std::vector<Op> ops;

    // ---- parallel replay (threads > 1)
    int threads = 1;
    bool planned = false;
    std::vector<std::vector<int>> lanes;   // op indices per context, recorded order
    std::vector<std::vector<int>> deps;    // per op: ops (of other lanes) issued before it
    std::unique_ptr<std::atomic<uint64_t>[]> done;  // per op: run generation of its last issue
    std::vector<std::thread> workers;      // lanes 1.. (lane 0 runs on the caller)
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> go{0};           // run generation the workers should execute
    std::atomic<int> finished{0};
    std::atomic<int> err{0}, err_op{-1};
    bool stop = false;
    uint64_t gen = 0;

    // $VX_SEQ_TIMING=1: host time per op kind over the single-thread replays, printed at destroy
    bool timing = false;
    double t_kind[5] = {0, 0, 0, 0, 0};
    long long n_kind[5] = {0, 0, 0, 0, 0};
    ~vx_seq() {
        shutdown();
        if (timing) {
            static const char* names[5] = {"wait", "record", "extract", "match", "ba_run"};
            for (int k = 0; k < 5; ++k)
                if (n_kind[k])
                    std::fprintf(stderr, "[vx_seq] %-8s %9lld calls %8.2f us/call\n", names[k], n_kind[k],
                                 t_kind[k] / (double)n_kind[k]);
        }
    }
    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : workers) t.join();
        workers.clear();
        stop = false;
        planned = false;
    }
};

namespace {
vx_seq::Op blank(vx_seq::Kind k, vx_ctx* c) {
    vx_seq::Op o{};
    o.kind = k;
    o.c = c;
    return o;
}

int run_op(const vx_seq::Op& o) {
    switch (o.kind) {
        case vx_seq::kWait: return vx_event_wait(o.c, o.ev);
        case vx_seq::kRecord: return vx_event_record(o.c, o.ev);
        case vx_seq::kExtract: return vx_orb_extract_async(o.c, &o.params, o.img, o.w, o.h, o.ch, o.stride, o.slot);
        case vx_seq::kMatch: return vx_match_device_async(o.c, o.q, o.nq, o.capq, o.t, o.nt, o.capt, o.ratio);
        case vx_seq::kBaRun: return vx_ba_plan_run_async(o.c, o.plan);
    }
    return VX_ERR_INVALID;
}

// lanes by context and the host-side edges that keep every event's record / wait order
void plan_lanes(vx_seq* s) {
    const int n = (int)s->ops.size();
    std::unordered_map<vx_ctx*, int> lane_of;
    s->lanes.clear();
    std::vector<int> lane(n);
    for (int i = 0; i < n; ++i) {
        auto it = lane_of.find(s->ops[i].c);
        if (it == lane_of.end()) {
            it = lane_of.emplace(s->ops[i].c, (int)s->lanes.size()).first;
            s->lanes.emplace_back();
        }
        lane[i] = it->second;
        s->lanes[it->second].push_back(i);
    }
    s->deps.assign(n, {});
    std::unordered_map<vx_event*, int> last_rec;                 // event -> last record op so far
    std::unordered_map<vx_event*, std::vector<int>> waits_since;  // event -> waits after that record
    for (int i = 0; i < n; ++i) {
        const vx_seq::Op& o = s->ops[i];
        if (o.kind == vx_seq::kWait) {
            auto r = last_rec.find(o.ev);
            if (r != last_rec.end() && lane[r->second] != lane[i]) s->deps[i].push_back(r->second);
            waits_since[o.ev].push_back(i);
        } else if (o.kind == vx_seq::kRecord) {
            for (int w : waits_since[o.ev])
                if (lane[w] != lane[i]) s->deps[i].push_back(w);
            waits_since[o.ev].clear();
            last_rec[o.ev] = i;
        }
    }
    s->done.reset(new std::atomic<uint64_t>[n > 0 ? n : 1]);
    for (int i = 0; i < n; ++i) s->done[i].store(0, std::memory_order_relaxed);
    s->planned = true;
}

// one lane of run generation g; after a failure the lane's remaining ops are marked issued (so no
// other lane spins on them) and the first error is kept
void run_lane(vx_seq* s, int l, uint64_t g) {
    bool failed = false;
    for (int i : s->lanes[l]) {
        if (!failed) {
            for (int d : s->deps[i])
                while (s->done[d].load(std::memory_order_acquire) < g) {
                    if (s->err.load(std::memory_order_relaxed)) break;  // (a failed lane marks its ops)
                    std::this_thread::yield();
                }
            // another lane failed: its ops were marked issued without running, so this op's
            // cross-context order is no longer guaranteed — issue nothing more
            if (s->err.load(std::memory_order_acquire)) failed = true;
        }
        if (!failed) {
            const int rc = run_op(s->ops[i]);
            if (rc != VX_OK) {
                failed = true;
                int zero = 0;
                if (s->err.compare_exchange_strong(zero, rc)) s->err_op.store(i);
            }
        }
        s->done[i].store(g, std::memory_order_release);
    }
}

// seen: the run generation current when the worker was created (its first run is the next one)
void worker_main(vx_seq* s, int l, uint64_t seen) {
    (void)hipSetDevice(s->ops[s->lanes[l][0]].c->device);  // (the lane's device current on this thread)
    for (;;) {
        // spin briefly for the next run (the timed loop calls back to back), then sleep
        uint64_t g = s->go.load(std::memory_order_acquire);
        for (int spin = 0; g == seen && spin < 20000; ++spin) {
            std::this_thread::yield();
            g = s->go.load(std::memory_order_acquire);
        }
        if (g == seen) {
            std::unique_lock<std::mutex> lk(s->mu);
            s->cv.wait(lk, [&] { return s->stop || s->go.load(std::memory_order_acquire) != seen; });
            if (s->stop) return;
            g = s->go.load(std::memory_order_acquire);
        }
        seen = g;
        run_lane(s, l, g);
        s->finished.fetch_add(1, std::memory_order_acq_rel);
    }
}

int run_parallel(vx_seq* s, int* failed_op) {
    if (!s->planned) {
        s->shutdown();
        plan_lanes(s);
        const uint64_t cur = s->go.load(std::memory_order_acquire);
        for (int l = 1; l < (int)s->lanes.size(); ++l) s->workers.emplace_back(worker_main, s, l, cur);
    }
    const int nw = (int)s->lanes.size() - 1;
    const uint64_t g = ++s->gen;
    s->err.store(0);
    s->err_op.store(-1);
    s->finished.store(0, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> lk(s->mu);
        s->go.store(g, std::memory_order_release);
    }
    s->cv.notify_all();
    if (!s->lanes.empty()) run_lane(s, 0, g);
    while (s->finished.load(std::memory_order_acquire) < nw) std::this_thread::yield();
    if (failed_op) *failed_op = s->err_op.load();
    return s->err.load();
}
}  // namespace

extern "C" {

int vx_seq_create(vx_seq** out) {
    if (!out) return VX_ERR_INVALID;
    *out = new vx_seq();
    const char* e = std::getenv("VX_SEQ_TIMING");
    (*out)->timing = e && e[0] == '1';
    return VX_OK;
}

void vx_seq_destroy(vx_seq* s) { delete s; }

static int seq_push(vx_seq* s, const vx_seq::Op& o) {
    if (s->planned) s->shutdown();  // (lanes are re-planned at the next parallel run)
    s->ops.push_back(o);
    return VX_OK;
}

int vx_seq_wait(vx_seq* s, vx_ctx* c, vx_event* e) {
    if (!s || !c || !e) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kWait, c);
    o.ev = e;
    return seq_push(s, o);
}

int vx_seq_record(vx_seq* s, vx_ctx* c, vx_event* e) {
    if (!s || !c || !e) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kRecord, c);
    o.ev = e;
    return seq_push(s, o);
}

int vx_seq_extract(vx_seq* s, vx_ctx* c, const vx_orb_params* p, const uint8_t* d_img, int w, int h, int channels,
                   int64_t stride, int slot) {
    if (!s || !c || !p) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kExtract, c);
    o.params = *p;
    o.img = d_img;
    o.w = w;
    o.h = h;
    o.ch = channels;
    o.stride = stride;
    o.slot = slot;
    return seq_push(s, o);
}

int vx_seq_match(vx_seq* s, vx_ctx* c, const uint8_t* d_query, const int32_t* d_n_query, int cap_query,
                 const uint8_t* d_train, const int32_t* d_n_train, int cap_train, float ratio) {
    if (!s || !c) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kMatch, c);
    o.q = d_query;
    o.nq = d_n_query;
    o.capq = cap_query;
    o.t = d_train;
    o.nt = d_n_train;
    o.capt = cap_train;
    o.ratio = ratio;
    return seq_push(s, o);
}

int vx_seq_ba_run(vx_seq* s, vx_ctx* c, vx_ba_plan* plan) {
    if (!s || !c || !plan) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kBaRun, c);
    o.plan = plan;
    return seq_push(s, o);
}

int vx_seq_length(const vx_seq* s) { return s ? (int)s->ops.size() : VX_ERR_INVALID; }

int vx_seq_set_threads(vx_seq* s, int threads) {
    if (!s || threads < 1) return VX_ERR_INVALID;
    if (threads != s->threads) s->shutdown();
    s->threads = threads;
    return VX_OK;
}

int vx_seq_run(vx_seq* s, int* failed_op) {
    if (!s) return VX_ERR_INVALID;
    if (s->threads > 1) return run_parallel(s, failed_op);
    for (size_t i = 0; i < s->ops.size(); ++i) {
        if (s->timing) {
            const auto t0 = std::chrono::steady_clock::now();
            const int rc = run_op(s->ops[i]);
            s->t_kind[s->ops[i].kind] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            ++s->n_kind[s->ops[i].kind];
            if (rc != VX_OK) {
                if (failed_op) *failed_op = (int)i;
                return rc;
            }
            continue;
        }
        const int rc = run_op(s->ops[i]);
        if (rc != VX_OK) {
            if (failed_op) *failed_op = (int)i;
            return rc;
        }
    }
    if (failed_op) *failed_op = -1;
    return VX_OK;
}

}  // extern "C"
