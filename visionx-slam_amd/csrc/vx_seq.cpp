// vx_seq.cpp — recorded enqueue sequences (vx_seq_*, include/vx_slam.h).
//
// A pipelined caller (bench.py's Extract | Match | LocalBA step over several contexts) issues, per
// frame, about eight C-ABI calls: event waits and records between the contexts and the three async
// entry points, each of which replays a captured hipGraph.  Through a language binding every call
// costs microseconds of host time on top of the HIP runtime's own.  A vx_seq records such a call
// list once, with every argument resolved, and vx_seq_run replays it from C: the same calls, in the
// same order, with the same device-side semantics (nothing is fused or reordered), so a whole step of
// F frames is one call from the binding.
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
};

namespace {
vx_seq::Op blank(vx_seq::Kind k, vx_ctx* c) {
    vx_seq::Op o{};
    o.kind = k;
    o.c = c;
    return o;
}
}  // namespace

extern "C" {

int vx_seq_create(vx_seq** out) {
    if (!out) return VX_ERR_INVALID;
    *out = new vx_seq();
    return VX_OK;
}

void vx_seq_destroy(vx_seq* s) { delete s; }

int vx_seq_wait(vx_seq* s, vx_ctx* c, vx_event* e) {
    if (!s || !c || !e) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kWait, c);
    o.ev = e;
    s->ops.push_back(o);
    return VX_OK;
}

int vx_seq_record(vx_seq* s, vx_ctx* c, vx_event* e) {
    if (!s || !c || !e) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kRecord, c);
    o.ev = e;
    s->ops.push_back(o);
    return VX_OK;
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
    s->ops.push_back(o);
    return VX_OK;
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
    s->ops.push_back(o);
    return VX_OK;
}

int vx_seq_ba_run(vx_seq* s, vx_ctx* c, vx_ba_plan* plan) {
    if (!s || !c || !plan) return VX_ERR_INVALID;
    auto o = blank(vx_seq::kBaRun, c);
    o.plan = plan;
    s->ops.push_back(o);
    return VX_OK;
}

int vx_seq_length(const vx_seq* s) { return s ? (int)s->ops.size() : VX_ERR_INVALID; }

int vx_seq_run(vx_seq* s, int* failed_op) {
    if (!s) return VX_ERR_INVALID;
    for (size_t i = 0; i < s->ops.size(); ++i) {
        const vx_seq::Op& o = s->ops[i];
        int rc = VX_OK;
        switch (o.kind) {
            case vx_seq::kWait: rc = vx_event_wait(o.c, o.ev); break;
            case vx_seq::kRecord: rc = vx_event_record(o.c, o.ev); break;
            case vx_seq::kExtract:
                rc = vx_orb_extract_async(o.c, &o.params, o.img, o.w, o.h, o.ch, o.stride, o.slot);
                break;
            case vx_seq::kMatch:
                rc = vx_match_device_async(o.c, o.q, o.nq, o.capq, o.t, o.nt, o.capt, o.ratio);
                break;
            case vx_seq::kBaRun: rc = vx_ba_plan_run_async(o.c, o.plan); break;
        }
        if (rc != VX_OK) {
            if (failed_op) *failed_op = (int)i;
            return rc;
        }
    }
    if (failed_op) *failed_op = -1;
    return VX_OK;
}

}  // extern "C"
