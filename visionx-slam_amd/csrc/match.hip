// match.hip — brute-force Hamming kNN-2 + ratio test on gfx950 (FeatureMatcher::Match drop-in).
//
// Replaces ORBMatcher::Match (core/feature/orb_matcher.cpp:11-43): BFMatcher(NORM_HAMMING)
// knnMatch(desc_last, desc_curr, k = 2) then keep knn[0] when m1.distance < nn_ratio *
// m2.distance.  OpenCV's top-K insertion keeps, per query, the two smallest (distance, train
// index) pairs in lexicographic order (ties -> lower train index).  That order is
// a total order, so the GPU splits the train set into chunks, keeps a per-(query, chunk) top-2
// of packed keys (distance << 22 | train index) and merges chunks with the same min/med3
// update — bit-identical to the sequential scan whatever the chunking.
//
//   k_knn_partial  one thread per query (32 B in 8 VGPRs), a chunk of train rows staged in LDS
//                  and read as wave-uniform broadcasts; per pair 8 v_xor + 8 v_bcnt + 2 v_min/
//                  v_med3: VALU-popcount bound.
//   k_knn_merge    one block: merge chunk partials, ratio test, ordered compaction (ascending
//                  query index) by block scan.
#include <cstring>

#include "vx_internal.hpp"

namespace vx {
namespace {

constexpr int kQB = 256;      // queries per block (one per thread)
constexpr int kTC = 64;       // train rows per chunk
constexpr int kMergeBlock = 1024;
constexpr int kMergeBatch = 32;   // chunk partials in flight per thread in k_knn_merge
constexpr int kMergeQB = 64;      // queries per k_knn_merge workgroup (one wave: more CUs, same loads)
constexpr unsigned kNone = 0xffffffffu;

__global__ __launch_bounds__(kQB) void k_knn_partial(const uint8_t* __restrict__ q,
                                                     const int* __restrict__ nq_p, int nq_host,
                                                     const uint8_t* __restrict__ t,
                                                     const int* __restrict__ nt_p, int nt_host,
                                                     int n_chunks_cap, uint2* __restrict__ partial,
                                                     int q_stride) {
    __shared__ uint4 st[kTC * 2];
    const int nq = nq_p ? min(*nq_p, nq_host) : nq_host;  // device count clamped to capacity
    const int nt = nt_p ? min(*nt_p, nt_host) : nt_host;
    const int chunk = blockIdx.y;
    const int t0 = chunk * kTC;
    const int qi = blockIdx.x * kQB + threadIdx.x;
    if (blockIdx.x * kQB >= nq || t0 >= nt) return;  // block-uniform
    const int tn = min(kTC, nt - t0);
    for (int i = threadIdx.x; i < tn * 2; i += kQB)
        st[i] = reinterpret_cast<const uint4*>(t + (long long)t0 * 32)[i];
    __syncthreads();
    if (qi >= nq) return;
    const uint4 a0 = reinterpret_cast<const uint4*>(q + (long long)qi * 32)[0];
    const uint4 a1 = reinterpret_cast<const uint4*>(q + (long long)qi * 32)[1];
    unsigned k1 = kNone, k2 = kNone;
#pragma unroll 8
    for (int j = 0; j < tn; ++j) {
        const uint4 b0 = st[2 * j], b1 = st[2 * j + 1];
        unsigned d = __builtin_popcount(a0.x ^ b0.x);
        d += __builtin_popcount(a0.y ^ b0.y);
        d += __builtin_popcount(a0.z ^ b0.z);
        d += __builtin_popcount(a0.w ^ b0.w);
        d += __builtin_popcount(a1.x ^ b1.x);
        d += __builtin_popcount(a1.y ^ b1.y);
        d += __builtin_popcount(a1.z ^ b1.z);
        d += __builtin_popcount(a1.w ^ b1.w);
        const unsigned key = (d << 22) | (unsigned)(t0 + j);
        k2 = max(min(k1, key), min(k2, max(k1, key)));  // second smallest of {k1, k2, key}
        k1 = min(k1, key);
    }
    partial[(long long)chunk * q_stride + qi] = make_uint2(k1, k2);
    (void)n_chunks_cap;
}

// Exclusive block scan: wave prefix by __shfl_up, then the NT/64 wave totals from LDS (two
// barriers per call instead of a Hillis-Steele pass per doubling step).
template <int NT>
__device__ __forceinline__ int scan_excl(int v, int* sh, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        const int t = sh[i];
        tot += t;
        pre += i < w ? t : 0;
    }
    total = tot;
    __syncthreads();
    return pre + x - v;
}

// Per-query merge of the chunk partials + ratio test, one thread per query over many blocks.
// best[qi] = winning key when the query passes the ratio test, kNone otherwise.
__global__ __launch_bounds__(kMergeQB) void k_knn_merge(const uint2* __restrict__ partial,
                                                   const int* __restrict__ nq_p, int nq_host,
                                                   const int* __restrict__ nt_p, int nt_host,
                                                   int q_stride, float ratio,
                                                   unsigned* __restrict__ best) {
    const int nq = nq_p ? min(*nq_p, nq_host) : nq_host;
    const int nt = nt_p ? min(*nt_p, nt_host) : nt_host;
    const int qi = blockIdx.x * kMergeQB + threadIdx.x;
    if (qi >= nq) return;
    const int nchunks = (nt + kTC - 1) / kTC;
    unsigned k1 = kNone, k2 = kNone;
    // the chunk partials of a batch are loaded together (one exposed L2 latency per kMergeBatch
    // chunks, not per chunk); the merge order is the chunk order either way
    for (int c0 = 0; c0 < nchunks; c0 += kMergeBatch) {
        uint2 p[kMergeBatch];
#pragma unroll
        for (int j = 0; j < kMergeBatch; ++j)
            p[j] = c0 + j < nchunks ? partial[(long long)(c0 + j) * q_stride + qi] : make_uint2(kNone, kNone);
#pragma unroll
        for (int j = 0; j < kMergeBatch; ++j) {
            k2 = max(min(k1, p[j].x), min(k2, max(k1, p[j].x)));
            k1 = min(k1, p[j].x);
            k2 = max(min(k1, p[j].y), min(k2, max(k1, p[j].y)));
            k1 = min(k1, p[j].y);
        }
    }
    bool keep = false;
    if (k2 != kNone) {  // knn.size() == 2 (orb_matcher.cpp:28)
        const float d1 = (float)(k1 >> 22), d2 = (float)(k2 >> 22);
        keep = d1 < ratio * d2;  // orb_matcher.cpp:33
    }
    best[qi] = keep ? k1 : kNone;
}

// Ordered compaction (ascending query index) of the per-query results, one block.
__global__ __launch_bounds__(kMergeBlock) void k_knn_compact(const unsigned* __restrict__ best,
                                                             const int* __restrict__ nq_p, int nq_host,
                                                             vx_match* __restrict__ out,
                                                             int* __restrict__ out_count) {
    __shared__ int sh[kMergeBlock / 64];
    const int nq = nq_p ? min(*nq_p, nq_host) : nq_host;
    int written = 0;
    for (int base = 0; base < nq; base += kMergeBlock) {
        const int qi = base + threadIdx.x;
        const unsigned k1 = qi < nq ? best[qi] : kNone;
        const int keep = k1 != kNone;
        int cnt;
        const int pos = scan_excl<kMergeBlock>(keep, sh, cnt);
        if (keep) {
            vx_match m;
            m.query_idx = qi;
            m.train_idx = (int)(k1 & 0x3fffffu);
            m.distance = (float)(k1 >> 22);
            out[written + pos] = m;
        }
        written += cnt;
    }
    if (threadIdx.x == 0) *out_count = written;
}

int match_enqueue(vx_ctx* c, const uint8_t* dq, const int* dnq, int nq_host, const uint8_t* dt,
                  const int* dnt, int nt_host, int q_cap, int t_cap, float ratio) {
    const int n_chunks = (t_cap + kTC - 1) / kTC;
    const int q_stride = q_cap;
    VX_HIP(c, c->partial.ensure((size_t)n_chunks * q_stride * sizeof(uint2) + (size_t)q_cap * sizeof(unsigned) + 16));
    VX_HIP(c, c->matches.ensure((size_t)std::max(q_cap, 1) * sizeof(vx_match)));
    VX_HIP(c, c->match_count.ensure(16));
    c->match_cap = q_cap;
    VX_HIP(c, launch(c, kStMatchPartial, k_knn_partial, dim3((q_cap + kQB - 1) / kQB, n_chunks), dim3(kQB), 0,
                     c->stream, dq, dnq, nq_host, dt, dnt, nt_host, n_chunks, c->partial.as<uint2>(), q_stride));
    {
        ProfScope ps(c, kStMatchMerge);
        unsigned* best = reinterpret_cast<unsigned*>(c->partial.as<uint2>() + (size_t)n_chunks * q_stride);
        hipLaunchKernelGGL(k_knn_merge, dim3((q_cap + kMergeQB - 1) / kMergeQB), dim3(kMergeQB), 0, c->stream, c->partial.as<uint2>(),
                           dnq, nq_host, dnt, nt_host, q_stride, ratio, best);
        VX_LAUNCH_CHECK(c, "k_knn_merge");
        hipLaunchKernelGGL(k_knn_compact, dim3(1), dim3(kMergeBlock), 0, c->stream, best, dnq, nq_host,
                           c->matches.as<vx_match>(), c->match_count.as<int>());
        VX_LAUNCH_CHECK(c, "k_knn_compact");
    }
    c->match_valid = true;
    return VX_OK;
}

}  // namespace
}  // namespace vx

using namespace vx;

extern "C" {

int vx_match_slots_async(vx_ctx* c, int qs, int ts, float ratio) {
    if (!c) return VX_ERR_INVALID;
    if (qs < 0 || qs >= VX_MAX_SLOTS || ts < 0 || ts >= VX_MAX_SLOTS || !c->slots[qs].valid ||
        !c->slots[ts].valid)
        return set_error(c, VX_ERR_STATE, "match slots %d/%d hold no extraction", qs, ts);
    const Slot& a = c->slots[qs];
    const Slot& b = c->slots[ts];
    return match_enqueue(c, a.desc.as<uint8_t>(), a.count.as<int>(), a.cap, b.desc.as<uint8_t>(),
                         b.count.as<int>(), b.cap, a.cap, b.cap, ratio);
}

int vx_match_device_async(vx_ctx* c, const uint8_t* dq, const int32_t* dnq, int q_cap, const uint8_t* dt,
                          const int32_t* dnt, int t_cap, float ratio) {
    if (!c) return VX_ERR_INVALID;
    if (!dq || !dnq || !dt || !dnt || q_cap < 0 || t_cap < 0)
        return set_error(c, VX_ERR_INVALID, "vx_match_device_async: null buffers or negative capacity");
    if (t_cap > (1 << 22)) return set_error(c, VX_ERR_INVALID, "train set larger than 2^22 rows");
    VX_HIP(c, hipSetDevice(c->device));
    struct A {
        const uint8_t *dq, *dt;
        const int32_t *dnq, *dnt;
        int q_cap, t_cap;
        float ratio;
    } a{dq, dt, dnq, dnt, q_cap, t_cap, ratio};
    uint32_t rbits;
    std::memcpy(&rbits, &ratio, 4);
    // the buffers match_enqueue bakes into the graph are part of the key (they grow on demand)
    return graph_run(c, {2, (uint64_t)(uintptr_t)dq, (uint64_t)(uintptr_t)dnq, (uint64_t)q_cap, (uint64_t)(uintptr_t)dt,
                         (uint64_t)(uintptr_t)dnt, (uint64_t)t_cap, rbits, (uint64_t)(uintptr_t)c->partial.p,
                         (uint64_t)(uintptr_t)c->matches.p, (uint64_t)(uintptr_t)c->match_count.p},
                     [](vx_ctx* cc, void* v) {
                         const A* x = static_cast<const A*>(v);
                         return match_enqueue(cc, x->dq, x->dnq, x->q_cap, x->dt, x->dnt, x->t_cap, x->q_cap, x->t_cap,
                                              x->ratio);
                     },
                     &a);
}

int vx_match_fetch(vx_ctx* c, vx_match* out, int cap, int* n_out) {
    if (!c || !n_out) return VX_ERR_INVALID;
    if (!c->match_valid) return set_error(c, VX_ERR_STATE, "no match enqueued");
    int n = 0;
    VX_HIP(c, hipMemcpyAsync(&n, c->match_count.p, sizeof n, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) prof_collect(c);
    *n_out = n;
    if (n > cap) return set_error(c, VX_ERR_CAPACITY, "need %d matches, cap %d", n, cap);
    if (n > 0 && out) {
        VX_HIP(c, hipMemcpyAsync(out, c->matches.p, (size_t)n * sizeof(vx_match), hipMemcpyDeviceToHost,
                                 c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));
    }
    return VX_OK;
}

int vx_match_knn2_ratio(vx_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, float ratio,
                        vx_match* out, int cap, int* n_out) {
    if (!c || !n_out) return VX_ERR_INVALID;
    *n_out = 0;
    if (nq < 0 || nt < 0) return set_error(c, VX_ERR_INVALID, "negative descriptor count");
    if (nq == 0 || nt == 0) return VX_OK;  // desc1.empty() || desc2.empty() -> 0 (orb_matcher.cpp:18-20)
    if (!q || !t) return set_error(c, VX_ERR_INVALID, "null descriptors");
    if (nt > (1 << 22)) return set_error(c, VX_ERR_INVALID, "train set larger than 2^22 rows");
    VX_HIP(c, hipSetDevice(c->device));
    VX_HIP(c, c->mq.ensure((size_t)nq * 32));
    VX_HIP(c, c->mt.ensure((size_t)nt * 32));
    VX_HIP(c, hipMemcpyAsync(c->mq.p, q, (size_t)nq * 32, hipMemcpyHostToDevice, c->stream));
    VX_HIP(c, hipMemcpyAsync(c->mt.p, t, (size_t)nt * 32, hipMemcpyHostToDevice, c->stream));
    int rc = match_enqueue(c, c->mq.as<uint8_t>(), nullptr, nq, c->mt.as<uint8_t>(), nullptr, nt, nq, nt, ratio);
    if (rc) return rc;
    return vx_match_fetch(c, out, cap, n_out);
}

}  // extern "C"
