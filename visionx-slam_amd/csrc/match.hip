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
#include <algorithm>
#include <cstdlib>
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

// Whole-row kNN-2 (default): a workgroup takes kRQ queries against the whole train set, so no
// chunk partials go through memory and no merge launch follows.  The queries are wave-uniform (their
// 32 B each in SGPRs: every v_xor takes its query word as the scalar operand); thread tid holds train
// rows tid, tid + kRT, ... (4 in registers per pass) and keeps a top-2 per query; the top-2s are
// merged per query by one wave (LDS transpose, then DPP), then the ratio test.
// The merge of two lexicographic top-2s is exact in any order, so the result is the sequential
// scan's (the chunked kernels above stay for comparison: VX_MATCH_CHUNKED=1).
constexpr int kRQ = 8;     // queries per workgroup (default shape)
constexpr int kRT = 512;   // threads per workgroup (default shape)

__device__ __forceinline__ void top2_merge(unsigned& k1, unsigned& k2, unsigned o1, unsigned o2) {
    const unsigned n2 = min(max(k1, o1), min(k2, o2));
    k1 = min(k1, o1);
    k2 = n2;
}

// one DPP step of the top-2 reduction: merge with the pair `CTRL` moves here (lanes of rows outside
// ROWS, or without a source, merge the empty pair)
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ void top2_dpp(unsigned& k1, unsigned& k2) {
    const unsigned o1 = (unsigned)__builtin_amdgcn_update_dpp((int)kNone, (int)k1, CTRL, ROWS, 0xF, false);
    const unsigned o2 = (unsigned)__builtin_amdgcn_update_dpp((int)kNone, (int)k2, CTRL, ROWS, 0xF, false);
    top2_merge(k1, k2, o1, o2);
}

// RQ queries (wave-uniform operands) against the whole train set by RT threads; then the LDS
// transpose, each wave reducing RQ / (RT / 64) queries.  The workgroups take query groups
// blockIdx.x, blockIdx.x + gridDim.x, ... (a grid smaller than the capacity's query groups loops).
// nq / nt: the counts (device), nq_cap / nt_cap: the buffers' rows.  (Requesting the first
// operands before the counts arrive was measured in round 5: 5.2 us uncapped, 6.8 capped, no change
// in the pipeline — not kept.)
template <int RQ, int RT>
__device__ __forceinline__ void knn_rows(const uint8_t* __restrict__ q, const int* __restrict__ nq_p, int nq_cap,
                                         const uint8_t* __restrict__ t, const int* __restrict__ nt_p, int nt_cap,
                                         float ratio, unsigned* __restrict__ best, uint2 (*tr)[RT]) {
    constexpr int kW = RT / 64, kQPW = RQ / kW;
    static_assert(RQ % kW == 0, "k_knn_rows: whole queries per reducing wave");
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    auto load_q = [&](int q0, uint4 (&A0)[RQ], uint4 (&A1)[RQ], int lim) {
#pragma unroll
        for (int i = 0; i < RQ; ++i) {
            const int qi = min(q0 + i, lim - 1);  // (past the end: a row that is not written)
            A0[i] = reinterpret_cast<const uint4*>(q + (long long)qi * 32)[0];
            A1[i] = reinterpret_cast<const uint4*>(q + (long long)qi * 32)[1];
        }
    };
    uint4 A0[RQ], A1[RQ];
    const int nq = nq_p ? min(*nq_p, nq_cap) : nq_cap;
    const int nt = nt_p ? min(*nt_p, nt_cap) : nt_cap;
    for (int q0 = blockIdx.x * RQ; q0 < nq; q0 += gridDim.x * RQ) {  // (block-uniform)
    load_q(q0, A0, A1, nq);
    unsigned k1[RQ], k2[RQ];
#pragma unroll
    for (int i = 0; i < RQ; ++i) k1[i] = k2[i] = kNone;
    for (int r0 = tid; r0 < nt; r0 += 4 * RT) {
        uint4 B0[4], B1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = min(r0 + j * RT, nt - 1);
            B0[j] = reinterpret_cast<const uint4*>(t + (long long)row * 32)[0];
            B1[j] = reinterpret_cast<const uint4*>(t + (long long)row * 32)[1];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = r0 + j * RT;
            const unsigned tag = row < nt ? (unsigned)row : 0u;
#pragma unroll
            for (int i = 0; i < RQ; ++i) {
                unsigned d = __builtin_popcount(A0[i].x ^ B0[j].x);
                d += __builtin_popcount(A0[i].y ^ B0[j].y);
                d += __builtin_popcount(A0[i].z ^ B0[j].z);
                d += __builtin_popcount(A0[i].w ^ B0[j].w);
                d += __builtin_popcount(A1[i].x ^ B1[j].x);
                d += __builtin_popcount(A1[i].y ^ B1[j].y);
                d += __builtin_popcount(A1[i].z ^ B1[j].z);
                d += __builtin_popcount(A1[i].w ^ B1[j].w);
                const unsigned key = row < nt ? (d << 22) | tag : kNone;
                k2[i] = max(min(k1[i], key), min(k2[i], max(k1[i], key)));
                k1[i] = min(k1[i], key);
            }
        }
    }
    // transpose through LDS: wave w then reduces queries w * kQPW .. — RT / 64 entries per lane,
    // then the 64 lanes by DPP (xor 1, xor 2, half-row and row mirrors, row broadcasts 15 / 31:
    // lane 63 ends with all)
#pragma unroll
    for (int i = 0; i < RQ; ++i) tr[i][tid] = make_uint2(k1[i], k2[i]);
    __syncthreads();
#pragma unroll
    for (int qq = 0; qq < kQPW; ++qq) {
        const int qw = wv * kQPW + qq;
        unsigned a1 = kNone, a2 = kNone;
#pragma unroll
        for (int g = 0; g < RT / 64; ++g) {
            const uint2 v = tr[qw][64 * g + lane];
            top2_merge(a1, a2, v.x, v.y);
        }
        top2_dpp<0xB1>(a1, a2);        // quad_perm [1,0,3,2]
        top2_dpp<0x4E>(a1, a2);        // quad_perm [2,3,0,1]
        top2_dpp<0x141>(a1, a2);       // row_half_mirror
        top2_dpp<0x140>(a1, a2);       // row_mirror
        top2_dpp<0x142, 0xA>(a1, a2);  // row_bcast:15 into rows 1, 3
        top2_dpp<0x143, 0xC>(a1, a2);  // row_bcast:31 into rows 2, 3
        if (lane == 63 && q0 + qw < nq) {
            bool keep = false;
            if (a2 != kNone) {  // knn.size() == 2 (orb_matcher.cpp:28)
                const float d1 = (float)(a1 >> 22), d2 = (float)(a2 >> 22);
                keep = d1 < ratio * d2;  // orb_matcher.cpp:33
            }
            best[q0 + qw] = keep ? a1 : kNone;
        }
    }
    __syncthreads();  // (the next group's transpose overwrites tr)
    }
}

template <int RQ, int RT>
__global__ __launch_bounds__(RT) void k_knn_rows(const uint8_t* __restrict__ q, const int* __restrict__ nq_p,
                                                 int nq_host, const uint8_t* __restrict__ t,
                                                 const int* __restrict__ nt_p, int nt_host, float ratio,
                                                 unsigned* __restrict__ best) {
    __shared__ uint2 tr[RQ][RT];  // the threads' top-2s, query-major
    knn_rows<RQ, RT>(q, nq_p, nq_host, t, nt_p, nt_host, ratio, best, tr);
}

// Batched matching (vx_match_batch_async): pair blockIdx.y's sets from the table, per-pair results
// at best + pair * q_cap.
struct PairTab {
    const uint8_t* q[VX_MAX_MATCH_PAIRS];
    const int* nq[VX_MAX_MATCH_PAIRS];
    const uint8_t* t[VX_MAX_MATCH_PAIRS];
    const int* nt[VX_MAX_MATCH_PAIRS];
};

__global__ __launch_bounds__(kRT) void k_knn_rows_batch(PairTab tab, int q_cap, int t_cap, float ratio,
                                                        unsigned* __restrict__ best) {
    __shared__ uint2 tr[kRQ][kRT];
    const int p = blockIdx.y;
    knn_rows<kRQ, kRT>(tab.q[p], tab.nq[p], q_cap, tab.t[p], tab.nt[p], t_cap, ratio, best + (long long)p * q_cap, tr);
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
// nq_p: the device count (null: cap), cap: the results' capacity.  The first pass's entries are
// requested before the count arrives (entries below the capacity are valid memory; those past the
// count are dropped after): one dependent memory latency before the scan instead of two.
template <int NT>
__device__ __forceinline__ void knn_compact(const unsigned* __restrict__ best, const int* __restrict__ nq_p, int cap,
                                            vx_match* __restrict__ out, int* __restrict__ out_count, int* sh) {
    int written = 0;
    unsigned k0[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) k0[j] = 4 * (int)threadIdx.x + j < cap ? best[4 * threadIdx.x + j] : kNone;
    const int nq = nq_p ? min(*nq_p, cap) : cap;
    // 4 consecutive queries per thread (one pass up to 4 NT queries: one load latency, one scan)
    for (int base = 0; base < nq; base += 4 * NT) {
        const int q4 = base + 4 * threadIdx.x;
        unsigned k[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = q4 + j < nq ? (base == 0 ? k0[j] : best[q4 + j]) : kNone;
        int n4 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) n4 += k[j] != kNone;
        int cnt;
        int pos = written + scan_excl<NT>(n4, sh, cnt);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k[j] != kNone) {
                vx_match m;
                m.query_idx = q4 + j;
                m.train_idx = (int)(k[j] & 0x3fffffu);
                m.distance = (float)(k[j] >> 22);
                out[pos++] = m;
            }
        written += cnt;
    }
    if (threadIdx.x == 0) *out_count = written;
}

__global__ __launch_bounds__(kMergeBlock) void k_knn_compact(const unsigned* __restrict__ best,
                                                             const int* __restrict__ nq_p, int nq_host,
                                                             vx_match* __restrict__ out,
                                                             int* __restrict__ out_count) {
    __shared__ int sh[kMergeBlock / 64];
    knn_compact<kMergeBlock>(best, nq_p, nq_host, out, out_count, sh);
}

// one workgroup per pair: matches of pair p at out + p * q_cap, its count at out_count[4 p]
__global__ __launch_bounds__(kMergeBlock) void k_knn_compact_batch(const unsigned* __restrict__ best, PairTab tab,
                                                                   int q_cap, vx_match* __restrict__ out,
                                                                   int* __restrict__ out_count) {
    __shared__ int sh[kMergeBlock / 64];
    const int p = blockIdx.x;
    knn_compact<kMergeBlock>(best + (long long)p * q_cap, tab.nq[p], q_cap, out + (long long)p * q_cap,
                out_count + 4 * p, sh);
}

// k_knn_rows' shape: $VX_MATCH_SHAPE = "<queries>x<threads>" (8x512 default; 4x256, 16x512,
// 16x1024, 8x256, 4x128 for A/B runs) and $VX_MATCH_GRID = workgroups, read once.  The grid is capped at one
// workgroup per CU by default: the query count is on the device, so an uncapped grid ($VX_MATCH_GRID=0)
// is sized for the capacity and most of its workgroups only read the count and leave (C3's
// 2000-of-4254: 6.64 us uncapped, 4.92 us capped, profiles/r05/match_shapes.txt)
template <int RQ, int RT>
int knn_rows_launch_t(vx_ctx* c, const uint8_t* dq, const int* dnq, int nq_host, const uint8_t* dt, const int* dnt,
                      int nt_host, int q_cap, float ratio, unsigned* best, int grid_cap) {
    int g = (q_cap + RQ - 1) / RQ;
    if (grid_cap > 0) g = std::min(g, grid_cap);
    VX_HIP(c, launch(c, kStMatchPartial, k_knn_rows<RQ, RT>, dim3(std::max(g, 1)), dim3(RT), 0, c->stream, dq, dnq,
                     nq_host, dt, dnt, nt_host, ratio, best));
    return VX_OK;
}
int knn_rows_launch(vx_ctx* c, const uint8_t* dq, const int* dnq, int nq_host, const uint8_t* dt, const int* dnt,
                    int nt_host, int q_cap, float ratio, unsigned* best) {

    static const int shape = [] {
        const char* e = getenv("VX_MATCH_SHAPE");
        if (!e) return 0;
        const std::string v(e);
        return v == "4x256" ? 1 : v == "16x512" ? 2 : v == "16x1024" ? 3 : v == "8x256" ? 4 : v == "4x128" ? 5 : 0;
    }();
    static const int grid_env = [] {
        const char* e = getenv("VX_MATCH_GRID");
        return e ? atoi(e) : -1;
    }();
    if (!c->n_cus) c->n_cus = std::max(vx_device_cus(c->device), 1);
    const int grid_cap = grid_env >= 0 ? grid_env : c->n_cus;
    switch (shape) {
        case 1: return knn_rows_launch_t<4, 256>(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best, grid_cap);
        case 2: return knn_rows_launch_t<16, 512>(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best, grid_cap);
        case 3: return knn_rows_launch_t<16, 1024>(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best, grid_cap);
        case 4: return knn_rows_launch_t<8, 256>(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best, grid_cap);
        case 5: return knn_rows_launch_t<4, 128>(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best, grid_cap);
        default: return knn_rows_launch_t<kRQ, kRT>(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best, grid_cap);
    }
}

int match_enqueue(vx_ctx* c, const uint8_t* dq, const int* dnq, int nq_host, const uint8_t* dt,
                  const int* dnt, int nt_host, int q_cap, int t_cap, float ratio) {
    int rc;
    const int n_chunks = (t_cap + kTC - 1) / kTC;
    const int q_stride = q_cap;
    VX_HIP(c, c->partial.ensure((size_t)n_chunks * q_stride * sizeof(uint2) + (size_t)q_cap * sizeof(unsigned) + 16));
    VX_HIP(c, c->matches.ensure((size_t)std::max(q_cap, 1) * sizeof(vx_match)));
    VX_HIP(c, c->match_count.ensure(16));
    c->match_cap = q_cap;
    static const bool chunked = [] {
        const char* e = getenv("VX_MATCH_CHUNKED");
        return e && e[0] == '1';
    }();
    if (!chunked) {
        unsigned* best = reinterpret_cast<unsigned*>(c->partial.as<uint2>() + (size_t)n_chunks * q_stride);
        if ((rc = knn_rows_launch(c, dq, dnq, nq_host, dt, dnt, nt_host, q_cap, ratio, best))) return rc;
        ProfScope ps(c, kStMatchMerge);
        hipLaunchKernelGGL(k_knn_compact, dim3(1), dim3(kMergeBlock), 0, c->stream, best, dnq, nq_host,
                           c->matches.as<vx_match>(), c->match_count.as<int>());
        VX_LAUNCH_CHECK(c, "k_knn_compact");
        c->match_valid = true;
        return VX_OK;
    }
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

int match_batch_enqueue(vx_ctx* c, const PairTab& tab, int n_pairs, int q_cap, int t_cap, float ratio) {
    unsigned* best = c->mb_best.as<unsigned>();
    // (two workgroups per CU over all the pairs: capped as in knn_rows_launch, the pairs' query
    // groups looped over)
    if (!c->n_cus) c->n_cus = std::max(vx_device_cus(c->device), 1);
    const int gx = std::max(1, std::min((q_cap + kRQ - 1) / kRQ, 2 * c->n_cus / std::max(n_pairs, 1)));
    VX_HIP(c, launch(c, kStMatchPartial, k_knn_rows_batch, dim3(gx, n_pairs), dim3(kRT), 0,
                     c->stream, tab, q_cap, t_cap, ratio, best));
    ProfScope ps(c, kStMatchMerge);
    hipLaunchKernelGGL(k_knn_compact_batch, dim3(n_pairs), dim3(kMergeBlock), 0, c->stream, (const unsigned*)best, tab,
                       q_cap, c->mb_matches.as<vx_match>(), c->mb_count.as<int>());
    VX_LAUNCH_CHECK(c, "k_knn_compact_batch");
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

int vx_match_batch_async(vx_ctx* c, int n_pairs, const uint8_t* const* dq, const int32_t* const* dnq, int q_cap,
                         const uint8_t* const* dt, const int32_t* const* dnt, int t_cap, float ratio) {
    if (!c) return VX_ERR_INVALID;
    if (n_pairs < 1 || n_pairs > VX_MAX_MATCH_PAIRS)
        return set_error(c, VX_ERR_INVALID, "n_pairs %d outside [1, %d]", n_pairs, VX_MAX_MATCH_PAIRS);
    if (!dq || !dnq || !dt || !dnt || q_cap < 0 || t_cap < 0)
        return set_error(c, VX_ERR_INVALID, "vx_match_batch_async: null buffers or negative capacity");
    if (t_cap > (1 << 22)) return set_error(c, VX_ERR_INVALID, "train set larger than 2^22 rows");
    PairTab tab;
    std::memset(&tab, 0, sizeof tab);
    for (int i = 0; i < n_pairs; ++i) {
        if (!dq[i] || !dnq[i] || !dt[i] || !dnt[i])
            return set_error(c, VX_ERR_INVALID, "vx_match_batch_async: null buffers of pair %d", i);
        tab.q[i] = dq[i];
        tab.nq[i] = dnq[i];
        tab.t[i] = dt[i];
        tab.nt[i] = dnt[i];
    }
    VX_HIP(c, hipSetDevice(c->device));
    c->mb_valid = 0;
    const size_t qc = (size_t)std::max(q_cap, 1);
    VX_HIP(c, c->mb_best.ensure(n_pairs * qc * sizeof(unsigned)));
    VX_HIP(c, c->mb_matches.ensure(n_pairs * qc * sizeof(vx_match)));
    VX_HIP(c, c->mb_count.ensure((size_t)n_pairs * 16));
    if (q_cap > 0) {
        struct A {
            const PairTab* tab;
            int n, q_cap, t_cap;
            float ratio;
        } a{&tab, n_pairs, q_cap, t_cap, ratio};
        uint32_t rbits;
        std::memcpy(&rbits, &ratio, 4);
        std::vector<uint64_t> key{4, (uint64_t)n_pairs, (uint64_t)q_cap, (uint64_t)t_cap, rbits,
                                  (uint64_t)(uintptr_t)c->mb_best.p, (uint64_t)(uintptr_t)c->mb_matches.p,
                                  (uint64_t)(uintptr_t)c->mb_count.p};
        for (int i = 0; i < n_pairs; ++i)
            for (const void* v : {(const void*)dq[i], (const void*)dnq[i], (const void*)dt[i], (const void*)dnt[i]})
                key.push_back((uint64_t)(uintptr_t)v);
        const int rc = graph_run(c, key,
                                 [](vx_ctx* cc, void* v) {
                                     const A* x = static_cast<const A*>(v);
                                     return match_batch_enqueue(cc, *x->tab, x->n, x->q_cap, x->t_cap, x->ratio);
                                 },
                                 &a);
        if (rc) return rc;
    } else {
        VX_HIP(c, hipMemsetAsync(c->mb_count.p, 0, (size_t)n_pairs * 16, c->stream));
    }
    c->mb_valid = n_pairs;
    c->mb_cap = q_cap;
    return VX_OK;
}

int vx_match_knn2_ratio_batch(vx_ctx* c, int n_pairs, const uint8_t* const* q, const int32_t* nq,
                              const uint8_t* const* t, const int32_t* nt, float ratio) {
    if (!c) return VX_ERR_INVALID;
    if (n_pairs < 1 || n_pairs > VX_MAX_MATCH_PAIRS)
        return set_error(c, VX_ERR_INVALID, "n_pairs %d outside [1, %d]", n_pairs, VX_MAX_MATCH_PAIRS);
    if (!q || !nq || !t || !nt) return set_error(c, VX_ERR_INVALID, "vx_match_knn2_ratio_batch: null arrays");
    int q_cap = 0, t_cap = 0;
    for (int i = 0; i < n_pairs; ++i) {
        if (nq[i] < 0 || nt[i] < 0) return set_error(c, VX_ERR_INVALID, "negative descriptor count (pair %d)", i);
        if ((nq[i] && !q[i]) || (nt[i] && !t[i])) return set_error(c, VX_ERR_INVALID, "null descriptors (pair %d)", i);
        q_cap = std::max(q_cap, (int)nq[i]);
        t_cap = std::max(t_cap, (int)nt[i]);
    }
    if (t_cap > (1 << 22)) return set_error(c, VX_ERR_INVALID, "train set larger than 2^22 rows");
    VX_HIP(c, hipSetDevice(c->device));
    // every pair's rows and both counts staged in one pinned block and uploaded with one copy
    // (an empty side counts 0 rows: the pair yields no match, orb_matcher.cpp:18-20)
    const size_t qb = (size_t)std::max(q_cap, 1) * 32, tb = (size_t)std::max(t_cap, 1) * 32;
    const size_t cnt_off = (size_t)n_pairs * (qb + tb), total = cnt_off + (size_t)n_pairs * 8;
    VX_HIP(c, hipStreamSynchronize(c->stream));  // the staging block may still feed a previous copy
    VX_HIP(c, c->mb_host.ensure(total));
    VX_HIP(c, c->mb_in.ensure(total));
    uint8_t* H = static_cast<uint8_t*>(c->mb_host.p);
    int32_t* hc = reinterpret_cast<int32_t*>(H + cnt_off);
    for (int i = 0; i < n_pairs; ++i) {
        if (nq[i]) std::memcpy(H + i * qb, q[i], (size_t)nq[i] * 32);
        if (nt[i]) std::memcpy(H + n_pairs * qb + i * tb, t[i], (size_t)nt[i] * 32);
        hc[2 * i] = nq[i] && nt[i] ? nq[i] : 0;
        hc[2 * i + 1] = nq[i] && nt[i] ? nt[i] : 0;
    }
    VX_HIP(c, hipMemcpyAsync(c->mb_in.p, H, total, hipMemcpyHostToDevice, c->stream));
    const uint8_t* D = c->mb_in.as<uint8_t>();
    const int32_t* dc = reinterpret_cast<const int32_t*>(D + cnt_off);
    std::vector<const uint8_t*> dq(n_pairs), dt(n_pairs);
    std::vector<const int32_t*> dnq(n_pairs), dnt(n_pairs);
    for (int i = 0; i < n_pairs; ++i) {
        dq[i] = D + i * qb;
        dt[i] = D + n_pairs * qb + i * tb;
        dnq[i] = dc + 2 * i;
        dnt[i] = dc + 2 * i + 1;
    }
    return vx_match_batch_async(c, n_pairs, dq.data(), dnq.data(), q_cap, dt.data(), dnt.data(), t_cap, ratio);
}

int vx_match_batch_fetch(vx_ctx* c, int pair, vx_match* out, int cap, int* n_out) {
    if (!c || !n_out) return VX_ERR_INVALID;
    if (pair < 0 || pair >= c->mb_valid) return set_error(c, VX_ERR_STATE, "no batched match pair %d enqueued", pair);
    int n = 0;
    VX_HIP(c, hipMemcpyAsync(&n, c->mb_count.as<int>() + 4 * pair, sizeof n, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) prof_collect(c);
    *n_out = n;
    if (n > cap) return set_error(c, VX_ERR_CAPACITY, "need %d matches, cap %d", n, cap);
    if (n > 0 && out) {
        VX_HIP(c, hipMemcpyAsync(out, c->mb_matches.as<vx_match>() + (size_t)pair * std::max(c->mb_cap, 1),
                                 (size_t)n * sizeof(vx_match), hipMemcpyDeviceToHost, c->stream));
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
