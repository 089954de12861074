// ba_fused_build.hip — the fused LocalBA layout (the tables k_ba_iter reads, ba.hip) built on the
// device from the plan's device CSRs (the per-keyframe build of LocalBA's
// problem, local_ba.cpp:42-108, is paid on every LocalBA::Optimize call).
//
// The host builder (ba.hip build_fused) is the specification: optimised landmarks in a stable order
// by first window keyframe, a greedy packing into workgroups of at most `cap` landmarks, `cap`
// landmark-stage observations and kBaFusedK keyframes, keyframe owners, per-workgroup keyframe entries
// with their pose observations in wave-major, 64-aligned order and the per-keyframe partial slots.
// Every step here produces the same tables byte for byte (tests/test_gpu_fused_build.py):
//   * first keyframe + keyframe bit set of every landmark (atomics over both observation lists), a
//     stable radix sort (rocPRIM) by first keyframe;
//   * the greedy packing as a chain: next(i) = where a workgroup starting at sorted landmark i ends
//     (one thread per i, the landmarks ahead staged in LDS; the greedy's state resets at every break,
//     so next(i) depends on i alone), then one workgroup walks 0 -> next(0) -> ... through LDS
//     windows of next[] (nb dependent LDS reads instead of n_opt greedy steps on the host);
//   * per workgroup its keyframe set (OR of its landmarks' sets; sorted = bit order), owners by
//     atomicMin; per keyframe one wave ranks its pose observations by workgroup in observation order
//     (ballot per distinct workgroup), giving entry sizes, positions and partial-slot ranks;
//   * per workgroup the wave-major entry offsets, a scan for the global bases, then the tables.
// Two small read-backs (the workgroup count; the padded pose-observation count and the largest
// slot count) size the buffers.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "vx_sort.hpp"

#include "ba_plan.hpp"

namespace vx {
namespace {

constexpr int kT = 256;
constexpr int kFK = kBaFusedK;
constexpr int kMaxW = (kBaMaxKfLds + 63) / 64;  // 64-bit words of a keyframe set
constexpr int kChainWin = 12288;                 // next[] window of the chain walk (ints of LDS)
constexpr int kMaxGroupsRank = kFusedMaxGroups;  // workgroup counters of k_fb_pose_rank (LDS)
constexpr int kMaxWaves = kBaFTLarge / 64;
static_assert(kBaFTLarge <= kChainWin / 2, "the chain walk advances at most cap landmarks per step");

inline unsigned grid(long long n) { return (unsigned)std::max(1ll, (n + kT - 1) / kT); }
enum : int { kFailObs = 1, kFailLmKf = 2, kFailOwnerKf = 4 };
// counters[]: 0 workgroups, 1 failure flags, 2 largest slot count of a keyframe
typedef unsigned long long u64;

__device__ __forceinline__ int popc_below(const u64* m, int W, int k) {
    int r = 0;
#pragma unroll
    for (int w = 0; w < kMaxW; ++w)
        if (w < W) {
            if (w < (k >> 6)) r += __popcll(m[w]);
            else if (w == (k >> 6)) r += __popcll(m[w] & ((1ull << (k & 63)) - 1));
        }
    return r;
}

__global__ void k_fb_init(int n_opt, int nk, int W, int* key, int* iota, u64* mask, int* owner, int* counters) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < 16) counters[i] = i < 4 ? 0 : -1;  // ([4..5]: the stop-rule workgroup's key, atomicMin)
    if (i < n_opt) {
        key[i] = nk;
        iota[i] = i;
        for (int w = 0; w < W; ++w) mask[(size_t)i * W + w] = 0;
    }
    if (i < nk) owner[i] = INT_MAX;
}

// keyframe row of each pose observation (kf_obs_ptr is keyframe-major)
__global__ void k_fb_pkf(const int* kptr, int nk, int n_pose, int* pkf) {
    const int o = blockIdx.x * kT + threadIdx.x;
    if (o >= n_pose) return;
    int lo = 0, hi = nk;  // kptr[lo] <= o < kptr[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (kptr[mid] <= o) lo = mid;
        else hi = mid;
    }
    pkf[o] = lo;
}

// first keyframe and keyframe set of every optimised landmark, over its landmark-stage and its
// pose-stage observations (build_fused: key[q], uk)
__global__ void k_fb_mask(int n_lobs, const int* llm, const int* lkf, int n_pose, const int* plm, const int* pkf,
                          int n_opt, int W, int* key, u64* mask) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n_lobs) {
        const int q = llm[i], k = lkf[i];
        atomicOr(&mask[(size_t)q * W + (k >> 6)], 1ull << (k & 63));
        atomicMin(&key[q], k);
    }
    if (i < n_pose && plm[i] < n_opt) {
        const int q = plm[i], k = pkf[i];
        atomicOr(&mask[(size_t)q * W + (k >> 6)], 1ull << (k & 63));
        atomicMin(&key[q], k);
    }
}

// sorted-order copies of the observation counts and keyframe sets; the landmarks that can never
// fit a workgroup (more observations than threads, more keyframes than entries)
__global__ void k_fb_sorted(const int* order, const int* firstS, int n_opt, const int* lptr, const u64* mask, int W,
                            int ft, int* cntS, u64* maskS, int* counters) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i == 0) cntS[n_opt] = 0;
    if (i >= n_opt) return;
    const int q = order[i];
    const int c = lptr[q + 1] - lptr[q];
    cntS[i] = c;
    int pc = 0, last = -1;
    for (int w = 0; w < W; ++w) {
        const u64 m = mask[(size_t)q * W + w];
        maskS[(size_t)i * W + w] = m;
        pc += __popcll(m);
        if (m) last = 64 * w + 63 - __clzll((long long)m);
    }
    int f = 0;
    if (c > ft) f |= kFailObs;
    if (pc > kFK) f |= kFailLmKf;
    if (f) atomicOr(&counters[1], f);
    if (last >= 0) atomicMax(&counters[3], last - firstS[i]);  // widest keyframe span of a landmark
}

// next[i]: the end of the greedy workgroup that starts at sorted landmark i (build_fused step 2:
// break before a landmark when the group is non-empty and one more landmark, its observations or its
// new keyframes would exceed cap, cap, kFK).  The landmarks i .. i + cap - 1 of the block's threads
// are staged in LDS (observation prefix sums, first keyframes, keyframe sets).  The landmark and
// observation caps alone give an end j1 by binary search over the prefix sums; the keyframe cap
// cannot bind before j1 when every keyframe of [i, j1) lies in [first(i), first(j1 - 1) + span]
// (landmarks sorted by first keyframe; span = the widest landmark, counters[3]) spans at most kFK
// rows — otherwise the thread replays the greedy over the staged sets.
__global__ __launch_bounds__(kT) void k_fb_next(const int* cntScan, const int* firstS, const u64* maskS, int n_opt,
                                               int W, int cap, const int* counters, int* next) {
    extern __shared__ u64 fb_lds[];
    const int span_cap = kT + cap;
    u64* mL = fb_lds;                                                 // [W][span_cap]
    int* cs = reinterpret_cast<int*>(fb_lds + (size_t)W * span_cap);  // [span_cap + 1]
    int* fs = cs + span_cap + 1;                                      // [span_cap]
    const int base = blockIdx.x * kT;
    const int span = min(n_opt - base, span_cap);
    for (int i = threadIdx.x; i <= span; i += kT) {
        cs[i] = cntScan[base + i];
        if (i < span) {
            fs[i] = firstS[base + i];
            for (int w = 0; w < W; ++w) mL[(size_t)w * span_cap + i] = maskS[(size_t)(base + i) * W + w];
        }
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (base + t >= n_opt) return;
    const int hi = min(t + cap, span);
    int lo = t + 1, h = hi;  // smallest j in (t, hi) whose observations overflow the group, else hi
    while (lo < h) {
        const int mid = (lo + h) >> 1;
        if (cs[mid + 1] - cs[t] > cap) h = mid;
        else lo = mid + 1;
    }
    const int j1 = lo;
    if (fs[j1 - 1] + counters[3] - fs[t] + 1 <= kFK) {
        next[base + t] = base + j1;
        return;
    }
    u64 cur[kMaxW];
#pragma unroll
    for (int w = 0; w < kMaxW; ++w) cur[w] = 0;
    int nl = 0, no = 0, kc = 0, i = t;
    for (; i < span; ++i) {
        if (nl >= cap) break;
        const int c = cs[i + 1] - cs[i];
        u64 m[kMaxW];
        int nn = 0;
#pragma unroll
        for (int w = 0; w < kMaxW; ++w) {
            m[w] = w < W ? mL[(size_t)w * span_cap + i] : 0;
            nn += __popcll(m[w] & ~cur[w]);
        }
        if (nl > 0 && (no + c > cap || kc + nn > kFK)) break;
#pragma unroll
        for (int w = 0; w < kMaxW; ++w) cur[w] |= m[w];
        kc += nn;
        ++nl;
        no += c;
    }
    next[base + t] = base + i;
}

// workgroup starts: 0, next(0), next(next(0)), ... (one workgroup; next[] through LDS windows)
__global__ __launch_bounds__(1024) void k_fb_chain(const int* next, int n, int* starts, int* counters) {
    __shared__ int win[kChainWin];
    __shared__ int sh[2];
    int pos = 0, t = 0;
    while (pos < n) {
        const int lim = min(n, pos + kChainWin);
        for (int i = threadIdx.x; i < lim - pos; i += blockDim.x) win[i] = next[pos + i];
        __syncthreads();
        if (threadIdx.x == 0) {
            int p = pos, tt = t;
            while (p < lim) {
                starts[tt++] = p;
                const int np = win[p - pos];
                p = np > p ? np : p + 1;  // (next[p] > p by construction; keeps the walk finite)
            }
            sh[0] = p;
            sh[1] = tt;
        }
        __syncthreads();
        pos = sh[0];
        t = sh[1];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        starts[t] = n;
        counters[0] = t;
    }
}

// per workgroup: its landmarks' workgroup / local index, its keyframe set, keyframe owners
__global__ __launch_bounds__(kT) void k_fb_group(const int* starts, const int* order, const u64* maskS, int W,
                                                int nk, int* lm_blk, int* lm_loc, u64* gmask, int* owner, int* cntE,
                                                int* erank) {
    __shared__ u64 gm[kMaxW];
    const int b = blockIdx.x;
    if (threadIdx.x < kMaxW) gm[threadIdx.x] = 0;
    if (threadIdx.x < kFK) {  // entry sizes and slot ranks, filled by k_fb_pose_rank
        cntE[(size_t)b * kFK + threadIdx.x] = 0;
        erank[(size_t)b * kFK + threadIdx.x] = -1;
    }
    __syncthreads();
    const int s = starts[b], e = starts[b + 1];
    u64 loc[kMaxW];
#pragma unroll
    for (int w = 0; w < kMaxW; ++w) loc[w] = 0;
    for (int i = s + threadIdx.x; i < e; i += kT) {
        const int q = order[i];
        lm_blk[q] = b;
        lm_loc[q] = i - s;
#pragma unroll
        for (int w = 0; w < kMaxW; ++w)
            if (w < W) loc[w] |= maskS[(size_t)i * W + w];
    }
#pragma unroll
    for (int w = 0; w < kMaxW; ++w)
        if (w < W && loc[w]) atomicOr(&gm[w], loc[w]);
    __syncthreads();
    if (threadIdx.x < W) gmask[(size_t)b * W + threadIdx.x] = gm[threadIdx.x];
    for (int k = threadIdx.x; k < nk; k += kT)
        if ((gm[k >> 6] >> (k & 63)) & 1) atomicMin(&owner[k], b);
}

// keyframes no workgroup touches: owned by workgroup 0 (build_fused step 3)
__global__ __launch_bounds__(kT) void k_fb_owner0(int nk, int W, int* owner, u64* gmask, int* counters) {
    __shared__ u64 g0[kMaxW];
    if (threadIdx.x < W) g0[threadIdx.x] = gmask[threadIdx.x];
    __syncthreads();
    for (int k = threadIdx.x; k < nk; k += kT)
        if (owner[k] == INT_MAX) {
            owner[k] = 0;
            atomicOr(&g0[k >> 6], 1ull << (k & 63));
        }
    __syncthreads();
    if (threadIdx.x < W) gmask[threadIdx.x] = g0[threadIdx.x];
    if (threadIdx.x == 0) {
        int pc = 0;
        for (int w = 0; w < W; ++w) pc += __popcll(g0[w]);
        if (pc > kFK) atomicOr(&counters[1], kFailOwnerKf);
    }
}

// one workgroup per keyframe row k: its pose observations (ascending index) split by workgroup — an
// optimised landmark's observation goes to the landmark's workgroup, a fixed landmark's to the
// keyframe's owner — with their rank inside the (workgroup, keyframe) entry; then the entry sizes and
// each entry's partial-slot rank among the keyframe's non-empty entries (workgroup order).  The S
// waves take consecutive segments: per wave counts by workgroup (a ballot per distinct workgroup of
// a 64-observation chunk), their exclusive prefix over the waves, then the ranks.
__device__ __forceinline__ void rank_chunk(int b, bool valid, int lane, int* cnt, int* prank, int* pblk, int o) {
    const u64 lt = (1ull << lane) - 1;
    u64 act = __ballot(valid);
    while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const int bl = __shfl(b, leader);
        const u64 m = __ballot(valid && b == bl);
        const int c0 = cnt[bl];
        if (prank && valid && b == bl) {
            prank[o] = c0 + __popcll(m & lt);
            pblk[o] = bl;
        }
        if (lane == leader) cnt[bl] = c0 + __popcll(m);  // (one wave: LDS accesses in program order)
        act &= ~m;
    }
}

__global__ __launch_bounds__(512) void k_fb_pose_rank(const int* kptr, const int* plm, int n_opt, const int* lm_blk,
                                                     const int* owner, int nb, const u64* gmask, int W, int* pblk,
                                                     int* prank, int* cntE, int* erank, int* rankk, int* counters) {
    extern __shared__ int cb[];  // [S][nb] per-wave counts, then [nb] totals
    const int S = blockDim.x >> 6;
    const int k = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int* tot = cb + (size_t)S * nb;
    for (int i = threadIdx.x; i < (S + 1) * nb; i += blockDim.x) cb[i] = 0;
    __syncthreads();
    const int o0 = kptr[k], o1 = kptr[k + 1], own = owner[k];
    const int seg = ((o1 - o0 + S - 1) / S + 63) & ~63;
    const int s0 = min(o1, o0 + wv * seg), s1 = min(o1, s0 + seg);
    int* mine = cb + (size_t)wv * nb;
    for (int pass = 0; pass < 2; ++pass) {
        for (int base = s0; base < s1; base += 64) {
            const int o = base + lane;
            const bool valid = o < s1;
            int b = -1;
            if (valid) {
                const int q = plm[o];
                b = q < n_opt ? lm_blk[q] : own;
            }
            rank_chunk(b, valid, lane, mine, pass ? prank : nullptr, pblk, o);
        }
        __syncthreads();
        if (pass == 0) {  // counts -> exclusive prefix over the waves; totals
            for (int b = threadIdx.x; b < nb; b += blockDim.x) {
                int run = 0;
                for (int w = 0; w < S; ++w) {
                    const int c = cb[(size_t)w * nb + b];
                    cb[(size_t)w * nb + b] = run;
                    run += c;
                }
                tot[b] = run;
            }
            __syncthreads();
        }
    }
    if (wv != 0) return;
    const u64 lt = (1ull << lane) - 1;
    int run = 0;
    for (int bb = 0; bb < nb; bb += 64) {
        const int b = bb + lane;
        const int c = b < nb ? tot[b] : 0;
        const u64 m = __ballot(c > 0);
        if (c > 0) {
            const int j = popc_below(gmask + (size_t)b * W, W, k);
            cntE[(size_t)b * kFK + j] = c;
            erank[(size_t)b * kFK + j] = run + __popcll(m & lt);
        }
        run += __popcll(m);
    }
    if (lane == 0) {
        rankk[k] = run;
        atomicMax(&counters[2], run);
    }
}

// per workgroup (lane = keyframe entry j): padded entry sizes, their offsets in wave-major order
// (wave w takes entries w, w + fw, ...), each wave's start and rounds, the workgroup's total
__global__ __launch_bounds__(64) void k_fb_entries(const u64* gmask, int W, int fw, const int* cntE, int* eoff,
                                                  int* wst, int* wrd, int* G, int nb, int* counters, int* epos,
                                                  int* npos) {
    __shared__ int pad[kFK], rnd[kFK], pos[kFK], sh_npos;
    const int b = blockIdx.x, j = threadIdx.x;
    int nent = 0;
    for (int w = 0; w < W; ++w) nent += __popcll(gmask[(size_t)b * W + w]);
    const int n = j < nent ? cntE[(size_t)b * kFK + j] : 0;
    pad[j] = j < nent ? (n + 63) / 64 * 64 : 0;
    rnd[j] = (n + 63) / 64;
    __syncthreads();
    if (j == 0) sh_npos = fused_place_entries(rnd, nent, pos);  // (SIMD-aware LPT, ba_plan.hpp)
    __syncthreads();
    const int P = j < nent ? pos[j] : INT_MAX;
    const int key = j < nent ? (P % fw) * kFK + P / fw : INT_MAX;  // wave-major over positions
    int off = 0, tot = 0, ws = 0, wr = 0;
    for (int i = 0; i < nent; ++i) {
        const int pi = pos[i], ki = (pi % fw) * kFK + pi / fw;
        if (ki < key) off += pad[i];
        tot += pad[i];
        if (j < fw) {
            if (pi % fw < j) ws += pad[i];
            if (pi % fw == j) wr += pad[i];
        }
    }
    eoff[(size_t)b * kFK + j] = off;
    epos[(size_t)b * kFK + j] = j < nent ? P : -1;
    if (j < fw) {
        wst[(size_t)b * kMaxWaves + j] = ws;
        wrd[(size_t)b * kMaxWaves + j] = wr / 64;
    }
    if (j == 0) {
        G[b] = tot;
        npos[b] = sh_npos;
        if (b == 0) G[nb] = 0;
    }
    // the lightest pose stage runs the stop rule (ba.hip fused_stop_key; lanes < fw hold the waves)
    int mr = j < fw ? wr / 64 : 0;
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) mr = max(mr, __shfl_xor(mr, m, 64));
    if (j == 0)
        atomicMin(reinterpret_cast<unsigned long long*>(counters + 4),
                  (unsigned long long)fused_stop_key(mr, sh_npos, b));
}

struct FusedTabs {
    int* blk;
    int* lm_slot;
    int2* lm_run;
    int4* lobs_rec;
    int* kent;
    int* lobs_src;
    int* pobs_src;
    int* pobs_code;
};

// per workgroup b (ft threads): landmark slots and runs, landmark-stage records, the header with the
// waves' starts, the keyframe entries, the padding of its pose-observation positions
__global__ void k_fb_fill_group(FusedTabs T, int ft, int fw, int blk_ints, int maxl, int nk, int W,
                                const int* starts, const int* order, const int* cntS, const int* cntScan,
                                const int* lptr, const int* lkf, const u64* gmask, const int* owner,
                                const int* rankk, const int* cntE, const int* erank, const int* eoff, const int* wst,
                                const int* wrd, const int* gbase, const int* epos, const int* npos) {
    __shared__ int jl[kBaMaxKfLds], kof[kFK], jof[kFK];
    __shared__ u64 gm[kMaxW];
    const int b = blockIdx.x, t = threadIdx.x;
    if (t < W) gm[t] = gmask[(size_t)b * W + t];
    if (t < kFK) jof[t] = -1;
    __syncthreads();
    for (int k = t; k < nk; k += ft) {  // keyframe -> entry position; position -> keyframe, sorted index
        const bool in = (gm[k >> 6] >> (k & 63)) & 1;
        const int j = in ? popc_below(gm, W, k) : -1;
        const int P = in ? epos[(size_t)b * kFK + j] : -1;
        jl[k] = P;
        if (in) {
            kof[P] = k;
            jof[P] = j;
        }
    }
    __syncthreads();
    int nent = 0;
    for (int w = 0; w < W; ++w) nent += __popcll(gm[w]);
    const int s = starts[b], e = starts[b + 1], nl = e - s;
    const int obase = cntScan[s], ob_total = cntScan[e] - obase;
    const size_t L = (size_t)b * ft;
    if (t < nl) {
        const int i = s + t, q = order[i];
        const int r0 = cntScan[i] - obase, r1 = r0 + cntS[i];
        T.lm_slot[L + t] = q;
        T.lm_run[L + t] = make_int2(r0, r1);
        for (int r = r0; r < r1; ++r) {
            const int o = lptr[q] + (r - r0);
            T.lobs_src[L + r] = o;
            T.lobs_rec[L + r] = make_int4(jl[lkf[o]], t, q, 0);
        }
    } else {
        T.lm_slot[L + t] = 0;
        T.lm_run[L + t] = make_int2(0, 0);
    }
    if (t >= ob_total) {
        T.lobs_src[L + t] = -1;
        T.lobs_rec[L + t] = make_int4(0, 0, 0, 0);
    }
    const int gb = gbase[b];
    if (t < blk_ints) {
        int v = 0;
        if (t == 0) v = nl;
        else if (t == 1) v = ob_total;
        else if (t == 2) v = npos[b];
        else if (t >= 4) {
            const int w = (t - 4) >> 1;
            v = (t & 1) ? wrd[(size_t)b * kMaxWaves + w] : gb + wst[(size_t)b * kMaxWaves + w];
        }
        T.blk[(size_t)b * blk_ints + t] = v;
    }
    for (int x = t; x < kFK * 8; x += ft) {  // entries by position (holes keep the defaults)
        const int P = x >> 3, f = x & 7, j = jof[P];
        int v = (f == 0 || f == 4) ? -1 : 0;
        if (j >= 0) {
            const int k = kof[P];
            const size_t ej = (size_t)b * kFK + j;
            const int st = gb + eoff[ej];
            if (f == 0) v = k | (owner[k] == b ? (1 << 30) : 0);
            else if (f == 1) v = rankk[k];
            else if (f == 2) v = st;
            else if (f == 3) v = st + cntE[ej];
            else if (f == 4) v = erank[ej] >= 0 ? k * maxl + erank[ej] : -1;
        }
        T.kent[((size_t)b * kFK) * 8 + x] = v;
    }
    for (int x = t; x < kFK * 64; x += ft) {  // (entry j, lane x): the positions after the last round's observations
        const int j = x >> 6, l = x & 63;
        if (j >= nent) continue;
        const size_t ej = (size_t)b * kFK + j;
        const int n = cntE[ej], pad = (n + 63) / 64 * 64;
        if (n + l < pad) {
            const int at = gb + eoff[ej] + n + l;
            T.pobs_src[at] = -1;
            T.pobs_code[at] = 0;
        }
    }
}

__global__ void k_fb_fill_pose(FusedTabs T, int n_pose, int n_opt, int W, const int* plm, const int* pkf,
                               const int* pblk, const int* prank, const int* lm_loc, const u64* gmask,
                               const int* eoff, const int* gbase) {
    const int o = blockIdx.x * kT + threadIdx.x;
    if (o >= n_pose) return;
    const int b = pblk[o];
    const int j = popc_below(gmask + (size_t)b * W, W, pkf[o]);
    const int at = gbase[b] + eoff[(size_t)b * kFK + j] + prank[o];
    const int q = plm[o];
    T.pobs_src[at] = o;
    T.pobs_code[at] = q < n_opt ? lm_loc[q] : -1 - q;
}

// carve typed arrays out of one scratch block (256-B aligned)
struct Carve {
    uint8_t* base;
    size_t at = 0;
    template <class X>
    X* take(size_t n) {
        X* r = reinterpret_cast<X*>(base + at);
        at += (n * sizeof(X) + 255) & ~(size_t)255;
        return r;
    }
};
template <class X>
size_t carve_bytes(size_t n) {
    return (n * sizeof(X) + 255) & ~(size_t)255;
}

}  // namespace

int build_fused_device(vx_ctx* c, vx_ba_plan* p) {
    p->fused = false;
    if (!fused_eligible(p)) return VX_OK;
    static const bool timing = getenv("VX_PLAN_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); };
    const int nk = p->n_kf, n_opt = p->n_opt, n_pose = (int)p->n_pose_obs, n_lobs = (int)p->n_lm_obs;
    const int W = (nk + 63) / 64;
    int cap = 0;
    const int ft = fused_threads(c, n_lobs, &cap);
    const int fw = ft / 64;
    hipStream_t s = c->stream;
    vx_ctx::PlanScratch& S = c->plan_scratch;
    const int* kptr = p->kf_obs_ptr.as<int>();
    const int* plm = p->pobs_lm.as<int>();
    const int* lptr = p->lobs_ptr.as<int>();
    const int* lkf = p->lobs_kf.as<int>();
    const int* llm = p->lobs_lm.as<int>();

    // ---- per-landmark / per-observation scratch
    const size_t no = (size_t)n_opt, np = (size_t)std::max(n_pose, 1);
    size_t need = carve_bytes<int>(np) * 3 + carve_bytes<int>(no) * 7 + carve_bytes<u64>(no * W) * 2 +
                  carve_bytes<int>(no + 1) * 3 + carve_bytes<int>(nk) * 2 + carve_bytes<int>(16);
    VX_HIP(c, S.fb.ensure(need));
    Carve cv{S.fb.as<uint8_t>()};
    int* pkf = cv.take<int>(np);
    int* pblk = cv.take<int>(np);
    int* prank = cv.take<int>(np);
    int* key = cv.take<int>(no);
    int* keys2 = cv.take<int>(no);
    int* iota = cv.take<int>(no);
    int* order = cv.take<int>(no);
    int* lm_blk = cv.take<int>(no);
    int* lm_loc = cv.take<int>(no);
    u64* mask = cv.take<u64>(no * W);
    u64* maskS = cv.take<u64>(no * W);
    int* cntS = cv.take<int>(no + 1);
    int* cntScan = cv.take<int>(no + 1);
    int* starts = cv.take<int>(no + 1);
    int* owner = cv.take<int>(nk);
    int* rankk = cv.take<int>(nk);
    int* counters = cv.take<int>(16);
    int* next = cv.take<int>(no);

    hipLaunchKernelGGL(k_fb_init, dim3(grid(std::max(std::max(n_opt, nk), 16))), dim3(kT), 0, s, n_opt, nk, W, key, iota,
                       mask, owner, counters);
    hipLaunchKernelGGL(k_fb_pkf, dim3(grid(n_pose)), dim3(kT), 0, s, kptr, nk, n_pose, pkf);
    hipLaunchKernelGGL(k_fb_mask, dim3(grid(std::max(n_lobs, n_pose))), dim3(kT), 0, s, n_lobs, llm, lkf, n_pose, plm,
                       (const int*)pkf, n_opt, W, key, mask);
    VX_LAUNCH_CHECK(c, "fused build: keyframe sets");
    unsigned bits = 1;
    while ((1 << bits) <= nk) ++bits;
    size_t tb = 0;
    VX_HIP(c, rocprim::radix_sort_pairs<OnesweepSort>(nullptr, tb, key, keys2, iota, order, no, 0, bits, s));
    size_t tb2 = 0;
    VX_HIP(c, rocprim::exclusive_scan(nullptr, tb2, cntS, cntScan, 0, no + 1, rocprim::plus<int>(), s));
    VX_HIP(c, S.fb_tmp.ensure(std::max<size_t>(std::max(tb, tb2), 16)));
    VX_HIP(c, rocprim::radix_sort_pairs<OnesweepSort>(S.fb_tmp.p, tb, key, keys2, iota, order, no, 0, bits, s));
    hipLaunchKernelGGL(k_fb_sorted, dim3(grid(n_opt)), dim3(kT), 0, s, (const int*)order, (const int*)keys2, n_opt,
                       lptr, (const u64*)mask, W, ft, cntS, maskS, counters);
    VX_LAUNCH_CHECK(c, "fused build: sorted order");
    VX_HIP(c, rocprim::exclusive_scan(S.fb_tmp.p, tb2, cntS, cntScan, 0, no + 1, rocprim::plus<int>(), s));
    const size_t next_lds = (size_t)(kT + cap) * (W * sizeof(u64) + 2 * sizeof(int)) + sizeof(int);
    static std::atomic<uint64_t> attr_done{0};
    VX_HIP(c, lds_attr_once(c->device, reinterpret_cast<const void*>(&k_fb_next),
                            (int)((kT + kBaFTLarge) * (kMaxW * sizeof(u64) + 2 * sizeof(int)) + sizeof(int)), attr_done));
    hipLaunchKernelGGL(k_fb_next, dim3(grid(n_opt)), dim3(kT), (uint32_t)next_lds, s, (const int*)cntScan,
                       (const int*)keys2, (const u64*)maskS, n_opt, W, cap, (const int*)counters, next);
    hipLaunchKernelGGL(k_fb_chain, dim3(1), dim3(1024), 0, s, (const int*)next, n_opt, starts, counters);
    VX_LAUNCH_CHECK(c, "fused build: packing");
    VX_HIP(c, S.fb_host.ensure(64));
    int* H = static_cast<int*>(S.fb_host.p);
    VX_HIP(c, hipMemcpyAsync(H, counters, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    VX_HIP(c, hipStreamSynchronize(s));
    const double t_pack = ms();
    const int nb = H[0];
    if (H[1] != 0 || nb < 1 || nb > kMaxGroupsRank) return VX_OK;  // (the host packing returns not fused alike)

    // ---- per-workgroup scratch
    const size_t nbs = (size_t)nb;
    need = carve_bytes<u64>(nbs * W) + carve_bytes<int>(nbs * kFK) * 4 + carve_bytes<int>(nbs * kMaxWaves) * 2 +
           carve_bytes<int>(nbs + 1) * 3;
    VX_HIP(c, S.fb_groups.ensure(need));
    Carve cg{S.fb_groups.as<uint8_t>()};
    u64* gmask = cg.take<u64>(nbs * W);
    int* cntE = cg.take<int>(nbs * kFK);
    int* erank = cg.take<int>(nbs * kFK);
    int* eoff = cg.take<int>(nbs * kFK);
    int* wst = cg.take<int>(nbs * kMaxWaves);
    int* wrd = cg.take<int>(nbs * kMaxWaves);
    int* G = cg.take<int>(nbs + 1);
    int* gbase = cg.take<int>(nbs + 1);
    int* epos = cg.take<int>(nbs * kFK);  // entry (sorted index) -> position
    int* npos = cg.take<int>(nbs + 1);    // positions per workgroup
    hipLaunchKernelGGL(k_fb_group, dim3(nb), dim3(kT), 0, s, (const int*)starts, (const int*)order, (const u64*)maskS,
                       W, nk, lm_blk, lm_loc, gmask, owner, cntE, erank);
    hipLaunchKernelGGL(k_fb_owner0, dim3(1), dim3(kT), 0, s, nk, W, owner, gmask, counters);
    const int nw = std::max(1, std::min(8, kMaxGroupsRank * 2 / nb - 1));  // waves per keyframe: (nw + 1) x nb ints of LDS
    hipLaunchKernelGGL(k_fb_pose_rank, dim3(nk), dim3(64 * nw), (uint32_t)((nw + 1) * nbs * sizeof(int)), s, kptr, plm, n_opt,
                       (const int*)lm_blk, (const int*)owner, nb, (const u64*)gmask, W, pblk, prank, cntE, erank,
                       rankk, counters);
    hipLaunchKernelGGL(k_fb_entries, dim3(nb), dim3(64), 0, s, (const u64*)gmask, W, fw, (const int*)cntE, eoff, wst,
                       wrd, G, nb, counters, epos, npos);
    VX_LAUNCH_CHECK(c, "fused build: entries");
    VX_HIP(c, rocprim::exclusive_scan(nullptr, tb, G, gbase, 0, nbs + 1, rocprim::plus<int>(), s));
    VX_HIP(c, S.fb_tmp.ensure(std::max<size_t>(tb, 16)));
    VX_HIP(c, rocprim::exclusive_scan(S.fb_tmp.p, tb, G, gbase, 0, nbs + 1, rocprim::plus<int>(), s));
    VX_HIP(c, hipMemcpyAsync(H, counters, 6 * sizeof(int), hipMemcpyDeviceToHost, s));
    VX_HIP(c, hipMemcpyAsync(H + 8, gbase + nb, sizeof(int), hipMemcpyDeviceToHost, s));
    VX_HIP(c, hipStreamSynchronize(s));
    const double t_entries = ms();
    if (H[1] != 0) return VX_OK;
    const int maxl = std::max(1, H[2]);
    const size_t n_pp = (size_t)H[8];
    const int stop_b = H[4];  // (low word of the minimal key)

    // ---- the tables, straight into f_tab
    FusedOffsets& F = p->f_off;
    const size_t at = fused_offsets(nb, ft, n_pp, F);
    VX_HIP(c, p->f_tab.ensure(at));
    uint8_t* TB = p->f_tab.as<uint8_t>();
    FusedTabs T{reinterpret_cast<int*>(TB + F.blk),      reinterpret_cast<int*>(TB + F.lm_slot),
                reinterpret_cast<int2*>(TB + F.lm_run),  reinterpret_cast<int4*>(TB + F.lobs_rec),
                reinterpret_cast<int*>(TB + F.kent),     reinterpret_cast<int*>(TB + F.lobs_src),
                reinterpret_cast<int*>(TB + F.pobs_src), reinterpret_cast<int*>(TB + F.pobs_code)};
    hipLaunchKernelGGL(k_fb_fill_group, dim3(nb), dim3(ft), 0, s, T, ft, fw, fused_blk_ints(ft), maxl, nk, W,
                       (const int*)starts, (const int*)order, (const int*)cntS, (const int*)cntScan, lptr, lkf,
                       (const u64*)gmask, (const int*)owner, (const int*)rankk, (const int*)cntE, (const int*)erank,
                       (const int*)eoff, (const int*)wst, (const int*)wrd, (const int*)gbase, (const int*)epos,
                       (const int*)npos);
    hipLaunchKernelGGL(k_fb_fill_pose, dim3(grid(n_pose)), dim3(kT), 0, s, T, n_pose, n_opt, W, plm, (const int*)pkf,
                       (const int*)pblk, (const int*)prank, (const int*)lm_loc, (const u64*)gmask, (const int*)eoff,
                       (const int*)gbase);
    VX_LAUNCH_CHECK(c, "fused build: tables");
    int rc;
    if ((rc = fused_finish(c, p, nb, ft, maxl, n_pp, stop_b))) return rc;
    if (timing) {
        VX_HIP(c, hipStreamSynchronize(s));
        fprintf(stderr, "[vx plan] fused layout on the device: packing %.3f ms, entries %.3f ms, tables %.3f ms (%d workgroups x %d)\n",
                t_pack, t_entries - t_pack, ms() - t_entries, nb, ft);
    }
    return VX_OK;
}

}  // namespace vx
