// orb.hip — ORB feature extraction on gfx950 (FeatureExtractor::Extract drop-in).
//
// Replaces ORBExtractor::Extract (core/feature/orb_extractor.cpp:9-27), i.e.
// cv::ORB::create(n, 1.2f, 8)->detectAndCompute(img, noArray(), kps, desc).  The pipeline
//  is re-designed as a chain of wavefront kernels on one HIP stream:
//
//   k_pyramid         BGR(A)->gray level 0 (fixed point) and the whole INTER_LINEAR_EXACT pyramid
//                     (8.8 / 16.16 fixed point) in ONE launch: per level-0 tile, level by level
//                     through LDS with host-computed halos (A.1); k_gray + k_resize x (L-1) is
//                     the fallback when the halo does not fit in LDS
//   k_fast            all levels in one launch: 64x16 tiles staged in LDS with a 4 px
//                     halo; FAST-9/16 corner test as 16-bit ring masks, cornerScore<16>, strict
//                     3x3 NMS, border filter, raster-ordered cells by wave ballot, wave-parallel Harris
//                     7x7 from the same LDS tile, per-level score histogram (A.3, A.4)
//   k_blur            GaussianBlur 7x7 sigma 2, float separable, reflect-101, all levels (A.5)
//   k_select          one workgroup per level: retainBest(2q) by FAST score via the histogram,
//                     retainBest(q) by Harris via an exact 4-pass radix select; both keep the
//                     OpenCV set {response >= k-th largest} in raster order (A.3)
//   k_describe        one wavefront per keypoint: intensity-centroid angle (fastAtan2), rotated
//                     BRIEF sampling of the blurred level, 256 comparisons packed by 4 ballots
//                     into the 32-byte descriptor (A.4, A.6)
//
// Every integer stage is exact; float stages are compiled with -ffp-contract=off and follow the
// OpenCV operation order, so results are bit-identical to the CPU restatement in oracle/.
#include <cfloat>
#include <cstdlib>
#include <cmath>
#include <cstring>

#include "vx_internal.hpp"
#include "vx_ktrace.hpp"

#include "orb_pattern_31.inc"

namespace vx {
namespace {

constexpr int kBlock = 256;
// FAST score histograms: one replica per XCD slot (blockIdx mod 8) so that k_fast's atomics from
// different XCDs never meet on one address; k_select sums the replicas
constexpr int kHistRep = 8;

VX_KT_TABLE();
VX_KP_TABLE();

__constant__ signed char c_pattern[1024];
__constant__ int c_umax[16];
// ICAngles row masks: row lane (v = lane - 15), byte k of the 32-byte window starting at u = -15
// is 0xff iff |k - 15| <= umax[|v|] (row 31 empty)
__constant__ __attribute__((aligned(16))) unsigned c_icmask[32][8];

struct LevelArgs {
    int L;
    int lw[kMaxLevels], lh[kMaxLevels];
    long long off[kMaxLevels];
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    int quota[kMaxLevels];
    int ntx[kMaxLevels], tile_base[kMaxLevels];     // FAST tiles (64 x 16) per level
    long long cell_base[kMaxLevels];                // first (row, tile column) cell of level l
    long long stage_base[kMaxLevels];               // selection staging of level l
    int level_cap[kMaxLevels];                      // max NMS corners of level l
    int fast_threshold, edge, out_cap;
    int raster_rank;                                // k_select_stl wrote the survivors' raster ranks
    // blur tiling
    int btx[kMaxLevels], bty[kMaxLevels], bbase[kMaxLevels];
    float gk[7];
    // fused pyramid: resize tables and tile rectangles (offsets into the int4 table buffer)
    long long xtab[kMaxLevels], ytab[kMaxLevels];
    long long pr_x, pr_y;
    int pr_buf;
    // batched launches (vx_orb_extract_batch_async): frame blockIdx.z's buffers start this many
    // elements after frame 0's (all zero-offset for a single frame: gridDim.z = 1)
    long long fs_img, fs_pyr, fs_cells, fs_hist, fs_stage;
};

// Copies n elements into LDS, element i = load(i), with every load of a thread issued before the
// first LDS store: one exposed memory latency per KMAX * NT elements instead of one per element
// (a plain strided loop waits on each load before the next iteration's).
template <int NT, int KMAX, class T, class F>
__device__ __forceinline__ void stage_lds(T* __restrict__ dst, int n, F load) {
    for (int base = 0; base < n; base += NT * KMAX) {
        T v[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int i = base + (int)threadIdx.x + k * NT;
            v[k] = i < n ? load(i) : T{};
        }
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int i = base + (int)threadIdx.x + k * NT;
            if (i < n) dst[i] = v[k];
        }
    }
}

// ------------------------------------------------------------------------------ gray
// cvtColor BGR2GRAY fixed point (B 1868, G 9617, R 4899, >> 14); 1 channel passes through
__device__ __forceinline__ uint8_t gray_px(const uint8_t* s, int ch) {
    if (ch == 1) return s[0];
    return (uint8_t)((s[0] * 1868 + s[1] * 9617 + s[2] * 4899 + (1 << 13)) >> 14);
}

// INTER_LINEAR_EXACT tap: u16 8.8 horizontal, u32 16.16 vertical, (v + 32768) >> 16
__device__ __forceinline__ uint8_t lin_px(const uint8_t* r0, const uint8_t* r1, int c0, int c1, int4 cx,
                                          int4 cy) {
    const uint32_t h0 = (uint32_t)(r0[c0] * cx.y + r0[c1] * cx.z);
    const uint32_t h1 = (uint32_t)(r1[c0] * cx.y + r1[c1] * cx.z);
    const uint32_t v = h0 * (uint32_t)cy.y + h1 * (uint32_t)cy.z;
    return (uint8_t)min((v + 32768u) >> 16, 255u);
}

// Unfused path only (the fused k_pyramid zeroes the histograms itself).
__global__ void k_gray(const uint8_t* __restrict__ img, int W, int ch, long long stride,
                       uint8_t* __restrict__ out, int* __restrict__ hist, int hist_n, long long fs_img,
                       long long fs_pyr, long long fs_hist) {
    img += blockIdx.z * fs_img;
    out += blockIdx.z * fs_pyr;
    hist += blockIdx.z * fs_hist;
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < hist_n; i += blockDim.x) hist[i] = 0;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    out[(long long)y * W + x] = gray_px(img + (long long)y * stride + (long long)x * ch, ch);
}

// ------------------------------------------------------------------------------ fused pyramid
// One launch for gray + every INTER_LINEAR_EXACT level.  Workgroup (tx, ty) owns a level-0 tile
// and, at level l, the proportional sub-rectangle of level l; it computes, level by level in two
// LDS ping-pong buffers, every pixel its deeper levels depend on (the "need" rectangle: own +
// a halo that grows as h <- 1.2 h + 1, prepared on the host from the same coefficient tables),
// and writes only the pixels it owns.  Each pixel is the same deterministic function of its
// sources whichever workgroup computes it, so the result is bit-identical to the level chain.
// Level-0 tile edge and workgroup size (template NT: 512 or 1024 threads, 64 x NT/64) trade
// parallelism against redundant halo work.  A 1024-thread workgroup occupies a whole CU, so the
// tile is the smallest edge (>= 32, step 4) whose grid fits the device's CUs in one round
// (640x480 on 256 CUs: 36 -> 18 x 14 workgroups; measured 13.9 us at 40 vs 17.3 us at 64 and
// 22.9 us at 32, which needs two rounds).  A context sharing the device with concurrent ones
// (vx_set_grid_share) sizes the grid for its share of the CUs instead: in the 3-context pipeline
// (share 1/3: tile 64, 80 workgroups) the LocalBA kernels find free CUs and the pipelined frame
// is ~5 % faster than with the one-round grid (scripts/sweep_pyr_pipe.sh).
// $VX_PYR_TILE / $VX_PYR_BLOCK override for sweeps.
constexpr int kPyBlockDef = 1024;
constexpr int kPyLdsMax = 64 * 1024;

template <int NT>
__global__ __launch_bounds__(NT) void k_pyramid(const uint8_t* __restrict__ img, int ch,
                                                      long long stride, uint8_t* __restrict__ pyr,
                                                      const int4* __restrict__ tabs, LevelArgs a,
                                                      int* __restrict__ hist, int hist_n, int raw_bytes) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_pyr[];
    __shared__ int4 srx[kMaxLevels], sry[kMaxLevels];
    __shared__ int sox[kMaxLevels + 1], soy[kMaxLevels + 1];
    uint8_t* raw = lds_pyr;                       // level-0 need rectangle, BGR(A) bytes
    uint8_t* cur = raw + raw_bytes;               // ping-pong level buffers
    uint8_t* prev = cur + a.pr_buf;
    int* stab = reinterpret_cast<int*>(prev + a.pr_buf);  // packed {ofs | c1 << 16} per level
    const int tid = threadIdx.x, lx = tid & 63, ly = tid >> 6;
    const int L = a.L;
    img += blockIdx.z * a.fs_img;
    pyr += blockIdx.z * a.fs_pyr;
    hist += blockIdx.z * a.fs_hist;
    VX_KT(0);
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = tid; i < hist_n; i += NT) hist[i] = 0;
    // tiles XCD by XCD (workgroup i of the dispatch runs on XCD i mod 8): XCD k takes the k-th
    // contiguous run of the raster tile order, so neighbouring tiles' overlapping need rectangles
    // meet in one L2 (the k_fast mapping)
    int bx, by;
    {
        const int nb = (int)(gridDim.x * gridDim.y), lin = (int)(blockIdx.x + blockIdx.y * gridDim.x);
        const int xcd = lin & 7, qb = nb >> 3, rem = nb & 7;
        const int t = xcd * qb + min(xcd, rem) + (lin >> 3);
        by = t / (int)gridDim.x;
        bx = t - by * (int)gridDim.x;
    }
    if (tid < L) srx[tid] = tabs[a.pr_x + (long long)bx * L + tid];
    if (tid >= 64 && tid < 64 + L) sry[tid - 64] = tabs[a.pr_y + (long long)by * L + tid - 64];
    __syncthreads();
    if (tid == 0) {
        int o = 0;
        sox[0] = soy[0] = 0;
        for (int l = 1; l < L; ++l) { sox[l] = o; o += srx[l].y - srx[l].x; }
        for (int l = 1; l < L; ++l) { soy[l] = o; o += sry[l].y - sry[l].x; }
        sox[L] = o;  // total entries
    }
    __syncthreads();
    // coefficient tables of this tile's need ranges, every level, all loads in flight at once
    stage_lds<NT, 2048 / NT>(stab, sox[L], [&](int i) {
        const bool isy = i >= soy[1];
        int l = 1;
        if (!isy) { while (l + 1 < L && i >= sox[l + 1]) ++l; }
        else { while (l + 1 < L && i >= soy[l + 1]) ++l; }
        const int idx = i - (isy ? soy[l] : sox[l]) + (isy ? sry[l].x : srx[l].x);
        const int4 e = tabs[(isy ? a.ytab[l] : a.xtab[l]) + idx];
        return e.x | (e.z << 16);
    });
    // level 0: stage the BGR(A) bytes of the need rectangle as 4-byte-aligned dwords (a byte
    // load per pixel channel would saturate the vector-memory pipe long before HBM), each LDS row
    // starting at the dword containing the row's first needed byte.  Only the dword holding the
    // image's very last byte may extend past the allocation: it is read bytewise.
    int4 rx = srx[0], ry = sry[0];
    int px0 = rx.x, py0 = ry.x, pw = rx.y - rx.x, ph = ry.y - ry.x;
    const int rb = pw * ch;
    const int rowdw = (rb + 6) >> 2;  // dwords per LDS row, any start alignment
    {
        // byte offsets (from img) of the image's last byte and of this tile's first needed byte
        const long long last = (long long)(a.lh[0] - 1) * stride + (long long)a.lw[0] * ch - 1;
        const long long first = (long long)py0 * stride + (long long)px0 * ch;
        const int mis0 = (int)(reinterpret_cast<uintptr_t>(img) & 3);
        uint32_t* rawd = reinterpret_cast<uint32_t*>(raw);
        constexpr int KR = 96 / (NT / 64), KC = 2;  // one batch covers 96 rows x 128 dwords
        for (int r0 = 0; r0 < ph; r0 += (NT / 64) * KR)
            for (int c0 = 0; c0 < rowdw; c0 += 64 * KC) {
                uint32_t v[KR][KC];
                unsigned fix = 0;  // elements whose dword would pass the image's last byte
#pragma unroll
                for (int i = 0; i < KR; ++i)
#pragma unroll
                    for (int j = 0; j < KC; ++j) {
                        const int r = r0 + ly + (NT / 64) * i, c = c0 + lx + 64 * j;
                        const long long ro = first + (long long)r * stride;
                        const long long off = ro - (long long)((mis0 + ro) & 3) + 4LL * c;  // aligned
                        const bool in = r < ph && c < rowdw;
                        const bool safe = in && off + 3 <= last;
                        v[i][j] = safe ? *reinterpret_cast<const uint32_t*>(img + off) : 0u;
                        if (in && !safe) fix |= 1u << (i * KC + j);
                    }
                if (fix) {  // at most one dword of the whole image: bytewise, outside the batch
#pragma unroll
                    for (int i = 0; i < KR; ++i)
#pragma unroll
                        for (int j = 0; j < KC; ++j)
                            if (fix & (1u << (i * KC + j))) {
                                const int r = r0 + ly + (NT / 64) * i, c = c0 + lx + 64 * j;
                                const long long ro = first + (long long)r * stride;
                                const long long off = ro - (long long)((mis0 + ro) & 3) + 4LL * c;
                                for (int q = 0; q < 4; ++q)
                                    if (off + q <= last) v[i][j] |= (uint32_t)img[off + q] << (8 * q);
                            }
                }
#pragma unroll
                for (int i = 0; i < KR; ++i)
#pragma unroll
                    for (int j = 0; j < KC; ++j) {
                        const int r = r0 + ly + (NT / 64) * i, c = c0 + lx + 64 * j;
                        if (r < ph && c < rowdw) rawd[r * rowdw + c] = v[i][j];
                    }
            }
    }
    __syncthreads();
    VX_KT(1);
    constexpr int RS = NT / 64;  // rows per pass
    for (int yy = ly; yy < ph; yy += RS) {
        const int y = py0 + yy;
        const bool oy = y >= ry.z && y < ry.w;
        uint8_t* drow = pyr + (long long)y * a.lw[0];
        const int ra = (int)((reinterpret_cast<uintptr_t>(img) + (uintptr_t)((long long)y * stride + (long long)px0 * ch)) & 3);
        const uint8_t* rrow = raw + yy * rowdw * 4 + ra;
        for (int xx = lx; xx < pw; xx += 64) {
            const int x = px0 + xx;
            const uint8_t g = gray_px(rrow + xx * ch, ch);
            cur[yy * pw + xx] = g;
            if (oy && x >= rx.z && x < rx.w) drow[x] = g;
        }
    }
    VX_KT(2);
    for (int l = 1; l < L; ++l) {
        uint8_t* t = cur;
        cur = prev;
        prev = t;
        __syncthreads();
        rx = srx[l];
        ry = sry[l];
        const int sw = a.lw[l - 1], sh = a.lh[l - 1], dw = a.lw[l];
        const int* xt = stab + sox[l] - rx.x;
        const int* yt = stab + soy[l] - ry.x;
        const int nw = rx.y - rx.x, nh = ry.y - ry.x;
        uint8_t* dst = pyr + a.off[l];
        for (int yy = ly; yy < nh; yy += RS) {
            const int y = ry.x + yy;
            const int ey = yt[y];
            const int4 cy = make_int4(ey & 0xffff, 256 - (ey >> 16), ey >> 16, 0);
            const uint8_t* r0 = prev + (cy.x - py0) * pw;
            const uint8_t* r1 = prev + (min(cy.x + 1, sh - 1) - py0) * pw;
            const bool oy = y >= ry.z && y < ry.w;
            for (int xx = lx; xx < nw; xx += 64) {
                const int x = rx.x + xx;
                const int ex = xt[x];
                const int4 cx = make_int4(ex & 0xffff, 256 - (ex >> 16), ex >> 16, 0);
                const uint8_t v = lin_px(r0, r1, cx.x - px0, min(cx.x + 1, sw - 1) - px0, cx, cy);
                cur[yy * nw + xx] = v;
                if (oy && x >= rx.z && x < rx.w) dst[(long long)y * dw + x] = v;
            }
        }
        px0 = rx.x;
        py0 = ry.x;
        pw = nw;
        ph = nh;
    }
    VX_KT(3);
}

// ------------------------------------------------------------------------------ resize
__global__ void k_resize(const uint8_t* __restrict__ src, int sw, int sh, uint8_t* __restrict__ dst,
                         int dw, const int4* __restrict__ xt, const int4* __restrict__ yt, long long fs_pyr) {
    src += blockIdx.z * fs_pyr;
    dst += blockIdx.z * fs_pyr;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= dw) return;
    const int4 cx = xt[x];
    const int4 cy = yt[y];
    const uint8_t* r0 = src + (long long)cy.x * sw;
    const uint8_t* r1 = src + (long long)min(cy.x + 1, sh - 1) * sw;
    dst[(long long)y * dw + x] = lin_px(r0, r1, cx.x, min(cx.x + 1, sw - 1), cx, cy);
}

// ------------------------------------------------------------------------------ FAST
// ring offsets (x, y), FAST_t<16> makeOffsets
__device__ __forceinline__ int ring_dx(int k) {
    const int t[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    return t[k];
}
__device__ __forceinline__ int ring_dy(int k) {
    const int t[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    return t[k];
}

__device__ __forceinline__ bool has_run9(uint32_t m16) {
    const uint32_t m = m16 | (m16 << 16);
    uint32_t r = m & (m >> 1);   // runs >= 2
    r &= r >> 2;                 // >= 4
    r &= r >> 4;                 // >= 8
    r &= m >> 8;                 // >= 9
    return r != 0;
}

// FAST test + cornerScore<16>; returns 0 for non-corners.  t = tile base at the pixel.
__device__ int fast_score(const uint8_t* t, int stride, int thr) {
    const int v = t[0];
    int p[16];
    uint32_t bright = 0, dark = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        p[k] = t[ring_dy(k) * stride + ring_dx(k)];
        bright |= (uint32_t)(p[k] > v + thr) << k;
        dark |= (uint32_t)(p[k] < v - thr) << k;
    }
    if (!has_run9(bright) && !has_run9(dark)) return 0;
    int d[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) d[k] = v - p[k & 15];
    int a0 = thr;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(d[k + 1], d[k + 2]);
        a = min(a, d[k + 3]);
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(d[k + 1], d[k + 2]);
        b = max(b, d[k + 3]);
        b = max(b, d[k + 4]);
        b = max(b, d[k + 5]);
        b = max(b, d[k + 6]);
        b = max(b, d[k + 7]);
        b = max(b, d[k + 8]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + 9]));
    }
    return -b0 - 1;
}

struct alignas(16) CandRec {  // 16 B per FAST candidate / selected keypoint
    unsigned xy;  // x | y << 16
    int score;
    float harris;
    int pad;
};

// Wave-scan based exclusive block scan (NT/64 waves, one barrier pair).  sh: >= NT/64 ints.
template <int NT>
__device__ __forceinline__ int block_scan_excl(int v, int* sh, int& total) {
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
        const int s = sh[i];
        tot += s;
        pre += i < w ? s : 0;
    }
    total = tot;
    __syncthreads();
    return pre + x - v;
}

// FAST-9/16 + strict 3x3 NMS + border filter + Harris, all levels in one launch.
// Block = 64 x 16 output tile (4 px halo staged in LDS).  Output is written per cell = (row,
// tile column) with a fixed capacity of 32 (strict NMS keeps at most every other pixel of a
// 64 px row segment), so cell order == raster order and the per-row compaction is one ballot.
//
// LDS is read a dword (4 pixels) at a time wherever a lane works on a pixel quad: the FAST ring
// test, the blur's row pass (3 dwords per 4 outputs) and its column pass (float4 rows), instead of
// one ds_read_u8 per tap — the byte-read version was LDS-issue bound (SQ_WAIT_INST_LDS, 234 LDS
// instructions per wave).  cornerScore<16> runs only for the compacted corner list (3-7 % of the
// pixels), not under a divergent branch that nearly every wave takes.
constexpr int kTX = 64, kTY = 16, kCellCap = 32;
// Candidate records are stored slot-major within a frame: slot i of cell c at i * fs_cells + c.
// Most cells hold 0-2 records, so the selection's gather (consecutive cells per thread, slot 0
// first) reads whole cache lines of records instead of one line per record.
__device__ __forceinline__ long long cand_at(long long cell, int i, long long fs_cells) {
    return (long long)i * fs_cells + cell;
}
constexpr int kTW = kTX + 12, kTH = kTY + 8;  // staged tile: x0-4 .. x0+71 (quad reads up to x0+71)
constexpr int kSW = kTX + 4, kSH = kTY + 2;   // score tile (66 used + 2 pad: dword rows)
constexpr int kSQ = 17;                       // score quads per row (68 columns)

// The GaussianBlur of the same 64 x 16 output tile (k_blur's arithmetic, reflect-101 halo of 3)
// is computed here too: the tile is already being read, and the separate blur launch was a
// dependent step of its own on the extraction chain.
constexpr int kBW = kTX + 8, kBH = kTY + 6;   // blur input tile x0-4 .. x0+67 (reflect-101), 3 row halo
static_assert(kTW % 4 == 0 && kSW % 4 == 0 && kBW % 4 == 0, "quad rows must be dword aligned");

// byte b (0..11) of a 12-byte window held as three dwords
__device__ __forceinline__ int win_byte(const uint32_t (&w)[3], int b) {
    return (int)((w[b >> 2] >> (8 * (b & 3))) & 255u);
}

// Two adjacent bytes b, b + 1 (b in 0..8) of a 12-byte window, zero-extended into the two 16-bit
// lanes of a register (one v_perm_b32): the FAST ring test below runs on pixel pairs with packed
// 16-bit arithmetic.  Selector bytes 0..3 pick the low source's bytes, 4..7 the high one's, 0x0c a zero.
typedef short vx_i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short vx_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ vx_i16x2 win_pair(const uint32_t (&w)[3], int b) {
    const int lo = b >= 7 ? 1 : 0, bb = b - 4 * lo;
    const uint32_t sel = (uint32_t)bb | 0x0c00u | ((uint32_t)(bb + 1) << 16) | 0x0c000000u;
    return __builtin_bit_cast(vx_i16x2, __builtin_amdgcn_perm(w[lo + 1], w[lo], sel));
}

// An interior tile (every staged byte inside the level, no clamp / reflection) staged a dword at a
// time: ROWS rows of 4*DW bytes from src (row pitch W, any byte alignment) into dst, each dword from
// two aligned loads and one v_alignbyte, all loads of a thread issued before its first LDS store.
template <int ROWS, int DW>
__device__ __forceinline__ void stage_dw(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int W) {
    constexpr int N = ROWS * DW, KM = (N + kBlock - 1) / kBlock;
    unsigned lo[KM], hi[KM], sh[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        const int i = (int)threadIdx.x + k * kBlock;
        lo[k] = hi[k] = sh[k] = 0;
        if (i < N) {
            const int r = i / DW, c = i - r * DW;
            const uintptr_t ad = (uintptr_t)(src + (long long)r * W + 4 * c);
            const unsigned* al = reinterpret_cast<const unsigned*>(ad & ~(uintptr_t)3);
            sh[k] = (unsigned)(ad & 3u);
            lo[k] = al[0];
            hi[k] = al[1];
        }
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        const int i = (int)threadIdx.x + k * kBlock;
        if (i < N) reinterpret_cast<unsigned*>(dst)[i] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh[k]);
    }
}

__device__ __forceinline__ int refl101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) {
        if (p < 0) p = -p;
        if (p >= n) p = 2 * n - 2 - p;
    }
    return p;
}

__global__ __launch_bounds__(kBlock) void k_fast(const uint8_t* __restrict__ pyr, LevelArgs a,
                                                 CandRec* __restrict__ cand,
                                                 int* __restrict__ cell_count,
                                                 int* __restrict__ hist,
                                                 uint8_t* __restrict__ blur) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[kTH * kTW];
    __shared__ __attribute__((aligned(16))) uint8_t sc[kSH * kSW];
    __shared__ int s_list[kTY * kCellCap];   // (cell slot << 16) | (row << 8) | local x
    __shared__ int s_n, s_nc;
    __shared__ uint16_t s_corner[kSH * kSW];  // FAST corners of the score tile: (row << 8) | col
    __shared__ int s_hist[256];               // this tile's NMS corners by FAST score
    __shared__ __attribute__((aligned(16))) uint8_t bin_[kBH * kBW];
    __shared__ __attribute__((aligned(16))) float brow[kBH * kTX];
    // Tiles XCD by XCD (block x runs on XCD x mod 8): XCD i takes the i-th contiguous run of the
    // (level, raster) tile order, so a tile's vertical and horizontal neighbours — which stage the
    // same halo rows and columns — mostly share its L2 instead of fetching them again from HBM.
    const int b = [] {
        const int nb = (int)gridDim.x, xcd = (int)(blockIdx.x & 7u), qb = nb >> 3, rem = nb & 7;
        return xcd * qb + min(xcd, rem) + (int)(blockIdx.x >> 3);
    }();
    pyr += blockIdx.z * a.fs_pyr;
    blur += blockIdx.z * a.fs_pyr;
    cand += blockIdx.z * a.fs_cells * kCellCap;
    cell_count += blockIdx.z * a.fs_cells;
    hist += blockIdx.z * a.fs_hist;
    int l = 0;
    while (l + 1 < a.L && b >= a.tile_base[l + 1]) ++l;
    const int W = a.lw[l], H = a.lh[l];
    const uint8_t* img = pyr + a.off[l];
    const int t = b - a.tile_base[l];
    const int ntx = a.ntx[l];
    const int tx = t % ntx, ty = t / ntx;
    const int x0 = tx * kTX, y0 = ty * kTY;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    VX_KT(4);
    if (tid == 0) s_n = s_nc = 0;
    s_hist[tid] = 0;
    static_assert(kBlock == 256, "one histogram bin per thread");
    // (interior tiles: the aligned dword reads of the last column reach 3 bytes past the staged row)
    if (x0 >= 4 && x0 + kTW <= W && y0 >= 4 && y0 - 4 + kTH <= H)
        stage_dw<kTH, kTW / 4>(tile, img + (long long)(y0 - 4) * W + (x0 - 4), W);
    else
        stage_lds<kBlock, (kTH * kTW + kBlock - 1) / kBlock>(tile, kTH * kTW, [&](int i) {
            const int r = i / kTW, c = i - r * kTW;
            const int gy = min(max(y0 - 4 + r, 0), H - 1);
            const int gx = min(max(x0 - 4 + c, 0), W - 1);
            return img[(long long)gy * W + gx];
        });
    if (x0 >= 4 && x0 + kBW <= W && y0 >= 3 && y0 - 3 + kBH <= H)
        stage_dw<kBH, kBW / 4>(bin_, img + (long long)(y0 - 3) * W + (x0 - 4), W);
    else
        stage_lds<kBlock, (kBH * kBW + kBlock - 1) / kBlock>(bin_, kBH * kBW, [&](int i) {
            const int r = i / kBW, c = i - r * kBW;
            return img[(long long)refl101(y0 - 3 + r, H) * W + refl101(x0 - 4 + c, W)];
        });
    __syncthreads();
    VX_KT(5);
    const int thr = a.fast_threshold;
    // FAST ring test per pixel quad: score-tile pixel (r, c) is (x0 - 1 + c, y0 - 1 + r), tile
    // (r + 3, c + 3); its 7 ring rows are tile rows r .. r + 6 and the quad's ring columns lie in
    // the 12 bytes from tile column 4g.  Corners go to a list; the score tile is zeroed.
    for (int i = tid; i < kSH * kSQ; i += kBlock) {
        const int r = i / kSQ, g = i - r * kSQ;
        const uint32_t* rp = reinterpret_cast<const uint32_t*>(tile + r * kTW) + g;
        uint32_t w[7][3];
#pragma unroll
        for (int d = 0; d < 7; ++d)
#pragma unroll
            for (int k = 0; k < 3; ++k) w[d][k] = rp[d * (kTW / 4) + k];
        const int y = y0 - 1 + r;
        unsigned cm = 0;
        // pixel pairs (4g + 2h, 4g + 2h + 1) in 16-bit lanes: bright <=> (v + thr) - p < 0 and dark
        // <=> p - (v - thr) < 0, exact in 16 bits (|results| <= 510); the sign bit of lane k's
        // difference becomes bit k of the pixel's ring mask — no per-sample compare-to-mask round
        // trip, and both masks branch-free
        const vx_i16x2 T2 = {(short)thr, (short)thr};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const vx_i16x2 V = win_pair(w[3], 2 * h + 3);
            const vx_i16x2 VT = V + T2, VM = V - T2;
            vx_u16x2 mb = {0, 0}, md = {0, 0};
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const vx_i16x2 P = win_pair(w[3 + ring_dy(k)], 2 * h + 3 + ring_dx(k));
                const vx_u16x2 db = __builtin_bit_cast(vx_u16x2, (vx_i16x2)(VT - P));
                const vx_u16x2 dd = __builtin_bit_cast(vx_u16x2, (vx_i16x2)(P - VM));
                const vx_u16x2 bit = {(unsigned short)(1u << k), (unsigned short)(1u << k)};
                mb |= (db >> (unsigned short)(15 - k)) & bit;
                md |= (dd >> (unsigned short)(15 - k)) & bit;
            }
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int j = 2 * h + jj;
                const int x = x0 - 1 + 4 * g + j;
                const uint32_t bright = jj ? mb.y : mb.x, dark = jj ? md.y : md.x;
                const bool ok = 4 * g + j < kSW - 2 && y >= 3 && y < H - 3 && x >= 3 && x < W - 3;
                cm |= ((unsigned)ok & ((unsigned)has_run9(bright) | (unsigned)has_run9(dark))) << j;
            }
        }
        *reinterpret_cast<uint32_t*>(sc + r * kSW + 4 * g) = 0u;
        if (cm) {
            int k = atomicAdd(&s_nc, __popc(cm));
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (cm & (1u << j)) s_corner[k++] = (uint16_t)((r << 8) | (4 * g + j));
        }
    }
    // blur row pass 8U -> 32F (float separable GaussianBlur): output columns 4q .. 4q+3
    // of blur row r take bin_ bytes 4q + j + 1 .. 4q + j + 7 (bin_ column 0 is x0 - 4)
    const float k0 = a.gk[0], k1 = a.gk[1], k2 = a.gk[2], k3 = a.gk[3], k4 = a.gk[4], k5 = a.gk[5], k6 = a.gk[6];
    for (int i = tid; i < kBH * (kTX / 4); i += kBlock) {
        const int r = i / (kTX / 4), q = i - r * (kTX / 4);
        const uint32_t* bp = reinterpret_cast<const uint32_t*>(bin_ + r * kBW) + q;
        const uint32_t w[3] = {bp[0], bp[1], bp[2]};
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float s = k0 * (float)win_byte(w, j + 1);
            s += k1 * (float)win_byte(w, j + 2);
            s += k2 * (float)win_byte(w, j + 3);
            s += k3 * (float)win_byte(w, j + 4);
            s += k4 * (float)win_byte(w, j + 5);
            s += k5 * (float)win_byte(w, j + 6);
            s += k6 * (float)win_byte(w, j + 7);
            o[j] = s;
        }
        *reinterpret_cast<float4*>(brow + r * kTX + 4 * q) = make_float4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
    VX_KT(6);
    // cornerScore<16> for the listed corners only
    {
        const int nc = s_nc;
        for (int i = tid; i < nc; i += kBlock) {
            const int v = s_corner[i], r = v >> 8, c = v & 255;
            sc[r * kSW + c] = (uint8_t)fast_score(tile + (r + 3) * kTW + c + 3, kTW, thr);
        }
    }
    {  // blur column pass 32F -> 8U (symmetric form, round half to even), one output quad per thread
        uint8_t* out = blur + a.off[l];
        const float4* b4 = reinterpret_cast<const float4*>(brow);
        for (int i = tid; i < kTY * (kTX / 4); i += kBlock) {
            const int r = i / (kTX / 4), q = i - r * (kTX / 4);
            const int y = y0 + r, xq = x0 + 4 * q;
            if (y >= H || xq >= W) continue;
            float4 m[7];
#pragma unroll
            for (int d = 0; d < 7; ++d) m[d] = b4[(r + d) * (kTX / 4) + q];
            int v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                auto at = [&](int d) { return j == 0 ? m[d].x : j == 1 ? m[d].y : j == 2 ? m[d].z : m[d].w; };
                float s = k3 * at(3) + 0.0f;
                s += k4 * (at(4) + at(2));
                s += k5 * (at(5) + at(1));
                s += k6 * (at(6) + at(0));
                v[j] = min(255, max(0, __float2int_rn(s)));
            }
            uint8_t* dst = out + (long long)y * W + xq;
            if (xq + 3 < W && ((reinterpret_cast<uintptr_t>(dst) & 3u) == 0)) {
                *reinterpret_cast<uint32_t*>(dst) = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) |
                                                    ((uint32_t)v[3] << 24);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (xq + j < W) dst[j] = (uint8_t)v[j];
            }
        }
    }
    __syncthreads();
    const int e = a.edge;
    for (int r = wv; r < kTY; r += kBlock / 64) {
        const int y = y0 + r, x = x0 + lane;
        bool is_c = false;
        if (y >= e && y < H - e && x >= e && x < W - e) {
            const uint8_t* q = sc + (r + 1) * kSW + lane + 1;
            const int s = q[0];
            is_c = s && s > q[-1] && s > q[1] && s > q[-kSW - 1] && s > q[-kSW] && s > q[-kSW + 1] &&
                   s > q[kSW - 1] && s > q[kSW] && s > q[kSW + 1];
        }
        const unsigned long long m = __ballot(is_c);
        if (y < H && lane == 0) cell_count[a.cell_base[l] + y * ntx + tx] = __popcll(m);
        if (is_c) {
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            const int j = atomicAdd(&s_n, 1);
            s_list[j] = (rank << 16) | (r << 8) | lane;
        }
    }
    __syncthreads();
    VX_KT(7);
    // Harris 7x7 (HarrisResponses): four candidates per wave, 16 lanes each; lane s of a group
    // takes window pixels s, s + 16, s + 32 (and 48) and the integer sums are reduced over the 16
    // lanes (exact in any order).
    const int n = s_n;
    const int grp = lane >> 4, sl = lane & 15;
    for (int j0 = wv * 4; j0 < n; j0 += (kBlock / 64) * 4) {
        const int j = j0 + grp;
        const bool valid = j < n;
        const int v = valid ? s_list[j] : 0;
        const int xl = v & 255, r = (v >> 8) & 255, rank = v >> 16;
        int ia = 0, ib = 0, ic = 0;
        if (valid) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = sl + 16 * q;
                if (e < 49) {
                    const int dy = e / 7 - 3, dx = e % 7 - 3;
                    const uint8_t* p = tile + (r + 4 + dy) * kTW + xl + 4 + dx;
                    const int Ix = (p[1] - p[-1]) * 2 + (p[-kTW + 1] - p[-kTW - 1]) + (p[kTW + 1] - p[kTW - 1]);
                    const int Iy = (p[kTW] - p[-kTW]) * 2 + (p[kTW - 1] - p[-kTW - 1]) + (p[kTW + 1] - p[-kTW + 1]);
                    ia += Ix * Ix;
                    ib += Iy * Iy;
                    ic += Ix * Iy;
                }
            }
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
            ia += __shfl_xor(ia, o, 64);
            ib += __shfl_xor(ib, o, 64);
            ic += __shfl_xor(ic, o, 64);
        }
        if (valid && sl == 0) {
            const float scale = 1.f / ((1 << 2) * 7 * 255.f);
            const float s4 = scale * scale * scale * scale;
            const float fa = (float)ia, fb = (float)ib, fc = (float)ic;
            const int sco = sc[(r + 1) * kSW + xl + 1];
            CandRec c;
            c.xy = (unsigned)(x0 + xl) | ((unsigned)(y0 + r) << 16);
            c.score = sco;
            c.harris = (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * s4;
            c.pad = 0;
            cand[cand_at(a.cell_base[l] + (y0 + r) * ntx + tx, rank, a.fs_cells)] = c;
            atomicAdd(&s_hist[sco], 1);
        }
    }
    __syncthreads();
    {
        const int hc = s_hist[tid];
        if (hc) atomicAdd(&hist[(l * kHistRep + (int)(blockIdx.x % kHistRep)) * 256 + tid], hc);
    }
    VX_KT(8);
}

// ------------------------------------------------------------------------------ select
__device__ __forceinline__ unsigned f2key(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
    const unsigned u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(u);
}

constexpr int kSelBlock = 1024;
constexpr int kCellsPer = 6;      // max cells per thread per gather pass
#ifndef VX_SEL_RECBATCH
#define VX_SEL_RECBATCH 8
#endif
constexpr int kRecBatch = VX_SEL_RECBATCH;  // candidate records per thread loaded in one batch
constexpr int kSelRecLds = 2048;  // survivors kept in LDS
constexpr int kSelBins = 2048;    // one-pass select: histogram of the keys' top 11 bits

// Descending-digit search over a 256-bin histogram held by threads 0..255: returns (via the
// block) the largest digit d with count(bins >= d) >= k, and the count strictly above d.
__device__ __forceinline__ void find_digit(int bin_count_desc, int k, int* sh, int* s_out) {
    int tot;
    const int ex = block_scan_excl<kSelBlock>(bin_count_desc, sh, tot);
    const int tid = threadIdx.x;
    if (tid < 256 && ex < k && ex + bin_count_desc >= k) {
        s_out[0] = 255 - tid;
        s_out[1] = ex;
    }
    __syncthreads();
}

// One workgroup per level: retainBest(2q) by FAST score, then retainBest(q) by Harris, both as
// the exact OpenCV sets {response >= k-th largest}, kept in raster (cell) order.
__global__ __launch_bounds__(kSelBlock) void k_select(const CandRec* __restrict__ cand,
                                                      const int* __restrict__ cell_count,
                                                      const int* __restrict__ hist, LevelArgs a,
                                                      CandRec* __restrict__ stage,
                                                      int* __restrict__ level_count) {
    __shared__ int sw[kSelBlock / 64];
    __shared__ int sh[kSelBins];  // radix histogram (256 bins) / the one-pass histogram (2048)
    __shared__ int s_out[2];
    __shared__ unsigned s_bucket[64];
    __shared__ CandRec srec[kSelRecLds];  // retainBest(2q) survivors (32 KB)
    const int l = blockIdx.x;
    const int tid = threadIdx.x;
    cand += blockIdx.z * a.fs_cells * kCellCap;
    cell_count += blockIdx.z * a.fs_cells;
    hist += blockIdx.z * a.fs_hist;
    stage += blockIdx.z * a.fs_stage;
    level_count += blockIdx.z * kMaxLevels;
    VX_KT(12);
    const int ncell = a.lh[l] * a.ntx[l];
    const long long cbase = a.cell_base[l];
    CandRec* kept = stage + a.stage_base[l];                      // retainBest(2q) result
    CandRec* fin = stage + a.stage_base[l] + a.level_cap[l];      // retainBest(q) result
    const int q = a.quota[l];
    const int k1 = 2 * q;
    // the first gather pass's cell counts do not depend on thr1: their loads are issued before the
    // histogram scan so that their latency passes during it
    const int cpt = min(kCellsPer, (ncell + kSelBlock - 1) / kSelBlock);
    int cnt0[kCellsPer];
#pragma unroll
    for (int j = 0; j < kCellsPer; ++j) {
        const int c = tid * cpt + j;
        cnt0[j] = (k1 > 0 && j < cpt && c < ncell) ? cell_count[cbase + c] : 0;
    }
    // the first pass's records depend only on the counts, not on thr1: they are requested now, so
    // their latency passes while wave 0 derives thr1 from the histogram (no block barrier there:
    // a barrier would wait for these loads)
    int tot0 = 0;
#pragma unroll
    for (int j = 0; j < kCellsPer; ++j) tot0 += cnt0[j];
    auto rec_index_of = [&](const int (&cn)[kCellsPer], int c0, int k) {
        int j = 0, i = k;
#pragma unroll
        for (int jj = 0; jj < kCellsPer; ++jj)
            if (j == jj && i >= cn[jj]) {
                i -= cn[jj];
                j = jj + 1;
            }
        return cand_at(cbase + c0 + j, i, a.fs_cells);
    };
    CandRec rr0[kRecBatch];
#pragma unroll
    for (int k = 0; k < kRecBatch; ++k) rr0[k] = k < tot0 ? cand[rec_index_of(cnt0, tid * cpt, k)] : CandRec{};
    // ---- level histogram of FAST scores (border-passing NMS corners) -> thr1, on wave 0: lane L
    // holds the bins 255 - 4L .. 252 - 4L (descending), an inclusive wave scan gives the count of
    // candidates at or above each bin; thr1 = the largest score whose count reaches 2q (A.3)
    if ((tid >> 6) == 0) {
        const int lane = tid & 63;
        int c[4], ls = 0;
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
            int h = 0;
#pragma unroll
            for (int r = 0; r < kHistRep; ++r) h += hist[(l * kHistRep + r) * 256 + 255 - (4 * lane + q2)];
            c[q2] = h;
            ls += h;
        }
        int incl = ls;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const int n = __shfl(incl, 63, 64);
        int t1 = 0;
        if (n > k1 && k1 > 0) {
            const unsigned long long m = __ballot(incl >= k1);
            const int first = __ffsll((long long)m) - 1;
            int cand_t = 0;
            if (lane == first) {
                int cum = incl - ls;
#pragma unroll
                for (int q2 = 0; q2 < 4; ++q2) {
                    cum += c[q2];
                    if (cum >= k1 && cand_t == 0 && c[q2] > 0) cand_t = 256 - (4 * lane + q2);  // score + 1
                }
            }
            t1 = __shfl(cand_t, first, 64) - 1;
        }
        if (lane == 0) s_out[0] = t1;
    }
    __syncthreads();
    const int thr1 = s_out[0];
    VX_KT(9);
    // ---- gather kept candidates (score >= thr1) in raster order.  Each thread owns cpt
    // consecutive cells: their counts are loaded in one batch, then up to kRecBatch of their
    // records in one batch (a per-record loop would expose one memory latency per record).
    // Survivors go to LDS (when they fit) and to the global staging list.
    int K1 = 0;
    if (k1 > 0) {
        for (int base = 0; base < ncell; base += kSelBlock * cpt) {
            const int c0 = base + tid * cpt;
            int cnts[kCellsPer];
            int tot = 0;
#pragma unroll
            for (int j = 0; j < kCellsPer; ++j) {
                cnts[j] = base == 0 ? cnt0[j] : (j < cpt && c0 + j < ncell) ? cell_count[cbase + c0 + j] : 0;
            }
#pragma unroll
            for (int j = 0; j < kCellsPer; ++j) tot += cnts[j];
            // k-th record of this thread -> cand index
            auto rec_index = [&](int k) { return rec_index_of(cnts, c0, k); };
            CandRec rr[kRecBatch];
#pragma unroll
            for (int k = 0; k < kRecBatch; ++k) rr[k] = base == 0 ? rr0[k] : k < tot ? cand[rec_index(k)] : CandRec{};
            int kc = 0;
#pragma unroll
            for (int k = 0; k < kRecBatch; ++k) kc += (k < tot && rr[k].score >= thr1) ? 1 : 0;
            for (int k0 = kRecBatch; k0 < tot; k0 += kRecBatch) {  // (a batch of loads at a time)
                CandRec rb[kRecBatch];
#pragma unroll
                for (int k = 0; k < kRecBatch; ++k) rb[k] = k0 + k < tot ? cand[rec_index(k0 + k)] : CandRec{};
#pragma unroll
                for (int k = 0; k < kRecBatch; ++k) kc += (k0 + k < tot && rb[k].score >= thr1) ? 1 : 0;
            }
            if (base == 0) VX_KT(10);
            int btot;
            int pos = K1 + block_scan_excl<kSelBlock>(kc, sw, btot);
            if (base == 0) VX_KT(11);
            auto put = [&](const CandRec& r) {
                if (pos < kSelRecLds) srec[pos] = r;
                kept[pos] = r;
                ++pos;
            };
#pragma unroll
            for (int k = 0; k < kRecBatch; ++k)
                if (k < tot && rr[k].score >= thr1) put(rr[k]);
            for (int k0 = kRecBatch; k0 < tot; k0 += kRecBatch) {
                CandRec rb[kRecBatch];
#pragma unroll
                for (int k = 0; k < kRecBatch; ++k) rb[k] = k0 + k < tot ? cand[rec_index(k0 + k)] : CandRec{};
#pragma unroll
                for (int k = 0; k < kRecBatch; ++k)
                    if (k0 + k < tot && rb[k].score >= thr1) put(rb[k]);
            }
            K1 += btot;
        }
    }
    __syncthreads();
    VX_KT(13);
    // ---- retainBest(q) by Harris: exact q-th largest key by a 4-pass radix select over the
    // survivors (keys held in registers when K1 <= 2 * kSelBlock), then an ordered compaction
    int K2 = 0;
    if (q > 0 && K1 > 0) {
        const CandRec* kr = K1 <= kSelRecLds ? srec : kept;
        float thr2 = -INFINITY;
        if (K1 > q) {
            const bool in_regs = K1 <= 2 * kSelBlock;
            unsigned key0 = 0, key1 = 0;
            if (in_regs) {
                if (tid < K1) key0 = f2key(kr[tid].harris);
                if (tid + kSelBlock < K1) key1 = f2key(kr[tid + kSelBlock].harris);
            }
            unsigned prefix = 0, mask = 0;
            int k = q;
            bool done = false;
            if (in_regs) {
                // one pass: a histogram of the keys over kSelBins equal bins of [min, max] (keys of
                // similar responses share their top bits, so fixed top-bit bins crowd); wave 0
                // finds the bin d holding the q-th largest key and the count above it; when that
                // bin holds <= 64 keys they are compacted to LDS and wave 0 ranks them exactly
                // (lane i: keys above / equal to its own) — the 4-pass radix below is the
                // fallback for a crowded bin.  The bin is a monotone function of the key, so the
                // counts above a bin are exact.
                unsigned kmn = ~0u, kmx = 0u;
                if (tid < K1) kmn = min(kmn, key0), kmx = max(kmx, key0);
                if (tid + kSelBlock < K1) kmn = min(kmn, key1), kmx = max(kmx, key1);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    kmn = min(kmn, (unsigned)__shfl_xor((int)kmn, o, 64));
                    kmx = max(kmx, (unsigned)__shfl_xor((int)kmx, o, 64));
                }
                if ((tid & 63) == 0) {
                    s_bucket[tid >> 6] = kmn;
                    s_bucket[32 + (tid >> 6)] = kmx;
                }
                for (int i = tid; i < kSelBins; i += kSelBlock) sh[i] = 0;
                if (tid == 0) s_out[0] = 0;
                __syncthreads();
#pragma unroll
                for (int w2 = 0; w2 < kSelBlock / 64; ++w2) {
                    kmn = min(kmn, s_bucket[w2]);
                    kmx = max(kmx, s_bucket[32 + w2]);
                }
                const float scale = (float)kSelBins / ((float)(kmx - kmn) + 1.0f);
                auto bin_of = [&](unsigned key) { return min(kSelBins - 1, (int)((float)(key - kmn) * scale)); };
                const int b0 = tid < K1 ? bin_of(key0) : -1, b1 = tid + kSelBlock < K1 ? bin_of(key1) : -1;
                if (b0 >= 0) atomicAdd(&sh[b0], 1);
                if (b1 >= 0) atomicAdd(&sh[b1], 1);
                __syncthreads();
                if ((tid >> 6) == 0) {
                    const int lane = tid & 63;
                    constexpr int kPer = kSelBins / 64;  // bins per lane, descending
                    int c[kPer], ls = 0;
#pragma unroll
                    for (int j = 0; j < kPer; ++j) {
                        c[j] = sh[kSelBins - 1 - (kPer * lane + j)];
                        ls += c[j];
                    }
                    int incl = ls;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int y = __shfl_up(incl, o, 64);
                        if (lane >= o) incl += y;
                    }
                    const unsigned long long m = __ballot(incl >= q);  // (K1 > q: some lane reaches q)
                    const int first = __ffsll((long long)m) - 1;
                    if (lane == first) {
                        int cum = incl - ls, d = -1, above = 0;
#pragma unroll
                        for (int j = 0; j < kPer; ++j)
                            if (d < 0) {
                                if (cum + c[j] >= q) {
                                    d = kSelBins - 1 - (kPer * lane + j);
                                    above = cum;
                                }
                                cum += c[j];
                            }
                        s_out[1] = d | (above << 12);
                    }
                }
                __syncthreads();
                const int d = s_out[1] & 0xfff, above = s_out[1] >> 12, nb = sh[d];
                if (nb <= 64) {
                    if (b0 == d) s_bucket[atomicAdd(&s_out[0], 1)] = key0;
                    if (b1 == d) s_bucket[atomicAdd(&s_out[0], 1)] = key1;
                    __syncthreads();
                    if ((tid >> 6) == 0) {
                        const int lane = tid & 63, kk = q - above;  // rank of the wanted key in the bin
                        const unsigned mine = lane < nb ? s_bucket[lane] : 0u;
                        int gt = 0, eq = 0;
                        for (int j = 0; j < nb; ++j) {
                            const unsigned o = (unsigned)__shfl((int)mine, j, 64);
                            gt += o > mine;
                            eq += o == mine;
                        }
                        if (lane < nb && gt < kk && gt + eq >= kk) s_out[1] = (int)mine;  // (equal keys: same value)
                    }
                    __syncthreads();
                    prefix = (unsigned)s_out[1];
                    done = true;
                }
                __syncthreads();  // (s_out / sh reused below)
            }
            for (int shift = 24; shift >= 0 && !done; shift -= 8) {
                if (tid < 256) sh[tid] = 0;
                __syncthreads();
                if (in_regs) {
                    if (tid < K1 && (key0 & mask) == prefix) atomicAdd(&sh[(key0 >> shift) & 255], 1);
                    if (tid + kSelBlock < K1 && (key1 & mask) == prefix) atomicAdd(&sh[(key1 >> shift) & 255], 1);
                } else {
                    for (int j = tid; j < K1; j += kSelBlock) {
                        const unsigned key = f2key(kr[j].harris);
                        if ((key & mask) == prefix) atomicAdd(&sh[(key >> shift) & 255], 1);
                    }
                }
                __syncthreads();
                const int v = tid < 256 ? sh[255 - tid] : 0;
                find_digit(v, k, sw, s_out);
                const unsigned digit = (unsigned)s_out[0];
                k -= s_out[1];
                prefix |= digit << shift;
                mask |= 255u << shift;
                __syncthreads();
            }
            thr2 = key2f(prefix);
        }
        VX_KT(14);
        for (int base = 0; base < K1; base += kSelBlock) {
            const int j = base + tid;
            CandRec r{};
            int f = 0;
            if (j < K1) {
                r = kr[j];
                f = r.harris >= thr2;
            }
            int cnt;
            const int pos = block_scan_excl<kSelBlock>(f, sw, cnt);
            if (f) fin[K2 + pos] = r;
            K2 += cnt;
        }
    }
    if (tid == 0) level_count[l] = K2;
    VX_KT(15);
}

// ------------------------------------------------------------------------------ select, libstdc++ order
// OpenCV's KeyPointsFilter::retainBest leaves the keypoints in the order std::nth_element +
// std::partition produce (ORB calls it twice per level: by FAST score, then by Harris; SURVEY.md
// App. A.3), and ORBExtractor::Extract numbers Frame::Features() in that order
// (core/feature/orb_extractor.cpp:13-24).  k_select_stl reproduces libstdc++'s permutation
// exactly: introselect (median-of-3 moved to the front, unguarded Hoare partition, depth limit
// 2*lg(n) -> heap select, insertion sort of the last <= 3), then the bidirectional std::partition.
//
// One Hoare partition is done as ONE parallel pass instead of two scanning pointers: with pivot
// value P, the left scanner stops at every x with !(x > P) ("L"), the right one at every x with
// !(P > x) ("R"); swap k exchanges the k-th L from the left with the k-th R from the right for
// k < K, K = max over x of min(#L before x, #R at or after x), and the returned cut is
// min(L[K], R[K-1]).  std::partition is the same pairing with complementary predicates.  The
// passes evaluate it without computing K (swap_l / swap_r below: each element's swap from its own
// L / R ranks, the cut from ballots).  That formulation and the K-free rules are checked against the
// real STL (random, tie-heavy, sorted and McIlroy-adversarial inputs reaching the heap select) by
// tests/cpp/stl_select_model.cpp.
//
// The passes run on a register-resident engine (below): the range stays in registers across
// them.  Elements are u32 (FAST score << 24 | raster index) for the first retainBest and u64
// (order-preserving Harris key << 32 | raster index) for the second; the arrays live in LDS when
// they fit, in the level's global scratch otherwise.
#ifndef VX_SEL_THREADS
#define VX_SEL_THREADS 1024
#endif
constexpr int kStlNT = VX_SEL_THREADS;
constexpr int kStlWaves = kStlNT / 64;
constexpr int kStlLds = 160 * 1024 - 256;      // dynamic LDS of k_select_stl: the engine's, then the arrays

__device__ __forceinline__ unsigned sel_key(unsigned v) { return v >> 24; }
__device__ __forceinline__ unsigned sel_key(unsigned long long v) { return (unsigned)(v >> 32); }

// order-preserving key of a Harris response (-0 and +0 compare equal as floats: one key)
__device__ __forceinline__ unsigned harris_key(float f) {
    unsigned u = __float_as_uint(f);
    if ((u << 1) == 0u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

typedef unsigned long long u64;
// a wave-uniform value read from memory, declared uniform (keeps the pass's control flow scalar)
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ unsigned uni(unsigned x) { return (unsigned)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ u64 uni(u64 x) { return ((u64)uni((unsigned)(x >> 32)) << 32) | uni((unsigned)x); }

__device__ __forceinline__ int lane_rank(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

template <int NW>
__device__ __forceinline__ void team_sync() {
    if (NW > 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// One partition pass over [f0, l) by the first NW waves of the workgroup (NW = 1: wave 0 only).
// m >= 0: position m is read as `oldf` (the median-of-3 swap with the pivot slot f0 - 1, which
// receives pv; both written here).  Returns the cut; n_r = number of R elements.
// s: LDS scratch of >= 3 * NW + 2 ints.
template <int NW, class T, class IsL, class IsR>
__device__ __forceinline__ int team_pass(T* __restrict__ A, T* __restrict__ bl, T* __restrict__ br, int f0, int l,
                                         int m, T oldf, T pv, IsL isl, IsR isr, int* s, int& n_r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nb = (l - f0 + 63) >> 6;
    const int b0 = w * nb / NW, b1 = (w + 1) * nb / NW;
    auto rd = [&](int p) -> T { return p == m ? oldf : A[p]; };
    int cl = 0, cr = 0;
    for (int b = b0; b < b1; ++b) {
        const int p = f0 + 64 * b + lane;
        const bool in = p < l;
        const T v = in ? rd(p) : T(0);
        cl += __popcll(__ballot(in && isl(v)));
        cr += __popcll(__ballot(in && isr(v)));
    }
    int pl = 0, pr = 0, nl = cl, nr = cr;
    if (NW > 1) {
        if (lane == 0) {
            s[2 * w] = cl;
            s[2 * w + 1] = cr;
        }
        __syncthreads();
        nl = nr = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int x = uni(s[2 * i]), y = uni(s[2 * i + 1]);
            pl += i < w ? x : 0;
            pr += i < w ? y : 0;
            nl += x;
            nr += y;
        }
    }
    // K = max over positions x of min(#L in [f0, x), #R in [x, l))
    int km = 0;
    {
        int ql = pl, qr = pr;
        for (int b = b0; b < b1; ++b) {
            const int p = f0 + 64 * b + lane;
            const bool in = p < l;
            const T v = in ? rd(p) : T(0);
            const unsigned long long ml = __ballot(in && isl(v)), mr = __ballot(in && isr(v));
            if (in) km = max(km, min(ql + lane_rank(ml), nr - (qr + lane_rank(mr))));
            ql += __popcll(ml);
            qr += __popcll(mr);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) km = max(km, __shfl_xor(km, o, 64));
    if (NW > 1) {
        if (lane == 0) s[2 * NW + w] = km;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NW; ++i) km = max(km, uni(s[2 * NW + i]));
    }
    const int K = km;
    // mailboxes: the k-th L and the k-th R from the right (k < K); the cut's two candidates
    {
        int ql = pl, qr = pr;
        for (int b = b0; b < b1; ++b) {
            const int p = f0 + 64 * b + lane;
            const bool in = p < l;
            const T v = in ? rd(p) : T(0);
            const bool il = in && isl(v), ir = in && isr(v);
            const unsigned long long ml = __ballot(il), mr = __ballot(ir);
            const int lb = ql + lane_rank(ml), rr = nr - 1 - (qr + lane_rank(mr));
            if (il) {
                if (lb < K) bl[lb] = v;
                else if (lb == K) s[3 * NW] = p;
            }
            if (ir) {
                if (rr < K) br[rr] = v;
                if (rr == K - 1) s[3 * NW + 1] = p;
            }
            ql += __popcll(ml);
            qr += __popcll(mr);
        }
    }
    team_sync<NW>();
    {
        int ql = pl, qr = pr;
        for (int b = b0; b < b1; ++b) {
            const int p = f0 + 64 * b + lane;
            const bool in = p < l;
            const T v = in ? rd(p) : T(0);
            const bool il = in && isl(v), ir = in && isr(v);
            const unsigned long long ml = __ballot(il), mr = __ballot(ir);
            const int lb = ql + lane_rank(ml), rr = nr - 1 - (qr + lane_rank(mr));
            if (il && lb < K) A[p] = br[lb];
            else if (ir && rr < K) A[p] = bl[rr];
            else if (p == m) A[p] = oldf;
            ql += __popcll(ml);
            qr += __popcll(mr);
        }
        if (m >= 0 && threadIdx.x == 0) A[f0 - 1] = pv;
    }
    team_sync<NW>();
    n_r = nr;
    int cut = INT_MAX;
    if (K < nl) cut = uni(s[3 * NW]);
    if (K > 0) cut = min(cut, uni(s[3 * NW + 1]));
    return cut;
}

// ---- the pass engine
// Between passes the array lives in memory (LDS, or the level's global scratch).  A pass loads
// exactly its range into registers, densely (block j = the 64 positions from 64 j, one per lane;
// NB blocks, a power of two fixed at compile time), partitions it there and writes back the
// elements that moved: its instruction count follows the range, so the long tail of short
// introselect steps stays cheap.  Ranges of up to kRgWave run on wave 0 alone (pivot candidates
// are broadcast loads, the swaps and the cut come from lane ranks and ballots (swap_l / swap_r
// below), the mailboxes need no barrier); the last steps of a range of <= 64 stay in wave 0's
// registers (rg_tail64).  Longer ranges (up to RgCap: 8192 u32 / 4096 u64) run as team passes
// spread over kRgSpread waves (16: four per SIMD, up to 8 blocks each): block counts, the swapped
// elements and per-wave cut candidates go through LDS, three barriers a pass.
template <class T> struct RgCap { static constexpr int v = sizeof(T) == 4 ? 8192 : 4096; };
constexpr int kRgCap32 = 8192;                 // C4 level 0: ~6.9k FAST candidates
#ifndef VX_SEL_WAVE
#define VX_SEL_WAVE 256
#endif
#ifndef VX_SEL_SPREAD
#define VX_SEL_SPREAD 16
#endif
constexpr int kRgWave = VX_SEL_WAVE;           // wave-0 passes up to this range (longer: team passes)
constexpr int kRgSpread = VX_SEL_SPREAD;       // team passes spread their blocks over this many waves
constexpr int kRgMail = 16400;                 // bytes per mailbox: (8192 / 2 + 1) u32 = (4096 / 2 + 1) u64
constexpr int kRgTrash = 4 * kRgMail + 32 + 64 * 4 + 32;  // + 4 spare slots + 64 ints; 16-aligned
constexpr int kRgBytes = kRgTrash + 64 * 8 + 64 * 4;       // + one value and one int trash slot per lane
static_assert(kRgBytes % 16 == 0, "engine scratch alignment");
static_assert(kRgCap32 <= 64 * 8 * kStlWaves && RgCap<u64>::v <= 64 * 8 * kStlWaves,
              "a team pass (<= 8 blocks a wave) must cover the engine's capacity: VX_SEL_THREADS >= 1024");

// the engine's LDS: value mailboxes bl / br, (unused) position mailboxes lp / rp, a few ints
// (per-wave counts and cut candidates, results)
struct RgLds {
    unsigned char* p;
    template <class T> __device__ __forceinline__ T* bl() const { return reinterpret_cast<T*>(p); }
    template <class T> __device__ __forceinline__ T* br() const { return reinterpret_cast<T*>(p + kRgMail); }
    __device__ __forceinline__ int* lp() const { return reinterpret_cast<int*>(p + 2 * kRgMail); }
    __device__ __forceinline__ int* rp() const { return reinterpret_cast<int*>(p + 3 * kRgMail); }
    __device__ __forceinline__ int* s() const { return reinterpret_cast<int*>(p + 4 * kRgMail + 32); }
    // per-lane trash slots: the target of a lane's write when it has nothing to write (keeps the
    // passes' LDS traffic free of divergent branches)
    template <class T> __device__ __forceinline__ T* tv() const {
        return reinterpret_cast<T*>(p + kRgTrash) + (threadIdx.x & 63);
    }
    // the same as element indices from p (selects between LDS slots stay integer selects: a select
    // between pointers is turned into branches around each access)
    template <class T> static constexpr int kBr = kRgMail / (int)sizeof(T);
    template <class T> static constexpr int kTv = kRgTrash / (int)sizeof(T);
};

// position x of the blocks starting at q0 := val (x anywhere; compares positions, never the block
// index with a runtime value: GVN would turn v[i] into a dynamically indexed v[j] -> scratch)
template <int NB, class T>
__device__ __forceinline__ void rg_put(T (&v)[NB], int q0, int x, T val) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NB; ++i)
        if (q0 + 64 * i + lane == x) v[i] = val;
}
// __move_median_to_first(first, a, b, c, greater): the median's position; pv its value
template <class T>
__device__ __forceinline__ int stl_median(int a, int b, int c, T va, T vb, T vc, T& pv) {
    const unsigned ka = sel_key(va), kb = sel_key(vb), kc = sel_key(vc);
    int m;
    if (ka > kb) m = kb > kc ? b : ka > kc ? c : a;
    else m = ka > kc ? a : kb > kc ? c : b;
    pv = m == a ? va : m == b ? vb : vc;
    return m;
}
template <int NB, class T>
__device__ __forceinline__ void rg_load(T (&v)[NB], const T* __restrict__ A, int q0, int len) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        v[j] = A[min(q0 + 64 * j + lane, len - 1)];  // (lanes past the range: masked out by rg_masks)
    }
}
template <int NB, class T>
__device__ __forceinline__ void rg_store(const T (&v)[NB], T* __restrict__ A, int q0, int len) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int q = q0 + 64 * j + lane;
        if (q < len) A[q] = v[j];
    }
}

// Per block the pass keeps the lane's L / R flags (lane masks; their ballots are the block's
// masks), its L rank (#L before it in the range) and its R rank from the left, both from mbcnt
// with the running prefix as base (ql / qr: the prefixes in, the totals out).  Block counts are
// scalar popcounts of the masks.
__device__ __forceinline__ int mbcnt(u64 m, int base) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, (unsigned)base));
}

// Flags and masks of the blocks from q0 over the range [lo, len): L = key <= P (pivot pass) /
// key < P (partition), R = key >= P
template <int NB, bool kPivot, class T>
__device__ __forceinline__ void rg_masks(const T (&v)[NB], int q0, int lo, int len, unsigned P, bool (&il)[NB],
                                         bool (&ir)[NB]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int x = q0 + 64 * j + lane;
        const bool in = x >= lo && x < len;
        const unsigned k = sel_key(v[j]);
        il[j] = in && (kPivot ? k <= P : k < P);
        ir[j] = in && k >= P;
    }
}
template <int NB>
__device__ __forceinline__ void rg_ranks(const bool (&il)[NB], const bool (&ir)[NB], int& ql, int& qr, int (&ra)[NB],
                                         int (&rb)[NB]) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const u64 ml = __ballot(il[j]), mr = __ballot(ir[j]);
        ra[j] = mbcnt(ml, ql);
        rb[j] = mbcnt(mr, qr);
        ql += __popcll(ml);
        qr += __popcll(mr);
    }
}

// Which elements a pass swaps, without the swap count K: the L of rank ra (#L before it) is swapped
// iff more than ra R lie after it (ra + rb + ir < nr, rb = #R before it), an R iff more L than its
// right rank (nr - 1 - rb) lie before it (ra + rb >= nr) — the k-th L from the left and the k-th R
// from the right are exchanged exactly while the former lies left of the latter.  The cut
// min(L[K], R[K - 1]) is the first position holding an unswapped L or a swapped R.  Both rules are
// checked against the K-based formulation and the real STL by tests/cpp/stl_select_model.cpp.
__device__ __forceinline__ bool swap_l(bool il, bool ir, int ra, int rb, int nr) { return il && ra + rb + (int)ir < nr; }
__device__ __forceinline__ bool swap_r(bool ir, int ra, int rb, int nr) { return ir && ra + rb >= nr; }

// inclusive prefix sum / max over each 16-lane row (DPP row shifts; lanes shifted in read 0)
__device__ __forceinline__ int row_scan_add(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
    return x;
}
__device__ __forceinline__ int row_scan_max(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));
    return x;
}
static_assert(kStlWaves <= 16, "team counts are scanned within one DPP row");

// One pass by wave 0 alone over A[0, len) (A = the range's first element): kPivot, an
// introselect step (median of (1, len / 2, len - 1) moved to 0, unguarded partition of [1, len)
// around it, L = !(x > P), R = !(P > x)); otherwise std::partition of [0, len) by key >= thr
// (L = key < thr, R = key >= thr).  The swapped L of rank k exchanges with the R of rank k from
// the right through the mailboxes (swap_l / swap_r: an element is swapped at most once).  Every
// LDS access is unconditional, lanes with nothing to move using their trash slot: the pass is
// straight-line VALU + LDS code, no exec-mask branches.  Returns the cut min(L[K], R[K - 1])
// (relative to A; the first unswapped L or swapped R, from the blocks' ballots); n_r = #R.
template <int NB, bool kPivot, class T>
__device__ __forceinline__ int rg_wave_pass(T* __restrict__ A, int len, unsigned thr, const RgLds& E, int& n_r) {
    const int lane = threadIdx.x & 63;
    T v[NB];
    rg_load(v, A, 0, len);
    unsigned P = thr;
    int lo = 0, m = -1;
    if (kPivot) {
        const int b = len / 2, c = len - 1;
        const T vf = uni(A[0]), va = uni(A[1]), vb = uni(A[b]), vc = uni(A[c]);
        T pv;
        m = stl_median(1, b, c, va, vb, vc, pv);
        P = sel_key(pv);
        rg_put(v, 0, 0, pv);
        rg_put(v, 0, m, vf);
        lo = 1;
    }
    bool il[NB], ir[NB], sl[NB], sr[NB];
    int ra[NB], rb[NB];
    rg_masks<NB, kPivot>(v, 0, lo, len, P, il, ir);
    int nl = 0, nr = 0;
    rg_ranks(il, ir, nl, nr, ra, rb);
    T* eb = E.bl<T>();  // element slots: bl, then br, then the trash
    constexpr int kBr = RgLds::kBr<T>, kTv = RgLds::kTv<T>;
    int cut = INT_MAX;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        sl[j] = swap_l(il[j], ir[j], ra[j], rb[j], nr);
        sr[j] = swap_r(ir[j], ra[j], rb[j], nr);
        eb[sl[j] ? ra[j] : sr[j] ? kBr + (nr - 1 - rb[j]) : kTv + lane] = v[j];
        if (kPivot) {
            const u64 c = __ballot((il[j] && !sl[j]) || sr[j]);
            cut = (cut == INT_MAX && c != 0ull) ? 64 * j + __ffsll((long long)c) - 1 : cut;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    T nv[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j)  // every read issued before the first store
        nv[j] = eb[sl[j] ? kBr + ra[j] : sr[j] ? nr - 1 - rb[j] : kTv + lane];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int x = 64 * j + lane;
        const bool sw = sl[j] || sr[j];
        if (sw || (kPivot && (x == 0 || x == m))) A[x] = sw ? nv[j] : v[j];
    }
    cut = min(max(cut, 1), len);  // (clamped: memory-safe whatever happens)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // (the next pass reloads; global scratch too)
    n_r = nr;
    return cut;
}

// The same pass by the workgroup over A[0, len), len <= 64 NB kStlWaves: wave w holds the blocks
// [NB w, NB (w + 1)); waves past the range only meet the barriers.  After the first barrier (block
// counts scanned over the waves) every swapped element goes to its mailbox and each wave posts its
// first cut candidate (an unswapped L or a swapped R); after the second the swaps are read back and
// the cut is the least candidate.  Branch-free LDS traffic as above.
template <int NB, bool kPivot, class T>
__device__ __forceinline__ int rg_team_pass(T* __restrict__ A, int len, unsigned thr, const RgLds& E, int& n_r) {
    constexpr int NW = kStlWaves;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int q0 = 64 * NB * w;
    const bool act = q0 < len;
    int* s = E.s();
    T* eb = E.bl<T>();
    constexpr int kBr = RgLds::kBr<T>, kTv = RgLds::kTv<T>;
    T v[NB];
    bool il[NB], ir[NB], sl[NB], sr[NB];
    int ra[NB], rb[NB];
    unsigned P = thr;
    int lo = 0, m = -1;
    if (kPivot) {
        const int b = len / 2, c = len - 1;
        const T vf = uni(A[0]), va = uni(A[1]), vb = uni(A[b]), vc = uni(A[c]);
        T pv;
        m = stl_median(1, b, c, va, vb, vc, pv);
        P = sel_key(pv);
        if (act) {
            rg_load(v, A, q0, len);
            rg_put(v, q0, 0, pv);
            rg_put(v, q0, m, vf);
        }
        lo = 1;
    } else if (act) {
        rg_load(v, A, q0, len);
    }
    int cl = 0, cr = 0;
    if (act) {
        rg_masks<NB, kPivot>(v, q0, lo, len, P, il, ir);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            cl += __popcll(__ballot(il[j]));
            cr += __popcll(__ballot(ir[j]));
        }
    }
    if (lane == 0) *reinterpret_cast<int2*>(s + 2 * w) = make_int2(cl, cr);
    __syncthreads();
    int pl, pr, nr;
    {
        const int2 c2 = lane < NW ? *reinterpret_cast<const int2*>(s + 2 * lane) : make_int2(0, 0);
        const int xl = row_scan_add(c2.x), xr = row_scan_add(c2.y);
        pl = w > 0 ? __builtin_amdgcn_readlane(xl, w - 1) : 0;
        pr = w > 0 ? __builtin_amdgcn_readlane(xr, w - 1) : 0;
        nr = __builtin_amdgcn_readlane(xr, NW - 1);
    }
    int cw = INT_MAX;  // this wave's first cut candidate
    if (act) {
        rg_ranks(il, ir, pl, pr, ra, rb);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            sl[j] = swap_l(il[j], ir[j], ra[j], rb[j], nr);
            sr[j] = swap_r(ir[j], ra[j], rb[j], nr);
            eb[sl[j] ? ra[j] : sr[j] ? kBr + (nr - 1 - rb[j]) : kTv + lane] = v[j];
            if (kPivot) {
                const u64 c = __ballot((il[j] && !sl[j]) || sr[j]);
                cw = (cw == INT_MAX && c != 0ull) ? q0 + 64 * j + __ffsll((long long)c) - 1 : cw;
            }
        }
    }
    if (kPivot && lane == 0) s[2 * NW + w] = INT_MAX - cw;  // (>= 0: max-reduced below)
    __syncthreads();
    int cut = len;
    if (kPivot) {
        cut = INT_MAX - __builtin_amdgcn_readlane(row_scan_max(lane < NW ? s[2 * NW + lane] : 0), NW - 1);
        cut = min(max(cut, 1), len);  // (clamped: memory-safe whatever happens)
    }
    if (act) {
        T nv[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) nv[j] = eb[sl[j] ? kBr + ra[j] : sr[j] ? nr - 1 - rb[j] : kTv + lane];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int x = q0 + 64 * j + lane;
            const bool sw = sl[j] || sr[j];
            if (sw || (kPivot && (x == 0 || x == m))) A[x] = sw ? nv[j] : v[j];
        }
    }
    __syncthreads();
    n_r = nr;
    return cut;
}

// dispatch on the range: the smallest power-of-two block count that holds it
template <bool kPivot, class T>
__device__ __forceinline__ int rg_wave_any(T* __restrict__ A, int len, unsigned thr, const RgLds& E, int& n_r) {
    if (len <= 64) return rg_wave_pass<1, kPivot>(A, len, thr, E, n_r);
    if (len <= 128) return rg_wave_pass<2, kPivot>(A, len, thr, E, n_r);
    if (len <= 256) return rg_wave_pass<4, kPivot>(A, len, thr, E, n_r);
    return rg_wave_pass<8, kPivot>(A, len, thr, E, n_r);
}
// team passes spread the blocks over kRgSpread waves (16: four per SIMD, so each SIMD hides the
// others' LDS latency; measured 20 -> 14 us for the first retainBest of a C3 level 0)
template <bool kPivot, class T>
__device__ __forceinline__ int rg_team_any(T* __restrict__ A, int len, unsigned thr, const RgLds& E, int& n_r) {
    const int per = ((len + 63) / 64 + kRgSpread - 1) / kRgSpread;
    if (per <= 1) return rg_team_pass<1, kPivot>(A, len, thr, E, n_r);
    if (per <= 2) return rg_team_pass<2, kPivot>(A, len, thr, E, n_r);
    if (per <= 4) return rg_team_pass<4, kPivot>(A, len, thr, E, n_r);
    return rg_team_pass<8, kPivot>(A, len, thr, E, n_r);
}

// v_readlane of a wave-uniform lane, for u32 / u64 elements
__device__ __forceinline__ unsigned rdl(unsigned v, int i) { return (unsigned)__builtin_amdgcn_readlane((int)v, i); }
__device__ __forceinline__ u64 rdl(u64 v, int i) {
    return ((u64)(unsigned)__builtin_amdgcn_readlane((int)(v >> 32), i) << 32) |
           (unsigned)__builtin_amdgcn_readlane((int)v, i);
}

// The introselect steps of a range of <= 64 elements on wave 0 with the range in registers: lane i
// holds A[f0 + i] for the whole tail, a step's range is a lane interval [lf, ll) and its pivot
// candidates come from v_readlane; only the swapped pairs go through the mailboxes (one LDS round
// trip a step, no loads or stores of A until the range is written back once).  Same step as
// rg_wave_pass<1, true>; stops at a range of <= 3 or at the depth limit (heap = true), with f / l
// the final range and A updated.
template <class T>
__device__ __forceinline__ void rg_tail64(T* __restrict__ A, int& f, int& l, int nth, int& depth, bool& heap,
                                          const RgLds& E) {
    const int lane = threadIdx.x & 63;
    // (the range bounds are wave-uniform: declared so, the step's control flow and the pivot
    // readlanes stay scalar instead of running under exec masks)
    const int f0 = uni(f), n0 = uni(l) - f0;
    T v = A[f0 + min(lane, n0 - 1)];
    T* eb = E.bl<T>();
    constexpr int kBr = RgLds::kBr<T>, kTv = RgLds::kTv<T>;
    const int kth = uni(nth) - f0;
    int lf = 0, ll = n0, dep = uni(depth);
    while (ll - lf > 3) {
        if (dep == 0) {
            heap = true;
            break;
        }
        --dep;
        const int a = lf + 1, b = lf + (ll - lf) / 2, c = ll - 1;
        const T vf = rdl(v, lf), va = rdl(v, a), vb = rdl(v, b), vc = rdl(v, c);
        T pv;
        const int m = stl_median(a, b, c, va, vb, vc, pv);
        const unsigned P = sel_key(pv);
        v = lane == lf ? pv : lane == m ? vf : v;
        const unsigned k = sel_key(v);
        const bool in = lane > lf && lane < ll;
        const bool il = in && k <= P, ir = in && k >= P;
        const u64 ml = __ballot(il), mr = __ballot(ir);
        const int ra = mbcnt(ml, 0), rb = mbcnt(mr, 0), nr = __popcll(mr);
        const bool sl = swap_l(il, ir, ra, rb, nr), sr = swap_r(ir, ra, rb, nr);
        eb[sl ? ra : sr ? kBr + (nr - 1 - rb) : kTv + lane] = v;
        const u64 cb = __ballot((il && !sl) || sr);  // the cut: the first unswapped L or swapped R
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const T nv = eb[sl ? kBr + ra : sr ? nr - 1 - rb : kTv + lane];
        int cut = cb ? __ffsll((long long)cb) - 1 : INT_MAX;
        cut = uni(min(max(cut, lf + 1), ll));  // (clamped: memory-safe whatever happens)
        v = (sl || sr) ? nv : v;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (next step's mailbox writes after these reads)
        __builtin_amdgcn_wave_barrier();
        if (cut <= kth) lf = cut;
        else ll = cut;
    }
    if (lane < n0) A[f0 + lane] = v;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    depth = dep;
    f = f0 + lf;
    l = f0 + ll;
}

// libstdc++'s closing __insertion_sort of A[0, n) (n <= 3; a stable sort by key, descending):
// every lane of the calling wave reads the elements, lane 0 writes them back
template <class T>
__device__ __forceinline__ void stl_small_sort(T* __restrict__ A, int n) {
    if (n < 2) return;
    T e0 = uni(A[0]), e1 = uni(A[1]), e2 = n > 2 ? uni(A[2]) : T(0);
    if (sel_key(e1) > sel_key(e0)) {
        const T t = e0;
        e0 = e1;
        e1 = t;
    }
    if (n > 2 && sel_key(e2) > sel_key(e1)) {
        const T t = e1;
        e1 = e2;
        e2 = t;
        if (sel_key(e1) > sel_key(e0)) {
            const T u = e0;
            e0 = e1;
            e1 = u;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        A[0] = e0;
        A[1] = e1;
        if (n > 2) A[2] = e2;
    }
}

// libstdc++ __adjust_heap / __push_heap / __make_heap / __heap_select with comp = greater (one lane)
template <class T>
__device__ void stl_adjust_heap(T* a, int hole, int len, T v) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (sel_key(a[child]) > sel_key(a[child - 1])) --child;
        a[hole] = a[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        a[hole] = a[child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && sel_key(a[parent]) > sel_key(v)) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = v;
}

template <class T>
__device__ void stl_heap_select(T* a, int mid, int last) {
    if (mid >= 2)
        for (int parent = (mid - 2) / 2;; --parent) {
            stl_adjust_heap(a, parent, mid, a[parent]);
            if (parent == 0) break;
        }
    for (int i = mid; i < last; ++i)
        if (sel_key(a[i]) > sel_key(a[0])) {
            const T v = a[i];
            a[i] = a[0];
            stl_adjust_heap(a, 0, mid, v);
        }
}

template <class T>
__device__ void stl_insertion_sort(T* A, int f, int l) {
    for (int i = f + 1; i < l; ++i) {
        const T v = A[i];
        if (sel_key(v) > sel_key(A[f])) {
            for (int j = i; j > f; --j) A[j] = A[j - 1];
            A[f] = v;
        } else {
            int j = i;
            while (sel_key(v) > sel_key(A[j - 1])) {
                A[j] = A[j - 1];
                --j;
            }
            A[j] = v;
        }
    }
}

// __unguarded_partition_pivot(first = f, last = l) as one team pass over memory (ranges longer than
// the engine takes); bl / br: mailboxes of (l - f) / 2 + 1 elements.  Returns the cut.
template <class T>
__device__ __forceinline__ int pivot_pass_mem(T* __restrict__ A, T* __restrict__ bl, T* __restrict__ br, int f, int l,
                                              int* s) {
    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const T vf = uni(A[f]), va = uni(A[a]), vb = uni(A[b]), vc = uni(A[c]);
    T pv;
    const int m = stl_median(a, b, c, va, vb, vc, pv);
    const unsigned P = sel_key(pv);
    int nr;
    return team_pass<kStlWaves>(A, bl, br, f + 1, l, m, vf, pv, [P](T v) { return sel_key(v) <= P; },
                                [P](T v) { return sel_key(v) >= P; }, s, nr);
}

// std::nth_element(A, A + nth, A + n, greater); every thread of the workgroup calls it.  Ranges
// beyond the engine's capacity first take team passes over memory (bl / br: n / 2 + 1 each).
template <class T>
__device__ __forceinline__ void stl_nth_element(T* __restrict__ A, T* __restrict__ bl, T* __restrict__ br, int n,
                                                int nth, const RgLds& E) {
    if (n <= 0 || nth >= n) return;
    int f = 0, l = n, depth = 2 * (31 - __clz(n));
    bool heap = false;
    while (l - f > RgCap<T>::v) {
        if (depth == 0) {
            heap = true;
            break;
        }
        --depth;
        VX_KP(l - f);
        const int cut = pivot_pass_mem(A, bl, br, f, l, E.s());
        if (cut <= nth) f = cut;
        else l = cut;
    }
    while (!heap && l - f > kRgWave) {
        if (depth == 0) {
            heap = true;
            break;
        }
        --depth;
        int nr;
        VX_KP((1 << 24) | (l - f));
        const int cut = f + rg_team_any<true>(A + f, l - f, 0u, E, nr);
        if (cut <= nth) f = cut;
        else l = cut;
    }
    VX_KT(2);
    if (uni((int)(threadIdx.x >> 6)) == 0) {  // (wave 0: a scalar branch)
        while (!heap && l - f > 3) {
            if (l - f <= 64) {  // the rest of the introselect in registers (rg_tail64)
                VX_KP((5 << 24) | (l - f));
                rg_tail64(A, f, l, nth, depth, heap, E);
                break;
            }
            if (depth == 0) {
                heap = true;
                break;
            }
            --depth;
            int nr;
            VX_KP((2 << 24) | (l - f));
            const int cut = f + rg_wave_any<true>(A + f, l - f, 0u, E, nr);
            if (cut <= nth) f = cut;
            else l = cut;
        }
        if (!heap) {
            stl_small_sort(A + f, l - f);
        } else {  // introselect's depth limit: __heap_select + iter_swap (one lane)
            if (threadIdx.x == 0) {
                stl_heap_select(A + f, nth + 1 - f, l - f);
                const T t = A[f];
                A[f] = A[nth];
                A[nth] = t;
            }
        }
        VX_KT(3);
    }
    __syncthreads();
}

// KeyPointsFilter::retainBest(A[0..size), npts): nth_element, then std::partition of the tail by
// key >= the npts-th key.  Returns the kept length; every thread calls it.
template <class T>
__device__ __forceinline__ int stl_retain_best(T* __restrict__ A, T* __restrict__ bl, T* __restrict__ br, int size,
                                               int npts, const RgLds& E) {
    if (size <= npts) return size;
    if (npts <= 0) return 0;
    stl_nth_element(A, bl, br, size, npts - 1, E);
    VX_KT(4);
    VX_KP((3 << 24) | (size - npts));
    const unsigned thr = uni(sel_key(A[npts - 1]));
    const int len = size - npts;
    int* s = E.s();
    int nr = 0;
    if (len > RgCap<T>::v) {
        team_pass<kStlWaves>(A, bl, br, npts, size, -1, T(0), T(0), [thr](T v) { return sel_key(v) < thr; },
                             [thr](T v) { return sel_key(v) >= thr; }, s, nr);
    } else if (len > kRgWave) {
        rg_team_any<false>(A + npts, len, thr, E, nr);
    } else {
        if (uni((int)(threadIdx.x >> 6)) == 0) {
            rg_wave_any<false>(A + npts, len, thr, E, nr);
            if (threadIdx.x == 0) s[60] = nr;
        }
        __syncthreads();
        nr = uni(s[60]);
    }
    VX_KT(5);
    VX_KP(4 << 24);
    return npts + nr;
}

// One workgroup per (level, frame): retainBest(2q) by FAST score and retainBest(q) by Harris in
// libstdc++ order.  Staging of level l: kept[0..cap) = every border-passing NMS corner in raster
// order, fin[0..cap) = the result, then 32 B x cap of selection scratch.
// dbg (test hook vx_orb_set_debug, single frame; nullptr otherwise): dbg[l] = candidates,
// dbg[kMaxLevels + l] = retainBest(2q) survivors, then per level (at the prefix of level_cap) the
// survivors' raster indices in output order.
__global__ __launch_bounds__(kStlNT) void k_select_stl(const CandRec* __restrict__ cand,
                                                       const int* __restrict__ cell_count, LevelArgs a,
                                                       CandRec* __restrict__ stage, int* __restrict__ level_count,
                                                       int* __restrict__ dbg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sdyn[];
    __shared__ int sw[kStlWaves];
    const RgLds E{sdyn};
    const int l = blockIdx.x;
    const int tid = threadIdx.x;
    VX_KP_RESET();
    cand += blockIdx.z * a.fs_cells * kCellCap;
    cell_count += blockIdx.z * a.fs_cells;
    stage += blockIdx.z * a.fs_stage;
    level_count += blockIdx.z * kMaxLevels;
    VX_KT(12);
    const int ncell = a.lh[l] * a.ntx[l];
    const long long cbase = a.cell_base[l];
    const int cap = a.level_cap[l];
    CandRec* kept = stage + a.stage_base[l];
    CandRec* fin = kept + cap;
    unsigned char* gscr = reinterpret_cast<unsigned char*>(kept + 2 * (long long)cap);
    unsigned* gA1 = reinterpret_cast<unsigned*>(gscr);
    const int q = a.quota[l];
    const int k1 = 2 * q;
    // LDS after the engine's scratch: the pass-1 elements and the candidates' Harris keys (up to
    // kRgCap32 each), later the pass-2 elements over them
    unsigned* lA1 = reinterpret_cast<unsigned*>(sdyn + kRgBytes);
    unsigned* lhk = lA1 + kRgCap32;
    static_assert(kRgBytes + 8 * kRgCap32 <= kStlLds, "k_select_stl LDS");
    // ---- every border-passing NMS corner in raster (cell) order: records to kept[], pass-1
    // elements (score << 24 | raster index) to the global scratch and (when they fit) to LDS with
    // the Harris keys
    const int cpt = min(kCellsPer, (ncell + kStlNT - 1) / kStlNT);
    int n0 = 0;
    for (int base = 0; base < ncell; base += kStlNT * cpt) {
        const int c0 = base + tid * cpt;
        int cnts[kCellsPer];
        int tot = 0;
#pragma unroll
        for (int j = 0; j < kCellsPer; ++j) cnts[j] = (j < cpt && c0 + j < ncell) ? cell_count[cbase + c0 + j] : 0;
#pragma unroll
        for (int j = 0; j < kCellsPer; ++j) tot += cnts[j];
        auto rec_index = [&](int k) {  // the thread's k-th record: cell j of its cells, slot i
            int j = 0, i = k;
#pragma unroll
            for (int jj = 0; jj < kCellsPer; ++jj)
                if (j == jj && i >= cnts[jj]) {
                    i -= cnts[jj];
                    j = jj + 1;
                }
            return cand_at(cbase + c0 + j, i, a.fs_cells);
        };
        CandRec rr[kRecBatch];
#pragma unroll
        for (int k = 0; k < kRecBatch; ++k) rr[k] = k < tot ? cand[rec_index(k)] : CandRec{};
        int btot;
        int pos = n0 + block_scan_excl<kStlNT>(tot, sw, btot);
        auto put = [&](const CandRec& r) {
            kept[pos] = r;
            const unsigned e = ((unsigned)r.score << 24) | (unsigned)pos;
            if (pos < kRgCap32) {  // (the global copy only when the level outgrows the LDS: below)
                lA1[pos] = e;
                lhk[pos] = harris_key(r.harris);
            } else {
                gA1[pos] = e;
            }
            ++pos;
        };
#pragma unroll
        for (int k = 0; k < kRecBatch; ++k)
            if (k < tot) put(rr[k]);
        // further records a batch of loads at a time (a thread over a textured half row holds 10-20:
        // one load per put would expose a memory latency per record on the level's longest thread)
        for (int k0 = kRecBatch; k0 < tot; k0 += kRecBatch) {
#pragma unroll
            for (int k = 0; k < kRecBatch; ++k) rr[k] = k0 + k < tot ? cand[rec_index(k0 + k)] : CandRec{};
#pragma unroll
            for (int k = 0; k < kRecBatch; ++k)
                if (k0 + k < tot) put(rr[k]);
        }
        n0 += uni(btot);
    }
    __syncthreads();
    // the output's bitmap of survivors (raster indices), in the engine's unused lp / rp region:
    // cleared here, visible after the passes' barriers
    unsigned* bm = reinterpret_cast<unsigned*>(E.lp());
    const int nw32 = (n0 + 31) >> 5;
    const bool bm_fits = 2 * nw32 * 4 <= 2 * kRgMail;
    if (bm_fits)
        for (int i = tid; i < nw32; i += kStlNT) bm[i] = 0u;
    if (n0 > kRgCap32) {  // the whole pass-1 array then lives in the global scratch
        for (int i = tid; i < kRgCap32; i += kStlNT) gA1[i] = lA1[i];
        __syncthreads();
    }
    VX_KT(9);
    // ---- retainBest(2q) by FAST score (u32 elements; beyond the engine's capacity the first
    // passes run over the global scratch with mailboxes of n0 / 2 + 1 each after it)
    const int hb = n0 / 2 + 1;
    int K1;
    const bool lds1 = n0 <= kRgCap32;
    if (lds1) K1 = stl_retain_best(lA1, (unsigned*)nullptr, (unsigned*)nullptr, n0, k1, E);
    else K1 = stl_retain_best(gA1, gA1 + n0, gA1 + n0 + hb, n0, k1, E);
    // ---- retainBest(q) by Harris over the survivors in their new order (u64 elements: in LDS over
    // the pass-1 arrays when they fit the engine, else in the global scratch after the pass-1 one)
    constexpr int kCap2 = RgCap<u64>::v;
    const bool lds2 = K1 <= kCap2;
    u64* L2 = reinterpret_cast<u64*>(sdyn + kRgBytes);
    u64* G2 = reinterpret_cast<u64*>(gscr + 16 * (long long)cap);
    VX_KT(10);
    long long doff = 2 * kMaxLevels;
    if (dbg) {
        for (int i = 0; i < l; ++i) doff += a.level_cap[i];
        if (tid == 0) {
            dbg[l] = n0;
            dbg[kMaxLevels + l] = K1;
        }
    }
    auto elem2 = [&](int j) -> u64 {
        const unsigned idx = (lds1 ? lA1[j] : gA1[j]) & 0xffffffu;
        if (dbg) dbg[doff + j] = (int)idx;
        const unsigned hk = lds1 ? lhk[idx] : harris_key(kept[idx].harris);
        return ((u64)hk << 32) | idx;
    };
    if (lds2) {
        constexpr int kPer = kCap2 / kStlNT;
        u64 e2[kPer];
#pragma unroll
        for (int i = 0; i < kPer; ++i) e2[i] = tid + i * kStlNT < K1 ? elem2(tid + i * kStlNT) : 0ull;
        __syncthreads();  // (L2 overlays the pass-1 arrays)
#pragma unroll
        for (int i = 0; i < kPer; ++i)
            if (tid + i * kStlNT < K1) L2[tid + i * kStlNT] = e2[i];
    } else {
        for (int j = tid; j < K1; j += kStlNT) G2[j] = elem2(j);
    }
    __syncthreads();
    VX_KT(11);
    int K2;
    if (lds2) {  // (separate call sites: the LDS one compiles to ds_ instructions)
        K2 = stl_retain_best(L2, (u64*)nullptr, (u64*)nullptr, K1, q, E);
    } else {
        const int hb2 = K1 / 2 + 1;
        K2 = stl_retain_best(G2, G2 + K1, G2 + K1 + hb2, K1, q, E);
    }
    VX_KT(13);
    // the first survivor record of each thread requested before the bitmap's barriers
    auto sidx = [&](int j) { return (unsigned)(lds2 ? L2[j] : G2[j]); };
    const CandRec f0 = tid < K2 ? kept[sidx(tid)] : CandRec{};
    if (tid == 0) level_count[l] = K2;
    // The survivors in raster order for k_describe's walk (rast[p] = output index of the p-th
    // survivor in raster order, over the dead pass-1 scratch): a bitmap of their raster indices in
    // LDS (cleared after the gather), word popcounts scanned, one rank per survivor.
    int* rast = reinterpret_cast<int*>(gscr);
    int* wpre = reinterpret_cast<int*>(bm + nw32);
    if (bm_fits) {
        for (int j = tid; j < K2; j += kStlNT) {
            const unsigned idx = sidx(j);
            atomicOr(&bm[idx >> 5], 1u << (idx & 31u));
        }
        __syncthreads();
        int base = 0;
        for (int i0 = 0; i0 < nw32; i0 += kStlNT) {
            const int i = i0 + tid;
            int tot;
            const int e = block_scan_excl<kStlNT>(i < nw32 ? __popc(bm[i]) : 0, sw, tot);
            if (i < nw32) wpre[i] = base + e;
            base += uni(tot);
        }
        __syncthreads();
        for (int j = tid; j < K2; j += kStlNT) {
            const unsigned idx = sidx(j);
            rast[wpre[idx >> 5] + __popc(bm[idx >> 5] & ((1u << (idx & 31u)) - 1u))] = j;
        }
    } else {
        for (int j = tid; j < K2; j += kStlNT) rast[j] = j;  // (no room: output order, no locality)
    }
    if (tid < K2) fin[tid] = f0;
    for (int j = tid + kStlNT; j < K2; j += kStlNT) fin[j] = kept[sidx(j)];
    VX_KT(15);
}

// Test hook (vx_test_retain_best): retainBest over caller keys through the device code above
// (A in LDS after the engine's scratch, or in the global scratch; mailboxes for the passes beyond
// the engine after A).
template <class T>
__device__ __forceinline__ void test_retain_body(T* A, const unsigned* __restrict__ keys, int n, int npts,
                                                 int* __restrict__ out, const RgLds& E) {
    const int hb = n / 2 + 1;
    for (int i = threadIdx.x; i < n; i += kStlNT)
        A[i] = sizeof(T) == 4 ? (T)((keys[i] << 24) | (unsigned)i) : (T)(((u64)keys[i] << 32) | (unsigned)i);
    __syncthreads();
    VX_KT(1);
    const int K = stl_retain_best(A, A + n, A + n + hb, n, npts, E);
    for (int j = threadIdx.x; j < K; j += kStlNT) out[1 + j] = (int)(sizeof(T) == 4 ? (A[j] & 0xffffffu) : (unsigned)A[j]);
    if (threadIdx.x == 0) out[0] = K;
    VX_KT(6);
}

__global__ __launch_bounds__(kStlNT) void k_test_retain(const unsigned* __restrict__ keys, int n, int npts, int wide,
                                                        int use_lds, unsigned char* __restrict__ gscr,
                                                        int* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sdyn[];
    VX_KT(0);
    VX_KP_RESET();
    const RgLds E{sdyn};
    unsigned char* ra = sdyn + kRgBytes;
    if (!wide) {
        if (use_lds) test_retain_body(reinterpret_cast<unsigned*>(ra), keys, n, npts, out, E);
        else test_retain_body(reinterpret_cast<unsigned*>(gscr), keys, n, npts, out, E);
    } else {
        if (use_lds) test_retain_body(reinterpret_cast<u64*>(ra), keys, n, npts, out, E);
        else test_retain_body(reinterpret_cast<u64*>(gscr), keys, n, npts, out, E);
    }
}

// ------------------------------------------------------------------------------ describe
__device__ __forceinline__ float ocv_fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float r, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        r = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        r = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) r = 180.f - r;
    if (y < 0) r = 360.f - r;
    return r;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(kBlock) void k_describe(const uint8_t* __restrict__ pyr,
                                                     const uint8_t* __restrict__ blur,
                                                     const CandRec* __restrict__ stage,
                                                     const int* __restrict__ level_count,
                                                     LevelArgs a, vx_keypoint* __restrict__ kp,
                                                     uint8_t* __restrict__ desc,
                                                     int* __restrict__ slot_count) {
    constexpr int kWpb = kBlock / 64;
    const int lane = threadIdx.x & 63;
    pyr += blockIdx.z * a.fs_pyr;
    blur += blockIdx.z * a.fs_pyr;
    stage += blockIdx.z * a.fs_stage;
    level_count += blockIdx.z * kMaxLevels;
    kp += blockIdx.z * (long long)a.out_cap;
    desc += blockIdx.z * (long long)a.out_cap * 32;
    slot_count += blockIdx.z * 4;
    int total = 0;
    for (int i = 0; i < a.L; ++i) total += level_count[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        slot_count[0] = total;
        slot_count[1] = total > a.out_cap;
    }
    // Wave rank rk walks the keypoints in (level, raster) order, and the first nact blocks take
    // the ranks XCD by XCD (block x runs on XCD x mod 8): each XCD's L2 fetches the rows of one
    // band of the levels instead of every XCD fetching every patch row.  Keypoint rk's output
    // index is its STL-order index (rast, from k_select_stl).  Overflow: output order.
    const bool remap = a.raster_rank && total <= a.out_cap;
    const int nact = (min(total, a.out_cap) + kWpb - 1) / kWpb;
    int bx = blockIdx.x;
    if (remap) {
        if ((int)blockIdx.x >= nact) return;
        const int xcd = blockIdx.x & 7, qb = nact >> 3, rem = nact & 7;
        bx = xcd * qb + min(xcd, rem) + (blockIdx.x >> 3);
    }
    const int rk = bx * kWpb + (threadIdx.x >> 6);
    int l = -1, j = 0, w = 0;
    {
        int pre = 0;
        for (int i = 0; i < a.L; ++i) {
            const int c = level_count[i];
            if (l < 0 && rk < pre + c) {
                l = i;
                j = rk - pre;
                w = pre;
            }
            pre += c;
        }
    }
    if (l < 0) return;
    if (remap) j = reinterpret_cast<const int*>(stage + a.stage_base[l] + 2 * (long long)a.level_cap[l])[j];
    w += j;
    if (w >= a.out_cap) return;
    const CandRec r = stage[a.stage_base[l] + a.level_cap[l] + j];
    const int W = a.lw[l];
    const int xl = (int)(r.xy & 0xffffu), yl = (int)(r.xy >> 16);
    const uint8_t* img = pyr + a.off[l];
    const float sc = a.scale[l];
    const float px = (float)xl * sc, py = (float)yl * sc;
    const float inv = a.inv_scale[l];
    const int cx = __float2int_rn(px * inv), cy = __float2int_rn(py * inv);
    // The blurred patch the rBRIEF tests sample (the pattern's points lie in [-13, 12]^2, so rotated
    // they stay within +-18 of the centre): rows cy-18..cy+18 on lanes 0..36, 40 bytes from cx-18
    // each.  Keypoints lie >= edge_threshold px from the level's edges and validate_params requires
    // edge_threshold >= 19, so every row is inside the level; the 11 aligned dwords of a row reach
    // from (cx-18) & ~3 >= cx-21 to cx+25, i.e. at most 2 bytes before the row's first pixel and 6
    // past its last — neighbouring rows of the same level buffer, whose bytes v_alignbyte drops
    // (tests/test_gpu_parity.py::test_orb_min_edge_threshold).  They are loaded together with
    // the IC-angle taps below and parked in this wave's LDS — the tests then read LDS instead of
    // waiting on 512 dependent L2 gathers after the angle.
    __shared__ unsigned s_patch[kBlock / 64][37 * 10];
    unsigned* patch = s_patch[threadIdx.x >> 6];
    unsigned pq[11];
    unsigned psh = 0;
    if (lane < 37) {
        const uintptr_t ad = (uintptr_t)(blur + a.off[l] + (long long)(cy + lane - 18) * W + (cx - 18));
        const unsigned* al = reinterpret_cast<const unsigned*>(ad & ~(uintptr_t)3);
        psh = (unsigned)(ad & 3u);
#pragma unroll
        for (int j = 0; j < 11; ++j) pq[j] = al[j];
    }
    // ICAngles (half_k 15): lane v+15 sums row v of the circular patch — the row's 32-byte window
    // (u = -15..16) from 9 aligned dwords, bytes outside |u| <= umax[|v|] masked, then
    // sum p and sum (u + 15) p as byte dot products (integer: exact in any order)
    int m10 = 0, m01 = 0;
    if (lane < 31) {
        const int v = lane - 15;
        const uintptr_t ad = (uintptr_t)(img + (long long)(yl + v) * W + (xl - 15));
        const unsigned* al = reinterpret_cast<const unsigned*>(ad & ~(uintptr_t)3);
        const unsigned sh = (unsigned)(ad & 3u);
        unsigned q[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) q[j] = al[j];
        const uint4* mk = reinterpret_cast<const uint4*>(c_icmask[lane]);
        const uint4 ma = mk[0], mb = mk[1];
        const unsigned mw[8] = {ma.x, ma.y, ma.z, ma.w, mb.x, mb.y, mb.z, mb.w};
        unsigned s = 0, sr = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned p = __builtin_amdgcn_alignbyte(q[j + 1], q[j], sh) & mw[j];
            const unsigned ramp = (unsigned)(4 * j) | (unsigned)(4 * j + 1) << 8 | (unsigned)(4 * j + 2) << 16 |
                                  (unsigned)(4 * j + 3) << 24;
            s = __builtin_amdgcn_udot4(p, 0x01010101u, s, false);
            sr = __builtin_amdgcn_udot4(p, ramp, sr, false);
        }
        m10 = (int)sr - 15 * (int)s;
        m01 = v * (int)s;
    }
    if (lane < 37) {
#pragma unroll
        for (int j = 0; j < 10; ++j) patch[lane * 10 + j] = __builtin_amdgcn_alignbyte(pq[j + 1], pq[j], psh);
    }
    m10 = wave_sum(m10);
    m01 = wave_sum(m01);
    const float angle = ocv_fast_atan2((float)m01, (float)m10);
    // computeOrbDescriptors
    float ang = angle;
    ang *= (float)(M_PI / 180.f);
    double sd, cd;  // OpenCV: (float)cos((double)angle), (float)sin(...); one shared argument reduction
    sincos((double)ang, &sd, &cd);
    const float ca = (float)cd, sa = (float)sd;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (the patch rows written above, by other lanes)
    __builtin_amdgcn_wave_barrier();
    const uint8_t* pb = reinterpret_cast<const uint8_t*>(patch);
    unsigned long long words[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int bit = lane + 64 * s;
        int v[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int pi = 2 * bit + e;
            const float qx = (float)c_pattern[2 * pi], qy = (float)c_pattern[2 * pi + 1];
            const float x = qx * ca - qy * sa;
            const float y = qx * sa + qy * ca;
            v[e] = pb[(__float2int_rn(y) + 18) * 40 + __float2int_rn(x) + 18];
        }
        words[s] = __ballot(v[0] < v[1]);
    }
    const long long o = (long long)w;
    if (lane < 4) {
        const unsigned long long wv = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
        reinterpret_cast<unsigned long long*>(desc + o * 32)[lane] = wv;
    }
    if (lane == 0) {
        vx_keypoint k;
        k.x = px;
        k.y = py;
        k.response = r.harris;
        k.angle = angle;
        k.octave = l;
        kp[o] = k;
    }
}

// ------------------------------------------------------------------------------ host side
inline int cv_round_host(double v) { return (int)std::nearbyint(v); }
inline int cv_floor_host(double v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil_host(double v) { int i = (int)v; return i + (i < v); }

void linear_table(int src, int dst, std::vector<int4>& t) {
    t.resize(dst);
    const double inv = (double)dst / (double)src;
    const double scale = 1.0 / inv;
    for (int d = 0; d < dst; ++d) {
        const double f = scale * ((double)d + 0.5) - 0.5;
        const int i = cv_floor_host(f);
        if (i >= 0 && src > 1) {
            if (i < src - 1) {
                const int al = cv_round_host((f - (double)i) * 256.0);
                t[d] = make_int4(i, 256 - al, al, 0);
            } else {
                t[d] = make_int4(src - 1, 256, 0, 0);
            }
        } else {
            t[d] = make_int4(0, 256, 0, 0);
        }
    }
}

// Rectangles of the fused pyramid along one axis.  For level-0 tile t the owned range of level l
// is [b(t), b(t+1)) with b(t) = min(n_l, t * kPyTile * n_l / n_0) (a partition of every level);
// the needed range of level l-1 is the owned range plus every source index (ofs, min(ofs+1,
// n-1)) of the needed range of level l, taken from the same coefficient tables k_resize uses.
static void pyramid_axis(const std::vector<int>& n, const std::vector<const int4*>& tab, int tiles, int tile,
                         std::vector<int4>& out) {
    const int L = (int)n.size();
    for (int t = 0; t < tiles; ++t) {
        std::vector<int4> r(L);
        for (int l = 0; l < L; ++l) {
            const int64_t lo = std::min<int64_t>(n[l], (int64_t)t * tile * n[l] / n[0]);
            const int64_t hi = std::min<int64_t>(n[l], (int64_t)(t + 1) * tile * n[l] / n[0]);
            r[l] = make_int4(0, 0, (int)lo, (int)hi);
        }
        r[L - 1].x = r[L - 1].z;
        r[L - 1].y = r[L - 1].w;
        for (int l = L - 1; l >= 1; --l) {
            int lo = r[l - 1].z, hi = r[l - 1].w;
            if (lo >= hi) lo = INT32_MAX, hi = INT32_MIN;
            for (int d = r[l].x; d < r[l].y; ++d) {
                const int s0 = tab[l][d].x;
                lo = std::min(lo, s0);
                hi = std::max(hi, std::min(s0 + 1, n[l - 1] - 1) + 1);
            }
            if (lo >= hi) lo = hi = 0;
            r[l - 1].x = lo;
            r[l - 1].y = hi;
        }
        out.insert(out.end(), r.begin(), r.end());
    }
}

// LDS bytes of k_pyramid's raw level-0 staging: h0 rows of ((w0 * ch + 6) / 4) dwords.
static int64_t pyr_raw_bytes(const OrbGeometry& g, int ch) {
    return (int64_t)g.pr_h0 * (((int64_t)g.pr_w0 * ch + 6) >> 2) * 4;
}

// Prepares k_pyramid's tables (appended to the coefficient table vector `all`, which already holds
// the per-level resize tables) and decides whether the largest need rectangle fits in LDS.
static void pyramid_rects(OrbGeometry& g, std::vector<int4>& all, int n_cu) {
    g.pyr_fused = false;
    if (g.L < 2) return;
    std::vector<int> nw(g.L), nh(g.L);
    std::vector<const int4*> tx(g.L, nullptr), ty(g.L, nullptr);
    for (int l = 0; l < g.L; ++l) {
        nw[l] = g.lw[l];
        nh[l] = g.lh[l];
        if (l) {
            tx[l] = all.data() + g.xtab[l];
            ty[l] = all.data() + g.ytab[l];
        }
    }
    g.pr_tile = 64;
    if (const char* e = std::getenv("VX_PYR_TILE")) {
        g.pr_tile = std::max(16, std::min(256, std::atoi(e)));
    } else {
        for (int t = 32; t <= 256; t += 4)
            if ((int64_t)((g.W + t - 1) / t) * ((g.H + t - 1) / t) <= n_cu) {
                g.pr_tile = t;
                break;
            }
    }
    g.pr_block = kPyBlockDef;
    if (const char* e = std::getenv("VX_PYR_BLOCK")) g.pr_block = std::atoi(e) == 512 ? 512 : 1024;
    g.pr_ntx = (g.W + g.pr_tile - 1) / g.pr_tile;
    g.pr_nty = (g.H + g.pr_tile - 1) / g.pr_tile;
    std::vector<int4> rx, ry;
    pyramid_axis(nw, tx, g.pr_ntx, g.pr_tile, rx);
    pyramid_axis(nh, ty, g.pr_nty, g.pr_tile, ry);
    int64_t buf = 0;
    for (int l = 0; l < g.L; ++l) {
        int mw = 0, mh = 0;
        for (int t = 0; t < g.pr_ntx; ++t) mw = std::max(mw, rx[t * g.L + l].y - rx[t * g.L + l].x);
        for (int t = 0; t < g.pr_nty; ++t) mh = std::max(mh, ry[t * g.L + l].y - ry[t * g.L + l].x);
        buf = std::max<int64_t>(buf, (int64_t)mw * mh);
    }
    buf = (buf + 15) & ~int64_t(15);
    int64_t area0 = 0, tabn = 0, tx_max = 0, ty_max = 0;
    for (int t = 0; t < g.pr_ntx; ++t) {
        int64_t s = 0;
        for (int l = 1; l < g.L; ++l) s += rx[t * g.L + l].y - rx[t * g.L + l].x;
        tx_max = std::max(tx_max, s);
    }
    for (int t = 0; t < g.pr_nty; ++t) {
        int64_t s = 0;
        for (int l = 1; l < g.L; ++l) s += ry[t * g.L + l].y - ry[t * g.L + l].x;
        ty_max = std::max(ty_max, s);
    }
    tabn = tx_max + ty_max;
    for (int tx = 0; tx < g.pr_ntx; ++tx)
        for (int ty = 0; ty < g.pr_nty; ++ty)
            area0 = std::max<int64_t>(area0, (int64_t)(rx[tx * g.L].y - rx[tx * g.L].x) * (ry[ty * g.L].y - ry[ty * g.L].x));
    int64_t w0 = 0, h0 = 0;
    for (int tx = 0; tx < g.pr_ntx; ++tx) w0 = std::max<int64_t>(w0, rx[tx * g.L].y - rx[tx * g.L].x);
    for (int ty = 0; ty < g.pr_nty; ++ty) h0 = std::max<int64_t>(h0, ry[ty * g.L].y - ry[ty * g.L].x);
    g.pr_w0 = (int)w0;
    g.pr_h0 = (int)h0;
    // worst case 4 channels for the raw level-0 staging (dword rows, see k_pyramid)
    if (pyr_raw_bytes(g, 4) + 2 * buf + 4 * tabn > kPyLdsMax) return;  // level chain instead
    g.pr_buf = (int)buf;
    g.pr_area0 = (int)area0;
    g.pr_tabn = (int)tabn;
    g.pr_x = (int64_t)all.size();
    all.insert(all.end(), rx.begin(), rx.end());
    g.pr_y = (int64_t)all.size();
    all.insert(all.end(), ry.begin(), ry.end());
    g.pyr_fused = true;
}

// (float) of getGaussianKernelBitExact(7, sigma 2)
void gauss_taps(float k[7]) {
    double v[3], sum = 0;
    for (int i = 0, x = -6; i < 3; ++i, x += 2) {
        v[i] = std::exp((double)(x * x) * (-0.125 / 4.0));
        sum += v[i];
    }
    sum = sum * 2 + 1;
    const double mul = 1.0 / sum;
    for (int i = 0; i < 3; ++i) k[i] = k[6 - i] = (float)(v[i] * mul);
    k[3] = (float)(1.0 * mul);
}

bool g_constants_uploaded[64] = {false};

int upload_constants(vx_ctx* c) {
    if (c->device >= 0 && c->device < 64 && g_constants_uploaded[c->device]) return VX_OK;
    VX_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), kBitPattern31, sizeof(kBitPattern31)));
    int umax[16] = {0};
    const int half = 15;
    const int vmax = cv_floor_host(half * std::sqrt(2.f) / 2 + 1);
    const int vmin = cv_ceil_host(half * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) umax[v] = cv_round_host(std::sqrt((double)half * half - v * v));
    for (int v = half, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
    VX_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(c_umax), umax, sizeof(umax)));
    unsigned icmask[32][8] = {{0}};
    for (int r = 0; r < 31; ++r) {
        const int d = umax[r < 15 ? 15 - r : r - 15];
        for (int k = 0; k < 32; ++k)
            if (k - 15 >= -d && k - 15 <= d) icmask[r][k >> 2] |= 0xffu << (8 * (k & 3));
    }
    VX_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(c_icmask), icmask, sizeof(icmask)));
    // the selection kernels' 160 KB of dynamic LDS, per device (set with the device current; a failure
    // is reported every time, since the device is only marked done after it succeeded: ADVICE r3)
    VX_HIP(c, hipFuncSetAttribute(reinterpret_cast<const void*>(&k_select_stl), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kStlLds));
    VX_HIP(c, hipFuncSetAttribute(reinterpret_cast<const void*>(&k_test_retain),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kStlLds));
    if (c->device >= 0 && c->device < 64) g_constants_uploaded[c->device] = true;
    return VX_OK;
}

LevelArgs level_args(const OrbGeometry& g) {
    LevelArgs a{};
    std::memset(&a, 0, sizeof a);
    a.L = g.L;
    for (int l = 0; l < g.L; ++l) {
        a.lw[l] = g.lw[l];
        a.lh[l] = g.lh[l];
        a.off[l] = g.off[l];
        a.scale[l] = g.scale[l];
        a.inv_scale[l] = g.inv_scale[l];
        a.quota[l] = g.quota[l];
        a.ntx[l] = g.ntx[l];
        a.tile_base[l] = g.tile_base[l];
        a.cell_base[l] = g.cell_base[l];
        a.stage_base[l] = g.stage_base[l];
        a.level_cap[l] = g.level_cap[l];
    }
    a.fast_threshold = std::min(std::max(g.p.fast_threshold, 0), 255);
    a.edge = g.p.edge_threshold;
    a.out_cap = g.out_cap;
    int bb = 0;
    for (int l = 0; l < g.L; ++l) {
        a.btx[l] = (g.lw[l] + 63) / 64;
        a.bty[l] = (g.lh[l] + 15) / 16;
        a.bbase[l] = bb;
        bb += a.btx[l] * a.bty[l];
    }
    gauss_taps(a.gk);
    for (int l = 0; l < g.L; ++l) {
        a.xtab[l] = g.xtab[l];
        a.ytab[l] = g.ytab[l];
    }
    a.pr_x = g.pr_x;
    a.pr_y = g.pr_y;
    a.pr_buf = g.pr_buf;
    a.fs_pyr = g.pyr_bytes;
    a.fs_cells = g.cells_total;
    a.fs_hist = (long long)g.L * kHistRep * 256;
    a.fs_stage = g.stage_total;
    return a;
}


bool same_params(const vx_orb_params& x, const vx_orb_params& y) {
    return x.n_features == y.n_features && x.scale_factor == y.scale_factor &&
           x.n_levels == y.n_levels && x.fast_threshold == y.fast_threshold &&
           x.edge_threshold == y.edge_threshold;
}

int validate_params(vx_ctx* c, const vx_orb_params* p, int w, int h) {
    if (!p) return set_error(c, VX_ERR_INVALID, "null params");
    if (p->n_levels < 1 || p->n_levels > kMaxLevels)
        return set_error(c, VX_ERR_INVALID, "n_levels must be in [1, %d]", kMaxLevels);
    if (!(p->scale_factor > 1.0f)) return set_error(c, VX_ERR_INVALID, "scale_factor must be > 1");
    if (p->n_features < 0) return set_error(c, VX_ERR_INVALID, "n_features < 0");
    if (p->edge_threshold < 19)
        return set_error(c, VX_ERR_INVALID, "edge_threshold must be >= 19 (descriptor footprint)");
    if (w < 1 || h < 1 || w > 4096 || h > 4096)
        return set_error(c, VX_ERR_INVALID, "image size %dx%d outside [1, 4096]", w, h);
    return VX_OK;
}

}  // namespace

int orb_prepare(vx_ctx* c, const vx_orb_params* p, int w, int h) {
    int rc = validate_params(c, p, w, h);
    if (rc) return rc;
    if (c->geo_valid && c->geo.W == w && c->geo.H == h && same_params(c->geo.p, *p)) return VX_OK;
    VX_HIP(c, hipSetDevice(c->device));
    rc = upload_constants(c);
    if (rc) return rc;
    OrbGeometry g;
    g.W = w;
    g.H = h;
    g.p = *p;
    g.L = p->n_levels;
    // level geometry (ORB_Impl::detectAndCompute): s_l = (float)pow((double)scaleFactor, l)
    const double sf = (double)p->scale_factor;
    int64_t off = 0;
    for (int l = 0; l < g.L; ++l) {
        const float s = (float)std::pow(sf, (double)l);
        const float inv = 1.0f / s;
        g.scale[l] = s;
        g.inv_scale[l] = inv;
        g.lw[l] = std::max(1, (int)std::nearbyintf((float)w * inv));
        g.lh[l] = std::max(1, (int)std::nearbyintf((float)h * inv));
        g.off[l] = off;
        off += ((int64_t)g.lw[l] * g.lh[l] + 255) & ~int64_t(255);
    }
    g.pyr_bytes = off;
    // quotas (computeKeyPoints)
    {
        const float factor = (float)(1.0 / sf);
        float nd = (float)p->n_features * (1 - factor) /
                   (1 - (float)std::pow((double)factor, (double)g.L));
        int sum = 0;
        for (int l = 0; l < g.L - 1; ++l) {
            g.quota[l] = (int)std::nearbyintf(nd);
            sum += g.quota[l];
            nd *= factor;
        }
        g.quota[g.L - 1] = std::max(p->n_features - sum, 0);
    }
    // resize tables
    std::vector<int4> all, t;
    for (int l = 1; l < g.L; ++l) {
        linear_table(g.lw[l - 1], g.lw[l], t);
        g.xtab[l] = (int64_t)all.size();
        all.insert(all.end(), t.begin(), t.end());
        linear_table(g.lh[l - 1], g.lh[l], t);
        g.ytab[l] = (int64_t)all.size();
        all.insert(all.end(), t.begin(), t.end());
    }
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device);
    g.n_cu = n_cu;
    pyramid_rects(g, all, std::max(1, (int)(n_cu * c->grid_share)));
    g.tab_entries = (int64_t)all.size();
    // FAST tiles / cells and selection staging
    int tiles = 0;
    int64_t cells = 0, stg = 0;
    g.max_w = 0;
    for (int l = 0; l < g.L; ++l) {
        g.ntx[l] = (g.lw[l] + kTX - 1) / kTX;
        g.nty[l] = (g.lh[l] + kTY - 1) / kTY;
        g.tile_base[l] = tiles;
        tiles += g.ntx[l] * g.nty[l];
        g.cell_base[l] = cells;
        cells += (int64_t)g.lh[l] * g.ntx[l];
        g.level_cap[l] = (g.lw[l] / 2 + 1) * (g.lh[l] / 2 + 1);
        g.stage_base[l] = stg;
        // kept + fin (level_cap records each) + k_select_stl's scratch (32 B x level_cap + slack)
        stg += 4 * (int64_t)g.level_cap[l] + 4;
        g.max_w = std::max(g.max_w, g.lw[l]);
    }
    g.total_tiles = tiles;
    g.cells_total = cells;
    g.stage_total = stg;
    g.out_cap = 2 * p->n_features + 256;

    VX_HIP(c, c->tabs.ensure(std::max<int64_t>(1, g.tab_entries) * sizeof(int4)));
    if (!all.empty())
        VX_HIP(c, hipMemcpy(c->tabs.p, all.data(), all.size() * sizeof(int4), hipMemcpyHostToDevice));
    VX_HIP(c, c->pyr.ensure(g.pyr_bytes));
    VX_HIP(c, c->blur.ensure(g.pyr_bytes));
    VX_HIP(c, c->cand.ensure(g.cells_total * kCellCap * sizeof(CandRec)));
    VX_HIP(c, c->stage.ensure(g.stage_total * sizeof(CandRec)));
    VX_HIP(c, c->band_count.ensure(g.cells_total * sizeof(int)));
    VX_HIP(c, c->hist.ensure(g.L * kHistRep * 256 * sizeof(int)));
    VX_HIP(c, c->level_count.ensure(kMaxLevels * sizeof(int)));
    if (c->orb_debug) {
        int64_t caps = 0;
        for (int l = 0; l < g.L; ++l) caps += g.level_cap[l];
        VX_HIP(c, c->orb_dbg.ensure((size_t)(2 * kMaxLevels + caps) * sizeof(int)));
    }
    for (auto& s : c->slots) {
        s.valid = false;
        VX_HIP(c, s.kp.ensure((size_t)g.out_cap * sizeof(vx_keypoint)));
        VX_HIP(c, s.desc.ensure((size_t)g.out_cap * 32));
        VX_HIP(c, s.count.ensure(16));
        s.cap = g.out_cap;
    }
    for (int b = 0; b < VX_BATCH_BANKS; ++b) c->batch_n[b] = 0;
    c->geo = g;
    c->geo_valid = true;
    ++c->geo_gen;
    return VX_OK;
}

// Enqueues the extraction of nf frames (frame f at d_img + f * fs_img) into the outputs kp / desc /
// count (frame f at kp + f * out_cap, desc + f * 32 * out_cap, count + 4 f): one launch per kernel,
// frame = blockIdx.z, the scratch buffers hold nf frames (orb_reserve_frames).
static int orb_enqueue_frames(vx_ctx* c, const uint8_t* d_img, int channels, int64_t stride, int64_t fs_img, int nf,
                              vx_keypoint* kp, uint8_t* desc, int* count) {
    const OrbGeometry& g = c->geo;
    LevelArgs a = level_args(g);
    a.raster_rank = c->kp_order == VX_ORDER_STL && !(c->orb_debug & VX_ORB_DEBUG_FAST_NO_BORDER);
    a.fs_img = fs_img;
    // test hooks (vx_orb_set_debug): the FAST list before runByImageBorder, the selection's stages
    if (c->orb_debug & VX_ORB_DEBUG_FAST_NO_BORDER) a.edge = 3;
    int* dbg = (c->orb_debug && nf == 1) ? c->orb_dbg.as<int>() : nullptr;
    uint8_t* pyr = c->pyr.as<uint8_t>();
    const int hist_n = g.L * kHistRep * 256;
    // the fused pyramid buys latency with redundant halo work; a batch whose fused grid would need more
    // than one round of the device's CUs takes the level chain instead (C3, 8 frames on 18 x 14 tiles:
    // 16.5 us per frame fused vs ~5.5 for gray + resizes; 2 and 4 frames with the grid share set to
    // 1/B keep the fused pyramid: 35.9 / 25.1 against 39.4 / 27.4 us per frame)
    if (g.pyr_fused && (nf == 1 || (int64_t)g.pr_ntx * g.pr_nty * nf <= g.n_cu)) {
        const int raw = (int)((pyr_raw_bytes(g, channels) + 15) & ~int64_t(15));
        VX_HIP(c, launch(c, kStPyramid, g.pr_block == 512 ? k_pyramid<512> : k_pyramid<1024>,
                         dim3(g.pr_ntx, g.pr_nty, nf), dim3(g.pr_block),
                         (uint32_t)(raw + 2 * g.pr_buf + 4 * g.pr_tabn), c->stream, d_img, channels,
                         (long long)stride, pyr, (const int4*)c->tabs.as<int4>(), a, c->hist.as<int>(), hist_n, raw));
    } else {
        {
            ProfScope ps(c, kStGray);
            hipLaunchKernelGGL(k_gray, dim3((g.W + kBlock - 1) / kBlock, g.H, nf), dim3(kBlock), 0, c->stream,
                               d_img, g.W, channels, (long long)stride, pyr, c->hist.as<int>(), hist_n,
                               (long long)fs_img, (long long)a.fs_pyr, (long long)a.fs_hist);
            VX_LAUNCH_CHECK(c, "k_gray");
        }
        ProfScope ps(c, kStResize);
        const int4* tabs = c->tabs.as<int4>();
        for (int l = 1; l < g.L; ++l) {
            hipLaunchKernelGGL(k_resize, dim3((g.lw[l] + kBlock - 1) / kBlock, g.lh[l], nf), dim3(kBlock), 0,
                               c->stream, pyr + g.off[l - 1], g.lw[l - 1], g.lh[l - 1], pyr + g.off[l],
                               g.lw[l], tabs + g.xtab[l], tabs + g.ytab[l], (long long)a.fs_pyr);
            VX_LAUNCH_CHECK(c, "k_resize");
        }
    }
    // FAST + NMS + Harris and the GaussianBlur of every level, one launch over 64 x 16 tiles
    VX_HIP(c, launch(c, kStFast, k_fast, dim3(g.total_tiles, 1, nf), dim3(kBlock), 0, c->stream, (const uint8_t*)pyr, a,
                     c->cand.as<CandRec>(), c->band_count.as<int>(), c->hist.as<int>(), c->blur.as<uint8_t>()));
    if (c->kp_order == VX_ORDER_STL) {
        VX_HIP(c, launch(c, kStSelect, k_select_stl, dim3(g.L, 1, nf), dim3(kStlNT), (uint32_t)kStlLds, c->stream,
                         (const CandRec*)c->cand.as<CandRec>(), (const int*)c->band_count.as<int>(), a,
                         c->stage.as<CandRec>(), c->level_count.as<int>(), dbg));
    } else {
        VX_HIP(c, launch(c, kStSelect, k_select, dim3(g.L, 1, nf), dim3(kSelBlock), 0, c->stream,
                         (const CandRec*)c->cand.as<CandRec>(), (const int*)c->band_count.as<int>(),
                         (const int*)c->hist.as<int>(), a, c->stage.as<CandRec>(), c->level_count.as<int>()));
    }
    if (c->orb_debug & VX_ORB_DEBUG_FAST_NO_BORDER) {
        // corners within 31 px of the edge are no keypoints: the descriptor patch would leave the
        // level.  The debug run only exposes the FAST list; it reports no keypoints.
        VX_HIP(c, hipMemsetAsync(count, 0, (size_t)nf * 16, c->stream));
    } else {
        const int waves_per_block = kBlock / 64;
        VX_HIP(c, launch(c, kStDescribe, k_describe, dim3((g.out_cap + waves_per_block - 1) / waves_per_block, 1, nf),
                         dim3(kBlock), 0, c->stream, (const uint8_t*)pyr, (const uint8_t*)c->blur.as<uint8_t>(),
                         (const CandRec*)c->stage.as<CandRec>(), (const int*)c->level_count.as<int>(), a, kp, desc,
                         count));
    }
    return VX_OK;
}

static int orb_enqueue(vx_ctx* c, const uint8_t* d_img, int channels, int64_t stride, int slot) {
    Slot& s = c->slots[slot];
    const int rc = orb_enqueue_frames(c, d_img, channels, stride, 0, 1, s.kp.as<vx_keypoint>(), s.desc.as<uint8_t>(),
                                      s.count.as<int>());
    if (rc) return rc;
    s.valid = true;
    return VX_OK;
}

// Scratch for nf frames of the current geometry and the batch bank's outputs.  A buffer that has to
// grow moves, so the geometry serial is bumped (captured graphs of this context bake the old
// pointers into their kernels and must not be replayed).
static int orb_reserve_frames(vx_ctx* c, int nf, int bank) {
    const OrbGeometry& g = c->geo;
    const void* before[8] = {c->pyr.p, c->blur.p, c->cand.p, c->stage.p, c->band_count.p, c->hist.p, c->level_count.p,
                             nullptr};
    VX_HIP(c, c->pyr.ensure((size_t)nf * g.pyr_bytes));
    VX_HIP(c, c->blur.ensure((size_t)nf * g.pyr_bytes));
    VX_HIP(c, c->cand.ensure((size_t)nf * g.cells_total * kCellCap * sizeof(CandRec)));
    VX_HIP(c, c->stage.ensure((size_t)nf * g.stage_total * sizeof(CandRec)));
    VX_HIP(c, c->band_count.ensure((size_t)nf * g.cells_total * sizeof(int)));
    VX_HIP(c, c->hist.ensure((size_t)nf * g.L * kHistRep * 256 * sizeof(int)));
    VX_HIP(c, c->level_count.ensure((size_t)nf * kMaxLevels * sizeof(int)));
    const void* after[8] = {c->pyr.p, c->blur.p, c->cand.p, c->stage.p, c->band_count.p, c->hist.p, c->level_count.p,
                            nullptr};
    if (std::memcmp(before, after, sizeof before)) ++c->geo_gen;
    Slot& s = c->batch[bank];
    VX_HIP(c, s.kp.ensure((size_t)nf * g.out_cap * sizeof(vx_keypoint)));
    VX_HIP(c, s.desc.ensure((size_t)nf * g.out_cap * 32));
    VX_HIP(c, s.count.ensure((size_t)nf * 16));
    s.cap = g.out_cap;
    return VX_OK;
}

}  // namespace vx

namespace vx {
VX_KP_EXPORT(vx_kpass_read_orb);
VX_KT_EXPORT(vx_ktrace_read_orb);  // extern "C": the namespace does not enter the symbol
}

using namespace vx;

extern "C" {

void vx_orb_default_params(vx_orb_params* p) {
    if (!p) return;
    p->n_features = 1000;
    p->scale_factor = 1.2f;
    p->n_levels = 8;
    p->fast_threshold = 20;
    p->edge_threshold = 31;
}

int vx_orb_set_order(vx_ctx* c, int order) {
    if (!c) return VX_ERR_INVALID;
    if (order != VX_ORDER_STL && order != VX_ORDER_RASTER)
        return set_error(c, VX_ERR_INVALID, "keypoint order must be VX_ORDER_STL or VX_ORDER_RASTER");
    if (order == c->kp_order) return VX_OK;
    VX_HIP(c, hipSetDevice(c->device));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    // captured extraction graphs bake the selection kernel in
    for (auto& e : c->graphs.entries)
        if (e.exec) (void)hipGraphExecDestroy(e.exec);
    c->graphs.entries.clear();
    c->kp_order = order;
    for (auto& s : c->slots) s.valid = false;
    for (int b = 0; b < VX_BATCH_BANKS; ++b) c->batch_n[b] = 0;
    return VX_OK;
}

int vx_orb_get_order(const vx_ctx* c) { return c ? c->kp_order : VX_ERR_INVALID; }

int vx_orb_set_debug(vx_ctx* c, int flags) {
    if (!c) return VX_ERR_INVALID;
    if (flags & ~(VX_ORB_DEBUG_FAST_NO_BORDER | VX_ORB_DEBUG_STAGES))
        return set_error(c, VX_ERR_INVALID, "unknown debug flags %#x", flags);
    if (flags == c->orb_debug) return VX_OK;
    VX_HIP(c, hipSetDevice(c->device));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    for (auto& e : c->graphs.entries)
        if (e.exec) (void)hipGraphExecDestroy(e.exec);
    c->graphs.entries.clear();
    c->orb_debug = flags;
    c->geo_valid = false;  // orb_prepare sizes the debug buffer
    return VX_OK;
}

int vx_orb_debug_read(vx_ctx* c, int level, int what, void* out, int64_t cap_bytes, int64_t* n_out) {
    if (!c || !n_out) return VX_ERR_INVALID;
    *n_out = 0;
    // the scratch (pyramid, blur, candidates, stages) is shared by every slot and the batches: it
    // must still hold slot 0's single-frame extraction
    if (!c->geo_valid || !c->slots[0].valid || c->scratch_slot != 0)
        return set_error(c, VX_ERR_STATE, "no single-frame extraction into slot 0 is the last one to inspect");
    const OrbGeometry& g = c->geo;
    if (level < 0 || level >= g.L) return set_error(c, VX_ERR_INVALID, "bad level %d", level);
    if (what >= 2 && (!c->orb_debug || c->kp_order != VX_ORDER_STL))
        return set_error(c, VX_ERR_STATE, "selection stages need vx_orb_set_debug and VX_ORDER_STL");
    VX_HIP(c, hipSetDevice(c->device));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    int info[2 * kMaxLevels];
    if (what >= 2) VX_HIP(c, hipMemcpy(info, c->orb_dbg.p, sizeof info, hipMemcpyDeviceToHost));
    const CandRec* st = c->stage.as<CandRec>() + g.stage_base[level];
    const void* src = nullptr;
    int64_t n = 0, esz = 1;
    switch (what) {
        case 0: src = c->pyr.as<uint8_t>() + g.off[level]; n = (int64_t)g.lw[level] * g.lh[level]; break;
        case 1: src = c->blur.as<uint8_t>() + g.off[level]; n = (int64_t)g.lw[level] * g.lh[level]; break;
        case 2: src = st; n = info[level]; esz = sizeof(CandRec); break;
        case 3: {
            int64_t off = 2 * kMaxLevels;
            for (int i = 0; i < level; ++i) off += g.level_cap[i];
            src = c->orb_dbg.as<int>() + off;
            n = info[kMaxLevels + level];
            esz = sizeof(int);
            break;
        }
        case 4: {
            int cnt[kMaxLevels];
            VX_HIP(c, hipMemcpy(cnt, c->level_count.p, sizeof cnt, hipMemcpyDeviceToHost));
            src = st + g.level_cap[level];
            n = cnt[level];
            esz = sizeof(CandRec);
            break;
        }
        default: return set_error(c, VX_ERR_INVALID, "bad stage %d", what);
    }
    *n_out = n;
    if (n * esz > cap_bytes) return set_error(c, VX_ERR_CAPACITY, "need %lld bytes", (long long)(n * esz));
    if (n > 0) VX_HIP(c, hipMemcpy(out, src, (size_t)(n * esz), hipMemcpyDeviceToHost));
    return VX_OK;
}

int vx_test_retain_best(vx_ctx* c, const uint32_t* keys, int n, int npts, int wide, int use_lds, int32_t* out_idx,
                        int* n_out) {
    if (!c || !n_out || (n > 0 && (!keys || !out_idx)) || n < 0 || n >= (1 << 24)) return VX_ERR_INVALID;
    *n_out = 0;
    if (!wide)
        for (int i = 0; i < n; ++i)
            if (keys[i] > 255u) return set_error(c, VX_ERR_INVALID, "narrow keys must be <= 255");
    const int64_t esz = wide ? 8 : 4, need = esz * ((int64_t)n + 2 * (n / 2 + 1));
    if (use_lds && need > kStlLds - kRgBytes)
        return set_error(c, VX_ERR_INVALID, "%lld bytes exceed the LDS", (long long)need);
    VX_HIP(c, hipSetDevice(c->device));
    void *dk = nullptr, *ds = nullptr, *dout = nullptr;
    int rc = VX_OK;
    if (hipMalloc(&dk, std::max<int64_t>(4, 4 * (int64_t)n)) != hipSuccess || hipMalloc(&ds, need) != hipSuccess ||
        hipMalloc(&dout, 4 * ((int64_t)n + 1)) != hipSuccess) {
        rc = set_error(c, VX_ERR_HIP, "hipMalloc failed");
    } else {
        hipError_t e = upload_constants(c) == VX_OK ? hipSuccess : hipErrorUnknown;  // (k_test_retain's LDS size)
        if (e == hipSuccess) e = hipMemcpyAsync(dk, keys, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_test_retain, dim3(1), dim3(kStlNT), kStlLds, c->stream,
                               (const unsigned*)dk, n, npts, wide, use_lds, (unsigned char*)ds, (int*)dout);
            e = hipGetLastError();
        }
        int k = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(&k, dout, 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess && k > 0) e = hipMemcpy(out_idx, (int*)dout + 1, 4 * (size_t)k, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = hip_fail(c, e, "vx_test_retain_best");
        else *n_out = k;
    }
    if (dk) (void)hipFree(dk);
    if (ds) (void)hipFree(ds);
    if (dout) (void)hipFree(dout);
    return rc;
}

int vx_orb_pattern(int32_t* out) {
    if (!out) return VX_ERR_INVALID;
    for (int i = 0; i < 1024; ++i) out[i] = kBitPattern31[i];
    return VX_OK;
}

int vx_orb_extract_async(vx_ctx* c, const vx_orb_params* p, const uint8_t* d_img, int w, int h,
                         int channels, int64_t stride, int slot) {
    if (!c) return VX_ERR_INVALID;
    if (slot < 0 || slot >= VX_MAX_SLOTS) return set_error(c, VX_ERR_INVALID, "bad slot %d", slot);
    if (!d_img) return set_error(c, VX_ERR_INVALID, "null image");
    if (channels != 1 && channels != 3 && channels != 4)
        return set_error(c, VX_ERR_INVALID, "channels must be 1, 3 or 4");
    if (stride < (int64_t)w * channels) return set_error(c, VX_ERR_INVALID, "row stride too small");
    int rc = orb_prepare(c, p, w, h);
    if (rc) return rc;
    struct A {
        const uint8_t* img;
        int channels;
        int64_t stride;
        int slot;
    } a{d_img, channels, stride, slot};
    rc = graph_run(c, {1, (uint64_t)(uintptr_t)d_img, (uint64_t)channels, (uint64_t)stride, (uint64_t)slot, c->geo_gen},
                   [](vx_ctx* cc, void* v) {
                       const A* x = static_cast<const A*>(v);
                       return orb_enqueue(cc, x->img, x->channels, x->stride, x->slot);
                   },
                   &a);
    c->scratch_slot = rc ? -1 : slot;  // (a graph replay writes the scratch too: set here, not in orb_enqueue)
    return rc;
}

int vx_orb_fetch(vx_ctx* c, int slot, vx_keypoint* out_kp, uint8_t* out_desc, int cap, int* n_out) {
    if (!c || !n_out) return VX_ERR_INVALID;
    if (slot < 0 || slot >= VX_MAX_SLOTS || !c->slots[slot].valid)
        return set_error(c, VX_ERR_STATE, "slot %d holds no extraction", slot);
    Slot& s = c->slots[slot];
    int cnt[2];
    VX_HIP(c, hipMemcpyAsync(cnt, s.count.p, sizeof cnt, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) prof_collect(c);
    *n_out = cnt[0];
    if (cnt[1]) return set_error(c, VX_ERR_CAPACITY, "keypoints %d exceed slot capacity %d", cnt[0], s.cap);
    if (cnt[0] > cap) return set_error(c, VX_ERR_CAPACITY, "need %d keypoints, cap %d", cnt[0], cap);
    if (cnt[0] > 0) {
        if (out_kp)
            VX_HIP(c, hipMemcpyAsync(out_kp, s.kp.p, (size_t)cnt[0] * sizeof(vx_keypoint),
                                     hipMemcpyDeviceToHost, c->stream));
        if (out_desc)
            VX_HIP(c, hipMemcpyAsync(out_desc, s.desc.p, (size_t)cnt[0] * 32, hipMemcpyDeviceToHost, c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));
    }
    return VX_OK;
}

int vx_orb_slot_device(vx_ctx* c, int slot, const uint8_t** d_desc, const int32_t** d_count, int32_t* cap) {
    if (!c || slot < 0 || slot >= VX_MAX_SLOTS || !c->slots[slot].valid) return VX_ERR_INVALID;
    if (d_desc) *d_desc = c->slots[slot].desc.as<uint8_t>();
    if (d_count) *d_count = c->slots[slot].count.as<int32_t>();
    if (cap) *cap = c->slots[slot].cap;
    return VX_OK;
}

int vx_orb_extract_batch_async(vx_ctx* c, const vx_orb_params* p, const uint8_t* d_imgs, int n_frames,
                               int64_t frame_stride, int w, int h, int channels, int64_t stride, int bank) {
    if (!c) return VX_ERR_INVALID;
    if (bank < 0 || bank >= VX_BATCH_BANKS) return set_error(c, VX_ERR_INVALID, "bad batch bank %d", bank);
    if (n_frames < 1 || n_frames > VX_MAX_BATCH)
        return set_error(c, VX_ERR_INVALID, "n_frames %d outside [1, %d]", n_frames, VX_MAX_BATCH);
    if (!d_imgs) return set_error(c, VX_ERR_INVALID, "null images");
    if (channels != 1 && channels != 3 && channels != 4)
        return set_error(c, VX_ERR_INVALID, "channels must be 1, 3 or 4");
    if (stride < (int64_t)w * channels) return set_error(c, VX_ERR_INVALID, "row stride too small");
    if (n_frames > 1 && frame_stride < (int64_t)(h - 1) * stride + (int64_t)w * channels)
        return set_error(c, VX_ERR_INVALID, "frame stride smaller than one frame");
    int rc = orb_prepare(c, p, w, h);
    if (rc) return rc;
    VX_HIP(c, hipSetDevice(c->device));
    rc = orb_reserve_frames(c, n_frames, bank);
    if (rc) return rc;
    c->batch_n[bank] = 0;
    Slot& s = c->batch[bank];
    struct A {
        const uint8_t* img;
        int channels, nf;
        int64_t stride, fs;
        Slot* s;
    } a{d_imgs, channels, n_frames, stride, n_frames > 1 ? frame_stride : 0, &s};
    rc = graph_run(c, {3, (uint64_t)(uintptr_t)d_imgs, (uint64_t)channels, (uint64_t)stride, (uint64_t)a.fs,
                       (uint64_t)n_frames, (uint64_t)(uintptr_t)s.kp.p, (uint64_t)(uintptr_t)s.desc.p,
                       (uint64_t)(uintptr_t)s.count.p, c->geo_gen},
                   [](vx_ctx* cc, void* v) {
                       const A* x = static_cast<const A*>(v);
                       return orb_enqueue_frames(cc, x->img, x->channels, x->stride, x->fs, x->nf,
                                                 x->s->kp.as<vx_keypoint>(), x->s->desc.as<uint8_t>(),
                                                 x->s->count.as<int>());
                   },
                   &a);
    c->scratch_slot = -1;  // the batch overwrote the shared scratch
    if (rc) return rc;
    c->batch_n[bank] = n_frames;
    return VX_OK;
}

int vx_orb_extract_batch(vx_ctx* c, const vx_orb_params* p, const uint8_t* const* imgs, int n_frames, int w, int h,
                         int channels, int64_t stride, int bank) {
    if (!c) return VX_ERR_INVALID;
    if (!imgs) return set_error(c, VX_ERR_INVALID, "null images");
    if (n_frames < 1 || n_frames > VX_MAX_BATCH)
        return set_error(c, VX_ERR_INVALID, "n_frames %d outside [1, %d]", n_frames, VX_MAX_BATCH);
    if (channels != 1 && channels != 3 && channels != 4)
        return set_error(c, VX_ERR_INVALID, "channels must be 1, 3 or 4");
    if (stride < (int64_t)w * channels) return set_error(c, VX_ERR_INVALID, "row stride too small");
    for (int f = 0; f < n_frames; ++f)
        if (!imgs[f]) return set_error(c, VX_ERR_INVALID, "null image %d", f);
    int rc = orb_prepare(c, p, w, h);
    if (rc) return rc;
    VX_HIP(c, hipSetDevice(c->device));
    // frames packed back to back in the context's upload buffer, then the device-resident batch
    const size_t packed = (size_t)w * channels, fbytes = packed * h;
    VX_HIP(c, c->img_in.ensure(fbytes * n_frames));
    for (int f = 0; f < n_frames; ++f)
        VX_HIP(c, hipMemcpy2DAsync(c->img_in.as<uint8_t>() + f * fbytes, packed, imgs[f], (size_t)stride, packed, h,
                                   hipMemcpyHostToDevice, c->stream));
    return vx_orb_extract_batch_async(c, p, c->img_in.as<uint8_t>(), n_frames, (int64_t)fbytes, w, h, channels,
                                      (int64_t)packed, bank);
}

int vx_orb_batch_device(vx_ctx* c, int bank, int frame, const uint8_t** d_desc, const int32_t** d_count,
                        int32_t* cap) {
    if (!c || bank < 0 || bank >= VX_BATCH_BANKS || frame < 0 || frame >= c->batch_n[bank]) return VX_ERR_INVALID;
    const Slot& s = c->batch[bank];
    if (d_desc) *d_desc = s.desc.as<uint8_t>() + (size_t)frame * s.cap * 32;
    if (d_count) *d_count = s.count.as<int32_t>() + 4 * (size_t)frame;
    if (cap) *cap = s.cap;
    return VX_OK;
}

int vx_orb_batch_fetch(vx_ctx* c, int bank, int frame, vx_keypoint* out_kp, uint8_t* out_desc, int cap, int* n_out) {
    if (!c || !n_out) return VX_ERR_INVALID;
    if (bank < 0 || bank >= VX_BATCH_BANKS || frame < 0 || frame >= c->batch_n[bank])
        return set_error(c, VX_ERR_STATE, "batch bank %d holds no frame %d", bank, frame);
    const Slot& s = c->batch[bank];
    int cnt[2];
    VX_HIP(c, hipMemcpyAsync(cnt, s.count.as<int>() + 4 * (size_t)frame, sizeof cnt, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) prof_collect(c);
    *n_out = cnt[0];
    if (cnt[1]) return set_error(c, VX_ERR_CAPACITY, "keypoints %d exceed slot capacity %d", cnt[0], s.cap);
    if (cnt[0] > cap) return set_error(c, VX_ERR_CAPACITY, "need %d keypoints, cap %d", cnt[0], cap);
    if (cnt[0] > 0) {
        if (out_kp)
            VX_HIP(c, hipMemcpyAsync(out_kp, s.kp.as<vx_keypoint>() + (size_t)frame * s.cap,
                                     (size_t)cnt[0] * sizeof(vx_keypoint), hipMemcpyDeviceToHost, c->stream));
        if (out_desc)
            VX_HIP(c, hipMemcpyAsync(out_desc, s.desc.as<uint8_t>() + (size_t)frame * s.cap * 32, (size_t)cnt[0] * 32,
                                     hipMemcpyDeviceToHost, c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));
    }
    return VX_OK;
}

int vx_orb_extract(vx_ctx* c, const vx_orb_params* p, const uint8_t* img, int w, int h, int channels,
                   int64_t stride, vx_keypoint* out_kp, uint8_t* out_desc, int cap, int* n_out) {
    if (!c || !img || !n_out) return VX_ERR_INVALID;
    *n_out = 0;
    if (channels != 1 && channels != 3 && channels != 4)
        return set_error(c, VX_ERR_INVALID, "channels must be 1, 3 or 4");
    if (stride < (int64_t)w * channels) return set_error(c, VX_ERR_INVALID, "row stride too small");
    int rc = orb_prepare(c, p, w, h);
    if (rc) return rc;
    const size_t packed = (size_t)w * channels;
    VX_HIP(c, c->img_in.ensure(packed * h));
    VX_HIP(c, hipMemcpy2DAsync(c->img_in.p, packed, img, (size_t)stride, packed, h, hipMemcpyHostToDevice,
                               c->stream));
    rc = orb_enqueue(c, c->img_in.as<uint8_t>(), channels, (int64_t)packed, 0);
    c->scratch_slot = rc ? -1 : 0;
    if (rc) return rc;
    return vx_orb_fetch(c, 0, out_kp, out_desc, cap, n_out);
}

}  // extern "C"
