// stl_select_model.cpp — CPU model of the device retainBest permutation (k_select_stl, orb.hip),
// checked against the C++ standard library it restates.  TEST INFRASTRUCTURE ONLY.
//
// OpenCV's KeyPointsFilter::retainBest (the two calls in ORB's computeKeyPoints, SURVEY.md App.
// A.3; reached from ORBExtractor::Extract, core/feature/orb_extractor.cpp:13) is
//     std::nth_element(kp.begin(), kp.begin() + n - 1, kp.end(), response-greater);
//     thr = kp[n - 1].response;
//     kp.resize(std::partition(kp.begin() + n, kp.end(), response >= thr) - kp.begin());
// and the keypoint ORDER it leaves is libstdc++'s (introselect: median-of-3 pivot moved to the
// front, unguarded Hoare partition, depth limit 2*lg(n) -> heap select, insertion sort <= 3).
//
// The device does one partition PASS in parallel: in [f+1, l) with pivot value P the left
// scanner stops at every x with !(x > P) ("L" elements), the right scanner at every x with
// !(P > x) ("R"); the k-th swap exchanges the k-th L from the left with the k-th R from the
// right, for k < K, and
//     K   = max over x in [f+1, l] of min(#L in [f+1, x), #R in [x, l))
//     cut = min(L[K], R[K-1])                       (absent terms are +inf)
// std::partition (bidirectional form) is the same pairing with complementary predicates.  This
// program restates exactly that formulation (prefix counts, K by the max-min rule, swaps through
// per-rank mailboxes as the device does) and compares the resulting permutation with the real
// std::nth_element / std::partition on random, tie-heavy, sorted and adversarial (McIlroy
// "antiqsort", which drives libstdc++ into its heap-select fallback) inputs.
//
// Build: g++ -O2 -std=c++17 stl_select_model.cpp; exit status 0 = every case identical.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

using u64 = uint64_t;
static inline uint32_t key(u64 v) { return (uint32_t)(v >> 32); }
static inline bool gt(u64 a, u64 b) { return key(a) > key(b); }  // comp = response-greater

static int lg(int n) { int r = 0; while (n >>= 1) ++r; return r; }

// libstdc++ __adjust_heap / __push_heap / __make_heap / __pop_heap / __heap_select with comp = gt
static void push_heap(u64* a, int hole, int top, u64 v) {
    int parent = (hole - 1) / 2;
    while (hole > top && gt(a[parent], v)) { a[hole] = a[parent]; hole = parent; parent = (hole - 1) / 2; }
    a[hole] = v;
}
static void adjust_heap(u64* a, int hole, int len, u64 v) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (gt(a[child], a[child - 1])) --child;
        a[hole] = a[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        a[hole] = a[child - 1];
        hole = child - 1;
    }
    push_heap(a, hole, top, v);
}
static void heap_select(u64* a, int mid, int last) {
    if (mid >= 2)
        for (int parent = (mid - 2) / 2;; --parent) {
            adjust_heap(a, parent, mid, a[parent]);
            if (parent == 0) break;
        }
    for (int i = mid; i < last; ++i)
        if (gt(a[i], a[0])) {
            const u64 v = a[i];
            a[i] = a[0];
            adjust_heap(a, 0, mid, v);
        }
}

// One partition pass of [f+1, l) around the pivot value at f, in the device formulation.
// isl / isr: the left / right scanner's stop predicates.  Returns the cut.
template <class IsL, class IsR>
static int pass(std::vector<u64>& A, int f0, int l, IsL isl, IsR isr) {
    int nL = 0, nR = 0;
    for (int p = f0; p < l; ++p) { nL += isl(A[p]); nR += isr(A[p]); }
    // K = max_x min(Lcount(x), Rcount(x)); L / R positions by rank
    std::vector<int> Lb(l - f0), Rb(l - f0);
    int lb = 0, rb = 0, K = 0;
    for (int p = f0; p < l; ++p) {
        Lb[p - f0] = lb; Rb[p - f0] = rb;
        K = std::max(K, std::min(lb, nR - rb));
        lb += isl(A[p]); rb += isr(A[p]);
    }
    int cut = INT32_MAX;
    std::vector<u64> boxL(K), boxR(K);
    for (int p = f0; p < l; ++p) {
        const int i = p - f0;
        if (isl(A[p]) && Lb[i] == K) cut = std::min(cut, p);          // L[K]
        if (isr(A[p]) && nR - 1 - Rb[i] == K - 1) cut = std::min(cut, p);  // R[K-1]
        if (isl(A[p]) && Lb[i] < K) boxL[Lb[i]] = A[p];
        if (isr(A[p]) && nR - 1 - Rb[i] < K) boxR[nR - 1 - Rb[i]] = A[p];
    }
    // The device passes decide every swap without K: an L of rank Lb is swapped iff more than Lb R
    // lie after it (Lb + Rb + isR < nR), an R iff more than its right rank of L lie before it
    // (Lb + Rb >= nR); the cut is the first position that is an unswapped L or a swapped R.
    int cut2 = INT32_MAX;
    for (int p = f0; p < l; ++p) {  // a position is never both a swapped L and a swapped R
        const int i = p - f0;
        const bool sl = isl(A[p]) && Lb[i] < K, sr = isr(A[p]) && nR - 1 - Rb[i] < K;
        if (sl && sr) { std::printf("position both swapped\n"); std::exit(3); }
        const bool sl2 = isl(A[p]) && Lb[i] + Rb[i] + (int)isr(A[p]) < nR;
        const bool sr2 = isr(A[p]) && Lb[i] + Rb[i] >= nR;
        if (sl2 != sl || sr2 != sr) { std::printf("rank-sum swap rule differs\n"); std::exit(3); }
        if (cut2 == INT32_MAX && ((isl(A[p]) && !sl2) || sr2)) cut2 = p;
    }
    if (cut2 != cut) { std::printf("first-position cut differs\n"); std::exit(3); }
    for (int p = f0; p < l; ++p) {
        const int i = p - f0;
        const bool sl = isl(A[p]) && Lb[i] < K, sr = isr(A[p]) && nR - 1 - Rb[i] < K;
        if (sl) A[p] = boxR[Lb[i]];
        else if (sr) A[p] = boxL[nR - 1 - Rb[i]];
    }
    return cut;
}

static bool g_heap_used = false;

static void nth_element_model(std::vector<u64>& A, int nth) {
    int f = 0, l = (int)A.size();
    if (f == l || nth == l) return;
    int depth = 2 * lg(l - f);
    while (l - f > 3) {
        if (depth == 0) {
            g_heap_used = true;
            heap_select(A.data() + f, nth + 1 - f, l - f);
            std::swap(A[f], A[nth]);
            return;
        }
        --depth;
        const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
        int m;  // __move_median_to_first(f, a, b, c)
        if (gt(A[a], A[b])) m = gt(A[b], A[c]) ? b : gt(A[a], A[c]) ? c : a;
        else m = gt(A[a], A[c]) ? a : gt(A[b], A[c]) ? c : b;
        std::swap(A[f], A[m]);
        const u64 P = A[f];
        const int cut = pass(A, f + 1, l, [&](u64 x) { return !gt(x, P); }, [&](u64 x) { return !gt(P, x); });
        if (cut <= nth) f = cut; else l = cut;
    }
    for (int i = f + 1; i < l; ++i) {  // __insertion_sort
        const u64 v = A[i];
        if (gt(v, A[f])) {
            for (int j = i; j > f; --j) A[j] = A[j - 1];
            A[f] = v;
        } else {
            int j = i;
            while (gt(v, A[j - 1])) { A[j] = A[j - 1]; --j; }
            A[j] = v;
        }
    }
}

// retainBest in the device formulation; returns the kept length
static int retain_best_model(std::vector<u64>& A, int n) {
    if ((int)A.size() <= n) return (int)A.size();
    nth_element_model(A, n - 1);
    const uint32_t thr = key(A[n - 1]);
    // std::partition(begin + n, end, >= thr): left stops at < thr, right stops at >= thr
    pass(A, n, (int)A.size(), [&](u64 x) { return key(x) < thr; }, [&](u64 x) { return key(x) >= thr; });
    int kept = n;
    for (size_t p = n; p < A.size(); ++p) kept += key(A[p]) >= thr;
    return kept;
}

static int retain_best_stl(std::vector<u64>& A, int n) {
    if ((int)A.size() <= n) return (int)A.size();
    std::nth_element(A.begin(), A.begin() + n - 1, A.end(), gt);
    const uint32_t thr = key(A[n - 1]);
    return (int)(std::partition(A.begin() + n, A.end(), [&](u64 x) { return key(x) >= thr; }) - A.begin());
}

// McIlroy's adversary, driven through the real std::nth_element: returns keys that defeat its
// median-of-3 pivots (so the depth limit and the heap select are reached).
static std::vector<uint32_t> antiqsort(int n, int nth) {
    std::vector<int> val(n, n - 1);  // gas = n - 1
    int nsolid = 0, candidate = 0;
    const int gas = n - 1;
    std::vector<int> ptr(n);
    for (int i = 0; i < n; ++i) ptr[i] = i;
    auto less = [&](int x, int y) {  // ordering "greater" over frozen values, as comp = gt
        if (val[x] == gas && val[y] == gas) { if (x == candidate) val[x] = nsolid++; else val[y] = nsolid++; }
        if (val[x] == gas) candidate = x;
        else if (val[y] == gas) candidate = y;
        return val[x] > val[y];
    };
    std::nth_element(ptr.begin(), ptr.begin() + nth, ptr.end(), less);
    std::vector<uint32_t> keys(n);
    for (int i = 0; i < n; ++i) keys[i] = (uint32_t)val[i];
    return keys;
}

static int check(const std::vector<uint32_t>& keys, int n, const char* what, long& cases) {
    std::vector<u64> a(keys.size()), b;
    for (size_t i = 0; i < keys.size(); ++i) a[i] = ((u64)keys[i] << 32) | i;
    b = a;
    const int ka = retain_best_model(a, n), kb = retain_best_stl(b, n);
    ++cases;
    if (ka != kb || !std::equal(a.begin(), a.begin() + ka, b.begin())) {
        std::printf("MISMATCH %s size %zu n %d (kept %d vs %d)\n", what, keys.size(), n, ka, kb);
        return 1;
    }
    return 0;
}

int main() {
    std::mt19937_64 rng(0x5EED);
    long cases = 0;
    int bad = 0;
    for (int it = 0; it < 20000 && !bad; ++it) {
        const int size = 1 + (int)(rng() % (it < 15000 ? 300 : 9000));
        const int n = 1 + (int)(rng() % size);
        const int mode = (int)(rng() % 6);
        const uint32_t range = mode == 0 ? 2 : mode == 1 ? 8 : mode == 2 ? 236 : mode == 3 ? 100000 : 1u << 31;
        std::vector<uint32_t> k(size);
        for (auto& x : k) x = (uint32_t)(rng() % range);
        if (mode == 4) std::sort(k.begin(), k.end());
        if (mode == 5) std::sort(k.rbegin(), k.rend());
        bad |= check(k, n, "random", cases);
    }
    bool heap_hit = false;
    for (int size : {16, 17, 31, 64, 100, 257, 1000, 1763, 4096, 6781}) {
        for (int n : {1, 2, size / 3, size / 2, size - 1}) {
            if (n < 1 || n >= size) continue;
            g_heap_used = false;
            bad |= check(antiqsort(size, n - 1), n, "antiqsort", cases);
            heap_hit |= g_heap_used;
        }
    }
    std::printf("%ld cases, %s, heap select %s\n", cases, bad ? "MISMATCH" : "all identical",
                heap_hit ? "exercised" : "NOT exercised");
    return bad ? 1 : (heap_hit ? 0 : 2);
}
