// pdqsort.h — Go 1.19 sort.Slice (pdqsort_func) on the device: the exact permutation
// the reference's unstable sort produces, one workgroup per node group.
//
// Reference: CA/estimator/binpacking_estimator.go:74 sorts the pods of a node group with
// sort.Slice(podInfos, score_i > score_j); Go 1.19's sort.Slice is pdqsort_func
// (src/sort/zsortfunc.go: insertionSort_func, heapSort_func, pdqsort_func,
// partition_func, partitionEqual_func, partialInsertionSort_func, breakPatterns_func,
// choosePivot_func, reverseRange_func; src/sort/sort.go xorshift, nextPowerOfTwo).  The
// C restatement the tests check against is oracle/gosort.c.
//
// The permutation depends only on the comparisons, i.e. on the dense rank of each pod's
// float64 score (equal scores share a rank; less(i, j) == rank_i < rank_j).  The device
// reproduces pdqsort_func's swaps with three reformulations, each exact:
//   * Independent frames.  After a partition the two sides are sorted by calls that read
//     and write only their own range, plus the element just left of it (the
//     partitionEqual test, a final pivot or equal-zone element no later step moves), so
//     every pending range (a, b, limit, wasBalanced, wasPartitioned) can run at once and
//     in any order.  A workgroup step runs one pdqsort_func loop iteration of up to MAXF
//     frames longer than T_SMALL together; shorter frames wait, then are sorted to the
//     end by one wavefront each, claimed in turn (no workgroup barrier).
//   * Partition as a rank-paired exchange.  partition_func / partitionEqual_func are
//     Hoare scans over [a+1, b-1] against the pivot moved to a: with m = #{pred}, the
//     k-th element of [a+1, a+m] failing pred (from the left) is swapped with the k-th
//     element of [a+m+1, b-1] passing it (from the right) — prefix counts, then one swap
//     per pair in parallel.  partition_func then swaps a with a+m (mid = a+m,
//     alreadyPartitioned = no pair); partitionEqual_func returns a+m+1.
//     pred = rank < pivot rank (partition) or rank <= pivot rank (partitionEqual).
//   * partialInsertionSort as search + shift: the two bubbling loops after a swap move one
//     element over a run it compares against unchanged values, so its landing place is a
//     parallel search and the run shifts by one.
// Validated against oracle/gosort.c on randomized inputs (tests/test_gosort.py runs the
// device kernel through ca_go_sort_ranks on every branch: heapSort, breakPatterns,
// reverse, partialInsertionSort).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>
#include <type_traits>

namespace casim {
namespace pdq {

#ifdef CASIM_PROF    // phase cycle counters of workgroup 0 (profiling build: ca_debug_pdq_prof)
__device__ unsigned long long g_pdq_prof[32 + 16 * 16];   // + per-step slots [32 + 16 step + k]
__device__ int g_pdq_step;
// wavefront partialInsertionSort, summed over the waves of workgroup 0: find cycles,
// rotate cycles, search loop trips, rotate loop trips, steps, calls, rotated quads
__device__ unsigned long long g_pdq_pis[8];
// per workgroup (group slot < 128): kernel cycles, prologue (ranks into the store) cycles,
// epilogue (ids out) cycles
__device__ unsigned long long g_pdq_wg[3 * 128];
#define PDQ_PIS(k, v) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) atomicAdd(&g_pdq_pis[k], (unsigned long long)(v)); } while (0)
#define PDQ_S(k, v) do { if (threadIdx.x == 0 && blockIdx.x == 0 && g_pdq_step < 16) g_pdq_prof[32 + 16 * g_pdq_step + (k)] += (unsigned long long)(v); } while (0)
#define PDQ_SMAXW(k, v) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 0 && g_pdq_step < 16) atomicMax(&g_pdq_prof[32 + 16 * g_pdq_step + (k)], (unsigned long long)(v)); } while (0)
#define PDQ_T(v) const uint64_t v = clock64()
#define PDQ_ADD(i, t) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_pdq_prof[i] += clock64() - (t); } while (0)
#define PDQ_CNT(i, n) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_pdq_prof[i] += (n); } while (0)
#define PDQ_WADD(i, t) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) atomicAdd(&g_pdq_prof[i], clock64() - (t)); } while (0)
// sum over steps of the slowest wave's duration: per-step maxima accumulate in slot i+32
#define PDQ_WMAX(i, t) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) atomicAdd(&g_pdq_prof[i], clock64() - (t)); } while (0)
#define PDQ_TMAX(i, v) do { if (blockIdx.x == 0) atomicMax(&g_pdq_prof[i], (unsigned long long)(v)); } while (0)
#define PDQ_TADD(i, v) do { if (blockIdx.x == 0) atomicAdd(&g_pdq_prof[i], (unsigned long long)(v)); } while (0)
#else
#define PDQ_S(k, v) (void)0
#define PDQ_SMAXW(k, v) (void)0
#define PDQ_PIS(k, v) (void)0
#define PDQ_WADD(i, t) (void)0
#define PDQ_WMAX(i, t) (void)0
#define PDQ_TMAX(i, v) (void)0
#define PDQ_TADD(i, v) (void)0
#define PDQ_T(v) (void)0
#define PDQ_ADD(i, t) (void)0
#define PDQ_CNT(i, n) (void)0
#endif

constexpr int NT = 1024;             // threads of the workgroup
constexpr int NW = NT / 64;          // wavefronts
#ifndef CASIM_PDQ_MAXF
#define CASIM_PDQ_MAXF 96
#endif
constexpr int MAXF = CASIM_PDQ_MAXF; // frames per workgroup step
constexpr int PIS_WAVE_MAX = 4096;   // LDS store: longer frames run partialInsertionSort on the workgroup
constexpr int MAX_INSERTION = 12;    // pdqsort_func maxInsertion
enum { HINT_UNKNOWN = 0, HINT_INC = 1, HINT_DEC = 2 };
enum { OP_DONE = 0, OP_PART = 1, OP_EQ = 2 };

// A pending pdqsort_func call / loop state: [a, b), limit | wasBalanced<<8 | wasPartitioned<<9
struct Frame { int32_t a, b, lf; };
__device__ inline int32_t lf_pack(int limit, bool wb, bool wp) { return limit | (wb ? 256 : 0) | (wp ? 512 : 0); }

__device__ inline int bits_len(uint32_t x) { return x ? 32 - __clz((int)x) : 0; }

// Element stores.  An element is a position of the group's pod list; key() is its rank.
// LDS: 16-bit positions + the 8-bit rank of the element at each index, the two arrays
// moved together (groups of <= PDQ_LDS_N pods, <= 256 ranks — C2 / C4): a comparison is
// one byte load.  Global: the rank packed above the position (32 or 64 bits).
struct LdsStore {
    using Elem = uint32_t;
    uint16_t* e;
    uint8_t* rk;
    uint64_t* rmb;           // workgroup partition: moved positions (LM | RM) per 64-position word
    uint16_t* rmp;           //   and their exclusive prefix counts per word
    __device__ Elem ld(int i) const { return ((uint32_t)rk[i] << 16) | e[i]; }
    __device__ void st(int i, Elem v) const { e[i] = (uint16_t)v; rk[i] = (uint8_t)(v >> 16); }
    __device__ uint32_t key_at(int i) const { return rk[i]; }
    __device__ static uint32_t key(Elem v) { return v >> 16; }
    __device__ static uint32_t pos(Elem v) { return v & 0xFFFFu; }
};
struct G32Store {   // rank < 4096, position < 2^20
    using Elem = uint32_t;
    uint32_t* e;
    __device__ Elem ld(int i) const { return e[i]; }
    __device__ void st(int i, Elem v) const { e[i] = v; }
    __device__ uint32_t key_at(int i) const { return e[i] >> 20; }
    __device__ static uint32_t key(Elem v) { return v >> 20; }
    __device__ static uint32_t pos(Elem v) { return v & 0xFFFFFu; }
};
struct G64Store {
    using Elem = uint64_t;
    uint64_t* e;
    __device__ Elem ld(int i) const { return e[i]; }
    __device__ void st(int i, Elem v) const { e[i] = v; }
    __device__ uint32_t key_at(int i) const { return (uint32_t)(e[i] >> 32); }
    __device__ static uint32_t key(Elem v) { return (uint32_t)(v >> 32); }
    __device__ static uint32_t pos(Elem v) { return (uint32_t)v; }
};

template <class S> __device__ inline uint32_t K(const S& s, int i) { return s.key_at(i); }
template <class S> __device__ inline void swp(const S& s, int i, int j) {
    const typename S::Elem x = s.ld(i), y = s.ld(j);
    s.st(i, y);
    s.st(j, x);
}

// one lane's stores visible to the other lanes (LDS and global)
__device__ inline void wfence() { __threadfence_block(); }
__device__ inline int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline uint64_t lanes_below() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// ---------------------------------------------------------------------------------
// serial pieces (one lane)
// ---------------------------------------------------------------------------------
// heapSort_func / siftDown_func
template <class S> __device__ void sift_down(const S& s, int lo, int hi, int first) {
    int root = lo;
    for (;;) {
        int child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && K(s, first + child) < K(s, first + child + 1)) child++;
        if (!(K(s, first + root) < K(s, first + child))) return;
        swp(s, first + root, first + child);
        root = child;
    }
}
template <class S> __device__ void heap_sort(const S& s, int a, int b) {
    const int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(s, i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
        swp(s, first, first + i);
        sift_down(s, lo, i, first);
    }
}

// breakPatterns_func with sort.go's xorshift (the shift triple is the one unpinned
// assumption of the restatement; oracle/gosort.c uses the same)
template <class S> __device__ void break_patterns(const S& s, int a, int b) {
    const int len = b - a;
    if (len < 8) return;
    uint64_t r = (uint64_t)len;
    const uint64_t mod = 1ull << bits_len((uint32_t)len);          // nextPowerOfTwo
    const int idx = a + (len / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> 17;
        r ^= r << 5;
        int other = (int)(r & (mod - 1));
        if (other >= len) other -= len;
        swp(s, idx - 1 + i, a + other);
    }
}

// ---------------------------------------------------------------------------------
// wavefront pieces (all 64 lanes, uniform control flow)
// ---------------------------------------------------------------------------------
// choosePivot_func: the (up to) nine sampled keys are loaded by nine lanes at once, then
// the median network runs on lane indices with uniform readlanes.  Returns the pivot
// position; *hint = increasing / decreasing / unknown.
template <class S> __device__ int w_choose_pivot(const S& s, int a, int b, int* hint) {
    const int lane = threadIdx.x & 63;
    const int l = b - a;
    const int pi = a + l / 4 * 1, pj = a + l / 4 * 2, pk = a + l / 4 * 3;
    // lane 3q + d holds position {pi, pj, pk}[q] + d - 1
    int mypos = 0;
    uint32_t mykey = 0;
    if (l >= 8 && lane < 9) {
        const int q = lane / 3, d = lane % 3;
        mypos = (q == 0 ? pi : q == 1 ? pj : pk) + d - 1;
        if (l >= 50 || d == 1) mykey = K(s, mypos);
    }
    int swaps = 0;
    auto key = [&](int ln) { return (uint32_t)__builtin_amdgcn_readlane(mykey, ln); };
    auto order2 = [&](int& x, int& y) {      // order2_func on lane ids
        if (key(y) < key(x)) { const int t = x; x = y; y = t; swaps++; }
    };
    auto median = [&](int x, int y, int z) { order2(x, y); order2(y, z); order2(x, y); return y; };
    int li = 1, lj = 4, lk = 7;
    int result = pj;
    if (l >= 8) {
        if (l >= 50) {
            li = median(0, 1, 2);
            lj = median(3, 4, 5);
            lk = median(6, 7, 8);
        }
        lj = median(li, lj, lk);
        result = __builtin_amdgcn_readlane(mypos, lj);
    }
    *hint = swaps == 0 ? HINT_INC : swaps == 12 ? HINT_DEC : HINT_UNKNOWN;
    return result;
}

// insertionSort_func on <= 12 elements: stable, so each element's place is its rank
template <class S> __device__ void w_insertion(const S& s, int a, int b) {
    const int lane = threadIdx.x & 63, n = b - a;
    typename S::Elem x = 0;
    uint32_t k = 0xFFFFFFFFu;
    if (lane < n) { x = s.ld(a + lane); k = S::key(x); }
    int dest = 0;
    for (int j = 0; j < n; j++) {
        const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane(k, j);
        dest += (kj < k || (kj == k && j < lane)) ? 1 : 0;
    }
    wfence();
    if (lane < n) s.st(a + dest, x);
    wfence();
}

// reverseRange_func
template <class S> __device__ void w_reverse(const S& s, int a, int b) {
    const int lane = threadIdx.x & 63, half = (b - a) / 2;
    for (int k0 = 0; k0 < half; k0 += 64) {
        const int k = k0 + lane;
        if (k < half) swp(s, a + k, b - 1 - k);
    }
    wfence();
}

// first i' in [i, b) with less(i', i'-1), or b (256 positions per step)
template <class S> __device__ int w_find_descent(const S& s, int i, int b) {
    const int lane = threadIdx.x & 63;
    for (int base = i; base < b; base += 256) {
        uint64_t m[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = base + u * 64 + lane;
            const bool d = p < b && K(s, p) < K(s, p - 1);
            m[u] = __ballot(d);
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (m[u]) return base + u * 64 + __builtin_ctzll(m[u]);
    }
    return b;
}

// shift [lo, hi] one place right (to [lo+1, hi+1]) / left (to [lo-1, hi-1])
template <class S> __device__ void w_shift_right(const S& s, int lo, int hi) {
    const int lane = threadIdx.x & 63;
    for (int top = hi; top >= lo; top -= 256) {                     // right to left, 256 per step
        typename S::Elem v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = top - u * 64 - lane;
            v[u] = p >= lo ? s.ld(p) : 0;
        }
        wfence();
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = top - u * 64 - lane;
            if (p >= lo) s.st(p + 1, v[u]);
        }
        wfence();
    }
}
template <class S> __device__ void w_shift_left(const S& s, int lo, int hi) {
    const int lane = threadIdx.x & 63;
    for (int bot = lo; bot <= hi; bot += 256) {                     // left to right, 256 per step
        typename S::Elem v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = bot + u * 64 + lane;
            v[u] = p <= hi ? s.ld(p) : 0;
        }
        wfence();
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = bot + u * 64 + lane;
            if (p <= hi) s.st(p - 1, v[u]);
        }
        wfence();
    }
}

// partialInsertionSort_func on [a, b) (true: the range is sorted)
template <class S> __device__ bool w_partial_insertion(const S& s, int a, int b) {
    const int lane = threadIdx.x & 63;
    constexpr int maxSteps = 5, shortestShifting = 50;
    int i = a + 1;
    for (int step = 0; step < maxSteps; step++) {
        i = w_find_descent(s, i, b);
        if (i == b) return true;
        if (b - a < shortestShifting) return false;
        if (lane == 0) swp(s, i, i - 1);
        wfence();
        if (i - a >= 2) {
            // shift the smaller one to the left: e (now at i-1) passes every q with key > key(e)
            const typename S::Elem e = s.ld(i - 1);
            const uint32_t ke = S::key(e);
            const int qmin = a > 0 ? a - 1 : 0;   // key(a-1) <= every key of [a, b): the walk stops there
            int land = 0;
            bool found = false;
            for (int top = i - 2; top >= qmin && !found; top -= 256) {   // 256 positions per step
                uint64_t m[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int q = top - u * 64 - lane;
                    m[u] = __ballot(q >= qmin && K(s, q) <= ke);
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (!found && m[u]) { land = top - u * 64 - (int)__builtin_ctzll(m[u]) + 1; found = true; }
            }
            if (!found) land = qmin == 0 ? 0 : qmin;   // (qmin == a-1 always stops: never reached)
            if (land < i - 1) {
                w_shift_right(s, land, i - 2);
                if (lane == 0) s.st(land, e);
                wfence();
            }
        }
        if (b - i >= 2) {
            // shift the greater one to the right: f (now at i) passes every j with key < key(f)
            const typename S::Elem f = s.ld(i);
            const uint32_t kf = S::key(f);
            int land = b - 1;
            bool found = false;
            for (int bot = i + 1; bot < b && !found; bot += 256) {        // 256 positions per step
                uint64_t m[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int j = bot + u * 64 + lane;
                    m[u] = __ballot(j < b && !(K(s, j) < kf));
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (!found && m[u]) { land = bot + u * 64 + (int)__builtin_ctzll(m[u]) - 1; found = true; }
            }
            if (land > i) {
                w_shift_left(s, i + 1, land);
                if (lane == 0) s.st(land, f);
                wfence();
            }
        }
    }
    return false;
}

// position of the k-th set bit (0-based) of m
__device__ inline int select_bit(uint64_t m, int k) {
    int pos = 0;
    for (int w = 32; w >= 1; w >>= 1) {
        const int c = __builtin_popcountll((m >> pos) & ((1ull << w) - 1));
        if (k >= c) { k -= c; pos += w; }
    }
    return pos;
}

// partition_func (eq = 0) / partitionEqual_func (eq = 1) on [a, b) whose pivot (key pk)
// is already at a: the rank-paired exchange, by one wavefront with no memory round trip.
// m = #pred over [a+1, b-1] (four 64-position windows per step); then a merge walks the
// left zone [a+1, a+m] upward and the right zone [a+m+1, b-1] downward one window each:
// the k-th failing element of the left window pairs with the k-th passing element of the
// right window (lane order = descending positions there), the pair is swapped through
// registers (ds_bpermute), and each window moves past what it consumed.
// Returns m and t = #pairs.
template <class S> __device__ void w_exchange(const S& s, int a, int b, uint32_t pk, int eq, int* m_out, int* t_out) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lanes_below();
    auto predk = [&](uint32_t k) { return eq ? k <= pk : k < pk; };
    int m = 0;
    for (int base = a + 1; base < b; base += 256) {
        uint64_t mk[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = base + u * 64 + lane;
            mk[u] = __ballot(p < b && predk(K(s, p)));
        }
#pragma unroll
        for (int u = 0; u < 4; u++) m += __builtin_popcountll(mk[u]);
    }
    const int z = a + m;
    int lpos = a + 1, rpos = b - 1, t = 0;
    while (lpos <= z && rpos > z) {
        const int pl = lpos + lane, pr = rpos - lane;
        typename S::Elem vl = 0, vr = 0;
        bool fl = false, fr = false;
        if (pl <= z) { vl = s.ld(pl); fl = !predk(S::key(vl)); }
        if (pr > z) { vr = s.ld(pr); fr = predk(S::key(vr)); }
        const uint64_t ml = __ballot(fl), mr = __ballot(fr);
        const int nl = __builtin_popcountll(ml), nr = __builtin_popcountll(mr);
        const int cn = min(nl, nr);
        const int k = __builtin_popcountll(ml & below);
        const int src = (fl && k < cn) ? select_bit(mr, k) : lane;
        typename S::Elem vx;
        if constexpr (sizeof(typename S::Elem) == 8) {
            const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)vr, src, 64);
            const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)vr >> 32), src, 64);
            vx = (typename S::Elem)(((uint64_t)hi << 32) | lo);
        } else {
            vx = (typename S::Elem)__shfl((int)vr, src, 64);
        }
        if (fl && k < cn) {
            s.st(pl, vx);
            s.st(rpos - src, vl);
        }
        t += cn;
        lpos = nl == cn ? min(lpos + 64, z + 1) : lpos + select_bit(ml, cn);
        rpos = nr == cn ? max(rpos - 64, z) : rpos - select_bit(mr, cn);
        wfence();
    }
    *m_out = m;
    *t_out = t;
}

// pdqsort_func on one frame, to the end, by one wavefront.  The frames it defers live in
// a VGPR stack (lane j holds entry j): it continues with the smaller side and defers the
// larger, so the depth stays below log2(len) + 1.
template <class S> __device__ void w_sort(const S& s, int a, int b, int lf) {
    const int lane = threadIdx.x & 63;
    int sa = 0, sb = 0, slf = 0, sp = 0;
    int limit = lf & 255;
    bool wb = (lf >> 8) & 1, wp = (lf >> 9) & 1;
    for (;;) {
        const int len = b - a;
        bool done = false;
        if (len <= MAX_INSERTION) {
            if (len > 1) w_insertion(s, a, b);
            done = true;
        } else if (limit == 0) {
            if (lane == 0) heap_sort(s, a, b);
            wfence();
            done = true;
        } else {
            if (!wb) {
                if (lane == 0) break_patterns(s, a, b);
                wfence();
                limit--;
            }
            int hint;
            int pivot = w_choose_pivot(s, a, b, &hint);
            if (hint == HINT_DEC) {
                w_reverse(s, a, b);
                pivot = (b - 1) - (pivot - a);
                hint = HINT_INC;
            }
            if (wb && wp && hint == HINT_INC && w_partial_insertion(s, a, b)) {
                done = true;
            } else {
                int eq = 0;
                uint32_t pk = 0;
                if (lane == 0) {
                    eq = (a > 0 && !(K(s, a - 1) < K(s, pivot))) ? 1 : 0;
                    swp(s, a, pivot);
                    pk = K(s, a);
                }
                eq = rfl(eq);
                pk = (uint32_t)rfl((int)pk);
                wfence();
                int m, t;
                w_exchange(s, a, b, pk, eq, &m, &t);
                if (eq) {
                    a = a + m + 1;                  // partitionEqual: continue with [mid, b)
                    continue;
                }
                const int mid = a + m;
                if (lane == 0) swp(s, a, mid);
                wfence();
                const int ll = mid - a, rl = b - mid, thr = len / 8;
                int la, lb, lfp;
                if (ll < rl) {                      // Go recurses left (fresh), continues right
                    la = mid + 1; lb = b; lfp = lf_pack(limit, ll >= thr, t == 0);
                    b = mid;
                } else {                            // Go recurses right (fresh), continues left
                    la = a; lb = mid; lfp = lf_pack(limit, rl >= thr, t == 0);
                    a = mid + 1;
                }
                if (lb - la >= 2) {                 // defer the larger side with its continued state
                    if (lane == sp) { sa = la; sb = lb; slf = lfp; }
                    sp++;
                }
                wb = true;                          // the smaller side: a fresh pdqsort_func call
                wp = true;
                continue;
            }
        }
        if (done) {
            if (sp == 0) return;
            sp--;
            a = __builtin_amdgcn_readlane(sa, sp);
            b = __builtin_amdgcn_readlane(sb, sp);
            const int l2 = __builtin_amdgcn_readlane(slf, sp);
            limit = l2 & 255;
            wb = (l2 >> 8) & 1;
            wp = (l2 >> 9) & 1;
        }
    }
}

// ---------------------------------------------------------------------------------
// workgroup steps
// ---------------------------------------------------------------------------------
#ifndef CASIM_PDQ_T_SMALL
#define CASIM_PDQ_T_SMALL 2048
#endif
constexpr int T_SMALL = CASIM_PDQ_T_SMALL;   // frames up to this length wait for the wavefront phase

struct Ctl {
    Frame f[MAXF];
    int32_t op[MAXF];
    uint32_t pk[MAXF];
    int32_t m[MAXF], t[MAXF];
    int32_t pl[MAXF];          // slots of the frames that partition this step, in slot order
    int32_t fo[MAXF + 1];      // prefix of their interior lengths
    int32_t po[MAXF + 1];      // prefix of their pair counts
    int32_t piv[MAXF];         // chosen pivot position (step A1)
    uint8_t pis[MAXF];         // partialInsertionSort runs for the frame (A1 -> workgroup)
    uint64_t wsum[NW];
    uint32_t wflag[NW];
    int32_t nf, np, top, base, nsmall, snext;
    uint32_t rmax;
    int32_t x0, x1;            // workgroup partialInsertionSort: search results
    int32_t sx[3];             //   (LDS store: descent, left landing, right landing)
    uint64_t pe, pf;           //   the two elements it moves
};

// index k with fo[k] <= x < fo[k+1] (every listed frame has a non-empty interior)
__device__ inline int find_frame(const int32_t* fo, int np, int x) {
    int lo = 0, hi = np;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (fo[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

// exclusive prefix of n entries of v[] into o[], o[n] = total; one wave
__device__ inline void w_prefix(const int32_t* v, int32_t* o, int n) {
    const int lane = threadIdx.x & 63;
    int carry = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        const int x = i < n ? v[i] : 0;
        int incl = x;
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (i < n) o[i] = carry + incl - x;
        carry += __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) o[n] = carry;
}

// segmented exclusive scan over the workgroup's threads of (v, start flag): the sum of v
// back to (and including) the nearest earlier thread whose chunk holds a segment start
__device__ inline uint64_t wg_seg_scan(uint64_t v, bool flag, Ctl& c) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint64_t iv = v;
    bool iflag = flag;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t yv = __shfl_up(iv, d, 64);
        const bool yf = __shfl_up((int)iflag, d, 64) != 0;
        if (lane >= d && !iflag) { iv += yv; iflag = yf; }
    }
    if (lane == 63) { c.wsum[w] = iv; c.wflag[w] = iflag ? 1u : 0u; }
    __syncthreads();
    uint64_t pv = 0;                        // combine the waves before w
    for (int q = 0; q < w; q++) {
        if (c.wflag[q]) pv = c.wsum[q]; else pv += c.wsum[q];
    }
    uint64_t ev = __shfl_up(iv, 1, 64);
    bool ef = __shfl_up((int)iflag, 1, 64) != 0;
    if (lane == 0) { ev = 0; ef = false; }
    return ef ? ev : pv + ev;
}

// m[slot] += cnt with one atomic per wave when the wave's lanes all end in one frame
__device__ inline void add_count(Ctl& c, bool active, int slot, int cnt) {
    const int s0 = rfl(slot);
    if (__ballot(active && slot != s0) == 0) {
        int tot = active ? cnt : 0;
        for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d, 64);
        if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&c.m[s0], tot);
    } else if (active && cnt) {
        atomicAdd(&c.m[slot], cnt);
    }
}

// t[slot] += cnt, same aggregation
__device__ inline void add_count_t(Ctl& c, bool active, int slot, int cnt) {
    const int s0 = rfl(slot);
    if (__ballot(active && slot != s0) == 0) {
        int tot = active ? cnt : 0;
        for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d, 64);
        if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&c.t[s0], tot);
    } else if (active && cnt) {
        atomicAdd(&c.t[slot], cnt);
    }
}

// A partitioning frame seen from a thread's chunk: interior [s, e) = [a+1, b), zone
// boundary z = a + m, exchange offset c1, pair count t.
struct PFrame {
    int s, e, a, c1, z, t, slot;
    uint32_t pk;
    bool eq;
    __device__ void load(const Ctl& c, int k, bool counted) {
        if (k < 0 || k >= c.np) { s = e = INT_MAX; a = c1 = z = t = slot = 0; pk = 0; eq = false; return; }
        slot = c.pl[k];
        a = c.f[slot].a;
        s = a + 1;
        e = c.f[slot].b;
        c1 = (e - a) / 2;
        pk = c.pk[slot];
        eq = c.op[slot] == OP_EQ;
        z = counted ? a + c.m[slot] : 0;
        t = counted ? c.t[slot] : 0;
    }
    __device__ bool pred(uint32_t key) const { return eq ? key <= pk : key < pk; }
};

// One partition_func / partitionEqual_func step of every listed frame (c.pl, ordered by
// start).  Positional chunks: thread t owns positions [t*cs, t*cs + cs) of the group and
// walks them with the frame it is in (F) and the next one (G); positions outside every
// interior are skipped.  The loops are rolled: the code of a step stays small enough for
// the instruction cache (fully unrolled chunk loops thrashed it).
// Exchange inside an interior [a+1, b) of length L: the k-th left-zone element failing
// pred (from the left) leaves its value at xs[a+1+k], the j-th right-zone element passing
// it (from the left) at xs[a+1+c1+j], c1 = (L+1)/2 (t <= L/2 pairs fit); then the k-th
// left failure takes the value of the k-th right pass from the right, and vice versa.
// xs: the group's exchange scratch (global memory, one element per position).
template <class S> __device__ void wg_partition(const S& s, Ctl& c, typename S::Elem* __restrict__ xs, int n) {
    const int tid = threadIdx.x;
    const int np = c.np;
    const int cs = (n + NT - 1) / NT;
    const int p0 = min(tid * cs, n), p1 = min(p0 + cs, n);
    const bool cache = cs <= 64;                     // pred bits of the chunk in one register pair
    int k0;
    {
        int lo = 0, hi = np;                         // frames with start a <= p0
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (c.f[c.pl[mid]].a <= p0) lo = mid + 1; else hi = mid;
        }
        k0 = lo - 1;
    }
    uint64_t pm = 0;
    PFrame F, G;
    // P1: m per frame
    {
        int k = k0;
        F.load(c, k, false);
        G.load(c, k + 1, false);
        int cnt = 0;
        for (int p = p0; p < p1; p++) {
            if (p >= G.s) {
                if (cnt) atomicAdd(&c.m[F.slot], cnt);
                cnt = 0;
                k++;
                F = G;
                G.load(c, k + 1, false);
            }
            if (p >= F.s && p < F.e) {
                const bool pr = F.pred(S::key(s.ld(p)));
                cnt += pr ? 1 : 0;
                if (pr) pm |= 1ull << ((p - p0) & 63);
            }
        }
        add_count(c, p0 < p1 && k >= 0, F.slot, cnt);
    }
    __syncthreads();
    PDQ_T(t_p2);
    auto pred_at = [&](const PFrame& f, int p) -> bool {
        return cache ? ((pm >> (p - p0)) & 1ull) != 0 : f.pred(S::key(s.ld(p)));
    };
    // P2: segmented counts of left-zone failures (lm) / right-zone passes (rm)
    uint32_t lm = 0, rm = 0;
    bool start;
    {
        int k = k0;
        F.load(c, k, true);
        G.load(c, k + 1, true);
        start = F.s >= p0;
        for (int p = p0; p < p1; p++) {
            if (p >= G.s) { k++; F = G; G.load(c, k + 1, true); lm = rm = 0; start = true; }
            if (p >= F.s && p < F.e) {
                const bool pr = pred_at(F, p);
                if (p <= F.z) lm += pr ? 0u : 1u; else rm += pr ? 1u : 0u;
            }
        }
    }
    const uint64_t ex = wg_seg_scan(((uint64_t)rm << 32) | lm, start, c);
    {
        int k = k0;
        F.load(c, k, true);
        G.load(c, k + 1, true);
        lm = F.s < p0 ? (uint32_t)ex : 0u;
        rm = F.s < p0 ? (uint32_t)(ex >> 32) : 0u;
        for (int p = p0; p < p1; p++) {
            if (p >= G.s) { k++; F = G; G.load(c, k + 1, true); lm = rm = 0; }
            if (p >= F.s && p < F.e) {
                const bool pr = pred_at(F, p);
                if (p <= F.z) {
                    if (!pr) xs[F.s + lm++] = s.ld(p);
                } else if (pr) {
                    xs[F.s + F.c1 + rm++] = s.ld(p);
                }
                if (p == F.e - 1) c.t[F.slot] = (int32_t)lm;     // the frame's pair count
            }
        }
    }
    __syncthreads();
    PDQ_ADD(6, t_p2);
    PDQ_T(t_p3);
    // P3: every misplaced position takes its partner's value (each thread writes only its
    // own chunk, so the pred recomputation above reads unchanged positions)
    {
        int k = k0;
        F.load(c, k, true);
        G.load(c, k + 1, true);
        lm = F.s < p0 ? (uint32_t)ex : 0u;
        rm = F.s < p0 ? (uint32_t)(ex >> 32) : 0u;
        for (int p = p0; p < p1; p++) {
            if (p >= G.s) { k++; F = G; G.load(c, k + 1, true); lm = rm = 0; }
            if (p >= F.s && p < F.e) {
                const bool pr = pred_at(F, p);
                if (p <= F.z) {
                    if (!pr) { const int kk = (int)lm++; s.st(p, xs[F.s + F.c1 + F.t - 1 - kk]); }
                } else if (pr) {
                    const int kk = F.t - 1 - (int)rm++;
                    s.st(p, xs[F.s + kk]);
                }
            }
        }
    }
    __syncthreads();
    PDQ_ADD(7, t_p3);
}

// LDS store: thread t owns the 64 positions of word t.  Frames here are longer than
// T_SMALL, so a word meets at most two interiors (F, then G); membership, pred, zone,
// left-zone failures (LM) and right-zone passes (RM) are 64-bit masks, counts are
// popcounts.  The pairs are found, not listed: each thread swaps its LM elements with
// their partners, whose positions it selects from the RM bitmap (one word per thread in
// LDS) through the words' prefix counts — the RM with global index gR is bit
// gR - rmp[w] of the word w with rmp[w] <= gR < rmp[w+1].  Global indices are frame-
// ordered because frames are ordered by position: frame f's RMs are base_f .. base_f +
// t_f - 1 with base_f the pairs of the frames before it, and so are its LMs; the k-th LM
// from the left (global base_f + k) pairs with RM global base_f + t_f - 1 - k.
// 4-bit mask of the bytes of x below bound (0 <= bound <= 256), byte i -> bit i
__device__ inline uint32_t swar_lt4(uint32_t x, uint32_t bound) {
    if (bound >= 256) return 0xFu;
    const uint32_t b = bound * 0x01010101u;
    // per byte x < b: with the high bits split off no borrow crosses a byte, so
    // d = (x | H) - (b & ~H) has bit 7 set iff x_lo >= b_lo
    const uint32_t H = 0x80808080u;
    const uint32_t d = (x | H) - (b & ~H);
    const uint32_t lt = ((~x & b) | (~(x ^ b) & ~d)) & H;      // bit 7 of each byte
    const uint32_t m = lt >> 7;                                  // bits 0, 8, 16, 24
    // gather bits 0/8/16/24 into 0..3: m * (1 + 2^7 + 2^14 + 2^21) puts them at 21..24 and
    // no other product lands there (no carries)
    return ((m * 0x00204081u) >> 21) & 0xFu;
}

__device__ inline uint64_t range_bits(int lo, int hi) {     // bits [lo, hi) of a word, clamped to [0, 64)
    lo = max(lo, 0);
    hi = min(hi, 64);
    if (hi <= lo) return 0ull;
    const uint64_t up = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
    return up & ~((1ull << lo) - 1);
}

__device__ void wg_partition(const LdsStore& s, Ctl& c, uint32_t* __restrict__, int n) {
    const int tid = threadIdx.x, lane = tid & 63;
    PDQ_T(t_p1);
    const int np = c.np;
    const int W = (n + 63) >> 6;
    const bool act = tid < W;
    const int p0 = tid * 64;
    // F: the last partitioning frame starting at or before the word's last position; G: the one before it
    int kF = -1;
    {
        int lo = 0, hi = np;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (c.f[c.pl[mid]].a <= p0 + 63) lo = mid + 1; else hi = mid;
        }
        kF = lo - 1;
    }
    PFrame A, B;                   // B = frame kF (later positions), A = frame kF - 1 (earlier)
    A.load(c, kF - 1, false);
    B.load(c, kF, false);
    const uint64_t memA = act ? range_bits(A.s - p0, A.e - p0) : 0ull;
    const uint64_t memB = act ? range_bits(B.s - p0, B.e - p0) : 0ull;
    // P1: pred bits, four ranks per 32-bit compare (SWAR), m per frame
    uint64_t pm = 0;
    if (memA | memB) {
        // pred = key < bound with bound = pk (+1 for partitionEqual's key <= pk); bound 256
        // (key <= 255) is every key
        const uint32_t bA = A.pk + (A.eq ? 1u : 0u), bB = B.pk + (B.eq ? 1u : 0u);
        const uint4* r16 = reinterpret_cast<const uint4*>(s.rk + p0);
        uint64_t pa = 0, pb = 0;
        // one bound for a word inside one frame (the SWAR compares are the phase's VALU
        // cost); a word holding two frames' positions takes both
        const bool two = memA != 0 && memB != 0;
        const uint32_t b1 = memA ? bA : bB;
        // quarter q = q0 + lane/4 (mod 4): the 16-byte reads of an LDS lane group then
        // cover distinct banks (lanes are 64 bytes apart)
#pragma unroll
        for (int q0 = 0; q0 < 4; q0++) {
            const int q = (q0 + (lane >> 2)) & 3;
            const uint4 x = r16[q];
            const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const int j = q * 16 + h * 4;
                pa |= (uint64_t)swar_lt4(wv[h], b1) << j;
                if (two) pb |= (uint64_t)swar_lt4(wv[h], bB) << j;
            }
        }
        pm = two ? (pa & memA) | (pb & memB) : pa & (memA | memB);
    }
    add_count(c, memA != 0, A.slot, __builtin_popcountll(pm & memA));
    add_count(c, memB != 0, B.slot, __builtin_popcountll(pm & memB));
    __syncthreads();
    PDQ_T(t_p2);
    PDQ_S(6, t_p2 - t_p1);
    // P2: zones, LM / RM masks, RM bitmap, pair counts, prefix counts
    A.z = A.a + (memA ? c.m[A.slot] : 0);
    B.z = B.a + (memB ? c.m[B.slot] : 0);
    const uint64_t leftA = range_bits(A.s - p0, A.z + 1 - p0), leftB = range_bits(B.s - p0, B.z + 1 - p0);
    const uint64_t lmA = ~pm & memA & leftA, lmB = ~pm & memB & leftB;
    const uint64_t rmask = (pm & memA & ~leftA) | (pm & memB & ~leftB);
    const uint64_t lmask = lmA | lmB;
    if (act) s.rmb[tid] = lmask | rmask;
    add_count_t(c, lmA != 0, A.slot, __builtin_popcountll(lmA));
    add_count_t(c, lmB != 0, B.slot, __builtin_popcountll(lmB));
    // exclusive block scan of (LM << 16 | RM) per word (counts < 2^16: n <= PDQ_LDS_N)
    uint32_t incl = ((uint32_t)__builtin_popcountll(lmask) << 16) | (uint32_t)__builtin_popcountll(rmask);
    const uint32_t own = incl;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) c.wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t pre = incl - own;
    for (int q = 0; q < (tid >> 6); q++) pre += (uint32_t)c.wsum[q];
    // combined (LM + RM) prefix per word: n <= PDQ_LDS_N < 2^16
    if (act) s.rmp[tid] = (uint16_t)((pre >> 16) + (pre & 0xFFFFu));
    if (tid == W - 1) s.rmp[W] = (uint16_t)(((pre + own) >> 16) + ((pre + own) & 0xFFFFu));
    if (tid < 64) {
        // pair base of every frame in position order (c.t holds the pair counts; t[] of
        // the frames is read again in P3)
        for (int i = lane; i < np; i += 64) c.po[i] = c.t[c.pl[i]];
        w_prefix(c.po, c.fo, np);           // fo[k] = base of frame k (position order)
    }
    __syncthreads();
    PDQ_ADD(6, t_p2);
    PDQ_T(t_p3);
    PDQ_S(7, t_p3 - t_p2);
    // P3: the pairs, split evenly over the workgroup's threads in runs of consecutive
    // global pair indices.  In combined (LM | RM) order frame f (pair base fs, end fe)
    // holds its LMs at [2fs, fs+fe) and its RMs at [fs+fe, 2fe): pair k of the frame joins
    // combined bits fs + k and 2fe - 1 - k + fs.  A run locates both ends once (binary
    // search of the combined prefix counts), then walks the bitmap, forwards on the left,
    // backwards on the right; four pairs per iteration (all loads, then all stores).
    {
        const int P = c.fo[np];
        const int per = (P + NT - 1) / NT;
        int k = tid * per;
        const int k1 = min(P, k + per);
        auto locate = [&](int ci, int& ww, int& bit, uint64_t& wb) {
            int lo = 0, hi = W;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if ((int)s.rmp[mid] <= ci) lo = mid; else hi = mid;
            }
            ww = lo;
            wb = s.rmb[ww];
            bit = select_bit(wb, ci - (int)s.rmp[ww]);
        };
        auto next_l = [&](int& ww, int& bit, uint64_t& wb) {
            uint64_t m = bit < 63 ? wb & (~0ull << (bit + 1)) : 0ull;
            while (!m) { wb = s.rmb[++ww]; m = wb; }
            bit = __builtin_ctzll(m);
        };
        auto prev_r = [&](int& ww, int& bit, uint64_t& wb) {
            uint64_t m = wb & ((1ull << bit) - 1);
            while (!m) { wb = s.rmb[--ww]; m = wb; }
            bit = 63 - __builtin_clzll(m);
        };
        while (k < k1) {
            int lo = 0, hi = np;                     // frame of pair k: the last f with fo[f] <= k
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (c.fo[mid] <= k) lo = mid; else hi = mid;
            }
            const int fs = c.fo[lo], fe = c.fo[lo + 1];
            const int kend = min(k1, fe);
            int wl, bl, wr, br;
            uint64_t wbl, wbr;
            locate(fs + k, wl, bl, wbl);
            locate(2 * fe - 1 - k + fs, wr, br, wbr);
            for (;;) {
                int pp[4], qq[4];
                const int cnt = min(4, kend - k);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (u >= cnt) { pp[u] = qq[u] = 0; continue; }
                    if (u > 0) { next_l(wl, bl, wbl); prev_r(wr, br, wbr); }
                    pp[u] = wl * 64 + bl;
                    qq[u] = wr * 64 + br;
                }
                uint32_t vp[4], vq[4];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (u < cnt) { vp[u] = s.ld(pp[u]); vq[u] = s.ld(qq[u]); }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (u < cnt) { s.st(pp[u], vq[u]); s.st(qq[u], vp[u]); }
                k += cnt;
                if (k >= kend) break;
                next_l(wl, bl, wbl);
                prev_r(wr, br, wbr);
            }
        }
    }
    __syncthreads();
    PDQ_ADD(7, t_p3);
    PDQ_S(8, clock64() - t_p3);
}

// partialInsertionSort_func on a frame longer than T_SMALL, by the whole workgroup: the
// descent search and the two landing searches are parallel min / max reductions, the two
// bubbling loops are block moves (read, barrier, write).  One wavefront alone spent
// ~10^5 cycles per call where a frame held a long run of one key (every step moved the
// run by one place).
template <class S> __device__ void wg_shift(const S& s, Ctl& c, int lo, int hi, int dir) {
    // [lo, hi] moves one place (dir +1: right, processed top-down; -1: left, bottom-up),
    // NT * PER positions per round
    constexpr int PER = 8;
    const int tid = threadIdx.x;
    const int len = hi - lo + 1;
    for (int done = 0; done < len; done += NT * PER) {
        typename S::Elem v[PER];
        const int base = dir > 0 ? hi - done : lo + done;      // first position of this round
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int off = u * NT + tid;
            const int p = dir > 0 ? base - off : base + off;
            v[u] = off < len - done ? s.ld(p) : 0;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int off = u * NT + tid;
            const int p = dir > 0 ? base - off : base + off;
            if (off < len - done) s.st(p + dir, v[u]);
        }
        __syncthreads();
    }
}

// LDS store: the same block move on 32-bit words of each array (two positions per word
// of e, four of rk), the one-element offset taken from the neighbouring word
template <int EB> __device__ void shift_words(uint32_t* __restrict__ w32, int dlo, int dhi, int dir) {
    constexpr int EPW = 32 / EB, PER = 8;
    const int tid = threadIdx.x;
    const int w0 = dlo / EPW, w1 = dhi / EPW, nw = w1 - w0 + 1;
    for (int done = 0; done < nw; done += NT * PER) {
        uint32_t nv[PER];
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int off = u * NT + tid;
            nv[u] = 0;
            if (off < nw - done) {
                const int w = dir > 0 ? w1 - done - off : w0 + done + off;
                const uint32_t cur = w32[w];
                const uint32_t nb = dir > 0 ? (w > 0 ? w32[w - 1] : 0u) : w32[w + 1];
                const uint32_t sh = dir > 0 ? (cur << EB) | (nb >> (32 - EB)) : (cur >> EB) | (nb << (32 - EB));
                const int e0 = max(dlo, w * EPW) - w * EPW, e1 = min(dhi, w * EPW + EPW - 1) - w * EPW;
                const uint32_t hi_m = e1 + 1 >= EPW ? ~0u : ((1u << ((e1 + 1) * EB)) - 1);
                const uint32_t m = hi_m & ~((1u << (e0 * EB)) - 1);
                nv[u] = (sh & m) | (cur & ~m);
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int off = u * NT + tid;
            if (off < nw - done) w32[dir > 0 ? w1 - done - off : w0 + done + off] = nv[u];
        }
        __syncthreads();
    }
}

__device__ void wg_shift(const LdsStore& s, Ctl&, int lo, int hi, int dir) {
    shift_words<16>(reinterpret_cast<uint32_t*>(s.e), lo + dir, hi + dir, dir);
    shift_words<8>(reinterpret_cast<uint32_t*>(s.rk), lo + dir, hi + dir, dir);
}

// Workgroup searches of partialInsertionSort, outward from the start in windows (one
// barrier per window): the first descent in [i, b), the last q in [lo, top] with key <=
// kmax, the first j in [bot, b) with key >= kmin.  Generic: one position per thread per
// window; LDS store: four per thread (32-bit rank words, SWAR byte compares).
template <class S> __device__ int wg_find_descent(const S& s, Ctl& c, int i, int b) {
    const int tid = threadIdx.x;
    if (tid == 0) c.x0 = b;
    __syncthreads();
    for (int q0 = i; q0 < b; q0 += NT) {
        const int q = q0 + tid;
        const bool d = q < b && K(s, q) < K(s, q - 1);
        if (d) atomicMin(&c.x0, q);
        if (__syncthreads_or(d)) break;
    }
    const int r = c.x0;
    __syncthreads();
    return r;
}
template <class S> __device__ int wg_find_left(const S& s, Ctl& c, int lo, int top, uint32_t kmax) {
    const int tid = threadIdx.x;
    if (tid == 0) c.x0 = -1;
    __syncthreads();
    for (int t0 = top; t0 >= lo; t0 -= NT) {
        const int q = t0 - tid;
        const bool d = q >= lo && K(s, q) <= kmax;
        if (d) atomicMax(&c.x0, q);
        if (__syncthreads_or(d)) break;
    }
    const int r = c.x0;
    __syncthreads();
    return r;
}
template <class S> __device__ int wg_find_right(const S& s, Ctl& c, int bot, int b, uint32_t kmin) {
    const int tid = threadIdx.x;
    if (tid == 0) c.x0 = b;
    __syncthreads();
    for (int b0 = bot; b0 < b; b0 += NT) {
        const int j = b0 + tid;
        const bool d = j < b && K(s, j) >= kmin;
        if (d) atomicMin(&c.x0, j);
        if (__syncthreads_or(d)) break;
    }
    const int r = c.x0;
    __syncthreads();
    return r;
}

// bytes of x below the bytes of y, byte i -> bit i
__device__ inline uint32_t swar_ltv4(uint32_t x, uint32_t y) {
    const uint32_t H = 0x80808080u;
    const uint32_t d = (x | H) - (y & ~H);
    const uint32_t lt = ((~x & y) | (~(x ^ y) & ~d)) & H;
    const uint32_t m = lt >> 7;
    return ((m * 0x00204081u) >> 21) & 0xFu;                   // (see swar_lt4)
}
__device__ inline uint32_t nib_range(int w, int lo, int hi) {     // bits of positions [lo, hi] in word w
    const int e0 = max(lo - 4 * w, 0), e1 = min(hi - 4 * w, 3);
    if (e1 < e0) return 0u;
    return ((2u << e1) - 1) & ~((1u << e0) - 1);
}

__device__ int wg_find_descent(const LdsStore& s, Ctl& c, int i, int b) {
    const int tid = threadIdx.x;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(s.rk);
    if (tid == 0) c.x0 = b;
    __syncthreads();
    for (int w0 = i >> 2; 4 * w0 < b; w0 += NT) {
        const int w = w0 + tid;
        int q = INT_MAX;
        if (4 * w < b) {
            const uint32_t x = r32[w];
            const uint32_t y = (x << 8) | (w > 0 ? r32[w - 1] >> 24 : 0u);      // rk[q - 1]
            const uint32_t m = swar_ltv4(x, y) & nib_range(w, i, b - 1);
            if (m) q = 4 * w + __builtin_ctz(m);
        }
        if (q != INT_MAX) atomicMin(&c.x0, q);
        if (__syncthreads_or(q != INT_MAX)) break;
    }
    const int r = c.x0;
    __syncthreads();
    return r;
}
__device__ int wg_find_left(const LdsStore& s, Ctl& c, int lo, int top, uint32_t kmax) {
    const int tid = threadIdx.x;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(s.rk);
    if (tid == 0) c.x0 = -1;
    __syncthreads();
    for (int w0 = top >> 2; 4 * w0 + 3 >= lo; w0 -= NT) {
        const int w = w0 - tid;
        int q = -1;
        if (w >= 0 && 4 * w + 3 >= lo) {
            const uint32_t m = swar_lt4(r32[w], kmax + 1) & nib_range(w, lo, top);
            if (m) q = 4 * w + 31 - __builtin_clz(m);
        }
        if (q >= 0) atomicMax(&c.x0, q);
        if (__syncthreads_or(q >= 0)) break;
    }
    const int r = c.x0;
    __syncthreads();
    return r;
}
__device__ int wg_find_right(const LdsStore& s, Ctl& c, int bot, int b, uint32_t kmin) {
    const int tid = threadIdx.x;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(s.rk);
    if (tid == 0) c.x0 = b;
    __syncthreads();
    for (int w0 = bot >> 2; 4 * w0 < b; w0 += NT) {
        const int w = w0 + tid;
        int j = INT_MAX;
        if (4 * w < b) {
            const uint32_t m = ~swar_lt4(r32[w], kmin) & nib_range(w, bot, b - 1);
            if (m) j = 4 * w + __builtin_ctz(m);
        }
        if (j != INT_MAX) atomicMin(&c.x0, j);
        if (__syncthreads_or(j != INT_MAX)) break;
    }
    const int r = c.x0;
    __syncthreads();
    return r;
}

template <class S> __device__ bool wg_partial_insertion(const S& s, Ctl& c, int a, int b) {
    constexpr int maxSteps = 5, shortestShifting = 50;
    const int tid = threadIdx.x;
    int i = a + 1;
    for (int step = 0; step < maxSteps; step++) {
        PDQ_T(t_d0);
        i = wg_find_descent(s, c, i, b);
        PDQ_ADD(21, t_d0);
        PDQ_CNT(26, 1);               // first i' in [i, b) with less(i', i'-1)
        if (i == b) return true;
        if (b - a < shortestShifting) return false;
        if (tid == 0) {
            swp(s, i, i - 1);
            c.pe = (uint64_t)s.ld(i - 1);          // the smaller one, bubbling left
            c.pf = (uint64_t)s.ld(i);              // the greater one, bubbling right
        }
        __syncthreads();
        const typename S::Elem e = (typename S::Elem)c.pe, f = (typename S::Elem)c.pf;
        const bool left = i - a >= 2, right = b - i >= 2;
        const int qmin = a > 0 ? a - 1 : 0;        // key(a-1) <= every key of [a, b): the walk stops there
        // left: the last q in [qmin, i-2] with key(q) <= key(e); right: the first j in
        // [i+1, b) with !(key(j) < key(f))
        PDQ_T(t_s0);
        const int landL = left ? wg_find_left(s, c, qmin, i - 2, S::key(e)) + 1 : i - 1;   // (none: qmin == 0 -> 0)
        const int landR = right ? wg_find_right(s, c, i + 1, b, S::key(f)) - 1 : i;
        PDQ_ADD(22, t_s0);
        PDQ_T(t_h0);
        if (left && landL < i - 1) {
            wg_shift(s, c, landL, i - 2, +1);
            if (tid == 0) s.st(landL, e);
        }
        if (right && landR > i) {
            wg_shift(s, c, i + 1, landR, -1);
            if (tid == 0) s.st(landR, f);
        }
        __threadfence_block();
        __syncthreads();
        PDQ_ADD(23, t_h0);
        PDQ_CNT(24, (uint64_t)max(i - 1 - landL, 0) + (uint64_t)max(landR - i, 0));
        PDQ_CNT(25, (uint64_t)(b - a));
    }
    return false;
}

// The previous step of the same call (pis_hint): when the descent is found at the same i
// and the moved element's rank repeats, its landing follows from the previous step without
// a search — ranks repeat a lot (C2: 64 distinct over 50k pods).  Left: the previous step
// left e (rank ev) at L and every element it passed, now (L, i-1], above ev; so with the
// same ev the last q <= i-2 with rank <= ev is L.  Right: the previous f (rank fv) sits at
// R and the elements it passed, now [i, R-1], are below fv; so with the same fv the first
// j >= i+1 with rank >= fv is R.
struct PisHint {
    int i = -1, L = 0, R = 0;
    uint32_t ev = 0, fv = 0;
};
// LDS store: one step is a descent search, the two landing searches and one rewrite of
// [landL, landR] — swap(i, i-1) and the two bubbling loops together are the rotation
//   new[landL] = old[i], new[p] = old[p-1] on (landL, i-1], new[p] = old[p+1] on [i, landR),
//   new[landR] = old[i-1]
// done on whole words (quads of positions: two 16-bit words of e, one 8-bit word of rk).
// Searches reduce per wavefront first (lanes cover ascending or descending words, so the
// first hit lane holds the wave's extreme) and publish one LDS atomic per wave into a
// slot set before the barrier that precedes its use; a step has no barrier beyond one per
// search window and two per rewrite round.
template <int EB> __device__ inline uint32_t slot_mask(int p0, int lo, int hi) {
    constexpr int EPW = 32 / EB;
    const int e0 = max(lo - p0, 0), e1 = min(hi - p0, EPW - 1);
    if (e1 < e0) return 0u;
    const uint32_t up = (e1 + 1) * EB >= 32 ? ~0u : ((1u << ((e1 + 1) * EB)) - 1);
    return up & ~((1u << (e0 * EB)) - 1);
}
template <int EB> __device__ inline uint32_t rotate_word(uint32_t cur, uint32_t prv, uint32_t nxt, int p0,
                                                        int L, int i, int R, uint32_t ev, uint32_t fv) {
    const uint32_t shl = (cur << EB) | (prv >> (32 - EB));      // old[p - 1]
    const uint32_t shr = (cur >> EB) | (nxt << (32 - EB));      // old[p + 1]
    const uint32_t mE = slot_mask<EB>(p0, L, L), mF = slot_mask<EB>(p0, R, R);
    const uint32_t mL = slot_mask<EB>(p0, L + 1, i - 1), mR = slot_mask<EB>(p0, i, R - 1);
    const uint32_t rep = EB == 8 ? 0x01010101u : 0x00010001u;
    return (cur & ~(mE | mF | mL | mR)) | (shl & mL) | (shr & mR) | ((ev * rep) & mE) | ((fv * rep) & mF);
}

__device__ bool wg_partial_insertion(const LdsStore& s, Ctl& c, int a, int b) {
    constexpr int maxSteps = 5, shortestShifting = 50;
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(s.rk);
    uint32_t* w32 = reinterpret_cast<uint32_t*>(s.rk);
    uint32_t* e32 = reinterpret_cast<uint32_t*>(s.e);
    if (tid == 0) { c.sx[0] = b; c.sx[1] = -1; c.sx[2] = b; }
    __syncthreads();
    int i = a + 1;
    PisHint hint;                          // (uniform: see w_pis_find)
    for (int step = 0; step < maxSteps; step++) {
        PDQ_T(t_d0);
        for (int w0 = i >> 2; 4 * w0 < b; w0 += NT) {          // first descent in [i, b)
            const int w = w0 + tid;
            bool hit = false;
            int q = 0;
            if (4 * w < b) {
                const uint32_t x = r32[w];
                const uint32_t y = (x << 8) | (w > 0 ? r32[w - 1] >> 24 : 0u);
                const uint32_t m = swar_ltv4(x, y) & nib_range(w, i, b - 1);
                hit = m != 0;
                q = 4 * w + __builtin_ctz(m | 16u);
            }
            const uint64_t bal = __ballot(hit);
            if (bal && lane == __builtin_ctzll(bal)) atomicMin(&c.sx[0], q);
            __syncthreads();
            if (c.sx[0] < 4 * (w0 + NT)) break;     // (a later window's hits lie beyond it)
        }
        i = c.sx[0];
        PDQ_ADD(21, t_d0);
        PDQ_CNT(26, 1);
        if (i == b) return true;
        if (b - a < shortestShifting) return false;
        PDQ_T(t_s0);
        const uint32_t ev = s.rk[i], fv = s.rk[i - 1];            // the smaller one bubbles left, the greater right
        const uint32_t ee = s.e[i], fe = s.e[i - 1];
        int landL = i - 1, landR = i;
        const bool same = hint.i == i;
        if (i - a >= 2 && same && ev == hint.ev && hint.L <= i - 2) {
            landL = hint.L + 1;
        } else if (i - a >= 2) {           // the last q in [qmin, i-2] with rk[q] <= ev, plus one
            const int lo = a > 0 ? a - 1 : 0, top = i - 2;
            for (int w0 = top >> 2; 4 * w0 + 3 >= lo; w0 -= NT) {
                const int w = w0 - tid;
                bool hit = false;
                int q = 0;
                if (w >= 0 && 4 * w + 3 >= lo) {
                    const uint32_t m = swar_lt4(r32[w], ev + 1) & nib_range(w, lo, top);
                    hit = m != 0;
                    q = 4 * w + 31 - __builtin_clz(m | 1u);
                }
                const uint64_t bal = __ballot(hit);
                if (bal && lane == __builtin_ctzll(bal)) atomicMax(&c.sx[1], q);
                __syncthreads();
                if (c.sx[1] >= 4 * (w0 - NT + 1)) break;
            }
            landL = c.sx[1] + 1;           // (none found: qmin == 0 and landL = 0)
        }
        if (b - i >= 2 && same && fv == hint.fv && hint.R > i) {
            landR = hint.R - 1;
        } else if (b - i >= 2) {           // the first j in [i+1, b) with rk[j] >= fv, minus one
            for (int w0 = (i + 1) >> 2; 4 * w0 < b; w0 += NT) {
                const int w = w0 + tid;
                bool hit = false;
                int q = 0;
                if (4 * w < b) {
                    const uint32_t m = ~swar_lt4(r32[w], fv) & nib_range(w, i + 1, b - 1);
                    hit = m != 0;
                    q = 4 * w + __builtin_ctz(m | 16u);
                }
                const uint64_t bal = __ballot(hit);
                if (bal && lane == __builtin_ctzll(bal)) atomicMin(&c.sx[2], q);
                __syncthreads();
                if (c.sx[2] < 4 * (w0 + NT)) break;
            }
            landR = c.sx[2] - 1;
        }
        hint.i = i; hint.L = landL; hint.R = landR; hint.ev = ev; hint.fv = fv;
        PDQ_ADD(22, t_s0);
        PDQ_T(t_h0);
        // rewrite [landL, landR] by quads: the quads strictly between qL and qc shift right by
        // one, those strictly between qc and qR left (two shifts and an or per word); the (at
        // most three) quads holding landL, i-1 and landR take the general masked rotation —
        // computed by threads 0-2 before any word changes, stored after every interior quad.
        // Interior rounds run outward from the centre and read only words no earlier round
        // wrote.
        const int qL = landL >> 2, qc = (i - 1) >> 2, qR = landR >> 2;
        uint32_t bnv[3] = {0u, 0u, 0u};
        int bv = -1;
        if (tid < 3) {
            const int v = tid == 0 ? qL : tid == 1 ? qc : qR;
            const bool dup = (tid == 1 && qc == qL) || (tid == 2 && (qR == qc || qR == qL));
            if (!dup) {
                const int p0 = 4 * v;
                const uint32_t lo = e32[2 * v], hi = e32[2 * v + 1];
                const uint32_t pe = v > 0 ? e32[2 * v - 1] : 0u;
                const bool up = p0 + 4 <= landR;
                const uint32_t ne = up ? e32[2 * v + 2] : 0u;
                const uint32_t cr = w32[v];
                const uint32_t pr = v > 0 ? w32[v - 1] : 0u, nr8 = up ? w32[v + 1] : 0u;
                bnv[0] = rotate_word<16>(lo, pe, hi, p0, landL, i, landR, ee, fe);
                bnv[1] = rotate_word<16>(hi, lo, ne, p0 + 2, landL, i, landR, ee, fe);
                bnv[2] = rotate_word<8>(cr, pr, nr8, p0, landL, i, landR, ev, fv);
                bv = v;
            }
        }
        const int nli = max(qc - qL - 1, 0), nri = max(qR - qc - 1, 0);
        for (int done = 0; done < max(nli, nri); done += NT) {
            const int k = done + tid;
            const bool okL = k < nli, okR = k < nri;
            const int vl = qc - 1 - k, vr = qc + 1 + k;
            uint32_t l0 = 0, l1 = 0, l2 = 0, r0 = 0, r1 = 0, r2 = 0;
            if (okL) {                    // new[p] = old[p - 1]
                const uint32_t lo = e32[2 * vl], hi = e32[2 * vl + 1], pe = e32[2 * vl - 1];
                const uint32_t cr = w32[vl], pr = w32[vl - 1];
                l0 = (lo << 16) | (pe >> 16);
                l1 = (hi << 16) | (lo >> 16);
                l2 = (cr << 8) | (pr >> 24);
            }
            if (okR) {                    // new[p] = old[p + 1]
                const uint32_t lo = e32[2 * vr], hi = e32[2 * vr + 1], ne = e32[2 * vr + 2];
                const uint32_t cr = w32[vr], nr8 = w32[vr + 1];
                r0 = (lo >> 16) | (hi << 16);
                r1 = (hi >> 16) | (ne << 16);
                r2 = (cr >> 8) | (nr8 << 24);
            }
            __syncthreads();
            if (okL) { e32[2 * vl] = l0; e32[2 * vl + 1] = l1; w32[vl] = l2; }
            if (okR) { e32[2 * vr] = r0; e32[2 * vr + 1] = r1; w32[vr] = r2; }
            __syncthreads();
        }
        if (bv >= 0) { e32[2 * bv] = bnv[0]; e32[2 * bv + 1] = bnv[1]; w32[bv] = bnv[2]; }
        __syncthreads();                  // (every thread has read this step's search slots)
        if (tid == 0) { c.sx[0] = b; c.sx[1] = -1; c.sx[2] = b; }   // the next step's slots
        __syncthreads();
        PDQ_ADD(23, t_h0);
        PDQ_CNT(24, (uint64_t)(i - 1 - landL) + (uint64_t)(landR - i));
        PDQ_CNT(25, (uint64_t)(b - a));
    }
    return false;
}

// The same on the LDS store by one wavefront (frames run it side by side in step A; the
// frames are disjoint and position a-1 is a placed pivot): ballots in place of the
// workgroup reductions, and no barrier — a wavefront's LDS accesses are in program order.
// w_pis_find: one step's searches — the first descent i in [i0, b) (b: the rest is
// sorted) and, when the step shifts (i < b, b - a >= 50), the landing places of the two
// bubbling loops.
__device__ void w_pis_find(const LdsStore& s, int a, int b, int i0, int& i_out, int& landL, int& landR,
                           PisHint* hint = nullptr) {
    constexpr int shortestShifting = 50;
    const int lane = threadIdx.x & 63;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(s.rk);
    PDQ_T(t_f0);
    [[maybe_unused]] int trips = 0;
    int i = i0;
    {
        int found = b;
        for (int w0 = i >> 2; 4 * w0 < b; w0 += 64) {           // first descent in [i, b)
            trips++;
            const int w = w0 + lane;
            int q = INT_MAX;
            if (4 * w < b) {
                const uint32_t x = r32[w];
                const uint32_t y = (x << 8) | (w > 0 ? r32[w - 1] >> 24 : 0u);
                const uint32_t m = swar_ltv4(x, y) & nib_range(w, i, b - 1);
                if (m) q = 4 * w + __builtin_ctz(m);
            }
            const uint64_t bal = __ballot(q != INT_MAX);
            if (bal) { found = __builtin_amdgcn_readlane(q, __builtin_ctzll(bal)); break; }
        }
        i = found;
    }
    i_out = i;
    landL = i - 1;
    landR = i;
    if (i == b || b - a < shortestShifting) { PDQ_PIS(0, clock64() - t_f0); PDQ_PIS(2, trips); return; }
    const uint32_t ev = s.rk[i], fv = s.rk[i - 1];
    const bool same = hint && hint->i == i;
    if (i - a >= 2 && same && ev == hint->ev && hint->L <= i - 2) {
        landL = hint->L + 1;
    } else if (i - a >= 2) {
        const int lo = a > 0 ? a - 1 : 0, top = i - 2;
        int q0 = -1;
        for (int w0 = top >> 2; 4 * w0 + 3 >= lo; w0 -= 64) {
            trips++;
            const int w = w0 - lane;
            int q = -1;
            if (w >= 0 && 4 * w + 3 >= lo) {
                const uint32_t m = swar_lt4(r32[w], ev + 1) & nib_range(w, lo, top);
                if (m) q = 4 * w + 31 - __builtin_clz(m);
            }
            const uint64_t bal = __ballot(q >= 0);
            if (bal) { q0 = __builtin_amdgcn_readlane(q, __builtin_ctzll(bal)); break; }
        }
        landL = q0 + 1;
    }
    if (b - i >= 2 && same && fv == hint->fv && hint->R > i) {
        landR = hint->R - 1;
    } else if (b - i >= 2) {
        int j0 = b;
        for (int w0 = (i + 1) >> 2; 4 * w0 < b; w0 += 64) {
            trips++;
            const int w = w0 + lane;
            int j = INT_MAX;
            if (4 * w < b) {
                const uint32_t m = ~swar_lt4(r32[w], fv) & nib_range(w, i + 1, b - 1);
                if (m) j = 4 * w + __builtin_ctz(m);
            }
            const uint64_t bal = __ballot(j != INT_MAX);
            if (bal) { j0 = __builtin_amdgcn_readlane(j, __builtin_ctzll(bal)); break; }
        }
        landR = j0 - 1;
    }
    if (hint) { hint->i = i; hint->L = landL; hint->R = landR; hint->ev = ev; hint->fv = fv; }
    PDQ_PIS(0, clock64() - t_f0);
    PDQ_PIS(2, trips);
}

// pi >= 0: the first step's searches were done already (w_pis_find from a + 1: pi, pL, pR)
__device__ bool w_partial_insertion(const LdsStore& s, int a, int b, int pi = -1, int pL = 0, int pR = 0) {
    constexpr int maxSteps = 5, shortestShifting = 50;
    const int lane = threadIdx.x & 63;
    uint32_t* w32 = reinterpret_cast<uint32_t*>(s.rk);
    uint32_t* e32 = reinterpret_cast<uint32_t*>(s.e);
    int i = a + 1;
    PDQ_PIS(5, 1);
    PisHint hint;
    for (int step = 0; step < maxSteps; step++) {
        int landL, landR;
        if (step == 0 && pi >= 0) {
            i = pi; landL = pL; landR = pR;
            if (i < b) { hint.i = i; hint.L = landL; hint.R = landR; hint.ev = s.rk[i]; hint.fv = s.rk[i - 1]; }
        } else {
            w_pis_find(s, a, b, i, i, landL, landR, &hint);
        }
        if (i == b) return true;
        if (b - a < shortestShifting) return false;
        const uint32_t ev = s.rk[i], fv = s.rk[i - 1];
        const uint32_t ee = s.e[i], fe = s.e[i - 1];
        const int qL = landL >> 2, qc = (i - 1) >> 2, qR = landR >> 2;
        PDQ_T(t_r0);
        PDQ_PIS(4, 1);
        // The quads strictly between qL and qc only shift right by one (new[p] = old[p-1]),
        // those strictly between qc and qR only left (new[p] = old[p+1]): two shifts and an
        // or per word.  The (at most three) quads holding landL, i-1 and landR take the
        // general masked rotation: computed by lanes 0-2 before any word changes, stored
        // after every interior quad.
        uint32_t bnv[3] = {0u, 0u, 0u};
        int bv = -1;
        if (lane < 3) {
            const int v = lane == 0 ? qL : lane == 1 ? qc : qR;
            const bool dup = (lane == 1 && qc == qL) || (lane == 2 && (qR == qc || qR == qL));
            if (!dup) {
                const int p0 = 4 * v;
                const uint32_t lo = e32[2 * v], hi = e32[2 * v + 1];
                const uint32_t pe = v > 0 ? e32[2 * v - 1] : 0u;
                const bool up = p0 + 4 <= landR;
                const uint32_t ne = up ? e32[2 * v + 2] : 0u;
                const uint32_t cr = w32[v];
                const uint32_t pr = v > 0 ? w32[v - 1] : 0u, nr8 = up ? w32[v + 1] : 0u;
                bnv[0] = rotate_word<16>(lo, pe, hi, p0, landL, i, landR, ee, fe);
                bnv[1] = rotate_word<16>(hi, lo, ne, p0 + 2, landL, i, landR, ee, fe);
                bnv[2] = rotate_word<8>(cr, pr, nr8, p0, landL, i, landR, ev, fv);
                bv = v;
            }
        }
        const int nli = max(qc - qL - 1, 0), nri = max(qR - qc - 1, 0);
        PDQ_PIS(3, (max(nli, nri) + 63) / 64);
        PDQ_PIS(6, nli + nri);
        for (int done = 0; done < max(nli, nri); done += 64) {
            const int k = done + lane;
            const bool okL = k < nli, okR = k < nri;
            const int vl = qc - 1 - k, vr = qc + 1 + k;
            uint32_t l0 = 0, l1 = 0, l2 = 0, r0 = 0, r1 = 0, r2 = 0;
            if (okL) {                    // new[p] = old[p - 1]
                const uint32_t lo = e32[2 * vl], hi = e32[2 * vl + 1], pe = e32[2 * vl - 1];
                const uint32_t cr = w32[vl], pr = w32[vl - 1];
                l0 = (lo << 16) | (pe >> 16);
                l1 = (hi << 16) | (lo >> 16);
                l2 = (cr << 8) | (pr >> 24);
            }
            if (okR) {                    // new[p] = old[p + 1]
                const uint32_t lo = e32[2 * vr], hi = e32[2 * vr + 1], ne = e32[2 * vr + 2];
                const uint32_t cr = w32[vr], nr8 = w32[vr + 1];
                r0 = (lo >> 16) | (hi << 16);
                r1 = (hi >> 16) | (ne << 16);
                r2 = (cr >> 8) | (nr8 << 24);
            }
            wfence();
            if (okL) { e32[2 * vl] = l0; e32[2 * vl + 1] = l1; w32[vl] = l2; }
            if (okR) { e32[2 * vr] = r0; e32[2 * vr + 1] = r1; w32[vr] = r2; }
            wfence();
        }
        if (bv >= 0) { e32[2 * bv] = bnv[0]; e32[2 * bv + 1] = bnv[1]; w32[bv] = bnv[2]; }
        wfence();
        PDQ_PIS(1, clock64() - t_r0);
    }
    return false;
}

// Sort positions [0, n) of one group (elements already in the store in list order).
// stack: the group's frame area (cap >= n/2 + 2 frames): pending frames longer than
// T_SMALL grow from its start, shorter ones from its end (they are sorted last, one
// wavefront each, with no workgroup barrier).  xs: n elements of exchange scratch.
// limit0 > 0 replaces sort.Slice's initial limit bits.Len(n) (tests: the heapSort fallback).
template <class S> __device__ void wg_sort(const S& s, int n, Frame* __restrict__ stack, int cap,
                                           typename S::Elem* __restrict__ xs, Ctl& c, int limit0) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    PDQ_T(t_all);
    if (tid == 0) {
        c.top = 0;
        c.nsmall = 0;
        c.snext = 0;
        if (n >= 2) {
            const Frame root{0, n, lf_pack(limit0 > 0 ? limit0 : bits_len((uint32_t)n), true, true)};
            if (n <= T_SMALL) { stack[cap - 1] = root; c.nsmall = 1; }
            else { stack[0] = root; c.top = 1; }
        }
    }
#ifdef CASIM_PROF
    if (tid == 0 && blockIdx.x == 0) g_pdq_step = -1;
#endif
    __syncthreads();
    for (;;) {
#ifdef CASIM_PROF
        if (tid == 0 && blockIdx.x == 0) g_pdq_step++;
#endif
        PDQ_T(t_pop);
        if (tid == 0) {
            const int nf = min(c.top, MAXF);
            c.nf = nf;
            c.top -= nf;
            c.base = c.top;
        }
        __syncthreads();
        const int nf = c.nf;
        if (nf == 0) break;
        for (int i = tid; i < nf; i += NT) {
            c.f[i] = stack[c.base + i];
            c.op[i] = OP_DONE;
            c.m[i] = 0;
            c.t[i] = 0;
        }
        __syncthreads();
        PDQ_ADD(2, t_pop);
        PDQ_CNT(11, 1);
        PDQ_CNT(12, nf);
        PDQ_S(0, nf);
        PDQ_T(t_a);
        // A: one pdqsort_func loop iteration's control per frame (a wavefront each)
        for (int i = w; i < nf; i += NW) {
            const Frame fr = c.f[i];
            const int a = fr.a, b = fr.b;
            int limit = fr.lf & 255;
            const bool wb = (fr.lf >> 8) & 1, wp = (fr.lf >> 9) & 1;
            if (limit == 0) {
                if (lane == 0) heap_sort(s, a, b);
                wfence();
                continue;
            }
            PDQ_T(t_bp);
            if (!wb) {
                if (lane == 0) break_patterns(s, a, b);
                wfence();
                limit--;
            }
            PDQ_WADD(16, t_bp);
            PDQ_T(t_cp);
            int hint;
            int pivot = w_choose_pivot(s, a, b, &hint);
            PDQ_WADD(17, t_cp);
            PDQ_SMAXW(14, clock64() - t_cp);
            PDQ_T(t_rv);
            if (hint == HINT_DEC) {
                w_reverse(s, a, b);
                pivot = (b - 1) - (pivot - a);
                hint = HINT_INC;
            }
            PDQ_WADD(18, t_rv);
            bool pis = wb && wp && hint == HINT_INC;
            if constexpr (std::is_same<S, LdsStore>::value) {
                // partialInsertionSort here, one wavefront per frame; long frames (its scans
                // run over the whole frame when it is sorted) go to the workgroup below
                if (pis && b - a <= PIS_WAVE_MAX) {
                    PDQ_T(t_pis);
                    int pi, pL, pR;
                    w_pis_find(s, a, b, a + 1, pi, pL, pR);
                    const bool sorted = w_partial_insertion(s, a, b, pi, pL, pR);
                    PDQ_WADD(19, t_pis);
                    PDQ_SMAXW(13, clock64() - t_pis);
                    PDQ_SMAXW(15, b - a);
                    PDQ_CNT(20, 1);
                    if (sorted) {
                        if (lane == 0) c.op[i] = OP_DONE;
                        wfence();
                        continue;
                    }
                    pis = false;
                }
            }
            if (lane == 0) {
                c.piv[i] = pivot;
                c.pis[i] = pis ? 1 : 0;
                c.op[i] = OP_PART;                  // (A2 decides)
                c.f[i].lf = lf_pack(limit, wb, wp);
            }
            wfence();
        }
        PDQ_SMAXW(11, clock64() - t_a);
        __syncthreads();
        PDQ_S(2, clock64() - t_a);
        PDQ_T(t_wp);
        // partialInsertionSort of the frames that run it, one after another, by the workgroup
        for (int i = 0; i < nf; i++) {
            if (c.op[i] == OP_DONE || !c.pis[i]) continue;
            PDQ_T(t_pis);
            const bool sorted = wg_partial_insertion(s, c, c.f[i].a, c.f[i].b);
            PDQ_WADD(19, t_pis);
            PDQ_CNT(20, 1);
            if (sorted && tid == 0) c.op[i] = OP_DONE;
            __syncthreads();
            PDQ_S(12, 1);
        }
        PDQ_S(3, clock64() - t_wp);
        PDQ_T(t_a2);
        // A2: partitionEqual or partition; the pivot moves to a
        for (int i = w; i < nf; i += NW) {
            if (c.op[i] == OP_DONE) continue;
            if (lane == 0) {
                const int a = c.f[i].a, pivot = c.piv[i];
                const bool eq = a > 0 && !(K(s, a - 1) < K(s, pivot));
                swp(s, a, pivot);
                c.pk[i] = K(s, a);
                c.op[i] = eq ? OP_EQ : OP_PART;
            }
            wfence();
        }
        __syncthreads();
        PDQ_ADD(3, t_a);
        PDQ_S(4, clock64() - t_a2);
        PDQ_T(t_pl);
        if (tid < 64) {                     // the partitioning frames, ordered by start
            static_assert(MAXF <= 128, "two frames per lane");
            // rank of frame i among the partitioning frames by start a (starts are distinct):
            // each lane holds two frames' starts (INT_MAX: not partitioning), the starts are
            // broadcast by readlane — no LDS load per comparison
            const bool on0 = lane < nf && c.op[lane] != OP_DONE;
            const bool on1 = 64 + lane < nf && c.op[64 + lane] != OP_DONE;
            const int a0 = on0 ? c.f[lane].a : INT_MAX, a1 = on1 ? c.f[64 + lane].a : INT_MAX;
            const int np = __builtin_popcountll(__ballot(on0)) + __builtin_popcountll(__ballot(on1));
            int r0 = 0, r1 = 0;
            for (int q = 0; q < min(nf, 64); q++) {
                const int aq = __builtin_amdgcn_readlane(a0, q);
                r0 += aq < a0 ? 1 : 0;
                r1 += aq < a1 ? 1 : 0;
            }
            for (int q = 64; q < nf; q++) {
                const int aq = __builtin_amdgcn_readlane(a1, q - 64);
                r0 += aq < a0 ? 1 : 0;
                r1 += aq < a1 ? 1 : 0;
            }
            if (on0) { c.pl[r0] = lane; c.po[r0] = c.f[lane].b - a0 - 1; }            // (staging for the prefix)
            if (on1) { c.pl[r1] = 64 + lane; c.po[r1] = c.f[64 + lane].b - a1 - 1; }
            if (lane == 0) c.np = np;
            w_prefix(c.po, c.fo, np);
        }
        __syncthreads();
        PDQ_ADD(4, t_pl);
        PDQ_S(5, clock64() - t_pl);
        PDQ_CNT(13, c.np);
        PDQ_CNT(15, c.fo[c.np]);
        PDQ_S(1, c.np);
        PDQ_S(10, c.fo[c.np]);
        PDQ_T(t_part);
        if (c.np > 0) wg_partition(s, c, xs, n);
        PDQ_ADD(5, t_part);
        PDQ_T(t_d);
        // D: finish partitioned frames, push the pending calls
        for (int i = w; i < nf; i += NW) {
            if (c.op[i] == OP_DONE || lane != 0) continue;
            const Frame fr = c.f[i];
            const int a = fr.a, b = fr.b, len = b - a, limit = fr.lf & 255;
            const bool wb = (fr.lf >> 8) & 1, wp = (fr.lf >> 9) & 1;
            auto push = [&](int pa, int pb, int plf) {
                if (pb - pa < 2) return;
                if (pb - pa <= T_SMALL) stack[cap - 1 - atomicAdd(&c.nsmall, 1)] = Frame{pa, pb, plf};
                else stack[atomicAdd(&c.top, 1)] = Frame{pa, pb, plf};
            };
            if (c.op[i] == OP_EQ) {
                push(a + c.m[i] + 1, b, lf_pack(limit, wb, wp));
            } else {
                const int mid = a + c.m[i];
                swp(s, a, mid);
                const int ll = mid - a, rl = b - mid, thr = len / 8;
                const bool already = c.t[i] == 0;
                if (ll < rl) {
                    push(a, mid, lf_pack(limit, true, true));
                    push(mid + 1, b, lf_pack(limit, ll >= thr, already));
                } else {
                    push(mid + 1, b, lf_pack(limit, true, true));
                    push(a, mid, lf_pack(limit, rl >= thr, already));
                }
            }
        }
        __threadfence_block();
        __syncthreads();
        PDQ_ADD(9, t_d);
        PDQ_S(9, clock64() - t_d);
    }
    // the short frames, one wavefront each, claimed in turn
    PDQ_T(t_small);
    const int ns = c.nsmall;
    PDQ_CNT(14, ns);
    for (;;) {
        int q = 0;
        if (lane == 0) q = atomicAdd(&c.snext, 1);
        q = rfl(q);
        if (q >= ns) break;
        const Frame fr = stack[cap - 1 - q];
        w_sort(s, fr.a, fr.b, fr.lf);
    }
    __threadfence_block();
    __syncthreads();
    PDQ_ADD(10, t_small);
    PDQ_ADD(0, t_all);
}

}  // namespace pdq
}  // namespace casim
