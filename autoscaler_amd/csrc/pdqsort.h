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
//     frames together; frames of at most WAVE_SMALL elements are sorted to the end by one
//     wavefront each.
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

namespace casim {
namespace pdq {

constexpr int NT = 1024;             // threads of the workgroup
constexpr int NW = NT / 64;          // wavefronts
constexpr int MAXF = 128;            // frames per workgroup step
constexpr int WAVE_SMALL = 512;      // frames up to this length: one wavefront sorts them to the end
constexpr int MAX_INSERTION = 12;    // pdqsort_func maxInsertion
enum { HINT_UNKNOWN = 0, HINT_INC = 1, HINT_DEC = 2 };
enum { OP_DONE = 0, OP_PART = 1, OP_EQ = 2 };

// A pending pdqsort_func call / loop state: [a, b), limit | wasBalanced<<8 | wasPartitioned<<9
struct Frame { int32_t a, b, lf; };
__device__ inline int32_t lf_pack(int limit, bool wb, bool wp) { return limit | (wb ? 256 : 0) | (wp ? 512 : 0); }

__device__ inline int bits_len(uint32_t x) { return x ? 32 - __clz((int)x) : 0; }

// Element stores.  An element is a position of the group's pod list; key() is its rank.
// LDS: 16-bit positions + an 8-bit rank per position (groups of <= ~52k pods, <= 256
// ranks — C2 / C4).  Global: the rank packed above the position (32 or 64 bits).
struct LdsStore {
    using Elem = uint32_t;
    uint16_t* e;
    const uint8_t* rk;
    __device__ Elem ld(int i) const { const uint32_t p = e[i]; return ((uint32_t)rk[p] << 16) | p; }
    __device__ void st(int i, Elem v) const { e[i] = (uint16_t)v; }
    __device__ static uint32_t key(Elem v) { return v >> 16; }
    __device__ static uint32_t pos(Elem v) { return v & 0xFFFFu; }
};
struct G32Store {   // rank < 4096, position < 2^20
    using Elem = uint32_t;
    uint32_t* e;
    __device__ Elem ld(int i) const { return e[i]; }
    __device__ void st(int i, Elem v) const { e[i] = v; }
    __device__ static uint32_t key(Elem v) { return v >> 20; }
    __device__ static uint32_t pos(Elem v) { return v & 0xFFFFFu; }
};
struct G64Store {
    using Elem = uint64_t;
    uint64_t* e;
    __device__ Elem ld(int i) const { return e[i]; }
    __device__ void st(int i, Elem v) const { e[i] = v; }
    __device__ static uint32_t key(Elem v) { return (uint32_t)(v >> 32); }
    __device__ static uint32_t pos(Elem v) { return (uint32_t)v; }
};

template <class S> __device__ inline uint32_t K(const S& s, int i) { return S::key(s.ld(i)); }
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
    for (int top = hi; top >= lo; top -= 64) {                      // right to left
        const int p = top - lane;
        typename S::Elem v = 0;
        if (p >= lo) v = s.ld(p);
        wfence();
        if (p >= lo) s.st(p + 1, v);
        wfence();
    }
}
template <class S> __device__ void w_shift_left(const S& s, int lo, int hi) {
    const int lane = threadIdx.x & 63;
    for (int bot = lo; bot <= hi; bot += 64) {                      // left to right
        const int p = bot + lane;
        typename S::Elem v = 0;
        if (p <= hi) v = s.ld(p);
        wfence();
        if (p <= hi) s.st(p - 1, v);
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
            for (int top = i - 2; top >= qmin && !found; top -= 64) {
                const int q = top - lane;
                const uint64_t m = __ballot(q >= qmin && K(s, q) <= ke);
                if (m) { land = top - (int)__builtin_ctzll(m) + 1; found = true; }
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
            for (int bot = i + 1; bot < b; bot += 64) {
                const int j = bot + lane;
                const uint64_t m = __ballot(j < b && !(K(s, j) < kf));
                if (m) { land = bot + (int)__builtin_ctzll(m) - 1; break; }
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

// partition_func (eq = 0) / partitionEqual_func (eq = 1) on [a, b) whose pivot (key pk)
// is already at a: the rank-paired exchange.  scr[a .. b) is the frame's own scratch.
// Returns m = #pred over [a+1, b-1] and t = #pairs swapped.
template <class S> __device__ void w_exchange(const S& s, int a, int b, uint32_t pk, int eq, uint32_t* __restrict__ scr,
                                            int* m_out, int* t_out) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lanes_below();
    auto pred = [&](int p) { const uint32_t k = K(s, p); return eq ? k <= pk : k < pk; };
    int m = 0;
    for (int base = a + 1; base < b; base += 64) {
        const int p = base + lane;
        m += __builtin_popcountll(__ballot(p < b && pred(p)));
    }
    const int z = a + m, c0 = (b - a + 1) / 2;
    int t = 0;
    for (int base = a + 1; base <= z; base += 64) {                 // left zone: the k-th failing pred
        const int p = base + lane;
        const bool f = p <= z && !pred(p);
        const uint64_t mk = __ballot(f);
        if (f) scr[a + t + __builtin_popcountll(mk & below)] = (uint32_t)p;
        t += __builtin_popcountll(mk);
    }
    int j = 0;
    for (int base = z + 1; base < b; base += 64) {                  // right zone: passing pred, left to right
        const int p = base + lane;
        const bool f = p < b && pred(p);
        const uint64_t mk = __ballot(f);
        if (f) scr[a + c0 + j + __builtin_popcountll(mk & below)] = (uint32_t)p;
        j += __builtin_popcountll(mk);
    }
    wfence();
    for (int k0 = 0; k0 < t; k0 += 64) {                            // k-th from the left <-> k-th from the right
        const int k = k0 + lane;
        if (k < t) swp(s, (int)scr[a + k], (int)scr[a + c0 + t - 1 - k]);
    }
    wfence();
    *m_out = m;
    *t_out = t;
}

// pdqsort_func on one frame, to the end, by one wavefront.  The frames it defers live in
// a VGPR stack (lane j holds entry j): it continues with the smaller side and defers the
// larger, so the depth stays below log2(len) + 1.
template <class S> __device__ void w_sort(const S& s, int a, int b, int lf, uint32_t* __restrict__ scr) {
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
                w_exchange(s, a, b, pk, eq, scr, &m, &t);
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
struct Ctl {
    Frame f[MAXF];
    int32_t op[MAXF];
    uint32_t pk[MAXF];
    int32_t m[MAXF], t[MAXF];
    int32_t fo[MAXF + 1];      // prefix of the frames' interior lengths (partitioned frames only)
    int32_t po[MAXF + 1];      // prefix of the frames' pair counts
    uint64_t wsum[NW];
    uint32_t wflag[NW];
    int32_t nf, top, base;
    uint32_t rmax;
};

// frame of concatenated index x: fo[f] <= x < fo[f+1]
__device__ inline int find_frame(const int32_t* fo, int nf, int x) {
    int lo = 0, hi = nf;                    // largest f with fo[f] <= x (then skip empty frames)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (fo[mid] <= x) lo = mid; else hi = mid;
    }
    while (lo < nf - 1 && fo[lo + 1] <= x) lo++;
    return lo;
}

// exclusive prefix (over lanes, then waves) of n entries of v[] into o[], o[n] = total; one wave
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
        carry += __shfl(incl, 63, 64);
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
    // exclusive inside the wave
    uint64_t ev = __shfl_up(iv, 1, 64);
    bool ef = __shfl_up((int)iflag, 1, 64) != 0;
    if (lane == 0) { ev = 0; ef = false; }
    return ef ? ev : pv + ev;
}

// One pdqsort_func partition (or partitionEqual) of every frame of the step with
// op != OP_DONE, as one pass over the concatenation of their interiors.
template <class S> __device__ void wg_partition(const S& s, Ctl& c, int nf, uint32_t* __restrict__ scr) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int TT = c.fo[nf];
    const int ch = (TT + NT - 1) / NT;
    const int x0 = min(tid * ch, TT), x1 = min(x0 + ch, TT);
    const bool cache = ch <= 64;
    // P1: m[f] = #pred over the interior
    uint64_t pm = 0;
    {
        int f = x0 < x1 ? find_frame(c.fo, nf, x0) : 0;
        int fend = x0 < x1 ? c.fo[f + 1] : 0, a1 = x0 < x1 ? c.f[f].a + 1 - c.fo[f] : 0;
        uint32_t pk = x0 < x1 ? c.pk[f] : 0;
        bool eq = x0 < x1 && c.op[f] == OP_EQ;
        int cnt = 0, flast = f;
        bool multi = false;
        for (int x = x0; x < x1; x++) {
            if (x >= fend) {
                atomicAdd(&c.m[f], cnt);
                cnt = 0;
                multi = true;
                do { f++; } while (c.fo[f + 1] <= x);
                fend = c.fo[f + 1]; a1 = c.f[f].a + 1 - c.fo[f]; pk = c.pk[f]; eq = c.op[f] == OP_EQ;
            }
            const uint32_t k = K(s, a1 + x);
            const bool pr = eq ? k <= pk : k < pk;
            cnt += pr ? 1 : 0;
            if (cache && pr) pm |= 1ull << (x - x0);
        }
        flast = f;
        // wave aggregation when every lane's (last) frame is the same
        const int f0 = rfl(flast);
        const bool same = __ballot(x0 < x1 && flast != f0) == 0;
        if (same) {
            int tot = cnt;
            for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d, 64);
            if (lane == 0 && tot) atomicAdd(&c.m[f0], tot);
        } else if (x0 < x1 && cnt) {
            atomicAdd(&c.m[flast], cnt);
        }
        (void)multi;
    }
    __syncthreads();
    // P2: the k-th left-zone element failing pred -> scr[a + k]; the j-th right-zone
    // element passing it (from the left) -> scr[a + c0 + j]
    {
        auto pred_at = [&](int x, int a1, uint32_t pk, bool eq) -> bool {
            if (cache) return (pm >> (x - x0)) & 1ull;
            const uint32_t k = K(s, a1 + x);
            return eq ? k <= pk : k < pk;
        };
        uint32_t lm = 0, rm = 0;
        bool has_start = false;
        if (x0 < x1) {
            int f = find_frame(c.fo, nf, x0);
            int fend = c.fo[f + 1], fbeg = c.fo[f], a = c.f[f].a, a1 = a + 1 - fbeg, z = a + c.m[f];
            uint32_t pk = c.pk[f];
            bool eq = c.op[f] == OP_EQ;
            for (int x = x0; x < x1; x++) {
                if (x >= fend) {
                    do { f++; } while (c.fo[f + 1] <= x);
                    fend = c.fo[f + 1]; fbeg = c.fo[f]; a = c.f[f].a; a1 = a + 1 - fbeg; z = a + c.m[f];
                    pk = c.pk[f]; eq = c.op[f] == OP_EQ;
                }
                if (x == fbeg) { lm = 0; rm = 0; has_start = true; }
                const int p = a1 + x;
                const bool pr = pred_at(x, a1, pk, eq);
                if (p <= z) lm += pr ? 0u : 1u; else rm += pr ? 1u : 0u;
            }
        }
        const uint64_t ex = wg_seg_scan(((uint64_t)rm << 32) | lm, has_start, c);
        lm = (uint32_t)ex;
        rm = (uint32_t)(ex >> 32);
        if (x0 < x1) {
            int f = find_frame(c.fo, nf, x0);
            int fend = c.fo[f + 1], fbeg = c.fo[f], a = c.f[f].a, a1 = a + 1 - fbeg, z = a + c.m[f];
            int c0 = (c.f[f].b - a + 1) / 2;
            uint32_t pk = c.pk[f];
            bool eq = c.op[f] == OP_EQ;
            for (int x = x0; x < x1; x++) {
                if (x >= fend) {
                    do { f++; } while (c.fo[f + 1] <= x);
                    fend = c.fo[f + 1]; fbeg = c.fo[f]; a = c.f[f].a; a1 = a + 1 - fbeg; z = a + c.m[f];
                    c0 = (c.f[f].b - a + 1) / 2; pk = c.pk[f]; eq = c.op[f] == OP_EQ;
                }
                if (x == fbeg) { lm = 0; rm = 0; }
                const int p = a1 + x;
                const bool pr = pred_at(x, a1, pk, eq);
                if (p <= z) {
                    if (!pr) scr[a + lm++] = (uint32_t)p;
                } else if (pr) {
                    scr[a + c0 + rm++] = (uint32_t)p;
                }
                if (x == fend - 1) c.t[f] = (int32_t)lm;     // the frame's pair count
            }
        }
    }
    __syncthreads();
    if (tid < 64) {
        // (frames that did not partition have t = 0)
        w_prefix(c.t, c.po, nf);
    }
    __syncthreads();
    // P3: pairs
    {
        const int TP = c.po[nf];
        const int cp = (TP + NT - 1) / NT;
        const int y0 = min(tid * cp, TP), y1 = min(y0 + cp, TP);
        if (y0 < y1) {
            int f = find_frame(c.po, nf, y0);
            int fend = c.po[f + 1], fbeg = c.po[f], a = c.f[f].a, t = c.t[f], c0 = (c.f[f].b - a + 1) / 2;
            for (int y = y0; y < y1; y++) {
                if (y >= fend) {
                    do { f++; } while (c.po[f + 1] <= y);
                    fend = c.po[f + 1]; fbeg = c.po[f]; a = c.f[f].a; t = c.t[f]; c0 = (c.f[f].b - a + 1) / 2;
                }
                const int k = y - fbeg;
                swp(s, (int)scr[a + k], (int)scr[a + c0 + t - 1 - k]);
            }
        }
    }
    __syncthreads();
}

// Sort positions [0, n) of one group (elements already in the store in list order).
// limit0 > 0 replaces sort.Slice's initial limit bits.Len(n) (tests: the heapSort fallback).
// stack: the group's pending frames (capacity n/2 + 2); scr: n entries of scratch.
template <class S> __device__ void wg_sort(const S& s, int n, Frame* __restrict__ stack, uint32_t* __restrict__ scr,
                                           Ctl& c, int limit0) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) {
        c.top = 0;
        if (n >= 2) { stack[0] = Frame{0, n, lf_pack(limit0 > 0 ? limit0 : bits_len((uint32_t)n), true, true)}; c.top = 1; }
    }
    __syncthreads();
    for (;;) {
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
        // A: one loop iteration's control per frame (a wavefront each); small frames to the end
        for (int i = w; i < nf; i += NW) {
            const Frame fr = c.f[i];
            int a = fr.a, b = fr.b, limit = fr.lf & 255;
            const bool wb = (fr.lf >> 8) & 1, wp = (fr.lf >> 9) & 1;
            if (b - a <= WAVE_SMALL) { w_sort(s, a, b, fr.lf, scr); continue; }
            if (limit == 0) {
                if (lane == 0) heap_sort(s, a, b);
                wfence();
                continue;
            }
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
            if (wb && wp && hint == HINT_INC && w_partial_insertion(s, a, b)) continue;
            if (lane == 0) {
                const bool eq = a > 0 && !(K(s, a - 1) < K(s, pivot));
                swp(s, a, pivot);
                c.pk[i] = K(s, a);
                c.op[i] = eq ? OP_EQ : OP_PART;
                c.f[i].lf = lf_pack(limit, wb, wp);
            }
            wfence();
        }
        __syncthreads();
        if (tid < 64) {
            // interior lengths of the partitioned frames (scratch: the m[] slots are 0 here)
            int32_t* len = c.t;                 // t[] is rewritten by wg_partition
            for (int i = lane; i < nf; i += 64) len[i] = c.op[i] != OP_DONE ? c.f[i].b - c.f[i].a - 1 : 0;
            w_prefix(len, c.fo, nf);
            for (int i = lane; i < nf; i += 64) len[i] = 0;
        }
        __syncthreads();
        if (c.fo[nf] > 0) wg_partition(s, c, nf, scr);
        // D: finish partitioned frames, push the pending calls
        for (int i = w; i < nf; i += NW) {
            if (c.op[i] == OP_DONE || lane != 0) continue;
            const Frame fr = c.f[i];
            const int a = fr.a, b = fr.b, len = b - a, limit = fr.lf & 255;
            const bool wb = (fr.lf >> 8) & 1, wp = (fr.lf >> 9) & 1;
            auto push = [&](int pa, int pb, int plf) {
                if (pb - pa >= 2) stack[atomicAdd(&c.top, 1)] = Frame{pa, pb, plf};
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
    }
}

}  // namespace pdq
}  // namespace casim
