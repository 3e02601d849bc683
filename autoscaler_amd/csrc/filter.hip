// filter.hip — FilterOutSchedulable: HintingSimulator.TrySchedulePods(pending pods,
// ScheduleAnywhere, breakOnFailure=false), committed into the mirror.
//
// Reference: CA/core/podlistprocessor/filter_out_schedulable.go:95-124,
// CA/simulator/scheduling/hinting_simulator.go:58-125 (findNodeWithHints / findNode),
// CA/simulator/scheduling/similar_pods.go:43-111 (the per-call unschedulable cache),
// CA/simulator/predicatechecker/schedulerbased.go:103-137 (FitsAnyNodeMatching's rotating
// scan from lastIndex) and :139-185 (CheckPredicates).
//
// The reference is a sequential loop over the pods: a hint check, then (unless a similar
// pod already failed) a rotating scan from lastIndex; a placed pod is added to the
// snapshot before the next pod runs.  One persistent workgroup (16 waves) runs that loop
// in speculative batches of FO_T pods, one pod per thread, every outcome computed against
// the node rows as they were when the batch started:
//   hint   CheckPredicates on the hinted node (findNodeWithHints);
//   skip   the pod's class is already marked unschedulable (IsSimilarUnschedulable);
//   short  a lane-private rotating scan of <= FO_SHORT_K positions from the pod's start,
//          start = lastIndex + the positions the earlier pods of the batch advanced it by.
//          The advances depend on the starts, so the starts are iterated to a fixed point
//          (a landing further along shifts the later starts; rarely more than 2 rounds);
//   long   nothing within FO_SHORT_K: a block-wide scan of the whole ring.  A scan of the
//          whole ring that finds nothing does not depend on where it starts, and stays a
//          failure whatever the earlier pods of the batch placed (placements only take
//          resources, pod slots and ports away; the other filters read static node
//          attributes), so failures commit in bulk.  A pod whose record equals an earlier
//          failed pod's takes that result without scanning; a pod whose class an earlier
//          failure of the batch marks is a skip.
// The batch commits its longest prefix whose outcomes are exact.  It ends at the first pod
// that (a) found a node with a long scan, (b) has an unconverged start, (c) read a node an
// earlier pod of the batch placed on (its hinted node or a scanned position), (d) is the
// first failure of a controller that can reach similar_pods' 10-class cap, or (e) fits
// where an earlier failure of its class says it cannot.  That pod then runs alone,
// block-wide, exactly as the reference's loop body, and the next batch starts after it.
#include "mirror.h"
#include "device_filters.h"

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstring>

namespace casim {

constexpr int FO_T = 1024;             // pods per batch = threads of the workgroup
constexpr int FO_W = FO_T / 64;
constexpr int FO_SHORT_K = 4;          // positions of the lane-private scan
constexpr int FO_ROUNDS = 4;           // fixed-point rounds of the starts
constexpr int FO_HT = 2048;            // LDS hash slots (>= 2 * FO_T)
constexpr int FO_HT_BITS = 11;
constexpr int FO_MAX_PER_OWNER = 10;   // maxPodsPerOwnerRef, similar_pods.go:53
static_assert((1 << FO_HT_BITS) == FO_HT, "FO_HT");

constexpr int SPEC_WORDS = (int)(sizeof(ca_pod_spec) / 8);
static_assert(sizeof(ca_pod_spec) % 8 == 0, "ca_pod_spec words");
constexpr int SPEC_CLS_WORD = (int)(offsetof(ca_pod_spec, similar_class) / 8);

struct FoCtl {
    int32_t L;                 // lastIndex in/out
    int32_t overflowing;       // controllers that overflowed the class cap
    int32_t batches, cuts;
    unsigned long long evals;
    int32_t bad_line, bad_val; // CASIM_FO_CHECKS builds: the first index check that failed
};

struct FoArgs {
    NodeHot* hot;
    NodeExt* ext;
    const NodeStatic* st;
    int32_t n;
    const PodHot* ph;
    const ca_pod_spec* specs;
    const ca_selector_term* terms;
    const ca_selector_req* reqs;
    const int32_t* names;
    const int32_t* order;
    int32_t P;
    int32_t* hints;            // per position, in/out
    int32_t* out_node;         // per position
    uint8_t* cls_mark;         // per class: items[uid] holds it
    const uint8_t* cls_capped; // per class: its controller has more than 10 classes in this call
    const int32_t* cls_owner;  // per class: dense controller id (-1: none); NULL: no cap
    int32_t* owner_cnt;        // per controller: classes remembered
    uint8_t* owner_over;       // per controller: overflowed
    unsigned long long* claim; // per node: (batch << 16) | (0xFFFF - position) of the earliest placement
    FoCtl* ctl;
    int32_t n_pods, n_classes, n_owners;
};

// Index checks of the diagnostics build (make checks: -DCASIM_FO_CHECKS): an index out of
// range is recorded in ctl (first failure) and replaced by 0 instead of faulting.
#ifdef CASIM_FO_CHECKS
__device__ inline int32_t fo_ck(const FoArgs& a, int32_t i, int32_t lim, int line) {
    if (i >= 0 && i < lim) return i;
    if (atomicCAS(&a.ctl->bad_line, 0, line) == 0) a.ctl->bad_val = i;
    return 0;
}
#define CK(i, lim) fo_ck(a, (i), (lim), __LINE__)
#else
#define CK(i, lim) (i)
#endif

struct FoSmem {
    int32_t red_i[FO_W];
    unsigned long long red_u[FO_W];
    unsigned long long fit[FO_W], vis[FO_W];
    int32_t ckey[FO_HT], cval[FO_HT];               // class -> first failing position of the batch
    unsigned long long skey[FO_HT];                 // record hash -> first long position
    int32_t sval[FO_HT];
    int16_t ulist[FO_T];                            // long pods that scan, in order
    int32_t lstart[FO_T];                           // per position: start of its scan
    uint32_t lev[FO_T];                             // per position: evaluations of its long scan
    int32_t bcast;
};

// ---- block primitives (all threads, uniform control flow) -----------------------
__device__ inline int32_t fo_excl(FoSmem& sm, int32_t v, int32_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) sm.red_i[w] = x;
    __syncthreads();
    int32_t base = 0, tot = 0;
    for (int k = 0; k < FO_W; k++) {
        const int32_t s = sm.red_i[k];
        base += (k < w) ? s : 0;
        tot += s;
    }
    total = tot;
    return base + x - v;
}

__device__ inline int32_t fo_min(FoSmem& sm, int32_t v) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if (lane == 0) sm.red_i[w] = v;
    __syncthreads();
    int32_t m = INT32_MAX;
    for (int k = 0; k < FO_W; k++) m = min(m, sm.red_i[k]);
    return m;
}

__device__ inline int32_t fo_max(FoSmem& sm, int32_t v) { return -fo_min(sm, -v); }

__device__ inline unsigned long long fo_sum64(FoSmem& sm, unsigned long long v) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) sm.red_u[w] = v;
    __syncthreads();
    unsigned long long s = 0;
    for (int k = 0; k < FO_W; k++) s += sm.red_u[k];
    return s;
}

// ---- LDS hash tables (open addressing; at most FO_T keys per batch) -------------
__device__ inline void ht_min_i(int32_t* keys, int32_t* vals, int32_t key, int32_t v) {
    uint32_t sl = ((uint32_t)key * 2654435761u) >> (32 - FO_HT_BITS);
    while (true) {
        const int32_t old = atomicCAS(&keys[sl], -1, key);
        if (old == -1 || old == key) { atomicMin(&vals[sl], v); return; }
        sl = (sl + 1) & (FO_HT - 1);
    }
}
__device__ inline int32_t ht_get_i(const int32_t* keys, const int32_t* vals, int32_t key) {
    uint32_t sl = ((uint32_t)key * 2654435761u) >> (32 - FO_HT_BITS);
    while (true) {
        const int32_t k = keys[sl];
        if (k == key) return vals[sl];
        if (k == -1) return INT32_MAX;
        sl = (sl + 1) & (FO_HT - 1);
    }
}
__device__ inline void ht_min_u(unsigned long long* keys, int32_t* vals, unsigned long long key, int32_t v) {
    uint32_t sl = (uint32_t)(key >> (64 - FO_HT_BITS));
    while (true) {
        const unsigned long long old = atomicCAS(&keys[sl], 0ull, key);
        if (old == 0ull || old == key) { atomicMin(&vals[sl], v); return; }
        sl = (sl + 1) & (FO_HT - 1);
    }
}
__device__ inline int32_t ht_get_u(const unsigned long long* keys, const int32_t* vals, unsigned long long key) {
    uint32_t sl = (uint32_t)(key >> (64 - FO_HT_BITS));
    while (true) {
        const unsigned long long k = keys[sl];
        if (k == key) return vals[sl];
        if (k == 0ull) return INT32_MAX;
        sl = (sl + 1) & (FO_HT - 1);
    }
}

// hash of a pod record without its similar_class (two pods with equal records get equal
// filter results on every node); never 0
__device__ inline unsigned long long spec_hash(const ca_pod_spec* s) {
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(s);
    unsigned long long h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < SPEC_WORDS; i++) {
        unsigned long long x = w[i];
        if (i == SPEC_CLS_WORD) x &= (offsetof(ca_pod_spec, similar_class) % 8) ? 0x00000000FFFFFFFFull
                                                                                    : 0xFFFFFFFF00000000ull;
        h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
        h *= 0xBF58476D1CE4E5B9ull;
    }
    return h | 1ull;
}
__device__ inline bool spec_equal(const ca_pod_spec* a, const ca_pod_spec* b) {
    const unsigned long long* x = reinterpret_cast<const unsigned long long*>(a);
    const unsigned long long* y = reinterpret_cast<const unsigned long long*>(b);
    const unsigned long long m = (offsetof(ca_pod_spec, similar_class) % 8) ? 0x00000000FFFFFFFFull
                                                                             : 0xFFFFFFFF00000000ull;
    bool eq = true;
    for (int i = 0; i < SPEC_WORDS; i++) {
        const unsigned long long mm = (i == SPEC_CLS_WORD) ? m : ~0ull;
        eq &= ((x[i] ^ y[i]) & mm) == 0;
    }
    return eq;
}

// ---- filters ------------------------------------------------------------------------
__device__ inline bool fo_names_ok(const ca_pod_spec& s, const int32_t* names, int32_t name_id) {
    bool ok = false;
    for (int32_t k = 0; k < s.prefilter_count; k++) ok |= names[s.prefilter_first + k] == name_id;
    return ok;
}
// FitsAnyNodeMatching visits the node (schedulerbased.go:116-127): PreFilter's NodeNames
// and Spec.Unschedulable skip a node without running the filters
__device__ inline bool fo_visible(const FoArgs& a, const PodHot& p, const ca_pod_spec& s, const NodeHot& h,
                                  int32_t pos) {
    if (h.flags & NF_UNSCHED) return false;
    if (p.flags & PF_PREFILTER_NAMES) return fo_names_ok(s, a.names, a.st[CK(pos, a.n)].name_id);
    return true;
}
__device__ inline bool fo_fits(const FoArgs& a, const PodHot& p, const ca_pod_spec& s, const NodeHot& h,
                               int32_t pos, bool apply_unsched) {
    uint32_t r;
    pos = CK(pos, a.n);
    return dev_full_filters(s, p, a.terms, a.reqs, h, a.ext + pos, a.st + pos, apply_unsched, &r) == CA_PLUGIN_NONE;
}

// Rows, marks and counters this kernel writes are read with device-coherent loads where
// the address is uniform: a uniform plain load may be served from the scalar cache, which
// the kernel's own vector stores do not update (waves could then disagree on a branch that
// must be block-uniform).
template <class T>
__device__ inline T ld_coh(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline NodeHot ld_hot_coh(const NodeHot* p) {
    const int64_t* q = reinterpret_cast<const int64_t*>(p);
    NodeHot h;
    h.cpu = ld_coh(q);
    h.mem = ld_coh(q + 1);
    h.eph = ld_coh(q + 2);
    const uint64_t w = (uint64_t)ld_coh(q + 3);
    h.pods = (int32_t)(uint32_t)w;
    h.flags = (uint32_t)(w >> 32);
    return h;
}
__device__ inline NodeExt ld_ext_coh(const NodeExt* p) {
    const int64_t* q = reinterpret_cast<const int64_t*>(p);
    NodeExt e;
    for (int k = 0; k < CA_MAX_SCALAR; k++) e.scalar[k] = ld_coh(q + k);
    for (int w = 0; w < CA_PORT_WORDS; w++) e.ports[w] = (uint64_t)ld_coh(q + CA_MAX_SCALAR + w);
    return e;
}
__device__ inline uint8_t ld_mark(const uint8_t* p) {
    // byte marks: a coherent load of the aligned word holding the byte
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t w = ld_coh(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3));
    return (uint8_t)(w >> (8 * (a & 3)));
}

// AddPod on the device rows (NodeInfo.AddPod's resource/port update, SF/types.go:672-692)
__device__ inline void fo_place(const FoArgs& a, const PodHot& p, const ca_pod_spec& s, int32_t node) {
    node = CK(node, a.n);
    NodeHot* h = a.hot + node;
    const NodeHot cur = ld_hot_coh(h);        // fo_single's address is uniform: no scalar-cache read
    h->cpu = wsub(cur.cpu, p.cpu);
    h->mem = wsub(cur.mem, p.mem);
    h->eph = wsub(cur.eph, p.eph);
    h->pods = cur.pods - 1;
    uint64_t pu = 0;
    for (int w = 0; w < CA_PORT_WORDS; w++) pu |= s.port_use[w];
    if (pu || (p.flags & PF_SCALAR_REQ)) {
        NodeExt* e = a.ext + node;
        const NodeExt ce = ld_ext_coh(e);
        for (int w = 0; w < CA_PORT_WORDS; w++) e->ports[w] = ce.ports[w] | s.port_use[w];
        for (int k = 0; k < CA_MAX_SCALAR; k++) e->scalar[k] = wsub(ce.scalar[k], s.req_scalar[k]);
        if (pu) h->flags = cur.flags | NF_PORTS;
    }
}

// SetUnschedulable (similar_pods.go:92-111); one thread
__device__ inline void fo_mark(const FoArgs& a, int32_t c) {
    c = CK(c, a.n_classes);
    int32_t o = a.cls_owner ? a.cls_owner[c] : -1;
    if (o >= 0) o = CK(o, a.n_owners);
    if (o < 0 || !a.cls_capped[c]) {
        a.cls_mark[c] = 1;
        return;
    }
    if (ld_coh(&a.owner_cnt[o]) >= FO_MAX_PER_OWNER) {
        if (!ld_mark(&a.owner_over[o])) {
            a.owner_over[o] = 1;
            a.ctl->overflowing = ld_coh(&a.ctl->overflowing) + 1;
        }
        return;
    }
    a.cls_mark[c] = 1;
    a.owner_cnt[o] = ld_coh(&a.owner_cnt[o]) + 1;
}

// FitsAnyNode's rotating scan of the whole ring from `start`, block-wide: the first node
// that fits (-1: none) and the evaluations up to it (every visible node if none fits)
__device__ void fo_ring_scan(const FoArgs& a, FoSmem& sm, const PodHot& p, const ca_pod_spec& s, int32_t start,
                             int32_t& found, uint32_t& evs) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int32_t n = a.n;
    found = -1;
    evs = 0;
    for (int32_t base = 0; base < n; base += FO_T) {
        const int32_t off = base + (int32_t)threadIdx.x;
        bool vis = false, fit = false;
        if (off < n) {
            int32_t pos = start + off;
            if (pos >= n) pos -= n;
            pos = CK(pos, n);
            const NodeHot h = a.hot[pos];
            vis = fo_visible(a, p, s, h, pos);
            fit = vis && fo_fits(a, p, s, h, pos, false);
        }
        const unsigned long long fm = __ballot(fit), vm = __ballot(vis);
        __syncthreads();
        if (lane == 0) { sm.fit[w] = fm; sm.vis[w] = vm; }
        __syncthreads();
        bool done = false;
        uint32_t cnt = 0;
        for (int k = 0; k < FO_W && !done; k++) {
            const unsigned long long f = sm.fit[k], v = sm.vis[k];
            if (f) {
                const int l = __builtin_ctzll(f);
                cnt += (uint32_t)__builtin_popcountll(v & ((2ull << l) - 1ull));
                found = base + k * 64 + l;
                done = true;
            } else {
                cnt += (uint32_t)__builtin_popcountll(v);
            }
        }
        evs += cnt;
        if (done) break;
    }
    if (found >= 0) {
        found += start;
        if (found >= n) found -= n;
    }
}

// the reference's loop body for one pod, block-wide (hinting_simulator.go:63-86)
__device__ void fo_single(const FoArgs& a, FoSmem& sm, int32_t k, int32_t& L, unsigned long long& evals) {
    const int32_t n = a.n;
    k = CK(k, a.P);
    const PodHot p = a.ph[CK(a.order[k], a.n_pods)];
    const ca_pod_spec& s = a.specs[CK(p.spec, a.n_pods)];
    const int32_t h = a.hints[k];
    const int32_t c = s.similar_class;
    // the block-uniform decisions are taken by thread 0 on coherent loads and broadcast:
    // 1 the hinted node fits (findNodeWithHints), 2 the class is marked (a skip), 0 scan
    if (threadIdx.x == 0) {
        int32_t dec = 0;
        if (h >= 0 && h < n && !(p.flags & PF_PREFILTER_FAIL)) {
            evals++;
            const NodeHot hh = ld_hot_coh(a.hot + h);
            const NodeExt he = ld_ext_coh(a.ext + h);
            uint32_t r;
            if (dev_full_filters(s, p, a.terms, a.reqs, hh, &he, a.st + h, true, &r) == CA_PLUGIN_NONE) dec = 1;
        }
        if (dec == 0 && c >= 0 && ld_mark(&a.cls_mark[CK(c, a.n_classes)])) dec = 2;
        sm.bcast = dec;
    }
    __syncthreads();
    const int32_t dec = sm.bcast;
    __syncthreads();
    int32_t node = (dec == 1) ? h : -1;
    if (node < 0) {                                                     // findNode
        if (dec != 2) {
            int32_t found = -1;
            uint32_t ev = 0;
            if (!(p.flags & PF_PREFILTER_FAIL) && n > 0) fo_ring_scan(a, sm, p, s, L % n, found, ev);
            if (threadIdx.x == 0) evals += ev;
            if (found >= 0) {
                node = found;
                L = (found + 1 == n) ? 0 : found + 1;                   // schedulerbased.go:131
            } else if (c >= 0 && !(p.flags & PF_DAEMONSET) && threadIdx.x == 0) {
                fo_mark(a, c);
            }
        }
    }
    if (threadIdx.x == 0) {
        a.out_node[k] = node;
        if (node >= 0) {
            a.hints[k] = node;
            fo_place(a, p, s, node);
        }
    }
    __syncthreads();
}

__device__ inline unsigned long long claim_key(unsigned long long gen, int32_t j) {
    return (gen << 16) | (unsigned long long)(0xFFFF - j);
}
// an earlier pod of batch `gen` placed on `pos`
__device__ inline bool claimed_before(const FoArgs& a, int32_t pos, unsigned long long gen, int32_t j) {
    pos = CK(pos, a.n);
    const unsigned long long c = __hip_atomic_load(&a.claim[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (c >> 16) == gen && (int32_t)(0xFFFF - (c & 0xFFFF)) < j;
}

__global__ void __launch_bounds__(FO_T) k_filter_out(FoArgs a) {
    __shared__ FoSmem sm;
    const int32_t tid = (int32_t)threadIdx.x;
    const int32_t n = a.n, P = a.P;
    int32_t L = a.ctl->L;
    bool any_success = false;
    unsigned long long evals = 0;
    int32_t batches = 0, cuts = 0;
    unsigned long long gen = 0;
    for (int32_t k0 = 0; k0 < P;) {
        gen++;
        batches++;
        const int32_t nb = min(FO_T, P - k0);
        const int32_t k = k0 + tid;
        const bool valid = tid < nb;
        for (int x = tid; x < FO_HT; x += FO_T) {
            sm.ckey[x] = -1; sm.cval[x] = INT32_MAX;
            sm.skey[x] = 0ull; sm.sval[x] = INT32_MAX;
        }
        sm.lev[tid] = 0;
        PodHot p = {};
        const ca_pod_spec* sp = a.specs;
        int32_t cls = -1, h = -1;
        if (valid) {
            p = a.ph[CK(a.order[CK(k, P)], a.n_pods)];
            sp = a.specs + CK(p.spec, a.n_pods);
            cls = sp->similar_class;
            if (cls >= 0) cls = CK(cls, a.n_classes);
            h = a.hints[k];
        }
        const ca_pod_spec& s = *sp;
        const bool ds = (p.flags & PF_DAEMONSET) != 0;
        // findNodeWithHints on the batch-start rows
        uint32_t ev = 0;
        bool hint_ok = false;
        if (valid && h >= 0 && h < n && !(p.flags & PF_PREFILTER_FAIL)) {
            ev = 1;
            hint_ok = fo_fits(a, p, s, a.hot[CK(h, n)], h, true);
        }
        const bool skip0 = valid && !hint_ok && cls >= 0 && a.cls_mark[cls];
        const bool active = valid && !hint_ok && !skip0;                     // runs FitsAnyNode
        const bool pff = active && ((p.flags & PF_PREFILTER_FAIL) || n == 0); // fails without a scan
        const bool scanner = active && !pff;
        const int32_t Lr = n > 0 ? L % n : 0;
#ifdef CASIM_FO_CHECKS
        if (n > 0) CK(Lr, n);
#endif
        // lane-private short scans, starts iterated to a fixed point
        int32_t adv = scanner ? 1 : 0, start = 0, start_ev = -1, fnode = -1;
        uint32_t sev = 0;
        bool sfound = false;
        for (int r = 0;; r++) {
            int32_t tot;
            const int32_t ex = fo_excl(sm, adv, tot);
#ifdef CASIM_FO_CHECKS
            CK(adv, FO_SHORT_K + 1);
            {
                __syncthreads();
                sm.lstart[tid] = adv;
                __syncthreads();
                int32_t ex2 = 0, t2 = 0;
                for (int j = 0; j < FO_T; j++) { ex2 += (j < tid) ? sm.lstart[j] : 0; t2 += sm.lstart[j]; }
                __syncthreads();
                if (ex2 != ex || t2 != tot) {
                    if (atomicCAS(&a.ctl->bad_line, 0, __LINE__) == 0)
                        a.ctl->bad_val = tid * 1000000 + (ex2 - ex) * 1000 + r;
                }
            }
#endif
            if (scanner) start = (int32_t)(((int64_t)Lr + ex) % n);
            const bool ch = scanner && start != start_ev;
            if (fo_min(sm, ch ? 0 : 1) != 0 || r == FO_ROUNDS) break;
            if (ch) {
                start_ev = start;
                sfound = false;
                sev = 0;
                int32_t pos = start;
                const int32_t lim = min(FO_SHORT_K, n);
                for (int t = 0; t < lim; t++) {
                    const NodeHot hh = a.hot[CK(pos, n)];
                    if (fo_visible(a, p, s, hh, pos)) {
                        sev++;
                        if (fo_fits(a, p, s, hh, pos, false)) {
                            sfound = true;
                            fnode = pos;
                            adv = t + 1;
                            break;
                        }
                    }
                    if (++pos == n) pos = 0;
                }
                if (!sfound) adv = 0;
            }
        }
        int32_t b = fo_min(sm, (scanner && sfound && start != start_ev) ? tid : INT32_MAX);   // (b)
        b = min(b, nb);
        // long pods before b: dedup by class (a later pod of a class whose earlier long pod
        // failed is a skip) and by record; the rest scan the whole ring, in order
        const bool is_long = scanner && !sfound && tid < b;
        if ((is_long || (pff && tid < b)) && cls >= 0 && !ds) ht_min_i(sm.ckey, sm.cval, cls, tid);
        if (is_long) sm.lstart[tid] = start;
        __syncthreads();
        // first failing candidate of the class (a long or PreFilter-failed pod)
        const int32_t first = (cls >= 0) ? ht_get_i(sm.ckey, sm.cval, cls) : INT32_MAX;
        const bool cdup = is_long && cls >= 0 && !ds && first < tid;   // a skip once its class failed
        unsigned long long shash = 0;
        if (is_long && !cdup) {
            shash = spec_hash(sp);
            ht_min_u(sm.skey, sm.sval, shash, tid);
        }
        __syncthreads();
        int32_t rep = -1;          // the earlier long pod with an equal record
        if (is_long && !cdup) {
            const int32_t f = ht_get_u(sm.skey, sm.sval, shash);
            if (f < tid && spec_equal(sp, a.specs + CK(a.ph[CK(a.order[CK(k0 + f, P)], a.n_pods)].spec, a.n_pods)))
                rep = f;
        }
        const bool uniq = is_long && !cdup && rep < 0;
        int32_t nu;
        const int32_t ui = fo_excl(sm, uniq ? 1 : 0, nu);
        if (uniq) sm.ulist[CK(ui, FO_T)] = (int16_t)tid;
        __syncthreads();
        int32_t b_long = INT32_MAX;
        for (int32_t x = 0; x < nu; x++) {
            const int32_t j = CK(sm.ulist[CK(x, FO_T)], FO_T);
            const PodHot pj = a.ph[CK(a.order[CK(k0 + j, P)], a.n_pods)];
            int32_t found;
            uint32_t evs;
            fo_ring_scan(a, sm, pj, a.specs[CK(pj.spec, a.n_pods)], CK(sm.lstart[j], n), found, evs);
            if (found >= 0) { b_long = j; break; }                                    // (a)
            if (tid == 0) sm.lev[j] = evs;
        }
        __syncthreads();
        b = min(b, b_long);
        // outcomes before b
        uint32_t lev = 0;
        if (is_long && tid < b && !cdup) lev = sm.lev[rep >= 0 ? rep : tid];
        const bool fail = tid < b && (pff || (is_long && !cdup));
        const bool marks = fail && cls >= 0 && !ds && first == tid;
        bool cut = false;
        if (marks && a.cls_capped[cls]) cut = true;                                     // (d)
        if (sfound && first < tid) cut = true;                                           // (e)
        const bool pskip = fail && !ds && cls >= 0 && first < tid;                       // class failed earlier
        b = min(b, fo_min(sm, (cut && tid < b) ? tid : INT32_MAX));
        // placements before b: claim the nodes, then check every pod's reads
        const int32_t place = (tid < b) ? (hint_ok ? h : (sfound ? fnode : -1)) : -1;
        if (place >= 0) atomicMax(&a.claim[CK(place, n)], claim_key(gen, tid));
        __builtin_amdgcn_s_waitcnt(0);         // the claims are performed before the barrier
        __syncthreads();
        bool coll = false;
        if (tid < b) {
            if (hint_ok) coll = claimed_before(a, h, gen, tid);
            if (sfound) {
                int32_t pos = start_ev;
                for (int32_t t = 0; t < n; t++) {
                    coll |= claimed_before(a, pos, gen, tid);
                    if (pos == fnode) break;
                    if (++pos == n) pos = 0;
#ifdef CASIM_FO_CHECKS
                    if (t == FO_SHORT_K) CK(-1 - t, 0);           // the short scan covers <= FO_SHORT_K
#endif
                }
            }
        }
        b = min(b, fo_min(sm, coll ? tid : INT32_MAX));                                  // (c)
        // commit the prefix [0, b)
        if (tid < b) {
            const int32_t node = hint_ok ? h : (sfound ? fnode : -1);
            a.out_node[k] = node;
            evals += ev + (sfound ? sev : 0) + ((fail && !pskip) ? lev : 0);
            if (node >= 0) {
                a.hints[k] = node;
                fo_place(a, p, s, node);
            }
            if (marks) a.cls_mark[CK(cls, a.n_classes)] = 1;
        }
        __builtin_amdgcn_s_waitcnt(0);         // row updates performed before the next reads
        const int32_t last = fo_max(sm, (tid < b && sfound) ? tid : -1);
        if (last >= 0) {
            if (tid == last) sm.bcast = fnode;
            __syncthreads();
            const int32_t f = CK(sm.bcast, n);
            L = (f + 1 == n) ? 0 : f + 1;
            any_success = true;
        }
        __syncthreads();
        if (b < nb) {
            const int32_t L0 = L;
            fo_single(a, sm, k0 + b, L, evals);
            if (L != L0) any_success = true;
            cuts++;
            k0 += b + 1;
        } else {
            k0 += nb;
        }
    }
    const unsigned long long tot = fo_sum64(sm, evals);
    if (tid == 0) {
        if (any_success) a.ctl->L = L;
        a.ctl->evals = tot;
        a.ctl->batches = batches;
        a.ctl->cuts = cuts;
    }
}

}  // namespace casim

using namespace casim;

extern "C" {

int ca_filter_out_schedulable(ca_mirror* m, const ca_pod_table* t, const ca_podset* s, const int32_t* order,
                              int32_t n, const int32_t* class_owner, int32_t n_classes, int32_t* hints,
                              int32_t* last_index, int32_t* out_node, int32_t* out_pod_id, int32_t* n_overflowing,
                              uint64_t* evals, int32_t* n_placed) {
    if (!m || !t || n < 0 || n_classes < 0 || !last_index || (n > 0 && !out_node)) return CA_EINVAL;
    if (s && (s->m != m || s->t.n_pods != t->n_pods)) return CA_EINVAL;
    const auto t0 = std::chrono::steady_clock::now();
    for (int32_t k = 0; k < n; k++) {
        const int32_t i = order ? order[k] : k;
        if (i < 0 || i >= t->n_pods) return CA_EINVAL;
        if (t->pods[i].similar_class >= n_classes) return CA_EINVAL;
    }
    if (n_overflowing) *n_overflowing = 0;
    if (n_placed) *n_placed = 0;
    FilterScratch& fo = m->fo;
    fo.kernel_ms = 0;
    fo.batches = fo.cuts = 0;
    if (n == 0) return CA_OK;
    CA_HIP_CHECK(hipSetDevice(m->device));
    int rc;
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    const DevPodTable* dp = s ? &s->t : nullptr;
    if (!dp) {
        if ((rc = fo.pods.upload(t->pods, t->n_pods, t->terms, t->n_terms, t->reqs, t->n_reqs, t->prefilter_names,
                                 t->n_prefilter_names, m->stream)) != CA_OK)
            return rc;
        dp = &fo.pods;
    }
    // similar-pods classes: controllers with more than maxPodsPerOwnerRef classes can hit the cap
    int32_t n_owners = 0;
    std::vector<uint8_t> capped((size_t)n_classes + 1, 0);
    if (class_owner) {
        for (int32_t c = 0; c < n_classes; c++) n_owners = std::max(n_owners, class_owner[c] + 1);
        std::vector<int32_t> per_owner((size_t)n_owners + 1, 0);
        for (int32_t c = 0; c < n_classes; c++) if (class_owner[c] >= 0) per_owner[class_owner[c]]++;
        for (int32_t c = 0; c < n_classes; c++)
            capped[c] = class_owner[c] >= 0 && per_owner[class_owner[c]] > FO_MAX_PER_OWNER;
    }
    const int32_t nn = (int32_t)m->nodes.size();
    // inputs: order | hints | class_owner | capped ; zeroed: ctl | claim | owner_cnt | cls_mark | owner_over
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_order = 0, o_hints = o_order + al(sizeof(int32_t) * n), o_owner = o_hints + al(sizeof(int32_t) * n),
                 o_capped = o_owner + al(sizeof(int32_t) * (n_classes + 1)), in_bytes = o_capped + al(n_classes + 1);
    const size_t z_ctl = 0, z_claim = al(sizeof(FoCtl)), z_ocnt = z_claim + al(sizeof(unsigned long long) * (nn + 1)),
                 z_mark = z_ocnt + al(sizeof(int32_t) * (n_owners + 1)), z_over = z_mark + al(n_classes + 1),
                 z_bytes = z_over + al(n_owners + 1);
    const size_t out_bytes = al(sizeof(int32_t) * n) * 2 + al(sizeof(FoCtl));
    if ((rc = fo.in.reserve(in_bytes)) != CA_OK || (rc = fo.h_in.reserve(in_bytes)) != CA_OK ||
        (rc = fo.zero.reserve(z_bytes)) != CA_OK || (rc = fo.out.reserve(out_bytes)) != CA_OK ||
        (rc = fo.h_out.reserve(out_bytes)) != CA_OK)
        return rc;
    char* hi = fo.h_in.as<char>();
    int32_t* h_order = reinterpret_cast<int32_t*>(hi + o_order);
    int32_t* h_hints = reinterpret_cast<int32_t*>(hi + o_hints);
    for (int32_t k = 0; k < n; k++) {
        h_order[k] = order ? order[k] : k;
        h_hints[k] = hints ? hints[k] : -1;
    }
    if (class_owner) std::memcpy(hi + o_owner, class_owner, sizeof(int32_t) * n_classes);
    std::memcpy(hi + o_capped, capped.data(), (size_t)n_classes);
    FoCtl ctl0;
    std::memset(&ctl0, 0, sizeof ctl0);
    ctl0.L = *last_index;
    char* di = fo.in.as<char>();
    char* dz = fo.zero.as<char>();
    char* dout = fo.out.as<char>();
    CA_HIP_CHECK(hipMemcpyAsync(di, hi, in_bytes, hipMemcpyHostToDevice, m->stream));
    CA_HIP_CHECK(hipMemsetAsync(dz, 0, z_bytes, m->stream));
    CA_HIP_CHECK(hipMemcpyAsync(dz + z_ctl, &ctl0, sizeof ctl0, hipMemcpyHostToDevice, m->stream));
    // hints are in/out: the kernel writes into a copy in the output block
    int32_t* d_hints = reinterpret_cast<int32_t*>(dout + al(sizeof(int32_t) * n));
    CA_HIP_CHECK(hipMemcpyAsync(d_hints, di + o_hints, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, m->stream));
    FoArgs a;
    a.hot = m->d_hot.as<NodeHot>();
    a.ext = m->d_ext.as<NodeExt>();
    a.st = m->d_static.as<const NodeStatic>();
    a.n = nn;
    a.ph = dp->hot.as<const PodHot>();
    a.specs = dp->spec.as<const ca_pod_spec>();
    a.terms = dp->terms.as<const ca_selector_term>();
    a.reqs = dp->reqs.as<const ca_selector_req>();
    a.names = dp->names.as<const int32_t>();
    a.order = reinterpret_cast<const int32_t*>(di + o_order);
    a.P = n;
    a.hints = d_hints;
    a.out_node = reinterpret_cast<int32_t*>(dout);
    a.cls_mark = reinterpret_cast<uint8_t*>(dz + z_mark);
    a.cls_capped = reinterpret_cast<const uint8_t*>(di + o_capped);
    a.cls_owner = class_owner ? reinterpret_cast<const int32_t*>(di + o_owner) : nullptr;
    a.owner_cnt = reinterpret_cast<int32_t*>(dz + z_ocnt);
    a.owner_over = reinterpret_cast<uint8_t*>(dz + z_over);
    a.claim = reinterpret_cast<unsigned long long*>(dz + z_claim);
    a.ctl = reinterpret_cast<FoCtl*>(dz + z_ctl);
    a.n_pods = dp->n_pods;
    a.n_classes = n_classes;
    a.n_owners = n_owners;
    CA_HIP_CHECK(hipEventRecord(m->ev0, m->stream));
    hipLaunchKernelGGL(k_filter_out, dim3(1), dim3(FO_T), 0, m->stream, a);
    CA_HIP_CHECK(hipGetLastError());
    CA_HIP_CHECK(hipEventRecord(m->ev1, m->stream));
    char* ho = fo.h_out.as<char>();
    CA_HIP_CHECK(hipMemcpyAsync(ho, dout, al(sizeof(int32_t) * n) + sizeof(int32_t) * n, hipMemcpyDeviceToHost,
                                m->stream));
    FoCtl* hctl = reinterpret_cast<FoCtl*>(ho + al(sizeof(int32_t) * n) * 2);
    CA_HIP_CHECK(hipMemcpyAsync(hctl, a.ctl, sizeof(FoCtl), hipMemcpyDeviceToHost, m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    CA_HIP_CHECK(hipEventElapsedTime(&fo.kernel_ms, m->ev0, m->ev1));
    if (hctl->bad_line) {
        set_last_error("k_filter_out: index check failed at filter.hip:" + std::to_string(hctl->bad_line) +
                       " (value " + std::to_string(hctl->bad_val) + ")");
        return CA_EDEVICE;
    }
    const int32_t* nodes_out = reinterpret_cast<const int32_t*>(ho);
    const int32_t* hints_out = reinterpret_cast<const int32_t*>(ho + al(sizeof(int32_t) * n));
    // AddPod of every placed pod on the host rows, in the reference's order
    int32_t placed = 0;
    for (int32_t k = 0; k < n; k++) {
        const int32_t node = nodes_out[k];
        out_node[k] = node;
        if (hints) hints[k] = hints_out[k];
        if (node >= 0) {
            const int32_t id = m->store_pod(t, h_order[k], node);
            m->add_pod_to_node(id, node);
            if (out_pod_id) out_pod_id[k] = id;
            placed++;
        } else if (out_pod_id) {
            out_pod_id[k] = -1;
        }
    }
    *last_index = hctl->L;
    if (evals) *evals += hctl->evals;
    if (n_overflowing) *n_overflowing = hctl->overflowing;
    fo.batches = hctl->batches;
    fo.cuts = hctl->cuts;
    fo.total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (n_placed) *n_placed = placed;
    return CA_OK;
}

int ca_filter_stats(const ca_mirror* m, float* out, int32_t cap) {
    if (!m || (!out && cap > 0)) return CA_EINVAL;
    const float v[4] = {m->fo.kernel_ms, m->fo.total_ms, (float)m->fo.batches, (float)m->fo.cuts};
    for (int32_t i = 0; i < cap && i < 4; i++) out[i] = v[i];
    return 4;
}

}  // extern "C"
