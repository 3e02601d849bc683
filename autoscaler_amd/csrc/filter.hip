// filter.hip — FilterOutSchedulable: HintingSimulator.TrySchedulePods(pending pods,
// ScheduleAnywhere, breakOnFailure=false), committed into the mirror.
//
// Reference: CA/core/podlistprocessor/filter_out_schedulable.go:95-124,
// CA/simulator/scheduling/hinting_simulator.go:58-125 (findNodeWithHints / findNode),
// CA/simulator/scheduling/similar_pods.go:43-111 (the per-call unschedulable cache),
// CA/simulator/predicatechecker/schedulerbased.go:103-137 (FitsAnyNodeMatching's rotating
// scan from lastIndex) and :139-185 (CheckPredicates).
//
// The reference is one sequential loop: a pod's scan starts where the previous successful
// scan stopped (lastIndex) and sees every earlier placement, so the pods are walked in
// order.  One workgroup (SQ_W = 8 waves of SQ_T = 512 threads) owns the node rows for the whole call:
//   window     the SQ_WIN node rows from lastIndex on (hot, ext and static columns) live
//              in LDS, updated there by the placements and written back when the window
//              moves.  Consecutive scans continue where the previous one stopped, so the
//              cursor walks the window and most scans never leave it;
//   slots      the next SQ_SLOTS pods are staged in LDS: PodHot, the full record, the
//              similar-pods mark of their class and a copy of their hinted node's rows;
//   sequencer  wave 0 walks the staged pods: the hint check on the window row (or the
//              staged copy), the similar-pods skip, then the scan over the window rows,
//              64 positions per step (ballot of visible / fits: first fit wins, the
//              evaluations are the visible positions up to it);
//   block step when a scan runs off the window (or the slots are used up, or a class
//              must be marked) all 8 waves take over: write back, scan the rest of the
//              ring in parallel (SQ_RING positions in flight per thread, first fit by a
//              min reduction), place or mark, reload the window at lastIndex and the slots.
// Every pod's outcome, lastIndex and the evaluation count are exactly the reference loop's.
#include "mirror.h"
#include "device_filters.h"

#include <algorithm>
#include <chrono>
#include <unordered_map>
#include <cstddef>
#include <cstring>
#include <string>

namespace casim {

constexpr int SQ_T = 512;              // threads: wave 0 sequences, all waves run the block steps
constexpr int SQ_W = SQ_T / 64;
constexpr int SQ_WIN = 512;            // node positions resident in LDS
constexpr int SQ_SLOTS = 64;           // pods staged per phase (one per sequencer lane)
constexpr int SQ_RING = 16;            // positions per thread per pass of the block-wide ring scan
constexpr int FO_MAX_PER_OWNER = 10;   // maxPodsPerOwnerRef, similar_pods.go:53

enum : int32_t { CMD_DONE = 0, CMD_PHASE = 1, CMD_WINDOW = 2, CMD_RING = 3, CMD_MARK = 4 };

struct FoCtl {
    int32_t L;                 // lastIndex in/out
    int32_t overflowing;       // controllers that overflowed the class cap
    int32_t phases, steps;     // slot phases, block steps
    unsigned long long evals;
    int32_t ring_scans, windows;
    int32_t bad_line, bad_val; // CASIM_FO_CHECKS builds: the first index check that failed
    unsigned long long seq_cycles, all_cycles;   // CASIM_PROF builds: wave 0's walk, the whole kernel
    unsigned long long fb_cyc[4];                 // CASIM_PROF builds, bitmap walk: hint, scan, place, batch loads
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

struct SqSmem {
    NodeHot win_hot[SQ_WIN];
    NodeExt win_ext[SQ_WIN];
    NodeStatic win_st[SQ_WIN];
    NodeHot slot_hot[SQ_SLOTS];
    NodeExt slot_ext[SQ_SLOTS];
    NodeStatic slot_st[SQ_SLOTS];
    ca_pod_spec slot_spec[SQ_SLOTS];
    PodHot slot_ph[SQ_SLOTS];
    int32_t slot_node[SQ_SLOTS];     // hinted node position, -1 none
    int32_t slot_cls[SQ_SLOTS];
    int32_t slot_out[SQ_SLOTS];      // node of the walked pod, -1 (flushed to HBM per phase)
    uint8_t slot_mark[SQ_SLOTS];     // the class is marked unschedulable
    uint8_t slot_dirty[SQ_SLOTS];
    uint8_t win_dirty[SQ_WIN];
    int32_t L, wb, wn, cur;          // lastIndex; window start position and length; cursor offset
    int32_t k0, ns, j;               // phase: first pod, staged pods, next slot
    int32_t cmd, arg;                // block step the sequencer asks for
    int32_t succ;                    // some scan succeeded (lastIndex moved)
    uint32_t carry;                  // CMD_RING: evaluations of the window part of the scan
    int32_t red_i[SQ_W];
};

// ---- block primitives (all threads, uniform control flow) -----------------------
__device__ inline int32_t sq_min(SqSmem& sm, int32_t v) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if (lane == 0) sm.red_i[w] = v;
    __syncthreads();
    int32_t m = INT32_MAX;
    for (int k = 0; k < SQ_W; k++) m = min(m, sm.red_i[k]);
    return m;
}
__device__ inline int32_t sq_sum(SqSmem& sm, int32_t v) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) sm.red_i[w] = v;
    __syncthreads();
    int32_t s = 0;
    for (int k = 0; k < SQ_W; k++) s += sm.red_i[k];
    return s;
}

// The mutable columns (hot, ext), the marks and the counters are read with device-coherent
// loads: a uniform plain load may be served from the scalar cache, which the kernel's own
// vector stores do not update, and the coherent form also skips a stale vector-L1 line.
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

// ---- filters ------------------------------------------------------------------------
// FitsAnyNodeMatching visits the node (schedulerbased.go:116-127): PreFilter's NodeNames
// and Spec.Unschedulable skip a node without running the filters
__device__ inline bool sq_visible(const FoArgs& a, const PodHot& p, const ca_pod_spec& s, const NodeHot& h,
                                  const NodeStatic& st) {
    if (h.flags & NF_UNSCHED) return false;
    if (p.flags & PF_PREFILTER_NAMES) {
        bool ok = false;
        for (int32_t k = 0; k < s.prefilter_count; k++) ok |= a.names[s.prefilter_first + k] == st.name_id;
        return ok;
    }
    return true;
}
__device__ inline bool sq_fits(const FoArgs& a, const PodHot& p, const ca_pod_spec& s, const NodeHot& h,
                               const NodeExt* e, const NodeStatic* st, bool apply_unsched) {
    uint32_t r;
    return dev_full_filters(s, p, a.terms, a.reqs, h, e, st, apply_unsched, &r) == CA_PLUGIN_NONE;
}

// AddPod's resource / port update (NodeInfo.AddPod, SF/types.go:672-692) on one row
__device__ inline void sq_place_row(NodeHot& h, NodeExt& e, const PodHot& p, const ca_pod_spec& s) {
    h.cpu = wsub(h.cpu, p.cpu);
    h.mem = wsub(h.mem, p.mem);
    h.eph = wsub(h.eph, p.eph);
    h.pods = h.pods - 1;
    uint64_t pu = 0;
    if (p.flags & PF_PORTS)                   // PF_PORTS clear: port_use is empty (no LDS read)
        for (int w = 0; w < CA_PORT_WORDS; w++) pu |= s.port_use[w];
    if (pu || (p.flags & PF_SCALAR_REQ)) {
        for (int w = 0; w < CA_PORT_WORDS; w++) e.ports[w] |= s.port_use[w];
        for (int k = 0; k < CA_MAX_SCALAR; k++) e.scalar[k] = wsub(e.scalar[k], s.req_scalar[k]);
        if (pu) h.flags |= NF_PORTS;
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

// ---- block steps ----------------------------------------------------------------------
// dirty window rows and staged copies back to HBM
__device__ __attribute__((always_inline)) void sq_write_back(const FoArgs& a, SqSmem& sm) {
    const int32_t n = a.n, wb = sm.wb, wn = sm.wn;
    for (int32_t o = (int32_t)threadIdx.x; o < wn; o += SQ_T) {
        if (sm.win_dirty[o]) {
            int32_t pos = wb + o;
            if (pos >= n) pos -= n;
            pos = CK(pos, n);
            a.hot[pos] = sm.win_hot[o];
            a.ext[pos] = sm.win_ext[o];
            sm.win_dirty[o] = 0;
        }
    }
    const int32_t t = (int32_t)threadIdx.x;
    if (t < sm.ns && sm.slot_dirty[t]) {
        const int32_t pos = CK(sm.slot_node[t], n);
        a.hot[pos] = sm.slot_hot[t];          // every dirty copy of a node holds the same row
        a.ext[pos] = sm.slot_ext[t];
        sm.slot_dirty[t] = 0;
    }
    __threadfence();                          // the rows are in L2 before any coherent re-read
    __syncthreads();
}

// the window: SQ_WIN rows from position L (all three columns)
__device__ __attribute__((always_inline)) void sq_load_window(const FoArgs& a, SqSmem& sm, int32_t L) {
    const int32_t n = a.n;
    const int32_t wn = min(SQ_WIN, n);
    for (int32_t o = (int32_t)threadIdx.x; o < wn; o += SQ_T) {
        int32_t pos = L + o;
        if (pos >= n) pos -= n;
        pos = CK(pos, n);
        sm.win_hot[o] = ld_hot_coh(a.hot + pos);
        sm.win_ext[o] = ld_ext_coh(a.ext + pos);
        sm.win_st[o] = a.st[pos];
        sm.win_dirty[o] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        sm.wb = L;
        sm.wn = wn;
        sm.cur = 0;
    }
    __syncthreads();
}

// stage pods k0 .. k0+ns-1 (full: their records too; else only the hinted rows and marks
// of the slots from sm.j on)
__device__ __attribute__((always_inline)) void sq_load_slots(const FoArgs& a, SqSmem& sm, bool full) {
    const int32_t t = (int32_t)threadIdx.x;
    const int32_t n = a.n;
    if (full) {
        // order -> PodHot once per slot, then every spec word in flight at once (one
        // dependent HBM round trip each instead of three per word batch)
        constexpr int SW = (int)(sizeof(ca_pod_spec) / 8);
        static_assert(sizeof(ca_pod_spec) % 8 == 0, "ca_pod_spec words");
        constexpr int PER = (SQ_SLOTS * SW + SQ_T - 1) / SQ_T;
        if (t < sm.ns) sm.slot_ph[t] = a.ph[CK(a.order[CK(sm.k0 + t, a.P)], a.n_pods)];
        __syncthreads();
        const int32_t words = sm.ns * SW;
        unsigned long long v[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int32_t x = t + q * SQ_T;
            if (x < words) {
                const int32_t j = x / SW, w = x % SW;
                v[q] = reinterpret_cast<const unsigned long long*>(a.specs + CK(sm.slot_ph[j].spec, a.n_pods))[w];
            }
        }
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int32_t x = t + q * SQ_T;
            if (x < words) reinterpret_cast<unsigned long long*>(&sm.slot_spec[x / SW])[x % SW] = v[q];
        }
        __syncthreads();
    }
    if (t >= sm.j && t < sm.ns) {
        const int32_t k = sm.k0 + t;
        const int32_t h = a.hints[CK(k, a.P)];
        const int32_t node = (h >= 0 && h < n) ? h : -1;
        sm.slot_node[t] = node;
        if (node >= 0) {
            sm.slot_hot[t] = ld_hot_coh(a.hot + node);
            sm.slot_ext[t] = ld_ext_coh(a.ext + node);
            sm.slot_st[t] = a.st[node];
        }
        const int32_t c = sm.slot_spec[t].similar_class;
        sm.slot_cls[t] = c;
        sm.slot_mark[t] = (c >= 0) ? ld_mark(&a.cls_mark[CK(c, a.n_classes)]) : 0;
        sm.slot_dirty[t] = 0;
    }
    __syncthreads();
}

// the rest of a pod's ring: R positions from X, block-wide.  First fitting offset (-1:
// none) and the visible positions up to it (every visible position if none fits).
__device__ __attribute__((always_inline)) void sq_ring_scan(const FoArgs& a, SqSmem& sm, const PodHot& p, const ca_pod_spec& s, int32_t X,
                             int32_t R, int32_t& found, uint32_t& evs) {
    const int32_t n = a.n;
    found = -1;
    evs = 0;
    for (int32_t base = 0; base < R; base += SQ_T * SQ_RING) {
        uint32_t vis = 0, fit = 0;
#pragma unroll
        for (int i = 0; i < SQ_RING; i++) {
            const int32_t off = base + i * SQ_T + (int32_t)threadIdx.x;
            if (off < R) {
                int32_t pos = X + off;
                if (pos >= n) pos -= n;
                pos = CK(pos, n);
                const NodeHot h = ld_hot_coh(a.hot + pos);
                const bool v = sq_visible(a, p, s, h, a.st[pos]);
                vis |= (uint32_t)v << i;
                if (v) {
                    bool ok;
                    if (((p.flags & PF_PORTS) && (h.flags & NF_PORTS)) || (p.flags & PF_SCALAR_REQ)) {
                        const NodeExt e = ld_ext_coh(a.ext + pos);
                        ok = sq_fits(a, p, s, h, &e, a.st + pos, false);
                    } else {
                        ok = sq_fits(a, p, s, h, a.ext + pos, a.st + pos, false);   // ext unread
                    }
                    if (ok) fit |= 1u << i;
                }
            }
        }
        // offsets of this thread are base + i * SQ_T + tid, increasing in i
        const int32_t mine = fit ? base + __builtin_ctz(fit) * SQ_T + (int32_t)threadIdx.x : INT32_MAX;
        const int32_t f = sq_min(sm, mine);
        int32_t cnt = 0;
#pragma unroll
        for (int i = 0; i < SQ_RING; i++) {
            const int32_t off = base + i * SQ_T + (int32_t)threadIdx.x;
            cnt += (((vis >> i) & 1u) && off <= f) ? 1 : 0;
        }
        evs += (uint32_t)sq_sum(sm, cnt);
        if (f != INT32_MAX) {
            found = f;
            break;
        }
    }
}

// ---- the sequencer (wave 0) ----------------------------------------------------------
// Walks slots sm.j .. sm.ns-1 and stops at the first pod that needs a block step.
__device__ __attribute__((always_inline)) void sq_sequence(const FoArgs& a, SqSmem& sm, unsigned long long& evals) {
    const int lane = (int)threadIdx.x;       // wave 0
    const int32_t n = a.n, ns = sm.ns, k0 = sm.k0;
    const int32_t wb = sm.wb, wn = sm.wn;
    int32_t j = sm.j, L = sm.L, cur = sm.cur;
    bool succ = false;
    int32_t cmd = (k0 + ns >= a.P) ? CMD_DONE : CMD_PHASE, arg = 0;
    // lane l holds slot l's scalars; the walk reads them with readlane (no LDS round trip)
    const int ll = lane < ns ? lane : 0;
    const PodHot lp = sm.slot_ph[ll];
    const int32_t l_node = sm.slot_node[ll], l_cls = sm.slot_cls[ll];
    const int32_t l_mark = sm.slot_mark[ll];
    for (; j < ns; j++) {
        if (n > 0 && cur >= wn) { cmd = CMD_WINDOW; break; }   // the cursor ran off the window
        PodHot p;
        p.cpu = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lp.cpu >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)lp.cpu, j));
        p.mem = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lp.mem >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)lp.mem, j));
        p.eph = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lp.eph >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)lp.eph, j));
        p.flags = (uint32_t)__builtin_amdgcn_readlane((int)lp.flags, j);
        p.spec = 0;
        const ca_pod_spec& s = sm.slot_spec[j];
        const uint32_t pf = p.flags;
        const int32_t h = __builtin_amdgcn_readlane(l_node, j);
        int32_t node = -1;
        if (h >= 0 && !(pf & PF_PREFILTER_FAIL)) {            // findNodeWithHints (:91-108)
            if (lane == 0) evals++;
            int32_t ho = h - wb;
            if (ho < 0) ho += n;
            const bool inw = ho < wn;
            bool ok;
            if (inw) ok = sq_fits(a, p, s, sm.win_hot[ho], &sm.win_ext[ho], &sm.win_st[ho], true);
            else ok = sq_fits(a, p, s, sm.slot_hot[j], &sm.slot_ext[j], &sm.slot_st[j], true);
            if (ok) {
                node = h;
                if (inw) {
                    if (lane == 0) {
                        sq_place_row(sm.win_hot[ho], sm.win_ext[ho], p, s);
                        sm.win_dirty[ho] = 1;
                    }
                } else if (lane < ns && sm.slot_node[lane] == h) {
                    // every live staged copy of the node takes the pod; the copies of the slots
                    // already walked are superseded (never read again, never written back)
                    if (lane >= j) {
                        sq_place_row(sm.slot_hot[lane], sm.slot_ext[lane], p, s);
                        sm.slot_dirty[lane] = 1;
                    } else {
                        sm.slot_dirty[lane] = 0;
                    }
                }
            }
        }
        if (node < 0 && !__builtin_amdgcn_readlane(l_mark, j)) {   // findNode (:110-125)
            const int32_t c = __builtin_amdgcn_readlane(l_cls, j);
            const bool can_mark = c >= 0 && !(pf & PF_DAEMONSET);
            if ((pf & PF_PREFILTER_FAIL) || n == 0) {          // fails without a scan
                if (can_mark) {
                    if (lane == 0) sm.slot_out[j] = -1;
                    cmd = CMD_MARK;
                    arg = j++;
                    break;
                }
            } else {
                // the scan over the window from the cursor, 64 positions a step
                uint32_t ev = 0;
                int32_t fo = -1;
                const int32_t lim = (wn == n) ? cur + n : wn;     // whole ring resident: wrap inside
                for (int32_t base = cur; base < lim; base += 64) {
                    int32_t o = base + lane;
                    bool vis = false, fit = false;
                    if (o < lim) {
                        if (o >= wn) o -= wn;
                        const NodeHot hh = sm.win_hot[o];
                        vis = sq_visible(a, p, s, hh, sm.win_st[o]);
                        fit = vis && sq_fits(a, p, s, hh, &sm.win_ext[o], &sm.win_st[o], false);
                    }
                    const unsigned long long fm = __ballot(fit), vm = __ballot(vis);
                    if (fm) {
                        const int l = __builtin_ctzll(fm);
                        ev += (uint32_t)__builtin_popcountll(vm & ((2ull << l) - 1ull));
                        fo = base + l;
                        if (fo >= wn) fo -= wn;
                        break;
                    }
                    ev += (uint32_t)__builtin_popcountll(vm);
                }
                if (fo >= 0) {
                    if (lane == 0) {
                        evals += ev;
                        sq_place_row(sm.win_hot[fo], sm.win_ext[fo], p, s);
                        sm.win_dirty[fo] = 1;
                    }
                    int32_t f = wb + fo;
                    if (f >= n) f -= n;
                    node = f;
                    L = (f + 1 == n) ? 0 : f + 1;                 // schedulerbased.go:131
                    succ = true;
                    cur = fo + 1;
                    if (wn == n && cur == n) cur = 0;            // whole ring resident: keep walking
                } else if (wn == n) {                            // the whole ring: no node fits
                    if (lane == 0) evals += ev;
                    if (can_mark) {
                        if (lane == 0) sm.slot_out[j] = -1;
                        cmd = CMD_MARK;
                        arg = j++;
                        break;
                    }
                } else {                                         // the rest of the ring: block step
                    if (lane == 0) sm.carry = ev;
                    cmd = CMD_RING;
                    arg = j;
                    break;
                }
            }
        }
        if (lane == 0) sm.slot_out[j] = node;
    }
    if (lane == 0) {
        sm.j = j;
        sm.L = L;
        sm.cur = cur;
        sm.cmd = cmd;
        sm.arg = arg;
        if (succ) sm.succ = 1;
    }
}

// the phase's outcomes to HBM: out_node, and Hints.Set (:95, :123) for the placed pods
__device__ inline void sq_flush(const FoArgs& a, SqSmem& sm) {
    const int32_t t = (int32_t)threadIdx.x;
    if (t < sm.ns) {
        const int32_t k = CK(sm.k0 + t, a.P), node = sm.slot_out[t];
        a.out_node[k] = node;
        if (node >= 0) a.hints[k] = node;
    }
}

__global__ void __launch_bounds__(SQ_T) k_filter_out(FoArgs a) {
    __shared__ SqSmem sm;
    const int32_t tid = (int32_t)threadIdx.x;
    const int32_t n = a.n;
    unsigned long long evals = 0;           // thread 0 (= the sequencer's lane 0)
    int32_t phases = 1, steps = 0, rings = 0, windows = 0;
    unsigned long long seq_cyc = 0;
#ifdef CASIM_PROF
    const unsigned long long k_c0 = clock64();
#endif
    if (tid == 0) {
        int32_t L0 = (n > 0) ? a.ctl->L % n : 0;
        if (L0 < 0) L0 += n;
        sm.L = L0;
        sm.k0 = 0;
        sm.ns = min(SQ_SLOTS, a.P);
        sm.j = 0;
        sm.succ = 0;
        sm.wb = 0;
        sm.wn = 0;
        sm.cur = 0;
    }
    __syncthreads();
    if (n > 0) sq_load_window(a, sm, sm.L);
    sq_load_slots(a, sm, true);
    while (true) {
#ifdef CASIM_PROF
        const unsigned long long c0 = clock64();
#endif
        if (tid < 64) sq_sequence(a, sm, evals);
#ifdef CASIM_PROF
        if (tid == 0) seq_cyc += clock64() - c0;
#endif
        __syncthreads();
        const int32_t cmd = sm.cmd;
        if (cmd != CMD_DONE) steps++;
        if (cmd == CMD_MARK) {
            const int32_t c = sm.slot_cls[sm.arg];
            if (tid == 0) fo_mark(a, c);
            __threadfence();
            __syncthreads();
            if (tid < sm.ns && sm.slot_cls[tid] == c) sm.slot_mark[tid] = ld_mark(&a.cls_mark[CK(c, a.n_classes)]);
            __syncthreads();
            continue;
        }
        if (n > 0) sq_write_back(a, sm);
        if (cmd == CMD_DONE || cmd == CMD_PHASE) sq_flush(a, sm);
        if (cmd == CMD_DONE) break;
        if (cmd == CMD_PHASE) {
            __syncthreads();
            if (tid == 0) {
                sm.k0 += sm.ns;
                sm.ns = min(SQ_SLOTS, a.P - sm.k0);
                sm.j = 0;
            }
            __syncthreads();
            phases++;
            sq_load_slots(a, sm, true);
            continue;
        }
        if (cmd == CMD_RING) {
            rings++;
            const int32_t j = sm.arg;
            const PodHot p = sm.slot_ph[j];
            const ca_pod_spec& s = sm.slot_spec[j];
            int32_t X = sm.wb + sm.wn;
            if (X >= n) X -= n;
            const int32_t R = n - (sm.wn - sm.cur);
            int32_t found;
            uint32_t ev;
            sq_ring_scan(a, sm, p, s, X, R, found, ev);
            const int32_t c = sm.slot_cls[j];
            if (found >= 0) {
                int32_t f = X + found;
                if (f >= n) f -= n;
                f = CK(f, n);
                if (tid == 0) {
                    NodeHot hr = ld_hot_coh(a.hot + f);
                    NodeExt he = ld_ext_coh(a.ext + f);
                    sq_place_row(hr, he, p, s);
                    a.hot[f] = hr;
                    a.ext[f] = he;
                    sm.slot_out[j] = f;
                    evals += sm.carry + ev;
                    sm.L = (f + 1 == n) ? 0 : f + 1;
                    sm.succ = 1;
                    sm.j = j + 1;
                }
                __threadfence();
                __syncthreads();
                windows++;
                sq_load_window(a, sm, sm.L);
                sq_load_slots(a, sm, false);
            } else {
                if (tid == 0) {
                    evals += sm.carry + ev;
                    sm.slot_out[j] = -1;
                    if (c >= 0 && !(p.flags & PF_DAEMONSET)) fo_mark(a, c);
                    sm.j = j + 1;
                }
                __threadfence();
                __syncthreads();
                if (c >= 0 && tid < sm.ns && sm.slot_cls[tid] == c)
                    sm.slot_mark[tid] = ld_mark(&a.cls_mark[CK(c, a.n_classes)]);
                __syncthreads();
            }
            continue;
        }
        // CMD_WINDOW: the cursor left the window
        windows++;
        sq_load_window(a, sm, sm.L);
        sq_load_slots(a, sm, false);
    }
    if (tid == 0) {
        if (sm.succ) a.ctl->L = sm.L;       // lastIndex moves only with a successful scan
        a.ctl->evals = evals;
        a.ctl->phases = phases;
        a.ctl->seq_cycles = seq_cyc;
#ifdef CASIM_PROF
        a.ctl->all_cycles = clock64() - k_c0;
#endif
        a.ctl->steps = steps;
        a.ctl->ring_scans = rings;
        a.ctl->windows = windows;
    }
}


// ===========================================================================================
// Feasibility-bitmap walk (the fast path).  For pending pods without host ports, scalar
// requests or PreFilter NodeNames, a filter verdict factors into
//   static[c][node]  TaintToleration, NodeAffinity, NodeName (node attributes: fixed for the
//                    call; c = the pod's static class, -1 when every node passes),
//   dyn[s][node]     NodeResourcesFit of the pod's resource shape s on the node's current
//                    free resources (changes only on the nodes that take a placement),
//   vis[node]        !Spec.Unschedulable (FitsAnyNodeMatching skips such nodes unfiltered,
//                    schedulerbased.go:125-127; CheckPredicates runs NodeUnschedulable).
// One bit per node, so FitsAnyNodeMatching's rotating first fit from lastIndex is a
// first-set-bit search over (dyn & static & vis) words from bit L — 64 words (4096 nodes)
// per wave step — and its evaluation count is the popcount of vis over the scanned range.
//
// Runs: the pods of one controller variant come in a row (same shape, static class,
// similar class and flags).  Without hints, k consecutive such pods take the first k
// set bits of (dyn & static & vis) from L — pod t's scan starts right after pod t-1's
// node and the placements behind it cannot change the nodes ahead — so one wave step
// finds a whole run's nodes (a prefix sum of per-word popcounts across the lanes), the
// placements update k rows in parallel lanes, and the evaluation count of the run is the
// visible nodes from L to the last node (prefix counts of vis, which the walk never
// changes).  A run stops at the end of one ring pass (the next pod then rescans the
// updated state), at a hinted pod, and at the end of the 64-pod batch.  A hinted pod's
// hint is checked alone (CheckPredicates); if it fails, its scan starts a run.
// Node rows: read from HBM (the hinted nodes' rows prefetched when a batch is loaded),
// written to an LDS buffer with a dirty bit per node, and flushed to HBM once per batch —
// a global store inside the batch would make every later load wait for it.
// ===========================================================================================
constexpr int FB_MAX_SHAPES = 64;        // one lane per shape for the bit updates
constexpr int FB_COLLECT_SHAPES = 1024;  // distinct shapes looked at before the dead ones are merged
constexpr int FB_T = 64;                 // the walk is one wavefront
#ifndef CASIM_FB_ROWWISE_MAX
#define CASIM_FB_ROWWISE_MAX 24
#endif
#ifndef CASIM_FB_BACKOFF
#define CASIM_FB_BACKOFF 1
#endif
constexpr int FB_ROWWISE_MAX = CASIM_FB_ROWWISE_MAX;   // mixed runs shorter than this update the bitmaps row by row
constexpr int FB_BACKOFF = CASIM_FB_BACKOFF;           // pods a short mixed run (< 2 placed) skips before the next try
constexpr size_t FB_LDS_MAX = 160 * 1024;

struct alignas(16) FbPod {               // per pending position (the walk order)
    int32_t shape, scls, simcls;         // resource shape, static class (-1: passes everywhere), similar class
    uint32_t flags;                      // PF_* (TOL_UNSCHED, PREFILTER_FAIL, DAEMONSET)
};
struct alignas(16) FbShape {
    int64_t cpu, mem, eph;
    uint32_t flags;                      // PF_ALL_ZERO
    int32_t pad;
};
struct alignas(16) FbRow {               // a placed node's new free resources (run scratch)
    int64_t cpu, mem, eph;
    int32_t pods, pad;
};
static_assert(sizeof(FbRow) == 32, "FbRow must be 32 B");

// Which shapes fit a row, for 64 shapes at once: per resource the shapes' distinct requests
// sorted, and for each count k of them the shapes whose request is at most the k-th
// (fit = pods >= 1 && (all-zero || cpu, mem and eph each within the row)).
struct alignas(16) FbThr {
    int64_t v[3][64];                    // distinct requests (cpu, mem, eph), ascending
    uint64_t t[3][65];                   // t[d][k]: shapes whose request d <= v[d][k-1] (t[d][0] = 0)
    int32_t u[3], pad;                   // distinct values per resource
    uint64_t zero;                       // PF_ALL_ZERO shapes
};

struct FbArgs {
    NodeHot* hot;
    int32_t n, nwords, P, S, K, n_classes, n_owners, stat_in_lds;
    const FbPod* pods;
    const FbShape* shapes;
    const FbThr* thr;
    const uint64_t* dyn0;                // [S][nwords] initial dyn words (copied into LDS)
    const uint64_t* vis0;                // [nwords]
    const uint64_t* stat;                // [K][nwords] (copied into LDS when stat_in_lds)
    int32_t* hints;                      // per position, in/out
    int32_t* out_node;
    uint8_t* cls_mark;                   // per similar class: the marks at the end (for the caller)
    const uint8_t* cls_capped;
    const int32_t* cls_owner;
    FoCtl* ctl;
};

// LDS layout of k_fb_walk, shared by the host sizing and the kernel
struct FbLds {
    size_t shapes, dyn, vis, stat, vpre, slot, bufrow, bufnode, dirty, ocnt, marks, oover, thr, total;
};
__host__ __device__ inline size_t fb_a16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline FbLds fb_lds(int32_t S, int32_t NW, int32_t K, int32_t stat_in_lds, int32_t n_classes,
                                        int32_t n_owners) {
    FbLds l;
    l.shapes = 0;
    l.dyn = l.shapes + sizeof(FbShape) * (size_t)(S > 0 ? S : 1);
    l.vis = l.dyn + sizeof(uint64_t) * (size_t)S * NW;
    l.stat = l.vis + sizeof(uint64_t) * (size_t)NW;
    l.vpre = l.stat + (stat_in_lds ? sizeof(uint64_t) * (size_t)K * NW : 0);
    l.slot = l.vpre + fb_a16(sizeof(int32_t) * (size_t)(NW + 1));
    l.bufrow = l.slot + sizeof(int32_t) * FB_T;
    l.bufnode = l.bufrow + sizeof(FbRow) * FB_T;
    l.dirty = l.bufnode + sizeof(int32_t) * FB_T;
    l.ocnt = l.dirty + sizeof(uint64_t) * (size_t)NW;
    l.marks = l.ocnt + fb_a16(sizeof(int32_t) * (size_t)(n_owners > 0 ? n_owners : 1));
    l.oover = l.marks + fb_a16((size_t)(n_classes > 0 ? n_classes : 1));
    l.thr = l.oover + fb_a16((size_t)(n_owners > 0 ? n_owners : 1));
    l.total = l.thr + sizeof(FbThr);
    return l;
}

// shape s fits the free resources (cpu, mem, eph, pods): dev_fit_reasons without scalars
__host__ __device__ inline bool fb_fit(const FbShape& sh, int64_t cpu, int64_t mem, int64_t eph, int32_t pods) {
    if (pods < 1) return false;                                           // fit.go:256-265
    if (sh.flags & PF_ALL_ZERO) return true;                             // :267-272
    return sh.cpu <= cpu && sh.mem <= mem && sh.eph <= eph;              // :274-300
}

// the shapes (of the first 64) that fit the free resources: fb_fit for all of them at once
__device__ inline uint64_t fb_fit_mask(const FbThr& t, int64_t cpu, int64_t mem, int64_t eph, int32_t pods) {
    if (pods < 1) return 0ull;
    const int64_t x[3] = {cpu, mem, eph};
    int32_t k[3] = {0, 0, 0};
#pragma unroll
    for (int st = 64; st; st >>= 1)
#pragma unroll
        for (int d = 0; d < 3; d++)
            if (k[d] + st <= t.u[d] && t.v[d][k[d] + st - 1] <= x[d]) k[d] += st;
    return t.zero | (t.t[0][k[0]] & t.t[1][k[1]] & t.t[2][k[2]]);
}

// dyn[s][w] and vis[w] for every word of every shape: block (word chunk, shape)
__global__ void __launch_bounds__(256) k_fb_dyn(const NodeHot* __restrict__ hot, int32_t n, int32_t nwords,
                                               const FbShape* __restrict__ shapes, int32_t S,
                                               uint64_t* __restrict__ dyn, uint64_t* __restrict__ vis) {
    const int32_t node = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int32_t s = (int32_t)blockIdx.y;                    // s == S: the visibility words
    bool b = false;
    if (node < n) {
        const NodeHot h = hot[node];
        b = s < S ? fb_fit(shapes[s], h.cpu, h.mem, h.eph, h.pods) : !(h.flags & NF_UNSCHED);
    }
    const uint64_t m = __ballot(b);
    const int32_t w = node >> 6;
    if ((threadIdx.x & 63) == 0 && w < nwords) {
        if (s < S) dyn[(size_t)s * nwords + w] = m;
        else vis[w] = m;
    }
}

// static[c][w]: TaintToleration / NodeAffinity / NodeName of class c's representative pod
__global__ void __launch_bounds__(256) k_fb_stat(const NodeStatic* __restrict__ st, int32_t n, int32_t nwords,
                                                const int32_t* __restrict__ rep, const PodHot* __restrict__ ph,
                                                const ca_pod_spec* __restrict__ specs,
                                                const ca_selector_term* __restrict__ terms,
                                                const ca_selector_req* __restrict__ reqs, uint64_t* __restrict__ stat) {
    const int32_t node = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int32_t c = (int32_t)blockIdx.y;
    bool b = false;
    if (node < n) {
        const PodHot p = ph[rep[c]];
        b = dev_static_filters(specs[p.spec], p.flags, terms, reqs, st[node], false) == CA_PLUGIN_NONE;
    }
    const uint64_t m = __ballot(b);
    const int32_t w = node >> 6;
    if ((threadIdx.x & 63) == 0 && w < nwords) stat[(size_t)c * nwords + w] = m;
}

__device__ inline uint64_t bits_from(int b) { return b >= 64 ? 0ull : (~0ull << b); }   // bits >= b
__device__ inline uint64_t bits_below(int b) { return b <= 0 ? 0ull : (b >= 64 ? ~0ull : ((1ull << b) - 1)); }
__device__ inline int64_t rlane64(int64_t v, int l) {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)v, l));
}

// inclusive prefix sum across the 64 lanes (DPP row shifts, then row broadcasts 15 / 31)
__device__ inline int32_t wave_incl_scan(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);     // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);     // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);     // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);     // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);     // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);     // row_bcast:31 -> rows 2, 3
    return v;
}

// SetUnschedulable (similar_pods.go:92-111): wave-uniform, LDS writes by lane 0
__device__ inline void fb_mark(const FbArgs& a, uint8_t* marks, int32_t* ocnt, uint8_t* oover, int32_t c,
                               int32_t& overflowing, int lane) {
    const int32_t o = a.cls_owner ? a.cls_owner[c] : -1;
    if (o < 0 || !a.cls_capped[c]) {
        if (lane == 0) marks[c] = 1;
        return;
    }
    if (ocnt[o] >= FO_MAX_PER_OWNER) {                                   // the controller's cache is full
        if (!oover[o]) {
            if (lane == 0) oover[o] = 1;
            overflowing++;
        }
        return;
    }
    if (lane == 0) {
        marks[c] = 1;
        ocnt[o] = ocnt[o] + 1;
    }
}

__global__ void __launch_bounds__(FB_T) k_fb_walk(FbArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fb_smem[];
    const int lane = (int)threadIdx.x;
    const int32_t n = a.n, NW = a.nwords, S = a.S;
    const FbLds lo = fb_lds(S, NW, a.K, a.stat_in_lds, a.n_classes, a.n_owners);
    FbShape* shp = reinterpret_cast<FbShape*>(fb_smem + lo.shapes);
    uint64_t* dyn = reinterpret_cast<uint64_t*>(fb_smem + lo.dyn);                // [S][NW]
    uint64_t* vis = reinterpret_cast<uint64_t*>(fb_smem + lo.vis);                // [NW]
    uint64_t* stat_l = reinterpret_cast<uint64_t*>(fb_smem + lo.stat);            // [K][NW] when in LDS
    int32_t* vpre = reinterpret_cast<int32_t*>(fb_smem + lo.vpre);                // [NW + 1]: visible nodes before word w
    int32_t* slot = reinterpret_cast<int32_t*>(fb_smem + lo.slot);                // a run's nodes
    FbRow* bufrow = reinterpret_cast<FbRow*>(fb_smem + lo.bufrow);                // the batch's written rows
    int32_t* bufnode = reinterpret_cast<int32_t*>(fb_smem + lo.bufnode);          // their nodes (-1: superseded)
    uint64_t* dirty = reinterpret_cast<uint64_t*>(fb_smem + lo.dirty);            // node has a row in the buffer
    int32_t* ocnt = reinterpret_cast<int32_t*>(fb_smem + lo.ocnt);
    uint8_t* marks = fb_smem + lo.marks;
    uint8_t* oover = fb_smem + lo.oover;
    const bool stat_lds = a.stat_in_lds != 0;
    for (int32_t i = lane; i < S; i += FB_T) shp[i] = a.shapes[i];
    FbThr* thr = reinterpret_cast<FbThr*>(fb_smem + lo.thr);
    for (int32_t i = lane; i < (int32_t)(sizeof(FbThr) / 8); i += FB_T)
        reinterpret_cast<uint64_t*>(thr)[i] = reinterpret_cast<const uint64_t*>(a.thr)[i];
    for (int32_t i = lane; i < S * NW; i += FB_T) dyn[i] = a.dyn0[i];
    if (stat_lds)
        for (int32_t i = lane; i < a.K * NW; i += FB_T) stat_l[i] = a.stat[i];
    for (int32_t i = lane; i < a.n_owners; i += FB_T) { ocnt[i] = 0; oover[i] = 0; }
    for (int32_t i = lane; i < a.n_classes; i += FB_T) marks[i] = 0;
    int32_t run_total = 0;                                                      // vis words and their prefix counts
    for (int32_t base = 0; base < NW; base += FB_T) {
        const int32_t w = base + lane;
        const uint64_t v = w < NW ? a.vis0[w] : 0ull;
        if (w < NW) { vis[w] = v; dirty[w] = 0; }
        const int32_t c = __builtin_popcountll(v);
        const int32_t inc = wave_incl_scan(c);
        if (w < NW) vpre[w] = run_total + inc - c;
        run_total += __builtin_amdgcn_readlane(inc, 63);
    }
    if (lane == 0) vpre[NW] = run_total;
    const int32_t vis_total = run_total;
    FbShape my_sh = {};                                                         // lane s: shape s (dyn updates)
    if (lane < S) my_sh = a.shapes[lane];
    __syncthreads();
    int32_t L = 0;
    if (n > 0) { L = a.ctl->L % n; if (L < 0) L += n; }
    int32_t vpL = 0;                                                            // visible nodes before L
    {
        const int32_t w = L >> 6;
        vpL = vpre[w] + __builtin_popcountll(vis[w] & bits_below(L & 63));
    }
    bool succ = false;
    unsigned long long evals = 0;
    int32_t overflowing = 0;
#ifdef CASIM_PROF
    unsigned long long prof_fb[3] = {0, 0, 0};
    unsigned long long prof_bk[4] = {0, 0, 0, 0};           // mixed runs: chain, row loads, updates; batch edges
    const unsigned long long w_c0 = clock64();
#endif
    // place k pods of shape s on slot[0..k) (lane t: slot[t]); `pre`: lane 0's row is given
    // (a hinted node, prefetched) unless the buffer has a newer one
    int32_t buf_n = 0;
    auto place = [&](int32_t k, int32_t s, bool pre, const NodeHot& prow) {
        const FbShape sh = shp[s];
        FbRow q = {};
        int32_t node = -1;
        if (lane < k) {
            node = slot[lane];
            const bool dj = (dirty[node >> 6] >> (node & 63)) & 1;
            int64_t cpu, mem, eph;
            int32_t pods;
            if (dj) {                                                           // the newest buffered row
                int32_t i = buf_n - 1;
                while (bufnode[i] != node) i--;
                const FbRow r = bufrow[i];
                bufnode[i] = -1;                                                // superseded below
                cpu = r.cpu; mem = r.mem; eph = r.eph; pods = r.pods;
            } else {
                const NodeHot r = pre ? prow : ld_hot_coh(a.hot + node);
                cpu = r.cpu; mem = r.mem; eph = r.eph; pods = r.pods;
            }
            q.cpu = wsub(cpu, sh.cpu);                                          // AddPod (SF/types.go:672-692)
            q.mem = wsub(mem, sh.mem);
            q.eph = wsub(eph, sh.eph);
            q.pods = pods - 1;
            q.pad = 0;
            bufrow[buf_n + lane] = q;
            bufnode[buf_n + lane] = node;
            __hip_atomic_fetch_or(&dirty[node >> 6], 1ull << (node & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        buf_n += k;
        for (int32_t t = 0; t < k; t++) {                                       // lane s': shape s' on each new row
            const int64_t c0 = rlane64(q.cpu, t), m0 = rlane64(q.mem, t), e0 = rlane64(q.eph, t);
            const int32_t p0 = __builtin_amdgcn_readlane(q.pods, t);
            const int32_t x = __builtin_amdgcn_readlane(node, t);
            if (lane < S && !fb_fit(my_sh, c0, m0, e0, p0))
                __hip_atomic_fetch_and(&dyn[(size_t)lane * NW + (x >> 6)], ~(1ull << (x & 63)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    // the batch's rows to HBM (one store per node: superseded entries are -1)
    auto flush = [&]() {
        if (lane < buf_n) {
            const int32_t node = bufnode[lane];
            if (node >= 0) {
                const FbRow q = bufrow[lane];
                NodeHot* d = a.hot + node;
                d->cpu = q.cpu; d->mem = q.mem; d->eph = q.eph; d->pods = q.pods;
                __hip_atomic_fetch_and(&dirty[node >> 6], ~(1ull << (node & 63)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        buf_n = 0;
    };
    int32_t bulk_from = 0;                                                      // next pod to try a mixed run at
    int32_t n_bulk = 0, n_bulk_pods = 0, n_runs = 0;                            // (stats: steps / ring_scans / windows)
    for (int32_t base = 0; base < a.P; base += FB_T) {
        const int32_t cnt = min(FB_T, a.P - base);
        FbPod lp = {0, -1, -1, 0};
        int32_t lh = -1;
        if (lane < cnt) { lp = a.pods[base + lane]; lh = a.hints[base + lane]; }
        const bool my_hinted = lane < cnt && lh >= 0 && lh < n && !(lp.flags & PF_PREFILTER_FAIL);
        const uint64_t hinted_mask = __ballot(my_hinted);
        NodeHot hrow = {};                                                      // prefetch: the hinted rows
        if (my_hinted) hrow = ld_hot_coh(a.hot + lh);
        // hint checks that can pass at all: the bits at the batch's start (placements only
        // clear bits, so a hint failing now fails later in the batch too)
        bool may = false;
        if (my_hinted) {
            const int32_t hw = lh >> 6;
            const uint64_t bit = 1ull << (lh & 63);
            const uint64_t hs = lp.scls >= 0 ? (stat_lds ? stat_l[(size_t)lp.scls * NW + hw]
                                                         : a.stat[(size_t)lp.scls * NW + hw]) : ~0ull;
            may = (dyn[(size_t)lp.shape * NW + hw] & hs & bit) && ((vis[hw] & bit) || (lp.flags & PF_TOL_UNSCHED));
        }
        const uint64_t may_mask = __ballot(may);
        // hinted pods whose hint fails for sure: one evaluation (CheckPredicates), then they
        // behave as unhinted pods, so they join runs
        const uint64_t nohope = hinted_mask & ~may_mask;
        auto hint_evals = [&](int32_t from, int32_t np) -> unsigned long long {
            if (np <= 0 || from >= 64) return 0ull;
            const uint64_t mk = (np >= 64 ? ~0ull : ((1ull << np) - 1)) << from;
            return (unsigned long long)__builtin_popcountll(nohope & mk);
        };
        int32_t out = -1;
        int32_t j = 0;
        while (j < cnt) {
#ifdef CASIM_PROF
            const unsigned long long pc0 = clock64();
#endif
            // Mixed runs (loose clusters).  A pod without a live hint scans from the node after
            // the previous such pod's node (L for the first) to its first fit; a pod whose hint
            // can pass takes its hinted node (CheckPredicates).  Every lane builds its pod's fit
            // mask over the 64 ring positions from L (the bitmaps as they are now); the
            // scanning pods' nodes follow from those masks: consecutive positions, checked for
            // all lanes at once, and a first-set-bit search at each pod that has to skip.
            // While the scans stay in the window, the hinted nodes lie outside it and every pod
            // passes there, the pods land on distinct nodes and no scan crosses an earlier
            // pod's node, so the masks stay exact and the placements are independent lane
            // updates.  The leading passes are placed together; the first failing pod goes on
            // below.  PreFilter failures and pods of a marked class end the run.  Short runs
            // back off for a while (tight clusters).
            if (base + j >= bulk_from) {
                const bool el = lane < cnt && !(lp.flags & PF_PREFILTER_FAIL) && !(lp.simcls >= 0 && marks[lp.simcls]);
                const uint64_t em = __ballot(el) >> j;
                const int32_t ne = em == ~0ull ? 64 : (int32_t)__builtin_ctzll(~em);
                int32_t f = 0;
                if (ne >= 2) {
#ifdef CASIM_PROF
                    const unsigned long long pk0 = clock64();
#endif
                    const int32_t ring = NW << 6;                               // raw positions (ids >= n never fit)
                    // the window's rows, in flight while the chain is worked out (position lane k: node L + k)
                    int32_t pk = L + lane;
                    if (pk >= ring) pk -= ring;
                    NodeHot wrow = {};
                    if (pk < n) wrow = ld_hot_coh(a.hot + pk);
                    const bool in = lane >= j && lane < j + ne;
                    const bool hin = in && (((hinted_mask & may_mask) >> lane) & 1);
                    const bool un = in && !hin;
                    const uint64_t um = __ballot(un);
                    const int32_t rk = __builtin_popcountll(um & bits_below(lane));   // scanning pods before me
                    const int32_t w0 = L >> 6, sh = L & 63, w1 = w0 + 1 == NW ? 0 : w0 + 1;
                    const size_t mso = lp.scls >= 0 ? (size_t)lp.scls * NW : 0;
                    uint64_t fm = 0;                                             // bit k: node L + k fits my pod
                    if (un) {
                        const size_t dso = (size_t)lp.shape * NW;
                        uint64_t g0 = dyn[dso + w0] & vis[w0], g1 = dyn[dso + w1] & vis[w1];
                        if (lp.scls >= 0) {
                            g0 &= stat_lds ? stat_l[mso + w0] : a.stat[mso + w0];
                            g1 &= stat_lds ? stat_l[mso + w1] : a.stat[mso + w1];
                        }
                        fm = NW == 1 ? (sh ? (g0 >> sh) | (g0 << (64 - sh)) : g0)
                                     : (sh ? (g0 >> sh) | (g1 << (64 - sh)) : g0);
                    }
                    // the scanning pods' window offsets: from scanning pod r0 on, each pod takes the
                    // position after the previous one's while it fits there; the first that does
                    // not searches its mask, and the pods after it shift behind it
                    int32_t xo = -1;
                    int32_t r0 = 0, pos0 = 0;                                    // the segment's first pod, its position
                    int32_t fs_rank = 64;                                        // the first scanning pod without a node
                    for (;;) {
                        const int32_t pos = pos0 + (rk - r0);
                        const bool seg = un && rk >= r0;
                        const bool fit = seg && pos < 64 && ((fm >> pos) & 1);
                        const uint64_t miss = __ballot(seg && !fit);
                        const int32_t m = miss ? (int32_t)__builtin_ctzll(miss) : 64;
                        const int32_t rm = miss ? __builtin_amdgcn_readlane(rk, m) : 64;
                        if (seg && rk < rm) xo = pos;
                        if (!miss) break;
                        const int32_t pm0 = pos0 + (rm - r0);                   // pod m's first position
                        const uint64_t fmm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(fm >> 32), m) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane((int)fm, m);
                        const uint64_t mk = pm0 >= 64 ? 0ull : fmm & (~0ull << pm0);
                        if (!mk) { fs_rank = rm; break; }
                        const int32_t o = __builtin_ctzll(mk);
                        if (lane == m) xo = o;
                        r0 = rm + 1;
                        pos0 = o + 1;
                    }
                    int32_t x = -1;
                    if (un && rk < fs_rank) { x = L + xo; if (x >= ring) x -= ring; }
                    bool ok = un && rk < fs_rank;
                    // my row: the buffer's newest, else the batch's prefetch (hinted pods) or the
                    // window's (scanning pods, taken once the run is known)
                    int64_t rc = 0, rm_ = 0, re = 0;
                    int32_t rp = 0, didx = -1;
                    if (hin) { x = lh; rc = hrow.cpu; rm_ = hrow.mem; re = hrow.eph; rp = hrow.pods; }
                    const bool dj = x >= 0 && ((dirty[x >> 6] >> (x & 63)) & 1);
                    if (dj) {
                        int32_t i = buf_n - 1;
                        while (bufnode[i] != x) i--;
                        const FbRow rr = bufrow[i];
                        rc = rr.cpu; rm_ = rr.mem; re = rr.eph; rp = rr.pods;
                        didx = i;
                    }
                    const int32_t xw = x >> 6;
                    const uint64_t bit = 1ull << (x & 63);
                    if (hin) {
                        int32_t dh = x - L;
                        if (dh < 0) dh += ring;
                        bool clash = dh < 64;                                           // inside the scanning window
                        for (uint64_t hmk = __ballot(hin); hmk; hmk &= hmk - 1) {      // an earlier hinted pod's node
                            const int u = __builtin_ctzll(hmk);
                            clash |= lane > u && __builtin_amdgcn_readlane(lh, u) == x;
                        }
                        const uint64_t hs = lp.scls >= 0 ? (stat_lds ? stat_l[mso + xw] : a.stat[mso + xw]) : ~0ull;
                        ok = !clash && (hs & bit) && ((vis[xw] & bit) || (lp.flags & PF_TOL_UNSCHED)) &&
                             fb_fit(shp[lp.shape], rc, rm_, re, rp);
                    }
                    const uint64_t bad = __ballot(in && !ok) >> j;
                    f = bad ? min(ne, (int32_t)__builtin_ctzll(bad)) : ne;
                    const int32_t f_scan = __builtin_popcountll(um & bits_below(j + f));
                    n_bulk++;
                    n_bulk_pods += f;
#ifdef CASIM_PROF
                    const unsigned long long pk1 = clock64();
                    prof_bk[0] += pk1 - pk0;
#endif
                    if (f > 0) {
                        const bool mine = lane >= j && lane < j + f;
                        {
                            const int32_t src = un && xo >= 0 ? xo : lane;
                            const int64_t wc = __shfl(wrow.cpu, src, FB_T), wm = __shfl(wrow.mem, src, FB_T),
                                          we = __shfl(wrow.eph, src, FB_T);
                            const int32_t wp = __shfl(wrow.pods, src, FB_T);
                            if (un && !dj) { rc = wc; rm_ = wm; re = we; rp = wp; }
                        }
                        FbRow qr = {};
                        if (mine) {
                            const FbShape sp = shp[lp.shape];
                            qr.cpu = wsub(rc, sp.cpu);                                  // AddPod (SF/types.go:672-692)
                            qr.mem = wsub(rm_, sp.mem);
                            qr.eph = wsub(re, sp.eph);
                            qr.pods = rp - 1;
                            if (didx >= 0) bufnode[didx] = -1;                          // superseded below
                            const int32_t at = buf_n + (lane - j);
                            bufrow[at] = qr;
                            bufnode[at] = x;
                            __hip_atomic_fetch_or(&dirty[xw], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            out = x;
                        }
                        buf_n += f;
#ifdef CASIM_PROF
                        const unsigned long long pk2 = clock64();
                        prof_bk[1] += pk2 - pk1;
#endif
                        // the shapes that no longer fit the new rows: every lane its row against all
                        // shapes at once (threshold tables), then one masked LDS update per shape
                        // that lost a node (a 65th shape is the dead row: nothing to clear)
                        const uint64_t pm = __ballot(mine);
                        const int32_t S64 = min(S, FB_MAX_SHAPES);
                        if (f < FB_ROWWISE_MAX) {                                       // short runs: row by row,
                            for (uint64_t fmk = pm; fmk; fmk &= fmk - 1) {              // lane s' checking shape s'
                                const int t = __builtin_ctzll(fmk);
                                const int64_t c0 = rlane64(qr.cpu, t), m0 = rlane64(qr.mem, t), e0 = rlane64(qr.eph, t);
                                const int32_t p0 = __builtin_amdgcn_readlane(qr.pods, t);
                                const int32_t xt = __builtin_amdgcn_readlane(x, t);
                                if (lane < S64 && !fb_fit(my_sh, c0, m0, e0, p0))
                                    __hip_atomic_fetch_and(&dyn[(size_t)lane * NW + (xt >> 6)], ~(1ull << (xt & 63)),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                        } else {
                            uint64_t gone = 0;
                            if (mine) gone = ~fb_fit_mask(*thr, qr.cpu, qr.mem, qr.eph, qr.pods) & bits_below(S64);
                            uint64_t any = gone;                                            // OR over the lanes
                            for (int32_t off = 1; off < FB_T; off <<= 1)
                                any |= ((uint64_t)(uint32_t)__shfl_xor((int)(any >> 32), off, FB_T) << 32) |
                                       (uint32_t)__shfl_xor((int)any, off, FB_T);
                            any = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(any >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)any);
                            for (uint64_t am = any; am; am &= am - 1) {
                                const int s2 = __builtin_ctzll(am);
                                if ((gone >> s2) & 1)
                                    __hip_atomic_fetch_and(&dyn[(size_t)s2 * NW + xw], ~bit, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                        }
                        // CheckPredicates per hinted pod (+ failed hints); the scans evaluated
                        // the visible nodes from L to the last scanning pod's node
                        evals += (unsigned long long)(f - f_scan) + hint_evals(j, f);
                        const uint64_t sm = pm & um;                                    // the scanning pods move L
                        if (sm) {
                            const int32_t xl = __builtin_amdgcn_readlane(x, 63 - __builtin_clzll(sm));
                            const int32_t lw = xl >> 6;
                            const int32_t vpx = vpre[lw] + __builtin_popcountll(vis[lw] & bits_below(xl & 63)) + 1;
                            evals += (unsigned long long)(xl >= L ? vpx - vpL : vis_total - vpL + vpx);
                            L = xl + 1 == n ? 0 : xl + 1;                               // schedulerbased.go:131
                            vpL = L == 0 ? 0 : vpx;
                            succ = true;
                        }
                        j += f;
#ifdef CASIM_PROF
                        prof_bk[2] += clock64() - pk2;
#endif
                    }
                }
                if (f < 2) bulk_from = base + j + FB_BACKOFF;
                if (f > 0) {
#ifdef CASIM_PROF
                    prof_fb[2] += clock64() - pc0;
#endif
                    continue;
                }
            }
            n_runs++;
            const int32_t s = __builtin_amdgcn_readlane(lp.shape, j);
            const int32_t c = __builtin_amdgcn_readlane(lp.scls, j);
            const int32_t sim = __builtin_amdgcn_readlane(lp.simcls, j);
            const uint32_t pf = (uint32_t)__builtin_amdgcn_readlane((int)lp.flags, j);
            const uint64_t* ds = dyn + (size_t)s * NW;
            const size_t so = c >= 0 ? (size_t)c * NW : 0;
            int32_t first = j;                                                  // the run starts here
            // Leading hinted pods in bulk: pod t of a row of hinted pods whose earlier pods
            // all went to their hinted nodes sees exactly those placements on its own
            // hinted node, so the hint checks (CheckPredicates: NodeUnschedulable, static,
            // NodeResourcesFit on the row minus the earlier pods on that node) are
            // independent lane checks; the leading successes are placed together, and the
            // first failing pod goes on alone below.
            const uint64_t hr = (may_mask >> j) & 3ull;
            if (hr == 3ull) {
                const uint64_t hrun = may_mask >> j;
                const int32_t lead = hrun == ~0ull ? 64 : (int32_t)__builtin_ctzll(~hrun);
                const bool in = lane >= j && lane < j + lead;
                const FbShape msh = shp[in ? lp.shape : 0];
                // the row of my hinted node: the batch buffer's newest entry, else the prefetch
                int64_t rc = hrow.cpu, rm = hrow.mem, re = hrow.eph;
                int32_t rp = hrow.pods;
                int32_t didx = -1;
                if (in && ((dirty[lh >> 6] >> (lh & 63)) & 1)) {
                    int32_t i = buf_n - 1;
                    while (bufnode[i] != lh) i--;
                    const FbRow r = bufrow[i];
                    rc = r.cpu; rm = r.mem; re = r.eph; rp = r.pods;
                    didx = i;
                }
                // the earlier pods of the row that go to the same node
                for (int32_t u = j; u < j + lead - 1; u++) {
                    const int32_t hu = __builtin_amdgcn_readlane(lh, u);
                    const FbShape su = shp[__builtin_amdgcn_readlane(lp.shape, u)];
                    if (in && lane > u && lh == hu) {
                        rc = wsub(rc, su.cpu); rm = wsub(rm, su.mem); re = wsub(re, su.eph); rp -= 1;
                    }
                }
                bool ok = false;
                if (in) {
                    const int32_t hw = lh >> 6;
                    const uint64_t bit = 1ull << (lh & 63);
                    const size_t mso = lp.scls >= 0 ? (size_t)lp.scls * NW : 0;
                    const uint64_t hs = lp.scls >= 0 ? (stat_lds ? stat_l[mso + hw] : a.stat[mso + hw]) : ~0ull;
                    ok = (hs & bit) && ((vis[hw] & bit) || (lp.flags & PF_TOL_UNSCHED)) && fb_fit(msh, rc, rm, re, rp);
                }
                const uint64_t okm = __ballot(ok) >> j;
                const int32_t f = min(lead, okm == ~0ull ? 64 : (int32_t)__builtin_ctzll(~okm));
                if (f > 0) {
                    const bool mine = lane >= j && lane < j + f;
                    // the last of the placed pods on each node commits the node's new row
                    bool later = false;
                    for (int32_t u = j + 1; u < j + f; u++) {
                        const int32_t hu = __builtin_amdgcn_readlane(lh, u);
                        later |= mine && lane < u && lh == hu;
                    }
                    const bool fin = mine && !later;
                    if (fin && didx >= 0) bufnode[didx] = -1;                   // superseded below
                    const int64_t qc = wsub(rc, msh.cpu), qm = wsub(rm, msh.mem), qe = wsub(re, msh.eph);
                    const int32_t qp = rp - 1;
                    const uint64_t finm = __ballot(fin);
                    if (fin) {
                        const int32_t at = buf_n + (int32_t)__builtin_popcountll(finm & bits_below(lane));
                        FbRow q;
                        q.cpu = qc; q.mem = qm; q.eph = qe; q.pods = qp; q.pad = 0;
                        bufrow[at] = q;
                        bufnode[at] = lh;
                        __hip_atomic_fetch_or(&dirty[lh >> 6], 1ull << (lh & 63), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    buf_n += (int32_t)__builtin_popcountll(finm);
                    for (uint64_t fm = finm; fm; fm &= fm - 1) {                 // lane s': shape s' on each new row
                        const int t = __builtin_ctzll(fm);
                        const int64_t c0 = rlane64(qc, t), m0 = rlane64(qm, t), e0 = rlane64(qe, t);
                        const int32_t p0 = __builtin_amdgcn_readlane(qp, t);
                        const int32_t x = __builtin_amdgcn_readlane(lh, t);
                        if (lane < S && !fb_fit(my_sh, c0, m0, e0, p0))
                            __hip_atomic_fetch_and(&dyn[(size_t)lane * NW + (x >> 6)], ~(1ull << (x & 63)),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    if (mine) out = lh;
                    evals += (unsigned long long)f;                             // CheckPredicates per pod
                    j += f;
#ifdef CASIM_PROF
                    prof_fb[0] += clock64() - pc0;
#endif
                    continue;                                                   // pod j (if any) fails its hint
                }
            }
            if ((may_mask >> j) & 1) {                                          // findNodeWithHints (:91-108)
                const int32_t h = __builtin_amdgcn_readlane(lh, j);
                const int32_t hw = h >> 6;
                const uint64_t bit = 1ull << (h & 63);
                evals++;                                                        // CheckPredicates ran the filters
                // NodeUnschedulable applies (tolerable), then static, then fit
                const uint64_t hs = c >= 0 ? (stat_lds ? stat_l[so + hw] : a.stat[so + hw]) : ~0ull;
                if ((ds[hw] & hs & bit) && ((vis[hw] & bit) || (pf & PF_TOL_UNSCHED))) {
                    if (lane == 0) slot[0] = h;
                    NodeHot pr;
                    pr.cpu = rlane64(hrow.cpu, j); pr.mem = rlane64(hrow.mem, j); pr.eph = rlane64(hrow.eph, j);
                    pr.pods = __builtin_amdgcn_readlane(hrow.pods, j); pr.flags = 0;
                    place(1, s, true, pr);
                    if (lane == j) out = h;
                    j++;
#ifdef CASIM_PROF
                    prof_fb[0] += clock64() - pc0;
#endif
                    continue;
                }
                first = j + 1;                                                  // the run's other pods: unhinted
            }
            // the run: pod j and the unhinted pods right after it with the same attributes
            const bool same = lane >= first && lane < cnt && lp.shape == s && lp.scls == c && lp.simcls == sim &&
                              lp.flags == pf;
            const uint64_t run_ok = __ballot(same) & ~(hinted_mask & may_mask);
            const uint64_t rest = first < 64 ? run_ok >> first : 0ull;          // consecutive ones from `first`
            const int32_t m = (first - j) + (rest == ~0ull ? 64 : (int32_t)__builtin_ctzll(~rest));
#ifdef CASIM_PROF
            const unsigned long long pc1 = clock64();
            prof_fb[0] += pc1 - pc0;
#endif
            const int32_t pre = first - j;                                      // pod j, already hint-checked
            if (sim >= 0 && marks[sim]) {                                       // similar pod known unschedulable
                evals += hint_evals(first, m - pre);
                j += m;
                continue;
            }
            if (pf & PF_PREFILTER_FAIL) {                                       // no node passes PreFilter (never hinted)
                if (sim >= 0 && !(pf & PF_DAEMONSET)) fb_mark(a, marks, ocnt, oover, sim, overflowing, lane);
                j += (sim >= 0 && !(pf & PF_DAEMONSET) && marks[sim]) ? m : 1;
                continue;
            }
            // findNode (:110-125): the first m fits from L, one ring pass, 64 words per step;
            // step r == NW revisits word w0 for the bits below L (the ring's tail)
            const int32_t w0 = L >> 6, b0 = L & 63;
            const int32_t last = b0 ? NW : NW - 1;
            int32_t k = 0;
            for (int32_t rb = 0; rb <= last && k < m; rb += FB_T) {
                const int32_t r = rb + lane;
                int32_t w = w0 + (r < NW ? r : 0);
                if (w >= NW) w -= NW;
                uint64_t mask = r == 0 ? bits_from(b0) : (r == NW ? bits_below(b0) : ~0ull);
                if (r > last) mask = 0;
                uint64_t f = ds[w] & vis[w] & mask;
                if (c >= 0) f &= stat_lds ? stat_l[so + w] : a.stat[so + w];
                const int32_t cf = __builtin_popcountll(f);
                const int32_t inc = wave_incl_scan(cf);
                const int32_t tot = __builtin_amdgcn_readlane(inc, 63);
                // lanes scatter their fits into slot[k + before ...] while the run needs them
                int32_t at = k + inc - cf;
                while (f && at < m) {
                    slot[at++] = (w << 6) + __builtin_ctzll(f);
                    f &= f - 1;
                }
                k = min(m, k + tot);
            }
#ifdef CASIM_PROF
            const unsigned long long pc2 = clock64();
            prof_fb[1] += pc2 - pc1;
#endif
            if (k == 0) {                                                       // no node fits: every run pod fails
                const bool can_mark = sim >= 0 && !(pf & PF_DAEMONSET);
                if (can_mark) fb_mark(a, marks, ocnt, oover, sim, overflowing, lane);
                // a marked class skips the rest of the run; otherwise (no class, DaemonSet, a
                // controller over its cap) each pod scans the whole ring again, unchanged
                const int32_t nfail = (can_mark && marks[sim]) ? 1 : m;
                evals += (unsigned long long)nfail * (unsigned long long)vis_total + hint_evals(first, m - pre);
                j += m;
                continue;
            }
            // the visible nodes from L to the last fit (inclusive) were evaluated
            const int32_t xl = slot[k - 1];
            const int32_t xw = xl >> 6;
            const int32_t vpx = vpre[xw] + __builtin_popcountll(vis[xw] & bits_below(xl & 63)) + 1;
            evals += (unsigned long long)(xl >= L ? vpx - vpL : vis_total - vpL + vpx);
            place(k, s, false, NodeHot{});
            evals += hint_evals(first, k - pre);
            if (lane >= j && lane < j + k) out = slot[lane - j];
            L = xl + 1 == n ? 0 : xl + 1;                                       // schedulerbased.go:131
            vpL = L == 0 ? 0 : vpx;
            succ = true;
            j += k;
#ifdef CASIM_PROF
            prof_fb[2] += clock64() - pc2;
#endif
        }
        flush();
        if (lane < cnt) {
            a.out_node[base + lane] = out;
            if (out >= 0) a.hints[base + lane] = out;                           // Hints.Set (:95, :123)
        }
    }
    for (int32_t i = lane; i < a.n_classes; i += FB_T) a.cls_mark[i] = marks[i];
    if (lane == 0) {
        if (succ) a.ctl->L = L;
        a.ctl->evals = evals;
        a.ctl->overflowing = overflowing;
        a.ctl->phases = (a.P + FB_T - 1) / FB_T;
        a.ctl->steps = n_bulk;                          // mixed-run attempts
        a.ctl->ring_scans = n_bulk_pods;                // pods they placed
        a.ctl->windows = n_runs;                        // pod steps of the one-by-one path
#ifdef CASIM_PROF
        // (CASIM_FB_PROF_BULK: the mixed runs' chain / row loads / updates in place of the
        // hint / scan / place split)
        for (int i = 0; i < 3; i++) a.ctl->fb_cyc[i] = a.ctl->fb_cyc[3] ? prof_bk[i] : prof_fb[i];
        a.ctl->seq_cycles = clock64() - w_c0;
        a.ctl->all_cycles = a.ctl->seq_cycles;
#endif
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
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    auto tmark = [&](const char* what) {
        if (dbg_t)
            fprintf(stderr, "[filter] %-12s %8.3f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    // (one pass over the records: the arguments first, then the kernel scope)
    bool oos = false;
    for (int32_t k = 0; k < n; k++) {
        const int32_t i = order ? order[k] : k;
        if (i < 0 || i >= t->n_pods) return CA_EINVAL;
        if (t->pods[i].similar_class >= n_classes) return CA_EINVAL;
        oos |= (t->pods[i].flags & CA_POD_OUT_OF_SCOPE) != 0;
    }
    // casim.h kernel scope: an out-of-scope pending pod, or required anti-affinity in the
    // snapshot, sends the whole call to the Go path (nothing placed)
    if (m->n_scope_blockers > 0 || oos) return CA_EUNSUPPORTED;
    if (n_overflowing) *n_overflowing = 0;
    if (n_placed) *n_placed = 0;
    FilterScratch& fo = m->fo;
    fo.kernel_ms = 0;
    fo.phases = fo.steps = fo.ring_scans = fo.windows = 0;
    if (n == 0) return CA_OK;
    CA_HIP_CHECK(hipSetDevice(m->device));
    int rc;
    tmark("validated");
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    tmark("synced");
    const DevPodTable* dp = s ? &s->t : nullptr;
    if (!dp) {
        // (queued: the shape preparation below runs while the records cross; the call's sync
        // after the kernel ends them before the staging is reused)
        if ((rc = fo.pods.upload_staged(t->pods, t->n_pods, t->terms, t->n_terms, t->reqs, t->n_reqs,
                                        t->prefilter_names, t->n_prefilter_names, fo.h_pods, m->stream)) != CA_OK) {
            (void)hipStreamSynchronize(m->stream);
            return rc;
        }
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
    // inputs: order | hints | class_owner | capped ; zeroed: ctl | owner_cnt | cls_mark | owner_over
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_order = 0, o_hints = o_order + al(sizeof(int32_t) * n), o_owner = o_hints + al(sizeof(int32_t) * n),
                 o_capped = o_owner + al(sizeof(int32_t) * (n_classes + 1)), in_bytes = o_capped + al(n_classes + 1);
    const size_t z_ctl = 0, z_ocnt = al(sizeof(FoCtl)), z_mark = z_ocnt + al(sizeof(int32_t) * (n_owners + 1)),
                 z_over = z_mark + al(n_classes + 1), z_bytes = z_over + al(n_owners + 1);
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
    tmark("inputs");
    if (class_owner) std::memcpy(hi + o_owner, class_owner, sizeof(int32_t) * n_classes);
    std::memcpy(hi + o_capped, capped.data(), (size_t)n_classes);
    FoCtl ctl0;
    std::memset(&ctl0, 0, sizeof ctl0);
    ctl0.L = *last_index;
    ctl0.fb_cyc[3] = knob_env("CASIM_FB_PROF_BULK") ? 1 : 0;     // (CASIM_PROF builds: which split)
    char* di = fo.in.as<char>();
    char* dz = fo.zero.as<char>();
    char* dout = fo.out.as<char>();
    CA_HIP_CHECK(hipMemcpyAsync(di, hi, in_bytes, hipMemcpyHostToDevice, m->stream));
    CA_HIP_CHECK(hipMemsetAsync(dz, 0, z_bytes, m->stream));
    CA_HIP_CHECK(hipMemcpyAsync(dz + z_ctl, &ctl0, sizeof ctl0, hipMemcpyHostToDevice, m->stream));
    // hints are in/out: the kernel writes into a copy in the output block
    int32_t* d_hints = reinterpret_cast<int32_t*>(dout + al(sizeof(int32_t) * n));
    CA_HIP_CHECK(hipMemcpyAsync(d_hints, di + o_hints, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, m->stream));
    tmark("staged");
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
    a.ctl = reinterpret_cast<FoCtl*>(dz + z_ctl);
    a.n_pods = dp->n_pods;
    a.n_classes = n_classes;
    a.n_owners = n_owners;
    // Feasibility-bitmap walk when every pending pod qualifies (no host ports, no scalar
    // requests, no PreFilter NodeNames; <= 64 resource shapes; the bitmaps fit LDS); the
    // window sequencer otherwise (CASIM_FO_WINDOW forces it, for tests of both).
    fo.path = 0;
    fo.fb_shapes = fo.fb_classes = 0;
    std::vector<FbPod> fb_pods;
    std::vector<FbShape> fb_shapes;
    std::vector<int32_t> fb_rep;
    int32_t fb_stat_in_lds = 0;
    bool fb = nn > 0 && !knob_env("CASIM_FO_WINDOW");
    const int32_t NW = (nn + 63) / 64;
    if (fb) {
        // one pass over the node rows (host workers): the taints any node has, and the largest
        // free cpu / memory / ephemeral of any node with a free pod slot (the dead-shape test below)
        uint64_t taint_union = 0;
        int64_t mx_c = INT64_MIN, mx_m = INT64_MIN, mx_e = INT64_MIN;
        {
            const size_t N = m->nodes.size();
            const int32_t T = (int32_t)std::max<size_t>(1, std::min<size_t>(8, N / 2048));
            struct Part { uint64_t tu; int64_t c, mm, e; };
            std::vector<Part> part((size_t)T, Part{0, INT64_MIN, INT64_MIN, INT64_MIN});
            casim::parallel_run(T, [&](int32_t w) {
                Part p{0, INT64_MIN, INT64_MIN, INT64_MIN};
                const size_t i0 = N * (size_t)w / (size_t)T, i1 = N * (size_t)(w + 1) / (size_t)T;
                for (size_t i = i0; i < i1; i++) {
                    const NodeRow& nd = m->nodes[i];
                    p.tu |= nd.spec.taints;
                    if (clamp_i32(nd.spec.alloc_pods - nd.npods) < 1) continue;
                    p.c = std::max(p.c, wsub(nd.spec.alloc_milli_cpu, nd.req_cpu));
                    p.mm = std::max(p.mm, wsub(nd.spec.alloc_memory, nd.req_mem));
                    p.e = std::max(p.e, wsub(nd.spec.alloc_ephemeral, nd.req_eph));
                }
                part[(size_t)w] = p;
            });
            for (const Part& p : part) {
                taint_union |= p.tu;
                mx_c = std::max(mx_c, p.c); mx_m = std::max(mx_m, p.mm); mx_e = std::max(mx_e, p.e);
            }
        }
        tmark("taints");
        struct KeyHash {
            size_t operator()(const std::string& k) const { return std::hash<std::string>()(k); }
        };
        struct ShapeKey {
            int64_t c, m, e;
            uint32_t z;
            bool operator==(const ShapeKey& o) const { return c == o.c && m == o.m && e == o.e && z == o.z; }
        };
        struct ShapeHash {
            size_t operator()(const ShapeKey& k) const {
                uint64_t h = (uint64_t)k.c * 0x9E3779B97F4A7C15ull;
                h ^= (uint64_t)k.m + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
                h ^= (uint64_t)k.e * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2);
                return (size_t)(h ^ k.z);
            }
        };
        std::unordered_map<ShapeKey, int32_t, ShapeHash> shape_id;   // (no per-pod allocation)
        std::unordered_map<std::string, int32_t, KeyHash> cls_id;
        shape_id.reserve(256);
        fb_pods.resize((size_t)n);
        const ca_pod_spec* prev = nullptr;               // pods of one controller variant come in a row
        std::vector<int32_t> cls_seen((size_t)n_classes, -1);              // a similar class's first position
        // which pods repeat the record before them (compared on the host workers first: the
        // loop below then classifies only the first of each row)
        std::vector<uint8_t> same((size_t)n, 0);
        {
            const int32_t T = std::max(1, std::min(8, n / 4096));
            casim::parallel_run(T, [&](int32_t w) {
                const int32_t k0 = (int32_t)((int64_t)n * w / T), k1 = (int32_t)((int64_t)n * (w + 1) / T);
                for (int32_t k = std::max(k0, 1); k < k1; k++)
                    same[(size_t)k] = std::memcmp(&t->pods[h_order[k - 1]], &t->pods[h_order[k]], sizeof(ca_pod_spec)) == 0;
            });
        }
        for (int32_t k = 0; k < n && fb; k++) {
            const ca_pod_spec& ps = t->pods[h_order[k]];
            if (prev && same[(size_t)k]) {                                 // the same record: same ids
                fb_pods[k] = fb_pods[k - 1];
                prev = &ps;
                continue;
            }
            const int32_t sc = ps.similar_class;                           // (interleaved controllers)
            if (sc >= 0) {
                const int32_t k0 = cls_seen[sc];
                if (k0 >= 0 && std::memcmp(&t->pods[h_order[k0]], &ps, sizeof ps) == 0) {
                    fb_pods[k] = fb_pods[k0];
                    prev = &ps;
                    continue;
                }
                if (k0 < 0) cls_seen[sc] = k;
            }
            prev = &ps;
            const uint32_t f = pod_dev_flags(ps);
            if (f & (PF_PORTS | PF_SCALAR_REQ | PF_PREFILTER_NAMES)) { fb = false; break; }
            const ShapeKey sk{ps.req_milli_cpu, ps.req_memory, ps.req_ephemeral, (f & PF_ALL_ZERO) ? 1u : 0u};
            auto it = shape_id.find(sk);
            if (it == shape_id.end()) {
                if ((int32_t)shape_id.size() >= FB_COLLECT_SHAPES) { fb = false; break; }
                it = shape_id.emplace(sk, (int32_t)shape_id.size()).first;
                FbShape sh;
                sh.cpu = ps.req_milli_cpu; sh.mem = ps.req_memory; sh.eph = ps.req_ephemeral;
                sh.flags = f & PF_ALL_ZERO; sh.pad = 0;
                fb_shapes.push_back(sh);
            }
            int32_t cid = -1;                   // the static part of the filter chain (dev_static_filters)
            if ((f & (PF_NODE_NAME | PF_AFFINITY)) || (ps.tolerated_taints & taint_union) != taint_union) {
                std::string ck(reinterpret_cast<const char*>(&ps.tolerated_taints), 8);
                const uint32_t sf = f & (PF_NODE_NAME | PF_AFFINITY);
                ck.append(reinterpret_cast<const char*>(&sf), 4);
                if (f & PF_NODE_NAME) ck.append(reinterpret_cast<const char*>(&ps.node_name_id), 4);
                if (f & PF_AFFINITY) {
                    ck.append(reinterpret_cast<const char*>(ps.node_selector), sizeof ps.node_selector);
                    ck.append(reinterpret_cast<const char*>(&ps.aff_term_count), 4);
                    for (int32_t q = 0; q < ps.aff_term_count; q++) {
                        const ca_selector_term& tm = t->terms[ps.aff_term_first + q];
                        ck.append(reinterpret_cast<const char*>(&tm.count), 4);
                        for (int32_t r = 0; r < tm.count; r++)
                            ck.append(reinterpret_cast<const char*>(&t->reqs[tm.first + r]), sizeof(ca_selector_req));
                    }
                }
                auto ct = cls_id.find(ck);
                if (ct == cls_id.end()) {
                    ct = cls_id.emplace(ck, (int32_t)cls_id.size()).first;
                    fb_rep.push_back(h_order[k]);
                }
                cid = ct->second;
            }
            FbPod& fp = fb_pods[k];
            fp.shape = it->second;
            fp.scls = cid;
            fp.simcls = ps.similar_class;
            fp.flags = f;
        }
        tmark("shapes");
        // Shapes that fit no node now never fit during the call (placements only take
        // resources away): their pods share one shape with an all-zero dyn row (requests no
        // node has), so only the live shapes count against the 64 lanes of the bit updates.
        if (fb) {
            const int32_t S0 = (int32_t)fb_shapes.size();
            std::vector<uint8_t> alive((size_t)S0, 0);
            std::vector<int32_t> open;
            // shapes beyond the largest free cpu / memory / ephemeral of any node with a free
            // pod slot fit no node: dead without the node walk below (RunOnce's backlog of
            // variants too large for every node would otherwise walk all nodes each)
            for (int32_t q = 0; q < S0; q++) {
                const FbShape& sh = fb_shapes[q];
                if (mx_c == INT64_MIN) continue;                               // no node has a slot
                if (!(sh.flags & PF_ALL_ZERO) && (sh.cpu > mx_c || sh.mem > mx_m || sh.eph > mx_e)) continue;
                open.push_back(q);
            }
            for (size_t i = 0; i < m->nodes.size() && !open.empty(); i++) {
                // the free resources of fill_hot, without its port / scalar flag scans (a
                // shape that fits no node walks every node here)
                const NodeRow& nd = m->nodes[i];
                const int64_t fc = wsub(nd.spec.alloc_milli_cpu, nd.req_cpu), fm = wsub(nd.spec.alloc_memory, nd.req_mem);
                const int64_t fe = wsub(nd.spec.alloc_ephemeral, nd.req_eph);
                const int32_t fp = clamp_i32(nd.spec.alloc_pods - nd.npods);
                for (size_t q = 0; q < open.size();) {
                    if (fb_fit(fb_shapes[open[q]], fc, fm, fe, fp)) {
                        alive[open[q]] = 1;
                        open[q] = open.back();
                        open.pop_back();
                    } else {
                        q++;
                    }
                }
            }
            tmark("alive");
            bool any_dead = false;
            for (int32_t q = 0; q < S0; q++) any_dead |= !alive[q];
            if (any_dead) {
                std::vector<int32_t> remap((size_t)S0, -1);
                std::vector<FbShape> live;
                for (int32_t q = 0; q < S0; q++)
                    if (alive[q]) { remap[q] = (int32_t)live.size(); live.push_back(fb_shapes[q]); }
                FbShape none;
                none.cpu = none.mem = none.eph = INT64_MAX;
                none.flags = 0; none.pad = 0;
                const int32_t dead = (int32_t)live.size();
                live.push_back(none);
                for (FbPod& fp : fb_pods) fp.shape = alive[fp.shape] ? remap[fp.shape] : dead;
                fb_shapes.swap(live);
            }
            // the live shapes take the bit-update lanes; the dead row (last) needs none
            const int32_t live = (int32_t)fb_shapes.size() - (any_dead ? 1 : 0);
            if (live > FB_MAX_SHAPES) fb = false;
        }
        // LDS: shapes, bitmaps, vis prefix counts, run scratch and the similar-pods state,
        // plus the static words when they fit too
        const int32_t S = (int32_t)fb_shapes.size(), K = (int32_t)fb_rep.size();
        fb_stat_in_lds = K > 0 && fb_lds(S, NW, K, 1, n_classes, n_owners).total <= FB_LDS_MAX ? 1 : 0;
        if (fb_lds(S, NW, K, fb_stat_in_lds, n_classes, n_owners).total > FB_LDS_MAX) fb = false;
    }
    tmark("prepared");
    CA_HIP_CHECK(hipEventRecord(m->ev0, m->stream));
    if (fb) {
        const int32_t S = (int32_t)fb_shapes.size(), K = (int32_t)fb_rep.size();
        const size_t b_pods = al(sizeof(FbPod) * n), b_sh = al(sizeof(FbShape) * std::max(S, 1)),
                     b_rep = al(sizeof(int32_t) * std::max(K, 1)), b_thr = al(sizeof(FbThr));
        if ((rc = fo.fb_in.reserve(b_pods + b_sh + b_rep + b_thr)) != CA_OK ||
            (rc = fo.h_fb.reserve(b_pods + b_sh + b_rep + b_thr)) != CA_OK)
            return rc;
        const size_t w_dyn = (size_t)S * NW, w_vis = (size_t)NW, w_stat = (size_t)K * NW;
        if ((rc = fo.fb_bits.reserve(sizeof(uint64_t) * (w_dyn + w_vis + std::max<size_t>(w_stat, 1)))) != CA_OK) return rc;
        char* hb = fo.h_fb.as<char>();
        std::memcpy(hb, fb_pods.data(), sizeof(FbPod) * n);
        std::memcpy(hb + b_pods, fb_shapes.data(), sizeof(FbShape) * S);
        if (K) std::memcpy(hb + b_pods + b_sh, fb_rep.data(), sizeof(int32_t) * K);
        {                                                   // the fit thresholds of the first 64 shapes
            FbThr& th = *reinterpret_cast<FbThr*>(hb + b_pods + b_sh + b_rep);
            std::memset(&th, 0, sizeof th);
            const int32_t S64 = std::min(S, FB_MAX_SHAPES);
            for (int32_t d = 0; d < 3; d++) {
                auto req = [&](int32_t q) { return d == 0 ? fb_shapes[q].cpu : d == 1 ? fb_shapes[q].mem : fb_shapes[q].eph; };
                std::vector<int64_t> vals;
                for (int32_t q = 0; q < S64; q++) vals.push_back(req(q));
                std::sort(vals.begin(), vals.end());
                vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
                th.u[d] = (int32_t)vals.size();
                for (size_t k = 0; k < vals.size(); k++) th.v[d][k] = vals[k];
                for (size_t k = 1; k <= vals.size(); k++)
                    for (int32_t q = 0; q < S64; q++)
                        if (req(q) <= vals[k - 1]) th.t[d][k] |= 1ull << q;
            }
            for (int32_t q = 0; q < S64; q++)
                if (fb_shapes[q].flags & PF_ALL_ZERO) th.zero |= 1ull << q;
        }
        char* db = fo.fb_in.as<char>();
        CA_HIP_CHECK(hipMemcpyAsync(db, hb, b_pods + b_sh + b_rep + b_thr, hipMemcpyHostToDevice, m->stream));
        uint64_t* d_dyn = fo.fb_bits.as<uint64_t>();
        uint64_t* d_vis = d_dyn + w_dyn;
        uint64_t* d_stat = d_vis + w_vis;
        hipLaunchKernelGGL(k_fb_dyn, dim3((nn + 255) / 256, S + 1), dim3(256), 0, m->stream, m->d_hot.as<const NodeHot>(),
                           nn, NW, reinterpret_cast<const FbShape*>(db + b_pods), S, d_dyn, d_vis);
        CA_HIP_CHECK(hipGetLastError());
        if (K) {
            hipLaunchKernelGGL(k_fb_stat, dim3((nn + 255) / 256, K), dim3(256), 0, m->stream,
                               m->d_static.as<const NodeStatic>(), nn, NW,
                               reinterpret_cast<const int32_t*>(db + b_pods + b_sh), dp->hot.as<const PodHot>(),
                               dp->spec.as<const ca_pod_spec>(), dp->terms.as<const ca_selector_term>(),
                               dp->reqs.as<const ca_selector_req>(), d_stat);
            CA_HIP_CHECK(hipGetLastError());
        }
        FbArgs fa;
        fa.hot = m->d_hot.as<NodeHot>();
        fa.n = nn; fa.nwords = NW; fa.P = n; fa.S = S; fa.K = K;
        fa.n_classes = n_classes; fa.n_owners = n_owners;
        fa.stat_in_lds = fb_stat_in_lds;
        fa.pods = reinterpret_cast<const FbPod*>(db);
        fa.shapes = reinterpret_cast<const FbShape*>(db + b_pods);
        fa.thr = reinterpret_cast<const FbThr*>(db + b_pods + b_sh + b_rep);
        fa.dyn0 = d_dyn; fa.vis0 = d_vis; fa.stat = d_stat;
        fa.hints = a.hints; fa.out_node = a.out_node;
        fa.cls_mark = a.cls_mark; fa.cls_capped = a.cls_capped; fa.cls_owner = a.cls_owner;
        fa.ctl = a.ctl;
        const size_t lds_all = fb_lds(S, NW, K, fb_stat_in_lds, n_classes, n_owners).total;
        if ((rc = ensure_dyn_lds((const void*)k_fb_walk, lds_all)) != CA_OK) return rc;
        hipLaunchKernelGGL(k_fb_walk, dim3(1), dim3(FB_T), lds_all, m->stream, fa);
        CA_HIP_CHECK(hipGetLastError());
        fo.path = 1;
        fo.fb_shapes = S;
        fo.fb_classes = K;
        fo.fb_stat_lds = fb_stat_in_lds;
    } else {
        hipLaunchKernelGGL(k_filter_out, dim3(1), dim3(SQ_T), 0, m->stream, a);
        CA_HIP_CHECK(hipGetLastError());
    }
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
    tmark("device");
    // AddPod of every placed pod on the host rows, in the reference's order
    int32_t placed = 0;
    for (int32_t k = 0; k < n; k++) {
        out_node[k] = nodes_out[k];
        if (hints) hints[k] = hints_out[k];
        placed += nodes_out[k] >= 0;
    }
    const size_t pods0 = m->pods.size(), terms0 = m->terms.size(), reqs0 = m->reqs.size(), names0 = m->pf_names.size();
    const bool dev_in_sync = m->d_pods_synced == pods0 && (size_t)m->d_pods.n_pods == pods0 && m->d_terms_synced == terms0 &&
                             (size_t)m->d_pods.n_reqs == reqs0 && (size_t)m->d_pods.n_names == names0;
    m->add_placed_batch(t, h_order, nodes_out, n, out_pod_id, fb, s && !s->any_refs);   // the walk flushed its rows to d_hot
    // the new mirror records are the podset's records: gathered on the device instead of
    // crossing PCIe at the next sync (only when no selector tables had to be re-based)
    if (s && dev_in_sync && placed > 0 && m->pods.size() == pods0 + (size_t)placed && m->terms.size() == terms0 &&
        m->reqs.size() == reqs0 && m->pf_names.size() == names0 && !knob_env("CASIM_NO_POD_GATHER")) {
        std::vector<int32_t> src;
        src.reserve((size_t)placed);
        for (int32_t k = 0; k < n; k++)
            if (nodes_out[k] >= 0) src.push_back(h_order[k]);
        if ((rc = m->d_pods.append_gather(s->t, src.data(), placed, fo.gather_idx, m->stream)) != CA_OK) return rc;
        m->d_pods_synced = m->pods.size();
    }
    *last_index = hctl->L;
    if (evals) *evals += hctl->evals;
    if (n_overflowing) *n_overflowing = hctl->overflowing;
    fo.phases = hctl->phases;
    fo.steps = hctl->steps;
    fo.ring_scans = hctl->ring_scans;
    fo.windows = hctl->windows;
    fo.seq_share = hctl->all_cycles ? (float)((double)hctl->seq_cycles / (double)hctl->all_cycles) : 0.0f;
    fo.walk_cycles_per_pod = n ? (float)((double)hctl->seq_cycles / n) : 0.0f;
    for (int i = 0; i < 3; i++) fo.fb_cyc_per_pod[i] = n ? (float)((double)hctl->fb_cyc[i] / n) : 0.0f;
    tmark("host rows");
    fo.total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (n_placed) *n_placed = placed;
    return CA_OK;
}

int ca_filter_stats(const ca_mirror* m, float* out, int32_t cap) {
    if (!m || (!out && cap > 0)) return CA_EINVAL;
    const casim::FilterScratch& fo = m->fo;
    const float v[16] = {fo.kernel_ms, fo.total_ms, (float)fo.phases, (float)fo.steps, (float)fo.ring_scans,
                         (float)fo.windows, fo.seq_share, fo.walk_cycles_per_pod, (float)fo.path,
                         (float)fo.fb_shapes, (float)fo.fb_classes, fo.fb_cyc_per_pod[0], fo.fb_cyc_per_pod[1],
                         fo.fb_cyc_per_pod[2], 0.0f, (float)fo.fb_stat_lds};
    for (int32_t i = 0; i < cap && i < 16; i++) out[i] = v[i];
    return 16;
}

}  // extern "C"
