// estimate.hip — BinpackingNodeEstimator.Estimate for a batch of node groups.
//
// Reference: CA/estimator/binpacking_estimator.go:65-193,
//            CA/estimator/threshold_based_limiter.go:27-64,
//            CA/utils/scheduler/scheduler.go:73-91 (template copies),
//            CA/simulator/predicatechecker/schedulerbased.go:90-136 (rotating scan).
//
// Pipeline of one headline step (C2: uniform score classes, no cross-class float64 ties —
// the decoupled Go order):
//   st3 (high priority)  k_pdq_sort      Go 1.19 sort.Slice's exact permutation of every
//                                        group (class ranks folded in), one 1024-thread
//                                        workgroup per group; writes the Go-order pod ids
//                                        and an epoch-stamped ready flag per group.
//   st  (heavy groups)   k_run_table     class ranks + per-class counts of each group's
//                                        list, each rank's first stream position, the
//                                        class's stream record against the template.
//                        k_emit_runs     run heads and the stream windows that hold them.
//                        k_ffd_chain     one 4-wave workgroup per group: the sequential
//                                        First-Fit-Decreasing loop (per pod, or per run of
//                                        identical pods in closed form) with the new-node
//                                        rows in LDS; pushes 4096-output tickets.
//   st2 (light groups)   the same three kernels for the groups outside the heavy set.
//   pub_stream           k_publish       claims tickets in completion order and writes the
//                                        scheduled pods (Go-order ids) into the caller's
//                                        page-locked buffer while the chains run.
//   host                 lastIndex fix-up: groups whose result depends on their lastIndex
//                        input are re-run until every input equals its predecessor's
//                        output (exact); the host joins the streams.
// Other paths: non-uniform podsets (C4) sort in Go order first (k_class_rank, k_pdq_sort,
// radix passes, k_emit_bucket) and then chain; > 4096 score classes use k_score_tiles +
// k_merge_runs + k_emit_stream; device-resident results expand the chains' segments with
// k_copy_segments; a publisher that gives up falls back to the same copy + D2H.
#include "mirror.h"
#include "device_filters.h"
#include "pdqsort.h"

#include <cstring>
#include <algorithm>
#include <functional>
#include <chrono>
#include <mutex>
#include <thread>
#include <cstdlib>

namespace casim {

// per (group, pod) static bits computed against the template (k_score_tiles)
enum : uint32_t {
    SF_EVAL    = 0x1u,   // FitsAnyNode visits new nodes with filters (counts evals)
    SF_FA_OK   = 0x2u,   // static filters pass on the template (FitsAnyNode path)
    SF_CP_EVAL = 0x4u,   // CheckPredicates runs filters (PreFilter ok)
    SF_CP_OK   = 0x8u,   // static filters incl. NodeUnschedulable pass (CheckPredicates path)
    SF_ZERO    = 0x10u,  // PF_ALL_ZERO
    SF_SCALAR  = 0x20u,  // PF_SCALAR_REQ
    SF_PORTS   = 0x40u,  // PF_PORTS
    SF_UNSUP   = 0x80u,  // PF_HOSTNAME_DEP / PF_OUT_OF_SCOPE: group unsupported (casim.h scope)
};

struct alignas(16) SortItem {
    uint64_t key;     // ~ordered(score): ascending key == descending score
    uint32_t pos;     // position in the group's pod list (tie-break, stable)
    uint32_t flags;   // SF_*
};
static_assert(sizeof(SortItem) == 16, "SortItem");

struct alignas(16) StreamPod {
    int64_t cpu, mem, eph;
    int32_t pod;      // pod set index
    uint32_t flags;   // SF_* | SF_HEAD | SF_BATCH
};
static_assert(sizeof(StreamPod) == 32, "StreamPod");

// stream-only bits (k_emit_stream)
enum : uint32_t {
    SF_HEAD  = 0x100u,   // first pod of a run of identical consecutive pods
    SF_BATCH = 0x200u,   // run-batchable: resource-only (no ports / scalars), requests >= 0
};

struct alignas(16) GroupMeta {
    int64_t tcpu, tmem, teph;      // template free (alloc - template pods)
    int32_t tpods;                 // template free pod slots
    int32_t off;                   // offset into the pod lists / streams
    int32_t count;                 // pods in the group
    int32_t tmpl;                  // template index
    uint32_t tflags;               // NF_* of the template
    int32_t moff;                  // offset of the group's 64-pod head masks
    int32_t toff;                  // unused (was: compaction tile counters)
    int32_t hoff;                  // offset of the group's radix histograms [256][rtiles]
    int32_t rtiles;                // radix tiles of the group (bucket sort)
    int32_t pad;
};
static_assert(sizeof(GroupMeta) == 64, "GroupMeta");
// Group handled by a block: the launch's group map (a subset of the batch, e.g. the
// heavy groups launched first) or the block index itself.
#define GSEL(b) (gmap ? gmap[(b)] : (int)(b))

struct alignas(16) ChainOut {
    int32_t node_count, n_sched, nodes_added, lin;
    int32_t lout, status, sensitive, had_success;
    uint64_t evals;
    uint64_t pad;        // diagnostics (ca_estimate_plan_group_ticks)
    int32_t nseg;        // run-placement segments written to the group's segment list
    int32_t pad2[3];
};
static_assert(sizeof(ChainOut) == 64, "ChainOut");

// A run placement: stream positions [src, src+len) were scheduled as outputs
// [dst, dst+len) of the group (k_copy_segments fills sched_pod from them).
struct alignas(16) Seg {
    int32_t dst, src, len, pad;
};

constexpr int TILE = 1024;

__device__ inline uint64_t ordered_bits(double d) {
    if (d == 0.0) d = 0.0;   // -0 == +0 for the comparator (binpacking_estimator.go:74)
    uint64_t u = (uint64_t)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__device__ inline bool item_less(const SortItem& a, const SortItem& b) {
    return a.key < b.key || (a.key == b.key && a.pos < b.pos);
}

// SF_* bits of a pod against a group's template: the template-only part of the
// filter chain (schedulerbased.go:107-129 PreFilter / Unschedulable skip, framework.go
// order via dev_static_filters), evaluated once per (group, pod).  The full pod record
// is read only when a static filter can matter.
__device__ inline uint32_t static_sf(const PodHot& p, const ca_template& tp, bool tunsched,
                                     const ca_pod_spec* __restrict__ specs, const ca_selector_term* __restrict__ terms,
                                     const ca_selector_req* __restrict__ reqs) {
    uint32_t sf = 0;
    const bool pre_fail = (p.flags & PF_PREFILTER_FAIL) != 0;
    bool static_ok = true;
    if ((p.flags & (PF_NODE_NAME | PF_AFFINITY)) || (tp.node.taints && !(p.flags & PF_TAINT_MASK_ALL))) {
        const ca_pod_spec& s = specs[p.spec];
        if ((p.flags & (PF_NODE_NAME | PF_AFFINITY)) || (tp.node.taints & ~s.tolerated_taints)) {
            NodeStatic ns;
            ns.taints = tp.node.taints;
            for (int w = 0; w < CA_LABEL_WORDS; w++) ns.labels[w] = tp.node.label_pairs[w];
            ns.keys = tp.node.label_keys;
            for (int k = 0; k < CA_MAX_INT_KEYS; k++) ns.ints[k] = tp.node.int_label[k];
            ns.int_valid = tp.node.int_label_valid;
            ns.name_id = tp.node.name_id;
            static_ok = dev_static_filters(s, p.flags, terms, reqs, ns, false) == CA_PLUGIN_NONE;
        }
    }
    if (!pre_fail && !tunsched) sf |= SF_EVAL;                           // schedulerbased.go:125
    if ((sf & SF_EVAL) && static_ok) sf |= SF_FA_OK;
    if (!pre_fail) sf |= SF_CP_EVAL;
    if (!pre_fail && (!tunsched || (p.flags & PF_TOL_UNSCHED)) && static_ok) sf |= SF_CP_OK;
    if (p.flags & PF_ALL_ZERO) sf |= SF_ZERO;
    if (p.flags & PF_SCALAR_REQ) sf |= SF_SCALAR;
    if (p.flags & PF_PORTS) sf |= SF_PORTS;
    if (p.flags & (PF_HOSTNAME_DEP | PF_OUT_OF_SCOPE)) sf |= SF_UNSUP;
    return sf;
}

// the score class of every (group, pod) item, gathered from the podset's class column
__global__ void __launch_bounds__(256) k_item_cls(const int32_t* __restrict__ pod_idx, const int32_t* __restrict__ cls,
                                                 int32_t* __restrict__ out, int32_t n) {
    for (int32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) out[i] = cls[pod_idx[i]];
}

// 1. score + static predicates + tile sort ----------------------------------
__global__ void __launch_bounds__(256) k_score_tiles(
    const GroupMeta* __restrict__ groups, const int32_t* __restrict__ pod_idx, const ca_template* __restrict__ tmpls,
    const PodHot* __restrict__ ph, const ca_pod_spec* __restrict__ specs, const ca_selector_term* __restrict__ terms,
    const ca_selector_req* __restrict__ reqs, SortItem* __restrict__ out, uint32_t* __restrict__ group_unsup) {
    __shared__ SortItem tile[TILE];
    const GroupMeta gm = groups[blockIdx.y];
    const int32_t base = (int32_t)blockIdx.x * TILE;
    if (base >= gm.count) return;
    const int32_t n = min(TILE, gm.count - base);
    const ca_template& tp = tmpls[gm.tmpl];
    const int64_t acpu = tp.node.alloc_milli_cpu, amem = tp.node.alloc_memory;
    const bool tunsched = (tp.node.flags & CA_NODE_UNSCHEDULABLE) != 0;
    uint32_t unsup = 0;
    for (int t = threadIdx.x; t < TILE; t += blockDim.x) {
        SortItem it;
        if (t < n) {
            const int32_t pos = base + t;
            const int32_t pidx = pod_idx[gm.off + pos];
            const PodHot p = ph[pidx];
            const ca_pod_spec& s = specs[p.spec];
            // calculatePodScore (binpacking_estimator.go:164-193): containers-only sums
            double score = 0.0;
            if (acpu > 0) score += (double)s.score_milli_cpu / (double)acpu;
            if (amem > 0) score += (double)s.score_memory / (double)amem;
            const uint32_t sf = static_sf(p, tp, tunsched, specs, terms, reqs);
            if (sf & SF_UNSUP) unsup = 1;
            it.key = ~ordered_bits(score);
            it.pos = (uint32_t)pos;
            it.flags = sf;
        } else {
            it.key = ~0ull;
            it.pos = 0xFFFFFFFFu;
            it.flags = 0;
        }
        tile[t] = it;
    }
    if (unsup) atomicOr(&group_unsup[blockIdx.y], 1u);
    __syncthreads();
    // bitonic sort of TILE items, ascending (key, pos)
    for (int k = 2; k <= TILE; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < TILE; t += blockDim.x) {
                const int ixj = t ^ j;
                if (ixj > t) {
                    const SortItem a = tile[t], b = tile[ixj];
                    const bool up = (t & k) == 0;
                    if (up ? item_less(b, a) : item_less(a, b)) { tile[t] = b; tile[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (int t = threadIdx.x; t < n; t += blockDim.x) out[gm.off + base + t] = tile[t];
}

// 2. merge pass: runs of `width` -> runs of 2*width --------------------------
__global__ void __launch_bounds__(256) k_merge_runs(const GroupMeta* __restrict__ groups, const SortItem* __restrict__ src,
                                                   SortItem* __restrict__ dst, int32_t width) {
    const GroupMeta gm = groups[blockIdx.y];
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= gm.count) return;
    const SortItem* g = src + gm.off;
    const SortItem me = g[i];
    const int32_t run = i / width;
    const int32_t pair = run ^ 1;
    const int32_t pstart = pair * width;
    int32_t rank = 0;
    if (pstart < gm.count) {
        const int32_t pend = min(pstart + width, gm.count);
        int32_t lo = pstart, hi = pend;             // count partner items < me
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (item_less(g[mid], me)) lo = mid + 1; else hi = mid;
        }
        rank = lo - pstart;
    }
    const int32_t start = min(run, pair) * width;
    dst[gm.off + start + (i - run * width) + rank] = me;
}

// 3. gather the stream + run heads -------------------------------------------
// A run is a maximal sequence of consecutive sorted pods that behave identically on
// every new node: equal requests and equal SF_* bits, resource-only.  heads[] holds
// one 64-bit mask per 64 stream positions (bit set = a run starts there; positions
// past the group end are heads).
__device__ inline bool batchable(const PodHot& p, uint32_t sf) {
    return !(sf & (SF_PORTS | SF_SCALAR | SF_UNSUP)) && p.cpu >= 0 && p.mem >= 0 && p.eph >= 0;
}

__global__ void __launch_bounds__(256) k_emit_stream(const GroupMeta* __restrict__ groups, const SortItem* __restrict__ src,
                                                    const int32_t* __restrict__ pod_idx, const PodHot* __restrict__ ph,
                                                    StreamPod* __restrict__ out, int32_t* __restrict__ spod,
                                                    uint64_t* __restrict__ heads) {
    const GroupMeta gm = groups[blockIdx.y];
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    bool head = true;
    if (i < gm.count) {
        const SortItem it = src[gm.off + i];
        const int32_t pidx = pod_idx[gm.off + (int32_t)it.pos];
        const PodHot p = ph[pidx];
        const bool bat = batchable(p, it.flags);
        if (i > 0 && bat) {
            const SortItem pv = src[gm.off + i - 1];
            const PodHot q = ph[pod_idx[gm.off + (int32_t)pv.pos]];
            head = !(pv.flags == it.flags && q.cpu == p.cpu && q.mem == p.mem && q.eph == p.eph);
        }
        StreamPod sp;
        sp.cpu = p.cpu; sp.mem = p.mem; sp.eph = p.eph;
        sp.pod = pidx;
        sp.flags = it.flags | (head ? SF_HEAD : 0u) | (bat ? SF_BATCH : 0u);
        out[gm.off + i] = sp;
        spod[gm.off + i] = pidx;
    }
    const uint64_t hb = __ballot(head);
    if ((threadIdx.x & 63) == 0 && i < gm.count) heads[gm.moff + (i >> 6)] = hb;
}

// 1'-3'. bucket sort over score classes ----------------------------------------
// The sort key (score desc, list position asc) depends on a pod only through its
// score class (ca_podset: equal score_milli_cpu and score_memory) and its position.  So
// when the pod set has at most CLS_MAX classes, each group ranks its classes by score
// (k_class_rank: dense rank, equal scores share a rank = the tie-by-position rule H2),
// and its pod list — already in position order — is stably sorted by that rank with
// 8-bit LSD counting passes (k_radix_hist / k_radix_scan / k_radix_scatter; ranks of
// equal digits inside a wave by ballot multisplit).  k_emit_bucket then builds the
// stream exactly as k_emit_stream does from the comparison sort.  Same output as
// k_score_tiles + k_merge_runs + k_emit_stream, ~8 B of HBM per item and pass instead
// of ~300.
constexpr int CLS_MAX = 4096;
constexpr int RT = 2048;               // items per radix tile
constexpr int RTHREADS = 256;
constexpr int RPT = RT / RTHREADS;     // items per thread
constexpr int RCH = RT / 64 / (RTHREADS / 64);   // 64-item chunks per wave

// Dense ranks of the U score classes against a group's template, by one 1024-thread
// workgroup: float64 score of every class, bitonic sort of the classes in LDS, dense rank
// (equal scores share a rank).  On return sc[i] is the rank of class idx[i], i < U.
// block_class_rank for NP <= 64 by one wavefront, the class score sums already loaded
// (lane i: class i's cpu / memory sums; any value past U): lane i holds class i's key; its
// place in the (key, class) order and its dense rank are counts over the other lanes
// (readlane broadcasts, no barrier per bitonic stage).  Every thread of the block calls it.
__device__ inline void wave_class_rank(const ca_template& tp, int64_t s_cpu, int64_t s_mem, int32_t U, int32_t NP,
                                       uint64_t* key, uint32_t* idx, int32_t* sc) {
    const int64_t acpu = tp.node.alloc_milli_cpu, amem = tp.node.alloc_memory;
    if (threadIdx.x < 64) {
        const int lane = (int)threadIdx.x;
        uint64_t k = ~0ull;
        if (lane < U) {
            double score = 0.0;               // calculatePodScore, same float64 operations
            if (acpu > 0) score += (double)s_cpu / (double)acpu;
            if (amem > 0) score += (double)s_mem / (double)amem;
            k = ~ordered_bits(score);
        }
        const uint32_t klo = (uint32_t)k, khi = (uint32_t)(k >> 32);
        int pos = 0, eq_before = 0;
        for (int j = 0; j < NP; j++) {
            const uint64_t kj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(khi, j) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane(klo, j);
            pos += (kj < k || (kj == k && j < lane)) ? 1 : 0;
            eq_before += (kj == k && j < lane) ? 1 : 0;
        }
        const int first = eq_before == 0 ? 1 : 0;           // the lowest class holding its key
        int dense = 0;
        for (int j = 0; j < NP; j++) {
            const uint64_t kj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(khi, j) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane(klo, j);
            dense += (__builtin_amdgcn_readlane(first, j) && kj < k) ? 1 : 0;
        }
        if (lane < NP) { key[pos] = k; idx[pos] = (uint32_t)lane; sc[pos] = dense; }
    }
    __syncthreads();
}

__device__ inline void block_class_rank(const ca_template& tp, const int64_t* __restrict__ cls_sc, int32_t U,
                                        int32_t NP, uint64_t* key, uint32_t* idx, int32_t* sc) {
    const int64_t acpu = tp.node.alloc_milli_cpu, amem = tp.node.alloc_memory;
    if (NP <= 64) {
        const int l = (int)threadIdx.x;
        const int64_t c0 = l < U ? cls_sc[2 * l] : 0, c1 = l < U ? cls_sc[2 * l + 1] : 0;
        wave_class_rank(tp, c0, c1, U, NP, key, idx, sc);
        return;
    }
    for (int i = threadIdx.x; i < NP; i += blockDim.x) {
        uint64_t k = ~0ull;
        if (i < U) {
            // calculatePodScore (binpacking_estimator.go:164-193), same float64 operations
            double score = 0.0;
            if (acpu > 0) score += (double)cls_sc[2 * i] / (double)acpu;
            if (amem > 0) score += (double)cls_sc[2 * i + 1] / (double)amem;
            k = ~ordered_bits(score);            // ascending key == descending score
        }
        key[i] = k;
        idx[i] = (uint32_t)i;
    }
    __syncthreads();
    for (int k = 2; k <= NP; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < NP; t += blockDim.x) {
                const int ixj = t ^ j;
                if (ixj > t) {
                    const uint64_t a = key[t], b = key[ixj];
                    const uint32_t ia = idx[t], ib = idx[ixj];
                    const bool up = (t & k) == 0;
                    const bool less_ba = b < a || (b == a && ib < ia);
                    const bool less_ab = a < b || (a == b && ia < ib);
                    if (up ? less_ba : less_ab) { key[t] = b; key[ixj] = a; idx[t] = ib; idx[ixj] = ia; }
                }
            }
            __syncthreads();
        }
    }
    // dense rank: number of distinct keys before
    for (int i = threadIdx.x; i < NP; i += blockDim.x) sc[i] = (i > 0 && key[i] != key[i - 1]) ? 1 : 0;
    __syncthreads();
    for (int o = 1; o < NP; o <<= 1) {
        int32_t v[CLS_MAX / 1024];
        int n = 0;
        for (int i = threadIdx.x; i < NP; i += blockDim.x) v[n++] = (i >= o ? sc[i - o] : 0);
        __syncthreads();
        n = 0;
        for (int i = threadIdx.x; i < NP; i += blockDim.x) sc[i] += v[n++];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(1024) k_class_rank(const GroupMeta* __restrict__ groups,
                                                    const ca_template* __restrict__ tmpls,
                                                    const int64_t* __restrict__ cls_sc, int32_t U, int32_t NP,
                                                    int32_t* __restrict__ crank,
    const int32_t* __restrict__ gmap) {
    __shared__ uint64_t key[CLS_MAX];
    __shared__ uint32_t idx[CLS_MAX];
    __shared__ int32_t sc[CLS_MAX];
    const int gi = GSEL(blockIdx.x);
    const GroupMeta gm = groups[gi];
    block_class_rank(tmpls[gm.tmpl], cls_sc, U, NP, key, idx, sc);
    for (int i = threadIdx.x; i < U; i += blockDim.x) crank[(size_t)gi * U + idx[i]] = sc[i];
}

__device__ inline uint32_t item_digit(const GroupMeta& gm, const uint32_t* __restrict__ src, int32_t i,
                                      const int32_t* __restrict__ pod_idx, const int32_t* __restrict__ pcls,
                                      const int32_t* __restrict__ crank_g, int shift, uint32_t* pos_out) {
    const uint32_t pos = src ? src[gm.off + i] : (uint32_t)i;
    *pos_out = pos;
    const int32_t pidx = pod_idx[gm.off + (int32_t)pos];
    return ((uint32_t)crank_g[pcls[pidx]] >> shift) & 255u;
}

__global__ void __launch_bounds__(RTHREADS) k_radix_hist(const GroupMeta* __restrict__ groups,
                                                        const uint32_t* __restrict__ src,
                                                        const int32_t* __restrict__ pod_idx,
                                                        const int32_t* __restrict__ pcls,
                                                        const int32_t* __restrict__ crank, int32_t U, int shift,
                                                        int32_t* __restrict__ hist, const int32_t* __restrict__ gmap) {
    __shared__ int32_t h[256];
    const int gi = GSEL(blockIdx.y);
    const GroupMeta gm = groups[gi];
    const int32_t t = (int32_t)blockIdx.x;
    if (t >= gm.rtiles) return;
    h[threadIdx.x] = 0;
    __syncthreads();
    const int32_t* cr = crank + (size_t)gi * U;
    const int32_t base = t * RT;
    for (int r = 0; r < RPT; r++) {
        const int32_t i = base + r * RTHREADS + (int32_t)threadIdx.x;
        if (i < gm.count) {
            uint32_t pos;
            atomicAdd(&h[item_digit(gm, src, i, pod_idx, pcls, cr, shift, &pos)], 1);
        }
    }
    __syncthreads();
    hist[gm.hoff + (int32_t)threadIdx.x * gm.rtiles + t] = h[threadIdx.x];
}

// exclusive scan of the group's [256][rtiles] histogram, digit-major: thread d owns
// digit d's row (its tiles, contiguous), so the scan is one row sum per thread, one
// block scan of the 256 row totals and one pass writing the row's prefixes — two
// barriers instead of two per 256 entries.
__global__ void __launch_bounds__(256) k_radix_scan(const GroupMeta* __restrict__ groups, int32_t* __restrict__ hist,
                                                   const int32_t* __restrict__ gmap) {
    __shared__ int32_t wsum[4];
    const GroupMeta gm = groups[GSEL(blockIdx.x)];
    const int32_t nt = gm.rtiles;
    int32_t* row = hist + gm.hoff + (int32_t)threadIdx.x * nt;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int32_t tot = 0;
    for (int32_t j = 0; j < nt; j++) tot += row[j];
    int32_t x = tot;                                     // inclusive wave scan of row totals
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int32_t pre = x - tot;
    for (int q = 0; q < w; q++) pre += wsum[q];
    for (int32_t j = 0; j < nt; j++) {
        const int32_t v = row[j];
        row[j] = pre;
        pre += v;
    }
}

__global__ void __launch_bounds__(RTHREADS) k_radix_scatter(const GroupMeta* __restrict__ groups,
                                                           const uint32_t* __restrict__ src,
                                                           const int32_t* __restrict__ pod_idx,
                                                           const int32_t* __restrict__ pcls,
                                                           const int32_t* __restrict__ crank, int32_t U, int shift,
                                                           const int32_t* __restrict__ hist,
                                                           uint32_t* __restrict__ dst, const int32_t* __restrict__ gmap) {
    __shared__ int32_t wcnt[RTHREADS / 64][256];
    const int gi = GSEL(blockIdx.y);
    const GroupMeta gm = groups[gi];
    const int32_t t = (int32_t)blockIdx.x;
    if (t >= gm.rtiles) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int d = lane; d < 256; d += 64) wcnt[w][d] = 0;
    __builtin_amdgcn_wave_barrier();
    const int32_t* cr = crank + (size_t)gi * U;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t dg[RCH], pv[RCH];
    int32_t rk[RCH];
    const int32_t wbase = t * RT + w * (RCH * 64);       // wave w owns RCH consecutive chunks
    for (int c = 0; c < RCH; c++) {
        const int32_t i = wbase + c * 64 + lane;
        const bool valid = i < gm.count;
        uint32_t pos = 0, d = 0;
        if (valid) d = item_digit(gm, src, i, pod_idx, pcls, cr, shift, &pos);
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const int32_t before = wcnt[w][valid ? d : 0];
        const int32_t r = before + __builtin_popcountll(peers & lt);
        __builtin_amdgcn_wave_barrier();
        if (valid && (peers & lt) == 0) wcnt[w][d] = before + __builtin_popcountll(peers);
        __builtin_amdgcn_wave_barrier();
        dg[c] = valid ? d : 0xFFFFFFFFu;
        pv[c] = pos;
        rk[c] = r;
    }
    __syncthreads();
    // offset of wave w inside each digit of the tile: the counts of waves before it
    int32_t pre[RTHREADS / 64];
    if (threadIdx.x < 256) {
        int32_t acc = 0;
        for (int q = 0; q < RTHREADS / 64; q++) { pre[q] = acc; acc += wcnt[q][threadIdx.x]; }
    }
    __syncthreads();
    if (threadIdx.x < 256)
        for (int q = 0; q < RTHREADS / 64; q++) wcnt[q][threadIdx.x] = pre[q] + hist[gm.hoff + (int32_t)threadIdx.x * gm.rtiles + t];
    __syncthreads();
    for (int c = 0; c < RCH; c++) {
        if (dg[c] == 0xFFFFFFFFu) continue;
        dst[gm.off + wcnt[w][dg[c]] + rk[c]] = pv[c];
    }
}

// 1*-3*. decoupled Go order: the stable class order of a group is its
// classes in rank order, each class's pods together, and every pod of a class is the same
// record but for its controller — so the chain stream follows from per-class counts alone,
// with no sort of the pod list.  k_run_table (one workgroup per group; the class ranks
// computed in its prologue): the class counts of the group's list, each rank's first
// stream position rstart[g][r] (r in [0, U]), and the stream record of the rank's class
// rsp[g][r] (its representative pod's requests and static bits against the template);
// round 1 without k_round_init it also sets the group's lastIndex input / need /
// unsupported flags.  k_emit_runs: the stream itself.  The pod id of a stream entry is not
// needed: decoupled chains emit stream positions and the consumers map them through the
// Go-order ids.
#ifdef CASIM_PROF
// k_run_table phase cycles per group slot (< 1024): ranking, counting, scan, records
__device__ unsigned long long g_rt_prof[1024][4];
#endif
__device__ inline int32_t run_rank(const int32_t* __restrict__ st, int32_t U, int32_t i) {
    int32_t lo = 0, hi = U;                  // the last r with st[r] <= i (st[U] is never read)
    while (hi - lo > 1) {
        const int32_t mid = (lo + hi) >> 1;
        if (st[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(1024) k_run_table(const GroupMeta* __restrict__ groups,
                                                   const int32_t* __restrict__ item_cls,
                                                   const int64_t* __restrict__ cls_sc, int32_t NP,
                                                   const int32_t* __restrict__ cls_rep,
                                                   int32_t U, const ca_template* __restrict__ tmpls,
                                                   const PodHot* __restrict__ ph, const ca_pod_spec* __restrict__ specs,
                                                   const ca_selector_term* __restrict__ terms,
                                                   const ca_selector_req* __restrict__ reqs, int32_t* __restrict__ rstart,
                                                   StreamPod* __restrict__ rsp, uint32_t* __restrict__ group_unsup,
                                                   const int32_t* __restrict__ gmap,
                                                   int32_t* __restrict__ lin, uint8_t* __restrict__ need, int32_t lin0) {
    // lin != null: round 1 without k_round_init — the group's lastIndex input, need flag and
    // unsupported flag are set here (stored, not or-ed)
    __shared__ int32_t cnt[CLS_MAX];
    __shared__ uint32_t s_unsup;
    __shared__ int32_t rc[CLS_MAX];
    __shared__ int32_t cr[CLS_MAX];           // rank of each class
    __shared__ uint64_t key[CLS_MAX];
    __shared__ uint32_t idx[CLS_MAX];
    __shared__ int32_t wsum[16];
    const int gi = GSEL(blockIdx.x);
    const GroupMeta gm = groups[gi];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_unsup = 0;
#ifdef CASIM_PROF
    const uint64_t t_r0 = clock64();
#endif
    // Each wave counts a contiguous region of the list, 64 positions per step (classes come
    // in runs: a wave adds a run to a register and touches the LDS counter once per run —
    // with every wave on a strided slice the same few counters took ~1 000 contended LDS
    // atomics per group).  The class scores (ranking, up to 64 classes) are requested
    // first and the region's first RUB steps right after — all of a C2 group's list (up to
    // 64 x 64 x 16 positions) — so the ranking waits only for the scores.  (Measured,
    // CASIM_PROF: counting stays ~40k of the kernel's ~65k cycles whether the loads go in
    // slices or all at once, and with strided or contiguous slices — not memory latency,
    // not the LDS atomics)
    constexpr int RUB = 64;
    const int32_t per_w = ((gm.count + 15) / 16 + 63) & ~63;
    const int32_t wb0 = min(gm.count, w * per_w), wb1 = min(gm.count, wb0 + per_w);
    const bool small = NP <= 64;
    int64_t s_cpu = 0, s_mem = 0;
    if (small && tid < U) { s_cpu = cls_sc[2 * tid]; s_mem = cls_sc[2 * tid + 1]; }
    int32_t cv[RUB];
#pragma unroll
    for (int u = 0; u < RUB; u++) {
        const int32_t i = wb0 + u * 64 + lane;
        cv[u] = i < wb1 ? item_cls[gm.off + i] : -1;
    }
    if (small) wave_class_rank(tmpls[gm.tmpl], s_cpu, s_mem, U, NP, key, idx, rc);   // (rc: scratch)
    else block_class_rank(tmpls[gm.tmpl], cls_sc, U, NP, key, idx, rc);
    for (int i = tid; i < U; i += 1024) cr[idx[i]] = rc[i];
    __syncthreads();
    for (int i = tid; i < U; i += 1024) { cnt[i] = 0; rc[i] = 0; }
    __syncthreads();
#ifdef CASIM_PROF
    const uint64_t t_r1 = clock64();
#endif
    // class counts over the wave's region
    int32_t cur = -1, acc = 0;                // (wave-uniform) the run being added up
    for (int32_t base = wb0; base < wb1; base += 64 * RUB) {
        if (base > wb0) {                     // (groups past 65 536 positions)
#pragma unroll
            for (int u = 0; u < RUB; u++) {
                const int32_t i = base + u * 64 + lane;
                cv[u] = i < wb1 ? item_cls[gm.off + i] : -1;
            }
        }
#pragma unroll
        for (int u = 0; u < RUB; u++) {
            const bool valid = cv[u] >= 0;
            const int32_t c = cv[u];
            const uint64_t vm = __ballot(valid);
            if (!vm) continue;
            const int32_t c0 = __builtin_amdgcn_readlane(c, __builtin_ctzll(vm));
            if (__ballot(valid && c != c0) == 0) {          // one class in this step
                if (c0 == cur) {
                    acc += __builtin_popcountll(vm);
                } else {
                    if (acc > 0 && lane == 0) atomicAdd(&cnt[cur], acc);
                    cur = c0;
                    acc = __builtin_popcountll(vm);
                }
                continue;
            }
            uint64_t act = vm;                                // a class boundary in the step
            while (act) {
                const int l = __builtin_ctzll(act);
                const int32_t cl = __builtin_amdgcn_readlane(c, l);
                const uint64_t m = __ballot(valid && c == cl) & act;
                if (lane == l) atomicAdd(&cnt[cl], __builtin_popcountll(m));
                act &= ~m;
            }
        }
    }
    if (acc > 0 && lane == 0) atomicAdd(&cnt[cur], acc);
    __syncthreads();
    for (int c = tid; c < U; c += 1024)
        if (cnt[c] > 0) atomicAdd(&rc[cr[c]], cnt[c]);
    __syncthreads();
#ifdef CASIM_PROF
    const uint64_t t_r2 = clock64();
#endif
    // exclusive scan of the counts by rank: thread t owns ranks [4t, 4t + 4)
    int32_t v[4], loc = 0;
    for (int q = 0; q < 4; q++) { const int r = 4 * tid + q; v[q] = r < U ? rc[r] : 0; loc += v[q]; }
    int32_t x = loc;
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int32_t pre = x - loc;
    for (int q = 0; q < w; q++) pre += wsum[q];
    int32_t* rs = rstart + (size_t)gi * (U + 1);
    for (int q = 0; q < 4; q++) {
        const int r = 4 * tid + q;
        if (r < U) rs[r] = pre;
        pre += v[q];
    }
    if (tid == 0) rs[U] = gm.count;
#ifdef CASIM_PROF
    const uint64_t t_r3 = clock64();
#endif
    // the record of each present class, at its rank
    const ca_template& tp = tmpls[gm.tmpl];
    const bool tunsched = (tp.node.flags & CA_NODE_UNSCHEDULABLE) != 0;
    uint32_t unsup = 0;
    for (int c = tid; c < U; c += 1024) {
        if (cnt[c] == 0) continue;
        const PodHot p = ph[cls_rep[c]];
        const uint32_t sf = static_sf(p, tp, tunsched, specs, terms, reqs);
        StreamPod sp;
        sp.cpu = p.cpu; sp.mem = p.mem; sp.eph = p.eph;
        sp.pod = cls_rep[c];
        sp.flags = sf | (batchable(p, sf) ? SF_BATCH : 0u);
        rsp[(size_t)gi * U + cr[c]] = sp;
        unsup |= sf & SF_UNSUP;
    }
    if (unsup) atomicOr(&s_unsup, 1u);
    __syncthreads();                              // s_unsup
    if (tid == 0) {
        if (lin) { lin[gi] = lin0; need[gi] = 1; group_unsup[gi] = s_unsup ? 1u : 0u; }
        else if (s_unsup) atomicOr(&group_unsup[gi], 1u);
#ifdef CASIM_PROF
        if (gi < 1024) {
            const uint64_t t_r4 = clock64();
            g_rt_prof[gi][0] = t_r1 - t_r0; g_rt_prof[gi][1] = t_r2 - t_r1;
            g_rt_prof[gi][2] = t_r3 - t_r2; g_rt_prof[gi][3] = t_r4 - t_r3;
        }
#endif
    }
}

// The stream from the run table: one thread per position — position -> rank by binary
// search of the rank starts in LDS, the record, run heads exactly as k_emit_bucket marks
// them.  (Measured against a variant inside k_run_table, one thread per 64-position
// window: 0.49 against 0.50 ms per headline step — the wide grid wins.)
__global__ void __launch_bounds__(256) k_emit_runs(const GroupMeta* __restrict__ groups,
                                                  const int32_t* __restrict__ rstart, const StreamPod* __restrict__ rsp,
                                                  int32_t U, StreamPod* __restrict__ out, uint64_t* __restrict__ heads,
                                                  const int32_t* __restrict__ gmap, int32_t all_windows) {
    __shared__ int32_t st[CLS_MAX + 1];
    const int gi = GSEL(blockIdx.y);
    const GroupMeta gm = groups[gi];
    const int32_t base = (int32_t)(blockIdx.x * blockDim.x);
    if (base >= gm.count) return;                                   // (uniform per block)
    const int32_t* rs = rstart + (size_t)gi * (U + 1);
    for (int r = threadIdx.x; r <= U; r += blockDim.x) st[r] = rs[r];
    __syncthreads();
    const int32_t i = base + (int32_t)threadIdx.x;
    const int lane = threadIdx.x & 63;
    if (base + (int32_t)(threadIdx.x & ~63u) >= gm.count) return;   // whole wave past the end
    bool head = true;
    StreamPod sp = {};
    if (i < gm.count) {
        const int32_t r = run_rank(st, U, i);
        sp = rsp[(size_t)gi * U + r];
        const bool bat = (sp.flags & SF_BATCH) != 0;
        if (i > 0 && bat) {
            head = false;
            if (i == st[r]) {                                       // first pod of its class
                const StreamPod q = rsp[(size_t)gi * U + run_rank(st, U, i - 1)];
                head = !((q.flags & ~SF_BATCH) == (sp.flags & ~SF_BATCH) && q.cpu == sp.cpu && q.mem == sp.mem &&
                         q.eph == sp.eph);
            }
        }
        sp.flags |= head ? SF_HEAD : 0u;
    }
    const uint64_t hb = __ballot(head);
    if (lane == 0) heads[gm.moff + (i >> 6)] = hb;
    // With run batching the chain reads a stream entry only at a run head or inside a
    // non-batchable run (whose every pod is a head), and only from the 64-entry window
    // holding it: windows without a head are never read, so they are not written (C2: ~1
    // window in 10 has a head).  The per-pod chain (CASIM_RUN_BATCH=0) reads every window.
    if ((hb != 0 || all_windows) && i < gm.count) out[gm.off + i] = sp;
}

// 1''-2''. Go 1.19 sort.Slice order (binpacking_estimator.go:74; pdqsort.h) ----------
// One 1024-thread workgroup per group: the rank of every position of the group's list
// (its class's dense rank, k_class_rank, or an explicit per-position rank from
// k_item_rank), then pdqsort_func's exact permutation.  Groups of at most lds_n pods with
// at most 256 ranks sort in LDS (16-bit positions + 8-bit ranks); the others in global
// memory (rank above position in 32 or 64 bits).  Output: sorted[off + k] = position of
// the k-th pod, the same layout as the radix sort's.  force (tests): 1 LDS, 2 / 3 global.
// Scratch per group: gE [off, off+n) (8 B), scr [off, off+n), stack from off/2 + 2g.
constexpr int PDQ_LDS_N = 50368;       // ~3.16 B per pod + the static control block (~4.6 KB) <= 160 KB
// dynamic LDS of k_pdq_sort for groups of up to lds_n pods: positions (2 B), ranks (1 B),
// the partition's right-zone bitmap (1 bit) and its per-word prefix counts (2 B / 64)
__host__ __device__ inline size_t pdq_lds_bytes(int32_t lds_n) {
    const size_t np = ((size_t)std::max(lds_n, 0) + 63) & ~(size_t)63;
    return (3 * np + np / 8 + 2 * (np / 64 + 1) + 15) & ~(size_t)15;
}

#ifndef CASIM_PDQ_UB
#define CASIM_PDQ_UB 8
#endif
constexpr int PDQ_UB = CASIM_PDQ_UB;   // list positions per thread whose gathers are in flight together
__global__ void __launch_bounds__(pdq::NT) k_pdq_sort(const GroupMeta* __restrict__ groups,
                                                     const int32_t* __restrict__ pod_idx,
                                                     const int32_t* __restrict__ pcls,
                                                     const int32_t* __restrict__ crank, int32_t U,
                                                     const uint32_t* __restrict__ item_rank,
                                                     uint32_t* __restrict__ sorted, uint64_t* __restrict__ gE,
                                                     uint64_t* __restrict__ xs_all, pdq::Frame* __restrict__ stack_all,
                                                     int32_t lds_n, int32_t force, int32_t limit0, const int32_t* __restrict__ gmap,
                                                     int32_t* __restrict__ ids_out, int32_t* __restrict__ ids_ready,
                                                     int32_t ids_epoch, const int32_t* __restrict__ item_cls,
                                                     const ca_template* __restrict__ tmpls,
                                                     const int64_t* __restrict__ cls_sc, int32_t NP) {
    extern __shared__ __align__(16) unsigned char pdq_dyn[];
    __shared__ pdq::Ctl ctl;
#ifdef CASIM_PROF
    const uint64_t t_k0 = clock64();
#endif
    const int gi = GSEL(blockIdx.x);
    const GroupMeta gm = groups[gi];
    const int32_t n = gm.count, off = gm.off;
    const int tid = threadIdx.x;
    uint32_t* scr = reinterpret_cast<uint32_t*>(xs_all + off);    // ranks, then the exchange scratch
    pdq::Frame* stack = stack_all + off / 2 + 2 * gi;
    if (tid == 0) ctl.rmax = 0;
    __syncthreads();
    const bool fit = n <= lds_n;
    const size_t npad = ((size_t)lds_n + 63) & ~(size_t)63;
    uint16_t* e16 = reinterpret_cast<uint16_t*>(pdq_dyn);
    uint8_t* rk = pdq_dyn + 2 * npad;
    uint64_t* rmb = reinterpret_cast<uint64_t*>(pdq_dyn + 3 * npad);
    uint16_t* rmp = reinterpret_cast<uint16_t*>(rmb + npad / 64);
    // cls_sc != null: the class ranks are computed here (k_class_rank's work, one launch
    // less on the sort's critical path): the bitonic scratch lives in the element store
    // (free until the ranks are loaded), the rank of each class in the partition bitmap
    // area (free until the first partition); the host checks both fit
    const uint16_t* crk = nullptr;
    // the first slice of the list's classes is requested before the class ranking, so its
    // latency hides behind the ranking's barriers
    int32_t pre[PDQ_UB];
    const bool preload = item_cls && !item_rank;
    if (preload) {
#pragma unroll
        for (int u = 0; u < PDQ_UB; u++) { const int32_t i = tid + u * pdq::NT; pre[u] = i < n ? item_cls[off + i] : 0; }
    }
    if (cls_sc) {
        uint64_t* key = reinterpret_cast<uint64_t*>(pdq_dyn);
        uint32_t* idx = reinterpret_cast<uint32_t*>(pdq_dyn + 8 * (size_t)NP);
        int32_t* scv = reinterpret_cast<int32_t*>(pdq_dyn + 12 * (size_t)NP);
        block_class_rank(tmpls[gm.tmpl], cls_sc, U, NP, key, idx, scv);
        uint16_t* w = reinterpret_cast<uint16_t*>(rmb);
        for (int i = tid; i < U; i += pdq::NT) w[idx[i]] = (uint16_t)scv[i];
        __syncthreads();
        crk = w;
    }
    uint32_t rmax = 0;
    // the ranks of the list: a chain of three dependent gathers per position (list -> pod ->
    // class -> rank), issued PDQ_UB positions at a time so their latencies overlap
    for (int32_t i0 = tid; i0 < n; i0 += pdq::NT * PDQ_UB) {
        uint32_t r[PDQ_UB];
        if (item_rank) {
#pragma unroll
            for (int u = 0; u < PDQ_UB; u++) { const int32_t i = i0 + u * pdq::NT; r[u] = i < n ? item_rank[off + i] : 0u; }
        } else {
            int32_t pi[PDQ_UB], cl[PDQ_UB];
            if (item_cls && preload && i0 == tid) {
#pragma unroll
                for (int u = 0; u < PDQ_UB; u++) cl[u] = pre[u];
            } else if (item_cls) {
#pragma unroll
                for (int u = 0; u < PDQ_UB; u++) { const int32_t i = i0 + u * pdq::NT; cl[u] = i < n ? item_cls[off + i] : 0; }
            } else {
#pragma unroll
                for (int u = 0; u < PDQ_UB; u++) { const int32_t i = i0 + u * pdq::NT; pi[u] = i < n ? pod_idx[off + i] : 0; }
#pragma unroll
                for (int u = 0; u < PDQ_UB; u++) { const int32_t i = i0 + u * pdq::NT; cl[u] = i < n ? pcls[pi[u]] : 0; }
            }
#pragma unroll
            for (int u = 0; u < PDQ_UB; u++) {
                const int32_t i = i0 + u * pdq::NT;
                r[u] = i < n ? (crk ? (uint32_t)crk[cl[u]] : (uint32_t)crank[(size_t)gi * U + cl[u]]) : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < PDQ_UB; u++) {
            const int32_t i = i0 + u * pdq::NT;
            if (i >= n) break;
            rmax = max(rmax, r[u]);
            if (fit) { e16[i] = (uint16_t)i; rk[i] = (uint8_t)r[u]; }
            else scr[i] = r[u];                        // (the LDS store keeps its ranks in LDS)
        }
    }
    for (int d = 32; d >= 1; d >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, d, 64));
    if ((tid & 63) == 0) atomicMax(&ctl.rmax, rmax);
    __syncthreads();
    const uint32_t R = ctl.rmax;
    int mode = (fit && R < 256) ? 1 : (n <= (1 << 20) && R < 4096) ? 2 : 3;
    if (force == 1 && fit && R < 256) mode = 1;
    else if (force == 2 && n <= (1 << 20) && R < 4096) mode = 2;
    else if (force == 3) mode = 3;
    if (mode != 1 && fit) {
        // the ranks went to LDS only (8 bits): gather them again for a global store (a group
        // that fits LDS but has >= 256 ranks, or a forced store in tests)
        for (int32_t i = tid; i < n; i += pdq::NT) {
            uint32_t r;
            if (item_rank) r = item_rank[off + i];
            else {
                const int32_t cl = item_cls ? item_cls[off + i] : pcls[pod_idx[off + i]];
                r = crk ? (uint32_t)crk[cl] : (uint32_t)crank[(size_t)gi * U + cl];
            }
            scr[i] = r;
        }
        __syncthreads();
    }
    if (mode == 1) {
        const pdq::LdsStore st{e16, rk, rmb, rmp};
#ifdef CASIM_PROF
        const uint64_t t_k1 = clock64();
#endif
        pdq::wg_sort(st, n, stack, n / 2 + 2, scr, ctl, limit0);
#ifdef CASIM_PROF
        const uint64_t t_k2 = clock64();
#endif
        if (ids_out) {
            // decoupled Go order: the pod ids in sorted order.  A gather pod_idx[off +
            // e16[k]] straight from memory was ~40 % of the slowest workgroup's time on C2
            // (random 4-byte reads, every group at once); instead the group's list goes
            // through the LDS the sort no longer needs (the rank bytes and the partition
            // bitmaps) in coalesced slices, and each pass picks the sorted positions that
            // fall in its slice.
            int32_t* const buf = reinterpret_cast<int32_t*>(rk);
            // (npad >= 64: at least 16 entries per slice)
            const int32_t cap = (int32_t)((npad + (npad / 64) * 10) / 4);
            for (int32_t lo = 0; lo < n; lo += cap) {
                const int32_t hi = min(n, lo + cap);
                __syncthreads();                       // (the previous slice is consumed)
                constexpr int SL = 16;                 // a slice is one round of loads per thread
                for (int32_t j0 = lo + tid; j0 < hi; j0 += pdq::NT * SL) {
                    int32_t v[SL];
#pragma unroll
                    for (int u = 0; u < SL; u++) {
                        const int32_t j = j0 + u * pdq::NT;
                        v[u] = j < hi ? pod_idx[off + j] : 0;
                    }
#pragma unroll
                    for (int u = 0; u < SL; u++) {
                        const int32_t j = j0 + u * pdq::NT;
                        if (j < hi) buf[j - lo] = v[u];
                    }
                }
                __syncthreads();
                for (int32_t k = tid; k < n; k += pdq::NT) {
                    const int32_t pos = e16[k];
                    if (pos >= lo && pos < hi) ids_out[off + k] = buf[pos - lo];
                }
            }
        } else
            for (int32_t k = tid; k < n; k += pdq::NT) sorted[off + k] = e16[k];
#ifdef CASIM_PROF
        __syncthreads();
        if (tid == 0 && gi < 128) {
            const uint64_t t_k3 = clock64();
            pdq::g_pdq_wg[3 * gi] = t_k3 - t_k0;
            pdq::g_pdq_wg[3 * gi + 1] = t_k1 - t_k0;
            pdq::g_pdq_wg[3 * gi + 2] = t_k3 - t_k2;
        }
#endif
    } else if (mode == 2) {
        uint32_t* e = reinterpret_cast<uint32_t*>(gE + off);
        for (int32_t i = tid; i < n; i += pdq::NT) e[i] = (scr[i] << 20) | (uint32_t)i;
        __syncthreads();
        const pdq::G32Store st{e};
        pdq::wg_sort(st, n, stack, n / 2 + 2, scr, ctl, limit0);
        if (ids_out)
            for (int32_t k = tid; k < n; k += pdq::NT) ids_out[off + k] = pod_idx[off + (int32_t)(e[k] & 0xFFFFFu)];
        else
            for (int32_t k = tid; k < n; k += pdq::NT) sorted[off + k] = e[k] & 0xFFFFFu;
    } else {
        uint64_t* e = gE + off;
        for (int32_t i = tid; i < n; i += pdq::NT) e[i] = ((uint64_t)scr[i] << 32) | (uint32_t)i;
        __syncthreads();
        const pdq::G64Store st{e};
        pdq::wg_sort(st, n, stack, n / 2 + 2, xs_all + off, ctl, limit0);
        if (ids_out)
            for (int32_t k = tid; k < n; k += pdq::NT) ids_out[off + k] = pod_idx[off + (int32_t)(uint32_t)e[k]];
        else
            for (int32_t k = tid; k < n; k += pdq::NT) sorted[off + k] = (uint32_t)e[k];
    }
    if (ids_ready) {                                   // this group's ids are final
        __syncthreads();
        if (tid == 0) {
            __threadfence();
            __hip_atomic_store(&ids_ready[gi], ids_epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Dense rank of every position of a group's list from the comparison-sorted items
// (k_score_tiles + k_merge_runs: ascending key == descending float64 score): equal scores
// share a rank.  The Go-order path for pod sets with more than CLS_MAX score classes.
__global__ void __launch_bounds__(1024) k_item_rank(const GroupMeta* __restrict__ groups,
                                                   const SortItem* __restrict__ items, uint32_t* __restrict__ item_rank) {
    __shared__ uint32_t wtot[16];
    const GroupMeta gm = groups[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t carry = 0;
    for (int32_t base = 0; base < gm.count; base += 1024) {
        const int32_t i = base + tid;
        const bool valid = i < gm.count;
        SortItem it = {};
        uint32_t f = 0;
        if (valid) {
            it = items[gm.off + i];
            f = (i > 0 && items[gm.off + i - 1].key != it.key) ? 1u : 0u;
        }
        uint32_t incl = f;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) wtot[w] = incl;
        __syncthreads();
        uint32_t pre = carry, tot = carry;
        for (int q = 0; q < 16; q++) { if (q < w) pre += wtot[q]; tot += wtot[q]; }
        if (valid) item_rank[gm.off + (int32_t)it.pos] = pre + incl;
        carry = tot;
        __syncthreads();
    }
}

// stream of one group from the bucket-sorted positions (same output as k_emit_stream)
__global__ void __launch_bounds__(256) k_emit_bucket(const GroupMeta* __restrict__ groups,
                                                    const uint32_t* __restrict__ sorted,
                                                    const int32_t* __restrict__ pod_idx, const ca_template* __restrict__ tmpls,
                                                    const PodHot* __restrict__ ph, const ca_pod_spec* __restrict__ specs,
                                                    const ca_selector_term* __restrict__ terms,
                                                    const ca_selector_req* __restrict__ reqs,
                                                    StreamPod* __restrict__ out, int32_t* __restrict__ spod,
                                                    uint64_t* __restrict__ heads, uint32_t* __restrict__ group_unsup,
                                                    const int32_t* __restrict__ gmap) {
    const int gi = GSEL(blockIdx.y);
    const GroupMeta gm = groups[gi];
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int lane = threadIdx.x & 63;
    if ((int32_t)(blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) >= gm.count) return;   // whole wave past the end
    const ca_template& tp = tmpls[gm.tmpl];
    const bool tunsched = (tp.node.flags & CA_NODE_UNSCHEDULABLE) != 0;
    const bool valid = i < gm.count;
    PodHot p = {};
    uint32_t sf = 0;
    int32_t pidx = 0;
    if (valid) {
        pidx = pod_idx[gm.off + (int32_t)sorted[gm.off + i]];
        p = ph[pidx];
        sf = static_sf(p, tp, tunsched, specs, terms, reqs);
    }
    // the previous stream entry: lane - 1, or recomputed by lane 0
    int64_t qc = __shfl_up(p.cpu, 1, 64), qm = __shfl_up(p.mem, 1, 64), qe = __shfl_up(p.eph, 1, 64);
    uint32_t qf = __shfl_up(sf, 1, 64);
    if (lane == 0 && valid && i > 0) {
        const PodHot q = ph[pod_idx[gm.off + (int32_t)sorted[gm.off + i - 1]]];
        qc = q.cpu; qm = q.mem; qe = q.eph;
        qf = static_sf(q, tp, tunsched, specs, terms, reqs);
    }
    bool head = true;
    if (valid) {
        const bool bat = batchable(p, sf);
        if (i > 0 && bat) head = !(qf == sf && qc == p.cpu && qm == p.mem && qe == p.eph);
        StreamPod sp;
        sp.cpu = p.cpu; sp.mem = p.mem; sp.eph = p.eph;
        sp.pod = pidx;
        sp.flags = sf | (head ? SF_HEAD : 0u) | (bat ? SF_BATCH : 0u);
        out[gm.off + i] = sp;
        spod[gm.off + i] = pidx;
        if (sf & SF_UNSUP) atomicOr(&group_unsup[gi], 1u);
    }
    const uint64_t hb = __ballot(head);
    if (lane == 0) heads[gm.moff + (i >> 6)] = hb;
}

// 4. the First-Fit-Decreasing chain -------------------------------------------
#ifdef CASIM_PROF   // section cycle counters of k_ffd_chain (profiling build only)
constexpr int NPROF = 15;   // + [12] loop top (window moves, head reads), [13] epilogue, [14] before the loop
__device__ unsigned long long g_chain_prof[1024][NPROF];
#define PROF_T(v) const uint64_t v = clock64()
#define PROF_ADD(i, t) prof[i] += clock64() - (t)
#define PROF_INC(i) prof[i]++
#else
#define PROF_T(v) (void)0
#define PROF_ADD(i, t) (void)0
#define PROF_INC(i) (void)0
#endif
__device__ inline int64_t rl64(int64_t v, int lane) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline int32_t rl32(int32_t v, int lane) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, lane); }

// wavefront reductions (device-library DPP reductions; all 64 lanes active at every call site)
extern "C" __device__ long long __ockl_wfred_add_i64(long long);
extern "C" __device__ long long __ockl_wfred_max_i64(long long);
__device__ inline int64_t wave_max64(int64_t v) { return __ockl_wfred_max_i64(v); }
__device__ inline int32_t wave_max32(int32_t v) { return __ockl_wfred_max_i32(v); }
__device__ inline int32_t wave_min32(int32_t v) { return __ockl_wfred_min_i32(v); }
__device__ inline int64_t wave_sum64(int64_t v) { return __ockl_wfred_add_i64(v); }
__device__ inline int32_t mbcnt(uint64_t m) {
    return (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The chain workgroup: CW wavefronts, one per SIMD of the CU.  Every wave runs the same
// sequential control flow on the same (uniform) state; the per-row loops over the
// group's new nodes are split across the waves (row j -> thread j mod CT), so the
// row work of a run — copy counts, revolution lists, row updates, opened rows — runs
// on all four SIMDs.  Cross-wave reductions go through LDS, double-buffered by a parity
// bit so that one barrier per reduction suffices (a wave cannot reach the next use of
// a buffer before every wave has read it: that needs the barrier in between).
// Barrier that orders LDS only.  __syncthreads() is also a workgroup fence for global
// memory, i.e. an s_waitcnt vmcnt(0) before s_barrier: every barrier would wait for the
// chain's result stores and the stream prefetch.  The waves of a chain workgroup share
// state through LDS only (their global stores are write-only results, released once at
// the end with __threadfence), so an LDS-scoped fence is all the barriers need.
__device__ inline void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// The chain's barrier: LDS-only while the rows are in LDS; a workgroup fence over every
// address space when the rows live in an HBM slab (GM), so row stores of one wave are
// visible to the others (all waves of the workgroup share the CU's L1).
template <bool GM> __device__ inline void cbar() {
    if (GM) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        lds_barrier();
    }
}
#ifndef CASIM_CW
#define CASIM_CW 4
#endif
constexpr int CW = CASIM_CW;
constexpr int CT = 64 * CW;
constexpr int RED_N = 5;
struct ChainRed {
    int64_t v[2][CW][RED_N];
    int32_t cnt[2][CW];
    int32_t pick;          // a value one wave found, for every wave (barrier-ordered)
};
enum { R_SUM = 0, R_MAX = 1, R_MIN = 2 };
extern "C" __device__ long long __ockl_wfred_min_i64(long long);
template <int OP> __device__ inline int64_t wred(int64_t v) {
    return OP == R_SUM ? __ockl_wfred_add_i64(v) : OP == R_MAX ? __ockl_wfred_max_i64(v) : __ockl_wfred_min_i64(v);
}
template <int OP> __device__ inline int64_t wcomb(int64_t a, int64_t b) {
    return OP == R_SUM ? a + b : OP == R_MAX ? (a > b ? a : b) : (a < b ? a : b);
}
template <int OA, int OB, int OC, bool GM = false>
__device__ inline void blk_red3(ChainRed& cr, int& par, int wv, int lane, int64_t& a, int64_t& b, int64_t& c) {
    a = wred<OA>(a); b = wred<OB>(b); c = wred<OC>(c);
    if (lane == 0) { cr.v[par][wv][0] = a; cr.v[par][wv][1] = b; cr.v[par][wv][2] = c; }
    cbar<GM>();
    a = cr.v[par][0][0]; b = cr.v[par][0][1]; c = cr.v[par][0][2];
    for (int w = 1; w < CW; w++) {
        a = wcomb<OA>(a, cr.v[par][w][0]); b = wcomb<OB>(b, cr.v[par][w][1]); c = wcomb<OC>(c, cr.v[par][w][2]);
    }
    par ^= 1;
}
// Five reductions with one barrier; the waves' partial values stay readable in
// cr.v[par ^ 1] (the buffer just used) until the reduction after next.
__device__ inline int64_t wred_rt(int op, int64_t v) {
    return op == R_SUM ? wred<R_SUM>(v) : op == R_MAX ? wred<R_MAX>(v) : wred<R_MIN>(v);
}
__device__ inline int64_t wcomb_rt(int op, int64_t a, int64_t b) {
    return op == R_SUM ? a + b : op == R_MAX ? (a > b ? a : b) : (a < b ? a : b);
}
template <bool GM = false>
__device__ inline void blk_red5(ChainRed& cr, int& par, int wv, int lane, int64_t (&x)[RED_N], const int (&op)[RED_N]) {
    for (int i = 0; i < RED_N; i++) x[i] = wred_rt(op[i], x[i]);
    if (lane == 0)
        for (int i = 0; i < RED_N; i++) cr.v[par][wv][i] = x[i];
    cbar<GM>();
    for (int i = 0; i < RED_N; i++) {
        int64_t a = cr.v[par][0][i];
        for (int w = 1; w < CW; w++) a = wcomb_rt(op[i], a, cr.v[par][w][i]);
        x[i] = a;
    }
    par ^= 1;
}
// Cross-wave step only: x[] already reduced within each wave (wave-uniform).
template <bool GM = false>
__device__ inline void blk_xchg5(ChainRed& cr, int& par, int wv, int lane, int64_t (&x)[RED_N], const int (&op)[RED_N]) {
    if (lane == 0)
        for (int i = 0; i < RED_N; i++) cr.v[par][wv][i] = x[i];
    cbar<GM>();
    for (int i = 0; i < RED_N; i++) {
        int64_t a = cr.v[par][0][i];
        for (int w = 1; w < CW; w++) a = wcomb_rt(op[i], a, cr.v[par][w][i]);
        x[i] = a;
    }
    par ^= 1;
}
__device__ inline int32_t hibit(uint64_t m) { return 63 - __builtin_clzll(m); }
// lanes below `n` (n in [0, 64])
__device__ inline uint64_t lanes_below(int32_t n) { return n >= 64 ? ~0ull : n <= 0 ? 0ull : ((1ull << n) - 1); }

// Rows of the group split in contiguous 64-row-aligned ranges, one per wave, so that
// per-wave counts in wave order are counts in row order.
__device__ inline void wave_rows(int32_t k, int wv, int32_t& lo, int32_t& hi) {
    const int32_t cpw = (((k + 63) >> 6) + CW - 1) / CW;      // 64-row chunks per wave
    lo = min(k, wv * cpw * 64);
    hi = min(k, lo + cpw * 64);
}
// Evals of opening n_open template copies for the rest of a run (closed form of the
// per-node sum: node i's opening pod fails FitsAnyNode over the k0+i rows before it
// (i > 0), passes CheckPredicates, and its next pi-2 pods scan k0+i+1 rows each, the
// first of them from j00 on node 0).
__device__ inline uint64_t open_evals(int32_t n_open, int32_t ct, int32_t placed2, int32_t k0, int32_t j00,
                                      uint64_t kev, bool cp_eval) {
    const uint64_t no = (uint64_t)n_open;
    uint64_t ev = kev * ((no - 1) * (uint64_t)k0 + (no - 1) * no / 2);
    if (cp_eval) ev += no;
    const uint64_t m = no - 1;                   // full nodes, ct pods each
    if (m > 0 && ct >= 2) ev += (uint64_t)(ct - 1) * (m * (uint64_t)(k0 + 1) + m * (m - 1) / 2) - (uint64_t)j00;
    const int32_t i = n_open - 1;                // the last node
    const int32_t pi = placed2 - i * ct;
    if (pi >= 2) {
        const int32_t j0i = i == 0 ? j00 : 0;
        ev += (uint64_t)(k0 + i - j0i + 1) + (uint64_t)(pi - 2) * (uint64_t)(k0 + i + 1);
    }
    return ev;
}

// Ordered compaction step over the workgroup: thread t contributes `keep` for index
// base + t; returns the thread's slot (exclusive prefix over the workgroup) and the total.
template <bool GM = false>
__device__ inline int32_t blk_compact(ChainRed& cr, int& par, int wv, bool keep, int32_t& total) {
    const uint64_t bm = __ballot(keep);
    if ((threadIdx.x & 63) == 0) cr.cnt[par][wv] = __builtin_popcountll(bm);
    cbar<GM>();
    int32_t before = 0;
    total = 0;
    for (int w = 0; w < CW; w++) {
        const int32_t c = cr.cnt[par][w];
        before += w < wv ? c : 0;
        total += c;
    }
    par ^= 1;
    return before + mbcnt(bm);
}

// New-node row in LDS: free resources of one template copy (32 B, two ds_read_b128).
struct alignas(16) NodeRec {
    int64_t cpu, mem, eph;
    int32_t pods;      // free pod slots
    int32_t used;      // newNodesWithPods membership
};
static_assert(sizeof(NodeRec) == 32, "NodeRec");

// NodeResourcesFit on a row (fit.go:256-300), branch-free so all loads issue together.
__device__ inline bool rec_fits(const NodeRec& r, int64_t pcpu, int64_t pmem, int64_t peph, bool zero) {
    const bool res = (pcpu <= r.cpu) & (pmem <= r.mem) & (peph <= r.eph);
    return (r.pods >= 1) & (zero | res);
}

// How many copies of a resource-only pod (requests >= 0) fit a row one after another:
// copy m+1 fits iff pods >= m+1 and (all-zero or every req <= free - m*req), so the
// count is min(pods, floor(free/req)) over the requested dimensions (fit.go:256-300;
// a zero request passes iff free >= 0).  Capped at `cap`.
__device__ inline int32_t dim_copies(int64_t free_, int64_t req, int32_t cap) {
    if (free_ < 0) return 0;
    if (req == 0) return cap;
    if (free_ < req) return 0;
    // floor(free/req) capped at cap, without a 64-bit integer division: the float64
    // quotient is within one of the exact one once capped, and one step each way fixes it.
    const double qd = (double)free_ / (double)req;
    uint64_t q = qd >= (double)cap ? (uint64_t)cap : (uint64_t)qd;
    const uint64_t f = (uint64_t)free_, r = (uint64_t)req;     // both < 2^63: no wrap below
    if (q * r > f) q--;
    else if (q < (uint64_t)cap && (q + 1) * r <= f) q++;
    return (int32_t)q;
}
__device__ inline int32_t rec_copies(const NodeRec& r, int64_t pcpu, int64_t pmem, int64_t peph, bool zero, int32_t cap) {
    int32_t c = r.pods < cap ? r.pods : cap;
    if (c <= 0) return 0;
    if (!zero) {
        c = min(c, dim_copies(r.cpu, pcpu, c));
        c = min(c, dim_copies(r.mem, pmem, c));
        c = min(c, dim_copies(r.eph, peph, c));
    }
    return c;
}

// rec_copies for the rows of one run: the pod's requests and reciprocals in float64,
// computed once per run.  Exact while every free value and request is below 2^53 (a
// template copy's free values bound every row of its group; checked once per run);
// otherwise the exact integer rec_copies.
struct RunDiv {
    double reqd[3], rcpd[3];
    bool f64;
};
__device__ inline RunDiv run_div(int64_t pcpu, int64_t pmem, int64_t peph, int64_t bound) {
    RunDiv d;
    constexpr int64_t E53 = 1ll << 53;
    d.f64 = bound < E53 && pcpu < E53 && pmem < E53 && peph < E53;
    const int64_t req[3] = {pcpu, pmem, peph};
    for (int i = 0; i < 3; i++) {
        d.reqd[i] = (double)req[i];
        // req == 0: rcp = +inf, the quotient inf (NaN for free == 0) and fmin(., cap)
        // gives cap — a zero request passes whenever free >= 0
        d.rcpd[i] = req[i] > 0 ? 1.0 / d.reqd[i] : __builtin_inf();
    }
    return d;
}
// floor(free/req) capped at cap with full-rate float64 ops only: below 2^53 the
// conversions are exact, the quotient is within one of the exact floor, and
// fma(-q, req, free) = free - q*req is an integer below 2^53 in magnitude, so it is
// computed exactly and one step each way makes q exact (no 64-bit integer multiply).
__device__ inline int32_t dim_copies_f64(int64_t free_, double rd, double rcpd, int32_t cap) {
    const double fd = (double)(free_ < 0 ? 0 : free_);
    const double cp = (double)cap;
    double q = fmin(floor(fd * rcpd), cp);              // NaN (0 * inf) -> cap
    const double t = fma(-q, rd, fd);
    q += ((t >= rd) & (q < cp)) ? 1.0 : 0.0;
    q -= (t < 0.0) ? 1.0 : 0.0;
    return free_ < 0 ? 0 : (int32_t)q;
}
__device__ inline int32_t rec_copies_run(const NodeRec& r, const RunDiv& d, bool zero, int32_t cap,
                                         int64_t pcpu, int64_t pmem, int64_t peph) {
    if (!d.f64) return rec_copies(r, pcpu, pmem, peph, zero, cap);     // uniform
    int32_t c = max(0, min(r.pods, cap));
    if (!zero) {     // uniform
        // independent per-dimension quotients (capped at the same c, min taken after);
        // a zero request only needs free >= 0 (uniform skip of the division)
        const int32_t cp = max(c, 1);
        const int32_t q0 = d.reqd[0] != 0.0 ? dim_copies_f64(r.cpu, d.reqd[0], d.rcpd[0], cp) : (r.cpu < 0 ? 0 : cp);
        const int32_t q1 = d.reqd[1] != 0.0 ? dim_copies_f64(r.mem, d.reqd[1], d.rcpd[1], cp) : (r.mem < 0 ? 0 : cp);
        const int32_t q2 = d.reqd[2] != 0.0 ? dim_copies_f64(r.eph, d.reqd[2], d.rcpd[2], cp) : (r.eph < 0 ? 0 : cp);
        c = min(c, min(q0, min(q1, q2)));
    }
    return c;
}

// first run head strictly after `pos` (positions >= P count as heads)
__device__ inline int32_t run_end(const uint64_t* __restrict__ hm, int32_t pos, int32_t P, int lane) {
    int32_t c = pos >> 6;
    const int32_t nc = (P + 63) >> 6;
    const int sh = (pos & 63) + 1;
    uint64_t m = hm[c];
    m = sh >= 64 ? 0ull : (m >> sh) << sh;
    if (m) return min(P, (c << 6) + __builtin_ctzll(m));
    for (c = c + 1; c < nc; c += 64) {
        const int32_t cc = c + lane;
        const uint64_t v = cc < nc ? hm[cc] : 0ull;
        const uint64_t b = __ballot(v != 0);
        if (b) {
            const int l = __builtin_ctzll(b);
            return min(P, ((c + l) << 6) + __builtin_ctzll((uint64_t)rl64((int64_t)v, l)));
        }
    }
    return P;
}
// run_end with the head words [pf_c, pf_c + 64) already in registers (lane l holds word
// pf_c + l, 0 past the end; loaded when the previous run started), so finding a run's
// end costs no global round trip unless the run is longer than the 4096 positions held.
__device__ inline int32_t run_end_pf(const uint64_t* __restrict__ hm, int32_t pos, int32_t P, int lane,
                                     int32_t pf_c, uint64_t pf_w) {
    const int32_t c = pos >> 6;
    if (c != pf_c) return run_end(hm, pos, P, lane);
    const int sh = (pos & 63) + 1;
    uint64_t m = (uint64_t)rl64((int64_t)pf_w, 0);
    m = sh >= 64 ? 0ull : (m >> sh) << sh;
    if (m) return min(P, (c << 6) + __builtin_ctzll(m));
    const uint64_t b = __ballot((lane > 0) & (pf_w != 0ull));
    if (b) {
        const int l = __builtin_ctzll(b);
        return min(P, ((c + l) << 6) + __builtin_ctzll((uint64_t)rl64((int64_t)pf_w, l)));
    }
    const int32_t nc = (P + 63) >> 6;
    for (int32_t c2 = c + 64; c2 < nc; c2 += 64) {
        const int32_t cc = c2 + lane;
        const uint64_t v = cc < nc ? hm[cc] : 0ull;
        const uint64_t b2 = __ballot(v != 0);
        if (b2) {
            const int l = __builtin_ctzll(b2);
            return min(P, ((c2 + l) << 6) + __builtin_ctzll((uint64_t)rl64((int64_t)v, l)));
        }
    }
    return P;
}

// Zero-copy results (page-locked sched_pod, no node ordinals): a group hands its output
// range to k_publish in pch-sized chunks ("tickets") as soon as each chunk is final —
// every output of [c*pch, (c+1)*pch) is scheduled — and the rest when it ends, so the
// results cross PCIe while the chains still run, the long ones included.  Each ticket
// carries the group's progress (segments written, pods scheduled) at its push.
// Release at agent scope: the L2s of the 8 XCDs are not coherent, the publisher may run
// on another XCD.  Called by one whole wavefront (the one that stores the results).
//
// A ticket is 64-bit: the chunk (g * nsub + c) in the low word and, for a **pure** chunk —
// every output of it comes from run segments with one stream offset `off` (output i is
// stream position i + off) — off + 1 in the high word.  The publisher copies a pure chunk
// from the stream's pod ids (written before the chains started) and reads nothing the
// chain wrote, so its push needs no release: an agent-scope release writes the XCD's L2
// back (gfx950: its L2 is not coherent with the other XCDs'), microseconds per push on the
// chain's critical path.  Other chunks (single placements, a segment boundary with another
// offset, the group's tail) go with the release and the progress record.
constexpr int PCH = 4096;      // default chunk (CASIM_PUB_CHUNK overrides, for tests)
#ifndef CASIM_PCH_DECOUPLED
#define CASIM_PCH_DECOUPLED 16384
#endif
constexpr int PCH_DECOUPLED = CASIM_PCH_DECOUPLED;   // ... with the decoupled Go order (scripts/gpu_pubsweep2.sh)
__device__ inline void push_chunks(int32_t g, int32_t c0, int32_t c1, int32_t nsub, int64_t* tickets, int32_t* qctl,
                                   int2* prog, int32_t nseg, int32_t nsched, int lane, int32_t pch = 0,
                                   int32_t pure_from = INT32_MAX, int32_t pure_off = 0) {
    if (c1 <= c0) return;
    const bool pure = pch > 0 && (int64_t)c0 * pch >= pure_from;
    if (!pure) __threadfence();
    if (lane == 0) {
        if (!pure)
            for (int32_t c = c0; c < c1; c++) prog[g * nsub + c] = make_int2(nseg, nsched);
        const int32_t base = atomicAdd(&qctl[1], c1 - c0);
        const int64_t hi = pure ? ((int64_t)pure_off + 1) << 32 : 0;
        for (int32_t i = 0; i < c1 - c0; i++) {
            const int64_t v = hi | (int64_t)(uint32_t)(g * nsub + c0 + i);
            if (pure) __hip_atomic_store(&tickets[base + i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(&tickets[base + i], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Data the chains write while the publisher runs (progress records, segments) is read
// with device-coherent loads: a uniform plain load may be served from the scalar cache,
// which the acquire does not invalidate, so a line cached for an earlier chunk (or a
// neighbouring group) could hand back entries written after it was filled.
__device__ inline int32_t ld_coh(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline Seg ld_seg(const Seg* p) {
    const int32_t* q = reinterpret_cast<const int32_t*>(p);
    Seg sg;
    sg.dst = ld_coh(q); sg.src = ld_coh(q + 1); sg.len = ld_coh(q + 2); sg.pad = 0;
    return sg;
}

// Publisher (second stream, concurrent with k_ffd_chain): block b claims the next ticket
// in completion order, waits for it, and writes outputs [sub*pch, +pch) of its group
// into the caller's page-locked buffer: single placements from the chain's sched_pod,
// run placements from the stream via the group's segments, -1 past n_scheduled.
// Every block exits once all `total` tickets are claimed.  HIP does not promise that the
// two kernels overlap, so the publisher never waits on a chain that has not started:
// the chains raise qctl[4] when they begin, and a publisher that sees no chain within
// `start_ticks` (100 MHz wall clock; the kernels were serialised) sets qctl[2] and ends,
// as does one whose ticket is not pushed within 200 ms of a started chain (a chain that
// died).  qctl[2] sends the host to the stream-ordered copy (k_copy_segments + D2H).
// T = int32_t: pod ids; T = uint16_t: pod ids of a podset of at most 65535 pods, 0xFFFF for
// "not scheduled" (ca_estimate_plan_run_u16: half the bytes over PCIe).
template <typename T>
__global__ void __launch_bounds__(256) k_publish(const GroupMeta* __restrict__ groups, const ChainOut* __restrict__ outs,
                                                const Seg* __restrict__ segs, const int32_t* __restrict__ spod,
                                                const int32_t* sched_dev, int64_t* __restrict__ tickets,
                                                int32_t* __restrict__ qctl, int32_t total, int32_t nsub,
                                                const int2* __restrict__ prog, int32_t pch,
                                                T* pub,              // pub may alias sched_dev (device results)
                                                uint64_t start_ticks, const int32_t* ids_ready, int32_t ids_epoch,
                                                int32_t* __restrict__ hflags) {
    // ids_ready != null (decoupled Go order): the stream's pod ids in spod
    // come from a sort that runs beside the chains — a group's are final once
    // ids_ready[g] holds this run's epoch — and the chains' single placements are stream positions
    __shared__ int32_t s_t, s_seg0;
    __shared__ int64_t s_tk;
    __shared__ Seg s_segs[64];
    for (;;) {
        if (threadIdx.x == 0) {
            s_t = atomicAdd(&qctl[0], 1);
            int64_t tk = -1;
            if (s_t < total) {
                const uint64_t t0 = wall_clock64();
                bool started = false;
                for (;;) {
                    // relaxed polls (an acquire per poll invalidates caches other kernels on
                    // the XCD are using); the acquire comes once, when the ticket is there
                    tk = __hip_atomic_load(&tickets[s_t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk >= 0) {      // consumed: the slot is -1 again for the next run
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        __hip_atomic_store(&tickets[s_t], -1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    if (__hip_atomic_load(&qctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;  // given up
                    if (!started) started = __hip_atomic_load(&qctl[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    const uint64_t dt = wall_clock64() - t0;
                    if ((!started && dt > start_ticks) || dt > 20000000ull) {               // 200 ms
                        __hip_atomic_store(&qctl[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (tk >= 0 && ids_ready) {                  // the group's Go-order ids
                    const int32_t g = (int32_t)(uint32_t)(tk & 0xFFFFFFFFll) / nsub;
                    for (;;) {
                        if (__hip_atomic_load(&ids_ready[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ids_epoch) {
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                            break;
                        }
                        if (__hip_atomic_load(&qctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { tk = -1; break; }
                        if (wall_clock64() - t0 > 20000000ull) {                            // 200 ms
                            __hip_atomic_store(&qctl[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            tk = -1;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
            }
            s_tk = tk;
        }
        lds_barrier();
        const int32_t t = s_t;
        const int64_t tk64 = s_tk;
        if (t >= total || tk64 < 0) {
            if (threadIdx.x == 0) {
                // gave up (qctl[2]): tell the host, which reads hflags after the round (no copy)
                if (t < total) hflags[2] = 1;
                // the last block out clears the control words for the next run (every ticket
                // was consumed, so no chain pushes any more; after a give-up the host
                // re-initialises them)
                if (atomicAdd(&qctl[5], 1) == (int32_t)gridDim.x - 1)
                    for (int k = 0; k < 6; k++) __hip_atomic_store(&qctl[k], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
        __threadfence();                                   // acquire for every thread of the block
        const int32_t tk = (int32_t)(uint32_t)(tk64 & 0xFFFFFFFFll);
        const int32_t pure_off = (int32_t)(tk64 >> 32) - 1;   // >= 0: a pure chunk (push_chunks)
        const int32_t g = tk / nsub, sub = tk - g * nsub;
        const GroupMeta gm = groups[g];
        const Seg* gs = segs + gm.off;
        const int32_t a = sub * pch, b = min(gm.count, a + pch);
        if (pure_off >= 0) {
            // one contiguous copy: 16-byte stores into the page-locked buffer (fewer, fuller
            // PCIe writes), scalar stores for the unaligned head and tail
            constexpr int V = 16 / (int)sizeof(T);
            T* const dst = pub + gm.off;
            const int32_t* const src = spod + gm.off + pure_off;
            int32_t h = a;
            while (h < b && ((uintptr_t)(dst + h) & 15u)) h++;                 // aligned from h on
            const int32_t nv = (b - h) / V;
            for (int32_t i = a + (int32_t)threadIdx.x; i < h; i += blockDim.x) dst[i] = (T)src[i];
            for (int32_t v = (int32_t)threadIdx.x; v < nv; v += blockDim.x) {
                const int32_t i0 = h + v * V;
                T w[V];
#pragma unroll
                for (int u = 0; u < V; u++) w[u] = (T)src[i0 + u];
                uint4 q;
                __builtin_memcpy(&q, w, 16);
                *reinterpret_cast<uint4*>(dst + i0) = q;
            }
            for (int32_t i = h + nv * V + (int32_t)threadIdx.x; i < b; i += blockDim.x) dst[i] = (T)src[i];
            lds_barrier();
            continue;
        }
        const int32_t* pr = reinterpret_cast<const int32_t*>(prog + tk);   // the group's progress at the push
        const int32_t nseg = ld_coh(pr);
        const int32_t ns = ld_coh(pr + 1);
        if (threadIdx.x < 64) {
            // first segment ending after a (segments are in output order): wave 0 probes 64
            // evenly spaced segments per step with coherent loads in flight together, so a
            // search is one or two round trips to L2 instead of one per bisection step
            const int lane = (int)threadIdx.x;
            int32_t lo = 0, hi = nseg;                     // answer in [lo, hi]
            while (hi - lo > 0) {
                const int32_t span = hi - lo;
                const int32_t step = (span + 63) / 64;
                const int32_t i = lo + lane * step;
                bool past = false;                         // segment i ends after a
                if (i < hi) {
                    const int32_t* q3 = reinterpret_cast<const int32_t*>(gs + i);
                    past = ld_coh(q3) + ld_coh(q3 + 2) > a;
                }
                const uint64_t m = __ballot(past);
                const int32_t f = m ? (int32_t)__builtin_ctzll(m) : -1;    // first probe past a
                if (step == 1) { lo = f >= 0 ? lo + f : hi; break; }
                const int32_t nlo = f > 0 ? lo + (f - 1) * step + 1 : (f == 0 ? lo : lo + ((span - 1) / step) * step + 1);
                hi = f >= 0 ? lo + f * step : hi;
                lo = nlo;
            }
            if (lane == 0) s_seg0 = lo;
        }
        lds_barrier();
        int32_t at = a, q = s_seg0;
        const int32_t end = min(b, ns);
        int32_t q0 = 0, qn = 0;                           // segments [q0, q0 + qn) cached in LDS
        while (at < end) {
            int32_t lim = end, src_off = 0;
            bool from_seg = false;
            if (q < nseg && (q < q0 || q >= q0 + qn)) {
                // the next 64 segments, loaded together (one round trip instead of one per segment)
                lds_barrier();                             // every thread is done with the old ones
                if (threadIdx.x < 64 && q + (int32_t)threadIdx.x < nseg) s_segs[threadIdx.x] = ld_seg(gs + q + threadIdx.x);
                q0 = q;
                qn = min(64, nseg - q);
                lds_barrier();
            }
            if (q < nseg) {
                const Seg sg = s_segs[q - q0];
                if (sg.dst <= at) {                            // inside segment q
                    from_seg = true;
                    src_off = sg.src - sg.dst;
                    lim = min(end, sg.dst + sg.len);
                    q++;
                } else {
                    lim = min(end, sg.dst);                    // single placements before it
                }
            }
            for (int32_t i = at + (int32_t)threadIdx.x; i < lim; i += blockDim.x)
                pub[gm.off + i] = (T)(from_seg ? spod[gm.off + src_off + i]
                                               : ids_ready ? spod[gm.off + ld_coh(sched_dev + gm.off + i)]
                                                           : sched_dev[gm.off + i]);
            at = lim;
        }
        for (int32_t i = max(a, ns) + (int32_t)threadIdx.x; i < b; i += blockDim.x) pub[gm.off + i] = (T)-1;
        lds_barrier();
    }
}

// One workgroup of CW (4) waves per node group (see ChainRed above: the waves share the
// row loops, the control flow is uniform).  LDS: NodeRec rows[kcap], block summaries[kcap/64]
// (per-dimension maxima over a 64-row block, allowed to be stale-high), the per-run
// scratch CAPA/ALIVE[kcap], and the optional port / scalar columns.
//
// The sequential loop of binpacking_estimator.go:86-141 runs pod by pod, except that a
// run of identical resource-only pods (SF_BATCH) is placed in closed form: the rotating
// first fit of schedulerbased.go:114-131 with identical pods visits the nodes that still
// have room in rotated order, one pod per node per revolution, so revolution r serves
// the nodes with c_j >= r copies left, and the run costs O(k/64) wave steps plus one
// step per node it opens instead of one k-node scan per pod.  Evals are exact: the t-th
// placement's scan ends at unwrapped position (rev-1)*k + rank, so a batch costs
// (r_last-1)*k + rank(last)+1 filter calls.  assign[pos] receives the new-node index of
// every placed stream position (-1 = not scheduled).
// PS: the batch has pods with host ports or extended-resource requests (their columns and
// checks compile out of the common instantiation)
template <bool GROWS, bool PS>
__global__ void __launch_bounds__(CT) k_ffd_chain(
    const GroupMeta* __restrict__ groups, const StreamPod* __restrict__ stream, const uint64_t* __restrict__ heads,
    const ca_template* __restrict__ tmpls, const ca_pod_spec* __restrict__ specs, const PodHot* __restrict__ ph,
    const int32_t* __restrict__ lin_arr, const uint8_t* __restrict__ need, const uint32_t* __restrict__ group_unsup,
    int32_t n_base, int32_t max_nodes, int32_t kcap, int32_t use_ports, int32_t use_scalar, int32_t batch_runs,
    int32_t* __restrict__ sched_pod, int32_t* __restrict__ sched_node, Seg* __restrict__ segs,
    int64_t* __restrict__ tickets, int32_t* __restrict__ qctl, int32_t nsub, int2* __restrict__ prog, int32_t pch,
    ChainOut* __restrict__ outs, const int32_t* __restrict__ gmap, unsigned char* __restrict__ gslab,
    const int64_t* __restrict__ slab_off, const int32_t* __restrict__ gkcap, int32_t pos_out,
    ChainOut* __restrict__ hout, int32_t* __restrict__ hflags) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int g = GSEL(blockIdx.x);
    // GROWS: the group's rows live in its own HBM slab (kcap = the group's pod count, for an
    // unlimited estimate too large for LDS); else in LDS with the batch-wide kcap
    if (GROWS) kcap = gkcap[g];
    unsigned char* const row_base = GROWS ? gslab + slab_off[g] : smem_raw;
    if (!need[g]) return;
    if (tickets && threadIdx.x == 0)              // a publisher may wait on this batch now
        __hip_atomic_store(&qctl[4], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t_begin = wall_clock64();      // diagnostics: ca_estimate_plan_group_ticks
    __builtin_amdgcn_s_setprio(3);                // the chain is the critical path: win issue over k_publish
#ifdef CASIM_PROF
    const uint64_t t_cyc0 = clock64();
#endif
    uint32_t n_single = 0;
#ifdef CASIM_PROF
    uint64_t prof[NPROF] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = tid >> 6;          // wave of the workgroup
    const bool w0 = wv == 0;          // the wave that stores single-pod results
    __shared__ ChainRed cred;
    int par = 0;
    const GroupMeta gm = groups[g];
    const int32_t lin = lin_arr[g];
    ChainOut res;
    res.node_count = 0; res.n_sched = 0; res.nodes_added = 0; res.lin = lin; res.lout = lin;
    res.status = CA_OK; res.sensitive = 0; res.had_success = 0; res.evals = 0; res.pad = 0;
    res.nseg = 0; res.pad2[0] = res.pad2[1] = res.pad2[2] = 0;
    if (group_unsup[g] || (gm.tflags & CA_NODE_ANTI_AFFINITY_PODS)) {
        res.status = CA_EUNSUPPORTED;
        if (tid == 0) { outs[g] = res; hout[g] = res; }
        if (tickets && w0) push_chunks(g, 0, (gm.count + pch - 1) / pch, nsub, tickets, qctl, prog, 0, 0, lane);
        return;
    }
    const int nb_cap = (kcap + 63) >> 6;
    NodeRec* R = reinterpret_cast<NodeRec*>(row_base);
    NodeRec* SUM = R + kcap;
    int32_t* CAPA = reinterpret_cast<int32_t*>(SUM + nb_cap);                   // [kcap]
    int32_t* ALIVE = CAPA + kcap;                                               // [kcap]
    uint64_t* PORTS = reinterpret_cast<uint64_t*>(ALIVE + kcap);                // [kcap][CA_PORT_WORDS]
    int64_t* SC = reinterpret_cast<int64_t*>(PORTS + (use_ports ? (size_t)CA_PORT_WORDS * kcap : 0));
    if (!PS) use_ports = use_scalar = 0;  // [8][kcap]

    const ca_template& tp = tmpls[gm.tmpl];
    NodeRec trec;                 // a fresh template copy
    trec.cpu = gm.tcpu; trec.mem = gm.tmem; trec.eph = gm.teph; trec.pods = gm.tpods; trec.used = 0;

    int32_t k = 0;              // new nodes so far
    int32_t granted = 0;        // limiter.nodes
    int32_t last_node = -1;     // lastNodeName
    int32_t L = lin;            // the checker's lastIndex
    int32_t nsched = 0;
    uint64_t evals = 0;
    bool first_success = false, sensitive = false;

    const int32_t P = gm.count;
    const StreamPod* gs = stream + gm.off;
    const uint64_t* hm = heads + gm.moff;
    // outputs in processing order (binpacking_estimator.go:143): the i-th scheduled pod of
    // the group and its new-node ordinal go to index i; placements happen in stream order
    Seg* gseg = segs + gm.off;
    int32_t nseg = 0;
    int32_t* so_pod = sched_pod + gm.off;
    int32_t* so_node = sched_node ? sched_node + gm.off : nullptr;
    // Stream double buffer: lane l holds entry (wbase + l) in `cur` and (wbase + 64 + l)
    // in `nxt`.  Single-pod placements are kept in the lane of their stream position and
    // stored when the window moves on, so no step waits on a store (vmcnt counts both).
    int32_t wbase = 0;
    StreamPod cur = {}, nxt = {};
    if (lane < P) cur = gs[lane];
    if (64 + lane < P) nxt = gs[64 + lane];
    int32_t out_node = -1, out_idx = 0;
    bool pend = false;
    bool stop = false;
    // Prefetch for the next run head, issued when a run starts: the stream window at the
    // run's end (pf_base, -1 none) and the head words from there (pf_hc, lane l holds word
    // pf_hc + l), so the global latency overlaps the run's LDS work instead of following it.
    int32_t pf_base = -1, pf_hc = -1;
    StreamPod pf_cur = {}, pf_nxt = {};
    uint64_t pf_hw = 0;
    const int32_t nhc = (P + 63) >> 6;

    // add a template copy as new node k (addNewNodeToSnapshot, :146-159)
    // (LDS writes by one thread; a barrier follows before any wave reads the row)
    auto open_node = [&]() -> int32_t {
        const int32_t nn = k;
        if (tid == 0) {
            R[nn] = trec;
            SUM[nn >> 6] = trec;   // a fresh copy is the largest a row can be
        }
        if (use_ports && tid < CA_PORT_WORDS) PORTS[(size_t)nn * CA_PORT_WORDS + tid] = tp.used_ports[tid];
        if (use_scalar && tid < CA_MAX_SCALAR)
            SC[(size_t)tid * kcap + nn] = wsub(tp.node.alloc_scalar[tid], tp.used_scalar[tid]);
        k++;
        last_node = nn;
        return nn;
    };
    auto note_success = [&]() {
        if (!first_success) { first_success = true; sensitive = k >= 2; }
    };
    // publish the chunks whose outputs are all scheduled (wave 0 stores every result in
    // publishing mode: segments by thread 0, single placements by its lanes)
    int32_t tk_next = 0;
    int32_t tk_bound = pch;         // (tk_next + 1) * pch: progress() divides only once it is reached
    // outputs [pure_from, nsched) all come from run segments with stream offset pure_off
    // (pure chunks: push_chunks); a single placement or a segment with another offset
    // restarts the range
    int32_t pure_from = 0, pure_off = 0;
    auto note_segment = [&](int32_t dst, int32_t src) {
        if (src - dst != pure_off || dst < pure_from) { pure_from = dst; pure_off = src - dst; }
    };
    auto progress = [&]() {
        if (!tickets || !w0 || nsched < tk_bound) return;
        const int32_t c1 = nsched / pch;
        tk_bound = (c1 + 1) * pch;
        if (pend) {                       // the pending single placement, stored now
            so_pod[out_idx] = pos_out ? wbase + lane : cur.pod;
            pend = false;
        }
        push_chunks(g, tk_next, c1, nsub, tickets, qctl, prog, nseg, nsched, lane, pch, pure_from, pure_off);
        tk_next = c1;
    };

    int32_t pos = 0;
#ifdef CASIM_PROF
    prof[14] = clock64() - t_cyc0;
#endif
    while (pos < P && !stop) {
        PROF_T(t_top);
        if (pos >= wbase + 64) {
            if (pend) {
                so_pod[out_idx] = pos_out ? wbase + lane : cur.pod;
                if (so_node) so_node[out_idx] = out_node;
            }
            pend = false;
            if (pos < wbase + 128) {
                cur = nxt;
                wbase += 64;
                nxt = StreamPod{};
                if (wbase + 64 + lane < P) nxt = gs[wbase + 64 + lane];
            } else if ((pos & ~63) == pf_base) {
                wbase = pf_base;            // prefetched when the run that ends here started
                cur = pf_cur;
                nxt = pf_nxt;
            } else {
                wbase = pos & ~63;
                cur = StreamPod{};
                if (wbase + lane < P) cur = gs[wbase + lane];
                nxt = StreamPod{};
                if (wbase + 64 + lane < P) nxt = gs[wbase + 64 + lane];
            }
            pf_base = -1;
        }
        const int sl = pos - wbase;
        const int64_t pcpu = rl64(cur.cpu, sl), pmem = rl64(cur.mem, sl), peph = rl64(cur.eph, sl);
        const int32_t pidx = rl32(cur.pod, sl);
        const uint32_t sf = (uint32_t)rl32((int32_t)cur.flags, sl);
        const bool zero = (sf & SF_ZERO) != 0;
#ifdef CASIM_PROF
        __builtin_amdgcn_s_waitcnt(0);       // (profiling: the head's loads land here, not in the run)
#endif
        PROF_ADD(12, t_top);

        // ---------------- a run of identical resource-only pods ----------------
        if (batch_runs && (sf & (SF_BATCH | SF_HEAD)) == (SF_BATCH | SF_HEAD)) {
            PROF_T(t_re);
            PROF_T(t_run);
            const int32_t e = run_end_pf(hm, pos, P, lane, pf_hc, pf_hw);
            if (e < P) {
                const int32_t pb = e & ~63;
                if (pb >= wbase + 128) {
                    pf_base = pb;
                    pf_cur = StreamPod{};
                    if (pb + lane < P) pf_cur = gs[pb + lane];
                    pf_nxt = StreamPod{};
                    if (pb + 64 + lane < P) pf_nxt = gs[pb + 64 + lane];
                }
                pf_hc = e >> 6;
                pf_hw = pf_hc + lane < nhc ? hm[pf_hc + lane] : 0ull;
            }
            PROF_ADD(0, t_re);
            if (e - pos >= 2) {
                PROF_INC(7);
                PROF_T(t_pro);
                const int32_t RN = e - pos;
                const uint64_t kev = (sf & SF_EVAL) ? 1u : 0u;
                // the pod's reciprocals, once per run (copy counts of every row, the last
                // row and the template: fast path while the cap is <= 2^20)
                const RunDiv dv = run_div(pcpu, pmem, peph, max(trec.cpu, max(trec.mem, trec.eph)));
                int32_t done = 0;
                bool exhausted = false;          // every row but last_node has no room left
                PROF_ADD(8, t_pro);
                while (done < RN) {
                    const int32_t rem = RN - done;
                    const int32_t len = n_base + k;
                    int32_t placed = 0;
                    // last_node's used bit after this iteration: its bit now (every row is
                    // visible here: a barrier ended the previous step) or a placement on it, so
                    // the empty-node check below needs no barrier after the row updates
                    bool last_used = last_node >= 0 && R[last_node].used;
                    if ((sf & SF_FA_OK) && k > 0) {
                        int32_t s0 = L;
                        if (s0 >= len) s0 = (int32_t)((uint32_t)s0 % (uint32_t)len);
                        const int32_t j0 = s0 > n_base ? s0 - n_base : 0;   // first new node visited
                        int32_t one = -1, n_one = 0, nalive = 0;
                        int64_t S = 0;
                        int64_t lv_cmin = 0;      // revolution 1: fewest copies among rows with room
                        int32_t lv_s = 0;         // ... and how many of them lie before j0
                        // blocks of this wave's row range whose copy counts were computed
                        // (bit i: rows [lo + 64 i, +64)); every other row has no room
                        uint64_t adm_w = 0;
                        if (exhausted) {
                            PROF_T(t_ex);
                            const NodeRec rl_ = R[last_node];
                            const int32_t c = rem <= (1 << 20) ? rec_copies_run(rl_, dv, zero, rem, pcpu, pmem, peph)
                                                               : rec_copies(rl_, pcpu, pmem, peph, zero, rem);
                            cbar<GROWS>();    // every wave has read the row before it changes
                            if (c > 0) { one = last_node; n_one = c; nalive = 1; }
                            PROF_ADD(10, t_ex);
                        } else {
                            PROF_T(t_ca);
                            // copies per row, and for revolution 1 (rows with room): count,
                            // last such row, fewest copies, count below j0 (rotation split)
                            int32_t lo, hi;
                            wave_rows(k, wv, lo, hi);
                            // counts, last row with room and the rotation split come from
                            // ballots (scalar); only the copy sum and minimum need reductions
                            int64_t s64 = 0;                          // copies (rem > 2^20 path)
                            int32_t s32 = 0, cm = INT32_MAX;          // copies (<= 2^24 per lane), fewest
                            int32_t na_w = 0, lt_w = 0, a1_w = -1;    // wave-uniform
                            auto acc = [&](int32_t b, int32_t c, bool in) -> int32_t {   // row b + lane
                                if (in) CAPA[b + lane] = c;
                                const bool room = in && c > 0;
                                cm = room ? min(cm, c) : cm;
                                const uint64_t m = __ballot(room);
                                na_w += __builtin_popcountll(m);
                                lt_w += __builtin_popcountll(m & lanes_below(j0 - b));
                                if (m) a1_w = b + hibit(m);
                                return in ? c : 0;
                            };
                            const bool fast = rem <= (1 << 20);
                            if (fast) {
                                // Block skip: a row has room for a copy iff the pod fits it
                                // (rec_fits: compares only), so the float64 copy counts run
                                // only for 64-row blocks where some row fits — in FFD most rows
                                // are full for most later pods (C2: ~5% of rows have room per
                                // pass).  The placement-list path (node ordinals) reads every
                                // row's count, so it computes them all.  Two blocks in flight.
                                const bool all = so_node != nullptr;
                                for (int32_t b = lo; b < hi; b += 128) {
                                    const int32_t j = b + lane;
                                    const bool in0 = j < hi, in1 = j + 64 < hi;
                                    const NodeRec r0 = R[in0 ? j : 0], r1 = R[in1 ? j + 64 : 0];
                                    const uint64_t f0 = __ballot(in0 && (all || rec_fits(r0, pcpu, pmem, peph, zero)));
                                    const uint64_t f1 = __ballot(in1 && (all || rec_fits(r1, pcpu, pmem, peph, zero)));
                                    if (f0) {
                                        adm_w |= 1ull << ((b - lo) >> 6);
                                        s32 += acc(b, rec_copies_run(r0, dv, zero, rem, pcpu, pmem, peph), in0);
                                    } else if (in0) {
                                        CAPA[j] = 0;      // (read by the other waves' pick)
                                    }
                                    if (f1) {
                                        adm_w |= 1ull << ((b + 64 - lo) >> 6);
                                        s32 += acc(b + 64, rec_copies_run(r1, dv, zero, rem, pcpu, pmem, peph), in1);
                                    } else if (in1) {
                                        CAPA[j + 64] = 0;
                                    }
                                }
                            } else {
                                adm_w = ~0ull;
                                for (int32_t b = lo; b < hi; b += 64) {
                                    const int32_t j = b + lane;
                                    const bool in = j < hi;
                                    s64 += acc(b, rec_copies(R[in ? j : 0], pcpu, pmem, peph, zero, rem), in);
                                }
                            }
                            int64_t x[RED_N];          // S, rows with room, last such row, fewest copies, rows < j0
                            x[0] = fast ? (int64_t)__ockl_wfred_add_i32(s32) : wave_sum64(s64);
                            x[1] = na_w; x[2] = a1_w; x[3] = wave_min32(cm); x[4] = lt_w;
                            constexpr int OPS[RED_N] = {R_SUM, R_SUM, R_MAX, R_MIN, R_SUM};
                            blk_xchg5<GROWS>(cred, par, wv, lane, x, OPS);     // + CAPA visible
                            S = x[0];
                            nalive = (int32_t)x[1];
                            lv_cmin = x[3];
                            lv_s = (int32_t)x[4];
                            if (nalive == 1) { one = (int32_t)x[2]; n_one = (int32_t)min(S, (int64_t)rem); }
                            PROF_ADD(1, t_ca);
                        }
                        if (nalive == 1) {
                            // every remaining copy goes to the one row with room
                            int32_t rho = one - j0;
                            if (rho < 0) rho += k;
                            evals += (uint64_t)rho + 1 + (uint64_t)(n_one - 1) * (uint64_t)k;
                            if (tid == 0) {
                                NodeRec r = R[one];
                                r.cpu -= (int64_t)n_one * pcpu;
                                r.mem -= (int64_t)n_one * pmem;
                                r.eph -= (int64_t)n_one * peph;
                                r.pods -= n_one;
                                r.used = 1;
                                R[one] = r;
                            }
                            if (so_node) for (int32_t t = tid; t < n_one; t += CT) so_node[nsched + t] = one;
                            L = n_base + one + 1;
                            if (L >= len) L -= len;
                            note_success();
                            placed = n_one;
                            last_used |= one == last_node;
                        } else if (nalive > 1) {
                            const int32_t n = (int32_t)min(S, (int64_t)rem);
                            PROF_T(t_rv);
                            int32_t got = 0, r = 1, last = -1;
                            int32_t* gdst = so_node ? so_node + nsched : nullptr;
                            if (!gdst) {
                            // Without node ordinals no placement list is needed: a level
                            // (revolutions r..cmin, rows with >= r copies) is a count, and
                            // only the last placement's row matters — the m-th row of its
                            // revolution in rotated order, i.e. the t-th qualifying row in
                            // row order, found from the waves' counts and one wave's ballots.
                            int32_t lv_na = nalive;
                            int lv_buf = par ^ 1;     // per-wave partial counts of this level (x[1])
                            for (;;) {
                                const int64_t avail = (lv_cmin - r + 1) * (int64_t)lv_na;
                                if ((int64_t)got + avail >= n) {
                                    const int32_t m0 = n - got;
                                    r += (m0 - 1) / lv_na;
                                    const int32_t m = (m0 - 1) % lv_na + 1;        // rank in rotated order
                                    const int32_t hiN = lv_na - lv_s;              // qualifying rows >= j0
                                    int32_t t = m <= hiN ? lv_s + m : m - hiN;     // rank in row order (1-based)
                                    int w = 0;
                                    for (; w < CW - 1; w++) {
                                        const int32_t cw_ = (int32_t)cred.v[lv_buf][w][1];
                                        if (t <= cw_) break;
                                        t -= cw_;
                                    }
                                    {   // every wave finds it in wave w's counts: no barrier
                                        int32_t lo, hi;
                                        wave_rows(k, w, lo, hi);
                                        for (int32_t b = lo; b < hi; b += 64) {
                                            const int32_t j = b + lane;
                                            const uint64_t bm = __ballot(j < hi && CAPA[j] >= r);
                                            const int32_t pc = __builtin_popcountll(bm);
                                            if (t <= pc) {
                                                const bool hit = ((bm >> lane) & 1ull) && mbcnt(bm) == t - 1;
                                                last = b + __builtin_ctzll(__ballot(hit));
                                                break;
                                            }
                                            t -= pc;
                                        }
                                    }
                                    got = n;
                                    PROF_INC(6);
                                    break;
                                }
                                got += (int32_t)avail;
                                r = (int32_t)lv_cmin + 1;
                                // the next level: rows with at least r copies
                                int32_t lo, hi;
                                wave_rows(k, wv, lo, hi);
                                int32_t cnt_w = 0, lt2 = 0, cm2 = INT32_MAX;
                                for (int32_t b = lo; b < hi; b += 64) {
                                    if (!((adm_w >> ((b - lo) >> 6)) & 1ull)) continue;
                                    const int32_t j = b + lane;
                                    const int32_t c = j < hi ? CAPA[j] : 0;
                                    const bool q = c >= r;
                                    cm2 = q ? min(cm2, c) : cm2;
                                    const uint64_t m = __ballot(q);
                                    cnt_w += __builtin_popcountll(m);
                                    lt2 += __builtin_popcountll(m & lanes_below(j0 - b));
                                }
                                int64_t y[RED_N] = {0, cnt_w, 0, wave_min32(cm2), lt2};   // -, count, -, min, count < j0
                                constexpr int OPS2[RED_N] = {R_SUM, R_SUM, R_SUM, R_MIN, R_SUM};
                                blk_xchg5<GROWS>(cred, par, wv, lane, y, OPS2);
                                lv_buf = par ^ 1;
                                lv_na = (int32_t)y[1];
                                lv_cmin = y[3];
                                lv_s = (int32_t)y[4];
                                PROF_INC(6);
                            }
                            } else {
                            // revolution 1: rows with room, in rotated order from j0
                            int32_t na = 0;
                            int64_t cmin = INT32_MAX, z0 = 0, z1 = 0;
                            for (int32_t b = 0; b < k; b += CT) {
                                const int32_t rr = b + tid;
                                int32_t j = j0 + rr;
                                if (j >= k) j -= k;
                                const int32_t c = rr < k ? CAPA[j] : 0;
                                const bool keep = c >= 1;
                                int32_t tot;
                                const int32_t slot = blk_compact<GROWS>(cred, par, wv, keep, tot);
                                if (keep) { ALIVE[na + slot] = j; cmin = min(cmin, (int64_t)c); }
                                na += tot;
                            }
                            blk_red3<R_MIN, R_SUM, R_SUM, GROWS>(cred, par, wv, lane, cmin, z0, z1);   // + ALIVE visible
                            // Revolutions r..cmin serve the same alive list (no row runs out
                            // before cmin), so the list is compacted once per distinct copy
                            // level, and the placements of those revolutions are the list
                            // repeated: placement t of the level goes to ALIVE[t % na].
                            for (;;) {
                                const int64_t avail = (int64_t)(cmin - r + 1) * na;
                                const bool fin = got + avail >= n;
                                const int32_t cnt = fin ? n - got : (int32_t)avail;
                                if (gdst) {
                                    const int32_t st = CT % na;
                                    int32_t q = tid % na;
                                    for (int32_t t = tid; t < cnt; t += CT) {
                                        gdst[got + t] = ALIVE[q];
                                        q += st;
                                        if (q >= na) q -= na;
                                    }
                                }
                                if (fin) {
                                    r += (cnt - 1) / na;                    // revolution of the last placement
                                    last = ALIVE[(cnt - 1) % na];
                                    got = n;
                                    PROF_INC(6);
                                    break;
                                }
                                got += cnt;
                                r = cmin + 1;
                                // the rows with at least r copies stay
                                // (in place: a chunk's writes land below its end, and the
                                // barrier in blk_compact orders them after the chunk's reads)
                                int32_t nn2 = 0;
                                int64_t cm2 = INT32_MAX;
                                for (int32_t b = 0; b < na; b += CT) {
                                    const int32_t i = b + tid;
                                    const int32_t j = i < na ? ALIVE[i] : 0;
                                    const int32_t c = i < na ? CAPA[j] : 0;
                                    const bool keep = c >= r;
                                    int32_t tot;
                                    const int32_t slot = blk_compact<GROWS>(cred, par, wv, keep, tot);
                                    if (keep) { ALIVE[nn2 + slot] = j; cm2 = min(cm2, (int64_t)c); }
                                    nn2 += tot;
                                }
                                na = nn2;
                                blk_red3<R_MIN, R_SUM, R_SUM, GROWS>(cred, par, wv, lane, cm2, z0, z1);   // + ALIVE visible
                                cmin = cm2;
                                PROF_INC(6);
                            }
                            }
                            PROF_ADD(2, t_rv);
                            PROF_T(t_up);
                            int32_t rl = last - j0;
                            if (rl < 0) rl += k;
                            evals += (uint64_t)(r - 1) * (uint64_t)k + (uint64_t)rl + 1;
                            {   // the wave's own rows, blocks with counts only (others: no room)
                                int32_t lo, hi;
                                wave_rows(k, wv, lo, hi);
                                for (int32_t b = lo; b < hi; b += 64) {
                                    if (!((adm_w >> ((b - lo) >> 6)) & 1ull)) continue;
                                    const int32_t j = b + lane;
                                    const int32_t c = j < hi ? CAPA[j] : 0;
                                    int32_t rj = j - j0;
                                    if (rj < 0) rj += k;
                                    const int32_t nj = min(c, r - 1) + ((c >= r && rj <= rl) ? 1 : 0);
                                    if (nj > 0) {
                                        NodeRec q = R[j];
                                        q.cpu -= (int64_t)nj * pcpu;
                                        q.mem -= (int64_t)nj * pmem;
                                        q.eph -= (int64_t)nj * peph;
                                        q.pods -= nj;
                                        q.used = 1;
                                        R[j] = q;
                                    }
                                }
                            }
                            PROF_ADD(3, t_up);
                            if (last_node >= 0 && !last_used) {      // (the update's nj of last_node)
                                const int32_t c = CAPA[last_node];
                                int32_t rj = last_node - j0;
                                if (rj < 0) rj += k;
                                last_used = min(c, r - 1) + ((c >= r && rj <= rl) ? 1 : 0) > 0;
                            }
                            L = n_base + last + 1;
                            if (L >= len) L -= len;
                            note_success();
                            placed = n;
                        }
                    }
                    PROF_T(t_pb);
                    // The row updates become visible to every wave at the next barrier: right
                    // below when the run ends here, else the node opening's (its rows are new,
                    // beyond every row read or written above)
                    if (tid == 0 && placed > 0) gseg[nseg] = Seg{nsched, pos + done, placed, 0};
                    if (placed > 0) note_segment(nsched, pos + done);
                    nseg += placed > 0 ? 1 : 0;
                    nsched += placed;
                    done += placed;
                    progress();
                    if (done == RN) { cbar<GROWS>(); break; }
                    exhausted = true;
                    // the next pod of the run fails FitsAnyNode: every new node visited
                    evals += kev * (uint64_t)k;
                    if (max_nodes > 0 && granted >= max_nodes) { stop = true; break; }
                    granted++;
                    PROF_ADD(9, t_pb);
                    if (last_node >= 0 && !last_used) {
                        // :114-116 — and every later pod of the run repeats this pod's fate
                        done++;
                        const int32_t q = RN - done;
                        if (max_nodes > 0 && q > max_nodes - granted) {
                            const int32_t allowed = max_nodes - granted;
                            evals += (uint64_t)(allowed + 1) * kev * (uint64_t)k;
                            granted = max_nodes;
                            stop = true;
                            break;
                        }
                        evals += (uint64_t)q * kev * (uint64_t)k;
                        granted += q;
                        done = RN;
                        cbar<GROWS>();
                        break;
                    }
                    if (k >= kcap) { res.status = CA_ECAPACITY; stop = true; break; }
                    const int32_t rem2 = RN - done;
                    if (!((sf & SF_CP_OK) && rec_fits(trec, pcpu, pmem, peph, zero))) {
                        // CheckPredicates on the new node fails: it stays empty and the
                        // next pod of the run takes the empty-node skip above
                        open_node();
                        if (sf & SF_CP_EVAL) evals++;
                        done++;
                        cbar<GROWS>();
                        continue;
                    }
                    // Every row is full for this pod, so each remaining pod group opens a
                    // fresh template copy: pod 1 by CheckPredicates (:132-135), the next
                    // ct-1 by FitsAnyNode, whose scan ends at the new (last) row, so after
                    // the first one lastIndex wraps to 0 and each costs k evals.  A
                    // node's opening pod first fails FitsAnyNode over the k rows before it
                    // and takes one limiter grant.  Closed form over n_open nodes.
                    PROF_T(t_op);
                    const int32_t ct = !(sf & SF_FA_OK) ? 1
                                       : rem2 <= (1 << 20) ? rec_copies_run(trec, dv, zero, rem2, pcpu, pmem, peph)
                                                           : rec_copies(trec, pcpu, pmem, peph, zero, rem2);
                    int32_t n_open = (rem2 + ct - 1) / ct;
                    if (max_nodes > 0) n_open = min(n_open, 1 + (max_nodes - granted));
                    n_open = min(n_open, kcap - k);
                    const int32_t k0 = k;
                    const int32_t placed2 = min(rem2, n_open * ct);
                    const int32_t len0 = n_base + k0 + 1;
                    int32_t s00 = L;
                    if (s00 >= len0) s00 = (int32_t)((uint32_t)s00 % (uint32_t)len0);
                    const int32_t j00 = s00 > n_base ? s00 - n_base : 0;
                    for (int32_t i = tid; i < n_open; i += CT) {
                        const int32_t pi = (i == n_open - 1) ? placed2 - i * ct : ct;
                        NodeRec r = trec;
                        r.cpu -= (int64_t)pi * pcpu;
                        r.mem -= (int64_t)pi * pmem;
                        r.eph -= (int64_t)pi * peph;
                        r.pods -= pi;
                        r.used = 1;
                        R[k0 + i] = r;
                    }
                    for (int32_t b = (k0 >> 6) + tid; b <= ((k0 + n_open - 1) >> 6); b += CT) SUM[b] = trec;
                    if (use_ports) {
                        for (int32_t i = tid; i < n_open * CA_PORT_WORDS; i += CT)
                            PORTS[(size_t)k0 * CA_PORT_WORDS + i] = tp.used_ports[i % CA_PORT_WORDS];
                    }
                    if (use_scalar) {
                        for (int32_t i = tid; i < n_open * CA_MAX_SCALAR; i += CT) {
                            const int32_t sc = i / n_open, node = k0 + i % n_open;
                            SC[(size_t)sc * kcap + node] = wsub(tp.node.alloc_scalar[sc], tp.used_scalar[sc]);
                        }
                    }
                    cbar<GROWS>();                                                  // new rows visible
                    evals += open_evals(n_open, ct, placed2, k0, j00, kev, (sf & SF_CP_EVAL) != 0);
                    if (so_node) for (int32_t t = tid; t < placed2; t += CT) so_node[nsched + t] = k0 + t / ct;
                    if (tid == 0 && placed2 > 0) gseg[nseg] = Seg{nsched, pos + done, placed2, 0};
                    if (placed2 > 0) note_segment(nsched, pos + done);
                    nseg += placed2 > 0 ? 1 : 0;
                    if (ct >= 2 && placed2 >= 2) {
                        if (!first_success) { first_success = true; sensitive = k0 + 1 >= 2; }
                        L = 0;       // n_base + (last row) + 1 == len
                    }
                    k = k0 + n_open;
                    last_node = k - 1;
                    granted += n_open - 1;
                    nsched += placed2;
                    done += placed2;
                    progress();
                    PROF_ADD(4, t_op);
                }
                pos = e;
                PROF_ADD(11, t_run);
                continue;
            }
        }

        // ---------------- one pod ----------------
        // rare per-pod data (ports / scalars) from the full record
        uint64_t pconf[CA_PORT_WORDS] = {0, 0}, puse[CA_PORT_WORDS] = {0, 0};
        int64_t psc[CA_MAX_SCALAR];
        for (int i = 0; i < CA_MAX_SCALAR; i++) psc[i] = 0;
        if (PS && (sf & (SF_PORTS | SF_SCALAR))) {
            const ca_pod_spec& s = specs[ph[pidx].spec];
            for (int w = 0; w < CA_PORT_WORDS; w++) { pconf[w] = s.port_conflict[w]; puse[w] = s.port_use[w]; }
            for (int i = 0; i < CA_MAX_SCALAR; i++) psc[i] = s.req_scalar[i];
        }
        pos++;
        n_single++;

        // ---- FitsAnyNodeMatching(newNodeNames) (binpacking_estimator.go:91-93) ----
        int32_t found = -1;
        if ((sf & SF_EVAL) && k > 0) {
            if (sf & SF_FA_OK) {
                const int32_t len = n_base + k;
                int32_t s0 = L;                                                // (lastIndex+i) % len at i = 0
                if (s0 >= len) s0 = (int32_t)((uint32_t)s0 % (uint32_t)len);   // only for a caller-supplied L
                const int32_t j0 = s0 > n_base ? s0 - n_base : 0;              // first new node visited
                const int32_t nb = (k + 63) >> 6;
                const int32_t b0 = j0 >> 6;
                const bool lower_part = (j0 & 63) != 0;    // block b0 is visited twice (>= j0, then < j0)
                for (int32_t rbase = 0; rbase <= nb && found < 0; rbase += 64) {
                    // visit order: rotated block r -> block (b0 + r) mod nb; r == nb is b0's lower part
                    const int32_t rb = rbase + lane;
                    int32_t b = rb < nb ? b0 + rb : b0;
                    if (b >= nb) b -= nb;
                    const bool rb_ok = (rb < nb) | ((rb == nb) & lower_part);
                    const NodeRec sr = SUM[rb_ok ? b : 0];
                    const bool adm = rb_ok & rec_fits(sr, pcpu, pmem, peph, zero);
                    uint64_t amask = __ballot(adm);
                    while (amask && found < 0) {
                        const int l = __builtin_ctzll(amask);
                        amask &= amask - 1;
                        const int32_t r = rbase + l;
                        int32_t bb = r < nb ? b0 + r : b0;
                        if (bb >= nb) bb -= nb;
                        const int32_t j = (bb << 6) + lane;
                        const bool valid = (j < k) & ((r != 0) | (j >= j0)) & ((r != nb) | (j < j0));
                        const NodeRec nr = R[j < k ? j : 0];
                        bool fit = valid & rec_fits(nr, pcpu, pmem, peph, zero);
                        if (PS && (sf & SF_SCALAR)) {
                            for (int i = 0; i < CA_MAX_SCALAR; i++)
                                fit = fit & !((psc[i] != 0) & (j < k) && psc[i] > SC[(size_t)i * kcap + (j < k ? j : 0)]);
                        }
                        if (PS && (sf & SF_PORTS)) {
                            uint64_t c = 0;
                            for (int w = 0; w < CA_PORT_WORDS; w++) c |= PORTS[(size_t)(j < k ? j : 0) * CA_PORT_WORDS + w] & pconf[w];
                            fit = fit & (c == 0);
                        }
                        const uint64_t fmask = __ballot(fit);
                        if (fmask) {
                            found = (bb << 6) + __builtin_ctzll(fmask);
                        } else {
                            // no row of the visited part fits: tighten the block summary
                            // to the exact per-dimension maxima of the whole block
                            const bool in = j < k;
                            const int64_t mc = wave_max64(in ? nr.cpu : INT64_MIN);
                            const int64_t mm = wave_max64(in ? nr.mem : INT64_MIN);
                            const int64_t me = wave_max64(in ? nr.eph : INT64_MIN);
                            const int32_t mp = wave_max32(in ? nr.pods : INT32_MIN);
                            // (one writer; another wave may read either value of any field:
                            // both bound every row of the block, so its `found` is the same)
                            if (tid == 0) {
                                NodeRec sm;
                                sm.cpu = mc; sm.mem = mm; sm.eph = me; sm.pods = mp; sm.used = 0;
                                SUM[bb] = sm;
                            }
                        }
                    }
                }
                if (found >= 0) {
                    int32_t off = found - j0;                                  // rotated offset among new nodes
                    if (off < 0) off += k;
                    evals += (uint64_t)off + 1;
                    note_success();
                    L = n_base + found + 1;                                    // schedulerbased.go:131
                    if (L >= len) L -= len;
                } else {
                    evals += (uint64_t)k;
                }
            } else {
                evals += (uint64_t)k;                  // every new node visited, filters fail
            }
        }
        if (found < 0) {
            // PermissionToAddNode (threshold_based_limiter.go:46-56), before the empty-node skip
            if (max_nodes > 0 && granted >= max_nodes) break;
            granted++;
            if (last_node >= 0 && !R[last_node].used) continue;               // :114-116
            if (k >= kcap) { res.status = CA_ECAPACITY; break; }
            cbar<GROWS>();                    // every wave's scan is done before rows change
            const int32_t nn = open_node();
            // CheckPredicates(pod, newNode) (:132-134)
            if (sf & SF_CP_EVAL) evals++;
            bool ok = (sf & SF_CP_OK) != 0;
            if (ok) {
                ok = rec_fits(trec, pcpu, pmem, peph, zero);
                if (PS && ok && (sf & SF_SCALAR)) {
                    for (int i = 0; i < CA_MAX_SCALAR; i++)
                        if (psc[i] != 0 && psc[i] > wsub(tp.node.alloc_scalar[i], tp.used_scalar[i])) ok = false;
                }
                if (PS && ok && (sf & SF_PORTS)) {
                    uint64_t c = 0;
                    for (int w = 0; w < CA_PORT_WORDS; w++) c |= tp.used_ports[w] & pconf[w];
                    ok = c == 0;
                }
            }
            if (!ok) { cbar<GROWS>(); continue; }
            found = nn;
        }
        cbar<GROWS>();                        // every wave's scan is done before R[found] changes
        // AddPod(pod, node) (:96 / :135) — NodeInfo.update on the new-node row
        if (tid == 0) {
            NodeRec r = R[found];
            r.cpu = wsub(r.cpu, pcpu);
            r.mem = wsub(r.mem, pmem);
            r.eph = wsub(r.eph, peph);
            r.pods -= 1;
            r.used = 1;
            R[found] = r;
        }
        if (w0 && lane == sl) { out_node = found; out_idx = nsched; pend = true; }
        if (PS && (sf & SF_SCALAR)) {
            if (tid < CA_MAX_SCALAR) {
                const size_t ix = (size_t)tid * kcap + found;
                SC[ix] = wsub(SC[ix], psc[tid]);
            }
        }
        if (PS && (sf & SF_PORTS)) {
            if (tid < CA_PORT_WORDS) PORTS[(size_t)found * CA_PORT_WORDS + tid] |= puse[tid];
        }
        nsched++;
        pure_from = nsched;                   // a single placement: written by the chain itself
        progress();
        cbar<GROWS>();                        // the placement is visible to every wave
    }
    PROF_T(t_epi);
    if (pend) {
        so_pod[out_idx] = pos_out ? wbase + lane : cur.pod;
        if (so_node) so_node[out_idx] = out_node;
    }
    // newNodesWithPods
    cbar<GROWS>();
    int64_t cnt = 0, z0 = 0, z1 = 0;
    for (int32_t j = tid; j < k; j += CT) cnt += R[j].used;
    blk_red3<R_SUM, R_SUM, R_SUM, GROWS>(cred, par, wv, lane, cnt, z0, z1);
    if (tid == 0) {
        res.node_count = (int32_t)cnt;
        res.n_sched = nsched;
        res.nodes_added = k;
        res.lout = L;
        res.sensitive = sensitive ? 1 : 0;
        res.had_success = first_success ? 1 : 0;
        res.evals = evals;
        res.nseg = nseg;
        res.pad = (uint64_t)(uint32_t)(wall_clock64() - t_begin) | ((uint64_t)n_single << 32);
        outs[g] = res;
        hout[g] = res;                          // zero-copy: the host reads it after the round's event
    }
    if (tickets) {
        __threadfence();                        // every wave's result stores, before the release
        __syncthreads();
        if (w0) {
            const bool ok = res.status == CA_OK;
            // a group that failed after publishing chunks: the host falls back to the copy
            if (!ok && tk_next > 0 && lane == 0) { atomicExch(&qctl[3], 1); hflags[3] = 1; }
            // every pod scheduled: the tail chunks are pure when one segment offset covers them
            // (the publisher copies them straight from the stream's ids, no segment reads)
            const bool all = ok && nsched == P;
            push_chunks(g, tk_next, (P + pch - 1) / pch, nsub, tickets, qctl, prog, ok ? nseg : 0, ok ? nsched : 0, lane,
                        all ? pch : 0, all ? pure_from : INT32_MAX, pure_off);
        }
    }
    if (tid == 0) {
#ifdef CASIM_PROF
        prof[13] = clock64() - t_epi;
        prof[5] = clock64() - t_cyc0;
        if (g < 1024) for (int i = 0; i < NPROF; i++) g_chain_prof[g][i] = prof[i];
#endif
    }
}

// Round-1 state of a batch in one launch instead of five copies/fills on the critical
// path: every group needed, every group from the caller's lastIndex, no unsupported
// group yet, publisher tickets empty, queue counters zero.
__global__ void __launch_bounds__(256) k_round_init(int32_t G, int32_t lin0, int32_t* __restrict__ lin,
                                                   uint8_t* __restrict__ need, uint32_t* __restrict__ unsup,
                                                   int64_t* __restrict__ tickets, int32_t n_tickets,
                                                   int32_t* __restrict__ qctl) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int32_t stride = (int32_t)(gridDim.x * blockDim.x);
    for (int32_t g = i; g < G; g += stride) { lin[g] = lin0; need[g] = 1; unsup[g] = 0; }
    if (tickets)
        for (int32_t t = i; t < n_tickets; t += stride) tickets[t] = -1;
    if (qctl && i < 6) qctl[i] = 0;
}

// 5. scheduled pods of the run placements: sched_pod[dst + t] = stream pod at src + t.
// Output i of a group lies in the last segment with dst <= i, or was written directly
// by the chain (single-pod placements).  One block per CPY_PER_BLOCK outputs: one
// binary search for the first segment reaching the block's range, then the segments
// of the range are copied in turn (coalesced reads of the stream's pod ids).
constexpr int CPY_PER_BLOCK = 2048;
__global__ void __launch_bounds__(256) k_copy_segments(const GroupMeta* __restrict__ groups,
                                                      const ChainOut* __restrict__ outs, const Seg* __restrict__ segs,
                                                      const int32_t* __restrict__ spod, int32_t* __restrict__ sched_pod,
                                                      int32_t* __restrict__ sched_node, int32_t map_singles) {
    const GroupMeta gm = groups[blockIdx.y];
    const ChainOut o = outs[blockIdx.y];
    const int32_t base = (int32_t)blockIdx.x * CPY_PER_BLOCK;
    if (base >= gm.count) return;
    const int32_t end = min(base + CPY_PER_BLOCK, gm.count);
    const int32_t ns = o.status == CA_OK ? o.n_sched : 0;
    const int32_t nseg = o.status == CA_OK ? o.nseg : 0;
    const Seg* gs = segs + gm.off;
    int32_t* sp = sched_pod + gm.off;
    const int32_t* src = spod + gm.off;
    // past n_scheduled (or a failed group): -1, also over what an earlier speculation
    // round of the group wrote
    for (int32_t i = max(base, ns) + (int32_t)threadIdx.x; i < end; i += blockDim.x) {
        sp[i] = -1;
        if (sched_node) sched_node[gm.off + i] = -1;
    }
    const int32_t lim = min(end, ns);
    if (base >= lim) return;
    int32_t lo = 0, hi = nseg;                     // first segment ending after base
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        const Seg sg = gs[mid];
        if (sg.dst + sg.len <= base) lo = mid + 1; else hi = mid;
    }
    int32_t at = base;                              // single placements before segment q
    for (int32_t q = lo; q <= nseg && at < lim; q++) {
        const Seg sg = q < nseg ? gs[q] : Seg{lim, 0, 0};
        const int32_t gap_end = min(lim, max(at, sg.dst));
        if (map_singles)                            // stream positions -> pod ids (decoupled Go order)
            for (int32_t i = at + (int32_t)threadIdx.x; i < gap_end; i += blockDim.x) sp[i] = src[sp[i]];
        if (q == nseg || sg.dst >= lim) break;
        const int32_t a = max(base, sg.dst), b = min(lim, sg.dst + sg.len);
        const int32_t off = sg.src - sg.dst;
        for (int32_t i = a + (int32_t)threadIdx.x; i < b; i += blockDim.x) sp[i] = src[off + i];
        at = max(at, b);
    }
}

}  // namespace casim

using namespace casim;

struct ca_estimate_plan {
    ca_mirror* m = nullptr;
    const ca_podset* s = nullptr;
    int32_t G = 0;
    int32_t total = 0;
    int32_t max_count = 0;
    std::vector<int32_t> h_off;
    std::vector<ca_template> h_tmpl;
    std::vector<GroupMeta> h_meta;
    bool use_ports = false, use_scalar = false;
    int32_t n_masks = 0, n_tiles = 0;
    DevBuf d_meta, d_pod_idx, d_tmpl, d_sortA, d_sortB, d_stream, d_spod, d_seg, d_heads, d_unsup, d_lin, d_need,
        d_out, d_sched_pod, d_sched_node, d_crank, d_hist, d_sched16;
    // Go sort.Slice order (k_pdq_sort): element store, list scratch, frame stacks, and the
    // per-position ranks of the comparison path
    DevBuf d_pdq_e, d_pdq_scr, d_pdq_stack, d_item_rank;
    // decoupled Go order (uniform classes): the chains run on the stable class order while
    // k_pdq_sort on st3 writes the Go-order ids into d_spod_go (d_sortC: the
    // permutation; d_ids_ready: per group, the run epoch whose ids are final there)
    DevBuf d_sortC, d_ids_ready, d_spod_go, d_crank2;
    DevBuf d_rstart, d_rsp;        // decoupled: per group, each rank's first stream position and record
    DevBuf d_item_cls;             // bucket path: the score class of every (group, pod) item, uploaded with the lists
    int32_t ids_epoch = 0;
    hipStream_t st3 = nullptr;
    hipEvent_t ev_emitA = nullptr, ev_emitB = nullptr, ev_ids = nullptr;
    // HBM-slab rows (k_ffd_chain<true>): per group kcap and slab offset, for the limiter
    // setting they were sized for (slab_max_nodes)
    DevBuf d_slab, d_slab_off, d_gkcap;
    int32_t slab_max_nodes = -2;
    int32_t n_hist = 0, max_rtiles = 0;
    bool bucket = false;           // bucket sort over score classes (podset has <= CLS_MAX classes)
    // decoupled Go order allowed: uniform classes, bucket path, and no
    // group holds two classes whose float64 scores against its template are equal
    bool decouple_ok = false;
    Stats stats;
    // per-phase device timings of the last run (ms): score, merge, emit, chain (all
    // rounds), compact, d2h; and the host wall time of the call
    enum { EV_START, EV_SCORE, EV_MERGE, EV_EMIT, EV_CHAIN0, EV_CHAIN1, EV_COMPACT, EV_D2H, EV_N };
    hipEvent_t ev[EV_N] = {};
    float t_ms[7] = {};
    int32_t pub_state = 0;         // last run: 0 results copied, 1 published zero-copy, 2 publisher gave up
    // the publisher's tickets are all -1 and its control words zero on the device: every
    // publisher consumed and reset its tickets and its last block cleared the words (round 1
    // then needs no k_round_init; false at first and after a publisher gave up)
    bool pub_clean = false;
    int32_t ran_decoupled = 0;     // last run took the decoupled Go order
    bool phase_events = true;      // record the per-phase timing events (ca_estimate_plan_set_phase_timing)
    std::vector<uint64_t> diag;     // per group: chain ticks (100 MHz) | single-pod steps << 32
    std::vector<uint8_t> grp_succ;  // last run, per group: a FitsAnyNode call succeeded (moved lastIndex)
    // zero-copy publishing (k_publish on its own stream, concurrent with the chains)
    hipStream_t pub_stream = nullptr;
    hipEvent_t ev_go = nullptr, ev_pub = nullptr;
    DevBuf d_tickets, d_qctl;
    int32_t n_tickets = 0, nsub = 0, pch = PCH;
    DevBuf d_prog;                 // progress record per ticket slot (segments, pods scheduled)
    // page-locked landing buffers of the per-round readback (chain outputs + publisher
    // counters): one small D2H each and one synchronisation per round
    HostBuf h_out, h_qc;
    // Heavy groups first: the chains of the groups whose closed-form FFD
    // runs longest start as soon as their own sort is done, while the other groups sort
    // on a second, lower-priority stream.  demand[g] = template copies the group's pods
    // need (max over cpu, memory, pod slots of sum / template free); the map
    // [heavy..., rest...] is rebuilt when the limiter's max_nodes changes.
    std::vector<double> demand;
    hipStream_t st2 = nullptr;
    hipEvent_t ev_init = nullptr, ev_b = nullptr, ev_rb = nullptr;
    DevBuf d_gmap;
    int32_t map_max_nodes = -1, n_heavy = 0;
    int32_t map_source = 0;        // 1: demand model, 2: the chains' measured times (previous run)
    int32_t res_device = -1;       // the streams and events below came from the pool of this device
    ~ca_estimate_plan();
};

namespace casim {
// Streams and events of an Estimate plan, kept per device after the plan is destroyed and
// handed to the next plan (RunOnce builds a plan per loop: creating three streams and
// sixteen events costs more than a loop's whole Estimate).  The plan's destructor drains its
// three streams first (a run that failed part-way may have left kernels queued), so a
// released set is idle.
struct PlanStreams {
    hipStream_t pub = nullptr, st2 = nullptr, st3 = nullptr;
    hipEvent_t ev[ca_estimate_plan::EV_N] = {};
    hipEvent_t go = nullptr, pub_ev = nullptr, emitA = nullptr, emitB = nullptr, ids = nullptr, init = nullptr, b = nullptr,
               rb = nullptr;
};
static std::mutex g_ps_mu;
static std::vector<std::pair<int32_t, PlanStreams>> g_ps_pool;

static int plan_streams_acquire(int32_t dev, PlanStreams& out) {
    {
        std::lock_guard<std::mutex> lk(g_ps_mu);
        for (size_t i = 0; i < g_ps_pool.size(); i++)
            if (g_ps_pool[i].first == dev) {
                out = g_ps_pool[i].second;
                g_ps_pool.erase(g_ps_pool.begin() + (ptrdiff_t)i);
                return CA_OK;
            }
    }
    PlanStreams ps;
    for (auto& e : ps.ev) CA_HIP_CHECK(hipEventCreate(&e));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.go, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.pub_ev, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.emitA, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.emitB, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.ids, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.init, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.b, hipEventDisableTiming));
    CA_HIP_CHECK(hipEventCreateWithFlags(&ps.rb, hipEventDisableTiming));
    CA_HIP_CHECK(hipStreamCreateWithFlags(&ps.pub, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CA_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CA_HIP_CHECK(hipStreamCreateWithPriority(&ps.st2, hipStreamNonBlocking, lo));   // light groups: lowest
    CA_HIP_CHECK(hipStreamCreateWithPriority(&ps.st3, hipStreamNonBlocking, hi));   // Go-order sort: highest
    out = ps;
    return CA_OK;
}
}  // namespace casim

ca_estimate_plan::~ca_estimate_plan() {
    casim::PlanStreams ps;
    for (int i = 0; i < EV_N; i++) ps.ev[i] = ev[i];
    ps.go = ev_go; ps.pub_ev = ev_pub; ps.emitA = ev_emitA; ps.emitB = ev_emitB; ps.ids = ev_ids; ps.init = ev_init;
    ps.b = ev_b; ps.rb = ev_rb;
    ps.pub = pub_stream; ps.st2 = st2; ps.st3 = st3;
    // a run that returned early on an error may have left kernels queued on these streams
    // (a publisher polls for up to its deadline): drain them before the set is pooled or
    // destroyed, and before the plan's buffers go back to the allocation cache
    if (res_device >= 0) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != res_device) (void)hipSetDevice(res_device);
        for (hipStream_t q : {ps.pub, ps.st2, ps.st3}) if (q) (void)hipStreamSynchronize(q);
        if (cur >= 0 && cur != res_device) (void)hipSetDevice(cur);
    }
    if (res_device >= 0 && pub_stream && st2 && st3) {
        std::lock_guard<std::mutex> lk(casim::g_ps_mu);
        casim::g_ps_pool.emplace_back(res_device, ps);
        return;
    }
    for (auto& e : ps.ev) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ps.go, ps.pub_ev, ps.emitA, ps.emitB, ps.ids, ps.init, ps.b, ps.rb}) if (e) (void)hipEventDestroy(e);
    for (hipStream_t q : {ps.pub, ps.st2, ps.st3}) if (q) (void)hipStreamDestroy(q);
}

namespace {

// The decoupled Go order runs the chains on the stable class order and takes the pod ids
// from Go's sort.Slice permutation at the same positions.  That is exact only if both
// orders hold the same class at every sorted position of a group: k_class_rank gives two
// classes with equal float64 scores one dense rank, and pdqsort interleaves their pods
// differently from list position.  So: no group may hold two classes of one score
// (binpacking_estimator.go:72-74, 164-193; same float64 operations as k_class_rank,
// -ffp-contract=off).  Per group, the U class scores against the template are sorted;
// only when a tie exists are the group's own classes looked up.
bool groups_tie_free(const ca_podset* s, const int32_t* pod_idx, const std::vector<GroupMeta>& meta,
                     const ca_template* templates) {
    const int32_t U = s->n_cls;
    if (U < 2) return true;
    std::vector<std::pair<uint64_t, int32_t>> key((size_t)U);
    std::vector<int32_t> seen((size_t)U, -1);
    std::vector<int32_t> runs;                        // classes of tied runs, -1 between runs
    for (size_t g = 0; g < meta.size(); g++) {
        const ca_template& tp = templates[meta[g].tmpl];
        const int64_t acpu = tp.node.alloc_milli_cpu, amem = tp.node.alloc_memory;
        for (int32_t c = 0; c < U; c++) {
            double score = 0.0;
            if (acpu > 0) score += (double)s->h_cls_sc[2 * c] / (double)acpu;
            if (amem > 0) score += (double)s->h_cls_sc[2 * c + 1] / (double)amem;
            uint64_t b;
            std::memcpy(&b, &score, sizeof b);
            key[c] = {b, c};
        }
        std::sort(key.begin(), key.end());
        runs.clear();
        for (int32_t i = 1; i < U; i++) {
            if (key[i].first != key[i - 1].first) continue;
            if (runs.empty() || runs.back() != key[i - 1].second) {
                if (!runs.empty()) runs.push_back(-1);
                runs.push_back(key[i - 1].second);
            }
            runs.push_back(key[i].second);
        }
        if (runs.empty()) continue;
        for (int32_t i = meta[g].off; i < meta[g].off + meta[g].count; i++) seen[s->h_cls[pod_idx[i]]] = (int32_t)g;
        int32_t present = 0;
        for (size_t i = 0; i <= runs.size(); i++) {
            if (i == runs.size() || runs[i] < 0) { present = 0; continue; }
            if (seen[runs[i]] == (int32_t)g && ++present >= 2) return false;
        }
    }
    return true;
}

int plan_prepare(ca_estimate_plan* p, ca_mirror* m, const ca_podset* s, const int32_t* group_off,
                 const int32_t* pod_idx, const ca_template* templates, int32_t G) {
    p->m = m; p->s = s; p->G = G;
    {
        PlanStreams ps;                      // (pooled per device: plan_streams_acquire)
        int rc0;
        if ((rc0 = plan_streams_acquire(m->device, ps)) != CA_OK) return rc0;
        for (int i = 0; i < ca_estimate_plan::EV_N; i++) p->ev[i] = ps.ev[i];
        p->ev_go = ps.go; p->ev_pub = ps.pub_ev; p->ev_emitA = ps.emitA; p->ev_emitB = ps.emitB; p->ev_ids = ps.ids;
        p->ev_init = ps.init; p->ev_b = ps.b; p->ev_rb = ps.rb;
        p->pub_stream = ps.pub; p->st2 = ps.st2; p->st3 = ps.st3;
        p->res_device = m->device;
    }
    {
        int rc0;
        if ((rc0 = p->h_out.reserve(sizeof(ChainOut) * (size_t)std::max(G, 1))) != CA_OK) return rc0;
        if ((rc0 = p->h_qc.reserve(sizeof(int32_t) * 5)) != CA_OK) return rc0;
    }
    p->h_off.assign(group_off, group_off + G + 1);
    p->h_tmpl.assign(templates, templates + G);
    p->total = group_off[G] - group_off[0];
    if (group_off[0] != 0) return CA_EINVAL;
    p->h_meta.resize(G);
    p->max_count = 0;
    p->n_masks = 0;
    p->n_tiles = 0;
    p->n_hist = 0;
    p->max_rtiles = 0;
    {
        const char* e = knob_env("CASIM_SORT");      // "merge" forces the comparison sort (tests run both)
        p->bucket = s->n_cls <= CLS_MAX && !(e && strcmp(e, "merge") == 0);
    }
    for (int32_t g = 0; g < G; g++) {
        const int32_t c = group_off[g + 1] - group_off[g];
        if (c < 0) return CA_EINVAL;
        GroupMeta& gm = p->h_meta[g];
        const ca_template& t = templates[g];
        gm.tcpu = wsub(t.node.alloc_milli_cpu, t.used_milli_cpu);
        gm.tmem = wsub(t.node.alloc_memory, t.used_memory);
        gm.teph = wsub(t.node.alloc_ephemeral, t.used_ephemeral);
        gm.tpods = clamp_i32(t.node.alloc_pods - t.used_pods);
        gm.off = group_off[g];
        gm.count = c;
        gm.tmpl = g;
        gm.tflags = t.node.flags;
        gm.moff = p->n_masks;
        gm.toff = p->n_tiles;
        gm.rtiles = (c + RT - 1) / RT;
        gm.hoff = p->n_hist;
        gm.pad = 0;
        p->n_hist += 256 * gm.rtiles;
        p->max_rtiles = std::max(p->max_rtiles, gm.rtiles);
        p->n_masks += (c + 63) / 64;
        p->max_count = std::max(p->max_count, c);
        for (int w = 0; w < CA_PORT_WORDS; w++) if (t.used_ports[w]) p->use_ports = true;
        for (int i = 0; i < CA_MAX_SCALAR; i++)
            if (t.node.alloc_scalar[i] || t.used_scalar[i]) p->use_scalar = true;
    }
    hipStream_t st = m->stream;
    int rc;
    const size_t tot = (size_t)std::max(p->total, 1);
    // One pass over the lists (per-pod summaries of the podset: compact arrays instead of
    // the 208-B records), split over host threads for big batches: index validation, the
    // port / extended-resource flags and each group's summed requests for the demand
    // order.  The lists travel to the device meanwhile (the caller's thread queues the copy);
    // the item classes are gathered there from the podset's class column (k_item_cls).
    {
        const int32_t total = p->total;
        const int32_t T = std::max(1, std::min(7, total / (1 << 17)));
        struct Part { bool bad = false; uint8_t fl = 0; std::vector<double> c, mm; };
        std::vector<Part> part((size_t)T);
        const bool want_fl = s->any_ports || s->any_scalar;
        auto work = [&](int32_t t) {
            Part& pt = part[(size_t)t];
            pt.c.assign((size_t)G, 0.0);
            pt.mm.assign((size_t)G, 0.0);
            const int32_t a = (int32_t)((int64_t)total * t / T), b = (int32_t)((int64_t)total * (t + 1) / T);
            int32_t g = (int32_t)(std::upper_bound(group_off, group_off + G + 1, a) - group_off) - 1;
            const int32_t np_ = s->t.n_pods;
            const int64_t* req = s->h_req.data();
            for (int32_t i = a; i < b && !pt.bad;) {
                while (g < G - 1 && group_off[g + 1] <= i) g++;
                const int32_t e = std::min(b, group_off[g + 1]);
                double c0 = 0, c1 = 0, m0 = 0, m1 = 0;   // (two chains each: the adds pipeline)
                bool bad = false;
                int32_t k = i;
                for (; k + 1 < e; k += 2) {
                    const int32_t p0 = pod_idx[k], p1 = pod_idx[k + 1];
                    bad |= (uint32_t)p0 >= (uint32_t)np_ || (uint32_t)p1 >= (uint32_t)np_;
                    if (bad) break;
                    c0 += (double)req[2 * (size_t)p0]; m0 += (double)req[2 * (size_t)p0 + 1];
                    c1 += (double)req[2 * (size_t)p1]; m1 += (double)req[2 * (size_t)p1 + 1];
                }
                if (!bad && k < e) {
                    const int32_t p0 = pod_idx[k];
                    bad = (uint32_t)p0 >= (uint32_t)np_;
                    if (!bad) { c0 += (double)req[2 * (size_t)p0]; m0 += (double)req[2 * (size_t)p0 + 1]; }
                }
                if (bad) { pt.bad = true; break; }
                if (want_fl)
                    for (int32_t q = i; q < e; q++) pt.fl |= s->h_pflags[pod_idx[q]];
                pt.c[(size_t)g] += c0 + c1;
                pt.mm[(size_t)g] += m0 + m1;
                i = e;
            }
        };
        hipError_t ce = hipSuccess;
        rc = CA_OK;
        // task 0 (the caller's thread) queues the list upload, tasks 1..T walk the items
        casim::parallel_run(T + 1, [&](int32_t t) {
            if (t > 0) { work(t - 1); return; }
            if ((rc = p->d_pod_idx.reserve(sizeof(int32_t) * tot)) == CA_OK && total)
                ce = hipMemcpyAsync(p->d_pod_idx.ptr, pod_idx, sizeof(int32_t) * total, hipMemcpyHostToDevice, st);
        });
        if (rc != CA_OK) return rc;
        CA_HIP_CHECK(ce);
        bool bad = false;
        p->demand.assign(G, 0.0);
        std::vector<double> c((size_t)G, 0.0), mm((size_t)G, 0.0);
        for (const Part& pt : part) {
            bad |= pt.bad;
            if (pt.fl & 1) p->use_ports = true;
            if (pt.fl & 2) p->use_scalar = true;
            for (int32_t g = 0; g < G; g++) { c[(size_t)g] += pt.c[(size_t)g]; mm[(size_t)g] += pt.mm[(size_t)g]; }
        }
        if (bad) {
            CA_HIP_CHECK(hipStreamSynchronize(st));    // (the list copy may still read pod_idx)
            return CA_EINVAL;
        }
        for (int32_t g = 0; g < G; g++) {
            const GroupMeta& gm = p->h_meta[g];
            double d = gm.tpods > 0 ? (double)gm.count / gm.tpods : 0.0;
            if (gm.tcpu > 0) d = std::max(d, c[(size_t)g] / (double)gm.tcpu);
            if (gm.tmem > 0) d = std::max(d, mm[(size_t)g] / (double)gm.tmem);
            p->demand[g] = d;
        }
    }
    p->decouple_ok = p->bucket && s->cls_uniform && groups_tie_free(s, pod_idx, p->h_meta, templates);
    if ((rc = p->d_meta.reserve(sizeof(GroupMeta) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_tmpl.reserve(sizeof(ca_template) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_sortA.reserve(sizeof(SortItem) * tot)) != CA_OK) return rc;
    if ((rc = p->d_sortB.reserve(sizeof(SortItem) * tot)) != CA_OK) return rc;
    if ((rc = p->d_stream.reserve(sizeof(StreamPod) * tot)) != CA_OK) return rc;
    if ((rc = p->d_heads.reserve(sizeof(uint64_t) * (size_t)std::max(p->n_masks, 1))) != CA_OK) return rc;
    if ((rc = p->d_spod.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
    if ((rc = p->d_seg.reserve(sizeof(Seg) * tot)) != CA_OK) return rc;
    {
        const char* so = knob_env("CASIM_SORT_ORDER");                 // (go_sort_order(), below)
        const bool go_ord = !(so && strcmp(so, "stable") == 0);
        p->pch = (p->decouple_ok && go_ord) ? PCH_DECOUPLED : PCH;
    }
    if (const char* e = knob_env("CASIM_PUB_CHUNK")) p->pch = std::max(1, atoi(e));
    const int32_t pch = p->pch;
    p->n_tickets = 0;
    for (int32_t g = 0; g < G; g++) p->n_tickets += (p->h_meta[g].count + pch - 1) / pch;
    p->nsub = std::max(1, (p->max_count + pch - 1) / pch);
    if ((rc = p->d_tickets.reserve(sizeof(int64_t) * (size_t)std::max(p->n_tickets, 1))) != CA_OK) return rc;
    if ((int64_t)G * p->nsub < INT32_MAX &&
        (rc = p->d_prog.reserve(sizeof(int2) * (size_t)G * (size_t)p->nsub)) != CA_OK) return rc;
    if ((rc = p->d_qctl.reserve(sizeof(int32_t) * 6)) != CA_OK) return rc;
    if ((rc = p->d_unsup.reserve(sizeof(uint32_t) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_lin.reserve(sizeof(int32_t) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_need.reserve((size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_out.reserve(sizeof(ChainOut) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_sched_pod.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
    if ((rc = p->d_sched_node.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
    if (p->bucket) {
        if ((rc = p->d_crank.reserve(sizeof(int32_t) * (size_t)std::max(G, 1) * (size_t)std::max(s->n_cls, 1))) != CA_OK)
            return rc;
        if ((rc = p->d_hist.reserve(sizeof(int32_t) * (size_t)std::max(p->n_hist, 1))) != CA_OK) return rc;
    }
    if ((rc = p->d_pdq_e.reserve(sizeof(uint64_t) * tot)) != CA_OK) return rc;
    if ((rc = p->d_pdq_scr.reserve(sizeof(uint64_t) * tot)) != CA_OK) return rc;
    if ((rc = p->d_pdq_stack.reserve(sizeof(pdq::Frame) * (tot / 2 + 2 * (size_t)std::max(G, 1) + 2))) != CA_OK)
        return rc;
    if (!p->bucket && (rc = p->d_item_rank.reserve(sizeof(uint32_t) * tot)) != CA_OK) return rc;
    if (p->decouple_ok) {
        if ((rc = p->d_sortC.reserve(sizeof(uint32_t) * tot)) != CA_OK) return rc;
        if ((rc = p->d_spod_go.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
        if ((rc = p->d_ids_ready.reserve(sizeof(int32_t) * (size_t)std::max(G, 1))) != CA_OK) return rc;
        CA_HIP_CHECK(hipMemset(p->d_ids_ready.ptr, 0, sizeof(int32_t) * (size_t)std::max(G, 1)));   // epoch 0: none
        p->ids_epoch = 0;
        if ((rc = p->d_crank2.reserve(sizeof(int32_t) * (size_t)std::max(G, 1) * (size_t)std::max(s->n_cls, 1))) != CA_OK)
            return rc;
        if ((rc = p->d_rstart.reserve(sizeof(int32_t) * (size_t)std::max(G, 1) * (size_t)(s->n_cls + 1))) != CA_OK)
            return rc;
        if ((rc = p->d_rsp.reserve(sizeof(StreamPod) * (size_t)std::max(G, 1) * (size_t)std::max(s->n_cls, 1))) != CA_OK)
            return rc;
    }
    if (G) CA_HIP_CHECK(hipMemcpyAsync(p->d_meta.ptr, p->h_meta.data(), sizeof(GroupMeta) * G, hipMemcpyHostToDevice, st));
    if (p->bucket && p->total > 0) {
        // the lists as (pod, class) pairs: the class of every item next to its pod index, so
        // the sorts and the run table read it in one coalesced load instead of two gathers
        if ((rc = p->d_item_cls.reserve(sizeof(int32_t) * (size_t)p->total)) != CA_OK) return rc;
        const int32_t nb = (int32_t)std::min<int64_t>(4096, (p->total + 255) / 256);
        hipLaunchKernelGGL(k_item_cls, dim3(nb), dim3(256), 0, st, p->d_pod_idx.as<int32_t>(),
                           s->d_cls.as<int32_t>(), p->d_item_cls.as<int32_t>(), p->total);
        CA_HIP_CHECK(hipGetLastError());
    }
    if (G) CA_HIP_CHECK(hipMemcpyAsync(p->d_tmpl.ptr, templates, sizeof(ca_template) * G, hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipStreamSynchronize(st));
    return CA_OK;
}

// how long a publisher waits for the first chain of its batch to start (100 MHz ticks):
// the chains are launched just before it, so a chain not running by then means the two
// kernels were serialised (CASIM_PUB_START_US overrides; default 2 ms)
uint64_t pub_start_ticks() {
    const char* e = knob_env("CASIM_PUB_START_US");
    const long us = e ? std::max(1L, atol(e)) : 2000L;
    return (uint64_t)us * 100ull;
}

__global__ void k_narrow16(const int32_t* __restrict__ src, uint16_t* __restrict__ dst, int32_t n) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = (uint16_t)src[i];
}

// the plan's device results (sched_pod layout) into the caller's buffer: int32 ids, or
// 16-bit ids narrowed on the device first (stream-ordered copies)
int results_to_host(ca_estimate_plan* p, hipStream_t st, int32_t* sched_pod, uint16_t* sched16) {
    const int32_t n = std::max(p->total, 0);
    if (!sched16) {
        CA_HIP_CHECK(hipMemcpyAsync(sched_pod, p->d_sched_pod.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
        return CA_OK;
    }
    int rc;
    if ((rc = p->d_sched16.reserve(sizeof(uint16_t) * (size_t)std::max(n, 1))) != CA_OK) return rc;
    if (n > 0) {
        hipLaunchKernelGGL(k_narrow16, dim3((n + 255) / 256), dim3(256), 0, st, p->d_sched_pod.as<int32_t>(),
                           p->d_sched16.as<uint16_t>(), n);
        CA_HIP_CHECK(hipGetLastError());
        CA_HIP_CHECK(hipMemcpyAsync(sched16, p->d_sched16.ptr, sizeof(uint16_t) * n, hipMemcpyDeviceToHost, st));
    }
    return CA_OK;
}

// Estimate's tie order: Go 1.19 sort.Slice (the reference, default) or, with
// CASIM_SORT_ORDER=stable, ties by list position (the radix / merge paths alone)
bool go_sort_order() {
    const char* e = knob_env("CASIM_SORT_ORDER");
    return !(e && strcmp(e, "stable") == 0);
}

// k_pdq_sort for `ng` groups (map gm) into d_sortA: ranks from the class ranks (crank, U)
// or from item_rank
int launch_pdq_sort(ca_estimate_plan* p, hipStream_t ss, const int32_t* gm, int32_t ng, const int32_t* crank,
                    int32_t U, const uint32_t* item_rank, int32_t force = 0, uint32_t* out = nullptr,
                    int32_t* ids_out = nullptr, int32_t* ids_ready = nullptr, int32_t ids_epoch = 0,
                    int32_t fold_np = 0) {
    const int32_t lds_n = std::min(p->max_count, PDQ_LDS_N);
    const size_t lds = pdq_lds_bytes(lds_n);
    int rc;
    if ((rc = ensure_dyn_lds((const void*)k_pdq_sort, lds)) != CA_OK) return rc;
    hipLaunchKernelGGL(k_pdq_sort, dim3(ng), dim3(pdq::NT), lds, ss, p->d_meta.as<GroupMeta>(),
                       p->d_pod_idx.as<int32_t>(), p->s ? p->s->d_cls.as<int32_t>() : nullptr, crank, U, item_rank,
                       out ? out : p->d_sortA.as<uint32_t>(), p->d_pdq_e.as<uint64_t>(), p->d_pdq_scr.as<uint64_t>(),
                       p->d_pdq_stack.as<pdq::Frame>(), lds_n, force, 0, gm, ids_out, ids_ready, ids_epoch,
                       (p->bucket && crank && !item_rank) ? p->d_item_cls.as<int32_t>() : nullptr,
                       p->d_tmpl.as<ca_template>(), fold_np > 0 ? p->s->d_cls_sc.as<int64_t>() : nullptr, fold_np);
    CA_HIP_CHECK(hipGetLastError());
    return CA_OK;
}

int32_t pub_blocks(bool decoupled) {
    const char* e = knob_env("CASIM_PUB_BLOCKS");
    // scripts/pub_sweep.sh on C2: stable order 32 x 4096-output chunks; decoupled Go order
    // 128 x 8192 in round 4 (each group's ids are ready when its own sort ends, from ~0.17 ms
    // on; more blocks in flight keep a block waiting on a late group from holding up the
    // ready ones — 0.474 against 0.478 ms for 64 x 16384, interleaved repeats,
    // scripts/gpu_pubsweep2.sh); with round 6's chains and sort, 64 x 16384 (A/Bs of variant
    // builds: profiles/r06_pub_chunk_ab.txt, r06_pub_blocks_ab.txt)
#ifndef CASIM_PUB_BLOCKS_DECOUPLED
#define CASIM_PUB_BLOCKS_DECOUPLED 64
#endif
    return e ? std::max(1, atoi(e)) : (decoupled ? CASIM_PUB_BLOCKS_DECOUPLED : 32);
}

size_t chain_lds_bytes(int32_t kcap, bool use_ports, bool use_scalar) {
    const size_t nb = (size_t)((kcap + 63) >> 6);
    size_t b = 32 * ((size_t)kcap + nb) + 8 * (size_t)kcap;   // rows, summaries, CAPA + ALIVE
    if (use_ports) b += 8 * CA_PORT_WORDS * (size_t)kcap;
    if (use_scalar) b += 8 * CA_MAX_SCALAR * (size_t)kcap;
    return (b + 15) & ~(size_t)15;
}

int plan_run(ca_estimate_plan* p, const ca_limiter* lim, int32_t* last_index, ca_estimate_result* results,
             int32_t* sched_pod, int32_t* sched_node, uint16_t* sched16 = nullptr) {
    ca_mirror* m = p->m;
    hipStream_t st = m->stream;
    const int32_t G = p->G;
    if (!lim || !last_index || !results) return CA_EINVAL;
    // sched_pod == NULL: the scheduled pods stay in device memory (ca_estimate_plan_fetch /
    // ca_estimate_plan_device_results); no node ordinals then
    const bool to_host = sched_pod != nullptr || sched16 != nullptr;
    if (!to_host && sched_node) return CA_EINVAL;
    // 16-bit results: pod ids of a podset of at most 65535 pods (0xFFFF: not scheduled)
    if (sched16 && (sched_pod || sched_node || p->s->n_host > 65535)) return CA_EINVAL;
    p->pub_state = 0;
    const auto t_start = std::chrono::steady_clock::now();
    // CASIM_STEP_TIMING (read once per process): host-side split of the steps, averaged over
    // 20 calls — entry to the first launch, to the last launch, to the join, to the return,
    // and the caller's time between a return and the next entry
    static const bool step_timing = knob_env("CASIM_STEP_TIMING") != nullptr;
    static double st_acc[6] = {0, 0, 0, 0, 0, 0};
    static int st_n = 0;
    static std::chrono::steady_clock::time_point st_last_exit;
    std::chrono::steady_clock::time_point st_t[4];
    auto st_mark = [&](int k) { if (step_timing) st_t[k] = std::chrono::steady_clock::now(); };
    CA_HIP_CHECK(hipSetDevice(m->device));
    const int32_t n_base = (int32_t)m->nodes.size();
    if (G == 0) return CA_OK;
    if (m->n_scope_blockers > 0) return CA_EUNSUPPORTED;    // casim.h scope: required anti-affinity in the snapshot
    // kcap: new nodes a group can add (limiter cap, or one per pod when unlimited: a group
    // never opens more nodes than it has pods)
    int32_t kcap = lim->max_nodes > 0 ? std::min(lim->max_nodes, std::max(p->max_count, 1)) : std::max(p->max_count, 1);
    kcap = ((kcap + 63) / 64) * 64;
    size_t lds = chain_lds_bytes(kcap, p->use_ports, p->use_scalar);
    // rows that do not fit the CU's LDS (an unlimited estimate of a large group) live in a
    // per-group HBM slab sized by the group's own pod count
    const bool grows = lds + sizeof(ChainRed) > 160 * 1024 || (knob_env("CASIM_CHAIN_GLOBAL") != nullptr);
    if (grows) {
        lds = 0;
        if (p->slab_max_nodes != lim->max_nodes) {
            std::vector<int64_t> off(G);
            std::vector<int32_t> kc(G);
            int64_t tot = 0;
            for (int32_t g = 0; g < G; g++) {
                const int32_t c = std::max(p->h_meta[g].count, 1);
                int32_t kg = lim->max_nodes > 0 ? std::min(lim->max_nodes, c) : c;
                kg = ((kg + 63) / 64) * 64;
                kc[g] = kg;
                off[g] = tot;
                tot += (int64_t)((chain_lds_bytes(kg, p->use_ports, p->use_scalar) + 255) & ~(size_t)255);
            }
            int rc;
            if ((rc = p->d_slab.reserve((size_t)std::max<int64_t>(tot, 256))) != CA_OK) return rc;
            if ((rc = p->d_slab_off.reserve(sizeof(int64_t) * (size_t)G)) != CA_OK) return rc;
            if ((rc = p->d_gkcap.reserve(sizeof(int32_t) * (size_t)G)) != CA_OK) return rc;
            CA_HIP_CHECK(hipMemcpy(p->d_slab_off.ptr, off.data(), sizeof(int64_t) * G, hipMemcpyHostToDevice));
            CA_HIP_CHECK(hipMemcpy(p->d_gkcap.ptr, kc.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice));
            p->slab_max_nodes = lim->max_nodes;
        }
    }
    // Zero-copy results: when the caller's sched_pod is page-locked (ca_host_alloc) and no
    // node ordinals are wanted, the chains publish straight into it (k_ffd_chain epilogue).
    // (Device-resident results could use the same publisher into the plan's own buffer;
    // measured on C2 it slows the chains more than k_copy_segments after them costs.)
    int32_t* publish = nullptr;
    if (to_host && !sched_node && p->total > 0 && (int64_t)G * p->nsub < INT32_MAX && !knob_env("CASIM_NO_PUBLISH")) {
        {
            hipPointerAttribute_t attr;
            const void* hp = sched16 ? (const void*)sched16 : (const void*)sched_pod;
            if (hipPointerGetAttributes(&attr, hp) == hipSuccess && attr.type == hipMemoryTypeHost &&
                attr.devicePointer != nullptr)
                publish = static_cast<int32_t*>(attr.devicePointer);
            else
                (void)hipGetLastError();
        }
    }
    // (no fill of the result buffers: k_copy_segments writes every output the chains do
    // not — run placements, and -1 past n_scheduled or for a failed group)
    const char* rb_env = knob_env("CASIM_RUN_BATCH");
    const int32_t batch_runs = (rb_env && rb_env[0] == '0') ? 0 : 1;
    const bool serial_pub = knob_env("CASIM_PUB_SERIAL") != nullptr;
    // (test hook: the publisher serialised in round 1 only — it gives up there, a later
    // lastIndex round publishes cleanly, and the fallback must still cover round 1's groups)
    const bool serial_pub_r1 = test_hook_env("CASIM_PUB_SERIAL_R1") != nullptr;
    int32_t tickets1 = 0;                               // publisher tickets of round 1 (every group)
    if (publish)
        for (int32_t g = 0; g < G; g++) tickets1 += (p->h_meta[g].count + p->pch - 1) / p->pch;
    // decoupled Go order (uniform classes, bucket path): chains on the stable order, Go's ids
    // beside them (CASIM_GO_DECOUPLE=0: the Go sort ahead of the stream, for tests)
    const bool go_order = go_sort_order();
    const bool decoupled = go_order && p->decouple_ok && p->total > 0 &&
                           !(knob_env("CASIM_GO_DECOUPLE") && atoi(knob_env("CASIM_GO_DECOUPLE")) == 0);
    p->ran_decoupled = decoupled ? 1 : 0;
    // Go's sort.Slice permutation of every group and its pod ids, on st3: its own class
    // ranks, k_pdq_sort, ids into d_spod_go and per-group ready flags holding this run's
    // epoch (no reset between runs; every run is synchronised before it returns).  The
    // chains meanwhile run on the stable class order (same class at every position).  It
    // is queued right after the heavy chains when the groups split (the heavy chains are the
    // step's critical path; the sort only bounds when the publisher can start and ends well
    // before them), else before anything else.
    // (the run's epoch is set before anything is queued: every consumer launched below reads it)
    if (decoupled) {
        if (p->ids_epoch == INT32_MAX) {                  // (wrapped: start over from a clean table)
            CA_HIP_CHECK(hipMemsetAsync(p->d_ids_ready.ptr, 0, sizeof(int32_t) * (size_t)G, p->st3));
            p->ids_epoch = 0;
        }
        p->ids_epoch++;
    }
    auto launch_go_sort = [&]() -> int {
        const int32_t U = p->s->n_cls;
        int32_t NP = 1;
        while (NP < U) NP <<= 1;
        // the class ranks inside the sort kernel when its LDS has room for the scratch
        const size_t npad = ((size_t)std::min(p->max_count, PDQ_LDS_N) + 63) & ~(size_t)63;
        const bool fold = 16 * (size_t)NP <= 3 * npad && 2 * (size_t)U <= npad / 8 && !knob_env("CASIM_NO_RANK_FOLD");
        if (!fold) {
            hipLaunchKernelGGL(k_class_rank, dim3(G), dim3(1024), 0, p->st3, p->d_meta.as<GroupMeta>(),
                               p->d_tmpl.as<ca_template>(), p->s->d_cls_sc.as<int64_t>(), U, NP,
                               p->d_crank2.as<int32_t>(), (const int32_t*)nullptr);
            CA_HIP_CHECK(hipGetLastError());
        }
        int rc0;
        if ((rc0 = launch_pdq_sort(p, p->st3, nullptr, G, p->d_crank2.as<int32_t>(), U, nullptr, 0,
                                   p->d_sortC.as<uint32_t>(), p->d_spod_go.as<int32_t>(),
                                   p->d_ids_ready.as<int32_t>(), p->ids_epoch, fold ? NP : 0)) != CA_OK)
            return rc0;
        st_mark(0);
        return CA_OK;
    };
    bool go_sort_queued = !decoupled;
    // (ev_ids is recorded on st3 once the heavy chains are queued: the host's launches ahead
    // of them pace the step's start)
    bool ids_recorded = !decoupled;
    auto record_ids = [&]() -> int {
        if (!ids_recorded) { CA_HIP_CHECK(hipEventRecord(p->ev_ids, p->st3)); ids_recorded = true; }
        return CA_OK;
    };
    if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_START], st));
    // decoupled: the stream from per-class counts (k_run_table) instead of the radix passes
    // and k_emit_bucket (CASIM_RUNS_STREAM=0: the radix path, for tests)
    const bool runs_stream = !(knob_env("CASIM_RUNS_STREAM") && atoi(knob_env("CASIM_RUNS_STREAM")) == 0);
    // round 1 without k_round_init: k_run_table sets each group's lastIndex / need /
    // unsupported flags, and the publisher's tickets and control words are clean from the
    // last run (ca_estimate_plan::pub_clean) — no launch and no cross-stream event ahead of
    // the chains
    const bool fast_init = decoupled && runs_stream && (!publish || p->pub_clean) && !serial_pub && !serial_pub_r1 &&
                           !knob_env("CASIM_NO_FAST_INIT");
    const int32_t lin0 = *last_index;
    if (publish) p->pub_clean = false;        // set again once this run's publishers all finished clean
    bool pub_gave_up = false;
    if (!fast_init) {
        const int32_t n = std::max(G, tickets1);
        hipLaunchKernelGGL(k_round_init, dim3(std::min((n + 255) / 256, 64)), dim3(256), 0, st, G, *last_index,
                           p->d_lin.as<int32_t>(), p->d_need.as<uint8_t>(), p->d_unsup.as<uint32_t>(),
                           publish ? p->d_tickets.as<int64_t>() : nullptr, tickets1,
                           publish ? p->d_qctl.as<int32_t>() : nullptr);
        CA_HIP_CHECK(hipGetLastError());
    }
    // heavy groups first (bucket path): see ca_estimate_plan::demand
    bool split = false;
    const int32_t* gmapA = nullptr;
    const int32_t* gmapB = nullptr;
    if (p->total > 0 && p->bucket && G >= 8 && !knob_env("CASIM_NO_SPLIT")) {
        // The heavy set: groups whose chain cost is within 60% of the largest, if that is
        // at most half the batch (a flat distribution gains nothing from the split).
        // First from the demand model, then once from the chain times the previous run
        // measured (ChainOut ticks) with the same max_nodes — a scheduling choice only:
        // every run computes everything.
        auto build_map = [&](const std::vector<double>& cost) -> int {
            double cmax = 0;
            for (int32_t g = 0; g < G; g++) cmax = std::max(cmax, cost[g]);
            std::vector<int32_t> map;
            map.reserve(G);
            for (int32_t g = 0; g < G; g++) if (cmax > 0 && cost[g] >= 0.6 * cmax) map.push_back(g);
            p->n_heavy = (int32_t)map.size() * 2 <= G ? (int32_t)map.size() : 0;
            for (int32_t g = 0; g < G; g++) if (!(cmax > 0 && cost[g] >= 0.6 * cmax)) map.push_back(g);
            int rc;
            if ((rc = p->d_gmap.reserve(sizeof(int32_t) * (size_t)G)) != CA_OK) return rc;
            CA_HIP_CHECK(hipMemcpy(p->d_gmap.ptr, map.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice));
            return CA_OK;
        };
        int rc;
        if (p->map_max_nodes != lim->max_nodes) {
            // chain length ~ the template copies a group opens over the runs it gets
            // through: `demand` below the limiter's cap, cap^2/demand above it (the
            // limiter stops the group after ~cap/demand of its pods)
            const double M = lim->max_nodes > 0 ? (double)lim->max_nodes : 0.0;
            std::vector<double> cost(G);
            for (int32_t g = 0; g < G; g++) {
                const double d = p->demand[g];
                cost[g] = (M > 0 && d > M) ? M * M / d : d;
            }
            if ((rc = build_map(cost)) != CA_OK) return rc;
            p->map_max_nodes = lim->max_nodes;
            p->map_source = 1;
        } else if (p->map_source == 1 && (int32_t)p->diag.size() == G) {
            std::vector<double> cost(G);
            for (int32_t g = 0; g < G; g++) cost[g] = (double)(uint32_t)(p->diag[g] & 0xFFFFFFFFull);
            if ((rc = build_map(cost)) != CA_OK) return rc;
            p->map_source = 2;
        }
        split = p->n_heavy > 0 && p->n_heavy < G;
        gmapA = p->d_gmap.as<int32_t>();
        gmapB = gmapA + p->n_heavy;
    }
    const int32_t nA = split ? p->n_heavy : G, nB = split ? G - p->n_heavy : 0;
    const bool sort_after_heavy = split && p->total > 0 && p->bucket && !knob_env("CASIM_SORT_FIRST");
    if (!go_sort_queued && !sort_after_heavy) {
        int rcs;
        if ((rcs = launch_go_sort()) != CA_OK) return rcs;
        go_sort_queued = true;
    }
    // where the consumers (publisher, segment copies) read the stream's pod ids
    const int32_t* const ids_src = decoupled ? p->d_spod_go.as<int32_t>() : p->d_spod.as<int32_t>();
    std::function<int()> sort_light;        // split: the light groups' sort, queued after the heavy chains
    // 1-3: score, sort, stream
    if (p->total > 0 && p->bucket) {
        const int32_t U = p->s->n_cls;
        int32_t NP = 1;
        while (NP < U) NP <<= 1;
        int32_t* crank = p->d_crank.as<int32_t>();
        const int32_t* pcls = p->s->d_cls.as<int32_t>();
        int32_t nb = 1, passes = 0;                       // buckets <= U: 8-bit digits
        while (nb < U) { nb <<= 8; passes++; }
        passes = std::max(passes, 1);
        const int32_t passes_run = (go_order && !decoupled) ? 0 : passes;
        const int32_t blocks = (p->max_count + 255) / 256;
        // class ranks, then Go's pdqsort (default) or the stable LSD radix passes, stream
        // emission for `ng` groups (map `gm`)
        // (by value: the light groups' call runs after this block's locals are gone)
        auto sort_groups = [=](hipStream_t ss, const int32_t* gm, int32_t ng, bool events) -> int {
            if (decoupled && runs_stream) {
                // the stream from per-class counts (no sort of the pod lists; the class ranks
                // are computed inside k_run_table)
                if (events && p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_SCORE], ss));
                hipLaunchKernelGGL(k_run_table, dim3(ng), dim3(1024), 0, ss, p->d_meta.as<GroupMeta>(),
                                   p->d_item_cls.as<int32_t>(), p->s->d_cls_sc.as<int64_t>(), NP,
                                   p->s->d_cls_rep.as<int32_t>(), U,
                                   p->d_tmpl.as<ca_template>(), p->s->t.hot.as<PodHot>(), p->s->t.spec.as<ca_pod_spec>(),
                                   p->s->t.terms.as<ca_selector_term>(), p->s->t.reqs.as<ca_selector_req>(),
                                   p->d_rstart.as<int32_t>(), p->d_rsp.as<StreamPod>(), p->d_unsup.as<uint32_t>(), gm,
                                   fast_init ? p->d_lin.as<int32_t>() : nullptr, p->d_need.as<uint8_t>(), lin0);
                CA_HIP_CHECK(hipGetLastError());
                hipLaunchKernelGGL(k_emit_runs, dim3(blocks, ng), dim3(256), 0, ss, p->d_meta.as<GroupMeta>(),
                                   p->d_rstart.as<int32_t>(), p->d_rsp.as<StreamPod>(), U, p->d_stream.as<StreamPod>(),
                                   p->d_heads.as<uint64_t>(), gm, batch_runs ? 0 : 1);
                CA_HIP_CHECK(hipGetLastError());
                if (events && p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_MERGE], ss));
                return CA_OK;
            }
            hipLaunchKernelGGL(k_class_rank, dim3(ng), dim3(1024), 0, ss, p->d_meta.as<GroupMeta>(),
                               p->d_tmpl.as<ca_template>(), p->s->d_cls_sc.as<int64_t>(), U, NP, crank, gm);
            CA_HIP_CHECK(hipGetLastError());
            if (events && p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_SCORE], ss));
            uint32_t* a = nullptr;                        // identity (position order)
            uint32_t* bufs[2] = {p->d_sortA.as<uint32_t>(), p->d_sortB.as<uint32_t>()};
            if (go_order && !decoupled) {
                int rc0;
                if ((rc0 = launch_pdq_sort(p, ss, gm, ng, crank, U, nullptr)) != CA_OK) return rc0;
                a = bufs[0];
            }
            for (int ps = 0; ps < passes_run; ps++) {
                uint32_t* b = bufs[ps & 1];
                hipLaunchKernelGGL(k_radix_hist, dim3(p->max_rtiles, ng), dim3(RTHREADS), 0, ss, p->d_meta.as<GroupMeta>(),
                                   a, p->d_pod_idx.as<int32_t>(), pcls, crank, U, 8 * ps, p->d_hist.as<int32_t>(), gm);
                CA_HIP_CHECK(hipGetLastError());
                hipLaunchKernelGGL(k_radix_scan, dim3(ng), dim3(256), 0, ss, p->d_meta.as<GroupMeta>(),
                                   p->d_hist.as<int32_t>(), gm);
                CA_HIP_CHECK(hipGetLastError());
                hipLaunchKernelGGL(k_radix_scatter, dim3(p->max_rtiles, ng), dim3(RTHREADS), 0, ss,
                                   p->d_meta.as<GroupMeta>(), a, p->d_pod_idx.as<int32_t>(), pcls, crank, U, 8 * ps,
                                   p->d_hist.as<int32_t>(), b, gm);
                CA_HIP_CHECK(hipGetLastError());
                a = b;
            }
            if (events && p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_MERGE], ss));
            hipLaunchKernelGGL(k_emit_bucket, dim3(blocks, ng), dim3(256), 0, ss, p->d_meta.as<GroupMeta>(), a,
                               p->d_pod_idx.as<int32_t>(), p->d_tmpl.as<ca_template>(), p->s->t.hot.as<PodHot>(),
                               p->s->t.spec.as<ca_pod_spec>(), p->s->t.terms.as<ca_selector_term>(),
                               p->s->t.reqs.as<ca_selector_req>(), p->d_stream.as<StreamPod>(), p->d_spod.as<int32_t>(),
                               p->d_heads.as<uint64_t>(), p->d_unsup.as<uint32_t>(), gm);
            CA_HIP_CHECK(hipGetLastError());
            return CA_OK;
        };
        int rc;
        if (split) {     // the light groups are sorted right after the heavy chains are queued
            // (fast_init: nothing of k_round_init to wait for)
            if (!fast_init) CA_HIP_CHECK(hipEventRecord(p->ev_init, st));
            if ((rc = sort_groups(st, gmapA, nA, true)) != CA_OK) return rc;
            sort_light = [=]() -> int {
                if (!fast_init) CA_HIP_CHECK(hipStreamWaitEvent(p->st2, p->ev_init, 0));
                return sort_groups(p->st2, gmapB, nB, false);
            };
        } else if ((rc = sort_groups(st, nullptr, G, true)) != CA_OK) {
            return rc;
        }
    } else if (p->total > 0) {
        const int32_t tiles = (p->max_count + TILE - 1) / TILE;
        hipLaunchKernelGGL(k_score_tiles, dim3(tiles, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(),
                           p->d_pod_idx.as<int32_t>(), p->d_tmpl.as<ca_template>(), p->s->t.hot.as<PodHot>(),
                           p->s->t.spec.as<ca_pod_spec>(), p->s->t.terms.as<ca_selector_term>(),
                           p->s->t.reqs.as<ca_selector_req>(), p->d_sortA.as<SortItem>(), p->d_unsup.as<uint32_t>());
        CA_HIP_CHECK(hipGetLastError());
        if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_SCORE], st));
        SortItem* a = p->d_sortA.as<SortItem>();
        SortItem* b = p->d_sortB.as<SortItem>();
        const int32_t blocks = (p->max_count + 255) / 256;
        for (int32_t w = TILE; w < p->max_count; w *= 2) {
            hipLaunchKernelGGL(k_merge_runs, dim3(blocks, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(), a, b, w);
            CA_HIP_CHECK(hipGetLastError());
            std::swap(a, b);
        }
        if (go_order) {
            // dense ranks from the comparison sort, then sort.Slice's permutation of them
            hipLaunchKernelGGL(k_item_rank, dim3(G), dim3(1024), 0, st, p->d_meta.as<GroupMeta>(), a,
                               p->d_item_rank.as<uint32_t>());
            CA_HIP_CHECK(hipGetLastError());
            int rc0;
            if ((rc0 = launch_pdq_sort(p, st, nullptr, G, nullptr, 0, p->d_item_rank.as<uint32_t>())) != CA_OK)
                return rc0;
        }
        if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_MERGE], st));
        if (go_order) {
            hipLaunchKernelGGL(k_emit_bucket, dim3(blocks, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(),
                               p->d_sortA.as<uint32_t>(), p->d_pod_idx.as<int32_t>(), p->d_tmpl.as<ca_template>(),
                               p->s->t.hot.as<PodHot>(), p->s->t.spec.as<ca_pod_spec>(),
                               p->s->t.terms.as<ca_selector_term>(), p->s->t.reqs.as<ca_selector_req>(),
                               p->d_stream.as<StreamPod>(), p->d_spod.as<int32_t>(), p->d_heads.as<uint64_t>(),
                               p->d_unsup.as<uint32_t>(), nullptr);
        } else {
            hipLaunchKernelGGL(k_emit_stream, dim3(blocks, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(), a,
                               p->d_pod_idx.as<int32_t>(), p->s->t.hot.as<PodHot>(), p->d_stream.as<StreamPod>(),
                               p->d_spod.as<int32_t>(), p->d_heads.as<uint64_t>());
        }
        CA_HIP_CHECK(hipGetLastError());
    }
    if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_EMIT], st));
    // 4-5: chains with lastIndex speculation
    std::vector<int32_t> lin(G, *last_index);
    std::vector<uint8_t> need(G, 1);
    std::vector<ChainOut> outs(G);
    std::vector<uint8_t> accepted(G, 0);
    std::vector<int32_t> true_lin(G, *last_index);
    int32_t cut = -1;                   // first unsupported group when later groups exist (prefix protocol)
    // the host joins the streams itself (publisher, heavy and light chains) instead of
    // queueing cross-stream waits ahead of the readback event on st
    const bool host_joins = publish && !p->phase_events;
    bool light_pending = false;
    int32_t rounds = 0;
    float chain_ms = 0;
    {
        int32_t* hq = p->h_qc.as<int32_t>();     // host-side failure flags ([2] per round, [3] sticky)
        hq[2] = hq[3] = 0;
    }
    for (;;) {
        rounds++;
        if (rounds > 1) p->h_qc.as<int32_t>()[2] = 0;
        const bool serial_now = serial_pub || (serial_pub_r1 && rounds == 1);
        if (rounds > 1) {      // round 1's state came from k_round_init
            CA_HIP_CHECK(hipMemcpyAsync(p->d_lin.ptr, lin.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
            CA_HIP_CHECK(hipMemcpyAsync(p->d_need.ptr, need.data(), G, hipMemcpyHostToDevice, st));
        }
        int32_t round_tickets = 0;
        // the publisher's start: after the ticket reset (k_round_init, or the memsets of a
        // later round); round 1 of a split run reuses ev_init (recorded right after
        // k_round_init), so no marker sits between the heavy stream and its chains
        hipEvent_t pub_go = p->ev_go;
        if (publish) {
            for (int32_t g = 0; g < G; g++) if (need[g]) round_tickets += (p->h_meta[g].count + p->pch - 1) / p->pch;
            if (rounds > 1) {
                CA_HIP_CHECK(hipStreamWaitEvent(st, p->ev_pub, 0));   // previous publisher done
                CA_HIP_CHECK(hipMemsetAsync(p->d_tickets.ptr, 0xFF, sizeof(int64_t) * (size_t)std::max(round_tickets, 1), st));
                CA_HIP_CHECK(hipMemsetAsync(p->d_qctl.ptr, 0, sizeof(int32_t) * 3, st));   // [3] stays: sticky
                CA_HIP_CHECK(hipMemsetAsync(p->d_qctl.as<int32_t>() + 4, 0, sizeof(int32_t) * 2, st));
            }
            if (rounds == 1 && fast_init) pub_go = nullptr;       // the tickets are clean already
            else if (rounds == 1 && split) pub_go = p->ev_init;
            else CA_HIP_CHECK(hipEventRecord(p->ev_go, st));
        }
        // CASIM_PUB_SERIAL (tests): the publisher goes first on the chains' own stream, i.e.
        // the two kernels are serialised — it must give up at its start deadline
        auto launch_pub = [&](hipStream_t ps) -> int {
            if (sched16)
                hipLaunchKernelGGL(k_publish<uint16_t>, dim3(std::min(round_tickets, pub_blocks(decoupled))), dim3(256), 0, ps,
                                   p->d_meta.as<GroupMeta>(), p->d_out.as<ChainOut>(), p->d_seg.as<Seg>(),
                                   ids_src, p->d_sched_pod.as<int32_t>(), p->d_tickets.as<int64_t>(),
                                   p->d_qctl.as<int32_t>(), round_tickets, p->nsub, p->d_prog.as<int2>(), p->pch,
                                   reinterpret_cast<uint16_t*>(publish), pub_start_ticks(),
                                   decoupled ? p->d_ids_ready.as<int32_t>() : nullptr, p->ids_epoch, p->h_qc.as<int32_t>());
            else
                hipLaunchKernelGGL(k_publish<int32_t>, dim3(std::min(round_tickets, pub_blocks(decoupled))), dim3(256), 0, ps,
                                   p->d_meta.as<GroupMeta>(), p->d_out.as<ChainOut>(), p->d_seg.as<Seg>(),
                                   ids_src, p->d_sched_pod.as<int32_t>(), p->d_tickets.as<int64_t>(),
                                   p->d_qctl.as<int32_t>(), round_tickets, p->nsub, p->d_prog.as<int2>(), p->pch,
                                   publish, pub_start_ticks(), decoupled ? p->d_ids_ready.as<int32_t>() : nullptr, p->ids_epoch,
                                   p->h_qc.as<int32_t>());
            CA_HIP_CHECK(hipGetLastError());
            return CA_OK;
        };
        if (publish && round_tickets > 0 && serial_now) {
            int rc0;
            if ((rc0 = launch_pub(st)) != CA_OK) return rc0;
            CA_HIP_CHECK(hipEventRecord(p->ev_pub, st));
        }
        if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_CHAIN0], st));
        const bool ps = p->use_ports || p->use_scalar;
        auto chain_kernel = grows ? (ps ? k_ffd_chain<true, true> : k_ffd_chain<true, false>)
                                  : (ps ? k_ffd_chain<false, true> : k_ffd_chain<false, false>);
        if (!grows) {
            int rcl;
            if ((rcl = ensure_dyn_lds((const void*)chain_kernel, lds)) != CA_OK) return rcl;
        }
        auto chain = [&](hipStream_t ss, const int32_t* gm, int32_t ng) -> int {
            hipLaunchKernelGGL(chain_kernel, dim3(ng), dim3(CT), lds, ss,
                               p->d_meta.as<GroupMeta>(),
                               p->d_stream.as<StreamPod>(), p->d_heads.as<uint64_t>(), p->d_tmpl.as<ca_template>(),
                               p->s->t.spec.as<ca_pod_spec>(), p->s->t.hot.as<PodHot>(), p->d_lin.as<int32_t>(),
                               p->d_need.as<uint8_t>(), p->d_unsup.as<uint32_t>(), n_base, lim->max_nodes, kcap,
                               p->use_ports ? 1 : 0, p->use_scalar ? 1 : 0, batch_runs,
                               p->d_sched_pod.as<int32_t>(), sched_node ? p->d_sched_node.as<int32_t>() : nullptr,
                               p->d_seg.as<Seg>(), publish ? p->d_tickets.as<int64_t>() : nullptr,
                               p->d_qctl.as<int32_t>(), p->nsub, p->d_prog.as<int2>(), p->pch, p->d_out.as<ChainOut>(),
                               gm, grows ? p->d_slab.as<unsigned char>() : nullptr,
                               grows ? p->d_slab_off.as<int64_t>() : nullptr, grows ? p->d_gkcap.as<int32_t>() : nullptr,
                               decoupled ? 1 : 0, p->h_out.as<ChainOut>(), p->h_qc.as<int32_t>());
            CA_HIP_CHECK(hipGetLastError());
            return CA_OK;
        };
        int rc;
        if (rounds == 1 && split) {         // heavy groups on st as soon as their sort is done
            if ((rc = chain(st, gmapA, nA)) != CA_OK) return rc;
            if (!go_sort_queued) {
                if ((rc = launch_go_sort()) != CA_OK) return rc;
                go_sort_queued = true;
            }
            if ((rc = record_ids()) != CA_OK) return rc;
            if ((rc = sort_light()) != CA_OK) return rc;
            if ((rc = chain(p->st2, gmapB, nB)) != CA_OK) return rc;
            CA_HIP_CHECK(hipEventRecord(p->ev_b, p->st2));
            // (publishing without phase events the host waits for ev_b itself: one
            // cross-stream hop less between the last chain and the host)
            if (!host_joins) CA_HIP_CHECK(hipStreamWaitEvent(st, p->ev_b, 0));
            light_pending = host_joins;
        } else if ((rc = chain(st, nullptr, G)) != CA_OK) {
            return rc;
        }
        if (!go_sort_queued) {             // (a later round of a split run: queued in round 1)
            if ((rc = launch_go_sort()) != CA_OK) return rc;
            go_sort_queued = true;
        }
        if ((rc = record_ids()) != CA_OK) return rc;
        if (publish && round_tickets > 0 && !serial_now) {
            if (pub_go) CA_HIP_CHECK(hipStreamWaitEvent(p->pub_stream, pub_go, 0));
            if ((rc = launch_pub(p->pub_stream)) != CA_OK) return rc;
            CA_HIP_CHECK(hipEventRecord(p->ev_pub, p->pub_stream));
        }
        if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_CHAIN1], st));
        // one readback per round: the chain outputs, and (publishing) the publisher's
        // counters once it is done — the results are then already in the caller's buffer
        // (the chains write their ChainOut records, and the chains / publisher their failure
        // flags, straight into page-locked h_out / h_qc: no copy kernels at the step's end)
        const ChainOut* fresh = p->h_out.as<ChainOut>();
        const bool pub_ran = publish && round_tickets > 0 && !serial_now;
        if (publish && !(host_joins && pub_ran)) CA_HIP_CHECK(hipStreamWaitEvent(st, p->ev_pub, 0));
        CA_HIP_CHECK(hipEventRecord(p->ev_rb, st));
        // results of this round, queued behind the readback: the device fills them while
        // the host walks the lastIndex chain (a later round queues them again)
        if (p->total > 0 && !publish && !decoupled) {
            hipLaunchKernelGGL(k_copy_segments, dim3((p->max_count + CPY_PER_BLOCK - 1) / CPY_PER_BLOCK, G), dim3(256), 0,
                               st, p->d_meta.as<GroupMeta>(), p->d_out.as<ChainOut>(), p->d_seg.as<Seg>(),
                               p->d_spod.as<int32_t>(), p->d_sched_pod.as<int32_t>(),
                               sched_node ? p->d_sched_node.as<int32_t>() : nullptr, 0);
            CA_HIP_CHECK(hipGetLastError());
        }
        if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_COMPACT], st));
        // (polling the events with hipEventQuery instead measured the same: 0.486 ms)
        if (rounds == 1) st_mark(1);
        if (host_joins && pub_ran) CA_HIP_CHECK(hipEventSynchronize(p->ev_pub));   // (finishes last)
        CA_HIP_CHECK(hipEventSynchronize(p->ev_rb));
        if (light_pending) { CA_HIP_CHECK(hipEventSynchronize(p->ev_b)); light_pending = false; }
        if (rounds == 1) st_mark(2);
        if (publish && p->h_qc.as<int32_t>()[2] != 0) pub_gave_up = true;
        float ms = 0;
        if (p->phase_events)
            (void)hipEventElapsedTime(&ms, p->ev[ca_estimate_plan::EV_CHAIN0], p->ev[ca_estimate_plan::EV_CHAIN1]);
        chain_ms += ms;
        for (int32_t g = 0; g < G; g++) if (need[g]) outs[g] = fresh[g];
        if (rounds == 1) {
            p->diag.resize(G);
            for (int32_t g = 0; g < G; g++) p->diag[g] = fresh[g].pad;
        }
        // walk the lastIndex chain
        int64_t cur = *last_index;
        cut = -1;
        bool known = true;
        bool all_ok = true;
        std::fill(need.begin(), need.end(), 0);
        for (int32_t g = 0; g < G; g++) {
            const ChainOut& o = outs[g];
            true_lin[g] = (int32_t)cur;     // exact once the walk converged (known stays true)
            if (o.status == CA_EUNSUPPORTED && known) {
                // prefix protocol (casim.h scope): groups after it are CA_ENOTRUN, the batch's
                // lastIndex is the one this group starts from
                for (int32_t h = g; h < G; h++) { accepted[h] = 1; need[h] = 0; }
                if (g + 1 < G) cut = g;
                break;
            }
            const bool insensitive = o.status != CA_OK || !o.sensitive;
            if (known && (o.lin == cur || insensitive)) {
                accepted[g] = 1;
                if (o.status == CA_OK && o.had_success) cur = o.lout;
                continue;
            }
            if (!known && insensitive) {
                accepted[g] = 1;                         // result independent of lastIndex
                if (o.status == CA_OK && o.had_success) { cur = o.lout; known = true; }
                continue;
            }
            // sensitive group run from a wrong lastIndex: re-run from the best guess
            accepted[g] = 0;
            all_ok = false;
            need[g] = 1;
            lin[g] = (int32_t)cur;
            if (known) {
                known = false;   // this group's output is unknown until it re-runs
            }
            // speculate: the stale output is the guess for the successors
            cur = o.had_success ? o.lout : cur;
        }
        if (all_ok) {
            *last_index = (int32_t)cur;
            break;
        }
        if (rounds > G + 2) { set_last_error("estimate speculation did not converge"); return CA_EDEVICE; }
    }
    // results: the chains wrote single placements directly, the last round's
    // k_copy_segments the run placements (or the publisher, into the caller's buffer)
    if (decoupled && !publish && p->total > 0) {
        // once, after the last round: stream positions -> Go-order ids
        CA_HIP_CHECK(hipStreamWaitEvent(st, p->ev_ids, 0));
        hipLaunchKernelGGL(k_copy_segments, dim3((p->max_count + CPY_PER_BLOCK - 1) / CPY_PER_BLOCK, G), dim3(256), 0,
                           st, p->d_meta.as<GroupMeta>(), p->d_out.as<ChainOut>(), p->d_seg.as<Seg>(),
                           ids_src, p->d_sched_pod.as<int32_t>(),
                           sched_node ? p->d_sched_node.as<int32_t>() : nullptr, 1);
        CA_HIP_CHECK(hipGetLastError());
    }
    if (publish) {
        p->pub_clean = !pub_gave_up;
        // the publisher of the last round wrote the results; a deadline hit (a chain that
        // died) falls back to the device copy + D2H
        const int32_t* qc = p->h_qc.as<int32_t>();      // read back with the last round's outputs
        p->pub_state = 1;
        // (a give-up in ANY round: qc[2] is reset per round and a later round publishes only
        // the groups it re-ran, so round 1's accepted groups would otherwise stay unwritten)
        if (pub_gave_up || qc[2] != 0 || qc[3] != 0) {
            p->pub_state = 2;
            set_last_error("estimate publisher missed a ticket; results copied instead");
            if (decoupled) CA_HIP_CHECK(hipStreamWaitEvent(st, p->ev_ids, 0));
            hipLaunchKernelGGL(k_copy_segments, dim3((p->max_count + CPY_PER_BLOCK - 1) / CPY_PER_BLOCK, G), dim3(256), 0,
                               st, p->d_meta.as<GroupMeta>(), p->d_out.as<ChainOut>(), p->d_seg.as<Seg>(),
                               ids_src, p->d_sched_pod.as<int32_t>(), nullptr, decoupled ? 1 : 0);
            CA_HIP_CHECK(hipGetLastError());
            int rc;
            if (to_host && (rc = results_to_host(p, st, sched_pod, sched16)) != CA_OK) return rc;
        }
    } else if (to_host) {
        int rc;
        if ((rc = results_to_host(p, st, sched_pod, sched16)) != CA_OK) return rc;
    }
    if (sched_node)
        CA_HIP_CHECK(hipMemcpyAsync(sched_node, p->d_sched_node.ptr, sizeof(int32_t) * std::max(p->total, 0),
                                    hipMemcpyDeviceToHost, st));
    if (p->phase_events) CA_HIP_CHECK(hipEventRecord(p->ev[ca_estimate_plan::EV_D2H], st));
    // (published with the host joining the streams: the round's event already covered
    // everything queued on st, nothing was queued since)
    if (!(host_joins && p->pub_state == 1)) CA_HIP_CHECK(hipStreamSynchronize(st));
    for (int32_t g = 0; g < G; g++) {
        const ChainOut& o = outs[g];
        ca_estimate_result& r = results[g];
        r.node_count = o.node_count;
        r.n_scheduled = o.n_sched;
        r.nodes_added = o.nodes_added;
        r.last_index_in = true_lin[g];
        r.last_index_out = o.status == CA_OK && o.had_success ? o.lout : true_lin[g];
        r.status = o.status;
        r.evals = o.evals;
        if (cut >= 0 && g > cut) {        // CA_ENOTRUN: nothing of it is reported
            r.node_count = r.n_scheduled = r.nodes_added = 0;
            r.last_index_in = r.last_index_out = true_lin[cut];
            r.status = CA_ENOTRUN;
            r.evals = 0;
        }
    }
    float sort_ms = 0;
    {
        using P = ca_estimate_plan;
        auto el = [&](int a, int b) {
            float v = 0;
            if (p->phase_events) (void)hipEventElapsedTime(&v, p->ev[a], p->ev[b]);
            return v;
        };
        const bool any = p->total > 0;
        p->t_ms[0] = any ? el(P::EV_START, P::EV_SCORE) : 0;
        p->t_ms[1] = any ? el(P::EV_SCORE, P::EV_MERGE) : 0;
        p->t_ms[2] = any ? el(P::EV_MERGE, P::EV_EMIT) : 0;
        p->t_ms[3] = chain_ms;
        p->t_ms[4] = el(P::EV_CHAIN1, P::EV_COMPACT);
        p->t_ms[5] = el(P::EV_COMPACT, P::EV_D2H);
        sort_ms = el(P::EV_START, P::EV_EMIT);
    }
    p->grp_succ.assign((size_t)G, 0);
    for (int32_t g = 0; g < G; g++)
        p->grp_succ[g] = outs[g].status == CA_OK && outs[g].had_success && !(cut >= 0 && g > cut) ? 1 : 0;
    // batch-level lastIndex dependence: the first group with a FitsAnyNode success decides
    p->stats.lin_sensitive = 0;
    p->stats.had_success = 0;
    for (int32_t g = 0; g < G; g++) {
        const ChainOut& o = outs[g];
        if (o.status != CA_OK || !o.had_success) continue;
        p->stats.lin_sensitive = o.sensitive;
        p->stats.had_success = 1;
        break;
    }
    p->stats.rounds = rounds;
    p->stats.kernel_ms = chain_ms;
    p->stats.sort_ms = sort_ms;
    p->stats.total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    p->t_ms[6] = p->stats.total_ms;
    if (step_timing) {
        const auto t_exit = std::chrono::steady_clock::now();
        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::micro>(b - a).count();
        };
        st_acc[0] += us(t_start, st_t[0]);
        st_acc[1] += us(st_t[0], st_t[1]);
        st_acc[2] += us(st_t[1], st_t[2]);
        st_acc[3] += us(st_t[2], t_exit);
        if (st_n > 0) st_acc[4] += us(st_last_exit, t_start);
        st_acc[5] += us(t_start, t_exit);
        st_last_exit = t_exit;
        if (++st_n == 20) {
            fprintf(stderr, "[step] us per call: to the sort launch %.1f, to the last launch %.1f, join wait %.1f, "
                    "to the return %.1f, caller between calls %.1f, call %.1f\n", st_acc[0] / 20, st_acc[1] / 20,
                    st_acc[2] / 20, st_acc[3] / 20, st_acc[4] / 19, st_acc[5] / 20);
            for (double& v : st_acc) v = 0;
            st_n = 0;
        }
    }
    return CA_OK;
}

}  // namespace

// Results of the plan's last run re-based to another input lastIndex, for a batch that is
// not lastIndex-sensitive (its outputs are the same from any input: multi.hip).  Returns
// the batch's output lastIndex from `lin`.
namespace casim {
int32_t estimate_plan_rebase(const ca_estimate_plan* p, ca_estimate_result* results, int32_t lin) {
    int32_t cur = lin;
    for (int32_t g = 0; g < p->G; g++) {
        ca_estimate_result& r = results[g];
        r.last_index_in = cur;
        if (r.status == CA_OK && g < (int32_t)p->grp_succ.size() && p->grp_succ[g]) cur = r.last_index_out;
        else r.last_index_out = cur;
    }
    return cur;
}
}  // namespace casim

extern "C" {

int ca_estimate_plan_rebase(const ca_estimate_plan* p, ca_estimate_result* results, int32_t last_index_in,
                            int32_t* last_index_out) {
    if (!p || (p->G > 0 && !results)) return CA_EINVAL;
    const int32_t lout = casim::estimate_plan_rebase(p, results, last_index_in);
    if (last_index_out) *last_index_out = lout;
    return CA_OK;
}

int ca_estimate_plan_create(ca_mirror* m, const ca_podset* s, const int32_t* group_off, const int32_t* pod_idx,
                            const ca_template* templates, int32_t n_groups, ca_estimate_plan** out) {
    if (!m || !s || !group_off || !out || n_groups < 0 || (n_groups > 0 && !templates)) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    ca_estimate_plan* p = new ca_estimate_plan();
    int rc = plan_prepare(p, m, s, group_off, pod_idx, templates, n_groups);
    if (rc != CA_OK) { delete p; return rc; }
    *out = p;
    return CA_OK;
}

int ca_estimate_plan_fetch(const ca_estimate_plan* p, int32_t* sched_pod) {
    if (!p || !sched_pod) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(p->m->device));
    if (p->total > 0)
        CA_HIP_CHECK(hipMemcpy(sched_pod, p->d_sched_pod.ptr, sizeof(int32_t) * (size_t)p->total, hipMemcpyDeviceToHost));
    return CA_OK;
}

int ca_estimate_plan_device_results(const ca_estimate_plan* p, const int32_t** sched_pod_dev) {
    if (!p || !sched_pod_dev) return CA_EINVAL;
    *sched_pod_dev = p->d_sched_pod.as<int32_t>();
    return CA_OK;
}

int ca_estimate_plan_run(ca_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                         ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node) {
    if (!p) return CA_EINVAL;
    return plan_run(p, limiter, last_index, results, sched_pod, sched_node);
}

int ca_estimate_plan_run_u16(ca_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                             ca_estimate_result* results, uint16_t* sched_pod16) {
    if (!p || !sched_pod16) return CA_EINVAL;
    return plan_run(p, limiter, last_index, results, nullptr, nullptr, sched_pod16);
}

int ca_estimate_plan_destroy(ca_estimate_plan* p) {
    if (!p) return CA_EINVAL;
    delete p;
    return CA_OK;
}

int ca_estimate_plan_stats(const ca_estimate_plan* p, int32_t* rounds, float* chain_ms, float* sort_ms, float* total_ms) {
    if (!p) return CA_EINVAL;
    if (rounds) *rounds = p->stats.rounds;
    if (chain_ms) *chain_ms = p->stats.kernel_ms;
    if (sort_ms) *sort_ms = p->stats.sort_ms;
    if (total_ms) *total_ms = p->stats.total_ms;
    return CA_OK;
}

int ca_estimate_plan_timings(const ca_estimate_plan* p, float* out, int32_t cap) {
    if (!p || (cap > 0 && !out)) return CA_EINVAL;
    const int32_t n = 9;
    for (int32_t i = 0; i < 7 && i < cap; i++) out[i] = p->t_ms[i];
    if (cap > 7) out[7] = (float)p->pub_state;
    if (cap > 8) out[8] = (float)p->ran_decoupled;
    return n;
}

int ca_estimate_plan_set_phase_timing(ca_estimate_plan* p, int32_t on) {
    if (!p) return CA_EINVAL;
    p->phase_events = on != 0;
    return CA_OK;
}

int ca_estimate_plan_group_ticks(const ca_estimate_plan* p, uint64_t* out, int32_t cap) {
    if (!p || (cap > 0 && !out)) return CA_EINVAL;
    const int32_t n = (int32_t)p->diag.size();
    for (int32_t i = 0; i < n && i < cap; i++) out[i] = p->diag[i];
    return n;
}

int ca_estimate_plan_chain_info(const ca_estimate_plan* p, int32_t* lin_sensitive, int32_t* had_success) {
    if (!p) return CA_EINVAL;
    if (lin_sensitive) *lin_sensitive = p->stats.lin_sensitive;
    if (had_success) *had_success = p->stats.had_success;
    return CA_OK;
}

int ca_estimate_batch(ca_mirror* m, const ca_podset* s, const int32_t* group_off, const int32_t* pod_idx,
                      const ca_template* templates, int32_t n_groups, const ca_limiter* limiter, int32_t* last_index,
                      ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node) {
    ca_estimate_plan* p = nullptr;
    int rc = ca_estimate_plan_create(m, s, group_off, pod_idx, templates, n_groups, &p);
    if (rc != CA_OK) return rc;
    rc = ca_estimate_plan_run(p, limiter, last_index, results, sched_pod, sched_node);
    ca_estimate_plan_destroy(p);
    return rc;
}

int ca_go_sort_ranks(int32_t device, const uint32_t* ranks, int32_t n, int32_t store, int32_t limit, int32_t* perm) {
    if (n < 0 || (n > 0 && (!ranks || !perm)) || store < 0 || store > 3) return CA_EINVAL;
    if (n == 0) return CA_OK;
    CA_HIP_CHECK(hipSetDevice(device));
    DevBuf meta, rk, sorted, e, scr, stack;
    int rc;
    if ((rc = meta.reserve(sizeof(GroupMeta))) != CA_OK || (rc = rk.reserve(sizeof(uint32_t) * (size_t)n)) != CA_OK ||
        (rc = sorted.reserve(sizeof(uint32_t) * (size_t)n)) != CA_OK ||
        (rc = e.reserve(sizeof(uint64_t) * (size_t)n)) != CA_OK || (rc = scr.reserve(sizeof(uint64_t) * (size_t)n)) != CA_OK ||
        (rc = stack.reserve(sizeof(pdq::Frame) * ((size_t)n / 2 + 4))) != CA_OK)
        return rc;
    GroupMeta gm = {};
    gm.off = 0;
    gm.count = n;
    CA_HIP_CHECK(hipMemcpy(meta.ptr, &gm, sizeof(gm), hipMemcpyHostToDevice));
    CA_HIP_CHECK(hipMemcpy(rk.ptr, ranks, sizeof(uint32_t) * (size_t)n, hipMemcpyHostToDevice));
    const int32_t lds_n = std::min(n, PDQ_LDS_N);
    const size_t lds = pdq_lds_bytes(lds_n);
    if ((rc = ensure_dyn_lds((const void*)k_pdq_sort, lds)) != CA_OK) return rc;
    hipLaunchKernelGGL(k_pdq_sort, dim3(1), dim3(pdq::NT), lds, 0, meta.as<GroupMeta>(), nullptr, nullptr, nullptr, 0,
                       rk.as<uint32_t>(), sorted.as<uint32_t>(), e.as<uint64_t>(), scr.as<uint64_t>(),
                       stack.as<pdq::Frame>(), lds_n, store, std::max(limit, 0), nullptr, nullptr, nullptr, 0,
                       (const int32_t*)nullptr, (const ca_template*)nullptr, (const int64_t*)nullptr, 0);
    CA_HIP_CHECK(hipGetLastError());
    CA_HIP_CHECK(hipMemcpy(perm, sorted.ptr, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost));
    return CA_OK;
}

#ifdef CASIM_PROF
int ca_debug_pdq_prof(uint64_t* out, int32_t reset) {
    CA_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(pdq::g_pdq_prof), sizeof(uint64_t) * (32 + 256)));
    CA_HIP_CHECK(hipMemcpyFromSymbol(out + 32 + 256, HIP_SYMBOL(pdq::g_pdq_pis), sizeof(uint64_t) * 8));
    CA_HIP_CHECK(hipMemcpyFromSymbol(out + 32 + 256 + 8, HIP_SYMBOL(pdq::g_pdq_wg), sizeof(uint64_t) * 3 * 128));
    if (reset) {
        static const uint64_t z[32 + 256] = {};
        CA_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(pdq::g_pdq_prof), z, sizeof z));
        CA_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(pdq::g_pdq_pis), z, sizeof(uint64_t) * 8));
    }
    return CA_OK;
}

int ca_debug_chain_prof(uint64_t* out, int32_t n_groups) {
    if (n_groups > 1024) n_groups = 1024;
    CA_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_prof), sizeof(uint64_t) * NPROF * (size_t)n_groups));
    return CA_OK;
}
int ca_debug_rt_prof(uint64_t* out, int32_t n_groups) {     // k_run_table phases: 4 per group
    if (n_groups > 1024) n_groups = 1024;
    CA_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_prof), sizeof(uint64_t) * 4 * (size_t)n_groups));
    return CA_OK;
}
#endif

}  // extern "C"
