// estimate.hip — BinpackingNodeEstimator.Estimate for a batch of node groups.
//
// Reference: CA/estimator/binpacking_estimator.go:65-193,
//            CA/estimator/threshold_based_limiter.go:27-64,
//            CA/utils/scheduler/scheduler.go:73-91 (template copies),
//            CA/simulator/predicatechecker/schedulerbased.go:90-136 (rotating scan).
//
// Pipeline per call:
//   1. k_score_tiles   score (float64, calculatePodScore) + static predicates of every
//                      (group, pod) against the group's template; bitonic sort of
//                      1024-item tiles in LDS by (score desc, list position asc).
//   2. k_merge_runs    log2(P/1024) merge passes (rank by binary search; keys unique).
//   3. k_emit_stream   gather the sorted pods into a 32-B/pod stream per group.
//   4. k_ffd_chain     one wavefront per group runs the sequential First-Fit-Decreasing
//                      loop with the new-node rows in LDS; the rotating first-fit is a
//                      64-lane ballot over block summaries, then over the block's nodes.
//   5. host fix-up     the groups share lastIndex: groups whose result
//                      depends on their lastIndex input are re-run until every group's
//                      input equals its predecessor's output (exact).
#include "mirror.h"
#include "device_filters.h"

#include <cstring>
#include <algorithm>
#include <chrono>

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
    SF_UNSUP   = 0x80u,  // PF_HOSTNAME_DEP: group unsupported
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
    uint32_t flags;   // SF_*
};
static_assert(sizeof(StreamPod) == 32, "StreamPod");

struct alignas(16) GroupMeta {
    int64_t tcpu, tmem, teph;      // template free (alloc - template pods)
    int32_t tpods;                 // template free pod slots
    int32_t off;                   // offset into the pod lists / streams
    int32_t count;                 // pods in the group
    int32_t tmpl;                  // template index
    uint32_t tflags;               // NF_* of the template
    int32_t pad;
};

struct alignas(16) ChainOut {
    int32_t node_count, n_sched, nodes_added, lin;
    int32_t lout, status, sensitive, had_success;
    uint64_t evals;
    uint64_t pad;
};
static_assert(sizeof(ChainOut) == 48, "ChainOut");

constexpr int TILE = 1024;

__device__ inline uint64_t ordered_bits(double d) {
    if (d == 0.0) d = 0.0;   // -0 == +0 for the comparator (binpacking_estimator.go:74)
    uint64_t u = (uint64_t)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__device__ inline bool item_less(const SortItem& a, const SortItem& b) {
    return a.key < b.key || (a.key == b.key && a.pos < b.pos);
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
            uint32_t sf = 0;
            const bool pre_fail = (p.flags & PF_PREFILTER_FAIL) != 0;
            bool static_ok = true;
            const bool need_static = (p.flags & (PF_NODE_NAME | PF_AFFINITY)) ||
                                     (tp.node.taints & ~s.tolerated_taints);
            if (need_static) {
                NodeStatic ns;
                ns.taints = tp.node.taints;
                for (int w = 0; w < CA_LABEL_WORDS; w++) ns.labels[w] = tp.node.label_pairs[w];
                ns.keys = tp.node.label_keys;
                for (int k = 0; k < CA_MAX_INT_KEYS; k++) ns.ints[k] = tp.node.int_label[k];
                ns.int_valid = tp.node.int_label_valid;
                ns.name_id = tp.node.name_id;
                static_ok = dev_static_filters(s, p.flags, terms, reqs, ns, false) == CA_PLUGIN_NONE;
            }
            if (!pre_fail && !tunsched) sf |= SF_EVAL;                           // schedulerbased.go:125
            if ((sf & SF_EVAL) && static_ok) sf |= SF_FA_OK;
            if (!pre_fail) sf |= SF_CP_EVAL;
            if (!pre_fail && (!tunsched || (p.flags & PF_TOL_UNSCHED)) && static_ok) sf |= SF_CP_OK;
            if (p.flags & PF_ALL_ZERO) sf |= SF_ZERO;
            if (p.flags & PF_SCALAR_REQ) sf |= SF_SCALAR;
            if (p.flags & PF_PORTS) sf |= SF_PORTS;
            if (p.flags & PF_HOSTNAME_DEP) { sf |= SF_UNSUP; unsup = 1; }
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

// 3. gather the stream ---------------------------------------------------------
__global__ void __launch_bounds__(256) k_emit_stream(const GroupMeta* __restrict__ groups, const SortItem* __restrict__ src,
                                                    const int32_t* __restrict__ pod_idx, const PodHot* __restrict__ ph,
                                                    StreamPod* __restrict__ out) {
    const GroupMeta gm = groups[blockIdx.y];
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= gm.count) return;
    const SortItem it = src[gm.off + i];
    const int32_t pidx = pod_idx[gm.off + (int32_t)it.pos];
    const PodHot p = ph[pidx];
    StreamPod sp;
    sp.cpu = p.cpu; sp.mem = p.mem; sp.eph = p.eph;
    sp.pod = pidx;
    sp.flags = it.flags;
    out[gm.off + i] = sp;
}

// 4. the First-Fit-Decreasing chain -------------------------------------------
__device__ inline int64_t rl64(int64_t v, int lane) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline int32_t rl32(int32_t v, int lane) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, lane); }

__device__ inline int64_t wave_max64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t x = __shfl_xor(v, o, 64);
        v = x > v ? x : v;
    }
    return v;
}
__device__ inline int32_t wave_max32(int32_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t x = __shfl_xor(v, o, 64);
        v = x > v ? x : v;
    }
    return v;
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

// One wavefront per node group.  LDS: NodeRec rows[kcap], block summaries[kcap/64]
// (per-dimension maxima over a 64-row block, allowed to be stale-high), and the
// optional port / scalar columns.
__global__ void __launch_bounds__(64) k_ffd_chain(
    const GroupMeta* __restrict__ groups, const StreamPod* __restrict__ stream, const ca_template* __restrict__ tmpls,
    const ca_pod_spec* __restrict__ specs, const PodHot* __restrict__ ph, const int32_t* __restrict__ lin_arr,
    const uint8_t* __restrict__ need, const uint32_t* __restrict__ group_unsup, int32_t n_base, int32_t max_nodes,
    int32_t kcap, int32_t use_ports, int32_t use_scalar, int32_t* __restrict__ sched_pod,
    int32_t* __restrict__ sched_node, ChainOut* __restrict__ outs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int g = blockIdx.x;
    if (!need[g]) return;
    const int lane = threadIdx.x;
    const GroupMeta gm = groups[g];
    const int32_t lin = lin_arr[g];
    ChainOut res;
    res.node_count = 0; res.n_sched = 0; res.nodes_added = 0; res.lin = lin; res.lout = lin;
    res.status = CA_OK; res.sensitive = 0; res.had_success = 0; res.evals = 0; res.pad = 0;
    if (group_unsup[g]) {
        res.status = CA_EUNSUPPORTED;
        if (lane == 0) outs[g] = res;
        return;
    }
    const int nb_cap = (kcap + 63) >> 6;
    NodeRec* R = reinterpret_cast<NodeRec*>(smem_raw);
    NodeRec* SUM = R + kcap;
    uint64_t* PORTS = reinterpret_cast<uint64_t*>(SUM + nb_cap);               // [kcap][CA_PORT_WORDS]
    int64_t* SC = reinterpret_cast<int64_t*>(PORTS + (use_ports ? (size_t)CA_PORT_WORDS * kcap : 0));  // [8][kcap]

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
    // Stream double buffer: lane l holds entry (window + l) in `cur` and (window + 64 + l)
    // in `nxt`; the next window is requested 64 steps before it is read.  Outputs are
    // kept in lanes (lane i = i-th placement of the window) and stored once per window,
    // before the prefetch, so no step waits on a store (vmcnt counts both).
    StreamPod cur = {}, nxt = {};
    if (lane < P) cur = gs[lane];
    if (64 + lane < P) nxt = gs[64 + lane];
    int32_t out_pod = -1, out_node = -1;
    int32_t flushed = 0;         // placements already stored

    for (int32_t step = 0; step < P; step++) {
        const int sl = step & 63;
        if (sl == 0 && step > 0) {
            const int32_t pend = nsched - flushed;
            if (lane < pend) {
                sched_pod[gm.off + flushed + lane] = out_pod;
                if (sched_node) sched_node[gm.off + flushed + lane] = out_node;
            }
            flushed = nsched;
            cur = nxt;
            if (step + 64 + lane < P) nxt = gs[step + 64 + lane];
        }
        const int64_t pcpu = rl64(cur.cpu, sl), pmem = rl64(cur.mem, sl), peph = rl64(cur.eph, sl);
        const int32_t pidx = rl32(cur.pod, sl);
        const uint32_t sf = (uint32_t)rl32((int32_t)cur.flags, sl);
        const bool zero = (sf & SF_ZERO) != 0;

        // rare per-pod data (ports / scalars) from the full record
        uint64_t pconf[CA_PORT_WORDS] = {0, 0}, puse[CA_PORT_WORDS] = {0, 0};
        int64_t psc[CA_MAX_SCALAR];
        for (int i = 0; i < CA_MAX_SCALAR; i++) psc[i] = 0;
        if (sf & (SF_PORTS | SF_SCALAR)) {
            const ca_pod_spec& s = specs[ph[pidx].spec];
            for (int w = 0; w < CA_PORT_WORDS; w++) { pconf[w] = s.port_conflict[w]; puse[w] = s.port_use[w]; }
            for (int i = 0; i < CA_MAX_SCALAR; i++) psc[i] = s.req_scalar[i];
        }

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
                        if (sf & SF_SCALAR) {
                            for (int i = 0; i < CA_MAX_SCALAR; i++)
                                fit = fit & !((psc[i] != 0) & (j < k) && psc[i] > SC[(size_t)i * kcap + (j < k ? j : 0)]);
                        }
                        if (sf & SF_PORTS) {
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
                            if (lane == 0) {
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
                    if (!first_success) { first_success = true; sensitive = k >= 2; }
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
            // addNewNodeToSnapshot: a template copy (:146-159)
            const int32_t nn = k;
            if (lane == 0) {
                R[nn] = trec;
                SUM[nn >> 6] = trec;   // a fresh copy is the largest a row can be
            }
            if (use_ports && lane < CA_PORT_WORDS) PORTS[(size_t)nn * CA_PORT_WORDS + lane] = tp.used_ports[lane];
            if (use_scalar && lane < CA_MAX_SCALAR)
                SC[(size_t)lane * kcap + nn] = wsub(tp.node.alloc_scalar[lane], tp.used_scalar[lane]);
            k++;
            last_node = nn;
            // CheckPredicates(pod, newNode) (:132-134)
            if (sf & SF_CP_EVAL) evals++;
            bool ok = (sf & SF_CP_OK) != 0;
            if (ok) {
                ok = rec_fits(trec, pcpu, pmem, peph, zero);
                if (ok && (sf & SF_SCALAR)) {
                    for (int i = 0; i < CA_MAX_SCALAR; i++)
                        if (psc[i] != 0 && psc[i] > wsub(tp.node.alloc_scalar[i], tp.used_scalar[i])) ok = false;
                }
                if (ok && (sf & SF_PORTS)) {
                    uint64_t c = 0;
                    for (int w = 0; w < CA_PORT_WORDS; w++) c |= tp.used_ports[w] & pconf[w];
                    ok = c == 0;
                }
            }
            if (!ok) continue;
            found = nn;
        }
        // AddPod(pod, node) (:96 / :135) — NodeInfo.update on the new-node row
        if (lane == 0) {
            NodeRec r = R[found];
            r.cpu = wsub(r.cpu, pcpu);
            r.mem = wsub(r.mem, pmem);
            r.eph = wsub(r.eph, peph);
            r.pods -= 1;
            r.used = 1;
            R[found] = r;
        }
        if (lane == nsched - flushed) { out_pod = pidx; out_node = found; }
        if (sf & SF_SCALAR) {
            if (lane < CA_MAX_SCALAR) {
                const size_t ix = (size_t)lane * kcap + found;
                SC[ix] = wsub(SC[ix], psc[lane]);
            }
        }
        if (sf & SF_PORTS) {
            if (lane < CA_PORT_WORDS) PORTS[(size_t)found * CA_PORT_WORDS + lane] |= puse[lane];
        }
        nsched++;
        __builtin_amdgcn_wave_barrier();
    }
    {
        const int32_t pend = nsched - flushed;
        if (lane < pend) {
            sched_pod[gm.off + flushed + lane] = out_pod;
            if (sched_node) sched_node[gm.off + flushed + lane] = out_node;
        }
    }
    // newNodesWithPods
    int32_t cnt = 0;
    for (int32_t j = lane; j < k; j += 64) cnt += R[j].used;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) {
        res.node_count = cnt;
        res.n_sched = nsched;
        res.nodes_added = k;
        res.lout = L;
        res.sensitive = sensitive ? 1 : 0;
        res.had_success = first_success ? 1 : 0;
        res.evals = evals;
        outs[g] = res;
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
    DevBuf d_meta, d_pod_idx, d_tmpl, d_sortA, d_sortB, d_stream, d_unsup, d_lin, d_need, d_out, d_sched_pod,
        d_sched_node;
    Stats stats;
};

namespace {

int plan_prepare(ca_estimate_plan* p, ca_mirror* m, const ca_podset* s, const int32_t* group_off,
                 const int32_t* pod_idx, const ca_template* templates, int32_t G) {
    p->m = m; p->s = s; p->G = G;
    p->h_off.assign(group_off, group_off + G + 1);
    p->h_tmpl.assign(templates, templates + G);
    p->total = group_off[G] - group_off[0];
    if (group_off[0] != 0) return CA_EINVAL;
    p->h_meta.resize(G);
    p->max_count = 0;
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
        gm.pad = 0;
        p->max_count = std::max(p->max_count, c);
        for (int w = 0; w < CA_PORT_WORDS; w++) if (t.used_ports[w]) p->use_ports = true;
        for (int i = 0; i < CA_MAX_SCALAR; i++)
            if (t.node.alloc_scalar[i] || t.used_scalar[i]) p->use_scalar = true;
    }
    for (int32_t i = 0; i < p->total; i++) {
        const int32_t pi = pod_idx[i];
        if (pi < 0 || pi >= s->t.n_pods) return CA_EINVAL;
        const uint32_t f = pod_dev_flags(s->h_pods[pi]);
        if (f & PF_PORTS) p->use_ports = true;
        if (f & PF_SCALAR_REQ) p->use_scalar = true;
    }
    hipStream_t st = m->stream;
    int rc;
    const size_t tot = (size_t)std::max(p->total, 1);
    if ((rc = p->d_meta.reserve(sizeof(GroupMeta) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_pod_idx.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
    if ((rc = p->d_tmpl.reserve(sizeof(ca_template) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_sortA.reserve(sizeof(SortItem) * tot)) != CA_OK) return rc;
    if ((rc = p->d_sortB.reserve(sizeof(SortItem) * tot)) != CA_OK) return rc;
    if ((rc = p->d_stream.reserve(sizeof(StreamPod) * tot)) != CA_OK) return rc;
    if ((rc = p->d_unsup.reserve(sizeof(uint32_t) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_lin.reserve(sizeof(int32_t) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_need.reserve((size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_out.reserve(sizeof(ChainOut) * (size_t)std::max(G, 1))) != CA_OK) return rc;
    if ((rc = p->d_sched_pod.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
    if ((rc = p->d_sched_node.reserve(sizeof(int32_t) * tot)) != CA_OK) return rc;
    if (G) CA_HIP_CHECK(hipMemcpyAsync(p->d_meta.ptr, p->h_meta.data(), sizeof(GroupMeta) * G, hipMemcpyHostToDevice, st));
    if (p->total) CA_HIP_CHECK(hipMemcpyAsync(p->d_pod_idx.ptr, pod_idx, sizeof(int32_t) * p->total, hipMemcpyHostToDevice, st));
    if (G) CA_HIP_CHECK(hipMemcpyAsync(p->d_tmpl.ptr, templates, sizeof(ca_template) * G, hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipStreamSynchronize(st));
    return CA_OK;
}

size_t chain_lds_bytes(int32_t kcap, bool use_ports, bool use_scalar) {
    const size_t nb = (size_t)((kcap + 63) >> 6);
    size_t b = 32 * ((size_t)kcap + nb);
    if (use_ports) b += 8 * CA_PORT_WORDS * (size_t)kcap;
    if (use_scalar) b += 8 * CA_MAX_SCALAR * (size_t)kcap;
    return (b + 15) & ~(size_t)15;
}

int plan_run(ca_estimate_plan* p, const ca_limiter* lim, int32_t* last_index, ca_estimate_result* results,
             int32_t* sched_pod, int32_t* sched_node) {
    ca_mirror* m = p->m;
    hipStream_t st = m->stream;
    const int32_t G = p->G;
    if (!lim || !last_index || !results || !sched_pod) return CA_EINVAL;
    const auto t_start = std::chrono::steady_clock::now();
    CA_HIP_CHECK(hipSetDevice(m->device));
    const int32_t n_base = (int32_t)m->nodes.size();
    if (G == 0) return CA_OK;
    // kcap: new nodes a group can add (limiter cap, or one per pod when unlimited)
    int32_t kcap = lim->max_nodes > 0 ? std::min(lim->max_nodes, std::max(p->max_count, 1)) : std::max(p->max_count, 1);
    kcap = ((kcap + 63) / 64) * 64;
    const size_t lds = chain_lds_bytes(kcap, p->use_ports, p->use_scalar);
    if (lds > 160 * 1024) return CA_EUNSUPPORTED;   // HBM-backed variant is future work
    CA_HIP_CHECK(hipMemsetAsync(p->d_unsup.ptr, 0, sizeof(uint32_t) * G, st));
    if (p->total > 0) {   // entries past n_scheduled read back as -1
        CA_HIP_CHECK(hipMemsetAsync(p->d_sched_pod.ptr, 0xFF, sizeof(int32_t) * p->total, st));
        CA_HIP_CHECK(hipMemsetAsync(p->d_sched_node.ptr, 0xFF, sizeof(int32_t) * p->total, st));
    }
    CA_HIP_CHECK(hipEventRecord(m->ev0, st));
    // 1-3: score, sort, stream
    if (p->total > 0) {
        const int32_t tiles = (p->max_count + TILE - 1) / TILE;
        hipLaunchKernelGGL(k_score_tiles, dim3(tiles, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(),
                           p->d_pod_idx.as<int32_t>(), p->d_tmpl.as<ca_template>(), p->s->t.hot.as<PodHot>(),
                           p->s->t.spec.as<ca_pod_spec>(), p->s->t.terms.as<ca_selector_term>(),
                           p->s->t.reqs.as<ca_selector_req>(), p->d_sortA.as<SortItem>(), p->d_unsup.as<uint32_t>());
        CA_HIP_CHECK(hipGetLastError());
        SortItem* a = p->d_sortA.as<SortItem>();
        SortItem* b = p->d_sortB.as<SortItem>();
        const int32_t blocks = (p->max_count + 255) / 256;
        for (int32_t w = TILE; w < p->max_count; w *= 2) {
            hipLaunchKernelGGL(k_merge_runs, dim3(blocks, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(), a, b, w);
            CA_HIP_CHECK(hipGetLastError());
            std::swap(a, b);
        }
        hipLaunchKernelGGL(k_emit_stream, dim3(blocks, G), dim3(256), 0, st, p->d_meta.as<GroupMeta>(), a,
                           p->d_pod_idx.as<int32_t>(), p->s->t.hot.as<PodHot>(), p->d_stream.as<StreamPod>());
        CA_HIP_CHECK(hipGetLastError());
    }
    CA_HIP_CHECK(hipEventRecord(m->ev1, st));
    // 4-5: chains with lastIndex speculation
    std::vector<int32_t> lin(G, *last_index);
    std::vector<uint8_t> need(G, 1);
    std::vector<ChainOut> outs(G);
    std::vector<uint8_t> accepted(G, 0);
    std::vector<int32_t> true_lin(G, *last_index);
    int32_t rounds = 0;
    float chain_ms = 0;
    for (;;) {
        rounds++;
        CA_HIP_CHECK(hipMemcpyAsync(p->d_lin.ptr, lin.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipMemcpyAsync(p->d_need.ptr, need.data(), G, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipEventRecord(m->ev2, st));
        CA_HIP_CHECK(hipFuncSetAttribute((const void*)k_ffd_chain, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k_ffd_chain, dim3(G), dim3(64), lds, st, p->d_meta.as<GroupMeta>(),
                           p->d_stream.as<StreamPod>(), p->d_tmpl.as<ca_template>(), p->s->t.spec.as<ca_pod_spec>(),
                           p->s->t.hot.as<PodHot>(), p->d_lin.as<int32_t>(), p->d_need.as<uint8_t>(),
                           p->d_unsup.as<uint32_t>(), n_base, lim->max_nodes, kcap, p->use_ports ? 1 : 0,
                           p->use_scalar ? 1 : 0, p->d_sched_pod.as<int32_t>(), p->d_sched_node.as<int32_t>(),
                           p->d_out.as<ChainOut>());
        CA_HIP_CHECK(hipGetLastError());
        hipEvent_t evc;
        CA_HIP_CHECK(hipEventCreate(&evc));
        CA_HIP_CHECK(hipEventRecord(evc, st));
        std::vector<ChainOut> fresh(G);
        CA_HIP_CHECK(hipMemcpyAsync(fresh.data(), p->d_out.ptr, sizeof(ChainOut) * G, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipStreamSynchronize(st));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, m->ev2, evc);
        (void)hipEventDestroy(evc);
        chain_ms += ms;
        for (int32_t g = 0; g < G; g++) if (need[g]) outs[g] = fresh[g];
        // walk the lastIndex chain
        int64_t cur = *last_index;
        bool known = true;
        bool all_ok = true;
        std::fill(need.begin(), need.end(), 0);
        for (int32_t g = 0; g < G; g++) {
            const ChainOut& o = outs[g];
            true_lin[g] = (int32_t)cur;     // exact once the walk converged (known stays true)
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
    // results
    CA_HIP_CHECK(hipMemcpyAsync(sched_pod, p->d_sched_pod.ptr, sizeof(int32_t) * std::max(p->total, 0),
                                hipMemcpyDeviceToHost, st));
    if (sched_node)
        CA_HIP_CHECK(hipMemcpyAsync(sched_node, p->d_sched_node.ptr, sizeof(int32_t) * std::max(p->total, 0),
                                    hipMemcpyDeviceToHost, st));
    CA_HIP_CHECK(hipStreamSynchronize(st));
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
    }
    float sort_ms = 0;
    (void)hipEventElapsedTime(&sort_ms, m->ev0, m->ev1);
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
    return CA_OK;
}

}  // namespace

extern "C" {

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

int ca_estimate_plan_run(ca_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                         ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node) {
    if (!p) return CA_EINVAL;
    return plan_run(p, limiter, last_index, results, sched_pod, sched_node);
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

}  // extern "C"
