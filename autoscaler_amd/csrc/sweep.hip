// sweep.hip — RemovalSimulator.FindNodesToRemove, legacy semantics (canPersist=false).
//
// Reference: CA/simulator/cluster.go:116-254 (FindNodesToRemove, SimulateNodeRemoval,
// withForkedSnapshot, findPlaceFor), CA/simulator/scheduling/hinting_simulator.go:58-125
// (TrySchedulePods, hints), CA/utils/tpu/tpu.go:57-79 (ClearTPURequests).
//
// Every candidate is simulated on a fork that is reverted afterwards, so candidates
// share no snapshot state; the only coupling is the checker's lastIndex.
// Two kernels:
//   k_sweep_table  one wavefront per candidate, one lastIndex per LANE: lane w runs the
//                  candidate from L = window_start + w and reports where lastIndex ends.
//                  The host composes these 64-wide tables along the candidate order to
//                  find every candidate's exact input lastIndex (re-centring the windows
//                  that missed).
//   k_sweep        one wavefront per candidate at its exact lastIndex: 64-node chunks of
//                  the rotating scan with an LDS overlay of the candidate's placements;
//                  produces every output (removable, destinations, hints, evals).
#include "mirror.h"
#include "device_filters.h"

#include <cstring>
#include <cstdlib>
#include <algorithm>
#include <chrono>

namespace casim {

constexpr int OV_CAP = CA_MAX_MOVED_PODS;   // distinct destination nodes per candidate (k_sweep)
constexpr int TB_MAXP = 128;    // moved pods per candidate handled by k_sweep_table
constexpr int TB_SCAN = 512;    // per-lane scan bound in k_sweep_table (longer: exact kernel)
constexpr int32_t TB_UNKNOWN = -1;

struct alignas(16) SweepOut {
    int32_t removable, reason, n_placed, lin;
    int32_t lout, fa_success, status, pad;
    uint64_t evals;
    uint64_t pad2;
};
static_assert(sizeof(SweepOut) == 48, "SweepOut");

struct OverlaySmem {
    int32_t node[OV_CAP];
    int32_t pods[OV_CAP];
    int64_t cpu[OV_CAP], mem[OV_CAP], eph[OV_CAP];
};
// port / extended-resource overlay columns: dynamic LDS, only when some pod of the
// mirror has host ports or extended requests (keeps 4 KB of LDS per block otherwise)
struct OverlayExt {
    uint64_t ports[OV_CAP][CA_PORT_WORDS];
    int64_t scalar[OV_CAP][CA_MAX_SCALAR];
};

__device__ inline int64_t rl64s(int64_t v, int lane) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline int32_t rl32s(int32_t v, int lane) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, lane); }
__device__ inline uint64_t lanes_below_u(int lane) { return lane == 0 ? 0ull : (~0ull >> (64 - lane)); }
extern "C" __device__ long long __ockl_wfred_add_i64(long long);

// moved-pod semantics: Spec.NodeName cleared (cluster.go:235-240), TPU requests
// cleared (tpu.go:57-79)
__device__ inline uint32_t moved_flags(uint32_t f) {
    uint32_t m = f & ~(PF_NODE_NAME | PF_ALL_ZERO | PF_SCALAR_REQ | PF_HAS_SCALAR_KEYS);
    if (f & PF_MOVED_ALL_ZERO) m |= PF_ALL_ZERO;
    if (f & PF_MOVED_SCALAR_REQ) m |= PF_SCALAR_REQ;
    if (f & PF_NONTPU_SCALAR) m |= PF_HAS_SCALAR_KEYS;
    return m;
}

// Resource part of NodeResourcesFit on a row, branch-free (fit.go:256-300).
__device__ inline bool hot_fits(const PodHot& p, const NodeHot& h) {
    const bool res = (p.cpu <= h.cpu) & (p.mem <= h.mem) & (p.eph <= h.eph);
    return (h.pods >= 1) & (((p.flags & PF_ALL_ZERO) != 0) | res);
}

// Per 64-node block of the ring: the largest free cpu / memory / ephemeral storage / pod
// slots over its visible nodes (destination, schedulable) and their bit mask.  A pod that
// fails the maxima fits no node of the block, so a scan passes the block without reading
// its rows and counts its visible nodes from the mask (tight clusters: the planner's later
// windows, RunOnce, where most scans cross long runs of full nodes).  Built per sweep call
// (the destination mask is an input of the call).
struct alignas(8) BlockSum {
    int64_t cpu, mem, eph;
    uint64_t vis;
    int32_t pods, pad;
};
static_assert(sizeof(BlockSum) == 40, "BlockSum");

__device__ inline bool block_may_fit(const PodHot& p, const BlockSum& b) {
    const bool res = (p.cpu <= b.cpu) & (p.mem <= b.mem) & (p.eph <= b.eph);
    return (b.vis != 0) & (b.pods >= 1) & (((p.flags & PF_ALL_ZERO) != 0) | res);
}

// visible nodes of block b in lanes [lo, hi), the candidate's node excluded
__device__ inline int32_t block_vis(const BlockSum& b, int32_t blk, int lo, int hi, int32_t node) {
    uint64_t m = b.vis;
    if (hi < 64) m &= (1ull << hi) - 1;
    m &= ~0ull << lo;
    if ((node >> 6) == blk) m &= ~(1ull << (node & 63));
    return __popcll(m);
}

__device__ inline int64_t wave_max_i64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

__global__ void __launch_bounds__(64) k_block_sum(const NodeHot* __restrict__ hot, const uint8_t* __restrict__ dest_mask,
                                                 int32_t n, BlockSum* __restrict__ bsum) {
    const int32_t j = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t pos = j * 64 + lane;
    bool v = false;
    NodeHot h = {};
    if (pos < n) {
        h = hot[pos];
        v = dest_mask[pos] != 0 && !(h.flags & NF_UNSCHED);
    }
    const uint64_t vm = __ballot(v);
    const int64_t lo = INT64_MIN;
    const int64_t c = wave_max_i64(v ? h.cpu : lo);
    const int64_t m = wave_max_i64(v ? h.mem : lo);
    const int64_t e = wave_max_i64(v ? h.eph : lo);
    const int64_t p = wave_max_i64(v ? (int64_t)h.pods : lo);
    if (lane == 0) {
        BlockSum b;
        b.cpu = c; b.mem = m; b.eph = e; b.vis = vm;
        b.pods = vm ? (int32_t)p : 0;
        b.pad = 0;
        bsum[j] = b;
    }
}

// Full filter chain on a (possibly overlay-adjusted) row; per lane.
__device__ inline bool eval_node(const ca_pod_spec& s, const PodHot& p, const int64_t* psc,
                                 const ca_selector_term* terms, const ca_selector_req* reqs,
                                 const NodeHot& h, const NodeExt& e, const NodeStatic* st_row, bool apply_unsched) {
    if (apply_unsched && (h.flags & NF_UNSCHED) && !(p.flags & PF_TOL_UNSCHED)) return false;
    const bool need_static = (p.flags & (PF_NODE_NAME | PF_AFFINITY)) ||
                             ((h.flags & NF_TAINTS) && !(p.flags & PF_TAINT_MASK_ALL));
    if (need_static) {
        const NodeStatic ns = *st_row;
        if (dev_static_filters(s, p.flags, terms, reqs, ns, false) != CA_PLUGIN_NONE) return false;
    }
    if (p.flags & PF_PORTS) {
        uint64_t c = 0;
        for (int w = 0; w < CA_PORT_WORDS; w++) c |= e.ports[w] & s.port_conflict[w];
        if (c) return false;
    }
    return dev_fit_reasons(p.cpu, p.mem, p.eph, p.flags, psc, h.cpu, h.mem, h.eph, h.pods, e.scalar) == 0;
}

// static filters only where the pod needs them (taints / affinity / names)
__device__ inline bool static_ok(const ca_pod_spec& s, const PodHot& p, const ca_selector_term* terms,
                                 const ca_selector_req* reqs, const NodeHot& h, const NodeStatic* st_row) {
    const bool need_static = (p.flags & (PF_NODE_NAME | PF_AFFINITY)) ||
                             ((h.flags & NF_TAINTS) && !(p.flags & PF_TAINT_MASK_ALL));
    if (!need_static) return true;
    const NodeStatic ns = *st_row;
    return dev_static_filters(s, p.flags, terms, reqs, ns, false) == CA_PLUGIN_NONE;
}

__device__ inline bool in_prefilter(const ca_pod_spec& s, const int32_t* names, int32_t name_id) {
    bool ok = false;
    for (int32_t k = 0; k < s.prefilter_count; k++) ok |= names[s.prefilter_first + k] == name_id;
    return ok;
}

// ---------------------------------------------------------------------------
// exact kernel: one wavefront per candidate at its exact lastIndex
// ---------------------------------------------------------------------------
// Occupancy: the sweep runs one wavefront per candidate (C3: 5 000) and each candidate is a
// latency-bound chain, so the kernel time is (rounds of resident waves) x (chain time);
// CASIM_SWEEP_WAVES bounds the VGPRs so more waves are resident per SIMD.
#ifndef CASIM_SWEEP_WAVES
#define CASIM_SWEEP_WAVES 4
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(CASIM_SWEEP_WAVES, 8))) k_sweep(
    const NodeHot* __restrict__ hot, const NodeExt* __restrict__ ext, const NodeStatic* __restrict__ st, int32_t n,
    const uint8_t* __restrict__ dest_mask, const int32_t* __restrict__ cands, const int32_t* __restrict__ cand_status,
    const int32_t* __restrict__ move_off, const int32_t* __restrict__ move_pods, const PodHot* __restrict__ ph,
    const ca_pod_spec* __restrict__ specs, const ca_selector_term* __restrict__ terms,
    const ca_selector_req* __restrict__ reqs, const int32_t* __restrict__ names, const int32_t* __restrict__ hints,
    const int32_t* __restrict__ lin_arr, const uint8_t* __restrict__ need, int32_t* __restrict__ out_dest,
    int32_t* __restrict__ hint_set, SweepOut* __restrict__ outs, int32_t* __restrict__ walk_lout, int32_t use_ext,
    const BlockSum* __restrict__ bsum, const int32_t* __restrict__ chain_list, int32_t n_chain,
    int32_t* __restrict__ chain) {
    __shared__ OverlaySmem ov;
    extern __shared__ __attribute__((aligned(16))) unsigned char ovx_raw[];
    OverlayExt& ox = *reinterpret_cast<OverlayExt*>(ovx_raw);
    // chain != null (the host walk's serial exact chain): one workgroup runs the candidates
    // chain_list[0..n_chain) in order, each from the lastIndex the previous one left (*chain
    // in and out), with the node rows warm in its XCD's L2 from one candidate to the next
    int32_t chain_v = chain ? *chain : 0;
    for (int32_t it = 0; it < (chain ? n_chain : 1); it++) {
    const int c = chain ? chain_list[it] : (int)blockIdx.x;
    if (!chain && !need[c]) continue;
    const uint64_t t_begin = wall_clock64();      // diagnostics: SweepOut.pad2 = device ticks (100 MHz)
    const int lane = threadIdx.x;
    const int32_t lin = chain ? chain_v : lin_arr[c];
    SweepOut res;
    res.removable = 0; res.reason = CA_UNREMOVABLE_NONE; res.n_placed = 0; res.lin = lin; res.lout = lin;
    res.fa_success = 0; res.status = CA_OK; res.pad = 0; res.evals = 0; res.pad2 = 0;
    const int32_t node = cands[c];
    const int32_t mo = move_off[c], mn = move_off[c + 1] - mo;
    if (node < 0 || node >= n || !dest_mask[node]) {                          // cluster.go:157-160
        for (int32_t i = lane; i < mn; i += 64) { out_dest[mo + i] = -1; hint_set[mo + i] = -1; }
        res.reason = CA_UNREMOVABLE_UNEXPECTED_ERROR;
        if (lane == 0) { outs[c] = res; walk_lout[c] = -1; }
        continue;
    }
    if (cand_status[c] != 0) {                                                 // :162-169
        for (int32_t i = lane; i < mn; i += 64) { out_dest[mo + i] = -1; hint_set[mo + i] = -1; }
        res.reason = cand_status[c];
        if (lane == 0) { outs[c] = res; walk_lout[c] = -1; }
        continue;
    }
    int32_t npl = 0;          // overlay entries
    int32_t L = lin;
    if (n > 0 && L >= n) L = (int32_t)((uint32_t)L % (uint32_t)n);
    uint64_t evals = 0;
    bool fa_success = false;
    int32_t placed = 0;
    bool failed = false;
    // lane i holds moved pod (batch + i): id, record, hint; outputs kept in lanes and
    // stored once per batch (no per-pod store for a later load to wait behind)
    int32_t my_id = -1, my_hint = -1, my_dest = -1, my_hset = -1;
    bool own_ok = false;          // the moved pods' request sums (hints to the candidate itself)
    int64_t own_c = 0, own_m = 0, own_e = 0;
    PodHot my_p = {};
    NodeHot my_hh = {};           // the hinted node's row, prefetched with the batch
    uint8_t my_hdm = 0;

    const int32_t nb = (n + 63) >> 6;
    // register block cache: raw hot row, base visibility, overlay delta per lane
    int32_t ja = -1, jb = -1;
    NodeHot Ah = {}, Bh = {};
    bool Avis = false, Bvis = false;
    int64_t Adc = 0, Adm = 0, Ade = 0, Bdc = 0, Bdm = 0, Bde = 0;
    int32_t Adp = 0, Bdp = 0;
    auto load_block = [&](int32_t j, NodeHot& h, bool& vis, int64_t& dc, int64_t& dmm, int64_t& de, int32_t& dp) {
        const int32_t pos = j * 64 + lane;
        const bool valid = pos < n;
        h = NodeHot{};
        uint8_t dm = 0;
        if (valid) { h = hot[pos]; dm = dest_mask[pos]; }
        dc = 0; dmm = 0; de = 0; dp = 0;
        for (int32_t q0 = 0; q0 < npl; q0 += 64) {           // this candidate's placements in block j
            const int32_t q = q0 + lane;
            const int32_t d = q < npl ? ov.node[q] - j * 64 : -1;
            uint64_t mm = __ballot(d >= 0 && d < 64);
            while (mm) {
                const int l = __builtin_ctzll(mm);
                mm &= mm - 1;
                const int32_t dl = __builtin_amdgcn_readlane(d, l);
                const int32_t slot = q0 + l;
                if (lane == dl) { dc = ov.cpu[slot]; dmm = ov.mem[slot]; de = ov.eph[slot]; dp = ov.pods[slot]; }
            }
        }
        vis = valid & (pos != node) & (dm != 0);   // & !unschedulable: applied at use
    };
    // A = block of lastIndex, B = the next one (prefetched)
    auto refill = [&]() {
        const int32_t j = L >> 6;
        if (j == ja) return;
        if (j == jb) {
            ja = jb; Ah = Bh; Avis = Bvis; Adc = Bdc; Adm = Bdm; Ade = Bde; Adp = Bdp;
        } else {
            ja = j;
            load_block(ja, Ah, Avis, Adc, Adm, Ade, Adp);
        }
        jb = ja + 1 < nb ? ja + 1 : (nb > 1 ? 0 : -1);
        if (jb == ja) jb = -1;
        if (jb >= 0) load_block(jb, Bh, Bvis, Bdc, Bdm, Bde, Bdp);
    };

    for (int32_t i = 0; i < mn; i++) {
        const int sl = i & 63;
        if (sl == 0) {
            if (i > 0) {   // flush the previous batch's outputs
                out_dest[mo + i - 64 + lane] = my_dest;
                hint_set[mo + i - 64 + lane] = my_hset;
            }
            my_dest = -1; my_hset = -1;
            if (i + lane < mn) {
                my_id = move_pods[mo + i + lane];
                my_p = ph[my_id];
                my_hint = hints[mo + i + lane];
                if (my_hint >= 0 && my_hint < n) { my_hh = hot[my_hint]; my_hdm = dest_mask[my_hint]; }
            }
        }
        // one wavefront per workgroup: its LDS accesses complete in order, so the overlay
        // needs only a compiler-level barrier here (an s_barrier would also wait for the
        // next block's prefetch and every outstanding load, each pod)
        __builtin_amdgcn_wave_barrier();
        if (sl == 0) {
            // ---- the batch's leading pods placed on their hints, in bulk ----
            // Pod i of a run whose earlier pods all went to their hinted nodes sees exactly
            // those placements (plus the overlay so far) on its own hinted node, so the
            // hint checks of the run are independent lane-parallel checks; the first pod
            // whose check fails (or that cannot take this path) continues sequentially.
            // The steady-state sweep (hints of the previous loop) is almost all such pods.
            const int32_t bn = min(64, mn - i);
            bool el = false;
            PodHot q = my_p;
            q.flags = moved_flags(my_p.flags);
            if (lane < bn)
                el = my_hint >= 0 && my_hint < n && my_hint != node && my_hdm != 0 &&
                     !(q.flags & (PF_PREFILTER_FAIL | PF_PORTS | PF_SCALAR_REQ));
            const uint64_t em = __ballot(el);
            const int32_t lead = min(bn, em == ~0ull ? 64 : __builtin_ctzll(~em));
            int32_t f = 0;
            if (lead > 0) {
                int64_t ac = 0, am = 0, ae = 0;
                int32_t ap = 0;
                for (int32_t j = 0; j + 1 < lead; j++) {          // earlier pods of the run, same node
                    const int32_t hj = rl32s(my_hint, j);
                    const int64_t cj = rl64s(my_p.cpu, j), mj = rl64s(my_p.mem, j), ej = rl64s(my_p.eph, j);
                    if ((lane > j) & (lane < lead) & (my_hint == hj)) { ac += cj; am += mj; ae += ej; ap += 1; }
                }
                for (int32_t qq = 0; qq < npl; qq++) {              // this candidate's overlay so far
                    const int32_t nd = ov.node[qq];
                    if ((lane < lead) & (my_hint == nd)) {
                        ac += ov.cpu[qq]; am += ov.mem[qq]; ae += ov.eph[qq]; ap += ov.pods[qq];
                    }
                }
                bool fit = false;
                if (lane < lead) {
                    NodeHot nh = my_hh;
                    nh.cpu = wsub(nh.cpu, ac); nh.mem = wsub(nh.mem, am); nh.eph = wsub(nh.eph, ae); nh.pods -= ap;
                    const NodeExt ne = {};
                    int64_t psc0[CA_MAX_SCALAR];
                    for (int k = 0; k < CA_MAX_SCALAR; k++) psc0[k] = 0;
                    fit = eval_node(specs[q.spec], q, psc0, terms, reqs, nh, ne, st + my_hint, true);
                }
                const uint64_t fm = __ballot(fit);
                f = min(lead, fm == ~0ull ? 64 : __builtin_ctzll(~fm));
                // AddPod of the run into the overlay, in order (:79)
                for (int32_t j = 0; j < f; j++) {
                    const int32_t hj = rl32s(my_hint, j);
                    const int64_t cj = rl64s(my_p.cpu, j), mj = rl64s(my_p.mem, j), ej = rl64s(my_p.eph, j);
                    int32_t slot = -1;
                    for (int32_t q0 = 0; q0 < npl; q0 += 64) {
                        const uint64_t mm = __ballot(q0 + lane < npl && ov.node[q0 + lane] == hj);
                        if (mm) { slot = q0 + __builtin_ctzll(mm); break; }
                    }
                    if (slot < 0) {
                        if (npl >= OV_CAP) { f = j; break; }            // the sequential path reports it
                        slot = npl++;
                        if (lane == 0) {
                            ov.node[slot] = hj; ov.pods[slot] = 0; ov.cpu[slot] = 0; ov.mem[slot] = 0; ov.eph[slot] = 0;
                            if (use_ext) {
                                for (int w = 0; w < CA_PORT_WORDS; w++) ox.ports[slot][w] = 0;
                                for (int k = 0; k < CA_MAX_SCALAR; k++) ox.scalar[slot][k] = 0;
                            }
                        }
                    }
                    if (lane == 0) {
                        ov.cpu[slot] = wadd(ov.cpu[slot], cj);
                        ov.mem[slot] = wadd(ov.mem[slot], mj);
                        ov.eph[slot] = wadd(ov.eph[slot], ej);
                        ov.pods[slot] += 1;
                    }
                    if (lane == (hj & 63)) {
                        if ((hj >> 6) == ja) { Adc = wadd(Adc, cj); Adm = wadd(Adm, mj); Ade = wadd(Ade, ej); Adp += 1; }
                        if ((hj >> 6) == jb) { Bdc = wadd(Bdc, cj); Bdm = wadd(Bdm, mj); Bde = wadd(Bde, ej); Bdp += 1; }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (f > 0) {
                if (lane < f) { my_dest = my_hint; my_hset = my_hint; }      // hints.Set + isNodeAcceptable
                evals += (uint64_t)f;
                placed += f;
                __builtin_amdgcn_wave_barrier();
                i += f - 1;
                continue;
            }
        }
        PodHot p;
        p.cpu = rl64s(my_p.cpu, sl); p.mem = rl64s(my_p.mem, sl); p.eph = rl64s(my_p.eph, sl);
        p.flags = moved_flags((uint32_t)rl32s((int32_t)my_p.flags, sl));
        p.spec = rl32s(my_p.spec, sl);
        const int32_t h = rl32s(my_hint, sl);
        const ca_pod_spec& s = specs[p.spec];
        int64_t psc[CA_MAX_SCALAR];
        for (int k = 0; k < CA_MAX_SCALAR; k++) psc[k] = 0;
        if (p.flags & PF_SCALAR_REQ)
            for (int k = 0; k < CA_MAX_SCALAR; k++) psc[k] = ((s.tpu_scalar_mask >> k) & 1u) ? 0 : s.req_scalar[k];
        const bool pre_fail = (p.flags & PF_PREFILTER_FAIL) != 0;
        int32_t target = -1;

        if (n > 0) refill();
        // ---- findNodeWithHints (hinting_simulator.go:91-108) ----
        if (h >= 0 && h < n && !pre_fail) {
            evals++;
            NodeHot nh;
            nh.cpu = rl64s(my_hh.cpu, sl); nh.mem = rl64s(my_hh.mem, sl); nh.eph = rl64s(my_hh.eph, sl);
            nh.pods = rl32s(my_hh.pods, sl);
            nh.flags = (uint32_t)rl32s((int32_t)my_hh.flags, sl);
            NodeExt ne = {};                 // read only by the port / extended-resource checks
            if (p.flags & (PF_PORTS | PF_SCALAR_REQ)) ne = ext[h];
            if (h == node) {
                // the candidate with every moved pod removed (cluster.go:228-233): the moved
                // pods' requests summed lane-parallel once per candidate (wrapping adds:
                // any order), the extended part only for pods that read it
                if (!own_ok) {
                    int64_t sc = 0, sm = 0, se = 0;
                    for (int32_t q = lane; q < mn; q += 64) {
                        const PodHot mp = ph[move_pods[mo + q]];
                        sc = wadd(sc, mp.cpu); sm = wadd(sm, mp.mem); se = wadd(se, mp.eph);
                    }
                    own_c = __ockl_wfred_add_i64(sc); own_m = __ockl_wfred_add_i64(sm); own_e = __ockl_wfred_add_i64(se);
                    own_ok = true;
                }
                nh.cpu = wadd(nh.cpu, own_c); nh.mem = wadd(nh.mem, own_m); nh.eph = wadd(nh.eph, own_e);
                nh.pods += mn;
                if (p.flags & (PF_PORTS | PF_SCALAR_REQ))
                    for (int32_t q = 0; q < mn; q++) {
                        const ca_pod_spec& ms = specs[ph[move_pods[mo + q]].spec];
                        for (int k = 0; k < CA_MAX_SCALAR; k++) ne.scalar[k] = wadd(ne.scalar[k], ms.req_scalar[k]);
                        for (int w = 0; w < CA_PORT_WORDS; w++) ne.ports[w] &= ~ms.port_use[w];
                    }
            } else {
                // this candidate's placements on h (a node has at most one overlay slot)
                int32_t q = -1;
                for (int32_t q0 = 0; q0 < npl && q < 0; q0 += 64) {
                    const uint64_t m = __ballot(q0 + lane < npl && ov.node[q0 + lane] == h);
                    if (m) q = q0 + __builtin_ctzll(m);
                }
                if (q >= 0) {
                    nh.cpu = wsub(nh.cpu, ov.cpu[q]); nh.mem = wsub(nh.mem, ov.mem[q]);
                    nh.eph = wsub(nh.eph, ov.eph[q]); nh.pods -= ov.pods[q];
                    if (use_ext) {
                        for (int w = 0; w < CA_PORT_WORDS; w++) ne.ports[w] |= ox.ports[q][w];
                        for (int k = 0; k < CA_MAX_SCALAR; k++) ne.scalar[k] = wsub(ne.scalar[k], ox.scalar[q][k]);
                    }
                }
            }
            if (eval_node(s, p, psc, terms, reqs, nh, ne, st + h, true)) {
                if (lane == sl) my_hset = h;                                    // :95
                if (h != node && rl32s((int32_t)my_hdm, sl) != 0) target = h;  // :102
            }
        }
        // ---- findNode -> FitsAnyNodeMatching(isCandidateNode) (:110-125) ----
        // slow path: pods with host ports / extended resources / PreFilter node names
        // evaluate 64-node chunks straight from HBM with the overlay applied per chunk
        const bool fast = !(p.flags & (PF_PORTS | PF_SCALAR_REQ | PF_PREFILTER_NAMES));
        if (target < 0 && !pre_fail && !fast) {
            for (int32_t base = 0; base < n; base += 64) {
                const int32_t off = base + lane;
                int32_t pos = L + off;                                        // (lastIndex+i) % len
                if (pos >= n) pos -= n;
                const int32_t rp = off < n ? pos : 0;
                const uint8_t dm = dest_mask[rp];                             // both loads issue together
                NodeHot nh = hot[rp];
                bool vis = (off < n) & (pos != node) & (dm != 0) & !(nh.flags & NF_UNSCHED);
                if (vis && (p.flags & PF_PREFILTER_NAMES)) vis = in_prefilter(s, names, st[pos].name_id);
                // overlay entries inside this chunk
                bool ov_here = false;
                int32_t ov_slot = -1;
                int32_t st0 = L + base;                                        // chunk start position
                if (st0 >= n) st0 -= n;
                for (int32_t q0 = 0; q0 < npl; q0 += 64) {
                    const int32_t q = q0 + lane;
                    bool in = false;
                    int32_t d = 0;
                    if (q < npl) {
                        d = ov.node[q] - st0;
                        if (d < 0) d += n;
                        in = d < 64;
                    }
                    uint64_t m = __ballot(in);
                    while (m) {
                        const int l = __builtin_ctzll(m);
                        m &= m - 1;
                        const int32_t dl = __builtin_amdgcn_readlane(d, l);
                        if (lane == dl) { ov_here = true; ov_slot = q0 + l; }
                    }
                }
                bool fit = false;
                if (vis) {
                    const bool need_ext = (p.flags & (PF_PORTS | PF_SCALAR_REQ)) || ov_here;
                    if (!need_ext) {
                        fit = hot_fits(p, nh) && static_ok(s, p, terms, reqs, nh, st + pos);
                    } else {
                        NodeExt ne = ext[pos];
                        if (ov_here) {
                            nh.cpu = wsub(nh.cpu, ov.cpu[ov_slot]); nh.mem = wsub(nh.mem, ov.mem[ov_slot]);
                            nh.eph = wsub(nh.eph, ov.eph[ov_slot]); nh.pods -= ov.pods[ov_slot];
                            if (use_ext) {
                                for (int w = 0; w < CA_PORT_WORDS; w++) ne.ports[w] |= ox.ports[ov_slot][w];
                                for (int k = 0; k < CA_MAX_SCALAR; k++)
                                    ne.scalar[k] = wsub(ne.scalar[k], ox.scalar[ov_slot][k]);
                            }
                        }
                        fit = eval_node(s, p, psc, terms, reqs, nh, ne, st + pos, false);
                    }
                }
                const uint64_t fm = __ballot(fit), vm = __ballot(vis);
                if (fm) {
                    const int f = __builtin_ctzll(fm);
                    const uint64_t below = (f == 63) ? ~0ull : ((2ull << f) - 1);
                    evals += (uint64_t)__popcll(vm & below);
                    const int32_t foff = base + f;
                    target = L + foff;
                    if (target >= n) target -= n;
                    L = target + 1;                                            // schedulerbased.go:131
                    if (L >= n) L -= n;
                    fa_success = true;
                    if (lane == sl) my_hset = target;                          // :123
                    break;
                }
                evals += (uint64_t)__popcll(vm);
            }
        }
        // fast path: aligned 64-node blocks; the block holding lastIndex (A) and the next
        // one (B) stay in registers with this candidate's overlay as per-lane deltas
        if (target < 0 && !pre_fail && fast) {
            const int32_t j0 = L >> 6, l0 = L & 63;
            // look-ahead window over 64 full blocks (lane i: block r = wr + i): a block passes
            // when the pod fails its maxima and it holds none of this candidate's placements
            // (whose deltas the maxima do not see).  The overlay and the maxima are fixed for
            // the whole scan (a placement ends it), so one window serves 64 blocks.
            int32_t wr = -1, my_nv = 0;
            uint64_t passm = 0;
            for (int32_t r = 0; r <= nb; r++) {
                if (r == nb && l0 == 0) break;
                int32_t j = j0 + r;
                if (j >= nb) j -= nb;
                if (r > 0 && r < nb) {
                    if (wr < 0 || r >= wr + 64) {
                        const int32_t rr = r + lane;
                        bool pass = false;
                        my_nv = 0;
                        if (rr < nb) {
                            int32_t jj = j0 + rr;
                            if (jj >= nb) jj -= nb;
                            const BlockSum b = bsum[jj];
                            bool ovh = false;
                            for (int32_t q = 0; q < npl; q++) ovh |= (ov.node[q] >> 6) == jj;
                            pass = !ovh && !block_may_fit(p, b);
                            my_nv = block_vis(b, jj, 0, 64, node);
                        }
                        passm = __ballot(pass);
                        wr = r;
                    }
                    // pass every leading block from r on, counting its visible nodes
                    const int32_t off = r - wr;
                    const uint64_t stop = ~passm & (~0ull << off);
                    const int32_t k = (stop ? __builtin_ctzll(stop) : 64) - off;
                    if (k > 0) {
                        evals += (uint64_t)__ockl_wfred_add_i64((lane >= off && lane < off + k) ? my_nv : 0);
                        r += k - 1;
                        continue;
                    }
                }
                NodeHot raw;
                bool bvis;
                int64_t dc, dmm, de;
                int32_t dp;
                if (j == ja) { raw = Ah; bvis = Avis; dc = Adc; dmm = Adm; de = Ade; dp = Adp; }
                else if (j == jb) { raw = Bh; bvis = Bvis; dc = Bdc; dmm = Bdm; de = Bde; dp = Bdp; }
                else load_block(j, raw, bvis, dc, dmm, de, dp);
                const bool inr = (r == 0) ? lane >= l0 : (r == nb ? lane < l0 : true);
                const bool vis = bvis & inr & !(raw.flags & NF_UNSCHED);
                NodeHot eff = raw;
                eff.cpu = wsub(raw.cpu, dc); eff.mem = wsub(raw.mem, dmm); eff.eph = wsub(raw.eph, de);
                eff.pods = raw.pods - dp;
                bool fit = vis && hot_fits(p, eff);
                if (fit) fit = static_ok(s, p, terms, reqs, eff, st + (j * 64 + lane));
                const uint64_t fm = __ballot(fit), vm = __ballot(vis);
                if (fm) {
                    const int f = __builtin_ctzll(fm);
                    const uint64_t below = (f == 63) ? ~0ull : ((2ull << f) - 1);
                    evals += (uint64_t)__popcll(vm & below);
                    target = j * 64 + f;
                    L = target + 1;                                            // schedulerbased.go:131
                    if (L >= n) L -= n;
                    fa_success = true;
                    if (lane == sl) my_hset = target;                          // :123
                    break;
                }
                evals += (uint64_t)__popcll(vm);
            }
        }
        if (target < 0) { failed = true; break; }                              // breakOnFailure
        // ---- AddPod(pod, target) into the overlay (:79) ----
        int32_t slot = -1;
        for (int32_t q0 = 0; q0 < npl; q0 += 64) {
            const int32_t q = q0 + lane;
            const uint64_t m = __ballot(q < npl && ov.node[q] == target);
            if (m) { slot = q0 + __builtin_ctzll(m); break; }
        }
        if (slot < 0) {
            if (npl >= OV_CAP) { res.status = CA_ECAPACITY; failed = true; break; }
            slot = npl++;
            if (lane == 0) {
                ov.node[slot] = target; ov.pods[slot] = 0; ov.cpu[slot] = 0; ov.mem[slot] = 0; ov.eph[slot] = 0;
                if (use_ext) {
                    for (int w = 0; w < CA_PORT_WORDS; w++) ox.ports[slot][w] = 0;
                    for (int k = 0; k < CA_MAX_SCALAR; k++) ox.scalar[slot][k] = 0;
                }
            }
        }
        if (lane == 0) {
            ov.cpu[slot] = wadd(ov.cpu[slot], p.cpu);
            ov.mem[slot] = wadd(ov.mem[slot], p.mem);
            ov.eph[slot] = wadd(ov.eph[slot], p.eph);
            ov.pods[slot] += 1;
            if (use_ext) {
                for (int w = 0; w < CA_PORT_WORDS; w++) ox.ports[slot][w] |= s.port_use[w];
                for (int k = 0; k < CA_MAX_SCALAR; k++) ox.scalar[slot][k] = wadd(ox.scalar[slot][k], psc[k]);
            }
        }
        if (lane == (target & 63)) {
            if ((target >> 6) == ja) { Adc = wadd(Adc, p.cpu); Adm = wadd(Adm, p.mem); Ade = wadd(Ade, p.eph); Adp += 1; }
            if ((target >> 6) == jb) { Bdc = wadd(Bdc, p.cpu); Bdm = wadd(Bdm, p.mem); Bde = wadd(Bde, p.eph); Bdp += 1; }
        }
        if (lane == sl) my_dest = target;
        placed++;
    }
    if (mn > 0) {
        // the batch that was being processed (the last one, or the one that failed)
        const int32_t bi = failed ? (placed >> 6) << 6 : ((mn - 1) >> 6) << 6;
        if (bi + lane < mn) { out_dest[mo + bi + lane] = my_dest; hint_set[mo + bi + lane] = my_hset; }
        // batches after it were never loaded
        for (int32_t i = bi + 64 + lane; i < mn; i += 64) { out_dest[mo + i] = -1; hint_set[mo + i] = -1; }
    }
    if (lane == 0) {
        res.n_placed = placed;
        if (!failed && placed == mn) { res.removable = 1; res.reason = CA_UNREMOVABLE_NONE; }
        else res.reason = CA_UNREMOVABLE_NO_PLACE;
        res.lout = L;
        res.fa_success = fa_success ? 1 : 0;
        res.evals = evals;
        res.pad2 = wall_clock64() - t_begin;
        outs[c] = res;
        walk_lout[c] = fa_success ? L : -1;    // host walk: -1 = the result does not depend on lastIndex
    }
    if (fa_success) chain_v = L;
    __builtin_amdgcn_wave_barrier();              // (the next candidate re-initialises the overlay)
    }
    if (chain && threadIdx.x == 0) *chain = chain_v;
}

// ---------------------------------------------------------------------------
// Fit-point classes of lastIndex.  A candidate's first FitsAnyNode scan from L lands on
// the first node at or after L where its first pod fits (schedulerbased.go:114-131),
// and everything after depends only on that node: every L in (f_{w-1}, f_w] between two
// consecutive fit points of the first pod has the outputs of L = f_w, except for the
// evaluations of the skipped visible nodes in [L, f_w).  A table row therefore holds 64
// classes: fp[0] = f_{-1}, fp[1 + w] = f_w, and lane w simulates L = f_w.  In a loose
// cluster every node fits and the classes are 64 consecutive positions; in a tight one a
// row covers 64 fit points (DESIGN.md §4 sweep).  Rows whose first pod has PreFilter
// node names, or a ring with fewer than 65 fit points, use 64 consecutive positions.
// ---------------------------------------------------------------------------
constexpr int FPW = SWEEP_FPW;

// class of lastIndex L in a row (fp[k * fs], k = 0..64), or -1 outside it
__host__ __device__ inline int32_t fp_class(const int32_t* fp, int32_t fs, int32_t n, int32_t L) {
    if (n < FPW) {                     // a ring shorter than a row: 64 consecutive positions cover it
        int32_t w = L - fp[fs];
        if (w < 0) w += n;
        return w;
    }
    const int32_t f0 = fp[0];
    int32_t d = L - f0;
    if (d < 0) d += n;
    if (d <= 0) return -1;
    auto D = [&](int32_t w) { int32_t x = fp[(size_t)(w + 1) * fs] - f0; return x <= 0 ? x + n : x; };
    const int32_t d63 = D(63);
    if (d > d63) return -1;
    // interpolation, then a few steps: the fit points of a row are spread about evenly
    int32_t w = (int32_t)((float)d * 64.0f / (float)d63) - 1;     // (no 64-bit division on the device)
    w = w < 0 ? 0 : (w > 63 ? 63 : w);
    while (w > 0 && D(w - 1) >= d) w--;
    while (D(w) < d) w++;
    return w;
}

// visible nodes (destination, schedulable, not the candidate) in the cyclic range [a, b)
__device__ inline int32_t vis_between(const int32_t* __restrict__ vp, int32_t n, int32_t a, int32_t b, int32_t node,
                                      bool node_vis) {
    int32_t v = a <= b ? vp[b] - vp[a] : vp[n] - vp[a] + vp[b];
    const bool in = a <= b ? (node >= a && node < b) : (node >= a || node < b);
    return v - ((in && node_vis) ? 1 : 0);
}

// vp[i] = destination, schedulable nodes among positions [0, i) (one block of 1024 threads)
__device__ void vis_prefix_block(const NodeHot* __restrict__ hot, const uint8_t* __restrict__ dest_mask, int32_t n,
                                 int32_t* __restrict__ vp) {
    __shared__ int32_t wsum[16];
    __shared__ int32_t carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) { carry = 0; vp[0] = 0; }
    __syncthreads();
    for (int32_t base = 0; base < n; base += 1024) {
        const int32_t i = base + tid;
        const int32_t v = (i < n && dest_mask[i] && !(hot[i].flags & NF_UNSCHED)) ? 1 : 0;
        const uint64_t m = __ballot(v != 0);
        const int32_t incl = __popcll(m & (lane == 63 ? ~0ull : ((2ull << lane) - 1)));
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int32_t pre = carry;
        for (int q = 0; q < w; q++) pre += wsum[q];
        if (i < n) vp[i + 1] = pre + incl;
        __syncthreads();
        if (tid == 0) { int32_t t = 0; for (int q = 0; q < 16; q++) t += wsum[q]; carry += t; }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// table kernel: lane w simulates the candidate from lastIndex = class w of its row.
// A lane's placements all lie in the cyclic interval its scans have passed
// ([L_start, L_cur)); a scan that would re-enter it (a full turn of the ring: a
// NoPlace failure or a revisit) is left to the exact kernel, as are candidates with
// hints or port/scalar pods.  Scans longer than TB_SCAN are left to it too.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_sweep_table(
    const NodeHot* __restrict__ hot, const NodeStatic* __restrict__ st, int32_t n,
    const uint8_t* __restrict__ dest_mask, const int32_t* __restrict__ cands, const int32_t* __restrict__ move_off,
    const int32_t* __restrict__ move_pods, const PodHot* __restrict__ ph, const ca_pod_spec* __restrict__ specs,
    const ca_selector_term* __restrict__ terms, const ca_selector_req* __restrict__ reqs,
    const int32_t* __restrict__ names, const int32_t* __restrict__ hints, const int32_t* __restrict__ todo,
    const int32_t* __restrict__ wstart, const int32_t* __restrict__ row_of, int32_t* __restrict__ table,
    int32_t stride, uint32_t* __restrict__ tev, int32_t* __restrict__ tdest, const int32_t* __restrict__ tdoff,
    int32_t* __restrict__ tfp, const int32_t* __restrict__ mode, const BlockSum* __restrict__ bsum) {
    // tev / tdest (first round, device walk): the lane's evaluation count and each moved
    // pod's destination, so a candidate the walk resolves through the table takes these
    // outputs (k_table_gather) instead of being simulated again
    __shared__ int32_t fps[FPW];
    const int t = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t c = todo[t];
    const int32_t node = cands[c];
    const int32_t mo = move_off[c], mn = move_off[c + 1] - mo;
    const int32_t row = row_of ? row_of[t] : t;
    const int32_t ws0 = wstart[t];
    // the row's classes: fit points of the first pod from the window start (wave-parallel,
    // 64 positions per step), or 64 consecutive positions
    bool classes = false;
    if (mode[0] && mn > 0 && n > 0) {
        const PodHot p0h = ph[move_pods[mo]];
        PodHot p0 = p0h;
        p0.flags = moved_flags(p0h.flags);
        if (!(p0.flags & (PF_PREFILTER_NAMES | PF_PREFILTER_FAIL | PF_PORTS | PF_SCALAR_REQ))) {
            const ca_pod_spec& s0 = specs[p0.spec];
            // ring order from the window start: the tail of its block, the blocks after it
            // (64 at a time passed on their maxima), the head of its block
            const int32_t nb = (n + 63) >> 6;
            int32_t ws = ws0;
            if (ws >= n) ws -= n;
            const int32_t j0 = ws >> 6, l0 = ws & 63;
            int32_t cnt = 0;
            for (int32_t r = 0; r <= nb && cnt < FPW; r++) {
                if (r == nb && l0 == 0) break;
                int32_t j = j0 + r;
                if (j >= nb) j -= nb;
                if (r > 0 && r < nb) {
                    const int32_t rr = r + lane;
                    bool pass = false;
                    if (rr < nb) {
                        int32_t jj = j0 + rr;
                        if (jj >= nb) jj -= nb;
                        pass = !block_may_fit(p0, bsum[jj]);
                    }
                    const uint64_t stop = __ballot(!pass);
                    const int32_t k = stop ? __builtin_ctzll(stop) : 64;
                    if (k > 0) { r += k - 1; continue; }
                }
                const int32_t pos = j * 64 + lane;
                const bool inr = (pos < n) & ((r == 0) ? lane >= l0 : (r == nb ? lane < l0 : true));
                bool fit = false;
                if (inr) {
                    const NodeHot nh = hot[pos];
                    fit = (pos != node) & (dest_mask[pos] != 0) & !(nh.flags & NF_UNSCHED) && hot_fits(p0, nh) &&
                          static_ok(s0, p0, terms, reqs, nh, st + pos);
                }
                const uint64_t m = __ballot(fit);
                const int32_t rk = cnt + __popcll(m & lanes_below_u(lane));
                if (fit && rk < FPW) fps[rk] = pos;
                cnt += __popcll(m);
            }
            classes = cnt >= FPW;
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (!classes) {
        for (int32_t i = lane; i < FPW; i += 64) {
            int32_t v = ws0 - 1 + i;
            if (v < 0) v += n;
            if (v >= n) v -= n;
            fps[i] = v;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (tfp) for (int32_t i = lane; i < FPW; i += 64) tfp[(size_t)i * stride + row] = fps[i];   // [FPW][stride]
    int32_t Ls = fps[1 + lane];
    int32_t Lcur = Ls;
    int32_t adv = 0;              // positions passed since Ls
    uint32_t ev = 0;              // visible nodes scanned (the exact kernel's evals)
    const int32_t dbase = tdoff ? tdoff[t] : -1;
    bool unknown = mn > TB_MAXP;
    // candidates with hints / ports / scalars go to the exact kernel.  A hint to the
    // candidate's own node (a pod committed onto it by the planner, planner.hip) is checked
    // (one evaluation) but never accepted (cluster.go:221-223), and the scan's Hints.Set
    // overrides the check's: such a pod is an unhinted one plus an evaluation while its scan
    // succeeds (a failing scan is left to the exact kernel anyway).
    for (int32_t i = lane; i < mn; i += 64) {
        const int32_t id = move_pods[mo + i];
        const uint32_t f = moved_flags(ph[id].flags);
        const int32_t h = hints[mo + i];
        if ((h >= 0 && h != node) | ((f & (PF_PORTS | PF_SCALAR_REQ)) != 0)) unknown = true;
    }
    unknown = __ballot(unknown) != 0;
    if (!unknown) {
        // lane-parallel prefetch of the moved pods' records (batch of 64)
        int32_t my_id = -1, my_h = -1;
        PodHot my_p = {};
        for (int32_t i = 0; i < mn; i++) {
            const int sl = i & 63;
            if (sl == 0 && i + lane < mn) { my_id = move_pods[mo + i + lane]; my_p = ph[my_id]; my_h = hints[mo + i + lane]; }
            ev += rl32s(my_h, sl) == node ? 1u : 0u;                             // the own-node hint check
            PodHot p;
            p.cpu = rl64s(my_p.cpu, sl); p.mem = rl64s(my_p.mem, sl); p.eph = rl64s(my_p.eph, sl);
            p.flags = moved_flags((uint32_t)rl32s((int32_t)my_p.flags, sl));
            p.spec = rl32s(my_p.spec, sl);
            if (p.flags & PF_PREFILTER_FAIL) { unknown = true; break; }         // FitsAnyNode error: exact kernel
            const ca_pod_spec& s = specs[p.spec];
            // lane-private rotating scan from this lane's lastIndex
            int32_t steps = 0, work = 0;
            int32_t pos = Lcur;
            bool lane_unknown = false;
            const bool skip_ok = !(p.flags & PF_PREFILTER_NAMES);
            int32_t okb = -1;             // block whose maxima the pod passes
            while (!unknown) {
                if (adv + steps >= n || work >= TB_SCAN) { lane_unknown = true; break; }
                const int32_t b = pos >> 6;
                // the node's row is requested with its block's summary: one global round trip
                // per step, not two (a row read for a block that passes is wasted bandwidth only)
                const NodeHot nh = hot[pos];
                const uint8_t dm = dest_mask[pos];
                if (skip_ok && b != okb) {
                    // the rest of a block whose maxima the pod fails: passed in one step (the
                    // lane's placements all lie behind it, so the committed rows are exact)
                    const BlockSum bs = bsum[b];
                    if (!block_may_fit(p, bs)) {
                        const int32_t end = min((b + 1) * 64, n);
                        ev += (uint32_t)block_vis(bs, b, pos & 63, end - b * 64, node);
                        steps += end - pos;
                        pos = end >= n ? 0 : end;
                        work++;
                        continue;
                    }
                    okb = b;
                }
                work++;
                bool vis = (pos != node) & (dm != 0) & !(nh.flags & NF_UNSCHED);
                if (vis && (p.flags & PF_PREFILTER_NAMES)) vis = in_prefilter(s, names, st[pos].name_id);
                ev += vis ? 1u : 0u;
                if (vis && hot_fits(p, nh) && static_ok(s, p, terms, reqs, nh, st + pos)) break;
                steps++;
                pos++;
                if (pos >= n) pos = 0;
            }
            if (lane_unknown) unknown = true;
            if (__ballot(!unknown) == 0) break;          // every lane handed over
            if (!unknown) {
                if (dbase >= 0) tdest[(size_t)(dbase + i) * 64 + lane] = pos;
                adv += steps + 1;
                Lcur = pos + 1;
                if (Lcur >= n) Lcur = 0;
            }
        }
    }
    table[(size_t)lane * stride + row] = unknown ? TB_UNKNOWN : Lcur;
    if (tev) tev[(size_t)lane * stride + row] = ev;
}

// ---------------------------------------------------------------------------
// window estimate for the first table round.  The probe pass (k_sweep at rough
// guesses) tells how far each candidate moved lastIndex; the advance barely depends on
// the starting point (a placement lands on the first node with room), so the prefix sum
// of the advances centres every window within a few positions of the true value.  A
// candidate that made no successful scan does not move lastIndex at all (advance 0).
// est_k = L0 + sum_{i<k} adv_i (mod n); window start = est_k - 32.  One block.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_sweep_est(const SweepOut* __restrict__ probe, const int32_t* __restrict__ sens,
                                                    int32_t S, int32_t n, int32_t* __restrict__ ws,
                                                    int32_t* __restrict__ mode, const NodeHot* __restrict__ hot,
                                                    const uint8_t* __restrict__ dest_mask, int32_t* __restrict__ vp) {
    const int64_t L0 = mode[2];                      // the chain's input lastIndex (mod n), copied in by the host
    // Rows of fit-point classes pay off where placements are sparse: the probe's positions
    // passed per placement decide it for the whole call (mode[0] = 1: classes, window start
    // = 32 x the candidate's mean gap before the estimate; 0: 64 consecutive positions).
    __shared__ int64_t part[2][16];
    int64_t my_adv = 0, my_placed = 0;
    for (int32_t k = threadIdx.x; k < S; k += blockDim.x) {
        const SweepOut o = probe[sens[k]];
        if (o.fa_success) {
            int64_t d = ((int64_t)o.lout - (int64_t)o.lin) % n;
            if (d < 0) d += n;
            my_adv += d;
            my_placed += max(1, o.n_placed);
        }
    }
    my_adv = __ockl_wfred_add_i64(my_adv);
    my_placed = __ockl_wfred_add_i64(my_placed);
    if ((threadIdx.x & 63) == 0) { part[0][threadIdx.x >> 6] = my_adv; part[1][threadIdx.x >> 6] = my_placed; }
    __syncthreads();
    int64_t sum_adv = 0, sum_placed = 0;
    for (int q = 0; q < 16; q++) { sum_adv += part[0][q]; sum_placed += part[1][q]; }
    // C3 (a loose cluster): 1.008 positions per placement; C5 RunOnce: 1.10, where the
    // few long gaps are what throws the consecutive windows off
    const bool classes = sum_adv * 100 > sum_placed * 104;
    if (threadIdx.x == 0) mode[0] = classes ? 1 : 0;
    if (classes && vp) vis_prefix_block(hot, dest_mask, n, vp);    // for k_table_gather's evaluation counts
    __shared__ int64_t wtot[16];
    __shared__ int64_t carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int32_t base = 0; base < S; base += 1024) {
        const int32_t k = base + tid;
        int64_t v = 0, gap = 1;
        if (k < S) {
            const SweepOut o = probe[sens[k]];
            if (o.fa_success) {
                int64_t d = ((int64_t)o.lout - (int64_t)o.lin) % n;
                if (d < 0) d += n;
                v = d;
                if (classes) gap = max((int64_t)1, min((int64_t)(n / 64), d / max(1, o.n_placed)));
            }
        }
        int64_t x = v;                                   // inclusive scan in the wave
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[w] = x;
        __syncthreads();
        int64_t pre = carry;
        for (int q = 0; q < w; q++) pre += wtot[q];
        if (k < S) {
            int64_t e = (L0 + pre + x - v - 32 * gap) % n;  // exclusive prefix, window start
            if (e < 0) e += n;
            ws[k] = (int32_t)e;
        }
        __syncthreads();
        if (tid == 0) {
            int64_t t = 0;
            for (int q = 0; q < 16; q++) t += wtot[q];
            carry += t;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// device walk of the lastIndex chain, replacing the host walk and its
// round trip in the common case.  The chain is cut into chunks of WK sensitive
// candidates.  k_walk_chunks: lane x of chunk j follows the chain through the chunk from
// input ws[first] + x (the 64 values around the estimate), applying each candidate's map
// (insensitive: identity; the probe's input: the probe's output; inside the candidate's
// table window: the table; otherwise: stop), with the table rows staged in LDS; it
// records every lane's trajectory.  k_walk_resolve: one thread chains the chunk maps
// from the true input, then every candidate of the resolved prefix reads its exact
// input and whether it needs the exact re-run from the trajectory of its chunk's true
// lane.  A stop (input outside every window, or a row the table cannot simulate) hands
// the rest of the chain to the host walk.
// ---------------------------------------------------------------------------
constexpr int WK = 64;
constexpr int WALK_MAX_CHUNKS = 256;

__global__ void __launch_bounds__(64) k_walk_chunks(const int32_t* __restrict__ sens, const int32_t* __restrict__ ws,
                                                   const int32_t* __restrict__ guess, const int32_t* __restrict__ wl,
                                                   const int32_t* __restrict__ tab, const int32_t* __restrict__ tfp,
                                                   const int32_t* __restrict__ mode, int32_t S, int32_t n,
                                                   int32_t* __restrict__ cmap, int32_t* __restrict__ traj) {
    __shared__ int32_t T[64][WK + 1];
    __shared__ int32_t FP[FPW][WK + 1];
    __shared__ int32_t cws[WK], cg[WK], cwl[WK];
    const int j = blockIdx.x, lane = threadIdx.x;
    const int32_t k0 = j * WK, kn = min(WK, S - k0);
    const bool classes = mode[0] != 0;
    for (int w = 0; w < 64; w++) T[w][lane] = lane < kn ? tab[(size_t)w * S + k0 + lane] : TB_UNKNOWN;
    if (classes)
        for (int i = 0; i < FPW; i++) FP[i][lane] = lane < kn ? tfp[(size_t)i * S + k0 + lane] : 0;
    if (lane < kn) {
        const int32_t c = sens[k0 + lane];
        cws[lane] = ws[k0 + lane];
        cg[lane] = guess[c];
        cwl[lane] = wl[c];
    }
    __syncthreads();
    // lane x: class x of the chunk's first row (its fit point, or position ws + x)
    int32_t cur = classes ? FP[1 + lane][0] : (int32_t)(((int64_t)cws[0] + lane) % n);
    int32_t stop = -1;
    for (int kk = 0; kk < kn; kk++) {
        int32_t enc = -1;
        if (stop < 0) {
            enc = cur * 2;                                  // lastIndex before candidate kk, re-run bit
            const int32_t wlv = cwl[kk];
            if (wlv >= 0) {
                if (cur == cg[kk]) {
                    cur = wlv;
                } else {
                    int32_t w;
                    if (classes) {
                        w = fp_class(&FP[0][kk], WK + 1, n, cur);
                    } else {
                        w = cur - cws[kk];
                        if (w < 0) w += n;
                        if (w >= 64) w = -1;
                    }
                    const int32_t v = w >= 0 ? T[w][kk] : TB_UNKNOWN;
                    if (v == TB_UNKNOWN) stop = kk;
                    else { cur = v; enc |= 1; }
                }
            }
        }
        traj[((size_t)k0 + kk) * 64 + lane] = enc;
    }
    cmap[(size_t)j * 64 + lane] = stop >= 0 ? -1 - stop : cur;
}

// info[0] = first unresolved sensitive candidate (S: all), info[1] = lastIndex before it
__global__ void __launch_bounds__(1024) k_walk_resolve(const int32_t* __restrict__ sens, const int32_t* __restrict__ tfp,
                                                      const int32_t* __restrict__ cmap, const int32_t* __restrict__ traj,
                                                      const int32_t* __restrict__ wl, const int32_t* __restrict__ mode,
                                                      int32_t S, int32_t n,
                                                      int32_t* __restrict__ lin, uint8_t* __restrict__ need,
                                                      int32_t* __restrict__ info) {
    const int32_t L0n = mode[2];                     // the chain's input lastIndex (mod n)
    // dynamic LDS: the chunk maps [nch][64] and the chunks' first rows [nch][FPW]
    extern __shared__ int32_t wr_lds[];
    __shared__ int32_t lane_of[WALK_MAX_CHUNKS], cin[WALK_MAX_CHUNKS];
    __shared__ int32_t stop_k, cur_out;
    const int32_t nch = (S + WK - 1) / WK;
    int32_t* const cm = wr_lds;
    int32_t* const heads = wr_lds + (size_t)nch * 64;
    for (int32_t i = threadIdx.x; i < nch * 64; i += blockDim.x) cm[i] = cmap[i];
    const bool classes = mode[0] != 0;
    if (classes)
        for (int32_t i = threadIdx.x; i < nch * FPW; i += blockDim.x)
            heads[i] = tfp[(size_t)(i % FPW) * S + (size_t)(i / FPW) * WK];
    else
        for (int32_t j = threadIdx.x; j < nch; j += blockDim.x) heads[(size_t)j * FPW + 1] = tfp[(size_t)S + (size_t)j * WK];
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t cur = L0n, sk = S;
        for (int32_t j = 0; j < nch; j++) {
            int32_t x;
            if (classes) {
                x = fp_class(heads + (size_t)j * FPW, 1, n, cur);
            } else {                          // consecutive positions from the row's first class
                x = cur - heads[(size_t)j * FPW + 1];
                if (x < 0) x += n;
                if (x >= 64) x = -1;
            }
            if (x < 0) { sk = j * WK; break; }
            lane_of[j] = x;
            cin[j] = cur;                     // the chunk's true input (its lane started at class x's point)
            const int32_t r = cm[j * 64 + x];
            if (r < 0) {
                sk = j * WK + (-1 - r);
                if (sk > j * WK) cur = traj[(size_t)sk * 64 + x] >> 1;
                break;
            }
            cur = r;
        }
        stop_k = sk;
        cur_out = cur;
    }
    __syncthreads();
    const int32_t sk = stop_k;
    for (int32_t k = threadIdx.x; k < sk; k += blockDim.x) {
        const int32_t e = traj[(size_t)k * 64 + lane_of[k / WK]];
        const int32_t c = sens[k];
        uint8_t nd = (uint8_t)((e & 1) ? 2 : 0);       // 2: resolved through the table (k_table_gather)
        if (k % WK == 0) {
            // the chunk's lane ran this candidate from its class's fit point: a probe taken at
            // that point has the chain's lastIndex out but not this input's outputs
            const int32_t L = cin[k / WK];
            if (!(e & 1) && wl[c] >= 0 && lin[c] != L) nd = 1;
            lin[c] = L;
        } else {
            lin[c] = e >> 1;
        }
        need[c] = nd;
    }
    if (threadIdx.x == 0) { info[0] = sk; info[1] = cur_out; }
}

// The block map of a candidate range (multi-device sweep, multi.hip): the same chunk maps
// as k_walk_resolve, chained from each of the 64 classes of the range's first row instead
// of from one known input.  out[x] = the range's lastIndex out when it starts in class x
// (-1: the walk leaves a window or meets a row the table cannot simulate);
// out[64 + i] = the first row's fit points (its class boundaries, FPW entries; in
// consecutive mode only [1], the window start, is meaningful); out[64 + FPW] = mode[0].
// The caller composes the ranges' maps in order from the true input: a range whose input
// falls inside its first window is resolved without re-running anything.
__global__ void __launch_bounds__(1024) k_walk_map(const int32_t* __restrict__ tfp, const int32_t* __restrict__ cmap,
                                                  const int32_t* __restrict__ mode, int32_t S, int32_t n,
                                                  int32_t* __restrict__ out) {
    extern __shared__ int32_t wr_lds[];
    const int32_t nch = (S + WK - 1) / WK;
    int32_t* const cm = wr_lds;
    int32_t* const heads = wr_lds + (size_t)nch * 64;
    for (int32_t i = threadIdx.x; i < nch * 64; i += blockDim.x) cm[i] = cmap[i];
    const bool classes = mode[0] != 0;
    if (classes)
        for (int32_t i = threadIdx.x; i < nch * FPW; i += blockDim.x)
            heads[i] = tfp[(size_t)(i % FPW) * S + (size_t)(i / FPW) * WK];
    else
        for (int32_t j = threadIdx.x; j < nch; j += blockDim.x) heads[(size_t)j * FPW + 1] = tfp[(size_t)S + (size_t)j * WK];
    __syncthreads();
    const int tid = threadIdx.x;
    if (tid < 64) {
        int32_t x = tid, cur = -1;
        bool ok = true;
        for (int32_t j = 0; j < nch && ok; j++) {
            if (j > 0) {
                if (classes) {
                    x = fp_class(heads + (size_t)j * FPW, 1, n, cur);
                } else {
                    x = cur - heads[(size_t)j * FPW + 1];
                    if (x < 0) x += n;
                    if (x >= 64) x = -1;
                }
                if (x < 0) { ok = false; break; }
            }
            const int32_t r = cm[j * 64 + x];
            if (r < 0) ok = false;
            else cur = r;
        }
        out[tid] = ok ? cur : -1;
    }
    if (tid < FPW) out[64 + tid] = classes ? heads[tid] : (tid == 1 ? heads[1] : 0);
    if (tid == 0) out[64 + FPW] = classes ? 1 : 0;
}

// Candidates the device walk resolved through the table (need == 2): the table lane at
// their exact input simulated them exactly (unhinted, no ports / extended requests, no
// ring wrap, every pod placed), so its outputs are theirs: removable, every pod at its
// recorded destination (Hints.Set to it), lastIndex out, evaluations.  One wavefront per
// sensitive candidate; need becomes 0 so the exact pass skips it.
__global__ void __launch_bounds__(64) k_table_gather(const int32_t* __restrict__ sens, const int32_t* __restrict__ tfp,
                                                    const int32_t* __restrict__ vp, const int32_t* __restrict__ cands,
                                                    const uint8_t* __restrict__ dest_mask, const NodeHot* __restrict__ hot,
                                                    int32_t S, int32_t n, const int32_t* __restrict__ lin,
                                                    uint8_t* __restrict__ need, const int32_t* __restrict__ tab,
                                                    const uint32_t* __restrict__ tev, const int32_t* __restrict__ tdest,
                                                    const int32_t* __restrict__ tdoff, const int32_t* __restrict__ move_off,
                                                    SweepOut* __restrict__ outs, int32_t* __restrict__ out_dest,
                                                    int32_t* __restrict__ hint_set, int32_t* __restrict__ walk_lout,
                                                    const int32_t* __restrict__ mode) {
    const int32_t k = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t c = sens[k];
    if (need[c] != 2) return;
    const int32_t* fp = tfp + k;                           // column k of [FPW][S]
    int32_t x;                                             // resolved: inside the row
    if (mode[0]) {
        x = fp_class(fp, S, n, lin[c]);
    } else {
        x = lin[c] - fp[S];
        if (x < 0) x += n;
    }
    const int32_t mo = move_off[c], mn = move_off[c + 1] - mo;
    const int32_t db = tdoff[k];
    for (int32_t i = lane; i < mn; i += 64) {
        const int32_t d = tdest[(size_t)(db + i) * 64 + x];
        out_dest[mo + i] = d;
        hint_set[mo + i] = d;
    }
    if (lane == 0) {
        SweepOut r;
        r.removable = 1; r.reason = CA_UNREMOVABLE_NONE; r.n_placed = mn; r.lin = lin[c];
        r.lout = tab[(size_t)x * S + k];
        r.fa_success = mn > 0 ? 1 : 0; r.status = CA_OK; r.pad = 0;
        // the lane ran from the class's fit point: add the visible nodes skipped before it
        const int32_t node = cands[c];
        const bool node_vis = dest_mask[node] != 0 && !(hot[node].flags & NF_UNSCHED);
        r.evals = tev[(size_t)x * S + k] +
                  (mode[0] ? (uint64_t)vis_between(vp, n, lin[c], fp[(size_t)(1 + x) * S], node, node_vis) : 0ull);
        r.pad2 = 0;
        outs[c] = r;
        walk_lout[c] = r.lout;
        need[c] = 0;
    }
}

// resident hints (per mirror pod): gather the moved pods' hints / apply the hint sets
__global__ void k_hints_gather(const int32_t* __restrict__ pod_hints, const int32_t* __restrict__ moves, int32_t M,
                               int32_t* __restrict__ hint_move) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < M) hint_move[i] = pod_hints[moves[i]];
}
__global__ void k_hints_apply(const int32_t* __restrict__ hset, const int32_t* __restrict__ moves, int32_t M,
                              int32_t* __restrict__ pod_hints) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < M && hset[i] >= 0) pod_hints[moves[i]] = hset[i];
}

}  // namespace casim

using namespace casim;

namespace casim {

inline int32_t wrap(int64_t v, int32_t n) {
    if (n <= 0) return 0;
    if (v >= 0 && v < n) return (int32_t)v;            // the common case: no division
    if (v >= n && v < 2 * (int64_t)n) return (int32_t)(v - n);
    if (v < 0 && v >= -(int64_t)n) return (int32_t)(v + n);
    int64_t r = v % n;
    if (r < 0) r += n;
    return (int32_t)r;
}

// a typed view into the packed input buffer
struct DevView {
    void* ptr;
    template <class T> T* as() const { return static_cast<T*>(ptr); }
};

// One FindNodesToRemove call: host copies (bookkeeping) and device views of the inputs.
struct SweepCall {
    int32_t C = 0, M = 0, n = 0;
    const int32_t *cand = nullptr, *status = nullptr, *move_off = nullptr, *move_pods = nullptr;
    const uint8_t* dest_mask = nullptr;
    DevView d_c{}, d_status{}, d_off{}, d_moves{}, d_hints{}, d_mask{};
};

int launch_exact(ca_mirror* m, hipStream_t st, const SweepCall& in, const int32_t* d_lin, const uint8_t* d_need,
                 DevView d_dest, DevView d_hset, DevView d_out, int32_t* d_wl, const int32_t* d_chain_list = nullptr,
                 int32_t n_chain = 0, int32_t* d_chain = nullptr) {
    const bool use_ext = m->n_ext_pods > 0;
    const size_t dyn = use_ext ? sizeof(OverlayExt) : 0;
    if (use_ext) {
        int rc;
        if ((rc = ensure_dyn_lds((const void*)k_sweep, dyn)) != CA_OK) return rc;
    }
    hipLaunchKernelGGL(k_sweep, dim3(d_chain ? 1 : in.C), dim3(64), dyn, st, m->d_hot.as<NodeHot>(), m->d_ext.as<NodeExt>(),
                       m->d_static.as<NodeStatic>(), in.n, in.d_mask.as<uint8_t>(), in.d_c.as<int32_t>(),
                       in.d_status.as<int32_t>(), in.d_off.as<int32_t>(), in.d_moves.as<int32_t>(),
                       m->d_pods.hot.as<PodHot>(), m->d_pods.spec.as<ca_pod_spec>(),
                       m->d_pods.terms.as<ca_selector_term>(), m->d_pods.reqs.as<ca_selector_req>(),
                       m->d_pods.names.as<int32_t>(), in.d_hints.as<int32_t>(), d_lin, d_need, d_dest.as<int32_t>(),
                       d_hset.as<int32_t>(), d_out.as<SweepOut>(), d_wl, use_ext ? 1 : 0,
                       m->sw.bsum.as<BlockSum>(), d_chain_list, n_chain, d_chain);
    CA_HIP_CHECK(hipGetLastError());
    return CA_OK;
}

// The sweep proper (DESIGN.md §4 sweep).  hints: per mirror pod, host (in/out; nullable);
// d_pod_hints: the mirror's resident per-pod hints (used and updated instead when
// non-null).  out_dest nullable.
int sweep_core(ca_mirror* m, const SweepCall& in, int32_t* hints, int32_t* d_pod_hints, int32_t* last_index,
               ca_removal_result* results, int32_t* out_dest, SweepPhase* ph = nullptr) {
    const auto t_start = std::chrono::steady_clock::now();
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    auto tmark = [&](const char* what) {
        if (dbg_t)
            fprintf(stderr, "[sweep] %-14s %8.3f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    };
    hipStream_t st = m->stream;
    const int32_t C = in.C, M = in.M, n = in.n;
    const int32_t *candidates = in.cand, *status = in.status, *move_off = in.move_off, *move_pods = in.move_pods;
    int rc;
    // candidates whose simulation can move lastIndex: valid, not blocked, pods to move
    std::vector<int32_t> sens;
    sens.reserve((size_t)C);
    for (int32_t c = 0; c < C; c++) {
        const int32_t nd = candidates[c];
        if (nd < 0 || nd >= n || !in.dest_mask[nd] || status[c] != 0) continue;
        if (move_off[c + 1] - move_off[c] == 0) continue;
        sens.push_back(c);
    }
    const int32_t S = (int32_t)sens.size();
    const int32_t nch = (S + WK - 1) / WK;
    const bool dev_walk = S > 0 && n > 0 && nch <= WALK_MAX_CHUNKS && !knob_env("CASIM_SWEEP_HOST_WALK");

    SweepScratch& sw = m->sw;
    // device scratch: [SweepOut C][walk lout C][info 2][dest M][hint set M] (one D2H; the
    // per-pod part only when the caller wants destinations or host hints),
    // [lin C][need C] (one H2D), [sens S][ws S], table [64][S], trajectories [S][64], chunk maps
    const size_t out_bytes = sizeof(SweepOut) * (size_t)C + sizeof(int32_t) * (2 * (size_t)std::max(M, 1) + C + 2);
    if ((rc = sw.out.reserve(out_bytes)) != CA_OK) return rc;
    if ((rc = sw.h_out.reserve(out_bytes)) != CA_OK) return rc;
    DevView d_out{sw.out.ptr};
    int32_t* const d_wl = reinterpret_cast<int32_t*>(sw.out.as<unsigned char>() + sizeof(SweepOut) * (size_t)C);
    int32_t* const d_info = d_wl + C;
    DevView d_dest{d_info + 2};
    DevView d_hset{d_dest.as<int32_t>() + std::max(M, 1)};
    const SweepOut* outs = sw.h_out.as<SweepOut>();
    const int32_t* h_wl = reinterpret_cast<const int32_t*>(outs + C);
    const int32_t* h_info = h_wl + C;
    const int32_t* h_dest = h_info + 2;
    const int32_t* hset = h_dest + std::max(M, 1);
    const size_t d2h_bytes = (out_dest || hints) ? out_bytes : sizeof(SweepOut) * (size_t)C + sizeof(int32_t) * (C + 2);
    if ((rc = sw.lin.reserve((sizeof(int32_t) + 1) * (size_t)C)) != CA_OK) return rc;
    if ((rc = sw.h_lin.reserve((sizeof(int32_t) + 1) * (size_t)C)) != CA_OK) return rc;
    int32_t* const d_lin = sw.lin.as<int32_t>();
    uint8_t* const d_need = reinterpret_cast<uint8_t*>(d_lin + C);
    int32_t* const h_lin = sw.h_lin.as<int32_t>();
    uint8_t* const h_need = reinterpret_cast<uint8_t*>(h_lin + C);
    const size_t Sx = (size_t)std::max(S, 1);
    if ((rc = sw.todo.reserve(sizeof(int32_t) * 12 * Sx)) != CA_OK) return rc;      // (a host round: 3 rows a candidate)
    {
        void* const was = sw.h_todo.ptr;
        if ((rc = sw.h_todo.reserve(sizeof(int32_t) * 12 * Sx)) != CA_OK) return rc;
        if (sw.h_todo.ptr != was) sw.dmap.clear();
    }
    if ((rc = sw.tab.reserve(sizeof(int32_t) * 64 * Sx)) != CA_OK) return rc;
    if ((rc = sw.h_tab.reserve(sizeof(int32_t) * 64 * Sx)) != CA_OK) return rc;
    if ((rc = sw.wl.reserve(sizeof(int32_t) * (64 * Sx + 64 * (size_t)std::max(nch, 1)))) != CA_OK) return rc;
    if ((rc = sw.tfp.reserve(sizeof(int32_t) * FPW * Sx)) != CA_OK) return rc;
    if ((rc = sw.h_tfp.reserve(sizeof(int32_t) * FPW * Sx)) != CA_OK) return rc;
    if ((rc = sw.vp.reserve(sizeof(int32_t) * ((size_t)n + 1))) != CA_OK) return rc;
    int32_t* const d_tfp = sw.tfp.as<int32_t>();
    int32_t* const h_tfp = sw.h_tfp.as<int32_t>();
    if ((rc = sw.mode.reserve(sizeof(int32_t) * 4)) != CA_OK) return rc;
    int32_t* const d_mode = sw.mode.as<int32_t>();
    int32_t* const d_traj = sw.wl.as<int32_t>();
    int32_t* const d_cmap = d_traj + 64 * Sx;
    int32_t* const tab = sw.h_tab.as<int32_t>();    // [64][S] host copy (host walk only)
    int32_t* const ht = sw.h_todo.as<int32_t>();
    int32_t* const d_sens = sw.todo.as<int32_t>();
    int32_t* const d_ws = d_sens + S;

    // ---- 1. probe: every candidate once, at a rough guess of its lastIndex ----
    // A candidate's outputs depend on its input lastIndex only from its first successful
    // FitsAnyNode scan on (hint checks and failed full scans do not depend on it).  The
    // probe's results are final for every candidate without a successful scan (steady
    // state: the hints of the previous loop place every pod), and for the others its
    // advances calibrate the table windows.
    const int64_t L0 = *last_index;               // raw until the first placement (Go keeps the int)
    std::vector<int32_t> guess((size_t)C, 0);
    {
        int64_t g = ph && ph->kind != SP_FULL ? ph->guess_base : L0;
        int32_t k = 0;
        for (int32_t c = 0; c < C; c++) {
            guess[c] = wrap(g, n);
            if (k < S && sens[k] == c) { g += move_off[c + 1] - move_off[c]; k++; }
        }
    }
    std::memcpy(h_lin, guess.data(), sizeof(int32_t) * C);
    std::memset(h_need, 1, (size_t)C);
    int32_t rounds = 1, exact_runs = 0;
    int32_t* const d_tdoff = d_sens + 2 * (size_t)S;     // per sensitive candidate: its pods in tdest
    int64_t tpods = 0;
    if (S > 0 && n > 0) {
        rounds++;
        std::memcpy(ht, sens.data(), sizeof(int32_t) * S);
        for (int32_t k = 0; k < S; k++) {
            const int32_t mn = move_off[sens[k] + 1] - move_off[sens[k]];
            ht[2 * S + k] = (int32_t)tpods;
            tpods += mn <= TB_MAXP ? mn : 0;
        }
        if (dev_walk) {
            if ((rc = sw.tev.reserve(sizeof(uint32_t) * 64 * Sx)) != CA_OK) return rc;
            if ((rc = sw.tdest.reserve(sizeof(int32_t) * 64 * (size_t)std::max<int64_t>(tpods, 1))) != CA_OK) return rc;
        }
    }
    if ((rc = sw.bsum.reserve(sizeof(BlockSum) * (size_t)std::max((n + 63) / 64, 1))) != CA_OK) return rc;
    if ((rc = sw.h_l0.reserve(sizeof(int32_t) * 4)) != CA_OK) return rc;
    // -> mode[2]: the chain's input (k_sweep_est, k_walk_resolve); a range's SP_MAP centres
    // its windows on the estimate of its input instead
    sw.h_l0.as<int32_t>()[0] = n > 0 ? wrap(ph && ph->kind == SP_MAP ? (int64_t)ph->est_base : L0, n) : 0;
    if (ph) ph->n_sensitive = S;
    const bool use_ext = m->n_ext_pods > 0;
    if (use_ext && (rc = ensure_dyn_lds((const void*)k_sweep, sizeof(OverlayExt))) != CA_OK) return rc;
    const size_t wr_bytes = sizeof(int32_t) * (size_t)nch * (64 + FPW);
    if (dev_walk && (rc = ensure_dyn_lds((const void*)k_walk_resolve,
                                         sizeof(int32_t) * (size_t)WALK_MAX_CHUNKS * (64 + FPW))) != CA_OK)
        return rc;
    if (dev_walk && ph && ph->kind == SP_MAP &&
        (rc = ensure_dyn_lds((const void*)k_walk_map, sizeof(int32_t) * (size_t)WALK_MAX_CHUNKS * (64 + FPW))) != CA_OK)
        return rc;
    // the resident hints: applied behind the exact pass, while the results travel (a host
    // walk below re-runs candidates and applies them again; its exact passes read the
    // gathered copy, not the resident table)
    auto apply_hints = [&]() -> int {
        if (d_pod_hints && M > 0) {
            hipLaunchKernelGGL(k_hints_apply, dim3((M + 255) / 256), dim3(256), 0, st, d_hset.as<int32_t>(),
                               in.d_moves.as<int32_t>(), M, d_pod_hints);
            CA_HIP_CHECK(hipGetLastError());
        }
        return CA_OK;
    };
    // ---- 1-3: the device pipeline (no host round trip in the common case) ----
    auto enqueue = [&]() -> int {
        int e;
        CA_HIP_CHECK(hipMemcpyAsync(d_lin, h_lin, (sizeof(int32_t) + 1) * (size_t)C, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipMemcpyAsync(d_mode + 2, sw.h_l0.ptr, sizeof(int32_t), hipMemcpyHostToDevice, st));
        if (d_pod_hints && M > 0) {
            hipLaunchKernelGGL(k_hints_gather, dim3((M + 255) / 256), dim3(256), 0, st, d_pod_hints,
                               in.d_moves.as<int32_t>(), M, in.d_hints.as<int32_t>());
            CA_HIP_CHECK(hipGetLastError());
        }
        if (n > 0) {
            hipLaunchKernelGGL(k_block_sum, dim3((n + 63) / 64), dim3(64), 0, st, m->d_hot.as<NodeHot>(),
                               in.d_mask.as<uint8_t>(), n, sw.bsum.as<BlockSum>());
            CA_HIP_CHECK(hipGetLastError());
        }
        // 1. probe: every candidate once, at a rough guess of its lastIndex
        if ((e = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl)) != CA_OK) return e;
        if (S > 0 && n > 0) {
            // 2. first table round, windows centred on the probe's advances
            CA_HIP_CHECK(hipMemcpyAsync(d_sens, ht, sizeof(int32_t) * S, hipMemcpyHostToDevice, st));
            CA_HIP_CHECK(hipMemcpyAsync(d_tdoff, ht + 2 * S, sizeof(int32_t) * S, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_sweep_est, dim3(1), dim3(1024), 0, st, d_out.as<SweepOut>(), d_sens, S, n, d_ws, d_mode,
                               m->d_hot.as<NodeHot>(), in.d_mask.as<uint8_t>(), dev_walk ? sw.vp.as<int32_t>() : nullptr);
            CA_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_sweep_table, dim3(S), dim3(64), 0, st, m->d_hot.as<NodeHot>(),
                               m->d_static.as<NodeStatic>(), n, in.d_mask.as<uint8_t>(), in.d_c.as<int32_t>(),
                               in.d_off.as<int32_t>(), in.d_moves.as<int32_t>(), m->d_pods.hot.as<PodHot>(),
                               m->d_pods.spec.as<ca_pod_spec>(), m->d_pods.terms.as<ca_selector_term>(),
                               m->d_pods.reqs.as<ca_selector_req>(), m->d_pods.names.as<int32_t>(),
                               in.d_hints.as<int32_t>(), d_sens, d_ws, (const int32_t*)nullptr, sw.tab.as<int32_t>(), S,
                               dev_walk ? sw.tev.as<uint32_t>() : nullptr, dev_walk ? sw.tdest.as<int32_t>() : nullptr,
                               dev_walk ? (const int32_t*)d_tdoff : nullptr, d_tfp, (const int32_t*)d_mode,
                               sw.bsum.as<BlockSum>());
            CA_HIP_CHECK(hipGetLastError());
        }
        if (dev_walk) {
            // 3. device walk, then the exact pass at the exact lastIndex values
            CA_HIP_CHECK(hipMemsetAsync(d_need, 0, (size_t)C, st));
            hipLaunchKernelGGL(k_walk_chunks, dim3(nch), dim3(64), 0, st, d_sens, d_ws, d_lin, d_wl, sw.tab.as<int32_t>(),
                               d_tfp, d_mode, S, n, d_cmap, d_traj);
            CA_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_walk_resolve, dim3(1), dim3(1024), wr_bytes, st, d_sens, d_tfp, d_cmap, d_traj, d_wl,
                               d_mode, S, n, d_lin, d_need, d_info);
            CA_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_table_gather, dim3(S), dim3(64), 0, st, d_sens, d_tfp, sw.vp.as<int32_t>(),
                               in.d_c.as<int32_t>(), in.d_mask.as<uint8_t>(), m->d_hot.as<NodeHot>(), S, n, d_lin, d_need,
                               sw.tab.as<int32_t>(), sw.tev.as<uint32_t>(), sw.tdest.as<int32_t>(), d_tdoff,
                               in.d_off.as<int32_t>(), d_out.as<SweepOut>(), d_dest.as<int32_t>(), d_hset.as<int32_t>(),
                               d_wl, d_mode);
            CA_HIP_CHECK(hipGetLastError());
            if ((e = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl)) != CA_OK) return e;
        }
        if ((e = apply_hints()) != CA_OK) return e;
        CA_HIP_CHECK(hipMemcpyAsync(sw.h_out.ptr, sw.out.ptr, d2h_bytes, hipMemcpyDeviceToHost, st));
        return CA_OK;
    };
    // ---- the three calls of a multi-device range (SweepPhase above) ----
    auto enqueue_phase = [&]() -> int {
        int e;
        CA_HIP_CHECK(hipMemcpyAsync(d_lin, h_lin, (sizeof(int32_t) + 1) * (size_t)C, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipMemcpyAsync(d_mode + 2, sw.h_l0.ptr, sizeof(int32_t), hipMemcpyHostToDevice, st));
        if (ph->kind == SP_PROBE) {
            if (d_pod_hints && M > 0) {
                hipLaunchKernelGGL(k_hints_gather, dim3((M + 255) / 256), dim3(256), 0, st, d_pod_hints,
                                   in.d_moves.as<int32_t>(), M, in.d_hints.as<int32_t>());
                CA_HIP_CHECK(hipGetLastError());
            }
            if (n > 0) {
                hipLaunchKernelGGL(k_block_sum, dim3((n + 63) / 64), dim3(64), 0, st, m->d_hot.as<NodeHot>(),
                                   in.d_mask.as<uint8_t>(), n, sw.bsum.as<BlockSum>());
                CA_HIP_CHECK(hipGetLastError());
            }
            if ((e = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl)) != CA_OK) return e;
            CA_HIP_CHECK(hipMemcpyAsync(sw.h_out.ptr, sw.out.ptr, sizeof(SweepOut) * (size_t)C, hipMemcpyDeviceToHost, st));
            return CA_OK;
        }
        if (ph->kind == SP_MAP) {
            ph->map_ran = 0;
            if (!(S > 0 && n > 0)) return CA_OK;
            ph->map_ran = 1;
            CA_HIP_CHECK(hipMemcpyAsync(d_sens, ht, sizeof(int32_t) * S, hipMemcpyHostToDevice, st));
            CA_HIP_CHECK(hipMemcpyAsync(d_tdoff, ht + 2 * S, sizeof(int32_t) * S, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_sweep_est, dim3(1), dim3(1024), 0, st, d_out.as<SweepOut>(), d_sens, S, n, d_ws, d_mode,
                               m->d_hot.as<NodeHot>(), in.d_mask.as<uint8_t>(), dev_walk ? sw.vp.as<int32_t>() : nullptr);
            CA_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_sweep_table, dim3(S), dim3(64), 0, st, m->d_hot.as<NodeHot>(),
                               m->d_static.as<NodeStatic>(), n, in.d_mask.as<uint8_t>(), in.d_c.as<int32_t>(),
                               in.d_off.as<int32_t>(), in.d_moves.as<int32_t>(), m->d_pods.hot.as<PodHot>(),
                               m->d_pods.spec.as<ca_pod_spec>(), m->d_pods.terms.as<ca_selector_term>(),
                               m->d_pods.reqs.as<ca_selector_req>(), m->d_pods.names.as<int32_t>(),
                               in.d_hints.as<int32_t>(), d_sens, d_ws, (const int32_t*)nullptr, sw.tab.as<int32_t>(), S,
                               dev_walk ? sw.tev.as<uint32_t>() : nullptr, dev_walk ? sw.tdest.as<int32_t>() : nullptr,
                               dev_walk ? (const int32_t*)d_tdoff : nullptr, d_tfp, (const int32_t*)d_mode,
                               sw.bsum.as<BlockSum>());
            CA_HIP_CHECK(hipGetLastError());
            if (!dev_walk) return CA_OK;            // (the range's resolve walks on the host)
            CA_HIP_CHECK(hipMemsetAsync(d_need, 0, (size_t)C, st));
            hipLaunchKernelGGL(k_walk_chunks, dim3(nch), dim3(64), 0, st, d_sens, d_ws, d_lin, d_wl, sw.tab.as<int32_t>(),
                               d_tfp, d_mode, S, n, d_cmap, d_traj);
            CA_HIP_CHECK(hipGetLastError());
            if ((e = sw.bmap.reserve(sizeof(int32_t) * SWEEP_MAP_INTS)) != CA_OK) return e;
            if ((e = sw.h_bmap.reserve(sizeof(int32_t) * SWEEP_MAP_INTS)) != CA_OK) return e;
            hipLaunchKernelGGL(k_walk_map, dim3(1), dim3(1024), wr_bytes, st, d_tfp, d_cmap, d_mode, S, n,
                               sw.bmap.as<int32_t>());
            CA_HIP_CHECK(hipGetLastError());
            CA_HIP_CHECK(hipMemcpyAsync(sw.h_bmap.ptr, sw.bmap.ptr, sizeof(int32_t) * SWEEP_MAP_INTS, hipMemcpyDeviceToHost,
                                        st));
            return CA_OK;
        }
        // SP_RESOLVE: the tail of enqueue() from the true input (mode[2]); it reads the
        // tables and chunk maps this range's SP_MAP built (multi.hip maps every range with
        // sensitive candidates), never an earlier call's
        if (S > 0 && n > 0 && !ph->map_ran) {
            set_last_error("sweep resolve phase without this call's map phase");
            return CA_EINVAL;
        }
        if (dev_walk) {
            // (the probe's results for the candidates the walk does not re-run stay in d_out;
            // d_lin was re-uploaded with the same guesses, need = 0 as the map phase left it)
            CA_HIP_CHECK(hipMemsetAsync(d_need, 0, (size_t)C, st));
            hipLaunchKernelGGL(k_walk_resolve, dim3(1), dim3(1024), wr_bytes, st, d_sens, d_tfp, d_cmap, d_traj, d_wl,
                               d_mode, S, n, d_lin, d_need, d_info);
            CA_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_table_gather, dim3(S), dim3(64), 0, st, d_sens, d_tfp, sw.vp.as<int32_t>(),
                               in.d_c.as<int32_t>(), in.d_mask.as<uint8_t>(), m->d_hot.as<NodeHot>(), S, n, d_lin, d_need,
                               sw.tab.as<int32_t>(), sw.tev.as<uint32_t>(), sw.tdest.as<int32_t>(), d_tdoff,
                               in.d_off.as<int32_t>(), d_out.as<SweepOut>(), d_dest.as<int32_t>(), d_hset.as<int32_t>(),
                               d_wl, d_mode);
            CA_HIP_CHECK(hipGetLastError());
            if ((e = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl)) != CA_OK) return e;
        }
        if ((e = apply_hints()) != CA_OK) return e;
        CA_HIP_CHECK(hipMemcpyAsync(sw.h_out.ptr, sw.out.ptr, d2h_bytes, hipMemcpyDeviceToHost, st));
        return CA_OK;
    };
    // The pipeline is a dozen launches and copies whose arguments depend only on the call's
    // shape (sizes, buffers, flags): a call with the shape of the previous one replays it
    // as a HIP graph captured on the second such call (no per-launch host cost, no gaps
    // between the kernels).  Everything that varies per call is read from the page-locked
    // inputs when the graph runs.  CASIM_NO_GRAPH: eager launches always.
    uint64_t gkey = 1469598103934665603ull;
    {
        const uint64_t v[] = {(uint64_t)(uintptr_t)m, (uint64_t)C, (uint64_t)M, (uint64_t)n, (uint64_t)S, (uint64_t)nch,
                              (uint64_t)dev_walk, (uint64_t)use_ext, (uint64_t)tpods, (uint64_t)d2h_bytes,
                              (uint64_t)(uintptr_t)d_pod_hints, (uint64_t)(uintptr_t)h_lin, (uint64_t)(uintptr_t)ht,
                              (uint64_t)(uintptr_t)sw.h_l0.ptr, (uint64_t)(uintptr_t)sw.h_out.ptr,
                              (uint64_t)(uintptr_t)sw.out.ptr, (uint64_t)(uintptr_t)sw.lin.ptr,
                              (uint64_t)(uintptr_t)sw.todo.ptr, (uint64_t)(uintptr_t)sw.tab.ptr,
                              (uint64_t)(uintptr_t)sw.wl.ptr, (uint64_t)(uintptr_t)sw.tev.ptr,
                              (uint64_t)(uintptr_t)sw.tdest.ptr, (uint64_t)(uintptr_t)sw.tfp.ptr,
                              (uint64_t)(uintptr_t)sw.vp.ptr, (uint64_t)(uintptr_t)sw.mode.ptr,
                              (uint64_t)(uintptr_t)sw.bsum.ptr, (uint64_t)(uintptr_t)m->d_hot.ptr,
                              (uint64_t)(uintptr_t)m->d_ext.ptr, (uint64_t)(uintptr_t)m->d_static.ptr,
                              (uint64_t)(uintptr_t)m->d_pods.hot.ptr, (uint64_t)(uintptr_t)m->d_pods.spec.ptr,
                              (uint64_t)(uintptr_t)m->d_pods.terms.ptr, (uint64_t)(uintptr_t)m->d_pods.reqs.ptr,
                              (uint64_t)(uintptr_t)m->d_pods.names.ptr, (uint64_t)(uintptr_t)in.d_mask.ptr,
                              (uint64_t)(uintptr_t)in.d_c.ptr, (uint64_t)(uintptr_t)in.d_status.ptr,
                              (uint64_t)(uintptr_t)in.d_off.ptr, (uint64_t)(uintptr_t)in.d_moves.ptr,
                              (uint64_t)(uintptr_t)in.d_hints.ptr, (uint64_t)(uintptr_t)st};
        for (uint64_t x : v) { gkey ^= x; gkey *= 1099511628211ull; }
    }
    // Serial-only call: every candidate in one k_sweep chain launch (no probe, tables or
    // walk).  Taken when the previous call of this mirror resolved most of its sensitive
    // candidates through the serial chain anyway (the planner's late windows), and kept
    // while it costs less per candidate than the last pipeline call (re-measured at least
    // every 8 calls); windows of at most 2 048 candidates only.
    // (CASIM_SWEEP_SERIAL: every call serial-only; CASIM_NO_SERIAL_CHAIN: never; tests)
    // The mode carries over only to a call of the same shape — candidates and sensitive
    // candidates within a factor of two of the call that measured it, most of them
    // sensitive — not to an unrelated call on the same mirror.
    const bool same_shape = C <= 2 * sw.serial_C && 2 * C >= sw.serial_C && S <= 2 * sw.serial_S &&
                            2 * S >= sw.serial_S && 2 * S >= C;
    const bool serial_only = !(ph && ph->kind != SP_FULL) && S > 0 && n > 0 && !knob_env("CASIM_NO_SERIAL_CHAIN") &&
                             ((C <= 2048 && sw.serial_next && same_shape) || knob_env("CASIM_SWEEP_SERIAL") != nullptr);
    auto enqueue_serial = [&]() -> int {
        int e;
        if ((e = sw.chainl.reserve(sizeof(int32_t) * (size_t)C)) != CA_OK) return e;
        if ((e = sw.h_chainl.reserve(sizeof(int32_t) * (size_t)C)) != CA_OK) return e;
        int32_t* const cl = sw.h_chainl.as<int32_t>();
        for (int32_t c = 0; c < C; c++) cl[c] = c;
        int32_t* const hc = sw.h_l0.as<int32_t>() + 1;
        hc[0] = (int32_t)L0;
        CA_HIP_CHECK(hipMemcpyAsync(sw.chainl.ptr, cl, sizeof(int32_t) * (size_t)C, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipMemcpyAsync(d_mode + 3, hc, sizeof(int32_t), hipMemcpyHostToDevice, st));
        if (d_pod_hints && M > 0) {
            hipLaunchKernelGGL(k_hints_gather, dim3((M + 255) / 256), dim3(256), 0, st, d_pod_hints,
                               in.d_moves.as<int32_t>(), M, in.d_hints.as<int32_t>());
            CA_HIP_CHECK(hipGetLastError());
        }
        hipLaunchKernelGGL(k_block_sum, dim3((n + 63) / 64), dim3(64), 0, st, m->d_hot.as<NodeHot>(),
                           in.d_mask.as<uint8_t>(), n, sw.bsum.as<BlockSum>());
        CA_HIP_CHECK(hipGetLastError());
        if ((e = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl, sw.chainl.as<int32_t>(), C,
                              d_mode + 3)) != CA_OK)
            return e;
        if ((e = apply_hints()) != CA_OK) return e;
        CA_HIP_CHECK(hipMemcpyAsync(sw.h_out.ptr, sw.out.ptr, d2h_bytes, hipMemcpyDeviceToHost, st));
        return CA_OK;
    };
    static const bool no_graph = knob_env("CASIM_NO_GRAPH") != nullptr;
    CA_HIP_CHECK(hipEventRecord(m->ev0, st));
    const bool phased = ph && ph->kind != SP_FULL;
    if (phased) {
        if ((rc = enqueue_phase()) != CA_OK) return rc;
    } else if (serial_only) {
        if ((rc = enqueue_serial()) != CA_OK) return rc;
    } else if (!no_graph && sw.gexec && sw.gkey == gkey) {
        CA_HIP_CHECK(hipGraphLaunch(sw.gexec, st));
    } else if (!no_graph && sw.gseen == gkey) {
        if (sw.gexec) { (void)hipGraphExecDestroy(sw.gexec); sw.gexec = nullptr; }
        hipGraph_t graph = nullptr;
        CA_HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        const int erc = enqueue();
        const hipError_t ce = hipStreamEndCapture(st, &graph);
        if (erc != CA_OK) { if (graph) (void)hipGraphDestroy(graph); return erc; }
        if (ce != hipSuccess) { set_last_error(hipGetErrorString(ce)); return CA_EDEVICE; }
        const hipError_t ie = hipGraphInstantiate(&sw.gexec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ie != hipSuccess) { sw.gexec = nullptr; set_last_error(hipGetErrorString(ie)); return CA_EDEVICE; }
        sw.gkey = gkey;
        CA_HIP_CHECK(hipGraphLaunch(sw.gexec, st));
    } else {
        if ((rc = enqueue()) != CA_OK) return rc;
        sw.gseen = gkey;
    }
    CA_HIP_CHECK(hipEventRecord(m->ev1, st));
    CA_HIP_CHECK(hipStreamSynchronize(st));
    if (phased && ph->kind == SP_PROBE) {
        // the range's advance as k_sweep_est sums it (successful scans only)
        int64_t adv = 0;
        int32_t succ = 0;
        for (int32_t k = 0; k < S; k++) {
            const SweepOut& o = outs[sens[k]];
            if (!o.fa_success) continue;
            succ++;
            int64_t d = ((int64_t)o.lout - (int64_t)o.lin) % n;
            if (d < 0) d += n;
            adv += d;
        }
        ph->adv = adv;
        ph->succ = succ;
        return CA_OK;
    }
    if (phased && ph->kind == SP_MAP) {
        ph->map_ok = (S > 0 && n > 0 && dev_walk) ? 1 : 0;
        if (ph->map_ok) std::memcpy(ph->map, sw.h_bmap.ptr, sizeof(int32_t) * SWEEP_MAP_INTS);
        return CA_OK;
    }
    float kms = 0;
    {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, m->ev0, m->ev1);
        kms += ms;
        if (dbg_t) fprintf(stderr, "[sweep] device %s: %d sensitive, kernels %.3f ms\n",
                           serial_only ? "serial chain (all candidates)" : "pipeline", S, ms);
        tmark("device");
    }
    // ---- 4. host walk from where the device walk stopped (or of everything) ----
    int32_t k0 = serial_only ? S : dev_walk ? h_info[0] : 0;   // first sensitive candidate not yet resolved
    int64_t cur = dev_walk ? (int64_t)h_info[1] : L0;
    if (dev_walk && k0 == 0) cur = L0;
    int32_t chained = 0;
    if (k0 < S) {
        std::vector<int32_t> ws((size_t)S, 0);
        std::vector<int32_t> wlc((size_t)C, 0);
        std::memcpy(wlc.data(), h_wl, sizeof(int32_t) * C);   // the probe's walk values (h_out is reused below)
        CA_HIP_CHECK(hipMemcpyAsync(tab, sw.tab.ptr, sizeof(int32_t) * 64 * (size_t)S, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipMemcpyAsync(h_tfp, d_tfp, sizeof(int32_t) * FPW * (size_t)S, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipMemcpyAsync(ht, d_ws, sizeof(int32_t) * S, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipStreamSynchronize(st));
        for (int32_t k = 0; k < S; k++) ws[k] = ht[k];
        // final[c] = 0: re-run at exact_lin in one exact pass
        std::vector<int32_t> exact_lin((size_t)C, 0);
        std::vector<uint8_t> final_((size_t)C, 1);
        std::vector<uint8_t> have((size_t)S, 1);
        std::vector<int32_t> todo, todo_ws, todo_k, todo_slot;
        // Side rows: a row whose estimate lies within SIDE_BAND classes of one of its edges gets
        // the adjacent window on that side in the next round (overlapping it by 8 mean gaps),
        // so an exact input that drifts a few positions past the edge still finds its class
        // instead of costing another round (C5: most misses fell 2-28 positions outside the
        // 64-wide windows).  Rows are not free — past ~500 a round's kernel grows — so one side
        // per row, near-edge rows only (C5 RunOnce sweep: 16 / 24 / 32 classes read 2.85 /
        // 2.6 / 3.0 ms, both sides at 16: 3.1, none: 3.5).
        const bool sides = !knob_env("CASIM_SWEEP_NO_SIDE_ROWS");
        // CASIM_SWEEP_RECENTRE_SIDES=1/2/3: a re-centred row gets its side row below / above /
        // both in the same round as its main row (A/B of wider windows for the drifting estimates)
        const int recentre_sides = knob_env("CASIM_SWEEP_RECENTRE_SIDES") ? atoi(knob_env("CASIM_SWEEP_RECENTRE_SIDES")) & 3 : 0;
#ifndef CASIM_SIDE_BAND
#define CASIM_SIDE_BAND 24
#endif
        constexpr int32_t SIDE_BAND = CASIM_SIDE_BAND;
        std::vector<uint8_t> have_side((size_t)S, 0), want_side((size_t)S, 0);   // want_side: bit 0 below, bit 1 above
        std::vector<int32_t> gapk((size_t)S, 1);
        std::vector<int32_t> dbg_rc;                // (CASIM_DEBUG_TIMING) round that re-centred each row
        int32_t dbg_first_rc = -1;                   // ... and the first row the last pass re-centred
        if (dbg_t) dbg_rc.assign((size_t)S, 0);
        // Where each candidate's rows are: the first pipeline's table ([64][S] values and
        // [FPW][S] fit points, copied once), or the compact rows of the table round that
        // rebuilt them, read in place in that round's page-locked buffer ([64][T], [FPW][T]:
        // the kernel writes them there, zero-copy) — no scatter of every round's rows into
        // one host table.  Slot 0: the main row, 1 / 2: the side rows below / above.
        struct RowRef {
            const int32_t* v;      // value of class w: v[w * s]
            const int32_t* f;      // fit point i: f[i * s]
            int32_t s;
        };
        std::vector<RowRef> rref((size_t)3 * S);
        for (int32_t k = 0; k < S; k++) rref[k] = RowRef{tab + k, h_tfp + k, S};
        RowRef* const mref = rref.data();
        int32_t round_buf = 0;                     // this call's table rounds so far (sw.rbuf)
        // the class of input L in candidate k's rows (main, then the sides), and that row
        auto lookup = [&](int32_t k, int32_t L, const RowRef*& rr) -> int32_t {
            rr = &mref[k];
            int32_t w = fp_class(rr->f, rr->s, n, L);
            if (w >= 0 || !have_side[k]) return w;
            for (int sd = 0; sd < 2; sd++) {
                if (!((have_side[k] >> sd) & 1)) continue;
                const RowRef* q = &rref[(size_t)(1 + sd) * S + k];
                w = fp_class(q->f, q->s, n, L);
                if (w >= 0) { rr = q; return w; }
            }
            return -1;
        };
        auto insensitive = [&](int32_t k) { return wlc[sens[k]] < 0; };
        // the device walk's re-runs already happened: only candidates from k0 on remain
        // each round looks LOOKAHEAD candidates ahead: the estimates drift with the distance
        // from the exact lastIndex, so rows further out would be re-centred again anyway
#ifndef CASIM_SWEEP_LOOKAHEAD_ROWS
#define CASIM_SWEEP_LOOKAHEAD_ROWS 512
#endif
        static const int32_t LOOKAHEAD = knob_env("CASIM_SWEEP_LOOKAHEAD") ? std::max(64, atoi(knob_env("CASIM_SWEEP_LOOKAHEAD")))
                                                                          : CASIM_SWEEP_LOOKAHEAD_ROWS;
        // Serial exact chain: when a table round resolves few candidates for its cost (late
        // planner windows over a nearly full cluster: long scans that no lane budget covers,
        // windows that miss again after every re-centring), the next candidates run exactly
        // in one launch: one workgroup walks them in order, each from the lastIndex the
        // previous one left (k_sweep chain mode), and one sync ends the batch.
        // Batches double while the tables keep losing; the costs compared are measured.
        double chain_ms_per = 0.03;          // per candidate; re-measured after each batch
        int32_t chain_batch = 64;
        int32_t* const h_chain = sw.h_l0.as<int32_t>() + 1;
        auto run_chain = [&](int32_t kend) -> int {
            const auto tc = std::chrono::steady_clock::now();
            h_chain[0] = (int32_t)cur;
            CA_HIP_CHECK(hipMemcpyAsync(d_mode + 3, h_chain, sizeof(int32_t), hipMemcpyHostToDevice, st));
            int32_t runs = 0;
            int e;
            if ((e = sw.chainl.reserve(sizeof(int32_t) * (size_t)std::max(kend - k0, 1))) != CA_OK) return e;
            if ((e = sw.h_chainl.reserve(sizeof(int32_t) * (size_t)std::max(kend - k0, 1))) != CA_OK) return e;
            int32_t* const cl = sw.h_chainl.as<int32_t>();
            for (int32_t k = k0; k < kend; k++)
                if (!insensitive(k)) cl[runs++] = sens[k];                          // others pass lastIndex through
            if (runs > 0) {
                CA_HIP_CHECK(hipMemcpyAsync(sw.chainl.ptr, cl, sizeof(int32_t) * (size_t)runs, hipMemcpyHostToDevice, st));
                if ((e = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl, sw.chainl.as<int32_t>(),
                                      runs, d_mode + 3)) != CA_OK)
                    return e;
            }
            CA_HIP_CHECK(hipMemcpyAsync(h_chain + 1, d_mode + 3, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            CA_HIP_CHECK(hipStreamSynchronize(st));
            cur = runs > 0 ? (int64_t)h_chain[1] : cur;
            chained += runs;
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count();
            if (runs > 0) chain_ms_per = ms / runs;
            if (dbg_t) {
                std::vector<SweepOut> o((size_t)C);
                CA_HIP_CHECK(hipMemcpy(o.data(), d_out.ptr, sizeof(SweepOut) * (size_t)C, hipMemcpyDeviceToHost));
                uint64_t ticks = 0, ev = 0, pl = 0;
                for (int32_t k = k0; k < kend; k++)
                    if (!insensitive(k)) { ticks += o[sens[k]].pad2; ev += o[sens[k]].evals; pl += o[sens[k]].n_placed; }
                fprintf(stderr, "[sweep] serial chain [%d,%d): %d runs, %.3f ms, in-kernel %.3f ms, %llu evals, %llu placed\n",
                        k0, kend, runs, ms, ticks * 1e-5, (unsigned long long)ev, (unsigned long long)pl);
            }
            k0 = kend;
            return CA_OK;
        };
        while (k0 < S) {
            const auto t_round = std::chrono::steady_clock::now();
            const int32_t k_round = k0;
            todo.clear(); todo_ws.clear(); todo_k.clear(); todo_slot.clear();
            const int32_t kend = std::min(S, k0 + LOOKAHEAD);
            for (int32_t k = k0; k < kend; k++) {
                if (insensitive(k)) continue;
                if (!have[k]) { todo.push_back(sens[k]); todo_ws.push_back(ws[k]); todo_k.push_back(k); todo_slot.push_back(0); }
                if (sides && want_side[k] && !have_side[k]) {
                    const int64_t sh = 56 * (int64_t)gapk[k];
                    for (int sd = 0; sd < 2; sd++) {
                        if (!((want_side[k] >> sd) & 1)) continue;
                        todo.push_back(sens[k]); todo_ws.push_back(wrap((int64_t)ws[k] + (sd ? sh : -sh), n));
                        todo_k.push_back(k); todo_slot.push_back(1 + sd);
                    }
                }
            }
            if (!todo.empty()) {
                rounds++;
                const int32_t T = (int32_t)todo.size();
                std::memcpy(ht, todo.data(), sizeof(int32_t) * T);
                std::memcpy(ht + T, todo_ws.data(), sizeof(int32_t) * T);
                std::memcpy(ht + 2 * T, todo_k.data(), sizeof(int32_t) * T);
                // zero-copy both ways: the kernel reads the rows to build from the page-locked
                // staging and writes the compact rows straight into this round's host buffer (no
                // copy launches around a 40 µs kernel; the round trip is what a round costs).
                // The round buffers are kept for the call (the walk reads the rows in place) and
                // pooled across calls, each sized once for a full round (LOOKAHEAD main rows
                // and their two side rows) so a later call never regrows one.
                if ((int32_t)sw.rbuf.size() <= round_buf) sw.rbuf.emplace_back();
                HostBuf& rbuf = sw.rbuf[round_buf++];
                void* const rb_was = rbuf.ptr;
                if ((rc = rbuf.reserve(sizeof(int32_t) * (64 + FPW) * (size_t)std::max(T, 3 * LOOKAHEAD))) != CA_OK)
                    return rc;
                if (rbuf.ptr != rb_was) sw.dmap.clear();
                int32_t* const ct = rbuf.as<int32_t>();
                void *d_ht = nullptr, *d_ct = nullptr;
                // (the device mappings of the staging and of each pooled round buffer, looked
                // up once per buffer: the runtime's lookup is a few µs per call)
                auto dev_of = [&](void* h, void*& d) -> bool {
                    for (const auto& e : sw.dmap)
                        if (e.first == h) { d = e.second; return true; }
                    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return false;
                    sw.dmap.emplace_back(h, d);
                    return true;
                };
                const bool zc = !knob_env("CASIM_SWEEP_COPY_ROUNDS") && dev_of(ht, d_ht) && dev_of(ct, d_ct);
                if (!zc) {
                    (void)hipGetLastError();
                    CA_HIP_CHECK(hipMemcpyAsync(sw.todo.ptr, ht, sizeof(int32_t) * 3 * T, hipMemcpyHostToDevice, st));
                }
                const int32_t* const k_todo = zc ? static_cast<const int32_t*>(d_ht) : sw.todo.as<int32_t>();
                int32_t* const k_tab = zc ? static_cast<int32_t*>(d_ct) : sw.tab.as<int32_t>();
                int32_t* const k_tfp = zc ? static_cast<int32_t*>(d_ct) + 64 * (size_t)T : d_tfp;
                CA_HIP_CHECK(hipEventRecord(m->ev0, st));
                hipLaunchKernelGGL(k_sweep_table, dim3(T), dim3(64), 0, st, m->d_hot.as<NodeHot>(),
                                   m->d_static.as<NodeStatic>(), n, in.d_mask.as<uint8_t>(), in.d_c.as<int32_t>(),
                                   in.d_off.as<int32_t>(), in.d_moves.as<int32_t>(), m->d_pods.hot.as<PodHot>(),
                                   m->d_pods.spec.as<ca_pod_spec>(), m->d_pods.terms.as<ca_selector_term>(),
                                   m->d_pods.reqs.as<ca_selector_req>(), m->d_pods.names.as<int32_t>(),
                                   in.d_hints.as<int32_t>(), k_todo, k_todo + T,
                                   (const int32_t*)nullptr, k_tab, T, nullptr, nullptr, nullptr, k_tfp,
                                   (const int32_t*)d_mode, sw.bsum.as<BlockSum>());
                CA_HIP_CHECK(hipGetLastError());
                CA_HIP_CHECK(hipEventRecord(m->ev1, st));
                tmark("table launched");
                // compact rows (row t of this round): only they cross PCIe, then go to their
                // places in the host copy, stored [lane][candidate] so the walk, whose class
                // stays near the centre, reads it nearly sequentially
                if (!zc) {
                    CA_HIP_CHECK(hipMemcpyAsync(ct, sw.tab.ptr, sizeof(int32_t) * 64 * (size_t)T, hipMemcpyDeviceToHost, st));
                    CA_HIP_CHECK(hipMemcpyAsync(ct + 64 * (size_t)T, d_tfp, sizeof(int32_t) * FPW * (size_t)T,
                                                hipMemcpyDeviceToHost, st));
                }
                CA_HIP_CHECK(hipStreamSynchronize(st));
                tmark("table sync");
                const int32_t* ctf = ct + 64 * (size_t)T;
                // the candidates' rows now live in this round's buffer (row t: column t)
                for (int32_t t = 0; t < T; t++)
                    rref[(size_t)todo_slot[t] * S + todo_k[t]] = RowRef{ct + t, ctf + t, T};
                for (int32_t t = 0; t < T; t++)
                    if (todo_slot[t] != 0) { have_side[todo_k[t]] |= (uint8_t)(1 << (todo_slot[t] - 1)); want_side[todo_k[t]] = 0; }
                float ms = 0;
                (void)hipEventElapsedTime(&ms, m->ev0, m->ev1);
                kms += ms;
                if (dbg_t) fprintf(stderr, "[sweep] table round %d: %d rows, kernel %.3f ms\n", rounds, T, ms);
                tmark("table");
            }
            for (int32_t k = k0; k < kend; k++) have[k] = 1;
            // walk the exact chain as far as the windows reach
            for (; k0 < S; k0++) {
                const int32_t c = sens[k0];
                const int32_t wlv = wlc[c];
                exact_lin[c] = (int32_t)cur;
                if (wlv < 0) continue;                                             // lastIndex passes through
                if (wrap(cur, n) == guess[c]) { cur = wlv; continue; }            // probed at the true value
                const RowRef* rr = nullptr;
                const int32_t w = lookup(k0, wrap(cur, n), rr);
                if (w < 0) {
                    if (dbg_t) {                  // where the exact input fell against the row's window
                        const int32_t* fp = mref[k0].f;
                        const int32_t lo = fp[0], hi = fp[(size_t)64 * mref[k0].s];
                        const int32_t gap = std::max(1, wrap((int64_t)hi - lo, n) / 64);
                        fprintf(stderr, "[sweep] miss at %d: input %d, window [%d, %d] (gap %d): %+d gaps from its start"
                                        " (row re-centred in round %d; %d rows after the last pass's first re-centred %d)\n",
                                k0, wrap(cur, n), lo, hi, gap, (int)(wrap((int64_t)wrap(cur, n) - lo + n / 2, n) - n / 2) / gap,
                                dbg_rc[k0], k0 - dbg_first_rc, dbg_first_rc);
                    }
                    break;
                }
                int32_t v = rr->v[(size_t)w * rr->s];
                if (v == TB_UNKNOWN) {
                    // hints / ports / long scans: exact kernel at the exact lastIndex, alone
                    std::memset(h_need, 0, (size_t)C);
                    h_need[c] = 1;
                    h_lin[c] = (int32_t)cur;
                    CA_HIP_CHECK(hipMemcpyAsync(d_lin, h_lin, (sizeof(int32_t) + 1) * (size_t)C, hipMemcpyHostToDevice, st));
                    if ((rc = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl)) != CA_OK) return rc;
                    SweepOut one;
                    CA_HIP_CHECK(hipMemcpyAsync(&one, d_out.as<SweepOut>() + c, sizeof(SweepOut), hipMemcpyDeviceToHost, st));
                    CA_HIP_CHECK(hipStreamSynchronize(st));
                    exact_runs++;
                    v = one.fa_success ? one.lout : (int32_t)cur;
                } else {
                    final_[c] = 0;
                }
                cur = v;
            }
            tmark("walk");
            if (k0 >= S) break;
            {
                const double round_ms =
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_round).count();
                const int32_t adv = k0 - k_round;
                if ((round_ms > 2.0 * chain_ms_per * std::max(adv, 1) || knob_env("CASIM_SWEEP_FORCE_CHAIN")) &&
                    !knob_env("CASIM_NO_SERIAL_CHAIN")) {
                    if ((rc = run_chain(std::min(S, k0 + chain_batch))) != CA_OK) return rc;
                    chain_batch = std::min(2 * chain_batch, 4096);
                    if (k0 >= S) break;
                } else {
                    chain_batch = 64;
                }
            }
            // re-centre the windows from k0 on: follow the tables where the estimate falls
            // inside a window, otherwise shift the nearest known entry
            int64_t est = cur;
            dbg_first_rc = -1;
            for (int32_t k = k0; k < std::min(S, k0 + LOOKAHEAD); k++) {
                if (insensitive(k)) continue;
                const RowRef& mr = mref[k];                          // the main row
                const int32_t* fp = mr.f;
                const int32_t ms = mr.s;
                const RowRef* rr = nullptr;
                const int32_t w = lookup(k, wrap(est, n), rr);
                const int32_t v = w >= 0 ? rr->v[(size_t)w * rr->s] : TB_UNKNOWN;
                // an estimate within SIDE_BAND classes of its row's edge: the next round adds the
                // side row there (the exact input drifts a few positions past the edge now and then)
                if (sides && w >= 0 && rr == &mr && (w < SIDE_BAND || w > 63 - SIDE_BAND) && !have_side[k]) {
                    gapk[k] = std::max(1, wrap((int64_t)fp[(size_t)64 * ms] - fp[0], n) / 64);
                    want_side[k] = w < SIDE_BAND ? 1 : 2;
                }
                if (w >= 0 && v != TB_UNKNOWN) { est = v; continue; }
                int64_t next = est + (move_off[sens[k] + 1] - move_off[sens[k]]);
                int best = -1;              // known entry nearest the window centre
                for (int d = 0; d <= 32 && best < 0; d++) {
                    if (32 - d >= 0 && mr.v[(size_t)(32 - d) * ms] != TB_UNKNOWN) best = 32 - d;
                    else if (32 + d < 64 && mr.v[(size_t)(32 + d) * ms] != TB_UNKNOWN) best = 32 + d;
                }
                if (best >= 0) next = est + wrap(mr.v[(size_t)best * ms] - fp[(size_t)(1 + best) * ms], n);
                if (w < 0) {                 // re-centre: 32 of the row's mean gaps before the estimate
                    const int32_t gap = std::max(1, wrap((int64_t)fp[(size_t)64 * ms] - fp[0], n) / 64);
                    ws[k] = wrap(est - 32 * (int64_t)gap, n);
                    gapk[k] = gap;
                    if (dbg_t) {
                        dbg_rc[k] = rounds + 1;
                        if (dbg_first_rc < 0) dbg_first_rc = k;
                    }
                    have[k] = 0;
                    have_side[k] = 0;
                    if (sides && recentre_sides) want_side[k] = (uint8_t)recentre_sides;   // (knob: A/B)
                }
                est = wrap(next, n);
            }
            tmark("re-centre");
            if (rounds > S + 4) { set_last_error("sweep speculation did not converge"); return CA_EDEVICE; }
        }
        tmark("host walk");
        // exact pass for the candidates the host walk resolved through the table
        int32_t n_rerun = 0;
        for (int32_t c = 0; c < C; c++) {
            h_need[c] = final_[c] ? 0 : 1;
            h_lin[c] = exact_lin[c];
            n_rerun += final_[c] ? 0 : 1;
        }
        if (n_rerun > 0) {
            rounds++;
            CA_HIP_CHECK(hipMemcpyAsync(d_lin, h_lin, (sizeof(int32_t) + 1) * (size_t)C, hipMemcpyHostToDevice, st));
            if ((rc = launch_exact(m, st, in, d_lin, d_need, d_dest, d_hset, d_out, d_wl)) != CA_OK) return rc;
        }
        if (n_rerun > 0 || exact_runs > 0 || chained > 0)
            if ((rc = apply_hints()) != CA_OK) return rc;
        CA_HIP_CHECK(hipMemcpyAsync(sw.h_out.ptr, sw.out.ptr, d2h_bytes, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipStreamSynchronize(st));
    }
    if (dbg_t) fprintf(stderr, "[sweep] exact fallbacks %d, device walk %s (stopped at %d of %d)\n", exact_runs,
                       dev_walk ? "on" : "off", dev_walk ? h_info[0] : 0, S);
    const auto t_exact = std::chrono::steady_clock::now();
    if (M && out_dest) std::memcpy(out_dest, h_dest, sizeof(int32_t) * M);
    // the outputs must reproduce the chain: each result with a successful scan was
    // computed at the lastIndex the chain gives it; the others do not move it
    int64_t Lrun = L0;
    bool any_success = false;
    for (int32_t c = 0; c < C; c++) {
        const SweepOut& o = outs[c];
        if (o.status != CA_OK) { set_last_error("overlay capacity exceeded"); return o.status; }
        if (o.fa_success && wrap(o.lin, n) != wrap(Lrun, n)) {
            if (knob_env("CASIM_DEBUG"))
                fprintf(stderr, "chain mismatch at candidate %d: o.lin=%d Lrun=%ld\n", c, o.lin, (long)Lrun);
            set_last_error("sweep lastIndex chain mismatch");
            return CA_EDEVICE;
        }
        ca_removal_result& r = results[c];
        r.removable = o.removable;
        r.reason = o.reason;
        r.n_placed = o.n_placed;
        r.last_index_in = (int32_t)Lrun;
        r.evals = o.evals;
        if (o.fa_success) { Lrun = o.lout; any_success = true; }
    }
    *last_index = (int32_t)Lrun;
    if (hints) {
        for (int32_t i = 0; i < M; i++) if (hset[i] >= 0) hints[move_pods[i]] = hset[i];
    }
    // (the hint update stays queued on the mirror's stream: every later call is ordered
    // behind it, and ca_mirror_get_hints synchronises)
    tmark("done");
    if (!phased) {   // the next call's mode (serial_only above)
        const float per = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_start).count() /
                          (float)std::max(C, 1);
        if (serial_only) {
            sw.serial_ms_per = per;
            sw.serial_calls++;
        } else {
            sw.pipe_ms_per = per;
            sw.serial_calls = 0;
        }
        sw.serial_next = serial_only ? (sw.serial_calls < 8 && sw.serial_ms_per < sw.pipe_ms_per)
                                     : (S > 0 && 2 * chained > S);
        sw.serial_C = C;
        sw.serial_S = S;
    }
    m->sweep_stats.rounds = rounds + exact_runs;
    // the sweep's output depends on its input lastIndex iff some scan succeeded
    m->sweep_stats.had_success = any_success ? 1 : 0;
    m->sweep_stats.lin_sensitive = m->sweep_stats.had_success;
    m->sweep_stats.exact_ms = 0;
    m->sweep_stats.walk_ms = std::chrono::duration<float, std::milli>(t_exact - t_start).count();
    m->sweep_stats.kernel_ms = kms;
    m->sweep_stats.total_ms =
        std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return CA_OK;
}

// Prefix protocol (include/casim.h kernel scope): the first candidate that would be
// simulated with a CA_POD_OUT_OF_SCOPE pod to move or with more than CA_MAX_MOVED_PODS
// pods to move (k_sweep's destination overlay holds OV_CAP nodes), or C.
int32_t scope_cut(const ca_mirror* m, int32_t C, const int32_t* candidates, const uint8_t* dest_mask,
                  const int32_t* status, const int32_t* move_off, const int32_t* move_pods) {
    const int32_t n = (int32_t)m->nodes.size(), np = (int32_t)m->pods.size();
    for (int32_t c = 0; c < C; c++) {
        const int32_t nd = candidates[c];
        if (nd < 0 || nd >= n || !dest_mask[nd] || (status && status[c] != 0)) continue;
        if (move_off[c + 1] - move_off[c] > CA_MAX_MOVED_PODS) return c;
        if (m->n_oos_pods == 0) continue;        // no out-of-scope record in the mirror: no per-pod reads
        for (int32_t i = move_off[c]; i < move_off[c + 1]; i++) {
            const int32_t id = move_pods[i];
            if (id >= 0 && id < np && (m->pods[id].spec.flags & CA_POD_OUT_OF_SCOPE)) return c;
        }
    }
    return C;
}

void fill_cut(ca_removal_result* results, int32_t cut, int32_t C, int32_t last_index, int32_t* out_dest,
              const int32_t* move_off) {
    for (int32_t c = cut; c < C; c++) {
        ca_removal_result& r = results[c];
        r.removable = 0;
        r.reason = c == cut ? CA_UNREMOVABLE_OUT_OF_SCOPE : CA_UNREMOVABLE_NOT_RUN;
        r.n_placed = 0;
        r.last_index_in = last_index;
        r.evals = 0;
        if (out_dest)
            for (int32_t i = move_off[c]; i < move_off[c + 1]; i++) out_dest[i] = -1;
    }
}

}  // namespace casim

extern "C" {

int ca_find_nodes_to_remove(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                            const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                            int32_t* hints, int32_t* last_index, ca_removal_result* results, int32_t* out_dest) {
    if (!m || (C > 0 && (!candidates || !dest_mask || !move_off || !results || !out_dest)) || !last_index || C < 0)
        return CA_EINVAL;
    const auto t_entry = std::chrono::steady_clock::now();
    CA_HIP_CHECK(hipSetDevice(m->device));
    hipStream_t st = m->stream;
    const int32_t n = (int32_t)m->nodes.size();
    m->sweep_stats.had_success = m->sweep_stats.lin_sensitive = 0;
    if (C == 0) return CA_OK;
    const int32_t M = move_off[C] - move_off[0];
    if (move_off[0] != 0 || M < 0) return CA_EINVAL;
    for (int32_t c = 0; c < C; c++)
        if (move_off[c + 1] < move_off[c]) return CA_EINVAL;
    if (m->n_scope_blockers > 0) return CA_EUNSUPPORTED;        // casim.h scope
    {
        const int32_t cut = scope_cut(m, C, candidates, dest_mask, cand_status, move_off, move_pods);
        if (cut < C) {                                            // prefix protocol
            int rc = cut > 0 ? ca_find_nodes_to_remove(m, candidates, cut, dest_mask, cand_status, move_off, move_pods,
                                                       hints, last_index, results, out_dest)
                             : CA_OK;
            if (rc != CA_OK) return rc;
            fill_cut(results, cut, C, *last_index, out_dest, move_off);
            return CA_OK;
        }
    }
    // duplicate candidates share hints between their simulations: run them in
    // separate sequential segments (Hints.Set of one is seen by the next).
    {
        std::vector<uint8_t> seen((size_t)std::max(n, 1), 0);
        for (int32_t c = 0; c < C; c++) {
            const int32_t nd = candidates[c];
            if (nd < 0 || nd >= n) continue;
            if (seen[nd]) {
                int rc = ca_find_nodes_to_remove(m, candidates, c, dest_mask, cand_status, move_off, move_pods, hints,
                                                 last_index, results, out_dest);
                if (rc != CA_OK) return rc;
                std::vector<int32_t> off2(C - c + 1);
                for (int32_t k = 0; k <= C - c; k++) off2[k] = move_off[c + k] - move_off[c];
                return ca_find_nodes_to_remove(m, candidates + c, C - c, dest_mask, cand_status ? cand_status + c : nullptr,
                                               off2.data(), move_pods + move_off[c], hints, last_index, results + c,
                                               out_dest + move_off[c]);
            }
            seen[nd] = 1;
        }
    }
    int rc;
    const auto t_sync = std::chrono::steady_clock::now();
    const size_t dirty = m->all_dirty ? m->nodes.size() : m->dirty_rows.size();
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    const auto t_sync1 = std::chrono::steady_clock::now();
    if ((rc = m->sync_pods()) != CA_OK) return rc;
    if (knob_env("CASIM_DEBUG_TIMING"))
        fprintf(stderr, "[sweep] sync           %8.3f ms (rows %zu dirty: %.3f ms; %zu pods)\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_sync).count(), dirty,
                std::chrono::duration<double, std::milli>(t_sync1 - t_sync).count(), m->pods.size());
    const int32_t* status = cand_status;
    std::vector<int32_t> zero_status;
    if (!status) { zero_status.assign((size_t)C, 0); status = zero_status.data(); }
    // one page-locked staging area and one H2D copy for every per-call input:
    // [cand C][status C][move_off C+1][move_pods M][hint per moved pod M][dest mask n bytes]
    SweepScratch& sw = m->sw;
    const size_t in_ints = (size_t)C * 3 + 1 + (size_t)M * 2;
    const size_t in_bytes = sizeof(int32_t) * in_ints + (size_t)std::max(n, 1);
    if ((rc = sw.h_in.reserve(in_bytes)) != CA_OK) return rc;
    if ((rc = sw.in.reserve(in_bytes)) != CA_OK) return rc;
    int32_t* hin = sw.h_in.as<int32_t>();
    std::memcpy(hin, candidates, sizeof(int32_t) * C);
    std::memcpy(hin + C, status, sizeof(int32_t) * C);
    std::memcpy(hin + 2 * C, move_off, sizeof(int32_t) * (C + 1));
    int32_t* hm = hin + 3 * C + 1;
    int32_t* hh = hm + M;
    const int32_t np = (int32_t)m->pods.size();
    for (int32_t i = 0; i < M; i++) {             // validate, stage, gather the hints in one pass
        const int32_t id = move_pods[i];
        if (id < 0 || id >= np) return CA_EINVAL;
        hm[i] = id;
        hh[i] = hints ? hints[id] : -1;
    }
    std::memcpy(reinterpret_cast<uint8_t*>(hin + in_ints), dest_mask, (size_t)n);
    CA_HIP_CHECK(hipMemcpyAsync(sw.in.ptr, sw.h_in.ptr, in_bytes, hipMemcpyHostToDevice, st));
    int32_t* const dptr = sw.in.as<int32_t>();
    SweepCall in;
    in.C = C; in.M = M; in.n = n;
    in.cand = candidates; in.status = status; in.move_off = move_off; in.move_pods = move_pods; in.dest_mask = dest_mask;
    in.d_c = DevView{dptr}; in.d_status = DevView{dptr + C}; in.d_off = DevView{dptr + 2 * C};
    in.d_moves = DevView{dptr + 3 * C + 1}; in.d_hints = DevView{dptr + 3 * C + 1 + M};
    in.d_mask = DevView{dptr + in_ints};
    if (knob_env("CASIM_DEBUG_TIMING"))
        fprintf(stderr, "[sweep] entry to core %8.3f ms (C %d, M %d)\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_entry).count(), C, M);
    return sweep_core(m, in, hints, nullptr, last_index, results, out_dest);
}

int ca_removal_timings(const ca_mirror* m, float* out, int32_t cap) {
    if (!m || (cap > 0 && !out)) return CA_EINVAL;
    const float t[4] = {m->sweep_stats.kernel_ms, m->sweep_stats.exact_ms, m->sweep_stats.walk_ms,
                        m->sweep_stats.total_ms};
    for (int32_t i = 0; i < 4 && i < cap; i++) out[i] = t[i];
    return 4;
}

int ca_removal_candidate_ticks(const ca_mirror* m, uint64_t* out, int32_t C) {
    if (!m || C < 0 || (C > 0 && !out)) return CA_EINVAL;
    if (m->sw.h_out.bytes < sizeof(SweepOut) * (size_t)C) return CA_EINVAL;
    const SweepOut* o = m->sw.h_out.as<SweepOut>();
    for (int32_t c = 0; c < C; c++) out[c] = o[c].pad2;
    return CA_OK;
}

int ca_removal_stats(const ca_mirror* m, int32_t* rounds, float* kernel_ms, float* total_ms) {
    if (!m) return CA_EINVAL;
    if (rounds) *rounds = m->sweep_stats.rounds;
    if (kernel_ms) *kernel_ms = m->sweep_stats.kernel_ms;
    if (total_ms) *total_ms = m->sweep_stats.total_ms;
    return CA_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// removal plan: the call's inputs resident in HBM across runs (FindNodesToRemove is
// called every loop with the same candidates while the cluster is stable)
// ---------------------------------------------------------------------------
struct ca_removal_plan {
    ca_mirror* m = nullptr;
    int32_t C = 0, M = 0, n = 0;
    int32_t C_all = 0;              // candidates of the call; C = the prefix before the scope cut
    std::vector<int32_t> off_all;
    std::vector<int32_t> cand, status, off, moves;
    std::vector<uint8_t> mask;
    casim::DevBuf d_in;
    casim::HostBuf h_hints;
    casim::SweepCall call() {
        casim::SweepCall in;
        in.C = C; in.M = M; in.n = n;
        in.cand = cand.data(); in.status = status.data(); in.move_off = off.data(); in.move_pods = moves.data();
        in.dest_mask = mask.data();
        int32_t* d = d_in.as<int32_t>();
        const size_t in_ints = (size_t)C * 3 + 1 + (size_t)M * 2;
        in.d_c = casim::DevView{d}; in.d_status = casim::DevView{d + C}; in.d_off = casim::DevView{d + 2 * C};
        in.d_moves = casim::DevView{d + 3 * C + 1}; in.d_hints = casim::DevView{d + 3 * C + 1 + M};
        in.d_mask = casim::DevView{d + in_ints};
        return in;
    }
};

extern "C" {

int ca_removal_plan_create(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                           const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                           ca_removal_plan** out) {
    if (!m || !out || C < 0 || (C > 0 && (!candidates || !dest_mask || !move_off))) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    const int32_t n = (int32_t)m->nodes.size();
    int32_t M = C > 0 ? move_off[C] - move_off[0] : 0;
    if (C > 0 && (move_off[0] != 0 || M < 0)) return CA_EINVAL;
    std::vector<uint8_t> seen((size_t)std::max(n, 1), 0);
    for (int32_t c = 0; c < C; c++) {
        if (move_off[c + 1] < move_off[c]) return CA_EINVAL;
        const int32_t nd = candidates[c];
        if (nd >= 0 && nd < n) {
            if (seen[nd]) return CA_EUNSUPPORTED;     // duplicates: ca_find_nodes_to_remove splits them
            seen[nd] = 1;
        }
    }
    const int32_t np = (int32_t)m->pods.size();
    for (int32_t i = 0; i < M; i++) if (move_pods[i] < 0 || move_pods[i] >= np) return CA_EINVAL;
    ca_removal_plan* p = new ca_removal_plan();
    p->C_all = C;
    p->off_all.assign(move_off, move_off + C + 1);
    // prefix protocol (casim.h scope): the plan simulates the candidates before the first
    // out-of-scope one; run() reports the rest
    C = casim::scope_cut(m, C, candidates, dest_mask, cand_status, move_off, move_pods);
    M = move_off[C] - move_off[0];
    p->m = m; p->C = C; p->M = M; p->n = n;
    p->cand.assign(candidates, candidates + C);
    p->status = cand_status ? std::vector<int32_t>(cand_status, cand_status + C) : std::vector<int32_t>((size_t)C, 0);
    p->off.assign(move_off, move_off + C + 1);
    p->moves.assign(move_pods, move_pods + M);
    p->mask.assign(dest_mask, dest_mask + n);
    const size_t in_ints = (size_t)C * 3 + 1 + (size_t)M * 2;
    std::vector<int32_t> h(in_ints + ((size_t)std::max(n, 1) + 3) / 4, 0);
    std::copy(p->cand.begin(), p->cand.end(), h.begin());
    std::copy(p->status.begin(), p->status.end(), h.begin() + C);
    std::copy(p->off.begin(), p->off.end(), h.begin() + 2 * C);
    std::copy(p->moves.begin(), p->moves.end(), h.begin() + 3 * C + 1);
    std::fill(h.begin() + 3 * C + 1 + M, h.begin() + 3 * C + 1 + 2 * M, -1);
    std::memcpy(h.data() + in_ints, p->mask.data(), (size_t)n);
    int rc = p->d_in.reserve(sizeof(int32_t) * h.size());
    if (rc != CA_OK) { delete p; return rc; }
    if (hipMemcpy(p->d_in.ptr, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice) != hipSuccess) {
        delete p;
        casim::set_last_error("plan upload failed");
        return CA_EDEVICE;
    }
    *out = p;
    return CA_OK;
}

int ca_removal_plan_run(ca_removal_plan* p, int32_t* hints, int32_t* last_index, ca_removal_result* results,
                        int32_t* out_dest) {
    return casim::removal_plan_run_phase(p, hints, last_index, results, out_dest, nullptr);
}

}  // extern "C"

namespace casim {

bool removal_plan_phase_ok(const ca_removal_plan* p) { return p->C == p->C_all; }
int32_t sweep_fp_class(const int32_t* fp, int32_t n, int32_t L) { return fp_class(fp, 1, n, L); }

// pods to move of the plan's sensitive candidates (the probe's guess step, sweep_core)
int64_t removal_plan_sensitive_pods(const ca_removal_plan* p) {
    int64_t t = 0;
    for (int32_t c = 0; c < p->C; c++) {
        const int32_t nd = p->cand[c];
        if (nd < 0 || nd >= p->n || !p->mask[nd] || p->status[c] != 0) continue;
        t += p->off[c + 1] - p->off[c];
    }
    return t;
}

// A phase of a multi-device range (SweepPhase in sweep_core); ph == nullptr: a whole call.
// A plan with a scope cut runs whole calls only (ph->kind must be SP_FULL).
int removal_plan_run_phase(ca_removal_plan* p, int32_t* hints, int32_t* last_index, ca_removal_result* results,
                           int32_t* out_dest, SweepPhase* ph) {
    if (!p || !last_index || (p->C_all > 0 && !results)) return CA_EINVAL;
    if (ph && ph->kind != SP_FULL && p->C < p->C_all) return CA_EINVAL;
    ca_mirror* m = p->m;
    CA_HIP_CHECK(hipSetDevice(m->device));
    m->sweep_stats.had_success = m->sweep_stats.lin_sensitive = 0;
    if (p->C_all == 0) return CA_OK;
    if ((int32_t)m->nodes.size() != p->n) return CA_EINVAL;   // the plan's dest mask covers the node list
    if (m->n_scope_blockers > 0) return CA_EUNSUPPORTED;        // casim.h scope
    if (p->C < p->C_all) {                                      // prefix protocol
        int rc = CA_OK;
        if (p->C > 0) {
            p->C_all = p->C;                                    // run the prefix as a full plan
            rc = ca_removal_plan_run(p, hints, last_index, results, out_dest);
            p->C_all = (int32_t)p->off_all.size() - 1;
        }
        if (rc != CA_OK) return rc;
        casim::fill_cut(results, p->C, p->C_all, *last_index, out_dest, p->off_all.data());
        return CA_OK;
    }
    int rc;
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    if ((rc = m->sync_pods()) != CA_OK) return rc;
    casim::SweepCall in = p->call();
    int32_t* d_pod_hints = nullptr;
    if (hints) {                    // caller-held hints: gather per moved pod, one H2D
        if ((rc = p->h_hints.reserve(sizeof(int32_t) * (size_t)std::max(p->M, 1))) != CA_OK) return rc;
        int32_t* hh = p->h_hints.as<int32_t>();
        for (int32_t i = 0; i < p->M; i++) hh[i] = hints[p->moves[i]];
        if (p->M) CA_HIP_CHECK(hipMemcpyAsync(in.d_hints.ptr, hh, sizeof(int32_t) * p->M, hipMemcpyHostToDevice, m->stream));
    } else {                        // the mirror's resident hints
        if ((rc = m->ensure_pod_hints()) != CA_OK) return rc;
        d_pod_hints = m->d_pod_hints.as<int32_t>();
    }
    return casim::sweep_core(m, in, hints, d_pod_hints, last_index, results, out_dest, ph);
}

}  // namespace casim

extern "C" {

int ca_removal_plan_sensitive_pods(const ca_removal_plan* p, int64_t* out) {
    if (!p || !out) return CA_EINVAL;
    *out = casim::removal_plan_sensitive_pods(p);
    return CA_OK;
}

int ca_removal_plan_phased(const ca_removal_plan* p, int32_t* out) {
    if (!p || !out) return CA_EINVAL;
    *out = casim::removal_plan_phase_ok(p) ? 1 : 0;
    return CA_OK;
}

int ca_removal_plan_run_phase(ca_removal_plan* p, ca_sweep_phase* ph, int32_t* hints, int32_t* last_index,
                              ca_removal_result* results, int32_t* out_dest) {
    if (!p || !ph || !hints) return CA_EINVAL;
    if (ph->kind != SP_PROBE && ph->kind != SP_MAP && ph->kind != SP_RESOLVE) return CA_EINVAL;
    return casim::removal_plan_run_phase(p, hints, last_index, results, out_dest, ph);
}

int ca_removal_plan_destroy(ca_removal_plan* p) {
    if (!p) return CA_EINVAL;
    delete p;
    return CA_OK;
}

}  // extern "C"
