// sweep.hip — RemovalSimulator.FindNodesToRemove, legacy semantics (canPersist=false).
//
// Reference: CA/simulator/cluster.go:116-254 (FindNodesToRemove, SimulateNodeRemoval,
// withForkedSnapshot, findPlaceFor), CA/simulator/scheduling/hinting_simulator.go:58-125
// (TrySchedulePods, hints), CA/utils/tpu/tpu.go:57-79 (ClearTPURequests).
//
// Every candidate is simulated on a fork that is reverted afterwards, so candidates
// share no snapshot state: one wavefront per candidate keeps its placements in an
// LDS overlay over the read-only base rows.  The only coupling is the checker's
// lastIndex; the host driver runs all candidates from guessed
// lastIndex values and re-runs the ones whose guess was wrong until every
// candidate's input equals its predecessor's output.
#include "mirror.h"
#include "device_filters.h"

#include <cstring>
#include <algorithm>
#include <chrono>

namespace casim {

constexpr int OV_CAP = 128;   // distinct destination nodes per candidate

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
    uint64_t ports[OV_CAP][CA_PORT_WORDS];
    int64_t scalar[OV_CAP][CA_MAX_SCALAR];
};

__device__ inline int64_t rl64s(int64_t v, int lane) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// moved-pod semantics: Spec.NodeName cleared (cluster.go:235-240), TPU requests
// cleared (tpu.go:57-79)
__device__ inline uint32_t moved_flags(uint32_t f) {
    uint32_t m = f & ~(PF_NODE_NAME | PF_ALL_ZERO | PF_SCALAR_REQ | PF_HAS_SCALAR_KEYS);
    if (f & PF_MOVED_ALL_ZERO) m |= PF_ALL_ZERO;
    if (f & PF_MOVED_SCALAR_REQ) m |= PF_SCALAR_REQ;
    if (f & PF_NONTPU_SCALAR) m |= PF_HAS_SCALAR_KEYS;
    return m;
}

// Evaluate the filter chain for one node with the candidate's overlay applied.
// All lanes hold the same (pod, node) — used for the hint check.
__device__ inline bool eval_node_uniform(const ca_pod_spec& s, const PodHot& p, const int64_t* psc,
                                         const ca_selector_term* terms, const ca_selector_req* reqs,
                                         NodeHot h, NodeExt e, const NodeStatic* st_row, bool apply_unsched) {
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

__global__ void __launch_bounds__(64) k_sweep(
    const NodeHot* __restrict__ hot, const NodeExt* __restrict__ ext, const NodeStatic* __restrict__ st, int32_t n,
    const uint8_t* __restrict__ dest_mask, const int32_t* __restrict__ cands, const int32_t* __restrict__ cand_status,
    const int32_t* __restrict__ move_off, const int32_t* __restrict__ move_pods, const PodHot* __restrict__ ph,
    const ca_pod_spec* __restrict__ specs, const ca_selector_term* __restrict__ terms,
    const ca_selector_req* __restrict__ reqs, const int32_t* __restrict__ names, const int32_t* __restrict__ hints,
    const int32_t* __restrict__ lin_arr, const uint8_t* __restrict__ need, int32_t* __restrict__ out_dest,
    int32_t* __restrict__ hint_set, SweepOut* __restrict__ outs) {
    __shared__ OverlaySmem ov;
    const int c = blockIdx.x;
    if (!need[c]) return;
    const int lane = threadIdx.x;
    const int32_t lin = lin_arr[c];
    SweepOut res;
    res.removable = 0; res.reason = CA_UNREMOVABLE_NONE; res.n_placed = 0; res.lin = lin; res.lout = lin;
    res.fa_success = 0; res.status = CA_OK; res.pad = 0; res.evals = 0; res.pad2 = 0;
    const int32_t node = cands[c];
    const int32_t mo = move_off[c], mn = move_off[c + 1] - mo;
    for (int32_t i = lane; i < mn; i += 64) { out_dest[mo + i] = -1; hint_set[mo + i] = -1; }
    if (node < 0 || node >= n || !dest_mask[node]) {                          // cluster.go:157-160
        res.reason = CA_UNREMOVABLE_UNEXPECTED_ERROR;
        if (lane == 0) outs[c] = res;
        return;
    }
    if (cand_status[c] != 0) {                                                 // :162-169
        res.reason = cand_status[c];
        if (lane == 0) outs[c] = res;
        return;
    }
    int32_t npl = 0;          // overlay entries
    int64_t L = lin;
    uint64_t evals = 0;
    bool fa_success = false;
    int32_t placed = 0;
    bool failed = false;

    for (int32_t i = 0; i < mn; i++) {
        __syncthreads();
        const int32_t id = move_pods[mo + i];
        PodHot p = ph[id];
        p.flags = moved_flags(p.flags);
        const ca_pod_spec& s = specs[p.spec];
        int64_t psc[CA_MAX_SCALAR];
        for (int k = 0; k < CA_MAX_SCALAR; k++) psc[k] = 0;
        if (p.flags & PF_SCALAR_REQ)
            for (int k = 0; k < CA_MAX_SCALAR; k++) psc[k] = ((s.tpu_scalar_mask >> k) & 1u) ? 0 : s.req_scalar[k];
        const bool pre_fail = (p.flags & PF_PREFILTER_FAIL) != 0;
        int32_t target = -1;

        // ---- findNodeWithHints (hinting_simulator.go:91-108) ----
        const int32_t h = hints[id];
        if (h >= 0 && h < n && !pre_fail) {
            evals++;
            NodeHot nh = hot[h];
            NodeExt ne = ext[h];
            if (h == node) {
                // the candidate with every moved pod removed (cluster.go:228-233)
                for (int32_t q = 0; q < mn; q++) {
                    const PodHot mp = ph[move_pods[mo + q]];
                    const ca_pod_spec& ms = specs[mp.spec];
                    nh.cpu = wadd(nh.cpu, mp.cpu); nh.mem = wadd(nh.mem, mp.mem); nh.eph = wadd(nh.eph, mp.eph);
                    nh.pods += 1;
                    for (int k = 0; k < CA_MAX_SCALAR; k++) ne.scalar[k] = wadd(ne.scalar[k], ms.req_scalar[k]);
                    for (int w = 0; w < CA_PORT_WORDS; w++) ne.ports[w] &= ~ms.port_use[w];
                }
            } else {
                for (int32_t q = 0; q < npl; q++) {
                    if (ov.node[q] == h) {
                        nh.cpu = wsub(nh.cpu, ov.cpu[q]); nh.mem = wsub(nh.mem, ov.mem[q]);
                        nh.eph = wsub(nh.eph, ov.eph[q]); nh.pods -= ov.pods[q];
                        for (int w = 0; w < CA_PORT_WORDS; w++) ne.ports[w] |= ov.ports[q][w];
                        for (int k = 0; k < CA_MAX_SCALAR; k++) ne.scalar[k] = wsub(ne.scalar[k], ov.scalar[q][k]);
                    }
                }
            }
            if (eval_node_uniform(s, p, psc, terms, reqs, nh, ne, st + h, true)) {
                if (lane == 0) hint_set[mo + i] = h;                          // :95
                if (h != node && dest_mask[h]) target = h;                      // :102
            }
        }
        // ---- findNode -> FitsAnyNodeMatching(isCandidateNode) (:110-125) ----
        if (target < 0 && !pre_fail) {
            for (int32_t base = 0; base < n; base += 64) {
                const int32_t off = base + lane;
                const int32_t pos = (int32_t)((L + off) % n);
                bool vis = false;
                NodeHot nh;
                if (off < n && pos != node && dest_mask[pos]) {
                    nh = hot[pos];
                    bool pf_ok = true;
                    if (p.flags & PF_PREFILTER_NAMES) {
                        const int32_t nm = st[pos].name_id;
                        pf_ok = false;
                        for (int32_t k = 0; k < s.prefilter_count; k++) pf_ok |= names[s.prefilter_first + k] == nm;
                    }
                    vis = pf_ok && !(nh.flags & NF_UNSCHED);
                }
                // overlay entries inside this chunk
                bool ov_here = false;
                int32_t ov_slot = -1;
                for (int32_t q0 = 0; q0 < npl; q0 += 64) {
                    const int32_t q = q0 + lane;
                    bool in = false;
                    int32_t d = 0;
                    if (q < npl) {
                        d = (int32_t)(((int64_t)ov.node[q] - (L + base)) % n);
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
                    NodeExt ne;
                    const bool need_ext = (p.flags & (PF_PORTS | PF_SCALAR_REQ)) || ov_here;
                    if (need_ext) ne = ext[pos];
                    if (ov_here) {
                        nh.cpu = wsub(nh.cpu, ov.cpu[ov_slot]); nh.mem = wsub(nh.mem, ov.mem[ov_slot]);
                        nh.eph = wsub(nh.eph, ov.eph[ov_slot]); nh.pods -= ov.pods[ov_slot];
                        for (int w = 0; w < CA_PORT_WORDS; w++) ne.ports[w] |= ov.ports[ov_slot][w];
                        for (int k = 0; k < CA_MAX_SCALAR; k++) ne.scalar[k] = wsub(ne.scalar[k], ov.scalar[ov_slot][k]);
                    }
                    if (!need_ext) {
                        // resource-only fast path: one 32-B row
                        const bool need_static = (p.flags & (PF_NODE_NAME | PF_AFFINITY)) ||
                                                 ((nh.flags & NF_TAINTS) && !(p.flags & PF_TAINT_MASK_ALL));
                        fit = true;
                        if (need_static) {
                            const NodeStatic ns = st[pos];
                            fit = dev_static_filters(s, p.flags, terms, reqs, ns, false) == CA_PLUGIN_NONE;
                        }
                        if (fit) {
                            fit = nh.pods >= 1;
                            if (!(p.flags & PF_ALL_ZERO))
                                fit = fit && p.cpu <= nh.cpu && p.mem <= nh.mem && p.eph <= nh.eph;
                        }
                    } else {
                        fit = eval_node_uniform(s, p, psc, terms, reqs, nh, ne, st + pos, false);
                    }
                }
                const uint64_t fm = __ballot(fit), vm = __ballot(vis);
                if (fm) {
                    const int f = __builtin_ctzll(fm);
                    const uint64_t below = (f == 63) ? ~0ull : ((2ull << f) - 1);
                    evals += (uint64_t)__popcll(vm & below);
                    const int32_t foff = base + f;
                    target = (int32_t)((L + foff) % n);
                    L = (L + foff + 1) % n;                                    // schedulerbased.go:131
                    fa_success = true;
                    if (lane == 0) hint_set[mo + i] = target;                  // :123
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
                for (int w = 0; w < CA_PORT_WORDS; w++) ov.ports[slot][w] = 0;
                for (int k = 0; k < CA_MAX_SCALAR; k++) ov.scalar[slot][k] = 0;
            }
        }
        if (lane == 0) {
            ov.cpu[slot] = wadd(ov.cpu[slot], p.cpu);
            ov.mem[slot] = wadd(ov.mem[slot], p.mem);
            ov.eph[slot] = wadd(ov.eph[slot], p.eph);
            ov.pods[slot] += 1;
            for (int w = 0; w < CA_PORT_WORDS; w++) ov.ports[slot][w] |= s.port_use[w];
            for (int k = 0; k < CA_MAX_SCALAR; k++) ov.scalar[slot][k] = wadd(ov.scalar[slot][k], psc[k]);
            out_dest[mo + i] = target;
        }
        placed++;
    }
    if (lane == 0) {
        res.n_placed = placed;
        if (!failed && placed == mn) { res.removable = 1; res.reason = CA_UNREMOVABLE_NONE; }
        else res.reason = CA_UNREMOVABLE_NO_PLACE;
        res.lout = (int32_t)L;
        res.fa_success = fa_success ? 1 : 0;
        res.evals = evals;
        outs[c] = res;
    }
}

}  // namespace casim

using namespace casim;

extern "C" {

int ca_find_nodes_to_remove(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                            const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                            int32_t* hints, int32_t* last_index, ca_removal_result* results, int32_t* out_dest) {
    if (!m || (C > 0 && (!candidates || !dest_mask || !move_off || !results || !out_dest)) || !last_index || C < 0)
        return CA_EINVAL;
    const auto t_start = std::chrono::steady_clock::now();
    CA_HIP_CHECK(hipSetDevice(m->device));
    hipStream_t st = m->stream;
    const int32_t n = (int32_t)m->nodes.size();
    if (C == 0) return CA_OK;
    const int32_t M = move_off[C] - move_off[0];
    if (move_off[0] != 0 || M < 0) return CA_EINVAL;
    for (int32_t c = 0; c < C; c++) {
        for (int32_t i = move_off[c]; i < move_off[c + 1]; i++) {
            const int32_t id = move_pods[i];
            if (id < 0 || (size_t)id >= m->pods.size()) return CA_EINVAL;
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
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    if ((rc = m->sync_pods()) != CA_OK) return rc;
    // per-call inputs
    std::vector<int32_t> status((size_t)C, 0);
    if (cand_status) std::copy(cand_status, cand_status + C, status.begin());
    const size_t hint_n = std::max<size_t>(m->pods.size(), 1);
    std::vector<int32_t> h_hints(hint_n, -1);
    if (hints) std::copy(hints, hints + m->pods.size(), h_hints.begin());
    DevBuf d_c, d_status, d_off, d_moves, d_hints, d_lin, d_need, d_dest, d_hset, d_out, d_mask;
    if ((rc = d_c.reserve(sizeof(int32_t) * C)) != CA_OK) return rc;
    if ((rc = d_status.reserve(sizeof(int32_t) * C)) != CA_OK) return rc;
    if ((rc = d_off.reserve(sizeof(int32_t) * (C + 1))) != CA_OK) return rc;
    if ((rc = d_moves.reserve(sizeof(int32_t) * std::max(M, 1))) != CA_OK) return rc;
    if ((rc = d_hints.reserve(sizeof(int32_t) * hint_n)) != CA_OK) return rc;
    if ((rc = d_lin.reserve(sizeof(int32_t) * C)) != CA_OK) return rc;
    if ((rc = d_need.reserve((size_t)C)) != CA_OK) return rc;
    if ((rc = d_dest.reserve(sizeof(int32_t) * std::max(M, 1))) != CA_OK) return rc;
    if ((rc = d_hset.reserve(sizeof(int32_t) * std::max(M, 1))) != CA_OK) return rc;
    if ((rc = d_out.reserve(sizeof(SweepOut) * C)) != CA_OK) return rc;
    if ((rc = d_mask.reserve((size_t)std::max(n, 1))) != CA_OK) return rc;
    CA_HIP_CHECK(hipMemcpyAsync(d_c.ptr, candidates, sizeof(int32_t) * C, hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipMemcpyAsync(d_status.ptr, status.data(), sizeof(int32_t) * C, hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipMemcpyAsync(d_off.ptr, move_off, sizeof(int32_t) * (C + 1), hipMemcpyHostToDevice, st));
    if (M) CA_HIP_CHECK(hipMemcpyAsync(d_moves.ptr, move_pods, sizeof(int32_t) * M, hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipMemcpyAsync(d_hints.ptr, h_hints.data(), sizeof(int32_t) * hint_n, hipMemcpyHostToDevice, st));
    if (n) CA_HIP_CHECK(hipMemcpyAsync(d_mask.ptr, dest_mask, (size_t)n, hipMemcpyHostToDevice, st));

    std::vector<int32_t> lin((size_t)C, *last_index);
    std::vector<uint8_t> need((size_t)C, 1);
    std::vector<SweepOut> outs((size_t)C), fresh((size_t)C);
    int32_t rounds = 0;
    float kms = 0;
    int32_t first_unconfirmed = 0;
    int64_t cur_true = *last_index;
    for (;;) {
        rounds++;
        CA_HIP_CHECK(hipMemcpyAsync(d_lin.ptr, lin.data(), sizeof(int32_t) * C, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipMemcpyAsync(d_need.ptr, need.data(), (size_t)C, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipEventRecord(m->ev0, st));
        hipLaunchKernelGGL(k_sweep, dim3(C), dim3(64), 0, st, m->d_hot.as<NodeHot>(), m->d_ext.as<NodeExt>(),
                           m->d_static.as<NodeStatic>(), n, d_mask.as<uint8_t>(), d_c.as<int32_t>(),
                           d_status.as<int32_t>(), d_off.as<int32_t>(), d_moves.as<int32_t>(),
                           m->d_pods.hot.as<PodHot>(), m->d_pods.spec.as<ca_pod_spec>(),
                           m->d_pods.terms.as<ca_selector_term>(), m->d_pods.reqs.as<ca_selector_req>(),
                           m->d_pods.names.as<int32_t>(), d_hints.as<int32_t>(), d_lin.as<int32_t>(),
                           d_need.as<uint8_t>(), d_dest.as<int32_t>(), d_hset.as<int32_t>(), d_out.as<SweepOut>());
        CA_HIP_CHECK(hipGetLastError());
        CA_HIP_CHECK(hipEventRecord(m->ev1, st));
        CA_HIP_CHECK(hipMemcpyAsync(fresh.data(), d_out.ptr, sizeof(SweepOut) * C, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipStreamSynchronize(st));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, m->ev0, m->ev1);
        kms += ms;
        for (int32_t c = 0; c < C; c++) if (need[c]) outs[c] = fresh[c];
        // confirm the exact prefix
        int32_t c = first_unconfirmed;
        for (; c < C; c++) {
            const SweepOut& o = outs[c];
            const bool insensitive = !o.fa_success;          // no FitsAnyNode placement: L untouched
            if (o.lin != cur_true && !insensitive) break;
            if (o.fa_success) cur_true = o.lout;
        }
        first_unconfirmed = c;
        if (c == C) break;
        // new guesses: exact lastIndex for the first unconfirmed candidate, then the
        // lastIndex advance each later candidate showed on its last run
        std::fill(need.begin(), need.end(), 0);
        int64_t guess = cur_true;
        for (int32_t k = c; k < C; k++) {
            const SweepOut& o = outs[k];
            if (o.fa_success) {
                if (o.lin != (int32_t)guess) { need[k] = 1; lin[k] = (int32_t)guess; }
                int64_t adv = ((int64_t)o.lout - (int64_t)o.lin) % n;
                if (adv < 0) adv += n;
                guess = (guess + adv) % n;
            }
        }
        need[c] = 1;
        lin[c] = (int32_t)cur_true;
        if (rounds > C + 2) { set_last_error("sweep speculation did not converge"); return CA_EDEVICE; }
    }
    *last_index = (int32_t)cur_true;
    std::vector<int32_t> hset((size_t)std::max(M, 1));
    if (M) {
        CA_HIP_CHECK(hipMemcpyAsync(out_dest, d_dest.ptr, sizeof(int32_t) * M, hipMemcpyDeviceToHost, st));
        CA_HIP_CHECK(hipMemcpyAsync(hset.data(), d_hset.ptr, sizeof(int32_t) * M, hipMemcpyDeviceToHost, st));
    }
    CA_HIP_CHECK(hipStreamSynchronize(st));
    for (int32_t c = 0; c < C; c++) {
        const SweepOut& o = outs[c];
        if (o.status != CA_OK) { set_last_error("overlay capacity exceeded"); return o.status; }
        ca_removal_result& r = results[c];
        r.removable = o.removable;
        r.reason = o.reason;
        r.n_placed = o.n_placed;
        r.last_index_in = o.lin;
        r.evals = o.evals;
    }
    if (hints) {
        for (int32_t i = 0; i < M; i++) if (hset[i] >= 0) hints[move_pods[i]] = hset[i];
    }
    m->sweep_stats.rounds = rounds;
    m->sweep_stats.kernel_ms = kms;
    m->sweep_stats.total_ms =
        std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_start).count();
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
