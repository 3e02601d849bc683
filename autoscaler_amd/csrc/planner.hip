// planner.hip — Planner.categorizeNodes with canPersist = true.
//
// Reference: CA/core/scaledown/planner/planner.go:252-296 (the candidate loop),
// CA/simulator/cluster.go:145-184,204-254 (SimulateNodeRemoval, withForkedSnapshot Commit,
// findPlaceFor), CA/core/scaledown/pdb/basic.go:58-95 (RemainingPdbTracker),
// CA/simulator/drain.go:73-90 (checkPdbs).
//
// The loop is sequential: every removable candidate commits its moves before the next one
// is simulated.  The device runs it speculatively (DESIGN.md §4 planner):
//   1. speculate: the legacy sweep (sweep.hip, every candidate on a reverted fork, exact
//      lastIndex chain) simulates a window of candidates from the committed state;
//   2. validate, in candidate order, on the host: a speculative simulation is the committed
//      one unless a commit made earlier in the same window changed something it read.
//      Commits only add pods to destination nodes and drop removed candidates from the
//      destination set, and every filter is monotone in the pods a node holds, so a node
//      the speculation rejected still rejects: only its chosen nodes (re-checked with the
//      committed rows), its hinted nodes that left the destination set and its own node
//      (which may have received pods to move) can differ.  Nodes that left the
//      destination set inside a scanned range are skipped instead of evaluated: the
//      evaluation count is corrected, lastIndex is positional and unchanged;
//   3. commit the valid prefix into the mirror (RemovePod + AddPod of the moved copies,
//      journaled at the caller's fork depth) and re-speculate from the first conflict,
//      whose own speculation is then exact (it is first in its window).
#include "mirror.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

using namespace casim;

namespace {

// moved-pod copy: Spec.NodeName cleared (cluster.go:235-240), TPU requests cleared
// (cluster.go:225, tpu.go:57-79)
ca_pod_spec moved_spec(const ca_pod_spec& p) {
    ca_pod_spec q = p;
    q.node_name_id = -1;
    for (int i = 0; i < CA_MAX_SCALAR; i++)
        if ((p.tpu_scalar_mask >> i) & 1u) q.req_scalar[i] = 0;
    if (!(p.flags & CA_POD_HAS_NONTPU_SCALAR_KEYS)) q.flags &= ~CA_POD_HAS_SCALAR_KEYS;
    return q;
}

// a candidate's own placements on one node so far (the fork's AddPods)
struct Own {
    int32_t node;
    int64_t cpu, mem, eph, pods;
    int64_t sc[CA_MAX_SCALAR];
    uint64_t ports[CA_PORT_WORDS];
};

// NodePorts + NodeResourcesFit on the committed row plus the candidate's own placements
// (the static filters passed in the speculation and do not depend on pods)
bool dyn_fits(const ca_mirror* m, int32_t f, const ca_pod_spec& q, const Own* own) {
    const NodeRow& nd = m->nodes[f];
    int64_t fc = wsub(nd.spec.alloc_milli_cpu, nd.req_cpu), fm = wsub(nd.spec.alloc_memory, nd.req_mem);
    int64_t fe = wsub(nd.spec.alloc_ephemeral, nd.req_eph), fp = nd.spec.alloc_pods - nd.npods;
    int64_t fs[CA_MAX_SCALAR];
    uint64_t used[CA_PORT_WORDS];
    for (int k = 0; k < CA_MAX_SCALAR; k++) fs[k] = wsub(nd.spec.alloc_scalar[k], nd.req_scalar[k]);
    for (int w = 0; w < CA_PORT_WORDS; w++) used[w] = nd.ports[w];
    if (own) {
        fc = wsub(fc, own->cpu); fm = wsub(fm, own->mem); fe = wsub(fe, own->eph); fp -= own->pods;
        for (int k = 0; k < CA_MAX_SCALAR; k++) fs[k] = wsub(fs[k], own->sc[k]);
        for (int w = 0; w < CA_PORT_WORDS; w++) used[w] |= own->ports[w];
    }
    for (int w = 0; w < CA_PORT_WORDS; w++)
        if (used[w] & q.port_conflict[w]) return false;
    return dev_fit_reasons(q.req_milli_cpu, q.req_memory, q.req_ephemeral, pod_dev_flags(q), q.req_scalar, fc, fm, fe,
                           clamp_i32(fp), fs) == 0;
}

// would FitsAnyNodeMatching evaluate node x for pod q (schedulerbased.go:114-129; x is in
// the destination set and is not the candidate)
bool scan_visits(const ca_mirror* m, int32_t x, const ca_pod_spec& q) {
    const ca_node_spec& ns = m->nodes[x].spec;
    if (ns.flags & CA_NODE_UNSCHEDULABLE) return false;                          // :125
    if (q.flags & CA_POD_PREFILTER_NAMES) {                                        // :120
        for (int32_t k = 0; k < q.prefilter_count; k++)
            if (m->pf_names[q.prefilter_first + k] == ns.name_id) return true;
        return false;
    }
    return true;
}

}  // namespace

int32_t ca_mirror::store_moved_copy(int32_t pod) {
    PodRow row;
    row.spec = moved_spec(pods[pod].spec);     // selector / name indices already on the mirror tables
    row.node = -1;
    if (pod_dev_flags(row.spec) & (PF_PORTS | PF_SCALAR_REQ | PF_MOVED_SCALAR_REQ)) n_ext_pods++;
    if (row.spec.req_ephemeral != 0) n_eph_pods++;
    if (row.spec.flags & CA_POD_OUT_OF_SCOPE) n_oos_pods++;
    pods.push_back(row);
    return (int32_t)pods.size() - 1;
}

int ca_mirror::replay_moves(const ca_plan_move* mv, int32_t nm) {
    if (nm <= 0) return CA_OK;
    const int32_t base = (int32_t)pods.size();
    for (int32_t t = 0; t < nm; t++) {
        if (mv[t].new_pod != base + t || mv[t].pod < 0 || mv[t].pod >= base + t || mv[t].node < 0 ||
            mv[t].node >= (int32_t)nodes.size()) {
            set_last_error("plan chain: copy ids out of step with the mirror");
            return CA_EDEVICE;
        }
    }
    int32_t T = std::min(8, nm / 4096);    // (serially ~40 ns a move; at 6k moves four threads are no faster)
    T = T >= 8 ? 8 : T >= 4 ? 4 : T >= 2 ? 2 : 1;              // (a power of two: 64-node block & (T - 1) picks the thread)
    const int32_t tm = T - 1;
    if (T <= 1) {
        for (int32_t k = 0; k < nm;) {
            const int32_t cand = mv[k].candidate;
            int32_t e = k;
            while (e < nm && mv[e].candidate == cand) e++;
            for (int32_t t = k; t < e; t++) {
                const int rc = ca_mirror_remove_pod(this, mv[t].pod);                 // cluster.go:228-233
                if (rc != CA_OK) return rc;
            }
            for (int32_t t = k; t < e; t++) add_pod_to_node(store_moved_copy(mv[t].pod), mv[t].node);   // AddPod (:79)
            k = e;
        }
        return CA_OK;
    }
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    const auto tr0 = std::chrono::steady_clock::now();
    auto tmark = [&](const char* what) {
        if (dbg_t)
            fprintf(stderr, "[replay] %-10s %8.3f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count());
    };
    // Large batches (the loop without a limit: ~68k moves on C3).  The copies' records first:
    // a copy of a copy is a copy of the original (moved_spec is idempotent), so record t
    // derives from its root pod below `base` and every record is independent.  Then the row
    // updates split by 64-node block (adjacent rows share cache lines): each thread walks the moves in order and applies the
    // RemovePods / AddPods on its own nodes, so every node sees its pods in order; journal
    // entries of different nodes commute (Revert undoes each node's in reverse).
    std::vector<int32_t> root((size_t)nm), src_node((size_t)nm);
    for (int32_t t = 0; t < nm; t++) {
        const int32_t p = mv[t].pod;
        root[t] = p < base ? p : root[p - base];
        src_node[t] = p < base ? pods[p].node : mv[p - base].node;
        if (src_node[t] < 0) return CA_ENOTFOUND;
    }
    pods.resize_for_overwrite((size_t)base + (size_t)nm);
    if (dirty_flag.size() < nodes.size()) dirty_flag.resize(nodes.size(), 0);
    if (depth > 0) reserve_more(0, 2 * (size_t)nm);
    struct Part {
        std::vector<JournalEntry> jr;
        std::vector<int32_t> dirty;
        int64_t ext = 0, eph = 0, blockers = 0, oos = 0;
        int rc = CA_OK;
    };
    std::vector<Part> part((size_t)T);
    const bool journaled = depth > 0;
    tmark("prepared");
    casim::parallel_run(T, [&](int32_t w) {
        Part& pt = part[w];
        const int32_t t0 = (int32_t)((int64_t)nm * w / T), t1 = (int32_t)((int64_t)nm * (w + 1) / T);
        for (int32_t t = t0; t < t1; t++) {                     // the records of moves [t0, t1)
            if (t + 8 < t1) __builtin_prefetch(&pods[root[t + 8]].spec);   // (random records: fetch ahead)
            PodRow& r = pods[(size_t)base + t];
            r.spec = moved_spec(pods[root[t]].spec);
            r.node = -1;
            if (pod_dev_flags(r.spec) & (PF_PORTS | PF_SCALAR_REQ | PF_MOVED_SCALAR_REQ)) pt.ext++;
            if (r.spec.req_ephemeral != 0) pt.eph++;
            if (r.spec.flags & CA_POD_OUT_OF_SCOPE) pt.oos++;
        }
    });
    tmark("records");
    casim::parallel_run(T, [&](int32_t w) {
        Part& pt = part[w];
        if (journaled) pt.jr.reserve(2 * (size_t)nm / (size_t)T + 1024);
        auto apply = [&](int32_t x, const ca_pod_spec& p, int sign) {
            NodeRow& nd = nodes[x];
            if (sign > 0) {
                nd.req_cpu = wadd(nd.req_cpu, p.req_milli_cpu);
                nd.req_mem = wadd(nd.req_mem, p.req_memory);
                nd.req_eph = wadd(nd.req_eph, p.req_ephemeral);
                for (int i = 0; i < CA_MAX_SCALAR; i++) nd.req_scalar[i] = wadd(nd.req_scalar[i], p.req_scalar[i]);
                for (int q = 0; q < CA_PORT_WORDS; q++) nd.ports[q] |= p.port_use[q];
            } else {
                nd.req_cpu = wsub(nd.req_cpu, p.req_milli_cpu);
                nd.req_mem = wsub(nd.req_mem, p.req_memory);
                nd.req_eph = wsub(nd.req_eph, p.req_ephemeral);
                for (int i = 0; i < CA_MAX_SCALAR; i++) nd.req_scalar[i] = wsub(nd.req_scalar[i], p.req_scalar[i]);
                for (int q = 0; q < CA_PORT_WORDS; q++) nd.ports[q] &= ~p.port_use[q];
            }
            nd.npods += sign;
            if (p.flags & CA_POD_REQUIRED_ANTI_AFFINITY) pt.blockers += sign;
            if (!dirty_flag[x]) { dirty_flag[x] = 1; pt.dirty.push_back(x); }
        };
        auto journal = [&](int32_t kind, int32_t x, int32_t pod, int32_t slot, const uint64_t* before) {
            if (!journaled) return;
            JournalEntry e;
            std::memset(&e, 0, sizeof e);
            e.kind = kind; e.node = x; e.pod = pod; e.slot = slot;
            std::memcpy(e.ports, before, sizeof e.ports);
            pt.jr.push_back(e);
        };
        for (int32_t k = 0; k < nm && pt.rc == CA_OK;) {
            const int32_t cand = mv[k].candidate;
            int32_t e = k;
            while (e < nm && mv[e].candidate == cand) e++;
            for (int32_t t = k; t < e; t++) {                   // RemovePod (cluster.go:228-233)
                if (t + 16 < nm && ((src_node[t + 16] >> 6) & tm) == w) {     // (random rows and records: fetch ahead)
                    __builtin_prefetch(&pods[mv[t + 16].pod].spec);
                    __builtin_prefetch(reinterpret_cast<const char*>(&pods[mv[t + 16].pod].spec) + 64);
                    __builtin_prefetch(&nodes[src_node[t + 16]]);
                }
                const int32_t x = src_node[t];
                if (((x >> 6) & tm) != w) continue;
                const int32_t pod = mv[t].pod;
                NodeRow& nd = nodes[x];
                int32_t slot = -1;
                for (size_t i = 0; i < nd.pods.size(); i++) if (nd.pods[i] == pod) { slot = (int32_t)i; break; }
                if (slot < 0) { pt.rc = CA_ENOTFOUND; break; }
                uint64_t before[CA_PORT_WORDS];
                std::memcpy(before, nd.ports, sizeof before);
                nd.pods[slot] = nd.pods.back();                 // swap-with-last (SF/types.go:660-663)
                nd.pods.pop_back();
                apply(x, pods[pod].spec, -1);
                pods[pod].node = -1;
                journal(J_REMOVE_POD, x, pod, slot, before);
            }
            for (int32_t t = k; t < e && pt.rc == CA_OK; t++) {    // AddPod of the copy (:79)
                if (t + 16 < nm && ((mv[t + 16].node >> 6) & tm) == w) {
                    __builtin_prefetch(&pods[(size_t)base + t + 16].spec);
                    __builtin_prefetch(&nodes[mv[t + 16].node]);
                }
                const int32_t x = mv[t].node;
                if (((x >> 6) & tm) != w) continue;
                const int32_t nid = base + t;
                NodeRow& nd = nodes[x];
                uint64_t before[CA_PORT_WORDS];
                std::memcpy(before, nd.ports, sizeof before);
                apply(x, pods[nid].spec, +1);
                nd.pods.push_back(nid);
                pods[nid].node = x;
                journal(J_ADD_POD, x, nid, (int32_t)nd.pods.size() - 1, before);
            }
            k = e;
        }
    });
    tmark("rows");
    // every part's changes are merged before an error is returned: a part that failed and the
    // parts after it have already changed rows, pod lists and pods[].node, and the caller's
    // revert-on-error (ca_plan_removals) can only undo what the journal holds and re-sync the
    // rows dirty_rows names
    int first_rc = CA_OK;
    for (Part& pt : part) {
        if (first_rc == CA_OK) first_rc = pt.rc;
        n_ext_pods += pt.ext;
        n_eph_pods += pt.eph;
        n_oos_pods += pt.oos;
        n_scope_blockers += pt.blockers;
        dirty_rows.insert(dirty_rows.end(), pt.dirty.begin(), pt.dirty.end());
        if (journaled) journal.insert(journal.end(), pt.jr.begin(), pt.jr.end());
    }
    tmark("merged");
    return first_rc;
}

// plan_chain.hip: the whole loop as one device-resident chain (1 = ran, 0 = outside its scope)
namespace casim {
int plan_chain_run(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                   const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                   int32_t max_removable, const ca_pdb_table* pdbs, int32_t* hints, int32_t n_pods,
                   int32_t* last_index, ca_plan_result* results, std::vector<ca_plan_move>& moves_out,
                   std::vector<std::pair<int32_t, int32_t>>& hint_sets, int32_t* simulated_out);
}  // namespace casim

namespace {

int plan_removals(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                  const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                  int32_t max_removable, const ca_pdb_table* pdbs, int32_t* hints, int32_t n_pods,
                  int32_t* last_index, ca_plan_result* results, ca_plan_move* moves, int32_t moves_cap,
                  int32_t* n_moves) {
    if (!m || C < 0 || !last_index || moves_cap < 0 || (moves_cap > 0 && !moves)) return CA_EINVAL;
    if (C > 0 && (!candidates || !dest_mask || !move_off || !results)) return CA_EINVAL;
    // pods past n_pods are records a Revert detached (ids are never reused): on no node
    if (n_pods < 0 || n_pods > (int32_t)m->pods.size()) return CA_EINVAL;
    const int P = pdbs ? pdbs->n_pdbs : 0;
    if (P < 0 || (P > 0 && (!pdbs->allowed || !pdbs->pod_off || !pdbs->pod_pdb))) return CA_EINVAL;
    const auto t0 = std::chrono::steady_clock::now();
    const int32_t N = (int32_t)m->nodes.size();
    PlanStats& ps = m->plan;
    ps.rounds = ps.conflicts = ps.simulated = 0;
    ps.moves.clear();
    if (C > 0 && (move_off[0] != 0)) return CA_EINVAL;
    for (int32_t c = 0; c < C; c++)
        if (move_off[c + 1] < move_off[c]) return CA_EINVAL;
    {   // every pod to move names a mirror pod (one flat pass: the offsets ascend)
        uint32_t bad = 0;
        const int32_t M = C > 0 ? move_off[C] : 0;
        for (int32_t i = 0; i < M; i++) bad |= (uint32_t)((uint32_t)move_pods[i] >= (uint32_t)n_pods);
        if (bad) return CA_EINVAL;
    }
    {   // the planner walks unique node names (planner.go:261)
        std::vector<uint8_t> seen((size_t)std::max(N, 1), 0);
        for (int32_t c = 0; c < C; c++) {
            const int32_t nd = candidates[c];
            if (nd < 0 || nd >= N) continue;
            if (seen[nd]) return CA_EINVAL;
            seen[nd] = 1;
        }
    }
    if (C == 0) {
        if (n_moves) *n_moves = 0;
        ps.total_ms = 0;
        return CA_OK;
    }
    if (m->n_scope_blockers > 0) return CA_EUNSUPPORTED;                         // casim.h scope
    const char* fail_env = test_hook_env("CASIM_PLAN_FAIL_ROUND");          // tests: an error in that round
    const int32_t fail_round = fail_env ? atoi(fail_env) : 0;
    {
        // the device-resident chain (plan_chain.hip); the speculative windows below otherwise
        int32_t sim = 0, Lc = *last_index;
        std::vector<std::pair<int32_t, int32_t>> hc;            // Hints.Set of the caller's pods (pod, node)
        const int rc = plan_chain_run(m, candidates, C, dest_mask, cand_status, move_off, move_pods, max_removable,
                                      pdbs, hints, n_pods, &Lc, results, ps.moves, hc, &sim);
        if (rc < 0) return rc;
        if (rc == 1) {
            ps.rounds = 1;
            ps.simulated = sim;
            ps.path = 1;
            if (fail_round == 1) {
                set_last_error("CASIM_PLAN_FAIL_ROUND: injected failure");
                return CA_EDEVICE;
            }
            *last_index = Lc;
            if (hints) for (const auto& e : hc) hints[e.first] = e.second;
            const int32_t nm = (int32_t)ps.moves.size();
            if (moves) std::memcpy(moves, ps.moves.data(), sizeof(ca_plan_move) * (size_t)std::min(nm, moves_cap));
            if (n_moves) *n_moves = nm;
            ps.total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
            return CA_OK;
        }
        ps.path = 0;
    }

    std::vector<uint8_t> mask(dest_mask, dest_mask + N);                         // podDestinations
    std::vector<int32_t> H(m->pods.size(), -1);                                   // Hints by pod (copies share)
    if (hints) std::memcpy(H.data(), hints, sizeof(int32_t) * (size_t)n_pods);
    std::vector<int32_t> origin(m->pods.size());                                  // pod -> caller pod (PDBs)
    for (size_t i = 0; i < origin.size(); i++) origin[i] = (int32_t)i;
    std::vector<std::vector<int32_t>> extra((size_t)N);                          // copies committed onto a node
    // this window's commits: nodes that gained pods, nodes that left the destination set
    std::vector<uint8_t> gained((size_t)std::max(N, 1), 0), gone((size_t)std::max(N, 1), 0);
    std::vector<int32_t> gained_list, gone_list;
    auto member = [&](int32_t pod, int p) {
        const int32_t o = origin[pod];
        for (int32_t k = pdbs->pod_off[o]; k < pdbs->pod_off[o + 1]; k++)
            if (pdbs->pod_pdb[k] == p) return true;
        return false;
    };

    int64_t L = *last_index;
    int32_t removed = 0;
    int32_t i = 0;
    int32_t W = std::min(C, 256);
    if (const char* e = test_hook_env("CASIM_PLAN_WINDOW")) W = std::max(1, std::min(C, atoi(e)));   // tests
    std::vector<int32_t> w_off, w_pods, w_status, w_dest, Hs;
    std::vector<ca_removal_result> w_res;
    std::vector<Own> own;
    std::vector<int32_t> list_tmp;
    bool done = false;
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    const char* why = "";

    auto not_run = [&](int32_t from) {
        for (int32_t c = from; c < C; c++) {
            ca_plan_result& r = results[c];
            std::memset(&r, 0, sizeof r);
            r.reason = CA_UNREMOVABLE_NOT_RUN;
            r.last_index_in = (int32_t)L;
            r.first_move = (int32_t)ps.moves.size();
            r.blocking_pod = -1;
        }
    };
    while (i < C && !done) {
        if (max_removable > 0 && removed >= max_removable) { not_run(i); break; }   // :268-271
        const int32_t j = std::min(C, i + std::max(W, 1));
        const auto t_build = std::chrono::steady_clock::now();
        // ---- 1. speculate candidates [i, j) from the committed state ----
        w_off.assign(1, 0);
        w_pods.clear();
        for (int32_t c = i; c < j; c++) {
            w_pods.insert(w_pods.end(), move_pods + move_off[c], move_pods + move_off[c + 1]);
            const int32_t nd = candidates[c];
            if (nd >= 0 && nd < N) w_pods.insert(w_pods.end(), extra[nd].begin(), extra[nd].end());
            w_off.push_back((int32_t)w_pods.size());
        }
        if (cand_status) w_status.assign(cand_status + i, cand_status + j);
        else w_status.assign((size_t)(j - i), 0);
        w_res.resize((size_t)(j - i));
        w_dest.assign(std::max<size_t>(w_pods.size(), 1), -1);
        Hs = H;
        int32_t Ls = (int32_t)L;
        if (w_pods.empty()) w_pods.push_back(0);          // (a valid pointer; move_off bounds it)
        const auto t_spec = std::chrono::steady_clock::now();
        int rc = ca_find_nodes_to_remove(m, candidates + i, j - i, mask.data(), w_status.data(), w_off.data(),
                                         w_pods.data(), Hs.data(), &Ls, w_res.data(), w_dest.data());
        if (rc == CA_OK && fail_round > 0 && ps.rounds + 1 == fail_round) {
            set_last_error("CASIM_PLAN_FAIL_ROUND: injected failure");
            rc = CA_EDEVICE;
        }
        if (rc != CA_OK) return rc;
        const auto t_val = std::chrono::steady_clock::now();
        ps.rounds++;
        ps.simulated += j - i;
        // ---- 2. validate in order, commit ----
        for (int32_t x : gained_list) gained[x] = 0;
        for (int32_t x : gone_list) gone[x] = 0;
        gained_list.clear();
        gone_list.clear();
        int32_t k = i;
        bool conflict = false;
        for (; k < j; k++) {
            if (max_removable > 0 && removed >= max_removable) break;
            const ca_removal_result& sr = w_res[k - i];
            const int32_t node = candidates[k];
            const int32_t mo = w_off[k - i], mn = w_off[k - i + 1] - mo;
            const int32_t* list = w_pods.data() + mo;
            const int64_t lout = k + 1 < j ? (int64_t)w_res[k + 1 - i].last_index_in : (int64_t)Ls;
            if (node >= 0 && node < N && gained[node]) { conflict = true; why = "grown"; break; }   // its pods to move grew
            ca_plan_result& r = results[k];
            std::memset(&r, 0, sizeof r);
            r.last_index_in = (int32_t)L;
            r.first_move = (int32_t)ps.moves.size();
            r.blocking_pod = -1;
            if (sr.reason == CA_UNREMOVABLE_OUT_OF_SCOPE) {                          // prefix protocol
                r.reason = sr.reason;
                not_run(k + 1);
                done = true;
                break;
            }
            const bool simulated = sr.reason == CA_UNREMOVABLE_NONE || sr.reason == CA_UNREMOVABLE_NO_PLACE;
            if (!simulated) { r.reason = sr.reason; continue; }                     // not in podDestinations / drain
            // checkPdbs with the remaining budgets (drain.go:73-90)
            for (int p = 0; p < P && r.blocking_pod < 0; p++) {
                if (pdbs->allowed[p] >= 1) continue;
                for (int32_t t = 0; t < mn; t++)
                    if (member(list[t], p)) { r.blocking_pod = list[t]; break; }
            }
            if (r.blocking_pod >= 0) {
                r.reason = CA_UNREMOVABLE_BLOCKED_BY_POD;
                // the speculation simulated it: later candidates started where it left lastIndex
                if (lout != L) { k++; conflict = true; why = "pdb"; break; }
                continue;
            }
            if (sr.last_index_in != (int32_t)L) { conflict = true; why = "chain"; break; }   // (cannot happen)
            // the trace under this window's commits
            const int32_t np = sr.n_placed;
            const bool failed = !sr.removable;
            int32_t Lc = N > 0 ? (int32_t)(((L % N) + N) % N) : 0;
            uint64_t skipped = 0;
            bool bad = false;
            own.clear();
            for (int32_t t = 0; t <= np && t < mn && !bad; t++) {
                if (t == np && !failed) break;
                const int32_t id = list[t];
                const ca_pod_spec q = moved_spec(m->pods[id].spec);
                const bool prefail = (q.flags & CA_POD_PREFILTER_FAIL) != 0;
                const int32_t h = H[id];
                if (h >= 0 && h < N && !prefail && gone[h]) { bad = true; why = "hint"; break; }   // the hint check may pass now
                if (t == np) {                                                       // the failed scan: all nodes
                    if (!prefail)
                        for (int32_t x : gone_list) skipped += scan_visits(m, x, q) ? 1 : 0;
                    break;
                }
                const int32_t f = w_dest[mo + t];
                if (f < 0 || f >= N || gone[f]) { bad = true; why = "gone"; break; }
                Own* o = nullptr;
                for (Own& e : own) if (e.node == f) { o = &e; break; }
                if (f != h) {                                                        // found by the scan [Lc, f]
                    const int32_t span = (f - Lc + N) % N;
                    for (int32_t x : gone_list)
                        if ((x - Lc + N) % N <= span && scan_visits(m, x, q)) skipped++;
                    Lc = f + 1 == N ? 0 : f + 1;
                }
                if (gained[f] && !dyn_fits(m, f, q, o)) { bad = true; why = "full"; break; }
                if (!o) {
                    own.push_back(Own{});
                    o = &own.back();
                    std::memset(o, 0, sizeof *o);
                    o->node = f;
                }
                o->cpu = wadd(o->cpu, q.req_milli_cpu); o->mem = wadd(o->mem, q.req_memory);
                o->eph = wadd(o->eph, q.req_ephemeral); o->pods++;
                for (int s = 0; s < CA_MAX_SCALAR; s++) o->sc[s] = wadd(o->sc[s], q.req_scalar[s]);
                for (int w = 0; w < CA_PORT_WORDS; w++) o->ports[w] |= q.port_use[w];
            }
            if (bad) { conflict = true; break; }
            // accepted: the committed simulation is the speculative one
            r.n_placed = np;
            r.evals = sr.evals - skipped;
            for (int32_t t = 0; t < mn; t++) H[list[t]] = Hs[list[t]];               // Hints.Set
            L = lout;
            if (!sr.removable) { r.reason = CA_UNREMOVABLE_NO_PLACE; continue; }
            // ---- commit (withForkedSnapshot, cluster.go:207-211) ----
            r.removable = 1;
            r.reason = CA_UNREMOVABLE_NONE;
            r.n_moves = mn;
            list_tmp.assign(list, list + mn);
            for (int32_t t = 0; t < mn; t++) (void)ca_mirror_remove_pod(m, list_tmp[t]);   // :228-233
            for (int32_t t = 0; t < mn; t++) {
                const int32_t f = w_dest[mo + t];
                const int32_t nid = m->store_moved_copy(list_tmp[t]);
                m->add_pod_to_node(nid, f);                                          // AddPod (:79)
                H.push_back(f);
                origin.push_back(origin[list_tmp[t]]);
                extra[f].push_back(nid);
                ps.moves.push_back(ca_plan_move{k, list_tmp[t], nid, f});
                if (!gained[f]) { gained[f] = 1; gained_list.push_back(f); }
            }
            mask[node] = 0;                                                          // planner.go:280
            gone[node] = 1;
            gone_list.push_back(node);
            removed++;
            if (P > 0) {
                for (int p = 0; p < P; p++) {                                        // CanRemovePods (basic.go:66-84)
                    int32_t count = 0;
                    for (int32_t t = 0; t < mn; t++)
                        if (member(list_tmp[t], p) && pdbs->allowed[p] < ++count) r.risky = 1;
                }
                for (int p = 0; p < P; p++)                                          // RemovePods (:86-95)
                    for (int32_t t = 0; t < mn; t++)
                        if (member(list_tmp[t], p)) pdbs->allowed[p]--;
            }
        }
        if (dbg_t)
            fprintf(stderr, "[plan] round %d: [%d,%d) build %.3f ms, spec %.3f ms, validate+commit %.3f ms, accepted %d%s%s\n",
                    ps.rounds, i, j, std::chrono::duration<double, std::milli>(t_spec - t_build).count(),
                    std::chrono::duration<double, std::milli>(t_val - t_spec).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_val).count(), k - i,
                    conflict ? ", conflict: " : "", conflict ? why : "");
        if (done) break;
        if (conflict) {
            ps.conflicts++;
            W = std::max(32, 2 * (k - i));
            i = k;
        } else {
            if (k == j) W = std::min(C, 2 * W);
            i = k;
        }
    }
    *last_index = (int32_t)L;
    if (hints) std::memcpy(hints, H.data(), sizeof(int32_t) * (size_t)n_pods);
    const int32_t nm = (int32_t)ps.moves.size();
    if (moves) std::memcpy(moves, ps.moves.data(), sizeof(ca_plan_move) * (size_t)std::min(nm, moves_cap));
    if (n_moves) *n_moves = nm;
    ps.total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CA_OK;
}

}  // namespace

extern "C" {

// All or nothing: the call runs inside a fork of its own, committed into the
// caller's state on success and reverted on any error — the mirror, the PDB budgets, the
// caller's hints and lastIndex are then exactly as before the call.
int ca_plan_removals(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                     const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                     int32_t max_removable, const ca_pdb_table* pdbs, int32_t* hints, int32_t n_pods,
                     int32_t* last_index, ca_plan_result* results, ca_plan_move* moves, int32_t moves_cap,
                     int32_t* n_moves) {
    if (!m) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));    // the chain's buffers and launches belong to the mirror's device
    std::vector<int32_t> allowed0;
    if (pdbs && pdbs->n_pdbs > 0 && pdbs->allowed) allowed0.assign(pdbs->allowed, pdbs->allowed + pdbs->n_pdbs);
    int rc = ca_mirror_fork(m);
    if (rc != CA_OK) return rc;
    rc = plan_removals(m, candidates, C, dest_mask, cand_status, move_off, move_pods, max_removable, pdbs, hints, n_pods,
                       last_index, results, moves, moves_cap, n_moves);
    if (rc != CA_OK) {
        const std::string err = last_error();
        (void)ca_mirror_revert(m);
        if (!allowed0.empty()) std::memcpy(pdbs->allowed, allowed0.data(), sizeof(int32_t) * allowed0.size());
        m->plan.moves.clear();
        if (n_moves) *n_moves = 0;
        set_last_error(err);
        return rc;
    }
    const auto t_c = std::chrono::steady_clock::now();
    rc = ca_mirror_commit(m);
    if (knob_env("CASIM_DEBUG_TIMING"))
        fprintf(stderr, "[plan] commit %.3f ms (journal %zu entries)\n",
                std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_c).count(), m->journal.size());
    return rc;
}

int ca_plan_last_path(const ca_mirror* m) { return m ? m->plan.path : CA_EINVAL; }

int ca_plan_chain_profile(const ca_mirror* m, uint64_t* cycles, int32_t cap, float* host_ms) {
    if (!m || cap < 0 || (cap > 0 && !cycles)) return CA_EINVAL;
    const int32_t k = (int32_t)m->plan.chain_prof.size();
    for (int32_t i = 0; i < k && i < cap; i++) cycles[i] = m->plan.chain_prof[i];
    if (host_ms) for (int i = 0; i < 5; i++) host_ms[i] = m->plan.host_ms[i];
    return k;
}

int ca_plan_last_moves(const ca_mirror* m, ca_plan_move* out, int32_t cap) {
    if (!m || cap < 0 || (cap > 0 && !out)) return CA_EINVAL;
    const int32_t nm = (int32_t)m->plan.moves.size();
    std::memcpy(out, m->plan.moves.data(), sizeof(ca_plan_move) * (size_t)std::min(nm, cap));
    return nm;
}

int ca_plan_stats(const ca_mirror* m, int32_t* rounds, int32_t* conflicts, int32_t* simulated, float* total_ms) {
    if (!m) return CA_EINVAL;
    // (the path of the last call: m->plan.path, 1 = device chain, 0 = speculative windows)
    if (rounds) *rounds = m->plan.rounds;
    if (conflicts) *conflicts = m->plan.conflicts;
    if (simulated) *simulated = m->plan.simulated;
    if (total_ms) *total_ms = m->plan.total_ms;
    return CA_OK;
}

}  // extern "C"
