// multi.hip — multi-GPU entry points of the C ABI.
//
// A Go caller holds one mirror per device and applies every snapshot change to each (the
// snapshot is replicated: a C5 mirror is < 80 MB of a 288 GB HBM).  Estimate's node groups
// and FindNodesToRemove's candidates are coupled only through the checker's lastIndex
// (CA/simulator/predicatechecker/schedulerbased.go:43,131; cluster.go:130-137 for the
// sweep), so a batch splits into contiguous blocks, one per device, that run concurrently
// (one host thread per device) from the caller's lastIndex.  The chain is then fixed up
// here: walking the blocks in order, a block that ran from a wrong lastIndex is re-run
// from the exact one when its output depends on it (a FitsAnyNode success whose scan
// started at the input), and otherwise only has its lastIndex fields re-based.  No data
// crosses devices: every block writes its own slice of the caller's result arrays.
#include <thread>
#include <chrono>

#include "mirror.h"

using namespace casim;

namespace casim {
int32_t estimate_plan_rebase(const ca_estimate_plan* p, ca_estimate_result* results, int32_t lin);
}

struct ca_multi {
    std::vector<ca_mirror*> m;
};

namespace {

// run fn(d) for every block d, block 0 on the calling thread; first failure wins
template <class F>
int for_blocks(int32_t D, F&& fn) {
    if (D <= 0) return CA_OK;
    std::vector<int> rc((size_t)D, CA_OK);
    std::vector<std::thread> th;
    for (int32_t d = 1; d < D; d++) th.emplace_back([&, d] { rc[d] = fn(d); });
    rc[0] = fn(0);
    for (auto& t : th) t.join();
    for (int32_t d = 0; d < D; d++) if (rc[d] != CA_OK) return rc[d];
    return CA_OK;
}

// contiguous blocks of [0, n) with about equal weight (w[i] >= 0), at most D of them, none empty
std::vector<int32_t> split_blocks(int32_t n, int32_t D, const std::vector<int64_t>& w) {
    std::vector<int32_t> b{0};
    if (n == 0) { b.push_back(0); return b; }
    D = std::max(1, std::min(D, n));
    int64_t tot = 0;
    for (int32_t i = 0; i < n; i++) tot += std::max<int64_t>(w[i], 1);
    int64_t acc = 0;
    for (int32_t i = 0; i < n; i++) {
        acc += std::max<int64_t>(w[i], 1);
        const int32_t k = (int32_t)b.size();       // blocks closed so far + 1
        const bool room = n - (i + 1) >= D - k;     // enough items left for the remaining blocks
        if (k < D && i + 1 < n && room && acc * D >= tot * k) b.push_back(i + 1);
    }
    b.push_back(n);
    return b;
}

}  // namespace

struct ca_multi_estimate_plan {
    ca_multi* mm = nullptr;
    int32_t G = 0;
    std::vector<int32_t> off;                 // the caller's group_off
    std::vector<int32_t> gb;                  // block d = groups [gb[d], gb[d+1]) on mirror d
    std::vector<ca_podset*> ps;
    std::vector<ca_estimate_plan*> pl;
    int32_t reruns = 0;
    int32_t rerun_units = 0;                  // groups in the re-run blocks of the last run
    ~ca_multi_estimate_plan() {
        for (auto* p : pl) if (p) ca_estimate_plan_destroy(p);
        for (auto* s : ps) if (s) ca_podset_destroy(s);
    }
};

struct ca_multi_removal_plan {
    ca_multi* mm = nullptr;
    int32_t C = 0;
    std::vector<int32_t> off;                 // the caller's move_off
    std::vector<int32_t> cb;                  // block d = candidates [cb[d], cb[d+1])
    std::vector<int32_t> moves;               // the caller's move_pods
    std::vector<ca_removal_plan*> pl;
    std::vector<std::vector<int32_t>> hb;     // per block: the hints its run reads and writes
    int32_t reruns = 0;
    int32_t rerun_units = 0;                  // candidates in the re-run blocks of the last run
    float phase_ms[5] = {0, 0, 0, 0, 0};      // last run (host wall): probe, map, compose, resolve, fix-up
    ~ca_multi_removal_plan() {
        for (auto* p : pl) if (p) ca_removal_plan_destroy(p);
    }
};

extern "C" {

int ca_multi_create(ca_mirror* const* mirrors, int32_t n, ca_multi** out) {
    if (!mirrors || n <= 0 || !out) return CA_EINVAL;
    for (int32_t i = 0; i < n; i++) if (!mirrors[i]) return CA_EINVAL;
    ca_multi* mm = new ca_multi();
    mm->m.assign(mirrors, mirrors + n);
    *out = mm;
    return CA_OK;
}

int ca_multi_destroy(ca_multi* mm) {
    if (!mm) return CA_EINVAL;
    delete mm;
    return CA_OK;
}

// ---- Estimate -------------------------------------------------------------------------

int ca_multi_estimate_plan_create(ca_multi* mm, const ca_pod_table* t, const int32_t* group_off,
                                  const int32_t* pod_idx, const ca_template* templates, int32_t n_groups,
                                  ca_multi_estimate_plan** out) {
    if (!mm || !t || !group_off || !out || n_groups < 0 || (n_groups > 0 && !templates)) return CA_EINVAL;
    if (group_off[0] != 0) return CA_EINVAL;
    for (int32_t g = 0; g < n_groups; g++) if (group_off[g + 1] < group_off[g]) return CA_EINVAL;
    auto* p = new ca_multi_estimate_plan();
    p->mm = mm;
    p->G = n_groups;
    p->off.assign(group_off, group_off + n_groups + 1);
    std::vector<int64_t> w((size_t)n_groups);
    for (int32_t g = 0; g < n_groups; g++) w[g] = group_off[g + 1] - group_off[g];
    p->gb = split_blocks(n_groups, (int32_t)mm->m.size(), w);
    const int32_t D = (int32_t)p->gb.size() - 1;
    p->ps.assign((size_t)D, nullptr);
    p->pl.assign((size_t)D, nullptr);
    const int rc = for_blocks(D, [&](int32_t d) {
        const int32_t g0 = p->gb[d], g1 = p->gb[d + 1];
        int r = ca_podset_create(mm->m[d], t, &p->ps[d]);
        if (r != CA_OK) return r;
        std::vector<int32_t> loff((size_t)(g1 - g0 + 1));
        for (int32_t g = g0; g <= g1; g++) loff[g - g0] = group_off[g] - group_off[g0];
        return ca_estimate_plan_create(mm->m[d], p->ps[d], loff.data(), pod_idx + group_off[g0], templates + g0,
                                       g1 - g0, &p->pl[d]);
    });
    if (rc != CA_OK) { delete p; return rc; }
    *out = p;
    return CA_OK;
}

int ca_multi_estimate_plan_run(ca_multi_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                               ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node) {
    if (!p || !limiter || !last_index || (p->G > 0 && (!results || !sched_pod))) return CA_EINVAL;
    const int32_t D = (int32_t)p->gb.size() - 1;
    const int32_t L0 = *last_index;
    std::vector<int32_t> lin((size_t)D, L0), lout((size_t)D, L0), sens((size_t)D, 0), succ((size_t)D, 0);
    auto run = [&](int32_t d, int32_t from) {
        const int32_t g0 = p->gb[d];
        int32_t li = from;
        int r = ca_estimate_plan_run(p->pl[d], limiter, &li, results + g0, sched_pod + p->off[g0],
                                     sched_node ? sched_node + p->off[g0] : nullptr);
        if (r != CA_OK) return r;
        lin[d] = from;
        lout[d] = li;
        return ca_estimate_plan_chain_info(p->pl[d], &sens[d], &succ[d]);
    };
    int rc = for_blocks(D, [&](int32_t d) { return run(d, L0); });
    if (rc != CA_OK) return rc;
    // the lastIndex chain over the blocks (prefix protocol: after a block that stopped at an
    // unsupported group, nothing runs)
    p->reruns = 0;
    p->rerun_units = 0;
    int32_t cur = L0;
    bool cut = false;
    for (int32_t d = 0; d < D; d++) {
        const int32_t g0 = p->gb[d], g1 = p->gb[d + 1];
        if (cut) {
            for (int32_t g = g0; g < g1; g++) {
                ca_estimate_result& r = results[g];
                r.node_count = r.n_scheduled = r.nodes_added = 0;
                r.last_index_in = r.last_index_out = cur;
                r.status = CA_ENOTRUN;
                r.evals = 0;
            }
            std::fill(sched_pod + p->off[g0], sched_pod + p->off[g1], -1);
            if (sched_node) std::fill(sched_node + p->off[g0], sched_node + p->off[g1], -1);
            continue;
        }
        if (lin[d] != cur) {
            if (sens[d]) {                                   // depends on its input: run it again
                if ((rc = run(d, cur)) != CA_OK) return rc;
                p->reruns++;
                p->rerun_units += g1 - g0;
            } else {                                         // same outputs from any input
                lout[d] = casim::estimate_plan_rebase(p->pl[d], results + g0, cur);
                lin[d] = cur;
            }
        }
        cur = lout[d];
        for (int32_t g = g0; g < g1; g++) if (results[g].status == CA_EUNSUPPORTED) cut = true;
    }
    *last_index = cur;
    return CA_OK;
}

int ca_multi_estimate_plan_stats(const ca_multi_estimate_plan* p, int32_t* n_blocks, int32_t* reruns,
                                 int32_t* block_first_group, int32_t cap) {
    if (!p) return CA_EINVAL;
    const int32_t D = (int32_t)p->gb.size() - 1;
    if (n_blocks) *n_blocks = D;
    if (reruns) *reruns = p->reruns;
    if (block_first_group)
        for (int32_t d = 0; d <= D && d < cap; d++) block_first_group[d] = p->gb[d];
    return CA_OK;
}

int ca_multi_estimate_plan_rerun_units(const ca_multi_estimate_plan* p, int32_t* groups_rerun) {
    if (!p || !groups_rerun) return CA_EINVAL;
    *groups_rerun = p->rerun_units;
    return CA_OK;
}

int ca_multi_estimate_plan_destroy(ca_multi_estimate_plan* p) {
    if (!p) return CA_EINVAL;
    delete p;
    return CA_OK;
}

int ca_multi_estimate_batch(ca_multi* mm, const ca_pod_table* t, const int32_t* group_off, const int32_t* pod_idx,
                            const ca_template* templates, int32_t n_groups, const ca_limiter* limiter,
                            int32_t* last_index, ca_estimate_result* results, int32_t* sched_pod,
                            int32_t* sched_node) {
    ca_multi_estimate_plan* p = nullptr;
    int rc = ca_multi_estimate_plan_create(mm, t, group_off, pod_idx, templates, n_groups, &p);
    if (rc != CA_OK) return rc;
    rc = ca_multi_estimate_plan_run(p, limiter, last_index, results, sched_pod, sched_node);
    ca_multi_estimate_plan_destroy(p);
    return rc;
}

// ---- FindNodesToRemove --------------------------------------------------------------------

int ca_multi_removal_plan_create(ca_multi* mm, const int32_t* candidates, int32_t n_candidates,
                                 const uint8_t* dest_mask, const int32_t* cand_status, const int32_t* move_off,
                                 const int32_t* move_pods, ca_multi_removal_plan** out) {
    const int32_t C = n_candidates;
    if (!mm || !out || C < 0 || (C > 0 && (!candidates || !dest_mask || !move_off))) return CA_EINVAL;
    if (C > 0 && move_off[0] != 0) return CA_EINVAL;
    for (int32_t c = 0; c < C; c++) if (move_off[c + 1] < move_off[c]) return CA_EINVAL;
    auto* p = new ca_multi_removal_plan();
    p->mm = mm;
    p->C = C;
    p->off.assign(move_off, move_off + C + 1);
    if (C > 0) p->moves.assign(move_pods, move_pods + move_off[C]);
    std::vector<int64_t> w((size_t)C);                 // work ~ pods to move
    for (int32_t c = 0; c < C; c++) w[c] = move_off[c + 1] - move_off[c];
    p->cb = split_blocks(C, (int32_t)mm->m.size(), w);
    const int32_t D = (int32_t)p->cb.size() - 1;
    p->pl.assign((size_t)D, nullptr);
    p->hb.resize((size_t)D);
    const int rc = for_blocks(D, [&](int32_t d) {
        const int32_t c0 = p->cb[d], c1 = p->cb[d + 1];
        std::vector<int32_t> loff((size_t)(c1 - c0 + 1));
        for (int32_t c = c0; c <= c1; c++) loff[c - c0] = move_off[c] - move_off[c0];
        return ca_removal_plan_create(mm->m[d], candidates + c0, c1 - c0, dest_mask, cand_status ? cand_status + c0 : nullptr,
                                      loff.data(), move_pods + move_off[c0], &p->pl[d]);
    });
    if (rc != CA_OK) { delete p; return rc; }
    *out = p;
    return CA_OK;
}

// The blocks' lastIndex chain from their MAP records: a block without a
// successful probe scan passes lastIndex through; otherwise the class of its input in its
// first row's fit points picks its map entry, the next block's input.  The walk stops at the
// first block whose map is missing or does not cover its input.
int ca_sweep_compose(const ca_sweep_phase* ph, int32_t D, int32_t n, int32_t L0, int32_t* lin_c, int32_t* n_reached) {
    if (D < 0 || (D > 0 && (!ph || !lin_c)) || n < 0) return CA_EINVAL;
    for (int32_t d = 0; d < D; d++) lin_c[d] = CA_SWEEP_NOT_REACHED;
    if (n_reached) *n_reached = 0;
    if (n == 0) return CA_OK;
    int64_t cur = L0;
    int32_t reached = 0;
    for (int32_t d = 0; d < D; d++) {
        if (ph[d].n_sensitive == 0 || ph[d].succ == 0) {   // no scan can succeed: lastIndex passes through
            lin_c[d] = (int32_t)cur;
            reached++;
            continue;
        }
        if (!ph[d].map_ok) break;
        const int32_t* mp = ph[d].map;
        const int32_t* head = mp + SWEEP_MAP_HEAD;
        const int32_t Lw = (int32_t)(((cur % n) + n) % n);
        int32_t x;
        if (mp[SWEEP_MAP_MODE]) {
            x = casim::sweep_fp_class(head, n, Lw);
        } else {
            x = Lw - head[1];
            if (x < 0) x += n;
            if (x >= 64) x = -1;
        }
        if (x < 0 || mp[x] < 0) break;
        lin_c[d] = (int32_t)cur;
        reached++;
        cur = mp[x];
    }
    if (n_reached) *n_reached = reached;
    return CA_OK;
}

int ca_multi_removal_plan_run(ca_multi_removal_plan* p, int32_t* hints, int32_t n_pods, int32_t* last_index,
                              ca_removal_result* results, int32_t* out_dest) {
    // (no resident-hint mode: a block re-run must start from the caller's hints again)
    if (!p || !last_index || n_pods < 0 || (p->C > 0 && !results)) return CA_EINVAL;
    const int32_t D = (int32_t)p->cb.size() - 1;
    for (int32_t d = 0; d < D; d++)
        if ((int32_t)p->mm->m[d]->pods.size() != n_pods) return CA_EINVAL;      // replicas: same pod ids
    const int32_t L0 = *last_index;
    const int32_t n = D > 0 ? (int32_t)p->mm->m[0]->nodes.size() : 0;
    std::vector<int32_t> lin((size_t)D, L0), lout((size_t)D, L0), succ((size_t)D, 0);
    std::vector<uint8_t> ran((size_t)D, 0);
    std::vector<int32_t> none;                              // (no caller hints: every pod unhinted)
    if (!hints) none.assign((size_t)std::max(n_pods, 1), -1);
    auto run = [&](int32_t d, int32_t from, SweepPhase* ph) {
        const int32_t c0 = p->cb[d];
        int32_t* hp;
        if (ph && (ph->kind == SP_PROBE || ph->kind == SP_MAP)) {
            hp = hints ? hints : none.data();               // (read only: gathered per moved pod)
        } else {
            std::vector<int32_t>& h = p->hb[d];             // the caller's hints, fresh for every run
            if (hints) h.assign(hints, hints + n_pods);
            else h.assign((size_t)n_pods, -1);
            hp = h.data();
        }
        int32_t li = from;
        int r = removal_plan_run_phase(p->pl[d], hp, &li, results + c0, out_dest ? out_dest + p->off[c0] : nullptr, ph);
        if (r != CA_OK) return r;
        if (ph && (ph->kind == SP_PROBE || ph->kind == SP_MAP)) return CA_OK;
        lin[d] = from;
        lout[d] = li;
        succ[d] = p->mm->m[d]->sweep_stats.had_success;
        ran[d] = 1;
        return CA_OK;
    };
    p->reruns = 0;
    p->rerun_units = 0;
    for (float& v : p->phase_ms) v = 0;
    auto clk = std::chrono::steady_clock::now();
    auto lap = [&](int i) {
        const auto t = std::chrono::steady_clock::now();
        p->phase_ms[i] = std::chrono::duration<float, std::milli>(t - clk).count();
        clk = t;
    };
    int rc;
    // ---- the ranges' lastIndex classes, composed on the host ----
    // 1. every range probes its candidates (guesses from the pods before it) and reports its
    //    advance; 2. every range centres its windows on the previous ranges' advances, builds
    //    its tables and its block map (lastIndex out by class of its first row's input);
    //    3. the maps compose in order from the true input, and every range whose input falls
    //    in its first window resolves from it, all at once.  A range the composition does
    //    not reach (a walk that leaves its windows, a scope cut) runs after its predecessor
    //    from the exact input, as before.
    bool phased = D > 1 && n > 0 && !knob_env("CASIM_MULTI_NO_MAP");
    for (int32_t d = 0; d < D && phased; d++) if (p->pl[d] && !removal_plan_phase_ok(p->pl[d])) phased = false;
    std::vector<int32_t> lin_c((size_t)D, CA_SWEEP_NOT_REACHED);   // composed input of each range
    if (phased) {
        std::vector<SweepPhase> ph((size_t)D);
        int64_t gb = L0;
        for (int32_t d = 0; d < D; d++) {
            ph[d].kind = SP_PROBE;
            ph[d].guess_base = gb;
            gb += removal_plan_sensitive_pods(p->pl[d]);
        }
        if ((rc = for_blocks(D, [&](int32_t d) { return run(d, L0, &ph[d]); })) != CA_OK) return rc;
        lap(0);
        int64_t est = L0;
        std::vector<int32_t> mapped;                          // ranges whose output can depend on their input
        for (int32_t d = 0; d < D; d++) {
            ph[d].kind = SP_MAP;
            ph[d].est_base = (int32_t)(((est % n) + n) % n);
            est += ph[d].adv;
            // every range with sensitive candidates builds its tables here, including one whose
            // probe made no successful scan (its lastIndex passes through the composition): its
            // resolve walks the tables from the true input, so they must be this call's (a range
            // left out would walk the tables and chunk maps of an earlier call)
            if (ph[d].n_sensitive > 0) mapped.push_back(d);
        }
        if ((rc = for_blocks((int32_t)mapped.size(), [&](int32_t i) { return run(mapped[i], L0, &ph[mapped[i]]); })) !=
            CA_OK)
            return rc;
        lap(1);
        ca_sweep_compose(ph.data(), D, n, L0, lin_c.data(), nullptr);
        lap(2);
        for (int32_t d = 0; d < D; d++) ph[d].kind = SP_RESOLVE;
        std::vector<int32_t> todo;
        for (int32_t d = 0; d < D; d++) if (lin_c[d] != CA_SWEEP_NOT_REACHED) todo.push_back(d);
        if ((rc = for_blocks((int32_t)todo.size(), [&](int32_t i) {
                 const int32_t d = todo[i];
                 return run(d, lin_c[d], &ph[d]);
             })) != CA_OK)
            return rc;
        lap(3);
    } else {
        if ((rc = for_blocks(D, [&](int32_t d) { return run(d, L0, nullptr); })) != CA_OK) return rc;
        lap(3);
    }
    int32_t cur = L0;
    bool cut = false;
    for (int32_t d = 0; d < D; d++) {
        const int32_t c0 = p->cb[d], c1 = p->cb[d + 1];
        if (cut) {                                            // prefix protocol: not run
            for (int32_t c = c0; c < c1; c++) {
                ca_removal_result& r = results[c];
                r.removable = 0;
                r.reason = CA_UNREMOVABLE_NOT_RUN;
                r.n_placed = 0;
                r.last_index_in = cur;
                r.evals = 0;
            }
            if (out_dest) std::fill(out_dest + p->off[c0], out_dest + p->off[c1], -1);
            continue;
        }
        if (!ran[d] || (lin[d] != cur && succ[d])) {         // not reached, or ran from a wrong input
            if ((rc = run(d, cur, nullptr)) != CA_OK) return rc;
            p->reruns++;
            p->rerun_units += c1 - c0;
        } else if (lin[d] != cur) {                          // no scan succeeded: lastIndex passes through
            for (int32_t c = c0; c < c1; c++) results[c].last_index_in = cur;
            lin[d] = lout[d] = cur;
        }
        cur = lout[d];
        for (int32_t c = c0; c < c1; c++) if (results[c].reason == CA_UNREMOVABLE_OUT_OF_SCOPE) cut = true;
        // Hints.Set by the block: the hints of its own candidates' pods (the pods of one node
        // belong to one candidate), from the buffer its accepted run wrote
        if (hints)
            for (int32_t i = p->off[c0]; i < p->off[c1]; i++) {
                const int32_t id = p->moves[i];
                hints[id] = p->hb[d][id];
            }
    }
    *last_index = cur;
    lap(4);
    return CA_OK;
}

}  // extern "C"

extern "C" {

int ca_multi_removal_plan_stats(const ca_multi_removal_plan* p, int32_t* n_blocks, int32_t* reruns,
                                int32_t* block_first_candidate, int32_t cap) {
    if (!p) return CA_EINVAL;
    const int32_t D = (int32_t)p->cb.size() - 1;
    if (n_blocks) *n_blocks = D;
    if (reruns) *reruns = p->reruns;
    if (block_first_candidate)
        for (int32_t d = 0; d <= D && d < cap; d++) block_first_candidate[d] = p->cb[d];
    return CA_OK;
}

int ca_multi_removal_plan_rerun_units(const ca_multi_removal_plan* p, int32_t* candidates_rerun) {
    if (!p || !candidates_rerun) return CA_EINVAL;
    *candidates_rerun = p->rerun_units;
    return CA_OK;
}

int ca_multi_removal_plan_timings(const ca_multi_removal_plan* p, float* ms, int32_t cap) {
    if (!p || (cap > 0 && !ms)) return CA_EINVAL;
    for (int32_t i = 0; i < cap && i < 5; i++) ms[i] = p->phase_ms[i];
    return 5;
}

int ca_multi_removal_plan_destroy(ca_multi_removal_plan* p) {
    if (!p) return CA_EINVAL;
    delete p;
    return CA_OK;
}

int ca_multi_find_nodes_to_remove(ca_multi* mm, const int32_t* candidates, int32_t n_candidates,
                                  const uint8_t* dest_mask, const int32_t* cand_status, const int32_t* move_off,
                                  const int32_t* move_pods, int32_t* hints, int32_t n_pods, int32_t* last_index,
                                  ca_removal_result* results, int32_t* out_dest) {
    ca_multi_removal_plan* p = nullptr;
    int rc = ca_multi_removal_plan_create(mm, candidates, n_candidates, dest_mask, cand_status, move_off, move_pods, &p);
    if (rc != CA_OK) return rc;
    rc = ca_multi_removal_plan_run(p, hints, n_pods, last_index, results, out_dest);
    ca_multi_removal_plan_destroy(p);
    return rc;
}

}  // extern "C"
