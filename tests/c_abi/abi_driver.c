/*
 * abi_driver.c — a C caller of libcasim.so through include/casim.h only (what a cgo shim
 * compiles against): mirror -> FitsAnyNode / CheckPredicates -> Estimate (BASELINE C1:
 * 1000 pods of 500m / 1 GiB on a 4000m / 16 GiB / 110-pod template = 125 nodes,
 * binpacking_estimator_test.go semantics) -> FindNodesToRemove (two drainable candidates
 * whose pods fit elsewhere; destinations follow the rotating first fit) -> the kernel-scope prefix protocol ->
 * the multi-GPU entry points over two replicas (device 1 when there is one, else 0).
 * Prints one "key value" line per check and exits non-zero on the first failure.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "casim.h"

#define CHECK(expr)                                                                      \
    do {                                                                                 \
        int _rc = (expr);                                                                \
        if (_rc != CA_OK) {                                                              \
            fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #expr, _rc,     \
                    ca_status_string(_rc));                                              \
            return 1;                                                                    \
        }                                                                                \
    } while (0)
#define EXPECT(cond)                                                                     \
    do {                                                                                 \
        if (!(cond)) { fprintf(stderr, "%s:%d expected %s\n", __FILE__, __LINE__, #cond); return 1; } \
    } while (0)

static ca_node_spec node(int64_t milli, int64_t mem, int64_t pods, int32_t name) {
    ca_node_spec n;
    memset(&n, 0, sizeof n);
    n.alloc_milli_cpu = milli;
    n.alloc_memory = mem;
    n.alloc_pods = pods;
    n.name_id = name;
    return n;
}

static ca_pod_spec pod(int64_t milli, int64_t mem) {
    ca_pod_spec p;
    memset(&p, 0, sizeof p);
    p.req_milli_cpu = p.score_milli_cpu = milli;
    p.req_memory = p.score_memory = mem;
    p.aff_term_count = -1;
    p.node_name_id = -1;
    p.similar_class = -1;
    return p;
}

static ca_pod_table table(const ca_pod_spec* pods, int32_t n) {
    ca_pod_table t;
    memset(&t, 0, sizeof t);
    t.pods = pods;
    t.n_pods = n;
    return t;
}

int main(void) {
    if (ca_abi_version() != CASIM_ABI_VERSION) { fprintf(stderr, "ABI version mismatch\n"); return 1; }
    int32_t ndev = 0;
    CHECK(ca_device_count(&ndev));
    printf("devices %d\n", ndev);
    EXPECT(ndev > 0);

    ca_mirror* m = NULL;
    CHECK(ca_mirror_create(0, &m));
    const int64_t GI = 1024ll * 1024 * 1024;
    /* cluster_test.go:169-177: n2 holds p1, p2 (100m each, ReplicaSet), n3 holds p3 */
    ca_node_spec nodes[3] = {node(1000, 2000000, 100, 1), node(1000, 2000000, 100, 2), node(1000, 2000000, 100, 3)};
    int32_t first = -1;
    CHECK(ca_mirror_add_nodes(m, nodes, 3, &first));
    ca_pod_spec running[3] = {pod(100, 100000), pod(100, 100000), pod(100, 100000)};
    ca_pod_table rt = table(running, 3);
    int32_t idx[3] = {0, 1, 2}, pos[3] = {1, 1, 2}, ids[3];
    CHECK(ca_mirror_add_pods(m, &rt, idx, pos, 3, ids));

    /* FitsAnyNode: 950m fits only n1 (free 1000m); lastIndex moves past it */
    ca_pod_spec big = pod(950, 1000);
    ca_pod_table bt = table(&big, 1);
    ca_match_spec all;
    memset(&all, 0, sizeof all);
    all.kind = CA_MATCH_ALL;
    all.exclude = -1;
    int32_t li = 0, out = -1, pf = 0;
    uint64_t evals = 0;
    CHECK(ca_fits_any_node(m, &bt, 0, &all, &li, &out, &pf, &evals));
    printf("fits_any_node %d last_index %d evals %llu\n", out, li, (unsigned long long)evals);
    EXPECT(out == 0 && li == 1 && evals == 1);
    ca_pred_result pr;
    CHECK(ca_check_predicates(m, &bt, 0, 1, &pr));        /* n2: 800m free -> Insufficient cpu */
    printf("check_predicates type %d plugin %d reasons %u\n", pr.type, pr.plugin, pr.reasons);
    EXPECT(pr.type == CA_PRED_NOT_SCHEDULABLE && pr.plugin == CA_PLUGIN_NODE_RESOURCES_FIT &&
           (pr.reasons & CA_REASON_INSUFF_CPU));

    /* FindNodesToRemove(candidates n2, n3): p1, p2 move to n1; n3's p3 moves too */
    int32_t cand[2] = {1, 2};
    uint8_t dest[3] = {1, 1, 1};
    int32_t st[2] = {0, 0}, moff[3] = {0, 2, 3}, moves[3] = {ids[0], ids[1], ids[2]}, hints[3] = {-1, -1, -1};
    ca_removal_result rr[2];
    int32_t odest[3];
    li = 0;
    CHECK(ca_find_nodes_to_remove(m, cand, 2, dest, st, moff, moves, hints, &li, rr, odest));
    printf("find_nodes_to_remove removable %d %d dest %d %d %d last_index %d\n", rr[0].removable, rr[1].removable,
           odest[0], odest[1], odest[2], li);
    /* rotating first fit: p1 -> n1 (lastIndex 1), p2 skips n2 (the candidate) -> n3
     * (lastIndex 3 = 0), n3's p3 -> n1 (lastIndex 1); the CPU restatement agrees */
    EXPECT(rr[0].removable == 1 && rr[1].removable == 1 && odest[0] == 0 && odest[1] == 2 && odest[2] == 0);
    EXPECT(li == 1 && rr[1].last_index_in == 0);
    EXPECT(hints[ids[0]] == 0 && hints[ids[1]] == 2 && hints[ids[2]] == 0);          /* Hints.Set */
    const int32_t li_sweep = li;

    /* Estimate, BASELINE C1 */
    ca_pod_spec* pods = malloc(sizeof(ca_pod_spec) * 1000);
    int32_t* pidx = malloc(sizeof(int32_t) * 1000);
    for (int i = 0; i < 1000; i++) { pods[i] = pod(500, GI); pidx[i] = i; }
    ca_pod_table pt = table(pods, 1000);
    ca_podset* ps = NULL;
    CHECK(ca_podset_create(m, &pt, &ps));
    ca_template tmpl;
    memset(&tmpl, 0, sizeof tmpl);
    tmpl.node = node(4000, 16 * GI, 110, -1000);
    int32_t goff[2] = {0, 1000};
    ca_limiter lim = {0, 0};
    ca_estimate_result er;
    int32_t* sched = malloc(sizeof(int32_t) * 1000);
    li = 0;
    CHECK(ca_estimate_batch(m, ps, goff, pidx, &tmpl, 1, &lim, &li, &er, sched, NULL));
    printf("estimate node_count %d n_scheduled %d evals %llu\n", er.node_count, er.n_scheduled,
           (unsigned long long)er.evals);
    EXPECT(er.status == CA_OK && er.node_count == 125 && er.n_scheduled == 1000);

    /* the prepared plan, scheduled pods as 16-bit podset indices into page-locked memory */
    {
        ca_estimate_plan* plan = NULL;
        CHECK(ca_estimate_plan_create(m, ps, goff, pidx, &tmpl, 1, &plan));
        void* buf16 = NULL;
        CHECK(ca_host_alloc(sizeof(uint16_t) * 1000, &buf16));
        uint16_t* s16 = (uint16_t*)buf16;
        ca_estimate_result ep;
        int32_t lp = 0;
        CHECK(ca_estimate_plan_run_u16(plan, &lim, &lp, &ep, s16));
        int same = ep.node_count == er.node_count && ep.n_scheduled == er.n_scheduled && lp == li;
        for (int i = 0; i < 1000; i++) same &= (int32_t)s16[i] == sched[i];
        printf("plan u16 node_count %d same %d\n", ep.node_count, same);
        EXPECT(same);
        CHECK(ca_host_free(buf16));
        CHECK(ca_estimate_plan_destroy(plan));
    }

    /* ComputeExpansionOption: one-shot and with the node group resident (page-locked verdicts) */
    {
        int32_t samples[2] = {0, 999};
        ca_template big = tmpl, small = tmpl;
        small.node = node(400, 16 * GI, 110, -1001);        /* 400m free: a 500m pod does not fit */
        ca_template ng[2] = {big, small};
        uint8_t ok1[4];
        CHECK(ca_check_templates(m, ps, samples, 2, ng, 2, NULL, ok1));
        ca_expansion_plan* ep = NULL;
        CHECK(ca_expansion_plan_create(m, ng, 2, &ep));
        void* okb = NULL;
        CHECK(ca_host_alloc(4, &okb));
        uint8_t* ok2 = (uint8_t*)okb;
        CHECK(ca_expansion_plan_run(ep, ps, samples, 2, NULL, ok2));
        float kms = -1;
        CHECK(ca_expansion_plan_kernel_ms(ep, &kms));
        printf("expansion verdicts %d %d %d %d plan same %d\n", ok1[0], ok1[1], ok1[2], ok1[3],
               memcmp(ok1, ok2, 4) == 0);
        EXPECT(ok1[0] == 1 && ok1[1] == 1 && ok1[2] == 0 && ok1[3] == 0 && memcmp(ok1, ok2, 4) == 0 && kms >= 0);
        CHECK(ca_host_free(okb));
        CHECK(ca_expansion_plan_destroy(ep));
    }

    /* kernel scope: a group with an out-of-scope pod stops the batch (prefix protocol) */
    pods[999].flags |= CA_POD_OUT_OF_SCOPE;
    ca_podset* ps2 = NULL;
    CHECK(ca_podset_create(m, &pt, &ps2));
    int32_t goff2[3] = {0, 500, 1000};
    ca_template t2[2] = {tmpl, tmpl};
    ca_estimate_result er2[2];
    li = 0;
    CHECK(ca_estimate_batch(m, ps2, goff2, pidx, t2, 2, &lim, &li, er2, sched, NULL));
    printf("prefix status %d %d\n", er2[0].status, er2[1].status);
    EXPECT(er2[0].status == CA_OK && er2[1].status == CA_EUNSUPPORTED);

    /* multi-GPU entry: a replica of the cluster (same calls, same order) on a second mirror
     * (device ndev > 1 ? 1 : 0), the C1 batch split into 4 groups of 250 pods over the two
     * replicas, results equal the single-mirror batch of the same groups */
    pods[999].flags &= ~CA_POD_OUT_OF_SCOPE;
    ca_mirror* m2 = NULL;
    CHECK(ca_mirror_create(ndev > 1 ? 1 : 0, &m2));
    CHECK(ca_mirror_add_nodes(m2, nodes, 3, &first));
    int32_t ids2[3];
    CHECK(ca_mirror_add_pods(m2, &rt, idx, pos, 3, ids2));
    ca_mirror* reps[2] = {m, m2};
    ca_multi* mm = NULL;
    CHECK(ca_multi_create(reps, 2, &mm));
    int32_t goff4[5] = {0, 250, 500, 750, 1000};
    ca_template t4[4] = {tmpl, tmpl, tmpl, tmpl};
    ca_estimate_result e1[4], e2[4];
    int32_t* sched2 = malloc(sizeof(int32_t) * 1000);
    ca_podset* ps3 = NULL;
    CHECK(ca_podset_create(m, &pt, &ps3));
    int32_t l1 = 3, l2 = 3;
    CHECK(ca_estimate_batch(m, ps3, goff4, pidx, t4, 4, &lim, &l1, e1, sched, NULL));
    CHECK(ca_multi_estimate_batch(mm, &pt, goff4, pidx, t4, 4, &lim, &l2, e2, sched2, NULL));
    printf("multi estimate node_count %d %d %d %d last_index %d\n", e2[0].node_count, e2[1].node_count,
           e2[2].node_count, e2[3].node_count, l2);
    EXPECT(l1 == l2 && memcmp(e1, e2, sizeof e1) == 0 && memcmp(sched, sched2, sizeof(int32_t) * 1000) == 0);
    int32_t hints2[3] = {-1, -1, -1};
    ca_removal_result rr2[2];
    int32_t odest2[3];
    l2 = 0;
    CHECK(ca_multi_find_nodes_to_remove(mm, cand, 2, dest, st, moff, moves, hints2, 3, &l2, rr2, odest2));
    printf("multi find_nodes_to_remove removable %d %d last_index %d\n", rr2[0].removable, rr2[1].removable, l2);
    EXPECT(memcmp(rr, rr2, sizeof rr) == 0 && memcmp(odest, odest2, sizeof odest) == 0 && l2 == li_sweep);
    EXPECT(memcmp(hints, hints2, sizeof hints) == 0);
    CHECK(ca_multi_destroy(mm));
    CHECK(ca_podset_destroy(ps3));
    CHECK(ca_mirror_destroy(m2));
    free(sched2);

    /* RemoveNode shifts positions; Revert restores them */
    CHECK(ca_mirror_fork(m));
    CHECK(ca_mirror_remove_node(m, 0));
    int32_t nn = 0;
    CHECK(ca_mirror_node_count(m, &nn));
    EXPECT(nn == 2);
    CHECK(ca_mirror_revert(m));
    CHECK(ca_mirror_node_count(m, &nn));
    EXPECT(nn == 3);

    /* planner (canPersist=true) inside a fork: n2 is removed first (p1 -> n1, p2 -> n3,
     * committed), so n3's pods to move are p3 and the copy of p2; n2 is no destination any
     * more: p3 -> n1, p2's copy -> n1 (its hint, n3 itself, is checked but not acceptable) */
    CHECK(ca_mirror_fork(m));
    ca_plan_result pr2[2];
    ca_plan_move mv[8];
    int32_t hints3[3] = {-1, -1, -1}, nmv = 0;
    li = 0;
    CHECK(ca_plan_removals(m, cand, 2, dest, st, moff, moves, 0, NULL, hints3, 3, &li, pr2, mv, 8, &nmv));
    printf("plan_removals removable %d %d moves %d evals %llu %llu last_index %d\n", pr2[0].removable,
           pr2[1].removable, nmv, (unsigned long long)pr2[0].evals, (unsigned long long)pr2[1].evals, li);
    EXPECT(pr2[0].removable == 1 && pr2[1].removable == 1 && nmv == 4 && li == 1);
    EXPECT(pr2[0].first_move == 0 && pr2[0].n_moves == 2 && pr2[1].first_move == 2 && pr2[1].n_moves == 2);
    EXPECT(mv[0].pod == ids[0] && mv[0].node == 0 && mv[1].pod == ids[1] && mv[1].node == 2);
    EXPECT(mv[2].pod == ids[2] && mv[2].node == 0 && mv[3].pod == mv[1].new_pod && mv[3].node == 0);
    EXPECT(pr2[0].evals == 2 && pr2[1].evals == 3);
    int32_t on_n1[8], k1 = 0;
    CHECK(ca_mirror_node_pods(m, 0, on_n1, 8, &k1));
    EXPECT(k1 == 3);                                       /* p1', p3', p2'' */
    CHECK(ca_mirror_revert(m));
    CHECK(ca_mirror_node_pods(m, 0, on_n1, 8, &k1));
    EXPECT(k1 == 0);

    CHECK(ca_podset_destroy(ps));
    CHECK(ca_podset_destroy(ps2));
    CHECK(ca_mirror_destroy(m));
    free(pods); free(pidx); free(sched);
    printf("abi_driver ok\n");
    return 0;
}
