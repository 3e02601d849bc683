/*
 * casim_oracle.c — CPU restatement of the scheduling-simulation hot path.
 * TEST INFRASTRUCTURE ONLY (see casim_oracle.h).  Single-threaded, like the
 * reference's RunOnce goroutine.
 *
 * CA/ = /root/reference/cluster-autoscaler/
 * SF/ = CA/vendor/k8s.io/kubernetes/pkg/scheduler/framework/
 */
#include "casim_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* growable arrays                                                            */
/* ------------------------------------------------------------------------- */
#define VEC(T) struct { T* a; int64_t n, cap; }
#define VEC_PUSH(v, x)                                                        \
    do {                                                                      \
        if ((v).n == (v).cap) {                                               \
            (v).cap = (v).cap ? (v).cap * 2 : 16;                             \
            (v).a = realloc((v).a, (size_t)(v).cap * sizeof(*(v).a));         \
        }                                                                     \
        (v).a[(v).n++] = (x);                                                 \
    } while (0)

typedef VEC(int32_t) vec_i32;

/* A node row: NodeInfo (SF/types.go:381-441).  Requested is kept as the
 * reference keeps it (sum of pod requests), the check is alloc - requested. */
typedef struct or_node {
    ca_node_spec spec;
    int64_t req_cpu, req_mem, req_eph;
    int64_t req_scalar[CA_MAX_SCALAR];
    int64_t npods;                    /* len(NodeInfo.Pods) (incl. template pods)  */
    uint64_t ports[CA_PORT_WORDS];    /* UsedPorts as a set of interned triples    */
    vec_i32 pods;                     /* NodeInfo.Pods order (mirror pod ids)      */
} or_node;

typedef struct or_pod {
    ca_pod_spec spec;                 /* terms re-indexed into the state's tables  */
    int32_t node;                     /* -1 when removed                           */
} or_pod;

/* undo journal entries (DeltaClusterSnapshot fork semantics, delta.go:43-475) */
enum { J_FORK = 1, J_ADD_NODE, J_ADD_POD, J_REMOVE_POD, J_REMOVE_NODE };
typedef struct or_jent {
    int32_t kind;
    int32_t node;
    int32_t pod;
    int32_t slot;                     /* index in node.pods the removed pod had    */
    uint64_t ports[CA_PORT_WORDS];    /* node ports before the operation           */
} or_jent;

struct or_state {
    VEC(or_node) nodes;
    VEC(or_pod) pods;
    VEC(ca_selector_term) terms;
    VEC(ca_selector_req) reqs;
    VEC(int32_t) pf_names;
    VEC(or_jent) journal;
    VEC(or_node) removed;             /* rows of journaled RemoveNode ops          */
    int32_t depth;
    int32_t next_new_name;            /* fresh name ids for template copies        */
    int64_t scope_blockers;           /* pods with CA_POD_REQUIRED_ANTI_AFFINITY   */
    int32_t sort_mode;                /* Estimate's sort.Slice: OR_SORT_STABLE / OR_SORT_GO_PDQ */
};

static int64_t wrap_sub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static int64_t wrap_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

or_state* or_create(void) {
    or_state* s = calloc(1, sizeof(or_state));
    if (s) s->sort_mode = OR_SORT_GO_PDQ;       /* the reference's sort.Slice (binpacking_estimator.go:74) */
    s->next_new_name = -2;
    return s;
}

static void free_nodes(or_state* s) {
    for (int64_t i = 0; i < s->nodes.n; i++) free(s->nodes.a[i].pods.a);
    s->nodes.n = 0;
}

static void free_removed(or_state* s) {
    for (int64_t i = 0; i < s->removed.n; i++) free(s->removed.a[i].pods.a);
    s->removed.n = 0;
}

void or_destroy(or_state* s) {
    if (!s) return;
    free_nodes(s);
    free_removed(s);
    free(s->nodes.a); free(s->pods.a); free(s->terms.a); free(s->reqs.a);
    free(s->pf_names.a); free(s->journal.a); free(s->removed.a);
    free(s);
}

int or_clear(or_state* s) {                       /* ClusterSnapshot.Clear() */
    free_nodes(s);
    free_removed(s);
    s->pods.n = s->terms.n = s->reqs.n = s->pf_names.n = s->journal.n = 0;
    s->depth = 0;
    s->next_new_name = -2;
    s->scope_blockers = 0;
    return CA_OK;
}

/* pods in the snapshot that make every simulation out of kernel scope (include/casim.h
 * "kernel scope"): InterPodAffinity's PreFilter does not Skip while a pod with required
 * anti-affinity exists (interpodaffinity/filtering.go:230-268) */
static void scope_count(or_state* s, const ca_pod_spec* p, int sign) {
    if (p->flags & CA_POD_REQUIRED_ANTI_AFFINITY) s->scope_blockers += sign;
}

int or_scope_blockers(const or_state* s) { return (int)s->scope_blockers; }

/* Estimate's sort of the pods by score (binpacking_estimator.go:74): OR_SORT_GO_PDQ (the
 * default) is the reference's Go 1.19 sort.Slice (gosort.c), OR_SORT_STABLE breaks score
 * ties by list position (the device's CASIM_SORT_ORDER=stable knob). */
int or_set_sort_mode(or_state* s, int32_t mode) {
    if (mode != OR_SORT_STABLE && mode != OR_SORT_GO_PDQ) return CA_EINVAL;
    s->sort_mode = mode;
    return CA_OK;
}

int or_node_count(const or_state* s) { return (int)s->nodes.n; }

static void journal(or_state* s, int32_t kind, int32_t node, int32_t pod, int32_t slot,
                    const uint64_t* ports) {
    if (s->depth == 0 && kind != J_FORK) return; /* unforked mutations are permanent */
    or_jent e;
    memset(&e, 0, sizeof e);
    e.kind = kind; e.node = node; e.pod = pod; e.slot = slot;
    if (ports) memcpy(e.ports, ports, sizeof e.ports);
    VEC_PUSH(s->journal, e);
}

static void add_node_row(or_state* s, const ca_node_spec* spec) {
    or_node nd;
    memset(&nd, 0, sizeof nd);
    nd.spec = *spec;
    VEC_PUSH(s->nodes, nd);
}

int or_add_nodes(or_state* s, const ca_node_spec* nodes, int32_t n, int32_t* out_first) {
    if (out_first) *out_first = (int32_t)s->nodes.n;
    for (int32_t i = 0; i < n; i++) {
        add_node_row(s, &nodes[i]);
        journal(s, J_ADD_NODE, (int32_t)s->nodes.n - 1, -1, -1, NULL);
    }
    return CA_OK;
}

/* NodeInfo.update(pod, +1) (SF/types.go:672-692) */
static void node_apply(or_node* nd, const ca_pod_spec* p, int sign) {
    nd->req_cpu = sign > 0 ? wrap_add(nd->req_cpu, p->req_milli_cpu) : wrap_sub(nd->req_cpu, p->req_milli_cpu);
    nd->req_mem = sign > 0 ? wrap_add(nd->req_mem, p->req_memory) : wrap_sub(nd->req_mem, p->req_memory);
    nd->req_eph = sign > 0 ? wrap_add(nd->req_eph, p->req_ephemeral) : wrap_sub(nd->req_eph, p->req_ephemeral);
    for (int i = 0; i < CA_MAX_SCALAR; i++)
        nd->req_scalar[i] = sign > 0 ? wrap_add(nd->req_scalar[i], p->req_scalar[i])
                                     : wrap_sub(nd->req_scalar[i], p->req_scalar[i]);
    nd->npods += sign;
    /* updateUsedPorts: HostPortInfo is a set; Remove deletes the triple even if
     * another pod on the node also uses it (SF/types.go:772-784, 863-880). */
    for (int w = 0; w < CA_PORT_WORDS; w++)
        nd->ports[w] = sign > 0 ? (nd->ports[w] | p->port_use[w]) : (nd->ports[w] & ~p->port_use[w]);
}

/* copy a pod record and its selector side tables into the state */
static int32_t store_pod(or_state* s, const ca_pod_table* t, int32_t idx, int32_t node) {
    or_pod op;
    op.spec = t->pods[idx];
    op.node = node;
    if (op.spec.aff_term_count > 0) {
        int32_t first = (int32_t)s->terms.n;
        for (int32_t k = 0; k < op.spec.aff_term_count; k++) {
            ca_selector_term tm = t->terms[op.spec.aff_term_first + k];
            int32_t rfirst = (int32_t)s->reqs.n;
            for (int32_t r = 0; r < tm.count; r++) VEC_PUSH(s->reqs, t->reqs[tm.first + r]);
            tm.first = rfirst;
            VEC_PUSH(s->terms, tm);
        }
        op.spec.aff_term_first = first;
    }
    if ((op.spec.flags & CA_POD_PREFILTER_NAMES) && op.spec.prefilter_count > 0) {
        int32_t first = (int32_t)s->pf_names.n;
        for (int32_t k = 0; k < op.spec.prefilter_count; k++)
            VEC_PUSH(s->pf_names, t->prefilter_names[op.spec.prefilter_first + k]);
        op.spec.prefilter_first = first;
    }
    VEC_PUSH(s->pods, op);
    return (int32_t)s->pods.n - 1;
}

/* ClusterSnapshot.AddPod (delta.go:209-230 -> NodeInfo.AddPod SF/types.go:602-619) */
static void add_pod_to_node(or_state* s, int32_t pod_id, int32_t node) {
    or_node* nd = &s->nodes.a[node];
    uint64_t before[CA_PORT_WORDS];
    memcpy(before, nd->ports, sizeof before);
    node_apply(nd, &s->pods.a[pod_id].spec, +1);
    scope_count(s, &s->pods.a[pod_id].spec, +1);
    VEC_PUSH(nd->pods, pod_id);
    s->pods.a[pod_id].node = node;
    journal(s, J_ADD_POD, node, pod_id, (int32_t)nd->pods.n - 1, before);
}

int or_add_pods(or_state* s, const ca_pod_table* t, const int32_t* pod_idx,
                const int32_t* node_pos, int32_t n, int32_t* out_ids) {
    for (int32_t i = 0; i < n; i++) {
        if (node_pos[i] < 0 || node_pos[i] >= s->nodes.n) return CA_ENOTFOUND;
        if (pod_idx[i] < 0 || pod_idx[i] >= t->n_pods) return CA_EINVAL;
        int32_t id = store_pod(s, t, pod_idx[i], node_pos[i]);
        add_pod_to_node(s, id, node_pos[i]);
        if (out_ids) out_ids[i] = id;
    }
    return CA_OK;
}

/* NodeInfo.RemovePod: swap-with-last removal (SF/types.go:645-670) */
int or_remove_pod(or_state* s, int32_t pod_id) {
    if (pod_id < 0 || pod_id >= s->pods.n || s->pods.a[pod_id].node < 0) return CA_ENOTFOUND;
    int32_t node = s->pods.a[pod_id].node;
    or_node* nd = &s->nodes.a[node];
    int64_t slot = -1;
    for (int64_t i = 0; i < nd->pods.n; i++)
        if (nd->pods.a[i] == pod_id) { slot = i; break; }
    if (slot < 0) return CA_ENOTFOUND;
    uint64_t before[CA_PORT_WORDS];
    memcpy(before, nd->ports, sizeof before);
    nd->pods.a[slot] = nd->pods.a[nd->pods.n - 1];
    nd->pods.n--;
    node_apply(nd, &s->pods.a[pod_id].spec, -1);
    scope_count(s, &s->pods.a[pod_id].spec, -1);
    s->pods.a[pod_id].node = -1;
    journal(s, J_REMOVE_POD, node, pod_id, (int32_t)slot, before);
    return CA_OK;
}

/* ClusterSnapshot.RemoveNode (clustersnapshot.go:38, delta.go:150-186): the NodeInfo and
 * its pods leave the snapshot; canonical order keeps the other nodes'
 * relative order, so later positions shift down by one. */
int or_remove_node(or_state* s, int32_t pos) {
    if (pos < 0 || pos >= s->nodes.n) return CA_ENOTFOUND;
    or_node row = s->nodes.a[pos];
    memmove(&s->nodes.a[pos], &s->nodes.a[pos + 1], (size_t)(s->nodes.n - pos - 1) * sizeof(or_node));
    s->nodes.n--;
    for (int64_t i = 0; i < row.pods.n; i++) {
        s->pods.a[row.pods.a[i]].node = -1;
        scope_count(s, &s->pods.a[row.pods.a[i]].spec, -1);
    }
    for (int64_t i = 0; i < s->pods.n; i++) if (s->pods.a[i].node > pos) s->pods.a[i].node--;
    if (s->depth > 0) {
        journal(s, J_REMOVE_NODE, pos, -1, (int32_t)s->removed.n, NULL);
        VEC_PUSH(s->removed, row);
    } else {
        free(row.pods.a);
    }
    return CA_OK;
}

int or_fork(or_state* s) {                        /* Fork (delta.go:428-431) */
    s->depth++;
    journal(s, J_FORK, -1, -1, -1, NULL);
    return CA_OK;
}

int or_revert(or_state* s) {                      /* Revert (delta.go:434-443) */
    if (s->depth == 0) return CA_ESTATE;
    while (s->journal.n > 0) {
        or_jent e = s->journal.a[--s->journal.n];
        if (e.kind == J_FORK) break;
        if (e.kind == J_ADD_NODE) {
            free(s->nodes.a[e.node].pods.a);
            s->nodes.n--;
        } else if (e.kind == J_ADD_POD) {
            or_node* nd = &s->nodes.a[e.node];
            node_apply(nd, &s->pods.a[e.pod].spec, -1);
            scope_count(s, &s->pods.a[e.pod].spec, -1);
            memcpy(nd->ports, e.ports, sizeof nd->ports);
            nd->pods.n--;
            s->pods.a[e.pod].node = -1;
        } else if (e.kind == J_REMOVE_POD) {
            or_node* nd = &s->nodes.a[e.node];
            node_apply(nd, &s->pods.a[e.pod].spec, +1);
            scope_count(s, &s->pods.a[e.pod].spec, +1);
            memcpy(nd->ports, e.ports, sizeof nd->ports);
            VEC_PUSH(nd->pods, nd->pods.a[e.slot]);
            nd->pods.a[e.slot] = e.pod;
            s->pods.a[e.pod].node = e.node;
        } else if (e.kind == J_REMOVE_NODE) {
            const int32_t pos = e.node;
            or_node row = s->removed.a[--s->removed.n];
            for (int64_t i = 0; i < s->pods.n; i++) if (s->pods.a[i].node >= pos) s->pods.a[i].node++;
            VEC_PUSH(s->nodes, row);                      /* grow by one, then shift into place */
            memmove(&s->nodes.a[pos + 1], &s->nodes.a[pos], (size_t)(s->nodes.n - 1 - pos) * sizeof(or_node));
            s->nodes.a[pos] = row;
            for (int64_t i = 0; i < row.pods.n; i++) {
                s->pods.a[row.pods.a[i]].node = pos;
                scope_count(s, &s->pods.a[row.pods.a[i]].spec, +1);
            }
        }
    }
    s->depth--;
    return CA_OK;
}

int or_commit(or_state* s) {                      /* Commit (delta.go:446-462) */
    if (s->depth == 0) return CA_ESTATE;
    /* drop the fork marker: the entries now belong to the enclosing fork (or
     * become permanent at depth 0). */
    int64_t i = s->journal.n - 1;
    while (i >= 0 && s->journal.a[i].kind != J_FORK) i--;
    if (i < 0) return CA_ESTATE;
    s->depth--;
    if (s->depth == 0) {
        s->journal.n = 0;
        free_removed(s);                          /* committed removals are permanent */
    } else {
        memmove(&s->journal.a[i], &s->journal.a[i + 1], (size_t)(s->journal.n - i - 1) * sizeof(or_jent));
        s->journal.n--;
    }
    return CA_OK;
}

int or_node_pods(const or_state* s, int32_t node, int32_t* out, int32_t cap) {
    if (node < 0 || node >= s->nodes.n) return -1;
    const or_node* nd = &s->nodes.a[node];
    for (int64_t i = 0; i < nd->pods.n && i < cap; i++) out[i] = nd->pods.a[i];
    return (int)nd->pods.n;
}

int or_pod_node(const or_state* s, int32_t pod_id) {
    if (pod_id < 0 || pod_id >= s->pods.n) return -1;
    return s->pods.a[pod_id].node;
}

int or_node_state(const or_state* s, int32_t node, int64_t* out4) {
    if (node < 0 || node >= s->nodes.n) return CA_ENOTFOUND;
    const or_node* nd = &s->nodes.a[node];
    out4[0] = wrap_sub(nd->spec.alloc_milli_cpu, nd->req_cpu);
    out4[1] = wrap_sub(nd->spec.alloc_memory, nd->req_mem);
    out4[2] = wrap_sub(nd->spec.alloc_ephemeral, nd->req_eph);
    out4[3] = nd->spec.alloc_pods - nd->npods;
    return CA_OK;
}

/* ------------------------------------------------------------------------- */
/* the filter chain                                                           */
/* ------------------------------------------------------------------------- */
typedef struct pod_ctx {
    const ca_pod_spec* p;
    const ca_selector_term* terms;
    const ca_selector_req* reqs;
    const int32_t* pf_names;
} pod_ctx;

static int any_bits(const uint64_t* a, const uint64_t* b, int w) {
    for (int i = 0; i < w; i++) if (a[i] & b[i]) return 1;
    return 0;
}

/* labels.Requirement.Matches (labels/selector.go:223-267) on interned form, and
 * the matchFields selector (nodeaffinity.go:207-217, 263-293). */
static int req_matches(const ca_selector_req* r, const ca_node_spec* n) {
    switch (r->op) {
    case CA_OP_IN: return any_bits(n->label_pairs, r->pairs, CA_LABEL_WORDS);
    case CA_OP_NOTIN: return !any_bits(n->label_pairs, r->pairs, CA_LABEL_WORDS);
    case CA_OP_EXISTS: return (int)((n->label_keys >> r->key) & 1u);
    case CA_OP_DOESNOTEXIST: return !(int)((n->label_keys >> r->key) & 1u);
    case CA_OP_GT:
        if (!((n->int_label_valid >> r->key) & 1u)) return 0;
        return n->int_label[r->key] > r->bound;
    case CA_OP_LT:
        if (!((n->int_label_valid >> r->key) & 1u)) return 0;
        return n->int_label[r->key] < r->bound;
    case CA_OP_FIELD_EQ: return n->name_id == r->key;
    case CA_OP_FIELD_NE: return n->name_id != r->key;
    default: return 0;
    }
}

/* RequiredNodeAffinity.Match (nodeaffinity.go:310-324): nodeSelector AND, then the
 * required terms ORed (LazyErrorNodeSelector.Match, nodeaffinity.go:104-123). */
static int affinity_matches(const pod_ctx* c, const ca_node_spec* n) {
    const ca_pod_spec* p = c->p;
    for (int w = 0; w < CA_LABEL_WORDS; w++)
        if ((n->label_pairs[w] & p->node_selector[w]) != p->node_selector[w]) return 0;
    if (p->aff_term_count < 0) return 1;
    for (int32_t k = 0; k < p->aff_term_count; k++) {
        const ca_selector_term* tm = &c->terms[p->aff_term_first + k];
        int ok = 1;
        for (int32_t r = 0; r < tm->count && ok; r++) ok = req_matches(&c->reqs[tm->first + r], n);
        if (ok) return 1;
    }
    return 0;
}

/* frameworkImpl.RunFilterPlugins (SF/runtime/framework.go:727-749) with the default
 * profile order (default_plugins.go:33-53); first failure wins.  Out-of-kernel filters
 * (volumes, topology spread, inter-pod affinity) are no-ops for the pods admitted here
 * (SURVEY §8a A12). */
static int run_filters(const or_node* nd, const pod_ctx* c, ca_pred_result* r) {
    const ca_pod_spec* p = c->p;
    const ca_node_spec* n = &nd->spec;
    if (r) memset(r, 0, sizeof *r);
    /* NodeUnschedulable (nodeunschedulable/node_unschedulable.go:61-75) */
    if ((n->flags & CA_NODE_UNSCHEDULABLE) && !(p->flags & CA_POD_TOLERATES_UNSCHED)) {
        if (r) { r->type = CA_PRED_NOT_SCHEDULABLE; r->plugin = CA_PLUGIN_NODE_UNSCHEDULABLE; }
        return 0;
    }
    /* NodeName (nodename/node_name.go:56-69) */
    if (p->node_name_id != -1 && p->node_name_id != n->name_id) {
        if (r) { r->type = CA_PRED_NOT_SCHEDULABLE; r->plugin = CA_PLUGIN_NODE_NAME; }
        return 0;
    }
    /* TaintToleration (tainttoleration/taint_toleration.go:64-77) */
    uint64_t untol = n->taints & ~p->tolerated_taints;
    if (untol) {
        if (r) {
            r->type = CA_PRED_NOT_SCHEDULABLE; r->plugin = CA_PLUGIN_TAINT_TOLERATION;
            r->taint = __builtin_ctzll(untol);
        }
        return 0;
    }
    /* NodeAffinity (nodeaffinity/node_affinity.go:150-170); skipped when PreFilter Skips */
    if ((p->flags & CA_POD_AFFINITY_FILTER) && !affinity_matches(c, n)) {
        if (r) { r->type = CA_PRED_NOT_SCHEDULABLE; r->plugin = CA_PLUGIN_NODE_AFFINITY; }
        return 0;
    }
    /* NodePorts (nodeports/node_ports.go:117-141) */
    if (any_bits(nd->ports, p->port_conflict, CA_PORT_WORDS)) {
        if (r) { r->type = CA_PRED_NOT_SCHEDULABLE; r->plugin = CA_PLUGIN_NODE_PORTS; }
        return 0;
    }
    /* NodeResourcesFit fitsRequest (noderesources/fit.go:253-331) */
    uint32_t reasons = 0;
    if (nd->npods + 1 > n->alloc_pods) reasons |= CA_REASON_TOO_MANY_PODS;
    int all_zero = p->req_milli_cpu == 0 && p->req_memory == 0 && p->req_ephemeral == 0 &&
                   !(p->flags & CA_POD_HAS_SCALAR_KEYS);
    if (!all_zero) {
        if (p->req_milli_cpu > wrap_sub(n->alloc_milli_cpu, nd->req_cpu)) reasons |= CA_REASON_INSUFF_CPU;
        if (p->req_memory > wrap_sub(n->alloc_memory, nd->req_mem)) reasons |= CA_REASON_INSUFF_MEMORY;
        if (p->req_ephemeral > wrap_sub(n->alloc_ephemeral, nd->req_eph)) reasons |= CA_REASON_INSUFF_EPHEMERAL;
        for (int i = 0; i < CA_MAX_SCALAR; i++) {
            if (p->req_scalar[i] == 0) continue;          /* fit.go:303-306 */
            if (p->req_scalar[i] > wrap_sub(n->alloc_scalar[i], nd->req_scalar[i]))
                reasons |= CA_REASON_INSUFF_SCALAR0 << i;
        }
    }
    if (reasons) {
        if (r) { r->type = CA_PRED_NOT_SCHEDULABLE; r->plugin = CA_PLUGIN_NODE_RESOURCES_FIT; r->reasons = reasons; }
        return 0;
    }
    return 1;
}

static int name_in_prefilter(const pod_ctx* c, int32_t name) {
    for (int32_t k = 0; k < c->p->prefilter_count; k++)
        if (c->pf_names[c->p->prefilter_first + k] == name) return 1;
    return 0;
}

static int match_pos(const ca_match_spec* m, int32_t pos) {
    if (!m) return 1;
    if (pos == m->exclude) return 0;
    switch (m->kind) {
    case CA_MATCH_ALL: return 1;
    case CA_MATCH_RANGE: return pos >= m->lo && pos < m->hi;
    case CA_MATCH_MASK: return m->mask[pos] != 0;
    default: return 0;
    }
}

/* SchedulerBasedPredicateChecker.FitsAnyNodeMatching (schedulerbased.go:90-136) */
static int32_t fits_any(or_state* s, const pod_ctx* c, const ca_match_spec* m, int32_t* last_index,
                        int32_t* prefilter_failed, uint64_t* evals) {
    if (prefilter_failed) *prefilter_failed = 0;
    if (c->p->flags & CA_POD_PREFILTER_FAIL) {          /* :109-112 */
        if (prefilter_failed) *prefilter_failed = 1;
        return -1;
    }
    const int64_t len = s->nodes.n;                      /* :95 List() */
    const int64_t L = *last_index;
    const int use_names = (c->p->flags & CA_POD_PREFILTER_NAMES) != 0;
    for (int64_t i = 0; i < len; i++) {                  /* :114-134 */
        const int32_t pos = (int32_t)((L + i) % len);
        if (!match_pos(m, pos)) continue;                /* :116 nodeMatches */
        const or_node* nd = &s->nodes.a[pos];
        if (use_names && !name_in_prefilter(c, nd->spec.name_id)) continue;  /* :120 */
        if (nd->spec.flags & CA_NODE_UNSCHEDULABLE) continue;               /* :125 */
        if (evals) (*evals)++;
        if (run_filters(nd, c, NULL)) {                                      /* :129 */
            *last_index = (int32_t)((L + i + 1) % len);                       /* :131 */
            return pos;
        }
    }
    return -1;
}

/* CheckPredicates (schedulerbased.go:139-185) */
static void check_pred(or_state* s, const pod_ctx* c, int32_t node, ca_pred_result* r,
                       uint64_t* evals) {
    memset(r, 0, sizeof *r);
    if (node < 0 || node >= s->nodes.n) { r->type = CA_PRED_INTERNAL; return; }   /* :143-147 */
    if (c->p->flags & CA_POD_PREFILTER_FAIL) { r->type = CA_PRED_INTERNAL; r->plugin = CA_PLUGIN_NODE_AFFINITY; return; }  /* :153-161 */
    if (evals) (*evals)++;
    run_filters(&s->nodes.a[node], c, r);
}

static pod_ctx table_ctx(const ca_pod_table* t, int32_t pod) {
    pod_ctx c;
    c.p = &t->pods[pod];
    c.terms = t->terms;
    c.reqs = t->reqs;
    c.pf_names = t->prefilter_names;
    return c;
}

int or_fits_any_node(or_state* s, const ca_pod_table* t, int32_t pod, const ca_match_spec* match,
                     int32_t* last_index, int32_t* out_node, int32_t* out_prefilter_failed,
                     uint64_t* evals) {
    if (pod < 0 || pod >= t->n_pods) return CA_EINVAL;
    if ((t->pods[pod].flags & CA_POD_OUT_OF_SCOPE) || s->scope_blockers > 0) return CA_EUNSUPPORTED;
    pod_ctx c = table_ctx(t, pod);
    *out_node = fits_any(s, &c, match, last_index, out_prefilter_failed, evals);
    return CA_OK;
}

int or_check_predicates(or_state* s, const ca_pod_table* t, int32_t pod, int32_t node,
                        ca_pred_result* out) {
    if (pod < 0 || pod >= t->n_pods) return CA_EINVAL;
    if ((t->pods[pod].flags & CA_POD_OUT_OF_SCOPE) || s->scope_blockers > 0) return CA_EUNSUPPORTED;
    pod_ctx c = table_ctx(t, pod);
    check_pred(s, &c, node, out, NULL);
    return CA_OK;
}

/* ------------------------------------------------------------------------- */
/* BinpackingNodeEstimator.Estimate (binpacking_estimator.go:65-159)           */
/* ------------------------------------------------------------------------- */
typedef struct scored { double score; int32_t pos; } scored;

/* stable merge sort, descending score: sort.Slice(podInfos, score_i > score_j)
 * (binpacking_estimator.go:74) with ties in input order. */
static void merge_sort_desc(scored* a, scored* tmp, int64_t n) {
    if (n < 2) return;
    int64_t h = n / 2;
    merge_sort_desc(a, tmp, h);
    merge_sort_desc(a + h, tmp, n - h);
    int64_t i = 0, j = h, k = 0;
    while (i < h && j < n) {
        if (a[j].score > a[i].score) tmp[k++] = a[j++];
        else tmp[k++] = a[i++];
    }
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, (size_t)n * sizeof(scored));
}

/* calculatePodScore (binpacking_estimator.go:164-193) */
static double pod_score(const ca_pod_spec* p, const ca_node_spec* tmpl) {
    double score = 0.0;
    if (tmpl->alloc_milli_cpu > 0)
        score += (double)p->score_milli_cpu / (double)tmpl->alloc_milli_cpu;
    if (tmpl->alloc_memory > 0)
        score += (double)p->score_memory / (double)tmpl->alloc_memory;
    return score;
}

/* addNewNodeToSnapshot + DeepCopyTemplateNode (binpacking_estimator.go:146-159,
 * utils/scheduler/scheduler.go:73-91): a copy of the template with a fresh name and
 * the template's pods (their aggregate requests and ports). */
static int32_t add_template_copy(or_state* s, const ca_template* tp) {
    ca_node_spec spec = tp->node;
    spec.name_id = s->next_new_name--;
    add_node_row(s, &spec);
    int32_t pos = (int32_t)s->nodes.n - 1;
    journal(s, J_ADD_NODE, pos, -1, -1, NULL);
    or_node* nd = &s->nodes.a[pos];
    nd->req_cpu = tp->used_milli_cpu;
    nd->req_mem = tp->used_memory;
    nd->req_eph = tp->used_ephemeral;
    for (int i = 0; i < CA_MAX_SCALAR; i++) nd->req_scalar[i] = tp->used_scalar[i];
    nd->npods = tp->used_pods;
    memcpy(nd->ports, tp->used_ports, sizeof nd->ports);
    return pos;
}

/* ComputeExpansionOption's feasibility check (CA/core/scaleup/orchestrator/
 * orchestrator.go:455-481), per node group: Fork, AddNodeWithPods(template node,
 * template pods), CheckPredicates(samplePod, node) for every equivalence group, Revert. */
int or_check_templates(or_state* s, const ca_pod_table* t, const int32_t* samples, int32_t n_samples,
                       const ca_template* templates, int32_t n_templates, ca_pred_result* out) {
    for (int32_t e = 0; e < n_samples; e++)
        if (samples[e] < 0 || samples[e] >= t->n_pods) return CA_EINVAL;
    if (s->scope_blockers > 0) return CA_EUNSUPPORTED;
    for (int32_t g = 0; g < n_templates; g++) {
        or_fork(s);                                                           /* :454 */
        const int32_t node = add_template_copy(s, &templates[g]);             /* :457-466 */
        for (int32_t e = 0; e < n_samples; e++) {                             /* :468-480 */
            pod_ctx c = table_ctx(t, samples[e]);
            ca_pred_result* r = &out[(size_t)g * n_samples + e];
            if ((c.p->flags & CA_POD_OUT_OF_SCOPE) || (templates[g].node.flags & CA_NODE_ANTI_AFFINITY_PODS)) {
                memset(r, 0, sizeof *r);
                r->type = CA_PRED_UNSUPPORTED;                                /* casim.h scope */
                continue;
            }
            check_pred(s, &c, node, r, NULL);
        }
        or_revert(s);                                                         /* :482 */
    }
    return CA_OK;
}

static int estimate_one(or_state* s, const ca_pod_table* t, const int32_t* pods, int32_t P,
                        const ca_template* tp, const ca_limiter* lim, int32_t* last_index,
                        ca_estimate_result* res, int32_t* sched_pod, int32_t* sched_node) {
    memset(res, 0, sizeof *res);
    res->last_index_in = *last_index;
    for (int32_t i = 0; i <= P; i++) {
        if (i == P ? (tp->node.flags & CA_NODE_ANTI_AFFINITY_PODS) != 0
                   : (t->pods[pods[i]].flags & (CA_POD_HOSTNAME_DEPENDENT | CA_POD_OUT_OF_SCOPE)) != 0) {
            res->status = CA_EUNSUPPORTED;
            res->last_index_out = *last_index;
            return CA_OK;
        }
    }
    /* limiter.StartEstimation (threshold_based_limiter.go:34-37) */
    int32_t granted = 0;
    scored* order = malloc(sizeof(scored) * (size_t)(P > 0 ? P : 1));
    scored* tmp = malloc(sizeof(scored) * (size_t)(P > 0 ? P : 1));
    for (int32_t i = 0; i < P; i++) {
        order[i].score = pod_score(&t->pods[pods[i]], &tp->node);
        order[i].pos = i;
    }
    if (s->sort_mode == OR_SORT_GO_PDQ) {                 /* sort.Slice (pdqsort_func) */
        double* key = malloc(sizeof(double) * (size_t)(P > 0 ? P : 1));
        int32_t* perm = malloc(sizeof(int32_t) * (size_t)(P > 0 ? P : 1));
        for (int32_t i = 0; i < P; i++) key[i] = order[i].score;
        go_sort_slice_desc(key, P, perm);
        for (int32_t i = 0; i < P; i++) { order[i].score = key[perm[i]]; order[i].pos = perm[i]; }
        free(key);
        free(perm);
    } else {
        merge_sort_desc(order, tmp, P);
    }
    free(tmp);

    or_fork(s);                                          /* :79 */
    const int32_t base = (int32_t)s->nodes.n;
    int32_t k = 0;                                       /* new nodes so far */
    uint8_t* has_pods = calloc((size_t)(P + 1), 1);       /* newNodesWithPods */
    int32_t last_node = -1;                              /* lastNodeName */
    int32_t nsched = 0;

    for (int32_t oi = 0; oi < P; oi++) {                 /* :88 */
        const int32_t pidx = pods[order[oi].pos];
        pod_ctx c = table_ctx(t, pidx);
        ca_match_spec m;
        memset(&m, 0, sizeof m);
        m.kind = CA_MATCH_RANGE; m.lo = base; m.hi = base + k; m.exclude = -1;
        int32_t node = fits_any(s, &c, &m, last_index, NULL, &res->evals);   /* :91-93 */
        if (node >= 0) {                                                      /* :94-102 */
            int32_t id = store_pod(s, t, pidx, node);
            add_pod_to_node(s, id, node);
            sched_pod[nsched] = pidx;
            if (sched_node) sched_node[nsched] = node - base;
            nsched++;
            has_pods[node - base] = 1;
            continue;
        }
        /* PermissionToAddNode consumes budget before the empty-node skip (:107-116) */
        if (lim->max_nodes > 0 && granted >= lim->max_nodes) break;
        granted++;
        if (last_node >= 0 && !has_pods[last_node - base]) continue;          /* :114 */
        int32_t nn = add_template_copy(s, tp);                               /* :119 */
        k++;
        last_node = nn;
        ca_pred_result pr;
        check_pred(s, &c, nn, &pr, &res->evals);                             /* :132 */
        if (pr.type != CA_PRED_OK) continue;
        int32_t id = store_pod(s, t, pidx, nn);
        add_pod_to_node(s, id, nn);                                          /* :135 */
        has_pods[nn - base] = 1;
        sched_pod[nsched] = pidx;
        if (sched_node) sched_node[nsched] = nn - base;
        nsched++;
    }
    int32_t count = 0;
    for (int32_t i = 0; i < k; i++) count += has_pods[i];
    or_revert(s);                                        /* :80-82 */
    /* pods stored during the estimate are dropped with the fork */
    free(has_pods);
    free(order);
    res->node_count = count;
    res->n_scheduled = nsched;
    res->nodes_added = k;
    res->last_index_out = *last_index;
    res->status = CA_OK;
    return CA_OK;
}

int or_estimate(or_state* s, const ca_pod_table* t, const int32_t* group_off,
                const int32_t* pod_idx, const ca_template* templates, int32_t n_groups,
                const ca_limiter* limiter, int32_t* last_index, ca_estimate_result* results,
                int32_t* sched_pod, int32_t* sched_node) {
    if (s->scope_blockers > 0 && n_groups > 0) return CA_EUNSUPPORTED;
    for (int32_t g = 0; g < n_groups; g++) {
        const int32_t off = group_off[g];
        const int64_t pods_before = s->pods.n, terms_before = s->terms.n, reqs_before = s->reqs.n,
                      pf_before = s->pf_names.n;
        int rc = estimate_one(s, t, pod_idx + off, group_off[g + 1] - off, &templates[g], limiter,
                              last_index, &results[g], sched_pod + off,
                              sched_node ? sched_node + off : NULL);
        s->pods.n = pods_before; s->terms.n = terms_before; s->reqs.n = reqs_before;
        s->pf_names.n = pf_before;
        if (rc != CA_OK) return rc;
        if (results[g].status == CA_EUNSUPPORTED) {       /* prefix protocol (casim.h scope) */
            for (int32_t h = g + 1; h < n_groups; h++) {
                memset(&results[h], 0, sizeof results[h]);
                results[h].last_index_in = results[h].last_index_out = *last_index;
                results[h].status = CA_ENOTRUN;
            }
            break;
        }
    }
    return CA_OK;
}

/* ------------------------------------------------------------------------- */
/* HintingSimulator.TrySchedulePods (hinting_simulator.go:58-125)              */
/* ------------------------------------------------------------------------- */
typedef struct similar_ent { int32_t cls; } similar_ent;

/* moved-pod copy: Spec.NodeName cleared (cluster.go:235-240) and TPU requests
 * cleared (tpu.go:57-79, applied at cluster.go:225). */
static ca_pod_spec moved_copy(const ca_pod_spec* p) {
    ca_pod_spec q = *p;
    q.node_name_id = -1;
    for (int i = 0; i < CA_MAX_SCALAR; i++)
        if ((p->tpu_scalar_mask >> i) & 1u) q.req_scalar[i] = 0;
    if (!(p->flags & CA_POD_HAS_NONTPU_SCALAR_KEYS)) q.flags &= ~CA_POD_HAS_SCALAR_KEYS;
    return q;
}

int or_try_schedule_pods(or_state* s, const int32_t* pod_ids, int32_t n,
                         const ca_match_spec* match, int32_t break_on_failure,
                         int32_t* hints, int32_t* last_index, int32_t* dest, uint64_t* evals) {
    /* SimilarPodsScheduling (similar_pods.go:43-111): unschedulable equivalence
     * classes seen in this call.  The class id is computed by the host from the
     * controller UID + labels + spec equality; <= 10 distinct entries per owner is
     * enforced by the host when it assigns class ids. */
    VEC(int32_t) unsched_cls = {0};
    int32_t placed = 0;
    for (int32_t i = 0; i < n; i++) dest[i] = -1;
    for (int32_t i = 0; i < n; i++) {
        const int32_t id = pod_ids[i];
        or_pod* op = &s->pods.a[id];
        ca_pod_spec q = moved_copy(&op->spec);
        pod_ctx c;
        c.p = &q; c.terms = s->terms.a; c.reqs = s->reqs.a; c.pf_names = s->pf_names.a;
        int32_t node = -1;
        /* findNodeWithHints (:91-108) */
        if (hints && hints[id] >= 0) {
            int32_t h = hints[id];
            ca_pred_result pr;
            check_pred(s, &c, h, &pr, evals);
            if (pr.type == CA_PRED_OK) {
                hints[id] = h;                                   /* :95 */
                if (match_pos(match, h)) node = h;               /* :102 */
            }
        }
        if (node < 0) {
            /* findNode (:110-125) */
            int similar = 0;
            if (q.similar_class >= 0)
                for (int64_t k = 0; k < unsched_cls.n; k++)
                    if (unsched_cls.a[k] == q.similar_class) { similar = 1; break; }
            if (!similar) {
                int32_t pf;
                node = fits_any(s, &c, match, last_index, &pf, evals);
                if (node < 0) {
                    if (q.similar_class >= 0 && !(q.flags & CA_POD_DAEMONSET))
                        VEC_PUSH(unsched_cls, q.similar_class);   /* SetUnschedulable */
                } else if (hints) {
                    hints[id] = node;                               /* :123 */
                }
            }
        }
        if (node >= 0) {                                            /* :77-82 */
            /* AddPod of the moved copy: a fresh pod record on the destination */
            or_pod np;
            np.spec = q;
            np.node = -1;
            VEC_PUSH(s->pods, np);
            int32_t nid = (int32_t)s->pods.n - 1;
            add_pod_to_node(s, nid, node);
            dest[i] = node;
            placed++;
        } else if (break_on_failure) {
            break;
        }
    }
    free(unsched_cls.a);
    return placed;
}

/* ------------------------------------------------------------------------- */
/* FilterOutSchedulable (filter_out_schedulable.go:95-124)                     */
/* ------------------------------------------------------------------------- */
#define OR_MAX_PODS_PER_OWNER 10                  /* similar_pods.go:53 */

int or_filter_out_schedulable(or_state* s, const ca_pod_table* t, const int32_t* order, int32_t n,
                              const int32_t* class_owner, int32_t n_classes, int32_t* hints,
                              int32_t* last_index, int32_t* out_node, int32_t* out_pod_id,
                              int32_t* n_overflowing, uint64_t* evals, int32_t* n_placed) {
    if (n < 0 || n_classes < 0) return CA_EINVAL;
    int32_t n_owners = 0;
    for (int32_t k = 0; k < n; k++) {
        const int32_t i = order ? order[k] : k;
        if (i < 0 || i >= t->n_pods) return CA_EINVAL;
        if (t->pods[i].similar_class >= n_classes) return CA_EINVAL;
    }
    if (s->scope_blockers > 0) return CA_EUNSUPPORTED;            /* casim.h scope: nothing runs */
    for (int32_t k = 0; k < n; k++)
        if (t->pods[order ? order[k] : k].flags & CA_POD_OUT_OF_SCOPE) return CA_EUNSUPPORTED;
    if (class_owner)
        for (int32_t c = 0; c < n_classes; c++) if (class_owner[c] + 1 > n_owners) n_owners = class_owner[c] + 1;
    uint8_t* marked = calloc((size_t)n_classes + 1, 1);       /* items[uid] holds this class */
    int32_t* owner_cnt = calloc((size_t)n_owners + 1, sizeof(int32_t));   /* len(items[uid]) */
    uint8_t* owner_over = calloc((size_t)n_owners + 1, 1);    /* overflowingControllers */
    ca_match_spec all;
    memset(&all, 0, sizeof all);
    all.kind = CA_MATCH_ALL; all.exclude = -1;                  /* ScheduleAnywhere */
    int32_t placed = 0;
    for (int32_t k = 0; k < n; k++) {                           /* hinting_simulator.go:63-86 */
        const int32_t i = order ? order[k] : k;
        pod_ctx c = table_ctx(t, i);
        int32_t node = -1;
        if (hints && hints[k] >= 0) {                           /* findNodeWithHints :91-108 */
            ca_pred_result pr;
            check_pred(s, &c, hints[k], &pr, evals);
            if (pr.type == CA_PRED_OK) node = hints[k];         /* :95 Set, :102 accepted */
        }
        if (node < 0) {                                         /* findNode :110-125 */
            const int32_t cls = c.p->similar_class;
            if (!(cls >= 0 && marked[cls])) {                   /* IsSimilarUnschedulable */
                node = fits_any(s, &c, &all, last_index, NULL, evals);
                if (node < 0) {
                    if (cls >= 0 && !(c.p->flags & CA_POD_DAEMONSET)) {   /* SetUnschedulable */
                        const int32_t o = class_owner ? class_owner[cls] : -1;
                        if (o < 0) {
                            marked[cls] = 1;
                        } else if (owner_cnt[o] >= OR_MAX_PODS_PER_OWNER) {
                            owner_over[o] = 1;
                        } else {
                            marked[cls] = 1;
                            owner_cnt[o]++;
                        }
                    }
                }
            }
        }
        if (node >= 0) {                                        /* :77-82 AddPod, no fork */
            if (hints) hints[k] = node;
            const int32_t id = store_pod(s, t, i, node);
            add_pod_to_node(s, id, node);
            out_node[k] = node;
            if (out_pod_id) out_pod_id[k] = id;
            placed++;
        } else {
            out_node[k] = -1;
            if (out_pod_id) out_pod_id[k] = -1;
        }
    }
    if (n_overflowing) {
        int32_t ov = 0;
        for (int32_t o = 0; o < n_owners; o++) ov += owner_over[o];
        *n_overflowing = ov;
    }
    free(marked); free(owner_cnt); free(owner_over);
    if (n_placed) *n_placed = placed;
    return CA_OK;
}

/* ------------------------------------------------------------------------- */
/* RemovalSimulator.FindNodesToRemove, legacy canPersist=false (cluster.go:116-254) */
/* ------------------------------------------------------------------------- */
int or_find_nodes_to_remove(or_state* s, const int32_t* candidates, int32_t n_candidates,
                            const uint8_t* dest_mask, const int32_t* cand_status,
                            const int32_t* move_off, const int32_t* move_pods,
                            int32_t* hints, int32_t* last_index,
                            ca_removal_result* results, int32_t* out_dest) {
    if (s->scope_blockers > 0 && n_candidates > 0) return CA_EUNSUPPORTED;
    int32_t cut = 0;
    for (int32_t ci = 0; ci < n_candidates; ci++) {
        ca_removal_result* r = &results[ci];
        memset(r, 0, sizeof *r);
        r->last_index_in = *last_index;
        const int32_t node = candidates[ci];
        const int32_t mo = move_off[ci], mn = move_off[ci + 1] - move_off[ci];
        for (int32_t i = 0; i < mn; i++) out_dest[mo + i] = -1;
        if (cut) {                                                        /* prefix protocol */
            r->reason = CA_UNREMOVABLE_NOT_RUN;
            continue;
        }
        if (node >= 0 && node < s->nodes.n && dest_mask[node] && !(cand_status && cand_status[ci] != 0)) {
            if (mn > CA_MAX_MOVED_PODS) cut = 1;                          /* casim.h scope */
            for (int32_t i = 0; i < mn && !cut; i++)
                if (s->pods.a[move_pods[mo + i]].spec.flags & CA_POD_OUT_OF_SCOPE) cut = 1;
            if (cut) {
                r->reason = CA_UNREMOVABLE_OUT_OF_SCOPE;                  /* casim.h scope */
                continue;
            }
        }
        if (node < 0 || node >= s->nodes.n || !dest_mask[node]) {        /* :157-160 */
            r->reason = CA_UNREMOVABLE_UNEXPECTED_ERROR;
            continue;
        }
        if (cand_status && cand_status[ci] != 0) {                        /* :162-169 */
            r->reason = cand_status[ci];
            continue;
        }
        /* withForkedSnapshot(findPlaceFor) (:171-173, :204-218) */
        const int64_t pods_before = s->pods.n;
        or_fork(s);
        for (int32_t i = 0; i < mn; i++) or_remove_pod(s, move_pods[mo + i]);   /* :228-233 */
        ca_match_spec m;
        memset(&m, 0, sizeof m);
        m.kind = CA_MATCH_MASK; m.mask = dest_mask; m.exclude = node;          /* :221-223 */
        int32_t placed = or_try_schedule_pods(s, move_pods + mo, mn, &m, 1, hints, last_index,
                                              out_dest + mo, &r->evals);      /* :242 */
        or_revert(s);
        s->pods.n = pods_before;
        r->n_placed = placed;
        if (placed == mn) {                                                     /* :246-248 */
            r->removable = 1;
            r->reason = CA_UNREMOVABLE_NONE;
        } else {
            r->reason = CA_UNREMOVABLE_NO_PLACE;                                /* :174-177 */
        }
    }
    return CA_OK;
}

/* ------------------------------------------------------------------------- */
/* Planner.categorizeNodes with canPersist=true (planner.go:252-296)           */
/* ------------------------------------------------------------------------- */
static int pdb_member(const ca_pdb_table* t, const int32_t* origin, int32_t pod, int32_t pdb) {
    const int32_t o = origin[pod];
    for (int32_t k = t->pod_off[o]; k < t->pod_off[o + 1]; k++)
        if (t->pod_pdb[k] == pdb) return 1;
    return 0;
}

int or_plan_removals(or_state* s, const int32_t* candidates, int32_t n_candidates,
                     const uint8_t* dest_mask, const int32_t* cand_status,
                     const int32_t* move_off, const int32_t* move_pods,
                     int32_t max_removable, const ca_pdb_table* pdbs,
                     int32_t* hints, int32_t n_pods, int32_t* last_index,
                     ca_plan_result* results, ca_plan_move* moves, int32_t moves_cap, int32_t* n_moves) {
    if (n_candidates < 0 || n_pods < 0 || n_pods > s->pods.n) return CA_EINVAL;   /* past n_pods: detached */
    if (s->scope_blockers > 0 && n_candidates > 0) return CA_EUNSUPPORTED;
    const int32_t N = (int32_t)s->nodes.n;
    const int P = pdbs ? pdbs->n_pdbs : 0;
    uint8_t* mask = malloc((size_t)N + 1);                  /* podDestinations (planner.go:280) */
    memcpy(mask, dest_mask, (size_t)N);
    /* Hints by pod key: a copy shares its original's key (hints.go:31-37) */
    VEC(int32_t) H = {0};
    VEC(int32_t) origin = {0};                              /* pod id -> caller pod id (PDBs) */
    for (int32_t i = 0; i < (int32_t)s->pods.n; i++) {
        VEC_PUSH(H, hints && i < n_pods ? hints[i] : -1);
        VEC_PUSH(origin, i);
    }
    /* copies committed onto a node, in commit order (NodeInfo.Pods appends) */
    vec_i32* extra = calloc((size_t)N + 1, sizeof(vec_i32));
    vec_i32 list = {0};
    int32_t removed = 0, cut = 0, nm = 0;
    for (int32_t ci = 0; ci < n_candidates; ci++) {
        ca_plan_result* r = &results[ci];
        memset(r, 0, sizeof *r);
        r->last_index_in = *last_index;
        r->first_move = nm;
        r->blocking_pod = -1;
        if (cut || (max_removable > 0 && removed >= max_removable)) {          /* :268-271 */
            r->reason = CA_UNREMOVABLE_NOT_RUN;
            cut = 1;
            continue;
        }
        const int32_t node = candidates[ci];
        const int valid = node >= 0 && node < N && mask[node];
        list.n = 0;
        for (int32_t i = move_off[ci]; i < move_off[ci + 1]; i++) VEC_PUSH(list, move_pods[i]);
        if (node >= 0 && node < N)
            for (int64_t i = 0; i < extra[node].n; i++) VEC_PUSH(list, extra[node].a[i]);
        if (valid && !(cand_status && cand_status[ci] != 0)) {
            if (list.n > CA_MAX_MOVED_PODS) cut = 1;                      /* casim.h scope */
            for (int64_t i = 0; i < list.n && !cut; i++)
                if (s->pods.a[list.a[i]].spec.flags & CA_POD_OUT_OF_SCOPE) cut = 1;
            if (cut) { r->reason = CA_UNREMOVABLE_OUT_OF_SCOPE; continue; }   /* casim.h scope */
        }
        if (!valid) { r->reason = CA_UNREMOVABLE_UNEXPECTED_ERROR; continue; } /* cluster.go:157-160 */
        if (cand_status && cand_status[ci] != 0) { r->reason = cand_status[ci]; continue; }
        /* GetPodsToMove's checkPdbs against the remaining budgets (drain.go:73-90) */
        for (int p = 0; p < P && r->blocking_pod < 0; p++) {
            if (pdbs->allowed[p] >= 1) continue;
            for (int64_t i = 0; i < list.n; i++)
                if (pdb_member(pdbs, origin.a, list.a[i], p)) { r->blocking_pod = list.a[i]; break; }
        }
        if (r->blocking_pod >= 0) { r->reason = CA_UNREMOVABLE_BLOCKED_BY_POD; continue; }
        /* withForkedSnapshot(findPlaceFor) (cluster.go:171-173, :204-218) */
        const int64_t pods_before = s->pods.n;
        int32_t* dest = malloc(sizeof(int32_t) * (size_t)(list.n + 1));
        or_fork(s);
        for (int64_t i = 0; i < list.n; i++) or_remove_pod(s, list.a[i]);           /* :228-233 */
        ca_match_spec m;
        memset(&m, 0, sizeof m);
        m.kind = CA_MATCH_MASK; m.mask = mask; m.exclude = node;                    /* :221-223 */
        const int32_t placed = or_try_schedule_pods(s, list.a, (int32_t)list.n, &m, 1, H.a, last_index, dest,
                                                    &r->evals);
        r->n_placed = placed;
        if (placed == list.n) {
            or_commit(s);                                                            /* :207-211 */
            r->removable = 1;
            r->reason = CA_UNREMOVABLE_NONE;
            r->n_moves = placed;
            for (int32_t i = 0; i < placed; i++) {                /* copies pods_before + i, in order */
                const int32_t nid = (int32_t)(pods_before + i);
                VEC_PUSH(H, dest[i]);
                VEC_PUSH(origin, origin.a[list.a[i]]);
                VEC_PUSH(extra[dest[i]], nid);
                if (nm < moves_cap) {
                    moves[nm].candidate = ci; moves[nm].pod = list.a[i];
                    moves[nm].new_pod = nid; moves[nm].node = dest[i];
                }
                nm++;
            }
            mask[node] = 0;                                                          /* planner.go:280 */
            removed++;
            /* CanRemovePods (basic.go:66-84) then RemovePods (:86-95) */
            for (int p = 0; p < P; p++) {
                int32_t count = 0;
                for (int64_t i = 0; i < list.n; i++)
                    if (pdb_member(pdbs, origin.a, list.a[i], p) && pdbs->allowed[p] < ++count) r->risky = 1;
            }
            for (int p = 0; p < P; p++)
                for (int64_t i = 0; i < list.n; i++)
                    if (pdb_member(pdbs, origin.a, list.a[i], p)) pdbs->allowed[p]--;
        } else {
            or_revert(s);
            s->pods.n = pods_before;
            r->reason = CA_UNREMOVABLE_NO_PLACE;                                     /* :174-177 */
        }
        free(dest);
    }
    if (hints) memcpy(hints, H.a, sizeof(int32_t) * (size_t)n_pods);
    if (n_moves) *n_moves = nm;
    for (int32_t i = 0; i < N; i++) free(extra[i].a);
    free(extra); free(list.a); free(H.a); free(origin.a); free(mask);
    return CA_OK;
}

/* ---------------------------------------------------------------------------
 * Scale-down eligibility: utilization.Calculate + FindEmptyNodesToRemove
 * ------------------------------------------------------------------------- */

/* drain.IsPodLongTerminating (CA/utils/drain/drain.go:294-306):
 * DeletionTimestamp + grace seconds + PodLongTerminatingExtraThreshold (30 s, :34) is
 * strictly before currentTime. */
static int or_pod_long_terminating(const ca_util_pod* p, int64_t now_ns) {
    if (!(p->flags & CA_UPOD_DELETED)) return 0;
    int64_t t = p->deletion_ns + p->grace_s * 1000000000LL;
    t += 30LL * 1000000000LL;
    return t < now_ns;
}

/* calculateUtilizationOfResource (info.go:83-127) for resource r (0 cpu, 1 mem, 2 gpu).
 * Returns 0 and *util, or the error code (absent / zero allocatable). */
static int or_util_of_resource(const ca_util_node* nd, const ca_util_pod* pods, int32_t b, int32_t e,
                               int r, int32_t skip_ds, int32_t skip_mirror, int64_t now_ns, double* util) {
    static const uint32_t has_bit[3] = {CA_UNODE_HAS_CPU, CA_UNODE_HAS_MEM, CA_UNODE_HAS_GPU};
    if (!(nd->flags & has_bit[r])) return 1;                   /* :84-87 not found */
    if (nd->alloc_milli[r] == 0) return 2;                     /* :88-90 zero       */
    int64_t pods_request = 0, ds_and_mirror = 0;
    for (int32_t i = b; i < e; i++) {
        const ca_util_pod* p = &pods[i];
        if (skip_ds && (p->flags & CA_UPOD_DAEMONSET)) {       /* :100-108 */
            ds_and_mirror += p->req_milli[r];
            continue;
        }
        if (skip_mirror && (p->flags & CA_UPOD_MIRROR)) {      /* :109-117 */
            ds_and_mirror += p->req_milli[r];
            continue;
        }
        if (or_pod_long_terminating(p, now_ns)) continue;      /* :118-121 */
        pods_request += p->req_milli[r];                       /* :122-124 */
    }
    *util = (double)pods_request / (double)(nd->alloc_milli[r] - ds_and_mirror);   /* :126 */
    return 0;
}

int or_node_utilization(const ca_util_node* nodes, int32_t n_nodes, const int32_t* pod_off,
                        const ca_util_pod* pods, int32_t skip_ds, int32_t skip_mirror,
                        int64_t now_ns, ca_util_info* out) {
    if (n_nodes < 0 || (n_nodes > 0 && (!nodes || !pod_off || !out))) return CA_EINVAL;
    for (int32_t n = 0; n < n_nodes; n++) {
        const ca_util_node* nd = &nodes[n];
        const int32_t b = pod_off[n], e = pod_off[n + 1];
        ca_util_info o;
        memset(&o, 0, sizeof o);
        o.resource = CA_UTIL_CPU;
        /* cluster.go:197-199: GetPodsToMove with nil listers has no error and no pods */
        o.empty = 1;
        for (int32_t i = b; i < e; i++)
            if (pods[i].flags & (CA_UPOD_MOVABLE | CA_UPOD_BLOCKING)) o.empty = 0;
        if (nd->flags & CA_UNODE_GPU_CONFIG) {                 /* info.go:49-58 */
            double g = 0.0;
            o.resource = CA_UTIL_GPU;
            if (or_util_of_resource(nd, pods, b, e, 2, skip_ds, skip_mirror, now_ns, &g) == 0) {
                o.gpu = g;
                o.utilization = g;
            }
        } else {                                               /* info.go:61-80 */
            double cpu = 0.0, mem = 0.0;
            int err = or_util_of_resource(nd, pods, b, e, 0, skip_ds, skip_mirror, now_ns, &cpu);
            if (err) {
                o.status = err == 1 ? CA_UTIL_NO_CPU : CA_UTIL_ZERO_CPU;
            } else if ((err = or_util_of_resource(nd, pods, b, e, 1, skip_ds, skip_mirror, now_ns, &mem))) {
                o.status = err == 1 ? CA_UTIL_NO_MEM : CA_UTIL_ZERO_MEM;
            } else {
                o.cpu = cpu;
                o.mem = mem;
                if (cpu > mem) { o.resource = CA_UTIL_CPU; o.utilization = cpu; }
                else           { o.resource = CA_UTIL_MEM; o.utilization = mem; }
            }
        }
        out[n] = o;
    }
    return CA_OK;
}
