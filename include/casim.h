/*
 * casim.h — C ABI of the MI355X scheduling-simulation library (libcasim.so).
 *
 * This is the drop-in boundary for cluster-autoscaler's scheduling-simulation
 * hot path.  A Go shim (cgo) or any C caller binds these entry points; no torch
 * or C++ types appear in any signature.  Every struct is plain-old-data with
 * fixed-size members so cgo can pass Go-allocated arrays of them directly.
 *
 * Reference interfaces replaced (CA/ = cluster-autoscaler/ in the reference):
 *   ClusterSnapshot data plane   CA/simulator/clustersnapshot/clustersnapshot.go:29-55
 *                                (DeltaClusterSnapshot CA/simulator/clustersnapshot/delta.go:43-475)
 *       -> ca_mirror_* (create/add_nodes/add_pods/remove_pod/fork/revert/commit/clear)
 *   PredicateChecker.FitsAnyNode / FitsAnyNodeMatching
 *                                CA/simulator/predicatechecker/interface.go:27-31,
 *                                CA/simulator/predicatechecker/schedulerbased.go:83-136
 *       -> ca_fits_any_node (closure nodeMatches -> ca_match_spec; lastIndex explicit in/out)
 *   PredicateChecker.CheckPredicates  schedulerbased.go:139-185, error.go:24-107
 *       -> ca_check_predicates (PredicateError -> ca_pred_result)
 *   Estimator.Estimate           CA/estimator/estimator.go:40-42,
 *                                CA/estimator/binpacking_estimator.go:65-193
 *   EstimationLimiter            CA/estimator/estimator.go:63-74, threshold_based_limiter.go:27-64
 *       -> ca_estimate_batch (one call = Estimate for every node group of one ScaleUp,
 *          CA/core/scaleup/orchestrator/orchestrator.go:139-178, :487-488)
 *   RemovalSimulator.FindNodesToRemove  CA/simulator/cluster.go:116-139 (+ SimulateNodeRemoval
 *                                :145-184, findPlaceFor :220-254, HintingSimulator.TrySchedulePods
 *                                CA/simulator/scheduling/hinting_simulator.go:58-125)
 *       -> ca_find_nodes_to_remove (legacy canPersist=false semantics)
 *
 * Node order.  Every node index in this ABI is a POSITION in the mirror's node
 * list.  The list is the canonical order of SURVEY.md fact 2: nodes in
 * ca_mirror_add_nodes order; nodes added in a fork are appended.  The caller
 * passes nodes in the order its own ClusterSnapshot.NodeInfos().List() returned
 * (the rotating scan of FitsAnyNodeMatching walks that order).
 *
 * Threading.  One mirror per caller thread; calls on one handle are serialised
 * by the caller (the reference checker is not thread-safe either,
 * schedulerbased.go:43,105-106).  No pointer passed in is retained after a call
 * returns.
 */
#ifndef CASIM_H
#define CASIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CASIM_ABI_VERSION 3

/* ---- status codes (int return of every entry point) -------------------- */
#define CA_OK            0
#define CA_EINVAL        1  /* malformed argument                                    */
#define CA_ENOTFOUND     2  /* node/pod not in the mirror (clustersnapshot.go:58 ErrNodeNotFound) */
#define CA_EEXISTS       3  /* object already present                                */
#define CA_EDEVICE       4  /* HIP runtime failure                                   */
#define CA_ECAPACITY     5  /* a fixed-width intern table (labels/ports/...) overflowed */
#define CA_EUNSUPPORTED  6  /* input needs a plugin the kernels do not implement:
                               the caller routes it to the Go scheduler framework      */
#define CA_ESTATE        7  /* fork/revert/commit misuse                              */
#define CA_ENOTRUN       8  /* per-item status: not evaluated because an EARLIER item of the
                               same batch was CA_EUNSUPPORTED (prefix protocol below)   */

/* ---- fixed widths of interned bitsets (host interning) -- */
#define CA_MAX_SCALAR    8   /* extended / hugepage / attachable-volume resources   */
#define CA_LABEL_WORDS   4   /* 256 interned (key,value) label pairs                  */
#define CA_PORT_WORDS    2   /* 128 interned (hostIP,protocol,hostPort) triples        */
#define CA_MAX_INT_KEYS  4   /* label keys referenced by Gt/Lt requirements           */
/* taint classes: 64 (one u64); label keys for Exists/DoesNotExist: 64 (one u64) */
#define CA_MAX_MOVED_PODS 128 /* pods to move of one scale-down candidate (kernel scope below) */

/* ---- node flags ---------------------------------------------------------- */
#define CA_NODE_UNSCHEDULABLE   0x1u  /* node.Spec.Unschedulable                       */
#define CA_NODE_ANTI_AFFINITY_PODS 0x2u /* ca_template only: one of the template's pods has
                                          required pod anti-affinity (the group is out of scope,
                                          interpodaffinity/filtering.go:230-268)              */

/* ---- pod flags ----------------------------------------------------------- */
#define CA_POD_HAS_SCALAR_KEYS        0x001u /* len(podRequest.ScalarResources) != 0 (fit.go:267-272) */
#define CA_POD_HAS_NONTPU_SCALAR_KEYS 0x002u /* same after tpu.ClearTPURequests (tpu.go:57-79)        */
#define CA_POD_TOLERATES_UNSCHED      0x004u /* tolerates node.kubernetes.io/unschedulable:NoSchedule
                                                (node_unschedulable.go:61-75)                         */
#define CA_POD_AFFINITY_FILTER        0x008u /* NodeAffinity PreFilter did not Skip (node_affinity.go:91-99):
                                                pod has nodeSelector or required node affinity        */
#define CA_POD_PREFILTER_FAIL         0x010u /* NodeAffinity PreFilter UnschedulableAndUnresolvable
                                                (empty matchFields intersection, node_affinity.go:125-127) */
#define CA_POD_PREFILTER_NAMES        0x020u /* PreFilterResult.NodeNames set (node_affinity.go:129-133) */
#define CA_POD_DAEMONSET              0x040u /* owned by a DaemonSet (similar_pods.go:94)            */
#define CA_POD_HOSTNAME_DEPENDENT     0x080u /* selector/affinity/nodeName refer to node identity:
                                                not evaluable once per template in ca_estimate_batch  */
#define CA_POD_OUT_OF_SCOPE           0x100u /* the pod needs a filter plugin the kernels do not
                                                implement: required pod (anti-)affinity
                                                (interpodaffinity/filtering.go:230-268), a DoNotSchedule
                                                topology spread constraint (podtopologyspread/
                                                filtering.go:151-158,238-258), or a volume a volume
                                                plugin reads (volume_binding.go:169, volume_zone.go:97-103,
                                                volume_restrictions.go:166-176, nodevolumelimits)       */
#define CA_POD_REQUIRED_ANTI_AFFINITY 0x200u /* the pod has required pod anti-affinity terms: while
                                                it is in the snapshot no other pod's InterPodAffinity
                                                PreFilter Skips (filtering.go:260-262), so every
                                                simulation over the mirror is out of scope           */

/* ---- selector requirement ops (labels/selector.go:223-267, nodeaffinity.go:297-324) */
#define CA_OP_IN            1  /* node has key with value in set:  node.pairs & req.pairs != 0   */
#define CA_OP_NOTIN         2  /* !(node.pairs & req.pairs)                                       */
#define CA_OP_EXISTS        3  /* node.label_keys bit key                                          */
#define CA_OP_DOESNOTEXIST  4
#define CA_OP_GT            5  /* int label key `key` present, parses as int64, value >  bound     */
#define CA_OP_LT            6  /*                                                 value <  bound     */
#define CA_OP_FIELD_EQ      7  /* matchFields metadata.name In [v]   -> node.name_id == key         */
#define CA_OP_FIELD_NE      8  /* matchFields metadata.name NotIn [v] -> node.name_id != key        */
#define CA_OP_FALSE         9  /* term never matches (parse error, unsupported field key)          */

/* ---- plugins (default_plugins.go:33-53 filter order) ---------------------- */
#define CA_PLUGIN_NONE               0
#define CA_PLUGIN_NODE_UNSCHEDULABLE 1
#define CA_PLUGIN_NODE_NAME          2
#define CA_PLUGIN_TAINT_TOLERATION   3
#define CA_PLUGIN_NODE_AFFINITY      4
#define CA_PLUGIN_NODE_PORTS         5
#define CA_PLUGIN_NODE_RESOURCES_FIT 6

/* ---- predicate result types (error.go:27-32) ----------------------------- */
#define CA_PRED_OK              0
#define CA_PRED_NOT_SCHEDULABLE 1  /* NotSchedulablePredicateError */
#define CA_PRED_INTERNAL        2  /* InternalPredicateError       */
#define CA_PRED_UNSUPPORTED     3  /* not evaluated: the pod (or the template's pods) is out of
                                      kernel scope; run this pair on the Go path          */

/* reason bits of NodeResourcesFit (fit.go:256-329), in the reference's append order */
#define CA_REASON_TOO_MANY_PODS   0x1u
#define CA_REASON_INSUFF_CPU      0x2u
#define CA_REASON_INSUFF_MEMORY   0x4u
#define CA_REASON_INSUFF_EPHEMERAL 0x8u
#define CA_REASON_INSUFF_SCALAR0  0x100u /* bit (8+i): "Insufficient <scalar resource i>" */

/* ---- match spec: the data form of the nodeMatches closure ---------------- */
#define CA_MATCH_ALL   0  /* FitsAnyNode (schedulerbased.go:83-87)                                */
#define CA_MATCH_RANGE 1  /* positions [lo,hi): nodes added since a fork (binpacking_estimator.go:91-93) */
#define CA_MATCH_MASK  2  /* mask[pos] != 0 (destinations, cluster.go:221-223)                     */

/* UnremovableReason values (cluster.go:58-90) used by ca_find_nodes_to_remove */
#define CA_UNREMOVABLE_NONE              0
#define CA_UNREMOVABLE_NO_PLACE          12 /* NoPlaceToMovePods */
#define CA_UNREMOVABLE_BLOCKED_BY_POD    13 /* BlockedByPod      */
#define CA_UNREMOVABLE_UNEXPECTED_ERROR  14 /* UnexpectedError   */
/* Not reference reasons: the prefix protocol of ca_find_nodes_to_remove. */
#define CA_UNREMOVABLE_OUT_OF_SCOPE     100 /* a pod to move is CA_POD_OUT_OF_SCOPE: simulate this
                                               candidate on the Go path                    */
#define CA_UNREMOVABLE_NOT_RUN          101 /* after an out-of-scope candidate: not simulated */

/* ------------------------------------------------------------------------- */

/* One node (NodeInfo.node + NodeInfo.Allocatable, SF/types.go:381-441, :791-796). */
typedef struct ca_node_spec {
    int64_t  alloc_milli_cpu;                 /* Allocatable.MilliCPU                    */
    int64_t  alloc_memory;                    /* Allocatable.Memory                      */
    int64_t  alloc_ephemeral;                 /* Allocatable.EphemeralStorage            */
    int64_t  alloc_pods;                      /* Allocatable.AllowedPodNumber            */
    int64_t  alloc_scalar[CA_MAX_SCALAR];     /* Allocatable.ScalarResources[interned i] */
    uint64_t taints;                          /* NoSchedule/NoExecute taint classes      */
    uint64_t label_pairs[CA_LABEL_WORDS];     /* interned (key,value) pairs on the node  */
    uint64_t label_keys;                      /* interned keys present                   */
    int64_t  int_label[CA_MAX_INT_KEYS];      /* int64 value of Gt/Lt key i              */
    uint32_t int_label_valid;                 /* bit i: key i present and ParseInt ok    */
    uint32_t flags;                           /* CA_NODE_*                               */
    int32_t  name_id;                         /* unique interned node name               */
    int32_t  reserved;
} ca_node_spec;

/* One pod (requests per computePodResourceRequest fit.go:160-176 == calculateResource
 * SF/types.go:726-757; scoring sums per calculatePodScore binpacking_estimator.go:164-193). */
typedef struct ca_pod_spec {
    int64_t  req_milli_cpu;                   /* max(sum containers, init) + overhead   */
    int64_t  req_memory;
    int64_t  req_ephemeral;
    int64_t  req_scalar[CA_MAX_SCALAR];
    int64_t  score_milli_cpu;                 /* containers-only cpu sum, MilliValue()   */
    int64_t  score_memory;                    /* containers-only memory sum, Value()     */
    uint64_t tolerated_taints;                /* bit t: some toleration tolerates class t */
    uint64_t port_conflict[CA_PORT_WORDS];    /* triples that conflict with wanted ports
                                                 (HostPortInfo.CheckConflict SF/types.go:887-921) */
    uint64_t port_use[CA_PORT_WORDS];         /* triples the pod occupies once placed    */
    uint64_t node_selector[CA_LABEL_WORDS];   /* spec.nodeSelector pairs (AND)           */
    int32_t  aff_term_first;                  /* required node affinity terms (ORed)     */
    int32_t  aff_term_count;                  /* -1: none; 0: present but no terms       */
    int32_t  prefilter_first;                 /* PreFilter NodeNames (node name ids)     */
    int32_t  prefilter_count;
    int32_t  node_name_id;                    /* spec.nodeName; -1 empty                 */
    uint32_t flags;                           /* CA_POD_*                                */
    int32_t  similar_class;                   /* SimilarPodsScheduling key, -1 none      */
    uint32_t tpu_scalar_mask;                 /* scalar indices cleared by ClearTPURequests */
} ca_pod_spec;

typedef struct ca_selector_req {
    int32_t  op;                              /* CA_OP_*                                 */
    int32_t  key;                             /* key id / int key id / name id           */
    int64_t  bound;                           /* Gt/Lt integer                           */
    uint64_t pairs[CA_LABEL_WORDS];           /* In/NotIn value pairs of `key`           */
} ca_selector_req;

typedef struct ca_selector_term {
    int32_t first;                            /* into ca_pod_table.reqs                  */
    int32_t count;                            /* 0 is never emitted (empty terms dropped, nodeaffinity.go:83-85) */
} ca_selector_term;

/* A set of pods plus the side tables their records index into. */
typedef struct ca_pod_table {
    const ca_pod_spec*      pods;
    int32_t                 n_pods;
    int32_t                 n_terms;
    const ca_selector_term* terms;
    const ca_selector_req*  reqs;
    int32_t                 n_reqs;
    int32_t                 n_prefilter_names;
    const int32_t*          prefilter_names;
} ca_pod_table;

typedef struct ca_match_spec {
    int32_t        kind;                      /* CA_MATCH_*                              */
    int32_t        lo, hi;                    /* CA_MATCH_RANGE                          */
    int32_t        exclude;                   /* position never matched, -1 none         */
    const uint8_t* mask;                      /* CA_MATCH_MASK, length = node count      */
} ca_match_spec;

typedef struct ca_pred_result {
    int32_t  type;                            /* CA_PRED_*                               */
    int32_t  plugin;                          /* CA_PLUGIN_* that failed                 */
    uint32_t reasons;                         /* CA_REASON_* (NodeResourcesFit)          */
    int32_t  taint;                           /* lowest untolerated taint class          */
} ca_pred_result;

/* Node-group template for Estimate: NodeInfo template (orchestrator.go:444-491) and the
 * aggregate of its pods (DaemonSets), copied onto every new node (scheduler.go:73-91). */
typedef struct ca_template {
    ca_node_spec node;
    int64_t  used_milli_cpu;
    int64_t  used_memory;
    int64_t  used_ephemeral;
    int64_t  used_scalar[CA_MAX_SCALAR];
    int64_t  used_pods;
    uint64_t used_ports[CA_PORT_WORDS];
} ca_template;

/* thresholdBasedEstimationLimiter (threshold_based_limiter.go:27-64).  Duration must be 0
 * for a deterministic result; the kernels implement the node cap only. */
typedef struct ca_limiter {
    int32_t max_nodes;                        /* 0 = unlimited                           */
    int32_t reserved;
} ca_limiter;

typedef struct ca_estimate_result {
    int32_t  node_count;                      /* len(newNodesWithPods)                   */
    int32_t  n_scheduled;                     /* len(scheduledPods)                      */
    int32_t  nodes_added;                     /* new nodes created (incl. empty ones)    */
    int32_t  last_index_in;                   /* lastIndex the group started from        */
    int32_t  last_index_out;                  /* lastIndex after the group               */
    int32_t  status;                          /* CA_OK or CA_EUNSUPPORTED                */
    uint64_t evals;                           /* filter-chain evaluations performed      */
} ca_estimate_result;

typedef struct ca_removal_result {
    int32_t  removable;                       /* 1: NodeToBeRemoved, 0: UnremovableNode  */
    int32_t  reason;                          /* CA_UNREMOVABLE_*                        */
    int32_t  n_placed;                        /* pods placed before success/failure      */
    int32_t  last_index_in;
    uint64_t evals;
} ca_removal_result;

typedef struct ca_mirror ca_mirror;
typedef struct ca_podset ca_podset;

/* ---- kernel scope ------------------------------------
 * The kernels implement the six default-profile filters of the path.  InterPodAffinity,
 * PodTopologySpread and the volume plugins are no-ops for pods without the features
 * above; a pod WITH them carries CA_POD_OUT_OF_SCOPE (the caller's interning classifies
 * it) and is never simulated:
 *   - while the mirror holds a pod flagged CA_POD_REQUIRED_ANTI_AFFINITY, every
 *     simulation entry point returns CA_EUNSUPPORTED without running;
 *   - ca_fits_any_node / ca_check_predicates / ca_fits_matrix / ca_filter_out_schedulable:
 *     an out-of-scope pod in the call -> CA_EUNSUPPORTED, nothing run or changed;
 *   - ca_check_templates: the pair's result type is CA_PRED_UNSUPPORTED (verdict 0);
 *   - batches (ca_estimate_batch / _plan_run, ca_find_nodes_to_remove / _plan_run) use a
 *     PREFIX protocol: items are evaluated in order up to the first out-of-scope item u
 *     (a group with an out-of-scope or hostname-dependent pod, or a template flagged
 *     CA_NODE_ANTI_AFFINITY_PODS; a candidate whose pods to move include an out-of-scope
 *     pod, or that has more than CA_MAX_MOVED_PODS pods to move: the sweep keeps a
 *     candidate's distinct destination nodes in a fixed on-chip table).  Item u is reported (status CA_EUNSUPPORTED / reason CA_UNREMOVABLE_OUT_OF_SCOPE),
 *     every later item is CA_ENOTRUN / CA_UNREMOVABLE_NOT_RUN, and *last_index is the
 *     lastIndex item u starts from.  The call returns CA_OK; the caller runs item u on the
 *     reference path and calls again with the remaining items. */

/* ---- library ---------------------------------------------------------------- */
int ca_abi_version(void);
/* sizes of every ABI struct, in declaration order, for binding checks */
int ca_abi_struct_sizes(int32_t* out, int32_t cap);
int ca_device_count(int32_t* out);
const char* ca_status_string(int status);
/* Page-locked host memory for result buffers (sched_pod/sched_node/dest): results are
 * DMA'd straight into it instead of through a pageable staging copy.  C memory, so a cgo
 * caller may keep it across calls. */
int ca_host_alloc(size_t bytes, void** out);
int ca_host_free(void* p);

/* ---- mirror: the SoA ClusterSnapshot data plane in HBM ---------------------- */
int ca_mirror_create(int32_t device, ca_mirror** out);
int ca_mirror_destroy(ca_mirror* m);
int ca_mirror_clear(ca_mirror* m);                                   /* Clear()          */
int ca_mirror_add_nodes(ca_mirror* m, const ca_node_spec* nodes, int32_t n,
                        int32_t* out_first_pos);                     /* AddNode*         */
/* Scheduled pods: AddPod(pod, nodeName) for each (t->pods[pod_idx[i]], node_pos[i]); the
 * mirror keeps a copy of each record and of its selector terms.  out_ids receive mirror
 * pod ids (stable for the mirror's lifetime). */
int ca_mirror_add_pods(ca_mirror* m, const ca_pod_table* t, const int32_t* pod_idx,
                       const int32_t* node_pos, int32_t n, int32_t* out_ids);
int ca_mirror_remove_pod(ca_mirror* m, int32_t pod_id);              /* RemovePod        */
int ca_mirror_fork(ca_mirror* m);                                    /* Fork             */
int ca_mirror_revert(ca_mirror* m);                                  /* Revert           */
int ca_mirror_commit(ca_mirror* m);                                  /* Commit           */
int ca_mirror_node_count(const ca_mirror* m, int32_t* out);
int ca_mirror_pod_node(const ca_mirror* m, int32_t pod_id, int32_t* out_node_pos);
/* node pods in NodeInfo.Pods order (ids), returns count in *out_n (CA_ECAPACITY if cap short) */
int ca_mirror_node_pods(const ca_mirror* m, int32_t node_pos, int32_t* out_ids, int32_t cap,
                        int32_t* out_n);
/* RemoveNode (clustersnapshot.go:38; delta.go:150-186): the node and the pods on it leave
 * the snapshot.  Positions after it shift down by one (canonical order);
 * mirror pod ids stay valid (the removed node's pods report node -1); the resident hints
 * (ca_mirror_set_hints) are remapped the same way (hints to the removed node become -1).
 * Journaled: a Revert of the enclosing fork restores node, position and pods. */
int ca_mirror_remove_node(ca_mirror* m, int32_t node_pos);
/* Pods in the mirror flagged CA_POD_REQUIRED_ANTI_AFFINITY (> 0: simulations unsupported). */
int ca_mirror_scope_blockers(const ca_mirror* m, int32_t* out_n);

/* ---- device-resident pod sets (pending pods for Estimate) ------------------ */
int ca_podset_create(ca_mirror* m, const ca_pod_table* t, ca_podset** out);
int ca_podset_destroy(ca_podset* s);

/* ---- predicate checker ------------------------------------------------------- */
/* FitsAnyNodeMatching: *out_node = position or -1.  *out_prefilter_failed = 1 when the
 * PreFilter failed (the reference returns an error without scanning).  *last_index is
 * updated exactly as schedulerbased.go:131.  evals (may be NULL) accumulates
 * RunFilterPlugins calls. */
int ca_fits_any_node(ca_mirror* m, const ca_pod_table* t, int32_t pod, const ca_match_spec* match,
                     int32_t* last_index, int32_t* out_node, int32_t* out_prefilter_failed,
                     uint64_t* evals);
int ca_check_predicates(ca_mirror* m, const ca_pod_table* t, int32_t pod, int32_t node_pos,
                        ca_pred_result* out);
/* Dense feasibility: out[p*n_nodes + n] = 1 iff RunFilterPlugins(pod p, node n) succeeds
 * (CheckPredicates semantics, PreFilter failure -> 0). */
int ca_fits_matrix(ca_mirror* m, const ca_podset* s, uint8_t* out);
/* ComputeExpansionOption's feasibility check (CA/core/scaleup/orchestrator/
 * orchestrator.go:455-481) for every (node group, pod equivalence group) at once:
 * CheckPredicates(pod set entry samples[e], a fresh copy of templates[g] — the node
 * with its template pods) as schedulerbased.go:139-185 returns it.
 * out[g * n_samples + e]: type CA_PRED_OK when group e's pods join g's option (the
 * failing plugin / reasons otherwise: eg.SchedulingErrors); out_ok[g * n_samples + e]:
 * the same verdict as one byte (either output may be NULL).
 * The snapshot is not modified (the reference forks, adds the test node, reverts). */
int ca_check_templates(ca_mirror* m, const ca_podset* s, const int32_t* samples, int32_t n_samples,
                       const ca_template* templates, int32_t n_templates, ca_pred_result* out,
                       uint8_t* out_ok);
/* The same check with the node groups resident (a loop's node groups rarely change; the
 * Estimate plan keeps its inputs the same way): _create uploads the templates' test-node
 * rows once; _run takes the pod set and the samples of one loop and writes out / out_ok
 * as ca_check_templates does, its samples and results passing through page-locked memory
 * the kernel reads and writes in place (no copy-engine round trips).  s must belong to
 * the plan's mirror.  _run reads only the plan's rows and the pod set (both fixed when
 * their create calls return) and runs on the plan's own stream: it does not wait for
 * work still queued on the mirror (e.g. FilterOutSchedulable's record gather).  Asking
 * only for out_ok (one byte per pair instead of a 16-byte ca_pred_result) is the fast
 * form when the caller needs only the option set. */
typedef struct ca_expansion_plan ca_expansion_plan;
int ca_expansion_plan_create(ca_mirror* m, const ca_template* templates, int32_t n_templates,
                             ca_expansion_plan** out);
int ca_expansion_plan_run(ca_expansion_plan* p, const ca_podset* s, const int32_t* samples, int32_t n_samples,
                          ca_pred_result* out, uint8_t* out_ok);
/* the last run's kernel time (HIP events) */
int ca_expansion_plan_kernel_ms(const ca_expansion_plan* p, float* kernel_ms);
int ca_expansion_plan_destroy(ca_expansion_plan* p);

/* ---- estimator ---------------------------------------------------------------- */
/* Estimate() for G node groups in order, sharing lastIndex as the reference's single
 * checker does.  Group g's pods are pod_idx[group_off[g] .. group_off[g+1])
 * (indices into the pod set, in the order Estimate receives them).  Outputs:
 * results[g]; sched_pod/sched_node[group_off[g] + i] = i-th scheduled pod (pod set index)
 * and the new-node ordinal it went to (sched_node may be NULL).  The pods are sorted by
 * float64 score in Go 1.19 sort.Slice order (binpacking_estimator.go:74: pdqsort_func,
 * ties included).  CASIM_SORT_ORDER=stable in the environment (with
 * CASIM_KNOBS=1: the Estimate path's switches are read only then) breaks ties by list
 * position instead (the round-2 order, kept for A/B measurements). */
int ca_estimate_batch(ca_mirror* m, const ca_podset* s,
                      const int32_t* group_off, const int32_t* pod_idx,
                      const ca_template* templates, int32_t n_groups,
                      const ca_limiter* limiter, int32_t* last_index,
                      ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node);

/* Go 1.19 sort.Slice on the device for one slice whose i-th element has dense rank
 * ranks[i] (less(i, j) == ranks[i] < ranks[j]): perm[k] = input index of the element
 * sorted to position k — the permutation Estimate's score sort uses.  store selects the
 * kernel's element store (0 automatic, 1 LDS, 2 32-bit global, 3 64-bit global; a store
 * that cannot hold the input falls back to automatic).  limit > 0 replaces sort.Slice's
 * initial recursion limit bits.Len(n) (tests: reaches the heapSort fallback).  For tests
 * and Go-side checks. */
int ca_go_sort_ranks(int32_t device, const uint32_t* ranks, int32_t n, int32_t store, int32_t limit,
                     int32_t* perm);

/* Prepared form for repeated calls (bench): uploads group lists/templates once. */
typedef struct ca_estimate_plan ca_estimate_plan;
int ca_estimate_plan_create(ca_mirror* m, const ca_podset* s, const int32_t* group_off,
                            const int32_t* pod_idx, const ca_template* templates,
                            int32_t n_groups, ca_estimate_plan** out);
int ca_estimate_plan_run(ca_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                         ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node);
/* sched_pod == NULL (and sched_node == NULL) in ca_estimate_plan_run keeps the scheduled
 * pods in device memory: results[] and last_index are returned as usual, the pod lists
 * stay in the plan (same layout as sched_pod) until the next run.  Fetch them with
 * ca_estimate_plan_fetch (one D2H), or hand the device pointer to a device consumer. */
int ca_estimate_plan_fetch(const ca_estimate_plan* p, int32_t* sched_pod);
/* ca_estimate_plan_run with the scheduled pods as 16-bit podset indices (the podset holds
 * at most 65535 pods, else CA_EINVAL; 0xFFFF = not scheduled), same layout as sched_pod:
 * half the bytes across PCIe.  Page-locked sched_pod16 (ca_host_alloc) is written by the
 * zero-copy publisher while the chains run; other memory gets a stream-ordered copy. */
int ca_estimate_plan_run_u16(ca_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                             ca_estimate_result* results, uint16_t* sched_pod16);
int ca_estimate_plan_device_results(const ca_estimate_plan* p, const int32_t** sched_pod_dev);
int ca_estimate_plan_destroy(ca_estimate_plan* p);
/* statistics of the last run: speculation rounds, kernel time of the chain kernel (ms) */
int ca_estimate_plan_stats(const ca_estimate_plan* p, int32_t* rounds, float* chain_ms,
                           float* sort_ms, float* total_ms);
/* Device time of each phase of the last run, in ms: [0] score+static predicates,
 * [1] merge passes, [2] stream emission, [3] FFD chains (all speculation rounds),
 * [4] result compaction, [5] D2H of the results; [6] host wall time of the call;
 * [7] how the results reached sched_pod: 0 copied after the chains, 1 published
 * zero-copy while they ran, 2 the publisher gave up (kernels serialised, or a chain
 * died) and the results were copied instead; [8] 1 if the run took the decoupled Go
 * order (chains on the stable class order, Go's ids beside them: uniform classes and no
 * two classes of a group with equal scores), else 0.  Writes min(cap, 9) values; returns 9. */
int ca_estimate_plan_timings(const ca_estimate_plan* p, float* out, int32_t cap);
/* Record the per-phase timing events of later runs (on: default) or not: 8 event records
 * per run on the host's launch path; with them off, ca_estimate_plan_timings[0..5] and the
 * chain time of ca_estimate_plan_stats read 0. */
int ca_estimate_plan_set_phase_timing(ca_estimate_plan* p, int32_t on);
/* Whether the last run's outputs depend on the lastIndex it started from (then a caller
 * that ran the batch from a guessed lastIndex must re-run it from the true one), and
 * whether any FitsAnyNode call succeeded (if not, lastIndex passed through unchanged).
 * Used to chain batches sharded across GPUs. */
int ca_estimate_plan_chain_info(const ca_estimate_plan* p, int32_t* lin_sensitive, int32_t* had_success);
/* A run whose outputs do not depend on its input lastIndex (chain_info: not sensitive) but
 * that started from a wrong one: rewrite its results' last_index_in / last_index_out fields
 * for the exact input last_index_in (the run's own results[], in place) and return the
 * batch's exact output in *last_index_out (may be NULL).  The one-process-per-GPU form of
 * the node-group chain calls it on every rank after the walk. */
int ca_estimate_plan_rebase(const ca_estimate_plan* p, ca_estimate_result* results, int32_t last_index_in,
                            int32_t* last_index_out);
/* Diagnostics of the last run's first chain launch, one entry per group: the chain's
 * device wall-clock ticks (100 MHz) in bits 0-31, the number of single-pod steps (pods
 * not placed by the closed-form run path) in bits 32-63.  Returns the group count. */
int ca_estimate_plan_group_ticks(const ca_estimate_plan* p, uint64_t* out, int32_t cap);

/* ---- removal simulator ------------------------------------------------------- */
/* FindNodesToRemove(candidates, destinations) with legacy semantics (canPersist=false).
 * cand_status[c] != 0 carries the host-side GetPodsToMove verdict (drain.go:50-90):
 * CA_UNREMOVABLE_BLOCKED_BY_POD / _UNEXPECTED_ERROR.  Pods to move for candidate c are
 * move_pods[move_off[c] .. move_off[c+1]) (mirror pod ids, NodeInfo.Pods order).
 * hints[pod_id]: hinted node position or -1 (Hints.Get), updated in place (Hints.Set).
 * out_dest[move_off[c]+i] = destination of the i-th moved pod or -1. */
int ca_find_nodes_to_remove(ca_mirror* m, const int32_t* candidates, int32_t n_candidates,
                            const uint8_t* dest_mask, const int32_t* cand_status,
                            const int32_t* move_off, const int32_t* move_pods,
                            int32_t* hints, int32_t* last_index,
                            ca_removal_result* results, int32_t* out_dest);
/* [0] device time of all sweep kernels, [1] of the exact pass, [2] host time until the
 * exact pass's results were on the host, [3] host wall time of the call (ms); returns 4. */
/* Removal plan: FindNodesToRemove's inputs (candidates, destination mask, host drain
 * verdicts, pods to move) uploaded once and resident in HBM, for repeated sweeps over an
 * unchanged candidate set (RunOnce calls FindNodesToRemove every loop, legacy.go:146).
 * Duplicate candidates: CA_EUNSUPPORTED (use ca_find_nodes_to_remove).  run: hints are
 * per mirror pod in/out as in ca_find_nodes_to_remove, or NULL to use and update the
 * mirror's resident hint table (ca_mirror_set_hints/get_hints: the HintingSimulator's
 * hints kept in HBM, hinting_simulator.go:32-43).  out_dest may be NULL. */
typedef struct ca_removal_plan ca_removal_plan;
int ca_removal_plan_create(ca_mirror* m, const int32_t* candidates, int32_t n_candidates,
                           const uint8_t* dest_mask, const int32_t* cand_status,
                           const int32_t* move_off, const int32_t* move_pods, ca_removal_plan** out);
int ca_removal_plan_run(ca_removal_plan* p, int32_t* hints, int32_t* last_index,
                        ca_removal_result* results, int32_t* out_dest);
int ca_removal_plan_destroy(ca_removal_plan* p);
int ca_mirror_set_hints(ca_mirror* m, const int32_t* hints, int32_t n_pods);
int ca_mirror_get_hints(ca_mirror* m, int32_t* hints, int32_t n_pods);
int ca_removal_timings(const ca_mirror* m, float* out, int32_t cap);
int ca_removal_stats(const ca_mirror* m, int32_t* rounds, float* kernel_ms, float* total_ms);
/* Diagnostics: device wall-clock ticks (100 MHz) each candidate's simulation took in the
 * last sweep's last exact pass that ran it (0 for candidates it did not run). */
int ca_removal_candidate_ticks(const ca_mirror* m, uint64_t* out, int32_t n_candidates);

/* ---- FilterOutSchedulable ------------------------------------------------------ */
/* filterOutSchedulableByPacking (CA/core/podlistprocessor/filter_out_schedulable.go:95-124):
 * HintingSimulator.TrySchedulePods(snapshot, pending, ScheduleAnywhere, breakOnFailure=false)
 * (CA/simulator/scheduling/hinting_simulator.go:58-125) over the pending pods
 * t->pods[order[k]], k = 0..n-1, in that order (order NULL: the table order).  The caller
 * does the priority sort (:97-99).  Every pod that fits is added to the mirror (AddPod,
 * :77-82), on the current fork level, so a later Revert drops it.
 *  s            optional device-resident copy of t (ca_podset_create(m, t)); NULL uploads t.
 *  hints[k]     hinted node position of pod k, or -1 (Hints.Get).  Updated in place
 *               (Hints.Set): the node of every placed pod.
 *  similar pods (similar_pods.go:43-111): t->pods[i].similar_class (< n_classes, or -1).
 *               class_owner[c] is the dense controller id of class c.  At most 10 classes per
 *               controller are remembered; the controllers that overflow are counted in
 *               *n_overflowing (may be NULL).  class_owner NULL: no cap.
 *  out_node[k]  node position of pod k, or -1 (still unschedulable).
 *  out_pod_id[k] mirror pod id of the added pod, or -1 (may be NULL).
 *  *last_index  FitsAnyNode's lastIndex, in/out;  *evals += predicate evaluations.
 *  *n_placed    number of placed pods (may be NULL). */
int ca_filter_out_schedulable(ca_mirror* m, const ca_pod_table* t, const ca_podset* s,
                              const int32_t* order, int32_t n, const int32_t* class_owner,
                              int32_t n_classes, int32_t* hints, int32_t* last_index,
                              int32_t* out_node, int32_t* out_pod_id, int32_t* n_overflowing,
                              uint64_t* evals, int32_t* n_placed);
/* [0] device time of the last call's kernels, [1] host wall time of the call (ms),
 * [2] slot phases, [3] block steps, [4] block-wide ring scans, [5] window loads, [6] share of the
 * kernel's cycles in wave 0's walk and [7] walk cycles per pod (both CASIM_PROF builds only, else 0),
 * [8] path (1: feasibility-bitmap walk, 0: window sequencer), [9] resource shapes and [10] static
 * classes of the bitmap walk, [11..13] the bitmap walk's cycles per pod in its head (attributes,
 * hints), run (scan) and place sections (CASIM_PROF builds), [14] 0 (reserved) and [15] 1 when
 * its static words sit in LDS; returns 16. */
int ca_filter_stats(const ca_mirror* m, float* out, int32_t cap);

/* ---- scale-down eligibility ----------------------------
 * utilization.Calculate (CA/simulator/utilization/info.go:48-127) for every node of a
 * device-resident table, plus the FindEmptyNodesToRemove verdict (CA/simulator/cluster.go:
 * 187-202) from per-pod drain flags the host classified (GetPodsToMove with nil listers,
 * CA/simulator/drain.go:50-90, stays on the host).  All quantities are
 * Quantity.MilliValue() int64s; the ratio is one IEEE float64 division, bit-exact. */
#define CA_UTIL_CPU 0                          /* Info.ResourceName                      */
#define CA_UTIL_MEM 1
#define CA_UTIL_GPU 2

#define CA_UNODE_HAS_CPU     0x1u              /* Allocatable[cpu] present               */
#define CA_UNODE_HAS_MEM     0x2u              /* Allocatable[memory] present            */
#define CA_UNODE_HAS_GPU     0x4u              /* Allocatable[gpuConfig.ResourceName]    */
#define CA_UNODE_GPU_CONFIG  0x8u              /* gpuConfig != nil (info.go:49)          */

#define CA_UPOD_DAEMONSET    0x01u             /* pod_util.IsDaemonSetPod (utils/pod/pod.go:32-43) */
#define CA_UPOD_MIRROR       0x02u             /* pod_util.IsMirrorPod (pod.go:46-52)    */
#define CA_UPOD_DELETED      0x04u             /* DeletionTimestamp != nil               */
#define CA_UPOD_MOVABLE      0x08u             /* GetPodsToMove lists it                  */
#define CA_UPOD_BLOCKING     0x10u             /* GetPodsToMove fails on it               */

/* ca_util_info.status: the error calculateUtilizationOfResource returns (info.go:88-94) */
#define CA_UTIL_OK           0
#define CA_UTIL_NO_CPU       1                 /* "failed to get cpu from <node>"        */
#define CA_UTIL_ZERO_CPU     2                 /* "cpu is 0 at <node>"                   */
#define CA_UTIL_NO_MEM       3
#define CA_UTIL_ZERO_MEM     4

typedef struct ca_util_node {
    int64_t  alloc_milli[3];                  /* Allocatable MilliValue: cpu, memory, gpu */
    uint32_t flags;                           /* CA_UNODE_*                              */
    uint32_t _pad;
} ca_util_node;

typedef struct ca_util_pod {
    int64_t  req_milli[3];                    /* Σ Containers[*].Requests MilliValue (cpu, memory,
                                                 gpu); init containers and overhead excluded */
    int64_t  deletion_ns;                     /* DeletionTimestamp (ns since epoch) if DELETED */
    int64_t  grace_s;                         /* TerminationGracePeriodSeconds (nil -> 30) */
    uint32_t flags;                           /* CA_UPOD_*                               */
    uint32_t _pad;
} ca_util_pod;

typedef struct ca_util_info {                 /* utilization.Info                        */
    double   cpu, mem, gpu, utilization;
    int32_t  resource;                        /* CA_UTIL_CPU / _MEM / _GPU               */
    int32_t  status;                          /* CA_UTIL_OK or the error                 */
    int32_t  empty;                           /* FindEmptyNodesToRemove would list it    */
    int32_t  _pad;
} ca_util_info;

typedef struct ca_util_table ca_util_table;

/* Uploads nodes[n_nodes] and their pods (pods[pod_off[i] .. pod_off[i+1]) belong to node
 * i) to HBM on `device`; they stay resident until destroy. */
int ca_util_table_create(int32_t device, const ca_util_node* nodes, int32_t n_nodes,
                         const int32_t* pod_off, const ca_util_pod* pods, ca_util_table** out);
int ca_util_table_destroy(ca_util_table* t);
/* Replaces the table's rows (the snapshot changed: next loop, or after FilterOutSchedulable
 * placed pods), reusing its device buffers. */
int ca_util_table_update(ca_util_table* t, const ca_util_node* nodes, int32_t n_nodes, const int32_t* pod_off,
                         const ca_util_pod* pods);
/* Pods added to the snapshot since the rows were set (AddPod: FilterOutSchedulable's
 * placements, static_autoscaler.go:528): pods[k] now runs on node[k], in any order.
 * Replaces the previous added set (n = 0 clears it; ca_util_table_update clears it too).
 * Calculate adds them to their nodes' sums — only these records cross PCIe, not the nodes'
 * whole pod lists.  The copy is asynchronous and stream-ordered before the next
 * ca_util_calculate; page-locked arrays (ca_host_alloc) are copied from in place, so keep
 * them unchanged until that calculate returns. */
int ca_util_table_set_added(ca_util_table* t, const int32_t* node, const ca_util_pod* pods, int32_t n);
/* Calculate(nodeInfo, skipDaemonSetPods, skipMirrorPods, gpuConfig, currentTime) for every
 * node.  out NULL keeps the results in HBM (ca_util_device_results); otherwise out[n_nodes]
 * is filled — by the kernel itself when out is page-locked (ca_host_alloc), else by a copy.
 * *kernel_ms (may be NULL) = device time of the kernel. */
int ca_util_calculate(ca_util_table* t, int32_t skip_daemonset_pods, int32_t skip_mirror_pods,
                      int64_t now_ns, ca_util_info* out, float* kernel_ms);
int ca_util_device_results(const ca_util_table* t, const ca_util_info** out);

/* ---- multi-GPU ---------------------------------------------
 * One mirror per device (ca_mirror_create(device)), kept identical by the caller: every
 * snapshot change (add/remove nodes and pods, fork/revert/commit, hints) is applied to
 * each, in the same order, so node positions and pod ids agree.  The batch calls below
 * split their units into contiguous blocks, one per mirror (balanced by pods), run the
 * blocks concurrently from the caller's lastIndex, and fix up the lastIndex chain in the
 * library: a block that ran from a wrong lastIndex is re-run from the exact one when its
 * output depends on it, otherwise its lastIndex fields are re-based.  The
 * results are those of the single-mirror calls, bit for bit.  Replaces the Go caller's
 * loop over node groups (orchestrator.go:139-178 → Estimate per group) and the candidate
 * loop of FindNodesToRemove (cluster.go:130-137) when they are spread over GPUs. */
typedef struct ca_multi ca_multi;
int ca_multi_create(ca_mirror* const* mirrors, int32_t n, ca_multi** out);
int ca_multi_destroy(ca_multi* mm);   /* the mirrors stay the caller's */

/* Estimate batch (ca_estimate_batch semantics, prefix protocol included) over the mirrors'
 * blocks of node groups.  sched_pod is required (host memory; page-locked memory from
 * ca_host_alloc lets each block publish zero-copy); sched_node may be NULL. */
typedef struct ca_multi_estimate_plan ca_multi_estimate_plan;
int ca_multi_estimate_plan_create(ca_multi* mm, const ca_pod_table* t, const int32_t* group_off,
                                  const int32_t* pod_idx, const ca_template* templates, int32_t n_groups,
                                  ca_multi_estimate_plan** out);
int ca_multi_estimate_plan_run(ca_multi_estimate_plan* p, const ca_limiter* limiter, int32_t* last_index,
                               ca_estimate_result* results, int32_t* sched_pod, int32_t* sched_node);
/* blocks, re-runs of the last run, and the first group of each block (n_blocks + 1 values) */
int ca_multi_estimate_plan_stats(const ca_multi_estimate_plan* p, int32_t* n_blocks, int32_t* reruns,
                                 int32_t* block_first_group, int32_t cap);
/* node groups in the blocks the last run had to run again (a block run from a wrong
 * lastIndex whose output depends on it) */
int ca_multi_estimate_plan_rerun_units(const ca_multi_estimate_plan* p, int32_t* groups_rerun);
int ca_multi_estimate_plan_destroy(ca_multi_estimate_plan* p);
int ca_multi_estimate_batch(ca_multi* mm, const ca_pod_table* t, const int32_t* group_off, const int32_t* pod_idx,
                            const ca_template* templates, int32_t n_groups, const ca_limiter* limiter,
                            int32_t* last_index, ca_estimate_result* results, int32_t* sched_pod,
                            int32_t* sched_node);

/* FindNodesToRemove (ca_find_nodes_to_remove semantics, prefix protocol included) over the
 * mirrors' blocks of candidates.  hints[n_pods] per mirror pod (or NULL: none), updated in
 * place; n_pods must equal every mirror's pod count.  out_dest may be NULL. */
typedef struct ca_multi_removal_plan ca_multi_removal_plan;
int ca_multi_removal_plan_create(ca_multi* mm, const int32_t* candidates, int32_t n_candidates,
                                 const uint8_t* dest_mask, const int32_t* cand_status, const int32_t* move_off,
                                 const int32_t* move_pods, ca_multi_removal_plan** out);
int ca_multi_removal_plan_run(ca_multi_removal_plan* p, int32_t* hints, int32_t n_pods, int32_t* last_index,
                              ca_removal_result* results, int32_t* out_dest);
int ca_multi_removal_plan_stats(const ca_multi_removal_plan* p, int32_t* n_blocks, int32_t* reruns,
                                int32_t* block_first_candidate, int32_t cap);
/* candidates in the blocks the last run had to run again */
int ca_multi_removal_plan_rerun_units(const ca_multi_removal_plan* p, int32_t* candidates_rerun);
/* host wall time (ms) of the last run's phases: probe, map, compose, resolve, fix-up
 * (the serial path reports its block runs as "resolve"); returns the count (5) */
int ca_multi_removal_plan_timings(const ca_multi_removal_plan* p, float* ms, int32_t cap);
int ca_multi_removal_plan_destroy(ca_multi_removal_plan* p);
int ca_multi_find_nodes_to_remove(ca_multi* mm, const int32_t* candidates, int32_t n_candidates,
                                  const uint8_t* dest_mask, const int32_t* cand_status, const int32_t* move_off,
                                  const int32_t* move_pods, int32_t* hints, int32_t n_pods, int32_t* last_index,
                                  ca_removal_result* results, int32_t* out_dest);

/* ---- one process per GPU: the sweep's phases ---------------------
 * A caller with one process per GPU (each holding its own mirror replica and a removal plan
 * over its contiguous block of candidates, blocks in candidate order) composes the blocks'
 * lastIndex chain itself, exchanging one fixed-size ca_sweep_phase record per block per
 * phase over its own transport (an RCCL all_gather over xGMI, or any all-gather) — the three
 * phases ca_multi_removal_plan_run runs inside one process:
 *   0. once per plan: ca_removal_plan_sensitive_pods; block d's guess_base = L0 + the sum
 *      over the blocks before it (the probe's rough guess of its input);
 *   1. PROBE   run_phase(kind = PROBE, guess_base): out adv (the block's lastIndex advance as
 *              its successful scans saw it), succ, n_sensitive.  All-gather the records.
 *   2. MAP     est_base = (L0 + the earlier blocks' adv) mod n_nodes; run_phase(kind = MAP):
 *              every block with n_sensitive > 0 builds its tables and its map (lastIndex out
 *              by class of its input).  All-gather the records.
 *   3. ca_sweep_compose(all records, L0) -> each block's exact input lastIndex, or
 *      CA_SWEEP_NOT_REACHED after the first block the maps cannot carry the chain through.
 *   4. RESOLVE run_phase(kind = RESOLVE, *last_index = the composed input): the block's
 *      results, out_dest and hints (Hints.Set of its candidates' pods), exact.  A block not
 *      reached runs ca_removal_plan_run from its exact input once its predecessors are final.
 * The chain is then the blocks' last_index outputs in order.  Between a plan's PROBE and its
 * RESOLVE nothing else may use its mirror; hints must not be NULL (caller-held hints); a plan
 * with a prefix-protocol cut (an out-of-scope candidate) runs whole calls only
 * (ca_removal_plan_phased reports 0). */
#define CA_SWEEP_PHASE_PROBE    1
#define CA_SWEEP_PHASE_MAP      2
#define CA_SWEEP_PHASE_RESOLVE  3
#define CA_SWEEP_MAP_INTS       130           /* 64 outputs + 65 fit points + class mode */
#define CA_SWEEP_NOT_REACHED    INT32_MIN

typedef struct ca_sweep_phase {
    int32_t kind;                             /* CA_SWEEP_PHASE_*                        */
    int32_t est_base;                         /* MAP in: the estimate of the block's input */
    int64_t guess_base;                       /* PROBE in                                */
    int64_t adv;                              /* PROBE out                               */
    int32_t succ;                             /* PROBE out: candidates with a successful scan */
    int32_t n_sensitive;                      /* PROBE/MAP out: lastIndex-sensitive candidates */
    int32_t map_ran;                          /* MAP out: tables built by this call      */
    int32_t map_ok;                           /* MAP out: map[] valid                    */
    int32_t map[CA_SWEEP_MAP_INTS];           /* MAP out                                 */
} ca_sweep_phase;

int ca_removal_plan_sensitive_pods(const ca_removal_plan* p, int64_t* out);
int ca_removal_plan_phased(const ca_removal_plan* p, int32_t* out);
/* hints[n_pods] caller-held (PROBE and MAP read them; RESOLVE updates the block's pods) */
int ca_removal_plan_run_phase(ca_removal_plan* p, ca_sweep_phase* ph, int32_t* hints, int32_t* last_index,
                              ca_removal_result* results, int32_t* out_dest);
/* recs[D]: every block's MAP record, in block order; lin[D] = each block's input lastIndex
 * or CA_SWEEP_NOT_REACHED; *n_reached (may be NULL) = the blocks reached. */
int ca_sweep_compose(const ca_sweep_phase* recs, int32_t n_blocks, int32_t n_nodes, int32_t last_index,
                     int32_t* lin, int32_t* n_reached);

/* ---- interning: API values -> the records' ids and bitsets --------
 * What a cgo shim does before it fills ca_node_spec / ca_pod_spec / ca_selector_req
 * records, here so the shim binds it instead of restating it:
 *   taint classes   NoSchedule/NoExecute (key, value, effect) — other effects are not
 *                   filter taints (V/k8s.io/component-helpers/scheduling/corev1/helpers.go:78-101)
 *   label pairs     (key, value) referenced by nodeSelector / In / NotIn
 *   label keys      keys referenced by Exists / DoesNotExist
 *   int keys        keys referenced by Gt / Lt (node values parsed as strconv.ParseInt)
 *   ports           (hostIP, protocol, hostPort), sanitised as HostPortInfo.sanitize
 *                   (SF/types.go:923-931: "" -> 0.0.0.0 / TCP; hostPort <= 0 ignored)
 *   scalars         IsScalarResourceName (scheduler/util/utils.go:158-161; fit.go:160-176)
 *   names           node names (spec.nodeName, matchFields metadata.name, name_id)
 * Protocol: intern every value of every object the call will see first (nodes, templates,
 * pods — autoscaler_amd/intern.py:Interner.observe), then encode the records: port
 * conflicts and toleration masks range over every value interned so far.  Universes have
 * the records' fixed widths; a value past a width gets id -1 (remembered as overflow: a
 * node taint past the width sets bit 63, which a pod's mask covers only when it tolerates
 * every overflow taint), and an encoder reports *out_of_scope = 1 for a pod whose
 * simulation would need such a value — the shim then sets CA_POD_OUT_OF_SCOPE (prefix
 * protocol).  Quantities (MilliValue / Value), score sums, PreFilter NodeNames, scope and
 * hostname flags stay with the shim (Go has them natively; intern.py shows each).  Pinned
 * with autoscaler_amd/intern.py by tests/golden/intern_fixtures.json (tests/c_abi/
 * intern_driver.c replays tests/golden/intern_calls.txt, generated from those cases). */
typedef struct ca_interner ca_interner;
#define CA_INTERN_NOT_INTERNED (-2)           /* not a value of the universe (effect, non-scalar, port <= 0) */
#define CA_U_TAINTS       0
#define CA_U_LABEL_PAIRS  1
#define CA_U_LABEL_KEYS   2
#define CA_U_INT_KEYS     3
#define CA_U_PORTS        4
#define CA_U_SCALARS      5
#define CA_U_NAMES        6

typedef struct ca_str_pair { const char* key; const char* value; } ca_str_pair;
typedef struct ca_taint_str { const char* key; const char* value; const char* effect; } ca_taint_str;
typedef struct ca_toleration_str {
    const char* key; const char* op;          /* op: "", "Equal" or "Exists"             */
    const char* value; const char* effect;
} ca_toleration_str;
typedef struct ca_port_str { const char* host_ip; const char* protocol; int32_t host_port; int32_t reserved; } ca_port_str;
typedef struct ca_requirement_str {
    const char* key;
    const char* op;                           /* In NotIn Exists DoesNotExist Gt Lt      */
    const char* const* values;
    int32_t n_values;
    int32_t is_field;                         /* 1: a matchFields requirement            */
} ca_requirement_str;

int ca_interner_create(ca_interner** out);
int ca_interner_destroy(ca_interner* it);
int ca_interner_size(const ca_interner* it, int32_t universe, int32_t* n, int32_t* n_overflow);
int ca_is_scalar_resource(const char* name);  /* 1 / 0 */
/* *id: the value's bit position, -1 past the width, or CA_INTERN_NOT_INTERNED */
int ca_intern_taint(ca_interner* it, const char* key, const char* value, const char* effect, int32_t* id);
int ca_intern_label_pair(ca_interner* it, const char* key, const char* value, int32_t* id);
int ca_intern_label_key(ca_interner* it, const char* key, int32_t* id);
int ca_intern_int_key(ca_interner* it, const char* key, int32_t* id);
int ca_intern_port(ca_interner* it, const char* host_ip, const char* protocol, int32_t host_port, int32_t* id);
int ca_intern_resource(ca_interner* it, const char* name, int32_t* id);
int ca_intern_name(ca_interner* it, const char* name, int32_t* id);
/* a node's taints (interned here), label_pairs, label_keys, int_label, int_label_valid */
int ca_intern_encode_node(ca_interner* it, const ca_str_pair* labels, int32_t n_labels, const ca_taint_str* taints,
                          int32_t n_taints, ca_node_spec* out);
/* a pod's tolerated_taints and its CA_POD_TOLERATES_UNSCHED flag (other flags kept) */
int ca_intern_encode_tolerations(const ca_interner* it, const ca_toleration_str* t, int32_t n, ca_pod_spec* out,
                                 int32_t* out_of_scope);
/* a pod's port_conflict / port_use over its containers' ports */
int ca_intern_encode_ports(ca_interner* it, const ca_port_str* p, int32_t n, ca_pod_spec* out, int32_t* out_of_scope);
/* a pod's node_selector bits */
int ca_intern_encode_node_selector(ca_interner* it, const ca_str_pair* sel, int32_t n, ca_pod_spec* out,
                                   int32_t* out_of_scope);
/* one non-empty nodeSelectorTerm (expressions, then fields) -> rows out[cap]; *n_rows = the
 * rows it needs (CA_ECAPACITY when cap is short).  An empty term matches nothing and is
 * dropped by the caller (nodeaffinity.go:83-85). */
int ca_intern_compile_term(ca_interner* it, const ca_requirement_str* reqs, int32_t n, ca_selector_req* out,
                           int32_t cap, int32_t* n_rows, int32_t* out_of_scope);

/* ---- planner: committing removal simulation ----------------------
 * Planner.categorizeNodes' simulation loop (CA/core/scaledown/planner/planner.go:252-296)
 * over a RemovalSimulator built with persistSuccessfulSimulations = true (planner.go:89):
 * candidates are simulated in order, each by SimulateNodeRemoval (CA/simulator/cluster.go:
 * 145-184) on the CURRENT snapshot.  A removable candidate's simulation is committed into
 * the mirror (withForkedSnapshot Commit, cluster.go:204-218): its pods to move leave it
 * (RemovePod, :228-233) and their copies (Spec.NodeName and TPU requests cleared, :235-240,
 * tpu.go:57-79) stay on their destinations (AddPod); the node leaves the destination set
 * (planner.go:280); its pods are charged to the PDB budgets (RemainingPdbTracker.RemovePods,
 * CA/core/scaledown/pdb/basic.go:86-95).  A later candidate's pods to move are its
 * caller-given pods followed by the copies committed onto it, in commit order (NodeInfo.Pods
 * appends).  The loop stops before the next candidate once max_removable candidates are
 * removable (planner.go:268-271, unneededNodesLimit; <= 0: no limit); the rest are
 * CA_UNREMOVABLE_NOT_RUN.  Prefix protocol and kernel scope as ca_find_nodes_to_remove. */
typedef struct ca_plan_result {
    int32_t  removable;                       /* NodeToBeRemoved, committed              */
    int32_t  reason;                          /* CA_UNREMOVABLE_*                        */
    int32_t  n_placed;
    int32_t  last_index_in;
    uint64_t evals;
    int32_t  first_move;                      /* removable: moves[first_move, +n_moves)  */
    int32_t  n_moves;                         /*   = PodsToReschedule, in order          */
    int32_t  blocking_pod;                    /* NotEnoughPdb (drain.go checkPdbs): mirror
                                                 pod id, else -1                          */
    int32_t  risky;                           /* CanRemovePods inParallel == false
                                                 (planner.go:274-278, basic.go:66-84)     */
} ca_plan_result;

typedef struct ca_plan_move {
    int32_t candidate;                        /* index into candidates[]                 */
    int32_t pod;                              /* mirror pod id that left the candidate   */
    int32_t new_pod;                          /* mirror pod id of its copy               */
    int32_t node;                             /* destination node position               */
} ca_plan_move;

/* RemainingPdbTracker (basic.go): PDB memberships of the mirror pods (namespace + selector
 * match, computed by the caller), pdb indices ascending per pod, CSR over pod ids <
 * n_pods; a copy inherits its original's memberships.  allowed[] = DisruptionsAllowed,
 * decremented in place.  n_pdbs == 0 (or a NULL table): no PDBs. */
typedef struct ca_pdb_table {
    int32_t        n_pdbs;
    int32_t*       allowed;
    const int32_t* pod_off;                   /* [n_pods + 1] */
    const int32_t* pod_pdb;
} ca_pdb_table;

/* hints[n_pods]: as ca_find_nodes_to_remove, n_pods = the mirror's pod count (a copy's hint
 * is its destination).  moves[moves_cap]: every committed move in order; *n_moves = their
 * number (if it exceeds moves_cap the first moves_cap are written and the call still
 * completes; ca_plan_last_moves returns all of them).  All or nothing: on an error return
 * the mirror, pdbs->allowed, hints and *last_index are exactly as before the call (it
 * runs inside a fork of its own, committed into the caller's state only on success);
 * only the pod ids its copies took stay consumed (ids are never reused). */
int ca_plan_removals(ca_mirror* m, const int32_t* candidates, int32_t n_candidates,
                     const uint8_t* dest_mask, const int32_t* cand_status,
                     const int32_t* move_off, const int32_t* move_pods,
                     int32_t max_removable, const ca_pdb_table* pdbs,
                     int32_t* hints, int32_t n_pods, int32_t* last_index,
                     ca_plan_result* results, ca_plan_move* moves, int32_t moves_cap, int32_t* n_moves);
int ca_plan_last_moves(const ca_mirror* m, ca_plan_move* out, int32_t cap);
/* last call: speculation rounds, rounds cut short by a commit conflict, candidates
 * simulated on the device (all rounds), host wall time (ms) */
int ca_plan_stats(const ca_mirror* m, int32_t* rounds, int32_t* conflicts, int32_t* simulated, float* total_ms);
/* how the last ca_plan_removals ran: 1 = one device-resident chain over every candidate
 * (node rows in LDS; no pod to move with host ports or extended resources), 0 = speculative
 * sweep windows validated on the host (every other case) */
int ca_plan_last_path(const ca_mirror* m);
/* diagnostics of the last device-chain call: shader-clock cycles per phase (init, pod lists,
 * PDB checks, fork, hint checks, scans, AddPod, commit, revert, total, scanned blocks,
 * skip windows) into cycles[cap]; host_ms[5] = mirror sync, launch + kernel, kernel,
 * readback, replay into the mirror.  Returns the number of counters. */
int ca_plan_chain_profile(const ca_mirror* m, uint64_t* cycles, int32_t cap, float* host_ms);

#ifdef __cplusplus
}
#endif
#endif /* CASIM_H */
