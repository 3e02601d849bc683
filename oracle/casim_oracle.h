/*
 * casim_oracle.h — CPU restatement of cluster-autoscaler's scheduling-simulation
 * hot path.  TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg as the checker.  The product (libcasim.so) never
 * links or calls it.
 *
 * It consumes the same interned records as the C ABI (include/casim.h) and restates
 * the reference algorithms independently of the HIP kernels: a ClusterSnapshot with
 * Delta-style fork/revert/commit (undo journal), the rotating FitsAnyNodeMatching
 * scan, the default-profile filter chain, BinpackingNodeEstimator.Estimate and the
 * legacy RemovalSimulator sweep with HintingSimulator.  Each function cites the
 * reference file:line it follows (CA/ = cluster-autoscaler/, SF/ = vendored
 * k8s.io/kubernetes/pkg/scheduler/framework/).
 *
 * Parity pinning: the restatement is checked against the reference's own known-answer
 * tests (tests/golden/ fixtures).  The Go reference cannot be built here
 * (no Go toolchain), so there is no oracle/_ref.
 */
#ifndef CASIM_ORACLE_H
#define CASIM_ORACLE_H
#include "casim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_state or_state;

or_state* or_create(void);
void      or_destroy(or_state* s);
int       or_clear(or_state* s);
int       or_add_nodes(or_state* s, const ca_node_spec* nodes, int32_t n, int32_t* out_first);
int       or_add_pods(or_state* s, const ca_pod_table* t, const int32_t* pod_idx,
                      const int32_t* node_pos, int32_t n, int32_t* out_ids);
int       or_remove_pod(or_state* s, int32_t pod_id);
int       or_remove_node(or_state* s, int32_t pos);
/* pods with CA_POD_REQUIRED_ANTI_AFFINITY in the snapshot (include/casim.h kernel scope) */
int       or_scope_blockers(const or_state* s);
/* Estimate's score sort: stable (ties by list position, the device order) or Go 1.19's
 * sort.Slice pdqsort (the reference; gosort.c) */
#define OR_SORT_STABLE 0
#define OR_SORT_GO_PDQ 1
int       or_set_sort_mode(or_state* s, int32_t mode);
/* gosort.c: sort.Slice(x, less) with less(i, j) = key[i] > key[j]; perm[k] = input index
 * at sorted position k.  go_sort_stats: breakPatterns and heapSort calls so far. */
void      go_sort_slice_desc(const double* key, int32_t n, int32_t* perm);
void      go_sort_slice_desc_limit(const double* key, int32_t n, int32_t limit, int32_t* perm);
void      go_sort_stats(int64_t* out2);
int       or_fork(or_state* s);
int       or_revert(or_state* s);
int       or_commit(or_state* s);
int       or_node_count(const or_state* s);
int       or_node_pods(const or_state* s, int32_t node, int32_t* out, int32_t cap);
int       or_pod_node(const or_state* s, int32_t pod_id);
/* free resources of a node (for white-box checks): cpu, mem, eph, pods */
int       or_node_state(const or_state* s, int32_t node, int64_t* out4);

int or_fits_any_node(or_state* s, const ca_pod_table* t, int32_t pod, const ca_match_spec* match,
                     int32_t* last_index, int32_t* out_node, int32_t* out_prefilter_failed,
                     uint64_t* evals);
int or_check_predicates(or_state* s, const ca_pod_table* t, int32_t pod, int32_t node,
                        ca_pred_result* out);
/* utilization.Calculate (CA/simulator/utilization/info.go:48-127) and the
 * FindEmptyNodesToRemove verdict (CA/simulator/cluster.go:187-202) per node; the table
 * layout of ca_util_table_create (pods[pod_off[i] .. pod_off[i+1]) on node i). */
int or_node_utilization(const ca_util_node* nodes, int32_t n_nodes, const int32_t* pod_off,
                        const ca_util_pod* pods, int32_t skip_daemonset_pods, int32_t skip_mirror_pods,
                        int64_t now_ns, ca_util_info* out);
int or_check_templates(or_state* s, const ca_pod_table* t, const int32_t* samples, int32_t n_samples,
                       const ca_template* templates, int32_t n_templates, ca_pred_result* out);
int or_estimate(or_state* s, const ca_pod_table* t, const int32_t* group_off,
                const int32_t* pod_idx, const ca_template* templates, int32_t n_groups,
                const ca_limiter* limiter, int32_t* last_index, ca_estimate_result* results,
                int32_t* sched_pod, int32_t* sched_node);
/* TrySchedulePods (hinting_simulator.go:58-89) over mirror pods pod_ids[] (moved-pod
 * semantics when `as_moved`: nodeName cleared, TPU requests cleared).  Returns the
 * number of statuses (placed pods); dest[i] = node or -1. */
int or_try_schedule_pods(or_state* s, const int32_t* pod_ids, int32_t n,
                         const ca_match_spec* match, int32_t break_on_failure,
                         int32_t* hints, int32_t* last_index, int32_t* dest, uint64_t* evals);
/* filterOutSchedulableByPacking (filter_out_schedulable.go:95-124): TrySchedulePods over
 * the pending pods t->pods[order[k]] with ScheduleAnywhere, breakOnFailure=false, the
 * similar-pods cache with its 10-per-controller cap (similar_pods.go:88-111); placed pods
 * are committed (no fork).  Same contract as ca_filter_out_schedulable. */
int or_filter_out_schedulable(or_state* s, const ca_pod_table* t, const int32_t* order, int32_t n,
                              const int32_t* class_owner, int32_t n_classes, int32_t* hints,
                              int32_t* last_index, int32_t* out_node, int32_t* out_pod_id,
                              int32_t* n_overflowing, uint64_t* evals, int32_t* n_placed);
int or_find_nodes_to_remove(or_state* s, const int32_t* candidates, int32_t n_candidates,
                            const uint8_t* dest_mask, const int32_t* cand_status,
                            const int32_t* move_off, const int32_t* move_pods,
                            int32_t* hints, int32_t* last_index,
                            ca_removal_result* results, int32_t* out_dest);
/* Planner.categorizeNodes' loop, canPersist=true (ca_plan_removals semantics) */
int or_plan_removals(or_state* s, const int32_t* candidates, int32_t n_candidates,
                     const uint8_t* dest_mask, const int32_t* cand_status,
                     const int32_t* move_off, const int32_t* move_pods,
                     int32_t max_removable, const ca_pdb_table* pdbs,
                     int32_t* hints, int32_t n_pods, int32_t* last_index,
                     ca_plan_result* results, ca_plan_move* moves, int32_t moves_cap, int32_t* n_moves);

#ifdef __cplusplus
}
#endif
#endif
