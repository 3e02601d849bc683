// mirror.h — the ClusterSnapshot mirror: host journal + device SoA rows.
//
// Host side keeps the authoritative rows (so Fork/Revert/Commit are O(changes),
// DeltaClusterSnapshot semantics, CA/simulator/clustersnapshot/delta.go:43-475);
// device rows are re-synchronised lazily (dirty rows only) before a kernel reads them.
#pragma once
#include "casim_internal.h"
#include <array>
#include <deque>
#include <cstdlib>
#include <new>
#include <sys/mman.h>

namespace casim {

enum { J_FORK = 1, J_ADD_NODE, J_ADD_POD, J_REMOVE_POD, J_REMOVE_NODE };

struct JournalEntry {
    int32_t kind, node, pod, slot;
    uint64_t ports[CA_PORT_WORDS];
};

struct NodeRow {
    ca_node_spec spec;
    int64_t req_cpu = 0, req_mem = 0, req_eph = 0;
    int64_t req_scalar[CA_MAX_SCALAR] = {0};
    int64_t npods = 0;
    uint64_t ports[CA_PORT_WORDS] = {0};
    std::vector<int32_t> pods;   // NodeInfo.Pods order
};

struct PodRow {
    ca_pod_spec spec;            // selector indices re-based on the mirror tables
    int32_t node = -1;
};

struct ca_mirror_impl;

// Device pod table: hot rows + full records + selector tables.
struct DevPodTable {
    DevBuf hot, spec, terms, reqs, names;
    int32_t n_pods = 0, n_terms = 0, n_reqs = 0, n_names = 0;
    int upload(const ca_pod_spec* pods, int32_t n, const ca_selector_term* terms, int32_t nt,
               const ca_selector_req* reqs, int32_t nr, const int32_t* names, int32_t nn, hipStream_t st);
    // the same with the hot rows and records copied into the page-locked `stage` first (host
    // threads) and the copies left queued on st: the caller syncs st before stage is reused
    int upload_staged(const ca_pod_spec* pods, int32_t n, const ca_selector_term* terms, int32_t nt,
                      const ca_selector_req* reqs, int32_t nr, const int32_t* names, int32_t nn, HostBuf& stage,
                      hipStream_t st);
    // append pods [n_pods, n_pods + k) and the selector tables' new tails (the mirror's
    // tables only grow between Clear()s), keeping what is on the device
    int append(const ca_pod_spec* new_pods, int32_t k, const ca_selector_term* terms, int32_t nt,
               const ca_selector_req* reqs, int32_t nr, const int32_t* names, int32_t nn, hipStream_t st);
    // append src's records idx[0..k) (already on the device: a podset), in order; the
    // records must hold no selector-table or PreFilter-name references
    int append_gather(const DevPodTable& src, const int32_t* idx, int32_t k, DevBuf& d_idx, hipStream_t st);
};

// Per-mirror scratch of ca_find_nodes_to_remove, kept across calls (no per-call
// hipMalloc); host staging is page-locked.
struct SweepScratch {
    DevBuf in, lin, need, out, todo, tab, wl;
    DevBuf tev, tdest;              // table lanes' evaluation counts and pod destinations (first round)
    DevBuf tfp, vp, mode;           // table rows' fit-point classes; visible-node prefix counts; class mode
    DevBuf bsum;                    // per 64-node block: maxima of the visible rows (sweep.hip BlockSum)
    DevBuf chainl;                  // the host walk's serial exact chain: candidates in order
    DevBuf bmap;                    // a multi-device range's block map (k_walk_map)
    HostBuf h_in, h_tab, h_out, h_todo, h_lin, h_wl, h_tfp, h_l0, h_chainl, h_bmap;
    // the host walk's table rounds: each round's compact rows (main and side rows), read in
    // place by the walk for the rest of the call; pooled across calls
    std::deque<HostBuf> rbuf;
    // device mappings of h_todo and the round buffers (cleared whenever one of them moves)
    std::vector<std::pair<void*, void*>> dmap;
    // the device pipeline of the last call shape, replayed as a graph (sweep.hip sweep_core)
    hipGraphExec_t gexec = nullptr;
    uint64_t gkey = 0, gseen = 0;
    // serial-only calls (sweep_core): the next call's mode and the measured ms per candidate
    bool serial_next = false;
    int32_t serial_calls = 0;
    int32_t serial_C = 0, serial_S = 0;     // shape of the call that decided serial_next
    float serial_ms_per = 0, pipe_ms_per = 0;
    ~SweepScratch() {
        if (gexec) (void)hipGraphExecDestroy(gexec);
    }
};

// Per-mirror scratch of ca_filter_out_schedulable (filter.hip).
struct FilterScratch {
    DevBuf in, zero, out;          // inputs (order, hints, class tables), zeroed state, outputs
    HostBuf h_in, h_out;
    DevPodTable pods;              // the pending table when the caller passes no podset
    HostBuf h_pods;                // ... staged in page-locked memory (its copies run beside the preparation)
    DevBuf gather_idx;             // podset indices of the placed pods (mirror records gathered on the device)
    float kernel_ms = 0, total_ms = 0;
    int32_t phases = 0, steps = 0, ring_scans = 0, windows = 0;
    float seq_share = 0, walk_cycles_per_pod = 0;   // CASIM_PROF builds: sequencer walk share, cycles/pod
    // feasibility-bitmap path (filter.hip k_fb_*): pods, shapes, static classes, bitmaps
    DevBuf fb_in, fb_bits;
    HostBuf h_fb;
    int32_t path = 0;              // last call: 1 bitmap walk, 0 window sequencer
    int32_t fb_shapes = 0, fb_classes = 0;
    float fb_cyc_per_pod[3] = {0, 0, 0};   // CASIM_PROF builds: bitmap walk cycles per pod (head, run, place)
    int32_t fb_stat_lds = 0;                // bitmap walk: static words in LDS
};

// Per-mirror scratch of the planner's device chain (plan_chain.hip), freed with the mirror
// and allocated on its device.
struct PlanChainScratch {
    DevBuf in, work, out;
    HostBuf h_in, h_out;
};

// Dirty-row staging of sync_nodes: one H2D copy + a scatter kernel.
struct RowStage {
    DevBuf d;
    HostBuf h;
    HostBuf full;                  // page-locked staging: full-table hot + ext columns, appended pod records
};

// ca_plan_removals (planner.hip): the last call's moves and counters.
struct PlanStats {
    int32_t rounds = 0, conflicts = 0, simulated = 0;
    int32_t path = 0;              // 1: the device chain (plan_chain.hip), 0: speculative windows
    std::vector<uint64_t> chain_prof;   // the chain's phase cycle counters (plan_chain.hip PC_*)
    float host_ms[5] = {0, 0, 0, 0, 0};  // sync, launch+kernel, kernel, readback, replay
    float total_ms = 0;
    std::vector<ca_plan_move> moves;
};

struct Stats {
    int32_t rounds = 0;
    float kernel_ms = 0, sort_ms = 0, total_ms = 0;
    int32_t lin_sensitive = 0;    // batch output depends on the input lastIndex
    int32_t had_success = 0;      // some FitsAnyNode call of the batch succeeded
    float exact_ms = 0;           // sweep: device time of the exact pass
    float walk_ms = 0;            // sweep: host time up to the end of the exact pass
};

}  // namespace casim

namespace casim {
// The mirror's pod records: ids are never reused (Revert detaches pods, Clear() starts over),
// so the table only grows — every planner run appends its committed copies, every
// FilterOutSchedulable call its placements.  Rows live in fixed chunks of 2^16 records that
// are never moved: growing a contiguous vector past its capacity copied every record
// (~40 MB at C3 size: a 30 ms stall inside whichever call crossed the boundary).  Chunks
// come from 2 MiB-aligned anonymous mappings with transparent huge pages asked for (4 KiB
// first-touch faults cost more than the records' copies).
template <class T> class ChunkVec {
  public:
    static constexpr size_t kBits = 16, kRows = (size_t)1 << kBits, kMask = kRows - 1;
    ChunkVec() = default;
    ChunkVec(const ChunkVec&) = delete;
    ChunkVec& operator=(const ChunkVec&) = delete;
    ~ChunkVec() {
        clear();
        for (T* c : chunks_) unmap(c);
    }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    size_t capacity() const { return chunks_.size() * kRows; }
    T& operator[](size_t i) { return chunks_[i >> kBits][i & kMask]; }
    const T& operator[](size_t i) const { return chunks_[i >> kBits][i & kMask]; }
    T& back() { return (*this)[n_ - 1]; }
    void reserve(size_t n) {
        while (capacity() < n) chunks_.push_back(map());
    }
    void push_back(const T& v) {
        reserve(n_ + 1);
        new (&(*this)[n_]) T(v);
        n_++;
    }
    void resize(size_t n) {                     // (grow: value-initialised rows; shrink: dropped)
        reserve(n);
        for (size_t i = n_; i < n; i++) new (&(*this)[i]) T();
        for (size_t i = n; i < n_; i++) (*this)[i].~T();
        n_ = n;
    }
    void clear() { resize(0); }                 // (the chunks stay mapped for the next load)
    void resize_for_overwrite(size_t n) {       // grow without initialising: the caller writes every new row
        static_assert(std::is_trivially_destructible<T>::value, "rows dropped without destructors");
        if (n <= n_) { resize(n); return; }
        reserve(n);
        n_ = n;
    }

  private:
    static constexpr size_t kHuge = (size_t)2 << 20;
    static size_t bytes() { return (kRows * sizeof(T) + kHuge - 1) & ~(kHuge - 1); }
    static T* map() {
        const size_t sz = bytes();
        char* base = static_cast<char*>(mmap(nullptr, sz + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
        if (base == MAP_FAILED) throw std::bad_alloc();
        char* al = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(base) + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
        if (al > base) munmap(base, (size_t)(al - base));                       // keep [al, al + sz)
        if (base + sz + kHuge > al + sz) munmap(al + sz, (size_t)(base + sz + kHuge - (al + sz)));
        (void)madvise(al, sz, MADV_HUGEPAGE);
        return reinterpret_cast<T*>(al);
    }
    static void unmap(T* c) { munmap(c, bytes()); }
    std::vector<T*> chunks_;
    size_t n_ = 0;
};
}  // namespace casim

namespace casim {
// A candidate range of a multi-device sweep (multi.hip) runs the pipeline in three calls
// on its own device, the host composing the ranges between them:
//   SP_PROBE    the probe at the guesses from guess_base (lastIndex + the pods to move of
//               every earlier sensitive candidate of the whole call); out: adv = the range's
//               advance as the probe saw it (the sum k_sweep_est would take)
//   SP_MAP      windows centred from est_base (the previous ranges' probe advances), the
//               tables, the chunk walks and k_walk_map; out: map[] (64 lastIndex-out values
//               by class of the first row, the row's fit points, the class mode), S
//   SP_RESOLVE  the walk from the true input (*last_index), the table gather and the exact
//               pass — the tail of a normal call, host walk included, so it is always exact
// Device state (probe outputs, guesses, tables, chunk maps) stays in the mirror's sweep
// scratch between the calls; nothing else may use the mirror meanwhile.
enum { SP_FULL = 0, SP_PROBE = CA_SWEEP_PHASE_PROBE, SP_MAP = CA_SWEEP_PHASE_MAP, SP_RESOLVE = CA_SWEEP_PHASE_RESOLVE };
// the map record k_walk_map writes (sweep.hip): 64 lastIndex-out values by class, then the
// first row's SWEEP_FPW fit points, then the class mode flag
constexpr int SWEEP_FPW = 65;
constexpr int SWEEP_MAP_HEAD = 64;                     // offset of the fit points
constexpr int SWEEP_MAP_MODE = 64 + SWEEP_FPW;         // offset of the mode flag
constexpr int SWEEP_MAP_INTS = 64 + SWEEP_FPW + 1;
static_assert(SWEEP_MAP_INTS == CA_SWEEP_MAP_INTS, "casim.h map record size");
// the public record (casim.h ca_sweep_phase): kind, guess_base (PROBE in), est_base (MAP
// in), adv / succ (PROBE out), n_sensitive, map_ran / map_ok / map (MAP out)
using SweepPhase = ca_sweep_phase;

int64_t removal_plan_sensitive_pods(const ca_removal_plan* p);
bool removal_plan_phase_ok(const ca_removal_plan* p);             // no scope cut in the range
int32_t sweep_fp_class(const int32_t* fp, int32_t n, int32_t L);  // class of L in a row's fit points
int removal_plan_run_phase(ca_removal_plan* p, int32_t* hints, int32_t* last_index, ca_removal_result* results,
                           int32_t* out_dest, SweepPhase* ph);
}  // namespace casim

struct ca_mirror {
    int32_t device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;

    std::vector<casim::NodeRow> nodes;
    casim::ChunkVec<casim::PodRow> pods;             // by pod id (never moved)
    std::vector<ca_selector_term> terms;
    std::vector<ca_selector_req> reqs;
    std::vector<int32_t> pf_names;
    std::vector<casim::JournalEntry> journal;
    std::vector<casim::NodeRow> removed_nodes;   // rows of journaled RemoveNode ops (J_REMOVE_NODE.slot)
    int32_t depth = 0;
    int64_t n_scope_blockers = 0;          // pods in the snapshot with CA_POD_REQUIRED_ANTI_AFFINITY

    // device rows
    casim::DevBuf d_hot, d_ext, d_static;
    size_t d_cap = 0;                      // rows allocated
    size_t d_rows = 0;                     // rows valid on device
    std::vector<int32_t> dirty_rows;       // rows whose dynamic part changed
    std::vector<uint8_t> dirty_flag;
    bool static_dirty = true;              // static/ext columns need a full upload
    bool all_dirty = true;

    // device pod table (mirror pods), appended lazily
    casim::DevPodTable d_pods;
    size_t d_pods_synced = 0;              // pods whose records are on device
    size_t d_terms_synced = 0;

    // scratch
    casim::DevBuf d_scratch0, d_scratch1, d_scratch2, d_scratch3;
    casim::DevBuf d_mask;                  // per-node match mask
    std::vector<uint8_t> h_scratch;
    casim::Stats sweep_stats;
    casim::PlanStats plan;
    casim::SweepScratch sw;
    casim::FilterScratch fo;
    casim::PlanChainScratch pc;
    casim::RowStage rs;
    casim::HostBuf podset_stage;           // ca_podset_create: the records' page-locked staging
    // resident HintingSimulator hints (hints.go:29-72): node per mirror pod, -1 = none
    casim::DevBuf d_pod_hints;
    size_t d_hints_n = 0;
    int ensure_pod_hints();                // grow to pods.size(), new entries -1
    int64_t n_ext_pods = 0;                // pods stored with host ports / extended requests
    int64_t n_eph_pods = 0;                // pods stored with ephemeral-storage requests
    int64_t n_oos_pods = 0;                // pods stored with CA_POD_OUT_OF_SCOPE (never decremented:
                                           // 0 lets the sweep's scope cut skip the per-pod check)

    int remap_hints_removed(int32_t pos, int32_t code, bool restore);   // resident hints around a RemoveNode
    int32_t removals = 0;                  // RemoveNode calls so far: hint codes of removed nodes
    int sync_nodes();                      // push dirty rows to the device
    int sync_pods();                       // push new pod records to the device
    void mark_dirty(int32_t node);
    void node_apply(int32_t node, const ca_pod_spec& p, int sign);
    void add_pod_to_node(int32_t pod, int32_t node);
    int32_t store_pod(const ca_pod_table* t, int32_t idx, int32_t node);
    void reserve_more(size_t n_pods_add, size_t n_journal_add);    // geometric growth before a batch
    // store_pod + add_pod_to_node of pod idx[k] on node[k] for every k with node[k] >= 0, in
    // order (ids in out_id, -1 for the others); large batches on a few host threads
    // device_rows: the caller's kernel already wrote the placed nodes' free resources to
    // d_hot (FilterOutSchedulable's bitmap walk), so they stay clean where fill_hot agrees
    void add_placed_batch(const ca_pod_table* t, const int32_t* idx, const int32_t* node, int32_t n,
                          int32_t* out_id, bool device_rows = false, bool known_plain = false);
    int32_t store_moved_copy(int32_t pod);  // the copy findPlaceFor schedules (cluster.go:235-240)
    // the planner's committed moves, candidate by candidate: RemovePod of each moved pod,
    // then the copies (ids pods.size() + t, t-th move) AddPod'ed on their nodes; large
    // batches on the worker pool, split by node (planner.hip).  CA_EDEVICE if mv[t].new_pod
    // is not the id the copy gets.
    int replay_moves(const ca_plan_move* mv, int32_t nm);
    void journal_push(int32_t kind, int32_t node, int32_t pod, int32_t slot, const uint64_t* ports);
    void fill_hot(int32_t i, casim::NodeHot& h) const;
    void fill_ext(int32_t i, casim::NodeExt& e) const;
    void fill_static(int32_t i, casim::NodeStatic& s) const;
};

struct ca_podset {
    ca_mirror* m = nullptr;
    casim::DevPodTable t;
    int32_t n_host = 0;                // pods in the set
    bool any_oos = false;              // some pod carries CA_POD_OUT_OF_SCOPE (no host copy of the records)
    bool any_refs = false;             // some pod references selector terms or PreFilter names
    // Score classes: pods with equal (score_milli_cpu, score_memory) — the only inputs of
    // calculatePodScore (binpacking_estimator.go:164-193) — share a class, numbered in
    // first-occurrence order.  d_cls[pod] = class, d_cls_sc[c] = {score_milli_cpu,
    // score_memory}.  Used by the Estimate bucket sort (estimate.hip).
    int32_t n_cls = 0;
    casim::DevBuf d_cls, d_cls_sc;
    casim::DevBuf d_cls_rep;           // a pod of each class (its first in the set)
    std::vector<int64_t> h_req;        // per pod: request cpu, memory (compact copies for plan creation)
    std::vector<uint8_t> h_pflags;     // per pod: 1 host ports, 2 extended-resource requests
    bool any_ports = false, any_scalar = false;
    std::vector<int32_t> h_cls;        // host copies: class per pod, {cpu, memory} per class
    std::vector<int64_t> h_cls_sc;
    // every class's pods carry identical records apart from their controller
    // (similar_class): interchangeable for the FFD chain, so Estimate can run the chain on
    // the stable class order while Go's sort.Slice order of their ids is computed beside it
    // — provided no two classes of a group tie on their float64 score against the group's
    // template (checked per plan: ca_estimate_plan::decouple_ok)
    bool cls_uniform = false;
};
