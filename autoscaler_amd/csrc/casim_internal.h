// casim_internal.h — device data layout of the ClusterSnapshot mirror and the
// pod records, shared by the HIP translation units of libcasim.so.
//
// Layout in HBM:
//   NodeHot   [cap]   32 B  free cpu/mem/eph (alloc - requested, int64 wrapping),
//                           free pod slots (int32), flags — the only row every
//                           predicate evaluation reads.
//   NodeExt   [cap]   80 B  free scalar resources + used host-port bitset; read only
//                           when the pod or the node has scalars / ports.
//   NodeStatic[cap]   96 B  taint classes, label pairs/keys, Gt/Lt ints, name id;
//                           read only when the pod carries a toleration-relevant
//                           taint, a selector, or a nodeName.
//   PodHot    [pods]  32 B  requests + flags of a pod record.
//   ca_pod_spec       full record for the rare fields (tolerations, selector...).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include <string>
#include <cstdlib>
#include <functional>
#include "../../include/casim.h"

namespace casim {

// NodeHot.flags
enum : uint32_t {
    NF_UNSCHED = 0x1u,     // Spec.Unschedulable
    NF_TAINTS  = 0x2u,     // node has NoSchedule/NoExecute taints
    NF_PORTS   = 0x4u,     // node has used host ports (may be stale-high)
    NF_SCALAR  = 0x8u,     // node allocatable has scalar resources
    NF_VALID   = 0x10u,    // row holds a node
    NF_OUT_OF_SCOPE = 0x20u, // template row: its pods include a required-anti-affinity pod
};

// PodHot.flags (device-side copy of the CA_POD_* bits plus derived bits)
enum : uint32_t {
    PF_HAS_SCALAR_KEYS = CA_POD_HAS_SCALAR_KEYS,
    PF_NONTPU_SCALAR   = CA_POD_HAS_NONTPU_SCALAR_KEYS,
    PF_TOL_UNSCHED     = CA_POD_TOLERATES_UNSCHED,
    PF_AFFINITY        = CA_POD_AFFINITY_FILTER,
    PF_PREFILTER_FAIL  = CA_POD_PREFILTER_FAIL,
    PF_PREFILTER_NAMES = CA_POD_PREFILTER_NAMES,
    PF_DAEMONSET       = CA_POD_DAEMONSET,
    PF_HOSTNAME_DEP    = CA_POD_HOSTNAME_DEPENDENT,
    PF_OUT_OF_SCOPE    = CA_POD_OUT_OF_SCOPE,
    PF_ANTI_AFFINITY   = CA_POD_REQUIRED_ANTI_AFFINITY,
    PF_SCALAR_REQ      = 0x1000u,  // some req_scalar[i] != 0
    PF_PORTS           = 0x2000u,  // port_conflict or port_use non-empty
    PF_NODE_NAME       = 0x4000u,  // node_name_id != -1
    PF_ALL_ZERO        = 0x8000u,  // cpu == mem == eph == 0 && !HAS_SCALAR_KEYS (fit.go:267-272)
    PF_TAINT_MASK_ALL  = 0x10000u, // tolerates every taint class (no taint check needed)
    PF_MOVED_ALL_ZERO  = 0x20000u, // PF_ALL_ZERO after tpu.ClearTPURequests
    PF_MOVED_SCALAR_REQ = 0x40000u,// PF_SCALAR_REQ after tpu.ClearTPURequests
};

struct alignas(16) NodeHot {
    int64_t cpu, mem, eph;
    int32_t pods;
    uint32_t flags;
};
static_assert(sizeof(NodeHot) == 32, "NodeHot must be 32 B");

struct alignas(16) NodeExt {
    int64_t scalar[CA_MAX_SCALAR];
    uint64_t ports[CA_PORT_WORDS];
};
static_assert(sizeof(NodeExt) == 80, "NodeExt must be 80 B");

struct alignas(16) NodeStatic {
    uint64_t taints;
    uint64_t labels[CA_LABEL_WORDS];
    uint64_t keys;
    int64_t ints[CA_MAX_INT_KEYS];
    uint32_t int_valid;
    int32_t name_id;
    uint64_t pad;
};
static_assert(sizeof(NodeStatic) == 96, "NodeStatic must be 96 B");

struct alignas(16) PodHot {
    int64_t cpu, mem, eph;
    uint32_t flags;
    int32_t spec;      // index of the full record
};
static_assert(sizeof(PodHot) == 32, "PodHot must be 32 B");

// Wrapping int64 arithmetic (Go int64 semantics).
__host__ __device__ inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__host__ __device__ inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

// Derived device flags of a pod record.
inline uint32_t pod_dev_flags(const ca_pod_spec& p) {
    uint32_t f = p.flags & 0xFFFu;
    for (int i = 0; i < CA_MAX_SCALAR; i++) if (p.req_scalar[i] != 0) f |= PF_SCALAR_REQ;
    for (int w = 0; w < CA_PORT_WORDS; w++) if (p.port_conflict[w] | p.port_use[w]) f |= PF_PORTS;
    if (p.node_name_id != -1) f |= PF_NODE_NAME;
    if (p.req_milli_cpu == 0 && p.req_memory == 0 && p.req_ephemeral == 0 && !(p.flags & CA_POD_HAS_SCALAR_KEYS))
        f |= PF_ALL_ZERO;
    if (p.tolerated_taints == ~0ull) f |= PF_TAINT_MASK_ALL;
    bool moved_scalar = false;
    for (int i = 0; i < CA_MAX_SCALAR; i++)
        if (p.req_scalar[i] != 0 && !((p.tpu_scalar_mask >> i) & 1u)) moved_scalar = true;
    if (moved_scalar) f |= PF_MOVED_SCALAR_REQ;
    if (p.req_milli_cpu == 0 && p.req_memory == 0 && p.req_ephemeral == 0 &&
        !(p.flags & CA_POD_HAS_NONTPU_SCALAR_KEYS))
        f |= PF_MOVED_ALL_ZERO;
    return f;
}

// ---------------------------------------------------------------------------
// Static (node-attribute) part of the filter chain: NodeUnschedulable, NodeName,
// TaintToleration, NodeAffinity — SF/runtime/framework.go:727-749 order.
// Returns the failing plugin (CA_PLUGIN_*) or CA_PLUGIN_NONE.
// ---------------------------------------------------------------------------
// n.ints[k] without a dynamic register-array index (which would put the row in scratch)
__host__ __device__ inline int64_t int_label_at(const NodeStatic& n, int32_t k) {
    static_assert(CA_MAX_INT_KEYS == 4, "int_label_at");
    const int64_t a = (k & 1) ? n.ints[1] : n.ints[0];
    const int64_t b = (k & 1) ? n.ints[3] : n.ints[2];
    return (k & 2) ? b : a;
}

__host__ __device__ inline bool dev_req_matches(const ca_selector_req& r, const NodeStatic& n) {
    switch (r.op) {
    case CA_OP_IN: {
        uint64_t a = 0;
        for (int w = 0; w < CA_LABEL_WORDS; w++) a |= n.labels[w] & r.pairs[w];
        return a != 0;
    }
    case CA_OP_NOTIN: {
        uint64_t a = 0;
        for (int w = 0; w < CA_LABEL_WORDS; w++) a |= n.labels[w] & r.pairs[w];
        return a == 0;
    }
    case CA_OP_EXISTS: return (n.keys >> r.key) & 1u;
    case CA_OP_DOESNOTEXIST: return !((n.keys >> r.key) & 1u);
    case CA_OP_GT: return ((n.int_valid >> r.key) & 1u) && int_label_at(n, r.key) > r.bound;
    case CA_OP_LT: return ((n.int_valid >> r.key) & 1u) && int_label_at(n, r.key) < r.bound;
    case CA_OP_FIELD_EQ: return n.name_id == r.key;
    case CA_OP_FIELD_NE: return n.name_id != r.key;
    default: return false;
    }
}

__host__ __device__ inline bool dev_affinity_matches(const ca_pod_spec& p, const ca_selector_term* terms,
                                                     const ca_selector_req* reqs, const NodeStatic& n) {
    for (int w = 0; w < CA_LABEL_WORDS; w++)
        if ((n.labels[w] & p.node_selector[w]) != p.node_selector[w]) return false;
    if (p.aff_term_count < 0) return true;
    for (int k = 0; k < p.aff_term_count; k++) {
        const ca_selector_term tm = terms[p.aff_term_first + k];
        bool ok = true;
        for (int r = 0; r < tm.count && ok; r++) ok = dev_req_matches(reqs[tm.first + r], n);
        if (ok) return true;
    }
    return false;
}

// static part; `unsched` applies NodeUnschedulable (CheckPredicates path; the
// FitsAnyNode scan skips unschedulable nodes before filtering).
__host__ __device__ inline int dev_static_filters(const ca_pod_spec& p, uint32_t pflags,
                                                  const ca_selector_term* terms, const ca_selector_req* reqs,
                                                  const NodeStatic& n, bool node_unsched) {
    if (node_unsched && !(pflags & PF_TOL_UNSCHED)) return CA_PLUGIN_NODE_UNSCHEDULABLE;
    if ((pflags & PF_NODE_NAME) && p.node_name_id != n.name_id) return CA_PLUGIN_NODE_NAME;
    if (n.taints & ~p.tolerated_taints) return CA_PLUGIN_TAINT_TOLERATION;
    if ((pflags & PF_AFFINITY) && !dev_affinity_matches(p, terms, reqs, n)) return CA_PLUGIN_NODE_AFFINITY;
    return CA_PLUGIN_NONE;
}

// NodeResourcesFit reasons (fit.go:253-331) for the dynamic part; ports first
// (NodePorts precedes NodeResourcesFit in the default profile).
__host__ __device__ inline uint32_t dev_fit_reasons(int64_t pcpu, int64_t pmem, int64_t peph, uint32_t pflags,
                                                    const int64_t* preq_scalar,
                                                    int64_t fcpu, int64_t fmem, int64_t feph, int32_t fpods,
                                                    const int64_t* fscalar) {
    uint32_t reasons = 0;
    if (fpods < 1) reasons |= CA_REASON_TOO_MANY_PODS;
    if (pflags & PF_ALL_ZERO) return reasons;
    if (pcpu > fcpu) reasons |= CA_REASON_INSUFF_CPU;
    if (pmem > fmem) reasons |= CA_REASON_INSUFF_MEMORY;
    if (peph > feph) reasons |= CA_REASON_INSUFF_EPHEMERAL;
    if (pflags & PF_SCALAR_REQ) {
        for (int i = 0; i < CA_MAX_SCALAR; i++)
            if (preq_scalar[i] != 0 && preq_scalar[i] > fscalar[i]) reasons |= CA_REASON_INSUFF_SCALAR0 << i;
    }
    return reasons;
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------
#define CA_HIP_CHECK(expr)                                                         \
    do {                                                                           \
        hipError_t _e = (expr);                                                    \
        if (_e != hipSuccess) {                                                    \
            casim::set_last_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
            return CA_EDEVICE;                                                     \
        }                                                                          \
    } while (0)

void set_last_error(const std::string& s);
// Fault-injection / trace hooks for tests and diagnosis scripts: the variable is read only
// when CASIM_TEST_HOOKS is set as well, so one stray variable cannot change a production
// call's behaviour.
inline const char* test_hook_env(const char* name) {
    return getenv("CASIM_TEST_HOOKS") ? getenv(name) : nullptr;
}

// Tuning / diagnostic switches of the Estimate path (CASIM_GO_DECOUPLE, CASIM_PUB_SERIAL,
// ...): read only when CASIM_TEST_HOOKS or CASIM_KNOBS is set in the process (checked once),
// so a production step reads no environment — each getenv is a scan of it, a dozen per
// step on the launch path.
inline bool knobs_enabled() {
    static const bool on = getenv("CASIM_TEST_HOOKS") != nullptr || getenv("CASIM_KNOBS") != nullptr;
    return on;
}
inline const char* knob_env(const char* name) { return knobs_enabled() ? getenv(name) : nullptr; }

const std::string& last_error();

// hipFuncAttributeMaxDynamicSharedMemorySize of a kernel, raised to `bytes` at most once
// per (device, kernel) and size: the call costs tens of microseconds, too much per launch.
int ensure_dyn_lds(const void* kernel, size_t bytes);

// A growable device buffer.
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    int dev = -1;               // device of ptr (the allocation cache is per device)
    int reserve(size_t need);   // grows (content not preserved)
    int reserve_keep(size_t need, hipStream_t st);  // grows, preserving content
    void release();
    ~DevBuf() { release(); }
    template <class T> T* as() const { return static_cast<T*>(ptr); }
};

// A growable page-locked host buffer (DMA target for results / tables).
struct HostBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    int reserve(size_t need);   // grows (content not preserved)
    void release();
    ~HostBuf() { release(); }
    template <class T> T* as() const { return static_cast<T*>(ptr); }
};

// Convert int64 allowed pods - count into the int32 free-slot column.
inline int32_t clamp_i32(int64_t v) {
    if (v > INT32_MAX) return INT32_MAX;
    if (v < INT32_MIN) return INT32_MIN;
    return (int32_t)v;
}

// Host worker threads kept for the library's parallel host passes (plan creation, the
// placement replay): fn(0 .. T-1), fn(0) on the caller, T <= 8.  Spawning the threads per
// call cost ~0.15 ms; parked workers wake in a few microseconds.  One region at a time
// (callers on several host threads queue); fn must not start a region itself.
void parallel_run(int32_t T, const std::function<void(int32_t)>& fn);

}  // namespace casim
