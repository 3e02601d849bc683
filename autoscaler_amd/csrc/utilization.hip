// utilization.hip — scale-down eligibility.
//
// utilization.Calculate (CA/simulator/utilization/info.go:48-127) for every node of a
// device-resident node/pod table, and the FindEmptyNodesToRemove verdict
// (CA/simulator/cluster.go:187-202) from the host's per-pod drain flags.
//
// The work is a segmented integer reduction over each node's pods followed by at most
// three float64 divisions: HBM-bound, no MFMA.  A 16-lane segment owns one node (four
// nodes per wavefront: C5 nodes hold ~20 pods, so a full wave per node left two thirds of
// its lanes idle and needed twice the waves); its lanes stride over the node's pod records
// (48 B each, consecutive per node, so a segment reads one contiguous span), accumulate
// six int64 sums (requests and the DaemonSet/mirror share for cpu, memory, gpu) and two
// flag bits, and reduce them with segment shuffles.  The segment's first lane finishes the
// node and writes its 48 B Info row.  16 nodes per 256-thread workgroup; 15 000 nodes
// (C5) launch 938 workgroups, 3 750 wavefronts: one resident round on 256 CUs.
#include "casim_internal.h"

#include <algorithm>
#include <cstring>
#include <vector>


struct ca_util_table {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_added = nullptr;       // the staging copy of the last set_added is done
    bool added_in_flight = false;
    int32_t n_nodes = 0, n_pods = 0;
    casim::DevBuf nodes, pod_off, pods, info;
    // pods added since the rows were set (ca_util_table_set_added), in the caller's order:
    // [node n_added][pad][pods n_added] in device memory, summed per node by atomics in
    // ca_util_calculate (k_added_sums) into acc, which the node kernel reads and clears
    int32_t n_added = 0;
    casim::DevBuf added;
    casim::HostBuf h_added;              // staging for pageable caller arrays
    casim::DevBuf acc;                   // AddedSum per node, all zero between calls
};

namespace {

// byte offset of the added pods behind their node indices in ca_util_table::added
inline size_t added_pods_at(int32_t n) { return ((sizeof(int32_t) * (size_t)std::max(n, 1)) + 63) & ~(size_t)63; }

// the added pods' sums of one node (k_added_sums), consumed and cleared by k_node_utilization
struct AddedSum {
    unsigned long long req[3], dsm[3];       // int64 sums (two's complement adds)
    int32_t drain, pad;
    int64_t pad2;
};
static_assert(sizeof(AddedSum) == 64, "AddedSum");

constexpr int kLanes = 16;                                    // lanes per node (C5: ~20 pods/node)
constexpr int kThreads = 256;
constexpr int64_t kNsPerS = 1000000000LL;
constexpr int64_t kLongTerminatingExtraNs = 30 * kNsPerS;   // drain.go:34 PodLongTerminatingExtraThreshold

// calculateUtilizationOfResource's final ratio (info.go:126): float64 / float64 of the
// MilliValue difference, one correctly rounded IEEE division (built -ffp-contract=off).
__device__ inline double util_ratio(int64_t pods, int64_t alloc, int64_t dsm) {
    return (double)pods / (double)(alloc - dsm);
}

__device__ inline int64_t seg_sum(int64_t v) {                // within a kLanes-lane segment
    for (int o = kLanes / 2; o; o >>= 1) v += __shfl_xor(v, o, kLanes);
    return v;
}

// one pod's share of its node's sums (info.go:100-124)
__device__ inline void pod_share(const ca_util_pod& p, int32_t skip_ds, int32_t skip_mirror, int64_t now_ns,
                                 int64_t (&req)[3], int64_t (&dsm)[3], int& drain) {
    drain |= (int)(p.flags & (CA_UPOD_MOVABLE | CA_UPOD_BLOCKING));
    const bool factored = (skip_ds && (p.flags & CA_UPOD_DAEMONSET)) || (skip_mirror && (p.flags & CA_UPOD_MIRROR));
    // drain.IsPodLongTerminating (utils/drain/drain.go:294-306): deleted, and deletion +
    // grace + 30 s strictly before now
    const bool long_term = !factored && (p.flags & CA_UPOD_DELETED) &&
                           p.deletion_ns + p.grace_s * kNsPerS + kLongTerminatingExtraNs < now_ns;
    for (int r = 0; r < 3; r++) {
        if (factored) dsm[r] += p.req_milli[r];
        else if (!long_term) req[r] += p.req_milli[r];
    }
}

// The pods added since the rows were set, one thread each, into their nodes' sums
// (integer sums and flag ORs: the order of a node's pods does not matter).
__global__ __launch_bounds__(kThreads) void k_added_sums(const int32_t* __restrict__ add_node,
                                                         const ca_util_pod* __restrict__ add_pods, int32_t n,
                                                         int32_t skip_ds, int32_t skip_mirror, int64_t now_ns,
                                                         AddedSum* __restrict__ acc) {
    const int32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const int32_t x = add_node[k];
    int64_t req[3] = {0, 0, 0}, dsm[3] = {0, 0, 0};
    int drain = 0;
    pod_share(add_pods[k], skip_ds, skip_mirror, now_ns, req, dsm, drain);
    AddedSum& a = acc[x];
    for (int r = 0; r < 3; r++) {
        if (req[r]) atomicAdd(&a.req[r], (unsigned long long)req[r]);
        if (dsm[r]) atomicAdd(&a.dsm[r], (unsigned long long)dsm[r]);
    }
    if (drain) atomicOr(&a.drain, drain);
}

__global__ __launch_bounds__(kThreads) void k_node_utilization(
    const ca_util_node* __restrict__ nodes, const int32_t* __restrict__ pod_off,
    const ca_util_pod* __restrict__ pods, int32_t n_nodes, int32_t skip_ds, int32_t skip_mirror,
    int64_t now_ns, ca_util_info* __restrict__ out, AddedSum* __restrict__ acc, ca_util_info* __restrict__ out_host) {
    const int sub = threadIdx.x & (kLanes - 1);
    const int32_t node = blockIdx.x * (kThreads / kLanes) + (int32_t)(threadIdx.x / kLanes);
    if (node >= n_nodes) return;                                  // whole segments only
    const int32_t b = pod_off[node], e = pod_off[node + 1];
    const ca_util_node nd = nodes[node];                          // in flight during the pod loop
    int64_t req[3] = {0, 0, 0}, dsm[3] = {0, 0, 0};
    int drain = 0;
    for (int32_t k = b + sub; k < e; k += kLanes)                 // info.go:100-124
        pod_share(pods[k], skip_ds, skip_mirror, now_ns, req, dsm, drain);
    for (int r = 0; r < 3; r++) {
        req[r] = seg_sum(req[r]);
        dsm[r] = seg_sum(dsm[r]);
    }
    for (int o = kLanes / 2; o; o >>= 1) drain |= __shfl_xor(drain, o, kLanes);
    if (sub != 0) return;
    if (acc) {                                                    // the added pods' sums, then cleared
        AddedSum a = acc[node];
        for (int r = 0; r < 3; r++) { req[r] += (int64_t)a.req[r]; dsm[r] += (int64_t)a.dsm[r]; }
        drain |= a.drain;
        if (a.drain | a.req[0] | a.req[1] | a.req[2] | a.dsm[0] | a.dsm[1] | a.dsm[2]) acc[node] = AddedSum{};
    }

    ca_util_info o;
    o.cpu = o.mem = o.gpu = o.utilization = 0.0;
    o.resource = CA_UTIL_CPU;
    o.status = CA_UTIL_OK;
    o._pad = 0;
    o.empty = drain == 0;                                         // cluster.go:197-199
    if (nd.flags & CA_UNODE_GPU_CONFIG) {                         // info.go:49-58
        o.resource = CA_UTIL_GPU;
        if ((nd.flags & CA_UNODE_HAS_GPU) && nd.alloc_milli[2] != 0) {
            o.gpu = util_ratio(req[2], nd.alloc_milli[2], dsm[2]);
            o.utilization = o.gpu;
        }                                                         // unready GPU: Info{Gpu 0, Util 0}, nil
    } else if (!(nd.flags & CA_UNODE_HAS_CPU)) {                  // info.go:88-94 -> Info{}, err
        o.status = CA_UTIL_NO_CPU;
    } else if (nd.alloc_milli[0] == 0) {
        o.status = CA_UTIL_ZERO_CPU;
    } else if (!(nd.flags & CA_UNODE_HAS_MEM)) {
        o.status = CA_UTIL_NO_MEM;
    } else if (nd.alloc_milli[1] == 0) {
        o.status = CA_UTIL_ZERO_MEM;
    } else {                                                      // info.go:61-80
        o.cpu = util_ratio(req[0], nd.alloc_milli[0], dsm[0]);
        o.mem = util_ratio(req[1], nd.alloc_milli[1], dsm[1]);
        if (o.cpu > o.mem) { o.resource = CA_UTIL_CPU; o.utilization = o.cpu; }
        else               { o.resource = CA_UTIL_MEM; o.utilization = o.mem; }
    }
    out[node] = o;
    if (out_host) out_host[node] = o;                             // page-locked caller rows (zero-copy)
}

}  // namespace

extern "C" {

int ca_util_table_create(int32_t device, const ca_util_node* nodes, int32_t n_nodes,
                         const int32_t* pod_off, const ca_util_pod* pods, ca_util_table** out) {
    if (!out || n_nodes < 0 || (n_nodes > 0 && (!nodes || !pod_off))) return CA_EINVAL;
    *out = nullptr;
    const int32_t n_pods = n_nodes > 0 ? pod_off[n_nodes] : 0;
    if (n_pods < 0 || (n_pods > 0 && !pods) || (n_nodes > 0 && pod_off[0] != 0)) return CA_EINVAL;
    for (int32_t i = 0; i < n_nodes; i++)                         // the kernel trusts the offsets
        if (pod_off[i + 1] < pod_off[i]) return CA_EINVAL;
    auto* t = new ca_util_table();
    t->device = device;
    t->n_nodes = n_nodes;
    t->n_pods = n_pods;
    auto fail = [&](int st) { ca_util_table_destroy(t); return st; };
    if (hipSetDevice(device) != hipSuccess) return fail(CA_EDEVICE);
    if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&t->ev0) != hipSuccess || hipEventCreate(&t->ev1) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_added, hipEventDisableTiming) != hipSuccess)
        return fail(CA_EDEVICE);
    int st;
    if ((st = t->nodes.reserve(sizeof(ca_util_node) * (size_t)n_nodes + 1)) ||
        (st = t->pod_off.reserve(sizeof(int32_t) * ((size_t)n_nodes + 1))) ||
        (st = t->pods.reserve(sizeof(ca_util_pod) * (size_t)n_pods + 1)) ||
        (st = t->info.reserve(sizeof(ca_util_info) * (size_t)n_nodes + 1)) ||
        (st = t->acc.reserve(sizeof(AddedSum) * ((size_t)n_nodes + 1))))
        return fail(st);
    if (hipMemsetAsync(t->acc.ptr, 0, sizeof(AddedSum) * ((size_t)n_nodes + 1), t->stream) != hipSuccess)
        return fail(CA_EDEVICE);
    if (n_nodes > 0) {
        if (hipMemcpyAsync(t->nodes.ptr, nodes, sizeof(ca_util_node) * n_nodes, hipMemcpyHostToDevice,
                           t->stream) != hipSuccess ||
            hipMemcpyAsync(t->pod_off.ptr, pod_off, sizeof(int32_t) * (n_nodes + 1), hipMemcpyHostToDevice,
                           t->stream) != hipSuccess)
            return fail(CA_EDEVICE);
        if (n_pods > 0 && hipMemcpyAsync(t->pods.ptr, pods, sizeof(ca_util_pod) * n_pods,
                                         hipMemcpyHostToDevice, t->stream) != hipSuccess)
            return fail(CA_EDEVICE);
    }
    if (hipStreamSynchronize(t->stream) != hipSuccess) return fail(CA_EDEVICE);
    *out = t;
    return CA_OK;
}

int ca_util_table_update(ca_util_table* t, const ca_util_node* nodes, int32_t n_nodes, const int32_t* pod_off,
                         const ca_util_pod* pods) {
    if (!t || n_nodes < 0 || (n_nodes > 0 && (!nodes || !pod_off))) return CA_EINVAL;
    const int32_t n_pods = n_nodes > 0 ? pod_off[n_nodes] : 0;
    if (n_pods < 0 || (n_pods > 0 && !pods) || (n_nodes > 0 && pod_off[0] != 0)) return CA_EINVAL;
    for (int32_t i = 0; i < n_nodes; i++)
        if (pod_off[i + 1] < pod_off[i]) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(t->device));
    int st;
    if ((st = t->nodes.reserve(sizeof(ca_util_node) * (size_t)n_nodes + 1)) ||
        (st = t->pod_off.reserve(sizeof(int32_t) * ((size_t)n_nodes + 1))) ||
        (st = t->pods.reserve(sizeof(ca_util_pod) * (size_t)n_pods + 1)) ||
        (st = t->info.reserve(sizeof(ca_util_info) * (size_t)n_nodes + 1)))
        return st;
    if (t->added_in_flight) {                                  // (a set_added copy may still read)
        CA_HIP_CHECK(hipEventSynchronize(t->ev_added));
        t->added_in_flight = false;
    }
    if ((st = t->acc.reserve_keep(sizeof(AddedSum) * ((size_t)n_nodes + 1), t->stream)) != CA_OK) return st;
    // (a table that grows gets its new sums zeroed; the old ones are zero between calls)
    CA_HIP_CHECK(hipMemsetAsync(t->acc.ptr, 0, sizeof(AddedSum) * ((size_t)n_nodes + 1), t->stream));
    if (n_nodes > 0) {
        CA_HIP_CHECK(hipMemcpyAsync(t->nodes.ptr, nodes, sizeof(ca_util_node) * n_nodes, hipMemcpyHostToDevice,
                                    t->stream));
        CA_HIP_CHECK(hipMemcpyAsync(t->pod_off.ptr, pod_off, sizeof(int32_t) * (n_nodes + 1), hipMemcpyHostToDevice,
                                    t->stream));
        if (n_pods > 0)
            CA_HIP_CHECK(hipMemcpyAsync(t->pods.ptr, pods, sizeof(ca_util_pod) * n_pods, hipMemcpyHostToDevice,
                                        t->stream));
    }
    CA_HIP_CHECK(hipStreamSynchronize(t->stream));
    t->n_nodes = n_nodes;
    t->n_pods = n_pods;
    t->n_added = 0;
    return CA_OK;
}

int ca_util_table_set_added(ca_util_table* t, const int32_t* node, const ca_util_pod* pods, int32_t n) {
    if (!t || n < 0 || (n > 0 && (!node || !pods))) return CA_EINVAL;
    for (int32_t k = 0; k < n; k++)                            // the kernel trusts the indices
        if ((uint32_t)node[k] >= (uint32_t)t->n_nodes) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(t->device));
    if (t->added_in_flight) {                                  // the staging buffer is reused
        CA_HIP_CHECK(hipEventSynchronize(t->ev_added));
        t->added_in_flight = false;
    }
    t->n_added = 0;
    if (n == 0) return CA_OK;
    // one DMA per array into device memory (no sort: the sums are order-free); page-locked
    // caller arrays (ca_host_alloc) are copied in place, others through page-locked staging
    const size_t at = added_pods_at(n);
    const size_t bytes = at + sizeof(ca_util_pod) * (size_t)n;
    int st;
    if ((st = t->added.reserve(bytes)) != CA_OK) return st;
    auto pinned = [](const void* h) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, h) == hipSuccess && a.type == hipMemoryTypeHost) return true;
        (void)hipGetLastError();
        return false;
    };
    const void* src_node = node;
    const void* src_pods = pods;
    if (!pinned(node) || !pinned(pods)) {
        if ((st = t->h_added.reserve(bytes)) != CA_OK) return st;
        std::memcpy(t->h_added.ptr, node, sizeof(int32_t) * (size_t)n);
        std::memcpy(t->h_added.as<unsigned char>() + at, pods, sizeof(ca_util_pod) * (size_t)n);
        src_node = t->h_added.ptr;
        src_pods = t->h_added.as<unsigned char>() + at;
    }
    // stream-ordered before the next calculate; the next set_added waits for the copies
    CA_HIP_CHECK(hipMemcpyAsync(t->added.ptr, src_node, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, t->stream));
    CA_HIP_CHECK(hipMemcpyAsync(t->added.as<unsigned char>() + at, src_pods, sizeof(ca_util_pod) * (size_t)n,
                                hipMemcpyHostToDevice, t->stream));
    CA_HIP_CHECK(hipEventRecord(t->ev_added, t->stream));
    t->added_in_flight = true;
    t->n_added = n;
    return CA_OK;
}

int ca_util_table_destroy(ca_util_table* t) {
    if (!t) return CA_EINVAL;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    t->nodes.release();
    t->pod_off.release();
    t->pods.release();
    t->info.release();
    t->added.release();
    t->h_added.release();
    t->acc.release();
    if (t->ev0) (void)hipEventDestroy(t->ev0);
    if (t->ev1) (void)hipEventDestroy(t->ev1);
    if (t->ev_added) (void)hipEventDestroy(t->ev_added);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
    return CA_OK;
}

int ca_util_calculate(ca_util_table* t, int32_t skip_daemonset_pods, int32_t skip_mirror_pods,
                      int64_t now_ns, ca_util_info* out, float* kernel_ms) {
    if (!t) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(t->device));
    if (t->n_nodes > 0) {
        // a page-locked `out` (ca_host_alloc) takes the rows straight from the kernel
        ca_util_info* dst = nullptr;
        bool zero_copy = false;
        if (out) {
            hipPointerAttribute_t attr;
            if (hipPointerGetAttributes(&attr, out) == hipSuccess && attr.type == hipMemoryTypeHost &&
                attr.devicePointer != nullptr) {
                dst = static_cast<ca_util_info*>(attr.devicePointer);
                zero_copy = true;
            } else {
                (void)hipGetLastError();
            }
        }
        CA_HIP_CHECK(hipEventRecord(t->ev0, t->stream));
        if (t->n_added > 0) {
            hipLaunchKernelGGL(k_added_sums, dim3((t->n_added + kThreads - 1) / kThreads), dim3(kThreads), 0, t->stream,
                               t->added.as<const int32_t>(),
                               reinterpret_cast<const ca_util_pod*>(t->added.as<unsigned char>() + added_pods_at(t->n_added)),
                               t->n_added, skip_daemonset_pods ? 1 : 0, skip_mirror_pods ? 1 : 0, now_ns,
                               t->acc.as<AddedSum>());
            CA_HIP_CHECK(hipGetLastError());
        }
        constexpr int per_block = kThreads / kLanes;
        const int blocks = (t->n_nodes + per_block - 1) / per_block;
        hipLaunchKernelGGL(k_node_utilization, dim3(blocks), dim3(kThreads), 0, t->stream,
                           t->nodes.as<const ca_util_node>(), t->pod_off.as<const int32_t>(),
                           t->pods.as<const ca_util_pod>(), t->n_nodes, skip_daemonset_pods ? 1 : 0,
                           skip_mirror_pods ? 1 : 0, now_ns, t->info.as<ca_util_info>(),
                           t->n_added > 0 ? t->acc.as<AddedSum>() : nullptr, dst);
        CA_HIP_CHECK(hipGetLastError());
        CA_HIP_CHECK(hipEventRecord(t->ev1, t->stream));
        if (out && !zero_copy)
            CA_HIP_CHECK(hipMemcpyAsync(out, t->info.ptr, sizeof(ca_util_info) * t->n_nodes,
                                        hipMemcpyDeviceToHost, t->stream));
    }
    CA_HIP_CHECK(hipStreamSynchronize(t->stream));
    if (kernel_ms) {
        *kernel_ms = 0.0f;
        if (t->n_nodes > 0) CA_HIP_CHECK(hipEventElapsedTime(kernel_ms, t->ev0, t->ev1));
    }
    return CA_OK;
}

int ca_util_device_results(const ca_util_table* t, const ca_util_info** out) {
    if (!t || !out) return CA_EINVAL;
    *out = t->info.as<const ca_util_info>();
    return CA_OK;
}

}  // extern "C"
