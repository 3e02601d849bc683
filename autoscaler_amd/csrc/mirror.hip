// mirror.hip — ClusterSnapshot mirror (host journal + device SoA), the C-ABI entry
// points for the snapshot data plane, and the single-pod predicate kernels
// (FitsAnyNode scan, CheckPredicates, dense feasibility matrix).
//
// Reference: CA/simulator/clustersnapshot/delta.go:43-475 (fork/revert/commit),
// SF/types.go:602-692 (AddPod/RemovePod/update), CA/simulator/predicatechecker/
// schedulerbased.go:83-185 (FitsAnyNodeMatching, CheckPredicates).
#include "mirror.h"
#include "device_filters.h"

#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <condition_variable>
#include <thread>
#include <unordered_map>
#include <algorithm>

namespace casim {

static thread_local std::string g_last_error;
void set_last_error(const std::string& s) { g_last_error = s; }
const std::string& last_error() { return g_last_error; }

int ensure_dyn_lds(const void* kernel, size_t bytes) {
    static std::mutex mu;
    static std::unordered_map<uint64_t, size_t> done;      // (device, kernel) -> limit set
    int dev = 0;
    CA_HIP_CHECK(hipGetDevice(&dev));
    const uint64_t key = ((uint64_t)(uint32_t)dev << 56) ^ (uint64_t)(uintptr_t)kernel;
    std::lock_guard<std::mutex> lock(mu);
    auto it = done.find(key);
    if (it != done.end() && it->second >= bytes) return CA_OK;
    CA_HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done[key] = bytes;
    return CA_OK;
}

// Both buffers grow geometrically: a hipMalloc / hipHostMalloc (and the free before it)
// costs up to milliseconds, and callers like the planner's rounds grow them step by step.
//
// Released blocks go to a per-process cache instead of hipFree / hipHostFree: a caller
// that builds and destroys its objects every loop (a podset of this loop's pending pods,
// an Estimate batch's plan: ~20 device and page-locked buffers) then pays no allocation
// after the first loop.  hipFree synchronises the device; a cached block is handed out
// again only after the same synchronisation, so no queued kernel or copy still uses it.
// The cache keeps at most 4 GiB per device and 1 GiB of page-locked memory, takes the
// smallest cached block of at least the request and at most twice it, and is never
// returned to the runtime (process exit reclaims it).
namespace {
struct BlockCache {
    std::mutex mu;
    std::multimap<size_t, std::pair<int, void*>> free;   // size -> (device or -1, block)
    size_t cached = 0;
    size_t cap = 0;
    void* take(size_t need, int dev, size_t& got) {
        std::lock_guard<std::mutex> lock(mu);
        for (auto it = free.lower_bound(need); it != free.end() && it->first <= 2 * need; ++it) {
            if (it->second.first != dev) continue;
            void* p = it->second.second;
            got = it->first;
            cached -= got;
            free.erase(it);
            return p;
        }
        return nullptr;
    }
    bool give(size_t bytes, int dev, void* p) {
        std::lock_guard<std::mutex> lock(mu);
        if (cached + bytes > cap) return false;
        free.emplace(bytes, std::make_pair(dev, p));
        cached += bytes;
        return true;
    }
};
BlockCache& dev_cache() {
    static BlockCache* c = [] { auto* b = new BlockCache(); b->cap = 4ull << 30; return b; }();   // leaked on purpose
    return *c;
}
BlockCache& host_cache() {
    static BlockCache* c = [] { auto* b = new BlockCache(); b->cap = 1ull << 30; return b; }();
    return *c;
}
// caller blocks (ca_host_alloc / ca_host_free) have a cache of their own: a block a caller
// freed while it still holds views of it can then never alias the library's staging
// buffers
BlockCache& caller_cache() {
    static BlockCache* c = [] { auto* b = new BlockCache(); b->cap = 1ull << 30; return b; }();
    return *c;
}
bool no_cache() {
    static const bool off = knob_env("CASIM_NO_ALLOC_CACHE") != nullptr;
    return off;
}
// the synchronisation hipFree would have done, on the block's device
void sync_device(int dev) {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (dev >= 0 && cur != dev) (void)hipSetDevice(dev);
    (void)hipDeviceSynchronize();
    if (dev >= 0 && cur != dev) (void)hipSetDevice(cur);
}
}  // namespace

int DevBuf::reserve(size_t need) {
    if (need <= bytes) return CA_OK;
    const size_t grown = bytes + bytes / 2;
    release();
    size_t sz = std::max<size_t>(need, std::max<size_t>(grown, 4096));
    int d = 0;
    CA_HIP_CHECK(hipGetDevice(&d));
    size_t got = 0;
    if (!no_cache() && (ptr = dev_cache().take(sz, d, got)) != nullptr) {
        bytes = got;
        dev = d;
        return CA_OK;
    }
    if (hipMalloc(&ptr, sz) != hipSuccess) { ptr = nullptr; bytes = 0; set_last_error("hipMalloc failed"); return CA_EDEVICE; }
    bytes = sz;
    dev = d;
    return CA_OK;
}

int DevBuf::reserve_keep(size_t need, hipStream_t st) {
    if (need <= bytes) return CA_OK;
    size_t sz = std::max<size_t>(need, bytes * 2);
    void* p = nullptr;
    if (hipMalloc(&p, sz) != hipSuccess) { set_last_error("hipMalloc failed"); return CA_EDEVICE; }
    if (ptr && bytes) {
        if (hipMemcpyAsync(p, ptr, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess) return CA_EDEVICE;
        if (hipStreamSynchronize(st) != hipSuccess) return CA_EDEVICE;
        release();
    }
    int d = 0;
    CA_HIP_CHECK(hipGetDevice(&d));
    ptr = p;
    bytes = sz;
    dev = d;
    return CA_OK;
}

void DevBuf::release() {
    if (ptr) {
        bool kept = false;
        if (!no_cache()) {
            sync_device(dev);
            kept = dev_cache().give(bytes, dev, ptr);
        }
        if (!kept) (void)hipFree(ptr);
    }
    ptr = nullptr;
    bytes = 0;
}

namespace {
class WorkerPool {
  public:
    explicit WorkerPool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this, i] { loop(i + 1); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(int32_t T, const std::function<void(int32_t)>& fn) {
        std::lock_guard<std::mutex> region(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &fn;
            njob_ = T;
            left_ = (int32_t)th_.size();
            gen_++;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return left_ == 0; });
    }
    int32_t workers() const { return (int32_t)th_.size(); }

  private:
    void loop(int32_t id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int32_t)>* f;
            int32_t nj;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                f = job_;
                nj = njob_;
            }
            if (id < nj) (*f)(id);
            std::lock_guard<std::mutex> lk(mu_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int32_t)>* job_ = nullptr;
    int32_t njob_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};
}  // namespace

void parallel_run(int32_t T, const std::function<void(int32_t)>& fn) {
    if (T <= 1) { fn(0); return; }
    static WorkerPool pool(7);
    if (T > pool.workers() + 1) T = pool.workers() + 1;
    pool.run(T, fn);
}

int HostBuf::reserve(size_t need) {
    if (need <= bytes) return CA_OK;
    const size_t grown = bytes + bytes / 2;
    release();
    size_t sz = std::max<size_t>(need, std::max<size_t>(grown, 4096));
    size_t got = 0;
    if (!no_cache() && (ptr = host_cache().take(sz, -1, got)) != nullptr) {
        bytes = got;
        return CA_OK;
    }
    if (hipHostMalloc(&ptr, sz, hipHostMallocNonCoherent) != hipSuccess) {
        ptr = nullptr; bytes = 0; set_last_error("hipHostMalloc failed"); return CA_EDEVICE;
    }
    bytes = sz;
    return CA_OK;
}

void HostBuf::release() {
    if (ptr) {
        bool kept = false;
        if (!no_cache()) {
            sync_device(-1);
            kept = host_cache().give(bytes, -1, ptr);
        }
        if (!kept) (void)hipHostFree(ptr);
    }
    ptr = nullptr;
    bytes = 0;
}

int DevPodTable::upload(const ca_pod_spec* pods, int32_t n, const ca_selector_term* tms, int32_t nt,
                        const ca_selector_req* rqs, int32_t nr, const int32_t* nms, int32_t nn,
                        hipStream_t st) {
    std::vector<PodHot> h((size_t)n);
    for (int32_t i = 0; i < n; i++) {
        h[i].cpu = pods[i].req_milli_cpu;
        h[i].mem = pods[i].req_memory;
        h[i].eph = pods[i].req_ephemeral;
        h[i].flags = pod_dev_flags(pods[i]);
        h[i].spec = i;
    }
    int rc;
    // headroom for the pods later calls append (FilterOutSchedulable's placements, the
    // planner's moved copies) without a reallocation
    const size_t room = (size_t)n + (size_t)n / 4 + 1024;
    if ((rc = hot.reserve(sizeof(PodHot) * room)) != CA_OK) return rc;
    if ((rc = spec.reserve(sizeof(ca_pod_spec) * room)) != CA_OK) return rc;
    if ((rc = terms.reserve(sizeof(ca_selector_term) * (size_t)(nt + 1))) != CA_OK) return rc;
    if ((rc = reqs.reserve(sizeof(ca_selector_req) * (size_t)(nr + 1))) != CA_OK) return rc;
    if ((rc = names.reserve(sizeof(int32_t) * (size_t)(nn + 1))) != CA_OK) return rc;
    if (n) CA_HIP_CHECK(hipMemcpyAsync(hot.ptr, h.data(), sizeof(PodHot) * n, hipMemcpyHostToDevice, st));
    if (n) CA_HIP_CHECK(hipMemcpyAsync(spec.ptr, pods, sizeof(ca_pod_spec) * n, hipMemcpyHostToDevice, st));
    if (nt) CA_HIP_CHECK(hipMemcpyAsync(terms.ptr, tms, sizeof(ca_selector_term) * nt, hipMemcpyHostToDevice, st));
    if (nr) CA_HIP_CHECK(hipMemcpyAsync(reqs.ptr, rqs, sizeof(ca_selector_req) * nr, hipMemcpyHostToDevice, st));
    if (nn) CA_HIP_CHECK(hipMemcpyAsync(names.ptr, nms, sizeof(int32_t) * nn, hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipStreamSynchronize(st));
    n_pods = n; n_terms = nt; n_reqs = nr; n_names = nn;
    return CA_OK;
}

int DevPodTable::upload_staged(const ca_pod_spec* pods, int32_t n, const ca_selector_term* tms, int32_t nt,
                               const ca_selector_req* rqs, int32_t nr, const int32_t* nms, int32_t nn, HostBuf& stage,
                               hipStream_t st) {
    // [hot n][records n] in one page-locked block: the DMA reads it while the caller goes on
    // (a pageable source is copied through the runtime's staging before the call returns)
    const size_t hb = ((sizeof(PodHot) * (size_t)n + 255) & ~(size_t)255);
    int rc;
    CA_HIP_CHECK(hipStreamSynchronize(st));      // (an earlier call's copies out of stage are done)
    if ((rc = stage.reserve(hb + sizeof(ca_pod_spec) * (size_t)std::max(n, 1))) != CA_OK) return rc;
    PodHot* const h = stage.as<PodHot>();
    ca_pod_spec* const rec = reinterpret_cast<ca_pod_spec*>(stage.as<unsigned char>() + hb);
    const int32_t T = n >= 8192 ? 8 : 1;
    parallel_run(T, [&](int32_t w) {
        const int32_t a = (int32_t)((int64_t)n * w / T), b = (int32_t)((int64_t)n * (w + 1) / T);
        std::memcpy(rec + a, pods + a, sizeof(ca_pod_spec) * (size_t)(b - a));
        for (int32_t i = a; i < b; i++) {
            h[i].cpu = pods[i].req_milli_cpu;
            h[i].mem = pods[i].req_memory;
            h[i].eph = pods[i].req_ephemeral;
            h[i].flags = pod_dev_flags(pods[i]);
            h[i].spec = i;
        }
    });
    const size_t room = (size_t)n + (size_t)n / 4 + 1024;
    if ((rc = hot.reserve(sizeof(PodHot) * room)) != CA_OK) return rc;
    if ((rc = spec.reserve(sizeof(ca_pod_spec) * room)) != CA_OK) return rc;
    if ((rc = terms.reserve(sizeof(ca_selector_term) * (size_t)(nt + 1))) != CA_OK) return rc;
    if ((rc = reqs.reserve(sizeof(ca_selector_req) * (size_t)(nr + 1))) != CA_OK) return rc;
    if ((rc = names.reserve(sizeof(int32_t) * (size_t)(nn + 1))) != CA_OK) return rc;
    if (n) CA_HIP_CHECK(hipMemcpyAsync(hot.ptr, h, sizeof(PodHot) * n, hipMemcpyHostToDevice, st));
    if (n) CA_HIP_CHECK(hipMemcpyAsync(spec.ptr, rec, sizeof(ca_pod_spec) * n, hipMemcpyHostToDevice, st));
    if (nt) CA_HIP_CHECK(hipMemcpyAsync(terms.ptr, tms, sizeof(ca_selector_term) * nt, hipMemcpyHostToDevice, st));
    if (nr) CA_HIP_CHECK(hipMemcpyAsync(reqs.ptr, rqs, sizeof(ca_selector_req) * nr, hipMemcpyHostToDevice, st));
    if (nn) CA_HIP_CHECK(hipMemcpyAsync(names.ptr, nms, sizeof(int32_t) * nn, hipMemcpyHostToDevice, st));
    n_pods = n; n_terms = nt; n_reqs = nr; n_names = nn;
    return CA_OK;
}

int DevPodTable::append(const ca_pod_spec* np, int32_t k, const ca_selector_term* tms, int32_t nt,
                        const ca_selector_req* rqs, int32_t nr, const int32_t* nms, int32_t nn, hipStream_t st) {
    const int32_t n0 = n_pods, n = n_pods + k;
    std::vector<PodHot> h((size_t)std::max(k, 0));
    for (int32_t i = 0; i < k; i++) {
        h[i].cpu = np[i].req_milli_cpu;
        h[i].mem = np[i].req_memory;
        h[i].eph = np[i].req_ephemeral;
        h[i].flags = pod_dev_flags(np[i]);
        h[i].spec = n0 + i;
    }
    int rc;
    if ((rc = hot.reserve_keep(sizeof(PodHot) * (size_t)(n + 1), st)) != CA_OK) return rc;
    if ((rc = spec.reserve_keep(sizeof(ca_pod_spec) * (size_t)(n + 1), st)) != CA_OK) return rc;
    if ((rc = terms.reserve_keep(sizeof(ca_selector_term) * (size_t)(nt + 1), st)) != CA_OK) return rc;
    if ((rc = reqs.reserve_keep(sizeof(ca_selector_req) * (size_t)(nr + 1), st)) != CA_OK) return rc;
    if ((rc = names.reserve_keep(sizeof(int32_t) * (size_t)(nn + 1), st)) != CA_OK) return rc;
    if (k > 0) {
        CA_HIP_CHECK(hipMemcpyAsync(hot.as<PodHot>() + n0, h.data(), sizeof(PodHot) * k, hipMemcpyHostToDevice, st));
        CA_HIP_CHECK(hipMemcpyAsync(spec.as<ca_pod_spec>() + n0, np, sizeof(ca_pod_spec) * k, hipMemcpyHostToDevice, st));
    }
    if (nt > n_terms)
        CA_HIP_CHECK(hipMemcpyAsync(terms.as<ca_selector_term>() + n_terms, tms + n_terms,
                                    sizeof(ca_selector_term) * (nt - n_terms), hipMemcpyHostToDevice, st));
    if (nr > n_reqs)
        CA_HIP_CHECK(hipMemcpyAsync(reqs.as<ca_selector_req>() + n_reqs, rqs + n_reqs,
                                    sizeof(ca_selector_req) * (nr - n_reqs), hipMemcpyHostToDevice, st));
    if (nn > n_names)
        CA_HIP_CHECK(hipMemcpyAsync(names.as<int32_t>() + n_names, nms + n_names, sizeof(int32_t) * (nn - n_names),
                                    hipMemcpyHostToDevice, st));
    CA_HIP_CHECK(hipStreamSynchronize(st));
    n_pods = n; n_terms = nt; n_reqs = nr; n_names = nn;
    return CA_OK;
}

__global__ void __launch_bounds__(256) k_gather_pods(const PodHot* __restrict__ sh, const ca_pod_spec* __restrict__ ss,
                                                     const int32_t* __restrict__ idx, int32_t k, int32_t n0,
                                                     PodHot* __restrict__ dh, ca_pod_spec* __restrict__ ds) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= k) return;
    const int32_t j = idx[i];
    PodHot h = sh[j];
    h.spec = n0 + i;
    dh[n0 + i] = h;
    ds[n0 + i] = ss[j];
}

int DevPodTable::append_gather(const DevPodTable& src, const int32_t* idx, int32_t k, DevBuf& d_idx, hipStream_t st) {
    const int32_t n0 = n_pods, n = n_pods + k;
    int rc;
    if ((rc = hot.reserve_keep(sizeof(PodHot) * (size_t)(n + 1), st)) != CA_OK) return rc;
    if ((rc = spec.reserve_keep(sizeof(ca_pod_spec) * (size_t)(n + 1), st)) != CA_OK) return rc;
    if (k > 0) {
        if ((rc = d_idx.reserve(sizeof(int32_t) * (size_t)k)) != CA_OK) return rc;
        CA_HIP_CHECK(hipMemcpyAsync(d_idx.ptr, idx, sizeof(int32_t) * (size_t)k, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_gather_pods, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, st, src.hot.as<const PodHot>(),
                           src.spec.as<const ca_pod_spec>(), d_idx.as<const int32_t>(), k, n0, hot.as<PodHot>(),
                           spec.as<ca_pod_spec>());
        CA_HIP_CHECK(hipGetLastError());
        CA_HIP_CHECK(hipStreamSynchronize(st));          // (idx is the caller's pageable memory)
    }
    n_pods = n;
    return CA_OK;
}

// a dirty row staged for sync_nodes
struct alignas(16) StagedRow {
    int32_t row, pad[3];
    NodeHot hot;
    NodeExt ext;
};

__global__ void k_scatter_rows(const StagedRow* __restrict__ rows, int32_t k, NodeHot* __restrict__ hot,
                               NodeExt* __restrict__ ext) {
    const int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j >= k) return;
    const int32_t r = rows[j].row;
    hot[r] = rows[j].hot;
    ext[r] = rows[j].ext;
}

// Resident hints around RemoveNode(pos) (positions after it shift down by one).  A hint
// to the removed node is kept as code = -2 - serial, where serial numbers the mirror's
// RemoveNode calls (no usable hint: kernels read h >= 0 only), so the Revert of that very
// removal restores it — two removals at the same position (node p, then the node that
// shifted into p) keep distinct codes.  The reference keeps hints by node NAME
// (hints.go:29-72) outside the snapshot, and the name is valid again after the Revert.
__global__ void k_remap_hints(int32_t* __restrict__ h, int32_t n, int32_t pos, int32_t code, int32_t restore) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    int32_t v = h[i];
    if (!restore) {
        if (v == pos) v = code;
        else if (v > pos) v--;
    } else {
        if (v == code) v = pos;
        else if (v >= pos) v++;
    }
    h[i] = v;
}

}  // namespace casim

using namespace casim;

// ---------------------------------------------------------------------------
// host row algebra (NodeInfo.update SF/types.go:672-692)
// ---------------------------------------------------------------------------
void ca_mirror::mark_dirty(int32_t node) {
    if ((size_t)node >= dirty_flag.size()) dirty_flag.resize(nodes.size(), 0);
    if (!dirty_flag[node]) {
        dirty_flag[node] = 1;
        dirty_rows.push_back(node);
    }
}

void ca_mirror::node_apply(int32_t node, const ca_pod_spec& p, int sign) {
    NodeRow& nd = nodes[node];
    if (sign > 0) {
        nd.req_cpu = wadd(nd.req_cpu, p.req_milli_cpu);
        nd.req_mem = wadd(nd.req_mem, p.req_memory);
        nd.req_eph = wadd(nd.req_eph, p.req_ephemeral);
        for (int i = 0; i < CA_MAX_SCALAR; i++) nd.req_scalar[i] = wadd(nd.req_scalar[i], p.req_scalar[i]);
        for (int w = 0; w < CA_PORT_WORDS; w++) nd.ports[w] |= p.port_use[w];
    } else {
        nd.req_cpu = wsub(nd.req_cpu, p.req_milli_cpu);
        nd.req_mem = wsub(nd.req_mem, p.req_memory);
        nd.req_eph = wsub(nd.req_eph, p.req_ephemeral);
        for (int i = 0; i < CA_MAX_SCALAR; i++) nd.req_scalar[i] = wsub(nd.req_scalar[i], p.req_scalar[i]);
        // HostPortInfo.Remove deletes the triple (set semantics, SF/types.go:863-880)
        for (int w = 0; w < CA_PORT_WORDS; w++) nd.ports[w] &= ~p.port_use[w];
    }
    nd.npods += sign;
    if (p.flags & CA_POD_REQUIRED_ANTI_AFFINITY) n_scope_blockers += sign;
    mark_dirty(node);
}

void ca_mirror::journal_push(int32_t kind, int32_t node, int32_t pod, int32_t slot, const uint64_t* ports) {
    if (depth == 0 && kind != J_FORK) return;
    JournalEntry e;
    std::memset(&e, 0, sizeof e);
    e.kind = kind; e.node = node; e.pod = pod; e.slot = slot;
    if (ports) std::memcpy(e.ports, ports, sizeof e.ports);
    journal.push_back(e);
}

void ca_mirror::add_pod_to_node(int32_t pod, int32_t node) {
    uint64_t before[CA_PORT_WORDS];
    std::memcpy(before, nodes[node].ports, sizeof before);
    node_apply(node, pods[pod].spec, +1);
    nodes[node].pods.push_back(pod);
    pods[pod].node = node;
    journal_push(J_ADD_POD, node, pod, (int32_t)nodes[node].pods.size() - 1, before);
}

void ca_mirror::reserve_more(size_t n_pods_add, size_t n_journal_add) {
    pods.reserve(pods.size() + n_pods_add);                 // (chunked: nothing moves)
    if (journal.capacity() < journal.size() + n_journal_add)
        journal.reserve(std::max(journal.capacity() * 2, journal.size() + n_journal_add));
}

void ca_mirror::add_placed_batch(const ca_pod_table* t, const int32_t* idx, const int32_t* node, int32_t n,
                                 int32_t* out_id, bool device_rows, bool known_plain) {
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto tmark = [&](const char* what) {
        if (dbg_t)
            fprintf(stderr, "[add_placed] %-10s %8.3f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    int32_t np = 0;
    bool plain = true;                      // no selector tables or PreFilter names to re-base
    // (known_plain: the caller's pod set holds no such references — no record reads here)
    for (int32_t k = 0; k < n; k++) {
        if (node[k] < 0) continue;
        np++;
        if (known_plain) continue;
        const ca_pod_spec& ps = t->pods[idx[k]];
        if (ps.aff_term_count > 0 || ((ps.flags & CA_POD_PREFILTER_NAMES) && ps.prefilter_count > 0)) plain = false;
    }
    reserve_more((size_t)np, depth > 0 ? (size_t)np : 0);
    tmark("reserved");
    int32_t T = plain ? std::min(8, np / 2048) : 1;
    T = T >= 8 ? 8 : T >= 4 ? 4 : T >= 2 ? 2 : 1;              // (a power of two: 64-node block & (T - 1) picks the thread)
    const int32_t tmask = T - 1;
    // rows dirty before this batch stay dirty; the batch's own marks are dropped below where
    // the kernel's row equals fill_hot's
    const size_t dirty0 = dirty_rows.size();
    auto keep_device_rows = [&]() {
        if (!device_rows) return;
        size_t w = dirty0;
        for (size_t i = dirty0; i < dirty_rows.size(); i++) {
            const int32_t x = dirty_rows[i];
            const NodeRow& nd = nodes[x];
            // the kernel's pods column is the old clamp minus one per pod: equal unless clamped
            const int64_t fp = nd.spec.alloc_pods - nd.npods;
            if (fp >= INT32_MIN && fp + np <= INT32_MAX && (size_t)x < d_rows) { dirty_flag[x] = 0; continue; }
            dirty_rows[w++] = x;
        }
        dirty_rows.resize(w);
    };
    if (T <= 1) {
        for (int32_t k = 0; k < n; k++) {
            if (node[k] < 0) { if (out_id) out_id[k] = -1; continue; }
            const int32_t id = store_pod(t, idx[k], node[k]);
            add_pod_to_node(id, node[k]);
            if (out_id) out_id[k] = id;
        }
        keep_device_rows();
        return;
    }
    // Threads own disjoint pod id ranges (the records) and disjoint node sets (64-node blocks: adjacent rows share cache lines): each
    // walks the placements in order for its nodes, so every node sees its pods in order; the
    // journal entries of different nodes commute (Revert undoes each node's in reverse).
    const size_t base = pods.size();
    pods.resize_for_overwrite(base + (size_t)np);                // (the threads write every record)
    if (dirty_flag.size() < nodes.size()) dirty_flag.resize(nodes.size(), 0);
    std::vector<int32_t> id_of((size_t)n, -1);
    // each thread's placements (its nodes' 64-node blocks), in order: a counting sort once
    // instead of every thread stepping over all n positions
    std::vector<int32_t> bk_off((size_t)T + 1, 0), bk((size_t)np);
    for (int32_t k = 0, c = 0; k < n; k++)
        if (node[k] >= 0) { id_of[k] = (int32_t)base + c++; bk_off[((node[k] >> 6) & tmask) + 1]++; }
    for (int32_t w = 0; w < T; w++) bk_off[w + 1] += bk_off[w];
    {
        std::vector<int32_t> fill(bk_off.begin(), bk_off.end() - 1);
        for (int32_t k = 0; k < n; k++)
            if (node[k] >= 0) bk[fill[(node[k] >> 6) & tmask]++] = k;
    }
    tmark("resized");
    struct Part {
        std::vector<int32_t> dirty;
        int64_t ext = 0, eph = 0, blockers = 0, oos = 0;
    };
    std::vector<Part> part((size_t)T);
    const bool journaled = depth > 0;
    // the journal grows by one entry per placement: thread w writes its placements' entries
    // at jbase + bk_off[w] ... in place (no per-thread lists to merge)
    const size_t jbase = journal.size();
    if (journaled) journal.resize(jbase + (size_t)np);
    std::vector<double> tw((size_t)T * 3, 0.0);          // (CASIM_DEBUG_TIMING: per-thread start / records / AddPods)
    auto work = [&](int32_t w) {
        if (dbg_t) tw[3 * w] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        Part& pt = part[w];
        const int32_t k0 = (int32_t)((int64_t)n * w / T), k1 = (int32_t)((int64_t)n * (w + 1) / T);
        for (int32_t k = k0; k < k1; k++) {             // the records of positions [k0, k1)
            if (id_of[k] < 0) continue;
            casim::PodRow& r = pods[id_of[k]];
            r.spec = t->pods[idx[k]];
            r.node = node[k];
            if (casim::pod_dev_flags(r.spec) & (casim::PF_PORTS | casim::PF_SCALAR_REQ | casim::PF_MOVED_SCALAR_REQ)) pt.ext++;
            if (r.spec.req_ephemeral != 0) pt.eph++;
            if (r.spec.flags & CA_POD_OUT_OF_SCOPE) pt.oos++;
        }
        if (dbg_t) tw[3 * w + 1] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        const int32_t b0 = bk_off[w], b1 = bk_off[w + 1];
        for (int32_t b = b0; b < b1; b++) {            // AddPod on my nodes, in order
            if (b + 16 < b1) {                           // (rows are cache misses: fetch ahead)
                const int32_t y = node[bk[b + 16]];
                __builtin_prefetch(&nodes[y], 1);
                __builtin_prefetch(reinterpret_cast<const char*>(&nodes[y]) + 256, 1);
            }
            const int32_t k = bk[b];
            const int32_t x = node[k];
            const ca_pod_spec& p = t->pods[idx[k]];
            casim::NodeRow& nd = nodes[x];
            if (journaled) {
                casim::JournalEntry& e = journal[jbase + (size_t)b];
                e.kind = casim::J_ADD_POD; e.node = x; e.pod = id_of[k];
                e.slot = (int32_t)nd.pods.size();                       // (the slot push_back below fills)
                std::memcpy(e.ports, nd.ports, sizeof e.ports);
            }
            nd.req_cpu = casim::wadd(nd.req_cpu, p.req_milli_cpu);       // node_apply(+1)
            nd.req_mem = casim::wadd(nd.req_mem, p.req_memory);
            nd.req_eph = casim::wadd(nd.req_eph, p.req_ephemeral);
            for (int i = 0; i < CA_MAX_SCALAR; i++) nd.req_scalar[i] = casim::wadd(nd.req_scalar[i], p.req_scalar[i]);
            for (int q = 0; q < CA_PORT_WORDS; q++) nd.ports[q] |= p.port_use[q];
            nd.npods += 1;
            if (p.flags & CA_POD_REQUIRED_ANTI_AFFINITY) pt.blockers++;
            if (!dirty_flag[x]) { dirty_flag[x] = 1; pt.dirty.push_back(x); }
            nd.pods.push_back(id_of[k]);
        }
        if (device_rows) {                              // keep_device_rows on my own new marks
            size_t o = 0;
            for (const int32_t x : pt.dirty) {
                const casim::NodeRow& nd = nodes[x];
                const int64_t fp = nd.spec.alloc_pods - nd.npods;
                if (fp >= INT32_MIN && fp + np <= INT32_MAX && (size_t)x < d_rows) { dirty_flag[x] = 0; continue; }
                pt.dirty[o++] = x;
            }
            pt.dirty.resize(o);
        }
        if (dbg_t) tw[3 * w + 2] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    casim::parallel_run(T, work);
    tmark("threads");
    if (dbg_t)
        for (int32_t w = 0; w < T; w++)
            fprintf(stderr, "[add_placed]   thread %d: start %.3f records %.3f addpods %.3f ms\n", w, tw[3 * w], tw[3 * w + 1],
                    tw[3 * w + 2]);
    for (Part& pt : part) {
        n_ext_pods += pt.ext;
        n_eph_pods += pt.eph;
        n_oos_pods += pt.oos;
        n_scope_blockers += pt.blockers;
        dirty_rows.insert(dirty_rows.end(), pt.dirty.begin(), pt.dirty.end());
    }
    if (out_id)
        for (int32_t k = 0; k < n; k++) out_id[k] = id_of[k];
    tmark("merged");
}

int32_t ca_mirror::store_pod(const ca_pod_table* t, int32_t idx, int32_t node) {
    PodRow row;
    row.spec = t->pods[idx];
    row.node = node;
    if (row.spec.aff_term_count > 0) {
        int32_t first = (int32_t)terms.size();
        for (int32_t k = 0; k < row.spec.aff_term_count; k++) {
            ca_selector_term tm = t->terms[row.spec.aff_term_first + k];
            int32_t rfirst = (int32_t)reqs.size();
            for (int32_t r = 0; r < tm.count; r++) reqs.push_back(t->reqs[tm.first + r]);
            tm.first = rfirst;
            terms.push_back(tm);
        }
        row.spec.aff_term_first = first;
    }
    if ((row.spec.flags & CA_POD_PREFILTER_NAMES) && row.spec.prefilter_count > 0) {
        int32_t first = (int32_t)pf_names.size();
        for (int32_t k = 0; k < row.spec.prefilter_count; k++)
            pf_names.push_back(t->prefilter_names[row.spec.prefilter_first + k]);
        row.spec.prefilter_first = first;
    }
    if (pod_dev_flags(row.spec) & (PF_PORTS | PF_SCALAR_REQ | PF_MOVED_SCALAR_REQ)) n_ext_pods++;
    if (row.spec.req_ephemeral != 0) n_eph_pods++;
    if (row.spec.flags & CA_POD_OUT_OF_SCOPE) n_oos_pods++;
    pods.push_back(row);
    return (int32_t)pods.size() - 1;
}

void ca_mirror::fill_hot(int32_t i, NodeHot& h) const {
    const NodeRow& nd = nodes[i];
    h.cpu = wsub(nd.spec.alloc_milli_cpu, nd.req_cpu);
    h.mem = wsub(nd.spec.alloc_memory, nd.req_mem);
    h.eph = wsub(nd.spec.alloc_ephemeral, nd.req_eph);
    h.pods = clamp_i32(nd.spec.alloc_pods - nd.npods);
    uint32_t f = NF_VALID;
    if (nd.spec.flags & CA_NODE_UNSCHEDULABLE) f |= NF_UNSCHED;
    if (nd.spec.taints) f |= NF_TAINTS;
    bool ports = false;
    for (int w = 0; w < CA_PORT_WORDS; w++) ports |= nd.ports[w] != 0;
    if (ports) f |= NF_PORTS;
    bool sc = false;
    for (int k = 0; k < CA_MAX_SCALAR; k++) sc |= nd.spec.alloc_scalar[k] != 0 || nd.req_scalar[k] != 0;
    if (sc) f |= NF_SCALAR;
    h.flags = f;
}

void ca_mirror::fill_ext(int32_t i, NodeExt& e) const {
    const NodeRow& nd = nodes[i];
    for (int k = 0; k < CA_MAX_SCALAR; k++) e.scalar[k] = wsub(nd.spec.alloc_scalar[k], nd.req_scalar[k]);
    for (int w = 0; w < CA_PORT_WORDS; w++) e.ports[w] = nd.ports[w];
}

void ca_mirror::fill_static(int32_t i, NodeStatic& s) const {
    const ca_node_spec& n = nodes[i].spec;
    std::memset(&s, 0, sizeof s);
    s.taints = n.taints;
    for (int w = 0; w < CA_LABEL_WORDS; w++) s.labels[w] = n.label_pairs[w];
    s.keys = n.label_keys;
    for (int k = 0; k < CA_MAX_INT_KEYS; k++) s.ints[k] = n.int_label[k];
    s.int_valid = n.int_label_valid;
    s.name_id = n.name_id;
}

int ca_mirror::remap_hints_removed(int32_t pos, int32_t code, bool restore) {
    if (d_hints_n == 0) return CA_OK;
    hipLaunchKernelGGL(k_remap_hints, dim3((unsigned)((d_hints_n + 255) / 256)), dim3(256), 0, stream,
                       d_pod_hints.as<int32_t>(), (int32_t)d_hints_n, pos, code, restore ? 1 : 0);
    CA_HIP_CHECK(hipGetLastError());
    return CA_OK;
}

int ca_mirror::sync_nodes() {
    const size_t n = nodes.size();
    int rc;
    static const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    struct Done {                                           // (CASIM_DEBUG_TIMING: the sync's size and time)
        bool on; const std::chrono::steady_clock::time_point t0; size_t rows; bool full, stat;
        ~Done() {
            if (on)
                fprintf(stderr, "[sync_nodes] %zu rows%s%s %.3f ms\n", rows, full ? " (full)" : "", stat ? " +static" : "",
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
    } done{dbg_t, t0, dirty_rows.size(), all_dirty, static_dirty};
    if (n > d_cap) {
        size_t cap = std::max<size_t>(n, std::max<size_t>(1024, d_cap * 2));
        if ((rc = d_hot.reserve(sizeof(NodeHot) * cap)) != CA_OK) return rc;
        if ((rc = d_ext.reserve(sizeof(NodeExt) * cap)) != CA_OK) return rc;
        if ((rc = d_static.reserve(sizeof(NodeStatic) * cap)) != CA_OK) return rc;
        d_cap = cap;
        all_dirty = true;
        static_dirty = true;
    }
    if (n > d_rows) {
        // new rows (AddNode): upload them fully
        for (size_t i = d_rows; i < n; i++) mark_dirty((int32_t)i);
        static_dirty = true;
    }
    if (all_dirty || dirty_rows.size() > std::max<size_t>(64, n / 4)) {
        // both columns built in page-locked memory: DMA straight from it, no staging copy
        if ((rc = rs.full.reserve((sizeof(NodeHot) + sizeof(NodeExt)) * std::max<size_t>(n, 1))) != CA_OK) return rc;
        NodeHot* h = rs.full.as<NodeHot>();
        NodeExt* e = reinterpret_cast<NodeExt*>(h + n);
        // (a revert's or a new snapshot's thousands of rows: filled by the host workers)
        const int32_t T = (int32_t)std::max<size_t>(1, std::min<size_t>(8, n / 2048));
        casim::parallel_run(T, [&](int32_t w) {
            const size_t i0 = n * (size_t)w / (size_t)T, i1 = n * (size_t)(w + 1) / (size_t)T;
            for (size_t i = i0; i < i1; i++) { fill_hot((int32_t)i, h[i]); fill_ext((int32_t)i, e[i]); }
        });
        if (dbg_t)
            fprintf(stderr, "[sync_nodes]   filled %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        if (n) CA_HIP_CHECK(hipMemcpyAsync(d_hot.ptr, h, sizeof(NodeHot) * n, hipMemcpyHostToDevice, stream));
        if (n) CA_HIP_CHECK(hipMemcpyAsync(d_ext.ptr, e, sizeof(NodeExt) * n, hipMemcpyHostToDevice, stream));
        CA_HIP_CHECK(hipStreamSynchronize(stream));
        // the staged path's buffers sized now, so the first partial sync (a revert's rows,
        // the next loop) allocates nothing
        const size_t kcap0 = std::max<size_t>(64, n / 4);
        if ((rc = rs.h.reserve(sizeof(StagedRow) * kcap0)) != CA_OK) return rc;
        if ((rc = rs.d.reserve(sizeof(StagedRow) * kcap0)) != CA_OK) return rc;
    } else if (!dirty_rows.empty()) {
        // few rows: stage them (row id + both columns) in pinned memory, one H2D copy, and
        // scatter them on the device
        const size_t k = dirty_rows.size();
        const size_t kcap = std::max<size_t>(k, std::max<size_t>(64, n / 4));   // the largest staged batch
        if ((rc = rs.h.reserve(sizeof(StagedRow) * kcap)) != CA_OK) return rc;
        if ((rc = rs.d.reserve(sizeof(StagedRow) * kcap)) != CA_OK) return rc;
        if (dbg_t)
            fprintf(stderr, "[sync_nodes]   staging reserved %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        StagedRow* sr = rs.h.as<StagedRow>();
        for (size_t j = 0; j < k; j++) {
            sr[j].row = dirty_rows[j];
            fill_hot(dirty_rows[j], sr[j].hot);
            fill_ext(dirty_rows[j], sr[j].ext);
        }
        CA_HIP_CHECK(hipMemcpyAsync(rs.d.ptr, sr, sizeof(StagedRow) * k, hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, stream,
                           rs.d.as<const StagedRow>(), (int32_t)k, d_hot.as<NodeHot>(), d_ext.as<NodeExt>());
        CA_HIP_CHECK(hipGetLastError());
        if (dbg_t)
            fprintf(stderr, "[sync_nodes]   staged + launched %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        CA_HIP_CHECK(hipStreamSynchronize(stream));        // the staging buffer is reused
    }
    if (static_dirty && n) {
        std::vector<NodeStatic> s(n);
        const int32_t T = (int32_t)std::max<size_t>(1, std::min<size_t>(8, n / 2048));
        casim::parallel_run(T, [&](int32_t w) {
            const size_t i0 = n * (size_t)w / (size_t)T, i1 = n * (size_t)(w + 1) / (size_t)T;
            for (size_t i = i0; i < i1; i++) fill_static((int32_t)i, s[i]);
        });
        CA_HIP_CHECK(hipMemcpyAsync(d_static.ptr, s.data(), sizeof(NodeStatic) * n, hipMemcpyHostToDevice, stream));
        CA_HIP_CHECK(hipStreamSynchronize(stream));
    }
    for (int32_t r : dirty_rows) if ((size_t)r < dirty_flag.size()) dirty_flag[r] = 0;
    dirty_rows.clear();
    all_dirty = false;
    static_dirty = false;
    d_rows = n;
    return CA_OK;
}

int ca_mirror::sync_pods() {
    if (d_pods_synced == pods.size() && d_terms_synced == terms.size() && (size_t)d_pods.n_reqs == reqs.size() &&
        (size_t)d_pods.n_names == pf_names.size())
        return CA_OK;
    // pod records and selector tables only grow between Clear()s (Revert detaches pods
    // from their nodes, ids are never reused): append the new tail
    if (pods.size() >= d_pods_synced && terms.size() >= d_terms_synced && d_pods_synced == (size_t)d_pods.n_pods &&
        reqs.size() >= (size_t)d_pods.n_reqs && pf_names.size() >= (size_t)d_pods.n_names && d_pods_synced > 0) {
        const size_t a = d_pods_synced, k = pods.size() - a;
        // the new records gathered into page-locked staging (shared with sync_nodes' full
        // path; both finish their copies before returning): DMA straight from it
        int rc = rs.full.reserve(sizeof(ca_pod_spec) * std::max<size_t>(k, 1));
        if (rc != CA_OK) return rc;
        ca_pod_spec* specs = rs.full.as<ca_pod_spec>();
        for (size_t i = 0; i < k; i++) specs[i] = pods[a + i].spec;
        rc = d_pods.append(specs, (int32_t)k, terms.data(), (int32_t)terms.size(), reqs.data(),
                           (int32_t)reqs.size(), pf_names.data(), (int32_t)pf_names.size(), stream);
        if (rc != CA_OK) return rc;
        d_pods_synced = pods.size();
        d_terms_synced = terms.size();
        return CA_OK;
    }
    std::vector<ca_pod_spec> specs(pods.size());
    for (size_t i = 0; i < pods.size(); i++) specs[i] = pods[i].spec;
    int rc = d_pods.upload(specs.data(), (int32_t)specs.size(), terms.data(), (int32_t)terms.size(),
                           reqs.data(), (int32_t)reqs.size(), pf_names.data(), (int32_t)pf_names.size(), stream);
    if (rc != CA_OK) return rc;
    d_pods_synced = pods.size();
    d_terms_synced = terms.size();
    return CA_OK;
}

// ---------------------------------------------------------------------------
// kernels: FitsAnyNodeMatching scan, CheckPredicates, feasibility matrix
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_fits_scan(
    const NodeHot* __restrict__ hot, const NodeExt* __restrict__ ext, const NodeStatic* __restrict__ st,
    int32_t n, const PodHot* __restrict__ ph, const ca_pod_spec* __restrict__ specs,
    const ca_selector_term* __restrict__ terms, const ca_selector_req* __restrict__ reqs,
    const int32_t* __restrict__ names, int32_t pod, int64_t L, int32_t kind, int32_t lo, int32_t hi,
    int32_t exclude, const uint8_t* __restrict__ mask, unsigned long long* __restrict__ out_fit,
    unsigned long long* __restrict__ out_vis) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);   // rotated offset
    const PodHot p = ph[pod];
    bool vis = false, fit = false;
    if (i < n) {
        int32_t pos = (int32_t)L + i;                                      // schedulerbased.go:115
        if (pos >= n) pos -= n;
        bool m = pos != exclude;
        if (kind == CA_MATCH_RANGE) m = m && pos >= lo && pos < hi;
        else if (kind == CA_MATCH_MASK) m = m && mask[pos] != 0;
        if (m) {
            const NodeHot h = hot[pos];
            bool pf_ok = true;
            if (p.flags & PF_PREFILTER_NAMES) {                            // :120
                const ca_pod_spec& s = specs[p.spec];
                const int32_t nm = st[pos].name_id;
                pf_ok = false;
                for (int32_t k = 0; k < s.prefilter_count; k++) pf_ok |= names[s.prefilter_first + k] == nm;
            }
            if (pf_ok && !(h.flags & NF_UNSCHED)) {                        // :125
                vis = true;
                uint32_t reasons;
                fit = dev_full_filters(specs[p.spec], p, terms, reqs, h, ext + pos, st + pos, false, &reasons)
                      == CA_PLUGIN_NONE;
            }
        }
    }
    const unsigned long long bf = __ballot(fit), bv = __ballot(vis);
    const int32_t w = i >> 6;
    if ((threadIdx.x & 63) == 0 && (int64_t)w * 64 < n) { out_fit[w] = bf; out_vis[w] = bv; }
}

__global__ void k_check_one(const NodeHot* __restrict__ hot, const NodeExt* __restrict__ ext,
                            const NodeStatic* __restrict__ st, const PodHot* __restrict__ ph,
                            const ca_pod_spec* __restrict__ specs, const ca_selector_term* __restrict__ terms,
                            const ca_selector_req* __restrict__ reqs, int32_t pod, int32_t node,
                            ca_pred_result* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const PodHot p = ph[pod];
    ca_pred_result r;
    r.type = CA_PRED_OK; r.plugin = 0; r.reasons = 0; r.taint = 0;
    uint32_t reasons = 0;
    const int plugin = dev_full_filters(specs[p.spec], p, terms, reqs, hot[node], ext + node, st + node, true, &reasons);
    if (plugin != CA_PLUGIN_NONE) {
        r.type = CA_PRED_NOT_SCHEDULABLE;
        r.plugin = plugin;
        r.reasons = reasons;
        if (plugin == CA_PLUGIN_TAINT_TOLERATION) {
            const uint64_t u = st[node].taints & ~specs[p.spec].tolerated_taints;
            r.taint = (int32_t)__builtin_ctzll(u);
        }
    }
    *out = r;
}

// ComputeExpansionOption's check (orchestrator.go:455-481) for every (node group, pod
// equivalence group): CheckPredicates(sample pod, fresh copy of the group's template)
// with the reference's result (schedulerbased.go:139-185; the PreFilter failure is an
// internal error).  One thread per (template, sample); templates on the grid's y axis.
__global__ void __launch_bounds__(256) k_check_templates(
    const NodeHot* __restrict__ thot, const NodeExt* __restrict__ text, const NodeStatic* __restrict__ tst,
    const int32_t* __restrict__ samples, int32_t n_samples, const PodHot* __restrict__ ph,
    const ca_pod_spec* __restrict__ specs, const ca_selector_term* __restrict__ terms,
    const ca_selector_req* __restrict__ reqs, ca_pred_result* __restrict__ out, uint8_t* __restrict__ out_ok) {
    const int32_t e = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int32_t g = (int32_t)blockIdx.y;
    if (e >= n_samples) return;
    const PodHot p = ph[samples[e]];
    ca_pred_result r;
    r.type = CA_PRED_OK; r.plugin = 0; r.reasons = 0; r.taint = 0;
    if ((p.flags & PF_OUT_OF_SCOPE) || (thot[g].flags & NF_OUT_OF_SCOPE)) {
        r.type = CA_PRED_UNSUPPORTED;                    // casim.h scope: the Go path evaluates it
    } else if (p.flags & PF_PREFILTER_FAIL) {
        r.type = CA_PRED_INTERNAL;
        r.plugin = CA_PLUGIN_NODE_AFFINITY;
    } else {
        uint32_t reasons = 0;
        const int plugin = dev_full_filters(specs[p.spec], p, terms, reqs, thot[g], text + g, tst + g, true, &reasons);
        if (plugin != CA_PLUGIN_NONE) {
            r.type = CA_PRED_NOT_SCHEDULABLE;
            r.plugin = plugin;
            r.reasons = reasons;
            if (plugin == CA_PLUGIN_TAINT_TOLERATION) {
                const uint64_t u = tst[g].taints & ~specs[p.spec].tolerated_taints;
                r.taint = (int32_t)__builtin_ctzll(u);
            }
        }
    }
    if (out) out[(size_t)g * n_samples + e] = r;
    if (out_ok) out_ok[(size_t)g * n_samples + e] = r.type == CA_PRED_OK ? 1 : 0;
}

// Dense pods x nodes feasibility (CheckPredicates semantics, PreFilter failure -> 0).
// One thread per (pod, node); nodes on the fast axis for coalesced node rows.
__global__ void __launch_bounds__(256) k_fits_matrix(
    const NodeHot* __restrict__ hot, const NodeExt* __restrict__ ext, const NodeStatic* __restrict__ st,
    int32_t n, const PodHot* __restrict__ ph, const ca_pod_spec* __restrict__ specs,
    const ca_selector_term* __restrict__ terms, const ca_selector_req* __restrict__ reqs,
    int32_t n_pods, uint8_t* __restrict__ out) {
    const int32_t node = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int32_t pod = (int32_t)blockIdx.y;
    if (node >= n || pod >= n_pods) return;
    const PodHot p = ph[pod];
    uint8_t ok = 0;
    if (!(p.flags & PF_PREFILTER_FAIL)) {
        uint32_t reasons;
        ok = dev_full_filters(specs[p.spec], p, terms, reqs, hot[node], ext + node, st + node, true, &reasons)
             == CA_PLUGIN_NONE;
    }
    out[(size_t)pod * n + node] = ok;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int ca_abi_version(void) { return CASIM_ABI_VERSION; }

int ca_abi_struct_sizes(int32_t* out, int32_t cap) {
    const int32_t s[] = {(int32_t)sizeof(ca_node_spec), (int32_t)sizeof(ca_pod_spec),
                         (int32_t)sizeof(ca_selector_req), (int32_t)sizeof(ca_selector_term),
                         (int32_t)sizeof(ca_pod_table), (int32_t)sizeof(ca_match_spec),
                         (int32_t)sizeof(ca_pred_result), (int32_t)sizeof(ca_template),
                         (int32_t)sizeof(ca_limiter), (int32_t)sizeof(ca_estimate_result),
                         (int32_t)sizeof(ca_removal_result), (int32_t)sizeof(ca_util_node),
                         (int32_t)sizeof(ca_util_pod), (int32_t)sizeof(ca_util_info),
                         (int32_t)sizeof(ca_plan_result), (int32_t)sizeof(ca_plan_move),
                         (int32_t)sizeof(ca_sweep_phase), (int32_t)sizeof(ca_str_pair), (int32_t)sizeof(ca_taint_str),
                         (int32_t)sizeof(ca_toleration_str), (int32_t)sizeof(ca_port_str),
                         (int32_t)sizeof(ca_requirement_str)};
    const int32_t n = (int32_t)(sizeof s / sizeof s[0]);
    for (int32_t i = 0; i < n && i < cap; i++) out[i] = s[i];
    return n;
}

int ca_device_count(int32_t* out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *out = 0; set_last_error(hipGetErrorString(e)); return CA_EDEVICE; }
    *out = n;
    return CA_OK;
}

// Page-locked blocks handed to callers are cached too (a caller that allocates its result
// buffers per call pays no hipHostMalloc after the first), in a cache separate from the
// library's own staging buffers (HostBuf).  The block sizes are remembered for ca_host_free.
static std::mutex g_host_mu;
static std::unordered_map<void*, size_t>* g_host_sizes = new std::unordered_map<void*, size_t>();   // leaked on purpose

int ca_host_alloc(size_t bytes, void** out) {
    if (!out) return CA_EINVAL;
    *out = nullptr;
    const size_t want = bytes ? bytes : 1;
    size_t got = 0;
    void* p = no_cache() ? nullptr : caller_cache().take(want, -1, got);
    if (!p) {
        got = std::max<size_t>(want, 4096);
        // portable: a caller's result buffer may be written by every device of a ca_multi
        // (each block publishes its slice zero-copy), so it is mapped for all of them
        if (hipHostMalloc(&p, got, hipHostMallocNonCoherent | hipHostMallocPortable) != hipSuccess) {
            set_last_error("hipHostMalloc failed");
            return CA_EDEVICE;
        }
    }
    {
        std::lock_guard<std::mutex> lock(g_host_mu);
        (*g_host_sizes)[p] = got;
    }
    *out = p;
    return CA_OK;
}

int ca_host_free(void* p) {
    if (!p) return CA_OK;
    size_t sz = 0;
    {
        std::lock_guard<std::mutex> lock(g_host_mu);
        auto it = g_host_sizes->find(p);
        if (it == g_host_sizes->end()) { set_last_error("ca_host_free: not a ca_host_alloc block"); return CA_EINVAL; }
        sz = it->second;
        g_host_sizes->erase(it);
    }
    bool kept = false;                  // released through the callers' cache
    if (!no_cache()) {
        sync_device(-1);
        kept = caller_cache().give(sz, -1, p);
    }
    if (!kept) (void)hipHostFree(p);
    return CA_OK;
}

const char* ca_status_string(int status) {
    switch (status) {
    case CA_OK: return "ok";
    case CA_EINVAL: return "invalid argument";
    case CA_ENOTFOUND: return "not found";
    case CA_EEXISTS: return "already exists";
    case CA_EDEVICE: return g_last_error.empty() ? "device error" : g_last_error.c_str();
    case CA_ECAPACITY: return "capacity exceeded";
    case CA_EUNSUPPORTED: return "unsupported by the kernels";
    case CA_ESTATE: return "invalid fork state";
    default: return "unknown status";
    }
}

int ca_mirror_create(int32_t device, ca_mirror** out) {
    if (!out) return CA_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) { set_last_error("no HIP device"); return CA_EDEVICE; }
    if (device < 0 || device >= n) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(device));
    ca_mirror* m = new ca_mirror();
    m->device = device;
    if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&m->ev0) != hipSuccess || hipEventCreate(&m->ev1) != hipSuccess ||
        hipEventCreate(&m->ev2) != hipSuccess) {
        delete m;
        set_last_error("stream/event creation failed");
        return CA_EDEVICE;
    }
    *out = m;
    return CA_OK;
}

int ca_mirror_destroy(ca_mirror* m) {
    if (!m) return CA_EINVAL;
    (void)hipSetDevice(m->device);
    (void)hipStreamSynchronize(m->stream);
    (void)hipEventDestroy(m->ev0); (void)hipEventDestroy(m->ev1); (void)hipEventDestroy(m->ev2);
    (void)hipStreamDestroy(m->stream);
    delete m;
    return CA_OK;
}

int ca_mirror_clear(ca_mirror* m) {
    if (!m) return CA_EINVAL;
    m->n_ext_pods = 0;
    m->n_eph_pods = 0;
    m->n_oos_pods = 0;
    m->nodes.clear(); m->pods.clear(); m->terms.clear(); m->reqs.clear(); m->pf_names.clear();
    m->journal.clear(); m->depth = 0; m->removed_nodes.clear(); m->n_scope_blockers = 0;
    m->dirty_rows.clear(); m->dirty_flag.clear();
    m->all_dirty = true; m->static_dirty = true; m->d_rows = 0;
    m->d_pods_synced = 0; m->d_terms_synced = 0;
    m->d_hints_n = 0;
    return CA_OK;
}

int ca_mirror::ensure_pod_hints() {
    const size_t np = pods.size();
    if (d_hints_n >= np) return CA_OK;
    int rc = d_pod_hints.reserve_keep(sizeof(int32_t) * std::max<size_t>(np, 1), stream);
    if (rc != CA_OK) return rc;
    CA_HIP_CHECK(hipMemsetAsync(d_pod_hints.as<int32_t>() + d_hints_n, 0xFF, sizeof(int32_t) * (np - d_hints_n), stream));
    d_hints_n = np;
    return CA_OK;
}

int ca_mirror_set_hints(ca_mirror* m, const int32_t* hints, int32_t n_pods) {
    if (!m || n_pods != (int32_t)m->pods.size() || (n_pods > 0 && !hints)) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    int rc = m->ensure_pod_hints();
    if (rc != CA_OK) return rc;
    if (n_pods) CA_HIP_CHECK(hipMemcpyAsync(m->d_pod_hints.ptr, hints, sizeof(int32_t) * n_pods, hipMemcpyHostToDevice,
                                            m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    return CA_OK;
}

int ca_mirror_get_hints(ca_mirror* m, int32_t* hints, int32_t n_pods) {
    if (!m || n_pods != (int32_t)m->pods.size() || (n_pods > 0 && !hints)) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    int rc = m->ensure_pod_hints();
    if (rc != CA_OK) return rc;
    if (n_pods) CA_HIP_CHECK(hipMemcpyAsync(hints, m->d_pod_hints.ptr, sizeof(int32_t) * n_pods, hipMemcpyDeviceToHost,
                                            m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    return CA_OK;
}

int ca_mirror_add_nodes(ca_mirror* m, const ca_node_spec* nodes, int32_t n, int32_t* out_first_pos) {
    if (!m || (n > 0 && !nodes) || n < 0) return CA_EINVAL;
    if (out_first_pos) *out_first_pos = (int32_t)m->nodes.size();
    for (int32_t i = 0; i < n; i++) {
        NodeRow r;
        r.spec = nodes[i];
        m->nodes.push_back(std::move(r));
        m->journal_push(J_ADD_NODE, (int32_t)m->nodes.size() - 1, -1, -1, nullptr);
    }
    m->static_dirty = true;
    return CA_OK;
}

int ca_mirror_add_pods(ca_mirror* m, const ca_pod_table* t, const int32_t* pod_idx,
                       const int32_t* node_pos, int32_t n, int32_t* out_ids) {
    if (!m || !t || n < 0) return CA_EINVAL;
    for (int32_t i = 0; i < n; i++) {
        if (node_pos[i] < 0 || (size_t)node_pos[i] >= m->nodes.size()) return CA_ENOTFOUND;
        if (pod_idx[i] < 0 || pod_idx[i] >= t->n_pods) return CA_EINVAL;
        int32_t id = m->store_pod(t, pod_idx[i], node_pos[i]);
        m->add_pod_to_node(id, node_pos[i]);
        if (out_ids) out_ids[i] = id;
    }
    return CA_OK;
}

int ca_mirror_remove_pod(ca_mirror* m, int32_t pod_id) {
    if (!m) return CA_EINVAL;
    if (pod_id < 0 || (size_t)pod_id >= m->pods.size() || m->pods[pod_id].node < 0) return CA_ENOTFOUND;
    const int32_t node = m->pods[pod_id].node;
    NodeRow& nd = m->nodes[node];
    int32_t slot = -1;
    for (size_t i = 0; i < nd.pods.size(); i++) if (nd.pods[i] == pod_id) { slot = (int32_t)i; break; }
    if (slot < 0) return CA_ENOTFOUND;
    uint64_t before[CA_PORT_WORDS];
    std::memcpy(before, nd.ports, sizeof before);
    nd.pods[slot] = nd.pods.back();          // swap-with-last (SF/types.go:660-663)
    nd.pods.pop_back();
    m->node_apply(node, m->pods[pod_id].spec, -1);
    m->pods[pod_id].node = -1;
    m->journal_push(J_REMOVE_POD, node, pod_id, slot, before);
    return CA_OK;
}

int ca_mirror_remove_node(ca_mirror* m, int32_t node_pos) {
    if (!m) return CA_EINVAL;
    if (node_pos < 0 || (size_t)node_pos >= m->nodes.size()) return CA_ENOTFOUND;   // ErrNodeNotFound
    CA_HIP_CHECK(hipSetDevice(m->device));
    NodeRow row = std::move(m->nodes[node_pos]);
    m->nodes.erase(m->nodes.begin() + node_pos);
    for (int32_t id : row.pods) {
        m->pods[id].node = -1;
        if (m->pods[id].spec.flags & CA_POD_REQUIRED_ANTI_AFFINITY) m->n_scope_blockers--;
    }
    for (size_t i = 0; i < m->pods.size(); i++) if (m->pods[i].node > node_pos) m->pods[i].node--;
    // positions moved: every row is re-uploaded before the next kernel
    m->dirty_rows.clear();
    m->dirty_flag.assign(m->nodes.size(), 0);
    m->all_dirty = true;
    m->static_dirty = true;
    if (m->d_rows > m->nodes.size()) m->d_rows = m->nodes.size();
    const int32_t code = -2 - (m->removals++ & 0x3FFFFFFF);     // this removal's hint code
    int rc = m->remap_hints_removed(node_pos, code, false);
    if (rc != CA_OK) return rc;
    if (m->depth > 0) {
        JournalEntry e;
        std::memset(&e, 0, sizeof e);
        e.kind = J_REMOVE_NODE; e.node = node_pos; e.pod = code; e.slot = (int32_t)m->removed_nodes.size();
        m->journal.push_back(e);
        m->removed_nodes.push_back(std::move(row));
    }
    return CA_OK;
}

int ca_mirror_scope_blockers(const ca_mirror* m, int32_t* out_n) {
    if (!m || !out_n) return CA_EINVAL;
    *out_n = (int32_t)m->n_scope_blockers;
    return CA_OK;
}

int ca_mirror_fork(ca_mirror* m) {
    if (!m) return CA_EINVAL;
    m->depth++;
    m->journal_push(J_FORK, -1, -1, -1, nullptr);
    return CA_OK;
}

int ca_mirror_revert(ca_mirror* m) {
    if (!m) return CA_EINVAL;
    if (m->depth == 0) return CA_ESTATE;
    while (!m->journal.empty()) {
        JournalEntry e = m->journal.back();
        m->journal.pop_back();
        if (e.kind == J_FORK) break;
        if (e.kind == J_ADD_NODE) {
            m->nodes.pop_back();
            if (m->d_rows > m->nodes.size()) m->d_rows = m->nodes.size();
            if (m->dirty_flag.size() > m->nodes.size()) m->dirty_flag.resize(m->nodes.size());
            m->dirty_rows.erase(std::remove_if(m->dirty_rows.begin(), m->dirty_rows.end(),
                                               [&](int32_t r) { return (size_t)r >= m->nodes.size(); }),
                                m->dirty_rows.end());
            m->static_dirty = true;
        } else if (e.kind == J_ADD_POD) {
            m->node_apply(e.node, m->pods[e.pod].spec, -1);
            std::memcpy(m->nodes[e.node].ports, e.ports, sizeof e.ports);
            m->nodes[e.node].pods.pop_back();
            m->pods[e.pod].node = -1;
        } else if (e.kind == J_REMOVE_POD) {
            NodeRow& nd = m->nodes[e.node];
            m->node_apply(e.node, m->pods[e.pod].spec, +1);
            std::memcpy(nd.ports, e.ports, sizeof e.ports);
            nd.pods.push_back(nd.pods[e.slot]);
            nd.pods[e.slot] = e.pod;
            m->pods[e.pod].node = e.node;
        } else if (e.kind == J_REMOVE_NODE) {
            const int32_t pos = e.node;
            for (size_t i = 0; i < m->pods.size(); i++) if (m->pods[i].node >= pos) m->pods[i].node++;
            m->nodes.insert(m->nodes.begin() + pos, std::move(m->removed_nodes.back()));
            m->removed_nodes.pop_back();
            for (int32_t id : m->nodes[pos].pods) {
                m->pods[id].node = pos;
                if (m->pods[id].spec.flags & CA_POD_REQUIRED_ANTI_AFFINITY) m->n_scope_blockers++;
            }
            m->dirty_rows.clear();
            m->dirty_flag.assign(m->nodes.size(), 0);
            m->all_dirty = true;
            m->static_dirty = true;
            int rc = m->remap_hints_removed(pos, e.pod, true);
            if (rc != CA_OK) return rc;
        }
    }
    m->depth--;
    return CA_OK;
}

int ca_mirror_commit(ca_mirror* m) {
    if (!m) return CA_EINVAL;
    if (m->depth == 0) return CA_ESTATE;
    int64_t i = (int64_t)m->journal.size() - 1;
    while (i >= 0 && m->journal[i].kind != J_FORK) i--;
    if (i < 0) return CA_ESTATE;
    m->depth--;
    if (m->depth == 0) {
        m->journal.clear();
        m->removed_nodes.clear();            // committed removals are permanent
    } else {
        m->journal.erase(m->journal.begin() + i);
    }
    return CA_OK;
}

int ca_mirror_node_count(const ca_mirror* m, int32_t* out) {
    if (!m || !out) return CA_EINVAL;
    *out = (int32_t)m->nodes.size();
    return CA_OK;
}

int ca_mirror_pod_node(const ca_mirror* m, int32_t pod_id, int32_t* out_node_pos) {
    if (!m || !out_node_pos) return CA_EINVAL;
    if (pod_id < 0 || (size_t)pod_id >= m->pods.size()) return CA_ENOTFOUND;
    *out_node_pos = m->pods[pod_id].node;
    return CA_OK;
}

int ca_mirror_node_pods(const ca_mirror* m, int32_t node_pos, int32_t* out_ids, int32_t cap, int32_t* out_n) {
    if (!m || !out_n) return CA_EINVAL;
    if (node_pos < 0 || (size_t)node_pos >= m->nodes.size()) return CA_ENOTFOUND;
    const auto& v = m->nodes[node_pos].pods;
    *out_n = (int32_t)v.size();
    if ((int32_t)v.size() > cap) return CA_ECAPACITY;
    for (size_t i = 0; i < v.size(); i++) out_ids[i] = v[i];
    return CA_OK;
}

int ca_podset_create(ca_mirror* m, const ca_pod_table* t, ca_podset** out) {
    if (!m || !t || !out || t->n_pods < 0) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    const auto t0 = std::chrono::steady_clock::now();
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    auto tmark = [&](const char* what) {
        if (dbg_t)
            fprintf(stderr, "[podset] %-10s %8.3f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    ca_podset* s = new ca_podset();
    s->m = m;
    s->n_host = t->n_pods;
    s->h_req.resize(2 * (size_t)t->n_pods);
    s->h_pflags.assign((size_t)t->n_pods, 0);
    for (int32_t i = 0; i < t->n_pods; i++) {
        const ca_pod_spec& ps = t->pods[i];
        s->any_oos |= (ps.flags & CA_POD_OUT_OF_SCOPE) != 0;
        s->any_refs |= ps.aff_term_count > 0 || ((ps.flags & CA_POD_PREFILTER_NAMES) && ps.prefilter_count > 0);
        s->h_req[2 * (size_t)i] = ps.req_milli_cpu;
        s->h_req[2 * (size_t)i + 1] = ps.req_memory;
        const uint32_t f = pod_dev_flags(ps);
        const uint8_t b = (uint8_t)(((f & PF_PORTS) ? 1 : 0) | ((f & PF_SCALAR_REQ) ? 2 : 0));
        s->h_pflags[i] = b;
        s->any_ports |= (b & 1) != 0;
        s->any_scalar |= (b & 2) != 0;
    }
    tmark("flags");
    // the records' copies stay queued while the score classes are worked out below; the
    // creation ends with one sync (a pod set is immutable and complete once created)
    int rc = s->t.upload_staged(t->pods, t->n_pods, t->terms, t->n_terms, t->reqs, t->n_reqs, t->prefilter_names,
                                t->n_prefilter_names, m->podset_stage, m->stream);
    if (rc != CA_OK) { (void)hipStreamSynchronize(m->stream); delete s; return rc; }
    tmark("uploaded");
    {   // score classes
        struct PairHash {
            size_t operator()(const std::pair<int64_t, int64_t>& k) const {
                return std::hash<int64_t>()(k.first * 0x9E3779B97F4A7C15ll ^ k.second);
            }
        };
        std::unordered_map<std::pair<int64_t, int64_t>, int32_t, PairHash> ids;
        std::vector<int32_t> cls((size_t)t->n_pods);
        std::vector<int64_t> sc;
        for (int32_t i = 0; i < t->n_pods; i++) {
            const auto key = std::make_pair(t->pods[i].score_milli_cpu, t->pods[i].score_memory);
            auto it = ids.find(key);
            if (it == ids.end()) {
                it = ids.emplace(key, (int32_t)ids.size()).first;
                sc.push_back(key.first);
                sc.push_back(key.second);
            }
            cls[i] = it->second;
        }
        s->n_cls = (int32_t)ids.size();
        {   // class uniformity (ca_podset::cls_uniform)
            std::vector<int32_t> first((size_t)s->n_cls, -1);
            bool uni = true;
            for (int32_t i = 0; i < t->n_pods && uni; i++) {
                int32_t& f = first[cls[i]];
                if (f < 0) { f = i; continue; }
                ca_pod_spec a = t->pods[f], b = t->pods[i];
                a.similar_class = b.similar_class = 0;
                uni = std::memcmp(&a, &b, sizeof a) == 0;
            }
            s->cls_uniform = uni;
        }
        s->h_cls = cls;
        s->h_cls_sc = sc;
        std::vector<int32_t> rep((size_t)std::max(s->n_cls, 1), 0);
        for (int32_t i = t->n_pods - 1; i >= 0; i--) rep[cls[i]] = i;
        if ((rc = s->d_cls_rep.reserve(sizeof(int32_t) * rep.size())) != CA_OK) { (void)hipStreamSynchronize(m->stream); delete s; return rc; }
        CA_HIP_CHECK(hipMemcpyAsync(s->d_cls_rep.ptr, rep.data(), sizeof(int32_t) * rep.size(), hipMemcpyHostToDevice,
                                    m->stream));
        if ((rc = s->d_cls.reserve(sizeof(int32_t) * (cls.size() + 1))) != CA_OK ||
            (rc = s->d_cls_sc.reserve(sizeof(int64_t) * (sc.size() + 2))) != CA_OK) { (void)hipStreamSynchronize(m->stream); delete s; return rc; }
        if (!cls.empty())
            CA_HIP_CHECK(hipMemcpyAsync(s->d_cls.ptr, cls.data(), sizeof(int32_t) * cls.size(), hipMemcpyHostToDevice,
                                        m->stream));
        if (!sc.empty())
            CA_HIP_CHECK(hipMemcpyAsync(s->d_cls_sc.ptr, sc.data(), sizeof(int64_t) * sc.size(), hipMemcpyHostToDevice,
                                        m->stream));
        CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    }
    tmark("classes");
    *out = s;
    return CA_OK;
}

int ca_podset_destroy(ca_podset* s) {
    if (!s) return CA_EINVAL;
    delete s;
    return CA_OK;
}

int ca_fits_any_node(ca_mirror* m, const ca_pod_table* t, int32_t pod, const ca_match_spec* match,
                     int32_t* last_index, int32_t* out_node, int32_t* out_prefilter_failed, uint64_t* evals) {
    if (!m || !t || !last_index || !out_node || pod < 0 || pod >= t->n_pods) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    *out_node = -1;
    if (out_prefilter_failed) *out_prefilter_failed = 0;
    const ca_pod_spec& ps = t->pods[pod];
    if ((ps.flags & CA_POD_OUT_OF_SCOPE) || m->n_scope_blockers > 0) return CA_EUNSUPPORTED;   // casim.h scope
    if (ps.flags & CA_POD_PREFILTER_FAIL) {                 // schedulerbased.go:109-112
        if (out_prefilter_failed) *out_prefilter_failed = 1;
        return CA_OK;
    }
    const int32_t n = (int32_t)m->nodes.size();
    if (n == 0) return CA_OK;
    int rc;
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    // single-pod table on device (pod record + its selector tables)
    ca_pod_spec one = ps;
    std::vector<ca_selector_term> tms;
    std::vector<ca_selector_req> rqs;
    std::vector<int32_t> nms;
    if (one.aff_term_count > 0) {
        for (int32_t k = 0; k < one.aff_term_count; k++) {
            ca_selector_term tm = t->terms[one.aff_term_first + k];
            int32_t rf = (int32_t)rqs.size();
            for (int32_t r = 0; r < tm.count; r++) rqs.push_back(t->reqs[tm.first + r]);
            tm.first = rf;
            tms.push_back(tm);
        }
        one.aff_term_first = 0;
    }
    if ((one.flags & CA_POD_PREFILTER_NAMES) && one.prefilter_count > 0) {
        for (int32_t k = 0; k < one.prefilter_count; k++) nms.push_back(t->prefilter_names[one.prefilter_first + k]);
        one.prefilter_first = 0;
    }
    DevPodTable dp;
    if ((rc = dp.upload(&one, 1, tms.data(), (int32_t)tms.size(), rqs.data(), (int32_t)rqs.size(), nms.data(),
                        (int32_t)nms.size(), m->stream)) != CA_OK)
        return rc;
    const int32_t kind = match ? match->kind : CA_MATCH_ALL;
    const uint8_t* dmask = nullptr;
    if (kind == CA_MATCH_MASK) {
        if (!match->mask) return CA_EINVAL;
        if ((rc = m->d_mask.reserve((size_t)n)) != CA_OK) return rc;
        CA_HIP_CHECK(hipMemcpyAsync(m->d_mask.ptr, match->mask, (size_t)n, hipMemcpyHostToDevice, m->stream));
        dmask = m->d_mask.as<uint8_t>();
    }
    const int32_t words = (n + 63) / 64;
    if ((rc = m->d_scratch0.reserve(sizeof(unsigned long long) * 2 * (size_t)words)) != CA_OK) return rc;
    unsigned long long* dfit = m->d_scratch0.as<unsigned long long>();
    unsigned long long* dvis = dfit + words;
    const int64_t L = (int64_t)((uint32_t)*last_index % (uint32_t)n);   // (lastIndex+i)%len
    hipLaunchKernelGGL(k_fits_scan, dim3((n + 255) / 256), dim3(256), 0, m->stream, m->d_hot.as<NodeHot>(),
                       m->d_ext.as<NodeExt>(), m->d_static.as<NodeStatic>(), n, dp.hot.as<PodHot>(),
                       dp.spec.as<ca_pod_spec>(), dp.terms.as<ca_selector_term>(), dp.reqs.as<ca_selector_req>(),
                       dp.names.as<int32_t>(), 0, L, kind, match ? match->lo : 0, match ? match->hi : 0,
                       match ? match->exclude : -1, dmask, dfit, dvis);
    CA_HIP_CHECK(hipGetLastError());
    std::vector<unsigned long long> h((size_t)words * 2);
    CA_HIP_CHECK(hipMemcpyAsync(h.data(), dfit, sizeof(unsigned long long) * 2 * words, hipMemcpyDeviceToHost, m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    // first fit in rotated order; evals = visited nodes up to and including it
    uint64_t ev = 0;
    for (int32_t w = 0; w < words; w++) {
        const unsigned long long f = h[w], v = h[words + w];
        if (f) {
            const int b = __builtin_ctzll(f);
            const unsigned long long below = (b == 63) ? ~0ull : ((2ull << b) - 1);
            ev += (uint64_t)__builtin_popcountll(v & below);
            const int64_t i = (int64_t)w * 64 + b;
            *out_node = (int32_t)((L + i) % n);
            *last_index = (int32_t)((L + i + 1) % n);     // schedulerbased.go:131
            if (evals) *evals += ev;
            return CA_OK;
        }
        ev += (uint64_t)__builtin_popcountll(v);
    }
    if (evals) *evals += ev;
    return CA_OK;
}

int ca_check_predicates(ca_mirror* m, const ca_pod_table* t, int32_t pod, int32_t node_pos, ca_pred_result* out) {
    if (!m || !t || !out || pod < 0 || pod >= t->n_pods) return CA_EINVAL;
    std::memset(out, 0, sizeof *out);
    if ((t->pods[pod].flags & CA_POD_OUT_OF_SCOPE) || m->n_scope_blockers > 0) return CA_EUNSUPPORTED;
    if (node_pos < 0 || (size_t)node_pos >= m->nodes.size()) {   // schedulerbased.go:143-147
        out->type = CA_PRED_INTERNAL;
        return CA_OK;
    }
    const ca_pod_spec& ps = t->pods[pod];
    if ((ps.flags & CA_POD_OUT_OF_SCOPE) || m->n_scope_blockers > 0) return CA_EUNSUPPORTED;   // casim.h scope
    if (ps.flags & CA_POD_PREFILTER_FAIL) {                       // :153-161
        out->type = CA_PRED_INTERNAL;
        out->plugin = CA_PLUGIN_NODE_AFFINITY;
        return CA_OK;
    }
    CA_HIP_CHECK(hipSetDevice(m->device));
    int rc;
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    ca_pod_spec one = ps;
    std::vector<ca_selector_term> tms;
    std::vector<ca_selector_req> rqs;
    if (one.aff_term_count > 0) {
        for (int32_t k = 0; k < one.aff_term_count; k++) {
            ca_selector_term tm = t->terms[one.aff_term_first + k];
            int32_t rf = (int32_t)rqs.size();
            for (int32_t r = 0; r < tm.count; r++) rqs.push_back(t->reqs[tm.first + r]);
            tm.first = rf;
            tms.push_back(tm);
        }
        one.aff_term_first = 0;
    }
    DevPodTable dp;
    if ((rc = dp.upload(&one, 1, tms.data(), (int32_t)tms.size(), rqs.data(), (int32_t)rqs.size(), nullptr, 0,
                        m->stream)) != CA_OK)
        return rc;
    if ((rc = m->d_scratch1.reserve(sizeof(ca_pred_result))) != CA_OK) return rc;
    hipLaunchKernelGGL(k_check_one, dim3(1), dim3(64), 0, m->stream, m->d_hot.as<NodeHot>(), m->d_ext.as<NodeExt>(),
                       m->d_static.as<NodeStatic>(), dp.hot.as<PodHot>(), dp.spec.as<ca_pod_spec>(),
                       dp.terms.as<ca_selector_term>(), dp.reqs.as<ca_selector_req>(), 0, node_pos,
                       m->d_scratch1.as<ca_pred_result>());
    CA_HIP_CHECK(hipGetLastError());
    CA_HIP_CHECK(hipMemcpyAsync(out, m->d_scratch1.ptr, sizeof(ca_pred_result), hipMemcpyDeviceToHost, m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    return CA_OK;
}

int ca_fits_matrix(ca_mirror* m, const ca_podset* s, uint8_t* out) {
    if (!m || !s || !out) return CA_EINVAL;
    CA_HIP_CHECK(hipSetDevice(m->device));
    int rc;
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    const int32_t n = (int32_t)m->nodes.size();
    const int32_t P = s->t.n_pods;
    if (m->n_scope_blockers > 0) return CA_EUNSUPPORTED;
    if (s->any_oos) return CA_EUNSUPPORTED;
    if (n == 0 || P == 0) return CA_OK;
    const size_t bytes = (size_t)n * (size_t)P;
    if ((rc = m->d_scratch2.reserve(bytes)) != CA_OK) return rc;
    hipLaunchKernelGGL(k_fits_matrix, dim3((n + 255) / 256, P), dim3(256), 0, m->stream, m->d_hot.as<NodeHot>(),
                       m->d_ext.as<NodeExt>(), m->d_static.as<NodeStatic>(), n, s->t.hot.as<PodHot>(),
                       s->t.spec.as<ca_pod_spec>(), s->t.terms.as<ca_selector_term>(), s->t.reqs.as<ca_selector_req>(),
                       P, m->d_scratch2.as<uint8_t>());
    CA_HIP_CHECK(hipGetLastError());
    CA_HIP_CHECK(hipMemcpyAsync(out, m->d_scratch2.ptr, bytes, hipMemcpyDeviceToHost, m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    return CA_OK;
}

}  // extern "C"

namespace {
// The test node of a node group (NodeInfo of a fresh template copy: the template with its pods)
void template_test_rows(const ca_template* templates, int32_t G, NodeHot* h, NodeExt* x, NodeStatic* st) {
    for (int32_t g = 0; g < G; g++) {
        const ca_template& tp = templates[g];
        const ca_node_spec& n = tp.node;
        h[g].cpu = wsub(n.alloc_milli_cpu, tp.used_milli_cpu);
        h[g].mem = wsub(n.alloc_memory, tp.used_memory);
        h[g].eph = wsub(n.alloc_ephemeral, tp.used_ephemeral);
        h[g].pods = clamp_i32(n.alloc_pods - tp.used_pods);
        uint32_t f = NF_VALID;
        if (n.flags & CA_NODE_UNSCHEDULABLE) f |= NF_UNSCHED;
        if (n.taints) f |= NF_TAINTS;
        bool ports = false, sc = false;
        for (int w = 0; w < CA_PORT_WORDS; w++) { x[g].ports[w] = tp.used_ports[w]; ports |= tp.used_ports[w] != 0; }
        for (int k = 0; k < CA_MAX_SCALAR; k++) {
            x[g].scalar[k] = wsub(n.alloc_scalar[k], tp.used_scalar[k]);
            sc |= n.alloc_scalar[k] != 0 || tp.used_scalar[k] != 0;
        }
        if (ports) f |= NF_PORTS;
        if (sc) f |= NF_SCALAR;
        if (n.flags & CA_NODE_ANTI_AFFINITY_PODS) f |= NF_OUT_OF_SCOPE;
        h[g].flags = f;
        std::memset(&st[g], 0, sizeof st[g]);
        st[g].taints = n.taints;
        for (int w = 0; w < CA_LABEL_WORDS; w++) st[g].labels[w] = n.label_pairs[w];
        st[g].keys = n.label_keys;
        for (int k = 0; k < CA_MAX_INT_KEYS; k++) st[g].ints[k] = n.int_label[k];
        st[g].int_valid = n.int_label_valid;
        st[g].name_id = n.name_id;
    }
}

int check_samples(const ca_mirror* m, const ca_podset* s, const int32_t* samples, int32_t n_samples) {
    for (int32_t e = 0; e < n_samples; e++)
        if (samples[e] < 0 || samples[e] >= s->t.n_pods) return CA_EINVAL;
    if (m->n_scope_blockers > 0) return CA_EUNSUPPORTED;
    return CA_OK;
}
}  // namespace

// Node groups resident for ComputeExpansionOption checks (ca_expansion_plan_*): the
// templates' test-node rows stay in HBM; a run passes samples and results through
// page-locked memory the kernel reads and writes in place.
struct ca_expansion_plan {
    ca_mirror* m = nullptr;
    int32_t G = 0;
    casim::DevBuf rows;        // NodeHot[G] | NodeExt[G] | NodeStatic[G]
    casim::HostBuf io;         // page-locked: samples | results | verdicts
    float kernel_ms = 0;       // the last run's kernel (events)
    // The check reads only the plan's rows and the podset's tables, both immutable once
    // their create call returned (each ends with a sync): it runs on a stream of its own, so
    // it neither waits behind nor holds up work queued on the mirror's stream (after
    // FilterOutSchedulable: the placed pods' record gather).
    hipStream_t st = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    void* io_host = nullptr;   // io.ptr when io_dev was looked up (a grown io re-queries)
    char* io_dev = nullptr;    // io's device mapping
    ~ca_expansion_plan() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (st) (void)hipStreamDestroy(st);
    }
};

extern "C" {

int ca_check_templates(ca_mirror* m, const ca_podset* s, const int32_t* samples, int32_t n_samples,
                       const ca_template* templates, int32_t n_templates, ca_pred_result* out, uint8_t* out_ok) {
    if (!m || !s || n_samples < 0 || n_templates < 0) return CA_EINVAL;
    if (n_samples == 0 || n_templates == 0) return CA_OK;
    if (!samples || !templates || (!out && !out_ok)) return CA_EINVAL;
    int rc;
    if ((rc = check_samples(m, s, samples, n_samples)) != CA_OK) return rc;
    CA_HIP_CHECK(hipSetDevice(m->device));
    std::vector<NodeHot> h(n_templates);
    std::vector<NodeExt> x(n_templates);
    std::vector<NodeStatic> st(n_templates);
    template_test_rows(templates, n_templates, h.data(), x.data(), st.data());
    const size_t nh = sizeof(NodeHot) * n_templates, nx = sizeof(NodeExt) * n_templates,
                 ns = sizeof(NodeStatic) * n_templates, nsm = sizeof(int32_t) * n_samples,
                 no = out ? sizeof(ca_pred_result) * (size_t)n_templates * (size_t)n_samples : 0,
                 nok = out_ok ? (size_t)n_templates * (size_t)n_samples : 0;
    if ((rc = m->d_scratch2.reserve(nh + nx + ns + nsm + no + nok + 64)) != CA_OK) return rc;
    char* base = m->d_scratch2.as<char>();
    NodeHot* dh = reinterpret_cast<NodeHot*>(base);
    NodeExt* dx = reinterpret_cast<NodeExt*>(base + nh);
    NodeStatic* ds = reinterpret_cast<NodeStatic*>(base + nh + nx);
    int32_t* dsm = reinterpret_cast<int32_t*>(base + nh + nx + ns);
    const size_t o_out = (nh + nx + ns + nsm + 15) & ~size_t(15);
    ca_pred_result* dout = out ? reinterpret_cast<ca_pred_result*>(base + o_out) : nullptr;
    uint8_t* dok = out_ok ? reinterpret_cast<uint8_t*>(base + o_out + no) : nullptr;
    CA_HIP_CHECK(hipMemcpyAsync(dh, h.data(), nh, hipMemcpyHostToDevice, m->stream));
    CA_HIP_CHECK(hipMemcpyAsync(dx, x.data(), nx, hipMemcpyHostToDevice, m->stream));
    CA_HIP_CHECK(hipMemcpyAsync(ds, st.data(), ns, hipMemcpyHostToDevice, m->stream));
    CA_HIP_CHECK(hipMemcpyAsync(dsm, samples, nsm, hipMemcpyHostToDevice, m->stream));
    hipLaunchKernelGGL(k_check_templates, dim3((n_samples + 255) / 256, n_templates), dim3(256), 0, m->stream,
                       dh, dx, ds, dsm, n_samples, s->t.hot.as<PodHot>(), s->t.spec.as<ca_pod_spec>(),
                       s->t.terms.as<ca_selector_term>(), s->t.reqs.as<ca_selector_req>(), dout, dok);
    CA_HIP_CHECK(hipGetLastError());
    if (out) CA_HIP_CHECK(hipMemcpyAsync(out, dout, no, hipMemcpyDeviceToHost, m->stream));
    if (out_ok) CA_HIP_CHECK(hipMemcpyAsync(out_ok, dok, nok, hipMemcpyDeviceToHost, m->stream));
    CA_HIP_CHECK(hipStreamSynchronize(m->stream));
    return CA_OK;
}

int ca_expansion_plan_create(ca_mirror* m, const ca_template* templates, int32_t n_templates,
                             ca_expansion_plan** out) {
    if (!m || !out || n_templates < 0 || (n_templates > 0 && !templates)) return CA_EINVAL;
    *out = nullptr;
    CA_HIP_CHECK(hipSetDevice(m->device));
    auto* p = new ca_expansion_plan();
    p->m = m;
    p->G = n_templates;
    const size_t G = (size_t)std::max(n_templates, 1);
    const size_t nh = sizeof(NodeHot) * G, nx = sizeof(NodeExt) * G, ns = sizeof(NodeStatic) * G;
    int rc;
    if ((rc = p->rows.reserve(nh + nx + ns)) != CA_OK) { delete p; return rc; }
    if (n_templates > 0) {
        std::vector<NodeHot> h(G);
        std::vector<NodeExt> x(G);
        std::vector<NodeStatic> st(G);
        template_test_rows(templates, n_templates, h.data(), x.data(), st.data());
        char* base = p->rows.as<char>();
        if (hipMemcpyAsync(base, h.data(), nh, hipMemcpyHostToDevice, m->stream) != hipSuccess ||
            hipMemcpyAsync(base + nh, x.data(), nx, hipMemcpyHostToDevice, m->stream) != hipSuccess ||
            hipMemcpyAsync(base + nh + nx, st.data(), ns, hipMemcpyHostToDevice, m->stream) != hipSuccess ||
            hipStreamSynchronize(m->stream) != hipSuccess) {
            delete p;
            set_last_error("ca_expansion_plan_create: template upload failed");
            return CA_EDEVICE;
        }
    }
    if (hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&p->ev0) != hipSuccess || hipEventCreate(&p->ev1) != hipSuccess) {
        delete p;
        set_last_error("ca_expansion_plan_create: stream / event creation failed");
        return CA_EDEVICE;
    }
    *out = p;
    return CA_OK;
}

int ca_expansion_plan_run(ca_expansion_plan* p, const ca_podset* s, const int32_t* samples, int32_t n_samples,
                          ca_pred_result* out, uint8_t* out_ok) {
    if (!p || !s || s->m != p->m || n_samples < 0) return CA_EINVAL;
    if (n_samples == 0 || p->G == 0) return CA_OK;
    if (!samples || (!out && !out_ok)) return CA_EINVAL;
    const auto t_entry = std::chrono::steady_clock::now();
    ca_mirror* m = p->m;
    int rc;
    if ((rc = check_samples(m, s, samples, n_samples)) != CA_OK) return rc;
    CA_HIP_CHECK(hipSetDevice(m->device));
    const size_t pairs = (size_t)p->G * (size_t)n_samples;
    const size_t nsm = (sizeof(int32_t) * (size_t)n_samples + 63) & ~(size_t)63;
    const size_t no = out ? ((sizeof(ca_pred_result) * pairs + 63) & ~(size_t)63) : 0;
    const size_t nok = out_ok ? pairs : 0;
    if ((rc = p->io.reserve(nsm + no + nok)) != CA_OK) return rc;
    // the samples are read and the results written in page-locked memory through its
    // device mapping: no copy-engine round trips for a call of a few kilobytes
    char* hio = p->io.as<char>();
    std::memcpy(hio, samples, sizeof(int32_t) * (size_t)n_samples);
    if (p->io_host != p->io.ptr) {
        void* dio_v = nullptr;
        CA_HIP_CHECK(hipHostGetDevicePointer(&dio_v, p->io.ptr, 0));
        p->io_dev = static_cast<char*>(dio_v);
        p->io_host = p->io.ptr;
    }
    char* dio = p->io_dev;
    // a page-locked output of the caller's (ca_host_alloc) takes large results straight from
    // the kernel; below 256 KiB the results land in the plan's own buffer and one memcpy moves
    // them (cheaper than the runtime's pointer lookup)
    auto mapped = [](void* h, size_t bytes) -> char* {
        if (!h || bytes < ((size_t)256 << 10)) return nullptr;
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, h) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer)
            return static_cast<char*>(at.devicePointer);
        (void)hipGetLastError();
        return nullptr;
    };
    char* d_out = out ? mapped(out, sizeof(ca_pred_result) * pairs) : nullptr;
    char* d_ok = out_ok ? mapped(out_ok, pairs) : nullptr;
    const auto t_mapped = std::chrono::steady_clock::now();
    const size_t G = (size_t)p->G;
    const char* rows = p->rows.as<const char>();
    CA_HIP_CHECK(hipEventRecord(p->ev0, p->st));
    hipLaunchKernelGGL(k_check_templates, dim3((n_samples + 255) / 256, p->G), dim3(256), 0, p->st,
                       reinterpret_cast<const NodeHot*>(rows),
                       reinterpret_cast<const NodeExt*>(rows + sizeof(NodeHot) * G),
                       reinterpret_cast<const NodeStatic*>(rows + (sizeof(NodeHot) + sizeof(NodeExt)) * G),
                       reinterpret_cast<const int32_t*>(dio), n_samples, s->t.hot.as<PodHot>(),
                       s->t.spec.as<ca_pod_spec>(), s->t.terms.as<ca_selector_term>(), s->t.reqs.as<ca_selector_req>(),
                       out ? reinterpret_cast<ca_pred_result*>(d_out ? d_out : dio + nsm) : nullptr,
                       out_ok ? reinterpret_cast<uint8_t*>(d_ok ? d_ok : dio + nsm + no) : nullptr);
    CA_HIP_CHECK(hipGetLastError());
    CA_HIP_CHECK(hipEventRecord(p->ev1, p->st));
    const auto t_launched = std::chrono::steady_clock::now();
    CA_HIP_CHECK(hipStreamSynchronize(p->st));
    CA_HIP_CHECK(hipEventElapsedTime(&p->kernel_ms, p->ev0, p->ev1));
    if (knob_env("CASIM_DEBUG_TIMING")) {
        const auto t_done = std::chrono::steady_clock::now();
        fprintf(stderr, "[expansion] mapped %.3f ms, launched %.3f ms, synced %.3f ms, kernel %.3f ms (%d x %d)\n",
                std::chrono::duration<double, std::milli>(t_mapped - t_entry).count(),
                std::chrono::duration<double, std::milli>(t_launched - t_entry).count(),
                std::chrono::duration<double, std::milli>(t_done - t_entry).count(), p->kernel_ms, p->G, n_samples);
    }
    if (out && !d_out) std::memcpy(out, hio + nsm, sizeof(ca_pred_result) * pairs);
    if (out_ok && !d_ok) std::memcpy(out_ok, hio + nsm + no, pairs);
    return CA_OK;
}

int ca_expansion_plan_kernel_ms(const ca_expansion_plan* p, float* kernel_ms) {
    if (!p || !kernel_ms) return CA_EINVAL;
    *kernel_ms = p->kernel_ms;
    return CA_OK;
}

int ca_expansion_plan_destroy(ca_expansion_plan* p) {
    if (!p) return CA_EINVAL;
    if (p->m) (void)hipSetDevice(p->m->device);
    delete p;
    return CA_OK;
}

}  // extern "C"
