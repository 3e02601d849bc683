// plan_chain.hip — the planner's committing candidate loop as one device-resident chain
// (Planner.categorizeNodes with canPersist = true).
//
// Reference: CA/core/scaledown/planner/planner.go:252-296 (the loop over unneeded nodes,
// podDestinations shrinking by every removal), CA/simulator/cluster.go:145-254
// (SimulateNodeRemoval, withForkedSnapshot + Commit, findPlaceFor: RemovePod of the pods to
// move, TrySchedulePods with breakOnFailure), CA/simulator/scheduling/hinting_simulator.go:58-125
// (hints first, then FitsAnyNodeMatching), CA/simulator/predicatechecker/schedulerbased.go:90-185
// (the rotating first-fit scan and lastIndex), CA/simulator/drain.go:73-90 + CA/core/scaledown/
// pdb/basic.go:58-95 (checkPdbs against the remaining budgets, CanRemovePods, RemovePods).
//
// The loop is strictly sequential: every candidate reads the snapshot its predecessors
// committed.  One wavefront walks all candidates in order with the committed node rows
// resident in LDS (free cpu / memory / ephemeral storage / pod slots, plus bit planes for
// podDestinations, schedulability, taints), so a pod's hint check and its scan touch only
// LDS: a 64-node block per step, blocks whose maxima the pod exceeds skipped 64 at a time.
// A candidate's simulation applies its RemovePods and AddPods to the rows in place; a
// failed candidate undoes them (Revert), a removable one keeps them (Commit) and appends its
// moved copies to the destination nodes' pod lists (which a later candidate on such a node
// must move too).  No host round trip per candidate or per conflict: one launch runs the
// whole loop, and the host replays the committed moves into the mirror's journal afterwards.
//
// Scope of the chain (planner.hip falls back to the speculative sweep windows otherwise):
// the node rows fit in LDS, and no pod to move has host ports or extended-resource requests
// (the only filters whose node state is not a resource column).
#include "mirror.h"

#include <algorithm>
#include <chrono>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <cstdio>

namespace casim {

constexpr int PC_LIST = CA_MAX_MOVED_PODS;   // pods to move per candidate (larger: prefix cut)
constexpr size_t PC_LDS_MAX = 163840;         // gfx950: one workgroup may own the CU's 160 KiB
constexpr int32_t PC_MAX_NODES = 8192;        // two 64-bit words of per-block dirty bits
#ifndef CASIM_PC_MVBUF
#define CASIM_PC_MVBUF 512
#endif
constexpr int32_t PC_MVBUF = CASIM_PC_MVBUF;  // moves staged in LDS between global writes
constexpr int PC_MAX_WAVES = 8;               // the chain wave + up to 7 helper waves (VGPR budget: 2 waves / SIMD)
// shader-clock counters of the chain's phases (info[4 + k]; CASIM_PROF builds only)
enum { PC_INIT, PC_LISTS, PC_PDB, PC_FORK, PC_HINT, PC_SCAN, PC_ADD, PC_COMMIT, PC_REVERT, PC_TOTAL, PC_BLOCKS,
       PC_WINDOWS, PC_HANDOFFS, PC_BULK, PC_PREP, PC_WIN, PC_LOADCHK, PC_SKYB,
       PC_R_POD, PC_R_WIN, PC_R_BLK, PC_R_SKY, PC_R_ADD, PC_R_NPODS, PC_R_NBLK, PC_R_NWIN, PC_R_NSKY, PC_R_NRUNS,
       PC_NPROF };
constexpr int PC_INFO = 4 + PC_NPROF + 3;     // int64 words of the kernel's info record
#ifdef CASIM_PROF
#define PC_T0() uint64_t tp_ = clock64()
#define PC_MARK(k) do { const uint64_t t_ = clock64(); prof[k] += t_ - tp_; tp_ = t_; } while (0)
#define PC_COUNT(k) (prof[k]++)
#else
#define PC_T0() do {} while (0)
#define PC_MARK(k) do {} while (0)
#define PC_COUNT(k) do {} while (0)
#endif

// One pod to move, as the chain reads it: requests, flags after the move (NodeName and TPU
// requests cleared), the hint it carries in, its record and its caller pod (PDBs).
struct alignas(16) PcPod {
    int64_t cpu, mem, eph;
    int32_t id, hint;
    uint32_t flags;
    int32_t spec, orig, pad;
};
static_assert(sizeof(PcPod) == 48, "PcPod");

struct PcArgs {
    const NodeHot* hot;
    const NodeStatic* st;
    int32_t n;
    const uint8_t* dest_mask;
    const int32_t* cands;
    const int32_t* status;
    const int32_t* move_off;
    const PcPod* pods;            // the caller's pods to move, packed in list order (+64 padding)
    int32_t C;
    const ca_pod_spec* specs;
    const ca_selector_term* terms;
    const ca_selector_req* reqs;
    const int32_t* names;
    int32_t base;                 // mirror pod id of the first copy this call stores
    int32_t max_removable;
    int32_t n_pdbs;
    int32_t* allowed;             // RemainingPdbTracker budgets (in place)
    const int32_t* pdb_off;       // memberships by caller pod [n_pods + 1]
    const int32_t* pdb_pod;
    int32_t* hout;                // Hints.Set of the caller's pods, by move index (page-locked host memory)
    const int32_t* ex_base;       // per node: first slot of its committed copies in ex_pods
    PcPod* ex_pods;               // copies committed onto a node, as their later candidacy reads them
    ca_plan_result* res;          // (results, moves and info: page-locked host memory, written in place)
    ca_plan_move* moves;
    int32_t* published;           // moves written out so far (page-locked): the host replays them
                                  // into the mirror while the chain runs
    int64_t* info;                // [0] lastIndex, [1] moves, [2] removed, [3] candidates simulated,
                                  // [4..4+PC_NPROF) phase cycle counters (PC_* above), [4+PC_NPROF] the
                                  // first candidate not run (C: none; the host fills their results)
    int64_t L0;
    int32_t copy_cap;
    int32_t dbg;                  // CASIM_PLAN_DBG bits: 1 no block cache, 2 no maxima refresh
    int32_t* trace;               // CASIM_PLAN_TRACE: per simulated pod {c, t, hint, hint_ok, target, evals, L, cnt}
    int32_t trace_cap;
    int32_t help_after;           // blocks a scan loads before handing the rest to the helper waves
};

// packs the pods to move (one thread per list entry; hints as the caller passed them, by move
// index: a pod's hint changes only while its own candidate is simulated)
__global__ void __launch_bounds__(256) k_plan_pack(const int32_t* __restrict__ move_pods, int32_t M,
                                                  const PodHot* __restrict__ ph, const int32_t* __restrict__ hint_move,
                                                  PcPod* __restrict__ out) {
    const int32_t i = (int32_t)(blockIdx.x * 256 + threadIdx.x);
    if (i >= M + 64) return;
    PcPod r = {};
    r.id = -1; r.hint = -1; r.orig = -1;
    if (i < M) {
        const int32_t id = move_pods[i];
        const PodHot p = ph[id];
        r.cpu = p.cpu; r.mem = p.mem; r.eph = p.eph;
        r.id = id; r.hint = hint_move ? hint_move[i] : -1; r.spec = p.spec; r.orig = id;
        // moved-pod semantics (cluster.go:235-240 clears Spec.NodeName, tpu.go:57-79 the TPU requests)
        uint32_t f = p.flags & ~(PF_NODE_NAME | PF_ALL_ZERO | PF_SCALAR_REQ | PF_HAS_SCALAR_KEYS);
        if (p.flags & PF_MOVED_ALL_ZERO) f |= PF_ALL_ZERO;
        if (p.flags & PF_MOVED_SCALAR_REQ) f |= PF_SCALAR_REQ;
        if (p.flags & PF_NONTPU_SCALAR) f |= PF_HAS_SCALAR_KEYS;
        r.flags = f;
    }
    out[i] = r;
}

// The committed node rows in LDS, one array per column (free cpu / memory / [ephemeral
// storage] / pod slots): a wave reads a block's column with one conflict-free access per
// lane.  ex_base (each node's first slot in the copy table) sits beside them.
struct PcRows {
    int64_t* c;
    int64_t* m;
    int64_t* e;                   // EPH_COLS only
    int32_t* p;
    int32_t* exb;                 // [n + 1]
};
// Per 64-node block: bit planes (podDestinations, visible = destination and schedulable,
// unschedulable, tainted, free ephemeral >= 0).
struct PcBlk {
    uint64_t dest, vis, usch, taint, eph;
};

// Per 64-node block: a 2-D skyline of its rows' free (cpu, memory) — the Pareto-maximal
// points over the visible rows with a free pod slot — so "can this pod fit any row of the
// block" is a handful of compares instead of loading the block.  The per-dimension maxima it
// replaces pass almost every block in a tight cluster (the most cpu and the most memory sit
// on different rows): on C3 without a limit 876 failing full-ring scans read 56k blocks
// whose maxima passed and that no exact skyline admits (scripts/plan_skyline_study.py).
// Invariant: every such row is dominated by a stored point (an over-approximation):
//   * points are 32-bit images rounded up — cpu clamped, memory in MiB rounded up; a pod
//     is compared through the same monotone maps, so a row that fits passes;
//   * at most PC_SKY points: past PC_SKY - 1 exact points the last one bounds the rest;
//   * a row that shrinks (AddPod, a node leaving podDestinations) leaves the points valid
//     (stale-high: a scan that loads the block without a fit rebuilds it); a row that grows
//     (the candidate's own RemovePods, a Revert) sets n = -1 (unknown: always loaded);
//   * the candidate being simulated is excluded (its scans exclude it, and its row grew).
// Stored point-major across blocks (c[i * nb + j]: point i of block j), so the window test —
// lane q checks block q — reads every point with one conflict-free access per lane, all of
// them issued at once.
#ifndef CASIM_PC_SKY
#define CASIM_PC_SKY 6
#endif
constexpr int PC_SKY = CASIM_PC_SKY;
struct PcSkyV {
    int32_t* n;                   // [nb] points stored (-1 = unknown)
    int32_t* c;                   // [PC_SKY][nb] cpu (points in no particular order)
    int32_t* m;                   // [PC_SKY][nb] memory (MiB, rounded up)
    int32_t nb;
};
__host__ __device__ inline int32_t sky_c(int64_t v) {
    return v > INT32_MAX ? INT32_MAX : (v < INT32_MIN ? INT32_MIN : (int32_t)v);
}
__host__ __device__ inline int32_t sky_m(int64_t v) {                 // ceil(v / 2^20), clamped
    const int64_t q = (v >> 20) + ((v & 0xFFFFF) != 0);
    return q > INT32_MAX ? INT32_MAX : (q < INT32_MIN ? INT32_MIN : (int32_t)q);
}

// LDS image of one call (byte offsets; every array 16-B aligned)
struct PcLayout {
    size_t rc, rm, re, rp, exb, blk, sky, excnt, scratch, resbuf, mvbuf, ctx, pdest, run, help, total;
};

__host__ __device__ inline PcLayout pc_layout(int32_t n, bool eph_cols) {
    PcLayout L;
    const size_t nn = (size_t)n, nb = (nn + 63) / 64;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += (bytes + 15) & ~(size_t)15; return r; };
    L.rc = take(8 * nn);
    L.rm = take(8 * nn);
    L.re = eph_cols ? take(8 * nn) : 0;
    L.rp = take(4 * nn);
    L.exb = take(4 * (nn + 1));
    L.blk = take(sizeof(PcBlk) * nb);
    L.sky = take(4 * nb * (1 + 2 * PC_SKY));
    L.excnt = take(2 * nn);
    L.scratch = take(4 * 64);
    L.resbuf = take(sizeof(ca_plan_result) * 64);       // results of the current 64 candidates
    L.mvbuf = take(sizeof(ca_plan_move) * PC_MVBUF);   // committed moves not yet written out
    L.ctx = take(512);                                 // PcCtx
    L.pdest = take(4 * PC_LIST);                       // destinations of a plain run's pods, by list index
    L.run = take(128);                                 // PcRun
    L.help = take(256);                                // PcHelp (scan requests to the helper waves)
    L.total = o;
    return L;
}

__device__ inline PcRows pc_rows(unsigned char* pc_raw, const PcLayout& Y) {
    PcRows r;
    r.c = reinterpret_cast<int64_t*>(pc_raw + Y.rc);
    r.m = reinterpret_cast<int64_t*>(pc_raw + Y.rm);
    r.e = reinterpret_cast<int64_t*>(pc_raw + Y.re);
    r.p = reinterpret_cast<int32_t*>(pc_raw + Y.rp);
    r.exb = reinterpret_cast<int32_t*>(pc_raw + Y.exb);
    return r;
}
__device__ inline PcSkyV pc_sky_view(unsigned char* pc_raw, const PcLayout& Y, int32_t nb) {
    PcSkyV v;
    v.n = reinterpret_cast<int32_t*>(pc_raw + Y.sky);
    v.c = v.n + nb;
    v.m = v.c + (size_t)PC_SKY * nb;
    v.nb = nb;
    return v;
}

extern "C" __device__ long long __ockl_wfred_add_i64(long long);
extern "C" __device__ long long __ockl_wfred_max_i64(long long);
extern "C" __device__ int __ockl_wfred_add_i32(int);
extern "C" __device__ int __ockl_wfred_min_i32(int);
extern "C" __device__ int __ockl_wfred_max_i32(int);

__device__ inline int64_t pc_rl64(int64_t v, int lane) {
    const uint64_t u = (uint64_t)v;
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)u, lane);   // (no sign extension)
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline int32_t pc_rl32(int32_t v, int lane) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, lane); }
__device__ inline uint64_t pc_below(int lane) { return lane == 0 ? 0ull : (~0ull >> (64 - lane)); }
__device__ inline bool pc_bit(const uint64_t* w, int32_t i) { return (w[i >> 6] >> (i & 63)) & 1ull; }
// a value every lane holds, as a scalar (SGPR) value
__device__ inline uint64_t pc_uni64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline int64_t pc_uni64s(int64_t v) { return (int64_t)pc_uni64((uint64_t)v); }

// Wave maximum of an unsigned value (0 = no value): DPP row shifts, then the row
// broadcasts 15 / 31; lane 63 ends with the maximum.  Seven VALU steps, against ~35
// instructions for the 64-bit __ockl reduction.
__device__ inline uint32_t pc_wmax_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Rebuilds a block's skyline from its 64 rows as one wave holds them (lane i: row j*64 + i;
// `valid`: visible, a free pod slot, not the candidate being simulated).  Extraction from
// both ends of the staircase at once: the largest (cpu, memory) key is a skyline point (the
// front), and so is the largest (memory, cpu) key (the back); every row with memory at most
// the front's memory, or cpu at most the back's cpu, is dominated; repeat on the rest.  The
// two ends' wave maxima are independent, so their latencies overlap: half the dependent
// steps of a one-ended extraction.  Past PC_SKY - 1 exact points, one point bounds the
// rest.  Keys are 32-bit images biased so that unsigned order is signed order (0: none).
// C3 blocks hold 4-5 points on average (p99 10).
__device__ void pc_sky_build(const PcSkyV sk, int32_t j, int64_t cc, int64_t cm, bool valid) {
    const int lane = threadIdx.x & 63;
    const int32_t C = sky_c(cc), M = sky_m(cm);
    const uint32_t Cu = (uint32_t)C ^ 0x80000000u, Mu = (uint32_t)M ^ 0x80000000u;
    bool alive = valid;
    int k = 0;
    auto put = [&](int slot, uint32_t cu, uint32_t mu) {
        if (lane == 0) { sk.c[slot * sk.nb + j] = (int32_t)(cu ^ 0x80000000u); sk.m[slot * sk.nb + j] = (int32_t)(mu ^ 0x80000000u); }
    };
    while (k <= PC_SKY - 3) {                        // room for two exact points and a bound
        if (!__ballot(alive)) break;
        const uint32_t cmax = pc_wmax_u32(alive ? Cu : 0u);
        const uint32_t mmax = pc_wmax_u32(alive ? Mu : 0u);
        const uint32_t m_at = pc_wmax_u32((alive && Cu == cmax) ? Mu : 0u);   // front: (cmax, m_at)
        const uint32_t c_at = pc_wmax_u32((alive && Mu == mmax) ? Cu : 0u);   // back: (c_at, mmax)
        put(k++, cmax, m_at);
        if (m_at != mmax) put(k++, c_at, mmax);      // (one point when the front is also the back)
        alive = alive && Mu > m_at && Cu > c_at;
    }
    while (k < PC_SKY - 1) {                         // the last slots one point at a time
        if (!__ballot(alive)) break;
        const uint32_t cmax = pc_wmax_u32(alive ? Cu : 0u);
        const uint32_t m_at = pc_wmax_u32((alive && Cu == cmax) ? Mu : 0u);
        put(k++, cmax, m_at);
        alive = alive && Mu > m_at;
    }
    if (k == PC_SKY - 1 && __ballot(alive)) {        // one point bounds the rest
        const uint32_t cmax = pc_wmax_u32(alive ? Cu : 0u);
        const uint32_t mmax = pc_wmax_u32(alive ? Mu : 0u);
        put(k++, cmax, mmax);
    }
    if (lane == 0) sk.n[j] = k;
}

// May some row of the block fit a pod with these 32-bit images (sky_c / sky_m of its
// requests; all_zero: only a visible row with a free slot is needed)?
__device__ inline bool pc_sky_maybe(const PcSkyV sk, int32_t j, int32_t pc, int32_t pm, bool all_zero) {
    const int32_t k = sk.n[j];
    int32_t c[PC_SKY], m[PC_SKY];
#pragma unroll
    for (int i = 0; i < PC_SKY; i++) { c[i] = sk.c[i * sk.nb + j]; m[i] = sk.m[i * sk.nb + j]; }   // (all issued at once)
    if (k < 0) return true;
    if (all_zero) return k > 0;
    bool hit = false;
#pragma unroll
    for (int i = 0; i < PC_SKY; i++) hit |= (i < k) & (pc <= c[i]) & (pm <= m[i]);
    return hit;
}

// The same test without branches (the window test: every lane's 18 loads in flight at once)
__device__ inline bool pc_sky_maybe_bf(const PcSkyV sk, int32_t j, int32_t pc, int32_t pm, bool all_zero) {
    const int32_t k = sk.n[j];
    bool hit = false;
#pragma unroll
    for (int i = 0; i < PC_SKY; i++) {
        const int32_t c = sk.c[i * sk.nb + j], m = sk.m[i * sk.nb + j];
        hit |= (i < k) & (pc <= c) & (pm <= m);
    }
    return (k < 0) | (all_zero ? (k > 0) : hit);
}

// workgroup-coherent global loads: the PDB budgets the chain's own atomics updated
__device__ inline int32_t pc_ld(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// a list entry held by a lane (pod t in lane t % 64 of half t / 64)
struct PcReg {
    int64_t cpu, mem, eph;
    int32_t id, hint, spec, orig;
    uint32_t flags;
};
__device__ inline PcReg pc_reg(const PcPod& p) {
    PcReg r;
    r.cpu = p.cpu; r.mem = p.mem; r.eph = p.eph; r.id = p.id; r.hint = p.hint; r.spec = p.spec; r.orig = p.orig;
    r.flags = p.flags;
    return r;
}
__device__ inline PcPod pc_load(const PcPod* p) {
    PcPod r;
    const int4* q = reinterpret_cast<const int4*>(p);
    int4 a = q[0], b = q[1], c = q[2];
    __builtin_memcpy(reinterpret_cast<int4*>(&r), &a, 16);
    __builtin_memcpy(reinterpret_cast<int4*>(&r) + 1, &b, 16);
    __builtin_memcpy(reinterpret_cast<int4*>(&r) + 2, &c, 16);
    return r;
}

// Out of line (rare: taints, affinity, node names), so the chain keeps its registers.  The
// tables are passed by value: a reference to the kernel's by-value PcArgs would make the
// compiler copy the whole argument block to scratch memory and read every field back from
// there (global-memory latency on the chain's critical path).
struct PcTabs {
    const NodeStatic* st;
    const ca_pod_spec* specs;
    const ca_selector_term* terms;
    const ca_selector_req* reqs;
    const int32_t* names;
};
__device__ __attribute__((always_inline)) inline bool pc_static_fit(PcTabs t, int32_t x, int32_t spec, uint32_t pf) {
    const NodeStatic ns = t.st[x];
    return dev_static_filters(t.specs[spec], pf, t.terms, t.reqs, ns, false) == CA_PLUGIN_NONE;
}
__device__ __attribute__((always_inline)) inline bool pc_in_names(PcTabs t, int32_t x, int32_t spec) {
    const ca_pod_spec& s = t.specs[spec];
    const int32_t nid = t.st[x].name_id;
    bool in = false;
    for (int32_t k = 0; k < s.prefilter_count; k++) in |= t.names[s.prefilter_first + k] == nid;
    return in;
}
__device__ inline PcTabs pc_tabs(const PcArgs& a) { return PcTabs{a.st, a.specs, a.terms, a.reqs, a.names}; }

// Helper waves (the workgroup's waves 1..H).  The chain is one wavefront; a rotating scan
// that has loaded PC_HELP_AFTER blocks without a fit (the tight phase: scans over most of
// the ring) hands the rest of the ring to the helpers and waits.  Nothing changes the rows
// while it waits, so a block's verdict is a pure function of the LDS rows, its bit planes
// and the pod: helper h checks rotated blocks rr_lo + h, rr_lo + h + H, ... (the maxima
// skip, then the rows and the static filters where they matter), lowers `best` (rr * 64 +
// first fitting lane) with an LDS atomic min and stops at the first fit of its own
// sequence or once its next block lies beyond `best`; blocks it read without a fit while
// their maxima were stale get the exact maxima (`refr` tells the chain which).  The chain
// then takes the fit at `best` and counts the visible nodes before it as evaluations —
// exactly the scan's outcome, in a fraction of its dependent steps.
// the bulk step's back-off: after PC_BULK_FAILS candidates in a row whose first bulk step
// placed nothing, the next PC_BULK_SKIP candidates start with the plain run
#ifndef CASIM_PC_BULK_FAILS
#define CASIM_PC_BULK_FAILS 3
#endif
#ifndef CASIM_PC_BULK_SKIP
#define CASIM_PC_BULK_SKIP 32
#endif
constexpr int PC_BULK_FAILS = CASIM_PC_BULK_FAILS, PC_BULK_SKIP = CASIM_PC_BULK_SKIP;
constexpr int PC_HELP_AFTER = 2;       // blocks the chain loads itself before handing off
struct PcHelp {
    int32_t seq, quit, done, best;
    int32_t rr_lo, rr_end, j0, l0, nb, node, spec, fl;
    int64_t pcpu, pmem, peph;
    uint32_t pf, pad;
    uint64_t dirty0, dirty1, refr0, refr1;
};
static_assert(sizeof(PcHelp) <= 256, "PcHelp");
enum { PH_ANY_STATIC = 1, PH_TAINT_ALL = 2, PH_ALL_ZERO = 4 };

__device__ inline int32_t ph_ld(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool EPH_COLS>
__device__ void pc_helper(const PcArgs& a, unsigned char* pc_raw, int h, int H) {
    const int lane = threadIdx.x & 63;
    const int32_t n = a.n;
    const PcLayout Y = pc_layout(n, EPH_COLS);
    const PcRows R_ = pc_rows(pc_raw, Y);
    int64_t* const rc = R_.c;
    int64_t* const rm = R_.m;
    int64_t* const re = R_.e;
    int32_t* const rp = R_.p;
    PcBlk* const blk = reinterpret_cast<PcBlk*>(pc_raw + Y.blk);
    const PcSkyV sky = pc_sky_view(pc_raw, Y, (n + 63) >> 6);
    PcHelp* const q = reinterpret_cast<PcHelp*>(pc_raw + Y.help);
    int32_t seen = 0;
    for (;;) {
        int32_t sq;
        for (;;) {
            sq = __builtin_amdgcn_readfirstlane(ph_ld(&q->seq));
            if (sq != seen || __builtin_amdgcn_readfirstlane(ph_ld(&q->quit))) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (sq == seen) break;                                   // quit
        seen = sq;
        const int32_t rr_lo = __builtin_amdgcn_readfirstlane(q->rr_lo), rr_end = __builtin_amdgcn_readfirstlane(q->rr_end);
        const int32_t j0 = __builtin_amdgcn_readfirstlane(q->j0), l0 = __builtin_amdgcn_readfirstlane(q->l0);
        const int32_t nb = __builtin_amdgcn_readfirstlane(q->nb), node = __builtin_amdgcn_readfirstlane(q->node);
        const int32_t spec = __builtin_amdgcn_readfirstlane(q->spec), fl = __builtin_amdgcn_readfirstlane(q->fl);
        const int64_t pcpu = pc_uni64s(q->pcpu), pmem = pc_uni64s(q->pmem), peph = pc_uni64s(q->peph);
        const uint32_t pf = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)q->pf);
        const uint64_t dirty0 = pc_uni64(q->dirty0), dirty1 = pc_uni64(q->dirty1);
        const bool any_static = fl & PH_ANY_STATIC, taint_all = fl & PH_TAINT_ALL, all_zero = fl & PH_ALL_ZERO;
        const int32_t jn = node >> 6;
        const uint64_t nbit = 1ull << (node & 63);
        const int32_t pc32 = sky_c(pcpu), pm32 = sky_m(pmem);
        uint64_t refr0 = 0, refr1 = 0;
        for (int32_t rr = rr_lo + h; rr <= rr_end; rr += H) {
            if (rr * 64 > __builtin_amdgcn_readfirstlane(ph_ld(&q->best))) break;   // a fit before this block
            int32_t j = j0 + rr;
            if (j >= nb) j -= nb;
            const uint64_t inr = rr == nb ? ((1ull << l0) - 1) : ~0ull;
            const uint64_t cvis = pc_uni64(blk[j].vis);
            const uint64_t vw = cvis & inr & (j == jn ? ~nbit : ~0ull);
            if (!vw) continue;
            if (!pc_sky_maybe(sky, j, pc32, pm32, all_zero)) continue;   // no row of the block can fit it
            const int32_t x = j * 64 + lane;
            const bool in = x < n;
            const int64_t cc = in ? rc[x] : 0, cm = in ? rm[x] : 0;
            const int64_t ce = (EPH_COLS && in) ? re[x] : 0;
            const int32_t cp = in ? rp[x] : INT32_MIN;
            uint64_t fitm = vw & __ballot(cp >= 1);
            if (!all_zero) {
                fitm &= __ballot(pcpu <= cc) & __ballot(pmem <= cm);
                fitm &= EPH_COLS ? __ballot(peph <= ce) : pc_uni64(blk[j].eph);
            }
            const uint64_t needm = any_static ? ~0ull : (taint_all ? 0ull : pc_uni64(blk[j].taint));
            if (fitm & needm) {
                bool ok = true;
                if ((fitm & needm) >> lane & 1ull) ok = pc_static_fit(pc_tabs(a), x, spec, pf);
                fitm &= __ballot(ok);
            }
            if (fitm) {
                if (lane == 0) atomicMin(&q->best, rr * 64 + (int32_t)__builtin_ctzll(fitm));
                break;
            }
            const bool dj = j < 64 ? ((dirty0 >> j) & 1ull) : ((dirty1 >> (j - 64)) & 1ull);
            if (dj) {                                               // the exact skyline of the rows just read
                pc_sky_build(sky, j, cc, cm, ((cvis >> lane) & 1ull) && cp >= 1 && x != node);
                if (j < 64) refr0 |= 1ull << j; else refr1 |= 1ull << (j - 64);
            }
        }
        if (lane == 0) {
            if (refr0) atomicOr(reinterpret_cast<unsigned long long*>(&q->refr0), (unsigned long long)refr0);
            if (refr1) atomicOr(reinterpret_cast<unsigned long long*>(&q->refr1), (unsigned long long)refr1);
            __hip_atomic_fetch_add(&q->done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// A plain run's pod whose hint names a node it may not take (the candidate itself, or a
// node outside podDestinations): findNodeWithHints still runs CheckPredicates on it
// (hinting_simulator.go:91-108: one evaluation; its Hints.Set would store the same node)
// and the pod goes on to the scan like an unhinted one.
constexpr uint32_t PC_QF_HINT_EVAL = 0x80000000u;

// The plain run is inlined: as a call, its entry waited for every memory operation in
// flight (the ABI's s_waitcnt at function entry: the next candidate's prefetched pods, the
// copies' records), its PcTabs argument went through scratch and its callee-saved registers
// were saved and restored in scratch — ≈ 3.7k cycles per call, 13 % of the limit-200 kernel
// (1.59 -> 1.38 ms) and 6 % without a limit (51.6 -> 48.4 ms).  CASIM_PC_NOINLINE builds
// the call for comparison.
#ifdef CASIM_PC_NOINLINE
#define PC_PLAIN_RUN_ATTR __attribute__((noinline))
#else
#define PC_PLAIN_RUN_ATTR __attribute__((always_inline)) inline
#endif

// Scalars a plain run (pc_plain_run) shares with the simulation, in LDS.
struct PcRun {
    int32_t Lw, adv, placed, failed;
    int32_t node, moved, pad0, pad1;
    uint64_t dirty0, dirty1, evals;
    uint64_t prof[8];             // CASIM_PROF builds: PC_R_* (cycles by region, counts)
};
static_assert(sizeof(PcRun) <= 128, "PcRun");

// A run of plain pods (no usable hint, no PreFilter names or failure, no NodeName or node
// affinity) of one candidate, one pod after another: rotating first fit from lastIndex over
// the committed rows (schedulerbased.go:114-131), the block skylines skipping blocks that
// cannot fit the pod, AddPod of each placement (cluster.go:79).  Lane i holds pod t0 + i's
// requests; destinations go to pdest[t0 + k] (LDS).  Its state crosses in the PcRun record
// (LDS) and its loop state is re-asserted uniform at every pod, so the inlined loop keeps
// it in scalars.  Stops at the first pod that fits nowhere (failed = 1) or after R pods.
template <bool EPH_COLS>
__device__ PC_PLAIN_RUN_ATTR void pc_plain_run(unsigned char* pc_raw, int32_t n_, int32_t t0_, int32_t R_,
                                                       int64_t qc, int64_t qm, int64_t qe, uint32_t qf, int32_t qs,
                                                       PcTabs tabs) {
    const int lane = threadIdx.x & 63;
    // (a device function's arguments arrive in vector registers as per-lane values: the
    // uniform ones go back to scalars, else every loop and branch below is divergent)
    const int32_t n = __builtin_amdgcn_readfirstlane(n_), t0 = __builtin_amdgcn_readfirstlane(t0_);
    const int32_t R = __builtin_amdgcn_readfirstlane(R_);
    const PcLayout Y = pc_layout(n, EPH_COLS);
    const PcRows RW = pc_rows(pc_raw, Y);
    int64_t* const rc = RW.c;
    int64_t* const rm = RW.m;
    int64_t* const re = RW.e;
    int32_t* const rp = RW.p;
    PcBlk* const blk = reinterpret_cast<PcBlk*>(pc_raw + Y.blk);
    const PcSkyV sky = pc_sky_view(pc_raw, Y, (n + 63) >> 6);
    int32_t* const pdest = reinterpret_cast<int32_t*>(pc_raw + Y.pdest);
    PcRun* const rs = reinterpret_cast<PcRun*>(pc_raw + Y.run);
    const int32_t nb = (n + 63) >> 6;
    int32_t Lw = __builtin_amdgcn_readfirstlane(rs->Lw);
    int32_t adv = __builtin_amdgcn_readfirstlane(rs->adv);
    const int32_t node = __builtin_amdgcn_readfirstlane(rs->node);
    uint64_t dirty0 = pc_uni64(rs->dirty0), dirty1 = pc_uni64(rs->dirty1);
    const int32_t jn = node >> 6;
    const uint64_t nbit = 1ull << (node & 63);
    uint64_t evals = 0;
    int32_t cj = -1;
    int64_t cc = 0, cm = 0, ce = 0;
    int32_t cp = 0;
    uint64_t cvis = 0, cok = 0, ctaint = 0;
    uint64_t cd0 = 0, cd1 = 0;            // the cached block's dirty bit
    bool cmod = false;                    // its rows in registers differ from LDS
    // AddPods change the cached block's rows in registers only; they go back to LDS when
    // another block is loaded and when the run ends (nothing else reads them meanwhile)
    auto flush = [&]() {
        if (cmod) {
            const int32_t x = cj * 64 + lane;
            if (x < n) {
                rc[x] = cc; rm[x] = cm; rp[x] = cp;
                if (EPH_COLS) re[x] = ce;
            }
            cmod = false;
        }
    };
    auto load_block = [&](int32_t j) {
        flush();
        const int32_t x = j * 64 + lane;
        const bool in = x < n;
        cc = in ? rc[x] : 0; cm = in ? rm[x] : 0; cp = in ? rp[x] : INT32_MIN;
        ce = (EPH_COLS && in) ? re[x] : 0;
        cvis = pc_uni64(blk[j].vis) & (j == jn ? ~nbit : ~0ull);   // (the candidate is never a destination)
        cok = EPH_COLS ? ~0ull : pc_uni64(blk[j].eph);
        ctaint = pc_uni64(blk[j].taint);
        cd0 = j < 64 ? 1ull << j : 0ull;
        cd1 = j < 64 ? 0ull : 1ull << (j - 64);
        cj = j;
    };
    int32_t k = 0, failed = 0;
#ifdef CASIM_PROF
    uint64_t rp_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t rt_ = clock64();
#define PR_MARK(i) do { const uint64_t t_ = clock64(); rp_[i] += t_ - rt_; rt_ = t_; } while (0)
#define PR_COUNT(i) (rp_[i]++)
#define PR_NSKY() (nsky_++)
    int32_t nsky_ = 0;
#else
#define PR_NSKY() do {} while (0)
#define PR_MARK(i) do {} while (0)
#define PR_COUNT(i) do {} while (0)
#endif
    for (; k < R; k++) {
        PR_COUNT(5);
        // (the loop state is uniform: said so at every pod, else a value the compiler cannot
        // prove uniform turns the whole scan below into exec-masked vector code)
        k = __builtin_amdgcn_readfirstlane(k);
        Lw = __builtin_amdgcn_readfirstlane(Lw);
        adv = __builtin_amdgcn_readfirstlane(adv);
        cj = __builtin_amdgcn_readfirstlane(cj);
        dirty0 = pc_uni64(dirty0); dirty1 = pc_uni64(dirty1);
        cvis = pc_uni64(cvis); cok = pc_uni64(cok); ctaint = pc_uni64(ctaint);
        cd0 = pc_uni64(cd0); cd1 = pc_uni64(cd1);
        const int64_t pcpu = pc_rl64(qc, k), pmem = pc_rl64(qm, k);
        const int64_t peph = EPH_COLS ? pc_rl64(qe, k) : 0;
        const uint32_t pf = (uint32_t)pc_rl32((int32_t)qf, k);
        const bool all_zero = (pf & PF_ALL_ZERO) != 0;
        const bool taint_all = (pf & PF_TAINT_MASK_ALL) != 0;
        if (pf & PC_QF_HINT_EVAL) evals += 1;        // the CheckPredicates of a hint it cannot take
        const int32_t j0 = Lw >> 6, l0 = Lw & 63;
        bool skip0 = false;                       // pod k fits no row of the cached block from l0 on
        // Fast path: a batch of pods whose first fits lie in the cached block (the block of the
        // previous placement), each past the previous one's.  Within the batch every pod's scan
        // starts past the rows the batch has taken (lastIndex = target + 1), so its fit test
        // reads rows as they were when the batch began: the tests need no dependent updates,
        // and the batch's AddPods, evaluations and lastIndex advance are applied once at its end.
        if (j0 == cj && !all_zero) {
            uint64_t P = 0;                       // rows the batch took (one pod each, ascending)
            int32_t l = l0, kk = k, nhint = 0;
            // (all uniform; said so, else the compiler keeps the loop state in vector lanes)
            const uint64_t vis_ = pc_uni64(cvis), ok_ = pc_uni64(cok), taint_ = pc_uni64(ctaint);
            const uint64_t free_ = vis_ & __ballot(cp >= 1) & (EPH_COLS ? ~0ull : ok_);
            bool go = true;
            while (go) {
                l = __builtin_amdgcn_readfirstlane(l);
                kk = __builtin_amdgcn_readfirstlane(kk);
                P = pc_uni64(P);
                // the fit masks of the next 4 pods first (independent of each other: their
                // loads and compares overlap), then the dependent first-fit chain over them
                uint64_t F[4];
                uint32_t FL[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int32_t kq = kk + q < R ? kk + q : R - 1;
                    FL[q] = (uint32_t)pc_rl32((int32_t)qf, kq);
                    const int64_t c_ = pc_rl64(qc, kq), m_ = pc_rl64(qm, kq);
                    uint64_t f_ = free_ & __ballot(c_ <= cc) & __ballot(m_ <= cm);
                    if (EPH_COLS) f_ &= __ballot(pc_rl64(qe, kq) <= ce);
                    F[q] = pc_uni64(f_);
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t bf = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)FL[q]);
                    if (bf & PF_ALL_ZERO) { go = false; break; }                  // (pod k: not all_zero)
                    const uint64_t fitm = F[q] & (~0ull << l);
                    if (kk == k && !fitm) skip0 = true;   // (the scan's first block: no fit, known)
                    const uint64_t first = fitm & (0ull - fitm);
                    if (!first || (first & ((bf & PF_TAINT_MASK_ALL) ? 0ull : taint_))) { go = false; break; }
                    P |= first;
                    if (kk > k && (bf & PC_QF_HINT_EVAL)) nhint++;               // (pod k's was counted above)
                    l = __builtin_ctzll(first) + 1;
                    if (++kk == R || l == 64) { go = false; break; }
                }
            }
            if (P) {
                const bool inP = (P >> lane) & 1ull;
                const int32_t src = k + __popcll(P & pc_below(lane));    // the pod that took this row
                const int32_t sa = (src & 63) * 4;
                const int64_t sc = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int32_t)(qc >> 32)) << 32) |
                                             (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int32_t)qc));
                const int64_t sm = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int32_t)(qm >> 32)) << 32) |
                                             (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int32_t)qm));
                cc = inP ? wsub(cc, sc) : cc;
                cm = inP ? wsub(cm, sm) : cm;
                cp = inP ? cp - 1 : cp;
                if (EPH_COLS) {
                    const int64_t se = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int32_t)(qe >> 32)) << 32) |
                                                 (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int32_t)qe));
                    ce = inP ? wsub(ce, se) : ce;
                }
                if (inP) pdest[t0 + src] = cj * 64 + lane;
                cmod = true;
                dirty0 |= cd0; dirty1 |= cd1;
                const int32_t tl = 63 - __builtin_clzll(P);              // the last pod's row
                evals += (uint64_t)__popcll(cvis & (~0ull << l0) & (tl == 63 ? ~0ull : ((2ull << tl) - 1))) + nhint;
                const int32_t nx = cj * 64 + tl + 1;
                adv += nx - Lw;
                Lw = nx == n ? 0 : nx;
                k = kk - 1;
                PR_MARK(4);
                continue;
            }
        }
        int32_t target = -1, wr = -1, my_nv = 0;
        uint64_t passm = 0;
        PR_MARK(0);
        // the batch attempt already tested the scan's first block (the cached one) for pod k
        skip0 = __builtin_amdgcn_readfirstlane((int)skip0) != 0;
        if (skip0) evals += (uint64_t)__popcll(cvis & (~0ull << l0));
        for (int32_t rr = skip0 ? 1 : 0; rr <= nb; rr++) {
            rr = __builtin_amdgcn_readfirstlane(rr);
            wr = __builtin_amdgcn_readfirstlane(wr);
            cj = __builtin_amdgcn_readfirstlane(cj);
            passm = pc_uni64(passm);
            if (rr == nb && l0 == 0) break;
            int32_t j = j0 + rr;
            if (j >= nb) j -= nb;
            if (rr > 0 && rr < nb && j != cj) {
                // 64 blocks at a time: a block passes when its skyline cannot fit the pod
                if (wr < 0 || rr >= wr + 64) {
                    const int32_t pc32 = sky_c(pcpu), pm32 = sky_m(pmem);   // (only scans that leave their block)
                    const int32_t q = rr + lane;
                    const bool qin = q < nb;
                    int32_t jj = j0 + (qin ? q : 0);             // (lanes past the ring read a valid block)
                    if (jj >= nb) jj -= nb;
                    const uint64_t vw = blk[jj].vis & (jj == jn ? ~nbit : ~0ull);
                    const bool maybe = pc_sky_maybe_bf(sky, jj, pc32, pm32, all_zero);
                    const bool pass = qin & !((vw != 0) & maybe) & (jj != cj);
                    my_nv = qin ? __popcll(vw) : 0;
                    passm = __ballot(pass);
                    wr = rr;
                    PR_COUNT(7);
                }
                const int32_t off = rr - wr;
                const uint64_t stop = ~passm & (~0ull << off);
                const int32_t kk = (stop ? __builtin_ctzll(stop) : 64) - off;
                if (kk > 0) {
                    evals += (uint64_t)__ockl_wfred_add_i32((lane >= off && lane < off + kk) ? my_nv : 0);
                    rr += kk - 1;
                    PR_MARK(1);
                    continue;
                }
                PR_MARK(1);
            }
            if (j != cj) { load_block(j); PR_COUNT(6); }
            const uint64_t inr = (rr == 0) ? (~0ull << l0) : (rr == nb ? ((1ull << l0) - 1) : ~0ull);
            const uint64_t vism = cvis & inr;
            uint64_t fitm = vism & __ballot(cp >= 1);
            if (!all_zero) {
                fitm &= __ballot(pcpu <= cc) & __ballot(pmem <= cm);
                fitm &= EPH_COLS ? __ballot(peph <= ce) : cok;
            }
            const uint64_t needm = taint_all ? 0ull : ctaint;
            if (fitm & needm) {                              // TaintToleration where the node has taints
                bool ok = true;
                if (((fitm & needm) >> lane) & 1ull) ok = pc_static_fit(tabs, j * 64 + lane, pc_rl32(qs, k), pf);
                fitm &= __ballot(ok);
            }
            if (fitm) {
                const int f = __builtin_ctzll(fitm);
                const uint64_t upto = (f == 63) ? ~0ull : ((2ull << f) - 1);
                evals += (uint64_t)__popcll(vism & upto);
                target = j * 64 + f;
                PR_MARK(2);
                break;
            }
            evals += (uint64_t)__popcll(vism);
            PR_MARK(2);
            // a block the skyline let through without a fit (a false positive): rebuild it.  Not
            // the scan's first block — read regardless of its skyline, and usually the block of
            // the previous placement: a rebuild there would buy nothing
            const bool dj = rr > 0 && (j < 64 ? ((dirty0 >> j) & 1ull) : ((dirty1 >> (j - 64)) & 1ull));
            if (dj) {
                pc_sky_build(sky, j, cc, cm, ((cvis >> lane) & 1ull) && cp >= 1 && j * 64 + lane != node);
                if (j < 64) dirty0 &= ~(1ull << j); else dirty1 &= ~(1ull << (j - 64));
                PR_NSKY();
                PR_MARK(3);
            }
        }
        if (target < 0) { failed = 1; break; }                                    // breakOnFailure
        // ---- AddPod of the moved copy (:79): the row is the cached block's lane f ----
        {
            const bool me = lane == (target & 63);
            cc = me ? wsub(cc, pcpu) : cc;
            cm = me ? wsub(cm, pmem) : cm;
            cp = me ? cp - 1 : cp;
            if (EPH_COLS) ce = me ? wsub(ce, peph) : ce;
            cmod = true;
        }
        dirty0 |= cd0; dirty1 |= cd1;                                            // (target's block is cj)
        adv += (target >= Lw ? target - Lw : target + n - Lw) + 1;
        Lw = target + 1 == n ? 0 : target + 1;                                   // schedulerbased.go:131
        if (lane == 0) pdest[t0 + k] = target;
        PR_MARK(4);
    }
    flush();
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        rs->Lw = Lw; rs->adv = adv; rs->dirty0 = dirty0; rs->dirty1 = dirty1; rs->evals = evals;
        rs->placed = k; rs->failed = failed; rs->moved = k > 0 ? 1 : 0;
#ifdef CASIM_PROF
        for (int i = 0; i < 8; i++) rs->prof[i] = rp_[i];
        rs->pad0 = nsky_;
#endif
    }
#undef PR_MARK
#undef PR_COUNT
#undef PR_NSKY
    __builtin_amdgcn_wave_barrier();
}

// Per-call scalar state the candidate loop and the simulation share (LDS).
struct PcCtx {
    int32_t Lw, Lraw, nm, mv_n, mv_first, removed;
    int32_t bulk_fail, bulk_skip;         // candidates whose first bulk step placed nothing; candidates to skip it
    uint64_t dirty0, dirty1;              // blocks whose skylines may be stale-high
    ca_plan_result r;                     // the current candidate's result
#ifdef CASIM_PROF
    uint64_t prof[PC_NPROF];
#endif
};
static_assert(sizeof(PcCtx) <= 512, "PcCtx (pc_layout ctx)");

__device__ inline void pc_flush_moves(const PcArgs& a, const ca_plan_move* mvbuf, PcCtx* ctx, int lane) {
    const int32_t k = __builtin_amdgcn_readfirstlane(ctx->mv_n), first = __builtin_amdgcn_readfirstlane(ctx->mv_first);
    for (int32_t i = lane; i < k; i += 64) a.moves[first + i] = mvbuf[i];
    // the records reach host memory before the count that publishes them (whole candidates:
    // a flush follows a Commit)
    __threadfence_system();
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        ctx->mv_first = first + k; ctx->mv_n = 0;
        __hip_atomic_store(a.published, first + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_wave_barrier();
}

#ifdef CASIM_PROF
#define PC_SIM_T0() uint64_t tp_ = clock64()
#define PC_SIM_MARK(k) do { const uint64_t t_ = clock64(); if (lane == 0) ctx->prof[k] += t_ - tp_; tp_ = t_; } while (0)
#define PC_SIM_COUNT(k) do { if (lane == 0) ctx->prof[k]++; } while (0)
#else
#define PC_SIM_T0() do {} while (0)
#define PC_SIM_MARK(k) do {} while (0)
#define PC_SIM_COUNT(k) do {} while (0)
#endif
#define PC_MARK_DIRTY(j) do { const int32_t j_ = (j); if (j_ < 64) dirty0 |= 1ull << j_; else dirty1 |= 1ull << (j_ - 64); } while (0)

// withForkedSnapshot(findPlaceFor) for one candidate on the committed rows: RemovePod of its
// pods, TrySchedulePods (hints, then the rotating scan), then Commit or Revert;
// the candidate loop keeps its scalar state in LDS (ctx), the simulation in registers.
// Updates ctx (lastIndex, moves, dirty blocks) and ctx->r.
template <bool EPH_COLS>
__device__ __attribute__((always_inline)) inline void pc_simulate(const PcArgs& a, unsigned char* pc_raw, PcCtx* ctx, const int32_t c,
                                                     const int32_t mo, const int32_t m0,
                                                     const int32_t node, const int32_t cnt, const PcReg r0,
                                                     const PcReg r1, const int nh) {
    const int lane = threadIdx.x;
    const int32_t n = a.n, nb = (n + 63) >> 6;
    const PcLayout Y = pc_layout(n, EPH_COLS);
    const PcRows R_ = pc_rows(pc_raw, Y);
    int64_t* const rc = R_.c;
    int64_t* const rm = R_.m;
    int64_t* const re = R_.e;
    int32_t* const rp = R_.p;
    PcBlk* const blk = reinterpret_cast<PcBlk*>(pc_raw + Y.blk);
    const PcSkyV sky = pc_sky_view(pc_raw, Y, (n + 63) >> 6);
    uint16_t* const excnt = reinterpret_cast<uint16_t*>(pc_raw + Y.excnt);
    int32_t* const scratch = reinterpret_cast<int32_t*>(pc_raw + Y.scratch);
    ca_plan_move* const mvbuf = reinterpret_cast<ca_plan_move*>(pc_raw + Y.mvbuf);
    PcHelp* const hq = reinterpret_cast<PcHelp*>(pc_raw + Y.help);
    // (the shared scalars come back through readfirstlane: an LDS load is a per-lane value to
    // the compiler, and everything derived from it would run on the vector unit — a wave64
    // VALU instruction costs four cycles on a 16-lane SIMD, an SALU one)
    int32_t Lw = __builtin_amdgcn_readfirstlane(ctx->Lw);
    const int32_t nm = __builtin_amdgcn_readfirstlane(ctx->nm);
    uint64_t dirty0 = pc_uni64(ctx->dirty0), dirty1 = pc_uni64(ctx->dirty1);
    ca_plan_result r = ctx->r;
    bool moved_L = false;                       // a scan succeeded: lastIndex is the wrapped value
    // ring positions the candidate's scans advanced lastIndex over, and whether a hint placed
    // a pod: scan placements lie at distinct positions while the advance stays within one
    // ring, so the commit then needs no grouping of equal destinations
    int32_t adv = 0;
    bool hinted = false;
    PC_SIM_T0();
    // register cache of one 64-node block of rows (lane i: node cj * 64 + i): the free
    // columns in VGPRs, the block's visibility / ephemeral-ok / taint bits as wave-uniform
    // masks (SGPRs), so a fit test is a few compares and mask ANDs
    int32_t cj = -1;
    int64_t cc = 0, cm = 0, ce = 0;
    int32_t cp = 0;
    uint64_t cvis = 0, cok = 0, ctaint = 0;
    auto load_block = [&](int32_t j) {
        const int32_t x = j * 64 + lane;
        const bool in = x < n;
        cc = in ? rc[x] : 0; cm = in ? rm[x] : 0; cp = in ? rp[x] : INT32_MIN;
        ce = (EPH_COLS && in) ? re[x] : 0;
        cvis = pc_uni64(blk[j].vis);
        cok = EPH_COLS ? ~0ull : pc_uni64(blk[j].eph);
        ctaint = pc_uni64(blk[j].taint);
        cj = j;
    };
        // ---- withForkedSnapshot(findPlaceFor): RemovePod of the pods to move (cluster.go:228-233) ----
        const bool in0 = lane < cnt, in1 = 64 + lane < cnt;
        const int64_t sc = __ockl_wfred_add_i64(wadd(in0 ? r0.cpu : 0, in1 ? r1.cpu : 0));
        const int64_t sm = __ockl_wfred_add_i64(wadd(in0 ? r0.mem : 0, in1 ? r1.mem : 0));
        const int64_t se = EPH_COLS ? __ockl_wfred_add_i64(wadd(in0 ? r0.eph : 0, in1 ? r1.eph : 0)) : 0;
        const int32_t jn = node >> 6;
        const uint64_t nbit = 1ull << (node & 63);
        {
            const int64_t oc = rc[node], om = rm[node], oe = EPH_COLS ? re[node] : 0;
            const int32_t op = rp[node];
            const int64_t nc = wadd(oc, sc), nmm = wadd(om, sm), ne2 = wadd(oe, se);
            const int32_t np = op + cnt;
            if (lane == 0) {
                rc[node] = nc; rm[node] = nmm; rp[node] = np;
                if (EPH_COLS) re[node] = ne2;
                sky.n[jn] = -1;             // a row that grows: the block's skyline is unknown
            }
            if (jn == cj && lane == (node & 63)) { cc = nc; cm = nmm; ce = ne2; cp = np; }
            PC_MARK_DIRTY(jn);
        }
        PC_SIM_MARK(PC_FORK);
        uint64_t evals = 0;
        int32_t placed = 0;
        int32_t d0 = -1, d1 = -1;                   // destinations of pods t = lane, 64 + lane
        int32_t hs0 = INT32_MIN, hs1 = INT32_MIN;   // Hints.Set of pods t = lane, 64 + lane
        bool failed = false;
        // one pod (uniform values): hint check, then the rotating scan, then AddPod
        auto place = [&](const int32_t t, const int64_t pcpu, const int64_t pmem, const int64_t peph, const uint32_t pf,
                         const int32_t h, const int32_t spec) -> bool {
            PC_SIM_MARK(PC_PREP);
            const bool prefail = (pf & PF_PREFILTER_FAIL) != 0;
            const bool all_zero = (pf & PF_ALL_ZERO) != 0;
            // TaintToleration / NodeAffinity / NodeName where the pod or the node needs them
            auto static_fit = [&](int32_t x) -> bool { return pc_static_fit(pc_tabs(a), x, spec, pf); };
            const bool any_static = (pf & (PF_NODE_NAME | PF_AFFINITY)) != 0;
            const bool taint_all = (pf & PF_TAINT_MASK_ALL) != 0;
            int32_t target = -1;
            int64_t tc = 0, tm = 0, te = 0;         // the target's row
            int32_t tpd = 0;
            const int tl = t & 63;
            // ---- findNodeWithHints (hinting_simulator.go:91-108): CheckPredicates ----
            if (h >= 0 && h < n && !prefail) {
                evals++;
                const int64_t hc = pc_uni64s(rc[h]), hm = pc_uni64s(rm[h]);
                const int64_t he = EPH_COLS ? pc_uni64s(re[h]) : 0;
                const int32_t hp = __builtin_amdgcn_readfirstlane(rp[h]);
                const int32_t jh = h >> 6;
                const uint64_t hb = 1ull << (h & 63);
                const uint64_t uw = pc_uni64(blk[jh].usch), tw = pc_uni64(blk[jh].taint), dw = pc_uni64(blk[jh].dest);
                const bool eok = EPH_COLS ? (peph <= he) : ((pc_uni64(blk[jh].eph) & hb) != 0);
                bool ok = !((uw & hb) && !(pf & PF_TOL_UNSCHED));
                ok = ok && (hp >= 1) && (all_zero || ((pcpu <= hc) && (pmem <= hm) && eok));
                // (the call's result is a per-lane value to the compiler; every lane checked the same
                // node: making it uniform keeps the whole pod loop on the scalar unit)
                if (ok && (any_static || ((tw & hb) && !taint_all))) ok = __builtin_amdgcn_readfirstlane(static_fit(h) ? 1 : 0) != 0;
                if (ok) {
                    if (lane == tl) { if (t >= 64) hs1 = h; else hs0 = h; }          // :95 Set
                    if (h != node && (dw & hb)) { target = h; tc = hc; tm = hm; te = he; tpd = hp; hinted = true; }   // :102
                }
            }
            PC_SIM_MARK(PC_HINT);
            // ---- findNode -> FitsAnyNodeMatching(isCandidateNode) (:110-125) ----
            if (target < 0 && !prefail && n > 0) {
                const bool names = (pf & PF_PREFILTER_NAMES) != 0;
                const int32_t pc32 = sky_c(pcpu), pm32 = sky_m(pmem);
                const int32_t j0 = Lw >> 6, l0 = Lw & 63;
                int32_t wr = -1, my_nv = 0;
                uint64_t passm = 0;
                int32_t loaded = 0;
                // visible nodes (the scan's evaluations) of rotated blocks [ra, rb]
                auto vis_count = [&](int32_t ra, int32_t rb) -> uint64_t {
                    uint64_t tot = 0;
                    for (int32_t b0 = ra; b0 <= rb; b0 += 64) {
                        const int32_t r2 = b0 + lane;
                        int32_t cn = 0;
                        if (r2 <= rb) {
                            int32_t jj = j0 + r2;
                            if (jj >= nb) jj -= nb;
                            const uint64_t inr2 = r2 == nb ? ((1ull << l0) - 1) : ~0ull;
                            cn = __popcll(blk[jj].vis & inr2 & (jj == jn ? ~nbit : ~0ull));
                        }
                        tot += (uint64_t)__ockl_wfred_add_i32(cn);
                    }
                    return tot;
                };
                for (int32_t rr = 0; rr <= nb; rr++) {
                    if (rr == nb && l0 == 0) break;
                    int32_t j = j0 + rr;
                    if (j >= nb) j -= nb;
                    if (rr > 0 && rr < nb && !names && j != cj) {
                        // 64 blocks at a time: a block passes when the pod exceeds its maxima
                        if (wr < 0 || rr >= wr + 64) {
                            PC_SIM_COUNT(PC_WINDOWS);
                            const int32_t q = rr + lane;
                            bool pass = false;
                            my_nv = 0;
                            if (q < nb) {
                                int32_t jj = j0 + q;
                                if (jj >= nb) jj -= nb;
                                const uint64_t vw = blk[jj].vis & (jj == jn ? ~nbit : ~0ull);
                                const bool fitb = (vw != 0) && pc_sky_maybe(sky, jj, pc32, pm32, all_zero);
                                pass = !fitb && jj != cj;
                                my_nv = __popcll(vw);
                            }
                            passm = __ballot(pass);
                            wr = rr;
                            PC_SIM_MARK(PC_WIN);
                        }
                        const int32_t off = rr - wr;
                        const uint64_t stop = ~passm & (~0ull << off);
                        const int32_t k = (stop ? __builtin_ctzll(stop) : 64) - off;
                        if (k > 0) {
                            evals += (uint64_t)__ockl_wfred_add_i32((lane >= off && lane < off + k) ? my_nv : 0);
                            rr += k - 1;
                            PC_SIM_MARK(PC_WIN);
                            continue;
                        }
                    }
                    if (nh > 0 && !names && loaded >= a.help_after) {
                        // ---- the rest of the ring to the helper waves (PcHelp) ----
                        PC_SIM_COUNT(PC_HANDOFFS);
                        const int32_t rr_end = l0 == 0 ? nb - 1 : nb;
                        if (lane == 0) {
                            hq->rr_lo = rr; hq->rr_end = rr_end; hq->j0 = j0; hq->l0 = l0; hq->nb = nb;
                            hq->node = node; hq->spec = spec;
                            hq->fl = (any_static ? PH_ANY_STATIC : 0) | (taint_all ? PH_TAINT_ALL : 0) |
                                     (all_zero ? PH_ALL_ZERO : 0);
                            hq->pcpu = pcpu; hq->pmem = pmem; hq->peph = peph; hq->pf = pf;
                            hq->dirty0 = dirty0; hq->dirty1 = dirty1; hq->refr0 = 0; hq->refr1 = 0;
                            hq->best = INT32_MAX; hq->done = 0;
                            __hip_atomic_store(&hq->seq, hq->seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        while (__builtin_amdgcn_readfirstlane(ph_ld(&hq->done)) < nh) __builtin_amdgcn_s_sleep(1);
                        const int32_t best = __builtin_amdgcn_readfirstlane(ph_ld(&hq->best));
                        dirty0 &= ~pc_uni64(hq->refr0);
                        dirty1 &= ~pc_uni64(hq->refr1);
                        if (best != INT32_MAX) {
                            const int32_t rb = best >> 6, f = best & 63;
                            int32_t jb = j0 + rb;
                            if (jb >= nb) jb -= nb;
                            const uint64_t inrb = rb == nb ? ((1ull << l0) - 1) : ~0ull;
                            const uint64_t vmb = pc_uni64(blk[jb].vis) & inrb & (jb == jn ? ~nbit : ~0ull);
                            const uint64_t upto = (f == 63) ? ~0ull : ((2ull << f) - 1);
                            evals += vis_count(rr, rb - 1) + (uint64_t)__popcll(vmb & upto);
                            target = jb * 64 + f;
                            tc = pc_uni64s(rc[target]); tm = pc_uni64s(rm[target]);
                            te = EPH_COLS ? pc_uni64s(re[target]) : 0;
                            tpd = __builtin_amdgcn_readfirstlane(rp[target]);
                            adv += (target >= Lw ? target - Lw : target + n - Lw) + 1;
                            Lw = target + 1 == n ? 0 : target + 1;                       // schedulerbased.go:131
                            moved_L = true;
                            if (lane == tl) { if (t >= 64) hs1 = target; else hs0 = target; }   // :123
                        } else {
                            evals += vis_count(rr, rr_end);
                        }
                        break;
                    }
                    loaded++;
                    PC_SIM_COUNT(PC_BLOCKS);
#ifdef CASIM_PROF
                    if (a.dbg & 1) cj = -1;
#endif
                    if (j != cj) load_block(j);
                    const uint64_t inr = (rr == 0) ? (~0ull << l0) : (rr == nb ? ((1ull << l0) - 1) : ~0ull);
                    uint64_t vism = cvis & inr & (j == jn ? ~nbit : ~0ull);
                    if (names && vism) {
                        bool in = false;
                        if ((vism >> lane) & 1ull) in = pc_in_names(pc_tabs(a), j * 64 + lane, spec);
                        vism &= __ballot(in);
                    }
                    uint64_t fitm = vism & __ballot(cp >= 1);
                    if (!all_zero) {
                        fitm &= __ballot(pcpu <= cc) & __ballot(pmem <= cm);
                        fitm &= EPH_COLS ? __ballot(peph <= ce) : cok;
                    }
                    const uint64_t needm = any_static ? ~0ull : (taint_all ? 0ull : ctaint);
                    if (fitm & needm) {
                        bool ok = true;
                        if ((fitm & needm) >> lane & 1ull) ok = static_fit(j * 64 + lane);
                        fitm &= __ballot(ok);
                    }
                    PC_SIM_MARK(PC_LOADCHK);
                    if (fitm) {
                        const int f = __builtin_ctzll(fitm);
                        const uint64_t upto = (f == 63) ? ~0ull : ((2ull << f) - 1);
                        evals += (uint64_t)__popcll(vism & upto);
                        target = j * 64 + f;
                        tc = pc_rl64(cc, f); tm = pc_rl64(cm, f); te = EPH_COLS ? pc_rl64(ce, f) : 0;
                        tpd = pc_rl32(cp, f);
                        adv += (target >= Lw ? target - Lw : target + n - Lw) + 1;
                        Lw = target + 1 == n ? 0 : target + 1;                       // schedulerbased.go:131
                        moved_L = true;
                        if (lane == tl) { if (t >= 64) hs1 = target; else hs0 = target; }   // :123
                        break;
                    }
                    evals += (uint64_t)__popcll(vism);
                    // the block passed: rebuild its skyline from the rows just read (not the
                    // scan's first block: read regardless of its skyline)
                    const bool dj = rr > 0 && (j < 64 ? ((dirty0 >> j) & 1ull) : ((dirty1 >> (j - 64)) & 1ull));
                    if (dj) {
                        pc_sky_build(sky, j, cc, cm, ((cvis >> lane) & 1ull) && cp >= 1 && j * 64 + lane != node);
                        if (j < 64) dirty0 &= ~(1ull << j); else dirty1 &= ~(1ull << (j - 64));
                        PC_SIM_MARK(PC_SKYB);
                    }
                }
            }
            PC_SIM_MARK(PC_SCAN);
#ifdef CASIM_PROF
            if (a.trace && lane == 0) {
                const int32_t k = atomicAdd(a.trace, 1);
                if (k < a.trace_cap) {
                    int32_t* e = a.trace + 16 + 16 * k;
                    const int32_t dn = a.trace[1];
                    e[0] = c; e[1] = t; e[2] = h; e[3] = (int32_t)pf; e[4] = target; e[5] = (int32_t)evals;
                    e[6] = Lw; e[7] = cnt; e[8] = (int32_t)pcpu; e[9] = (int32_t)(pmem >> 20);
                    e[10] = (int32_t)rc[dn]; e[11] = (int32_t)(rm[dn] >> 20); e[12] = rp[dn];
                    e[13] = (int32_t)((blk[(dn) >> 6].vis >> ((dn) & 63)) & 1ull) | ((int32_t)((blk[(dn) >> 6].taint >> ((dn) & 63)) & 1ull) << 1) |
                            ((int32_t)(EPH_COLS ? 1 : ((blk[(dn) >> 6].eph >> ((dn) & 63)) & 1ull)) << 2);
                    e[14] = spec; e[15] = -1;
                }
            }
#endif
            if (target < 0) return false;                                            // breakOnFailure
            // ---- AddPod of the moved copy (:79) ----
            const int64_t nc = wsub(tc, pcpu), nmm = wsub(tm, pmem), ne2 = wsub(te, peph);
            const int32_t np = tpd - 1;
            if (lane == 0) {
                rc[target] = nc; rm[target] = nmm; rp[target] = np;
                if (EPH_COLS) re[target] = ne2;
            }
            if ((target >> 6) == cj && lane == (target & 63)) { cc = nc; cm = nmm; ce = ne2; cp = np; }
            PC_MARK_DIRTY(target >> 6);
            if (lane == tl) { if (t >= 64) d1 = target; else d0 = target; }
            PC_SIM_MARK(PC_ADD);
            return true;
        };
        // Bulk placement of a run of plain pods (no usable hint, no PreFilter names or
        // failure, no static filter): pod t0 + k's scan from lastIndex lands on the first
        // visible node at or after it, so while every pod fits the next visible node in
        // turn, pod t0 + k goes to the k-th visible node of the window [L, L + 64) — a node
        // that receives nothing else.  Lane i holds node L + i: its rank among the visible
        // nodes names its pod; the leading ranks that fit are placed at once, lane-parallel,
        // with one evaluation each.  The first pod that does not fit its node continues on
        // the exact per-pod path.  Pods of one half (t < 64 / t >= 64) per step.
        auto bulk = [&](const int32_t t0) -> int32_t {
            const bool hi = t0 >= 64;
            const int32_t hend = hi ? cnt : (cnt < 64 ? cnt : 64);
            const int32_t tl0 = t0 & 63;
            // run of plain pods: pod lane i = pod t0 + i
            const int32_t src_i = (tl0 + lane) & 63;
            const int32_t hh = __shfl(hi ? r1.hint : r0.hint, src_i, 64);
            const uint32_t ff = (uint32_t)__shfl((int32_t)(hi ? r1.flags : r0.flags), src_i, 64);
            const bool plain = t0 + lane < hend && (hh < 0 || hh >= n) &&
                               !(ff & (PF_PREFILTER_FAIL | PF_PREFILTER_NAMES | PF_NODE_NAME | PF_AFFINITY));
            const uint64_t pm = __ballot(plain);
            const int32_t R = (~pm) ? __builtin_ctzll(~pm) : 64;
            if (R == 0) return 0;
            // node lanes: window [L, L + 64)
            const int32_t span = n < 64 ? n : 64;
            int32_t x = Lw + lane;
            if (x >= n) x -= n;
            const bool inw = lane < span;
            const bool vis = inw && x != node && ((blk[x >> 6].vis >> (x & 63)) & 1ull);
            const uint64_t vm = __ballot(vis);
            const int32_t rank = __popcll(vm & pc_below(lane));
            const bool mine = vis && rank < R;
            const int32_t src = (tl0 + (rank < 63 ? rank : 63)) & 63;
            const int64_t pc2 = __shfl(hi ? r1.cpu : r0.cpu, src, 64);
            const int64_t pm2 = __shfl(hi ? r1.mem : r0.mem, src, 64);
            const int64_t pe2 = EPH_COLS ? __shfl(hi ? r1.eph : r0.eph, src, 64) : 0;
            const uint32_t pf2 = (uint32_t)__shfl((int32_t)(hi ? r1.flags : r0.flags), src, 64);
            bool fit = false;
            if (mine) {
                const bool eok = EPH_COLS ? (pe2 <= re[x]) : ((blk[x >> 6].eph >> (x & 63)) & 1ull);
                const bool tnt = (blk[x >> 6].taint >> (x & 63)) & 1ull;
                fit = (rp[x] >= 1) && ((pf2 & PF_ALL_ZERO) || ((pc2 <= rc[x]) && (pm2 <= rm[x]) && eok)) &&
                      !(tnt && !(pf2 & PF_TAINT_MASK_ALL));
            }
            const uint64_t failm = __ballot(mine && !fit);
            const uint64_t okm = failm ? (vm & pc_below(__builtin_ctzll(failm))) : vm;
            int32_t k = __popcll(okm);
            if (k > R) k = R;
            if (k == 0) return 0;
            const bool put = vis && rank < k;
            if (put) {                                                                // AddPod (:79)
                rc[x] = wsub(rc[x], pc2); rm[x] = wsub(rm[x], pm2); rp[x] -= 1;
                if (EPH_COLS) re[x] = wsub(re[x], pe2);
                scratch[(tl0 + rank) & 63] = x;
            }
            __builtin_amdgcn_wave_barrier();
            const int32_t last = __builtin_amdgcn_readfirstlane(scratch[(tl0 + k - 1) & 63]);
            if (lane >= tl0 && lane < tl0 + k) {                                    // pods t0 .. t0+k-1
                const int32_t v = scratch[lane];
                if (hi) { d1 = v; hs1 = v; } else { d0 = v; hs0 = v; }                // :123 Set
            }
            __builtin_amdgcn_wave_barrier();
            PC_MARK_DIRTY(Lw >> 6);
            PC_MARK_DIRTY((Lw + span - 1 < n ? Lw + span - 1 : Lw + span - 1 - n) >> 6);
            evals += (uint64_t)k;
            adv += (last >= Lw ? last - Lw : last + n - Lw) + 1;
            Lw = last + 1 == n ? 0 : last + 1;                                       // schedulerbased.go:131
            moved_L = true;
            cj = -1;                                                                 // rows changed
            return k;
        };
        // plain pods of a half from t: the leading pods without a usable hint, PreFilter names or
        // failure, NodeName or node affinity (lane i: pod t + i)
        // (a hint to the candidate itself or to a node outside podDestinations cannot be taken:
        // such a pod is plain but for the evaluation of the hint, PC_QF_HINT_EVAL)
        auto hint_eval = [&](const int32_t hh) -> bool { return hh >= 0 && hh < n; };
        auto hint_usable = [&](const int32_t hh) -> bool {
            return hint_eval(hh) && hh != node && ((blk[hh >> 6].dest >> (hh & 63)) & 1ull);
        };
        auto plain_len = [&](const int32_t t0) -> int32_t {
            const bool hi = t0 >= 64;
            const int32_t hend = hi ? cnt : (cnt < 64 ? cnt : 64);
            const int32_t src_i = ((t0 & 63) + lane) & 63;
            const int32_t hh = __shfl(hi ? r1.hint : r0.hint, src_i, 64);
            const uint32_t ff = (uint32_t)__shfl((int32_t)(hi ? r1.flags : r0.flags), src_i, 64);
            const bool plain = t0 + lane < hend && !hint_usable(hh) &&
                               !(ff & (PF_PREFILTER_FAIL | PF_PREFILTER_NAMES | PF_NODE_NAME | PF_AFFINITY));
            const uint64_t pm = __ballot(plain);
            return (~pm) ? __builtin_ctzll(~pm) : 64;
        };
        PcRun* const rs = reinterpret_cast<PcRun*>(pc_raw + Y.run);
        int32_t* const pdest = reinterpret_cast<int32_t*>(pc_raw + Y.pdest);
        {
            int32_t t = 0;
            // the bulk step pays off in a loose cluster; in a tight one it keeps failing at the
            // first pod: after PC_BULK_FAILS candidates in a row whose first bulk step placed nothing,
            // the next PC_BULK_SKIP candidates start with the plain run
            int32_t bfail = __builtin_amdgcn_readfirstlane(ctx->bulk_fail);
            int32_t bskip = __builtin_amdgcn_readfirstlane(ctx->bulk_skip);
            bool try_bulk = bskip == 0;
            if (bskip > 0) bskip--;
            bool first_bulk = true, bulk_hit = false;
            while (t < cnt && !failed) {
                if (try_bulk && n > 1) {
                    const int32_t k = bulk(t);
                    PC_SIM_MARK(PC_BULK);
                    if (first_bulk) {
                        first_bulk = false;
                        if (k > 0) bfail = 0;
                        else if (++bfail >= PC_BULK_FAILS) { bfail = 0; bskip = PC_BULK_SKIP; }
                    }
                    placed += k;
                    t += k;
                    if (k > 0) { bulk_hit = true; continue; }
                }
                try_bulk = false;
                const int32_t R = plain_len(t);
                if (R > 0) {
                    // ---- a run of plain pods: the lean scan, out of line ----
                    const bool hi = t >= 64;
                    const int32_t src_i = ((t & 63) + lane) & 63;
                    const int64_t qc = __shfl(hi ? r1.cpu : r0.cpu, src_i, 64);
                    const int64_t qm = __shfl(hi ? r1.mem : r0.mem, src_i, 64);
                    const int64_t qe = EPH_COLS ? __shfl(hi ? r1.eph : r0.eph, src_i, 64) : 0;
                    const int32_t qh = __shfl(hi ? r1.hint : r0.hint, src_i, 64);
                    const uint32_t qf = (uint32_t)__shfl((int32_t)(hi ? r1.flags : r0.flags), src_i, 64) |
                                        (hint_eval(qh) ? PC_QF_HINT_EVAL : 0u);
                    const int32_t qs = __shfl(hi ? r1.spec : r0.spec, src_i, 64);
                    if (lane == 0) {
                        rs->Lw = Lw; rs->adv = adv; rs->node = node; rs->dirty0 = dirty0; rs->dirty1 = dirty1;
                    }
                    __builtin_amdgcn_wave_barrier();
                    pc_plain_run<EPH_COLS>(pc_raw, n, t, R, qc, qm, qe, qf, qs, pc_tabs(a));
                    Lw = __builtin_amdgcn_readfirstlane(rs->Lw);
                    adv = __builtin_amdgcn_readfirstlane(rs->adv);
                    dirty0 = pc_uni64(rs->dirty0);
                    dirty1 = pc_uni64(rs->dirty1);
                    evals += pc_uni64(rs->evals);
                    const int32_t kp = __builtin_amdgcn_readfirstlane(rs->placed);
                    const bool fl = __builtin_amdgcn_readfirstlane(rs->failed) != 0;
#ifdef CASIM_PROF
                    if (lane == 0) {
                        for (int i = 0; i < 8; i++) ctx->prof[PC_R_POD + i] += rs->prof[i];
                        ctx->prof[PC_R_NSKY] += (uint64_t)rs->pad0;
                        ctx->prof[PC_R_NRUNS] += 1;
                    }
#endif
                    if (kp > 0) moved_L = true;
                    const int32_t tl0 = t & 63;
                    if (lane >= tl0 && lane < tl0 + kp) {                         // :123 Set
                        const int32_t v = pdest[(hi ? 64 : 0) + lane];
                        if (hi) { d1 = v; hs1 = v; } else { d0 = v; hs0 = v; }
                    }
                    cj = -1;                                                      // rows changed
                    placed += kp;
                    t += kp;
                    PC_SIM_MARK(PC_SCAN);
                    if (fl) { failed = true; break; }
                    try_bulk = bulk_hit;
                    continue;
                }
                bool ok;
                if (t < 64)
                    ok = place(t, pc_rl64(r0.cpu, t), pc_rl64(r0.mem, t), EPH_COLS ? pc_rl64(r0.eph, t) : 0,
                               (uint32_t)pc_rl32((int32_t)r0.flags, t), pc_rl32(r0.hint, t), pc_rl32(r0.spec, t));
                else
                    ok = place(t, pc_rl64(r1.cpu, t - 64), pc_rl64(r1.mem, t - 64),
                               EPH_COLS ? pc_rl64(r1.eph, t - 64) : 0, (uint32_t)pc_rl32((int32_t)r1.flags, t - 64),
                               pc_rl32(r1.hint, t - 64), pc_rl32(r1.spec, t - 64));
                if (!ok) { failed = true; break; }
                placed++;
                t++;
                try_bulk = bulk_hit;
            }
            if (lane == 0) { ctx->bulk_fail = bfail; ctx->bulk_skip = bskip; }
        }
        r.n_placed = placed;
        r.evals = evals;
        if (!failed) {
            // ---- Commit (cluster.go:207-211) ----
            r.removable = 1;
            r.n_moves = cnt;
            // distinct destinations (no hint placement, the scans within one ring): each copy
            // is its node's next entry — no grouping pass
            const bool distinct = !hinted && adv <= n;
            const int32_t mvn = __builtin_amdgcn_readfirstlane(ctx->mv_n);
            for (int half = 0; half < 2 && half * 64 < cnt; half++) {
                const int32_t t = half * 64 + lane;
                const bool act = t < cnt;
                const PcReg& q = half ? r1 : r0;
                const int32_t f = half ? d1 : d0;
                const int32_t fb = act ? R_.exb[f] : 0;                              // the copies' slots of node f
                const int32_t s = nm + t;
                if (act) {
                    ca_plan_move mv;
                    mv.candidate = c; mv.pod = q.id; mv.new_pod = a.base + s; mv.node = f;
                    mvbuf[mvn + t] = mv;                // (the copy's hint is f: it travels in its record)
                }
                // the copies join their destinations' pod lists in list order
                int32_t slot = 0;
                if (distinct) {
                    if (act) {
                        const int32_t old = excnt[f];
                        excnt[f] = (uint16_t)(old + 1);
                        slot = fb + old;
                    }
                } else {
                    int32_t rank = 0, lead = -1;
                    uint64_t pend = __ballot(act);
                    while (pend) {
                        const int l = __builtin_ctzll(pend);
                        const int32_t f0 = pc_rl32(f, l);
                        const uint64_t mm = __ballot(act && f == f0);
                        if (act && f == f0) { rank = __popcll(mm & pc_below(lane)); lead = l; }
                        if (lane == l) scratch[l] = __popcll(mm);
                        pend &= ~mm;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (act && lead == lane) {
                        const int32_t old = excnt[f];
                        excnt[f] = (uint16_t)(old + scratch[lane]);
                        scratch[lane] = old;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (act) slot = fb + scratch[lead] + rank;
                }
                if (act) {
                    PcPod cp2;
                    cp2.cpu = q.cpu; cp2.mem = q.mem; cp2.eph = q.eph;
                    cp2.id = a.base + s; cp2.hint = f; cp2.flags = q.flags; cp2.spec = q.spec; cp2.orig = q.orig;
                    cp2.pad = 0;
                    a.ex_pods[slot] = cp2;
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (lane == 0) { blk[jn].dest &= ~nbit; blk[jn].vis &= ~nbit; }               // planner.go:280
            if (jn == cj) cvis &= ~nbit;
            PC_MARK_DIRTY(jn);
            // CanRemovePods, then RemovePods (basic.go:66-95)
            if (a.n_pdbs > 0) {
                bool risky = false;
                for (int half = 0; half < 2; half++) {
                    const int32_t t = half * 64 + lane;
                    if (t >= cnt) continue;
                    const int32_t o = half ? r1.orig : r0.orig;
                    for (int32_t k = a.pdb_off[o]; k < a.pdb_off[o + 1]; k++)
                        risky |= atomicSub(a.allowed + a.pdb_pod[k], 1) <= 0;
                }
                r.risky = __ballot(risky) ? 1 : 0;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) { ctx->removed++; ctx->nm = nm + cnt; ctx->mv_n += cnt; }
            __builtin_amdgcn_wave_barrier();
            if (mvn + cnt + PC_LIST > PC_MVBUF) pc_flush_moves(a, mvbuf, ctx, lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            PC_SIM_MARK(PC_COMMIT);
        } else {
            // ---- Revert: undo the AddPods, then the RemovePods ----
            for (int half = 0; half < 2; half++) {
                const int32_t t = half * 64 + lane;
                if (t >= placed) continue;
                const PcReg& q = half ? r1 : r0;
                const int32_t f = half ? d1 : d0;
                atomicAdd(reinterpret_cast<unsigned long long*>(&rc[f]), (unsigned long long)q.cpu);
                atomicAdd(reinterpret_cast<unsigned long long*>(&rm[f]), (unsigned long long)q.mem);
                if (EPH_COLS) atomicAdd(reinterpret_cast<unsigned long long*>(reinterpret_cast<unsigned long long*>(&re[f])), (unsigned long long)q.eph);
                atomicAdd(&rp[f], 1);
            }
            // the destinations' rows grew back: their blocks' skylines are unknown (and dirty);
            // the candidate's own block is unknown already (its RemovePods)
            uint64_t* const dmask = reinterpret_cast<uint64_t*>(scratch);
            if (lane < 2) dmask[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            for (int half = 0; half < 2; half++) {
                const int32_t t = half * 64 + lane;
                if (t >= placed) continue;
                const int32_t f = half ? d1 : d0, j = f >> 6;
                sky.n[j] = -1;
                atomicOr(reinterpret_cast<unsigned long long*>(dmask + (j >> 6)), 1ull << (j & 63));
            }
            __builtin_amdgcn_wave_barrier();
            dirty0 |= pc_uni64(dmask[0]);
            dirty1 |= pc_uni64(dmask[1]);
            if (lane == 0) {
                rc[node] = wsub(rc[node], sc); rm[node] = wsub(rm[node], sm); rp[node] -= cnt;
                if (EPH_COLS) re[node] = wsub(re[node], se);
                sky.n[jn] = -1;             // (built without this candidate while it ran)
            }
            PC_MARK_DIRTY(jn);
            cj = -1;                                                                 // rows changed
            r.reason = CA_UNREMOVABLE_NO_PLACE;                                      // cluster.go:174-177
            PC_SIM_MARK(PC_REVERT);
        }
        // Hints.Set of this candidate's pods (hints persist whether or not it is removable): the
        // caller's pods (the first m0 of the list) by move index; the copies' keys are not the
        // caller's (a later candidacy reads a copy's hint from its record)
        if (hs0 != INT32_MIN && lane < m0) a.hout[mo + lane] = hs0;
        if (hs1 != INT32_MIN && 64 + lane < m0) a.hout[mo + 64 + lane] = hs1;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        ctx->Lw = Lw;
        if (moved_L) ctx->Lraw = Lw;
        ctx->dirty0 = dirty0;
        ctx->dirty1 = dirty1;
        ctx->r = r;
    }
    __builtin_amdgcn_wave_barrier();
}

template <bool EPH_COLS>
__global__ void __launch_bounds__(PC_MAX_WAVES * 64) k_plan_chain(PcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pc_raw[];
    const int32_t n = a.n, nb = (n + 63) >> 6;
    const PcLayout Y = pc_layout(n, EPH_COLS);
    const int nh = (int)(blockDim.x >> 6) - 1;                  // helper waves
#ifdef CASIM_PROF
    const uint64_t t_init0 = clock64();
#endif
    {
        // ---- the committed rows and bit planes into LDS: every wave of the workgroup
        // loads its share of the 64-node blocks (4 in flight per lane) ----
        const PcRows R_ = pc_rows(pc_raw, Y);
        int64_t* const rc = R_.c;
        int64_t* const rm = R_.m;
        int64_t* const re = R_.e;
        int32_t* const rp = R_.p;
        PcBlk* const blk = reinterpret_cast<PcBlk*>(pc_raw + Y.blk);
        uint16_t* const excnt = reinterpret_cast<uint16_t*>(pc_raw + Y.excnt);
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
        for (int32_t i = (int32_t)threadIdx.x; i <= n; i += (int32_t)blockDim.x) R_.exb[i] = a.ex_base[i];
        for (int32_t b0 = 4 * wv; b0 < nb; b0 += 4 * nw) {
            NodeHot h[4];
            uint8_t dm[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int32_t i = (b0 + u) * 64 + lane;
                h[u] = NodeHot{};
                dm[u] = 0;
                if (b0 + u < nb && i < n) { h[u] = a.hot[i]; dm[u] = a.dest_mask[i]; }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int32_t j = b0 + u;
                if (j >= nb) break;
                const int32_t i = j * 64 + lane;
                const bool valid = i < n;
                if (valid) {
                    rc[i] = h[u].cpu; rm[i] = h[u].mem; rp[i] = h[u].pods; excnt[i] = 0;
                    if (EPH_COLS) re[i] = h[u].eph;
                }
                const uint64_t dw = __ballot(valid && dm[u] != 0);
                const uint64_t uw = __ballot(valid && (h[u].flags & NF_UNSCHED));
                const uint64_t tw = __ballot(valid && (h[u].flags & NF_TAINTS));
                const uint64_t ew = __ballot(valid && h[u].eph >= 0);
                if (lane == 0) {
                    blk[j].dest = dw; blk[j].vis = dw & ~uw; blk[j].usch = uw; blk[j].taint = tw;
                    if (!EPH_COLS) blk[j].eph = ew;
                    reinterpret_cast<int32_t*>(pc_raw + Y.sky)[j] = -1;      // unknown until a scan reads it
                }
            }
        }
        PcHelp* const hq = reinterpret_cast<PcHelp*>(pc_raw + Y.help);
        if (threadIdx.x == 0) { hq->seq = 0; hq->quit = 0; hq->done = 0; hq->best = INT32_MAX; }
        __syncthreads();                                        // (the one workgroup barrier)
        if (threadIdx.x >= 64) {
            pc_helper<EPH_COLS>(a, pc_raw, (int)(threadIdx.x >> 6) - 1, nh);
            return;
        }
    }
    const int lane = threadIdx.x;
    PcBlk* const blk = reinterpret_cast<PcBlk*>(pc_raw + Y.blk);
    uint16_t* const excnt = reinterpret_cast<uint16_t*>(pc_raw + Y.excnt);  // copies committed per node
    ca_plan_result* const resbuf = reinterpret_cast<ca_plan_result*>(pc_raw + Y.resbuf);
    ca_plan_move* const mvbuf = reinterpret_cast<ca_plan_move*>(pc_raw + Y.mvbuf);
    // Global stores are kept out of the pod loop: on gfx9 a store counts in vmcnt, so any
    // later vmcnt wait (the compiler's, for a register a load may still write) would wait
    // for it.  Results and moves are staged in LDS and written in bulk; hints and the
    // copies' records are written once per candidate, behind the next candidate's prefetch.
    auto flush_res = [&](int32_t c0, int32_t k) {       // resbuf[0, k) -> res[c0, c0 + k)
        if (lane < k) {
            const int32_t* src = reinterpret_cast<const int32_t*>(resbuf + lane);
            int32_t* dst = reinterpret_cast<int32_t*>(a.res + c0 + lane);
            for (int w = 0; w < (int)(sizeof(ca_plan_result) / 4); w++) dst[w] = src[w];
        }
    };
    PcCtx* const ctx = reinterpret_cast<PcCtx*>(pc_raw + Y.ctx);
#ifdef CASIM_PROF
    uint64_t prof[PC_NPROF];
    for (int k = 0; k < PC_NPROF; k++) prof[k] = 0;
    const uint64_t t_start = t_init0;
#endif

    __builtin_amdgcn_wave_barrier();
#ifdef CASIM_PROF
    prof[PC_INIT] = clock64() - t_init0;
#endif

    if (lane == 0) {
        int32_t Lw = 0;
        if (n > 0) { Lw = (int32_t)(a.L0 % n); if (Lw < 0) Lw += n; }
        ctx->Lw = Lw;
        ctx->Lraw = (int32_t)a.L0;                    // Go keeps the int until a scan succeeds
        ctx->nm = 0; ctx->mv_n = 0; ctx->mv_first = 0; ctx->removed = 0; ctx->bulk_fail = 0; ctx->bulk_skip = 0;
        ctx->dirty0 = ~0ull; ctx->dirty1 = ~0ull;
#ifdef CASIM_PROF
        for (int k = 0; k < PC_NPROF; k++) ctx->prof[k] = 0;
#endif
    }
    __builtin_amdgcn_wave_barrier();
    int32_t nm = 0, removed = 0, simulated = 0;
    bool cut = false, stopped = false;
    int32_t stop_c = a.C;
    int32_t hb_node = -1, hb_st = 0, hb_mo = 0, hb_m1 = 0;    // candidate headers, lane k = c0 + k
    // the next candidate's first 64 pods, loaded while the current one runs
    PcPod nx = {};
    if (a.C > 0) nx = pc_load(a.pods + a.move_off[0] + lane);

    for (int32_t c = 0; c < a.C; c++) {
        const int sl = c & 63;
        if (sl == 0) {
            const int32_t k = c + lane;
            if (k < a.C) {
                hb_node = a.cands[k];
                hb_st = a.status ? a.status[k] : 0;
                hb_mo = a.move_off[k];
                hb_m1 = a.move_off[k + 1];
            }
        }
        PcReg r0 = pc_reg(nx);                                    // pods t = lane
        PcReg r1 = {};                                            // pods t = 64 + lane
        r1.id = -1; r1.hint = -1; r1.orig = -1;
        const int32_t mo1 = pc_rl32(hb_m1, sl);                  // = the next candidate's move_off
        if (c + 1 < a.C) nx = pc_load(a.pods + mo1 + lane);
        if (cut || (a.max_removable > 0 && removed >= a.max_removable)) {       // planner.go:268-271
            flush_res(c - sl, sl);
            stopped = true;
            stop_c = c;                                  // (the host fills the rest: NOT_RUN)
            break;
        }
        PC_T0();
        const int32_t node = pc_rl32(hb_node, sl), stc = pc_rl32(hb_st, sl);
        const int32_t mo = pc_rl32(hb_mo, sl), m0 = mo1 - mo;
        ca_plan_result r;
        r.removable = 0; r.reason = CA_UNREMOVABLE_NONE; r.n_placed = 0;
        r.last_index_in = __builtin_amdgcn_readfirstlane(ctx->Lraw);
        r.evals = 0; r.first_move = nm; r.n_moves = 0; r.blocking_pod = -1; r.risky = 0;
        const bool valid = node >= 0 && node < n && ((pc_uni64(blk[(node) >> 6].dest) >> ((node) & 63)) & 1ull);
        int32_t cnt = m0;
        if (valid && stc == 0) {
            // GetPodsToMove on the committed snapshot: the caller's list, then the copies
            // committed onto this node (NodeInfo.Pods appends)
            const int32_t ne = __builtin_amdgcn_readfirstlane(excnt[node]);
            cnt = m0 + ne;
            if (cnt > PC_LIST) {
                cut = true;                                                         // casim.h scope
            } else {
                if (m0 > 64) r1 = pc_reg(pc_load(a.pods + mo + 64 + lane));
                if (ne > 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    const PcPod* ex = a.ex_pods + __builtin_amdgcn_readfirstlane(
                                                      reinterpret_cast<const int32_t*>(pc_raw + Y.exb)[node]);
                    const int32_t t0 = lane, t1 = 64 + lane;
                    if (t0 >= m0 && t0 < cnt) r0 = pc_reg(pc_load(ex + (t0 - m0)));
                    if (t1 >= m0 && t1 < cnt) r1 = pc_reg(pc_load(ex + (t1 - m0)));
                }
                const bool oos = (lane < cnt && (r0.flags & PF_OUT_OF_SCOPE)) ||
                                 (64 + lane < cnt && (r1.flags & PF_OUT_OF_SCOPE));
                if (__ballot(oos)) cut = true;
            }
            if (cut) {
                r.reason = CA_UNREMOVABLE_OUT_OF_SCOPE;
                if (lane == 0) resbuf[sl] = r;
                if (sl == 63) flush_res(c - 63, 64);
                continue;
            }
        }
        PC_MARK(PC_LISTS);
        if (!valid) {
            r.reason = CA_UNREMOVABLE_UNEXPECTED_ERROR;                              // cluster.go:157-160
        } else if (stc != 0) {
            r.reason = stc;                                                          // :162-169
        } else if (a.n_pdbs > 0) {
            // ---- checkPdbs against the remaining budgets (drain.go:73-90) ----
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            auto lowest = [&](int32_t t, int32_t o) {           // lowest blocked PDB of pod t
                int32_t best = INT32_MAX;
                if (t < cnt)
                    for (int32_t k = a.pdb_off[o]; k < a.pdb_off[o + 1]; k++) {
                        const int32_t p = a.pdb_pod[k];
                        if (pc_ld(a.allowed + p) < 1) { best = p; break; }   // memberships ascend
                    }
                return best;
            };
            const int32_t pm0 = lowest(lane, r0.orig), pm1 = lowest(64 + lane, r1.orig);
            const int32_t pmin = __ockl_wfred_min_i32(pm0 < pm1 ? pm0 : pm1);
            if (pmin != INT32_MAX) {
                const uint64_t b0 = __ballot(pm0 == pmin), b1 = __ballot(pm1 == pmin);
                r.blocking_pod = b0 ? pc_rl32(r0.id, __builtin_ctzll(b0)) : pc_rl32(r1.id, __builtin_ctzll(b1));
                r.reason = CA_UNREMOVABLE_BLOCKED_BY_POD;
            }
        }
        PC_MARK(PC_PDB);
        if (r.reason != CA_UNREMOVABLE_NONE) {
            if (lane == 0) resbuf[sl] = r;
            if (sl == 63) flush_res(c - 63, 64);
            continue;
        }
        simulated++;
        if (lane == 0) ctx->r = r;
        __builtin_amdgcn_wave_barrier();
        pc_simulate<EPH_COLS>(a, pc_raw, ctx, c, mo, m0, node, cnt, r0, r1, nh);
        r = ctx->r;
        nm = __builtin_amdgcn_readfirstlane(ctx->nm);
        removed = __builtin_amdgcn_readfirstlane(ctx->removed);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) resbuf[sl] = r;
        if (sl == 63) flush_res(c - 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {                                            // the helper waves exit
        PcHelp* const hq = reinterpret_cast<PcHelp*>(pc_raw + Y.help);
        __hip_atomic_store(&hq->quit, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (!stopped && a.C > 0 && ((a.C - 1) & 63) != 63) flush_res((a.C - 1) & ~63, ((a.C - 1) & 63) + 1);
    pc_flush_moves(a, mvbuf, ctx, lane);
    if (lane == 0) {
        a.info[0] = ctx->Lraw;
        a.info[1] = nm;
        a.info[2] = removed;
        a.info[3] = simulated;
        a.info[4 + PC_NPROF] = stop_c;
#ifdef CASIM_PROF
        prof[PC_TOTAL] = clock64() - t_start;
        for (int k = 0; k < PC_NPROF; k++) a.info[4 + k] = (int64_t)(prof[k] + ctx->prof[k]);
#else
        for (int k = 0; k < PC_NPROF; k++) a.info[4 + k] = 0;
#endif
    }
}

}  // namespace casim

using namespace casim;

namespace casim {

// 1 = ran, 0 = outside the chain's scope (the caller takes the speculative path), < 0 error.
// *last_index is an out-value only (the caller passes a copy); hints come back in hints_out.
int plan_chain_run(ca_mirror* m, const int32_t* candidates, int32_t C, const uint8_t* dest_mask,
                   const int32_t* cand_status, const int32_t* move_off, const int32_t* move_pods,
                   int32_t max_removable, const ca_pdb_table* pdbs, int32_t* hints, int32_t n_pods,
                   int32_t* last_index, ca_plan_result* results, std::vector<ca_plan_move>& moves_out,
                   std::vector<std::pair<int32_t, int32_t>>& hint_sets, int32_t* simulated_out) {
    if (knob_env("CASIM_PLAN_SPECULATIVE")) return 0;
    const auto t_entry = std::chrono::steady_clock::now();
    const int32_t N = (int32_t)m->nodes.size();
    if (N <= 0 || C <= 0) return 0;
    const int32_t M = move_off[C];
    // (mirror-wide counters first: no per-pod pass when no pod has ports, extended
    // resources or ephemeral requests)
    bool eph_cols = false;
    if (m->n_ext_pods > 0 || m->n_eph_pods > 0)
        for (int32_t i = 0; i < M; i++) {
            const ca_pod_spec& s = m->pods[move_pods[i]].spec;
            if (m->n_ext_pods > 0 && (pod_dev_flags(s) & (PF_PORTS | PF_MOVED_SCALAR_REQ))) return 0;
            if (s.req_ephemeral != 0) eph_cols = true;
        }
    const PcLayout Y = pc_layout(N, eph_cols);
    if (Y.total > PC_LDS_MAX || N > PC_MAX_NODES) return 0;
    const int P = pdbs ? pdbs->n_pdbs : 0;
    {   // each pod in at most one candidate's list (its hint is packed before the loop runs)
        std::vector<uint8_t> seen((size_t)std::max(n_pods, 1), 0);
        for (int32_t i = 0; i < M; i++) {
            if (seen[move_pods[i]]) return 0;
            seen[move_pods[i]] = 1;
        }
    }

    // copies: at most one per free pod slot of its destination (every AddPod passes the
    // pod-count check; a node's own pods leave only when it is removed)
    std::vector<int32_t> ex_base((size_t)N + 1);
    int64_t cap = 0;
    for (int32_t i = 0; i < N; i++) {
        ex_base[i] = (int32_t)cap;
        const NodeRow& nd = m->nodes[i];
        const int64_t free_slots = nd.spec.alloc_pods - nd.npods;
        if (free_slots > 65535) return 0;                       // the per-node copy counters are 16-bit
        cap += free_slots > 0 ? free_slots : 0;
        if (cap > INT32_MAX / 64) return 0;
    }
    ex_base[N] = (int32_t)cap;
    const int32_t copy_cap = (int32_t)std::max<int64_t>(cap, 1);
    const int32_t base = (int32_t)m->pods.size();
    if ((int64_t)base + copy_cap > INT32_MAX) return 0;

    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    if ((rc = m->sync_nodes()) != CA_OK) return rc;
    // the chain reads the device records of the caller's pods only (copies it packs itself)
    if (m->d_pods_synced < (size_t)n_pods && (rc = m->sync_pods()) != CA_OK) return rc;
    const auto t_sync = std::chrono::steady_clock::now();
    PlanChainScratch& S = m->pc;
    hipStream_t st = m->stream;

    // packed inputs (one H2D): cands, status, move_off, move_pods, ex_base, pdb tables, the
    // caller's hint of every pod to move (by move index); mask
    const size_t n_pdb_members = P > 0 ? (size_t)pdbs->pod_off[n_pods] : 0;
    const size_t in_words = (size_t)C + C + (C + 1) + std::max(M, 1) + (N + 1) + (P > 0 ? (size_t)n_pods + 1 : 1) +
                            std::max<size_t>(n_pdb_members, 1) + std::max(P, 1) + std::max(M, 1);
    const size_t in_bytes = 4 * in_words + ((size_t)N + 15) / 16 * 16 + 16;      // (+ the hints' alignment)
    if ((rc = S.in.reserve(in_bytes)) != CA_OK) return rc;
    if ((rc = S.h_in.reserve(in_bytes)) != CA_OK) return rc;
    int32_t* hw = S.h_in.as<int32_t>();
    size_t o = 0;
    auto put = [&](const int32_t* src, size_t k, size_t room) {
        const size_t at = o;
        if (src && k) std::memcpy(hw + o, src, 4 * k);
        else if (room) std::memset(hw + o, 0, 4 * room);
        o += room;
        return at;
    };
    const size_t o_c = put(candidates, C, C);
    const size_t o_st = put(cand_status, cand_status ? C : 0, C);
    const size_t o_off = put(move_off, C + 1, C + 1);
    const size_t o_mv = put(move_pods, M, std::max(M, 1));
    const size_t o_exb = put(ex_base.data(), N + 1, N + 1);
    const size_t o_pof = put(P > 0 ? pdbs->pod_off : nullptr, P > 0 ? n_pods + 1 : 0, P > 0 ? (size_t)n_pods + 1 : 1);
    const size_t o_pp = put(P > 0 ? pdbs->pod_pdb : nullptr, n_pdb_members, std::max<size_t>(n_pdb_members, 1));
    const size_t o_al = put(P > 0 ? pdbs->allowed : nullptr, P, std::max(P, 1));
    const size_t o_mask = 4 * o;
    std::memcpy(reinterpret_cast<unsigned char*>(hw) + o_mask, dest_mask, (size_t)N);
    // the hints by move index last: not uploaded when none is set (a fresh loop's)
    const size_t o_hm = (o_mask + (size_t)N + 15) / 16 * 4;
    int32_t any_hint = 0;
    for (int32_t i = 0; i < M; i++) {
        const int32_t h = hints ? hints[move_pods[i]] : -1;
        hw[o_hm + i] = h;
        any_hint |= h + 1;                      // (hints are >= -1)
    }
    const size_t up_bytes = any_hint ? 4 * (o_hm + (size_t)std::max(M, 1)) : o_mask + (size_t)N;
    int32_t* const din = S.in.as<int32_t>();
    const auto t_pack = std::chrono::steady_clock::now();
    const bool dbg_t = knob_env("CASIM_DEBUG_TIMING") != nullptr;
    struct DbgEvents {                                            // (CASIM_DEBUG_TIMING: H2D and pack times)
        hipEvent_t e[3] = {nullptr, nullptr, nullptr};
        ~DbgEvents() { for (auto& x : e) if (x) (void)hipEventDestroy(x); }
    } dbg_ev;
    hipEvent_t* const dev = dbg_ev.e;                            // (destroyed on every return path)
    if (dbg_t) for (int i = 0; i < 3; i++) if (hipEventCreate(&dev[i]) != hipSuccess) dev[i] = nullptr;
    if (dev[0]) (void)hipEventRecord(dev[0], st);
    CA_HIP_CHECK(hipMemcpyAsync(din, hw, up_bytes, hipMemcpyHostToDevice, st));
    if (dev[1]) (void)hipEventRecord(dev[1], st);

    // device work: the packed pods to move [M + 64], the copies [copy_cap]
    const size_t w_bytes = sizeof(PcPod) * ((size_t)M + 64) + sizeof(PcPod) * (size_t)copy_cap;
    if ((rc = S.work.reserve(w_bytes)) != CA_OK) return rc;
    PcPod* const dpods = S.work.as<PcPod>();
    PcPod* const dex = dpods + M + 64;
    hipLaunchKernelGGL(k_plan_pack, dim3((unsigned)((M + 64 + 255) / 256)), dim3(256), 0, st, din + o_mv, M,
                       m->d_pods.hot.as<PodHot>(), any_hint ? (const int32_t*)(din + o_hm) : nullptr, dpods);
    CA_HIP_CHECK(hipGetLastError());
    if (dev[2]) (void)hipEventRecord(dev[2], st);
    // outputs, written by the kernel straight into page-locked memory (no copies, one sync):
    // results [C], info [PC_INFO], moves [copy_cap], the caller's pods' hints by move index [M]
    const size_t out_bytes = sizeof(ca_plan_result) * C + PC_INFO * sizeof(int64_t) + sizeof(ca_plan_move) * copy_cap +
                             sizeof(int32_t) * (size_t)std::max(M, 1) + 64;
    if ((rc = S.h_out.reserve(out_bytes)) != CA_OK) return rc;
    ca_plan_result* const hres = S.h_out.as<ca_plan_result>();
    int64_t* const hinfo = reinterpret_cast<int64_t*>(hres + C);
    ca_plan_move* const hmoves = reinterpret_cast<ca_plan_move*>(hinfo + PC_INFO);
    int32_t* const hhout = reinterpret_cast<int32_t*>(hmoves + copy_cap);
    std::memcpy(hhout, hw + o_hm, sizeof(int32_t) * (size_t)M);     // unchanged unless Hints.Set
    int32_t* const hpub = hhout + std::max(M, 1);                      // moves published so far
    __atomic_store_n(hpub, 0, __ATOMIC_RELAXED);
    void* dout = nullptr;
    CA_HIP_CHECK(hipHostGetDevicePointer(&dout, S.h_out.ptr, 0));
    ca_plan_result* const dres = static_cast<ca_plan_result*>(dout);
    int64_t* const dinfo = reinterpret_cast<int64_t*>(dres + C);
    ca_plan_move* const dmoves = reinterpret_cast<ca_plan_move*>(dinfo + PC_INFO);
    int32_t* const dhout = reinterpret_cast<int32_t*>(dmoves + copy_cap);
    int32_t* const dpub = dhout + std::max(M, 1);

    PcArgs A;
    A.hot = m->d_hot.as<NodeHot>();
    A.st = m->d_static.as<NodeStatic>();
    A.n = N;
    A.dest_mask = reinterpret_cast<const uint8_t*>(reinterpret_cast<unsigned char*>(din) + o_mask);
    A.cands = din + o_c;
    A.status = din + o_st;
    A.move_off = din + o_off;
    A.pods = dpods;
    A.C = C;
    A.specs = m->d_pods.spec.as<ca_pod_spec>();
    A.terms = m->d_pods.terms.as<ca_selector_term>();
    A.reqs = m->d_pods.reqs.as<ca_selector_req>();
    A.names = m->d_pods.names.as<int32_t>();
    A.base = base;
    A.max_removable = max_removable;
    A.n_pdbs = P;
    A.allowed = din + o_al;
    A.pdb_off = din + o_pof;
    A.pdb_pod = din + o_pp;
    A.hout = dhout;
    A.ex_base = din + o_exb;
    A.ex_pods = dex;
    A.res = dres;
    A.moves = dmoves;
    A.published = dpub;
    A.info = dinfo;
    A.L0 = *last_index;
    A.copy_cap = copy_cap;
    A.trace = nullptr;
    A.trace_cap = 0;
    A.help_after = PC_HELP_AFTER;
    if (const char* e = knob_env("CASIM_PLAN_HELP_AFTER")) A.help_after = std::max(1, atoi(e));
    A.dbg = test_hook_env("CASIM_PLAN_DBG") ? atoi(test_hook_env("CASIM_PLAN_DBG")) : 0;
    const char* tr_env = test_hook_env("CASIM_PLAN_TRACE");
    DevBuf trace;
    if (tr_env) {
        A.trace_cap = 4096;
        if ((rc = trace.reserve(sizeof(int32_t) * (16 + 16 * (size_t)A.trace_cap))) != CA_OK) return rc;
        int32_t hdr[2] = {0, std::max(0, std::min(N - 1, atoi(tr_env)))};
        CA_HIP_CHECK(hipMemcpy(trace.ptr, hdr, sizeof hdr, hipMemcpyHostToDevice));
        A.trace = trace.as<int32_t>();
    }
    const void* kfn = eph_cols ? (const void*)k_plan_chain<true> : (const void*)k_plan_chain<false>;
    if ((rc = ensure_dyn_lds(kfn, Y.total)) != CA_OK) return rc;
    CA_HIP_CHECK(hipEventRecord(m->ev0, st));
    // the chain wave plus helper waves for long scans (CASIM_PLAN_HELPERS: 0..7, default 7)
    int waves = PC_MAX_WAVES;
    if (const char* e = knob_env("CASIM_PLAN_HELPERS")) waves = 1 + std::max(0, std::min(PC_MAX_WAVES - 1, atoi(e)));
    if (eph_cols) hipLaunchKernelGGL(k_plan_chain<true>, dim3(1), dim3(64 * waves), Y.total, st, A);
    else hipLaunchKernelGGL(k_plan_chain<false>, dim3(1), dim3(64 * waves), Y.total, st, A);
    CA_HIP_CHECK(hipGetLastError());
    CA_HIP_CHECK(hipEventRecord(m->ev1, st));
    if (P > 0) CA_HIP_CHECK(hipMemcpyAsync(hw + o_al, din + o_al, 4 * (size_t)P, hipMemcpyDeviceToHost, st));
    // ---- replay the committed moves into the mirror (journaled at the caller's depth) while
    // the chain runs: it publishes each flushed batch of whole candidates' moves through *hpub
    // (cluster.go:228-240, :79) ----
    int32_t replayed = 0;
    float replay_ms = 0;
    auto replay_upto = [&](int32_t upto) -> int {
        const auto tr = std::chrono::steady_clock::now();
        const int e = m->replay_moves(hmoves + replayed, upto - replayed);
        replay_ms += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - tr).count();
        replayed = upto;
        return e;
    };
    for (;;) {
        const int32_t pub = __atomic_load_n(hpub, __ATOMIC_ACQUIRE);
        if (pub > replayed && pub <= copy_cap) {
            if ((rc = replay_upto(pub)) != CA_OK) {
                (void)hipStreamSynchronize(st);           // (the chain still writes into the buffers)
                return rc;
            }
            continue;
        }
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) CA_HIP_CHECK(q);
        std::this_thread::yield();
    }
    CA_HIP_CHECK(hipStreamSynchronize(st));
    const auto t_kernel = std::chrono::steady_clock::now();
    if (tr_env) {
        std::vector<int32_t> tb(16 + 16 * (size_t)A.trace_cap);
        CA_HIP_CHECK(hipMemcpy(tb.data(), trace.ptr, sizeof(int32_t) * tb.size(), hipMemcpyDeviceToHost));
        for (int32_t k = 0; k < std::min(tb[0], A.trace_cap); k++) {
            const int32_t* e = tb.data() + 16 + 16 * k;
            fprintf(stderr, "[plan trace] cand %d pod %d/%d (id %d spec %d cpu %d mem %dMi) hint %d flags %x -> %d evals %d "
                    "L %d | node %d: cpu %d mem %dMi pods %d bits %x\n", e[0], e[1], e[7], e[15], e[14], e[8], e[9],
                    e[2], e[3], e[4], e[5], e[6], tb[1], e[10], e[11], e[12], e[13]);
        }
    }
    const int32_t nm = (int32_t)hinfo[1];
    const int32_t stop_c = (int32_t)hinfo[4 + PC_NPROF];
    if (nm < replayed || nm > copy_cap || stop_c < 0 || stop_c > C) {
        set_last_error("plan chain: move count out of range");
        return CA_EDEVICE;
    }
    std::memcpy(results, hres, sizeof(ca_plan_result) * (size_t)stop_c);
    for (int32_t k = stop_c; k < C; k++) {                     // planner.go:268-271: not run
        ca_plan_result& r = results[k];
        r.removable = 0; r.reason = CA_UNREMOVABLE_NOT_RUN; r.n_placed = 0; r.last_index_in = (int32_t)hinfo[0];
        r.evals = 0; r.first_move = nm; r.n_moves = 0; r.blocking_pod = -1; r.risky = 0;
    }
    *last_index = (int32_t)hinfo[0];
    if (simulated_out) *simulated_out = (int32_t)hinfo[3];
    hint_sets.clear();
    if (hints)                                                  // Hints.Set of the caller's pods that ran
        for (int32_t i = 0; i < move_off[stop_c]; i++)
            if (hhout[i] != hw[o_hm + i]) hint_sets.emplace_back(move_pods[i], hhout[i]);
    if (P > 0) std::memcpy(pdbs->allowed, hw + o_al, 4 * (size_t)P);
    const auto t_read = std::chrono::steady_clock::now();
    const float overlapped_ms = replay_ms;
    if (nm > replayed && (rc = replay_upto(nm)) != CA_OK) return rc;        // the rest (the last flush)
    const auto t_end = std::chrono::steady_clock::now();
    moves_out.assign(hmoves, hmoves + nm);
    {
        PlanStats& ps = m->plan;
        auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<float, std::milli>(b - a).count();
        };
        float kms = 0;
        (void)hipEventElapsedTime(&kms, m->ev0, m->ev1);
        ps.chain_prof.assign(hinfo + 4, hinfo + 4 + PC_NPROF);
        ps.host_ms[0] = ms(t0, t_sync);          // mirror row / pod sync
        ps.host_ms[1] = ms(t_sync, t_kernel);    // inputs, kernel, results back
        ps.host_ms[2] = kms;                     // the kernel (events)
        ps.host_ms[3] = ms(t_kernel, t_read);    // moves, hints, budgets back
        ps.host_ms[4] = ms(t_read, t_end);       // replay into the mirror after the chain (the rest overlapped it)
        if (dbg_t && dev[0] && dev[1] && dev[2]) {
            float h2d = 0, pk = 0, gap = 0;
            (void)hipEventElapsedTime(&h2d, dev[0], dev[1]);
            (void)hipEventElapsedTime(&pk, dev[1], dev[2]);
            (void)hipEventElapsedTime(&gap, dev[2], m->ev0);
            fprintf(stderr, "[plan chain] device: H2D %.3f (%zu B)  pack %.3f  to the chain %.3f ms\n", h2d,
                    up_bytes, pk, gap);
        }
        if (dbg_t)
            fprintf(stderr, "[plan chain] checks %.3f  sync %.3f  pack %.3f  launch+kernel %.3f (kernel %.3f)  readback %.3f  "
                    "replay %.3f ms after the chain, %.3f ms beside it (C %d, M %d, N %d)\n", ms(t_entry, t0), ps.host_ms[0],
                    ms(t_sync, t_pack), ms(t_pack, t_kernel), ps.host_ms[2], ps.host_ms[3], ps.host_ms[4], overlapped_ms, C, M, N);
    }
    return 1;
}

}  // namespace casim
