// dgn_api.cpp — the extern "C" boundary (include/dgn.h): contexts, workspaces, launch
// sequencing, per-kernel event timing, host staging and the synthetic batch generator.
// Nothing here computes results on the CPU: there is no fallback path; without a GPU every
// compute entry point returns DGN_ERR_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/dgn.h"
#include "dgn_internal.hpp"

using namespace dgn;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    hipError_t ensure(size_t want) {
        if (want <= bytes && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t b = std::max<size_t>(want, 256);
        hipError_t e = hipMalloc(&p, b);
        if (e == hipSuccess) bytes = b;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

struct KernelStat {
    int64_t launches = 0;
    double total_ms = 0.0;
    double bytes = 0.0;
    double flops = 0.0;
};

struct PendingEvent {
    std::string name;
    hipEvent_t start, stop;
};

struct Scalars {  // device-side scalars, one allocation
    int64_t total;
    unsigned long long sum_sq;  // sum over atoms of (candidates + 1)^2
    unsigned long long sum_m;   // sum over atoms of candidates (every neighbour within rc)
    unsigned long long wide_atoms;  // atoms with 64 < candidates + 1 <= kWideRegular (low), above (high)
    uint32_t max_candidates;
    uint32_t max_natoms;        // largest structure of the batch (prep)
    uint32_t graph_flag;        // graph error bits kGErr* (prep, emit, Betti search)
    uint32_t error_flag;        // Betti reduction error bits
    uint32_t work_counter;      // betti main launch queue
    uint32_t work_counter2;     // betti overflow launch queue
    uint32_t overflow_len;      // complexes routed to the overflow launch
    uint32_t wide_queue;        // betti wide launch queue
    uint32_t wide_len;          // complexes routed to the wide launch
    uint32_t retry_len;         // complexes routed to the capacity-retry launch
    uint32_t retry_queue;       // capacity-retry launch queue
    uint32_t dense_len;         // complexes routed to the dense (NP = 64) launch by the main one
    uint32_t dense_queue;       // betti dense launch queue
    uint32_t retry2_len;        // second-level list of the device-driven retry launch (host entry points)
};

// one neighbour pass's device workspace and the facts its count recorded (count -> emit handshake)
struct GraphWork {
    DevBuf meta, counts, block_sums, block_aux, atom_struct, cell_start, cell_pos, mask, weight, defer;
    bool have = false;
    bool has_weight = false;  // weight[] holds the 1/count(species) Betti weights of this batch
    const double* pos = nullptr;
    const int32_t* species = nullptr;  // the species array the weights were computed from
    int64_t atoms = -1, structs = -1;
    double rc = 0, eps = 0;
    uint64_t k = 0;
    int qa = kQA;  // query atoms per count / emit block (graph_tile_atoms)
    uint32_t max_candidates = 0, max_natoms = 0;
    int64_t edges = 0;
    double sum_sq = 0;
    double sum_m = 0;  // neighbours within rc over the batch (the K = inf edge count)
    int64_t wide_atoms = 0, huge_atoms = 0;  // local complexes of 65..kWideRegular / more points
};

// host-pinned mirror: the scalars after a count pass, and the emit's deferred error flag
struct HostScalars {
    Scalars s;
    uint32_t emit_flag;  // copied asynchronously after every graph emit
    uint32_t pad;
    uint32_t betti_flags[2];  // copied asynchronously after every Betti pass: search, reduction bits
};

// sticky device words of the Betti pass (context lifetime; never cleared by a count pass): the
// Betti search's consistency bits, the reduction's error bits, and the number of complexes the
// capacity-retry launches reduced. A pass ORs into the first two; take_betti_flag clears them once
// the host has read them.
enum { kBFSearch = 0, kBFReduce = 1, kBFRetried = 2, kBFWords = 4 };

}  // namespace

struct dgn_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string last_error;
    // neighbour-pass workspaces: `gw` for dgn_dev_graph_count -> dgn_dev_graph_emit, `bw` for the
    // Betti pass's own NeighborList(rc, SIZE_MAX) (so a Betti call between a graph count and its
    // emit does not disturb the handshake)
    GraphWork gw, bw;
    DevBuf scalars;
    HostScalars* host = nullptr;  // pinned
    bool emit_pending = false;    // an emit's error flag is on its way to host->emit_flag
    bool betti_pending = false;   // a Betti pass's flags are on their way to host->betti_flags
    DevBuf bflags;                // [kBFWords] sticky Betti words (above)
    int big_nmax = 0, big_waves = 0;  // capacity-retry workspace (b_big) the tables were initialised for
    int64_t big_budget = 0;           // bytes the device-driven retry workspace may take (first use)
    int64_t host_syncs = 0;           // host waits on the stream (dgn_debug_host_syncs)
    // betti workspace
    DevBuf b_scratch, b_list, b_lower, b_np, b_w, b_wlist, b_wide, b_rlist, b_rlist2, b_big, b_rank, b_rscal, b_rank16,
        b_rscal16, b_walk;
    int betti_slots = 0;
    bool scratch_fresh = false;  // b_scratch (re)allocated: min-cofacet tables need initialising
    // overflow-tier fork (side stream + events), created on first use
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int cus = 0;  // compute units of the device (device_cus)
    int wide_nmax = 0, wide_waves = 0, wide_cap = 0;  // layout the wide scratch's tables were initialised for
    int wide_pre = -1;
    // debug / A-B knobs (dgn_ctx_set_debug; never read from the environment)
    bool dbg_force_retry = false;  // every complex of a Betti pass through the capacity-retry launch
    int dbg_wide_waves = 0;        // cap on the wide launch's resident waves (0 = none)
    int dbg_wide_cap = 0;          // regular wide layout's column / pivot / pair table cap (0 = natural)
    bool dbg_wide_c16 = true;      // u16 rank codes for wide complexes of <= kC16MaxPoints points
    hipStream_t rstream = nullptr;  // the 10 A reductions beside the next slice's walk pass
    hipEvent_t ev_walk[2] = {nullptr, nullptr}, ev_red[2] = {nullptr, nullptr};
    bool dbg_wide_walk = true;     // the u16-coded complexes' dim-2 walk as a workgroup-per-complex pass
    int dbg_split_chunk = 0;       // clouds per chunk of the component split (0 = its byte budget)
    int dbg_big_log2 = 0;          // capacity-retry layout's first-level table size log2 (0 = natural 24)
    int dbg_emit_chunk = 0;        // tiles per launch of the large-row emit (0 = the byte budget's)
    // host staging
    DevBuf h_lat, h_pos, h_spec, h_off;
    DevBuf dist_scratch;  // emit distance rows when the caller wants an RBF but no distances
    DevBuf emit_keys;     // the large-row emit's per-wave key rows (graph_emit_cap == kEmitGlobalKeys)
    // timing
    bool timing = false;
    std::vector<PendingEvent> pending;
    std::vector<hipEvent_t> free_events;
    std::map<std::string, KernelStat> stats;
    std::vector<std::string> order;
};

namespace {

int fail(dgn_ctx* c, int status, const std::string& msg) {
    if (c) c->last_error = msg;
    return status;
}
int hip_fail(dgn_ctx* c, hipError_t e, const char* where) {
    return fail(c, DGN_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}
// every wait of the host for the context's stream goes through here (dgn_debug_host_syncs)
hipError_t stream_sync(dgn_ctx* c) {
    ++c->host_syncs;
    return hipStreamSynchronize(c->stream);
}
#define HIP_TRY(ctx, expr)                                      \
    do {                                                        \
        hipError_t e_ = (expr);                                 \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr);  \
    } while (0)

hipEvent_t get_event(dgn_ctx* c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

struct TimedLaunch {
    dgn_ctx* c;
    const char* name;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(dgn_ctx* c_, const char* n, double bytes, double flops) : c(c_), name(n) {
        if (!c->timing) return;
        auto it = c->stats.find(name);
        if (it == c->stats.end()) {
            c->order.push_back(name);
            it = c->stats.emplace(name, KernelStat{}).first;
        }
        it->second.bytes += bytes;
        it->second.flops += flops;
        it->second.launches += 1;
        a = get_event(c);
        b = get_event(c);
        (void)hipEventRecord(a, c->stream);
    }
    ~TimedLaunch() {
        if (!c->timing || !a) return;
        (void)hipEventRecord(b, c->stream);
        c->pending.push_back({name, a, b});
    }
};

void fold_events(dgn_ctx* c) {
    for (auto& p : c->pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.stop) == hipSuccess && hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess)
            c->stats[p.name].total_ms += ms;
        c->free_events.push_back(p.start);
        c->free_events.push_back(p.stop);
    }
    c->pending.clear();
}

bool batch_ok(const dgn_batch* b) {
    return b && b->num_structures >= 0 && b->num_atoms >= 0 && b->lattice && b->positions && b->atom_offset &&
           (b->num_atoms == 0 || b->num_structures > 0);
}

RbfSpec make_rbf(const dgn_graph_params* p) {
    RbfSpec r{};
    r.dtype = p->rbf_dtype;
    r.nbins = dgn_rbf_bins(p->rbf_cutoff, p->rbf_dr);
    r.dr = p->rbf_dr;
    // edge_features.cpp:13-16
    const double sigma = p->rbf_cutoff / 3;
    r.inv_sigma2 = 1 / std::pow(sigma, 2);
    r.norm = 1 / (sigma * std::sqrt(2 * M_PI));
    r.c2 = -0.5 * r.inv_sigma2 * 1.4426950408889634074;  // exponent scale of the f32 path (log2 e)
    r.inv_nbins = r.nbins > 0 ? 1.0f / (float)r.nbins : 0.0f;
    r.norm_f = (float)r.norm;
    return r;
}

// A graph emit reports its consistency flag asynchronously (host->emit_flag); the next call
// that synchronizes the stream surfaces it.
int take_emit_flag(dgn_ctx* c) {
    if (!c->emit_pending) return DGN_OK;
    c->emit_pending = false;
    const uint32_t f = c->host->emit_flag;
    if (!f) return DGN_OK;
    std::string why;
    if (f & kGErrCap) why += " [more candidates than the count pass reported]";
    if (f & kGErrMismatch) why += " [kept rows differ from the count pass]";
    if (f & kGErrMissedHit) why += " [a count-pass hit failed the exact test]";
    return fail(c, DGN_ERR_INTERNAL, "graph emit disagreed with the count pass (flags " + std::to_string(f) + ")" + why);
}

// A Betti pass reports its flags asynchronously (host->betti_flags, copied at the end of the pass on
// its stream); the next call that synchronizes the stream surfaces them, and clears the sticky
// device words it reported.
int take_betti_flag(dgn_ctx* c) {
    if (!c->betti_pending) return DGN_OK;
    c->betti_pending = false;
    const uint32_t g = c->host->betti_flags[kBFSearch], f = c->host->betti_flags[kBFReduce];
    if (!g && !f) return DGN_OK;
    HIP_TRY(c, hipMemsetAsync(c->bflags.p, 0, 2 * sizeof(uint32_t), c->stream));
    if (g)
        return fail(c, DGN_ERR_INTERNAL, "Betti neighbour search disagreed with the count pass (flags " + std::to_string(g) + ")");
    if (f & 1u) return fail(c, DGN_ERR_UNSUPPORTED, "local complex exceeds the kernel's point envelope");
    if (f & 64u) return fail(c, DGN_ERR_INTERNAL, "reduction order check failed");
    return fail(c, DGN_ERR_CAPACITY, "per-complex workspace overflow, flags " + std::to_string(f));
}

// every deferred device-side report of this context (after a stream synchronization)
int take_flags(dgn_ctx* c) {
    if (int st = take_emit_flag(c)) {
        (void)take_betti_flag(c);
        return st;
    }
    return take_betti_flag(c);
}

int device_cus(dgn_ctx* c) {
    if (c->cus <= 0) {
        hipDeviceProp_t p;
        c->cus = hipGetDeviceProperties(&p, c->device) == hipSuccess ? p.multiProcessorCount : 256;
    }
    return c->cus;
}

GraphLaunch graph_launch(GraphWork& W, const dgn_batch* b, double rc, double eps, uint64_t kmax, bool use_mask) {
    return GraphLaunch{W.meta.as<StructMeta>(),  W.atom_struct.as<int32_t>(),
                       b->atom_offset,           b->positions,
                       W.cell_start.as<int32_t>(), W.cell_pos.as<double4>(),
                       use_mask ? W.mask.as<uint64_t>() : nullptr,
                       b->num_structures,        b->num_atoms,
                       rc * rc,                  eps,
                       kmax,                     W.qa};
}

// neighbour counting pass shared by the graph and Betti entry points: prep (geometry, atom map,
// cell lists, Betti weights) + per-atom counts and exact hit masks + block scan; one stream
// synchronization. `betti` = the neighbour pass internal to dgn_*_betti (its own workspace, timed
// under its own names so the graph kernels' roofline is never mixed with it; also computes the
// per-atom 1/count(species) weight)
int graph_count_impl(dgn_ctx* c, const dgn_batch* b, double rc, uint64_t kmax, double eps, int64_t* num_edges,
                     bool betti = false) {
    GraphWork& W = betti ? c->bw : c->gw;
    const int64_t A = b->num_atoms, B = b->num_structures;
    W.qa = graph_tile_atoms(A, device_cus(c));
    const int64_t nblocks = graph_blocks(A, W.qa);
    const size_t A1 = (size_t)std::max<int64_t>(A, 1);
    HIP_TRY(c, W.meta.ensure(sizeof(StructMeta) * (size_t)std::max<int64_t>(B, 1)));
    HIP_TRY(c, W.counts.ensure(sizeof(int32_t) * A1));
    HIP_TRY(c, W.block_sums.ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(nblocks, 1)));
    HIP_TRY(c, W.block_aux.ensure(kAux * sizeof(uint64_t) * (size_t)std::max<int64_t>(nblocks, 1)));
    HIP_TRY(c, W.defer.ensure((size_t)std::max<int64_t>(nblocks, 1)));  // a flag byte per count tile
    HIP_TRY(c, W.atom_struct.ensure(sizeof(int32_t) * A1));
    HIP_TRY(c, W.cell_start.ensure(sizeof(int32_t) * (size_t)(A + B + 1)));
    HIP_TRY(c, W.cell_pos.ensure(sizeof(double4) * A1));
    // hit masks: kMaskWords per atom, whole tiles (word-major per tile, graph_kernels.hip mask_index)
    HIP_TRY(c, W.mask.ensure(sizeof(uint64_t) * kMaskWords * (size_t)std::max<int64_t>(nblocks * W.qa, 1)));
    // the Betti weights ride along with any pass that has species, so a Betti pass at the same
    // cutoff can reuse this one (betti_impl)
    const bool want_weight = b->species != nullptr;
    (void)betti;
    if (want_weight) HIP_TRY(c, W.weight.ensure(sizeof(double) * A1));
    HIP_TRY(c, c->scalars.ensure(sizeof(Scalars)));
    Scalars* sc = c->scalars.as<Scalars>();
    HIP_TRY(c, hipMemsetAsync(sc, 0, sizeof(Scalars), c->stream));
    W.have = false;
    {
        TimedLaunch t(c, betti ? "betti_nl_prep" : "prep_structures", (double)B * (72 + 16 + sizeof(StructMeta)) + 4.0 * A, 0);
        HIP_TRY(c, launch_prep_structures(c->stream, b->lattice, b->atom_offset, b->positions,
                                          want_weight ? b->species : nullptr, B, rc, W.meta.as<StructMeta>(),
                                          W.atom_struct.as<int32_t>(), W.cell_start.as<int32_t>(),
                                          W.cell_pos.as<double4>(), want_weight ? W.weight.as<double>() : nullptr,
                                          &sc->graph_flag));
    }
    const GraphLaunch g = graph_launch(W, b, rc, eps, kmax, false);
    {
        // compulsory traffic: positions in, per-atom counts out (+ the structure metadata)
        TimedLaunch t(c, betti ? "betti_nl_count" : "graph_count", (double)A * (24 + 4) + (double)B * sizeof(StructMeta), 0);
        HIP_TRY(c, launch_graph_count(c->stream, g, W.counts.as<int32_t>(), W.block_sums.as<int64_t>(),
                                      W.block_aux.as<uint64_t>(), W.mask.as<uint64_t>(), W.defer.as<uint8_t>()));
    }
    {
        TimedLaunch t(c, betti ? "betti_nl_scan" : "block_scan", (double)nblocks * 32, 0);
        HIP_TRY(c, launch_block_scan(c->stream, W.block_sums.as<int64_t>(), W.block_aux.as<uint64_t>(), nblocks,
                                     &sc->total, &sc->max_candidates, &sc->sum_sq, &sc->max_natoms, &sc->sum_m, &sc->wide_atoms));
    }
    HIP_TRY(c, hipMemcpyAsync(&c->host->s, sc, sizeof(Scalars), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_sync(c));
    int st = take_flags(c);
    if (st) return st;
    if (c->host->s.graph_flag & kGErrFar)
        return fail(c, DGN_ERR_UNSUPPORTED, "an atom lies more than 500 lattice periods from the origin");
    W.have = true;
    W.pos = b->positions;
    W.atoms = A;
    W.structs = B;
    W.rc = rc;
    W.eps = eps;
    W.k = kmax;
    W.max_candidates = c->host->s.max_candidates;
    W.max_natoms = c->host->s.max_natoms;
    W.edges = c->host->s.total;
    W.sum_sq = (double)c->host->s.sum_sq;
    W.sum_m = (double)c->host->s.sum_m;
    W.wide_atoms = (int64_t)(c->host->s.wide_atoms & 0xFFFFFFFFull);
    W.huge_atoms = (int64_t)(c->host->s.wide_atoms >> 32);
    W.has_weight = want_weight;
    W.species = b->species;
    if (num_edges) *num_edges = W.edges;
    return DGN_OK;
}

int graph_emit_impl(dgn_ctx* c, const dgn_batch* b, const int64_t* row_ptr, int32_t* col, double* dist,
                    double* disp, void* rbf, const RbfSpec& rs) {
    GraphWork& W = c->gw;
    if (!W.have || W.pos != b->positions || W.atoms != b->num_atoms)
        return fail(c, DGN_ERR_ARG, "dgn_dev_graph_emit: no matching dgn_dev_graph_count on this context");
    const int cap = graph_emit_cap(W.max_candidates, W.k);
    if (b->num_atoms == 0) return DGN_OK;
    double* key_rows = nullptr;
    if (cap == kEmitGlobalKeys) {
        // rows of more candidates than the LDS holds (neighbor_list.cpp:27-66 has no cap): per-wave
        // key rows in HBM for one chunk of tiles (<= kEmitGkChunkBytes), kept for reuse
        HIP_TRY(c, c->emit_keys.ensure((size_t)emit_key_rows_per_chunk(W.max_candidates) *
                                       (size_t)emit_key_row_doubles(W.max_candidates) *
                                       sizeof(double)));
        key_rows = c->emit_keys.as<double>();
    }
    Scalars* sc = c->scalars.as<Scalars>();
    HIP_TRY(c, hipMemsetAsync(&sc->graph_flag, 0, sizeof(uint32_t), c->stream));
    const GraphLaunch g = graph_launch(W, b, W.rc, W.eps, W.k, true);
    const double E = (double)W.edges, A = (double)W.atoms, B = (double)W.structs;
    const double rbf_bytes = rs.dtype == DGN_F32 ? 4.0 : (rs.dtype == DGN_F64 ? 8.0 : 0.0);
    // compulsory traffic: positions + lattice + counts in; CSR + edge features out
    const double bytes = 24 * A + 72 * B + 4 * A + 8 * (A + 1) + E * (4 + (dist ? 8 : 0)) + (disp ? 24 * E : 0) +
                         (rbf ? E * rs.nbins * rbf_bytes : 0);
    const int stage = (int)std::min<uint32_t>(W.max_natoms, (uint32_t)kStage);
    // the block RBF stream re-reads the block's distance rows
    double* dist_rows = dist;
    if (!dist && rbf && rs.dtype != DGN_NONE) {
        HIP_TRY(c, c->dist_scratch.ensure((size_t)std::max<int64_t>(W.edges, 1) * sizeof(double)));
        dist_rows = c->dist_scratch.as<double>();
    }
    {
        TimedLaunch t(c, "graph_emit", bytes, 0);
        HIP_TRY(c, launch_graph_emit(c->stream, g, cap, stage, W.counts.as<int32_t>(), W.block_sums.as<int64_t>(),
                                     const_cast<int64_t*>(row_ptr), col, dist_rows, disp, rbf, rs, &sc->graph_flag,
                                     key_rows, W.max_candidates, c->dbg_emit_chunk));
    }
    HIP_TRY(c, hipMemcpyAsync(&c->host->emit_flag, &sc->graph_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    c->emit_pending = true;
    return DGN_OK;
}

int check_emit_flag(dgn_ctx* c) {
    HIP_TRY(c, stream_sync(c));
    return take_flags(c);
}

int betti_impl(dgn_ctx* c, const dgn_batch* b, double rc, double* features, int32_t* counts, const double* clouds,
               const int32_t* npoints, int32_t cloud_stride, int64_t num_clouds, float* pairs_out, int32_t pair_cap,
               const float* lower = nullptr, bool reuse_graph = false, bool async_report = false) {
    const bool given = clouds || lower;
    const int64_t A = given ? num_clouds : b->num_atoms;
    auto nw = [&]() -> GraphWork& { return reuse_graph ? c->gw : c->bw; };
    if (A == 0) return DGN_OK;
    int max_points = cloud_stride;
    if (!given) {
        // NeighborList(rc, SIZE_MAX) counts (betti_features.cpp:107): the largest local complex,
        // sum n^2 for the byte accounting, the per-atom weights
        // dgn_dev_graph_betti: the graph pass's count at the same cutoff already holds every
        // neighbour within rc (NeighborList(rc, K) and NeighborList(rc, SIZE_MAX) see the same
        // candidates, neighbor_list.cpp:27-66); its per-atom counts, hit masks, cell lists and
        // weights serve the Betti search unchanged
        if (!reuse_graph) {
            int64_t E = 0;
            int st = graph_count_impl(c, b, rc, UINT64_MAX, 1e-10, &E, true);
            if (st) return st;
        }
        max_points = (int)nw().max_candidates + 1;
    }
    // caller-given triangles (one connected component at a time, dgn_host_persistence's split) reach
    // the GIANT instantiation; clouds and atom-centred complexes stop at the distance kernels' 2,048
    const int envelope = lower ? kWideGiantPoints : betti_max_points();
    if (max_points > envelope)
        return fail(c, DGN_ERR_UNSUPPORTED,
                    "local complex with " + std::to_string(max_points) + " points exceeds the " +
                        std::to_string(envelope) + "-point kernel envelope (see DESIGN.md)");
    // scratch slots: the main grid's plus kOverflowWaves for the forked overflow tier
    constexpr int kOverflowWaves = 512;
    if (c->betti_slots == 0) c->betti_slots = betti_grid_waves(c->device) + kOverflowWaves;
    if (!c->side) {
        HIP_TRY(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    }
    const BettiFork fork{c->side, c->ev_fork, c->ev_join, kOverflowWaves};
    const int64_t spw = betti_scratch_bytes_per_wave();
    if (c->b_scratch.bytes < (size_t)spw * c->betti_slots) {
        HIP_TRY(c, c->b_scratch.ensure((size_t)spw * c->betti_slots));
        c->scratch_fresh = true;
    }
    if (c->scratch_fresh) {
        // every slot's one-byte min-cofacet tables start as "no cofacet" (0xFF): the kernels keep
        // that invariant for every entry they touch, so a stray byte can never read as a clearing mark
        HIP_TRY(c, betti_init_scratch(c->stream, c->b_scratch.as<uint8_t>(), c->betti_slots));
        c->scratch_fresh = false;
    }
    HIP_TRY(c, c->scalars.ensure(sizeof(Scalars)));
    Scalars* sc = c->scalars.as<Scalars>();
    HIP_TRY(c, hipMemsetAsync(&sc->graph_flag, 0, 5 * sizeof(uint32_t), c->stream));
    if (!c->bflags.p) {
        HIP_TRY(c, c->bflags.ensure(kBFWords * sizeof(uint32_t)));
        HIP_TRY(c, hipMemsetAsync(c->bflags.p, 0, kBFWords * sizeof(uint32_t), c->stream));
    }
    uint32_t* bflags = c->bflags.as<uint32_t>();
    HIP_TRY(c, c->b_list.ensure(2 * sizeof(int32_t) * (size_t)A));  // overflow list, dense list
    // complexes above 64 points: the wide kernel, one wave per complex with a per-wave scratch
    // (distance matrix, min-cofacet tables, sorted columns, pivot hash) sized for max_points
    WideLayout wl{};
    int wide_waves = 0;
    // wide complexes of <= kC16MaxPoints points run on u16 rank codes, and their dim-2 apparent walk
    // runs as a workgroup-per-complex pass before the per-wave launch (betti_walk_kernel)
    const bool c16 = c->dbg_wide_c16 && max_points > 64 && max_points <= kC16MaxPoints;
    const bool prewalk = c16 && c->dbg_wide_walk;
    if (max_points > 64) {
        const int wide_nmax = std::min(max_points, kWideRegular);  // larger: the coded retry launch
        wl = betti_wide_layout(wide_nmax, false, c->dbg_wide_cap, 0, 24, prewalk);
        // as many waves as the device keeps resident (dynamic LDS sized by
        // max_points), each with its own scratch, within half of the HBM that is free or already
        // this workspace's (288 GB per MI355X; at least 8 GB) -- counting the workspace in the pool
        // keeps the wave count, hence the layout, the same from one call to the next (a changed
        // layout re-initialises every wave's tables)
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        const int64_t budget =
            std::max<int64_t>(int64_t(8) << 30, ((int64_t)free_b + (int64_t)c->b_wide.bytes) / 2);
        const int64_t resident = betti_wide_resident_waves(c->device, wide_nmax, c16, prewalk);
        wide_waves = (int)std::max<int64_t>(1, std::min<int64_t>({budget / wl.total, resident, A}));
        if (c->dbg_wide_waves > 0 && c->dbg_wide_waves < wide_waves) wide_waves = c->dbg_wide_waves;  // A/B only
        const size_t want = (size_t)wl.total * (size_t)wide_waves;
        const bool grown = c->b_wide.bytes < want;
        if (grown) HIP_TRY(c, c->b_wide.ensure(want));
        wl.base = c->b_wide.as<uint8_t>();
        if (grown || c->wide_nmax != wide_nmax || c->wide_waves != wide_waves || c->wide_cap != wl.na_cap ||
            c->wide_pre != (int)prewalk) {
            // the layout depends on max_points: every wave's pivot hash table starts empty (key 0)
            // and its u16 min-cofacet tables "no cofacet" (0xFFFF); afterwards each reduction
            // restores both for the entries it used
            HIP_TRY(c, betti_wide_init_scratch(c->stream, wl, wide_waves));
            c->wide_nmax = wide_nmax;
            c->wide_waves = wide_waves;
            c->wide_cap = wl.na_cap;
            c->wide_pre = (int)prewalk;
        }
        HIP_TRY(c, c->b_wlist.ensure(sizeof(int32_t) * (size_t)A));
    }
    BettiLaunch bl{};
    bl.num_atoms = A;
    bl.thr = (float)rc;  // ripser_wrapper.cpp:28
    bl.features = features;
    bl.counts = counts;
    bl.error_flag = bflags + kBFReduce;
    bl.work_counter = &sc->work_counter;
    bl.work_counter2 = &sc->work_counter2;
    bl.overflow_list = c->b_list.as<int32_t>();
    bl.overflow_len = &sc->overflow_len;
    bl.dense_list = c->b_list.as<int32_t>() + A;
    bl.dense_len = &sc->dense_len;
    bl.dense_queue = &sc->dense_queue;
    bl.scratch = c->b_scratch.as<uint8_t>();
    bl.scratch_per_wave = spw;
    bl.clouds = clouds;
    bl.npoints = npoints;
    bl.cloud_stride = cloud_stride;
    bl.pairs_out = pairs_out;
    bl.pair_cap = pair_cap;
    bl.wide_list = max_points > 64 ? c->b_wlist.as<int32_t>() : nullptr;
    bl.wide_len = &sc->wide_len;
    bl.wide_queue = &sc->wide_queue;
    HIP_TRY(c, c->b_rlist.ensure(sizeof(int32_t) * (size_t)A));
    bl.retry_list = c->b_rlist.as<int32_t>();
    bl.retry_len = &sc->retry_len;
    bl.force_retry = c->dbg_force_retry ? 1 : 0;  // tests only (dgn_ctx_set_debug)
    // Betti pass over complexes [c0, c0 + cnt) whose triangles are in `lower`
    auto vr_pass = [&](int64_t c0, int64_t cnt, const float* tri, int64_t tri_stride, const int32_t* np,
                       const double* w, double bytes) -> int {
        BettiLaunch pb = bl;
        pb.lower = tri;
        pb.npoints = np;
        pb.weight = w;
        pb.tri_stride = tri_stride;
        pb.num_atoms = cnt;
        pb.features = features ? features + 35 * c0 : nullptr;
        pb.counts = counts ? counts + 4 * c0 : nullptr;
        pb.pairs_out = pairs_out ? pairs_out + c0 * 3 * (int64_t)pair_cap * 2 : nullptr;
        static_assert(offsetof(Scalars, dense_queue) - offsetof(Scalars, work_counter) == 8 * sizeof(uint32_t),
                      "queue and list counters are contiguous");
        HIP_TRY(c, hipMemsetAsync(&sc->work_counter, 0, 9 * sizeof(uint32_t), c->stream));
        // wide complexes of <= 362 points run on u16 rank codes (half the per-wave distance matrix
        // the scattered walk and pivot-search reads miss on): the narrow launches and the bucket
        // pass first, then per slice of the wide list its codes (betti_rank_codes) and a wide launch
        {
            TimedLaunch t(c, "betti_vr", bytes, 0.0);
            HIP_TRY(c, launch_betti(c->stream, pb, max_points, c->betti_slots,
                                    max_points > 64 && !c16 ? &wl : nullptr, wide_waves, &fork));
            if (c16) {
                // slices of the wide list sized on the host from an upper bound of its length (the
                // count pass's census of 65..kWideRegular-point complexes, which the host already
                // holds), their lengths derived on the device from the bucket pass's wide_len: no
                // host read, no stream synchronization
                const int64_t nwide = given ? cnt : std::min<int64_t>(cnt, nw().wide_atoms);
                if (nwide > 0) {
                    const int64_t rstride = ((int64_t)max_points * (max_points - 1) / 2 + 63) / 64 * 64;
                    int64_t slice = std::max<int64_t>(
                        1, std::min<int64_t>({nwide, (int64_t(16) << 30) / (20 * rstride), INT32_MAX / rstride}));
                    // The walk pass's per-complex outputs (matrix, lists: ~1.7 MB at 340 points), two
                    // slices' worth within half of the HBM that is free or already theirs, <= 32 GB
                    // (a quarter cut the slices below the reductions' 8,192 resident waves in a process
                    // holding ~40 GB elsewhere, the bench's config-4 shard: 7-9 % slower at 10 A).
                    // Slice q's walk pass (LDS- and issue-bound, one workgroup per CU) runs on the context
                    // stream while slice q - 1's reductions (LDS-free, latency-bound) run on a second
                    // stream: double-buffered codes and walk outputs, ordered by events
                    const int64_t walk_bytes = prewalk ? betti_walk_out_bytes(max_points) : 0;
                    const int nbuf = prewalk ? 2 : 1;
                    if (prewalk) {
                        size_t free_b = 0, total_b = 0;
                        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
                        const int64_t wbudget = std::min<int64_t>(
                            int64_t(32) << 30, std::max<int64_t>(int64_t(1) << 30, ((int64_t)free_b + (int64_t)c->b_walk.bytes) / 2));
                        slice = std::max<int64_t>(1, std::min<int64_t>(slice, wbudget / (nbuf * walk_bytes)));
                    }
                    // equal slices: a short last slice leaves its launch's resident waves idle behind
                    // a tail of single complexes
                    slice = (nwide + (nwide + slice - 1) / slice - 1) / ((nwide + slice - 1) / slice);
                    const size_t tmp_bytes = betti_rank_temp_bytes(slice, rstride);
                    const size_t rank_buf = (8 * (size_t)slice * rstride + tmp_bytes + 255) / 256 * 256;
                    const size_t walk_buf = ((size_t)walk_bytes * (size_t)slice + 255) / 256 * 256;
                    if (prewalk) HIP_TRY(c, c->b_walk.ensure(walk_buf * nbuf));
                    HIP_TRY(c, c->b_rank16.ensure(rank_buf * nbuf));
                    const int64_t nsl = (nwide + slice - 1) / slice;
                    HIP_TRY(c, c->b_rscal16.ensure(sizeof(uint32_t) * 2 * (size_t)nsl));
                    uint32_t* sl = c->b_rscal16.as<uint32_t>();
                    HIP_TRY(c, launch_slice_lengths(c->stream, &sc->wide_len, slice, nsl, sl));
                    hipStream_t rs = c->stream;  // the reductions' stream
                    if (prewalk && nsl > 1) {
                        if (!c->rstream) {
                            HIP_TRY(c, hipStreamCreateWithFlags(&c->rstream, hipStreamNonBlocking));
                            for (int k = 0; k < 2; ++k) {
                                HIP_TRY(c, hipEventCreateWithFlags(&c->ev_walk[k], hipEventDisableTiming));
                                HIP_TRY(c, hipEventCreateWithFlags(&c->ev_red[k], hipEventDisableTiming));
                            }
                        }
                        rs = c->rstream;
                    }
                    for (int64_t q = 0; q < nsl; ++q) {
                        const int k = (int)(q % nbuf);
                        uint32_t* codes = reinterpret_cast<uint32_t*>(c->b_rank16.as<uint8_t>() + k * rank_buf);
                        uint32_t* sorted = codes + slice * rstride;
                        BettiLaunch wb = pb;
                        wb.wide_list = c->b_wlist.as<int32_t>() + q * slice;
                        wb.wide_len = sl + 2 * q;
                        wb.wide_queue = sl + 2 * q + 1;
                        const int64_t ub = std::min<int64_t>(slice, nwide - q * slice);
                        // buffer k was last read by slice q - 2's reductions
                        if (rs != c->stream && q >= 2) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_red[k], 0));
                        HIP_TRY(c, betti_rank_codes(c->stream, pb.lower, pb.tri_stride, pb.npoints, wb.wide_list, ub,
                                                    rstride, codes, sorted, sorted + slice * rstride, tmp_bytes,
                                                    wb.wide_len));
                        wb.rank_codes = codes;
                        wb.rank_sorted = sorted;
                        wb.rank_stride = rstride;
                        if (prewalk) {
                            WalkOut wo = betti_walk_out_layout(max_points);
                            uint8_t* p = c->b_walk.as<uint8_t>() + k * walk_buf;
                            auto carve = [&](int64_t bytes_per_complex) {
                                uint8_t* r = p;
                                p += (size_t)bytes_per_complex * (size_t)slice;
                                return r;
                            };
                            wo.dmat = reinterpret_cast<uint16_t*>(carve(2 * wo.dstride));
                            wo.meta = reinterpret_cast<uint32_t*>(carve(32));
                            wo.d0 = reinterpret_cast<float*>(carve(4 * wo.d0stride));
                            wo.mce = reinterpret_cast<uint16_t*>(carve(2 * wo.mstride));
                            wo.e1 = reinterpret_cast<uint64_t*>(carve(8 * (int64_t)wo.cap1));
                            wo.cl = reinterpret_cast<uint32_t*>(carve(4 * (int64_t)wo.cap1));
                            wo.ent = reinterpret_cast<uint64_t*>(carve(8 * (int64_t)wo.cap));
                            wb.walk = wo;
                            HIP_TRY(c, launch_betti_walk(c->stream, wb, ub, max_points));
                        }
                        if (rs != c->stream) {
                            HIP_TRY(c, hipEventRecord(c->ev_walk[k], c->stream));
                            HIP_TRY(c, hipStreamWaitEvent(rs, c->ev_walk[k], 0));
                        }
                        HIP_TRY(c, launch_betti_wide(rs, wb, wl, (int)std::min<int64_t>(wide_waves, ub)));
                        if (rs != c->stream) HIP_TRY(c, hipEventRecord(c->ev_red[k], rs));
                    }
                    if (rs != c->stream) {  // join: the retry launch and the outputs follow on the context stream
                        HIP_TRY(c, hipEventRecord(c->ev_red[0], rs));
                        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_red[0], 0));
                    }
                }
            }
        }
        if (pb.force_retry) {
            // test knob (no kernel checks it: a per-complex flag read cost 0.8 % of the narrow
            // launch): every complex of the pass is listed for the retry launch, which overwrites
            // its outputs
            std::vector<int32_t> all((size_t)cnt);
            for (int64_t i = 0; i < cnt; ++i) all[(size_t)i] = (int32_t)i;
            const uint32_t n32 = (uint32_t)cnt;
            HIP_TRY(c, hipMemcpyAsync(c->b_rlist.p, all.data(), sizeof(int32_t) * (size_t)cnt, hipMemcpyHostToDevice,
                                      c->stream));
            HIP_TRY(c, hipMemcpyAsync(&sc->retry_len, &n32, sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, stream_sync(c));
        }
        // complexes whose reduction outgrew a kernel's workspace (the reference's Ripser has no
        // caps, ripser.cpp:514-1269): reduced again with the big wide layout
        const int nmax = std::max(max_points, 64);
        const bool coded = nmax > kWideRegular;
        HIP_TRY(c, c->b_rlist2.ensure(sizeof(int32_t) * (size_t)A));
        int32_t* cur = c->b_rlist.as<int32_t>();
        int32_t* nxt = c->b_rlist2.as<int32_t>();
        int64_t nretry = -1;
        int grow0 = 0;
        if (!coded && c->dbg_big_log2 == 0) {
            // Device-driven retry (complexes of up to kWideRegular points: the 5 A and 10 A paths):
            // the launch reads the retry list's length on the device and its waves leave at once when
            // nothing overflowed, so the pass never waits for the host. Its workspace (first growth
            // level, >= 8 waves) is kept for the context's lifetime, its tables restored by every
            // reduction; it takes at most an eighth of the HBM that is free or already its own, and
            // 32 GB (288 GB per MI355X).
            WideLayout big = betti_wide_layout(nmax, true);
            if (c->big_budget == 0) {
                size_t free_b = 0, total_b = 0;
                if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
                c->big_budget = std::min<int64_t>(int64_t(32) << 30, ((int64_t)free_b + (int64_t)c->b_big.bytes) / 8);
            }
            const int64_t waves =
                std::min<int64_t>({c->big_budget / big.total, betti_wide_resident_waves(c->device, nmax), 32});
            if (waves >= 8) {
                if (c->big_nmax != nmax || c->big_waves < waves) {
                    HIP_TRY(c, c->b_big.ensure((size_t)big.total * (size_t)waves));
                    big.base = c->b_big.as<uint8_t>();
                    HIP_TRY(c, betti_wide_init_scratch(c->stream, big, (int)waves));
                    c->big_nmax = nmax;
                    c->big_waves = (int)waves;
                }
                big.base = c->b_big.as<uint8_t>();
                BettiLaunch rb = pb;
                rb.rank_codes = nullptr;
                rb.rank_sorted = nullptr;
                // a complex that outgrows this level: the device entry points report DGN_ERR_CAPACITY
                // at their next synchronizing call (no host read here); the host entry points list it
                // for the growing levels below
                rb.retry_list = async_report ? nullptr : nxt;
                rb.retry_len = async_report ? nullptr : &sc->retry2_len;
                rb.force_retry = 0;
                rb.retried = bflags + kBFRetried;
                rb.wide_list = c->b_rlist.as<int32_t>();
                rb.wide_len = &sc->retry_len;
                rb.wide_queue = &sc->retry_queue;
                if (!async_report) HIP_TRY(c, hipMemsetAsync(&sc->retry2_len, 0, sizeof(uint32_t), c->stream));
                {
                    TimedLaunch t(c, "betti_retry", 0.0, 0.0);
                    HIP_TRY(c, launch_betti_wide(c->stream, rb, big, (int)waves));
                }
                HIP_TRY(c, hipMemsetAsync(&sc->retry_len, 0, 2 * sizeof(uint32_t), c->stream));
                if (async_report) return DGN_OK;
                HIP_TRY(c, hipMemcpyAsync(&c->host->s.retry2_len, &sc->retry2_len, sizeof(uint32_t),
                                          hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, stream_sync(c));
                nretry = c->host->s.retry2_len;
                if (nretry == 0) return DGN_OK;
                std::swap(cur, nxt);
                grow0 = 1;
            }
        }
        if (nretry < 0) {
            // larger complexes: the retry workspace is sized by the number of complexes that
            // overflowed (one host read of the list length)
            HIP_TRY(c, hipMemcpyAsync(&c->host->s.retry_len, &sc->retry_len, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                      c->stream));
            HIP_TRY(c, stream_sync(c));
            nretry = c->host->s.retry_len;
            if (nretry == 0) return DGN_OK;
        }
        // complexes above kWideRegular points (listed by the bucket pass) run on rank codes
        // (betti_rank_codes, the BIG / HUGE instantiations), in slices of at most 512 complexes.
        // The tables grow with the complexes (the reference's Ripser has no caps): a complex that
        // outgrows level `grow` is listed again and reduced at the next level, 4x the tables
        c->big_nmax = 0;  // the workspace below is laid out per call
        const int64_t rstride = ((int64_t)nmax * (nmax - 1) / 2 + 63) / 64 * 64;
        for (int grow = grow0;; ++grow) {
            const bool last = grow == kWideMaxGrow;
            WideLayout big = betti_wide_layout(nmax, true, 0, grow, c->dbg_big_log2 ? c->dbg_big_log2 : 24);
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
            // (GIANT: 8.4 M distances per 4,096-point complex; a slice keeps its codes below 16 GB and
            // its segmented-sort offsets in int32)
            const int64_t slice = coded ? std::max<int64_t>(1, std::min<int64_t>({nretry, 512, INT32_MAX / rstride,
                                                                                   (int64_t(16) << 30) / (8 * rstride)}))
                                        : nretry;
            const int64_t nsl = (nretry + slice - 1) / slice;
            const size_t rank_bytes = coded ? betti_rank_temp_bytes(slice, rstride) + 8 * (size_t)slice * rstride : 0;
            const int64_t budget =
                (int64_t)(free_b / 2) + (int64_t)c->b_big.bytes + (int64_t)c->b_rank.bytes - (int64_t)rank_bytes;
            const int64_t waves =
                std::min<int64_t>({slice, budget / big.total, betti_wide_resident_waves(c->device, nmax)});
            if (waves < 1)
                return fail(c, DGN_ERR_CAPACITY, "capacity retry: no device memory for a " +
                                                     std::to_string(big.total) + "-byte workspace");
            HIP_TRY(c, c->b_big.ensure((size_t)big.total * (size_t)waves));
            big.base = c->b_big.as<uint8_t>();
            HIP_TRY(c, betti_wide_init_scratch(c->stream, big, (int)waves));
            if (coded) HIP_TRY(c, c->b_rank.ensure(rank_bytes));
            // per slice (length, queue), then the next level's list length
            HIP_TRY(c, c->b_rscal.ensure(sizeof(uint32_t) * (2 * (size_t)nsl + 2)));
            uint32_t* sl0 = c->b_rscal.as<uint32_t>();
            uint32_t* next_len = sl0 + 2 * nsl;
            std::vector<uint32_t> lens((size_t)nsl);
            for (int64_t q = 0; q < nsl; ++q) lens[q] = (uint32_t)std::min<int64_t>(slice, nretry - q * slice);
            HIP_TRY(c, hipMemsetAsync(sl0, 0, sizeof(uint32_t) * (2 * (size_t)nsl + 2), c->stream));
            for (int64_t q = 0; q < nsl; ++q)
                HIP_TRY(c, hipMemcpyAsync(sl0 + 2 * q, &lens[q], sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
            BettiLaunch rb = pb;
            rb.rank_codes = nullptr;  // set per slice below when coded
            rb.rank_sorted = nullptr;
            rb.retry_list = last ? nullptr : nxt;  // last level: a further overflow is DGN_ERR_CAPACITY
            rb.retry_len = last ? nullptr : next_len;
            rb.force_retry = 0;
            rb.retried = bflags + kBFRetried;
            for (int64_t q = 0; q < nsl; ++q) {
                rb.wide_list = cur + q * slice;
                if (coded) {
                    uint32_t* codes = c->b_rank.as<uint32_t>();
                    uint32_t* sorted = codes + slice * rstride;
                    void* tmp = sorted + slice * rstride;
                    HIP_TRY(c, betti_rank_codes(c->stream, pb.lower, pb.tri_stride, pb.npoints, rb.wide_list,
                                                (int64_t)lens[q], rstride, codes, sorted, tmp,
                                                rank_bytes - 8 * (size_t)slice * rstride));
                    rb.rank_codes = codes;
                    rb.rank_sorted = sorted;
                    rb.rank_stride = rstride;
                }
                rb.wide_len = sl0 + 2 * q;
                rb.wide_queue = sl0 + 2 * q + 1;
                TimedLaunch t(c, "betti_retry", 0.0, 0.0);
                HIP_TRY(c, launch_betti_wide(c->stream, rb, big, (int)std::min<int64_t>(waves, lens[q])));
            }
            HIP_TRY(c, hipMemcpyAsync(&c->host->s.retry_len, next_len, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                      c->stream));
            HIP_TRY(c, stream_sync(c));  // `lens` leaves scope; the next level's count
            nretry = last ? 0 : c->host->s.retry_len;
            if (nretry == 0) break;
            std::swap(cur, nxt);
        }
        // the regular wide layout's tables are not touched; the big buffer is kept for reuse
        HIP_TRY(c, hipMemsetAsync(&sc->retry_len, 0, 2 * sizeof(uint32_t), c->stream));
        HIP_TRY(c, stream_sync(c));
        return DGN_OK;
    };
    // triangles: floats per complex, padded to a multiple of 4 (16-byte aligned complexes)
    const int64_t tri_stride = std::max<int64_t>(4, ((int64_t)max_points * (max_points - 1) / 2 + 3) / 4 * 4);
    if (lower) {
        // caller-given triangles: the Betti pass alone
        int st = vr_pass(0, A, lower, (int64_t)cloud_stride * (cloud_stride - 1) / 2, npoints, nullptr, 0.0);
        if (st) return st;
    } else {
        // distance pass (f64 VALU pairs; matrix cores above 64 points) + Betti pass per chunk of complexes; the triangle buffer is
        // bounded (~16 GB of the 288 GB HBM) so arbitrarily large shards stream through it
        const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(A, (int64_t(16) << 30) / (4 * tri_stride)));
        HIP_TRY(c, c->b_lower.ensure(sizeof(float) * (size_t)(chunk * tri_stride)));
        HIP_TRY(c, c->b_np.ensure(sizeof(int32_t) * (size_t)chunk));
        HIP_TRY(c, c->b_w.ensure(sizeof(double) * (size_t)chunk));
        // per-complex averages over the batch: points n (sum n = E + A), sum n^2 from the count pass
        const double En = given ? 0.0 : nw().sum_m, An = (double)A;
        const double sum_n2 = given ? 0.0 : nw().sum_sq;
        const GraphLaunch g = given ? GraphLaunch{} : graph_launch(nw(), b, rc, 1e-10, UINT64_MAX, true);
        for (int64_t c0 = 0; c0 < A; c0 += chunk) {
            const int64_t cnt = std::min<int64_t>(chunk, A - c0);
            const double f = (double)cnt / An;
            {
                // algorithmic bytes: the structures' positions in, triangles (4 C(n,2)) + point count
                // out; useful flops 6 n^2 per complex
                const double bytes = given ? 0.0 : f * (24 * An + 2 * (sum_n2 - (En + An)) + 4 * An);
                TimedLaunch t(c, "betti_dist", bytes, given ? 0.0 : f * 6.0 * sum_n2);
                if (given) {
                    BettiLaunch db = bl;
                    db.tri_stride = tri_stride;
                    DistLaunch dl{c0, cnt, c->b_lower.as<float>(), c->b_np.as<int32_t>(), c->b_w.as<double>()};
                    HIP_TRY(c, launch_betti_dist(c->stream, db, dl));
                } else {
                    HIP_TRY(c, launch_betti_dist_search(c->stream, g, c0, cnt, max_points, tri_stride,
                                                        nw().counts.as<int32_t>(), c->b_lower.as<float>(),
                                                        c->b_np.as<int32_t>(), bflags + kBFSearch));
                }
            }
            // Betti pass: triangles in, 35 f64 + 4 i32 out
            const double bytes = given ? 0.0 : f * (2 * (sum_n2 - (En + An)) + 12 * An + An * (35 * 8 + 16));
            const double* w = given ? c->b_w.as<double>() : (b->species ? nw().weight.as<double>() + c0 : nullptr);
            int st = vr_pass(c0, cnt, c->b_lower.as<float>(), tri_stride, c->b_np.as<int32_t>(), w, bytes);
            if (st) return st;
        }
    }
    // the pass's flags travel to the host behind its work; the device entry points return here
    // (asynchronous: the next synchronizing call reports them), the host ones wait and report
    HIP_TRY(c, hipMemcpyAsync(c->host->betti_flags, bflags, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    c->betti_pending = true;
    if (async_report) return DGN_OK;
    HIP_TRY(c, stream_sync(c));
    return take_flags(c);
}

// stage a host batch into context-owned device buffers
int stage_batch(dgn_ctx* c, const dgn_batch* h, dgn_batch* d) {
    if (!batch_ok(h)) return fail(c, DGN_ERR_ARG, "invalid batch");
    const int64_t A = h->num_atoms, B = h->num_structures;
    HIP_TRY(c, c->h_lat.ensure(sizeof(double) * 9 * (size_t)std::max<int64_t>(B, 1)));
    HIP_TRY(c, c->h_pos.ensure(sizeof(double) * 3 * (size_t)std::max<int64_t>(A, 1)));
    HIP_TRY(c, c->h_spec.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(A, 1)));
    HIP_TRY(c, c->h_off.ensure(sizeof(int64_t) * (size_t)(B + 1)));
    HIP_TRY(c, hipMemcpyAsync(c->h_lat.p, h->lattice, sizeof(double) * 9 * B, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->h_pos.p, h->positions, sizeof(double) * 3 * A, hipMemcpyHostToDevice, c->stream));
    if (h->species)
        HIP_TRY(c, hipMemcpyAsync(c->h_spec.p, h->species, sizeof(int32_t) * A, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->h_off.p, h->atom_offset, sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, c->stream));
    *d = *h;
    d->lattice = c->h_lat.as<double>();
    d->positions = c->h_pos.as<double>();
    d->species = h->species ? c->h_spec.as<int32_t>() : nullptr;
    d->atom_offset = c->h_off.as<int64_t>();
    return DGN_OK;
}

// splitmix64 (see defect-gnn-cpp_amd/python/dgn/synth.py for the contract)
inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

// ======================================= C ABI ============================================
extern "C" {

const char* dgn_status_string(int s) {
    switch (s) {
        case DGN_OK: return "ok";
        case DGN_ERR_ARG: return "invalid argument";
        case DGN_ERR_HIP: return "HIP runtime error";
        case DGN_ERR_CAPACITY: return "capacity exceeded";
        case DGN_ERR_NODEVICE: return "no GPU device (there is no CPU fallback)";
        case DGN_ERR_UNSUPPORTED: return "outside the implemented envelope";
        case DGN_ERR_INTERNAL: return "internal consistency check failed";
        default: return "unknown status";
    }
}

int dgn_ctx_create(int device, dgn_ctx** out) {
    if (!out) return DGN_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return DGN_ERR_NODEVICE;
    if (device < 0 || device >= n) return DGN_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return DGN_ERR_HIP;
    dgn_ctx* c = new dgn_ctx();
    c->device = device;
    // a blocking stream: ordered after (and before) the legacy null stream, which is where a
    // caller's default-stream work (torch's default stream reports handle 0) runs
    if (hipStreamCreateWithFlags(&c->own, hipStreamDefault) != hipSuccess) {
        delete c;
        return DGN_ERR_HIP;
    }
    c->stream = c->own;
    if (hipHostMalloc((void**)&c->host, sizeof(HostScalars), hipHostMallocDefault) != hipSuccess) {
        (void)hipStreamDestroy(c->own);
        delete c;
        return DGN_ERR_HIP;
    }
    std::memset(c->host, 0, sizeof(HostScalars));
    *out = c;
    return DGN_OK;
}

void dgn_ctx_destroy(dgn_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);
    fold_events(c);
    for (hipEvent_t e : c->free_events) (void)hipEventDestroy(e);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->rstream) (void)hipStreamSynchronize(c->rstream);
    for (int k = 0; k < 2; ++k) {
        if (c->ev_walk[k]) (void)hipEventDestroy(c->ev_walk[k]);
        if (c->ev_red[k]) (void)hipEventDestroy(c->ev_red[k]);
    }
    if (c->rstream) (void)hipStreamDestroy(c->rstream);
    if (c->host) (void)hipHostFree(c->host);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;  // DevBuf destructors free the device workspaces
}

int dgn_ctx_set_stream(dgn_ctx* c, void* s) {
    if (!c) return DGN_ERR_ARG;
    // a graph emit's consistency flag is still being copied on the old stream: let it land before
    // the stream is swapped, so the next synchronizing call reads it (take_emit_flag syncs only
    // the current stream)
    if (c->emit_pending || c->betti_pending) HIP_TRY(c, stream_sync(c));
    // NULL (the legacy null stream, e.g. torch's default stream) -> the context's own blocking
    // stream, which the null stream orders against; anything else is used as given
    c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own;
    return DGN_OK;
}

int dgn_ctx_set_debug(dgn_ctx* c, int knob, int value) {
    if (!c) return DGN_ERR_ARG;
    switch (knob) {
        case DGN_DEBUG_FORCE_RETRY: c->dbg_force_retry = value != 0; return DGN_OK;
        case DGN_DEBUG_WIDE_WAVES: c->dbg_wide_waves = value > 0 ? value : 0; return DGN_OK;
        case DGN_DEBUG_WIDE_C16: c->dbg_wide_c16 = value != 0; return DGN_OK;
        case DGN_DEBUG_WIDE_WALK: c->dbg_wide_walk = value != 0; return DGN_OK;
        case DGN_DEBUG_SPLIT_CHUNK: c->dbg_split_chunk = value > 0 ? value : 0; return DGN_OK;
        case DGN_DEBUG_WIDE_CAP: c->dbg_wide_cap = value > 0 ? value : 0; return DGN_OK;
        case DGN_DEBUG_BIG_LOG2: c->dbg_big_log2 = value > 0 && value < 24 ? value : 0; return DGN_OK;
        case DGN_DEBUG_EMIT_CHUNK: c->dbg_emit_chunk = value > 0 ? value : 0; return DGN_OK;
        default: return fail(c, DGN_ERR_ARG, "dgn_ctx_set_debug: unknown knob " + std::to_string(knob));
    }
}

int dgn_ctx_synchronize(dgn_ctx* c) {
    if (!c) return DGN_ERR_ARG;
    HIP_TRY(c, stream_sync(c));
    return take_flags(c);  // a pending graph-emit or Betti failure surfaces here
}

int dgn_debug_retry_count(dgn_ctx* c, int64_t* out) {
    if (!c || !out) return DGN_ERR_ARG;
    *out = 0;
    if (!c->bflags.p) return DGN_OK;
    uint32_t v = 0;
    HIP_TRY(c, hipMemcpyAsync(&c->host->pad, c->bflags.as<uint32_t>() + kBFRetried, sizeof(uint32_t),
                              hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->bflags.as<uint32_t>() + kBFRetried, 0, sizeof(uint32_t), c->stream));
    HIP_TRY(c, stream_sync(c));
    v = c->host->pad;
    *out = v;
    return take_flags(c);
}

int dgn_debug_host_syncs(dgn_ctx* c, int64_t* out) {
    if (!c || !out) return DGN_ERR_ARG;
    *out = c->host_syncs;
    c->host_syncs = 0;
    return DGN_OK;
}

int dgn_debug_check_wide_layouts(int64_t* first_bad) {
    if (!first_bad) return DGN_ERR_ARG;
    *first_bad = -1;
    auto pow2 = [](int64_t x) { return x > 0 && x <= INT32_MAX && (x & (x - 1)) == 0; };
    for (int nmax = 65; nmax <= kWideGiantPoints; ++nmax)
        for (int big = 0; big <= 1; ++big)
            for (int grow = 0; grow <= (big ? kWideMaxGrow : 0); ++grow) {
                const WideLayout l = betti_wide_layout(nmax, big != 0, 0, grow);
                if (!pow2(l.na_cap) || !pow2(l.p_cap) || !pow2(l.h_cap) || !pow2(l.vs_cap) || !pow2(l.vl_cap) ||
                    l.h_cap != 2 * (int64_t)l.na_cap || l.total <= 0) {
                    *first_bad = (int64_t)nmax * 64 + big * 16 + grow;
                    return DGN_ERR_INTERNAL;
                }
            }
    return DGN_OK;
}

const char* dgn_ctx_last_error(const dgn_ctx* c) { return c ? c->last_error.c_str() : "null context"; }

int dgn_ctx_enable_timing(dgn_ctx* c, int on) {
    if (!c) return DGN_ERR_ARG;
    c->timing = on != 0;
    return DGN_OK;
}

int dgn_ctx_reset_timing(dgn_ctx* c) {
    if (!c) return DGN_ERR_ARG;
    (void)hipStreamSynchronize(c->stream);
    fold_events(c);
    c->stats.clear();
    c->order.clear();
    return DGN_OK;
}

int dgn_ctx_kernel_times(dgn_ctx* c, dgn_kernel_time* out, int cap) {
    if (!c) return -DGN_ERR_ARG;
    (void)hipStreamSynchronize(c->stream);
    fold_events(c);
    int k = 0;
    for (const std::string& name : c->order) {
        if (out && k < cap) {
            const KernelStat& s = c->stats[name];
            std::memset(&out[k], 0, sizeof(dgn_kernel_time));
            std::snprintf(out[k].name, sizeof(out[k].name), "%s", name.c_str());
            out[k].launches = s.launches;
            out[k].total_ms = s.total_ms;
            out[k].bytes = s.bytes;
            out[k].flops = s.flops;
        }
        ++k;
    }
    return k;
}

void dgn_graph_params_default(dgn_graph_params* p) {
    if (!p) return;
    // include/graph/neighbor_list.hpp:19-22 and include/graph/crystal_graph.hpp:14-19
    p->r_cutoff = 10.0;
    p->max_neighbors = 20;
    p->epsilon = 1e-10;
    p->rbf_cutoff = 10.0;
    p->rbf_dr = 0.1;
    p->rbf_dtype = DGN_F32;
    p->write_displacement = 0;
}

int dgn_rbf_bins(double rc, double dr) { return (int)std::floor(rc / dr); }  // edge_features.cpp:13

int dgn_dev_graph_count(dgn_ctx* c, const dgn_batch* b, const dgn_graph_params* p, int64_t* num_edges) {
    if (!c || !p || !batch_ok(b) || !(p->r_cutoff > 0)) return fail(c, DGN_ERR_ARG, "dgn_dev_graph_count: bad args");
    HIP_TRY(c, hipSetDevice(c->device));
    return graph_count_impl(c, b, p->r_cutoff, p->max_neighbors, p->epsilon, num_edges);
}

int dgn_dev_graph_emit(dgn_ctx* c, const dgn_batch* b, const dgn_graph_params* p, int64_t* row_ptr,
                       const dgn_graph_out* o) {
    if (!c || !p || !batch_ok(b) || !o || !row_ptr || !o->col_idx) return fail(c, DGN_ERR_ARG, "dgn_dev_graph_emit: bad args");
    if (p->r_cutoff != c->gw.rc || p->max_neighbors != c->gw.k || p->epsilon != c->gw.eps)
        return fail(c, DGN_ERR_ARG, "dgn_dev_graph_emit: parameters differ from the count pass");
    if (p->rbf_dtype != DGN_NONE && (!(p->rbf_dr > 0) || dgn_rbf_bins(p->rbf_cutoff, p->rbf_dr) <= 0))
        return fail(c, DGN_ERR_ARG, "dgn_dev_graph_emit: bad RBF parameters");
    HIP_TRY(c, hipSetDevice(c->device));
    const RbfSpec rs = make_rbf(p);
    return graph_emit_impl(c, b, row_ptr, o->col_idx, o->distance, p->write_displacement ? o->displacement : nullptr,
                           p->rbf_dtype != DGN_NONE ? o->rbf : nullptr, rs);
}

int dgn_host_graph(dgn_ctx* c, const dgn_batch* h, const dgn_graph_params* p, dgn_graph_result** out) {
    if (!c || !p || !out) return fail(c, DGN_ERR_ARG, "dgn_host_graph: bad args");
    *out = nullptr;
    HIP_TRY(c, hipSetDevice(c->device));
    dgn_batch d;
    int st = stage_batch(c, h, &d);
    if (st) return st;
    int64_t E = 0;
    if ((st = dgn_dev_graph_count(c, &d, p, &E))) return st;
    const int nb = p->rbf_dtype != DGN_NONE ? dgn_rbf_bins(p->rbf_cutoff, p->rbf_dr) : 0;
    const size_t rbf_elem = p->rbf_dtype == DGN_F64 ? 8 : 4;
    const int64_t A = h->num_atoms;
    DevBuf rp, col, dist, disp, rbf;
    auto cleanup = [&]() {
        rp.release();
        col.release();
        dist.release();
        disp.release();
        rbf.release();
    };
    hipError_t e;
    if ((e = rp.ensure(8 * (A + 1))) || (e = col.ensure(4 * std::max<int64_t>(E, 1))) ||
        (e = dist.ensure(8 * std::max<int64_t>(E, 1))) ||
        (p->write_displacement && (e = disp.ensure(24 * std::max<int64_t>(E, 1)))) ||
        (nb && (e = rbf.ensure(rbf_elem * nb * std::max<int64_t>(E, 1))))) {
        cleanup();
        return hip_fail(c, e, "dgn_host_graph: device allocation");
    }
    if (A == 0) HIP_TRY(c, hipMemsetAsync(rp.p, 0, 8, c->stream));
    dgn_graph_out o{col.as<int32_t>(), dist.as<double>(), disp.as<double>(), rbf.p};
    if ((st = dgn_dev_graph_emit(c, &d, p, rp.as<int64_t>(), &o)) || (st = check_emit_flag(c))) {
        cleanup();
        return st;
    }
    dgn_graph_result* r = new dgn_graph_result();
    std::memset(r, 0, sizeof(*r));
    r->num_atoms = A;
    r->num_edges = E;
    r->n_rbf = nb;
    r->rbf_dtype = nb ? p->rbf_dtype : DGN_NONE;
    r->row_ptr = new int64_t[A + 1];
    r->col_idx = new int32_t[std::max<int64_t>(E, 1)];
    r->distance = new double[std::max<int64_t>(E, 1)];
    if (p->write_displacement) r->displacement = new double[3 * std::max<int64_t>(E, 1)];
    if (nb) r->rbf = ::operator new(rbf_elem * nb * std::max<int64_t>(E, 1));
    e = hipMemcpy(r->row_ptr, rp.p, 8 * (A + 1), hipMemcpyDeviceToHost);
    if (!e && E) e = hipMemcpy(r->col_idx, col.p, 4 * E, hipMemcpyDeviceToHost);
    if (!e && E) e = hipMemcpy(r->distance, dist.p, 8 * E, hipMemcpyDeviceToHost);
    if (!e && E && r->displacement) e = hipMemcpy(r->displacement, disp.p, 24 * E, hipMemcpyDeviceToHost);
    if (!e && E && r->rbf) e = hipMemcpy(r->rbf, rbf.p, rbf_elem * nb * E, hipMemcpyDeviceToHost);
    cleanup();
    if (e) {
        dgn_graph_result_free(r);
        return hip_fail(c, e, "dgn_host_graph: copy back");
    }
    *out = r;
    return DGN_OK;
}

void dgn_graph_result_free(dgn_graph_result* r) {
    if (!r) return;
    delete[] r->row_ptr;
    delete[] r->col_idx;
    delete[] r->distance;
    delete[] r->displacement;
    ::operator delete(r->rbf);
    delete r;
}

int dgn_dev_betti(dgn_ctx* c, const dgn_batch* b, const dgn_betti_params* p, double* features, int32_t* counts) {
    if (!c || !p || !batch_ok(b) || !b->species || !features || !(p->r_cutoff > 0))
        return fail(c, DGN_ERR_ARG, "dgn_dev_betti: bad args");
    HIP_TRY(c, hipSetDevice(c->device));
    return betti_impl(c, b, p->r_cutoff, features, counts, nullptr, nullptr, 0, 0, nullptr, 0, nullptr, false, true);
}

int dgn_dev_graph_betti(dgn_ctx* c, const dgn_batch* b, const dgn_graph_params* p, int64_t* row_ptr,
                        const dgn_graph_out* o, const dgn_betti_params* bp, double* features, int32_t* counts) {
    if (!c || !p || !bp || !batch_ok(b) || !b->species || !features || !(bp->r_cutoff > 0))
        return fail(c, DGN_ERR_ARG, "dgn_dev_graph_betti: bad args");
    if (p->r_cutoff != c->gw.rc || p->max_neighbors != c->gw.k || p->epsilon != c->gw.eps || !c->gw.have ||
        c->gw.pos != b->positions || c->gw.atoms != b->num_atoms)
        return fail(c, DGN_ERR_ARG, "dgn_dev_graph_betti: no matching dgn_dev_graph_count on this context");
    int st = dgn_dev_graph_emit(c, b, p, row_ptr, o);
    if (st) return st;
    // one neighbour count for both passes when the cutoffs agree (the bench's config: rc 5 / 5)
    // (the 1/count(species) weights are reused only for the species array the count saw)
    const bool reuse = bp->r_cutoff == p->r_cutoff && p->epsilon == 1e-10 && c->gw.has_weight &&
                       c->gw.species == b->species;
    return betti_impl(c, b, bp->r_cutoff, features, counts, nullptr, nullptr, 0, 0, nullptr, 0, nullptr, reuse, true);
}

int dgn_dev_node_features(dgn_ctx* c, const dgn_batch* b, const double* embed, int32_t num_keys, int32_t D,
                          const double* betti, const double* pca_mean, const double* pca_components, int32_t k,
                          double* out) {
    if (!c || !b || b->num_atoms < 0 || (b->num_atoms > 0 && (!b->species || !out)) || !embed || num_keys <= 0 ||
        D < 0 || k < 0 || k > 35 || (k > 0 && (!betti || !pca_mean || !pca_components)))
        return fail(c, DGN_ERR_ARG, "dgn_dev_node_features: bad args");
    if (b->num_atoms == 0) return DGN_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int st = take_emit_flag(c)) return st;
    HIP_TRY(c, c->scalars.ensure(sizeof(Scalars)));
    Scalars* sc = c->scalars.as<Scalars>();
    HIP_TRY(c, hipMemsetAsync(&sc->error_flag, 0, sizeof(uint32_t), c->stream));
    const double A = (double)b->num_atoms;
    {
        TimedLaunch t(c, "node_features", A * (4 + (k ? 35 * 8 : 0) + 8.0 * (D + k)), A * 2.0 * 35 * k);
        HIP_TRY(c, launch_node_features(c->stream, b->species, b->num_atoms, embed, num_keys, D, k ? betti : nullptr,
                                        pca_mean, pca_components, k, out, &sc->error_flag));
    }
    HIP_TRY(c, hipMemcpyAsync(&c->host->s.error_flag, &sc->error_flag, sizeof(uint32_t), hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, stream_sync(c));
    if (c->host->s.error_flag)
        return fail(c, DGN_ERR_ARG, "dgn_dev_node_features: a species key has no embedding row (atom_embeddings.at)");
    return DGN_OK;
}

int dgn_dev_edge_arrays(dgn_ctx* c, const dgn_batch* b, const int64_t* row_ptr, const int32_t* col_idx,
                        const double* distance, const double* displacement, int32_t* sources, int32_t* targets,
                        float* distances_f32, float* displacements_f32) {
    if (!c || !batch_ok(b) || !row_ptr || (targets && !col_idx) || (distances_f32 && !distance) ||
        (displacements_f32 && !displacement))
        return fail(c, DGN_ERR_ARG, "dgn_dev_edge_arrays: bad args");
    if (b->num_atoms == 0) return DGN_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    const double A = (double)b->num_atoms;
    TimedLaunch t(c, "edge_arrays", 8 * (A + 1), 0.0);  // + per edge: in 4 + 8 + 24 B, out 4 + 4 + 4 + 12 B
    HIP_TRY(c, launch_edge_arrays(c->stream, row_ptr, b->atom_offset, b->num_structures, b->num_atoms, col_idx, distance,
                                  displacement, sources, targets, distances_f32, displacements_f32));
    return DGN_OK;
}

int dgn_host_edge_arrays(dgn_ctx* c, const dgn_batch* h, double r_cutoff, uint64_t max_neighbors, double epsilon,
                         dgn_edge_arrays** out) {
    if (!c || !out) return fail(c, DGN_ERR_ARG, "dgn_host_edge_arrays: bad args");
    *out = nullptr;
    HIP_TRY(c, hipSetDevice(c->device));
    dgn_batch d;
    int st = stage_batch(c, h, &d);
    if (st) return st;
    dgn_graph_params p;
    dgn_graph_params_default(&p);
    p.r_cutoff = r_cutoff;
    p.max_neighbors = max_neighbors;
    p.epsilon = epsilon;
    p.rbf_dtype = DGN_NONE;
    p.write_displacement = 1;
    int64_t E = 0;
    if ((st = dgn_dev_graph_count(c, &d, &p, &E))) return st;
    const int64_t A = h->num_atoms, Em = std::max<int64_t>(E, 1);
    DevBuf rp, col, dist, disp, src, tgt, d32, p32;
    HIP_TRY(c, rp.ensure(8 * (A + 1)));
    HIP_TRY(c, col.ensure(4 * Em));
    HIP_TRY(c, dist.ensure(8 * Em));
    HIP_TRY(c, disp.ensure(24 * Em));
    HIP_TRY(c, src.ensure(4 * Em));
    HIP_TRY(c, tgt.ensure(4 * Em));
    HIP_TRY(c, d32.ensure(4 * Em));
    HIP_TRY(c, p32.ensure(12 * Em));
    if (A == 0) HIP_TRY(c, hipMemsetAsync(rp.p, 0, 8, c->stream));
    dgn_graph_out o{col.as<int32_t>(), dist.as<double>(), disp.as<double>(), nullptr};
    if ((st = dgn_dev_graph_emit(c, &d, &p, rp.as<int64_t>(), &o)) || (st = check_emit_flag(c))) return st;
    if ((st = dgn_dev_edge_arrays(c, &d, rp.as<int64_t>(), col.as<int32_t>(), dist.as<double>(), disp.as<double>(),
                                  src.as<int32_t>(), tgt.as<int32_t>(), d32.as<float>(), p32.as<float>())))
        return st;
    HIP_TRY(c, stream_sync(c));
    dgn_edge_arrays* r = new dgn_edge_arrays();
    r->num_edges = E;
    r->sources = new int32_t[Em];
    r->targets = new int32_t[Em];
    r->distances = new float[Em];
    r->displacements = new float[3 * Em];
    hipError_t e = hipSuccess;
    if (E) {
        if (!e) e = hipMemcpy(r->sources, src.p, 4 * E, hipMemcpyDeviceToHost);
        if (!e) e = hipMemcpy(r->targets, tgt.p, 4 * E, hipMemcpyDeviceToHost);
        if (!e) e = hipMemcpy(r->distances, d32.p, 4 * E, hipMemcpyDeviceToHost);
        if (!e) e = hipMemcpy(r->displacements, p32.p, 12 * E, hipMemcpyDeviceToHost);
    }
    if (e) {
        dgn_edge_arrays_free(r);
        return hip_fail(c, e, "dgn_host_edge_arrays: copy back");
    }
    *out = r;
    return DGN_OK;
}

void dgn_edge_arrays_free(dgn_edge_arrays* a) {
    if (!a) return;
    delete[] a->sources;
    delete[] a->targets;
    delete[] a->distances;
    delete[] a->displacements;
    delete a;
}

int dgn_host_betti(dgn_ctx* c, const dgn_batch* h, const dgn_betti_params* p, double* features, int32_t* counts) {
    if (!c || !p || !features || !h || !h->species) return fail(c, DGN_ERR_ARG, "dgn_host_betti: bad args");
    HIP_TRY(c, hipSetDevice(c->device));
    dgn_batch d;
    int st = stage_batch(c, h, &d);
    if (st) return st;
    const int64_t A = h->num_atoms;
    DevBuf f, k;
    hipError_t e;
    if ((e = f.ensure(8 * 35 * std::max<int64_t>(A, 1))) || (e = k.ensure(16 * std::max<int64_t>(A, 1))))
        return hip_fail(c, e, "dgn_host_betti: allocation");
    // NaN features / -1 counts unless a kernel writes them (a call rejected before any launch
    // returns those rather than uninitialised device memory)
    HIP_TRY(c, hipMemsetAsync(f.p, 0xFF, 8 * 35 * (size_t)A, c->stream));
    HIP_TRY(c, hipMemsetAsync(k.p, 0xFF, 16 * (size_t)A, c->stream));
    st = dgn_dev_betti(c, &d, p, f.as<double>(), k.as<int32_t>());
    if (st == DGN_OK || st == DGN_ERR_CAPACITY || st == DGN_ERR_UNSUPPORTED) {
        if (A) {
            e = hipMemcpy(features, f.p, 8 * 35 * A, hipMemcpyDeviceToHost);
            if (!e && counts) e = hipMemcpy(counts, k.p, 16 * A, hipMemcpyDeviceToHost);
            if (e) st = hip_fail(c, e, "dgn_host_betti: copy back");
        }
    }
    return st;
}

int dgn_debug_betti_clouds(dgn_ctx* c, const dgn_batch* h, double rc, int64_t first, int64_t count, int32_t max_points,
                           float* lower, int32_t* npoints, int64_t* keys) {
    if (!c || !h || !lower || !npoints || first < 0 || count < 0 || first + count > h->num_atoms || max_points < 1)
        return fail(c, DGN_ERR_ARG, "dgn_debug_betti_clouds: bad args");
    if (count == 0) return DGN_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    dgn_batch d;
    int st = stage_batch(c, h, &d);
    if (st) return st;
    int64_t E = 0;
    st = graph_count_impl(c, &d, rc, UINT64_MAX, 1e-10, &E, true);
    if (st) return st;
    if ((int64_t)c->bw.max_candidates + 1 > max_points || max_points > betti_max_points())
        return fail(c, DGN_ERR_CAPACITY, "dgn_debug_betti_clouds: a complex has " +
                                             std::to_string(c->bw.max_candidates + 1) + " points");
    const int64_t tri = (int64_t)max_points * (max_points - 1) / 2;
    const int64_t tri_stride = std::max<int64_t>(4, (tri + 3) / 4 * 4);
    DevBuf dl, dn, dk;
    hipError_t e;
    if ((e = dl.ensure(4 * (size_t)(count * tri_stride))) || (e = dn.ensure(4 * (size_t)count)) ||
        (e = dk.ensure(8 * (size_t)(count * max_points))))
        return hip_fail(c, e, "dgn_debug_betti_clouds: allocation");
    HIP_TRY(c, hipMemsetAsync(dl.p, 0, 4 * (size_t)(count * tri_stride), c->stream));
    HIP_TRY(c, hipMemsetAsync(dk.p, 0, 8 * (size_t)(count * max_points), c->stream));
    HIP_TRY(c, c->scalars.ensure(sizeof(Scalars)));
    Scalars* sc = c->scalars.as<Scalars>();
    HIP_TRY(c, hipMemsetAsync(&sc->graph_flag, 0, sizeof(uint32_t), c->stream));
    const GraphLaunch g = graph_launch(c->bw, &d, rc, 1e-10, UINT64_MAX, true);
    HIP_TRY(c, launch_betti_dist_search(c->stream, g, first, count, max_points, tri_stride, c->bw.counts.as<int32_t>(),
                                        dl.as<float>(), dn.as<int32_t>(), &sc->graph_flag, dk.as<uint64_t>(),
                                        max_points));
    HIP_TRY(c, hipMemcpyAsync(&c->host->s.graph_flag, &sc->graph_flag, sizeof(uint32_t), hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, stream_sync(c));
    if (c->host->s.graph_flag)
        return fail(c, DGN_ERR_INTERNAL, "dgn_debug_betti_clouds: search disagreed with the count pass");
    std::vector<float> tmp((size_t)(count * tri_stride));
    if ((e = hipMemcpy(tmp.data(), dl.p, 4 * tmp.size(), hipMemcpyDeviceToHost)) ||
        (e = hipMemcpy(npoints, dn.p, 4 * (size_t)count, hipMemcpyDeviceToHost)) ||
        (keys && (e = hipMemcpy(keys, dk.p, 8 * (size_t)(count * max_points), hipMemcpyDeviceToHost))))
        return hip_fail(c, e, "dgn_debug_betti_clouds: copy back");
    for (int64_t i = 0; i < count; ++i) std::memcpy(lower + i * tri, tmp.data() + i * tri_stride, 4 * (size_t)tri);
    return DGN_OK;
}

// Complexes above the kernels' kWideMaxPoints-point envelope (betti_split.hip): split into the
// connected components of their threshold graph, whose persistence pairs union to the complex's
// (ripser.cpp:386-395, 514-1269 on a block-diagonal coboundary matrix); each component of two or
// more points is reduced by the ordinary Betti pass as a caller-given triangle, a one-point
// component adds one essential dim-0 class. pairs [C][3][cap][2] (unsorted here) and kk [C][4] are
// filled on the host. A component above kWideGiantPoints points (or a GIANT one with 2^20 or more
// distances within the threshold): DGN_ERR_UNSUPPORTED.
static int persistence_split(dgn_ctx* c, const double* d_clouds, const float* d_lower, const int32_t* d_np,
                             const int32_t* npoints, int64_t C, int32_t max_points, double threshold, float* pairs,
                             int32_t cap, std::vector<int32_t>& kk) {
    const int64_t tri_in = (int64_t)max_points * (max_points - 1) / 2;  // caller-given packing
    const int64_t tri_stride = (tri_in + 3) / 4 * 4;
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(C, (int64_t(8) << 30) / (4 * tri_stride)));
    if (c->dbg_split_chunk > 0) chunk = std::min<int64_t>(chunk, c->dbg_split_chunk);  // tests only
    DevBuf tri, lab, dmap, doff, dsize, dsrc, sub, snp, spairs, scnt;
    if (d_clouds) HIP_TRY(c, tri.ensure(4 * (size_t)(chunk * tri_stride)));
    HIP_TRY(c, lab.ensure(4 * (size_t)(chunk * max_points)));
    std::vector<int32_t> labels((size_t)(chunk * max_points));
    std::fill(kk.begin(), kk.end(), 0);
    for (int64_t c0 = 0; c0 < C; c0 += chunk) {
        const int64_t cnt = std::min<int64_t>(chunk, C - c0);
        const float* T = d_lower ? d_lower + c0 * tri_in : tri.as<float>();
        const int64_t ts = d_lower ? tri_in : tri_stride;
        if (d_clouds) HIP_TRY(c, launch_big_gram(c->stream, d_clouds, max_points, d_np, c0, cnt, tri.as<float>(), tri_stride));
        HIP_TRY(c, launch_components(c->stream, T, ts, d_np, c0, cnt, (float)threshold, lab.as<int32_t>(), max_points));
        HIP_TRY(c, hipMemcpyAsync(labels.data(), lab.p, 4 * (size_t)(cnt * max_points), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_sync(c));
        // components (a root is its component's smallest vertex): vertex lists in ascending order
        std::vector<int32_t> map, src, size;
        std::vector<int64_t> off;
        int32_t smax = 1;
        for (int64_t i = 0; i < cnt; ++i) {
            const int32_t n = npoints[c0 + i];
            const int32_t* L = labels.data() + i * max_points;
            std::vector<int32_t> count((size_t)n, 0);
            for (int32_t v = 0; v < n; ++v) ++count[(size_t)L[v]];
            std::vector<int64_t> first((size_t)n, -1);
            for (int32_t r = 0; r < n; ++r) {
                if (count[(size_t)r] == 0) continue;
                if (count[(size_t)r] == 1) {
                    ++kk[4 * (size_t)(c0 + i) + 1];  // one point: an essential dim-0 class, no pairs
                    continue;
                }
                if (count[(size_t)r] > kWideGiantPoints)
                    return fail(c, DGN_ERR_UNSUPPORTED,
                                "a connected component of " + std::to_string(count[(size_t)r]) +
                                    " points at this threshold exceeds the " + std::to_string(kWideGiantPoints) +
                                    "-point kernel envelope (see DESIGN.md)");
                first[(size_t)r] = (int64_t)map.size();
                off.push_back((int64_t)map.size());
                size.push_back(count[(size_t)r]);
                src.push_back((int32_t)i);
                smax = std::max(smax, count[(size_t)r]);
                map.resize(map.size() + (size_t)count[(size_t)r]);
            }
            std::vector<int32_t> fill((size_t)n, 0);
            for (int32_t v = 0; v < n; ++v) {
                const int32_t r = L[v];
                if (first[(size_t)r] >= 0) map[(size_t)(first[(size_t)r] + fill[(size_t)r]++)] = v;
            }
        }
        const int64_t nsub = (int64_t)size.size();
        if (nsub == 0) continue;
        (void)smax;
        // Components in groups of similar size (largest first), each group one Betti pass whose
        // triangle stride and pair capacity are its largest member's -- not the chunk's: a cloud with
        // one 2,000-point cluster and thousands of 2-point components would otherwise give every
        // component a 2,000-point triangle and a full pair block -- and whose sub-triangles and pairs
        // stay within a byte budget
        std::vector<int64_t> order((size_t)nsub);
        for (int64_t q = 0; q < nsub; ++q) order[(size_t)q] = q;
        std::stable_sort(order.begin(), order.end(),
                         [&](int64_t x, int64_t y) { return size[(size_t)x] > size[(size_t)y]; });
        hipError_t e;
        if ((e = dmap.ensure(4 * map.size())))
            return hip_fail(c, e, "dgn_host_persistence: component split allocation");
        HIP_TRY(c, hipMemcpyAsync(dmap.p, map.data(), 4 * map.size(), hipMemcpyHostToDevice, c->stream));
        constexpr int64_t kGroupBytes = int64_t(2) << 30;
        for (int64_t g0 = 0; g0 < nsub;) {
            const int32_t gmax = size[(size_t)order[(size_t)g0]];
            const int64_t gstride = std::max<int64_t>(1, (int64_t)gmax * (gmax - 1) / 2);
            // pairs per diagram of a gmax-point complex: dim 0 < gmax, dim 1 < C(gmax, 2), dim 2 < C(gmax, 3)
            const int64_t c3 = (int64_t)gmax * (gmax - 1) * (gmax - 2) / 6;
            const int32_t gcap = (int32_t)std::min<int64_t>(cap, std::max<int64_t>({(int64_t)gmax, gstride, c3, 1}));
            const int64_t per = 4 * gstride + 24 * (int64_t)gcap + 64;
            const int64_t gn = std::max<int64_t>(1, std::min<int64_t>(nsub - g0, kGroupBytes / per));
            std::vector<int64_t> goff((size_t)gn);
            std::vector<int32_t> gsize((size_t)gn), gsrc((size_t)gn);
            for (int64_t t = 0; t < gn; ++t) {
                const int64_t q = order[(size_t)(g0 + t)];
                goff[(size_t)t] = off[(size_t)q];
                gsize[(size_t)t] = size[(size_t)q];
                gsrc[(size_t)t] = src[(size_t)q];
            }
            if ((e = doff.ensure(8 * (size_t)gn)) || (e = dsize.ensure(4 * (size_t)gn)) || (e = dsrc.ensure(4 * (size_t)gn)) ||
                (e = sub.ensure(4 * (size_t)(gn * gstride))) || (e = snp.ensure(4 * (size_t)gn)) ||
                (e = spairs.ensure(8 * 3 * (size_t)gn * gcap)) || (e = scnt.ensure(16 * (size_t)gn)))
                return hip_fail(c, e, "dgn_host_persistence: component split allocation");
            HIP_TRY(c, hipMemcpyAsync(doff.p, goff.data(), 8 * (size_t)gn, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemcpyAsync(dsize.p, gsize.data(), 4 * (size_t)gn, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemcpyAsync(dsrc.p, gsrc.data(), 4 * (size_t)gn, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemcpyAsync(snp.p, gsize.data(), 4 * (size_t)gn, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, launch_gather_sub(c->stream, T, ts, dsrc.as<int32_t>(), doff.as<int64_t>(), dsize.as<int32_t>(),
                                         dmap.as<int32_t>(), gn, sub.as<float>(), gstride));
            int st = betti_impl(c, nullptr, threshold, nullptr, scnt.as<int32_t>(), nullptr, snp.as<int32_t>(),
                                std::max<int32_t>(gmax, 2), gn, spairs.as<float>(), gcap, sub.as<float>());
            if (st) return st;
            std::vector<int32_t> sk(4 * (size_t)gn);
            std::vector<float> sp(2 * 3 * (size_t)gn * gcap);
            HIP_TRY(c, hipMemcpy(sk.data(), scnt.p, 16 * (size_t)gn, hipMemcpyDeviceToHost));
            HIP_TRY(c, hipMemcpy(sp.data(), spairs.p, 8 * 3 * (size_t)gn * gcap, hipMemcpyDeviceToHost));
            // the union of the components' pairs (counts past cap are reported by the caller)
            for (int64_t t = 0; t < gn; ++t) {
                const int64_t i = c0 + gsrc[(size_t)t];
                int32_t* k = kk.data() + 4 * i;
                k[1] += sk[4 * (size_t)t + 1];
                const int col[3] = {0, 2, 3};
                for (int d = 0; d < 3; ++d) {
                    const int32_t m = sk[4 * (size_t)t + col[d]];
                    for (int32_t u = 0; u < m && u < gcap; ++u) {
                        const int32_t slot = k[col[d]] + u;
                        if (slot >= cap) break;
                        const float* from = sp.data() + ((size_t)(t * 3 + d) * gcap + u) * 2;
                        float* to = pairs + ((size_t)(i * 3 + d) * cap + slot) * 2;
                        to[0] = from[0];
                        to[1] = from[1];
                    }
                    k[col[d]] += m;
                }
            }
            g0 += gn;
        }
    }
    return DGN_OK;
}

static int host_persistence_common(dgn_ctx* c, const double* clouds, const float* lower, const int32_t* npoints,
                                   int64_t C, int32_t max_points, double threshold, float* pairs, int32_t cap,
                                   int32_t* counts) {
    if (!c || (!clouds && !lower) || !npoints || C < 0 || max_points <= 0 || cap <= 0 || !pairs)
        return fail(c, DGN_ERR_ARG, "dgn_host_persistence: bad args");
    if (max_points > kSplitMaxPoints)
        return fail(c, DGN_ERR_UNSUPPORTED, "dgn_host_persistence: clouds above " + std::to_string(kSplitMaxPoints) +
                                                " points");
    if (C == 0) return DGN_OK;
    for (int64_t i = 0; i < C; ++i)
        if (npoints[i] < 1 || npoints[i] > max_points) return fail(c, DGN_ERR_ARG, "npoints out of range");
    HIP_TRY(c, hipSetDevice(c->device));
    DevBuf dc, dn, dp, dk;
    const size_t in_bytes = clouds ? 24 * (size_t)C * max_points
                                   : 4 * (size_t)C * ((size_t)max_points * (max_points - 1) / 2);
    hipError_t e;
    if ((e = dc.ensure(in_bytes)) || (e = dn.ensure(4 * (size_t)C)) || (e = dp.ensure(8 * 3 * (size_t)C * cap)) ||
        (e = dk.ensure(16 * (size_t)C)))
        return hip_fail(c, e, "dgn_host_persistence: allocation");
    HIP_TRY(c, hipMemcpy(dc.p, clouds ? (const void*)clouds : (const void*)lower, in_bytes, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(dn.p, npoints, 4 * (size_t)C, hipMemcpyHostToDevice));
    std::vector<int32_t> kk(4 * C);
    const bool split = max_points > kWideMaxPoints;  // complexes above the kernels' envelope
    int st = split ? persistence_split(c, clouds ? dc.as<double>() : nullptr, clouds ? nullptr : dc.as<float>(),
                                       dn.as<int32_t>(), npoints, C, max_points, threshold, pairs, cap, kk)
                   : betti_impl(c, nullptr, threshold, nullptr, dk.as<int32_t>(), clouds ? dc.as<double>() : nullptr,
                                dn.as<int32_t>(), max_points, C, dp.as<float>(), cap, clouds ? nullptr : dc.as<float>());
    if (!st) {
        if (!split) {
            HIP_TRY(c, hipMemcpy(kk.data(), dk.p, 16 * (size_t)C, hipMemcpyDeviceToHost));
            HIP_TRY(c, hipMemcpy(pairs, dp.p, 8 * 3 * (size_t)C * cap, hipMemcpyDeviceToHost));
        }
        // sort each diagram ascending by (birth, death) for a canonical order
        for (int64_t i = 0; i < C; ++i) {
            const int n_per[3] = {kk[4 * i], kk[4 * i + 2], kk[4 * i + 3]};
            for (int d = 0; d < 3; ++d) {
                std::pair<float, float>* P = reinterpret_cast<std::pair<float, float>*>(pairs + ((i * 3 + d) * cap) * 2);
                std::sort(P, P + std::min(n_per[d], cap));
            }
        }
        if (counts) std::memcpy(counts, kk.data(), 16 * (size_t)C);
        for (int64_t i = 0; i < C; ++i)
            if (kk[4 * i] > cap || kk[4 * i + 2] > cap || kk[4 * i + 3] > cap) st = fail(c, DGN_ERR_CAPACITY, "pair cap");
    }
    return st;
}

int dgn_host_persistence(dgn_ctx* c, const double* clouds, const int32_t* npoints, int64_t C, int32_t max_points,
                         double threshold, float* pairs, int32_t cap, int32_t* counts) {
    if (!clouds) return fail(c, DGN_ERR_ARG, "dgn_host_persistence: null clouds");
    return host_persistence_common(c, clouds, nullptr, npoints, C, max_points, threshold, pairs, cap, counts);
}

int dgn_host_persistence_lower(dgn_ctx* c, const float* lower, const int32_t* npoints, int64_t C, int32_t max_points,
                               double threshold, float* pairs, int32_t cap, int32_t* counts) {
    if (!lower) return fail(c, DGN_ERR_ARG, "dgn_host_persistence_lower: null matrix");
    return host_persistence_common(c, nullptr, lower, npoints, C, max_points, threshold, pairs, cap, counts);
}

int dgn_host_rbf(dgn_ctx* c, const double* distances, int64_t E, double rbf_cutoff, double rbf_dr, int32_t dtype,
                 int32_t layout, void* out) {
    if (!c || E < 0 || (E && (!distances || !out)) || (dtype != DGN_F32 && dtype != DGN_F64) ||
        (layout != 0 && layout != 1) || !(rbf_dr > 0) || dgn_rbf_bins(rbf_cutoff, rbf_dr) <= 0)
        return fail(c, DGN_ERR_ARG, "dgn_host_rbf: bad args");
    if (E == 0) return DGN_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    dgn_graph_params p;
    dgn_graph_params_default(&p);
    p.rbf_cutoff = rbf_cutoff;
    p.rbf_dr = rbf_dr;
    p.rbf_dtype = dtype;
    const RbfSpec rs = make_rbf(&p);
    const size_t elem = dtype == DGN_F32 ? 4 : 8;
    DevBuf dd, dout;
    hipError_t e;
    if ((e = dd.ensure(8 * (size_t)E)) || (e = dout.ensure(elem * (size_t)E * rs.nbins)))
        return hip_fail(c, e, "dgn_host_rbf: allocation");
    HIP_TRY(c, hipMemcpyAsync(dd.p, distances, 8 * (size_t)E, hipMemcpyHostToDevice, c->stream));
    {
        TimedLaunch t(c, "rbf", (double)E * 8 + (double)E * rs.nbins * elem, 0);
        HIP_TRY(c, launch_rbf(c->stream, dd.as<double>(), E, rs, layout, dout.p));
    }
    HIP_TRY(c, hipMemcpyAsync(out, dout.p, elem * (size_t)E * rs.nbins, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_sync(c));
    return DGN_OK;
}


int64_t dgn_synth_atoms_per_structure(int kind, int m) {
    if (m <= 0) return -1;
    return kind == 0 ? (int64_t)m * m * m : kind == 1 ? 4LL * m * m * m : -1;
}

int dgn_synth_batch(int kind, int m, int64_t B, int64_t first_id, double* lattice, double* positions, int32_t* species,
                    int64_t* atom_offset) {
    const int64_t n = dgn_synth_atoms_per_structure(kind, m);
    if (n <= 0 || B < 0 || !lattice || !positions || !atom_offset) return DGN_ERR_ARG;
    const double s = kind == 0 ? 2.32 : std::pow(4.0 / 0.08, 1.0 / 3.0);
    const double L = m * s;
    static const double basis[4][3] = {{0, 0, 0}, {0.5, 0.5, 0}, {0.5, 0, 0.5}, {0, 0.5, 0.5}};
    for (int64_t b = 0; b < B; ++b) {
        double* lat = lattice + 9 * b;
        for (int k = 0; k < 9; ++k) lat[k] = 0.0;
        lat[0] = lat[4] = lat[8] = L;
        atom_offset[b] = b * n;
        const uint64_t seed = 0x5EED0000ull + (uint64_t)(first_id + b);
        uint64_t draw = 0;
        for (int64_t i = 0; i < n; ++i) {
            double base[3];
            int sp;
            if (kind == 0) {
                const int64_t ix = i / ((int64_t)m * m), iy = (i / m) % m, iz = i % m;
                base[0] = (double)ix + 0.5;
                base[1] = (double)iy + 0.5;
                base[2] = (double)iz + 0.5;
                sp = (int)((ix + iy + iz) % 2);
            } else {
                const int64_t cell = i / 4, bb = i % 4;
                const int64_t cx = cell / ((int64_t)m * m), cy = (cell / m) % m, cz = cell % m;
                base[0] = ((double)cx + basis[bb][0]) + 0.25;
                base[1] = ((double)cy + basis[bb][1]) + 0.25;
                base[2] = ((double)cz + basis[bb][2]) + 0.25;
                sp = (int)(bb % 2);
            }
            double* p = positions + 3 * (b * n + i);
            for (int k = 0; k < 3; ++k) {
                ++draw;
                const uint64_t z = mix64(seed + draw * 0x9E3779B97F4A7C15ull);
                const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
                p[k] = base[k] * s + (0.1 * u - 0.05) * s;
            }
            if (species) species[b * n + i] = sp;
        }
    }
    atom_offset[B] = B * n;
    return DGN_OK;
}

}  // extern "C"
