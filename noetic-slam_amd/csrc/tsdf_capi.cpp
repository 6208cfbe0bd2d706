// tsdf_capi.cpp — extern "C" boundary of libtsdf_hip.so (declared in include/tsdf_hip.h).
//
// One tsdf_ctx = one HIP device + one non-blocking stream + the brick hash table, brick pool and
// batch work buffers, all allocated once at create (no allocation on the integrate path).  The
// host-pointer integrate packs the caller's PointCloud2-style records (any point_step/xyz_offset,
// f32 or f64 xyz) into one of two pinned staging buffers, copies them into the device staging
// area of the pending batch and returns; the batch is launched when max_batch scans are pending
// or when any other call needs the field (see "Batching" in the header).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tsdf_hip.h"
#include "../../include/tsdf_mc_tables.h"
#include "pack_pool.h"
#include "tsdf_device.h"

using namespace tsdf;

static_assert(TSDF_MAX_BATCH == MAX_BATCH, "header and device batch limits differ");
static_assert(TSDF_TILE_WORDS == TILE_WORDS && TSDF_MAX_WORLD == MAX_WORLD, "border tile layout differs");
static_assert(TSDF_MC_TABLES == MC_TABLES, "marching-cubes table count differs");

namespace {

// Diagnostic host timing of launch() sections (TSDF_HOST_TIMING=1: averages printed at destroy).
struct HostTiming {
    bool on = std::getenv("TSDF_HOST_TIMING") != nullptr;
    double acc[12] = {};
    uint64_t n = 0;
    std::chrono::steady_clock::time_point t;
    void start() { if (on) t = std::chrono::steady_clock::now(); }
    void lap(int k) {
        if (!on) return;
        const auto u = std::chrono::steady_clock::now();
        acc[k] += std::chrono::duration<double, std::micro>(u - t).count();
        t = u;
    }
    ~HostTiming() {
        if (!on || !n) return;
        std::fprintf(stderr, "host launch timing (us/batch over %llu):", (unsigned long long)n);
        for (int k = 0; k < 12; k++) std::fprintf(stderr, " %d:%.2f", k, acc[k] / n);
        std::fprintf(stderr, "\n");
    }
};

struct EventTimer final : KernelTimer {
    struct Rec { int kind; uint64_t batch; hipEvent_t a, b; bool own_a; };
    uint64_t cur_batch = 0;  // the batch being launched (set by launch())
    bool per_batch = false;  // keep per-batch times for the metrics log
    std::vector<std::pair<uint64_t, std::array<double, KIND_N>>> batch_ms;
    std::vector<hipEvent_t> free_ev;
    std::vector<Rec> pending;
    hipEvent_t open_ev[KIND_N] = {};
    bool open_own[KIND_N] = {};  // open_ev[k] is not also the end of an earlier record
    uint32_t every_mask = ~0u;   // kinds timed on every batch (tsdf_set_profiling_period)
    uint32_t period = 1;         // the other kinds: every period-th batch
    bool want(int kind) const { return ((every_mask >> kind) & 1u) || cur_batch % period == 0; }
    double ms[KIND_N] = {};
    uint64_t launches[KIND_N] = {};

    hipEvent_t get() {
        if (free_ev.empty()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            return e;
        }
        hipEvent_t e = free_ev.back();
        free_ev.pop_back();
        return e;
    }
    void begin(int kind, hipStream_t st) override {
        open_ev[kind] = get();
        open_own[kind] = true;
        if (open_ev[kind]) (void)hipEventRecord(open_ev[kind], st);
    }
    void end(int kind, hipStream_t st) override {
        hipEvent_t e = get();
        if (!e || !open_ev[kind]) return;
        (void)hipEventRecord(e, st);
        pending.push_back({kind, cur_batch, open_ev[kind], e, open_own[kind]});
        open_ev[kind] = nullptr;
    }
    // events the kernel launch itself records (its dispatch packet's timestamps: KTime)
    KTime timing(int kind) {
        hipEvent_t a = get(), b = get();
        if (!a || !b) return {};
        pending.push_back({kind, cur_batch, a, b, true});
        return {a, b};
    }
    // end `done` and begin `open` with ONE event, for kernels launched back to back on one stream
    // (every timing event is a queue barrier with a timestamp: ~4 us each per batch)
    void next(int done, int open, hipStream_t st) {
        hipEvent_t e = get();
        if (!e || !open_ev[done]) return begin(open, st);
        (void)hipEventRecord(e, st);
        pending.push_back({done, cur_batch, open_ev[done], e, open_own[done]});
        open_ev[done] = nullptr;
        open_ev[open] = e;
        open_own[open] = false;
    }
    // call only after the stream drained
    void harvest() {
        for (auto& r : pending) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
                ms[r.kind] += t;
                launches[r.kind]++;
                if (per_batch) {
                    if (batch_ms.empty() || batch_ms.back().first != r.batch)
                        batch_ms.push_back({r.batch, std::array<double, KIND_N>{}});
                    batch_ms.back().second[r.kind] += t;
                }
            }
            if (r.own_a) free_ev.push_back(r.a);  // else it is an earlier record's b
            free_ev.push_back(r.b);
        }
        pending.clear();
    }
    void reset() {
        std::fill(ms, ms + KIND_N, 0.0);
        std::fill(launches, launches + KIND_N, 0);
    }
    ~EventTimer() override {
        for (auto& r : pending) {
            if (r.own_a) (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        for (auto e : free_ev) (void)hipEventDestroy(e);
    }
};

uint64_t next_pow2(uint64_t v) {
    uint64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

// Sector k of n starts at the pseudo-angle of yaw0 + 2 pi k / n (include/tsdf_hip.h
// tsdf_sector_of); the oracle computes the same bounds with the same operations.
float sector_start(double yaw0, uint32_t k, uint32_t n) {
    const double th = yaw0 + 6.283185307179586476925286766559 * (double)k / (double)n;
    return pseudo_angle((float)std::cos(th), (float)std::sin(th));
}

void sector_bounds(double yaw0, uint32_t sector, uint32_t n, RayConst& R) {
    R.sec_on = n > 1 ? 1 : 0;
    if (!R.sec_on) return;
    R.sec_lo = sector_start(yaw0, sector, n);
    R.sec_hi = sector_start(yaw0, (sector + 1) % n, n);
    R.sec_wrap = R.sec_hi <= R.sec_lo ? 1 : 0;
}

// The smallest double x >= 0 with (float)sqrt(x) >= tau (bisection over the ordered bit patterns
// of non-negative doubles): behind the hit, VDBFusion's gate -(float)dist > -tau holds iff
// d2 < this threshold (TSDF_SEM_VDBFUSION_F64; the oracle gates on the sqrt itself).
double gate_threshold(float tau) {
    auto ok = [&](uint64_t b) {
        double x;
        std::memcpy(&x, &b, 8);
        return (float)std::sqrt(x) >= tau;
    };
    double hi_d = 4.0 * (double)tau * (double)tau + 1.0;
    uint64_t lo = 0, hi;
    std::memcpy(&hi, &hi_d, 8);
    while (hi - lo > 1) {  // ok(lo) false, ok(hi) true
        const uint64_t mid = lo + (hi - lo) / 2;
        if (ok(mid)) hi = mid;
        else lo = mid;
    }
    double x;
    std::memcpy(&x, &hi, 8);
    return x;
}

}  // namespace

struct tsdf_ctx {
    tsdf_params p{};
    int device = -1;
    hipStream_t stream = nullptr;
    RayConst R{};
    Table T{};
    Pool Pl{};
    Work Wk{};
    Globals* G = nullptr;
    uint64_t cap = 0;
    uint64_t max_points = 0;  // per scan
    uint32_t max_batch = 0;
    uint64_t batch_points = 0;  // pair-slot capacity / maxp: points one batch may hold
    uint32_t max_blocks = 0;    // k_count / k_place workgroups one batch may need
    uint64_t slots = 0;         // pair slots of one batch
    // single walk: k_walk + k_spans instead of k_count + k_place, when asked for
    // (tsdf_params.walk) and the band's walk fits nstep register slots per ray
    bool fused = false;
    int nstep = 0;
    // batches of at most small_ns scans take k_integrate_small (TSDF_SMALL_NS; 0: never; measured
    // break-even with k_integrate at 6 scans)
    int small_ns = 5;
    // batches of at most count_wide k_count blocks (about 4 full scans: too few workgroups of 256
    // lanes to fill the chip) run k_count with 1024-lane workgroups (TSDF_COUNT_WIDE; 0: never)
    uint32_t count_wide = 512;
    // TSDF_COUNT_PAIRED=1: larger batches run k_count with two blocks per 512-lane workgroup
    // (bit-exact, ~29% fewer cell atomics, but measured slower: DESIGN.md §10, round 4)
    bool count_paired = false;
    // host-pointer path: pinned double buffer per scan; the pending batch's points are staged in
    // stage2[batch parity]
    float* h_stage[2] = {nullptr, nullptr};
    hipEvent_t stage_done[2] = {nullptr, nullptr};
    int stage_cur = 0;
    // Batch pipeline: batch b runs on bst[b & 1] with its own work buffers (W2), per-scan cells
    // (cell2) and device staging (stage2), so batch b + 1's count / compact / place overlap batch
    // b's place / integrate.  Cross-batch order: k_count(b+1) after k_compact(b)
    // (the table's `touched` words), k_integrate(b+1) after k_finish(b) (per-brick fuse order).
    hipStream_t bst[2] = {nullptr, nullptr};
    Work W2[2]{};
    uint32_t* cell2[2] = {nullptr, nullptr};  // u64 cells with the single walk
    float* stage2[2] = {nullptr, nullptr};
    hipEvent_t ev_main = nullptr;
    hipEvent_t ev_compact[2] = {nullptr, nullptr};
    // the end of the last batch of each parity: the ring event of that batch's slot (one marker
    // per batch; every marker in the stream costs the GPU a few microseconds)
    hipEvent_t ev_integ[2] = {nullptr, nullptr};
    BatchDesc pend{};  // pending host scans (points in stage2[pend_stage])
    // Device staging ownership (independent of batch parity, which replays can shift): the pending
    // batch's buffer, and per buffer the last batch that read it (its id and completion event).
    int pend_stage = 0;
    int last_stage = 1;  // the buffer of the most recently launched host batch
    uint64_t stage_reader[2] = {~0ull, ~0ull};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    // batch records for the kernels: a pinned host ring and its device twin (launch() copies a
    // batch's n_scans + 1 records into the next slot on the batch's stream)
    static constexpr int RING = 16;
    HostTiming ht;
    ScanRec* h_ring = nullptr;
    ScanRec* d_ring = nullptr;
    const ScanRec* d_ring_src = nullptr;  // h_ring as the device addresses it (k_upload)
    // ring progress: k_upload of launch q stores q + 1 here once it has read its slot
    unsigned long long* h_ring_done = nullptr;
    unsigned long long* d_ring_done = nullptr;
    hipEvent_t ring_ev[RING] = {};
    uint64_t ring_next = 0;
    uint64_t batch_id = 0;
    uint64_t n_scans = 0, n_batches = 0, n_points_in = 0;
    EventTimer* timer = nullptr;
    std::string err;
    // Capacity growth: batches launched since the last check, replayable from their
    // still-valid input (caller device memory until tsdf_sync; host scans in stage2 until the
    // staging of batch id + 2, where a checkpoint runs first).
    struct Logged { uint64_t id; const float* xyz; BatchDesc D; };
    std::vector<Logged> log;
    bool can_grow = false;  // G->retry: overflowed batches are skipped and replayed
    bool in_replay = false;
    // metrics log (tsdf_set_metrics_log): one JSON line per finished batch
    FILE* metrics = nullptr;
    uint64_t metrics_next = 0;  // the next batch id to report
    struct BatchInfo { uint64_t id; uint32_t scans; uint64_t points; };
    std::vector<BatchInfo> metrics_info;  // host-side facts of the batches not yet reported
    PackPool* pack = nullptr;  // host staging threads (tsdf_integrate of strided records)
    // tsdf_integrate_sectors' packed scan (xyz, then the sector per point) when this context
    // leads the split: cache-resident between its two passes
    std::vector<float> split_xyz;
    std::vector<int8_t> split_sec;
    HostTiming split_ht;  // TSDF_HOST_TIMING: prep, classify, scatter, copies + queue (us/scan)
    uint64_t n_grows = 0, n_replayed = 0;
    // Voxblox MergedTsdfIntegrator (tsdf_params.voxblox_method): the bundling pre-pass' buffers,
    // one set per batch parity (tsdf_merged.hip)
    bool merged = false;
    // TSDF_SECTOR_RULE_INDEX sharding (ABI v10): the context takes points [share_lo, share_hi) of
    // every cloud (idx_share); the kernels' azimuth filter is off (R.sec_on = 0)
    bool idx_rule = false;
    MgBufs mg[2];
    // tsdf_create_sharded: the contexts whose device memory this one reaches directly (peer access
    // or the same device); tsdf_integrate_sectors' fan-out: its copy-done event (this device)
    uint64_t peer_mask = 0;
    hipEvent_t bc_ev = nullptr;
    // tsdf_integrate_sectors' fan-out, batch-granular: a follower's pending points [fan_lo, fan_hi)
    // are still in its leader's staging buffer fan_buf (same offsets: the contexts' batches run in
    // lockstep) and are copied in ONE device-to-device copy before the follower's batch launches
    // (fan_copy); the leader keeps its followers, so it never reuses a buffer they still read
    tsdf_ctx* fan_src = nullptr;
    const float* fan_buf = nullptr;
    uint64_t fan_lo = 0, fan_hi = 0;
    std::vector<tsdf_ctx*> fan_followers;
    // border-reduce transaction (ABI v9): the pool slots the open reduce's pack sent
    // (reset at commit) and, per merge, the received bricks' pre-merge tiles (written back at
    // abort).  While a reduce is open the context takes no scan and no import.
    bool brd_open = false;
    uint32_t* brd_sent = nullptr;
    uint64_t brd_n_sent = 0;
    std::vector<std::pair<uint32_t*, uint64_t>> brd_backup;
};

// A context with an open border reduce refuses new mass until the reduce is committed or aborted
// (a commit resets the sent bricks: mass integrated into them meanwhile would be lost).
static bool border_busy(tsdf_ctx* c);

// Weight cap of the weighted-mean merges (import, border reduce): Voxblox's max_weight, else none
static float merge_cap(const tsdf_ctx* c) {
    return c->p.semantics == TSDF_SEM_VOXBLOX ? c->p.max_weight : INFINITY;
}

static int fail(tsdf_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

#define HIPCHK(c, expr)                                                                        \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((c), TSDF_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));      \
    } while (0)

// Pair slots per ray: the distinct bricks a DDA over the band can visit.  A segment of length L
// (voxels) covers at most E = floor(L) + 2 cells along an axis, E cells cross at most
// floor((E - 1) / 8) + 1 brick boundaries, and a line crosses them monotonically, one axis per
// step: 1 + 3 * crossings bricks.  (5 cm / 15 cm: 4.)  Exceeding it is reported (OVF_PAIRS).
static uint32_t pairs_per_ray(const tsdf_params& p) {
    double band;  // band length in voxels along the ray
    if (p.space_carving) band = (p.max_range + p.sdf_trunc) / p.voxel_size;
    else band = 2.0 * p.sdf_trunc / p.voxel_size;
    const double e = std::floor(band) + 2.0;
    const double crossings = std::floor((e - 1.0) / TSDF_BRICK_SIDE) + 1.0;
    return (uint32_t)(1.0 + 3.0 * crossings);
}

// Sample slots per ray: a ray's gated voxels are among its DDA voxels, at most
// 1 + 3 (floor(band) + 2) (5 cm / 15 cm: 25).
static uint32_t samples_per_ray(const tsdf_params& p) {
    double band;
    if (p.space_carving) band = (p.max_range + p.sdf_trunc) / p.voxel_size;
    else band = 2.0 * p.sdf_trunc / p.voxel_size;
    return (uint32_t)(1.0 + 3.0 * (std::floor(band) + 2.0));
}

// Launch one batch (desc offsets relative to d_xyz); fills the workgroup prefix of D.
static int check_and_replay(tsdf_ctx* c);
static int drain_all(tsdf_ctx* c);
static int emit_metrics(tsdf_ctx* c);

// Before launch seq rewrites its host ring slot: launch seq - RING (the slot's previous user) must
// have read it (its k_upload raised the progress word to seq - RING + 1).  Waits like an event
// synchronize (spin, then yield), and checks the batch streams for errors while it waits.
static int ring_wait(tsdf_ctx* c, uint64_t seq) {
    if (seq < (uint64_t)tsdf_ctx::RING) return TSDF_OK;
    const unsigned long long need = seq - tsdf_ctx::RING + 1;
    for (uint64_t i = 0;; i++) {
        if (__atomic_load_n(c->h_ring_done, __ATOMIC_ACQUIRE) >= need) return TSDF_OK;
        if (i < 64) continue;
        std::this_thread::yield();
        if ((i & 1023) == 0) {
            bool idle = true;
            for (int q = 0; q < 2; q++) {
                const hipError_t e = hipStreamQuery(c->bst[q]);
                if (e == hipErrorNotReady) idle = false;
                else if (e != hipSuccess) HIPCHK(c, e);
            }
            if (idle && __atomic_load_n(c->h_ring_done, __ATOMIC_ACQUIRE) < need)
                return fail(c, TSDF_EHIP, "scan-record ring: upload %llu never completed",
                            (unsigned long long)(need - 1));
        }
    }
}

static int launch(tsdf_ctx* c, const float* d_xyz, BatchDesc& D) {
    if (D.n_scans == 0) return TSDF_OK;
    c->ht.start();
    if (c->metrics && !c->in_replay && c->batch_id - c->metrics_next >= METRIC_RING - 8) {
        int rc = drain_all(c);  // the device ring of batch records would wrap
        if (!rc) rc = check_and_replay(c);
        if (!rc) rc = emit_metrics(c);
        if (rc) return rc;
    }
    if (c->can_grow && !c->in_replay && c->log.size() >= 1024) {
        // device-pointer batches stay replayable until a check: bound the log
        int rc = drain_all(c);
        if (!rc) rc = check_and_replay(c);
        if (rc) return rc;
    }
    D.s[0].blk = 0;
    for (uint32_t s = 0; s < D.n_scans; s++)
        D.s[s + 1].blk = D.s[s].blk + (D.s[s + 1].off - D.s[s].off + RPB - 1) / RPB;
    D.n_blocks = D.s[D.n_scans].blk;
    if (D.n_blocks > c->max_blocks)
        return fail(c, TSDF_EINVAL, "batch needs %u workgroups > %u", D.n_blocks, c->max_blocks);
    const int par = (int)(c->batch_id & 1);
    c->ht.lap(0);
#ifndef TSDF_TWO_STREAM_SERIAL
    // serial batches share one stream (stream order replaces the cross-stream waits); pipelined
    // batches alternate between two
    const bool cross = c->p.pipeline != 0;
#else
    const bool cross = true;
#endif
    hipStream_t st = c->bst[cross ? par : 0];
    Table T = c->T;
    T.cell = c->cell2[par];
    const Work& W = c->W2[par];
    EventTimer* tm = c->timer;
    if (tm) tm->cur_batch = c->batch_id;
    if (c->metrics) c->metrics_info.push_back({c->batch_id, D.n_scans, D.s[D.n_scans].off});
    // staging uploads, imports, ... (an idle context stream has nothing to order against)
    if (hipStreamQuery(c->stream) != hipSuccess) {
        HIPCHK(c, hipEventRecord(c->ev_main, c->stream));
        HIPCHK(c, hipStreamWaitEvent(st, c->ev_main, 0));
    }
    if (c->batch_id > 0 && cross)  // pipelined: after the previous batch's compact; else after all of it
        HIPCHK(c, hipStreamWaitEvent(st, c->p.pipeline ? c->ev_compact[par ^ 1]
                                                       : c->ev_integ[par ^ 1], 0));
    c->ht.lap(1);
    // the batch's scan records -> the device (a ring slot; the host slot is reused once its copy ran)
    const uint64_t seq = c->ring_next++;
    const int slot = (int)(seq % tsdf_ctx::RING);
    {
        int rc = ring_wait(c, seq);
        if (rc) return rc;
    }
    c->ht.lap(8);
    ScanRec* hs = c->h_ring + (size_t)slot * (MAX_BATCH + 1);
    ScanRec* ds = c->d_ring + (size_t)slot * (MAX_BATCH + 1);
    std::memcpy(hs, D.s, (D.n_scans + 1) * sizeof(ScanRec));
    c->ht.lap(9);
#ifdef TSDF_RING_MEMCPY
    HIPCHK(c, hipMemcpyAsync(ds, hs, (D.n_scans + 1) * sizeof(ScanRec), hipMemcpyHostToDevice, st));
#error "TSDF_RING_MEMCPY: the ring progress word is written by k_upload"
#else
    HIPCHK(c, launch_upload(c->d_ring_src + (size_t)slot * (MAX_BATCH + 1), ds,
                            (uint32_t)((D.n_scans + 1) * sizeof(ScanRec)), c->d_ring_done, seq + 1,
                            st));
#endif
    c->ht.lap(10);
    c->ht.lap(2);
    const BatchRef B{D.n_scans, D.n_blocks, ds};
    // MergedTsdfIntegrator: the batch's points bundled per (scan, voxel) first; the walk kernels
    // then read one ray per bundle, in the slot of its first point (tsdf_merged.hip)
    RayConst R = c->R;
    const float* d_rays = d_xyz;
    if (c->merged && D.n_blocks) {
        HIPCHK(c, launch_mg_prepass(d_xyz, B, D.n_blocks, D.s[D.n_scans].off, c->R, c->mg[par],
                                    &c->G->ctr[par].ovf, st));
        d_rays = c->mg[par].xyz_out;
        R.ray_w = c->mg[par].w_out;
    }
    // a small batch (a live node's 1-8 scans) fuses wave-per-brick, in table order (no k_order)
    const bool small = !c->fused && D.n_scans <= (uint32_t)c->small_ns;
    const int k_front = c->fused ? KIND_WALK : KIND_COUNT;
    const int k_back = c->fused ? KIND_SPANS : KIND_PLACE;
    // per-kernel times: the two-walk kernels record their own dispatch timestamps (KTime, no
    // marker packets); the single walk's stages are bracketed by marker events
    auto kt = [&](int kind) { return tm && !c->fused && tm->want(kind) ? tm->timing(kind) : KTime{}; };
    if (D.n_blocks) {
        if (tm && c->fused) tm->begin(k_front, st);
        if (c->R.sec_on) HIPCHK(c, launch_sector_flags(d_rays, B, R, W, c->G, par, st));
        if (c->fused) HIPCHK(c, launch_walk(d_rays, B, R, T, W, c->G, par, c->nstep, st));
        else HIPCHK(c, launch_count(d_rays, B, R, T, W, c->G, par, st, kt(KIND_COUNT),
                                    !c->R.sec_on && D.n_blocks <= c->count_wide,
                                    !c->R.sec_on && c->count_paired));
        c->ht.lap(3);
        if (tm && c->fused) tm->next(k_front, KIND_COMPACT, st);
        HIPCHK(c, launch_compact(B, T, W, c->G, par, c->fused, st, kt(KIND_COMPACT)));
        c->ht.lap(4);
#if defined(TSDF_SEPARATE_ORDER) && !defined(TSDF_NO_ORDER)
        if (!small) HIPCHK(c, launch_order(W, c->G, par, st));
#endif
    }
    // pipeline 1: batch b+1's front end waits for this batch's compact (it may run beside this
    // batch's place and integrate); pipeline 2: for its place, and this batch's place waits for
    // batch b-1's end, so only k_count / k_compact of b+1 overlap k_integrate of b and k_place
    // always runs alone
    const bool lean = c->p.pipeline == 2;
    if (cross && c->p.pipeline && !lean) HIPCHK(c, hipEventRecord(c->ev_compact[par], st));
    if (lean && c->batch_id > 0) HIPCHK(c, hipStreamWaitEvent(st, c->ev_integ[par ^ 1], 0));
    if (D.n_blocks) {
        if (tm && c->fused) tm->next(KIND_COMPACT, k_back, st);
        if (c->fused) HIPCHK(c, launch_spans(B, c->R, T, W, c->G, par, c->nstep, st));
        else HIPCHK(c, launch_place(d_rays, B, R, T, W, c->G, par, st, kt(KIND_PLACE)));
        c->ht.lap(5);
        if (tm && c->fused) tm->end(k_back, st);
    }
    if (lean) HIPCHK(c, hipEventRecord(c->ev_compact[par], st));  // batch b+1's front-end wait
    if (c->batch_id > 0 && cross && !lean) HIPCHK(c, hipStreamWaitEvent(st, c->ev_integ[par ^ 1], 0));
    if (D.n_blocks) {
        if (tm && c->fused) tm->begin(KIND_INTEGRATE, st);
        if (small) {
            HIPCHK(c, launch_integrate_small(B, c->R, T, W, c->Pl, c->G, par, st, kt(KIND_INTEGRATE)));
        } else {
#ifndef TSDF_NO_ORDER
            Work Wi = W;
            Wi.active = W.active_ord;  // largest bricks first (k_compact's size order)
#else
            const Work& Wi = W;
#endif
            HIPCHK(c, launch_integrate(B, c->R, T, Wi, c->Pl, c->G, par, c->fused, c->max_batch > 64, st,
                                       kt(KIND_INTEGRATE)));
        }
        if (tm && c->fused) tm->end(KIND_INTEGRATE, st);
        c->ht.lap(6);
    }
    HIPCHK(c, launch_finish(c->G, par, (uint32_t)c->batch_id, st));
    if (cross) {  // pipelined: the other stream's next batches wait on this batch's end
        HIPCHK(c, hipEventRecord(c->ring_ev[slot], st));
        c->ev_integ[par] = c->ring_ev[slot];
    }
    if (c->can_grow) c->log.push_back({c->batch_id, d_xyz, D});
    for (int k = 0; k < 2; k++)  // a host batch: its staging buffer's last reader
        if (d_xyz == c->stage2[k]) {
            c->stage_reader[k] = c->batch_id;
            HIPCHK(c, hipEventRecord(c->stage_ev[k], st));
        }
    c->ht.lap(7);
    c->ht.n++;
    c->batch_id++;
    c->n_batches++;
    c->n_scans += D.n_scans;
    if (tm && tm->pending.size() > 8192) {
        HIPCHK(c, hipStreamSynchronize(c->bst[0]));
        HIPCHK(c, hipStreamSynchronize(c->bst[1]));
        tm->harvest();
    }
    return TSDF_OK;
}

// The context stream waits for every launched batch (read-outs, imports, sync).
static int join(tsdf_ctx* c) {
    if (c->batch_id == 0) return TSDF_OK;
#ifndef TSDF_TWO_STREAM_SERIAL
    if (!c->p.pipeline) {  // serial batches: one stream, no per-batch marker; one now
        HIPCHK(c, hipEventRecord(c->ev_main, c->bst[0]));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_main, 0));
        return TSDF_OK;
    }
#endif
    for (int q = 0; q < 2; q++)
        if (c->batch_id > (uint64_t)q) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_integ[q], 0));
    return TSDF_OK;
}

// A fan-out follower's pending points, still in its leader's staging, copied into its own staging
// (device to device, xGMI between GPUs) after the leader's H2D copies; the leader's stream then
// waits for the copy, so the leader never rewrites that region first.  Leaves the current device
// as it found it.
static int fan_copy_range(tsdf_ctx* c, tsdf_ctx* s, float* dst, const float* src, uint64_t bytes) {
    int dev = 0;
    HIPCHK(c, hipGetDevice(&dev));
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamWaitEvent(c->stream, s->bc_ev, 0));  // the leader's H2D copies so far
    HIPCHK(c, c->device == s->device
                  ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream)
                  : hipMemcpyPeerAsync(dst, c->device, src, s->device, bytes, c->stream));
    if (!c->bc_ev) HIPCHK(c, hipEventCreateWithFlags(&c->bc_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->bc_ev, c->stream));
    HIPCHK(s, hipSetDevice(s->device));
    HIPCHK(s, hipStreamWaitEvent(s->stream, c->bc_ev, 0));
    HIPCHK(c, hipSetDevice(dev));
    return TSDF_OK;
}

static int fan_copy(tsdf_ctx* c) {
    if (!c->fan_src || !c->fan_buf || c->fan_hi <= c->fan_lo) {
        c->fan_lo = c->fan_hi;
        return TSDF_OK;
    }
    const int rc = fan_copy_range(c, c->fan_src, c->stage2[c->pend_stage] + 3 * c->fan_lo,
                                  c->fan_buf + 3 * c->fan_lo, (c->fan_hi - c->fan_lo) * 12);
    c->fan_lo = c->fan_hi;
    return rc;
}

// Launch the queued host scans (integrate paths: no join, so batches keep overlapping).
static int flush(tsdf_ctx* c) {
    if (c->pend.n_scans == 0) return TSDF_OK;
    if (c->fan_src) {  // a fan-out follower: its points first
        const int rc = fan_copy(c);
        if (rc) return rc;
    }
    // the buffer the pending scans were staged into; a replay that runs inside launch() (metrics
    // drain, log bound) re-reads only logged batches, none of which uses this buffer any more
    const int rc = launch(c, c->stage2[c->pend_stage], c->pend);
    c->last_stage = c->pend_stage;
    c->pend.n_scans = 0;
    c->pend.s[0].off = 0;
    return rc;
}

// flush + make the context stream wait for every batch (read-out, import, sync paths)
static int settle(tsdf_ctx* c) {
    const int rc = flush(c);
    return rc ? rc : join(c);
}

// ---- capacity: brick pool, hash table and per-brick work lists -----------------

struct Capacity {
    uint64_t max_bricks = 0, cap = 0;
    uint32_t max_active = 0;
    uint64_t* keys = nullptr;
    uint32_t* slots = nullptr;
    uint32_t* touched = nullptr;
    uint64_t* brick_keys = nullptr;
    float* sdf = nullptr;
    float* weight = nullptr;
    uint32_t* cell[2] = {nullptr, nullptr};
    uint4* active[2] = {nullptr, nullptr};
    uint4* active_ord[2] = {nullptr, nullptr};
    uint4* cagg[2] = {nullptr, nullptr};

    void free_all() {
        void* d[] = {keys, slots, touched, brick_keys, sdf, weight, cell[0], cell[1], active[0],
                     active[1], active_ord[0], active_ord[1], cagg[0], cagg[1]};
        for (void* q : d)
            if (q) (void)hipFree(q);
        *this = Capacity{};
    }
};

// Allocate (and clear: empty table, zero cells) the capacity-dependent buffers for max_bricks bricks;
// the pool's contents are the caller's.  Allocation failure is TSDF_ENOMEM with nothing leaked.
static int alloc_capacity(tsdf_ctx* c, uint64_t max_bricks, Capacity& K) {
    K = Capacity{};
    K.max_bricks = max_bricks;
    K.cap = next_pow2(2 * max_bricks);
    K.max_active = (uint32_t)std::min<uint64_t>(K.cap, c->slots);
    const size_t cells = K.cap * c->T.cell_stride * (c->fused ? sizeof(uint64_t) : sizeof(uint32_t));
    hipError_t e = hipMalloc(&K.keys, K.cap * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&K.slots, K.cap * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&K.touched, K.cap * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&K.brick_keys, max_bricks * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&K.sdf, max_bricks * BRICK_VOX * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&K.weight, max_bricks * BRICK_VOX * sizeof(float));
    for (int q = 0; q < 2 && e == hipSuccess; q++) {
        e = hipMalloc(&K.cell[q], cells);
        if (e == hipSuccess) e = hipMalloc(&K.active[q], (size_t)K.max_active * sizeof(uint4));
        if (e == hipSuccess) e = hipMalloc(&K.active_ord[q], (size_t)K.max_active * sizeof(uint4));
        if (e == hipSuccess) e = hipMalloc(&K.cagg[q], compact_chunks(K.cap) * 2 * sizeof(uint4));
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        K.free_all();
        return fail(c, TSDF_ENOMEM, "device allocation for %llu bricks failed",
                    (unsigned long long)max_bricks);
    }
    e = launch_fill_u64(K.keys, EMPTY_KEY, K.cap, c->stream);
    if (e == hipSuccess) e = launch_fill_u32(K.slots, UNASSIGNED, K.cap, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(K.touched, 0, K.cap * sizeof(uint32_t), c->stream);
    for (int q = 0; q < 2 && e == hipSuccess; q++) e = hipMemsetAsync(K.cell[q], 0, cells, c->stream);
    if (e != hipSuccess) {
        K.free_all();
        return fail(c, TSDF_EHIP, "capacity init: %s", hipGetErrorString(e));
    }
    return TSDF_OK;
}

// Make K the context's capacity (the previous buffers are freed; K is emptied).
static void install_capacity(tsdf_ctx* c, Capacity& K) {
    Capacity old;
    old.keys = c->T.keys; old.slots = c->T.slots; old.touched = c->T.touched;
    old.brick_keys = c->T.brick_keys; old.sdf = c->Pl.sdf; old.weight = c->Pl.weight;
    for (int q = 0; q < 2; q++) {
        old.cell[q] = c->cell2[q];
        old.active[q] = c->W2[q].active;
        old.active_ord[q] = c->W2[q].active_ord;
        old.cagg[q] = c->W2[q].cagg;
    }
    old.free_all();
    c->cap = K.cap;
    c->T.keys = K.keys; c->T.slots = K.slots; c->T.touched = K.touched;
    c->T.brick_keys = K.brick_keys;
    c->T.mask = K.cap - 1;
    c->T.max_bricks = (uint32_t)K.max_bricks;
    c->T.cell = K.cell[0];
    c->Pl.sdf = K.sdf; c->Pl.weight = K.weight;
    c->Wk.max_active = K.max_active;
    for (int q = 0; q < 2; q++) {
        c->cell2[q] = K.cell[q];
        c->W2[q].active = K.active[q];
        c->W2[q].active_ord = K.active_ord[q];
        c->W2[q].cagg = K.cagg[q];
        c->W2[q].max_active = K.max_active;
    }
    K = Capacity{};
}

// Grow the pool (and table, cells, lists) to hold at least `need` bricks: x2 or more, capped by
// max_bricks_hard.  Every batch must be complete.  The pool keeps its bricks (same slots); the
// table is rebuilt from the slot -> key map.  TSDF_ENOMEM: no growth possible.
static int grow_capacity(tsdf_ctx* c, uint64_t need) {
    const uint64_t old = c->T.max_bricks;
    uint64_t nb = std::max<uint64_t>(2 * old, need + need / 4);
    if (c->p.max_bricks_hard) nb = std::min<uint64_t>(nb, c->p.max_bricks_hard);
    nb = std::min<uint64_t>(nb, 0xFFFFFFEFull);
    if (nb <= old) return fail(c, TSDF_ENOMEM, "brick pool at its hard limit (%llu bricks)",
                               (unsigned long long)old);
    uint32_t pc = 0;
    HIPCHK(c, hipMemcpy(&pc, &c->G->pool_count, 4, hipMemcpyDeviceToHost));
    const uint64_t valid = std::min<uint64_t>(pc, old);
    Capacity K;
    int rc = alloc_capacity(c, nb, K);
    if (rc) return rc;
    hipError_t e = hipSuccess;
    if (valid) {
        e = hipMemcpyAsync(K.sdf, c->Pl.sdf, valid * BRICK_VOX * 4, hipMemcpyDeviceToDevice, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(K.weight, c->Pl.weight, valid * BRICK_VOX * 4, hipMemcpyDeviceToDevice,
                               c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(K.brick_keys, c->T.brick_keys, valid * 8, hipMemcpyDeviceToDevice,
                               c->stream);
    }
    if (e == hipSuccess) e = launch_fill(K.sdf + valid * BRICK_VOX, c->R.bg, (nb - valid) * BRICK_VOX, c->stream);
    if (e == hipSuccess)
        e = hipMemsetAsync(K.weight + valid * BRICK_VOX, 0, (nb - valid) * BRICK_VOX * 4, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the old pool is read before the free
    if (e != hipSuccess) {
        K.free_all();
        return fail(c, TSDF_EHIP, "grow: %s", hipGetErrorString(e));
    }
    install_capacity(c, K);
    HIPCHK(c, launch_rehash(c->T, (uint32_t)valid, c->G, c->stream));
    // the failed batches' counters and flags go; the pool keeps its valid bricks
    const uint32_t pcv = (uint32_t)valid;
    HIPCHK(c, hipMemsetAsync(c->G, 0, offsetof(Globals, tot_vox), c->stream));
    HIPCHK(c, hipMemcpyAsync(&c->G->pool_count, &pcv, 4, hipMemcpyHostToDevice, c->stream));
    const uint32_t retry = 1u;
    HIPCHK(c, hipMemcpyAsync(&c->G->retry, &retry, 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->n_grows++;
    return TSDF_OK;
}

// Double the fallback-pair lists (OVF_FB) of both batch parities, up to the 26-bit index space.
static int grow_fb(tsdf_ctx* c) {
    const uint64_t nf = std::min<uint64_t>(2ull * c->Wk.max_fb, 1ull << 26);
    if (nf <= c->Wk.max_fb) return fail(c, TSDF_ENOMEM, "fallback pair list at its limit");
    uint4* f[2] = {nullptr, nullptr};
    hipError_t e = hipMalloc(&f[0], nf * sizeof(uint4));
    if (e == hipSuccess) e = hipMalloc(&f[1], nf * sizeof(uint4));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        for (auto q : f) if (q) (void)hipFree(q);
        return fail(c, TSDF_ENOMEM, "fallback pair list allocation failed");
    }
    for (int q = 0; q < 2; q++) {
        (void)hipFree(c->W2[q].fb);
        c->W2[q].fb = f[q];
        c->W2[q].max_fb = (uint32_t)nf;
    }
    c->Wk.max_fb = (uint32_t)nf;
    return TSDF_OK;
}

// Every launched batch complete: the context stream waits for them and drains.
static int drain_all(tsdf_ctx* c) {
    int rc = join(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TSDF_OK;
}

// With every batch complete: if a batch overflowed, grow the capacity it lacked and re-run the
// batches from it (their inputs are still valid), until a round succeeds.  Without growth (hard
// limit, or a non-growable overflow) the batches are re-run committing what fits, and tsdf_sync
// reports the overflow.
// Double both parities' sample lists (OVF_SMP), up to the 32-bit sample index (single walk: the
// workgroup regions, up to the span record's 30-bit sample position).
static uint64_t smp_limit(const tsdf_ctx* c) { return c->fused ? (1ull << 30) : 0xFFFFFFF0ull; }
static int grow_smp(tsdf_ctx* c) {
    const uint64_t ns = std::min<uint64_t>(2ull * c->Wk.max_smp, smp_limit(c));
    if (ns <= c->Wk.max_smp) return fail(c, TSDF_ENOMEM, "sample list at its limit");
    uint2* f[2] = {nullptr, nullptr};
    hipError_t e = hipMalloc(&f[0], ns * smp_bytes(c->R.sem));
    if (e == hipSuccess) e = hipMalloc(&f[1], ns * smp_bytes(c->R.sem));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        for (auto q : f) if (q) (void)hipFree(q);
        return fail(c, TSDF_ENOMEM, "sample list allocation failed");
    }
    for (int q = 0; q < 2; q++) {
        (void)hipFree(c->W2[q].smp);
        c->W2[q].smp = f[q];
        c->W2[q].max_smp = (uint32_t)ns;
    }
    c->Wk.max_smp = (uint32_t)ns;
    c->n_grows++;
    return TSDF_OK;
}

// Double both parities' span lists (OVF_SPN, single walk).
static int grow_spn(tsdf_ctx* c) {
    const uint64_t ns = std::min<uint64_t>(2ull * c->Wk.max_spn, 0xFFFFFFF0ull);
    if (ns <= c->Wk.max_spn) return fail(c, TSDF_ENOMEM, "span list at its limit");
    uint32_t* f[2] = {nullptr, nullptr};
    hipError_t e = hipMalloc(&f[0], ns * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&f[1], ns * sizeof(uint32_t));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        for (auto q : f) if (q) (void)hipFree(q);
        return fail(c, TSDF_ENOMEM, "span list allocation failed");
    }
    for (int q = 0; q < 2; q++) {
        (void)hipFree(c->W2[q].spn);
        c->W2[q].spn = f[q];
        c->W2[q].max_spn = (uint32_t)ns;
    }
    c->Wk.max_spn = (uint32_t)ns;
    c->n_grows++;
    return TSDF_OK;
}

static int check_and_replay(tsdf_ctx* c) {
    for (int round = 0; round < 64; round++) {
        struct { uint32_t pool_count, overflow, failed, retry, fail_id; } g;
        HIPCHK(c, hipMemcpy(&g, c->G, sizeof g, hipMemcpyDeviceToHost));
        if (!g.failed) {
            c->log.clear();
            return TSDF_OK;
        }
        if (!c->can_grow) {  // committed anyway (G->retry = 0): the overflow stays for tsdf_sync
            const uint32_t z[2] = {0u, 0u};
            HIPCHK(c, hipMemcpy(&c->G->failed, z, 4, hipMemcpyHostToDevice));
            c->log.clear();
            return TSDF_OK;
        }
        int rc = TSDF_ENOMEM;
        // pair slots per ray are a geometric bound, and a merged bucket's distinct keys exceed its
        // LDS table only for scans of more than ~2^22 points: not capacities to grow
        if (!(g.overflow & (OVF_PAIRS | OVF_MG))) {
            rc = TSDF_OK;
            if (g.overflow & (OVF_TABLE | OVF_POOL | OVF_ACTIVE))
                rc = grow_capacity(c, std::max<uint64_t>(g.pool_count, c->T.max_bricks + 1));
            if (rc == TSDF_OK && (g.overflow & OVF_FB)) rc = grow_fb(c);
            if (rc == TSDF_OK && (g.overflow & OVF_SMP)) rc = grow_smp(c);
            if (rc == TSDF_OK && (g.overflow & OVF_SPN)) rc = grow_spn(c);
            if (rc == TSDF_EHIP) return rc;
        }
        // the replay: from the first failed batch on, in order
        size_t first = 0;
        while (first < c->log.size() && (uint32_t)c->log[first].id != g.fail_id) first++;
        if (first == c->log.size()) first = 0;
        std::vector<tsdf_ctx::Logged> rep(c->log.begin() + first, c->log.end());
        c->log.clear();
        if (rc != TSDF_OK) {  // cannot grow: commit what fits from now on
            c->can_grow = false;
            const uint32_t z[2] = {0u, 0u};  // failed, retry
            HIPCHK(c, hipMemcpy(&c->G->failed, z, 8, hipMemcpyHostToDevice));
        } else {  // grown: the replay re-raises whatever still does not fit
            const uint32_t z[2] = {0u, 0u};  // overflow, failed
            HIPCHK(c, hipMemcpy(&c->G->overflow, z, 8, hipMemcpyHostToDevice));
        }
        c->in_replay = true;
        for (auto& L : rep) {
            c->n_scans -= L.D.n_scans;
            c->n_batches--;
            c->n_replayed++;
            rc = launch(c, L.xyz, L.D);
            if (rc) break;
        }
        c->in_replay = false;
        if (rc) return rc;
        rc = drain_all(c);
        if (rc) return rc;
    }
    return fail(c, TSDF_ENOMEM, "capacity growth did not converge");
}

// Metrics log: one JSON line per finished batch, from the device ring of batch records (k_finish)
// and the host's facts (points) and kernel times (profiling on).  Called with every batch done.
static int emit_metrics(tsdf_ctx* c) {
    if (!c->metrics) return TSDF_OK;
    if (c->timer) c->timer->harvest();
    const uint64_t end = c->batch_id;
    if (end == c->metrics_next) return TSDF_OK;
    std::vector<BatchRecord> ring(METRIC_RING);
    HIPCHK(c, hipMemcpy(ring.data(), c->G->ring, sizeof(BatchRecord) * METRIC_RING,
                        hipMemcpyDeviceToHost));
    size_t ti = 0;
    for (uint64_t b = std::max<uint64_t>(c->metrics_next, end > METRIC_RING ? end - METRIC_RING : 0);
         b < end; b++) {
        const BatchRecord& r = ring[b % METRIC_RING];
        if (r.batch_id != (uint32_t)b) continue;  // not written (ring wrapped)
        uint32_t scans = 0;
        uint64_t points = 0;
        for (auto& i : c->metrics_info)
            if (i.id == b) { scans = i.scans; points = i.points; }
        const double bytes = 12.0 * (double)r.rays + 16.0 * (double)r.vox;  // SURVEY §8d B_scan
        fprintf(c->metrics,
                "{\"batch\": %llu, \"scans\": %u, \"points\": %llu, \"rays\": %llu, \"pairs\": %llu, "
                "\"voxel_updates\": %llu, \"dirty_voxels\": %llu, \"active_bricks\": %u, "
                "\"new_bricks\": %u, \"bricks\": %u, \"overflow\": %u, \"committed\": %s, "
                "\"algorithmic_bytes\": %.0f",
                (unsigned long long)b, scans, (unsigned long long)points,
                (unsigned long long)r.rays, (unsigned long long)r.pairs, (unsigned long long)r.vox,
                (unsigned long long)r.dirty, r.n_active, r.n_new,
                std::min<uint32_t>(r.pool_count, c->T.max_bricks), r.ovf,
                r.committed ? "true" : "false", bytes);
        const std::array<double, KIND_N>* ms = nullptr;
        if (c->timer) {
            auto& bm = c->timer->batch_ms;
            while (ti < bm.size() && bm[ti].first < b) ti++;
            if (ti < bm.size() && bm[ti].first == b) ms = &bm[ti].second;
        }
        if (ms) {
            double path = 0;
            for (int k = 0; k < KIND_N; k++) path += (*ms)[k];
            if (c->fused)
                fprintf(c->metrics,
                        ", \"kernel_ms\": {\"walk\": %.5f, \"compact\": %.5f, \"spans\": %.5f, "
                        "\"integrate\": %.5f}",
                        (*ms)[KIND_WALK], (*ms)[KIND_COMPACT], (*ms)[KIND_SPANS], (*ms)[KIND_INTEGRATE]);
            else
                fprintf(c->metrics,
                        ", \"kernel_ms\": {\"count\": %.5f, \"compact\": %.5f, \"place\": %.5f, "
                        "\"integrate\": %.5f}",
                        (*ms)[KIND_COUNT], (*ms)[KIND_COMPACT], (*ms)[KIND_PLACE], (*ms)[KIND_INTEGRATE]);
            fprintf(c->metrics, ", \"path_ms\": %.5f, \"gbs\": %.2f", path,
                    path > 0 ? bytes / (path * 1e-3) / 1e9 : 0.0);
        }
        fprintf(c->metrics, "}\n");
    }
    fflush(c->metrics);
    c->metrics_next = end;
    c->metrics_info.clear();
    if (c->timer) c->timer->batch_ms.clear();
    return TSDF_OK;
}

// Marching-cubes case table, generated (the same construction as the oracle's
// mc_build): per cube face the sign-change edges are paired into segments (ambiguous faces pair the
// crossings around their inside corners, so neighbouring cubes agree), each directed with the
// face's inside corners (S < 0) on its right seen from outside; the segments chain into cycles,
// fanned into triangles.  Corner c = (c & 1, c >> 1 & 1, c >> 2 & 1); edges axis-major.
struct McTable {
    uint8_t tab[256][32];  // [case][0] = triangles, then 3 edge ids each
    uint8_t edge[12][2];   // edge -> (a, b), b = a | axis bit
};

// lorensen: the classic table's ambiguity rule instead (Lorensen & Cline's complement symmetry;
// TSDF_MC_LORENSEN_RULE, a restatement of the published table's topology): an ambiguous face pairs its crossings
// around the inside corners when at most 4 corners of the cube are inside, around the outside
// corners otherwise; the two cubes sharing a face can then disagree (the classic cracks).
static McTable build_mc_table(bool lorensen) {
    McTable M{};
    int ne = 0;
    for (int d = 0; d < 3; d++)
        for (int base = 0; base < 8; base++)
            if (!(base & (1 << d))) {
                M.edge[ne][0] = (uint8_t)base;
                M.edge[ne][1] = (uint8_t)(base | (1 << d));
                ne++;
            }
    auto edge_of = [&](int a, int b) {
        for (int e = 0; e < 12; e++)
            if ((M.edge[e][0] == a && M.edge[e][1] == b) || (M.edge[e][0] == b && M.edge[e][1] == a))
                return e;
        return -1;
    };
    for (int k = 0; k < 256; k++) {
        int next[12];
        std::fill(next, next + 12, -1);
        for (int d = 0; d < 3; d++) {
            const int u = (d + 1) % 3, w = (d + 2) % 3;
            for (int side = 0; side < 2; side++) {
                // face corners counter-clockwise seen from outside (outward normal (2 side - 1) e_d)
                const int ou[4] = {0, 1, 1, 0}, ow[4] = {0, 0, 1, 1};
                int q[4], in[4];
                for (int i = 0; i < 4; i++) {
                    const int cu = side ? ou[i] : ow[i], cw = side ? ow[i] : ou[i];
                    q[i] = (side << d) | (cu << u) | (cw << w);
                    in[i] = (k >> q[i]) & 1;
                }
                int cr[4], ncr = 0;
                for (int i = 0; i < 4; i++)
                    if (in[i] != in[(i + 1) & 3]) cr[ncr++] = i;
                std::vector<std::pair<int, int>> pairs;
                if (ncr == 2) pairs.push_back({cr[0], cr[1]});
                if (ncr == 4) {
                    // around the inside corners (generated; Lorensen with <= 4 inside corners), else
                    // around the outside ones
                    const bool around_in = !lorensen || __builtin_popcount((unsigned)k) <= 4;
                    if (in[0] == (around_in ? 1 : 0)) pairs = {{3, 0}, {1, 2}};
                    else pairs = {{0, 1}, {2, 3}};
                }
                for (auto [i, j] : pairs) {
                    const int ei = edge_of(q[i], q[(i + 1) & 3]), ej = edge_of(q[j], q[(j + 1) & 3]);
                    // the corners q[i+1 .. j] are on the right of the segment i -> j
                    if (in[(i + 1) & 3]) next[ei] = ej;
                    else next[ej] = ei;
                }
            }
        }
        bool used[12] = {};
        int nt = 0;
        for (int e0 = 0; e0 < 12; e0++) {
            if (next[e0] < 0 || used[e0]) continue;
            int poly[12], n = 0;
            for (int e = e0; !used[e] && n < 12; e = next[e]) {
                used[e] = true;
                poly[n++] = e;
            }
            for (int m = 1; m + 1 < n; m++) {
                M.tab[k][1 + 3 * nt] = (uint8_t)poly[0];
                M.tab[k][2 + 3 * nt] = (uint8_t)poly[m];
                M.tab[k][3 + 3 * nt] = (uint8_t)poly[m + 1];
                nt++;
            }
        }
        M.tab[k][0] = (uint8_t)nt;
    }
    return M;
}

// TSDF_MC_LORENSEN: the published table (include/tsdf_mc_tables.h, VDBFusion's), renumbered into
// this library's corners and edges: Bourke vertex v -> corner kV[v], edge e -> edge kE[e]; the
// triangles keep their order and winding.
static McTable literal_mc_table() {
    McTable M = build_mc_table(false);  // the edge list
    static const int kV[8] = {0, 1, 3, 2, 4, 5, 7, 6};
    static const int kE[12] = {0, 5, 1, 4, 2, 7, 3, 6, 8, 9, 11, 10};
    for (int b = 0; b < 256; b++) {
        int k = 0;
        for (int v = 0; v < 8; v++)
            if (b >> v & 1) k |= 1 << kV[v];
        int nt = 0;
        for (int i = 0; i < 15 && tsdf_mc_tri_table[b][i] >= 0; i += 3, nt++)
            for (int j = 0; j < 3; j++) M.tab[k][1 + 3 * nt + j] = (uint8_t)kE[tsdf_mc_tri_table[b][i + j]];
        M.tab[k][0] = (uint8_t)nt;
    }
    return M;
}

static const McTable& mc_table(int which = TSDF_MC_GENERATED) {
    static const McTable G = build_mc_table(false), L = literal_mc_table(), R = build_mc_table(true);
    return which == TSDF_MC_LORENSEN ? L : which == TSDF_MC_LORENSEN_RULE ? R : G;
}

extern "C" {

void tsdf_default_params(tsdf_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->voxel_size = 0.05;
    p->sdf_trunc = 0.15;
    p->space_carving = 0;
    p->weight_mode = TSDF_WEIGHT_CONSTANT;
    p->min_range = 0.0;
    p->max_range = INFINITY;
    p->max_bricks = 1u << 20;
    p->max_points = 1u << 18;
    p->max_pairs = 0;
    p->device_id = 0;
    p->brick_side = TSDF_BRICK_SIDE;
    p->max_batch = 32;
    p->semantics = TSDF_SEM_VDBFUSION_F64;  // ABI v8: the mode matching VDBFusion exactly
    p->voxblox_method = TSDF_VB_SIMPLE;
    p->sector_input = TSDF_SECTOR_INPUT_FANOUT;
    p->sector_rule = TSDF_SECTOR_RULE_INDEX;  // ABI v10: SURVEY §8e's contiguous column sectors
    p->allow_clear = 1;  // voxblox TsdfIntegratorBase::Config defaults
    p->use_weight_dropoff = 1;
    p->max_weight = 10000.0f;
    p->depth_weight = 1;  // voxblox use_const_weight = false (upstream's default)
}

int tsdf_abi_version(void) { return TSDF_ABI_VERSION; }

const char* tsdf_last_error(const tsdf_ctx* c) { return c ? c->err.c_str() : "null context"; }

void tsdf_destroy(tsdf_ctx* c) {
    if (!c) return;
    // fan-out links (tsdf_integrate_sectors): a leader hands its followers their pending points
    // before its staging goes; a follower leaves its leader's list
    for (tsdf_ctx* f : c->fan_followers) {
        (void)fan_copy(f);
        f->fan_src = nullptr;
        f->fan_buf = nullptr;
    }
    c->fan_followers.clear();
    if (c->fan_src) {
        auto& v = c->fan_src->fan_followers;
        v.erase(std::remove(v.begin(), v.end(), c), v.end());
    }
    if (c->device >= 0) {
        (void)hipSetDevice(c->device);
        if (c->stream) {
            (void)settle(c);
            (void)hipStreamSynchronize(c->stream);
            for (int q = 0; q < 2; q++)
                if (c->bst[q]) (void)hipStreamSynchronize(c->bst[q]);
        }
    }
    if (c->metrics) fclose(c->metrics);
    if (c->brd_sent) (void)hipFree(c->brd_sent);
    for (auto& b : c->brd_backup) (void)hipFree(b.first);
    delete c->timer;
    delete c->pack;
    void* dev[] = {c->T.keys,        c->T.slots,
                   c->T.touched,
                   c->T.brick_keys,  c->Pl.sdf,          c->Pl.weight,     c->G,
                   c->cell2[0],      c->cell2[1],        c->stage2[0],     c->stage2[1],
                   c->W2[0].pair,    c->W2[0].blk,       c->W2[0].blk_n, c->W2[0].fb,
                   c->W2[0].smp,     c->W2[0].active,  c->W2[0].active_ord, c->W2[1].active_ord,
                   c->W2[0].ord_hist, c->W2[1].ord_hist,    c->W2[1].pair,    c->W2[1].blk,
                   c->W2[1].blk_n, c->W2[1].fb,        c->W2[1].smp,     c->W2[1].active,
                   c->W2[0].cagg,    c->W2[1].cagg,      c->W2[0].act,     c->W2[1].act,
                   c->W2[0].spn,     c->W2[1].spn,
                   c->W2[0].plan,    c->W2[1].plan,      c->W2[0].rsv,     c->W2[1].rsv,
                   c->W2[0].rsv_n,   c->W2[1].rsv_n};
    for (void* d : dev)
        if (d) (void)hipFree(d);
    for (int i = 0; i < 2; i++) {
        if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
        if (c->stage_done[i]) (void)hipEventDestroy(c->stage_done[i]);
        MgBufs& M = c->mg[i];
        for (void* q : {(void*)M.xyz_out, (void*)M.w_out, (void*)M.ekey, (void*)M.eidx,
                        (void*)M.bcnt, (void*)M.bst, (void*)M.bscan})
            if (q) (void)hipFree(q);
    }
    if (c->bc_ev) (void)hipEventDestroy(c->bc_ev);
    for (int q = 0; q < 2; q++) {
        if (c->bst[q]) (void)hipStreamDestroy(c->bst[q]);
        if (c->ev_compact[q]) (void)hipEventDestroy(c->ev_compact[q]);
        if (c->stage_ev[q]) (void)hipEventDestroy(c->stage_ev[q]);
    }
    if (c->ev_main) (void)hipEventDestroy(c->ev_main);
    for (int k = 0; k < tsdf_ctx::RING; k++)
        if (c->ring_ev[k]) (void)hipEventDestroy(c->ring_ev[k]);
    if (c->h_ring) (void)hipHostFree(c->h_ring);
    if (c->h_ring_done) (void)hipHostFree(c->h_ring_done);
    if (c->d_ring) (void)hipFree(c->d_ring);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static int create_impl(tsdf_ctx* c, const tsdf_params* p) {
    c->p = *p;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(c, TSDF_ENODEV, "no HIP device available");
    if (p->device_id < 0 || p->device_id >= ndev)
        return fail(c, TSDF_EINVAL, "device_id %d out of range (%d devices)", p->device_id, ndev);
    c->device = p->device_id;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int q = 0; q < 2; q++) {
        HIPCHK(c, hipStreamCreateWithFlags(&c->bst[q], hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_compact[q], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->stage_ev[q], hipEventDisableTiming));
    }
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming));

    c->R.vs = (float)p->voxel_size;
    c->R.inv_vs = 1.0f / c->R.vs;
    c->R.tau = (float)p->sdf_trunc;
    c->R.min_range = (float)p->min_range;
    c->R.max_range = (float)p->max_range;
    c->R.carving = p->space_carving ? 1 : 0;
    c->R.tau2_lo = (float)(((double)c->R.tau * (1.0 - 0x1p-20)) * ((double)c->R.tau * (1.0 - 0x1p-20)));
    c->R.tau2_hi = (float)(((double)c->R.tau * (1.0 + 0x1p-20)) * ((double)c->R.tau * (1.0 + 0x1p-20)));
    // internal sem 3: Voxblox with the 1/z^2 weight (per-sample weights stored by k_place)
    c->R.depth_w = p->semantics == TSDF_SEM_VOXBLOX && p->depth_weight ? 1 : 0;
    // MergedTsdfIntegrator: bundles carry summed weights, so per-sample weights too (sem 3)
    c->merged = p->semantics == TSDF_SEM_VOXBLOX && p->voxblox_method == TSDF_VB_MERGED;
    c->R.sem = c->R.depth_w || c->merged ? 3 : p->semantics;
    c->R.ray_w = nullptr;  // set per launch to the pre-pass output (merged)
    c->R.allow_clear = p->allow_clear ? 1 : 0;
    c->R.dropoff = p->use_weight_dropoff ? 1 : 0;
    c->R.max_weight = p->max_weight;
    c->R.w0_cap = p->max_weight > 0.0f && p->max_weight < TSDF_W0_CAP ? p->max_weight : TSDF_W0_CAP;
    c->R.bg = p->semantics == TSDF_SEM_VOXBLOX ? 0.0f : c->R.tau;
    c->R.tau_m_vs = c->R.tau - c->R.vs;
    c->idx_rule = p->n_sectors > 1 && p->sector_rule == TSDF_SECTOR_RULE_INDEX;
    if (c->idx_rule) c->R.sec_on = 0;
    else sector_bounds(p->sector_yaw0, p->sector, p->n_sectors, c->R);
    const double vs_d = (double)c->R.vs;  // VDBVolume keeps voxel_size as float
    c->R.hvs_d = vs_d * 0.5;               // exact
    c->R.inv_s_d = 1.0 / vs_d;
    c->R.gate_d2 = gate_threshold(c->R.tau);
    {
        const double band = p->space_carving ? (p->max_range + p->sdf_trunc) / p->voxel_size
                                             : 2.0 * p->sdf_trunc / p->voxel_size;
        c->R.band_vox = (int)std::min(std::ceil(band) + 4.0, (double)(VOX_LIMIT / 2));
    }

    // Points one batch may hold: max_batch full scans, unless the per-ray worst cases (pair slots,
    // sample slots — large with space carving) exceed the u32 index space or the sample budget;
    // the host queue then cuts batches by points.  A single scan must always fit.
    const uint32_t maxp = pairs_per_ray(*p);
    const uint32_t spr = samples_per_ray(*p);
    // sample list: the worst case (spr per ray) of the rays a context keeps — 1 / n_sectors of them
    // when sharded — capped at 2^30 samples (8 GiB); an overflow grows it (OVF_SMP)
    const uint64_t smp_budget = 1ull << 30;
    c->max_batch = p->max_batch;
    uint64_t bp = p->max_points * c->max_batch;
    bp = std::min<uint64_t>(bp, 0xFFFFFFF0ull / maxp);
    if (p->max_pairs) bp = std::min<uint64_t>(bp, p->max_pairs / maxp);  // caller-imposed cap
    if (bp < p->max_points)
        return fail(c, TSDF_EINVAL,
                    "max_points %llu exceeds what one batch can hold (%llu: %u pair and %u sample "
                    "slots per ray)", (unsigned long long)p->max_points, (unsigned long long)bp,
                    maxp, spr);
    // Single walk: k_walk keeps a ray's samples in one register slot per DDA step, so
    // the band's walk must have a proven bound: a segment of L voxels crosses at most floor(L |u_a|)
    // + 1 boundaries per axis, i.e. visits <= sqrt(3) L + 4 voxels.  Carving and Voxblox clearing
    // rays (length up to max_range) keep the two-walk path, the default (tsdf_params.walk).
    {
        const double band = 2.0 * p->sdf_trunc / p->voxel_size;
        const double steps = std::floor(std::sqrt(3.0) * band * (1.0 + 1e-4)) + 5.0;
        const bool clearing = p->semantics == TSDF_SEM_VOXBLOX && p->allow_clear &&
                              std::isfinite(p->max_range);
        c->fused = p->walk == TSDF_WALK_SINGLE && !p->space_carving && !clearing && maxp <= 4 &&
                   c->R.sem != 3 &&
                   steps <= 32.0;
        c->nstep = steps <= 16.0 ? 16 : 32;
    }
    const uint64_t stg = (uint64_t)WLK_THREADS * (uint64_t)c->nstep;  // samples per k_walk region
    if (c->fused) {
        // the span record addresses 2^30 samples: at most 2^30 / stg k_walk workgroups per batch
        const uint64_t lim = ((1ull << 30) / (2 * stg) - MAX_BATCH - 1) * RPB;
        bp = std::min<uint64_t>(bp, lim);
        if (bp < p->max_points)
            return fail(c, TSDF_EINVAL, "max_points %llu exceeds a single-walk batch (%llu)",
                        (unsigned long long)p->max_points, (unsigned long long)bp);
    }
    c->max_points = p->max_points;
    c->batch_points = bp;
    const uint64_t slots = bp * maxp;
    c->slots = slots;
    c->max_blocks = (uint32_t)(c->batch_points / RPB + MAX_BATCH + 1);
    const uint32_t nsec = std::max<uint32_t>(1u, p->n_sectors);
    if (c->fused) {
        // 64-bit cells and a totals cell after the last scan; the pair and fallback lists are not
        // used; one region of stg samples per k_walk workgroup (sharded: this GPU's share of the
        // blocks, grown on OVF_SMP); span records ~ samples / SPAN + one partial span per run
        c->T.cell_stride = (c->max_batch + 2u) & ~1u;
        c->Wk.maxp = maxp;
        const uint64_t reg_blocks = nsec > 1 ? std::min<uint64_t>(
            c->max_blocks, c->max_blocks * 5ull / (4ull * nsec) + 2ull * c->max_batch + 64) : c->max_blocks;
        c->Wk.max_smp = (uint32_t)std::min<uint64_t>(2 * reg_blocks * stg, 1ull << 30);
        c->Wk.max_spn = (uint32_t)std::min<uint64_t>(
            bp * spr / SPAN / nsec + 2 * reg_blocks * 256, 0xFFFFFFF0ull);
        c->Wk.max_fb = 4;
    } else {
        c->T.cell_stride = (c->max_batch + 3u) & ~3u;
        c->Wk.maxp = maxp;
        c->Wk.max_smp = (uint32_t)std::min<uint64_t>(
            std::min<uint64_t>(bp * spr / nsec, smp_budget), 0xFFFFFFF0ull);
        // fallback pairs (a workgroup's LDS brick hash is full): rare without carving, the rule with
        // it (the fallback index has 26 bits; past it pairs are dropped and OVF_FB reported)
        c->Wk.max_fb = (uint32_t)std::min<uint64_t>(
            p->space_carving ? slots : std::max<uint64_t>(slots / 16, 1u << 20), 1u << 26);
        c->Wk.max_spn = 4;
    }

    for (int q = 0; q < 2; q++) {  // one set per batch parity (capacity-independent part)
        Work& W = c->W2[q];
        W = c->Wk;
        HIPCHK(c, hipMalloc(&W.pair, (c->fused ? 4 : slots) * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc(&W.blk, (size_t)c->max_blocks * 2 * HCAP * sizeof(uint4)));
        HIPCHK(c, hipMalloc(&W.blk_n, (size_t)c->max_blocks * 2 * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc(&W.plan, (size_t)c->max_blocks * 2 * PLAN_STRIDE * sizeof(uint32_t)));
#ifdef TSDF_CNT_SPLIT
        HIPCHK(c, hipMalloc(&W.rsv, (size_t)c->max_blocks * HCAP * sizeof(uint4)));
        HIPCHK(c, hipMalloc(&W.rsv_n, (size_t)c->max_blocks * sizeof(uint32_t)));
#endif
        HIPCHK(c, hipMalloc(&W.fb, (size_t)W.max_fb * sizeof(uint4)));
        HIPCHK(c, hipMalloc(&W.smp, (size_t)W.max_smp * smp_bytes(c->R.sem)));
        HIPCHK(c, hipMalloc(&W.spn, (size_t)W.max_spn * sizeof(uint32_t)));
        // (slice, size class) histogram, then first positions (k_compact; zero between batches)
        HIPCHK(c, hipMalloc(&W.ord_hist, 2 * 64 * 32 * sizeof(uint32_t)));
        HIPCHK(c, hipMemset(W.ord_hist, 0, 2 * 64 * 32 * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc(&W.act, (size_t)c->max_blocks * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc(&c->stage2[q], c->batch_points * 3 * sizeof(float)));
        if (c->merged) {  // the bundling pre-pass: one set per parity, batch_points entries
            MgBufs& M = c->mg[q];
            const uint64_t n = c->batch_points;
            M.cap = n;
            M.nb_cap = mg_buckets_max(n);
            HIPCHK(c, hipMalloc(&M.ekey, n * 8));
            HIPCHK(c, hipMalloc(&M.eidx, n * 4));
            HIPCHK(c, hipMalloc(&M.bcnt, (size_t)4 * MG_REPLICAS * M.nb_cap));
            HIPCHK(c, hipMemset(M.bcnt, 0, (size_t)4 * MG_REPLICAS * M.nb_cap));  // zero between batches
            HIPCHK(c, hipMalloc(&M.bst, (size_t)4 * (M.nb_cap + 1)));
            HIPCHK(c, hipMalloc(&M.bscan, (size_t)4 * M.nb_cap));
            HIPCHK(c, hipMalloc(&M.xyz_out, n * 12));
            HIPCHK(c, hipMalloc(&M.w_out, n * 4));
        }
    }
    HIPCHK(c, hipMalloc(&c->G, sizeof(Globals)));
    if (const char* e = std::getenv("TSDF_SMALL_NS")) c->small_ns = std::max(0, std::min(8, std::atoi(e)));
    if (const char* e = std::getenv("TSDF_COUNT_WIDE")) c->count_wide = (uint32_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("TSDF_COUNT_PAIRED")) c->count_paired = std::atoi(e) != 0;
    {
        // host staging threads: 3 workers + the caller (TSDF_PACK_THREADS overrides; 1 = none)
        int nt = 4;
        if (const char* e = std::getenv("TSDF_PACK_THREADS")) nt = std::max(1, std::atoi(e));
        nt = std::min<int>(nt, (int)std::max(1u, std::thread::hardware_concurrency()));
        if (nt > 1) {
            try {
                c->pack = new PackPool(nt - 1);
            } catch (...) {  // no threads: the caller's thread stages alone
                c->pack = nullptr;
            }
        }
    }
    HIPCHK(c, hipHostMalloc(&c->h_ring, tsdf_ctx::RING * (MAX_BATCH + 1) * sizeof(ScanRec),
                            hipHostMallocDefault));
    HIPCHK(c, hipMalloc(&c->d_ring, tsdf_ctx::RING * (MAX_BATCH + 1) * sizeof(ScanRec)));
    {
        void* dp = nullptr;
        HIPCHK(c, hipHostGetDevicePointer(&dp, c->h_ring, 0));
        c->d_ring_src = static_cast<const ScanRec*>(dp);
        HIPCHK(c, hipHostMalloc(&c->h_ring_done, 64, hipHostMallocDefault));
        *c->h_ring_done = 0;
        HIPCHK(c, hipHostGetDevicePointer(&dp, c->h_ring_done, 0));
        c->d_ring_done = static_cast<unsigned long long*>(dp);
    }
    for (int k = 0; k < tsdf_ctx::RING; k++)
        HIPCHK(c, hipEventCreateWithFlags(&c->ring_ev[k], hipEventDisableTiming));
    HIPCHK(c, hipMemsetAsync(c->G, 0, sizeof(Globals), c->stream));
    // the brick pool, hash table and per-brick work lists (grown later by grow_capacity)
    {
        Capacity K;
        const int rc = alloc_capacity(c, p->max_bricks, K);
        if (rc) return rc;
        HIPCHK(c, launch_fill(K.sdf, c->R.bg, p->max_bricks * BRICK_VOX, c->stream));
        HIPCHK(c, hipMemsetAsync(K.weight, 0, p->max_bricks * BRICK_VOX * sizeof(float), c->stream));
        install_capacity(c, K);
    }
    c->T.cell = c->cell2[0];
    for (int i = 0; i < 2; i++) {
        HIPCHK(c, hipHostMalloc(&c->h_stage[i], c->max_points * 3 * sizeof(float),
                                hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&c->stage_done[i], hipEventDisableTiming));
    }
    c->can_grow = p->max_bricks_hard == 0 || p->max_bricks_hard > p->max_bricks;
    {
        const uint32_t retry = c->can_grow ? 1u : 0u;
        HIPCHK(c, hipMemcpyAsync(&c->G->retry, &retry, 4, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    {
        static uint8_t all[TSDF_MC_TABLES][256][32];
        for (int t = 0; t < TSDF_MC_TABLES; t++) std::memcpy(all[t], mc_table(t).tab, sizeof all[t]);
        HIPCHK(c, upload_mc_table(all, mc_table().edge));
    }
    return TSDF_OK;
}

int tsdf_create(const tsdf_params* p, tsdf_ctx** out) {
    if (!p || !out) return TSDF_EINVAL;
    *out = nullptr;
    if (!(p->voxel_size > 0) || !(p->sdf_trunc > 0) || p->brick_side != TSDF_BRICK_SIDE ||
        p->weight_mode != TSDF_WEIGHT_CONSTANT || p->max_bricks == 0 ||
        p->max_bricks >= 0xFFFFFFF0ull || p->max_points == 0 || !(p->min_range >= 0) ||
        !(p->max_range > p->min_range) || p->max_batch == 0 || p->max_batch > TSDF_MAX_BATCH ||
        (p->semantics != TSDF_SEM_VDBFUSION && p->semantics != TSDF_SEM_VOXBLOX &&
         p->semantics != TSDF_SEM_VDBFUSION_F64) ||
        (p->semantics == TSDF_SEM_VOXBLOX && !(p->max_weight > 0.0f)) ||
        (p->voxblox_method != TSDF_VB_SIMPLE && p->voxblox_method != TSDF_VB_MERGED) ||
        p->sector_input < TSDF_SECTOR_INPUT_FANOUT || p->sector_input > TSDF_SECTOR_INPUT_SPLIT ||
        (p->sector_rule != TSDF_SECTOR_RULE_WORLD && p->sector_rule != TSDF_SECTOR_RULE_INDEX) ||
        (p->n_sectors > 1 && p->sector >= p->n_sectors) || !std::isfinite(p->sector_yaw0) ||
        (p->max_bricks_hard && p->max_bricks_hard < p->max_bricks))
        return TSDF_EINVAL;
    if (p->space_carving && !std::isfinite(p->max_range)) return TSDF_EINVAL;
    tsdf_ctx* c = new (std::nothrow) tsdf_ctx();
    if (!c) return TSDF_ENOMEM;
    const int rc = create_impl(c, p);
    if (rc != TSDF_OK) {
        fprintf(stderr, "tsdf_create: %s\n", c->err.c_str());
        tsdf_destroy(c);
        return rc;
    }
    *out = c;
    return TSDF_OK;
}

// A scan's ray origin and sensor z axis (the world frame's z axis unless a pose gives it)
struct ScanPose {
    double o[3];
    float z[3];
};

// An origin without an orientation: the zero axis tells the walk to use Voxblox's constant weight
// (the 1/z^2 weight needs the sensor axis, which only the pose entry points carry)
static ScanPose pose_of_origin(const double o[3]) {
    return ScanPose{{o[0], o[1], o[2]}, {0.0f, 0.0f, 0.0f}};
}

// pose = (x, y, z, qx, qy, qz, qw): the z axis is the third column of the rotation of the
// normalised quaternion, computed in double and rounded to float (the oracle does the same)
static ScanPose pose_of(const double q[7]) {
    ScanPose P = pose_of_origin(q);
    const double n = std::sqrt(q[3] * q[3] + q[4] * q[4] + q[5] * q[5] + q[6] * q[6]);
    const double x = q[3] / n, y = q[4] / n, z = q[5] / n, w = q[6] / n;
    P.z[0] = (float)(2.0 * (x * z + w * y));
    P.z[1] = (float)(2.0 * (y * z - w * x));
    P.z[2] = (float)(1.0 - 2.0 * (x * x + y * y));
    return P;
}

static void set_pose(BatchDesc& D, uint32_t s, const ScanPose& P) {
    D.s[s].ox = (float)P.o[0];
    D.s[s].oy = (float)P.o[1];
    D.s[s].oz = (float)P.o[2];
    D.s[s].odx = P.o[0];
    D.s[s].ody = P.o[1];
    D.s[s].odz = P.o[2];
    D.s[s].zx = P.z[0];
    D.s[s].zy = P.z[1];
    D.s[s].zz = P.z[2];
}

// The pending batch's device staging buffer (host and single device scans are queued there).  A
// new pending batch takes the buffer the last launched host batch did not use; that buffer's
// previous reader must be complete and, with growth possible, committed: an overflowed batch is
// re-run from its logged input, so that input stays until then.
static int pend_stage_buffer(tsdf_ctx* c) {
    if (c->pend.n_scans != 0) return TSDF_OK;
    const int k = c->last_stage ^ 1;
    for (tsdf_ctx* f : c->fan_followers)  // fan-out followers still reading buffer k copy first
        if (f->fan_buf == c->stage2[k] && f->fan_hi > f->fan_lo) {
            const int rc = fan_copy(f);
            if (rc) return rc;
        }
    if (c->stage_reader[k] != ~0ull) {
        if (c->can_grow) {
            HIPCHK(c, hipEventSynchronize(c->stage_ev[k]));
            uint32_t failed = 0;
            HIPCHK(c, hipMemcpy(&failed, &c->G->failed, 4, hipMemcpyDeviceToHost));
            if (failed) {  // replays re-read stage2[k]: it is written only after them
                int rc = drain_all(c);
                if (!rc) rc = check_and_replay(c);
                if (rc) return rc;
            } else {  // every batch up to stage2[k]'s reader committed
                const uint64_t done = c->stage_reader[k];
                size_t j = 0;
                while (j < c->log.size() && c->log[j].id <= done) j++;
                c->log.erase(c->log.begin(), c->log.begin() + j);
            }
        }
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->stage_ev[k], 0));
    }
    c->pend_stage = k;
    return TSDF_OK;
}

// Append a staged scan of n points seen from pose P to the pending batch; launch it when full.
static int pend_push(tsdf_ctx* c, uint64_t n, const ScanPose& P) {
    BatchDesc& D = c->pend;
    const uint32_t s = D.n_scans;
    set_pose(D, s, P);
    D.s[s].xoff = 0;  // staged scans are contiguous
    D.s[s + 1].off = D.s[s].off + (uint32_t)n;
    D.n_scans = s + 1;
    c->n_points_in += n;
    if (D.n_scans == c->max_batch) return flush(c);
    return TSDF_OK;
}

// Room for a scan of n points in the pending batch (flushing it first if needed).
static int pend_room(tsdf_ctx* c, uint64_t n) {
    if (c->pend.n_scans == c->max_batch || c->pend.s[c->pend.n_scans].off + n > c->batch_points)
        return flush(c);
    return TSDF_OK;
}

// TSDF_SECTOR_RULE_INDEX (ABI v10): sector k of N holds points
// [floor(k n / N), floor((k + 1) n / N)) of an n-point cloud -- contiguous column ranges of the
// spin for DLIO's time-sorted cloud (odom.cc:635-636).  The oracle's idx_share is the same.
static void idx_share(const tsdf_ctx* c, uint64_t n, uint64_t& lo, uint64_t& hi) {
    if (!c->idx_rule) {
        lo = 0;
        hi = n;
        return;
    }
    const unsigned __int128 N = c->p.n_sectors, k = c->p.sector;
    lo = (uint64_t)((unsigned __int128)n * k / N);
    hi = (uint64_t)((unsigned __int128)n * (k + 1) / N);
}

static int integrate_impl(tsdf_ctx* c, const void* pts, uint64_t n, uint32_t point_step,
                          uint32_t xyz_offset, int32_t xyz_is_f64, const ScanPose& P) {
    if (border_busy(c)) return TSDF_EINVAL;
    const uint32_t need = xyz_is_f64 ? 24u : 12u;
    if (point_step < need || xyz_offset > point_step - need)
        return fail(c, TSDF_EINVAL, "point_step/xyz_offset inconsistent");
    {  // the context's share of the cloud (all of it unless index-sharded)
        uint64_t lo, hi;
        idx_share(c, n, lo, hi);
        if (pts) pts = static_cast<const char*>(pts) + lo * point_step;
        n = hi - lo;
    }
    if (n > c->max_points)
        return fail(c, TSDF_EINVAL, "scan of %llu points exceeds max_points %llu",
                    (unsigned long long)n, (unsigned long long)c->max_points);
    HIPCHK(c, hipSetDevice(c->device));
    {
        const int rc = pend_room(c, n);
        if (rc) return rc;
    }
    const int b = c->stage_cur;
    c->stage_cur ^= 1;
    HIPCHK(c, hipEventSynchronize(c->stage_done[b]));  // previous copy out of this buffer is done
    float* h = c->h_stage[b];
    const char* base = static_cast<const char*>(pts);
    if (!xyz_is_f64 && point_step == 12 && xyz_offset == 0) {
        std::memcpy(h, base, n * 12);
    } else {
        auto pack = [&](uint64_t i0, uint64_t i1) {
            for (uint64_t i = i0; i < i1; i++) {
                const char* q = base + i * point_step + xyz_offset;
                if (xyz_is_f64) {
                    double d[3];
                    std::memcpy(d, q, sizeof d);
                    h[3 * i] = (float)d[0];
                    h[3 * i + 1] = (float)d[1];
                    h[3 * i + 2] = (float)d[2];
                } else {
                    std::memcpy(h + 3 * i, q, 12);
                }
            }
        };
        if (c->pack && n >= (1u << 15)) {
            const uint64_t parts = (uint64_t)c->pack->parts();
            c->pack->run([&](int k) { pack(n * k / parts, n * (k + 1) / parts); });
        } else {
            pack(0, n);
        }
    }
    int rc = pend_stage_buffer(c);
    if (rc) return rc;
    if (n) {
        HIPCHK(c, hipMemcpyAsync(c->stage2[c->pend_stage] + 3 * (uint64_t)c->pend.s[c->pend.n_scans].off,
                                 h, n * 12, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->stage_done[b], c->stream));
    return pend_push(c, n, P);
}

int tsdf_integrate(tsdf_ctx* c, const void* pts, uint64_t n, uint32_t point_step,
                   uint32_t xyz_offset, int32_t xyz_is_f64, const double origin[3]) {
    if (!c) return TSDF_EINVAL;
    if ((!pts && n) || !origin) return fail(c, TSDF_EINVAL, "null argument");
    return integrate_impl(c, pts, n, point_step, xyz_offset, xyz_is_f64, pose_of_origin(origin));
}

}  // extern "C"

// tsdf_integrate_sectors without a host split (tsdf_params.sector_input FANOUT / H2D): the cloud
// is packed ONCE into ctxs[0]'s pinned buffer h[0] (on every context's staging threads), and every
// context receives all of it -- its kernels drop the other sectors' rays (R.sec_on), so the fields
// are those of the split, bit for bit.
//   FANOUT: one H2D copy into ctxs[0]'s staging (the leader); the other contexts (followers) take
//           the scan into their pending batch and copy the batch's points from the leader's staging
//           in ONE device-to-device copy before they launch it (fan_copy: hipMemcpyPeerAsync, xGMI
//           with peer access, tsdf_create_sharded) -- O(1) API calls per follower per scan.
//   H2D:    every context copies h[0] over its own PCIe link; ctxs[0]'s stream waits for them all
//           before it records h[0]'s reuse event.
static int sectors_broadcast(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts, uint64_t n,
                             uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64,
                             const ScanPose& P, float* const* h, const int* hb, bool fanout) {
    tsdf_ctx* c0 = ctxs[0];
    float* hx = h[0];
    const char* base = static_cast<const char*>(pts);
    auto pack = [&](uint64_t i0, uint64_t i1) {
        if (!xyz_is_f64 && point_step == 12 && xyz_offset == 0) {
            std::memcpy(hx + 3 * i0, base + 12 * i0, (i1 - i0) * 12);
            return;
        }
        for (uint64_t i = i0; i < i1; i++) {
            const char* q = base + i * point_step + xyz_offset;
            if (xyz_is_f64) {
                double d[3];
                std::memcpy(d, q, sizeof d);
                hx[3 * i] = (float)d[0];
                hx[3 * i + 1] = (float)d[1];
                hx[3 * i + 2] = (float)d[2];
            } else {
                std::memcpy(hx + 3 * i, q, 12);
            }
        }
    };
    // every context's staging threads pack a share of the points
    int pbase[TSDF_MAX_WORLD + 1];
    pbase[0] = 0;
    for (uint32_t k = 0; k < n_ctx; k++)
        pbase[k + 1] = pbase[k] + (ctxs[k]->pack ? ctxs[k]->pack->parts() - (k ? 1 : 0) : (k ? 0 : 1));
    const int parts = n >= (1u << 15) ? pbase[n_ctx] : 1;
    auto part = [&](int q) { pack(n * (uint64_t)q / parts, n * (uint64_t)(q + 1) / parts); };
    if (parts == 1) {
        part(0);
    } else {
        for (uint32_t k = 1; k < n_ctx; k++)
            if (ctxs[k]->pack) ctxs[k]->pack->start(part, pbase[k] - 1);
        if (c0->pack) c0->pack->run(part);
        else part(0);
        for (uint32_t k = 1; k < n_ctx; k++)
            if (ctxs[k]->pack) ctxs[k]->pack->wait();
    }
    c0->split_ht.lap(1);  // TSDF_HOST_TIMING: 0 prep, 1 pack, 2 copies + queue
    // the leader's H2D copy first
    HIPCHK(c0, hipSetDevice(c0->device));
    int rc = pend_stage_buffer(c0);
    if (rc) return rc;
    const uint64_t off0 = c0->pend.s[c0->pend.n_scans].off;
    float* buf0 = c0->stage2[c0->pend_stage];
    if (n) HIPCHK(c0, hipMemcpyAsync(buf0 + 3 * off0, hx, n * 12, hipMemcpyHostToDevice, c0->stream));
    if (!c0->bc_ev) HIPCHK(c0, hipEventCreateWithFlags(&c0->bc_ev, hipEventDisableTiming));
    HIPCHK(c0, hipEventRecord(c0->bc_ev, c0->stream));
    for (uint32_t k = 1; k < n_ctx; k++) {
        tsdf_ctx* c = ctxs[k];
        HIPCHK(c, hipSetDevice(c->device));
        rc = pend_stage_buffer(c);
        if (rc) return rc;
        const uint64_t off = c->pend.s[c->pend.n_scans].off;
        if (fanout) {
            // batch-granular: extend the follower's uncopied range when it continues in the same
            // leader buffer at the same offset (lockstep batches), else copy what it holds first
            if (c->fan_src != c0 || c->fan_buf != buf0 || c->fan_hi != off || off != off0) {
                rc = fan_copy(c);
                if (rc) return rc;
                if (c->fan_src && c->fan_src != c0) {  // a new leader
                    auto& v = c->fan_src->fan_followers;
                    v.erase(std::remove(v.begin(), v.end(), c), v.end());
                }
                if (std::find(c0->fan_followers.begin(), c0->fan_followers.end(), c) ==
                    c0->fan_followers.end())
                    c0->fan_followers.push_back(c);
                c->fan_src = c0;
                c->fan_buf = buf0;
                c->fan_lo = c->fan_hi = off;
                if (off != off0) {  // out of lockstep: this scan alone, now
                    c->fan_buf = nullptr;  // nothing pending; the next scan starts afresh
                    if (n) {
                        rc = fan_copy_range(c, c0, c->stage2[c->pend_stage] + 3 * off,
                                            buf0 + 3 * off0, n * 12);
                        if (rc) return rc;
                    }
                }
            }
            if (c->fan_buf) c->fan_hi = off + n;
        } else if (n) {
            // H2D: this context's own PCIe copy of h[0]; the leader must not reuse h[0] first
            HIPCHK(c, hipMemcpyAsync(c->stage2[c->pend_stage] + 3 * off, hx, n * 12,
                                     hipMemcpyHostToDevice, c->stream));
            if (!c->bc_ev) HIPCHK(c, hipEventCreateWithFlags(&c->bc_ev, hipEventDisableTiming));
            HIPCHK(c, hipEventRecord(c->bc_ev, c->stream));
            HIPCHK(c0, hipStreamWaitEvent(c0->stream, c->bc_ev, 0));
        }
        rc = pend_push(c, n, P);  // a full batch launches here (fan-out: after its copy)
        if (rc) return rc;
    }
    HIPCHK(c0, hipSetDevice(c0->device));
    HIPCHK(c0, hipEventRecord(c0->stage_done[hb[0]], c0->stream));
    rc = pend_push(c0, n, P);
    if (rc) return rc;
    c0->split_ht.lap(2);
    return TSDF_OK;
}

extern "C" {

// One host cloud for N sector-sharded contexts (the live N-GPU input path): every
// point is classified once (the kernels' in_sector rule on each context's bounds) and packed into
// its context's pinned staging; each context then copies only its sector's points to its GPU, so a
// scan crosses PCIe once in total, split over the N links.
static int sectors_impl(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts, uint64_t n,
                        uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64,
                        const ScanPose& P);

int tsdf_integrate_sectors(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts, uint64_t n,
                           uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64,
                           const double pose[7]) {
    if (!ctxs || n_ctx == 0 || n_ctx > TSDF_MAX_WORLD) return TSDF_EINVAL;
    for (uint32_t k = 0; k < n_ctx; k++)
        if (!ctxs[k]) return TSDF_EINVAL;
    if (!pose) return fail(ctxs[0], TSDF_EINVAL, "null argument");
    const double qn = pose[3] * pose[3] + pose[4] * pose[4] + pose[5] * pose[5] + pose[6] * pose[6];
    if (!(qn > 0.0) || !std::isfinite(qn)) return fail(ctxs[0], TSDF_EINVAL, "pose quaternion is zero");
    return sectors_impl(ctxs, n_ctx, pts, n, point_step, xyz_offset, xyz_is_f64, pose_of(pose));
}

// ABI v9: the sectors path with a bare origin keeps tsdf_integrate's "no orientation"
// (Voxblox's constant weight), so the sharded field equals the unsharded one for every semantics
int tsdf_integrate_sectors_origin(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts,
                                  uint64_t n, uint32_t point_step, uint32_t xyz_offset,
                                  int32_t xyz_is_f64, const double origin[3]) {
    if (!ctxs || n_ctx == 0 || n_ctx > TSDF_MAX_WORLD) return TSDF_EINVAL;
    for (uint32_t k = 0; k < n_ctx; k++)
        if (!ctxs[k]) return TSDF_EINVAL;
    if (!origin) return fail(ctxs[0], TSDF_EINVAL, "null argument");
    return sectors_impl(ctxs, n_ctx, pts, n, point_step, xyz_offset, xyz_is_f64,
                        pose_of_origin(origin));
}

}  // extern "C"

// tsdf_integrate_sectors under TSDF_SECTOR_RULE_INDEX: context k receives points [lo_k, hi_k)
// (idx_share).  The packing is one parallel pass on the staging threads of ALL the contexts (each
// part of the cloud to the pinned buffers of the contexts whose shares it covers), then per
// context one H2D copy of its share and the scan joins its pending batch.
static int sectors_shares(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts, uint64_t n,
                          uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64,
                          const ScanPose& P) {
    tsdf_ctx* c0 = ctxs[0];
    HostTiming& ht = c0->split_ht;
    ht.start();
    uint64_t lo[TSDF_MAX_WORLD + 1];
    for (uint32_t k = 0; k < n_ctx; k++) {
        uint64_t l, h;
        idx_share(ctxs[k], n, l, h);
        lo[k] = l;
        if (h - l > ctxs[k]->max_points)
            return fail(c0, TSDF_EINVAL, "share of %llu points exceeds max_points of context %u",
                        (unsigned long long)(h - l), k);
    }
    lo[n_ctx] = n;
    float* h[TSDF_MAX_WORLD];
    int hb[TSDF_MAX_WORLD];
    for (uint32_t k = 0; k < n_ctx; k++) {  // room in every pending batch, a free pinned buffer
        tsdf_ctx* c = ctxs[k];
        HIPCHK(c, hipSetDevice(c->device));
        const int rc = pend_room(c, lo[k + 1] - lo[k]);
        if (rc) {
            if (k) c0->err = c->err;
            return rc;
        }
        hb[k] = c->stage_cur;
        c->stage_cur ^= 1;
        HIPCHK(c, hipEventSynchronize(c->stage_done[hb[k]]));
        h[k] = c->h_stage[hb[k]];
    }
    ht.lap(0);
    const char* base = static_cast<const char*>(pts);
    auto pack = [&](uint64_t i0, uint64_t i1) {
        uint32_t k = 0;
        while (k + 1 < n_ctx && lo[k + 1] <= i0) k++;
        for (uint64_t i = i0; i < i1;) {
            const uint64_t e = std::min(i1, lo[k + 1]);  // this context's part of [i0, i1)
            float* dst = h[k] + 3 * (i - lo[k]);
            if (!xyz_is_f64 && point_step == 12 && xyz_offset == 0) {
                std::memcpy(dst, base + 12 * i, (e - i) * 12);
            } else {
                for (uint64_t j = i; j < e; j++, dst += 3) {
                    const char* q = base + j * point_step + xyz_offset;
                    if (xyz_is_f64) {
                        double d[3];
                        std::memcpy(d, q, sizeof d);
                        dst[0] = (float)d[0];
                        dst[1] = (float)d[1];
                        dst[2] = (float)d[2];
                    } else {
                        std::memcpy(dst, q, 12);
                    }
                }
            }
            i = e;
            k++;
        }
    };
    // the staging pools of the first few contexts only: every pool's workers spin ~100 us after a
    // job, so N pools' workers (4 N threads) would crowd the calling thread off a 16-CPU share
    // (TSDF_SECTOR_PACK_POOLS, default 2: 8 threads)
    static const uint32_t max_pools = [] {
        const char* e = std::getenv("TSDF_SECTOR_PACK_POOLS");
        return e ? (uint32_t)std::max(1, std::atoi(e)) : 2u;
    }();
    const uint32_t np = std::min(n_ctx, max_pools);
    int pbase[TSDF_MAX_WORLD + 1];
    pbase[0] = 0;
    for (uint32_t k = 0; k < np; k++)
        pbase[k + 1] = pbase[k] + (ctxs[k]->pack ? ctxs[k]->pack->parts() - (k ? 1 : 0) : (k ? 0 : 1));
    const int parts = n >= (1u << 15) ? pbase[np] : 1;
    auto part = [&](int q) { pack(n * (uint64_t)q / parts, n * (uint64_t)(q + 1) / parts); };
    if (parts == 1) {
        part(0);
    } else {
        for (uint32_t k = 1; k < np; k++)
            if (ctxs[k]->pack) ctxs[k]->pack->start(part, pbase[k] - 1);
        if (c0->pack) c0->pack->run(part);
        else part(0);
        for (uint32_t k = 1; k < np; k++)
            if (ctxs[k]->pack) ctxs[k]->pack->wait();
    }
    ht.lap(1);
    for (uint32_t k = 0; k < n_ctx; k++) {
        tsdf_ctx* c = ctxs[k];
        const uint64_t nk = lo[k + 1] - lo[k];
        HIPCHK(c, hipSetDevice(c->device));
        int rc = pend_stage_buffer(c);
        if (!rc && nk)
            HIPCHK(c, hipMemcpyAsync(c->stage2[c->pend_stage] + 3 * (uint64_t)c->pend.s[c->pend.n_scans].off,
                                     h[k], nk * 12, hipMemcpyHostToDevice, c->stream));
        if (!rc) HIPCHK(c, hipEventRecord(c->stage_done[hb[k]], c->stream));
        if (!rc) rc = pend_push(c, nk, P);
        if (rc) {
            if (k) c0->err = c->err;
            return rc;
        }
    }
    HIPCHK(c0, hipSetDevice(c0->device));
    ht.lap(3);
    ht.n++;
    return TSDF_OK;
}

static int sectors_impl(tsdf_ctx* const* ctxs, uint32_t n_ctx, const void* pts, uint64_t n,
                        uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64,
                        const ScanPose& P) {
    tsdf_ctx* c0 = ctxs[0];
    if (!pts && n) return fail(c0, TSDF_EINVAL, "null argument");
    const uint32_t need = xyz_is_f64 ? 24u : 12u;
    if (point_step < need || xyz_offset > point_step - need)
        return fail(c0, TSDF_EINVAL, "point_step/xyz_offset inconsistent");
    for (uint32_t k = 0; k < n_ctx; k++)
        if (border_busy(ctxs[k])) {
            if (k) c0->err = ctxs[k]->err;
            return TSDF_EINVAL;
        }
    for (uint32_t k = 0; k < n_ctx; k++) {
        const tsdf_ctx* c = ctxs[k];
        const bool sharded = n_ctx == 1 ? c->p.n_sectors <= 1 : c->p.n_sectors == n_ctx;
        if (!sharded || (n_ctx > 1 && (c->p.sector != k || c->p.sector_yaw0 != c0->p.sector_yaw0 ||
                                       c->p.sector_rule != c0->p.sector_rule)))
            return fail(c0, TSDF_EINVAL,
                        "context %u is not sector %u of %u (same sector_yaw0 and sector_rule)", k, k,
                        n_ctx);
    }
    // TSDF_SECTOR_RULE_INDEX (ABI v10): context k's share is a contiguous index range of the
    // cloud: every context's staging threads pack the whole cloud once, each point into its own
    // context's pinned buffer, then each context copies only its share over its own PCIe link --
    // one pass over the cloud, no classification, no fan-out (a Merged context bundles its share)
    if (n_ctx > 1 && c0->idx_rule) return sectors_shares(ctxs, n_ctx, pts, n, point_step,
                                                         xyz_offset, xyz_is_f64, P);
    for (uint32_t k = 0; k < n_ctx; k++) {
        const tsdf_ctx* c = ctxs[k];
        if (n > c->max_points)  // a context may receive every point
            return fail(c0, TSDF_EINVAL, "scan of %llu points exceeds max_points of context %u",
                        (unsigned long long)n, k);
    }
    const float ox = (float)P.o[0], oy = (float)P.o[1];
    HostTiming& ht = c0->split_ht;
    ht.start();
    // room in every pending batch, and each context's free pinned buffer
    float* h[TSDF_MAX_WORLD];
    int hb[TSDF_MAX_WORLD];
    for (uint32_t k = 0; k < n_ctx; k++) {
        tsdf_ctx* c = ctxs[k];
        HIPCHK(c, hipSetDevice(c->device));
        const int rc = pend_room(c, n);
        if (rc) return rc;
        hb[k] = c->stage_cur;
        c->stage_cur ^= 1;
        HIPCHK(c, hipEventSynchronize(c->stage_done[hb[k]]));
        h[k] = c->h_stage[hb[k]];
    }
    int mode = n_ctx > 1 ? c0->p.sector_input : TSDF_SECTOR_INPUT_SPLIT;
    // MergedTsdfIntegrator bundles the whole scan's points before the sector filter: a host split
    // would bundle each sector's points apart
    if (mode == TSDF_SECTOR_INPUT_SPLIT && n_ctx > 1 && c0->merged) mode = TSDF_SECTOR_INPUT_FANOUT;
    if (mode == TSDF_SECTOR_INPUT_FANOUT || mode == TSDF_SECTOR_INPUT_H2D) {
        ht.lap(0);
        const int rc = sectors_broadcast(ctxs, n_ctx, pts, n, point_step, xyz_offset, xyz_is_f64,
                                         P, h, hb, mode == TSDF_SECTOR_INPUT_FANOUT);
        if (rc) return rc;
        ht.lap(3);
        ht.n++;
        return TSDF_OK;
    }
    // Two passes over point chunks, on the staging threads of ALL the contexts (each GPU's host
    // share): (1) read the records once, pack xyz into c0's scratch and classify each point,
    // counting per (part, sector); (2) copy the packed points, still in cache, to their sector's
    // pinned buffer at the part's prefix (the parts keep the input order within a sector).
    const char* base = static_cast<const char*>(pts);
    // The sector of a point: the starts s_k of the N sectors, rotated to ascending order
    // u_j = s_(r+j), give sector (r + #{j: a >= u_j} - 1) mod N -- the kernels' in_sector test on
    // every context's [lo, hi) bounds (the wrap sector holds a < u_0 and a >= u_(N-1)), one
    // pseudo-angle and N compares per point.  NaN: no sector (every kernel drops the ray).
    const bool sharded = n_ctx > 1 && c0->R.sec_on;
    float u[TSDF_MAX_WORLD];
    uint32_t r0 = 0;
    if (sharded) {
        for (uint32_t k = 1; k < n_ctx; k++)
            if (ctxs[k]->R.sec_lo < ctxs[r0]->R.sec_lo) r0 = k;
        for (uint32_t j = 0; j < n_ctx; j++) {
            u[j] = ctxs[(r0 + j) % n_ctx]->R.sec_lo;
            if (j && !(u[j] > u[j - 1]))
                return fail(c0, TSDF_EINVAL, "sector starts of the contexts are not distinct");
        }
    }
    // parts: c0's pool (caller + workers), then every other context's workers
    int pbase[TSDF_MAX_WORLD + 1];
    pbase[0] = 0;
    for (uint32_t k = 0; k < n_ctx; k++)
        pbase[k + 1] = pbase[k] + (ctxs[k]->pack ? ctxs[k]->pack->parts() - (k ? 1 : 0) : (k ? 0 : 1));
    const int parts = n >= (1u << 15) ? pbase[n_ctx] : 1;
    auto run_parts = [&](const std::function<void(int)>& f) {
        if (parts == 1) return f(0);
        for (uint32_t k = 1; k < n_ctx; k++)
            if (ctxs[k]->pack) ctxs[k]->pack->start(f, pbase[k] - 1);
        if (c0->pack) c0->pack->run(f);
        else f(0);
        for (uint32_t k = 1; k < n_ctx; k++)
            if (ctxs[k]->pack) ctxs[k]->pack->wait();
    };
    if (c0->split_xyz.size() < 3 * n) {
        c0->split_xyz.resize(3 * n);
        c0->split_sec.resize(n);
    }
    float* xyz = c0->split_xyz.data();
    int8_t* sec = c0->split_sec.data();
    std::vector<uint64_t> cnt((size_t)parts * n_ctx, 0), at((size_t)parts * n_ctx, 0);
    auto classify = [&](int part) {
        const uint64_t i0 = n * part / parts, i1 = n * (part + 1) / parts;
        uint64_t cl[TSDF_MAX_WORLD] = {};  // local counts (the parts' rows share cache lines)
        for (uint64_t i = i0; i < i1; i++) {
            const char* q = base + i * point_step + xyz_offset;
            float* v = xyz + 3 * i;
            if (xyz_is_f64) {
                double d[3];
                std::memcpy(d, q, sizeof d);
                v[0] = (float)d[0];
                v[1] = (float)d[1];
                v[2] = (float)d[2];
            } else {
                std::memcpy(v, q, 12);
            }
            int k = 0;
            if (sharded) {
                const float a = pseudo_angle(v[0] - ox, v[1] - oy);
                uint32_t c = 0;
                for (uint32_t j = 0; j < n_ctx; j++) c += a >= u[j] ? 1u : 0u;
                uint32_t m = r0 + c + n_ctx - 1u;  // (r0 + c - 1) mod N without a division: m < 3N
                m -= m >= n_ctx ? n_ctx : 0u;
                m -= m >= n_ctx ? n_ctx : 0u;
                k = a != a ? -1 : (int)m;
            }
            sec[i] = (int8_t)k;
            if (k >= 0) cl[k]++;
        }
        for (uint32_t k = 0; k < n_ctx; k++) cnt[(size_t)part * n_ctx + k] = cl[k];
    };
    auto scatter = [&](int part) {
        const uint64_t i0 = n * part / parts, i1 = n * (part + 1) / parts;
        float* dst[TSDF_MAX_WORLD];
        for (uint32_t k = 0; k < n_ctx; k++) dst[k] = h[k] + 3 * at[(size_t)part * n_ctx + k];
        for (uint64_t i = i0; i < i1; i++) {
            const int k = sec[i];
            if (k < 0) continue;
            std::memcpy(dst[k], xyz + 3 * i, 12);
            dst[k] += 3;
        }
    };
    ht.lap(0);
    run_parts(classify);
    ht.lap(1);
    std::vector<uint64_t> tot(n_ctx, 0);
    for (uint32_t k = 0; k < n_ctx; k++)
        for (int q = 0; q < parts; q++) {
            at[(size_t)q * n_ctx + k] = tot[k];
            tot[k] += cnt[(size_t)q * n_ctx + k];
        }
    run_parts(scatter);
    ht.lap(2);
    // each context: its sector's points to its GPU, into its pending batch -- the contexts are
    // independent, so the staging threads issue them side by side (the copy and launch API calls
    // cost ~10 us each on the host)
    int crc[TSDF_MAX_WORLD] = {};
    auto push_ctx = [&](uint32_t k) -> int {
        tsdf_ctx* c = ctxs[k];
        HIPCHK(c, hipSetDevice(c->device));
        int rc = pend_stage_buffer(c);
        if (rc) return rc;
        if (tot[k])
            HIPCHK(c, hipMemcpyAsync(c->stage2[c->pend_stage] + 3 * (uint64_t)c->pend.s[c->pend.n_scans].off,
                                     h[k], tot[k] * 12, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipEventRecord(c->stage_done[hb[k]], c->stream));
        return pend_push(c, tot[k], P);
    };
    const int cparts = c0->pack && n_ctx > 1 ? std::min<int>(c0->pack->parts(), (int)n_ctx) : 1;
    if (cparts > 1) {
        c0->pack->run([&](int part) {
            if (part >= cparts) return;
            for (uint32_t k = (uint32_t)part; k < n_ctx; k += (uint32_t)cparts) crc[k] = push_ctx(k);
        });
    } else {
        for (uint32_t k = 0; k < n_ctx; k++) crc[k] = push_ctx(k);
    }
    for (uint32_t k = 0; k < n_ctx; k++)
        if (crc[k]) return crc[k];
    ht.lap(3);
    ht.n++;
    return TSDF_OK;
}

extern "C" {

int tsdf_integrate_pose(tsdf_ctx* c, const void* pts, uint64_t n, uint32_t point_step,
                        uint32_t xyz_offset, int32_t xyz_is_f64, const double pose[7]) {
    if (!c) return TSDF_EINVAL;
    if ((!pts && n) || !pose) return fail(c, TSDF_EINVAL, "null argument");
    const double qn = pose[3] * pose[3] + pose[4] * pose[4] + pose[5] * pose[5] + pose[6] * pose[6];
    if (!(qn > 0.0) || !std::isfinite(qn)) return fail(c, TSDF_EINVAL, "pose quaternion is zero");
    return integrate_impl(c, pts, n, point_step, xyz_offset, xyz_is_f64, pose_of(pose));
}

// origins: 3 doubles per scan (pose_stride 3) or poses: 7 per scan (pose_stride 7)
static int batch_device_impl(tsdf_ctx* c, const float* d_xyz, const uint64_t* offs,
                             uint32_t n_scans, const double* origins, int pose_stride) {
    if (!c) return TSDF_EINVAL;
    if (border_busy(c)) return TSDF_EINVAL;
    if (!offs || !origins || (!d_xyz && n_scans)) return fail(c, TSDF_EINVAL, "null argument");
    for (uint32_t s = 0; s < n_scans; s++) {
        if (offs[s + 1] < offs[s]) return fail(c, TSDF_EINVAL, "scan_offsets not monotone");
        if (offs[s + 1] - offs[s] > c->max_points)
            return fail(c, TSDF_EINVAL, "scan %u of %llu points exceeds max_points %llu", s,
                        (unsigned long long)(offs[s + 1] - offs[s]),
                        (unsigned long long)c->max_points);
    }
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush(c);
    if (rc) return rc;
    // Each scan's share (all of it unless index-sharded: then only [lo, hi) of it is read, and the
    // shares of a batch's scans are not contiguous -- ScanRec.xoff = the gap before each share)
    uint32_t s = 0;
    while (s < n_scans) {
        BatchDesc D;
        D.n_scans = 0;
        D.s[0].off = 0;
        uint64_t lo, hi;
        idx_share(c, offs[s + 1] - offs[s], lo, hi);
        const uint64_t b0 = offs[s] + lo;
        while (s < n_scans && D.n_scans < c->max_batch) {
            idx_share(c, offs[s + 1] - offs[s], lo, hi);
            const uint64_t x0 = offs[s] + lo - b0, nb = D.s[D.n_scans].off + (hi - lo);
            if (nb > c->batch_points || x0 + (hi - lo) > 0xFFFFFFFFull) break;
            const double* q = origins + (uint64_t)pose_stride * s;
            set_pose(D, D.n_scans, pose_stride == 7 ? pose_of(q) : pose_of_origin(q));
            D.s[D.n_scans].xoff = (uint32_t)(x0 - D.s[D.n_scans].off);
            D.s[D.n_scans + 1].off = (uint32_t)nb;
            D.n_scans++;
            s++;
        }
        rc = launch(c, d_xyz + 3 * b0, D);
        if (rc) return rc;
        c->n_points_in += D.s[D.n_scans].off;
    }
    return TSDF_OK;
}

int tsdf_integrate_batch_device(tsdf_ctx* c, const float* d_xyz, const uint64_t* offs,
                                uint32_t n_scans, const double* origins) {
    return batch_device_impl(c, d_xyz, offs, n_scans, origins, 3);
}

int tsdf_integrate_batch_device_pose(tsdf_ctx* c, const float* d_xyz, const uint64_t* offs,
                                     uint32_t n_scans, const double* poses) {
    if (c && poses)
        for (uint32_t s = 0; s < n_scans; s++) {
            const double* q = poses + 7 * (uint64_t)s;
            const double qn = q[3] * q[3] + q[4] * q[4] + q[5] * q[5] + q[6] * q[6];
            if (!(qn > 0.0) || !std::isfinite(qn))
                return fail(c, TSDF_EINVAL, "pose %u: quaternion is zero", s);
        }
    return batch_device_impl(c, d_xyz, offs, n_scans, poses, 7);
}

// A single device scan joins the pending batch like a host scan: its points are copied into the
// pending batch's device staging before the call returns, so the caller's buffer is free at once
// (and a capacity replay re-reads the library's copy, not the caller's memory).
int tsdf_integrate_device(tsdf_ctx* c, const float* d_xyz, uint64_t n, const double origin[3]) {
    if (!c) return TSDF_EINVAL;
    if (border_busy(c)) return TSDF_EINVAL;
    if ((!d_xyz && n) || !origin) return fail(c, TSDF_EINVAL, "null argument");
    {  // the context's share of the scan (all of it unless index-sharded)
        uint64_t lo, hi;
        idx_share(c, n, lo, hi);
        if (d_xyz) d_xyz += 3 * lo;
        n = hi - lo;
    }
    if (n > c->max_points)
        return fail(c, TSDF_EINVAL, "scan of %llu points exceeds max_points %llu",
                    (unsigned long long)n, (unsigned long long)c->max_points);
    HIPCHK(c, hipSetDevice(c->device));
    int rc = pend_room(c, n);
    if (!rc) rc = pend_stage_buffer(c);
    if (rc) return rc;
    if (n) {
        HIPCHK(c, hipMemcpyAsync(c->stage2[c->pend_stage] + 3 * (uint64_t)c->pend.s[c->pend.n_scans].off,
                                 d_xyz, n * 12, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return pend_push(c, n, pose_of_origin(origin));
}

int tsdf_sync(tsdf_ctx* c) {
    if (!c) return TSDF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = settle(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    rc = check_and_replay(c);
    if (rc) return rc;
    if (c->timer) c->timer->harvest();
    rc = emit_metrics(c);
    if (rc) return rc;
    uint32_t ovf = 0;
    HIPCHK(c, hipMemcpy(&ovf, &c->G->overflow, sizeof ovf, hipMemcpyDeviceToHost));
    if (ovf) {
        HIPCHK(c, hipMemset(&c->G->overflow, 0, sizeof ovf));
        if (ovf & ERR_MERGE_KEY)
            return fail(c, TSDF_EINVAL, "border merge: a tile's brick is not held by this context");
        return fail(c, TSDF_ENOMEM, "capacity overflow (%s%s%s%s%s%s%s): updates were dropped",
                    (ovf & OVF_TABLE) ? "hash table full; " : "",
                    (ovf & OVF_POOL) ? "brick pool exhausted; " : "",
                    (ovf & OVF_PAIRS) ? "ray brick-pair slots exceeded; " : "",
                    (ovf & OVF_ACTIVE) ? "active-brick list full; " : "",
                    (ovf & OVF_SMP) ? "sample list full; " : "",
                    (ovf & OVF_FB) ? "fallback pair list full; " : "",
                    (ovf & OVF_SPN) ? "span list full; " : "");
    }
    return TSDF_OK;
}

// flush + drain, ignoring (but keeping) the overflow flag for read-out calls
static int drain(tsdf_ctx* c) {
    HIPCHK(c, hipSetDevice(c->device));
    int rc = settle(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    rc = check_and_replay(c);
    if (rc) return rc;
    if (c->timer) c->timer->harvest();
    return emit_metrics(c);
}

int tsdf_query_dense(tsdf_ctx* c, const int64_t lo[3], const int64_t hi[3], float* sdf,
                     float* weight) {
    if (!c) return TSDF_EINVAL;
    if (!lo || !hi) return fail(c, TSDF_EINVAL, "null argument");
    int dims[3];
    for (int a = 0; a < 3; a++) {
        if (hi[a] < lo[a]) return fail(c, TSDF_EINVAL, "hi < lo");
        // (the extent as unsigned: hi - lo of int64 bounds may exceed the int64 range)
        const uint64_t ext = (uint64_t)hi[a] - (uint64_t)lo[a];
        if (ext >= (1ull << 31)) return fail(c, TSDF_EINVAL, "query extent >= 2^31 voxels");
        dims[a] = (int)ext;
    }
    uint64_t total = 0;  // (dims[0] dims[1] < 2^62; the third factor may overflow)
    if (__builtin_mul_overflow((uint64_t)dims[0] * (uint64_t)dims[1], (uint64_t)dims[2], &total) ||
        total >= (1ull << 40))
        return fail(c, TSDF_EINVAL, "query box >= 2^40 voxels");
    int rc = drain(c);
    if (rc) return rc;
    if (!total) return TSDF_OK;
    float *ds = nullptr, *dw = nullptr;
    HIPCHK(c, hipMalloc(&ds, total * sizeof(float)));
    hipError_t e = hipMalloc(&dw, total * sizeof(float));
    if (e == hipSuccess) e = launch_query_dense(c->T, c->Pl, lo, dims, c->R.bg, ds,
                                                dw, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && sdf) e = hipMemcpy(sdf, ds, total * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && weight) e = hipMemcpy(weight, dw, total * 4, hipMemcpyDeviceToHost);
    (void)hipFree(ds);
    if (dw) (void)hipFree(dw);
    if (e != hipSuccess) return fail(c, TSDF_EHIP, "query_dense: %s", hipGetErrorString(e));
    return TSDF_OK;
}

static int pool_bricks(tsdf_ctx* c, uint64_t* n) {
    const int rc = drain(c);
    if (rc) return rc;
    uint32_t pc = 0;
    HIPCHK(c, hipMemcpy(&pc, &c->G->pool_count, sizeof pc, hipMemcpyDeviceToHost));
    *n = std::min<uint64_t>(pc, c->T.max_bricks);
    return TSDF_OK;
}

int tsdf_num_bricks(tsdf_ctx* c, uint64_t* n) {
    if (!c || !n) return TSDF_EINVAL;
    return pool_bricks(c, n);
}

int tsdf_export_bricks(tsdf_ctx* c, int32_t* coords, float* sdf, float* weight, uint64_t cap,
                       uint64_t* n_out) {
    if (!c || !n_out) return TSDF_EINVAL;
    uint64_t nb = 0;
    int rc = pool_bricks(c, &nb);
    if (rc) return rc;
    *n_out = nb;
    if (nb > cap) return fail(c, TSDF_EOVERFLOW, "export needs %llu bricks", (unsigned long long)nb);
    if (!nb) return TSDF_OK;
    std::vector<uint64_t> keys(nb);
    std::vector<float> s, w;
    HIPCHK(c, hipMemcpy(keys.data(), c->T.brick_keys, nb * 8, hipMemcpyDeviceToHost));
    if (sdf) {
        s.resize(nb * BRICK_VOX);
        HIPCHK(c, hipMemcpy(s.data(), c->Pl.sdf, nb * BRICK_VOX * 4, hipMemcpyDeviceToHost));
    }
    if (weight) {
        w.resize(nb * BRICK_VOX);
        HIPCHK(c, hipMemcpy(w.data(), c->Pl.weight, nb * BRICK_VOX * 4, hipMemcpyDeviceToHost));
    }
    auto coord = [&](uint64_t k, int a) {
        return (int32_t)((keys[k] >> (21 * a)) & 0x1FFFFF) - BRICK_COORD_BIAS;
    };
    std::vector<uint64_t> order(nb);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) {
        for (int ax = 2; ax >= 0; ax--)
            if (coord(a, ax) != coord(b, ax)) return coord(a, ax) < coord(b, ax);
        return false;
    });
    for (uint64_t i = 0; i < nb; i++) {
        const uint64_t k = order[i];
        if (coords)
            for (int a = 0; a < 3; a++) coords[3 * i + a] = coord(k, a);
        if (sdf) std::memcpy(sdf + i * BRICK_VOX, s.data() + k * BRICK_VOX, BRICK_VOX * 4);
        if (weight) std::memcpy(weight + i * BRICK_VOX, w.data() + k * BRICK_VOX, BRICK_VOX * 4);
    }
    return TSDF_OK;
}

// Ouster packet layouts per UDP profile (ouster_client/src/parsing.cpp:42-175): header / column /
// footer sizes and, for RANGE, SIGNAL, REFLECTIVITY, NEAR_IR: (bytes, offset, mask, shift).
static bool os_layout(const tsdf_os_format* f, OsLayout& L) {
    if (!f || f->pixels_per_column == 0 || f->columns_per_packet == 0 || f->columns_per_frame == 0 ||
        f->pixels_per_column > 4096)
        return false;
    L = OsLayout{};
    L.h = f->pixels_per_column;
    L.w = f->columns_per_frame;
    L.cols_per_packet = f->columns_per_packet;
    switch (f->profile) {
        case TSDF_OS_LEGACY:
            L.pixel_bytes = 12;
            L.f[0] = {4, 0, 0x000FFFFFu, 0};
            L.f[1] = {2, 6, 0, 0};
            L.f[2] = {2, 4, 0, 0};
            L.f[3] = {2, 8, 0, 0};
            break;
        case TSDF_OS_RNG19_RFL8_SIG16_NIR16:
            L.pixel_bytes = 12;
            L.f[0] = {4, 0, 0x0007FFFFu, 0};
            L.f[1] = {2, 6, 0, 0};
            L.f[2] = {1, 4, 0, 0};
            L.f[3] = {2, 8, 0, 0};
            break;
        case TSDF_OS_RNG19_RFL8_SIG16_NIR16_DUAL:
            L.pixel_bytes = 16;
            L.f[0] = {4, 0, 0x0007FFFFu, 0};
            L.f[1] = {2, 8, 0, 0};
            L.f[2] = {1, 3, 0, 0};
            L.f[3] = {2, 12, 0, 0};
            break;
        case TSDF_OS_RNG15_RFL8_NIR8:
            L.pixel_bytes = 4;
            L.f[0] = {2, 0, 0x7FFFu, -3};
            L.f[1] = {0, 0, 0, 0};
            L.f[2] = {1, 2, 0, 0};
            L.f[3] = {1, 3, 0, -4};
            break;
        default:
            return false;
    }
    L.legacy = f->profile == TSDF_OS_LEGACY ? 1u : 0u;
    L.packet_header = L.legacy ? 0u : 32u;
    L.col_header = L.legacy ? 16u : 12u;
    const uint32_t col_footer = L.legacy ? 4u : 0u, packet_footer = L.legacy ? 0u : 32u;
    L.col_bytes = L.col_header + L.h * L.pixel_bytes + col_footer;
    L.packet_bytes = L.packet_header + L.cols_per_packet * L.col_bytes + packet_footer;
    return true;
}

int tsdf_os_packet_bytes(const tsdf_os_format* fmt, uint32_t* bytes) {
    OsLayout L;
    if (!bytes || !os_layout(fmt, L)) return TSDF_EINVAL;
    *bytes = L.packet_bytes;
    return TSDF_OK;
}

int tsdf_os_decode_device(tsdf_ctx* c, const tsdf_os_format* fmt, const uint8_t* d_packets,
                          uint32_t n_packets, uint32_t* d_range, uint32_t* d_signal,
                          uint32_t* d_reflectivity, uint32_t* d_near_ir) {
    if (!c) return TSDF_EINVAL;
    OsLayout L;
    if (!os_layout(fmt, L)) return fail(c, TSDF_EINVAL, "bad Ouster packet format");
    if (n_packets && !d_packets) return fail(c, TSDF_EINVAL, "null packets");
    HIPCHK(c, hipSetDevice(c->device));
    uint32_t* out[4] = {d_range, d_signal, d_reflectivity, d_near_ir};
    const size_t img = (size_t)L.h * L.w * sizeof(uint32_t);
    for (int k = 0; k < 4; k++)
        if (out[k]) HIPCHK(c, hipMemsetAsync(out[k], 0, img, c->stream));
    HIPCHK(c, launch_os_decode(d_packets, n_packets, L, out, c->stream));
    return TSDF_OK;
}

int tsdf_os_cartesian_device(tsdf_ctx* c, const uint32_t* d_range, uint64_t n, const float* d_dir,
                             const float* d_off, const double pose[12], float* d_xyz) {
    if (!c) return TSDF_EINVAL;
    if (n && (!d_range || !d_dir || !d_off || !d_xyz)) return fail(c, TSDF_EINVAL, "null argument");
    if (!pose) return fail(c, TSDF_EINVAL, "null pose");
    HIPCHK(c, hipSetDevice(c->device));
    OsPose P;
    for (int k = 0; k < 12; k++) P.m[k] = (float)pose[k];
    HIPCHK(c, launch_os_xyz(d_range, n, d_dir, d_off, P, d_xyz, c->stream));
    return TSDF_OK;
}

}  // extern "C"

// A context's halo for meshing (ABI v9): received tiles as a small hash table + pool on the
// context's device (the mesh kernels look neighbours up there first).
struct Halo {
    Table H{};
    Pool HP{};
    void* mem[4] = {};
    void release() {
        for (void*& q : mem)
            if (q) {
                (void)hipFree(q);
                q = nullptr;
            }
    }
};

static int halo_build(tsdf_ctx* c, const uint32_t* d_halo, uint64_t n_halo, Halo& h) {
    if (!n_halo) return TSDF_OK;
    if (!d_halo) return fail(c, TSDF_EINVAL, "null halo tiles");
    if (n_halo >= (1ull << 30)) return fail(c, TSDF_EINVAL, "too many halo tiles");
    const uint64_t cap = next_pow2(2 * n_halo);
    hipError_t e = hipMalloc(&h.mem[0], cap * 8);
    if (e == hipSuccess) e = hipMalloc(&h.mem[1], cap * 4);
    if (e == hipSuccess) e = hipMalloc(&h.mem[2], n_halo * BRICK_VOX * 8);
    if (e == hipSuccess) e = hipMalloc(&h.mem[3], 16);
    if (e == hipSuccess) {
        h.H.keys = static_cast<uint64_t*>(h.mem[0]);
        h.H.slots = static_cast<uint32_t*>(h.mem[1]);
        h.H.mask = cap - 1;
        h.H.max_bricks = (uint32_t)n_halo;
        h.HP.sdf = static_cast<float*>(h.mem[2]);
        h.HP.weight = h.HP.sdf + n_halo * BRICK_VOX;
        e = launch_fill_u64(h.H.keys, EMPTY_KEY, cap, c->stream);
    }
    if (e == hipSuccess) e = hipMemsetAsync(h.mem[3], 0, 16, c->stream);
    if (e == hipSuccess)
        e = launch_halo_build(h.H, h.HP, d_halo, (uint32_t)n_halo, static_cast<uint32_t*>(h.mem[3]),
                              c->stream);
    uint32_t ovf = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&ovf, h.mem[3], 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        h.release();
        return fail(c, TSDF_EHIP, "halo: %s", hipGetErrorString(e));
    }
    if (ovf) {
        h.release();
        return fail(c, TSDF_EINVAL, "halo: table overflow");
    }
    return TSDF_OK;
}

// tsdf_extract_mesh_table, with optional halo tiles (device, TSDF_TILE_WORDS rows) looked up before
// the context's own table for the +x/+y/+z neighbours of its bricks
static int mesh_impl(tsdf_ctx* c, float min_weight, int32_t table, const uint32_t* d_halo,
                     uint64_t n_halo, float* tri, uint64_t cap, uint64_t* n_tri) {
    if (!c || !n_tri) return TSDF_EINVAL;
    if (table < 0 || table >= TSDF_MC_TABLES)
        return fail(c, TSDF_EINVAL, "unknown marching-cubes table %d", table);
    uint64_t nb = 0;
    int rc = pool_bricks(c, &nb);
    if (rc) return rc;
    *n_tri = 0;
    if (!nb) return TSDF_OK;
    if (nb >= 0xFFFFFFFFull) return fail(c, TSDF_EINVAL, "too many bricks");
    HIPCHK(c, hipSetDevice(c->device));
    Halo halo;
    rc = halo_build(c, d_halo, n_halo, halo);
    if (rc) return rc;
    // bricks in (z, y, x) order: the triangle soup's order (and the oracle's)
    std::vector<uint64_t> keys(nb);
    hipError_t e = hipMemcpy(keys.data(), c->T.brick_keys, nb * 8, hipMemcpyDeviceToHost);
    std::sort(keys.begin(), keys.end(), [](uint64_t a, uint64_t b) {
        for (int ax = 2; ax >= 0; ax--) {
            const uint64_t x = (a >> (21 * ax)) & 0x1FFFFF, y = (b >> (21 * ax)) & 0x1FFFFF;
            if (x != y) return x < y;
        }
        return false;
    });
    uint64_t* dk = nullptr;
    uint32_t* dc = nullptr;
    uint64_t* doff = nullptr;
    float* dt = nullptr;
    std::vector<uint32_t> cnt(nb);
    std::vector<uint64_t> off(nb);
    uint64_t total = 0;
    if (e == hipSuccess) e = hipMalloc(&dk, nb * 8);
    if (e == hipSuccess) e = hipMalloc(&dc, nb * 4);
    if (e == hipSuccess) e = hipMemcpyAsync(dk, keys.data(), nb * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = launch_mesh_count(c->T, c->Pl, halo.H, halo.HP, dk, (uint32_t)nb, min_weight, table, dc,
                              c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(cnt.data(), dc, nb * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) {
        for (uint64_t i = 0; i < nb; i++) {
            off[i] = total;
            total += cnt[i];
        }
        *n_tri = total;
    }
    if (e == hipSuccess && tri && total <= cap && total) {
        e = hipMalloc(&doff, nb * 8);
        if (e == hipSuccess) e = hipMalloc(&dt, total * 36);
        if (e == hipSuccess)
            e = hipMemcpyAsync(doff, off.data(), nb * 8, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess)
            e = launch_mesh_emit(c->T, c->Pl, halo.H, halo.HP, dk, (uint32_t)nb, min_weight, table,
                                 c->R.vs, doff, dt, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(tri, dt, total * 36, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    for (void* p : {(void*)dk, (void*)dc, (void*)doff, (void*)dt})
        if (p) (void)hipFree(p);
    halo.release();
    if (e != hipSuccess) return fail(c, TSDF_EHIP, "extract_mesh: %s", hipGetErrorString(e));
    if (tri && total > cap)
        return fail(c, TSDF_EOVERFLOW, "mesh has %llu triangles", (unsigned long long)total);
    return TSDF_OK;
}

extern "C" {

int tsdf_mc_table(uint8_t* out) {
    if (!out) return TSDF_EINVAL;
    std::memcpy(out, mc_table().tab, sizeof(mc_table().tab));
    return TSDF_OK;
}

int tsdf_mc_table_of(int32_t table, uint8_t* out) {
    if (!out || table < 0 || table >= TSDF_MC_TABLES) return TSDF_EINVAL;
    std::memcpy(out, mc_table(table).tab, sizeof(mc_table(table).tab));
    return TSDF_OK;
}

int tsdf_extract_mesh(tsdf_ctx* c, float min_weight, float* tri, uint64_t cap, uint64_t* n_tri) {
    return tsdf_extract_mesh_table(c, min_weight, TSDF_MC_GENERATED, tri, cap, n_tri);
}

int tsdf_extract_mesh_table(tsdf_ctx* c, float min_weight, int32_t table, float* tri, uint64_t cap,
                            uint64_t* n_tri) {
    return mesh_impl(c, min_weight, table, nullptr, 0, tri, cap, n_tri);
}

int tsdf_import_bricks(tsdf_ctx* c, const int32_t* coords, const float* sdf, const float* weight,
                       uint64_t n) {
    if (!c) return TSDF_EINVAL;
    if (border_busy(c)) return TSDF_EINVAL;
    if (!n) return TSDF_OK;
    if (!coords || !sdf || !weight) return fail(c, TSDF_EINVAL, "null argument");
    if (n >= 0xFFFFFFF0ull) return fail(c, TSDF_EINVAL, "too many bricks");
    {  // bricks must be unique and inside the packable range
        std::vector<uint64_t> k(n);
        for (uint64_t i = 0; i < n; i++) {
            for (int a = 0; a < 3; a++)
                if (coords[3 * i + a] < -BRICK_COORD_BIAS || coords[3 * i + a] >= BRICK_COORD_BIAS)
                    return fail(c, TSDF_EINVAL, "brick coordinate out of range");
            k[i] = (uint64_t)(coords[3 * i] + BRICK_COORD_BIAS) |
                   ((uint64_t)(coords[3 * i + 1] + BRICK_COORD_BIAS) << 21) |
                   ((uint64_t)(coords[3 * i + 2] + BRICK_COORD_BIAS) << 42);
        }
        std::sort(k.begin(), k.end());
        if (std::adjacent_find(k.begin(), k.end()) != k.end())
            return fail(c, TSDF_EINVAL, "duplicate brick in import");
    }
    int rc = drain(c);
    if (rc) return rc;
    {  // room for n new bricks (import is not a replayable batch: grow first)
        uint32_t pc = 0;
        HIPCHK(c, hipMemcpy(&pc, &c->G->pool_count, 4, hipMemcpyDeviceToHost));
        if (c->can_grow && (uint64_t)pc + n > c->T.max_bricks) {
            rc = grow_capacity(c, (uint64_t)pc + n);
            if (rc == TSDF_EHIP) return rc;
        }
    }
    int32_t* dc = nullptr;
    float *ds = nullptr, *dw = nullptr;
    uint32_t* dt = nullptr;
    hipError_t e = hipMalloc(&dc, n * 12);
    if (e == hipSuccess) e = hipMalloc(&ds, n * BRICK_VOX * 4);
    if (e == hipSuccess) e = hipMalloc(&dw, n * BRICK_VOX * 4);
    if (e == hipSuccess) e = hipMalloc(&dt, n * 4);
    if (e == hipSuccess) e = hipMemcpyAsync(dc, coords, n * 12, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ds, sdf, n * BRICK_VOX * 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(dw, weight, n * BRICK_VOX * 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_import(c->T, c->Pl, dc, (uint32_t)n, ds, dw, dt, c->G, merge_cap(c),
                                           c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(dc);
    (void)hipFree(ds);
    (void)hipFree(dw);
    (void)hipFree(dt);
    if (e != hipSuccess) return fail(c, TSDF_EHIP, "import: %s", hipGetErrorString(e));
    return tsdf_sync(c);
}

int tsdf_get_stats(tsdf_ctx* c, tsdf_stats* out) {
    if (!c || !out) return TSDF_EINVAL;
    const int rc = drain(c);
    if (rc) return rc;
    Globals g;
    HIPCHK(c, hipMemcpy(&g, c->G, sizeof g, hipMemcpyDeviceToHost));
    std::memset(out, 0, sizeof *out);
    out->n_scans = c->n_scans;
    out->n_batches = c->n_batches;
    out->n_points_in = c->n_points_in;
    out->n_bricks = std::min<uint64_t>(g.pool_count, c->T.max_bricks);
    out->n_grows = c->n_grows;
    out->n_replayed = c->n_replayed;
    out->max_bricks = c->T.max_bricks;
    out->peer_mask = c->peer_mask;
    if (c->batch_id) {
        const Counters& L = g.last;
        out->n_active_last = L.n_active;
        for (int k = 0; k < 8; k++) {
            out->n_voxels_last += L.n_vox[k];
            out->n_pairs_last += L.n_pairs[k];
        }
    }
    for (int k = 0; k < 8; k++) {
        out->n_voxels_total += g.tot_vox[k];
        out->n_rays_total += g.tot_rays[k];
        out->n_dirty_total += g.tot_dirty[k];
    }
    if (c->timer)
        for (int k = 0; k < KIND_N; k++) {
            out->kernel_ms[k] = c->timer->ms[k];
            out->kernel_launches[k] = c->timer->launches[k];
        }
    return TSDF_OK;
}

int tsdf_reset_stats(tsdf_ctx* c) {
    if (!c) return TSDF_EINVAL;
    const int rc = drain(c);
    if (rc) return rc;
    if (c->timer) c->timer->reset();
    HIPCHK(c, hipMemset(c->G->tot_vox, 0, sizeof(c->G->tot_vox) * 4));
    c->n_points_in = 0;
    c->n_scans = 0;
    c->n_batches = 0;
    return TSDF_OK;
}

int tsdf_set_profiling(tsdf_ctx* c, int32_t on) {
    if (!c) return TSDF_EINVAL;
    const int rc = drain(c);
    if (rc) return rc;
    if (on && !c->timer) {
        c->timer = new (std::nothrow) EventTimer();
        if (c->timer) c->timer->per_batch = c->metrics != nullptr;
    }
    if (!on && c->timer) { delete c->timer; c->timer = nullptr; }
    return (on && !c->timer) ? TSDF_ENOMEM : TSDF_OK;
}

int tsdf_set_profiling_period(tsdf_ctx* c, uint32_t every_mask, uint32_t period) {
    if (!c) return TSDF_EINVAL;
    if (period == 0) return fail(c, TSDF_EINVAL, "profiling period must be >= 1");
    if (!c->timer) return fail(c, TSDF_EINVAL, "profiling is off (tsdf_set_profiling)");
    c->timer->every_mask = every_mask;
    c->timer->period = period;
    return TSDF_OK;
}

int tsdf_set_metrics_log(tsdf_ctx* c, const char* path) {
    if (!c) return TSDF_EINVAL;
    int rc = drain(c);  // report (or drop) what came before
    if (rc) return rc;
    if (c->metrics) {
        fclose(c->metrics);
        c->metrics = nullptr;
    }
    if (c->timer) c->timer->per_batch = false;
    c->metrics_info.clear();
    c->metrics_next = c->batch_id;
    if (!path || !*path) return TSDF_OK;
    c->metrics = fopen(path, "a");
    if (!c->metrics) return fail(c, TSDF_EINVAL, "cannot open metrics log %s", path);
    if (c->timer) c->timer->per_batch = true;
    return TSDF_OK;
}

int32_t tsdf_sector_of(float px, float py, const double origin[3], double yaw0,
                       uint32_t n_sectors) {
    if (!origin || n_sectors == 0) return -1;
    const float dx = px - (float)origin[0], dy = py - (float)origin[1];
    if (!(dx == dx) || !(dy == dy)) return -1;
    if (n_sectors == 1) return 0;
    // the sector whose [start, next start) holds a, cyclically
    for (uint32_t k = 0; k < n_sectors; k++) {
        RayConst R{};
        sector_bounds(yaw0, k, n_sectors, R);
        if (in_sector(R, dx, dy)) return (int32_t)k;
    }
    return -1;
}

int tsdf_select_sector(const float* xyz, uint64_t n, const double origin[3], double yaw0,
                       uint32_t sector, uint32_t n_sectors, float* out_xyz, uint64_t* n_out) {
    if (!xyz || !origin || !out_xyz || !n_out || n_sectors == 0 || sector >= n_sectors)
        return TSDF_EINVAL;
    RayConst R{};
    sector_bounds(yaw0, sector, n_sectors, R);
    const float ox = (float)origin[0], oy = (float)origin[1];
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (!in_sector(R, xyz[3 * i] - ox, xyz[3 * i + 1] - oy)) continue;
        std::memcpy(out_xyz + 3 * k, xyz + 3 * i, 12);
        k++;
    }
    *n_out = k;
    return TSDF_OK;
}

// ---- border-brick reduce (include/tsdf_hip.h; kernels in tsdf_border.hip) ----------------------

int tsdf_brick_keys_device(tsdf_ctx* c, uint64_t* d_keys, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return TSDF_EINVAL;
    uint64_t nb = 0;
    int rc = pool_bricks(c, &nb);
    if (rc) return rc;
    *n_out = nb;
    if (nb > cap) return fail(c, TSDF_EOVERFLOW, "brick keys need %llu entries", (unsigned long long)nb);
    if (!nb) return TSDF_OK;
    if (!d_keys) return fail(c, TSDF_EINVAL, "null key buffer");
    HIPCHK(c, hipMemcpyAsync(d_keys, c->T.brick_keys, nb * 8, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TSDF_OK;
}

}  // extern "C"

// tsdf_border_pack_device with the reset optional: keep_rows (not null) receives the device list
// of the packed bricks' pool slots (caller frees it; null when nothing was packed) and their count,
// so the caller can reset them later (launch_border_reset)
static int border_pack_impl(tsdf_ctx* c, const uint64_t* d_all_keys, const uint64_t* counts,
                            uint64_t stride, uint32_t world, uint32_t rank, uint32_t* d_send,
                            uint64_t cap_rows, uint64_t* send_counts, bool reset,
                            uint32_t** keep_rows, uint64_t* kept) {
    if (keep_rows) *keep_rows = nullptr;
    if (kept) *kept = 0;
    if (!counts || !send_counts || world == 0 || world > TSDF_MAX_WORLD || rank >= world)
        return fail(c, TSDF_EINVAL, "bad world/rank or null counts");
    WorldCounts wc{};
    for (uint32_t r = 0; r < world; r++) {
        if (counts[r] > stride) return fail(c, TSDF_EINVAL, "counts[%u] > stride", r);
        wc.n[r] = counts[r];
        send_counts[r] = 0;
    }
    uint64_t nb = 0;
    int rc = pool_bricks(c, &nb);
    if (rc) return rc;
    if (!nb || rank == 0) return TSDF_OK;  // rank 0 owns everything it holds
    bool lower = false;
    for (uint32_t r = 0; r < rank; r++) lower |= wc.n[r] > 0;
    if (!lower) return TSDF_OK;
    if (!d_all_keys) return fail(c, TSDF_EINVAL, "null key buffer");
    uint32_t *d_owner = nullptr, *d_aux = nullptr, *d_rows = nullptr;
    uint32_t dest[MAX_WORLD] = {}, cursor[MAX_WORLD] = {};
    uint64_t rows = 0;
    hipError_t e = hipMalloc(&d_owner, nb * 4);
    if (e == hipSuccess) e = hipMalloc(&d_aux, 2 * MAX_WORLD * 4);
    if (e == hipSuccess)
        e = launch_border_owner(c->T, (uint32_t)nb, d_all_keys, wc, stride, rank, d_owner, d_aux,
                                c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dest, d_aux, sizeof dest, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) {
        for (uint32_t r = 0; r < world; r++) {
            cursor[r] = (uint32_t)rows;
            send_counts[r] = dest[r];
            rows += dest[r];
        }
    }
    if (e == hipSuccess && d_send && rows) {
        if (rows > cap_rows) {
            (void)hipFree(d_owner);
            (void)hipFree(d_aux);
            return fail(c, TSDF_EOVERFLOW, "border pack needs %llu rows", (unsigned long long)rows);
        }
        e = hipMalloc(&d_rows, rows * 4);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_aux + MAX_WORLD, cursor, sizeof cursor, hipMemcpyHostToDevice,
                               c->stream);
        if (e == hipSuccess)
            e = launch_border_pack(c->T, c->Pl, c->R.bg, (uint32_t)nb, rank, d_owner,
                                   d_aux + MAX_WORLD, d_rows, (uint32_t)rows, d_send, reset,
                                   c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    if (e == hipSuccess && keep_rows && d_rows) {  // handed to the caller
        *keep_rows = d_rows;
        *kept = rows;
        d_rows = nullptr;
    }
    for (void* q : {(void*)d_owner, (void*)d_aux, (void*)d_rows})
        if (q) (void)hipFree(q);
    if (e != hipSuccess) return fail(c, TSDF_EHIP, "border pack: %s", hipGetErrorString(e));
    return TSDF_OK;
}

static bool border_busy(tsdf_ctx* c) {
    if (!c->brd_open) return false;
    fail(c, TSDF_EINVAL, "a border reduce is open on this context: commit or abort it first "
                         "(tsdf_border_commit_device)");
    return true;
}

extern "C" {

// ABI v9: the pack no longer resets the sent bricks -- their mass stays here until
// tsdf_border_commit_device(ctx, 1) after the collective and every rank's merge succeeded; an
// abort keeps it.  The call opens the context's border transaction when it packs rows.
int tsdf_border_pack_device(tsdf_ctx* c, const uint64_t* d_all_keys, const uint64_t* counts,
                            uint64_t stride, uint32_t world, uint32_t rank, uint32_t* d_send,
                            uint64_t cap_rows, uint64_t* send_counts) {
    if (!c) return TSDF_EINVAL;
    if (c->brd_n_sent)
        return fail(c, TSDF_EINVAL, "border pack: the open reduce has packed already (commit first)");
    HIPCHK(c, hipSetDevice(c->device));
    uint32_t* rows = nullptr;
    uint64_t n = 0;
    const int rc = border_pack_impl(c, d_all_keys, counts, stride, world, rank, d_send, cap_rows,
                                    send_counts, false, d_send ? &rows : nullptr, &n);
    if (rc) return rc;
    if (d_send) {
        c->brd_open = true;
        c->brd_sent = rows;
        c->brd_n_sent = n;
    }
    return TSDF_OK;
}

// The owner's merge of received tiles; the bricks it touches are snapshot first (ABI v9) so an
// aborted reduce restores them.
int tsdf_border_merge_device(tsdf_ctx* c, const uint32_t* d_recv, const uint64_t* recv_counts,
                             uint32_t world) {
    if (!c) return TSDF_EINVAL;
    if (!recv_counts || world == 0 || world > TSDF_MAX_WORLD)
        return fail(c, TSDF_EINVAL, "bad world or null counts");
    uint64_t total = 0;
    for (uint32_t r = 0; r < world; r++) total += recv_counts[r];
    c->brd_open = true;  // a merge is part of the reduce even when this rank received nothing
    if (!total) return TSDF_OK;
    if (!d_recv) return fail(c, TSDF_EINVAL, "null tile buffer");
    int rc = drain(c);
    if (rc) return rc;
    uint32_t* bk = nullptr;
    HIPCHK(c, hipMalloc(&bk, total * TSDF_TILE_WORDS * 4));
    // the backup joins the abort's restore list only once its snapshot is launched (a
    // failed launch left uninitialised rows for the restore to write over held bricks)
    {
        const hipError_t e = launch_border_snapshot(c->T, c->Pl, d_recv, total, bk, c->stream);
        if (e != hipSuccess) {
            (void)hipFree(bk);
            return fail(c, TSDF_EHIP, "border snapshot: %s", hipGetErrorString(e));
        }
    }
    c->brd_backup.push_back({bk, total});
    uint64_t row = 0;
    for (uint32_t r = 0; r < world; r++) {  // sources in ascending rank order
        if (recv_counts[r])
            HIPCHK(c, launch_border_merge(c->T, c->Pl, d_recv + row * TSDF_TILE_WORDS,
                                          recv_counts[r], c->G, merge_cap(c), c->stream));
        row += recv_counts[r];
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return tsdf_sync(c);
}

// ABI v9: close the context's border transaction.  commit = 1 (the collective and EVERY rank's
// merge succeeded): the bricks this rank sent are reset to the background -- their mass now lives
// at their owners.  commit = 0 (abort): the bricks the merges touched are written back as they
// were, the sent bricks keep their mass; the field is the one before the reduce, bit for bit.
int tsdf_border_commit_device(tsdf_ctx* c, int32_t commit) {
    if (!c) return TSDF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    hipError_t e = hipSuccess;
    if (commit) {
        if (c->brd_n_sent)
            e = launch_border_reset(c->Pl, c->R.bg, c->brd_sent, (uint32_t)c->brd_n_sent, c->stream);
    } else {
        for (size_t k = c->brd_backup.size(); k-- > 0 && e == hipSuccess;)
            e = launch_border_restore(c->T, c->Pl, c->brd_backup[k].first, c->brd_backup[k].second,
                                      c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess)  // the transaction stays open: the caller may retry
        return fail(c, TSDF_EHIP, "border %s: %s", commit ? "commit" : "abort",
                    hipGetErrorString(e));
    if (c->brd_sent) (void)hipFree(c->brd_sent);
    c->brd_sent = nullptr;
    c->brd_n_sent = 0;
    for (auto& b : c->brd_backup) (void)hipFree(b.first);
    c->brd_backup.clear();
    c->brd_open = false;
    return TSDF_OK;
}

// ---- one process, several GPUs (SURVEY §8b's num_gpus / device_ids) ------------------------------

int tsdf_create_sharded(const tsdf_params* p, uint32_t n, const int32_t* device_ids, tsdf_ctx** out) {
    if (!p || !out || n == 0 || n > TSDF_MAX_WORLD) return TSDF_EINVAL;
    int dev0 = 0;
    if (hipGetDevice(&dev0) != hipSuccess) dev0 = -1;  // the caller's device, restored at the end
    for (uint32_t k = 0; k < n; k++) out[k] = nullptr;
    int rc = TSDF_OK;
    for (uint32_t k = 0; k < n && rc == TSDF_OK; k++) {
        tsdf_params q = *p;
        q.device_id = device_ids ? device_ids[k] : (int32_t)k;
        q.n_sectors = n > 1 ? n : 0;
        q.sector = k;
        rc = tsdf_create(&q, &out[k]);
        if (rc) {
            for (uint32_t j = 0; j < k; j++) {
                tsdf_destroy(out[j]);
                out[j] = nullptr;
            }
        }
    }
    // peer access between every pair of distinct devices that supports it, so the input fan-out
    // (tsdf_integrate_sectors) and the border reduce's tile copies go GPU to GPU over xGMI
    for (uint32_t k = 0; k < n && rc == TSDF_OK; k++) {
        tsdf_ctx* c = out[k];
        for (uint32_t j = 0; j < n; j++) {
            const int dk = c->device, dj = out[j]->device;
            if (dk == dj) {
                c->peer_mask |= 1ull << j;
                continue;
            }
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, dk, dj) != hipSuccess || !can) continue;
            if (hipSetDevice(dk) != hipSuccess) continue;
            const hipError_t e = hipDeviceEnablePeerAccess(dj, 0);
            if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) c->peer_mask |= 1ull << j;
            (void)hipGetLastError();  // an already-enabled pair leaves its error code behind
        }
    }
    if (dev0 >= 0) (void)hipSetDevice(dev0);  // the caller's device as it was
    return rc;
}

}  // extern "C"

// Tiles of `rows` rows from context src's device buffer to context dst's (xGMI peer copy, or a
// device copy when both share a GPU)
static hipError_t copy_tiles(tsdf_ctx* dst, uint32_t* d_dst, tsdf_ctx* src, const uint32_t* d_src,
                             uint64_t rows) {
    const size_t bytes = rows * TSDF_TILE_WORDS * 4;
    if (!bytes) return hipSuccess;
    return src->device == dst->device ? hipMemcpy(d_dst, d_src, bytes, hipMemcpyDeviceToDevice)
                                      : hipMemcpyPeer(d_dst, dst->device, d_src, src->device, bytes);
}

// Device buffers of several contexts, freed on their devices at scope end.
struct DevBufs {
    std::vector<std::pair<int, void*>> v;
    int get(tsdf_ctx* c, size_t bytes, void** p) {
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipMalloc(p, std::max<size_t>(bytes, 16)));
        v.push_back({c->device, *p});
        return TSDF_OK;
    }
    ~DevBufs() {
        for (auto& q : v) {
            (void)hipSetDevice(q.first);
            (void)hipFree(q.second);
        }
    }
};

// A failure in a multi-context call: the failing context holds the message, the first gets a copy
static int first_error(tsdf_ctx* const* ctxs, uint32_t n, int rc) {
    for (uint32_t k = 1; k < n && ctxs[0]->err.empty(); k++) ctxs[0]->err = ctxs[k]->err;
    return rc;
}

extern "C" {

// The border reduce of tsdf_brick_keys_device / tsdf_border_pack_device / tsdf_border_merge_device
// among the contexts of one process: the keys meet on the host, and each source's tiles go to
// their owner's GPU with one peer copy per (source, owner) pair (xGMI between GPUs; a device copy
// when two contexts share a GPU).  Transactional (ABI v9): every context packs without
// resetting and every owner snapshots before it merges; only when every copy and merge succeeded
// are the sent bricks reset (commit), otherwise every context is rolled back (abort), so a failed
// reduce neither loses nor double-counts mass.  Synchronous.
int tsdf_border_reduce_local(tsdf_ctx* const* ctxs, uint32_t n, uint64_t* bricks_moved) {
    if (!ctxs || n == 0 || n > TSDF_MAX_WORLD) return TSDF_EINVAL;
    for (uint32_t k = 0; k < n; k++)
        if (!ctxs[k]) return TSDF_EINVAL;
    if (bricks_moved) *bricks_moved = 0;
    if (n == 1) return TSDF_OK;
    for (uint32_t k = 0; k < n; k++)
        if (border_busy(ctxs[k])) return first_error(ctxs, n, TSDF_EINVAL);
    int dev0 = 0;
    if (hipGetDevice(&dev0) != hipSuccess) dev0 = -1;
    int rc = TSDF_OK;
    {
        DevBufs bufs;
        // 1. every context's keys, gathered on the host
        std::vector<uint64_t> counts(n, 0);
        std::vector<std::vector<uint64_t>> hkeys(n);
        for (uint32_t k = 0; k < n && !rc; k++) {
            tsdf_ctx* c = ctxs[k];
            uint64_t nb = 0;
            rc = pool_bricks(c, &nb);
            void* d = nullptr;
            if (!rc) rc = bufs.get(c, nb * 8, &d);
            if (!rc) rc = tsdf_brick_keys_device(c, static_cast<uint64_t*>(d), nb, &counts[k]);
            if (!rc) {
                hkeys[k].resize(counts[k]);
                if (counts[k] &&
                    hipMemcpy(hkeys[k].data(), d, counts[k] * 8, hipMemcpyDeviceToHost) != hipSuccess)
                    rc = fail(c, TSDF_EHIP, "border reduce: key read-back failed");
            }
        }
        uint64_t stride = 1;
        for (uint32_t k = 0; k < n; k++) stride = std::max(stride, counts[k]);
        std::vector<uint64_t> all(stride * n, ~0ull);
        for (uint32_t k = 0; k < n; k++)
            std::copy(hkeys[k].begin(), hkeys[k].end(), all.begin() + k * stride);
        // 2. each context packs the bricks a lower rank owns (no reset: the transaction)
        std::vector<uint32_t*> send(n, nullptr);
        std::vector<std::vector<uint64_t>> sc(n, std::vector<uint64_t>(n, 0));
        for (uint32_t k = 0; k < n && !rc; k++) {
            tsdf_ctx* c = ctxs[k];
            void *dk = nullptr, *ds = nullptr;
            rc = bufs.get(c, all.size() * 8, &dk);
            if (!rc && hipMemcpy(dk, all.data(), all.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
                rc = fail(c, TSDF_EHIP, "border reduce: key upload failed");
            if (!rc) rc = bufs.get(c, counts[k] * TSDF_TILE_WORDS * 4, &ds);
            if (!rc)
                rc = tsdf_border_pack_device(c, static_cast<uint64_t*>(dk), counts.data(), stride, n,
                                             k, static_cast<uint32_t*>(ds), counts[k], sc[k].data());
            send[k] = static_cast<uint32_t*>(ds);
        }
        // 3. every owner d receives block d of every source, sources ascending; 4. merge
        uint64_t moved = 0;
        for (uint32_t d = 0; d < n && !rc; d++) {
            tsdf_ctx* c = ctxs[d];
            std::vector<uint64_t> rcnt(n, 0);
            uint64_t total = 0;
            for (uint32_t r = 0; r < n; r++) {
                rcnt[r] = sc[r][d];
                total += rcnt[r];
            }
            if (!total) continue;
            void* dr = nullptr;
            rc = bufs.get(c, total * TSDF_TILE_WORDS * 4, &dr);
            uint64_t row = 0;
            for (uint32_t r = 0; r < n && !rc; r++) {
                if (!rcnt[r]) continue;
                uint64_t off = 0;
                for (uint32_t q = 0; q < d; q++) off += sc[r][q];
                const hipError_t e = copy_tiles(c, static_cast<uint32_t*>(dr) + row * TSDF_TILE_WORDS,
                                                ctxs[r], send[r] + off * TSDF_TILE_WORDS, rcnt[r]);
                if (e != hipSuccess)
                    rc = fail(c, TSDF_EHIP, "border reduce: tile copy: %s", hipGetErrorString(e));
                row += rcnt[r];
            }
            if (!rc) rc = tsdf_border_merge_device(c, static_cast<uint32_t*>(dr), rcnt.data(), n);
            moved += total;
        }
        // 5. commit everywhere when everything succeeded, else roll every context back
        const int commit = rc == TSDF_OK ? 1 : 0;
        for (uint32_t k = 0; k < n; k++) {
            const int crc = tsdf_border_commit_device(ctxs[k], commit);
            if (crc && !rc) rc = crc;
        }
        if (!rc && bricks_moved) *bricks_moved = moved;
    }
    if (dev0 >= 0) (void)hipSetDevice(dev0);
    return rc ? first_error(ctxs, n, rc) : TSDF_OK;
}

// ---- mesh halo (ABI v9): meshing a sector-sharded field, one owner per cube ---------------------

// The keys of the bricks this context needs to mesh its own and does not observe: for every brick
// holding an observed voxel, its 7 +x / +y / +z neighbours that hold none here (sorted, unique).
int tsdf_halo_keys_device(tsdf_ctx* c, uint64_t* d_keys, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return TSDF_EINVAL;
    *n_out = 0;
    uint64_t nb = 0;
    int rc = drain(c);
    if (!rc) rc = pool_bricks(c, &nb);
    if (rc) return rc;
    if (!nb) return TSDF_OK;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<uint64_t> keys(nb);
    std::vector<uint32_t> obs(nb);
    uint32_t* d_obs = nullptr;
    hipError_t e = hipMalloc(&d_obs, nb * 4);
    if (e == hipSuccess) e = launch_brick_observed(c->Pl, (uint32_t)nb, d_obs, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(obs.data(), d_obs, nb * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(keys.data(), c->T.brick_keys, nb * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (d_obs) (void)hipFree(d_obs);
    if (e != hipSuccess) return fail(c, TSDF_EHIP, "halo keys: %s", hipGetErrorString(e));
    std::vector<uint64_t> have;
    for (uint64_t i = 0; i < nb; i++)
        if (obs[i]) have.push_back(keys[i]);
    std::sort(have.begin(), have.end());
    std::vector<uint64_t> need;
    for (uint64_t k : have) {
        const int64_t bx = (int64_t)(k & 0x1FFFFF), by = (int64_t)((k >> 21) & 0x1FFFFF),
                      bz = (int64_t)((k >> 42) & 0x1FFFFF);
        for (int d = 1; d < 8; d++) {
            const int64_t nx = bx + (d & 1), ny = by + ((d >> 1) & 1), nz = bz + (d >> 2);
            if (nx > 0x1FFFFF || ny > 0x1FFFFF || nz > 0x1FFFFF) continue;
            const uint64_t q = (uint64_t)nx | ((uint64_t)ny << 21) | ((uint64_t)nz << 42);
            if (!std::binary_search(have.begin(), have.end(), q)) need.push_back(q);
        }
    }
    std::sort(need.begin(), need.end());
    need.erase(std::unique(need.begin(), need.end()), need.end());
    *n_out = need.size();
    if (need.size() > cap)
        return fail(c, TSDF_EOVERFLOW, "halo keys need %llu entries", (unsigned long long)need.size());
    if (need.empty()) return TSDF_OK;
    if (!d_keys) return fail(c, TSDF_EINVAL, "null key buffer");
    HIPCHK(c, hipMemcpy(d_keys, need.data(), need.size() * 8, hipMemcpyHostToDevice));
    return TSDF_OK;
}

// The tiles of the requested bricks (device keys) that this context observes, into d_send (device,
// cap_rows rows; row order unspecified); *n_rows = the tiles (TSDF_EOVERFLOW above cap_rows).
int tsdf_halo_pack_device(tsdf_ctx* c, const uint64_t* d_req, uint64_t n_req, uint32_t* d_send,
                          uint64_t cap_rows, uint64_t* n_rows) {
    if (!c || !n_rows) return TSDF_EINVAL;
    *n_rows = 0;
    if (!n_req) return TSDF_OK;
    if (!d_req || !d_send) return fail(c, TSDF_EINVAL, "null buffer");
    if (n_req >= 0xFFFFFFFFull || cap_rows >= 0xFFFFFFFFull)
        return fail(c, TSDF_EINVAL, "too many halo requests");
    int rc = drain(c);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    uint32_t* d_n = nullptr;
    uint32_t nr = 0;
    hipError_t e = hipMalloc(&d_n, 4);
    if (e == hipSuccess) e = hipMemsetAsync(d_n, 0, 4, c->stream);
    if (e == hipSuccess)
        e = launch_halo_pack(c->T, c->Pl, d_req, (uint32_t)n_req, d_send, (uint32_t)cap_rows, d_n,
                             c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&nr, d_n, 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (d_n) (void)hipFree(d_n);
    if (e != hipSuccess) return fail(c, TSDF_EHIP, "halo pack: %s", hipGetErrorString(e));
    *n_rows = nr;
    if (nr > cap_rows) return fail(c, TSDF_EOVERFLOW, "halo pack needs %u rows", nr);
    return TSDF_OK;
}

// tsdf_extract_mesh_table over this context's bricks, with the halo tiles (device) looked up first
// for their neighbours: after a border reduce, the union of every context's mesh is the mesh of
// the union field, each cube meshed by the owner of its min voxel's brick.
int tsdf_extract_mesh_halo(tsdf_ctx* c, float min_weight, int32_t table, const uint32_t* d_halo,
                           uint64_t n_halo, float* tri, uint64_t cap, uint64_t* n_tri) {
    return mesh_impl(c, min_weight, table, d_halo, n_halo, tri, cap, n_tri);
}

// The sharded mesh among the contexts of one process (2 cm + marching cubes on N
// GPUs): border reduce, halo exchange with one peer copy per (holder, requester) pair, one mesh per
// context; tri holds the contexts' soups one after another in context order (tri == NULL: count).
int tsdf_extract_mesh_local(tsdf_ctx* const* ctxs, uint32_t n, float min_weight, int32_t table,
                            float* tri, uint64_t cap, uint64_t* n_tri) {
    if (!ctxs || n == 0 || n > TSDF_MAX_WORLD || !n_tri) return TSDF_EINVAL;
    for (uint32_t k = 0; k < n; k++)
        if (!ctxs[k]) return TSDF_EINVAL;
    *n_tri = 0;
    if (n == 1) return tsdf_extract_mesh_table(ctxs[0], min_weight, table, tri, cap, n_tri);
    int rc = tsdf_border_reduce_local(ctxs, n, nullptr);
    if (rc) return rc;
    int dev0 = 0;
    if (hipGetDevice(&dev0) != hipSuccess) dev0 = -1;
    {
        DevBufs bufs;
        // every context's requests
        std::vector<void*> req(n, nullptr);
        std::vector<uint64_t> nreq(n, 0);
        for (uint32_t k = 0; k < n && !rc; k++) {
            rc = tsdf_halo_keys_device(ctxs[k], nullptr, 0, &nreq[k]);
            if (rc == TSDF_EOVERFLOW) rc = TSDF_OK;
            if (!rc) rc = bufs.get(ctxs[k], nreq[k] * 8, &req[k]);
            uint64_t got = 0;
            if (!rc) rc = tsdf_halo_keys_device(ctxs[k], static_cast<uint64_t*>(req[k]), nreq[k], &got);
        }
        // holder j packs for requester k on j's GPU; the tiles go to k's halo buffer
        std::vector<void*> halo(n, nullptr);
        std::vector<uint64_t> nh(n, 0);
        for (uint32_t k = 0; k < n && !rc; k++) {
            if (!nreq[k]) continue;
            rc = bufs.get(ctxs[k], nreq[k] * TSDF_TILE_WORDS * 4, &halo[k]);
            for (uint32_t j = 0; j < n && !rc; j++) {
                if (j == k) continue;
                void *dq = nullptr, *ds = nullptr;
                rc = bufs.get(ctxs[j], nreq[k] * 8, &dq);
                if (!rc) {
                    const hipError_t e =
                        ctxs[j]->device == ctxs[k]->device
                            ? hipMemcpy(dq, req[k], nreq[k] * 8, hipMemcpyDeviceToDevice)
                            : hipMemcpyPeer(dq, ctxs[j]->device, req[k], ctxs[k]->device, nreq[k] * 8);
                    if (e != hipSuccess)
                        rc = fail(ctxs[j], TSDF_EHIP, "halo: key copy: %s", hipGetErrorString(e));
                }
                if (!rc) rc = bufs.get(ctxs[j], nreq[k] * TSDF_TILE_WORDS * 4, &ds);
                uint64_t rows = 0;
                if (!rc)
                    rc = tsdf_halo_pack_device(ctxs[j], static_cast<uint64_t*>(dq), nreq[k],
                                               static_cast<uint32_t*>(ds), nreq[k] - nh[k], &rows);
                if (!rc) {
                    const hipError_t e = copy_tiles(
                        ctxs[k], static_cast<uint32_t*>(halo[k]) + nh[k] * TSDF_TILE_WORDS, ctxs[j],
                        static_cast<uint32_t*>(ds), rows);
                    if (e != hipSuccess)
                        rc = fail(ctxs[k], TSDF_EHIP, "halo: tile copy: %s", hipGetErrorString(e));
                }
                nh[k] += rows;
            }
        }
        // one mesh per context, soups concatenated
        uint64_t total = 0;
        for (uint32_t k = 0; k < n && !rc; k++) {
            uint64_t nt = 0;
            float* out = tri && total <= cap ? tri + 9 * total : nullptr;
            rc = mesh_impl(ctxs[k], min_weight, table, static_cast<uint32_t*>(halo[k]), nh[k], out,
                           tri && total <= cap ? cap - total : 0, &nt);
            if (rc == TSDF_EOVERFLOW) rc = TSDF_OK;  // the total decides below
            total += nt;
        }
        *n_tri = total;
        if (!rc && tri && total > cap)
            rc = fail(ctxs[0], TSDF_EOVERFLOW, "mesh has %llu triangles", (unsigned long long)total);
    }
    if (dev0 >= 0) (void)hipSetDevice(dev0);
    return rc ? first_error(ctxs, n, rc) : TSDF_OK;
}

}  // extern "C"
