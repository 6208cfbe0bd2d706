// tsdf_device.h — device-side data layout shared by the kernels and the C-ABI host code.
//
// The unit of GPU work is a BATCH of up to MAX_BATCH consecutive scans.  Ray
// walking, brick allocation and bucketing do not depend on the field, so they run for every ray of
// the batch at once; only the per-scan fuse has a cross-scan order, and k_integrate applies it scan
// by scan inside each brick — bitwise the same field as integrating the scans one at a time.
//
// HBM layout:
//   Table   open-addressing brick hash, capacity 2^k >= 2 * max_bricks, linear probing:
//           keys[cap]  u64  packed brick coords (21 bits/axis, biased by 2^20); EMPTY = ~0
//           slots[cap] u32  brick-pool slot (UNASSIGNED until the batch's compaction pass)
//           touched[cap] u32  1 if the batch touches the brick (k_count sets, k_compact clears)
//           cell[cap * cell_stride] u32  per (brick, scan) SAMPLE counts (k_count), then the
//                                        absolute position of those samples (k_compact);
//                                        single walk: u64 (samples | spans << 32), then (relative
//                                        sample prefix | absolute span position << 32)
//   Pool    sdf[max_bricks][512] f32, weight[max_bricks][512] f32 — voxel l = z*64 + y*8 + x;
//           brick_keys[max_bricks] u64 (slot -> key, for export)
//   Work    pair[max_batch_points * maxp] u32    per-ray pair codes (see PAIR_*)
//           blk[n_blocks * HCAP] uint4          per-block dense run list (tidx, cell rank -> sample
//                                               position, offset of the run in the block, samples)
//           fb[..] uint4                        fallback pairs (block's LDS hash full)
//           smp[..] uint2                       the batch's samples: (sdf bits, scan << 9 | voxel),
//                                               per brick contiguous and scan-ordered
//           active[..] uint4                    bricks touched by the batch: (table index, pool
//                                               slot, sample segment offset, sample count)
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tsdf {

constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr uint32_t UNASSIGNED = 0xFFFFFFFFu;    // table entry inserted, pool slot not yet given
constexpr uint32_t INVALID_SLOT = 0xFFFFFFFEu;  // pool exhausted for this brick
constexpr uint32_t NO_PAIR = 0xFFFFFFFFu;
constexpr int BRICK_VOX = 512;
constexpr int BRICK_COORD_BIAS = 1 << 20;
constexpr int VOX_LIMIT = 1 << 23;  // |voxel index| < 2^23 on every axis (same as the oracle)
constexpr int MAX_DDA_STEPS = 1 << 20;
constexpr int MAX_BATCH = 512;         // scans per batch
#ifndef TSDF_RPB
#define TSDF_RPB 1024
#endif
#ifndef TSDF_HCAP
#define TSDF_HCAP 2048
#endif
constexpr int RPB = TSDF_RPB;          // rays per k_count / k_place block (one scan per block)
constexpr int HCAP = TSDF_HCAP;        // LDS brick-hash slots per k_count block (~300-800 used)
constexpr int LDS_PROBES = 64;         // probe limit before a pair takes the global fallback
constexpr int MAX_IN_BRICK = 22;       // a line visits at most 8+8+8-2 voxels of an 8^3 brick
// k_place's LDS staging: samples per workgroup (6 B each), the bitmap words of run starts, and the
// staging plan k_count hands over per half block (Work::plan: the bitmap words, their exclusive
// popcount prefix as u16 per word, then the staged sample count).  5600 samples hold nearly a whole
// half block's samples (~4.8 k on average) at 50 KB of LDS, three workgroups per CU: fewer samples
// go out as scattered 8-B stores, which cost more than the fourth workgroup per CU bought
// (k_place 0.407 -> 0.390 ms against 3800 samples / four workgroups; 6000 no longer fits three)
#ifndef TSDF_PLC_STAGE
#define TSDF_PLC_STAGE 5600
#endif
constexpr int PLC_STAGE = TSDF_PLC_STAGE;
// Voxblox with 1/z^2 weights (sem 3): the sample's ray is staged beside it (8 B a sample; the
// weight is formed at copy-out from a per-ray LDS table), and its rays carry more samples, so it
// stages more: two workgroups per CU with nearly a whole half block staged beat three with less
// (round 5: 4352 / 4096 / 5600 / 7744 samples).  k_count<3>'s plan covers it.
#ifndef TSDF_PLC_STAGE3
#define TSDF_PLC_STAGE3 7744
#endif
constexpr int PLC_STAGE3 = TSDF_PLC_STAGE3;
// staging capacity and plan bitmap words of semantics SEM
__host__ __device__ constexpr int plan_cap(int sem) { return sem == 3 ? PLC_STAGE3 : PLC_STAGE; }
__host__ __device__ constexpr int plan_words(int sem) { return (plan_cap(sem) + 31) / 32; }
constexpr int PLC_WORDS = plan_words(0);
constexpr int PLC_WORDS_MAX = plan_words(0) > plan_words(3) ? plan_words(0) : plan_words(3);
constexpr int PLAN_STRIDE = ((PLC_WORDS_MAX + (PLC_WORDS_MAX + 1) / 2 + 1) + 15) & ~15;
// single-walk front end (tsdf_walk.hip): rays per k_walk workgroup (one per lane; half an RPB
// block) and samples per span record
constexpr int WLK_THREADS = RPB / 2;
constexpr int SPAN = 4;

// pair codes (one u32 per (ray, k-th brick) slot); count = the pair's in-brick samples
//   local:    bit 31 = 0 | count << 26 | lid << 15 | local sample offset  (lid < HCAP,
//             offset < RPB * MAX_IN_BRICK < 2^15)
//   fallback: bit 31 = 1 | count << 26 | fb index                         (fb index < 2^26)
//   dead:     PAIR_DEAD (the pair was dropped on a capacity overflow; keeps k_place's pair index
//             aligned with k_count's)
//   none:     NO_PAIR
constexpr uint32_t PAIR_FB = 0x80000000u;
constexpr uint32_t PAIR_DEAD = 0xFFFFFFFEu;  // count field 31: never a real pair
constexpr int PAIR_CNT_SHIFT = 26;
constexpr int PAIR_LID_SHIFT = 15;
static_assert(RPB * MAX_IN_BRICK < (1 << PAIR_LID_SHIFT), "local sample offset overflows");
static_assert(HCAP <= (1 << (PAIR_CNT_SHIFT - PAIR_LID_SHIFT)), "lid overflows");

// overflow bits (sticky until tsdf_sync reads them)
constexpr uint32_t OVF_TABLE = 1u, OVF_POOL = 2u, OVF_PAIRS = 4u, OVF_ACTIVE = 8u, OVF_FB = 16u,
                   OVF_SMP = 32u,  // the batch's samples exceed the sample list (single walk:
                                   // the workgroup regions)
                   OVF_SPN = 64u,  // single walk: the batch's spans exceed the span list
                   OVF_MG = 128u;  // merged pre-pass: a bucket holds more distinct bundle keys
                                   // than k_mg_group's LDS table (a scan of more than ~2^22
                                   // points; not a growable capacity)
// a border tile whose brick this context lacks (tsdf_border_merge_device; sticky like OVF_*)
constexpr uint32_t ERR_MERGE_KEY = 1u << 8;

// per-context constants of the ray model
struct RayConst {
    float vs, inv_vs, tau, min_range, max_range;
    int carving;
    // backend semantics (TSDF_SEM_*) and the Voxblox mode's constants
    int sem, allow_clear, dropoff;
    float max_weight;
    float bg;        // background distance of unobserved voxels: tau (VDBFusion) or 0 (Voxblox)
    float tau_m_vs;  // tau - vs (Voxblox dropoff denominator)
    int band_vox;    // bound on any axis' index span of a ray's walk (+ margin), in voxels
    // squared-distance bounds bracketing tau by 2^-20 relative: d2 < tau2_lo implies
    // sqrt_rn(d2) < tau, d2 > tau2_hi implies sqrt_rn(d2) > tau (voxel_gate skips the sqrt)
    float tau2_lo, tau2_hi;
    // azimuth-sector sharding (tsdf_params.n_sectors > 1): keep rays whose pseudo-angle lies in
    // [sec_lo, sec_hi), or outside [sec_hi, sec_lo) when the sector wraps past 4 (sec_wrap)
    int sec_on, sec_wrap;
    float sec_lo, sec_hi;
    // TSDF_SEM_VDBFUSION_F64: vs / 2 and 1/vs in double, and the gate's threshold
    // on the squared distance behind the hit: (float)sqrt(d2) < tau  <=>  d2 < gate_d2.  vs / 2 is
    // GetVoxelCenter's half voxel, precomputed so the walk reads it as a scalar kernel argument
    // (formed per voxel it cost a double multiply and two readfirstlanes at every DDA step)
    double hvs_d, inv_s_d, gate_d2;
    // Voxblox 1/z^2 sample weights (tsdf_params.depth_weight; sem 3 internally, each sample record
    // carrying its weight: smp_store / smp_load)
    int depth_w;
    float w0_cap;  // cap of a sample's 1/z^2 weight: min(max_weight, 2^16) (TSDF_W0_CAP)
    // Voxblox MergedTsdfIntegrator (tsdf_params.voxblox_method; sem 3): per ray slot of the
    // batch, its bundle's weight (< 0: a clearing bundle; 0: no bundle ray in this slot), set per
    // launch to the bundling pre-pass's output (tsdf_merged.hip); null otherwise
    const float* ray_w;
};

// fp32 pseudo-angle of (x, y) in [0, 4), monotone in atan2 (include/tsdf_hip.h tsdf_sector_of):
// one IEEE division, so host and GPU agree bit for bit (built with -ffp-contract=off)
__host__ __device__ inline float pseudo_angle(float x, float y) {
    if (y >= 0.0f) {
        if (x >= 0.0f) {
            const float d = x + y;
            return d > 0.0f ? y / d : 0.0f;
        }
        return 1.0f - x / (y - x);
    }
    if (x < 0.0f) return 2.0f - y / (-x - y);
    return 3.0f + x / (x - y);
}

__host__ __device__ inline bool in_sector(const RayConst& R, float dx, float dy) {
    if (!R.sec_on) return true;
    const float a = pseudo_angle(dx, dy);
    return R.sec_wrap ? (a >= R.sec_lo || a < R.sec_hi) : (a >= R.sec_lo && a < R.sec_hi);
}

// One batch: scan s = points [s[s].off, s[s+1].off) seen from s[s].ox/oy/oz (fp32; the origin as
// given in odx/ody/odz, TSDF_SEM_VDBFUSION_F64); k_count / k_place blocks [s[s].blk, s[s+1].blk)
// cover scan s, RPB rays each.  The host fills a BatchDesc; launch() uploads its n_scans + 1 used
// records to a device ring slot, and the kernels get a BatchRef to them (a batch of up to 512
// scans does not fit the kernel-argument segment).
// zx, zy, zz: the sensor's z axis in the world frame (Voxblox's 1/z^2 weight, RayConst::depth_w)
// xoff (ABI v10): the scan's points are d_xyz[3 (i + xoff)] for its batch rays i -- nonzero only
// for device batches of a TSDF_SECTOR_RULE_INDEX context, whose scans' shares are not contiguous
struct ScanRec {
    uint32_t off, blk;
    float ox, oy, oz;
    float zx;
    double odx, ody, odz;
    float zy, zz;
    uint32_t xoff, pad;
};
static_assert(sizeof(ScanRec) == 64, "ScanRec layout");
struct BatchDesc {
    uint32_t n_scans;
    uint32_t n_blocks;
    ScanRec s[MAX_BATCH + 1];
};
struct BatchRef {
    uint32_t n_scans;
    uint32_t n_blocks;
    const ScanRec* __restrict__ s;
};

struct Table {
    uint64_t* keys;
    uint32_t* slots;
    uint32_t* touched;  // set (plain store) by k_count for every brick the batch touches
    uint32_t* cell;
    uint64_t* brick_keys;  // pool slot -> key
    uint64_t mask;
    uint32_t max_bricks;
    uint32_t cell_stride;  // cells per row: u32 >= max_batch, multiple of 4 (two walks); u64 >=
                           // max_batch + 1, even (single walk: a totals cell after the last scan)
};

struct Pool {
    float* sdf;
    float* weight;
};

struct Work {
    uint32_t* pair;
    uint4* blk;      // n_blocks * 2 * HCAP: per k_count workgroup and half its DENSE run list (table index,
                     // rank in the (brick, scan) cell,
                     // run offset in the workgroup's sample order, run samples | LDS slot << 16)
    uint32_t* blk_n; // n_blocks * 2: runs in each list
    uint32_t* plan;  // n_blocks * 2 * PLAN_STRIDE: k_place's staging plan per half (k_count)
    uint4* fb;       // fallback pairs: (tidx, scan, rank, 0)
    uint2* smp;  // x = truncated sdf (f32 bits), y = scan << 9 | local voxel; Voxblox 1/z^2 (sem 3):
                 // 12-B records (x, y, weight f32 bits), smp_store / smp_load
    uint4* active;  // (h, slot, toff, cnt) per active brick (k_compact)
    uint4* active_ord;  // the same records, largest size class first (k_order; k_integrate's list)
    uint32_t* ord_hist; // per (slice, size class): counts [64][32], then first positions [64][32]
    uint4* cagg;    // k_compact: per table chunk (touched bricks, samples, new bricks), then bases
    uint32_t* act;  // sector sharding: the k_count blocks holding a ray of this GPU's sector (n_act)
    uint4* rsv;     // TSDF_CNT_SPLIT variant: per k_count block, its distinct bricks for k_resolve
    uint32_t* rsv_n;  // (key, n0 | n1 << 16, run-list index 0 | index 1 << 11 | scan << 22); count
    uint32_t* spn;  // single walk: span records (sample position | (samples - 1) << 30), per brick
                    // contiguous and scan-ordered (k_spans)
    uint32_t maxp;        // pair slots per ray
    uint32_t max_active;  // capacity of `active`
    uint32_t max_fb;      // capacity of `fb`
    uint32_t max_smp;     // capacity of smp
    uint32_t max_spn;     // capacity of spn
};

// Sample records: 8 B (sdf bits, scan << 9 | voxel); Voxblox 1/z^2 (sem 3) 12 B with the sample's
// weight, one store and one load per sample instead of a parallel weight array (round 5)
constexpr size_t smp_bytes(int sem) { return sem == 3 ? 12 : 8; }
template <int SEM>
__device__ __forceinline__ void smp_store(const Work& W, uint32_t i, float s, uint32_t tl, float w) {
    if constexpr (SEM == 3)
        reinterpret_cast<uint3*>(W.smp)[i] = make_uint3(__float_as_uint(s), tl, __float_as_uint(w));
    else
        W.smp[i] = make_uint2(__float_as_uint(s), tl);
}
template <int SEM>
__device__ __forceinline__ uint2 smp_load(const Work& W, uint32_t i, float& w) {
    if constexpr (SEM == 3) {
        const uint3 v = reinterpret_cast<const uint3*>(W.smp)[i];
        w = __uint_as_float(v.z);
        return make_uint2(v.x, v.y);
    } else {
        return W.smp[i];
    }
}

// per-batch counters, double-buffered by batch parity (zeroed by k_finish at the end of a batch)
struct Counters {
    uint32_t n_active;
    uint32_t cursor;
    uint32_t n_fb;
    uint32_t ovf;  // OVF_* raised by this batch's kernels
    uint32_t n_new;  // bricks the batch allocated (k_compact_scan)
    uint32_t n_act;  // sector sharding: k_count blocks with a ray of this GPU's sector (k_sector_flags)
    uint32_t pad1[2];
    unsigned long long n_vox[8];    // sum over scans of U_vox, sharded by blockIdx & 7
    unsigned long long n_rays[8];   // valid rays
    unsigned long long n_pairs[8];
    unsigned long long n_dirty[8];  // distinct voxels updated by the batch
};

// persistent device globals (one allocation, zeroed at create)
// One finished batch, as the metrics log reports it (tsdf_set_metrics_log; k_finish writes it to
// Globals::ring[batch_id % METRIC_RING], the host drains the ring at its checks).
constexpr uint32_t METRIC_RING = 256;
struct BatchRecord {
    uint32_t batch_id, n_active, n_new, ovf;
    uint32_t committed, pool_count, pad[2];
    unsigned long long rays, pairs, vox, dirty;
};

// Capacity growth: with `retry` set (the context can still grow), a batch that
// raised an overflow — or any batch after it — does not commit: k_integrate skips its field writes
// and k_finish its stats, so the host can grow the buffers and replay the batches from `fail_id`.
struct Globals {
    uint32_t pool_count;
    uint32_t overflow;  // OVF_* of every batch since the host's last check (sticky)
    uint32_t failed;    // a batch raised an overflow since the host's last check
    uint32_t retry;     // host: failed batches will be replayed (skip their writes)
    uint32_t fail_id;   // host batch id of the first failed batch
    uint32_t pad[3];
    Counters ctr[2];
    unsigned long long tot_vox[8];  // running totals since the last stats reset (sharded)
    unsigned long long tot_rays[8];
    unsigned long long tot_pairs[8];
    unsigned long long tot_dirty[8];
    Counters last;  // the last finished batch's counters (k_finish)
    BatchRecord ring[METRIC_RING];  // per-batch records (k_finish), drained by the host's metrics log
};

enum KernelKind {
    KIND_COUNT = 0, KIND_COMPACT = 1, KIND_PLACE = 2, KIND_INTEGRATE = 3,
    KIND_WALK = 4, KIND_SPANS = 5,  // the single-walk front end
    KIND_N = 6
};

// Optional per-kernel HIP-event timing (profiling mode); implemented in tsdf_capi.cpp.
// Kernel timing through the dispatch packets: a launch given start / stop events records the
// kernel's own begin / end timestamps (hipExtLaunchKernel), with no marker packet in the stream.
// A stage of several kernels takes start on its first launch and stop on its last.
struct KTime {
    hipEvent_t start = nullptr, stop = nullptr;
};
template <typename... KArgs, typename... Args>
inline void tlaunch(void (*kern)(KArgs...), dim3 grid, dim3 block, hipStream_t st, hipEvent_t e0,
                    hipEvent_t e1, Args... args) {
    if (!e0 && !e1) {
        kern<<<grid, block, 0, st>>>(args...);
        return;
    }
    hipExtLaunchKernelGGL(kern, grid, block, 0, st, e0, e1, 0, args...);
}

struct KernelTimer {
    virtual void begin(int kind, hipStream_t st) = 0;
    virtual void end(int kind, hipStream_t st) = 0;
    virtual ~KernelTimer() {}
};

hipError_t launch_count(const float* d_xyz, const BatchRef& D, const RayConst& R, const Table& T,
                        const Work& Wk, Globals* G, int parity, hipStream_t st, const KTime& kt = {},
                        bool wide = false, bool paired = false);
// table chunks of k_compact (Work::cagg holds two uint4 per chunk)
#ifndef TSDF_CMP_CHUNK
#define TSDF_CMP_CHUNK 1024
#endif
constexpr uint32_t CMP_CHUNK = TSDF_CMP_CHUNK;
inline uint64_t compact_chunks(uint64_t cap) { return (cap + CMP_CHUNK - 1) / CMP_CHUNK; }
// Sector sharding (n_sectors > 1): which k_count blocks hold a ray of this GPU's sector; the walk
// kernels' other workgroups leave after one load.
hipError_t launch_sector_flags(const float* d_xyz, const BatchRef& D, const RayConst& R,
                               const Work& Wk, Globals* G, int parity, hipStream_t st);
// fused: the single-walk path's 64-bit cells (samples | spans << 32; after k_compact_write the
// relative sample prefix | absolute span position, with the totals at scan n_scans)
hipError_t launch_compact(const BatchRef& D, const Table& T, const Work& Wk, Globals* G,
                          int parity, bool fused, hipStream_t st, const KTime& kt = {});
// single-walk front end (tsdf_walk.hip); nstep = 16 or 32 register slots per ray
hipError_t launch_walk(const float* d_xyz, const BatchRef& D, const RayConst& R, const Table& T,
                       const Work& Wk, Globals* G, int parity, int nstep, hipStream_t st);
hipError_t launch_spans(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                        Globals* G, int parity, int nstep, hipStream_t st);
hipError_t launch_place(const float* d_xyz, const BatchRef& D, const RayConst& R, const Table& T,
                        const Work& Wk, Globals* G, int parity, hipStream_t st, const KTime& kt = {});
hipError_t launch_finish(Globals* G, int parity, uint32_t batch_id, hipStream_t st);
// bytes (a multiple of 16) from device-accessible pinned host memory to device memory, then
// *done = seq (done: device address of a pinned host word)
hipError_t launch_upload(const void* host_src, void* dst, uint32_t bytes,
                         unsigned long long* done, unsigned long long seq, hipStream_t st);
// capacity growth: re-insert pool slots [0, n) of the new table from brick_keys
hipError_t launch_rehash(const Table& T, uint32_t n, Globals* G, hipStream_t st);
// Orders the batch's active bricks by size class, largest first (k_integrate's load balance).
hipError_t launch_order(const Work& Wk, Globals* G, int parity, hipStream_t st);
// fused: samples through the span list (single walk); big: batches of more than 64 scans
// k_integrate_small: batches of at most a few scans, one wave per brick (tsdf_integrate.hip)
hipError_t launch_integrate_small(const BatchRef& D, const RayConst& R, const Table& T,
                                  const Work& Wk, const Pool& Pl, Globals* G, int parity,
                                  hipStream_t st, const KTime& kt = {});
hipError_t launch_integrate(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                            const Pool& Pl, Globals* G, int parity, bool fused, bool big,
                            hipStream_t st, const KTime& kt = {});
hipError_t launch_query_dense(const Table& T, const Pool& Pl, const int64_t lo[3], const int dims[3],
                              float bg, float* d_sdf, float* d_w, hipStream_t st);
hipError_t launch_import(const Table& T, const Pool& Pl, const int32_t* d_coords, uint32_t n,
                         const float* d_sdf, const float* d_w, uint32_t* d_tidx, Globals* G,
                         float max_w, hipStream_t st);
hipError_t launch_fill(float* p, float v, uint64_t n, hipStream_t st);
// border-brick reduce (tsdf_border.hip)
constexpr int TILE_WORDS = 1028;  // include/tsdf_hip.h TSDF_TILE_WORDS
constexpr int MAX_WORLD = 64;
struct WorldCounts { uint64_t n[MAX_WORLD]; };
// owner[slot] = the lowest rank (< rank) holding the brick, else rank
hipError_t launch_border_owner(const Table& T, uint32_t n_bricks, const uint64_t* d_all_keys,
                               const WorldCounts& counts, uint64_t stride, uint32_t rank,
                               uint32_t* d_owner, uint32_t* d_dest_n, hipStream_t st);
// rows of the bricks owned elsewhere (cursor[r] = first row of destination r), tiles packed and,
// with reset, the bricks reset to the background
hipError_t launch_border_pack(const Table& T, const Pool& Pl, float bg, uint32_t n_bricks,
                              uint32_t rank, const uint32_t* d_owner, uint32_t* d_cursor,
                              uint32_t* d_rows, uint32_t n_rows, uint32_t* d_send, bool reset,
                              hipStream_t st);
// the bricks of rows[0, n_rows) reset to the background (after a pack without reset)
hipError_t launch_border_reset(const Pool& Pl, float bg, const uint32_t* d_rows, uint32_t n_rows,
                               hipStream_t st);
// max_w: the merged weight's cap (Voxblox max_weight; +inf for VDBFusion)
hipError_t launch_border_merge(const Table& T, const Pool& Pl, const uint32_t* d_recv,
                               uint64_t n_rows, Globals* G, float max_w, hipStream_t st);
// ABI v9 border transaction: the bricks of n_rows received tiles as they are before the merge
// (tiles; key EMPTY_KEY when the brick is not held), and their restore on abort
hipError_t launch_border_snapshot(const Table& T, const Pool& Pl, const uint32_t* d_recv,
                                  uint64_t n_rows, uint32_t* d_backup, hipStream_t st);
hipError_t launch_border_restore(const Table& T, const Pool& Pl, const uint32_t* d_backup,
                                 uint64_t n_rows, hipStream_t st);
// mesh halo (ABI v9): per pool slot, 1 when the brick holds an observed voxel
hipError_t launch_brick_observed(const Pool& Pl, uint32_t n_bricks, uint32_t* d_obs,
                                 hipStream_t st);
// tiles of the requested bricks observed here (rows counted in *d_n_rows, atomic order)
hipError_t launch_halo_pack(const Table& T, const Pool& Pl, const uint64_t* d_req, uint32_t n_req,
                            uint32_t* d_send, uint32_t cap_rows, uint32_t* d_n_rows,
                            hipStream_t st);
// received halo tiles -> a hash table H (slot = row) and pool HP (the mesh's second lookup)
hipError_t launch_halo_build(const Table& H, const Pool& HP, const uint32_t* d_tiles,
                             uint32_t n_rows, uint32_t* d_ovf, hipStream_t st);
// Voxblox MergedTsdfIntegrator's bundling pre-pass (tsdf_merged.hip): per batch, the points of
// every scan bundled by voxel; xyz_out / w_out hold one ray per bundle at its first point's slot
// (other slots: NaN point, weight 0), so the batch keeps its ray layout and block counts
// Merged pre-pass buffers (tsdf_merged.hip), one set per batch parity
struct MgBufs {
    float* xyz_out = nullptr;  // per point slot: the bundle ray's end point (NaN: no ray)
    float* w_out = nullptr;    // its weight (negative: clearing)
    uint64_t cap = 0;          // points
    // the batch's (key, point) entries, grouped by bucket (a hash of the key among its scan's
    // buckets of ~1024 points): bucket b holds entries [bst[b], bst[b + 1])
    uint64_t* ekey = nullptr;
    uint32_t* eidx = nullptr;
    uint32_t* bcnt = nullptr;  // per (replica, bucket): size, then cursor; zero between batches
    uint32_t* bst = nullptr;   // per bucket: first entry (nb_cap + 1)
    uint32_t* bscan = nullptr; // per bucket: its scan (k_mg_scan)
    uint32_t nb_cap = 0;       // buckets
};
uint32_t mg_buckets_max(uint64_t n_points);
constexpr uint32_t MG_REPLICAS = 8;  // bucket counter replicas (tsdf_merged.hip MG_REP)
hipError_t launch_mg_prepass(const float* d_xyz, const BatchRef& B, uint32_t n_blocks,
                             uint64_t n_points, const RayConst& R, MgBufs& M, uint32_t* ovf,
                             hipStream_t st);
// Ouster packets (tsdf_ouster.hip)
struct OsField {
    uint32_t nbytes;  // little-endian source bytes (0: the profile has no such field)
    uint32_t offset;  // byte offset in the pixel
    uint32_t mask;    // 0: none
    int32_t shift;    // > 0: right, < 0: left
};
struct OsLayout {
    uint32_t h, w, cols_per_packet, packet_bytes, packet_header, col_header, col_bytes,
        pixel_bytes, legacy;
    OsField f[4];  // RANGE, SIGNAL, REFLECTIVITY, NEAR_IR
};
struct OsPose {
    float m[12];  // 3x4 row-major (rotation | translation), fp32
};
hipError_t launch_os_decode(const uint8_t* d_packets, uint32_t n_packets, const OsLayout& L,
                            uint32_t* const out[4], hipStream_t st);
hipError_t launch_os_xyz(const uint32_t* d_range, uint64_t n, const float* d_dir,
                         const float* d_off, const OsPose& P, float* d_xyz, hipStream_t st);
// marching cubes (tsdf_mesh.hip)
// both case tables (TSDF_MC_GENERATED, TSDF_MC_LORENSEN); `tab` selects one per launch
constexpr int MC_TABLES = 3;  // include/tsdf_hip.h TSDF_MC_TABLES
hipError_t upload_mc_table(const uint8_t tab[MC_TABLES][256][32], const uint8_t edge[12][2]);
// H / HP: halo bricks looked up before the context's own table (ABI v9: bricks another rank
// owns; H.keys == nullptr: none)
hipError_t launch_mesh_count(const Table& T, const Pool& Pl, const Table& H, const Pool& HP,
                             const uint64_t* d_keys, uint32_t nb, float min_weight, int tab,
                             uint32_t* d_counts, hipStream_t st);
hipError_t launch_mesh_emit(const Table& T, const Pool& Pl, const Table& H, const Pool& HP,
                            const uint64_t* d_keys, uint32_t nb, float min_weight, int tab,
                            float vs, const uint64_t* d_offsets, float* d_tri, hipStream_t st);
hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t st);
hipError_t launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t st);

}  // namespace tsdf
