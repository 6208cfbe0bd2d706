// tsdf_device.h — device-side data layout shared by the kernels and the C-ABI host code.
//
// HBM layout:
//   Table   open-addressing brick hash, capacity 2^k >= 2 * max_bricks, linear probing:
//           keys[cap]  u64  packed brick coords (21 bits/axis, biased by 2^20); EMPTY = ~0
//           slots[cap] u32  brick-pool slot (UNASSIGNED until the scan's compaction pass)
//           cnt[cap]   u32  this scan's (ray, brick) pair count (zeroed by k_integrate)
//           toff[cap]  u32  this scan's ray-list segment offset
//   Pool    sdf[max_bricks][512] f32, weight[max_bricks][512] f32 — voxel l = z*64 + y*8 + x;
//           brick_keys[max_bricks] u64 (slot -> key, for export)
//   Work    per-ray fixed pair slots: pair_tidx / pair_local[max_points * maxp] u32,
//           ray_list[max_points * maxp] u32, active[max_points * maxp] u32
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tsdf {

constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr uint32_t UNASSIGNED = 0xFFFFFFFFu;  // table entry inserted, pool slot not yet given
constexpr uint32_t INVALID_SLOT = 0xFFFFFFFEu;  // pool exhausted for this brick
constexpr uint32_t NO_PAIR = 0xFFFFFFFFu;
constexpr int BRICK_VOX = 512;
constexpr int BRICK_COORD_BIAS = 1 << 20;
constexpr int VOX_LIMIT = 1 << 23;  // |voxel index| < 2^23 on every axis (same as the oracle)
constexpr int MAX_DDA_STEPS = 1 << 20;

// overflow bits (sticky until tsdf_sync reads them)
constexpr uint32_t OVF_TABLE = 1u, OVF_POOL = 2u, OVF_PAIRS = 4u;

struct ScanParams {
    float vs, inv_vs, tau, min_range, max_range;
    float ox, oy, oz;  // sensor origin (world), fp32
    int carving;
};

struct Table {
    uint64_t* keys;
    uint32_t* slots;
    uint32_t* cnt;
    uint32_t* toff;
    uint64_t* brick_keys;  // pool slot -> key
    uint64_t mask;
    uint32_t max_bricks;
};

struct Pool {
    float* sdf;
    float* weight;
};

struct Work {
    uint32_t* pair_tidx;
    uint32_t* pair_local;
    uint32_t* ray_list;
    uint32_t* active;
    uint32_t maxp;  // pair slots per ray
};

// per-scan counters, double-buffered by scan parity (k_rays zeroes the other set)
struct Counters {
    uint32_t n_active;
    uint32_t cursor;
    uint32_t n_new;
    uint32_t pad0;
    unsigned long long n_vox[8];   // U_vox of this scan, sharded by blockIdx & 7
    unsigned long long n_rays[8];  // valid rays of this scan
    unsigned long long n_pairs[8];
};

// persistent device globals (one allocation, zeroed at create)
struct Globals {
    uint32_t pool_count;
    uint32_t overflow;
    uint32_t pad[2];
    Counters ctr[2];
    unsigned long long tot_vox[8];  // running totals since the last stats reset (sharded)
    unsigned long long tot_rays[8];
    unsigned long long tot_pairs[8];
};

enum KernelKind { KIND_RAYS = 0, KIND_OFFSETS = 1, KIND_SCATTER = 2, KIND_INTEGRATE = 3, KIND_N = 4 };

// Optional per-kernel HIP-event timing (profiling mode); implemented in tsdf_capi.cpp.
struct KernelTimer {
    virtual void begin(int kind, hipStream_t st) = 0;
    virtual void end(int kind, hipStream_t st) = 0;
    virtual ~KernelTimer() {}
};

hipError_t launch_scan(const float* d_xyz, uint32_t n, const ScanParams& P, const Table& T,
                       const Work& Wk, const Pool& Pl, Globals* G, int parity, hipStream_t st,
                       KernelTimer* timer);
hipError_t launch_query_dense(const Table& T, const Pool& Pl, const int lo[3], const int dims[3],
                              float bg, float* d_sdf, float* d_w, hipStream_t st);
hipError_t launch_import(const Table& T, const Pool& Pl, const int32_t* d_coords, uint32_t n,
                         const float* d_sdf, const float* d_w, uint32_t* d_tidx, Globals* G,
                         hipStream_t st);
hipError_t launch_fill(float* p, float v, uint64_t n, hipStream_t st);
hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t st);
hipError_t launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t st);

}  // namespace tsdf
