// tsdf_kernels.hip — gfx950 kernels of the TSDF integration hot path (MAP_BACKEND_IDX = 4).
//
// One launch sequence integrates a BATCH of up to 64 consecutive scans:
//   k_rays      one lane per ray of every scan of the batch: range filter, DDA over the truncation
//               band, and at every step where some lanes enter a new brick, a wave-level
//               aggregation round: lanes with the same (brick, scan) elect a leader (ballot + shfl,
//               no LDS), the leaders find-or-insert their brick in the open-addressing table and
//               reserve their lanes' ranks with ONE atomicAdd per group on the brick count and one
//               on the (brick, scan) cell count; every (ray, brick) pair goes to the ray's fixed pair
//               slots.  Bricks first touched in the batch are listed in LDS and appended to the
//               active list with one atomic per flush.
//   k_compact   per active brick: block-wide scans give its contiguous ray-list segment, its pool
//               slot if it is new, and the prefix of its per-scan cells (ray lists scan-ordered)
//   k_scatter   pair -> ray list position (segment + cell prefix + rank)
//   k_integrate one wave per active brick: the brick's (sdf, weight) live in the wave's registers
//               (8 voxels per lane) for the whole batch; for each scan in order, the scan's rays
//               re-walk their DDA and add their in-brick samples as exact fixed point into an LDS
//               tile, then each lane fuses its own voxels — so each touched brick is read once
//               and its dirty voxels written once per batch instead of once per scan.
//
// Semantics: VDBFusion's VDBVolume::Integrate, restated in oracle/tsdf_oracle.c, which is the
// bit-exact CPU twin of this file's arithmetic.  Ray arithmetic is fp32 with contraction off
// (-ffp-contract=off) and correctly rounded div/sqrt, so the voxel sequence, the gate and every
// sample are the oracle's bits.  Per scan, the samples of a voxel are summed as exact 64-bit fixed
// point (trunc(s * 2^32)) plus a count, and fused in scan order, so the field does not depend on
// lane, wave, atomic or batch composition: it is bitwise reproducible and equal to the oracle's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsdf_device.h"

namespace tsdf {

// ------------------------------------------------------------------------------------------------
// ray setup and walk (same op order as oracle/tsdf_oracle.c walk_ray)

struct RayState {
    float px, py, pz;  // hit point (world)
    float t1i;         // band end (index units)
    float tnx, tny, tnz;
    float tdx, tdy, tdz;
    int vx, vy, vz;
    int sx, sy, sz;
};

__device__ __forceinline__ void axis_init(float u, float s, float t0i, int v, float& tn, float& td,
                                          int& st) {
    if (u > 0.0f) {
        const float inv = 1.0f / u;
        st = 1;
        td = inv;
        tn = t0i + ((float)(v + 1) - s) * inv;
    } else if (u < 0.0f) {
        const float inv = 1.0f / u;
        st = -1;
        td = -inv;
        tn = t0i + ((float)v - s) * inv;
    } else {
        st = 0;
        td = __builtin_inff();
        tn = __builtin_inff();
    }
}

// Returns false when the ray is filtered out (zero/NaN length, outside [min_range, max_range]).
__device__ __forceinline__ bool ray_init(const RayConst& R, float ox, float oy, float oz, float px,
                                         float py, float pz, RayState& r) {
    const float dx = px - ox, dy = py - oy, dz = pz - oz;
    const float depth = __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
    if (!(depth > 0.0f)) return false;
    if (!(depth >= R.min_range) || !(depth <= R.max_range)) return false;
    const float ux = dx / depth, uy = dy / depth, uz = dz / depth;
    const float t0 = R.carving ? 0.0f : depth - R.tau;
    const float t1 = depth + R.tau;
    const float t0i = t0 * R.inv_vs;
    r.t1i = t1 * R.inv_vs;
    const float sx = ox * R.inv_vs + ux * t0i;
    const float sy = oy * R.inv_vs + uy * t0i;
    const float sz = oz * R.inv_vs + uz * t0i;
    r.vx = (int)__builtin_floorf(sx);
    r.vy = (int)__builtin_floorf(sy);
    r.vz = (int)__builtin_floorf(sz);
    axis_init(ux, sx, t0i, r.vx, r.tnx, r.tdx, r.sx);
    axis_init(uy, sy, t0i, r.vy, r.tny, r.tdy, r.sy);
    axis_init(uz, sz, t0i, r.vz, r.tnz, r.tdz, r.sz);
    r.px = px;
    r.py = py;
    r.pz = pz;
    return true;
}

// ComputeSDF at the current voxel; true (and the truncated sample) when it passes sdf > -tau.
__device__ __forceinline__ bool voxel_sample(const RayConst& R, float ox, float oy, float oz,
                                             const RayState& r, float& s) {
    if (!(r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT && r.vy < VOX_LIMIT &&
          r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT))
        return false;
    const float cx = ((float)r.vx + 0.5f) * R.vs;
    const float cy = ((float)r.vy + 0.5f) * R.vs;
    const float cz = ((float)r.vz + 0.5f) * R.vs;
    const float ax = cx - ox, ay = cy - oy, az = cz - oz;
    const float bx = r.px - cx, by = r.py - cy, bz = r.pz - cz;
    const float dist = __builtin_sqrtf(bx * bx + by * by + bz * bz);
    const float proj = ax * bx + ay * by + az * bz;
    if (!(proj > 0.0f || proj < 0.0f)) return false;
    const float sdf = proj > 0.0f ? dist : -dist;
    if (!(sdf > -R.tau)) return false;
    s = sdf < R.tau ? sdf : R.tau;
    return true;
}

// One DDA step (math::MinIndex tie-break: equal entries resolve to the higher axis).
// Returns false when the next entry time is past the band end.
// Written with selects only: an axis index would make hipcc spill the state to scratch.
__device__ __forceinline__ bool ray_step(RayState& r) {
    const bool mx = (r.tnx < r.tny) && (r.tnx < r.tnz);  // == oracle: a = 0
    const bool my = !mx && (r.tny < r.tnz);              // == oracle: a = 1
    const bool mz = !mx && !my;                          // == oracle: a = 2 (ties -> higher)
    const float t = mx ? r.tnx : (my ? r.tny : r.tnz);
    if (!(t <= r.t1i)) return false;
    r.tnx = mx ? r.tnx + r.tdx : r.tnx;
    r.tny = my ? r.tny + r.tdy : r.tny;
    r.tnz = mz ? r.tnz + r.tdz : r.tnz;
    r.vx += mx ? r.sx : 0;
    r.vy += my ? r.sy : 0;
    r.vz += mz ? r.sz : 0;
    return true;
}

__device__ __forceinline__ uint64_t pack_brick(int bx, int by, int bz) {
    return (uint64_t)(bx + BRICK_COORD_BIAS) | ((uint64_t)(by + BRICK_COORD_BIAS) << 21) |
           ((uint64_t)(bz + BRICK_COORD_BIAS) << 42);
}

__device__ __forceinline__ uint64_t brick_key_of(int vx, int vy, int vz) {
    return pack_brick(vx >> 3, vy >> 3, vz >> 3);
}

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// Find-or-insert a brick key; returns the table index or -1 when the table is full.  Keys are
// never removed, so a stale EMPTY read is resolved by the CAS and a non-EMPTY read is final.
__device__ __forceinline__ int64_t table_insert(const Table& T, uint64_t key, uint32_t* overflow) {
    uint64_t h = mix64(key) & T.mask;
    for (uint64_t probe = 0; probe <= T.mask; probe++) {
        const uint64_t k = T.keys[h];
        if (k == key) return (int64_t)h;
        if (k == EMPTY_KEY) {
            const unsigned long long old =
                atomicCAS((unsigned long long*)&T.keys[h], (unsigned long long)EMPTY_KEY,
                          (unsigned long long)key);
            if (old == EMPTY_KEY || old == key) return (int64_t)h;
        }
        h = (h + 1) & T.mask;
    }
    atomicOr(overflow, OVF_TABLE);
    return -1;
}

__device__ __forceinline__ int64_t table_find(const Table& T, uint64_t key) {
    uint64_t h = mix64(key) & T.mask;
    for (uint64_t probe = 0; probe <= T.mask; probe++) {
        const uint64_t k = T.keys[h];
        if (k == key) return (int64_t)h;
        if (k == EMPTY_KEY) return -1;
        h = (h + 1) & T.mask;
    }
    return -1;
}

template <typename Tv>
__device__ __forceinline__ Tv wave_sum(Tv v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------------------------------------
// k_rays

constexpr int ACT_LDS = 2048;  // block-local list of bricks first touched by this block

__device__ __forceinline__ void push_active(uint32_t h, uint32_t* s_act, uint32_t* s_nact,
                                            Counters* C, const Work& Wk, Globals* G) {
    const uint32_t q = atomicAdd(s_nact, 1u);
    if (q < (uint32_t)ACT_LDS) {
        s_act[q] = h;
    } else {  // LDS list full (only long carving rays get here): append directly
        const uint32_t g = atomicAdd(&C->n_active, 1u);
        if (g < Wk.max_active) Wk.active[g] = h;
        else atomicOr(&G->overflow, OVF_ACTIVE);
    }
}

// Block-wide flush of the LDS first-touch list (called by all threads, uniform).
__device__ __forceinline__ void flush_active(uint32_t* s_act, uint32_t* s_nact, uint32_t* s_base,
                                             Counters* C, const Work& Wk, Globals* G) {
    __syncthreads();
    const uint32_t n = min(*s_nact, (uint32_t)ACT_LDS);
    if (n) {
        if (threadIdx.x == 0) *s_base = atomicAdd(&C->n_active, n);
        __syncthreads();
        const uint32_t b = *s_base;
        for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
            if (b + j < Wk.max_active) Wk.active[b + j] = s_act[j];
            else atomicOr(&G->overflow, OVF_ACTIVE);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *s_nact = 0;
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_rays(const float* __restrict__ xyz, BatchDesc D,
                                              RayConst R, Table T, Work Wk, Globals* G,
                                              int parity) {
    __shared__ uint32_t s_off[MAX_BATCH + 1];
    __shared__ float s_o[3][MAX_BATCH];
    __shared__ uint32_t s_act[ACT_LDS];
    __shared__ uint32_t s_nact, s_base;
    __shared__ unsigned long long red[2][4];
    Counters* C = &G->ctr[parity];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(Counters) / 4)
        reinterpret_cast<uint32_t*>(&G->ctr[parity ^ 1])[threadIdx.x] = 0u;  // next batch's set
    const uint32_t ns = D.n_scans;
    for (uint32_t j = threadIdx.x; j <= ns; j += blockDim.x) s_off[j] = D.off[j];
    for (uint32_t j = threadIdx.x; j < ns; j += blockDim.x) {
        s_o[0][j] = D.ox[j];
        s_o[1][j] = D.oy[j];
        s_o[2][j] = D.oz[j];
    }
    if (threadIdx.x == 0) s_nact = 0;
    __syncthreads();
    const uint32_t total = s_off[ns];
    const uint32_t maxp = Wk.maxp;
    const int lane = threadIdx.x & 63;
    uint32_t valid = 0, npairs = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const bool live = i < total;
        uint32_t t = 0;  // scan of ray i: the largest t with off[t] <= i
        if (live) {
            uint32_t lo = 0, hi = ns;  // off[lo] <= i < off[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_off[mid] <= i) lo = mid;
                else hi = mid;
            }
            t = lo;
        }
        const float ox = s_o[0][t], oy = s_o[1][t], oz = s_o[2][t];
        RayState r;
        bool walking = live && ray_init(R, ox, oy, oz, xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1],
                                        xyz[3 * (size_t)i + 2], r);
        valid += walking ? 1u : 0u;
        uint32_t* pt = Wk.pair_tidx + (size_t)i * maxp;
        uint32_t* pl = Wk.pair_local + (size_t)i * maxp;
        uint32_t k = 0;
        uint64_t last = EMPTY_KEY;
        int it = 0;
        while (__any(walking)) {
            bool emit = false;
            uint64_t key = 0;
            if (walking) {
                float s;
                if (voxel_sample(R, ox, oy, oz, r, s)) {
                    key = brick_key_of(r.vx, r.vy, r.vz);
                    if (key != last) {
                        last = key;
                        if (k < maxp) emit = true;
                        else atomicOr(&G->overflow, OVF_PAIRS);
                    }
                }
            }
            if (__ballot(emit)) {
                // --- wave-level aggregation: one leader per distinct (brick, scan) ---
                uint64_t pending = __ballot(emit);
                int leader = lane;
                uint32_t gcount = 0, myrank = 0;
                while (pending) {
                    const int ld = __ffsll((unsigned long long)pending) - 1;
                    const uint64_t lk = __shfl(key, ld, 64);
                    const uint32_t lt = __shfl(t, ld, 64);
                    const uint64_t grp = __ballot(emit && key == lk && t == lt) & pending;
                    if ((grp >> lane) & 1ull) {
                        leader = ld;
                        myrank = __popcll(grp & ((1ull << lane) - 1ull));
                    }
                    if (lane == ld) gcount = __popcll(grp);
                    pending &= ~grp;
                }
                uint32_t hh = NO_PAIR, cbase = 0;
                if (emit && leader == lane) {
                    const int64_t hx = table_insert(T, key, &G->overflow);
                    if (hx >= 0) {
                        hh = (uint32_t)hx;
                        const uint32_t c = atomicAdd(&T.cnt[hh], gcount);
                        if (c == 0) push_active(hh, s_act, &s_nact, C, Wk, G);
                        cbase = atomicAdd(&T.cell[(size_t)hh * T.cell_stride + t], gcount);
                    }
                }
                const uint32_t h = __shfl(hh, leader, 64);
                const uint32_t rank = __shfl(cbase, leader, 64) + myrank;
                if (emit && h != NO_PAIR) {
                    pt[k] = h;
                    pl[k] = (t << RANK_BITS) | rank;
                    k++;
                }
            }
            if (walking) walking = ray_step(r) && (++it < MAX_DDA_STEPS);
        }
        npairs += k;
        if (live)
            for (uint32_t j = k; j < maxp; j++) pt[j] = NO_PAIR;
        __syncthreads();
        if (s_nact > (uint32_t)ACT_LDS / 2)  // uniform: read after the barrier
            flush_active(s_act, &s_nact, &s_base, C, Wk, G);
    }
    flush_active(s_act, &s_nact, &s_base, C, Wk, G);
    // block-reduce the stats, one atomic per block on a shard picked by block index
    unsigned long long v = wave_sum<unsigned long long>(valid);
    unsigned long long q = wave_sum<unsigned long long>(npairs);
    const int wid = threadIdx.x >> 6;
    if (lane == 0) { red[0][wid] = v; red[1][wid] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        v = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        q = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        if (v) {
            atomicAdd(&C->n_rays[blockIdx.x & 7], v);
            atomicAdd(&G->tot_rays[blockIdx.x & 7], v);
        }
        if (q) {
            atomicAdd(&C->n_pairs[blockIdx.x & 7], q);
            atomicAdd(&G->tot_pairs[blockIdx.x & 7], q);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_compact: per active brick — ray-list segment, new pool slot, per-scan cell prefix

constexpr int CMP_THREADS = 1024;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d, 64);
        if (lane >= d) v += y;
    }
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    if (threadIdx.x < 16) {
        uint32_t u = s_w[threadIdx.x];
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t y = __shfl_up(u, d, 16);
            if ((int)threadIdx.x >= d) u += y;
        }
        s_w[threadIdx.x] = u;
    }
    __syncthreads();
    *total = s_w[15];
    const uint32_t r = v - x + (wid ? s_w[wid - 1] : 0u);
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(CMP_THREADS) void k_compact(uint32_t n_scans, Table T, Work Wk,
                                                         Globals* G, int parity) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t base_c, base_n;
    Counters* C = &G->ctr[parity];
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    for (uint32_t chunk = blockIdx.x * CMP_THREADS; chunk < n_active;
         chunk += gridDim.x * CMP_THREADS) {
        const uint32_t a = chunk + threadIdx.x;
        const uint32_t h = a < n_active ? Wk.active[a] : NO_PAIR;
        const uint32_t n = h != NO_PAIR ? T.cnt[h] : 0u;
        const uint32_t isnew = (h != NO_PAIR && T.slots[h] == UNASSIGNED) ? 1u : 0u;
        uint32_t tot_c, tot_n;
        const uint32_t ec = block_excl_scan(n, s_w, &tot_c);
        const uint32_t en = block_excl_scan(isnew, s_w, &tot_n);
        if (threadIdx.x == 0) {
            base_c = tot_c ? atomicAdd(&C->cursor, tot_c) : 0u;
            base_n = tot_n ? atomicAdd(&G->pool_count, tot_n) : 0u;
        }
        __syncthreads();
        if (h != NO_PAIR) {
            T.toff[h] = base_c + ec;
            if (isnew) {
                const uint32_t slot = base_n + en;
                if (slot < T.max_bricks) {
                    T.slots[h] = slot;
                    T.brick_keys[slot] = T.keys[h];
                } else {
                    T.slots[h] = INVALID_SLOT;
                    atomicOr(&G->overflow, OVF_POOL);
                }
            }
            // exclusive prefix of the per-scan cell counts (cell_stride is a multiple of 4)
            uint4* cp = reinterpret_cast<uint4*>(T.cell + (size_t)h * T.cell_stride);
            uint32_t run = 0;
            for (uint32_t q = 0; q < (n_scans + 3) / 4; q++) {
                uint4 v = cp[q];
                const uint32_t x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
                v.x = run; run += x0;
                v.y = run; run += x1;
                v.z = run; run += x2;
                v.w = run; run += x3;
                cp[q] = v;
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// k_scatter: pair -> ray list

__global__ __launch_bounds__(256) void k_scatter(uint32_t n_slots, Table T, Work Wk) {
    const uint32_t maxp = Wk.maxp;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n_slots;
         s += gridDim.x * blockDim.x) {
        const uint32_t h = Wk.pair_tidx[s];
        if (h == NO_PAIR) continue;
        const uint32_t pk = Wk.pair_local[s];
        const uint32_t t = pk >> RANK_BITS, r = pk & RANK_MASK;
        Wk.ray_list[T.toff[h] + T.cell[(size_t)h * T.cell_stride + t] + r] = s / maxp;
    }
}

// ------------------------------------------------------------------------------------------------
// k_integrate: one wave per active brick; brick in registers, per-scan LDS tile, fused in order

constexpr int INT_WAVES = 4;  // waves per 256-thread workgroup, one brick tile each

__global__ __launch_bounds__(256) void k_integrate(const float* __restrict__ xyz, BatchDesc D,
                                                  RayConst R, Table T, Work Wk, Pool Pl,
                                                  Globals* G, int parity) {
    __shared__ unsigned long long tileA[INT_WAVES][BRICK_VOX];  // sum of trunc(s * 2^32)
    __shared__ uint32_t tileB[INT_WAVES][BRICK_VOX];            // sample count
    Counters* C = &G->ctr[parity];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long* A = tileA[wid];
    uint32_t* B = tileB[wid];
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
#pragma unroll
    for (int k = 0; k < BRICK_VOX / 64; k++) {
        A[lane + 64 * k] = 0ull;
        B[lane + 64 * k] = 0u;
    }
    wave_sync_lds();
    uint32_t nvox = 0, ndirty = 0;
    for (uint32_t a = blockIdx.x * INT_WAVES + wid; a < n_active; a += gridDim.x * INT_WAVES) {
        const uint32_t h = Wk.active[a];
        const uint32_t slot = T.slots[h];
        const uint32_t n = T.cnt[h];
        const uint32_t base = T.toff[h];
        const uint32_t* cellp = T.cell + (size_t)h * T.cell_stride;
        const uint32_t cs = (uint32_t)lane < ns ? cellp[lane] : n;  // start of scan `lane`'s rays
        const uint64_t key = T.keys[h];
        const int bx = (int)(key & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int by = (int)((key >> 21) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int bz = (int)((key >> 42) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const bool has_slot = slot < T.max_bricks;
        float* Sg = Pl.sdf + (size_t)(has_slot ? slot : 0) * BRICK_VOX;
        float* Wg = Pl.weight + (size_t)(has_slot ? slot : 0) * BRICK_VOX;
        float sv[BRICK_VOX / 64], wv[BRICK_VOX / 64];
#pragma unroll
        for (int k = 0; k < BRICK_VOX / 64; k++) {
            sv[k] = has_slot ? Sg[lane + 64 * k] : R.tau;
            wv[k] = has_slot ? Wg[lane + 64 * k] : 0.0f;
        }
        uint32_t dirty = 0;
        for (uint32_t t = 0; t < ns; t++) {
            const uint32_t c0 = __shfl(cs, (int)t, 64);
            const uint32_t c1 = __shfl(cs, (int)t + 1, 64);  // lane ns holds n
            if (c0 == c1) continue;
            const float ox = D.ox[t], oy = D.oy[t], oz = D.oz[t];
            for (uint32_t j = c0 + lane; j < c1; j += 64) {
                const size_t i = Wk.ray_list[base + j];
                RayState r;
                if (!ray_init(R, ox, oy, oz, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], r))
                    continue;
                for (int it = 0; it < MAX_DDA_STEPS; it++) {
                    if ((r.vx >> 3) == bx && (r.vy >> 3) == by && (r.vz >> 3) == bz) {
                        float s;
                        if (voxel_sample(R, ox, oy, oz, r, s)) {
                            const int l = ((r.vz & 7) << 6) | ((r.vy & 7) << 3) | (r.vx & 7);
                            const long long q = (long long)(s * 4294967296.0f);
                            atomicAdd(&A[l], (unsigned long long)q);
                            atomicAdd(&B[l], 1u);
                        }
                    }
                    if (!ray_step(r)) break;
                }
            }
            wave_sync_lds();
#pragma unroll
            for (int k = 0; k < BRICK_VOX / 64; k++) {
                const int l = lane + 64 * k;
                const uint32_t b = B[l];
                if (b) {
                    const float bf = (float)b;
                    const float af = (float)((double)(long long)A[l] * (1.0 / 4294967296.0));
                    const float nw = wv[k] + bf;
                    sv[k] = (sv[k] * wv[k] + af) / nw;
                    wv[k] = nw;
                    A[l] = 0ull;
                    B[l] = 0u;
                    dirty |= 1u << k;
                    nvox++;
                }
            }
            wave_sync_lds();
        }
        if (has_slot) {
#pragma unroll
            for (int k = 0; k < BRICK_VOX / 64; k++) {
                if (dirty & (1u << k)) {
                    Sg[lane + 64 * k] = sv[k];
                    Wg[lane + 64 * k] = wv[k];
                }
            }
        }
        ndirty += __popc(dirty);
        if (lane == 0) T.cnt[h] = 0u;  // ready for the next batch
        if ((uint32_t)lane < ns) T.cell[(size_t)h * T.cell_stride + lane] = 0u;
    }
    __shared__ unsigned long long red[2][INT_WAVES];
    const unsigned long long v = wave_sum<unsigned long long>(nvox);
    const unsigned long long d = wave_sum<unsigned long long>(ndirty);
    if (lane == 0) { red[0][wid] = v; red[1][wid] = d; }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long tv = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        const unsigned long long td = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        if (tv) {
            atomicAdd(&C->n_vox[blockIdx.x & 7], tv);
            atomicAdd(&G->tot_vox[blockIdx.x & 7], tv);
        }
        if (td) {
            atomicAdd(&C->n_dirty[blockIdx.x & 7], td);
            atomicAdd(&G->tot_dirty[blockIdx.x & 7], td);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// read-out / import

__global__ void k_query_dense(Table T, Pool Pl, int lo0, int lo1, int lo2, int nx, int ny, int nz,
                              float bg_sdf, float* __restrict__ out_sdf,
                              float* __restrict__ out_w) {
    const uint64_t total = (uint64_t)nx * ny * nz;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const int x = lo0 + (int)(i % nx);
        const int y = lo1 + (int)((i / nx) % ny);
        const int z = lo2 + (int)(i / ((uint64_t)nx * ny));
        float s = bg_sdf, w = 0.0f;
        if (x > -VOX_LIMIT && x < VOX_LIMIT && y > -VOX_LIMIT && y < VOX_LIMIT &&
            z > -VOX_LIMIT && z < VOX_LIMIT) {
            const int64_t h = table_find(T, brick_key_of(x, y, z));
            if (h >= 0) {
                const uint32_t slot = T.slots[h];
                if (slot < T.max_bricks) {
                    const int l = ((z & 7) << 6) | ((y & 7) << 3) | (x & 7);
                    s = Pl.sdf[(size_t)slot * BRICK_VOX + l];
                    w = Pl.weight[(size_t)slot * BRICK_VOX + l];
                }
            }
        }
        if (out_sdf) out_sdf[i] = s;
        if (out_w) out_w[i] = w;
    }
}

// Import is not on the hot path: per-brick slot claims use a plain atomicAdd.  Bricks in one
// import call are unique (checked on the host).
__global__ void k_import_insert(Table T, const int32_t* __restrict__ coords, uint32_t n,
                                uint32_t* __restrict__ tidx_out, Globals* G) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t key = pack_brick(coords[3 * i], coords[3 * i + 1], coords[3 * i + 2]);
        const int64_t h = table_insert(T, key, &G->overflow);
        if (h < 0) { tidx_out[i] = NO_PAIR; continue; }
        tidx_out[i] = (uint32_t)h;
        if (T.slots[h] == UNASSIGNED) {
            const uint32_t slot = atomicAdd(&G->pool_count, 1u);
            if (slot < T.max_bricks) {
                T.brick_keys[slot] = key;
                T.slots[h] = slot;
            } else {
                T.slots[h] = INVALID_SLOT;
                atomicOr(&G->overflow, OVF_POOL);
            }
        }
    }
}

__global__ void k_import_merge(Table T, Pool Pl, const uint32_t* __restrict__ tidx, uint32_t n,
                               const float* __restrict__ sdf_in, const float* __restrict__ w_in) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (uint64_t)n * BRICK_VOX;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(i / BRICK_VOX);
        const int l = (int)(i % BRICK_VOX);
        const uint32_t h = tidx[b];
        if (h == NO_PAIR) continue;
        const uint32_t slot = T.slots[h];
        if (slot >= T.max_bricks) continue;
        const float wi = w_in[i];
        if (!(wi > 0.0f)) continue;
        float* S = Pl.sdf + (size_t)slot * BRICK_VOX + l;
        float* W = Pl.weight + (size_t)slot * BRICK_VOX + l;
        const float w0 = *W;
        if (w0 == 0.0f) {  // unobserved: copy, so single-owner voxels stay bit-exact
            *S = sdf_in[i];
            *W = wi;
            continue;
        }
        const float nw = w0 + wi;
        *S = (*S * w0 + sdf_in[i] * wi) / nw;
        *W = nw;
    }
}

template <typename Tv>
__global__ void k_fill(Tv* __restrict__ p, Tv v, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// ------------------------------------------------------------------------------------------------
// launchers (called from tsdf_capi.cpp; every kernel on the context's stream)

static int grid_for(uint64_t items, int per_block, int cap) {
    const uint64_t g = (items + per_block - 1) / per_block;
    return (int)(g < 1 ? 1 : (g > (uint64_t)cap ? (uint64_t)cap : g));
}

hipError_t launch_batch(const float* d_xyz, const BatchDesc& D, const RayConst& R, const Table& T,
                        const Work& Wk, const Pool& Pl, Globals* G, int parity, hipStream_t st,
                        KernelTimer* timer) {
    const uint32_t total = D.off[D.n_scans];
    const uint32_t n_slots = total * Wk.maxp;
    if (timer) timer->begin(KIND_RAYS, st);
    k_rays<<<grid_for(total, 256, 2048), 256, 0, st>>>(d_xyz, D, R, T, Wk, G, parity);
    if (timer) timer->end(KIND_RAYS, st);
    if (timer) timer->begin(KIND_OFFSETS, st);
    k_compact<<<64, CMP_THREADS, 0, st>>>(D.n_scans, T, Wk, G, parity);
    if (timer) timer->end(KIND_OFFSETS, st);
    if (timer) timer->begin(KIND_SCATTER, st);
    k_scatter<<<grid_for(n_slots, 256, 8192), 256, 0, st>>>(n_slots, T, Wk);
    if (timer) timer->end(KIND_SCATTER, st);
    if (timer) timer->begin(KIND_INTEGRATE, st);
    k_integrate<<<1536, 256, 0, st>>>(d_xyz, D, R, T, Wk, Pl, G, parity);
    if (timer) timer->end(KIND_INTEGRATE, st);
    return hipGetLastError();
}

hipError_t launch_query_dense(const Table& T, const Pool& Pl, const int lo[3], const int dims[3],
                              float bg, float* d_sdf, float* d_w, hipStream_t st) {
    const uint64_t total = (uint64_t)dims[0] * dims[1] * dims[2];
    k_query_dense<<<grid_for(total, 256, 8192), 256, 0, st>>>(T, Pl, lo[0], lo[1], lo[2], dims[0],
                                                              dims[1], dims[2], bg, d_sdf, d_w);
    return hipGetLastError();
}

hipError_t launch_import(const Table& T, const Pool& Pl, const int32_t* d_coords, uint32_t n,
                         const float* d_sdf, const float* d_w, uint32_t* d_tidx, Globals* G,
                         hipStream_t st) {
    k_import_insert<<<grid_for(n, 256, 4096), 256, 0, st>>>(T, d_coords, n, d_tidx, G);
    k_import_merge<<<grid_for((uint64_t)n * BRICK_VOX, 256, 8192), 256, 0, st>>>(T, Pl, d_tidx, n,
                                                                                 d_sdf, d_w);
    return hipGetLastError();
}

hipError_t launch_fill(float* p, float v, uint64_t n, hipStream_t st) {
    k_fill<float><<<grid_for(n, 256, 8192), 256, 0, st>>>(p, v, n);
    return hipGetLastError();
}

hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t st) {
    k_fill<uint32_t><<<grid_for(n, 256, 8192), 256, 0, st>>>(p, v, n);
    return hipGetLastError();
}

hipError_t launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t st) {
    k_fill<uint64_t><<<grid_for(n, 256, 8192), 256, 0, st>>>(p, v, n);
    return hipGetLastError();
}

}  // namespace tsdf
