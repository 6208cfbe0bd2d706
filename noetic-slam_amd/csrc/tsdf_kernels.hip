// tsdf_kernels.hip — gfx950 kernels of the TSDF integration hot path (MAP_BACKEND_IDX = 4).
//
// One launch sequence integrates a BATCH of up to 64 consecutive scans:
//   k_count     one workgroup per 1024 consecutive rays of one scan: every lane walks its rays' DDA
//               over the truncation band; each distinct brick a ray updates goes into the
//               workgroup's LDS hash (one LDS CAS + one LDS atomicAdd per (ray, brick) pair, which
//               also gives the pair its rank).  Then one lane per distinct brick finds-or-inserts it
//               in the global open-addressing table and reserves the workgroup's ranks with ONE
//               atomicAdd on the brick's pair count and one on its (brick, scan) cell — global
//               atomics per distinct brick per workgroup instead of per pair.
//   k_compact   per active brick: block-wide scans give its contiguous ray-record segment, its pool
//               slot if it is new, and the prefix of its per-scan cells (records scan-ordered)
//   k_place     same workgroups as k_count: coalesced read of the rays, one record
//               (x, y, z, in-brick sample count) written per pair to its brick segment
//   k_integrate one wave per active brick: the brick's (sdf, weight) live in registers (8 voxels
//               per lane) for the whole batch.  The brick's records are read 64 at a time
//               (coalesced); every lane walks its ray and writes its in-brick samples to an LDS
//               buffer (positions from a wave prefix of the counts); then, for each scan of the
//               chunk in order, the scan's samples are added as exact fixed point into an LDS tile
//               and — once the scan is complete — each lane fuses its own voxels.  Each touched
//               brick is read once and its dirty voxels written once per batch.
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
// shared helpers of the batch kernels

// Scan and ray range of k_count / k_place workgroup b (uniform: scalar loads of the descriptor).
__device__ __forceinline__ void block_range(const BatchDesc& D, uint32_t b, uint32_t& t,
                                            uint32_t& r0, uint32_t& r1) {
    uint32_t lo = 0, hi = D.n_scans;  // blk[lo] <= b < blk[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (D.blk[mid] <= b) lo = mid;
        else hi = mid;
    }
    t = lo;
    r0 = D.off[t] + (b - D.blk[t]) * RPB;
    r1 = min(D.off[t + 1], r0 + RPB);
}

// LDS brick hash of one k_count workgroup: slot index of key (inserted if new), -1 when no slot
// is found within LDS_PROBES probes (the pair then takes the global fallback).
__device__ __forceinline__ int lds_insert(unsigned long long* s_key, uint64_t key) {
    uint32_t hs = (uint32_t)(mix64(key) >> 40) & (HCAP - 1);
    for (int p = 0; p < LDS_PROBES; p++) {
        const unsigned long long k = s_key[hs];
        if (k == key) return (int)hs;
        if (k == EMPTY_KEY) {
            const unsigned long long old = atomicCAS(&s_key[hs], EMPTY_KEY, key);
            if (old == EMPTY_KEY || old == key) return (int)hs;
        }
        hs = (hs + 1) & (HCAP - 1);
    }
    return -1;
}

// ------------------------------------------------------------------------------------------------
// k_count

constexpr int CNT_THREADS = 256;

__global__ __launch_bounds__(CNT_THREADS) void k_count(const float* __restrict__ xyz, BatchDesc D,
                                                      RayConst R, Table T, Work Wk, Globals* G,
                                                      int parity) {
    __shared__ unsigned long long s_key[HCAP];
    __shared__ uint32_t s_cnt[HCAP];
    __shared__ uint32_t s_occ[HCAP / 32];
    __shared__ unsigned long long red[2][CNT_THREADS / 64];
    Counters* C = &G->ctr[parity];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(Counters) / 4)
        reinterpret_cast<uint32_t*>(&G->ctr[parity ^ 1])[threadIdx.x] = 0u;  // next batch's set
    for (int j = threadIdx.x; j < HCAP; j += CNT_THREADS) {
        s_key[j] = EMPTY_KEY;
        s_cnt[j] = 0u;
    }
    if (threadIdx.x < HCAP / 32) s_occ[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const float ox = D.ox[t], oy = D.oy[t], oz = D.oz[t];
    const uint32_t maxp = Wk.maxp;
    uint32_t valid = 0, npairs = 0;
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += CNT_THREADS) {
        uint32_t* pc = Wk.pair + (size_t)i * maxp;
        uint32_t k = 0;
        RayState r;
        if (ray_init(R, ox, oy, oz, xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1],
                     xyz[3 * (size_t)i + 2], r)) {
            valid++;
            // One pair per distinct brick; a line visits a brick in one contiguous run of DDA
            // voxels, so the pair is closed when the next gated voxel's brick differs.  cnt_in =
            // the pair's gated voxels (<= MAX_IN_BRICK), sizes k_integrate's sample buffer.
            auto emit = [&](uint64_t bkey, uint32_t cnt_in) {
                if (k >= maxp) {
                    atomicOr(&G->overflow, OVF_PAIRS);
                    return;
                }
                const int lid = lds_insert(s_key, bkey);
                if (lid >= 0) {
                    const uint32_t lr = atomicAdd(&s_cnt[lid], 1u);  // < RPB: one pair per ray
                    pc[k++] = (cnt_in << PAIR_CNT_SHIFT) | ((uint32_t)lid << 10) | lr;
                    return;
                }
                // LDS hash full: this pair takes the global path
                const uint32_t f = atomicAdd(&C->n_fb, 1u);
                if (f >= Wk.max_fb) {
                    atomicOr(&G->overflow, OVF_FB);
                    return;
                }
                const int64_t hx = table_insert(T, bkey, &G->overflow);
                if (hx < 0) return;
                const uint32_t h = (uint32_t)hx;
                T.touched[h] = 1u;
                const uint32_t rk = atomicAdd(&T.cell[(size_t)h * T.cell_stride + t], 1u);
                Wk.fb[f] = make_uint4(h, t, rk, 0u);
                pc[k++] = PAIR_FB | (cnt_in << PAIR_CNT_SHIFT) | f;
            };
            uint64_t cur = EMPTY_KEY;
            uint32_t ccount = 0;
            for (int it = 0; it < MAX_DDA_STEPS; it++) {
                float s;
                if (voxel_sample(R, ox, oy, oz, r, s)) {
                    const uint64_t key = brick_key_of(r.vx, r.vy, r.vz);
                    if (key != cur) {
                        if (cur != EMPTY_KEY) emit(cur, ccount);
                        cur = key;
                        ccount = 0;
                    }
                    ccount++;
                }
                if (!ray_step(r)) break;
            }
            if (cur != EMPTY_KEY) emit(cur, ccount);
        }
        npairs += k;
        for (uint32_t j = k; j < maxp; j++) pc[j] = NO_PAIR;
    }
    __syncthreads();
    // one global find-or-insert + one atomic per distinct brick of the workgroup: the cell
    // (brick, scan) count reserves the workgroup's ranks; `touched` (a plain store) lists the brick
    // for k_compact, which also derives the brick's total from its cells
    uint2* bt = Wk.blk + (size_t)blockIdx.x * HCAP;
    for (int slot = threadIdx.x; slot < HCAP; slot += CNT_THREADS) {
        const uint64_t key = s_key[slot];
        if (key == EMPTY_KEY) continue;
        const uint32_t n = s_cnt[slot];
        const int64_t hx = table_insert(T, key, &G->overflow);
        uint2 e = make_uint2(NO_PAIR, 0u);
        if (hx >= 0) {
            const uint32_t h = (uint32_t)hx;
            T.touched[h] = 1u;
            e = make_uint2(h, atomicAdd(&T.cell[(size_t)h * T.cell_stride + t], n));
        }
        bt[slot] = e;
        atomicOr(&s_occ[slot >> 5], 1u << (slot & 31));
    }
    __syncthreads();
    if (threadIdx.x < HCAP / 32) Wk.blk_occ[(size_t)blockIdx.x * (HCAP / 32) + threadIdx.x] =
        s_occ[threadIdx.x];
    // block-reduce the stats, one atomic per block on a shard picked by block index
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long v = wave_sum<unsigned long long>(valid);
    unsigned long long q = wave_sum<unsigned long long>(npairs);
    if (lane == 0) { red[0][wid] = v; red[1][wid] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        v = 0;
        q = 0;
        for (int w = 0; w < CNT_THREADS / 64; w++) { v += red[0][w]; q += red[1][w]; }
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
// k_compact: per active brick — record segment, new pool slot, per-scan cell prefix

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

// Sweeps the `touched` words of the whole table (coalesced, cap * 4 B) — cheaper than any
// per-brick first-touch atomic in k_count.  For each touched brick: its per-scan cell counts
// become their exclusive prefix (and their sum its pair count), it gets its record segment, a pool
// slot if it is new, and an active-list entry; three atomics per CMP_THREADS table entries.
__global__ __launch_bounds__(CMP_THREADS) void k_compact(uint32_t n_scans, Table T, Work Wk,
                                                         Globals* G, int parity) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t base_a, base_c, base_n;
    Counters* C = &G->ctr[parity];
    const uint32_t cap = (uint32_t)(T.mask + 1);
    for (uint32_t chunk = blockIdx.x * CMP_THREADS; chunk < cap;
         chunk += gridDim.x * CMP_THREADS) {
        const uint32_t h = chunk + threadIdx.x;
        const bool hit = T.touched[h] != 0u;
        uint32_t n = 0, isnew = 0;
        if (hit) {
            T.touched[h] = 0u;
            isnew = T.slots[h] == UNASSIGNED ? 1u : 0u;
            // exclusive prefix of the per-scan cell counts (cell_stride is a multiple of 4)
            uint4* cp = reinterpret_cast<uint4*>(T.cell + (size_t)h * T.cell_stride);
            for (uint32_t q = 0; q < (n_scans + 3) / 4; q++) {
                uint4 v = cp[q];
                const uint32_t x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
                v.x = n; n += x0;
                v.y = n; n += x1;
                v.z = n; n += x2;
                v.w = n; n += x3;
                cp[q] = v;
            }
            T.cnt[h] = n;
        }
        uint32_t tot_a, tot_c, tot_n;
        const uint32_t ea = block_excl_scan(hit ? 1u : 0u, s_w, &tot_a);
        const uint32_t ec = block_excl_scan(n, s_w, &tot_c);
        const uint32_t en = block_excl_scan(isnew, s_w, &tot_n);
        if (threadIdx.x == 0) {
            base_a = tot_a ? atomicAdd(&C->n_active, tot_a) : 0u;
            base_c = tot_c ? atomicAdd(&C->cursor, tot_c) : 0u;
            base_n = tot_n ? atomicAdd(&G->pool_count, tot_n) : 0u;
        }
        __syncthreads();
        if (hit) {
            if (base_a + ea < Wk.max_active) Wk.active[base_a + ea] = h;
            else atomicOr(&G->overflow, OVF_ACTIVE);
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
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// k_place: ray records into the bricks' scan-ordered segments

__global__ __launch_bounds__(CNT_THREADS) void k_place(const float* __restrict__ xyz, BatchDesc D,
                                                      Table T, Work Wk) {
    __shared__ uint32_t s_base[HCAP];
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const uint2* bt = Wk.blk + (size_t)blockIdx.x * HCAP;
    const uint32_t* occ = Wk.blk_occ + (size_t)blockIdx.x * (HCAP / 32);
    for (int slot = threadIdx.x; slot < HCAP; slot += CNT_THREADS) {
        uint32_t b = NO_PAIR;
        if ((occ[slot >> 5] >> (slot & 31)) & 1u) {
            const uint2 e = bt[slot];
            if (e.x != NO_PAIR)
                b = T.toff[e.x] + T.cell[(size_t)e.x * T.cell_stride + t] + e.y;
        }
        s_base[slot] = b;
    }
    __syncthreads();
    const uint32_t maxp = Wk.maxp;
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += CNT_THREADS) {
        const uint32_t* pc = Wk.pair + (size_t)i * maxp;
        const float px = xyz[3 * (size_t)i], py = xyz[3 * (size_t)i + 1],
                    pz = xyz[3 * (size_t)i + 2];
        for (uint32_t k = 0; k < maxp; k++) {
            const uint32_t code = pc[k];
            if (code == NO_PAIR) break;
            const uint32_t cnt_in = (code >> PAIR_CNT_SHIFT) & 31u;
            uint32_t pos;
            if (code & PAIR_FB) {
                const uint4 f = Wk.fb[code & ((1u << PAIR_CNT_SHIFT) - 1u)];
                pos = T.toff[f.x] + T.cell[(size_t)f.x * T.cell_stride + f.y] + f.z;
            } else {
                const uint32_t b = s_base[(code >> 10) & (HCAP - 1)];
                if (b == NO_PAIR) continue;
                pos = b + (code & 1023u);
            }
            if (pos < Wk.max_rec) Wk.rec[pos] = make_float4(px, py, pz, __uint_as_float(cnt_in));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_integrate: one wave per active brick; brick in registers, samples and tile in LDS

constexpr int SBUF = 64 * MAX_IN_BRICK;

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, int lane) {
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d, 64);
        if (lane >= d) v += y;
    }
    return v - x;
}

__global__ __launch_bounds__(64) void k_integrate(BatchDesc D, RayConst R, Table T, Work Wk,
                                                 Pool Pl, Globals* G, int parity) {
    __shared__ __attribute__((aligned(16))) unsigned long long A[BRICK_VOX];  // sum trunc(s*2^32)
    __shared__ __attribute__((aligned(16))) uint32_t B[BRICK_VOX];            // sample count
    __shared__ float smp_s[SBUF];
    __shared__ uint16_t smp_l[SBUF];
    Counters* C = &G->ctr[parity];
    const int lane = threadIdx.x;
    const int l0 = lane * 8;  // this lane owns voxels l0 .. l0 + 7
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        A[l0 + k] = 0ull;
        B[l0 + k] = 0u;
    }
    wave_sync_lds();
    uint32_t nvox = 0, ndirty = 0;
    for (uint32_t a = blockIdx.x; a < n_active; a += gridDim.x) {
        const uint32_t h = Wk.active[a];
        const uint32_t slot = T.slots[h];
        const uint32_t n = T.cnt[h];
        const uint32_t base = T.toff[h];
        const uint32_t cs = (uint32_t)lane < ns ? T.cell[(size_t)h * T.cell_stride + lane] : n;
        const uint64_t key = T.keys[h];
        const int bx = (int)(key & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int by = (int)((key >> 21) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int bz = (int)((key >> 42) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const bool has_slot = slot < T.max_bricks;
        float4* Sg = reinterpret_cast<float4*>(Pl.sdf + (size_t)(has_slot ? slot : 0) * BRICK_VOX + l0);
        float4* Wg = reinterpret_cast<float4*>(Pl.weight + (size_t)(has_slot ? slot : 0) * BRICK_VOX + l0);
        float sv[8], wv[8];
        {
            const float4 s0 = has_slot ? Sg[0] : make_float4(R.tau, R.tau, R.tau, R.tau);
            const float4 s1 = has_slot ? Sg[1] : make_float4(R.tau, R.tau, R.tau, R.tau);
            const float4 w0 = has_slot ? Wg[0] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 w1 = has_slot ? Wg[1] : make_float4(0.f, 0.f, 0.f, 0.f);
            sv[0] = s0.x; sv[1] = s0.y; sv[2] = s0.z; sv[3] = s0.w;
            sv[4] = s1.x; sv[5] = s1.y; sv[6] = s1.z; sv[7] = s1.w;
            wv[0] = w0.x; wv[1] = w0.y; wv[2] = w0.z; wv[3] = w0.w;
            wv[4] = w1.x; wv[5] = w1.y; wv[6] = w1.z; wv[7] = w1.w;
        }
        uint32_t dirty = 0;
        for (uint32_t j0 = 0; j0 < n; j0 += 64) {
            const uint32_t j = j0 + lane;
            const bool valid = j < n;
            const float4 rc = valid ? Wk.rec[base + j] : make_float4(0.f, 0.f, 0.f, 0.f);
            const uint32_t cnt_j = valid ? __float_as_uint(rc.w) : 0u;
            // scan of ray j: the largest t < ns with cs_t <= j (lane t holds cs_t; cs_0 = 0).
            // Branch-free search whose trip count depends on ns only, so every lane runs every
            // __shfl (a shfl from a lane that left a divergent loop reads garbage).
            uint32_t tj = 0;
            for (uint32_t len = ns; len > 1;) {
                const uint32_t half = len >> 1;
                const uint32_t v = (uint32_t)__shfl(cs, (int)(tj + half), 64);
                tj = (v <= j) ? tj + half : tj;
                len -= half;
            }
            const uint32_t off = wave_excl_scan(cnt_j, lane);
            if (valid && cnt_j) {
                const float ox = D.ox[tj], oy = D.oy[tj], oz = D.oz[tj];
                RayState r;
                if (ray_init(R, ox, oy, oz, rc.x, rc.y, rc.z, r)) {
                    uint32_t w = 0;
                    for (int it = 0; it < MAX_DDA_STEPS; it++) {
                        if ((r.vx >> 3) == bx && (r.vy >> 3) == by && (r.vz >> 3) == bz) {
                            float s;
                            if (voxel_sample(R, ox, oy, oz, r, s) && w < cnt_j) {
                                smp_s[off + w] = s;
                                smp_l[off + w] =
                                    (uint16_t)(((r.vz & 7) << 6) | ((r.vy & 7) << 3) | (r.vx & 7));
                                w++;
                            }
                        }
                        if (!ray_step(r)) break;
                    }
                }
            }
            wave_sync_lds();
            const uint32_t last_lane = min(63u, n - 1 - j0);
            const uint32_t t_first = __shfl(tj, 0, 64);
            const uint32_t t_last = __shfl(tj, (int)last_lane, 64);
            for (uint32_t t = t_first; t <= t_last; t++) {
                const unsigned long long m = __ballot(valid && tj == t);
                if (!m) continue;
                const int fl = __ffsll(m) - 1;
                const int ll = 63 - __clzll(m);
                const uint32_t sa = __shfl(off, fl, 64);
                const uint32_t sb = __shfl(off + cnt_j, ll, 64);
                for (uint32_t q = sa + lane; q < sb; q += 64) {
                    const int l = smp_l[q];
                    const long long fx = (long long)(smp_s[q] * 4294967296.0f);
                    atomicAdd(&A[l], (unsigned long long)fx);
                    atomicAdd(&B[l], 1u);
                }
                const uint32_t end_t = (t + 1 < ns) ? (uint32_t)__shfl(cs, (int)t + 1, 64) : n;
                if (end_t <= j0 + 64) {  // every ray of scan t has been accumulated: fuse
                    wave_sync_lds();
                    const uint4 b0 = *reinterpret_cast<const uint4*>(&B[l0]);
                    const uint4 b1 = *reinterpret_cast<const uint4*>(&B[l0 + 4]);
                    const uint32_t bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        if (bb[k]) {
                            const float bf = (float)bb[k];
                            const float af =
                                (float)((double)(long long)A[l0 + k] * (1.0 / 4294967296.0));
                            const float nw = wv[k] + bf;
                            sv[k] = (sv[k] * wv[k] + af) / nw;
                            wv[k] = nw;
                            A[l0 + k] = 0ull;
                            B[l0 + k] = 0u;
                            dirty |= 1u << k;
                            nvox++;
                        }
                    }
                }
                wave_sync_lds();
            }
        }
        if (has_slot) {
            if (dirty & 0x0Fu) {
                Sg[0] = make_float4(sv[0], sv[1], sv[2], sv[3]);
                Wg[0] = make_float4(wv[0], wv[1], wv[2], wv[3]);
            }
            if (dirty & 0xF0u) {
                Sg[1] = make_float4(sv[4], sv[5], sv[6], sv[7]);
                Wg[1] = make_float4(wv[4], wv[5], wv[6], wv[7]);
            }
        }
        ndirty += __popc(dirty);
        // zero every cell of the brick (k_compact prefixes whole uint4 groups) for the next batch
        if ((uint32_t)lane < T.cell_stride) T.cell[(size_t)h * T.cell_stride + lane] = 0u;
    }
    const unsigned long long v = wave_sum<unsigned long long>(nvox);
    const unsigned long long d = wave_sum<unsigned long long>(ndirty);
    if (lane == 0) {
        if (v) {
            atomicAdd(&C->n_vox[blockIdx.x & 7], v);
            atomicAdd(&G->tot_vox[blockIdx.x & 7], v);
        }
        if (d) {
            atomicAdd(&C->n_dirty[blockIdx.x & 7], d);
            atomicAdd(&G->tot_dirty[blockIdx.x & 7], d);
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

constexpr int INT_GRID = 2560;  // k_integrate: 256 CUs x 10 resident one-wave workgroups (LDS)

hipError_t launch_batch(const float* d_xyz, const BatchDesc& D, const RayConst& R, const Table& T,
                        const Work& Wk, const Pool& Pl, Globals* G, int parity, hipStream_t st,
                        KernelTimer* timer) {
    if (D.n_blocks == 0) return hipSuccess;
    if (timer) timer->begin(KIND_COUNT, st);
    k_count<<<D.n_blocks, CNT_THREADS, 0, st>>>(d_xyz, D, R, T, Wk, G, parity);
    if (timer) timer->end(KIND_COUNT, st);
    if (timer) timer->begin(KIND_COMPACT, st);
    k_compact<<<grid_for(T.mask + 1, CMP_THREADS, 256), CMP_THREADS, 0, st>>>(D.n_scans, T, Wk,
                                                                                G, parity);
    if (timer) timer->end(KIND_COMPACT, st);
    if (timer) timer->begin(KIND_PLACE, st);
    k_place<<<D.n_blocks, CNT_THREADS, 0, st>>>(d_xyz, D, T, Wk);
    if (timer) timer->end(KIND_PLACE, st);
    if (timer) timer->begin(KIND_INTEGRATE, st);
    k_integrate<<<INT_GRID, 64, 0, st>>>(D, R, T, Wk, Pl, G, parity);
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
