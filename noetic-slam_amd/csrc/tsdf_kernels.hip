// tsdf_kernels.hip — gfx950 kernels of the TSDF integration hot path (MAP_BACKEND_IDX = 4).
//
// Per scan, four stream-ordered launches:
//   k_rays      one lane per ray: range filter, DDA over the truncation band, brick find-or-insert
//               (CAS on the open-addressing table), one (ray, brick) pair per distinct brick the ray
//               updates, written to the ray's FIXED pair slots (no global counter); the pair's rank
//               inside its brick comes from a per-brick atomicAdd (spread over ~31k addresses)
//   k_compact   8 pair slots per lane, block-wide scans: the first pair of every brick makes the
//               brick active (compacted active list), reserves its contiguous ray-list segment and,
//               for a brick new to the map, its pool slot — 3 atomics per 8192 pair slots
//   k_scatter   pair -> ray-list segment
//   k_integrate one wave per active brick: 8^3 tile of (fixed-point sum, count) in LDS; the brick's
//               rays re-walk their DDA and add their in-brick samples with LDS atomics; the wave then
//               fuses the tile into the persistent (sdf, weight) brick, reading and writing only the
//               voxels it updated
//
// Semantics: VDBFusion's VDBVolume::Integrate, restated in oracle/tsdf_oracle.c, which is the
// bit-exact CPU twin of this file's arithmetic.  Ray arithmetic is fp32 with contraction off
// (-ffp-contract=off) and correctly rounded div/sqrt, so the voxel sequence, the gate and every
// sample are the oracle's bits.  Per scan, the samples of a voxel are summed as exact 64-bit fixed
// point (trunc(s * 2^32)) plus a count, so the fused result does not depend on lane, wave or atomic
// order: the field is bitwise reproducible and bitwise equal to the oracle's.
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
__device__ __forceinline__ bool ray_init(const ScanParams& P, float px, float py, float pz,
                                         RayState& r) {
    const float dx = px - P.ox, dy = py - P.oy, dz = pz - P.oz;
    const float depth = __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
    if (!(depth > 0.0f)) return false;
    if (!(depth >= P.min_range) || !(depth <= P.max_range)) return false;
    const float ux = dx / depth, uy = dy / depth, uz = dz / depth;
    const float t0 = P.carving ? 0.0f : depth - P.tau;
    const float t1 = depth + P.tau;
    const float t0i = t0 * P.inv_vs;
    r.t1i = t1 * P.inv_vs;
    const float sx = P.ox * P.inv_vs + ux * t0i;
    const float sy = P.oy * P.inv_vs + uy * t0i;
    const float sz = P.oz * P.inv_vs + uz * t0i;
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
__device__ __forceinline__ bool voxel_sample(const ScanParams& P, const RayState& r, float& s) {
    if (!(r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT && r.vy < VOX_LIMIT &&
          r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT))
        return false;
    const float cx = ((float)r.vx + 0.5f) * P.vs;
    const float cy = ((float)r.vy + 0.5f) * P.vs;
    const float cz = ((float)r.vz + 0.5f) * P.vs;
    const float ax = cx - P.ox, ay = cy - P.oy, az = cz - P.oz;
    const float bx = r.px - cx, by = r.py - cy, bz = r.pz - cz;
    const float dist = __builtin_sqrtf(bx * bx + by * by + bz * bz);
    const float proj = ax * bx + ay * by + az * bz;
    if (!(proj > 0.0f || proj < 0.0f)) return false;
    const float sdf = proj > 0.0f ? dist : -dist;
    if (!(sdf > -P.tau)) return false;
    s = sdf < P.tau ? sdf : P.tau;
    return true;
}

// One DDA step (math::MinIndex tie-break: equal entries resolve to the higher axis).
// Returns false when the next entry time is past the band end.
__device__ __forceinline__ bool ray_step(RayState& r) {
    int a;
    if (r.tnx < r.tny) a = (r.tnx < r.tnz) ? 0 : 2;
    else a = (r.tny < r.tnz) ? 1 : 2;
    const float t = a == 0 ? r.tnx : (a == 1 ? r.tny : r.tnz);
    if (!(t <= r.t1i)) return false;
    if (a == 0) { r.tnx += r.tdx; r.vx += r.sx; }
    else if (a == 1) { r.tny += r.tdy; r.vy += r.sy; }
    else { r.tnz += r.tdz; r.vz += r.sz; }
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

// ------------------------------------------------------------------------------------------------
// k_rays

__global__ __launch_bounds__(256) void k_rays(const float* __restrict__ xyz, uint32_t n,
                                              ScanParams P, Table T, Work Wk, Globals* G,
                                              int parity) {
    __shared__ unsigned long long red[2][4];
    Counters* C = &G->ctr[parity];
    if (blockIdx.x == 0 && threadIdx.x < sizeof(Counters) / 4)
        reinterpret_cast<uint32_t*>(&G->ctr[parity ^ 1])[threadIdx.x] = 0u;  // next scan's set
    const uint32_t maxp = Wk.maxp;
    uint32_t valid = 0, npairs = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t* pt = Wk.pair_tidx + (size_t)i * maxp;
        uint32_t* pl = Wk.pair_local + (size_t)i * maxp;
        uint32_t k = 0;
        RayState r;
        if (ray_init(P, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], r)) {
            valid++;
            uint64_t last = EMPTY_KEY;
            for (int it = 0; it < MAX_DDA_STEPS; it++) {
                float s;
                if (voxel_sample(P, r, s)) {
                    const uint64_t key = brick_key_of(r.vx, r.vy, r.vz);
                    if (key != last) {
                        last = key;
                        if (k < maxp) {
                            const int64_t h = table_insert(T, key, &G->overflow);
                            if (h >= 0) {
                                pl[k] = atomicAdd(&T.cnt[h], 1u);
                                pt[k] = (uint32_t)h;
                                k++;
                            }
                        } else {
                            atomicOr(&G->overflow, OVF_PAIRS);
                        }
                    }
                }
                if (!ray_step(r)) break;
            }
        }
        npairs += k;
        for (uint32_t j = k; j < maxp; j++) pt[j] = NO_PAIR;
    }
    // block-reduce the stats, one atomic per block on a shard picked by block index
    unsigned long long v = wave_sum<unsigned long long>(valid);
    unsigned long long q = wave_sum<unsigned long long>(npairs);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
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
// k_compact: active-brick list, ray-list segments and new pool slots, block-aggregated

constexpr int CMP_THREADS = 1024, CMP_ITEMS = 8, CMP_CHUNK = CMP_THREADS * CMP_ITEMS;

__global__ __launch_bounds__(CMP_THREADS) void k_compact(uint32_t n_slots, Table T, Work Wk,
                                                         Globals* G, int parity) {
    __shared__ uint32_t s_a[16], s_c[16];
    __shared__ uint32_t base_a, base_c, base_n;
    Counters* C = &G->ctr[parity];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t chunk = blockIdx.x * CMP_CHUNK; chunk < n_slots; chunk += gridDim.x * CMP_CHUNK) {
        const uint32_t s0 = chunk + threadIdx.x * CMP_ITEMS;
        uint32_t tid[CMP_ITEMS], cnt[CMP_ITEMS];
        uint32_t fa = 0, fn = 0, fc = 0;  // first-pair flags, new-brick flags (bit per item), counts
#pragma unroll
        for (int j = 0; j < CMP_ITEMS; j++) {
            const uint32_t s = s0 + j;
            tid[j] = NO_PAIR;
            cnt[j] = 0;
            if (s < n_slots) {
                const uint32_t h = Wk.pair_tidx[s];
                if (h != NO_PAIR && Wk.pair_local[s] == 0u) {
                    tid[j] = h;
                    cnt[j] = T.cnt[h];
                    fa += 1;
                    fc += cnt[j];
                    if (T.slots[h] == UNASSIGNED) fn |= 1u << j;
                }
            }
        }
        const uint32_t nnew = __builtin_popcount(fn);
        // block exclusive scan of (fa | nnew << 16) and fc
        uint32_t x = fa | (nnew << 16), y = fc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t xs = __shfl_up(x, d, 64), ys = __shfl_up(y, d, 64);
            if (lane >= d) { x += xs; y += ys; }
        }
        if (lane == 63) { s_a[wid] = x; s_c[wid] = y; }
        __syncthreads();
        if (threadIdx.x < 16) {
            uint32_t u = s_a[threadIdx.x], w = s_c[threadIdx.x];
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) {
                const uint32_t us = __shfl_up(u, d, 16), ws = __shfl_up(w, d, 16);
                if ((int)threadIdx.x >= d) { u += us; w += ws; }
            }
            s_a[threadIdx.x] = u;
            s_c[threadIdx.x] = w;
            if (threadIdx.x == 15) {
                base_a = (u & 0xFFFFu) ? atomicAdd(&C->n_active, u & 0xFFFFu) : 0u;
                base_c = w ? atomicAdd(&C->cursor, w) : 0u;
                base_n = (u >> 16) ? atomicAdd(&G->pool_count, u >> 16) : 0u;
            }
        }
        __syncthreads();
        const uint32_t pa = x - (fa | (nnew << 16)) + (wid ? s_a[wid - 1] : 0u);
        uint32_t ia = base_a + (pa & 0xFFFFu);
        uint32_t in = base_n + (pa >> 16);
        uint32_t ic = base_c + y - fc + (wid ? s_c[wid - 1] : 0u);
#pragma unroll
        for (int j = 0; j < CMP_ITEMS; j++) {
            if (tid[j] == NO_PAIR) continue;
            const uint32_t h = tid[j];
            Wk.active[ia++] = h;
            T.toff[h] = ic;
            ic += cnt[j];
            if (fn & (1u << j)) {
                const uint32_t slot = in++;
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
// k_scatter: pair -> ray list

__global__ __launch_bounds__(256) void k_scatter(uint32_t n_slots, Table T, Work Wk) {
    const uint32_t maxp = Wk.maxp;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n_slots;
         s += gridDim.x * blockDim.x) {
        const uint32_t h = Wk.pair_tidx[s];
        if (h == NO_PAIR) continue;
        Wk.ray_list[T.toff[h] + Wk.pair_local[s]] = s / maxp;
    }
}

// ------------------------------------------------------------------------------------------------
// k_integrate: one wave per active brick, LDS tile, fused write-back

constexpr int INT_WAVES = 4;  // waves per 256-thread workgroup, one brick tile each

__global__ __launch_bounds__(256) void k_integrate(const float* __restrict__ xyz, ScanParams P,
                                                  Table T, Work Wk, Pool Pl, Globals* G,
                                                  int parity) {
    __shared__ unsigned long long tileA[INT_WAVES][BRICK_VOX];  // sum of trunc(s * 2^32)
    __shared__ uint32_t tileB[INT_WAVES][BRICK_VOX];            // sample count
    Counters* C = &G->ctr[parity];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long* A = tileA[wid];
    uint32_t* B = tileB[wid];
    const uint32_t n_active = C->n_active;
    uint32_t nvox = 0;
    for (uint32_t a = blockIdx.x * INT_WAVES + wid; a < n_active; a += gridDim.x * INT_WAVES) {
        const uint32_t h = Wk.active[a];
        const uint32_t slot = T.slots[h];
        const uint32_t n = T.cnt[h];
        const uint32_t off = T.toff[h];
        const uint64_t key = T.keys[h];
        const int bx = (int)(key & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int by = (int)((key >> 21) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int bz = (int)((key >> 42) & 0x1FFFFF) - BRICK_COORD_BIAS;
#pragma unroll
        for (int k = 0; k < BRICK_VOX / 64; k++) {
            A[lane + 64 * k] = 0ull;
            B[lane + 64 * k] = 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t j = lane; j < n; j += 64) {
            const uint32_t i = Wk.ray_list[off + j];
            RayState r;
            if (!ray_init(P, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], r)) continue;
            for (int it = 0; it < MAX_DDA_STEPS; it++) {
                if ((r.vx >> 3) == bx && (r.vy >> 3) == by && (r.vz >> 3) == bz) {
                    float s;
                    if (voxel_sample(P, r, s)) {
                        const int l = ((r.vz & 7) << 6) | ((r.vy & 7) << 3) | (r.vx & 7);
                        const long long q = (long long)(s * 4294967296.0f);
                        atomicAdd(&A[l], (unsigned long long)q);
                        atomicAdd(&B[l], 1u);
                    }
                }
                if (!ray_step(r)) break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (slot < T.max_bricks) {
            float* S = Pl.sdf + (size_t)slot * BRICK_VOX;
            float* W = Pl.weight + (size_t)slot * BRICK_VOX;
#pragma unroll
            for (int k = 0; k < BRICK_VOX / 64; k++) {
                const int l = lane + 64 * k;
                const uint32_t b = B[l];
                if (b) {
                    const float s0 = S[l], w0 = W[l];
                    const float bf = (float)b;
                    const float af = (float)((double)(long long)A[l] * (1.0 / 4294967296.0));
                    const float nw = w0 + bf;
                    S[l] = (s0 * w0 + af) / nw;
                    W[l] = nw;
                    nvox++;
                }
            }
        }
        if (lane == 0) T.cnt[h] = 0u;  // ready for the next scan
    }
    __shared__ unsigned long long red[INT_WAVES];
    const unsigned long long v = wave_sum<unsigned long long>(nvox);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = red[0] + red[1] + red[2] + red[3];
        if (t) {
            atomicAdd(&C->n_vox[blockIdx.x & 7], t);
            atomicAdd(&G->tot_vox[blockIdx.x & 7], t);
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

// Import is not on the hot path: per-brick slot claims use a plain atomicAdd + CAS.  Bricks in one
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

hipError_t launch_scan(const float* d_xyz, uint32_t n, const ScanParams& P, const Table& T,
                       const Work& Wk, const Pool& Pl, Globals* G, int parity, hipStream_t st,
                       KernelTimer* timer) {
    const uint32_t n_slots = n * Wk.maxp;
    if (timer) timer->begin(KIND_RAYS, st);
    k_rays<<<grid_for(n, 256, 8192), 256, 0, st>>>(d_xyz, n, P, T, Wk, G, parity);
    if (timer) timer->end(KIND_RAYS, st);
    if (timer) timer->begin(KIND_OFFSETS, st);
    k_compact<<<grid_for(n_slots, CMP_CHUNK, 256), CMP_THREADS, 0, st>>>(n_slots, T, Wk, G,
                                                                        parity);
    if (timer) timer->end(KIND_OFFSETS, st);
    if (timer) timer->begin(KIND_SCATTER, st);
    k_scatter<<<grid_for(n_slots, 256, 4096), 256, 0, st>>>(n_slots, T, Wk);
    if (timer) timer->end(KIND_SCATTER, st);
    if (timer) timer->begin(KIND_INTEGRATE, st);
    k_integrate<<<1536, 256, 0, st>>>(d_xyz, P, T, Wk, Pl, G, parity);
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
