// tsdf_ray.h — device helpers shared by the hot-path kernels: the fp32 ray model (the bit-exact
// twin of oracle/tsdf_oracle.c walk_ray), brick keys, the global brick hash and wave utilities.
#pragma once
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
    if (!in_sector(R, dx, dy)) return false;  // another GPU's azimuth sector
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
                                             const RayState& r, float& s, bool check = true) {
    if (check && !(r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT && r.vy < VOX_LIMIT &&
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

// voxel_sample without early exits (same fp32 ops, same verdict and sample): for walks whose lanes
// diverge, where straight-line selects beat branches.
__device__ __forceinline__ bool voxel_sample_sel(const RayConst& R, float ox, float oy, float oz,
                                                 const RayState& r, float& s, bool check = true) {
    const bool inl = !check || (r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT &&
                                r.vy < VOX_LIMIT && r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT);
    const float cx = ((float)r.vx + 0.5f) * R.vs;
    const float cy = ((float)r.vy + 0.5f) * R.vs;
    const float cz = ((float)r.vz + 0.5f) * R.vs;
    const float ax = cx - ox, ay = cy - oy, az = cz - oz;
    const float bx = r.px - cx, by = r.py - cy, bz = r.pz - cz;
    const float dist = __builtin_sqrtf(bx * bx + by * by + bz * bz);
    const float proj = ax * bx + ay * by + az * bz;
    const float sdf = proj > 0.0f ? dist : -dist;
    s = sdf < R.tau ? sdf : R.tau;
    return inl && (proj > 0.0f || proj < 0.0f) && sdf > -R.tau;
}

// voxel_sample's verdict alone (k_count needs no sample value): the same fp32 ops up to the
// projection; a voxel in front of the hit (proj > 0) always passes, and behind it the sqrt is only
// evaluated when d2 lies within 2^-20 of tau^2, so the result equals voxel_sample's bit for bit.
__device__ __forceinline__ bool voxel_gate(const RayConst& R, float ox, float oy, float oz,
                                           const RayState& r, bool check = true) {
    if (check && !(r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT && r.vy < VOX_LIMIT &&
          r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT))
        return false;
    const float cx = ((float)r.vx + 0.5f) * R.vs;
    const float cy = ((float)r.vy + 0.5f) * R.vs;
    const float cz = ((float)r.vz + 0.5f) * R.vs;
    const float ax = cx - ox, ay = cy - oy, az = cz - oz;
    const float bx = r.px - cx, by = r.py - cy, bz = r.pz - cz;
    const float proj = ax * bx + ay * by + az * bz;
    if (proj > 0.0f) return true;       // sdf = +dist > -tau
    if (!(proj < 0.0f)) return false;   // proj == 0 (or NaN): skipped
    const float d2 = bx * bx + by * by + bz * bz;
    if (d2 < R.tau2_lo) return true;    // dist < tau
    if (!(d2 <= R.tau2_hi)) return false;
    return __builtin_sqrtf(d2) < R.tau;  // -dist > -tau
}

// voxel_gate without early exits (same verdict, bit for bit): the squared distance is always formed
// and only the rare near-tau case (|d2 - tau^2| within 2^-20) takes the sqrt, in a branch the wave
// skips when none of its lanes needs it.
__device__ __forceinline__ bool voxel_gate_sel(const RayConst& R, float ox, float oy, float oz,
                                               const RayState& r, bool check = true) {
    const bool inl = !check || (r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT &&
                                r.vy < VOX_LIMIT && r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT);
    const float cx = ((float)r.vx + 0.5f) * R.vs;
    const float cy = ((float)r.vy + 0.5f) * R.vs;
    const float cz = ((float)r.vz + 0.5f) * R.vs;
    const float ax = cx - ox, ay = cy - oy, az = cz - oz;
    const float bx = r.px - cx, by = r.py - cy, bz = r.pz - cz;
    const float proj = ax * bx + ay * by + az * bz;
    const float d2 = bx * bx + by * by + bz * bz;
    bool behind = d2 < R.tau2_lo;  // dist < tau, so -dist > -tau
    const bool near = !behind && d2 <= R.tau2_hi;
    if (near) behind = __builtin_sqrtf(d2) < R.tau;
    return inl && (proj > 0.0f || (proj < 0.0f && behind));
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

// ray_step without the early return: the state advances only when the step is taken, with selects
// (for the single walk's unrolled loop, where every branch would split the wave's exec mask)
__device__ __forceinline__ bool ray_step_sel(RayState& r) {
    const bool mx = (r.tnx < r.tny) && (r.tnx < r.tnz);
    const bool my = !mx && (r.tny < r.tnz);
    const bool mz = !mx && !my;
    const float t = mx ? r.tnx : (my ? r.tny : r.tnz);
    const bool adv = t <= r.t1i;
    r.tnx = (mx && adv) ? r.tnx + r.tdx : r.tnx;
    r.tny = (my && adv) ? r.tny + r.tdy : r.tny;
    r.tnz = (mz && adv) ? r.tnz + r.tdz : r.tnz;
    r.vx += (mx && adv) ? r.sx : 0;
    r.vy += (my && adv) ? r.sy : 0;
    r.vz += (mz && adv) ? r.sz : 0;
    return adv;
}

// ------------------------------------------------------------------------------------------------
// Voxblox ray model (TSDF_SEM_VOXBLOX; the bit-exact twin of oracle/tsdf_oracle.c walk_ray_vb,
// which restates voxblox SimpleTsdfIntegrator / RayCaster / updateTsdfVoxel — DESIGN.md §2b)

// Scan and ray range of k_count / k_place workgroup b, and of the merged pre-pass' k_mg_count /
// k_mg_scatter (uniform: scalar loads of the descriptor).
__device__ __forceinline__ void block_range(const BatchRef& D, uint32_t b, uint32_t& t,
                                            uint32_t& r0, uint32_t& r1) {
    uint32_t lo = 0, hi = D.n_scans;  // blk[lo] <= b < blk[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (D.s[mid].blk <= b) lo = mid;
        else hi = mid;
    }
    t = lo;
    r0 = D.s[t].off + (b - D.s[t].blk) * RPB;
    r1 = min(D.s[t + 1].off, r0 + RPB);
}

// The points of scan t for its batch rays i (ABI v10): xyz[3 (i + xoff)], xoff nonzero only for
// the device batches of an index-sharded context.  The merged pre-pass writes its bundle rays in
// batch-ray order (RayConst::ray_w set), so the walk kernels read that output without the gap.
__device__ __forceinline__ const float* scan_xyz(const float* xyz, const BatchRef& D, uint32_t t,
                                                 const RayConst& R) {
    return R.ray_w ? xyz : xyz + 3 * (size_t)D.s[t].xoff;
}

constexpr float VB_MIN_WEIGHT = 1.0f / 65536.0f;  // lighter samples are dropped whole

struct VbState {
    float px;              // hit x (diagnostic builds only)
    float dx, dy, dz;      // p - o
    float depth;           // |p - o| (Eigen association: x + (y + z))
    float tnx, tny, tnz;   // t_to_next_boundary
    float tdx, tdy, tdz;   // t_step_size
    int vx, vy, vz;
    int sx, sy, sz;
    int rem;               // steps left (RayCaster: ray_length_in_steps - current_step)
    float w0;              // getVoxelWeight: 1, or 1 / z^2 (tsdf_params.depth_weight)
};

__device__ __forceinline__ void vb_axis(float ss, float es, int& v, int& st, float& tn, float& td,
                                        int& steps) {
    v = (int)__builtin_floorf(ss + 1e-6f);  // getGridIndexFromPoint: floor(x + kCoordinateEpsilon)
    const int e = (int)__builtin_floorf(es + 1e-6f);
    steps += e > v ? e - v : v - e;
    const float r = es - ss;
    st = (0.0f < r) - (r < 0.0f);
    const float corr = st > 0 ? 1.0f : 0.0f;
    tn = st == 0 ? __builtin_inff() : (corr - (ss - (float)v)) / r;
    td = st == 0 ? __builtin_inff() : (float)st / r;
}

// isPointValid + RayCaster setup; false when the ray is dropped.
// Ray slot i of the batch (R.ray_w: MergedTsdfIntegrator bundles, see RayConst).
__device__ __forceinline__ bool vb_init(const RayConst& R, const BatchRef& D, uint32_t t,
                                        uint32_t i, float px, float py, float pz, VbState& r) {
    const float ox = D.s[t].ox, oy = D.s[t].oy, oz = D.s[t].oz;
    const float dx = px - ox, dy = py - oy, dz = pz - oz;
    if (!in_sector(R, dx, dy)) return false;  // another GPU's azimuth sector
    const float depth = __builtin_sqrtf(dx * dx + (dy * dy + dz * dz));
    if (!(depth > 0.0f)) return false;
    bool clearing;
    float bw = 0.0f;
    if (R.ray_w) {
        // a bundle's ray: integrateVoxel passes the clearing flag and the summed weight, the ray's
        // length is not tested again
        bw = R.ray_w[i];
        if (bw == 0.0f) return false;
        clearing = bw < 0.0f;
    } else {
        if (depth < R.min_range) return false;
        clearing = depth > R.max_range;
        if (clearing && !R.allow_clear) return false;
    }
    const float ux = dx / depth, uy = dy / depth, uz = dz / depth;
    float ex, ey, ez, sx, sy, sz;
    if (clearing) {
        float len = depth - R.tau;
        len = len > 0.0f ? len : 0.0f;
        len = R.max_range < len ? R.max_range : len;
        ex = ox + ux * len;
        ey = oy + uy * len;
        ez = oz + uz * len;
        sx = ex;
        sy = ey;
        sz = ez;
    } else {
        ex = px + ux * R.tau;
        ey = py + uy * R.tau;
        ez = pz + uz * R.tau;
        sx = px - ux * R.tau;
        sy = py - uy * R.tau;
        sz = pz - uz * R.tau;
    }
    if (R.carving) {
        sx = ox;
        sy = oy;
        sz = oz;
    }
    int steps = 0;
    vb_axis(sx * R.inv_vs, ex * R.inv_vs, r.vx, r.sx, r.tnx, r.tdx, steps);
    vb_axis(sy * R.inv_vs, ey * R.inv_vs, r.vy, r.sy, r.tny, r.tdy, steps);
    vb_axis(sz * R.inv_vs, ez * R.inv_vs, r.vz, r.sz, r.tnz, r.tdz, steps);
    r.rem = min(steps, MAX_DDA_STEPS - 1);
    // TsdfIntegratorBase::getVoxelWeight: 1 / z^2 of the point's sensor-frame depth z (the scan's
    // z axis dotted with p - o, Eigen's x + (y + z)); |z| <= kEpsilon (1e-6) gives 0.  The weight
    // is capped at R.w0_cap = min(max_weight, 2^16) so the int64 fixed-point sums cannot overflow
    // (upstream's per-update max_weight cap bounds the fused weight the same way).  A scan without
    // an orientation (origin-only entry points: zero axis) takes the constant weight 1.
    r.w0 = 1.0f;
    if (R.ray_w) {
        r.w0 = fabsf(bw);
    } else if (R.depth_w) {
        const float zx = D.s[t].zx, zy = D.s[t].zy, zz = D.s[t].zz;
        if (zx != 0.0f || zy != 0.0f || zz != 0.0f) {
            const float z = fabsf(zx * dx + (zy * dy + zz * dz));
            r.w0 = z > 1e-6f ? fminf(1.0f / (z * z), R.w0_cap) : 0.0f;
        }
    }
    r.px = px;
    r.dx = dx;
    r.dy = dy;
    r.dz = dz;
    r.depth = depth;
    return true;
}

// updateTsdfVoxel's weight for a sample: the ray's getVoxelWeight w0, then the optional dropoff
__device__ __forceinline__ float vb_weight(const RayConst& R, float w0, float sdf) {
    float w = w0;
    if (R.dropoff && sdf < -R.vs) {
        w = (w * (R.tau + sdf)) / R.tau_m_vs;
        w = w > 0.0f ? w : 0.0f;
    }
    return w;
}

// computeDistance at the current voxel (projective sdf, untruncated); true when its weight is kept
__device__ __forceinline__ bool vb_sample(const RayConst& R, float ox, float oy, float oz,
                                          const VbState& r, float& s, bool check = true) {
    const bool inl = !check || (r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT &&
                                r.vy < VOX_LIMIT && r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT);
    const float cx = ((float)r.vx + 0.5f) * R.vs;
    const float cy = ((float)r.vy + 0.5f) * R.vs;
    const float cz = ((float)r.vz + 0.5f) * R.vs;
    const float ax = cx - ox, ay = cy - oy, az = cz - oz;
    const float proj = (ax * r.dx + (ay * r.dy + az * r.dz)) / r.depth;
    const float sdf = r.depth - proj;
    s = sdf;
    return inl && vb_weight(R, r.w0, sdf) >= VB_MIN_WEIGHT;
}

// nextRayIndex's advance: the first minimum of t_next (Eigen minCoeff) steps by its sign
__device__ __forceinline__ bool vb_step(VbState& r) {
    if (r.rem <= 0) return false;
    r.rem--;
    const bool y0 = r.tny < r.tnx;
    const float m01 = y0 ? r.tny : r.tnx;
    const bool mz = r.tnz < m01;
    const bool my = y0 && !mz;
    const bool mx = !y0 && !mz;
    r.tnx = mx ? r.tnx + r.tdx : r.tnx;
    r.tny = my ? r.tny + r.tdy : r.tny;
    r.tnz = mz ? r.tnz + r.tdz : r.tnz;
    r.vx += mx ? r.sx : 0;
    r.vy += my ? r.sy : 0;
    r.vz += mz ? r.sz : 0;
    return true;
}

// vb_step with selects (see ray_step_sel)
__device__ __forceinline__ bool vb_step_sel(VbState& r) {
    const bool adv = r.rem > 0;
    r.rem -= adv ? 1 : 0;
    const bool y0 = r.tny < r.tnx;
    const float m01 = y0 ? r.tny : r.tnx;
    const bool mz = (r.tnz < m01) && adv;
    const bool my = y0 && !(r.tnz < m01) && adv;
    const bool mx = !y0 && !(r.tnz < m01) && adv;
    r.tnx = mx ? r.tnx + r.tdx : r.tnx;
    r.tny = my ? r.tny + r.tdy : r.tny;
    r.tnz = mz ? r.tnz + r.tdz : r.tnz;
    r.vx += mx ? r.sx : 0;
    r.vy += my ? r.sy : 0;
    r.vz += mz ? r.sz : 0;
    return adv;
}

// The ray model of each semantics, as one interface for the walk kernels (k_count / k_place).
template <int SEM>
struct Walk;

template <>
struct Walk<0> {  // TSDF_SEM_VDBFUSION
    typedef RayState State;
    __device__ static __forceinline__ bool init(const RayConst& R, const BatchRef& D, uint32_t t,
                                                uint32_t i, float px, float py, float pz, State& r) {
        (void)i;
        return ray_init(R, D.s[t].ox, D.s[t].oy, D.s[t].oz, px, py, pz, r);
    }
    __device__ static __forceinline__ bool gate(const RayConst& R, float ox, float oy, float oz,
                                                const State& r, bool check = true) {
        return voxel_gate(R, ox, oy, oz, r, check);
    }
    __device__ static __forceinline__ bool gate_sel(const RayConst& R, float ox, float oy, float oz,
                                                    const State& r, bool check = true) {
        return voxel_gate_sel(R, ox, oy, oz, r, check);
    }
    __device__ static __forceinline__ bool sample(const RayConst& R, float ox, float oy, float oz,
                                                  const State& r, float& s, bool check = true) {
        return voxel_sample(R, ox, oy, oz, r, s, check);
    }
    __device__ static __forceinline__ bool sample_sel(const RayConst& R, float ox, float oy,
                                                      float oz, const State& r, float& s,
                                                      bool check = true) {
        return voxel_sample_sel(R, ox, oy, oz, r, s, check);
    }
    // the ray's voxels all lie inside |index| < VOX_LIMIT (so the per-voxel check can go)
    __device__ static __forceinline__ bool inside(const RayConst& R, const State& r) {
        const int m = max(max(abs(r.vx), abs(r.vy)), abs(r.vz));
        return m < VOX_LIMIT - R.band_vox;
    }
    __device__ static __forceinline__ bool step(State& r) { return ray_step(r); }
    __device__ static __forceinline__ bool step_sel(State& r) { return ray_step_sel(r); }
};

template <>
struct Walk<1> {  // TSDF_SEM_VOXBLOX
    typedef VbState State;
    __device__ static __forceinline__ bool init(const RayConst& R, const BatchRef& D, uint32_t t,
                                                uint32_t i, float px, float py, float pz, State& r) {
        return vb_init(R, D, t, i, px, py, pz, r);
    }
    __device__ static __forceinline__ bool gate(const RayConst& R, float ox, float oy, float oz,
                                                const State& r, bool check = true) {
        float s;
        return vb_sample(R, ox, oy, oz, r, s, check);
    }
    __device__ static __forceinline__ bool gate_sel(const RayConst& R, float ox, float oy, float oz,
                                                    const State& r, bool check = true) {
        float s;
        return vb_sample(R, ox, oy, oz, r, s, check);
    }
    __device__ static __forceinline__ bool sample(const RayConst& R, float ox, float oy, float oz,
                                                  const State& r, float& s, bool check = true) {
        return vb_sample(R, ox, oy, oz, r, s, check);
    }
    __device__ static __forceinline__ bool sample_sel(const RayConst& R, float ox, float oy,
                                                      float oz, const State& r, float& s,
                                                      bool check = true) {
        return vb_sample(R, ox, oy, oz, r, s, check);
    }
    __device__ static __forceinline__ bool inside(const RayConst& R, const State& r) {
        const int m = max(max(abs(r.vx), abs(r.vy)), abs(r.vz));
        return m < VOX_LIMIT - R.band_vox;
    }
    __device__ static __forceinline__ bool step(State& r) { return vb_step(r); }
    __device__ static __forceinline__ bool step_sel(State& r) { return vb_step_sel(r); }
};

// Voxblox with the 1/z^2 weight (internal sem 3): the same walk; k_place stores every sample's
// weight in its 12-B record (smp_store) because k_integrate cannot recompute it from the sample
template <>
struct Walk<3> : Walk<1> {};

// ------------------------------------------------------------------------------------------------
// VDBFusion at upstream's own precisions (TSDF_SEM_VDBFUSION_F64; the bit-exact twin of
// oracle/tsdf_oracle.c walk_ray_vdb): the Ray<float> VDBVolume::Integrate builds
// from double points and maps to index space (double scale), openvdb's float DDA, and
// GetVoxelCenter / ComputeSDF in double (Eigen's x + (y + z) reductions).  No contraction; double
// division and sqrt are IEEE (LLVM's correctly rounded f64 expansions).

// A wave-uniform double, declared so (its halves through readfirstlane): the compiler then keeps it
// in an SGPR pair instead of a VGPR pair.
__device__ __forceinline__ double uniform_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// (float)sqrt(x) of a double x >= 0 (ComputeSDF's (float)dist, VDBFusion's depth): LLVM's correctly
// rounded f64 sqrt sequence (v_rsq_f64 and two Newton-Raphson corrections; the hardware v_sqrt_f64
// is only ~2^-25 accurate, profiles/tools/sqrt_check) without its input scaling, which acts only
// below 2^-767: a nonzero squared distance is at least 2^-298 (p and the centre lie on the float
// grid, |b| >= 2^-149), a nonzero depth^2 far above it.  x = 0 gives 0, as the sequence's class
// check does.  RN_f of the correctly rounded double equals RN_f(sqrt(x)) (double rounding is
// innocuous for sqrt at 53 >= 2 * 24 + 2 bits).
__device__ __forceinline__ float vdb_sqrt_f(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r, h = r * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    h = __builtin_fma(h, e, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return x == 0.0 ? 0.0f : (float)g;
}

struct VdbState : RayState {
    double oxd, oyd, ozd;  // the origin as given (uniform over a k_count / k_place workgroup)
    const ScanRec* sr;     // its scan record (k_count's filter re-reads the origin from it)
    // k_count's fp32 filter of the double gate (vdb_gate_filtered): |proj_f - proj| <= ep and
    // |d2_f - d2| <= e2 hold for every voxel with d2_f <= bchk (so |p - c| <= bn); glo / ghi are
    // gate_d2 -/+ 2 e2
    float ep, glo, ghi, bchk;
};

__device__ __forceinline__ void vdb_axis(float di, float inv, float pos, float t0i, int v,
                                         float& tn, float& td, int& st) {
    if (di == 0.0f) {  // math::isZero: the axis is disabled
        st = 0;
        tn = 3.402823466e+38f;
        td = 3.402823466e+38f;
    } else if (inv > 0.0f) {
        st = 1;
        tn = t0i + ((float)(v + 1) - pos) * inv;
        td = inv;
    } else {
        st = -1;
        tn = t0i + ((float)v - pos) * inv;
        td = -inv;
    }
}

__device__ __forceinline__ bool vdb_init(const RayConst& R, const BatchRef& D, uint32_t t,
                                         float px, float py, float pz, VdbState& r) {
    if (!in_sector(R, px - D.s[t].ox, py - D.s[t].oy)) return false;  // another GPU's azimuth sector
    r.oxd = uniform_f64(D.s[t].odx);  // the workgroup's scan: keep the origin in SGPRs
    r.oyd = uniform_f64(D.s[t].ody);
    r.ozd = uniform_f64(D.s[t].odz);
    r.sr = D.s + t;
    const double dx = (double)px - r.oxd, dy = (double)py - r.oyd, dz = (double)pz - r.ozd;
    const float depth = (float)__builtin_sqrt(dx * dx + (dy * dy + dz * dz));  // direction.norm()
    if (!(depth > 0.0f)) return false;
    if (!(depth >= R.min_range) || !(depth <= R.max_range)) return false;
    const double il = 1.0 / __builtin_sqrt((dx * dx + dy * dy) + dz * dz);  // Vec3R::normalize
    const float t0 = R.carving ? 0.0f : depth - R.tau;
    const float t1 = depth + R.tau;
    // Ray<float>(eye, dir, t0, t1).worldToIndex(grid)
    const float ex = (float)((double)D.s[t].ox * R.inv_s_d);
    const float ey = (float)((double)D.s[t].oy * R.inv_s_d);
    const float ez = (float)((double)D.s[t].oz * R.inv_s_d);
    const float jx = (float)((double)(float)(dx * il) * R.inv_s_d);
    const float jy = (float)((double)(float)(dy * il) * R.inv_s_d);
    const float jz = (float)((double)(float)(dz * il) * R.inv_s_d);
    const float L = __builtin_sqrtf((jx * jx + jy * jy) + jz * jz);
    const float dix = jx / L, diy = jy / L, diz = jz / L;
    const float t0i = L * t0;
    r.t1i = L * t1;
    // math::DDA::init
    const float qx = ex + dix * t0i, qy = ey + diy * t0i, qz = ez + diz * t0i;
    r.vx = (int)__builtin_floorf(qx);
    r.vy = (int)__builtin_floorf(qy);
    r.vz = (int)__builtin_floorf(qz);
    vdb_axis(dix, 1.0f / dix, qx, t0i, r.vx, r.tnx, r.tdx, r.sx);
    vdb_axis(diy, 1.0f / diy, qy, t0i, r.vy, r.tny, r.tdy, r.sy);
    vdb_axis(diz, 1.0f / diz, qz, t0i, r.vz, r.tnz, r.tdz, r.sz);
    r.px = px;
    r.py = py;
    r.pz = pz;
    // Bounds of k_count's fp32 filter (u = 2^-24; every factor (1 + 2^-20) and the final 1.01
    // absorb the rounding of this bound arithmetic itself).  bn is any radius; a voxel whose fp32
    // squared distance d2_f <= bchk has |b_f| <= bn - sqrt3 db, hence for the exact b* = p - c*:
    //   |c*_i| <= (|p_i| + |b_f|)(1 + 3u) <= cmax           (c_f = fl(c*), b_f = fl(p - c_f))
    //   |b_f,i - b*_i| <= u (cmax + bn) = db,  |b*| <= bn,   |a*| <= |p - o| + bn <= amax
    //   |a_f,i - a*_i| <= u (cmax + omax + amax) = da         (a_f = fl(fl(c*) - fl(o)))
    //   |proj_f - proj_d| <= 3.0001u |a_f||b_f| + sqrt3 (amax db + bn da) + 3 da db + 2^-50 amax bn
    //   |d2_f - d2_d|     <= 3.0001u |b_f|^2 + 2 sqrt3 bn db + 3 db^2 + 2^-50 bn^2
    // (Cauchy-Schwarz for the sums of products; 2^-50 covers the double evaluation's own error).
    {
        constexpr float u = 5.9604645e-8f, s3 = 1.7320509f, g = 1.00000095f;  // 2^-24, sqrt 3, 1 + 2^-20
        const float bn = fmaxf(depth - t0, R.tau) + 2.0f * R.vs;
        const float pmax = fmaxf(fmaxf(fabsf(px), fabsf(py)), fabsf(pz));
        const float omax = fmaxf(fmaxf(fabsf(D.s[t].ox), fabsf(D.s[t].oy)), fabsf(D.s[t].oz)) * g;
        const float cmax = (pmax + bn) * g;
        const float amax = depth * g + bn;
        const float db = u * (cmax + bn) * g;
        const float da = u * (cmax + omax + amax) * g;
        const float am = amax + s3 * da, bm = bn + s3 * db;
        r.ep = 1.01f * (3.0001f * u * am * bm + s3 * (amax * db + bn * da) + 3.0f * da * db +
                        8.9e-16f * amax * bn);
        const float e2 = 1.01f * (3.0001f * u * bm * bm + 2.0f * s3 * bn * db + 3.0f * db * db +
                                  8.9e-16f * bn * bn);
        const float gf = (float)R.gate_d2;
        r.glo = gf - 2.0f * e2;
        r.ghi = gf + 2.0f * e2;
        const float bc = bn - s3 * db;
        r.bchk = bc * bc * (1.0f - 8.0f * u);
    }
    return true;
}

// GetVoxelCenter + ComputeSDF in double at the current voxel: proj and the squared distance.
// GetVoxelCenter's v vs + vs / 2 is exact in double ((2v + 1) < 2^25 times the 24-bit float vs),
// so it is formed as (2v + 1) (vs / 2): one conversion and one product per axis.  The axes are
// taken z, y, then x (Eigen's x + (y + z) reductions), so few double temporaries are live.
__device__ __forceinline__ void vdb_geom_at(double hv, double ox, double oy, double oz, float px,
                                            float py, float pz, int vx, int vy, int vz,
                                            double& proj, double& d2) {
    double c = (double)(int)(2u * (uint32_t)vz + 1u) * hv;
    double b = (double)pz - c;
    proj = (c - oz) * b;
    d2 = b * b;
    c = (double)(int)(2u * (uint32_t)vy + 1u) * hv;
    b = (double)py - c;
    proj = (c - oy) * b + proj;
    d2 = b * b + d2;
    c = (double)(int)(2u * (uint32_t)vx + 1u) * hv;
    b = (double)px - c;
    proj = (c - ox) * b + proj;
    d2 = b * b + d2;
}

__device__ __forceinline__ void vdb_geom(const RayConst& R, const VdbState& r, double& proj,
                                         double& d2) {
    // the point's double conversions are loop-invariant: the compiler hoists them out of the walk
    // (4 more VGPRs in k_place, whose occupancy LDS sets; 3 double conversions less per DDA step)
    float px = r.px, py = r.py, pz = r.pz;
#ifdef TSDF_F64_PER_VOXEL_P
    asm volatile("" : "+v"(px), "+v"(py), "+v"(pz));
#endif
    vdb_geom_at(R.hvs_d, r.oxd, r.oyd, r.ozd, px, py, pz, r.vx, r.vy, r.vz, proj,
                d2);
}

// The double gate's verdict (proj > 0, or proj < 0 and d2 < gate_d2) from fp32 arithmetic: the
// fp32 centre, offsets, projection and squared distance with the per-ray error bounds of vdb_init;
// a voxel whose verdict the bounds leave open (|proj_f| <= ep, d2_f within 2 e2 of gate_d2, d2_f
// beyond bchk, NaN) takes the double evaluation, in a branch the wave skips when none of its lanes
// needs it.  Bit-identical verdict to the double gate by construction.
__device__ __forceinline__ bool vdb_gate_filtered(const RayConst& R, float ox, float oy, float oz,
                                                  const VdbState& r) {
    const float cx = ((float)r.vx + 0.5f) * R.vs;
    const float cy = ((float)r.vy + 0.5f) * R.vs;
    const float cz = ((float)r.vz + 0.5f) * R.vs;
    const float ax = cx - ox, ay = cy - oy, az = cz - oz;
    const float bx = r.px - cx, by = r.py - cy, bz = r.pz - cz;
    const float proj = ax * bx + ay * by + az * bz;
    const float d2 = bx * bx + by * by + bz * bz;
    const bool pos = proj > r.ep, neg = proj < -r.ep;
    const bool in = d2 < r.glo, out = d2 >= r.ghi;
    bool g = pos || (neg && in);
    const bool open = !(d2 <= r.bchk) || !(pos || neg) || (neg && !(in || out));
    if (__builtin_expect(__any(open), 0)) {
#ifdef TSDF_F64_GATE_R05  // A/B only: round 5's branch (8 VGPR spills at the 6-wave bound)
        if (open) {
            // the origin, vs / 2 and the point re-read or re-converted here (opaque to hoisting),
            // so that the rare branch keeps no double live across the walk loop
            const ScanRec* q = r.sr;
            float px = r.px, py = r.py, pz = r.pz, vs = R.vs;
            asm volatile("" : "+v"(q), "+v"(px), "+v"(py), "+v"(pz), "+v"(vs));
            double pd, dd;
            vdb_geom_at((double)vs * 0.5, q->odx, q->ody, q->odz, px, py, pz, r.vx, r.vy, r.vz, pd, dd);
            g = pd > 0.0 || (pd < 0.0 && dd < R.gate_d2);
        }
#else
        if (open) {
            // the origin, vs / 2 and the point re-read or re-converted here (opaque to hoisting),
            // so that the rare branch keeps no double live across the walk loop
            // (the scan record and vs are wave-uniform, as vdb_init's origin: scalar registers, and
            // the record is read with scalar loads)
            // (readfirstlane returns int: both halves go through uint32_t, or the low half of the
            // address would be sign-extended into the high one)
            const uint64_t qv = (uint64_t)r.sr;
            const uint32_t qlo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)qv);
            const uint32_t qhi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(qv >> 32));
            uint64_t qa = ((uint64_t)qhi << 32) | qlo;
            float px = r.px, py = r.py, pz = r.pz;
            float vs = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, R.vs)));
            asm volatile("" : "+s"(qa), "+v"(px), "+v"(py), "+v"(pz), "+s"(vs));
            typedef const __attribute__((address_space(4))) ScanRec* ConstRec;
            const ConstRec q = (ConstRec)qa;
            // one origin component at a time, and the squared distance formed eagerly beside the
            // projection (no short-circuit): the branch then holds ~12 VGPRs of doubles and the
            // walk's registers stay where they are (no scratch spills at the 6-wave bound)
            const double hv = (double)vs * 0.5;
            double c = (double)(int)(2u * (uint32_t)r.vz + 1u) * hv;
            double b = (double)pz - c;
            double pd = (c - q->odz) * b;
            double dd = b * b;
            asm volatile("" : "+v"(pd), "+v"(dd));
            c = (double)(int)(2u * (uint32_t)r.vy + 1u) * hv;
            b = (double)py - c;
            pd = (c - q->ody) * b + pd;
            dd = b * b + dd;
            asm volatile("" : "+v"(pd), "+v"(dd));
            c = (double)(int)(2u * (uint32_t)r.vx + 1u) * hv;
            b = (double)px - c;
            pd = (c - q->odx) * b + pd;
            dd = b * b + dd;
            g = (pd > 0.0) | ((pd < 0.0) & (dd < R.gate_d2));
        }
#endif
    }
    return g;
}

__device__ __forceinline__ bool vdb_inside(const VdbState& r) {
    return r.vx > -VOX_LIMIT && r.vx < VOX_LIMIT && r.vy > -VOX_LIMIT && r.vy < VOX_LIMIT &&
           r.vz > -VOX_LIMIT && r.vz < VOX_LIMIT;
}

template <>
struct Walk<2> {  // TSDF_SEM_VDBFUSION_F64
    typedef VdbState State;
    __device__ static __forceinline__ bool init(const RayConst& R, const BatchRef& D, uint32_t t,
                                                uint32_t i, float px, float py, float pz, State& r) {
        (void)i;
        return vdb_init(R, D, t, px, py, pz, r);
    }
    // k_count: the verdict alone ((float)sqrt(d2) < tau, i.e. -dist > -tau, is d2 < gate_d2)
    __device__ static __forceinline__ bool gate(const RayConst& R, float ox, float oy, float oz,
                                                const State& r, bool check = true) {
        if (check && !vdb_inside(r)) return false;
        return vdb_gate_filtered(R, ox, oy, oz, r);
    }
    __device__ static __forceinline__ bool gate_sel(const RayConst& R, float ox, float oy, float oz,
                                                    const State& r, bool check = true) {
        const bool inl = !check || vdb_inside(r);
        return inl && vdb_gate_filtered(R, ox, oy, oz, r);
    }
    __device__ static __forceinline__ bool sample(const RayConst& R, float, float, float,
                                                  const State& r, float& s, bool check = true) {
        if (check && !vdb_inside(r)) return false;
        double proj, d2;
        vdb_geom(R, r, proj, d2);
        if (!(proj > 0.0 || proj < 0.0)) return false;
        const float dist = vdb_sqrt_f(d2);
        const float sdf = proj > 0.0 ? dist : -dist;
        if (!(sdf > -R.tau)) return false;
        s = sdf < R.tau ? sdf : R.tau;
        return true;
    }
    __device__ static __forceinline__ bool sample_sel(const RayConst& R, float ox, float oy,
                                                      float oz, const State& r, float& s,
                                                      bool check = true) {
        const bool inl = !check || vdb_inside(r);
        double proj, d2;
        vdb_geom(R, r, proj, d2);
        const float dist = vdb_sqrt_f(d2);
        const float sdf = proj > 0.0 ? dist : -dist;
        s = sdf < R.tau ? sdf : R.tau;
        return inl && (proj > 0.0 || proj < 0.0) && sdf > -R.tau;
    }
    __device__ static __forceinline__ bool inside(const RayConst& R, const State& r) {
        const int m = max(max(abs(r.vx), abs(r.vy)), abs(r.vz));
        return m < VOX_LIMIT - R.band_vox;
    }
    __device__ static __forceinline__ bool step(State& r) { return ray_step(r); }
    __device__ static __forceinline__ bool step_sel(State& r) { return ray_step_sel(r); }
};

__device__ __forceinline__ uint64_t pack_brick(int bx, int by, int bz) {
    return (uint64_t)(bx + BRICK_COORD_BIAS) | ((uint64_t)(by + BRICK_COORD_BIAS) << 21) |
           ((uint64_t)(bz + BRICK_COORD_BIAS) << 42);
}

__device__ __forceinline__ uint64_t brick_key_of(int vx, int vy, int vz) {
    return pack_brick(vx >> 3, vy >> 3, vz >> 3);
}

// A ray's brick, truncated to 10 bits per axis: consecutive gated voxels of a ray lie in the same
// or adjacent bricks (a monotone line, gated voxels contiguous up to isolated skips), so equal
// codes mean the same brick; a pair boundary is a code change (one 32-bit compare per voxel).
__device__ __forceinline__ uint32_t brick_code_of(int vx, int vy, int vz) {
    return ((uint32_t)(vx >> 3) & 1023u) | (((uint32_t)(vy >> 3) & 1023u) << 10) |
           (((uint32_t)(vz >> 3) & 1023u) << 20);
}

// The full key of a pair from its brick code and the ray's first brick: a ray's bricks lie within
// 511 bricks of each other per axis (in practice within one), so the truncated difference is exact.
__device__ __forceinline__ int code_axis(uint32_t c, int b0) {
    const int d = (int)((c - (uint32_t)b0) & 1023u);
    return b0 + ((d << 22) >> 22);
}

__device__ __forceinline__ uint64_t code_key(uint32_t code, int bx0, int by0, int bz0) {
    return pack_brick(code_axis(code & 1023u, bx0), code_axis((code >> 10) & 1023u, by0),
                      code_axis((code >> 20) & 1023u, bz0));
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

// Inclusive prefix sum over a wave's 64 lanes in DPP (row shifts 1/2/4/8 scan each 16-lane row,
// row broadcasts 15/31 carry the row totals): six VALU ops instead of six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Inclusive prefix sum within each aligned 16-lane row (the first four steps of wave_incl_scan).
__device__ __forceinline__ uint32_t row16_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    return x;
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

}  // namespace tsdf
