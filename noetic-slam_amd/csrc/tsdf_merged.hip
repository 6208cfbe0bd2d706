// tsdf_merged.hip — Voxblox MergedTsdfIntegrator's bundling pre-pass (tsdf_params.voxblox_method =
// TSDF_VB_MERGED).  The bit-exact CPU twin is oracle/tsdf_oracle.c mg_bundle.
//
// A bundle is the points of ONE scan that fall into one (clearing, voxel) key; it casts one ray from
// the running weighted mean of its points in cloud order.  About 97 % of a scan's points are alone in
// their bundle, so the pre-pass (round 6) never sorts: it finds the multi-point bundles through a
// batch-wide key table whose records carry per-scan bitmasks, merges only those, in place.
//   k_mg_keys    one lane per point (k_count's block layout: RPB points of one scan per block):
//                isPointValid and the bundle key (clearing bit | the point's voxel, 21 biased bits per
//                axis) inserted into the table of {key, seen, dup} records (its record h is the
//                point's `slot`), then seen[h] |= bit(scan) -- a second point of the scan in h also
//                sets dup[h] |= bit(scan)
//   k_mg_single  one lane per point: a point whose (slot, scan) is not dup is a one-point bundle and
//                writes its ray at once (the merge's arithmetic for one point, bit for bit); a dup
//                point joins its (slot, scan) group in a second table: the member count, the first
//                and last members (atomic max of ~index / index) and a member chain (atomic exchange
//                of the chain head; `next` per point)
//   k_mg_lead    one lane per point (the key table is emptied by a fill after k_mg_single): a
//                group's first point merges the group's members in cloud order and writes the
//                bundle's ray into its own slot, then frees the group record.  A group of at most
//                MG_SMALL members (nearly all) is read from its chain into registers and sorted
//                there -- its members may lie anywhere in the cloud (a voxel on the seam of the
//                spin has members at both ends); a larger one (a near-range blob) walks the scan's
//                slots from its first member to its last
// Scans t and t + 64 of one batch share a mask bit: two one-point bundles of such scans in one voxel
// both take the group path, which is exact too (each group merges its own scan's points).
// The walk kernels then run unchanged over the batch's slots (RayConst::ray_w), so block counts,
// offsets and the ray layout stay those of the input; empty slots (NaN point, weight 0) leave at the
// walk's init.
#include <hip/hip_runtime.h>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

namespace {

constexpr int MG_THREADS = 256;
constexpr float MG_W_CAP = 1048576.0f;  // a bundle's weight cap (the fixed-point sums' headroom)
constexpr int MG_VOX_LIM = 1 << 20;     // voxel indices beyond drop the point (21-bit key axes)
// an empty key-table slot: no key is 0 (a kept voxel's biased axes lie in [1, 2^21 - 1])
constexpr uint64_t MG_EMPTY = 0ull;
constexpr uint32_t MG_NONE = ~0u;  // a dropped point's slot / a one-point bundle's group
constexpr int MG_SMALL = 8;        // a group of up to this many members merges from its chain

// One point's bundle facts, shared by the three kernels (the oracle's mg_bundle, op for op):
// validity, the clearing flag, the bundle key, p - o and getVoxelWeight.
struct MgPoint {
    bool ok, clearing;
    uint64_t key;
    float dx, dy, dz, pw;
};

__device__ __forceinline__ MgPoint mg_point(const RayConst& R, float px, float py, float pz,
                                            float ox, float oy, float oz, float zx, float zy,
                                            float zz, bool axis) {
    MgPoint m;
    m.dx = px - ox;
    m.dy = py - oy;
    m.dz = pz - oz;
    const float depth = __builtin_sqrtf(m.dx * m.dx + (m.dy * m.dy + m.dz * m.dz));
    bool ok = depth > 0.0f && !(depth < R.min_range);
    m.clearing = depth > R.max_range;
    ok = ok && (!m.clearing || R.allow_clear);
    // getGridIndexFromPoint(point_G, 1 / voxel_size): floor(x / vs + kCoordinateEpsilon)
    const float fx = __builtin_floorf(px * R.inv_vs + 1e-6f);
    const float fy = __builtin_floorf(py * R.inv_vs + 1e-6f);
    const float fz = __builtin_floorf(pz * R.inv_vs + 1e-6f);
    const float lim = (float)MG_VOX_LIM;
    m.ok = ok && fx > -lim && fx < lim && fy > -lim && fy < lim && fz > -lim && fz < lim;
    m.key = m.ok ? ((uint64_t)(m.clearing ? 1u : 0u) << 63) |
                       ((uint64_t)(uint32_t)((int)fz + MG_VOX_LIM) << 42) |
                       ((uint64_t)(uint32_t)((int)fy + MG_VOX_LIM) << 21) |
                       (uint64_t)(uint32_t)((int)fx + MG_VOX_LIM)
                 : MG_EMPTY;
    m.pw = 1.0f;  // getVoxelWeight (vb_init's w0)
    if (R.depth_w && axis) {
        const float z = fabsf(zx * m.dx + (zy * m.dy + zz * m.dz));
        m.pw = z > 1e-6f ? fminf(1.0f / (z * z), R.w0_cap) : 0.0f;
    }
    return m;
}

// A key's home slot in a table of n records (n need not be a power of two: the tables are sized
// 1.25 x the batch's points, so the key table of a 64-scan batch fits the 256 MiB MALL)
__device__ __forceinline__ uint32_t mg_home(uint64_t key, uint32_t n) {
    return (uint32_t)(((mix64(key) >> 32) * (uint64_t)n) >> 32);
}
__device__ __forceinline__ uint32_t mg_next(uint32_t q, uint32_t n) { return q + 1u == n ? 0u : q + 1u; }

// integrateVoxel's merge step (kEpsilon; a clearing bundle keeps its first kept point only)
__device__ __forceinline__ void mg_step(const MgPoint& p, bool clearing, float& mx, float& my,
                                        float& mz, float& mw) {
    if (p.pw < 1e-6f || (clearing && mw > 0.0f)) return;
    const float nw = mw + p.pw;
    mx = (mx * mw + p.dx * p.pw) / nw;
    my = (my * mw + p.dy * p.pw) / nw;
    mz = (mz * mw + p.dz * p.pw) / nw;
    mw = mw + p.pw;
}

// The bundle's ray in the slot of its first point (no ray: NaN point, weight 0)
__device__ __forceinline__ void mg_out(const MgBufs& M, uint32_t i, const ScanRec& s, bool clearing,
                                       float mx, float my, float mz, float mw) {
    float x = __builtin_nanf(""), y = x, z = x, w = 0.0f;
    if (mw > 0.0f) {
        x = s.ox + mx;
        y = s.oy + my;
        z = s.oz + mz;
        const float bw = mw < MG_W_CAP ? mw : MG_W_CAP;
        w = clearing ? -bw : bw;
    }
    M.xyz_out[3 * (size_t)i] = x;
    M.xyz_out[3 * (size_t)i + 1] = y;
    M.xyz_out[3 * (size_t)i + 2] = z;
    M.w_out[i] = w;
}

__global__ __launch_bounds__(MG_THREADS) void k_mg_keys(const float* __restrict__ xyz, BatchRef D,
                                                        RayConst R, MgBufs M, uint32_t* ovf) {
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const ScanRec s = D.s[t];
    const bool axis = s.zx != 0.0f || s.zy != 0.0f || s.zz != 0.0f;
    const float* __restrict__ xs = xyz + 3 * (size_t)s.xoff;  // the input (ABI v10 xoff)
    const uint64_t bit = 1ull << (t & 63u);
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += MG_THREADS) {
        const MgPoint p = mg_point(R, xs[3 * (size_t)i], xs[3 * (size_t)i + 1],
                                   xs[3 * (size_t)i + 2], s.ox, s.oy, s.oz, s.zx, s.zy, s.zz, axis);
        uint32_t h = MG_NONE;
        if (p.ok) {
            // the table holds >= 1.25 x the batch's points, so a free slot exists; the probe count
            // is capped all the same (an exhausted probe drops the point and raises OVF_MG)
            uint32_t q = mg_home(p.key, M.tab_n);
            for (uint32_t n = 0; n < M.tab_n; n++, q = mg_next(q, M.tab_n)) {
                const uint64_t k = M.tab[3 * (size_t)q];
                if (k == p.key) {
                    h = q;
                    break;
                }
                if (k == MG_EMPTY) {
                    const unsigned long long old = atomicCAS((unsigned long long*)&M.tab[3 * (size_t)q],
                                                             (unsigned long long)MG_EMPTY,
                                                             (unsigned long long)p.key);
                    if (old == MG_EMPTY || old == p.key) {
                        h = q;
                        break;
                    }
                }
            }
            if (h == MG_NONE) {
                atomicOr(ovf, OVF_MG);
            } else {
                const unsigned long long old = atomicOr((unsigned long long*)&M.tab[3 * (size_t)h + 1], bit);
                if (old & bit) atomicOr((unsigned long long*)&M.tab[3 * (size_t)h + 2], bit);
            }
        }
        M.slot[i] = h;
    }
}

__global__ __launch_bounds__(MG_THREADS) void k_mg_single(const float* __restrict__ xyz, BatchRef D,
                                                          RayConst R, MgBufs M, uint32_t* ovf) {
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const ScanRec s = D.s[t];
    const bool axis = s.zx != 0.0f || s.zy != 0.0f || s.zz != 0.0f;
    const float* __restrict__ xs = xyz + 3 * (size_t)s.xoff;
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += MG_THREADS) {
        const uint32_t h = M.slot[i];
        uint32_t g = MG_NONE;
        bool single = false;
        if (h != MG_NONE) single = ((M.tab[3 * (size_t)h + 2] >> (t & 63u)) & 1ull) == 0ull;
        if (single) {  // a one-point bundle: its ray now
            const MgPoint p = mg_point(R, xs[3 * (size_t)i], xs[3 * (size_t)i + 1],
                                       xs[3 * (size_t)i + 2], s.ox, s.oy, s.oz, s.zx, s.zy, s.zz,
                                       axis);
            float mx = 0.0f, my = 0.0f, mz = 0.0f, mw = 0.0f;
            mg_step(p, p.clearing, mx, my, mz, mw);
            mg_out(M, i, s, p.clearing, mx, my, mz, mw);
        } else {
            mg_out(M, i, s, false, 0.0f, 0.0f, 0.0f, 0.0f);  // no ray here (a group's leader's later)
            if (h != MG_NONE) {  // join the (slot, scan) group
                const uint64_t key = ((uint64_t)h << 16) | (uint64_t)(t + 1u);  // never 0
                uint32_t q = mg_home(key, M.grp_n);
                for (uint32_t n = 0; n < M.grp_n; n++, q = mg_next(q, M.grp_n)) {
                    const uint64_t k = M.grp[4 * (size_t)q];
                    if (k == key) {
                        g = q;
                        break;
                    }
                    if (k == MG_EMPTY) {
                        const unsigned long long old = atomicCAS((unsigned long long*)&M.grp[4 * (size_t)q],
                                                                 (unsigned long long)MG_EMPTY,
                                                                 (unsigned long long)key);
                        if (old == MG_EMPTY || old == key) {
                            g = q;
                            break;
                        }
                    }
                }
                if (g == MG_NONE) {
                    atomicOr(ovf, OVF_MG);
                } else {
                    uint32_t* v = reinterpret_cast<uint32_t*>(&M.grp[4 * (size_t)g + 1]);
                    atomicMax(&v[0], ~i);                 // the first member (~index; 0: none)
                    atomicAdd(&v[1], 1u);                 // the members
                    atomicMax(&v[2], i);                  // the last member
                    M.next[i] = atomicExch(&v[3], i + 1u);  // the chain (index + 1; 0 ends it)
                }
            }
        }
        M.gid[i] = g;
    }
}

__global__ __launch_bounds__(MG_THREADS) void k_mg_lead(const float* __restrict__ xyz, BatchRef D,
                                                        RayConst R, MgBufs M) {
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const ScanRec s = D.s[t];
    const uint32_t hi = D.s[t + 1].off;  // scan t's points end here
    const bool axis = s.zx != 0.0f || s.zy != 0.0f || s.zz != 0.0f;
    const float* __restrict__ xs = xyz + 3 * (size_t)s.xoff;
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += MG_THREADS) {
        const uint32_t g = M.gid[i];
        if (g == MG_NONE) continue;
        const uint64_t v = M.grp[4 * (size_t)g + 1];
        if (~(uint32_t)v != i) continue;  // not the group's first point (or already freed: 0)
        const uint32_t h = M.slot[i];
        const uint32_t cnt = (uint32_t)(v >> 32);
        const uint64_t v2 = M.grp[4 * (size_t)g + 2];
        const uint32_t last = (uint32_t)v2, head = (uint32_t)(v2 >> 32);
        // the group record is read by its members only for this test: the leader frees it now (a
        // member reading the zeros afterwards sees ~0 != its index, i.e. not the leader, as before)
        *reinterpret_cast<ulonglong2*>(&M.grp[4 * (size_t)g]) = make_ulonglong2(0ull, 0ull);
        M.grp[4 * (size_t)g + 2] = 0ull;
        // the members are the points of scan t in slot h, in cloud order from this one on
        float mx = 0.0f, my = 0.0f, mz = 0.0f, mw = 0.0f;
        bool clearing = false;
        auto merge_at = [&](uint32_t j) {
            const MgPoint p = mg_point(R, xs[3 * (size_t)j], xs[3 * (size_t)j + 1],
                                       xs[3 * (size_t)j + 2], s.ox, s.oy, s.oz, s.zx, s.zy, s.zz,
                                       axis);
            clearing = p.clearing;  // (the slot's key carries it: the same for every member)
            mg_step(p, clearing, mx, my, mz, mw);
        };
        if (cnt <= MG_SMALL) {
            // a small group (nearly all of them: two or three points): its chain, loaded once into
            // registers (a static index per slot: no scratch), sorted by a compare-exchange
            // network, merged in cloud order; cnt dependent loads, wherever the members lie (a
            // voxel on the seam of the spin has members at both ends of the cloud)
            uint32_t m[MG_SMALL];
            uint32_t e = head;
#pragma unroll
            for (int q = 0; q < MG_SMALL; q++) {
                const bool on = e != 0u;
                m[q] = on ? e - 1u : ~0u;
                e = on ? M.next[e - 1u] : 0u;
            }
#pragma unroll
            for (int a = 0; a < MG_SMALL; a++)  // odd-even transposition sort (MG_SMALL rounds)
#pragma unroll
                for (int q = a & 1; q + 1 < MG_SMALL; q += 2) {
                    const uint32_t lo_ = min(m[q], m[q + 1]), hi_ = max(m[q], m[q + 1]);
                    m[q] = lo_;
                    m[q + 1] = hi_;
                }
#pragma unroll
            for (int q = 0; q < MG_SMALL; q++)
                if (m[q] != ~0u) merge_at(m[q]);
        } else {
            // a large group (a near-range blob): forward over the scan's slots from the first
            // member to the last, four slots per 16-B load
            uint32_t found = 0;
            const uint32_t end = min(last + 1u, hi);
            for (uint32_t j0 = i & ~3u; j0 < end && found < cnt; j0 += 4u) {
                const uint4 q4 = *reinterpret_cast<const uint4*>(M.slot + j0);
                const uint32_t sl[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t j = j0 + (uint32_t)u;
                    if (j >= i && j < end && sl[u] == h) {
                        merge_at(j);
                        found++;
                    }
                }
            }
        }
        mg_out(M, i, s, clearing, mx, my, mz, mw);
    }
}

// Empties the key table for the next batch: one grid-stride streaming fill of 16-B stores (the
// table is 24 B x a multiple of 64 records)
__global__ __launch_bounds__(256) void k_mg_clear(uint4* __restrict__ p, uint64_t n16) {
    for (uint64_t q = blockIdx.x * 256ull + threadIdx.x; q < n16; q += (uint64_t)gridDim.x * 256ull)
        p[q] = make_uint4(0u, 0u, 0u, 0u);
}

}  // namespace

uint32_t mg_table_records(uint64_t n_points) {
    // >= 1.25 x the batch's points, a multiple of 64 records (k_mg_clear's 16-B stores)
    const uint64_t n = (n_points + n_points / 4 + 127) & ~63ull;
    return (uint32_t)std::min<uint64_t>(n, 0xFFFFFFC0ull);
}

hipError_t launch_mg_prepass(const float* d_xyz, const BatchRef& B, uint32_t n_blocks,
                             uint64_t n_points, const RayConst& R, MgBufs& M, uint32_t* ovf,
                             hipStream_t st) {
    if (!n_points) return hipSuccess;
    if (n_points > M.cap) return hipErrorInvalidValue;
    k_mg_keys<<<n_blocks, MG_THREADS, 0, st>>>(d_xyz, B, R, M, ovf);
    k_mg_single<<<n_blocks, MG_THREADS, 0, st>>>(d_xyz, B, R, M, ovf);
    k_mg_lead<<<n_blocks, MG_THREADS, 0, st>>>(d_xyz, B, R, M);
    // the key table's last readers ran (k_mg_single): empty it for the next batch in one streaming
    // fill (24 B a record; clearing each point's record from k_mg_lead cost 0.4 ms of scattered
    // partial-line stores per 64-scan batch)
    const uint64_t n16 = (uint64_t)24 * M.tab_n / 16;
    k_mg_clear<<<(uint32_t)std::min<uint64_t>((n16 + 255) / 256, 8192), 256, 0, st>>>(
        reinterpret_cast<uint4*>(M.tab), n16);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        // a pre-pass cut short may leave groups in the group table: empty it too, so the next batch
        // starts from empty tables
        (void)hipMemsetAsync(M.grp, 0, (size_t)32 * M.grp_n, st);
    }
    return e;
}

}  // namespace tsdf
