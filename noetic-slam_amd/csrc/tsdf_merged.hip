// tsdf_merged.hip — Voxblox MergedTsdfIntegrator's bundling pre-pass (tsdf_params.voxblox_method =
// TSDF_VB_MERGED).  The bit-exact CPU twin is oracle/tsdf_oracle.c mg_bundle.
//
// Per batch, before the walk kernels:
//   k_mg_keys   one lane per point (k_count's block layout: RPB points of one scan per block):
//               isPointValid, getVoxelWeight and the bundle key (clearing bit | the point's voxel,
//               21 biased bits per axis), inserted into a per-batch table whose slot becomes the
//               point's bundle id (2^tab_bits for a dropped point); every output ray slot starts
//               empty (NaN point, weight 0)
//   radix sort  (bundle id, point index) pairs over the whole batch, tab_bits + 1 key bits
//               (hipcub, stable: a bundle's points stay in cloud order, and equal voxels of
//               different scans in scan order)
//   k_mg_merge  one lane per sorted entry; the first entry of each (scan, key) run computes the
//               bundle's running weighted mean of p - o (integrateVoxel's merge, in the run's
//               order; a clearing bundle keeps its first kept point) and writes ONE ray -- o + mean,
//               weight (negative: clearing) -- into the slot of the bundle's first point; the
//               run's entries are loaded MG_U at a time ahead of the sequential merge.
// The walk kernels then run unchanged over the batch's slots (RayConst::ray_w), so block counts,
// offsets and the ray layout stay those of the input; empty slots leave at the walk's init.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

namespace {

constexpr int MG_THREADS = 256;
constexpr float MG_W_CAP = 1048576.0f;  // a bundle's weight cap (the fixed-point sums' headroom)
constexpr int MG_VOX_LIM = 1 << 20;     // voxel indices beyond drop the point (21-bit key axes)
// an empty key-table slot: no key is 0 (a kept voxel's biased axes lie in [1, 2^21 - 1])
constexpr uint64_t MG_EMPTY = 0ull;

__global__ __launch_bounds__(MG_THREADS) void k_mg_keys(const float* __restrict__ xyz, BatchRef D,
                                                        RayConst R, MgBufs M) {
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const float ox = D.s[t].ox, oy = D.s[t].oy, oz = D.s[t].oz;
    const float zx = D.s[t].zx, zy = D.s[t].zy, zz = D.s[t].zz;
    const bool axis = zx != 0.0f || zy != 0.0f || zz != 0.0f;
    const float nan = __builtin_nanf("");
    const float* __restrict__ xs = xyz + 3 * (size_t)D.s[t].xoff;  // the input (ABI v10 xoff)
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += MG_THREADS) {
        const float px = xs[3 * (size_t)i], py = xs[3 * (size_t)i + 1], pz = xs[3 * (size_t)i + 2];
        const float dx = px - ox, dy = py - oy, dz = pz - oz;
        const float depth = __builtin_sqrtf(dx * dx + (dy * dy + dz * dz));
        bool ok = depth > 0.0f && !(depth < R.min_range);
        const bool clearing = depth > R.max_range;
        ok = ok && (!clearing || R.allow_clear);
        // getGridIndexFromPoint(point_G, 1 / voxel_size): floor(x / vs + kCoordinateEpsilon)
        const float fx = __builtin_floorf(px * R.inv_vs + 1e-6f);
        const float fy = __builtin_floorf(py * R.inv_vs + 1e-6f);
        const float fz = __builtin_floorf(pz * R.inv_vs + 1e-6f);
        const float lim = (float)MG_VOX_LIM;
        ok = ok && fx > -lim && fx < lim && fy > -lim && fy < lim && fz > -lim && fz < lim;
        float pw = 1.0f;  // getVoxelWeight (vb_init's w0)
        if (R.depth_w && axis) {
            const float z = fabsf(zx * dx + (zy * dy + zz * dz));
            pw = z > 1e-6f ? fminf(1.0f / (z * z), R.w0_cap) : 0.0f;
        }
        // the bundle id: the slot of (clearing, voxel) in the batch's key table; a dropped point
        // sorts past every bundle
        uint32_t id = 1u << M.tab_bits;
        if (ok) {
            const uint64_t key = ((uint64_t)(clearing ? 1u : 0u) << 63) |
                                 ((uint64_t)(uint32_t)((int)fz + MG_VOX_LIM) << 42) |
                                 ((uint64_t)(uint32_t)((int)fy + MG_VOX_LIM) << 21) |
                                 (uint64_t)(uint32_t)((int)fx + MG_VOX_LIM);
            const uint64_t mask = (1ull << M.tab_bits) - 1ull;
            // the table holds >= 2x the batch's points, so a free slot always exists
            for (uint64_t h = mix64(key) & mask;; h = (h + 1) & mask) {
                const uint64_t k = M.tab[h];
                if (k == key) { id = (uint32_t)h; break; }
                if (k == MG_EMPTY) {
                    const unsigned long long old = atomicCAS((unsigned long long*)&M.tab[h],
                                                             (unsigned long long)MG_EMPTY,
                                                             (unsigned long long)key);
                    if (old == MG_EMPTY || old == key) { id = (uint32_t)h; break; }
                }
            }
        }
        M.key[i] = id;
        M.idx[i] = i;
        M.dw[i] = make_float4(dx, dy, dz, pw);
        M.sid[i] = (uint16_t)(t | (clearing ? 0x8000u : 0u));
        M.xyz_out[3 * (size_t)i] = nan;
        M.xyz_out[3 * (size_t)i + 1] = nan;
        M.xyz_out[3 * (size_t)i + 2] = nan;
        M.w_out[i] = 0.0f;
    }
}

// One lane per sorted entry; the lane at a (scan, key) run start merges the run.  The merge is a
// sequential running mean (bit for bit integrateVoxel's), but its operands need not arrive one
// dependent round trip at a time: the lane loads MG_U entries ahead (keys and indices contiguous,
// then the points' (d, w) gathers, all in flight together) and merges them from registers, so a
// long bundle (a near-range blob: thousands of points in one voxel) costs ~MG_U times fewer
// memory round trips.  A run ends at the next key or at the first point of a later scan (the sort
// is stable and a batch's points are in scan order, so the run's indices stay below the scan's end).
constexpr int MG_U = 8;
__global__ __launch_bounds__(MG_THREADS) void k_mg_merge(BatchRef D, MgBufs M, uint32_t n) {
    const uint32_t j = blockIdx.x * MG_THREADS + threadIdx.x;
    if (j >= n) return;
    const uint32_t key = M.key2[j];
    if (key >= (1u << M.tab_bits)) return;  // dropped points
    const uint32_t i0 = M.idx2[j];
    const uint32_t st = M.sid[i0];
    const uint32_t t = st & 0x7FFFu;
    const uint32_t lo = D.s[t].off, hi = D.s[t + 1].off;  // scan t's points
    const bool first = j == 0 || M.key2[j - 1] != key;   // the bundle id's first run
    if (!first && M.idx2[j - 1] >= lo) return;            // not a run start
    if (first) M.tab[key] = MG_EMPTY;                      // the slot is free for the next batch
    const bool clearing = (st & 0x8000u) != 0;
    float mx = 0.0f, my = 0.0f, mz = 0.0f, mw = 0.0f;
    for (uint32_t q = j;; q += MG_U) {
        uint32_t kk[MG_U];
        uint32_t ii[MG_U];
#pragma unroll
        for (int u = 0; u < MG_U; u++) {
            const bool in = q + u < n;
            kk[u] = in ? M.key2[q + u] : ~key;
            ii[u] = in ? M.idx2[q + u] : hi;
        }
        float4 dd[MG_U];
#pragma unroll
        for (int u = 0; u < MG_U; u++)
            dd[u] = (kk[u] == key && ii[u] < hi) ? M.dw[ii[u]] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        bool end = false;
#pragma unroll
        for (int u = 0; u < MG_U; u++) {
            end = end || kk[u] != key || ii[u] >= hi;
            const float4 d = dd[u];
            // kEpsilon; a clearing bundle keeps its first kept point only
            if (end || d.w < 1e-6f || (clearing && mw > 0.0f)) continue;
            const float nw = mw + d.w;
            mx = (mx * mw + d.x * d.w) / nw;
            my = (my * mw + d.y * d.w) / nw;
            mz = (mz * mw + d.z * d.w) / nw;
            mw = mw + d.w;
        }
        if (end) break;
    }
    if (!(mw > 0.0f)) return;
    M.xyz_out[3 * (size_t)i0] = D.s[t].ox + mx;
    M.xyz_out[3 * (size_t)i0 + 1] = D.s[t].oy + my;
    M.xyz_out[3 * (size_t)i0 + 2] = D.s[t].oz + mz;
    const float bw = mw < MG_W_CAP ? mw : MG_W_CAP;
    M.w_out[i0] = clearing ? -bw : bw;
}

}  // namespace

uint32_t mg_tab_bits(uint64_t n_points) {
    uint32_t b = 4;
    while ((1ull << b) < 2 * n_points) b++;
    return b;
}

size_t mg_sort_scratch(uint64_t n_points) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (int)n_points, 0,
                                             (int)mg_tab_bits(n_points) + 1);
    return bytes;
}

hipError_t launch_mg_prepass(const float* d_xyz, const BatchRef& B, uint32_t n_blocks,
                             uint64_t n_points, const RayConst& R, MgBufs& M, hipStream_t st) {
    if (!n_points) return hipSuccess;
    if (n_points > M.cap) return hipErrorInvalidValue;
    k_mg_keys<<<n_blocks, MG_THREADS, 0, st>>>(d_xyz, B, R, M);
    size_t bytes = M.tmp_bytes;
    // bundle ids are table slots (< 2^tab_bits) or 2^tab_bits for a dropped point: tab_bits + 1
    // key bits instead of the 64 of the voxel keys (4 sort passes instead of 8)
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(M.tmp, bytes, M.key, M.key2, M.idx, M.idx2,
                                                      (int)n_points, 0, (int)M.tab_bits + 1, st);
    if (e != hipSuccess) return e;
    k_mg_merge<<<(uint32_t)((n_points + MG_THREADS - 1) / MG_THREADS), MG_THREADS, 0, st>>>(
        B, M, (uint32_t)n_points);
    return hipGetLastError();
}

}  // namespace tsdf
