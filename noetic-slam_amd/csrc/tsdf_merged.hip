// tsdf_merged.hip — Voxblox MergedTsdfIntegrator's bundling pre-pass (tsdf_params.voxblox_method =
// TSDF_VB_MERGED).  The bit-exact CPU twin is oracle/tsdf_oracle.c mg_bundle.
//
// A bundle is the points of ONE scan that fall into one (clearing, voxel) key; it casts one ray from
// the running weighted mean of its points in cloud order.  About 97 % of a scan's points are alone in
// their bundle.  The pre-pass (round 6, second form) keeps every random access in LDS: the points are
// partitioned by a hash of their key into buckets of about 1024 points of one scan, and one
// workgroup per bucket finds and merges that bucket's multi-point bundles in an LDS table.
//   k_mg_count    one lane per point (k_count's block layout: RPB points of one scan per block):
//                 isPointValid, the bundle key (clearing bit | the point's voxel, 21 biased bits per
//                 axis) and its bucket; the point's ray as a one-point bundle (the merge's arithmetic
//                 for one point, bit for bit; no ray for a dropped one); bucket sizes through an LDS
//                 histogram, one global add per (block, bucket) to one of MG_REP replica counters
//   k_mg_scan     one workgroup: bucket starts (exclusive prefix); the sizes zeroed for use as
//                 cursors; each bucket's scan
//   k_mg_scatter  the same blocks again: (key, point) entries into their buckets (an LDS rank plus
//                 one returning global add per (block, bucket) on its replica's cursor)
//   k_mg_group    one workgroup per bucket: its keys into an LDS hash table (a key met again is
//                 marked); the entries of keys seen more than once (the multi-point bundles' members) gathered in
//                 LDS as (table slot, point) and sorted, so each bundle's members lie together in
//                 cloud order; the first member's lane merges them and writes the bundle's ray into
//                 its slot, the other members write "no ray" over their one-point rays.  A bucket with
//                 more members than the LDS list holds (a coarse voxel near the sensor) walks each
//                 bundle's points from its first member to its last instead.
// The walk kernels then run unchanged over the batch's slots (RayConst::ray_w), so block counts,
// offsets and the ray layout stay those of the input; empty slots (NaN point, weight 0) leave at the
// walk's init.  Limit: a bucket holds at most MG_TAB distinct keys (about 2 x its expected count;
// scans of more than ~2^22 points may exceed it): beyond, the batch fails with OVF_MG.
#include <hip/hip_runtime.h>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

namespace {

constexpr int MG_THREADS = 256;
constexpr float MG_W_CAP = 1048576.0f;  // a bundle's weight cap (the fixed-point sums' headroom)
constexpr int MG_VOX_LIM = 1 << 20;     // voxel indices beyond drop the point (21-bit key axes)
// an empty LDS table slot: no key is 0 (a kept voxel's biased axes lie in [1, 2^21 - 1])
constexpr uint64_t MG_EMPTY = 0ull;
constexpr uint32_t MG_NONE = ~0u;
constexpr int MG_BSHIFT = 10;       // a scan's buckets hold about 2^MG_BSHIFT points each
constexpr uint32_t MG_PMAX = 4096;  // buckets per scan at most (the LDS histograms)
constexpr uint32_t MG_TAB = 2048;   // k_mg_group: distinct keys per bucket (LDS hash table)
constexpr uint32_t MG_GM = 2048;    // k_mg_group: multi-point bundle members sorted in LDS
constexpr int MG_PPT = RPB / MG_THREADS;  // points per lane in k_mg_scatter
// bucket counters in MG_REP replicas (replica r = block index mod MG_REP, each replica's counters
// contiguous): the ~100 blocks of a scan reserve their runs in the same buckets at the same time,
// and one counter per bucket queued their returning atomics at the memory side
constexpr uint32_t MG_REP = MG_REPLICAS;
static_assert(RPB % MG_THREADS == 0, "k_mg_scatter keeps RPB / MG_THREADS points per lane");

// scan t's bucket count and first bucket: base(t) = off(t) / 2^MG_BSHIFT + t, so that
// base(t) + buckets(t) <= base(t + 1), and a batch has n_points / 2^MG_BSHIFT + scans buckets
__device__ __forceinline__ uint32_t mg_buckets(uint32_t n) {
    return min(max((n + (1u << MG_BSHIFT) - 1u) >> MG_BSHIFT, 1u), MG_PMAX);
}
__device__ __forceinline__ uint32_t mg_bucket_base(uint32_t off, uint32_t t) {
    return (off >> MG_BSHIFT) + t;
}
// a key's bucket among P (the hash's high half; the LDS table takes its low half)
__device__ __forceinline__ uint32_t mg_bucket(uint64_t key, uint32_t P) {
    return (uint32_t)(((mix64(key) >> 32) * (uint64_t)P) >> 32);
}

// One point's bundle facts, shared by the kernels (the oracle's mg_bundle, op for op): validity,
// the clearing flag, the bundle key, p - o and getVoxelWeight.
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

__global__ __launch_bounds__(MG_THREADS) void k_mg_count(const float* __restrict__ xyz, BatchRef D,
                                                         RayConst R, MgBufs M) {
    __shared__ uint32_t hist[MG_PMAX];
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const ScanRec s = D.s[t];
    const uint32_t P = mg_buckets(D.s[t + 1].off - s.off);
    const bool axis = s.zx != 0.0f || s.zy != 0.0f || s.zz != 0.0f;
    const float* __restrict__ xs = xyz + 3 * (size_t)s.xoff;  // the input (ABI v10 xoff)
    for (uint32_t j = threadIdx.x; j < P; j += MG_THREADS) hist[j] = 0u;
    __syncthreads();
    float px[MG_PPT], py[MG_PPT], pz[MG_PPT];  // the block's points, all loads in flight at once
#pragma unroll
    for (int k = 0; k < MG_PPT; k++) {
        const uint32_t i = min(r0 + threadIdx.x + k * MG_THREADS, r1 - 1u);
        px[k] = xs[3 * (size_t)i];
        py[k] = xs[3 * (size_t)i + 1];
        pz[k] = xs[3 * (size_t)i + 2];
    }
#pragma unroll
    for (int k = 0; k < MG_PPT; k++) {
        const uint32_t i = r0 + threadIdx.x + k * MG_THREADS;
        if (i >= r1) break;
        const MgPoint p = mg_point(R, px[k], py[k], pz[k], s.ox, s.oy, s.oz, s.zx, s.zy, s.zz, axis);
        // every point's ray as a one-point bundle (k_mg_group rewrites the multi-point ones)
        float mx = 0.0f, my = 0.0f, mz = 0.0f, mw = 0.0f;
        if (p.ok) {
            mg_step(p, p.clearing, mx, my, mz, mw);
            atomicAdd(&hist[mg_bucket(p.key, P)], 1u);
        }
        mg_out(M, i, s, p.clearing, mx, my, mz, mw);
    }
    __syncthreads();
    const uint32_t base = mg_bucket_base(s.off, t);
    for (uint32_t j = threadIdx.x; j < P; j += MG_THREADS)
        if (hist[j]) atomicAdd(&M.bcnt[(blockIdx.x % MG_REP) * M.nb_cap + base + j], hist[j]);
}

// bucket starts: bst[b] = the sizes of the buckets before b, bst[nb] = the entries; each replica
// counter becomes its runs' first entry (k_mg_scatter's cursor: bucket b's entries hold replica 0's
// runs, then replica 1's, ...)
constexpr int MG_SCAN_THREADS = 1024;
__global__ __launch_bounds__(MG_SCAN_THREADS) void k_mg_scan(BatchRef D, MgBufs M, uint32_t nb) {
    __shared__ uint32_t s_w[MG_SCAN_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    // 1. bucket sizes over the replicas into bst (lanes on consecutive buckets: coalesced)
    for (uint32_t j = tid; j < nb; j += MG_SCAN_THREADS) {
        uint32_t c = 0;
#pragma unroll
        for (uint32_t r = 0; r < MG_REP; r++) c += M.bcnt[r * M.nb_cap + j];
        M.bst[j] = c;
    }
    __syncthreads();
    // 2. their exclusive prefix (a contiguous range of buckets per lane)
    const uint32_t per = (nb + MG_SCAN_THREADS - 1) / MG_SCAN_THREADS;
    const uint32_t j0 = min(nb, tid * per), j1 = min(nb, j0 + per);
    uint32_t sum = 0;
    for (uint32_t j = j0; j < j1; j++) sum += M.bst[j];
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63u) s_w[wid] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < MG_SCAN_THREADS / 64; k++) {
        off += k < wid ? s_w[k] : 0u;
        tot += s_w[k];
    }
    uint32_t run = incl - sum + off;
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t c = M.bst[j];
        M.bst[j] = run;
        run += c;
    }
    __syncthreads();
    // 3. each replica's first entry (coalesced again)
    for (uint32_t j = tid; j < nb; j += MG_SCAN_THREADS) {
        uint32_t r0 = M.bst[j];
#pragma unroll
        for (uint32_t r = 0; r < MG_REP; r++) {
            const uint32_t c = M.bcnt[r * M.nb_cap + j];
            M.bcnt[r * M.nb_cap + j] = r0;
            r0 += c;
        }
    }
    if (tid == 0) M.bst[nb] = tot;
    // each bucket's scan, for k_mg_group (a table instead of its binary search over the scans:
    // nine dependent scalar loads per workgroup)
    for (uint32_t t = tid; t < D.n_scans; t += MG_SCAN_THREADS) {
        const uint32_t b0 = mg_bucket_base(D.s[t].off, t), P = mg_buckets(D.s[t + 1].off - D.s[t].off);
        for (uint32_t j = 0; j < P; j++) M.bscan[b0 + j] = t;
    }
}

__global__ __launch_bounds__(MG_THREADS) void k_mg_scatter(const float* __restrict__ xyz, BatchRef D,
                                                           RayConst R, MgBufs M) {
    __shared__ uint32_t hist[MG_PMAX];
    uint32_t t, r0, r1;
    block_range(D, blockIdx.x, t, r0, r1);
    const ScanRec s = D.s[t];
    const uint32_t P = mg_buckets(D.s[t + 1].off - s.off);
    const float* __restrict__ xs = xyz + 3 * (size_t)s.xoff;
    for (uint32_t j = threadIdx.x; j < P; j += MG_THREADS) hist[j] = 0u;
    __syncthreads();
    uint64_t key[MG_PPT];
    uint32_t bk[MG_PPT], rk[MG_PPT];
    float px[MG_PPT], py[MG_PPT], pz[MG_PPT];  // all loads in flight at once
#pragma unroll
    for (int k = 0; k < MG_PPT; k++) {
        const uint32_t i = min(r0 + threadIdx.x + k * MG_THREADS, r1 - 1u);
        px[k] = xs[3 * (size_t)i];
        py[k] = xs[3 * (size_t)i + 1];
        pz[k] = xs[3 * (size_t)i + 2];
    }
#pragma unroll
    for (int k = 0; k < MG_PPT; k++) {
        const uint32_t i = r0 + threadIdx.x + k * MG_THREADS;
        bk[k] = MG_NONE;
        key[k] = MG_EMPTY;
        rk[k] = 0u;
        if (i < r1) {
            // (the key and validity only: the weight's inputs do not enter them)
            const MgPoint p = mg_point(R, px[k], py[k], pz[k], s.ox, s.oy, s.oz, 0.0f, 0.0f, 0.0f,
                                       false);
            if (p.ok) {
                key[k] = p.key;
                bk[k] = mg_bucket(p.key, P);
                rk[k] = atomicAdd(&hist[bk[k]], 1u);
            }
        }
    }
    __syncthreads();
    // the block's run in each of its buckets (its replica's cursor): its first entry replaces the
    // count
    const uint32_t base = mg_bucket_base(s.off, t);
    for (uint32_t j = threadIdx.x; j < P; j += MG_THREADS) {
        const uint32_t c = hist[j];
        if (c) hist[j] = atomicAdd(&M.bcnt[(blockIdx.x % MG_REP) * M.nb_cap + base + j], c);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MG_PPT; k++) {
        if (bk[k] == MG_NONE) continue;
        const uint32_t e = hist[bk[k]] + rk[k];
        M.ekey[e] = key[k];
        M.eidx[e] = r0 + threadIdx.x + k * MG_THREADS;
    }
}

constexpr int MG_GTHREADS = 512;  // k_mg_group: lanes per bucket
constexpr int MG_EPT = 3;         // k_mg_group: entries per lane kept in registers
__global__ __launch_bounds__(MG_GTHREADS) void k_mg_group(const float* __restrict__ xyz, BatchRef D,
                                                          RayConst R, MgBufs M, uint32_t* ovf) {
    __shared__ uint64_t tkey[MG_TAB];  // the bucket's keys (open addressing)
    __shared__ uint8_t tdup[MG_TAB];   // the key was seen more than once
    __shared__ uint64_t gm[MG_GM];     // the multi-point bundles' members: slot << 32 | point
    __shared__ uint32_t n_gm;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t e0 = M.bst[b], e1 = M.bst[b + 1];
    if (tid < MG_REP) M.bcnt[tid * M.nb_cap + b] = 0u;  // the cursors: zero for the next batch
    if (e0 == e1) return;
    if (tid == 0) n_gm = 0u;
    const ScanRec s = D.s[M.bscan[b]];  // the bucket's scan (k_mg_scan's table)
    const bool axis = s.zx != 0.0f || s.zy != 0.0f || s.zz != 0.0f;
    const float* __restrict__ xs = xyz + 3 * (size_t)s.xoff;
    // the first MG_EPT x MG_GTHREADS entries stay in registers (nearly every bucket: ~1024)
    uint64_t ek[MG_EPT];
    uint32_t ei[MG_EPT], eq[MG_EPT];
#pragma unroll
    for (int k = 0; k < MG_EPT; k++) {
        const uint32_t e = min(e0 + tid + k * MG_GTHREADS, e1 - 1u);
        ek[k] = M.ekey[e];
        ei[k] = M.eidx[e];
    }
    for (uint32_t j = tid; j < MG_TAB; j += MG_GTHREADS) {
        tkey[j] = MG_EMPTY;
        tdup[j] = 0;
    }
    __syncthreads();
    // the key's slot; insert: a key already present (or inserted meanwhile) is marked as seen twice
    auto find = [&](uint64_t key, bool insert) {
        uint32_t q = (uint32_t)mix64(key) & (MG_TAB - 1u);
        for (uint32_t n = 0; n < MG_TAB; n++, q = (q + 1u) & (MG_TAB - 1u)) {
            uint64_t k = tkey[q];
            if (k == MG_EMPTY && insert)
                k = atomicCAS((unsigned long long*)&tkey[q], (unsigned long long)MG_EMPTY,
                              (unsigned long long)key);
            if (k == key) {
                if (insert) tdup[q] = 1;
                return q;
            }
            if (k == MG_EMPTY) {
                if (!insert) return MG_NONE;
                return q;  // this lane inserted it
            }
        }
        return MG_NONE;
    };
    const uint32_t e_reg = e0 + MG_EPT * MG_GTHREADS;  // entries from here on are re-read
#pragma unroll
    for (int k = 0; k < MG_EPT; k++) {
        eq[k] = MG_NONE;
        if (e0 + tid + k * MG_GTHREADS < e1) {
            eq[k] = find(ek[k], true);
            if (eq[k] == MG_NONE) atomicOr(ovf, OVF_MG);  // more distinct keys than MG_TAB
        }
    }
    for (uint32_t e = e_reg + tid; e < e1; e += MG_GTHREADS)
        if (find(M.ekey[e], true) == MG_NONE) atomicOr(ovf, OVF_MG);
    __syncthreads();
    auto add_member = [&](uint32_t q, uint32_t i) {
        if (q != MG_NONE && tdup[q]) {
            const uint32_t g = atomicAdd(&n_gm, 1u);
            if (g < MG_GM) gm[g] = ((uint64_t)q << 32) | i;
        }
    };
#pragma unroll
    for (int k = 0; k < MG_EPT; k++) add_member(eq[k], ei[k]);
    for (uint32_t e = e_reg + tid; e < e1; e += MG_GTHREADS) add_member(find(M.ekey[e], false), M.eidx[e]);
    __syncthreads();
    const uint32_t ng = n_gm;
    if (ng == 0) return;
    float mx, my, mz, mw;
    bool clearing;
    auto merge_at = [&](float px, float py, float pz) {
        const MgPoint p = mg_point(R, px, py, pz, s.ox, s.oy, s.oz, s.zx, s.zy, s.zz, axis);
        clearing = p.clearing;  // (the key carries it: the same for every member)
        mg_step(p, clearing, mx, my, mz, mw);
    };
    if (ng <= MG_GM) {
        // sort (slot, point): a bundle's members together, in cloud order
        if (ng <= (uint32_t)MG_GTHREADS) {
            // one member per lane: its rank among the (distinct) members is its place
            const uint64_t v = tid < ng ? gm[tid] : 0ull;
            uint32_t rank = 0;
            if (tid < ng)
                for (uint32_t g = 0; g < ng; g++) rank += gm[g] < v ? 1u : 0u;
            __syncthreads();
            if (tid < ng) gm[rank] = v;
            __syncthreads();
        } else {  // bitonic
            uint32_t N = 2;
            while (N < ng) N <<= 1;
            for (uint32_t j = ng + tid; j < N; j += MG_GTHREADS) gm[j] = ~0ull;
            __syncthreads();
            for (uint32_t k = 2; k <= N; k <<= 1)
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t x = tid; x < N; x += MG_GTHREADS) {
                        const uint32_t y = x ^ j;
                        if (y > x) {
                            const uint64_t u = gm[x], v = gm[y];
                            if ((u > v) == ((x & k) == 0u)) {
                                gm[x] = v;
                                gm[y] = u;
                            }
                        }
                    }
                    __syncthreads();
                }
        }
        for (uint32_t g = tid; g < ng; g += MG_GTHREADS) {
            const uint64_t cur = gm[g];
            const uint32_t i = (uint32_t)cur, q0 = (uint32_t)(cur >> 32);
            if (g > 0 && (uint32_t)(gm[g - 1] >> 32) == q0) {  // a later member: no ray here
                mg_out(M, i, s, false, 0.0f, 0.0f, 0.0f, 0.0f);
                continue;
            }
            // the first member merges the bundle, four members' points in flight at a time
            mx = my = mz = mw = 0.0f;
            clearing = false;
            for (uint32_t q = g; q < ng;) {
                float px[4], py[4], pz[4];
                uint32_t m = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint64_t c = q + u < ng ? gm[q + u] : ~0ull;
                    const bool on = m == (uint32_t)u && (uint32_t)(c >> 32) == q0;
                    const uint32_t j = on ? (uint32_t)c : i;
                    m += on ? 1u : 0u;
                    px[u] = xs[3 * (size_t)j];
                    py[u] = xs[3 * (size_t)j + 1];
                    pz[u] = xs[3 * (size_t)j + 2];
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if ((uint32_t)u < m) merge_at(px[u], py[u], pz[u]);
                if (m < 4u) break;
                q += 4u;
            }
            mg_out(M, i, s, clearing, mx, my, mz, mw);
        }
    } else {
        // too many members for the list: each bundle's first member walks the scan's points from
        // itself to its last member (first / last per slot, in the list's space)
        uint32_t* tfirst = reinterpret_cast<uint32_t*>(gm);
        uint32_t* tlast = tfirst + MG_TAB;
        static_assert(2 * MG_TAB * sizeof(uint32_t) <= MG_GM * sizeof(uint64_t), "first / last fit");
        for (uint32_t j = tid; j < MG_TAB; j += MG_GTHREADS) {
            tfirst[j] = MG_NONE;
            tlast[j] = 0u;
        }
        __syncthreads();
        for (uint32_t e = e0 + tid; e < e1; e += MG_GTHREADS) {
            const uint32_t q = find(M.ekey[e], false);
            if (q != MG_NONE && tdup[q]) {
                atomicMin(&tfirst[q], M.eidx[e]);
                atomicMax(&tlast[q], M.eidx[e]);
            }
        }
        __syncthreads();
        for (uint32_t q = tid; q < MG_TAB; q += MG_GTHREADS) {
            if (!tdup[q]) continue;
            const uint64_t key = tkey[q];
            const uint32_t i = tfirst[q], last = tlast[q];
            mx = my = mz = mw = 0.0f;
            clearing = false;
            for (uint32_t j0 = i; j0 <= last; j0 += 4u) {  // four points in flight at a time
                float px[4], py[4], pz[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t j = min(j0 + u, last);
                    px[u] = xs[3 * (size_t)j];
                    py[u] = xs[3 * (size_t)j + 1];
                    pz[u] = xs[3 * (size_t)j + 2];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t j = j0 + u;
                    if (j > last) break;
                    const MgPoint p = mg_point(R, px[u], py[u], pz[u], s.ox, s.oy, s.oz, s.zx,
                                               s.zy, s.zz, axis);
                    if (!p.ok || p.key != key) continue;
                    clearing = p.clearing;
                    mg_step(p, clearing, mx, my, mz, mw);
                    if (j != i) mg_out(M, j, s, false, 0.0f, 0.0f, 0.0f, 0.0f);
                }
            }
            mg_out(M, i, s, clearing, mx, my, mz, mw);
        }
    }
}

}  // namespace

uint32_t mg_buckets_max(uint64_t n_points) {
    return (uint32_t)std::min<uint64_t>((n_points >> MG_BSHIFT) + MAX_BATCH + 1, 0xFFFFFFF0ull);
}

hipError_t launch_mg_prepass(const float* d_xyz, const BatchRef& B, uint32_t n_blocks,
                             uint64_t n_points, const RayConst& R, MgBufs& M, uint32_t* ovf,
                             hipStream_t st) {
    if (!n_points) return hipSuccess;
    const uint64_t nb = (n_points >> MG_BSHIFT) + B.n_scans;
    if (n_points > M.cap || nb > M.nb_cap) return hipErrorInvalidValue;
    k_mg_count<<<n_blocks, MG_THREADS, 0, st>>>(d_xyz, B, R, M);
    k_mg_scan<<<1, MG_SCAN_THREADS, 0, st>>>(B, M, (uint32_t)nb);
    k_mg_scatter<<<n_blocks, MG_THREADS, 0, st>>>(d_xyz, B, R, M);
    k_mg_group<<<(uint32_t)nb, MG_GTHREADS, 0, st>>>(d_xyz, B, R, M, ovf);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        // a pre-pass cut short may leave bucket counters set: zero them, so the next batch starts
        // from zero counters
        (void)hipMemsetAsync(M.bcnt, 0, (size_t)4 * MG_REP * M.nb_cap, st);
    }
    return e;
}

}  // namespace tsdf
