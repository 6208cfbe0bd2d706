// tsdf_integrate.hip — k_integrate, the per-brick stage of the batch pipeline.
//
// One two-wave workgroup per active brick (grid-stride over the active list).  Thread `tid` OWNS
// voxels 4 tid .. 4 tid + 3: their (sdf, weight) live in its registers for the whole batch, read
// once (one coalesced float4 each) and written back once if dirty.  The brick's ray records
// (x, y, z, in-brick sample count; scan-ordered and contiguous, from k_place) are consumed in
// chunks of up to 128 rays:
//   1. every lane walks its ray's DDA (the same fp32 walk as k_count and the oracle) and writes its
//      in-brick gated samples (sdf, voxel << 6 | scan) into an LDS buffer at positions from a
//      workgroup prefix of the record counts (a chunk is cut where the buffer would overflow),
//      counting samples per voxel;
//   2. a counting sort by voxel (prefix of the 512 counts, one LDS atomic per sample) gives every
//      owner the buffer indices of its voxels' samples; an insertion sort of each (tiny) bucket by
//      buffer index puts them in scan order, because records — hence samples — are scan-ordered;
//   3. each owner walks its buckets: samples of one scan are summed as exact fixed point
//      (trunc(s * 2^32), int64) and counted; when the scan changes, the pending scan is fused
//          S <- (S W + A 2^-32) / (W + B),  W <- W + B
//      The pending (scan, sum, count) of each voxel stays in registers across chunks, so a scan
//      split over chunks is still fused once.
// Five barriers per chunk, whatever the number of scans in it; the fuse order per voxel is scan
// order, so the field is bitwise the one scan-at-a-time integration gives for any batch
// composition (tests/test_gpu_parity.py::test_batch_composition_is_invisible).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

constexpr int INT_THREADS = 128;        // two waves per brick; 4 owned voxels per thread
constexpr int INT_SB = 1024;            // LDS sample buffer entries (>= 46 rays of 22 samples)
constexpr int INT_BLOCKS_PER_CU = 12;   // LDS-bound residency (~13 KB per workgroup)
constexpr uint32_t NO_SCAN = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t excl_scan128(uint32_t x, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d, 64);
        if (lane >= d) v += y;
    }
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    *total = s_w[0] + s_w[1];
    const uint32_t r = v - x + (wid ? s_w[0] : 0u);
    __syncthreads();  // s_w is reused by the next call
    return r;
}

// largest t < ns with cs[t] <= j (cs[0] = 0); trip count depends on ns only
__device__ __forceinline__ uint32_t scan_of(const uint32_t* cs, uint32_t ns, uint32_t j) {
    uint32_t t = 0;
    for (uint32_t len = ns; len > 1;) {
        const uint32_t half = len >> 1;
        t = (cs[t + half] <= j) ? t + half : t;
        len -= half;
    }
    return t;
}

__global__ __launch_bounds__(INT_THREADS) void k_integrate(BatchDesc D, RayConst R, Table T,
                                                          Work Wk, Pool Pl, Globals* G,
                                                          int parity) {
    __shared__ float smp_s[INT_SB];      // sample sdf (truncated)
    __shared__ uint16_t smp_lt[INT_SB];  // voxel << 6 | scan
    __shared__ uint16_t s_idx[INT_SB];   // sample indices grouped by voxel
    __shared__ uint32_t s_cur[BRICK_VOX];     // per-voxel count, then bucket cursor
    __shared__ uint16_t s_bs[BRICK_VOX];      // bucket start
    __shared__ uint32_t s_cs[MAX_BATCH + 1];  // brick's per-scan record prefix; s_cs[ns] = n
    __shared__ uint32_t s_nchunk;
    __shared__ uint32_t s_w[2], s_m[2];
    Counters* C = &G->ctr[parity];
    const int tid = threadIdx.x;
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
    uint32_t nvox = 0, ndirty = 0;
    for (uint32_t a = blockIdx.x; a < n_active; a += gridDim.x) {
        const uint32_t h = Wk.active[a];
        const uint32_t slot = T.slots[h];
        const uint32_t n = T.cnt[h];
        const uint32_t base = T.toff[h];
        const uint64_t key = T.keys[h];
        const int bx = (int)(key & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int by = (int)((key >> 21) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const int bz = (int)((key >> 42) & 0x1FFFFF) - BRICK_COORD_BIAS;
        const bool has_slot = slot < T.max_bricks;
        if ((uint32_t)tid < ns) s_cs[tid] = T.cell[(size_t)h * T.cell_stride + tid];
        if (tid == 0) s_cs[ns] = n;
        float4* Sg = reinterpret_cast<float4*>(Pl.sdf + (size_t)(has_slot ? slot : 0) * BRICK_VOX);
        float4* Wg = reinterpret_cast<float4*>(Pl.weight + (size_t)(has_slot ? slot : 0) * BRICK_VOX);
        float sv[4], wv[4];
        {
            const float4 s4 = has_slot ? Sg[tid] : make_float4(R.tau, R.tau, R.tau, R.tau);
            const float4 w4 = has_slot ? Wg[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
            sv[0] = s4.x; sv[1] = s4.y; sv[2] = s4.z; sv[3] = s4.w;
            wv[0] = w4.x; wv[1] = w4.y; wv[2] = w4.z; wv[3] = w4.w;
        }
        uint32_t pt[4] = {NO_SCAN, NO_SCAN, NO_SCAN, NO_SCAN};  // pending scan per owned voxel
        long long pa[4] = {0, 0, 0, 0};                           // its fixed-point sum
        uint32_t pb[4] = {0u, 0u, 0u, 0u};                        // its sample count
        uint32_t dirty = 0;
        auto fuse = [&](int k) {
            const float bf = (float)pb[k];
            const float af = (float)((double)pa[k] * (1.0 / 4294967296.0));
            const float nw = wv[k] + bf;
            sv[k] = (sv[k] * wv[k] + af) / nw;
            wv[k] = nw;
            dirty |= 1u << k;
            nvox++;
        };
        __syncthreads();
        for (uint32_t j0 = 0; j0 < n;) {
            const uint32_t j = j0 + tid;
            const bool valid = j < n;
            const float4 rc = valid ? Wk.rec[base + j] : make_float4(0.f, 0.f, 0.f, 0.f);
            const uint32_t cnt_j = valid ? __float_as_uint(rc.w) : 0u;
            const uint32_t tj = scan_of(s_cs, ns, valid ? j : j0);
#pragma unroll
            for (int k = 0; k < 4; k++) s_cur[4 * tid + k] = 0u;
            uint32_t total;
            const uint32_t off = excl_scan128(cnt_j, s_w, &total);
            // the chunk: the leading rays whose samples fit the buffer (off is monotone in tid)
            const bool in_chunk = valid && off + cnt_j <= (uint32_t)INT_SB;
            const unsigned long long bal = __ballot(in_chunk);
            if ((tid & 63) == 0) s_m[tid >> 6] = (uint32_t)__popcll(bal);
            __syncthreads();
            const uint32_t m = s_m[0] + s_m[1];
            if ((uint32_t)tid == m - 1) s_nchunk = off + cnt_j;  // samples in the chunk
            // 1. walk: samples into the buffer, per-voxel counts
#ifdef TSDF_ABLATE_WALK  // diagnostic build only: dummy samples, no DDA (timing share of the walk)
            if (in_chunk)
                for (uint32_t w = 0; w < cnt_j; w++) {
                    const uint32_t l = (off + w) & 511u;
                    smp_s[off + w] = 0.01f;
                    smp_lt[off + w] = (uint16_t)((l << 6) | tj);
                    atomicAdd(&s_cur[l], 1u);
                }
#else
            if (in_chunk && cnt_j) {
                const float ox = D.ox[tj], oy = D.oy[tj], oz = D.oz[tj];
                RayState r;
                if (ray_init(R, ox, oy, oz, rc.x, rc.y, rc.z, r)) {
                    uint32_t w = 0;
                    for (int it = 0; it < MAX_DDA_STEPS; it++) {
                        if ((r.vx >> 3) == bx && (r.vy >> 3) == by && (r.vz >> 3) == bz) {
                            float s;
                            if (voxel_sample(R, ox, oy, oz, r, s) && w < cnt_j) {
                                const uint32_t l =
                                    ((r.vz & 7) << 6) | ((r.vy & 7) << 3) | (r.vx & 7);
                                smp_s[off + w] = s;
                                smp_lt[off + w] = (uint16_t)((l << 6) | tj);
                                atomicAdd(&s_cur[l], 1u);
                                w++;
                            }
                        }
                        if (!ray_step(r)) break;
                    }
                }
            }
#endif
            __syncthreads();
            const uint32_t nchunk = s_nchunk;
#ifndef TSDF_ABLATE_OWN  // diagnostic build only: skip the sort and the fuse
            // 2. counting sort by voxel
            {
                uint32_t c[4], sum = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    c[k] = s_cur[4 * tid + k];
                    sum += c[k];
                }
                uint32_t tot;
                uint32_t st = excl_scan128(sum, s_w, &tot);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    s_bs[4 * tid + k] = (uint16_t)st;
                    s_cur[4 * tid + k] = st;
                    st += c[k];
                }
            }
            __syncthreads();
            for (uint32_t q = tid; q < nchunk; q += INT_THREADS) {
                const uint32_t l = smp_lt[q] >> 6;
                s_idx[atomicAdd(&s_cur[l], 1u)] = (uint16_t)q;
            }
            __syncthreads();
            // 3. owners: samples of each voxel in scan order, fused once per scan
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t l = 4 * tid + k;
                const uint32_t b0 = s_bs[l], b1 = s_cur[l];
                for (uint32_t i = b0 + 1; i < b1; i++) {  // insertion sort by buffer index
                    const uint16_t v = s_idx[i];
                    uint32_t p = i;
                    while (p > b0 && s_idx[p - 1] > v) {
                        s_idx[p] = s_idx[p - 1];
                        p--;
                    }
                    s_idx[p] = v;
                }
                for (uint32_t i = b0; i < b1; i++) {
                    const uint32_t q = s_idx[i];
                    const uint32_t t = smp_lt[q] & 63u;
                    const long long fx = (long long)(smp_s[q] * 4294967296.0f);
                    if (t != pt[k]) {
                        if (pb[k]) fuse(k);
                        pt[k] = t;
                        pa[k] = fx;
                        pb[k] = 1u;
                    } else {
                        pa[k] += fx;
                        pb[k]++;
                    }
                }
            }
#else
            (void)nchunk;
#endif
            __syncthreads();
            j0 += m;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (pb[k]) fuse(k);
        if (has_slot && dirty) {
            Sg[tid] = make_float4(sv[0], sv[1], sv[2], sv[3]);
            Wg[tid] = make_float4(wv[0], wv[1], wv[2], wv[3]);
        }
        ndirty += __popc(dirty);
        // zero every cell of the brick (k_compact prefixes whole uint4 groups) for the next batch
        if ((uint32_t)tid < T.cell_stride) T.cell[(size_t)h * T.cell_stride + tid] = 0u;
        __syncthreads();
    }
    const unsigned long long v = wave_sum<unsigned long long>(nvox);
    const unsigned long long d = wave_sum<unsigned long long>(ndirty);
    if ((tid & 63) == 0) {
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

hipError_t launch_integrate(const BatchDesc& D, const RayConst& R, const Table& T, const Work& Wk,
                            const Pool& Pl, Globals* G, int parity, hipStream_t st) {
    k_integrate<<<256 * INT_BLOCKS_PER_CU, INT_THREADS, 0, st>>>(D, R, T, Wk, Pl, G, parity);
    return hipGetLastError();
}

}  // namespace tsdf
