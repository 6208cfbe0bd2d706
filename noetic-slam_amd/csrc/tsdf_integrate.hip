// tsdf_integrate.hip — k_integrate, the per-brick stage of the batch pipeline.
//
// One 256-thread workgroup per active brick (grid-stride over the active list).  Thread `tid` OWNS
// voxels 2 tid and 2 tid + 1: their (sdf, weight) live in its registers for the whole batch — read
// once (coalesced float2), written back once if dirty.  k_place left the brick's samples
// (sdf bits, scan << 9 | voxel) contiguous and scan-ordered in HBM.  The batch's scans are taken
// in windows of INT_WIN consecutive scans:
//   1. every thread streams its share of the window's samples from HBM (coalesced 8-byte loads)
//      and adds each into an LDS tile indexed by (scan within the window, voxel): exact fixed point
//      (trunc(s * 2^32), int64) and a count, with LDS atomics;
//   2. each owner then fuses its two voxels through the window's scans, in scan order:
//          S <- (S W + A 2^-32) / (W + B),  W <- W + B      (for every scan with B > 0)
//      and clears its tile entries.
// Two barriers per window (four windows for a 32-scan batch), no sort, no dependence on how the
// samples of a scan are spread; the per-voxel fuse order is scan order, so the field is bitwise
// the one scan-at-a-time integration gives, for any batch composition
// (tests/test_gpu_parity.py::test_batch_composition_is_invisible).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

constexpr int INT_THREADS = 256;      // four waves per brick; 2 owned voxels per thread
constexpr int INT_WIN = 8;            // scans per window (LDS tile: INT_WIN x 512 x 12 B = 48 KB)
constexpr int INT_BLOCKS_PER_CU = 3;  // LDS-bound residency

__global__ __launch_bounds__(INT_THREADS) void k_integrate(BatchDesc D, Table T, Work Wk, Pool Pl,
                                                          Globals* G, int parity, float tau) {
    __shared__ unsigned long long sA[INT_WIN][BRICK_VOX];  // sum of trunc(s * 2^32)
    __shared__ uint32_t sB[INT_WIN][BRICK_VOX];            // sample count
    __shared__ uint32_t s_cs[MAX_BATCH + 1];               // brick's per-scan sample prefix
    Counters* C = &G->ctr[parity];
    const int tid = threadIdx.x;
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
    for (int w = 0; w < INT_WIN; w++) {
        sA[w][2 * tid] = 0ull;
        sA[w][2 * tid + 1] = 0ull;
        sB[w][2 * tid] = 0u;
        sB[w][2 * tid + 1] = 0u;
    }
    uint32_t nvox = 0, ndirty = 0;
    for (uint32_t a = blockIdx.x; a < n_active; a += gridDim.x) {
        const uint32_t h = Wk.active[a];
        const uint32_t slot = T.slots[h];
        const uint32_t n = T.cnt[h];
        const uint32_t base = T.toff[h];
        const bool has_slot = slot < T.max_bricks;
        if ((uint32_t)tid < ns) s_cs[tid] = T.cell[(size_t)h * T.cell_stride + tid];
        if (tid == 0) s_cs[ns] = n;
        float2* Sg = reinterpret_cast<float2*>(Pl.sdf + (size_t)(has_slot ? slot : 0) * BRICK_VOX);
        float2* Wg = reinterpret_cast<float2*>(Pl.weight + (size_t)(has_slot ? slot : 0) * BRICK_VOX);
        const float2 s2 = has_slot ? Sg[tid] : make_float2(tau, tau);
        const float2 w2 = has_slot ? Wg[tid] : make_float2(0.f, 0.f);
        float sv[2] = {s2.x, s2.y}, wv[2] = {w2.x, w2.y};
        uint32_t dirty = 0;
        __syncthreads();  // s_cs visible
        for (uint32_t t0 = 0; t0 < ns; t0 += INT_WIN) {
            const uint32_t t1 = min(t0 + (uint32_t)INT_WIN, ns);
            const uint32_t q0 = s_cs[t0], q1 = s_cs[t1];
            if (q0 == q1) continue;  // uniform: no sample of this brick in the window
            // 1. accumulate the window's samples
            for (uint32_t q = q0 + tid; q < q1; q += INT_THREADS) {
                const uint32_t g = base + q;
                if (g >= Wk.max_smp) break;  // capacity overflow (reported by k_compact)
                const uint2 v = Wk.smp[g];
                const uint32_t l = v.y & 511u, w = (v.y >> 9) - t0;
                const long long fx = (long long)(__uint_as_float(v.x) * 4294967296.0f);
                atomicAdd(&sA[w][l], (unsigned long long)fx);
                atomicAdd(&sB[w][l], 1u);
            }
            __syncthreads();
            // 2. owners fuse their voxels through the window's scans, in order
            for (uint32_t w = 0; w < t1 - t0; w++) {
                const uint2 b2 = *reinterpret_cast<const uint2*>(&sB[w][2 * tid]);
                const uint32_t bb[2] = {b2.x, b2.y};
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    if (bb[k]) {
                        const int l = 2 * tid + k;
                        const float bf = (float)bb[k];
                        const float af =
                            (float)((double)(long long)sA[w][l] * (1.0 / 4294967296.0));
                        const float nw = wv[k] + bf;
                        sv[k] = (sv[k] * wv[k] + af) / nw;
                        wv[k] = nw;
                        sA[w][l] = 0ull;
                        sB[w][l] = 0u;
                        dirty |= 1u << k;
                        nvox++;
                    }
                }
            }
            __syncthreads();
        }
        if (has_slot && dirty) {
            Sg[tid] = make_float2(sv[0], sv[1]);
            Wg[tid] = make_float2(wv[0], wv[1]);
        }
        ndirty += __popc(dirty);
        // zero every cell of the brick (k_compact prefixes whole uint4 groups) for the next batch
        if ((uint32_t)tid < T.cell_stride) T.cell[(size_t)h * T.cell_stride + tid] = 0u;
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
    k_integrate<<<256 * INT_BLOCKS_PER_CU, INT_THREADS, 0, st>>>(D, T, Wk, Pl, G, parity, R.tau);
    return hipGetLastError();
}

}  // namespace tsdf
