// tsdf_integrate.hip — k_integrate, the per-brick stage of the batch pipeline.
//
// One 256-thread workgroup per active brick (grid-stride over k_compact's active records).  k_place
// left the brick's samples (sdf bits, scan << 9 | voxel) contiguous and scan-ordered in HBM.  The
// brick's (sdf, weight) are staged in LDS for the whole batch.  Its scans are taken in windows of
// consecutive scans holding at most INT_CAP samples (one window for a typical brick), each window:
//   P1  every sample sets bit (scan - t0) of its voxel's LDS scan mask;
//   P2  a block scan over the 512 masks' popcounts gives every voxel a contiguous, scan-ordered
//       run of "live cells" (one per (voxel, scan) the window observed; <= INT_CAP of them), plus
//       the list of live voxels;
//   P3  every sample adds its exact fixed-point value trunc(s * 2^32) (int64) and a count into its
//       cell: base[voxel] + popc(mask & lower scans);
//   P4  lanes take live voxels from an LDS work queue and fuse each one's cells in scan order:
//          S <- (S W + A 2^-32) / (W + B),  W <- W + B
//       so the wave time is ~(live cells / 64), not (64 lanes x longest chain).
// The per-voxel fuse order is scan order, so the field is bitwise the one scan-at-a-time
// integration gives, for any batch composition
// (tests/test_gpu_parity.py::test_batch_composition_is_invisible).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

constexpr int INT_THREADS = 256;
constexpr int INT_PER = 8;                           // register-cached samples per thread
constexpr uint32_t INT_CAP = INT_PER * INT_THREADS;  // samples (>= live cells) per window
constexpr int INT_BLOCKS_PER_CU = 4;                 // LDS ~34 KB per workgroup
constexpr uint32_t INT_MAX_WIN = 32;                 // scans per window (u32 masks)

// Diagnostic build only (-DTSDF_PHASE_TIMING, never shipped): thread 0 of a few workgroups drains
// its memory counters at each phase boundary and prints the cycles spent per phase.
#ifdef TSDF_PHASE_TIMING
#define PHASE(k)                                 \
    do {                                         \
        __builtin_amdgcn_s_waitcnt(0);           \
        const unsigned long long t_ = clock64(); \
        ph[k] += t_ - t_last;                    \
        t_last = t_;                             \
    } while (0)
#else
#define PHASE(k) \
    do {         \
    } while (0)
#endif

__global__ __launch_bounds__(INT_THREADS) void k_integrate(BatchDesc D, Table T, Work Wk, Pool Pl,
                                                          Globals* G, int parity, float tau) {
    __shared__ unsigned long long cA[INT_CAP];  // live cell: sum of trunc(s * 2^32)
    __shared__ uint32_t cB[INT_CAP];            // live cell: sample count
    __shared__ uint32_t sMask[BRICK_VOX];       // voxel: scans (bit t - t0) observed in the window
    __shared__ uint32_t sBase[BRICK_VOX];       // voxel: first live cell
    __shared__ float sS[BRICK_VOX], sW[BRICK_VOX];
    __shared__ uint16_t sLive[BRICK_VOX];  // live voxels of the window
    // brick's per-scan sample prefix, double-buffered by brick parity: a wave may still read the
    // previous brick's prefix while another writes the next one
    __shared__ uint32_t s_csb[2][MAX_BATCH + 1];
    __shared__ uint32_t s_red[INT_THREADS / 64];
    __shared__ uint32_t s_nlive, s_q;
    Counters* C = &G->ctr[parity];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
    for (uint32_t j = tid; j < INT_CAP; j += INT_THREADS) {
        cA[j] = 0ull;
        cB[j] = 0u;
    }
    sMask[tid] = 0u;
    sMask[tid + 256] = 0u;
    uint32_t nvox = 0, ndirty = 0, par = 0;
#ifdef TSDF_PHASE_TIMING
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last = clock64();
    uint32_t nb = 0;
#endif
    for (uint32_t a = blockIdx.x; a < n_active; a += gridDim.x, par ^= 1u) {
        uint32_t* s_cs = s_csb[par];
        const uint4 rec = Wk.active[a];  // (h, slot, toff, n)
        const uint32_t h = rec.x, n = rec.w, base = rec.z;
        const bool has_slot = rec.y < T.max_bricks;
        if ((uint32_t)tid < ns) s_cs[tid] = T.cell[(size_t)h * T.cell_stride + tid];
        if (tid == 0) s_cs[ns] = n;
        float* Sg = Pl.sdf + (size_t)(has_slot ? rec.y : 0) * BRICK_VOX;
        float* Wg = Pl.weight + (size_t)(has_slot ? rec.y : 0) * BRICK_VOX;
        // sS / sW of voxels tid, tid + 256: the previous brick's last readers are past a barrier
        sS[tid] = has_slot ? Sg[tid] : tau;
        sS[tid + 256] = has_slot ? Sg[tid + 256] : tau;
        sW[tid] = has_slot ? Wg[tid] : 0.0f;
        sW[tid + 256] = has_slot ? Wg[tid + 256] : 0.0f;
        uint32_t dirty = 0;  // voxels 2 tid, 2 tid + 1 (bits 0, 1)
        PHASE(0);
        __syncthreads();  // s_cs, sS, sW visible
        PHASE(1);
        uint2 c[INT_PER];
        uint32_t cq = ~0u;  // samples [cq, cq + INT_CAP) are in c[] (uniform)
        for (uint32_t t0 = 0; t0 < ns;) {
            // window [t0, t1): as many scans as keep its samples <= INT_CAP (at least one)
            const uint32_t q0 = s_cs[t0];
            uint32_t t1 = t0 + 1;
            while (t1 < ns && t1 - t0 < INT_MAX_WIN && s_cs[t1 + 1] - q0 <= INT_CAP) t1++;
            const uint32_t q1 = s_cs[t1], nw = t1 - t0;
            if (q0 == q1) {  // uniform: no sample of this brick in the window
                t0 = t1;
                continue;
            }
            // P1: scan masks (a one-scan window may exceed INT_CAP samples: chunked)
            for (uint32_t qc = q0; qc < q1; qc += INT_CAP) {
                if (cq != qc) {
                    cq = qc;
#pragma unroll
                    for (int j = 0; j < INT_PER; j++) {
                        const uint32_t i = cq + tid + j * INT_THREADS;
                        // base + i >= max_smp: capacity overflow (reported by k_compact)
                        c[j] = (i < n && base + i < Wk.max_smp) ? Wk.smp[base + i]
                                                                : make_uint2(0u, ~0u);
                    }
                    PHASE(2);
                }
#pragma unroll
                for (int j = 0; j < INT_PER; j++) {
                    const uint32_t w = (c[j].y >> 9) - t0;
                    if (w < nw) atomicOr(&sMask[c[j].y & 511u], 1u << w);
                }
            }
            __syncthreads();
            PHASE(3);
            // P2: live cells and live voxels (packed block scan: cells | voxels << 16)
            {
                const uint32_t m0 = sMask[2 * tid], m1 = sMask[2 * tid + 1];
                const uint32_t c0 = __popc(m0), c1 = __popc(m1);
                const uint32_t v0 = m0 ? 1u : 0u, v1 = m1 ? 1u : 0u;
                dirty |= v0 | (v1 << 1);
                const uint32_t x = (c0 + c1) | ((v0 + v1) << 16);
                uint32_t incl = x;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += y;
                }
                if (lane == 63) s_red[wid] = incl;
                __syncthreads();
                uint32_t off = 0, tot = 0;
#pragma unroll
                for (int k = 0; k < INT_THREADS / 64; k++) {
                    const uint32_t r = s_red[k];
                    off += k < wid ? r : 0u;
                    tot += r;
                }
                const uint32_t ex = incl - x + off;
                const uint32_t cb = ex & 0xFFFFu, vb = ex >> 16;
                sBase[2 * tid] = cb;
                sBase[2 * tid + 1] = cb + c0;
                if (v0) sLive[vb] = (uint16_t)(2 * tid);
                if (v1) sLive[vb + v0] = (uint16_t)(2 * tid + 1);
                if (tid == 0) {
                    s_nlive = tot >> 16;
                    s_q = 0u;
                    nvox += tot & 0xFFFFu;  // (voxel, scan) updates of the window
                }
            }
            __syncthreads();
            PHASE(4);
            // P3: accumulate into the live cells
            for (uint32_t qc = q0; qc < q1; qc += INT_CAP) {
                if (cq != qc) {
                    cq = qc;
#pragma unroll
                    for (int j = 0; j < INT_PER; j++) {
                        const uint32_t i = cq + tid + j * INT_THREADS;
                        c[j] = (i < n && base + i < Wk.max_smp) ? Wk.smp[base + i]
                                                                : make_uint2(0u, ~0u);
                    }
                }
#pragma unroll
                for (int j = 0; j < INT_PER; j++) {
                    const uint32_t w = (c[j].y >> 9) - t0;
                    if (w < nw) {
                        const uint32_t l = c[j].y & 511u;
                        const uint32_t cell = sBase[l] + __popc(sMask[l] & ((1u << w) - 1u));
                        const long long fx = (long long)(__uint_as_float(c[j].x) * 4294967296.0f);
                        atomicAdd(&cA[cell], (unsigned long long)fx);
                        atomicAdd(&cB[cell], 1u);
                    }
                }
            }
            __syncthreads();
            PHASE(5);
            // P4: fuse, live voxels from a work queue; each lane runs one voxel's chain at a time
            {
                const uint32_t nlive = s_nlive;
                uint32_t l = 0, cell = 0, rem = 0;
                float s = 0.0f, wt = 0.0f;
                while (true) {
                    if (rem == 0) {
                        const uint32_t vi = atomicAdd(&s_q, 1u);
                        if (vi >= nlive) break;
                        l = sLive[vi];
                        cell = sBase[l];
                        const uint32_t m = sMask[l];
                        sMask[l] = 0u;
                        rem = __popc(m);
                        s = sS[l];
                        wt = sW[l];
                    }
                    const float bf = (float)cB[cell];
                    const float af = (float)((double)(long long)cA[cell] * (1.0 / 4294967296.0));
                    cA[cell] = 0ull;
                    cB[cell] = 0u;
                    const float nwt = wt + bf;
                    s = (s * wt + af) / nwt;
                    wt = nwt;
                    cell++;
                    if (--rem == 0) {
                        sS[l] = s;
                        sW[l] = wt;
                    }
                }
            }
            __syncthreads();
            PHASE(6);
            t0 = t1;
        }
        if (has_slot) {
            if (dirty & 1u) {
                Sg[2 * tid] = sS[2 * tid];
                Wg[2 * tid] = sW[2 * tid];
            }
            if (dirty & 2u) {
                Sg[2 * tid + 1] = sS[2 * tid + 1];
                Wg[2 * tid + 1] = sW[2 * tid + 1];
            }
        }
        ndirty += __popc(dirty);
        // zero every cell of the brick (k_compact prefixes whole uint4 groups) for the next batch
        if ((uint32_t)tid < T.cell_stride) T.cell[(size_t)h * T.cell_stride + tid] = 0u;
#ifdef TSDF_PHASE_TIMING
        nb++;
#endif
        PHASE(7);
        __syncthreads();  // write-back reads of sS / sW done before the next brick stages its own
    }
#ifdef TSDF_PHASE_TIMING
    if (tid == 0 && (blockIdx.x % 97) == 0)
        printf("phase blk %u bricks %u meta %llu bar0 %llu load %llu mask %llu scan %llu acc %llu "
               "fuse %llu tail %llu\n", blockIdx.x, nb, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5],
               ph[6], ph[7]);
#endif
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

hipError_t launch_integrate(const BatchDesc& D, const RayConst& R, const Table& T, const Work& Wk,
                            const Pool& Pl, Globals* G, int parity, hipStream_t st) {
    k_integrate<<<256 * INT_BLOCKS_PER_CU, INT_THREADS, 0, st>>>(D, T, Wk, Pl, G, parity, R.tau);
    return hipGetLastError();
}

}  // namespace tsdf
