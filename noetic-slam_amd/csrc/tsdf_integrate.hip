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

#include <type_traits>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

constexpr int INT_THREADS = 256;
#ifndef TSDF_INT_PER
#define TSDF_INT_PER 6
#endif
constexpr int INT_PER = TSDF_INT_PER;                // register-cached samples per thread
constexpr uint32_t INT_CAP = INT_PER * INT_THREADS;  // samples (>= live cells) per window
// Voxblox with per-sample weights (sem 3): register-cached samples per thread (A/B knob; 5 keeps
// five workgroups per CU with 16-B cells but measured slower than 6: DESIGN.md §10)
#ifndef TSDF_INT_PER3
#define TSDF_INT_PER3 TSDF_INT_PER
#endif
// LDS: 12 B per cell + ~9.5 KB per workgroup; residency as LDS allows
constexpr int INT_BLOCKS_PER_CU = (160 * 1024) / (INT_CAP * 12 + 10 * 1024);
#ifndef TSDF_INT_WIN
#define TSDF_INT_WIN 64
#endif
#if TSDF_INT_WIN == 64
typedef unsigned long long MaskT;  // a voxel's scans in the window, one bit per scan
#define MASK_POPC(m) __popcll(m)
#else
typedef uint32_t MaskT;
#define MASK_POPC(m) __popc(m)
#endif
// LDS position of brick voxel l = (z * 8 + y) * 8 + x in k_integrate's per-voxel arrays.  A/B knob
// (round 6): TSDF_INT_SKEW=1 skews each z layer by one element, so voxels of one (x, y) column (64
// elements apart: one bank) fall in different banks -- measured slower (k_integrate 0.399 vs 0.377
// ms headline, 1.18 vs 1.07 ms C4: the index arithmetic costs more than the conflicts it removes)
// A/B knob (round 6): TSDF_INT_ZERO_IN_FUSE=1 zeroes the live cells in the fuse chains that
// consumed them instead of in a pass before each window's accumulation -- measured slower
// (k_integrate 0.385 vs 0.375 ms headline, 1.085 vs 1.065 ms C4: the stores lengthen the chains)
#ifndef TSDF_INT_ZERO_IN_FUSE
#define TSDF_INT_ZERO_IN_FUSE 0
#endif
#ifndef TSDF_INT_SKEW
#define TSDF_INT_SKEW 0
#endif
#define VOXL(l) ((l) + TSDF_INT_SKEW * ((l) >> 6))
constexpr int BRICK_VOX_LDS = BRICK_VOX + TSDF_INT_SKEW * (BRICK_VOX / 64);
constexpr uint32_t INT_MAX_WIN = TSDF_INT_WIN;       // scans per window (mask bits)
// single walk (FUSED): the register cache holds INT_SPT span records' samples per thread, so a
// chunk is INT_SCH spans; a window also keeps its spans <= INT_SCH (one chunk per window)
#ifndef TSDF_INT_SPT
#define TSDF_INT_SPT 2
#endif
constexpr int INT_SPT = TSDF_INT_SPT;
constexpr uint32_t INT_SCH = INT_SPT * INT_THREADS;
constexpr uint32_t NO_SPAN = 0xFFFFFFFFu;

#ifdef TSDF_ABLATE_PHASE  // `make ablate ABLATE=PHASE`
#define TSDF_PHASE_TIMING
#endif
// Diagnostic build only (-DTSDF_PHASE_TIMING, never shipped): thread 0 of a few workgroups reads
// the clock at each phase boundary (no counter drain: outstanding loads stay in flight) and
// prints the cycles spent per phase.
#ifdef TSDF_PHASE_TIMING
#define PHASE(k)                                 \
    do {                                         \
        const unsigned long long t_ = clock64(); \
        ph[k] += t_ - t_last;                    \
        t_last = t_;                             \
    } while (0)
#else
#define PHASE(k) \
    do {         \
    } while (0)
#endif

// SEM = TSDF_SEM_*.  VDBFusion (0): a cell holds (sum of trunc(s 2^32), sample count) and the fuse
// is the running average.  Voxblox (1): a cell holds (sum of trunc(s w 2^32), sum of
// trunc(w 2^32)), w the sample's dropoff weight recomputed from its stored distance, and the fuse
// clamps the distance to +-tau and the weight to max_weight.
// MAXS: the most scans a batch of this instantiation holds (64: the LDS of the single-GPU batches;
// 512: the sector-sharded multi-GPU batches, one batch per step).
// FUSED (single walk, tsdf_walk.hip): a brick's samples are read through its span records (active
// record = (table index, slot, first span, spans); 64-bit cells = relative sample prefix | absolute
// span position, the totals at scan n_scans).  Otherwise they are one contiguous segment (k_place).
#ifndef TSDF_INT_WAVES
#define TSDF_INT_WAVES 1
#endif
template <int SEM, int MAXS, bool FUSED>
__global__ __launch_bounds__(INT_THREADS, TSDF_INT_WAVES) void k_integrate(BatchRef D, Table T, Work Wk, Pool Pl,
                                                          Globals* G, int parity, RayConst R) {
    constexpr int PER = SEM == 3 ? TSDF_INT_PER3 : INT_PER;  // register-cached samples per thread
    constexpr uint32_t CAP = PER * INT_THREADS;                // samples (>= live cells) per window
    constexpr int NSLOT = FUSED ? INT_SPT * SPAN : PER;  // register-cached samples per thread
    constexpr bool VB = SEM == 1 || SEM == 3;  // Voxblox fuse (3: per-sample weights in the records)
    constexpr int NW = SEM == 3 ? NSLOT : 1;    // register-cached sample weights per thread
    typedef typename std::conditional<VB, unsigned long long, uint32_t>::type CellB;
    __shared__ unsigned long long cA[CAP];  // live cell: sum of trunc(s w * 2^32)
    __shared__ CellB cB[CAP];               // live cell: sample count / sum of trunc(w 2^32)
    const float tau = R.tau;
    __shared__ MaskT sMask[BRICK_VOX_LDS];     // voxel: scans (bit t - t0) observed in the window
    __shared__ uint32_t sBase[BRICK_VOX_LDS];  // voxel: first live cell
    __shared__ float sS[BRICK_VOX_LDS], sW[BRICK_VOX_LDS];
    __shared__ uint16_t sLive[BRICK_VOX];  // live voxels of the window
    // brick's per-scan sample prefix, double-buffered by brick parity: a wave may still read the
    // previous brick's prefix while another writes the next one
    __shared__ uint32_t s_csb[2][MAXS + 1];
    __shared__ uint32_t s_psb[FUSED ? 2 : 1][FUSED ? MAXS + 1 : 1];  // FUSED: per-scan span positions
    static_assert(MAXS <= 2 * INT_THREADS, "two cells per thread");
    __shared__ uint32_t s_red[INT_THREADS / 64];
    __shared__ uint32_t s_nlive, s_ncell;
    float2* cF = reinterpret_cast<float2*>(cA);  // P4: cells converted to (A 2^-32, B) as f32
    Counters* C = &G->ctr[parity];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
    // a batch that overflowed (or follows one) is replayed after the host grows the buffers: its
    // field writes are skipped, everything else (cell clean-up) runs
    const bool commit = !(G->retry && (C->ovf || G->failed));
    sMask[VOXL(tid)] = 0;
    sMask[VOXL(tid + 256)] = 0;
#if TSDF_INT_ZERO_IN_FUSE
    // every cell starts at zero; each window's fuse chains zero the cells they consumed
    for (uint32_t j = tid; j < CAP; j += INT_THREADS) {
        cA[j] = 0ull;
        cB[j] = 0;
    }
#endif
    uint32_t nvox = 0, ndirty = 0, par = 0;
#ifdef TSDF_PHASE_TIMING
    unsigned long long ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t_last = clock64();
    const unsigned long long t_first = __builtin_amdgcn_s_memrealtime();
    uint32_t nb = 0, nwin = 0;
#endif
    // Software pipeline over the workgroup's bricks: while brick a is processed, brick a + G's
    // cell row, (S, W) and first CAP samples are in flight to registers (BrickRegs), and
    // brick a + 2G's active record is loading.  A brick then starts with its data at hand.
    typedef typename std::conditional<FUSED, unsigned long long, uint32_t>::type CellT;
    const CellT* cells = reinterpret_cast<const CellT*>(T.cell);
    struct BrickRegs {
        uint2 c[NSLOT];
        float cw[NW];
        float s0, s1, w0, w1;
        CellT cell, cell2;
    };
    // FUSED: span records [p, min(p + INT_SCH, pend)) -> sp; their samples -> c (a span of cnt
    // samples fills slots j * SPAN .. j * SPAN + cnt - 1; empty slots hold scan ~0: never in a window)
    auto load_spans = [&](uint32_t p, uint32_t pend, uint32_t (&sp)[INT_SPT]) {
#pragma unroll
        for (int j = 0; j < INT_SPT; j++) {
            const uint32_t q = p + tid + j * INT_THREADS;
            sp[j] = (q < pend && q < Wk.max_spn) ? Wk.spn[q] : NO_SPAN;
        }
    };
    auto load_span_samples = [&](const uint32_t (&sp)[INT_SPT], uint2 (&c)[NSLOT]) {
#pragma unroll
        for (int j = 0; j < INT_SPT; j++) {
            const uint32_t e = sp[j];
            const uint32_t src = e & 0x3FFFFFFFu, cnt = e == NO_SPAN ? 0u : (e >> 30) + 1u;
#pragma unroll
            for (int k = 0; k < SPAN; k++)
                c[j * SPAN + k] = ((uint32_t)k < cnt && src + k < Wk.max_smp) ? Wk.smp[src + k]
                                                                           : make_uint2(0u, ~0u);
        }
    };
    uint32_t SP[INT_SPT];  // FUSED: span records of the next brick to load
    auto load_brick = [&](const uint4& r, BrickRegs& B) {
        const uint32_t n = r.w, base = r.z;
        const bool has = r.y < T.max_bricks;
        if constexpr (FUSED) {
            load_span_samples(SP, B.c);
        } else {
#pragma unroll
            for (int j = 0; j < PER; j++) {
                const uint32_t i = tid + j * INT_THREADS;
                // base + i >= max_smp: capacity overflow (reported by k_compact)
                float wv = 0.0f;
                B.c[j] = (i < n && base + i < Wk.max_smp) ? smp_load<SEM>(Wk, base + i, wv) : make_uint2(0u, ~0u);
                if constexpr (SEM == 3) B.cw[j] = wv;
            }
        }
        // two walks: absolute position of the brick's scan-tid samples -> relative to its segment
        // (made relative to the segment where it is consumed: a use here, or a load inside a
        // branch, would make the compiler wait for this prefetch at once); FUSED: the cell as is
        B.cell = cells[(size_t)r.x * T.cell_stride + min((uint32_t)tid, T.cell_stride - 1u)];
        if (MAXS > INT_THREADS)
            B.cell2 = cells[(size_t)r.x * T.cell_stride +
                            min((uint32_t)tid + INT_THREADS, T.cell_stride - 1u)];
        const float* Sg = Pl.sdf + (size_t)(has ? r.y : 0) * BRICK_VOX;
        const float* Wg = Pl.weight + (size_t)(has ? r.y : 0) * BRICK_VOX;
        B.s0 = has ? Sg[tid] : R.bg;
        B.s1 = has ? Sg[tid + 256] : R.bg;
        B.w0 = has ? Wg[tid] : 0.0f;
        B.w1 = has ? Wg[tid + 256] : 0.0f;
    };
    const uint32_t G0 = gridDim.x;
    const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);
    auto rec_at = [&](uint32_t a) { return a < n_active ? Wk.active[a] : zero4; };
    BrickRegs P;
    uint4 rec = rec_at(blockIdx.x);
    uint4 rec_next = rec_at(blockIdx.x + G0);
    uint4 rec_next2 = FUSED ? rec_at(blockIdx.x + 2 * G0) : zero4;
    if constexpr (FUSED) {
        // three-stage pipeline: records three bricks ahead, span records two, samples one
        if (blockIdx.x < n_active) {
            load_spans(rec.z, rec.z + rec.w, SP);
            load_brick(rec, P);
        }
        if (blockIdx.x + G0 < n_active) load_spans(rec_next.z, rec_next.z + rec_next.w, SP);
    } else {
        if (blockIdx.x < n_active) load_brick(rec, P);
    }
    for (uint32_t a = blockIdx.x; a < n_active; a += G0, par ^= 1u) {
        uint32_t* s_cs = s_csb[par];
        uint32_t* s_ps = s_psb[FUSED ? par : 0];
        const uint4 cur = rec;  // (h, slot, toff, n); FUSED: (h, slot, first span, spans)
        const BrickRegs B = P;
        rec = rec_next;
        if (a + G0 < n_active) load_brick(rec, P);  // brick a + G
        if constexpr (FUSED) {
            rec_next = rec_next2;
            if (a + 2 * G0 < n_active) load_spans(rec_next.z, rec_next.z + rec_next.w, SP);  // a + 2G
            if (a + 3 * G0 < n_active) rec_next2 = Wk.active[a + 3 * G0];                  // a + 3G
        } else {
            if (a + 2 * G0 < n_active) rec_next = Wk.active[a + 2 * G0];  // record of a + 2G
        }
        const uint32_t h = cur.x, n = cur.w, base = cur.z;
        uint2 c[NSLOT];
        float cw[NW];
#pragma unroll
        for (int j = 0; j < NSLOT; j++) c[j] = B.c[j];
#pragma unroll
        for (int j = 0; j < NW; j++) cw[j] = B.cw[j];
        // samples [cq, cq + CAP) (FUSED: spans [cq, cq + INT_SCH)) are in c[] (uniform)
        uint32_t cq = FUSED ? base : 0u;
        const uint32_t pend = FUSED ? base + n : 0u;  // FUSED: the brick's span end
        auto load_chunk = [&](uint32_t q) {
            cq = q;
            if constexpr (FUSED) {
                uint32_t sp[INT_SPT];
                load_spans(q, pend, sp);
                load_span_samples(sp, c);
            } else {
#pragma unroll
                for (int j = 0; j < PER; j++) {
                    const uint32_t i = q + tid + j * INT_THREADS;
                    float wv = 0.0f;
                    c[j] = (i < n && base + i < Wk.max_smp) ? smp_load<SEM>(Wk, base + i, wv) : make_uint2(0u, ~0u);
                    if constexpr (SEM == 3) cw[j] = wv;
                }
            }
        };
        const bool has_slot = cur.y < T.max_bricks;
        if constexpr (FUSED) {
            // per scan: relative sample prefix, absolute span position (scan ns: the totals)
            if ((uint32_t)tid <= ns) {
                s_cs[tid] = (uint32_t)B.cell;
                s_ps[tid] = (uint32_t)(B.cell >> 32);
            }
            if (MAXS > INT_THREADS && (uint32_t)tid + INT_THREADS <= ns) {
                s_cs[tid + INT_THREADS] = (uint32_t)B.cell2;
                s_ps[tid + INT_THREADS] = (uint32_t)(B.cell2 >> 32);
            }
        } else {
            if ((uint32_t)tid < ns) s_cs[tid] = B.cell - base;
            if (MAXS > INT_THREADS && (uint32_t)tid + INT_THREADS < ns) s_cs[tid + INT_THREADS] = B.cell2 - base;
            if (tid == 0) s_cs[ns] = n;
        }
        float* Sg = Pl.sdf + (size_t)(has_slot ? cur.y : 0) * BRICK_VOX;
        float* Wg = Pl.weight + (size_t)(has_slot ? cur.y : 0) * BRICK_VOX;
        // sS / sW of voxels tid, tid + 256: the previous brick's last readers are past a barrier
        sS[VOXL(tid)] = B.s0;
        sS[VOXL(tid + 256)] = B.s1;
        sW[VOXL(tid)] = B.w0;
        sW[VOXL(tid + 256)] = B.w1;
        uint32_t dirty = 0;  // voxels 2 tid, 2 tid + 1 (bits 0, 1)
        PHASE(0);
        __syncthreads();  // s_cs, sS, sW visible
        PHASE(1);
        for (uint32_t t0 = 0; t0 < ns;) {
            // window [t0, t1): as many scans as keep its samples <= CAP (at least one)
            // (the extension test is monotone in the scan: one lane per candidate, one ballot)
            const uint32_t q0 = s_cs[t0];
            const uint32_t p0 = FUSED ? s_ps[t0] : 0u;
            const uint32_t tt = t0 + 1 + lane;
            const bool ext = tt < ns && tt - t0 < INT_MAX_WIN && s_cs[min(tt + 1, ns)] - q0 <= CAP &&
                             (!FUSED || s_ps[min(tt + 1, ns)] - p0 <= INT_SCH);
            const uint32_t t1 = t0 + 1 + (uint32_t)__popcll(__ballot(ext));
            const uint32_t q1 = s_cs[t1], nw = t1 - t0;
            const uint32_t p1 = FUSED ? s_ps[t1] : 0u;
            // the window's chunks: samples [q0, q1) in CAP steps, FUSED spans [p0, p1) in INT_SCH
            const uint32_t ck0 = FUSED ? p0 : q0, ck1 = FUSED ? p1 : q1;
            constexpr uint32_t CK = FUSED ? INT_SCH : CAP;
            if (q0 == q1) {  // uniform: no sample of this brick in the window
                t0 = t1;
                continue;
            }
#ifdef TSDF_PHASE_TIMING
            nwin++;
#endif
            // P1: scan masks (a one-scan window may exceed CAP samples: chunked)
            for (uint32_t qc = ck0; qc < ck1; qc += CK) {
                if (cq != qc) {
                    load_chunk(qc);
                    PHASE(2);
                }
#pragma unroll
                for (int j = 0; j < NSLOT; j++) {
                    const uint32_t w = (c[j].y >> 9) - t0;
#ifdef TSDF_ABLATE_INT_NOP1
                    if (w < nw && c[j].x == 0x7FFFFFFFu)
#else
                    if (w < nw)
#endif
                        atomicOr(&sMask[VOXL(c[j].y & 511u)], (MaskT)1 << w);
                }
            }
            __syncthreads();
            PHASE(3);
            // P2: live cells and live voxels (packed block scan: cells | voxels << 16)
            {
                const MaskT m0 = sMask[VOXL(2 * tid)], m1 = sMask[VOXL(2 * tid + 1)];
                const uint32_t c0 = MASK_POPC(m0), c1 = MASK_POPC(m1);
                const uint32_t v0 = m0 ? 1u : 0u, v1 = m1 ? 1u : 0u;
                dirty |= v0 | (v1 << 1);
                const uint32_t x = (c0 + c1) | ((v0 + v1) << 16);
#ifdef TSDF_SHFL_SCAN
                uint32_t incl = x;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += y;
                }
#else
                const uint32_t incl = wave_incl_scan(x);
#endif
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
                sBase[VOXL(2 * tid)] = cb;
                sBase[VOXL(2 * tid + 1)] = cb + c0;
                if (v0) sLive[vb] = (uint16_t)(2 * tid);
                if (v1) sLive[vb + v0] = (uint16_t)(2 * tid + 1);
                if (tid == 0) {
                    s_nlive = tot >> 16;
                    s_ncell = tot & 0xFFFFu;
                    nvox += tot & 0xFFFFu;  // (voxel, scan) updates of the window
                }
#if !TSDF_INT_ZERO_IN_FUSE
                // the window's cells start at zero (the previous window's P4 is past a barrier)
                for (uint32_t j = tid; j < (tot & 0xFFFFu); j += INT_THREADS) {
                    cA[j] = 0ull;
                    cB[j] = 0;
                }
#endif
            }
            __syncthreads();
            PHASE(4);
            // P3: accumulate into the live cells
            for (uint32_t qc = ck0; qc < ck1; qc += CK) {
                if (cq != qc) {
                    load_chunk(qc);
                }
#pragma unroll
                for (int j = 0; j < NSLOT; j++) {
                    const uint32_t w = (c[j].y >> 9) - t0;
                    if (w < nw) {
                        const uint32_t l = VOXL(c[j].y & 511u);
                        const uint32_t cell = sBase[l] + MASK_POPC(sMask[l] & (((MaskT)1 << w) - 1));
                        const float sv = __uint_as_float(c[j].x);
                        if constexpr (VB) {
                            float wv;
                            if constexpr (SEM == 3) wv = cw[j];
                            else wv = vb_weight(R, 1.0f, sv);
                            const long long fa = (long long)((sv * wv) * 4294967296.0f);
                            const long long fb = (long long)(wv * 4294967296.0f);
                            atomicAdd(&cA[cell], (unsigned long long)fa);
                            atomicAdd(&cB[cell], (unsigned long long)fb);
                        } else {
                            const long long fx = (long long)(sv * 4294967296.0f);
#ifdef TSDF_ABLATE_INT_NOP3
                            if (fx == 12345)
#endif
                            {
                                atomicAdd(&cA[cell], (unsigned long long)fx);
                                atomicAdd(&cB[cell], 1u);
                            }
                        }
                    }
                }
            }
            // the next window starts at q1: its samples load while this one converts and fuses
            if (FUSED ? p1 < pend : q1 < n) load_chunk(ck1);
            __syncthreads();
            PHASE(5);
#ifndef TSDF_FUSE_P4A
            // VDBFusion: the chains convert their raw cells themselves, two steps ahead of use
            // (off the chain's critical path), so there is no conversion pass and no barrier
            constexpr bool inline_cvt = SEM == 0;
#else
            constexpr bool inline_cvt = false;
#endif
            // P4a: convert every live cell to (A 2^-32, B) in f32, in parallel, so the serial
            // per-voxel chains below are one LDS read, a multiply-add and a division per step
            if constexpr (!inline_cvt) {
                const uint32_t ncell = s_ncell;
                for (uint32_t j = tid; j < ncell; j += INT_THREADS) {
                    const long long av = (long long)cA[j];
                    const float af = (float)((double)av * (1.0 / 4294967296.0));
                    if constexpr (VB)
                        cF[j] = make_float2(af, (float)((double)(long long)cB[j] * (1.0 / 4294967296.0)));
                    else
                        cF[j] = make_float2(af, (float)cB[j]);
                }
            }
            if constexpr (!inline_cvt) __syncthreads();
            PHASE(8);
            // P4b: fuse.  Lane tid takes live voxels tid, tid + 256 and runs each one's chain in scan
            // order; the next cell is read from LDS while the current step divides, so a step costs
            // the arithmetic only (the critical path of a window is its longest chain).
            {
#ifdef TSDF_ABLATE_INT_NOP4
                const uint32_t nlive = 0;
#else
                const uint32_t nlive = s_nlive;
#endif
                for (uint32_t vi = tid; vi < nlive; vi += INT_THREADS) {
                    const uint32_t l = VOXL(sLive[vi]);
                    const uint32_t cell = sBase[l];
                    const uint32_t rem = MASK_POPC(sMask[l]);
                    sMask[l] = 0;
                    float s = sS[l], wt = sW[l];
                    if constexpr (inline_cvt) {
                        typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64r;
                        typedef const volatile __attribute__((address_space(3))) uint32_t lds_u32r;
                        lds_u64r* rA = (lds_u64r*)(cA);
                        lds_u32r* rB = (lds_u32r*)(cB);
                        uint64_t a0 = rA[cell], a1 = rA[min(cell + 1u, CAP - 1u)];
                        uint32_t b0 = rB[cell], b1 = rB[min(cell + 1u, CAP - 1u)];
                        for (uint32_t k = 0; k < rem; k += 2) {
                            const uint64_t na0 = rA[min(cell + k + 2, CAP - 1u)];
                            const uint32_t nb0 = rB[min(cell + k + 2, CAP - 1u)];
                            const uint64_t na1 = rA[min(cell + k + 3, CAP - 1u)];
                            const uint32_t nb1 = rB[min(cell + k + 3, CAP - 1u)];
                            const float fa0 = (float)((double)(long long)a0 * (1.0 / 4294967296.0));
                            const float fa1 = (float)((double)(long long)a1 * (1.0 / 4294967296.0));
                            float nwt = wt + (float)b0;
                            s = (s * wt + fa0) / nwt;
                            wt = nwt;
                            nwt = wt + (float)b1;
                            const float s2 = (s * wt + fa1) / nwt;
                            const bool more = k + 1 < rem;
                            s = more ? s2 : s;
                            wt = more ? nwt : wt;
                            a0 = na0;
                            a1 = na1;
                            b0 = nb0;
                            b1 = nb1;
#if TSDF_INT_ZERO_IN_FUSE
                            cA[cell + k] = 0ull;  // consumed (read two steps ago)
                            cB[cell + k] = 0;
                            if (more) {
                                cA[cell + k + 1] = 0ull;
                                cB[cell + k + 1] = 0;
                            }
#endif
                        }
                        sS[l] = s;
                        sW[l] = wt;
                        continue;
                    }
                    // two cells in flight: a step's operand was read one step earlier
                    float2 va = cF[cell], vb = cF[min(cell + 1u, CAP - 1u)];
                    // branch-free body (one basic block, so the reads stay ahead of their use);
                    // the second step of a pair is dropped past the chain's end
                    typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64;
                    lds_u64* cV = (lds_u64*)(cA);
                    // Voxblox updateTsdfVoxel on a cell (a, b) = (sum s w, sum w):
                    // W' = W + b (no update below kFloatEpsilon), S' = (a + S W) / W' clamped to
                    // +-tau, W = min(max_weight, W')
                    auto vb_fuse = [&](float2 v, float& s_, float& w_) {
                        const float nw = w_ + v.y;
                        float ns = (v.x + s_ * w_) / nw;
                        ns = ns > 0.0f ? (ns < tau ? ns : tau) : (-tau < ns ? ns : -tau);
                        const bool ok = !(nw < 1e-6f);
                        s_ = ok ? ns : s_;
                        w_ = ok ? (nw < R.max_weight ? nw : R.max_weight) : w_;
                    };
                    for (uint32_t k = 0; k < rem; k += 2) {
                        const uint64_t na = cV[min(cell + k + 2, CAP - 1u)];
                        uint64_t nb;
                        if constexpr (VB) {
                            vb_fuse(va, s, wt);
                            nb = cV[min(cell + k + 3, CAP - 1u)];
                            float s2 = s, w2 = wt;
                            vb_fuse(vb, s2, w2);
                            const bool more = k + 1 < rem;
                            s = more ? s2 : s;
                            wt = more ? w2 : wt;
                        } else {
                            float nwt = wt + va.y;
                            s = (s * wt + va.x) / nwt;
                            wt = nwt;
                            nb = cV[min(cell + k + 3, CAP - 1u)];
                            nwt = wt + vb.y;
                            const float s2 = (s * wt + vb.x) / nwt;
                            const bool more = k + 1 < rem;
                            s = more ? s2 : s;
                            wt = more ? nwt : wt;
                        }
                        va = make_float2(__uint_as_float((uint32_t)na), __uint_as_float((uint32_t)(na >> 32)));
                        vb = make_float2(__uint_as_float((uint32_t)nb), __uint_as_float((uint32_t)(nb >> 32)));
#if TSDF_INT_ZERO_IN_FUSE
                        cA[cell + k] = 0ull;  // consumed (cF aliases cA)
                        cB[cell + k] = 0;
                        if (k + 1 < rem) {
                            cA[cell + k + 1] = 0ull;
                            cB[cell + k + 1] = 0;
                        }
#endif
                    }
                    sS[l] = s;
                    sW[l] = wt;
                }
            }
            __syncthreads();
            PHASE(6);
            t0 = t1;
        }
        if (has_slot && commit) {
            if (dirty & 1u) {
                Sg[2 * tid] = sS[VOXL(2 * tid)];
                Wg[2 * tid] = sW[VOXL(2 * tid)];
            }
            if (dirty & 2u) {
                Sg[2 * tid + 1] = sS[VOXL(2 * tid + 1)];
                Wg[2 * tid + 1] = sW[VOXL(2 * tid + 1)];
            }
        }
        ndirty += __popc(dirty);
        // zero every cell of the brick (k_compact prefixes whole uint4 groups) for the next batch
        for (uint32_t q = tid; q < T.cell_stride; q += INT_THREADS)
            const_cast<CellT*>(cells)[(size_t)h * T.cell_stride + q] = 0u;
#ifdef TSDF_PHASE_TIMING
        nb++;
#endif
        PHASE(7);
        __syncthreads();  // write-back reads of sS / sW done before the next brick stages its own
    }
#ifdef TSDF_PHASE_TIMING
#ifdef TSDF_PHASE_ALL
    if (tid == 0)
        printf("wg %u bricks %u total %llu start %llu\n", blockIdx.x, nb,
               ph[0] + ph[1] + ph[2] + ph[3] + ph[4] + ph[5] + ph[6] + ph[7] + ph[8], t_first);
    if (false)
#else
    if (tid == 0 && (blockIdx.x % 97) == 0)
#endif
        printf("phase blk %u bricks %u windows %u meta %llu bar0 %llu load %llu mask %llu scan %llu "
               "acc %llu conv %llu fuse %llu tail %llu\n", blockIdx.x, nb, nwin, ph[0], ph[1], ph[2],
               ph[3], ph[4], ph[5], ph[8], ph[6], ph[7]);
#endif
    const unsigned long long v = wave_sum<unsigned long long>(nvox);
    const unsigned long long d = wave_sum<unsigned long long>(ndirty);
    if (lane == 0) {
        if (v) atomicAdd(&C->n_vox[blockIdx.x & 7], v);  // -> G->tot_vox at k_finish
        if (d) atomicAdd(&C->n_dirty[blockIdx.x & 7], d);
    }
}

// ------------------------------------------------------------------------------------------------
// k_integrate_small: the same update for batches of at most SMALL_NS scans (a live node's 1-8 scan
// batches), one WAVE per brick instead of a workgroup.  With few scans a voxel's chain is at most
// SMALL_NS steps, so the window / mask / live-cell machinery of k_integrate (six workgroup barriers
// per brick) costs more than it saves: here a wave keeps its brick's 512 (S, W) in registers (voxel
// lane + 64 k, k < 8), and takes the brick's scans in order:
//   accumulate scan t's samples (one contiguous segment) into dense per-voxel LDS cells
//   (int64 fixed-point sum, count / weight sum) with LDS atomics, then every lane fuses its 8
//   voxels' cells with the same arithmetic as k_integrate's chains and clears them.
// No barrier (wave-private LDS), no size order (the list is taken in table order), four bricks per
// workgroup.  Software-pipelined like k_integrate: while brick a is fused, brick a + G's cell row,
// (S, W) and first SML_K x 64 samples (the record gives the segment, so they need not wait for the
// cell row) are in flight to registers, and brick a + 2G's record is loading.
// The field is bitwise k_integrate's (tests/test_gpu_parity.py::test_small_batch_kernel_bitwise).
constexpr int SML_WAVES = 4;
#ifndef TSDF_SML_K
#define TSDF_SML_K 8
#endif
constexpr int SML_K = TSDF_SML_K;  // register-cached samples per lane
template <int SEM>
__global__ __launch_bounds__(SML_WAVES * 64) void k_integrate_small(BatchRef D, Table T, Work Wk,
                                                                   Pool Pl, Globals* G, int parity,
                                                                   RayConst R) {
    constexpr bool VB = SEM == 1 || SEM == 3;
    constexpr int NW = SEM == 3 ? SML_K : 1;
    typedef typename std::conditional<VB, unsigned long long, uint32_t>::type CellB;
    __shared__ unsigned long long sA[SML_WAVES][BRICK_VOX];
    __shared__ CellB sB[SML_WAVES][BRICK_VOX];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long* A = sA[wid];
    CellB* Bc = sB[wid];
    Counters* C = &G->ctr[parity];
    const uint32_t n_active = min(C->n_active, Wk.max_active);
    const uint32_t ns = D.n_scans;
    const bool commit = !(G->retry && (C->ovf || G->failed));
    const float tau = R.tau;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        A[lane + 64 * k] = 0ull;
        Bc[lane + 64 * k] = 0;
    }
    struct Regs {
        uint32_t cell;     // lane t < ns: absolute position of the brick's scan-t samples
        float s[8], w[8];  // voxels lane + 64 k
        uint2 c[SML_K];    // samples lane + 64 j of the segment
        float cw[NW];      // SEM 3: their weights
    };
    auto load = [&](const uint4& r, Regs& P) {
        const uint32_t base = r.z, n = r.w;
        const bool has = r.y < T.max_bricks;
        P.cell = (uint32_t)lane < ns ? T.cell[(size_t)r.x * T.cell_stride + lane] : 0u;
        const float* Sg = Pl.sdf + (size_t)(has ? r.y : 0) * BRICK_VOX;
        const float* Wg = Pl.weight + (size_t)(has ? r.y : 0) * BRICK_VOX;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            P.s[k] = has ? Sg[lane + 64 * k] : R.bg;
            P.w[k] = has ? Wg[lane + 64 * k] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < SML_K; j++) {
            const uint32_t i = lane + 64 * j;
            const bool ok = i < n && base + i < Wk.max_smp;  // past max_smp: overflow (k_compact)
            float wv = 0.0f;
            P.c[j] = ok ? smp_load<SEM>(Wk, base + i, wv) : make_uint2(0u, 0u);
            if constexpr (SEM == 3) P.cw[j] = wv;
        }
    };
    auto add = [&](uint2 c, float wv_stored) {
        const uint32_t l = c.y & 511u;
        const float sv = __uint_as_float(c.x);
        if constexpr (VB) {
            float wv;
            if constexpr (SEM == 3) wv = wv_stored;
            else wv = vb_weight(R, 1.0f, sv);
            atomicAdd(&A[l], (unsigned long long)(long long)((sv * wv) * 4294967296.0f));
            atomicAdd(&Bc[l], (unsigned long long)(long long)(wv * 4294967296.0f));
        } else {
            (void)wv_stored;
            atomicAdd(&A[l], (unsigned long long)(long long)(sv * 4294967296.0f));
            atomicAdd(&Bc[l], 1u);
        }
    };
    uint32_t nvox = 0, ndirty = 0;
    const uint32_t stride = gridDim.x * SML_WAVES;
    const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);
    uint32_t a = blockIdx.x * SML_WAVES + wid;
    uint4 rec = a < n_active ? Wk.active[a] : zero4;
    uint4 rec_next = a + stride < n_active ? Wk.active[a + stride] : zero4;
    Regs P;
    if (a < n_active) load(rec, P);
    for (; a < n_active; a += stride) {
        const uint4 cur = rec;
        const Regs B = P;
        rec = rec_next;
        if (a + stride < n_active) load(rec, P);                                  // brick a + G
        if (a + 2 * stride < n_active) rec_next = Wk.active[a + 2 * stride];       // record of a + 2G
        const uint32_t h = cur.x, base = cur.z, n = cur.w;
        const bool has = cur.y < T.max_bricks;
        // lane t <= ns: start of scan t's samples relative to the segment (ns: the end)
        const uint32_t cst = (uint32_t)lane < ns ? B.cell - base : n;
        float s[8], w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            s[k] = B.s[k];
            w[k] = B.w[k];
        }
        uint32_t dirty = 0;
        for (uint32_t t = 0; t < ns; t++) {
            const uint32_t q0 = __shfl(cst, (int)t), q1 = __shfl(cst, (int)t + 1);
            if (q0 == q1) continue;  // uniform: no sample of scan t in this brick
#pragma unroll
            for (int j = 0; j < SML_K; j++) {
                const uint32_t i = lane + 64 * j;
                if (i >= q0 && i < q1) add(B.c[j], B.cw[SEM == 3 ? j : 0]);
            }
            for (uint32_t i = max(q0, 64u * SML_K) + lane; i < q1; i += 64) {  // past the cache
                if (base + i >= Wk.max_smp) continue;
                float wv = 0.0f;
                const uint2 cs = smp_load<SEM>(Wk, base + i, wv);
                add(cs, wv);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the cells complete
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t v = lane + 64 * k;
                const CellB b = Bc[v];
                if (b == 0) continue;  // every live cell has b > 0 (Voxblox: w >= 2^-16)
                const float fa = (float)((double)(long long)A[v] * (1.0 / 4294967296.0));
                A[v] = 0ull;
                Bc[v] = 0;
                if constexpr (VB) {
                    const float fb = (float)((double)(long long)b * (1.0 / 4294967296.0));
                    const float nw = w[k] + fb;
                    float sn = (fa + s[k] * w[k]) / nw;
                    sn = sn > 0.0f ? (sn < tau ? sn : tau) : (-tau < sn ? sn : -tau);
                    const bool ok = !(nw < 1e-6f);
                    s[k] = ok ? sn : s[k];
                    w[k] = ok ? (nw < R.max_weight ? nw : R.max_weight) : w[k];
                } else {
                    const float nw = w[k] + (float)b;
                    s[k] = (s[k] * w[k] + fa) / nw;
                    w[k] = nw;
                }
                dirty |= 1u << k;
                nvox++;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // cleared before the next scan
            __builtin_amdgcn_wave_barrier();
        }
        if (has && commit) {
            float* So = Pl.sdf + (size_t)cur.y * BRICK_VOX;
            float* Wo = Pl.weight + (size_t)cur.y * BRICK_VOX;
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (dirty & (1u << k)) {
                    So[lane + 64 * k] = s[k];
                    Wo[lane + 64 * k] = w[k];
                }
        }
        ndirty += __popc(dirty);
        // zero the brick's cell row (k_compact prefixes whole uint4 groups) for the next batch
        for (uint32_t q = lane; q < T.cell_stride; q += 64) T.cell[(size_t)h * T.cell_stride + q] = 0u;
    }
    const unsigned long long v = wave_sum<unsigned long long>(nvox);
    const unsigned long long d = wave_sum<unsigned long long>(ndirty);
    if (lane == 0) {
        if (v) atomicAdd(&C->n_vox[blockIdx.x & 7], v);  // -> G->tot_vox at k_finish
        if (d) atomicAdd(&C->n_dirty[blockIdx.x & 7], d);
    }
}

// Grid = exactly the workgroups the device holds at once (CUs x resident workgroups per CU, from
// the occupancy API: VGPRs or LDS, whichever binds): every workgroup of the grid-stride loop starts
// at once, none waits for a second dispatch round.
template <typename K>
static int resident_grid(K kernel, int threads, int fallback_per_cu) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess ||
        cus <= 0 || per_cu <= 0) {
        cus = 256;
        per_cu = fallback_per_cu;
    }
    return cus * per_cu;
}

template <int SEM, int MAXS, bool FUSED>
static int integrate_grid() {
    static int grid = 0;
    if (grid == 0) grid = resident_grid(k_integrate<SEM, MAXS, FUSED>, INT_THREADS, INT_BLOCKS_PER_CU);
    return grid;
}

template <int SEM>
static void integrate_small_sem(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                                const Pool& Pl, Globals* G, int parity, hipStream_t st,
                                const KTime& kt) {
    static int grid = 0;
    if (grid == 0) grid = resident_grid(k_integrate_small<SEM>, SML_WAVES * 64, 4);
    tlaunch(k_integrate_small<SEM>, grid, SML_WAVES * 64, st, kt.start, kt.stop, D, T, Wk, Pl, G,
            parity, R);
}

hipError_t launch_integrate_small(const BatchRef& D, const RayConst& R, const Table& T,
                                  const Work& Wk, const Pool& Pl, Globals* G, int parity,
                                  hipStream_t st, const KTime& kt) {
    // SEM 2 (VDBFusion at double precision) fuses like SEM 0
    if (R.sem == 1) integrate_small_sem<1>(D, R, T, Wk, Pl, G, parity, st, kt);
    else if (R.sem == 3) integrate_small_sem<3>(D, R, T, Wk, Pl, G, parity, st, kt);
    else integrate_small_sem<0>(D, R, T, Wk, Pl, G, parity, st, kt);
    return hipGetLastError();
}

template <int SEM, int MAXS, bool FUSED>
static void integrate_sem(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                          const Pool& Pl, Globals* G, int parity, hipStream_t st, const KTime& kt) {
    tlaunch(k_integrate<SEM, MAXS, FUSED>, integrate_grid<SEM, MAXS, FUSED>(), INT_THREADS, st,
            kt.start, kt.stop, D, T, Wk, Pl, G, parity, R);
}

template <bool FUSED>
static void integrate_mode(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                           const Pool& Pl, Globals* G, int parity, bool big, hipStream_t st,
                           const KTime& kt) {
    // SEM 2 (VDBFusion at double precision) fuses like SEM 0; SEM 3 (Voxblox 1/z^2) never takes
    // the single walk (tsdf_capi.cpp)
    if (R.sem == 1) {
        if (big) integrate_sem<1, MAX_BATCH, FUSED>(D, R, T, Wk, Pl, G, parity, st, kt);
        else integrate_sem<1, 64, FUSED>(D, R, T, Wk, Pl, G, parity, st, kt);
    } else if (R.sem == 3) {
        if constexpr (!FUSED) {
            if (big) integrate_sem<3, MAX_BATCH, false>(D, R, T, Wk, Pl, G, parity, st, kt);
            else integrate_sem<3, 64, false>(D, R, T, Wk, Pl, G, parity, st, kt);
        }
    } else {
        if (big) integrate_sem<0, MAX_BATCH, FUSED>(D, R, T, Wk, Pl, G, parity, st, kt);
        else integrate_sem<0, 64, FUSED>(D, R, T, Wk, Pl, G, parity, st, kt);
    }
}

hipError_t launch_integrate(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                            const Pool& Pl, Globals* G, int parity, bool fused, bool big,
                            hipStream_t st, const KTime& kt) {
    if (fused) integrate_mode<true>(D, R, T, Wk, Pl, G, parity, big, st, kt);
    else integrate_mode<false>(D, R, T, Wk, Pl, G, parity, big, st, kt);
    return hipGetLastError();
}

}  // namespace tsdf
