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
//               slot if it is new, and the prefix of its per-scan cells (records scan-ordered);
//               it sweeps the table's `touched` words, so k_count needs no first-touch atomics
//   k_place     same workgroups as k_count: coalesced read of the rays, one record
//               (x, y, z, in-brick sample count) written per pair to its brick segment
//   k_integrate (tsdf_integrate.hip) one workgroup per active brick: brick in LDS for the whole
//               batch, samples accumulated and fused scan by scan, touched voxels only.
// (Global atomics in k_count: one cell atomicAdd per distinct brick per workgroup, plus the
//  find-or-insert CAS of bricks new to the map.)
//
// Semantics: VDBFusion's VDBVolume::Integrate, restated in oracle/tsdf_oracle.c, which is the
// bit-exact CPU twin of this file's arithmetic.  Ray arithmetic is fp32 with contraction off
// (-ffp-contract=off) and correctly rounded div/sqrt, so the voxel sequence, the gate and every
// sample are the oracle's bits.  Per scan, the samples of a voxel are summed as exact 64-bit fixed
// point (trunc(s * 2^32)) plus a count, and fused in scan order, so the field does not depend on
// lane, wave, atomic or batch composition: it is bitwise reproducible and equal to the oracle's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

// ------------------------------------------------------------------------------------------------
// shared helpers of the batch kernels

// XCD-aware block order: the hardware deals workgroup p to XCD p % 8, so consecutive blocks --
// adjacent azimuth wedges of a scan -- would land on different XCDs, and a brick on a wedge border
// would have its cell row fetched into two L2s.  Within every aligned group of 8 G workgroups,
// physical p = 8 r + x takes logical block G x + r: XCD x gets G contiguous wedges (a full scan's
// 128 k_count blocks are one group of 8 x 16; its 256 k_place halves one group of 8 x 32), and the
// same wedges of every scan.  Measured: k_place 0.419 -> 0.404 ms, 50.9 k -> 51.8-52.2 k scans/s
// (profiles/r03/xcd/; TSDF_NO_XCD_WEDGE builds the plain order).
__device__ __forceinline__ uint32_t xcd_wedge(uint32_t p, uint32_t n, uint32_t G) {
#ifndef TSDF_NO_XCD_WEDGE
    const uint32_t grp = 8u * G, g0 = p - p % grp;
    if (g0 + grp > n) return p;  // the last, partial group keeps its order
    const uint32_t i = p - g0;
    return g0 + (i % 8u) * G + i / 8u;
#else
    (void)n;
    (void)G;
    return p;
#endif
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

// A workgroup-wide OR in one barrier: each wave publishes its vote in its own LDS slot
// (__syncthreads_or takes three barriers: store, atomic OR, load).  Every lane of the workgroup
// must call it; the slots may be reused after the next barrier.
template <int NT>
__device__ __forceinline__ bool block_any(bool p, uint32_t* s_vote) {
#ifdef TSDF_SYNC_OR
    (void)s_vote;
    return __syncthreads_or(p);
#else
    const uint32_t w = __any(p) ? 1u : 0u;
    if ((threadIdx.x & 63) == 0) s_vote[threadIdx.x >> 6] = w;
    __syncthreads();
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; k++) r |= s_vote[k];
    return r != 0;
#endif
}

// ------------------------------------------------------------------------------------------------
// k_count

#ifndef TSDF_CNT_THREADS
#define TSDF_CNT_THREADS 256
#endif
// Diagnostic build only (-DTSDF_CNT_PHASE, never shipped): thread 0 of every 61st k_count
// workgroup prints its wall-clock cycles per phase (walk and pair emission summed over its rays).
#ifdef TSDF_CNT_PHASE
#define CPH(k)                                             \
    do {                                                   \
        const unsigned long long t_ = __builtin_readcyclecounter(); \
        cph[k] += t_ - cpl;                                \
        cpl = t_;                                          \
    } while (0)
#else
#define CPH(k) \
    do {       \
    } while (0)
#endif
constexpr int CNT_THREADS = TSDF_CNT_THREADS;

// NT: threads per workgroup (1024 for batches too small to fill the chip, one ray per lane, so
// each SIMD holds four waves of one workgroup).  G: RPB-ray blocks per workgroup.  G = 2 (the
// default for full batches) takes two adjacent blocks of a scan in one 512-lane
// workgroup with one LDS brick hash, so a brick both wedges reach costs ONE global probe and ONE
// cell atomic instead of two (runs per 64-scan launch ~5.2 M -> ~3.7 M).  The run lists, staging
// plans and pair codes stay per (block, half), exactly as k_place reads them; a brick's LDS slot
// counts its samples in 2G 16-bit sub-counters, one per (block, half).  Two blocks of different
// scans (a scan with an odd block count) keep their bricks apart by a block bit in the LDS key.
template <int SEM, int NT = CNT_THREADS, int G = 1>
// TSDF_SEM_VDBFUSION_F64: the fp32 filter's rare double branch would lift k_count to 93 VGPRs (5
// waves per SIMD); the bound keeps the LDS-limited 6, spilling only inside that branch
#ifndef TSDF_F64_COUNT_WAVES
#define TSDF_F64_COUNT_WAVES 6
#endif
#ifndef TSDF_F64_PLACE_WAVES
#define TSDF_F64_PLACE_WAVES 1
#endif
__global__ __launch_bounds__(NT, SEM == 2 && (NT == CNT_THREADS || G == 2) ? TSDF_F64_COUNT_WAVES : 1) void k_count(const float* __restrict__ xyz, BatchRef D,
                                                      RayConst R, Table T, Work Wk, Globals* G_,
                                                      int parity) {
    static_assert(G == 1 || G == 2, "one or two blocks per workgroup");
    static_assert(G == 1 || RPB % NT == 0, "a pass over the rays stays inside one block");
    using CntT = typename std::conditional<G == 2, unsigned long long, uint32_t>::type;
    constexpr int PCAP = plan_cap(SEM), PW = plan_words(SEM);  // k_place<SEM>'s staging plan
#ifdef TSDF_CNT_SPLIT
    // variant build: the global phase (find-or-insert, cell atomic) runs in k_resolve
    constexpr bool SPLIT = G == 1;
#else
    constexpr bool SPLIT = false;
#endif
    __shared__ uint32_t s_wsl[SPLIT ? NT / 64 : 1];
    constexpr int NSUB = 2 * G;  // (block, half) sub-runs
    constexpr uint64_t KEY_G1 = 1ull << 63;  // LDS key bit: block 1 of a workgroup spanning two scans
    __shared__ unsigned long long s_key[HCAP];
    __shared__ CntT s_cnt[HCAP];
    __shared__ unsigned long long red[2][NT / 64];
    __shared__ unsigned long long s_wsum[G][NT / 64];
    __shared__ uint32_t s_wcnt[G][NT / 64];
    __shared__ uint32_t s_bm[NSUB][PW];  // per sub-run list: staging positions where a run starts
    Counters* C = &G_->ctr[parity];  // zeroed by the previous batch of this parity (k_finish)
    // sector sharding: every GPU sees every scan, and a block of 1024 consecutive rays (~3 degrees
    // of azimuth) usually lies wholly in one sector; the workgroups take the blocks k_sector_flags
    // listed, the rest of the grid leaves at once (G = 1 only)
    uint32_t bx = xcd_wedge(blockIdx.x, gridDim.x, 16 / G);
    if constexpr (G == 1) {
        if (R.sec_on) {
            if (blockIdx.x >= C->n_act) return;
            bx = Wk.act[blockIdx.x];
        }
    }
#ifdef TSDF_CNT_PHASE
    unsigned long long cph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, cpl = __builtin_readcyclecounter();
#endif
    // block g of the workgroup is G bx + g (past the batch's last block: an empty range)
    uint32_t tb[G], r0b[G], r1b[G];
#pragma unroll
    for (int g = 0; g < G; g++) block_range(D, G * bx + g, tb[g], r0b[g], r1b[g]);
    const bool split = G == 2 && tb[G - 1] != tb[0];
    for (int j = threadIdx.x; j < HCAP; j += NT) {
        s_key[j] = EMPTY_KEY;
        s_cnt[j] = 0u;
    }
    for (int j = threadIdx.x; j < NSUB * PW; j += NT) (&s_bm[0][0])[j] = 0u;
    __syncthreads();
    CPH(0);  // LDS init
    const uint32_t maxp = Wk.maxp;
    uint32_t valid = 0, npairs = 0;
    // The pair code of (ray, brick run): LDS-hash rank in the workgroup's run for the brick, or a
    // fallback record when the LDS hash is full.  cnt_in = the pair's gated voxels (<= MAX_IN_BRICK).
    // A run's samples are counted per (block, half) -- rays [0, RPB/2) and [RPB/2, RPB) of the
    // block: k_place runs one 512-lane workgroup per half -- as 16-bit fields of s_cnt, field
    // sub = 2 g + half (a field holds at most RPB/2 * MAX_IN_BRICK samples); the pair's rank is
    // within its sub-run.
    auto pair_code = [&](uint64_t bkey, uint32_t cnt_in, uint32_t sub, uint32_t t) -> uint32_t {
        const uint64_t lkey = split && sub >= 2 ? bkey | KEY_G1 : bkey;
        const int lid = lds_insert(s_key, lkey);
        if (lid >= 0) {
            const CntT old = atomicAdd(&s_cnt[lid], (CntT)cnt_in << (16 * sub));
            const uint32_t lr = (uint32_t)(old >> (16 * sub)) & 0xFFFFu;
            return (cnt_in << PAIR_CNT_SHIFT) | ((uint32_t)lid << PAIR_LID_SHIFT) | lr;
        }
        const uint32_t f = atomicAdd(&C->n_fb, 1u);  // LDS hash full: the global path
        if (f >= Wk.max_fb) {
            atomicOr(&C->ovf, OVF_FB);
            return PAIR_DEAD;
        }
        const int64_t hx = table_insert(T, bkey, &C->ovf);
        if (hx < 0) return PAIR_DEAD;
        const uint32_t h = (uint32_t)hx;
        T.touched[h] = 1u;
        const uint32_t rk = atomicAdd(&T.cell[(size_t)h * T.cell_stride + t], cnt_in);
        Wk.fb[f] = make_uint4(h, t, rk, 0u);
        return PAIR_FB | (cnt_in << PAIR_CNT_SHIFT) | f;
    };
    // G = 1: the lanes stride the block's rays; G = 2: pass q covers rays [q NT, (q + 1) NT) of
    // the workgroup's 2 RPB, so the block (and its scan) is uniform in a pass
    constexpr int PASSES = G == 1 ? 1 : G * RPB / NT;
#pragma unroll 1
    for (int pass = 0; pass < PASSES; pass++) {
        const int g = G == 1 ? 0 : pass * NT / RPB;
        // selects, not array indexing: a dynamically indexed private array would live in scratch
        const uint32_t t = g ? tb[G - 1] : tb[0], r0 = g ? r0b[G - 1] : r0b[0];
        const uint32_t r1 = g ? r1b[G - 1] : r1b[0];
        const float ox = D.s[t].ox, oy = D.s[t].oy, oz = D.s[t].oz;
        const float* __restrict__ xs = scan_xyz(xyz, D, t, R);
        const uint32_t lo = G == 1 ? r0 + threadIdx.x : r0 + (uint32_t)(pass * NT) % RPB + threadIdx.x;
        const uint32_t hi = G == 1 ? r1 : min(r1, r0 + (uint32_t)(pass * NT) % RPB + NT);
        for (uint32_t i = lo; i < hi; i += NT) {
            uint32_t* pc = Wk.pair + (size_t)i * maxp;
            uint32_t k = 0;
            typename Walk<SEM>::State r;
            const bool ok = Walk<SEM>::init(R, D, t, i, xs[3 * (size_t)i], xs[3 * (size_t)i + 1],
                                            xs[3 * (size_t)i + 2], r);
            valid += ok ? 1u : 0u;
            const uint32_t sub = 2u * (uint32_t)g + (i - r0 >= (uint32_t)(RPB / 2) ? 1u : 0u);
            // One pair per distinct brick; a line visits a brick in one contiguous run of DDA
            // voxels, so a pair closes when the next gated voxel's brick differs.
            if (maxp <= 4) {
                // Short rays (no carving): the walk only records its <= 4 pairs in registers; all
                // lanes then emit pair j together, so the LDS hash work runs convergent, not once
                // per lane.
                uint64_t q0 = EMPTY_KEY, q1 = EMPTY_KEY, q2 = EMPTY_KEY, q3 = EMPTY_KEY;
                uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0, np = 0;
#ifdef TSDF_ABLATE_CNT_NOWALK
                if (ok && r.px == 1e30f) {
#else
                if (ok) {
#endif
                    // Branch-free walk (lanes are at different steps of different rays): the gate
                    // and the pair bookkeeping are selects on 32-bit brick codes; the 64-bit keys
                    // are built from the codes after the walk (code_key: a ray's bricks lie within
                    // one brick of its first one per axis).
                    const int bx0 = r.vx >> 3, by0 = r.vy >> 3, bz0 = r.vz >> 3;
                    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, curc = ~0u, ccount = 0;
                    auto walk = [&](auto chk) {
                        for (int it = 0; it < MAX_DDA_STEPS; it++) {
                            const bool gt = Walk<SEM>::gate_sel(R, ox, oy, oz, r, decltype(chk)::value);
                            const uint32_t bc = brick_code_of(r.vx, r.vy, r.vz);
                            const bool nb = gt && bc != curc;
                            const bool cl = nb && curc != ~0u;  // the previous pair closes
                            c0 = (cl && np == 0) ? curc : c0; n0 = (cl && np == 0) ? ccount : n0;
                            c1 = (cl && np == 1) ? curc : c1; n1 = (cl && np == 1) ? ccount : n1;
                            c2 = (cl && np == 2) ? curc : c2; n2 = (cl && np == 2) ? ccount : n2;
                            c3 = (cl && np == 3) ? curc : c3; n3 = (cl && np == 3) ? ccount : n3;
                            np += cl ? 1u : 0u;
                            curc = nb ? bc : curc;
                            ccount = (nb ? 0u : ccount) + (gt ? 1u : 0u);
                            if (!Walk<SEM>::step(r)) break;
                        }
                    };
                    // rays far from the index-domain edge (all, in practice) skip the per-voxel check
                    if (__all(Walk<SEM>::inside(R, r))) walk(std::false_type{});
                    else walk(std::true_type{});
                    if (curc != ~0u) {
                        c0 = np == 0 ? curc : c0; n0 = np == 0 ? ccount : n0;
                        c1 = np == 1 ? curc : c1; n1 = np == 1 ? ccount : n1;
                        c2 = np == 2 ? curc : c2; n2 = np == 2 ? ccount : n2;
                        c3 = np == 3 ? curc : c3; n3 = np == 3 ? ccount : n3;
                        np++;
                    }
                    if (np > 0) q0 = code_key(c0, bx0, by0, bz0);
                    if (np > 1) q1 = code_key(c1, bx0, by0, bz0);
                    if (np > 2) q2 = code_key(c2, bx0, by0, bz0);
                    if (np > 3) q3 = code_key(c3, bx0, by0, bz0);
                }
                CPH(1);  // point load + walk
                if (np > maxp) atomicOr(&C->ovf, OVF_PAIRS);  // beyond the geometric bound
                k = min(np, maxp);
                uint4 code = make_uint4(NO_PAIR, NO_PAIR, NO_PAIR, NO_PAIR);
                if (k > 0) code.x = pair_code(q0, n0, sub, t);
                if (k > 1) code.y = pair_code(q1, n1, sub, t);
                if (k > 2) code.z = pair_code(q2, n2, sub, t);
                if (k > 3) code.w = pair_code(q3, n3, sub, t);
                if (maxp == 4) {
                    *reinterpret_cast<uint4*>(pc) = code;  // one 16-B store per ray
                } else {
                    const uint32_t cv[4] = {code.x, code.y, code.z, code.w};
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++)
                        if (j < maxp) pc[j] = cv[j];
                }
            } else {
                if (ok) {
                    uint64_t cur = EMPTY_KEY;
                    uint32_t curc = ~0u, ccount = 0;
                    auto emit = [&](uint64_t bkey, uint32_t cnt_in) {
                        if (k >= maxp) {
                            atomicOr(&C->ovf, OVF_PAIRS);
                            return;
                        }
                        pc[k++] = pair_code(bkey, cnt_in, sub, t);
                    };
                    for (int it = 0; it < MAX_DDA_STEPS; it++) {
                        if (Walk<SEM>::gate(R, ox, oy, oz, r)) {
                            const uint32_t bc = brick_code_of(r.vx, r.vy, r.vz);
                            if (bc != curc) {
                                if (cur != EMPTY_KEY) emit(cur, ccount);
                                cur = brick_key_of(r.vx, r.vy, r.vz);
                                curc = bc;
                                ccount = 0;
                            }
                            ccount++;
                        }
                        if (!Walk<SEM>::step(r)) break;
                    }
                    if (cur != EMPTY_KEY) emit(cur, ccount);
                }
                for (uint32_t j = k; j < maxp; j++) pc[j] = NO_PAIR;
            }
            npairs += k;
            CPH(2);  // pair emission (LDS hash) + pair-code store
        }
    }
    __syncthreads();
    CPH(3);  // the block's slowest wave
    // one global find-or-insert + one atomic per distinct brick of the workgroup: the cell
    // (brick, scan) count reserves the workgroup's ranks; `touched` (a plain store) lists the brick
    // for k_compact, which also derives the brick's total from its cells.  Each thread takes
    // HCAP / NT consecutive slots; a block scan over their sample and run counts gives every
    // sub-run its offset in its (block, half)'s sample order (k_place stages the samples in that
    // order) and its index in the (block, half)'s DENSE run list (slot order = sample order).
    constexpr int SPT = HCAP / NT;
    static_assert(SPT >= 1, "LDS hash slots per thread");
    // The thread's SPT slots go to the global table in three batched stages, so their round trips
    // overlap instead of running one slot after another: (1) first-probe loads of all keys, issued
    // before the block scan so that their round trip overlaps it, (2) resolve (a hit needs nothing
    // more; an empty or taken first slot takes the probing path), (3) the cell atomics of all
    // found bricks, in flight while the run-start bitmap is built.
    // (only the loads are kept across the scan; keys, hashes and scans are re-derived after it)
    uint64_t key[SPT], k0[SPT];
    uint32_t ts[SPT];
    auto slot_key = [&](int j) {
        const uint64_t lk = s_key[threadIdx.x * SPT + j];
        const bool g1 = split && lk != EMPTY_KEY && (lk & KEY_G1);
        key[j] = g1 ? lk & ~KEY_G1 : lk;
        ts[j] = g1 ? tb[G - 1] : tb[0];
    };
    if constexpr (!SPLIT) {
#pragma unroll
        for (int j = 0; j < SPT; j++) {
            slot_key(j);
            k0[j] = key[j] != EMPTY_KEY ? T.keys[mix64(key[j]) & T.mask] : EMPTY_KEY;
        }
    }
    // one dense run list per (block, half): k_place workgroup 2 b + half
    uint32_t ns[NSUB], cc[G];
#pragma unroll
    for (int s = 0; s < NSUB; s++) ns[s] = 0u;
#pragma unroll
    for (int g = 0; g < G; g++) cc[g] = 0u;
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        const int slot = threadIdx.x * SPT + j;
        const CntT c = s_key[slot] != EMPTY_KEY ? s_cnt[slot] : (CntT)0;
#pragma unroll
        for (int s = 0; s < NSUB; s++) {
            const uint32_t n = (uint32_t)(c >> (16 * s)) & 0xFFFFu;
            ns[s] += n;
            cc[s >> 1] += (n ? 1u : 0u) << (16 * (s & 1));
        }
    }
    uint32_t nsl = 0, rbase = 0;  // SPLIT: the thread's distinct bricks, their first record
    if constexpr (SPLIT) {
#pragma unroll
        for (int j = 0; j < SPT; j++) nsl += s_key[threadIdx.x * SPT + j] != EMPTY_KEY ? 1u : 0u;
    }
    uint32_t off[NSUB], idx[NSUB];
    {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        const uint32_t isl = SPLIT ? wave_incl_scan(nsl) : 0u;
        if (SPLIT && lane == 63) s_wsl[wid] = isl;
        uint32_t in[NSUB], ic[G];
#pragma unroll
        for (int s = 0; s < NSUB; s++) in[s] = wave_incl_scan(ns[s]);
#pragma unroll
        for (int g = 0; g < G; g++) ic[g] = wave_incl_scan(cc[g]);
        if (lane == 63) {
#pragma unroll
            for (int g = 0; g < G; g++) {
                s_wsum[g][wid] = (unsigned long long)in[2 * g] | ((unsigned long long)in[2 * g + 1] << 32);
                s_wcnt[g][wid] = ic[g];
            }
        }
        __syncthreads();
        if constexpr (SPLIT) {
            uint32_t ex = 0, tot = 0;
            for (int w = 0; w < NT / 64; w++) {
                ex += w < wid ? s_wsl[w] : 0u;
                tot += s_wsl[w];
            }
            rbase = ex + isl - nsl;
            if (threadIdx.x == NT - 1) Wk.rsv_n[bx] = tot;
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            unsigned long long ex = 0, tot = 0;
            uint32_t exc = 0, totc = 0;
            for (int w = 0; w < NT / 64; w++) {
                ex += w < wid ? s_wsum[g][w] : 0ull;
                exc += w < wid ? s_wcnt[g][w] : 0u;
                tot += s_wsum[g][w];
                totc += s_wcnt[g][w];
            }
            off[2 * g] = (uint32_t)ex + (in[2 * g] - ns[2 * g]);
            off[2 * g + 1] = (uint32_t)(ex >> 32) + (in[2 * g + 1] - ns[2 * g + 1]);
            idx[2 * g] = (exc & 0xFFFFu) + ((ic[g] - cc[g]) & 0xFFFFu);
            idx[2 * g + 1] = (exc >> 16) + ((ic[g] - cc[g]) >> 16);
            if (threadIdx.x == NT - 1) {
                const uint32_t b = G * bx + g;
                Wk.blk_n[2 * b] = totc & 0xFFFFu;
                Wk.blk_n[2 * b + 1] = totc >> 16;
                // each half's staged sample count: its samples, up to the staging capacity
                Wk.plan[(size_t)(2 * b) * PLAN_STRIDE + PLAN_STRIDE - 1] =
                    min((uint32_t)tot, (uint32_t)PCAP);
                Wk.plan[(size_t)(2 * b + 1) * PLAN_STRIDE + PLAN_STRIDE - 1] =
                    min((uint32_t)(tot >> 32), (uint32_t)PCAP);
            }
        }
    }
    CPH(4);  // block scan
    if constexpr (SPLIT) {
        // one record per distinct brick for k_resolve, which fills the runs' (table index, cell
        // rank); this kernel writes the runs' (offset, samples | slot) and the run-start bits
        static_assert(G == 1 && HCAP <= 2048 && MAX_BATCH <= 1024, "record packing");
        uint32_t r = rbase;
#pragma unroll
        for (int j = 0; j < SPT; j++) {
            const int slot = threadIdx.x * SPT + j;
            slot_key(j);
            if (key[j] == EMPTY_KEY) continue;
            const uint32_t c = (uint32_t)s_cnt[slot], n0 = c & 0xFFFFu, n1 = c >> 16;
            uint32_t w = ts[j] << 22;
            uint4* bt = Wk.blk + (size_t)(2 * bx) * HCAP;
            if (n0) {
                reinterpret_cast<uint2*>(bt + idx[0])[1] = make_uint2(off[0], n0 | ((uint32_t)slot << 16));
                if (off[0] < (uint32_t)PCAP) atomicOr(&s_bm[0][off[0] >> 5], 1u << (off[0] & 31));
                w |= idx[0]++;
                off[0] += n0;
            }
            if (n1) {
                reinterpret_cast<uint2*>(bt + HCAP + idx[NSUB - 1])[1] =
                    make_uint2(off[NSUB - 1], n1 | ((uint32_t)slot << 16));
                if (off[NSUB - 1] < (uint32_t)PCAP)
                    atomicOr(&s_bm[NSUB - 1][off[NSUB - 1] >> 5], 1u << (off[NSUB - 1] & 31));
                w |= idx[NSUB - 1]++ << 11;
                off[NSUB - 1] += n1;
            }
            Wk.rsv[(size_t)bx * HCAP + r++] = make_uint4((uint32_t)key[j], (uint32_t)(key[j] >> 32), c, w);
        }
    } else {
    int64_t hx[SPT];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        slot_key(j);
        hx[j] = -1;
        if (key[j] != EMPTY_KEY)
            hx[j] = k0[j] == key[j] ? (int64_t)(mix64(key[j]) & T.mask) : table_insert(T, key[j], &C->ovf);
    }
    CPH(5);  // first probes + inserts
    uint32_t old[SPT];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        const int slot = threadIdx.x * SPT + j;
        const CntT c = s_cnt[slot];
        uint32_t tot = 0;
#pragma unroll
        for (int s = 0; s < NSUB; s++) tot += (uint32_t)(c >> (16 * s)) & 0xFFFFu;
#ifndef TSDF_ABLATE_CNT_NORET
        old[j] = hx[j] >= 0 ? atomicAdd(&T.cell[(size_t)hx[j] * T.cell_stride + ts[j]], tot) : 0u;
#else  // diagnostic: the cell atomics not waited for (every run ranked 0: wrong, in-bounds)
        if (hx[j] >= 0) atomicAdd(&T.cell[(size_t)hx[j] * T.cell_stride + ts[j]], tot);
        old[j] = 0u;
#endif
    }
    // dense run lists: (table index | NO_PAIR, rank in the (brick, scan) cell, run offset in the
    // sub-run's sample order, run samples | slot << 16); in the cell the sub-runs follow each
    // other in (block, half) order
    static_assert((RPB / 2) * MAX_IN_BRICK < (1 << 16) && HCAP <= (1 << 16), "run record packing");
    // the run-start bits need only the offsets: set them while the atomics are in flight
    uint32_t boff[NSUB];
#pragma unroll
    for (int s = 0; s < NSUB; s++) boff[s] = off[s];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        const int slot = threadIdx.x * SPT + j;
        if (key[j] == EMPTY_KEY) continue;
        const CntT c = s_cnt[slot];
#pragma unroll
        for (int s = 0; s < NSUB; s++) {
            const uint32_t n = (uint32_t)(c >> (16 * s)) & 0xFFFFu;
            if (n) {
                if (boff[s] < (uint32_t)PCAP) atomicOr(&s_bm[s][boff[s] >> 5], 1u << (boff[s] & 31));
                boff[s] += n;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        const int slot = threadIdx.x * SPT + j;
        if (key[j] == EMPTY_KEY) continue;
        const CntT c = s_cnt[slot];
        uint32_t tx = NO_PAIR, rk = 0u;
        if (hx[j] >= 0) {
            tx = (uint32_t)hx[j];
            rk = old[j];
            // the brick's first run of this scan marks it (one store per (brick, scan), not one
            // per (workgroup, brick): partial-line stores from every XCD cost HBM writes)
            if (old[j] == 0u) T.touched[tx] = 1u;
        }
#pragma unroll
        for (int s = 0; s < NSUB; s++) {
            const uint32_t n = (uint32_t)(c >> (16 * s)) & 0xFFFFu;
            if (n) {
                uint4* bt = Wk.blk + (size_t)(2 * (G * bx + (s >> 1)) + (s & 1)) * HCAP;
                bt[idx[s]++] = make_uint4(tx, rk, off[s], n | ((uint32_t)slot << 16));
                off[s] += n;
                rk += n;
            }
        }
    }
    }  // !SPLIT
    CPH(6);  // cell atomics + run lists
    // k_place's staging plan for each (block, half): the run-start bitmap and its exclusive
    // popcount prefix per word (wave s writes sub-run list s's)
    __syncthreads();
    CPH(7);
    {
        const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        static_assert(NT / 64 >= NSUB, "one wave per sub-run list");
        if (wv < NSUB) {
            // WPL consecutive bitmap words per lane; the prefix is one u16 per word
            constexpr int WPL = (PW + 63) / 64;
            static_assert(WPL >= 1 && WPL <= 4, "bitmap words per lane");
            uint32_t* pl = Wk.plan + (size_t)(2 * (G * bx + (wv >> 1)) + (wv & 1)) * PLAN_STRIDE;
            uint16_t* pp = reinterpret_cast<uint16_t*>(pl + PW);
            uint32_t b[WPL], cs = 0;
#pragma unroll
            for (int q = 0; q < WPL; q++) {
                const int wd = WPL * ln + q;
                b[q] = wd < PW ? s_bm[wv][wd] : 0u;
                cs += (uint32_t)__popc(b[q]);
            }
            uint32_t pre = wave_incl_scan(cs) - cs;
#pragma unroll
            for (int q = 0; q < WPL; q++) {
                const int wd = WPL * ln + q;
                if (wd < PW) {
                    pl[wd] = b[q];
                    pp[wd] = (uint16_t)pre;
                }
                pre += (uint32_t)__popc(b[q]);
            }
        }
    }
    // block-reduce the stats, one atomic per block on a shard picked by block index
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long v = wave_sum<unsigned long long>(valid);
    unsigned long long q = wave_sum<unsigned long long>(npairs);
    if (lane == 0) { red[0][wid] = v; red[1][wid] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        v = 0;
        q = 0;
        for (int w = 0; w < NT / 64; w++) { v += red[0][w]; q += red[1][w]; }
        if (v) atomicAdd(&C->n_rays[blockIdx.x & 7], v);  // -> G->tot_rays at k_finish
        if (q) atomicAdd(&C->n_pairs[blockIdx.x & 7], q);
    }
#ifdef TSDF_CNT_PHASE
    CPH(8);  // plan + stats
    if (threadIdx.x == 0 && blockIdx.x % 61 == 0 && NT == CNT_THREADS * G)
        printf("cntphase %u init %llu walk %llu emit %llu bar %llu scan %llu probe %llu atom %llu "
               "bar2 %llu tail %llu\n", blockIdx.x, cph[0], cph[1], cph[2], cph[3], cph[4], cph[5],
               cph[6], cph[7], cph[8]);
#endif
}

#ifdef TSDF_CNT_SPLIT
// k_resolve (TSDF_CNT_SPLIT variant): k_count's global phase as its own launch, so the LDS-bound
// k_count workgroups do not hold their LDS through the find-or-insert and cell-atomic round trips.
// One workgroup per k_count block, one lane per distinct brick of the block's LDS hash: find or
// insert the brick, reserve its samples in the (brick, scan) cell, and write the (table index,
// cell rank) half of the block's run records.
constexpr int RSV_THREADS = 256;
__global__ __launch_bounds__(RSV_THREADS) void k_resolve(BatchRef D, RayConst R, Table T, Work Wk,
                                                        Globals* G, int parity) {
    Counters* C = &G->ctr[parity];
    uint32_t b = blockIdx.x;
    if (R.sec_on) {
        if (blockIdx.x >= C->n_act) return;
        b = Wk.act[blockIdx.x];
    }
    if (b >= D.n_blocks) return;
    const uint32_t n = Wk.rsv_n[b];
    const uint4* rec = Wk.rsv + (size_t)b * HCAP;
    uint4* bt = Wk.blk + (size_t)(2 * b) * HCAP;
    for (uint32_t i = threadIdx.x; i < n; i += RSV_THREADS) {
        const uint4 q = rec[i];
        const uint64_t key = (uint64_t)q.x | ((uint64_t)q.y << 32);
        const uint32_t n0 = q.z & 0xFFFFu, n1 = q.z >> 16, t = q.w >> 22;
        const uint64_t h0 = mix64(key) & T.mask;
        const int64_t hx = T.keys[h0] == key ? (int64_t)h0 : table_insert(T, key, &C->ovf);
        uint32_t tx = NO_PAIR, rk = 0u;
        if (hx >= 0) {
            tx = (uint32_t)hx;
            rk = atomicAdd(&T.cell[(size_t)hx * T.cell_stride + t], n0 + n1);
            if (rk == 0u) T.touched[tx] = 1u;
        }
        if (n0) reinterpret_cast<uint2*>(bt + (q.w & 2047u))[0] = make_uint2(tx, rk);
        if (n1) reinterpret_cast<uint2*>(bt + HCAP + ((q.w >> 11) & 2047u))[0] = make_uint2(tx, rk + n0);
    }
}
#endif

// ------------------------------------------------------------------------------------------------
// k_sector_flags (sector sharding only): one wave per k_count block of RPB rays, 16 points per lane,
// a wave vote; no LDS, so the pass runs at full occupancy and the walk kernels' blocks of other
// sectors cost one byte load each instead of their point reads and LDS set-up.
constexpr int FLG_THREADS = 256;
__global__ __launch_bounds__(FLG_THREADS) void k_sector_flags(const float* __restrict__ xyz,
                                                             BatchRef D, RayConst R, Work Wk,
                                                             Globals* G, int parity) {
    const uint32_t b = blockIdx.x * (FLG_THREADS / 64) + (threadIdx.x >> 6);
    if (b >= D.n_blocks) return;  // wave-uniform
    uint32_t t, r0, r1;
    block_range(D, b, t, r0, r1);
    const float ox = D.s[t].ox, oy = D.s[t].oy;
    const float* __restrict__ xs = scan_xyz(xyz, D, t, R);
    bool any = false;
    for (uint32_t i = r0 + (threadIdx.x & 63); i < r1; i += 64)
        any |= in_sector(R, xs[3 * (size_t)i] - ox, xs[3 * (size_t)i + 1] - oy);
    const bool v = __any(any);
    // the block joins the walk kernels' list (order is immaterial: blocks are independent)
    if ((threadIdx.x & 63) == 0 && v) Wk.act[atomicAdd(&G->ctr[parity].n_act, 1u)] = b;
}

hipError_t launch_sector_flags(const float* d_xyz, const BatchRef& D, const RayConst& R,
                               const Work& Wk, Globals* G, int parity, hipStream_t st) {
    const uint32_t per = FLG_THREADS / 64;
    k_sector_flags<<<(D.n_blocks + per - 1) / per, FLG_THREADS, 0, st>>>(d_xyz, D, R, Wk, G,
                                                                        parity);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Size order: k_integrate hands its workgroups bricks in list order (grid stride), and bricks hold
// from a few to ~40 k samples, so a random order leaves the kernel waiting on the workgroups that
// drew several large bricks.  A counting sort by size class (floor(log2(samples)), largest class
// first) deals the large bricks out first and evenly (greedy largest-first).  Order inside a class
// is whatever the atomics give: each brick is fused independently, so the field does not depend
// on it.  k_compact builds the sorted list as it writes the records: k_compact_sum counts the
// (table slice, size class) histogram, k_compact_scan turns it into first positions, and
// k_compact_write ranks each record in its (slice, class) with one global atomic (a separate
// three-launch k_order remains for the ablation build TSDF_SEPARATE_ORDER).

constexpr int ORD_THREADS = 256;
constexpr int ORD_BLOCKS = 64;  // slices: of the active list (k_order), of the table's chunks (k_compact)
constexpr int ORD_CLASSES = 32;

__device__ __forceinline__ uint32_t size_class(uint32_t n) {
    return (uint32_t)__clz(max(n, 1u));  // 31 - floor(log2 n): large bricks -> small index
}
// the slice of table chunk c of nch (k_compact's size order)
__device__ __forceinline__ uint32_t ord_chunk_slice(uint32_t c, uint32_t nch) {
    return (uint32_t)(((uint64_t)c * ORD_BLOCKS) / nch);
}

// ------------------------------------------------------------------------------------------------
// k_compact: per active brick — record segment, new pool slot, per-scan cell prefix

constexpr int CMP_THREADS = 256;
constexpr int CMP_PER = CMP_CHUNK / CMP_THREADS;  // table entries per thread
constexpr int CMP_GROUP = 16;  // lanes per touched brick: one uint4 of its cell row each per 64 scans
constexpr int CMP_SCAN_THREADS = 1024;

template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w, uint32_t* total) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t v = wave_incl_scan(x);
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const uint32_t r = s_w[k];
        off += k < wid ? r : 0u;
        tot += r;
    }
    *total = tot;
    __syncthreads();  // s_w reusable
    return v - x + off;
}

// k_compact gives every brick touched by the batch its sample segment (a global prefix over the
// bricks), a pool slot if new and an active record, and rewrites its per-scan cells as absolute
// sample positions.  The global prefix is taken over table chunks in three launches, without any
// atomic (a counter shared by thousands of workgroups serializes at ~11 ns per add):
//   k_compact_sum    per chunk of CMP_CHUNK table entries: touched bricks, their samples (16 lanes
//                    per brick read its cell row, one uint4 each) and new bricks -> cagg[chunk];
//   k_compact_scan   one workgroup: exclusive prefix of the chunk totals -> cagg[nch + chunk], the
//                    batch's counters and the pool count;
//   k_compact_write  per chunk again: records, slots and the rewritten cell rows.
// The chunk's touched bricks, listed in LDS in table order (<= CMP_CHUNK of them).
__device__ __forceinline__ uint32_t compact_list(const Table& T, uint32_t chunk, uint32_t* s_h,
                                                 uint32_t* s_w, bool clear) {
    uint32_t hit[CMP_PER], cnt = 0;
#pragma unroll
    for (int j = 0; j < CMP_PER; j++) {  // thread-consecutive entries keep the list in table order
        const uint32_t h = chunk + threadIdx.x * CMP_PER + j;
        hit[j] = h <= T.mask && T.touched[h] != 0u ? 1u : 0u;
        cnt += hit[j];
    }
    uint32_t nh;
    uint32_t e = block_excl_scan<CMP_THREADS>(cnt, s_w, &nh);
#pragma unroll
    for (int j = 0; j < CMP_PER; j++) {
        if (hit[j]) {
            const uint32_t h = chunk + threadIdx.x * CMP_PER + j;
            s_h[e++] = h;
            if (clear) T.touched[h] = 0u;
        }
    }
    __syncthreads();
    return nh;
}

// A brick's cell row as uint4 groups, and the group's count (fused: u64 cells, two per group, the
// span counts in the high words; the row runs to the totals cell at n_scans).
template <bool FUSED>
__device__ __forceinline__ uint32_t row_groups(uint32_t n_scans) {
    return FUSED ? (n_scans + 2) / 2 : (n_scans + 3) / 4;
}
template <bool FUSED>
__device__ __forceinline__ uint32_t group_count(const uint4& v) {
    return FUSED ? v.y + v.w : v.x + v.y + v.z + v.w;
}
template <bool FUSED>
__device__ __forceinline__ const uint4* cell_row(const Table& T, uint32_t h) {
    return FUSED ? reinterpret_cast<const uint4*>(reinterpret_cast<const uint64_t*>(T.cell) +
                                                  (size_t)h * T.cell_stride)
                 : reinterpret_cast<const uint4*>(T.cell + (size_t)h * T.cell_stride);
}

template <bool FUSED>
__global__ __launch_bounds__(CMP_THREADS) void k_compact_sum(uint32_t n_scans, Table T, Work Wk) {
    __shared__ uint32_t s_w[CMP_THREADS / 64];
    __shared__ uint32_t s_h[CMP_CHUNK];
    __shared__ uint32_t s_acc[2];  // samples, new bricks
    if (threadIdx.x == 0) {
        s_acc[0] = 0u;
        s_acc[1] = 0u;
    }
#ifndef TSDF_SEPARATE_ORDER
    __shared__ uint32_t s_cls[ORD_CLASSES];  // the chunk's bricks per size class
    if (threadIdx.x < ORD_CLASSES) s_cls[threadIdx.x] = 0u;
#endif
    const uint32_t nh = compact_list(T, blockIdx.x * CMP_CHUNK, s_h, s_w, false);
    const uint32_t nq = row_groups<FUSED>(n_scans);  // whole uint4 groups (see cell_stride)
    const uint32_t grp = threadIdx.x / CMP_GROUP, li = threadIdx.x % CMP_GROUP;
    uint32_t samples = 0, nnew = 0;  // fused: spans
    for (uint32_t k = grp; k < nh; k += CMP_THREADS / CMP_GROUP) {
        const uint32_t h = s_h[k];
        const uint4* cp = cell_row<FUSED>(T, h);
        uint32_t sum = 0;
        for (uint32_t q = li; q < nq; q += CMP_GROUP) sum += group_count<FUSED>(cp[q]);
        samples += sum;
#ifndef TSDF_SEPARATE_ORDER
#pragma unroll
        for (int d = CMP_GROUP / 2; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, CMP_GROUP);
        if (li == 0) atomicAdd(&s_cls[size_class(sum)], 1u);
#endif
        if (li == 0 && T.slots[h] == UNASSIGNED) nnew++;
    }
    samples = wave_sum<uint32_t>(samples);
    nnew = wave_sum<uint32_t>(nnew);
    if ((threadIdx.x & 63) == 0) {
        if (samples) atomicAdd(&s_acc[0], samples);
        if (nnew) atomicAdd(&s_acc[1], nnew);
    }
    __syncthreads();
    if (threadIdx.x == 0) Wk.cagg[blockIdx.x] = make_uint4(nh, s_acc[0], s_acc[1], 0u);
#ifndef TSDF_SEPARATE_ORDER
    // the chunk's slice histogram (zeroed again by k_compact_scan once read)
    if (threadIdx.x < ORD_CLASSES && s_cls[threadIdx.x])
        atomicAdd(&Wk.ord_hist[ord_chunk_slice(blockIdx.x, gridDim.x) * ORD_CLASSES + threadIdx.x],
                  s_cls[threadIdx.x]);
#endif
}

__global__ __launch_bounds__(CMP_SCAN_THREADS) void k_compact_scan(uint32_t nch, Work Wk,
                                                                   Globals* G, int parity,
                                                                   int fused) {
    __shared__ uint32_t s_w[3][CMP_SCAN_THREADS / 64];
    __shared__ uint32_t s_carry[3];
    Counters* C = &G->ctr[parity];
    if (threadIdx.x == 0) {
        s_carry[0] = 0u;
        s_carry[1] = 0u;
        s_carry[2] = G->pool_count;
    }
    __syncthreads();
    // the three prefixes (touched bricks, samples, new bricks) in one pass: thread t takes the
    // chunks [t P, t P + P) (all loads issued at once), per-wave DPP scans of the threads' totals,
    // the waves' totals through LDS
    constexpr int NWS = CMP_SCAN_THREADS / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t P = (nch + CMP_SCAN_THREADS - 1) / CMP_SCAN_THREADS;
    const uint32_t c0 = threadIdx.x * P;
    uint32_t sa = 0, sc = 0, sn = 0;
#pragma unroll 4
    for (uint32_t q = 0; q < P; q++) {
        const uint4 a = c0 + q < nch ? Wk.cagg[c0 + q] : make_uint4(0u, 0u, 0u, 0u);
        sa += a.x;
        sc += a.y;
        sn += a.z;
    }
    const uint32_t ia = wave_incl_scan(sa), ic = wave_incl_scan(sc), in = wave_incl_scan(sn);
    if (lane == 63) {
        s_w[0][wid] = ia;
        s_w[1][wid] = ic;
        s_w[2][wid] = in;
    }
    __syncthreads();
    uint32_t oa = s_carry[0], oc = s_carry[1], on = s_carry[2], ta = 0, tc = 0, tn = 0;
#pragma unroll
    for (int k = 0; k < NWS; k++) {
        const uint32_t xa = s_w[0][k], xc = s_w[1][k], xn = s_w[2][k];
        oa += k < wid ? xa : 0u;
        oc += k < wid ? xc : 0u;
        on += k < wid ? xn : 0u;
        ta += xa;
        tc += xc;
        tn += xn;
    }
    oa += ia - sa;
    oc += ic - sc;
    on += in - sn;
    for (uint32_t q = 0; q < P && c0 + q < nch; q++) {  // re-read: L2-resident, and no registers held
        const uint4 a = Wk.cagg[c0 + q];
        Wk.cagg[nch + c0 + q] = make_uint4(oa, oc, on, 0u);
        oa += a.x;
        oc += a.y;
        on += a.z;
    }
    if (threadIdx.x == 0) {
        s_carry[0] += ta;
        s_carry[1] += tc;
        s_carry[2] += tn;
    }
    __syncthreads();
#ifndef TSDF_SEPARATE_ORDER
    // size order: (slice, class) first positions = the records of larger classes + class k's
    // records in the slices before (k_order_scan's rule); the histogram is zeroed for the next
    // batch.  Wave w takes classes w and w + 16 with lane = slice (ORD_BLOCKS = 64): one DPP scan
    // per class gives the slices' prefix, wave 0 the classes' bases.
    static_assert(ORD_BLOCKS == 64 && ORD_CLASSES == 32 && CMP_SCAN_THREADS == 1024, "layout");
    {
        __shared__ uint32_t s_tot[ORD_CLASSES], s_cbase[ORD_CLASSES];
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t v[2], ex[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int cls = w + 16 * q;
            v[q] = Wk.ord_hist[lane * ORD_CLASSES + cls];
            const uint32_t incl = wave_incl_scan(v[q]);
            ex[q] = incl - v[q];
            if (lane == 63) s_tot[cls] = incl;
            Wk.ord_hist[lane * ORD_CLASSES + cls] = 0u;
        }
        __syncthreads();
        if (w == 0) {
            const uint32_t t = lane < ORD_CLASSES ? s_tot[lane] : 0u;
            const uint32_t incl = wave_incl_scan(t);
            if (lane < ORD_CLASSES) s_cbase[lane] = incl - t;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int cls = w + 16 * q;
            Wk.ord_hist[ORD_BLOCKS * ORD_CLASSES + lane * ORD_CLASSES + cls] = s_cbase[cls] + ex[q];
        }
    }
#endif
    if (threadIdx.x == 0) {
        C->n_active = s_carry[0];
        C->cursor = s_carry[1];
        C->n_new = s_carry[2] - G->pool_count;
        G->pool_count = s_carry[2];
        if (fused ? s_carry[1] > Wk.max_spn : s_carry[1] > Wk.max_smp)
            atomicOr(&C->ovf, fused ? OVF_SPN : OVF_SMP);
        if (s_carry[0] > Wk.max_active) atomicOr(&C->ovf, OVF_ACTIVE);
    }
}

template <bool FUSED>
__global__ __launch_bounds__(CMP_THREADS) void k_compact_write(uint32_t n_scans, uint32_t nch,
                                                               Table T, Work Wk, Globals* G,
                                                               int parity) {
    __shared__ uint32_t s_w[CMP_THREADS / 64];
    __shared__ uint32_t s_h[CMP_CHUNK];
    __shared__ uint32_t s_n[CMP_CHUNK];  // the bricks' samples, then their segment starts
    const uint32_t chunk = blockIdx.x * CMP_CHUNK;
    const uint32_t nh = compact_list(T, chunk, s_h, s_w, true);
    if (nh == 0) return;  // uniform
    const uint32_t nq = row_groups<FUSED>(n_scans);
    const uint32_t grp = threadIdx.x / CMP_GROUP, li = threadIdx.x % CMP_GROUP;
    for (uint32_t k = grp; k < nh; k += CMP_THREADS / CMP_GROUP) {
        const uint4* cp = cell_row<FUSED>(T, s_h[k]);
        uint32_t sum = 0;  // fused: spans
        for (uint32_t q = li; q < nq; q += CMP_GROUP) sum += group_count<FUSED>(cp[q]);
#pragma unroll
        for (int d = CMP_GROUP / 2; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, CMP_GROUP);
        if (li == 0) s_n[k] = sum;
    }
    __syncthreads();
    const uint4 base = Wk.cagg[nch + blockIdx.x];  // (active, sample, pool) bases of the chunk
    // per brick, in table order: CMP_PER consecutive bricks per thread
    uint32_t n[CMP_PER], isnew[CMP_PER], sn = 0, snew = 0;
#pragma unroll
    for (int j = 0; j < CMP_PER; j++) {
        const uint32_t k = threadIdx.x * CMP_PER + j;
        n[j] = k < nh ? s_n[k] : 0u;
        isnew[j] = k < nh && T.slots[s_h[k]] == UNASSIGNED ? 1u : 0u;
        sn += n[j];
        snew += isnew[j];
    }
    uint32_t tc, tn;
    uint32_t ec = block_excl_scan<CMP_THREADS>(sn, s_w, &tc);
    uint32_t en = block_excl_scan<CMP_THREADS>(snew, s_w, &tn);
#pragma unroll
    for (int j = 0; j < CMP_PER; j++) {
        const uint32_t k = threadIdx.x * CMP_PER + j;
        if (k < nh) {
            const uint32_t h = s_h[k];
            uint32_t slot = isnew[j] ? base.z + en : T.slots[h];
            if (isnew[j]) {
                if (slot < T.max_bricks) {
                    T.brick_keys[slot] = T.keys[h];
                } else {
                    slot = INVALID_SLOT;
                    atomicOr(&G->ctr[parity].ovf, OVF_POOL);
                }
                T.slots[h] = slot;
            }
            // k_integrate's whole per-brick header in one record
            const uint4 rec = make_uint4(h, slot, base.y + ec, n[j]);
            if (base.x + k < Wk.max_active) Wk.active[base.x + k] = rec;
#ifndef TSDF_SEPARATE_ORDER
            const uint32_t op = atomicAdd(&Wk.ord_hist[ORD_BLOCKS * ORD_CLASSES +
                                                       ord_chunk_slice(blockIdx.x, gridDim.x) * ORD_CLASSES +
                                                       size_class(n[j])], 1u);
            if (op < Wk.max_active) Wk.active_ord[op] = rec;
#endif
            s_n[k] = base.y + ec;
        }
        ec += n[j];
        en += isnew[j];
    }
    __syncthreads();
    if constexpr (FUSED) {
        // the per-scan cells become (sample prefix relative to the brick | absolute span position):
        // the totals cell at n_scans (zero until now) receives (samples | span end), and k_spans
        // finds a run's span position with one gather
        for (uint32_t k = grp; k < nh; k += CMP_THREADS / CMP_GROUP) {
            uint4* cp = const_cast<uint4*>(cell_row<true>(T, s_h[k]));
            uint32_t cs = 0, cp_ = s_n[k];
            for (uint32_t q0 = 0; q0 < nq; q0 += CMP_GROUP) {
                const uint32_t q = q0 + li;
                uint4 v = q < nq ? cp[q] : make_uint4(0u, 0u, 0u, 0u);
                const uint32_t s2 = v.x + v.z, p2 = v.y + v.w;
                static_assert(CMP_GROUP == 16, "a cell row pass is one 16-lane DPP row");
                const uint32_t is = row16_incl_scan(s2), ip = row16_incl_scan(p2);
                const uint32_t ps = cs + is - s2, pp = cp_ + ip - p2;
                v = make_uint4(ps, pp, ps + v.x, pp + v.y);
                if (q < nq) cp[q] = v;
                cs += __shfl(is, CMP_GROUP - 1, CMP_GROUP);
                cp_ += __shfl(ip, CMP_GROUP - 1, CMP_GROUP);
            }
        }
        return;
    }
    // the per-scan cells become absolute sample positions: segment start + exclusive prefix
    // (k_place then finds a run's position with one gather)
    for (uint32_t k = grp; k < nh; k += CMP_THREADS / CMP_GROUP) {
        uint4* cp = reinterpret_cast<uint4*>(T.cell + (size_t)s_h[k] * T.cell_stride);
        uint32_t carry = s_n[k];
        for (uint32_t q0 = 0; q0 < nq; q0 += CMP_GROUP) {  // 64 scans per pass, carried
            const uint32_t q = q0 + li;
            uint4 v = q < nq ? cp[q] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t s4 = v.x + v.y + v.z + v.w;
            static_assert(CMP_GROUP == 16, "a cell row pass is one 16-lane DPP row");
            const uint32_t incl = row16_incl_scan(s4);
            uint32_t p = carry + incl - s4;
            const uint32_t x0 = v.x, x1 = v.y, x2 = v.z;
            v.x = p; p += x0;
            v.y = p; p += x1;
            v.z = p; p += x2;
            v.w = p;
            if (q < nq) cp[q] = v;
            carry += __shfl(incl, CMP_GROUP - 1, CMP_GROUP);  // the pass's row total
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_place: every ray walks its DDA once more (one lane per ray, the same ray ranges as k_count's
// workgroups) and produces each gated sample (truncated sdf, local voxel) for its brick's segment:
// segment start + (brick, scan) cell prefix + the workgroup's run base + the pair's local offset.
// Samples are therefore per-brick contiguous and scan-ordered.  Scattered 8-byte stores cost ~4x
// their bytes in HBM writes, so the workgroup stages its samples in LDS in run order (run offsets
// from k_count's block scan) and then copies each (brick) run out as one contiguous write; samples
// past the staging capacity, and fallback pairs, are stored directly.

#ifdef TSDF_ABLATE_PHASE  // `make ablate ABLATE=PHASE`
#define TSDF_PLC_PHASE
#endif
constexpr int PLC_THREADS = RPB / 2;  // one ray per lane, half a k_count workgroup's rays

template <int SEM>
__global__ __launch_bounds__(PLC_THREADS, SEM == 2 ? TSDF_F64_PLACE_WAVES : 1) void k_place(const float* __restrict__ xyz, BatchRef D,
                                                      RayConst R, Table T, Work Wk,
                                                      const Globals* __restrict__ G, int parity) {
    // staging capacity (tsdf_device.h plan_cap: Voxblox 1/z^2 stages more, at 8 B a sample);
    // samples past it are stored directly
    constexpr int STG = plan_cap(SEM), PW = plan_words(SEM);  // k_count<SEM> plans as much
    __shared__ uint32_t s_base[HCAP];      // run -> first sample of the run in the brick segment
    __shared__ uint16_t s_loff[HCAP];      // run -> offset in the workgroup's sample order
    __shared__ uint16_t s_ord[HCAP];       // staged runs in staging order
    __shared__ uint32_t s_bits[PW]; // staging positions where a run starts
    __shared__ uint16_t s_wpre[(PW + 1) & ~1]; // run starts in the words before
    __shared__ float st_s[STG];      // staged samples
    // the staged sample's voxel; Voxblox 1/z^2 (sem 3): | its ray (lane) << 9, whose 1/z^2 weight
    // s_w0 holds (the sample's weight is formed at copy-out: 8 B of staging a sample, not 10)
    typedef typename std::conditional<SEM == 3, uint32_t, uint16_t>::type StL;
    __shared__ StL st_l[STG];
    __shared__ float s_w0[SEM == 3 ? PLC_THREADS : 1];
    __shared__ uint32_t s_vote[2][PLC_THREADS / 64];  // block_any: sector test, second pass
#ifdef TSDF_ABLATE_PL_EMPTY
    __shared__ uint32_t s_nst;             // staged samples (end of the last staged run)
#endif
#ifdef TSDF_PLC_PHASE  // diagnostic build: thread 0's clock at the phase boundaries
    unsigned long long pt[6];
    if (threadIdx.x == 0) pt[0] = clock64();
#endif
#ifdef TSDF_ABLATE_PL_EMPTY  // diagnostic build: the workgroups' dispatch and LDS allocation only
    if (threadIdx.x < 2 && D.n_scans == 0xFFFFFFFFu) {
        s_base[threadIdx.x] = 0u; s_loff[threadIdx.x] = 0; s_ord[threadIdx.x] = 0;
        s_bits[threadIdx.x] = 0u; s_wpre[threadIdx.x] = 0; st_s[threadIdx.x] = 0.0f;
        st_l[threadIdx.x] = 0; s_nst = 0u;
    }
    return;
#endif
    // workgroup 2 b + hf takes half hf of k_count block b's rays, and that half's run list
    // (sector sharding: block b is the (w / 2)-th of k_sector_flags' list, the rest leave)
    uint32_t wb = xcd_wedge(blockIdx.x, gridDim.x, 32);
    if (R.sec_on) {
        if ((blockIdx.x >> 1) >= G->ctr[parity].n_act) return;
        wb = 2 * Wk.act[blockIdx.x >> 1] + (blockIdx.x & 1u);
    }
    uint32_t t, r0, r1;
    block_range(D, wb >> 1, t, r0, r1);
    r0 += (wb & 1u) * PLC_THREADS;
    const uint4* bt = Wk.blk + (size_t)wb * HCAP;
    const uint32_t maxp = Wk.maxp;
    const uint32_t i = r0 + threadIdx.x;
    // Every independent global load is issued first, so the prologue waits two memory round trips
    // (list entry -> its cell) instead of four (point -> pair codes, list -> cell): the ray's point
    // and pair codes, the list length, and each lane's first list entry.
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    uint4 code4 = make_uint4(NO_PAIR, NO_PAIR, NO_PAIR, NO_PAIR);
    const uint32_t* pc = Wk.pair + (size_t)i * maxp;
    if (i < r1) {
        const float* __restrict__ xs = scan_xyz(xyz, D, t, R);
        px = xs[3 * (size_t)i];
        py = xs[3 * (size_t)i + 1];
        pz = xs[3 * (size_t)i + 2];
        if (maxp == 4) code4 = *reinterpret_cast<const uint4*>(pc);
    }
    const uint32_t nruns = Wk.blk_n[wb];
    static_assert(PLC_THREADS <= HCAP, "a lane's first list entry lies inside the list");
    const uint4 e0 = bt[threadIdx.x];
    // k_count's staging plan: bitmap words, their prefix (u16 pairs) and the staged count
    const uint32_t* pl = Wk.plan + (size_t)wb * PLAN_STRIDE;
    static_assert(PW <= PLC_THREADS, "one bitmap word per lane");
    const uint32_t plan_bits = threadIdx.x < (uint32_t)PW ? pl[threadIdx.x] : 0u;
    const uint32_t plan_pre =
        threadIdx.x < (uint32_t)((PW + 1) / 2) ? pl[PW + threadIdx.x] : 0u;
    const uint32_t plan_nst = pl[PLAN_STRIDE - 1];
    // a run's absolute sample position is its (brick, scan) cell (absolute after k_compact) + its
    // rank.  The gather is issued here; for short rays (maxp <= 4) its value is first needed after
    // the walk (the copy-out, and the rare samples the staging cannot hold), so the walk hides it.
    const bool late = maxp <= 4;
    const uint32_t cell0 = (threadIdx.x < nruns && e0.x != NO_PAIR)
                               ? T.cell[(size_t)e0.x * T.cell_stride + t]
                               : NO_PAIR;
    const float ox = D.s[t].ox, oy = D.s[t].oy, oz = D.s[t].oz;
    typename Walk<SEM>::State r;
    const bool ok = i < r1 && Walk<SEM>::init(R, D, t, i, px, py, pz, r);
    // sector sharding: a half block without a ray of this GPU's sector has no samples to place
    if (R.sec_on && !block_any<PLC_THREADS>(ok, s_vote[0])) return;
    if constexpr (SEM == 3) s_w0[threadIdx.x] = ok ? r.w0 : 0.0f;
    if (threadIdx.x < (uint32_t)PW) s_bits[threadIdx.x] = plan_bits;
    if (threadIdx.x < (uint32_t)((PW + 1) / 2))
        reinterpret_cast<uint32_t*>(s_wpre)[threadIdx.x] = plan_pre;
#ifdef TSDF_PLC_PHASE
    if (threadIdx.x == 0) pt[1] = clock64();
#endif
    // run table from the dense run list (k_count order = sample order); staged runs are a prefix
    // of the list, so a staged run's list index is its staging rank
    auto fill = [&](uint32_t j, const uint4& e) {
        const uint32_t slot = e.w >> 16;
        // runs starting past the staging capacity are stored directly (0xFFFF: not staged)
        const bool stg = e.z < (uint32_t)STG;
        s_loff[slot] = stg ? (uint16_t)e.z : (uint16_t)0xFFFFu;
        if (stg) s_ord[j] = (uint16_t)slot;
    };
    auto run_base = [&](const uint4& e, uint32_t cell) {
        return e.x != NO_PAIR ? cell + e.y : NO_PAIR;
    };
    if (threadIdx.x < nruns) {
        fill(threadIdx.x, e0);
        if (!late) s_base[e0.w >> 16] = run_base(e0, cell0);
    }
    for (uint32_t j = threadIdx.x + PLC_THREADS; j < nruns; j += PLC_THREADS) {
        const uint4 e = bt[j];
        fill(j, e);
        if (!late) s_base[e.w >> 16] = run_base(e, e.x != NO_PAIR ? T.cell[(size_t)e.x * T.cell_stride + t] : 0u);
    }
    __syncthreads();
#ifdef TSDF_PLC_PHASE
    if (threadIdx.x == 0) pt[2] = clock64();
#endif
#ifdef TSDF_ABLATE_PL_PROLOGUE  // diagnostic build: the prologue (loads, run tables) only
    if (D.n_scans != 0xFFFFFFFFu) return;
#endif
#ifdef TSDF_PLC_PHASE
    if (threadIdx.x == 0) pt[3] = clock64();
#endif
    // Voxblox 1/z^2: a sample's weight (the ray's 1/z^2, then the dropoff); 0 for the others
    auto sample_w = [&](const typename Walk<SEM>::State& st, float s) -> float {
        if constexpr (SEM == 3) return vb_weight(R, st.w0, s);
        else return 0.0f;
    };
    // a pair code -> its samples' global position (when `with_pos`: s_base is filled), staging
    // position (lpos < STG), count
    auto resolve = [&](uint32_t code, bool with_pos, uint32_t& pos, uint32_t& lpos, uint32_t& cnt) {
        pos = NO_PAIR;
        lpos = NO_PAIR;
        cnt = 0;
        if (code == NO_PAIR || code == PAIR_DEAD) return;
        cnt = (code >> PAIR_CNT_SHIFT) & 31u;
        if (code & PAIR_FB) {
            if (with_pos) {
                const uint4 f = Wk.fb[code & ((1u << PAIR_CNT_SHIFT) - 1u)];
                pos = T.cell[(size_t)f.x * T.cell_stride + f.y] + f.z;
            }
        } else {
            const uint32_t slot = (code >> PAIR_LID_SHIFT) & (HCAP - 1);
            const uint32_t lr = code & ((1u << PAIR_LID_SHIFT) - 1u);
            const uint32_t b = with_pos ? s_base[slot] : 0u;
            if (b != NO_PAIR) {
                if (with_pos) pos = b + lr;
                const uint32_t lo = s_loff[slot];
                if (lo != 0xFFFFu) lpos = lo + lr;
            }
        }
    };
    // Short rays (maxp <= 4): all of the ray's pairs are resolved up front, convergent across
    // lanes; the walk then only selects the k-th.  Branch-free (lanes are at different steps of
    // different pairs, so every data-dependent branch would run for the whole wave).
    //   pass 0 (late: the bases are not known yet): the samples the staging holds go to LDS, and a
    //          lane whose ray has others (past the staging, fallback pairs) notes it;
    //   pass 1 (after the bases; only those lanes): the ray walks again and stores the others.
    // Without `late` one pass does both, with the bases from the prologue.
    bool ovf = false;
    auto walk_short = [&](auto stage_c, auto direct_c, typename Walk<SEM>::State& rs) {
        constexpr bool STAGE = decltype(stage_c)::value, DIRECT = decltype(direct_c)::value;
        constexpr bool WITH_POS = DIRECT;
        uint4 code = make_uint4(NO_PAIR, NO_PAIR, NO_PAIR, NO_PAIR);
        if (maxp == 4) {
            code = code4;
        } else {
            code.x = pc[0];
            if (maxp > 1) code.y = pc[1];
            if (maxp > 2) code.z = pc[2];
        }
        // pair queue: global position P, and (staging position | count << 16) Q; a staging
        // position of 0xFFFF (>= STG) means not staged
        uint32_t P0 = NO_PAIR, P1 = NO_PAIR, P2 = NO_PAIR, P3 = NO_PAIR;
        uint32_t Q0 = 0xFFFFu, Q1 = 0xFFFFu, Q2 = 0xFFFFu, Q3 = 0xFFFFu;
        static_assert(STG < 0xFFFF, "staging positions are 16-bit");
        auto resolve_q = [&](uint32_t c, uint32_t& P, uint32_t& Q) {
            uint32_t lp, n;
            resolve(c, WITH_POS, P, lp, n);
            Q = min(lp, 0xFFFFu) | (n << 16);
        };
        resolve_q(code.x, P0, Q0);
        resolve_q(code.y, P1, Q1);
        resolve_q(code.z, P2, Q2);
        resolve_q(code.w, P3, Q3);
        uint32_t cur = ~0u;          // brick code of the current pair
        uint32_t pos = NO_PAIR, w = 0;
        uint32_t lq = 0xFFFFu;       // current pair's (staging position | count << 16)
        auto walk = [&](auto chk) {
            for (int it = 0; it < MAX_DDA_STEPS; it++) {
                float s;
                const bool g = Walk<SEM>::sample_sel(R, ox, oy, oz, rs, s, decltype(chk)::value);
                const uint32_t key = brick_code_of(rs.vx, rs.vy, rs.vz);
                const uint32_t l = ((rs.vz & 7) << 6) | ((rs.vy & 7) << 3) | (rs.vx & 7);
                // the next DDA step now, in the same basic block as the sample's double chain
                // (after the staging branch the scheduler could not overlap the two)
                const bool adv = Walk<SEM>::step_sel(rs);
                const bool nb = g && key != cur;  // the ray's next pair, in k_count's order
                cur = nb ? key : cur;
                // take the head of the ray's pair queue and shift the queue: plain selects (a
                // select on the pair index k compiles to branches)
                pos = nb ? P0 : pos;
                lq = nb ? Q0 : lq;
                P0 = nb ? P1 : P0;
                P1 = nb ? P2 : P1;
                P2 = nb ? P3 : P2;
                P3 = nb ? NO_PAIR : P3;
                Q0 = nb ? Q1 : Q0;
                Q1 = nb ? Q2 : Q1;
                Q2 = nb ? Q3 : Q2;
                Q3 = nb ? 0xFFFFu : Q3;
                w = nb ? 0u : w;
                const uint32_t lpos = lq & 0xFFFFu, cnt = lq >> 16;
                const bool st = g && w < cnt;
                const bool staged = lpos + w < (uint32_t)STG;
                if (STAGE && st && staged) {
                    st_s[lpos + w] = s;
                    st_l[lpos + w] = (StL)(SEM == 3 ? l | (threadIdx.x << 9) : l);
                } else if (st && !staged) {
                    if constexpr (DIRECT) {
                        if (pos != NO_PAIR && pos + w < Wk.max_smp) {
                            smp_store<SEM>(Wk, pos + w, s, (t << 9) | l, sample_w(rs, s));
                        }
                    } else {
                        ovf = true;
                    }
                }
                w += g ? 1u : 0u;
                if (!adv) break;
            }
        };
        if (__all(Walk<SEM>::inside(R, rs))) walk(std::false_type{});
        else walk(std::true_type{});
    };
#ifdef TSDF_ABLATE_PL_NOWALK
    if (ok && r.px == 1e30f) {
#else
    if (ok) {
#endif
        if (late) {
            walk_short(std::true_type{}, std::false_type{}, r);
        } else {
            uint32_t cur = ~0u;  // brick code of the current pair
            uint32_t k = 0, pos = NO_PAIR, lpos = NO_PAIR, cnt = 0, w = 0;
            for (int it = 0; it < MAX_DDA_STEPS; it++) {
                float s;
                if (Walk<SEM>::sample(R, ox, oy, oz, r, s)) {
                    const uint32_t key = brick_code_of(r.vx, r.vy, r.vz);
                    if (key != cur) {  // the ray's next pair, in k_count's order
                        cur = key;
                        resolve(k < maxp ? pc[k] : NO_PAIR, true, pos, lpos, cnt);
                        k++;
                        w = 0;
                    }
                    if (w < cnt) {
                        const uint32_t l = ((r.vz & 7) << 6) | ((r.vy & 7) << 3) | (r.vx & 7);
                        if (lpos != NO_PAIR && lpos + w < (uint32_t)STG) {
                            st_s[lpos + w] = s;
                            st_l[lpos + w] = (StL)(SEM == 3 ? l | (threadIdx.x << 9) : l);
                        } else if (pos != NO_PAIR && pos + w < Wk.max_smp) {
                            smp_store<SEM>(Wk, pos + w, s, (t << 9) | l, sample_w(r, s));
                        }
                    }
                    w++;
                }
                if (!Walk<SEM>::step(r)) break;
            }
        }
    }
    if (late) {
        // the bases, now that the walk has covered the gather; then the second pass where needed
        if (threadIdx.x < nruns) s_base[e0.w >> 16] = run_base(e0, cell0);
        for (uint32_t j = threadIdx.x + PLC_THREADS; j < nruns; j += PLC_THREADS) {
            const uint4 e = bt[j];
            s_base[e.w >> 16] = run_base(e, e.x != NO_PAIR ? T.cell[(size_t)e.x * T.cell_stride + t] : 0u);
        }
        if (block_any<PLC_THREADS>(ovf, s_vote[1]) && ovf) {
            // a fresh state: the first pass's is dead after its loop (kept, it would be carried
            // out of that loop and cost register copies at every step)
            typename Walk<SEM>::State r2;
            Walk<SEM>::init(R, D, t, i, px, py, pz, r2);
            walk_short(std::false_type{}, std::true_type{}, r2);
        }
    } else {
        __syncthreads();  // (late: the barrier above already published the staging and the bases)
    }
#ifdef TSDF_PLC_PHASE
    if (threadIdx.x == 0) pt[4] = clock64();
#endif
    // copy-out: one lane per staged sample; its run = the last run start at or before it
#ifdef TSDF_ABLATE_PL_NOCOPY
    const uint32_t nst = 0;
#else
    const uint32_t nst = min(plan_nst, (uint32_t)STG);
#endif
    for (uint32_t j = threadIdx.x; j < nst; j += PLC_THREADS) {
        const uint32_t wd = j >> 5;
        const uint32_t rank = s_wpre[wd] + __popc(s_bits[wd] & ((2u << (j & 31)) - 1u)) - 1u;
        const uint32_t slot = s_ord[rank];
        const uint32_t b = s_base[slot];
        if (b != NO_PAIR) {
            const uint32_t dst = b + (j - s_loff[slot]);
            if (dst < Wk.max_smp) {
                const uint32_t sl = st_l[j];
                smp_store<SEM>(Wk, dst, st_s[j], (t << 9) | (sl & 511u),
                               SEM == 3 ? vb_weight(R, s_w0[sl >> 9], st_s[j]) : 0.0f);
            }
        }
    }
#ifdef TSDF_PLC_PHASE
    if (threadIdx.x == 0 && (blockIdx.x % 61) == 0) {
        pt[5] = clock64();
        printf("place %u prol0 %llu prol1 %llu prol2 %llu walk %llu copy %llu\n", blockIdx.x,
               pt[1] - pt[0], pt[2] - pt[1], pt[3] - pt[2], pt[4] - pt[3], pt[5] - pt[4]);
    }
#endif
}

// ------------------------------------------------------------------------------------------------
// read-out / import

// ABI v10: int64 bounds; a voxel outside the index domain reads the background
__global__ void k_query_dense(Table T, Pool Pl, int64_t lo0, int64_t lo1, int64_t lo2, int nx,
                              int ny, int nz, float bg_sdf, float* __restrict__ out_sdf,
                              float* __restrict__ out_w) {
    const uint64_t total = (uint64_t)nx * ny * nz;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t xl = lo0 + (int64_t)(i % nx);
        const int64_t yl = lo1 + (int64_t)((i / nx) % ny);
        const int64_t zl = lo2 + (int64_t)(i / ((uint64_t)nx * ny));
        float s = bg_sdf, w = 0.0f;
        if (xl > -VOX_LIMIT && xl < VOX_LIMIT && yl > -VOX_LIMIT && yl < VOX_LIMIT &&
            zl > -VOX_LIMIT && zl < VOX_LIMIT) {
            const int x = (int)xl, y = (int)yl, z = (int)zl;
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
                               const float* __restrict__ sdf_in, const float* __restrict__ w_in,
                               float max_w) {
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
        *W = nw > max_w ? max_w : nw;  // Voxblox: capped at max_weight (else +inf)
    }
}

template <typename Tv>
__global__ void k_fill(Tv* __restrict__ p, Tv v, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// ------------------------------------------------------------------------------------------------
// launchers (called from tsdf_capi.cpp)

static int grid_for(uint64_t items, int per_block, int cap) {
    const uint64_t g = (items + per_block - 1) / per_block;
    return (int)(g < 1 ? 1 : (g > (uint64_t)cap ? (uint64_t)cap : g));
}

// One batch is k_count -> k_compact -> k_place -> k_integrate -> k_finish on one stream; the host
// (tsdf_capi.cpp) interleaves the cross-batch waits between them.
hipError_t launch_count(const float* d_xyz, const BatchRef& D, const RayConst& R, const Table& T,
                        const Work& Wk, Globals* G, int parity, hipStream_t st, const KTime& kt,
                        bool wide, bool paired) {
    // sem 3 (Voxblox 1/z^2) walks as Walk<1> (Walk<3> derives from it); its own instantiation
    // plans k_place<3>'s larger staging
    if (wide) {  // a batch too small to fill the chip: 1024-lane workgroups
        auto k = R.sem == 3 ? k_count<3, 1024> : R.sem == 1 ? k_count<1, 1024> : R.sem == 2 ? k_count<2, 1024> : k_count<0, 1024>;
#ifndef TSDF_CNT_SPLIT
        tlaunch(k, D.n_blocks, 1024, st, kt.start, kt.stop, d_xyz, D, R, T, Wk, G, parity);
#else
        tlaunch(k, D.n_blocks, 1024, st, kt.start, nullptr, d_xyz, D, R, T, Wk, G, parity);
#endif
    } else if (paired) {  // two blocks per 512-lane workgroup (no sector sharding)
        constexpr int NT2 = 2 * CNT_THREADS;
        auto k = R.sem == 3 ? k_count<3, NT2, 2> : R.sem == 1 ? k_count<1, NT2, 2> : R.sem == 2 ? k_count<2, NT2, 2> : k_count<0, NT2, 2>;
        tlaunch(k, (D.n_blocks + 1) / 2, NT2, st, kt.start, kt.stop, d_xyz, D, R, T, Wk, G, parity);
    } else {
        auto k = R.sem == 3 ? k_count<3> : R.sem == 1 ? k_count<1> : R.sem == 2 ? k_count<2> : k_count<0>;
#ifndef TSDF_CNT_SPLIT
        tlaunch(k, D.n_blocks, CNT_THREADS, st, kt.start, kt.stop, d_xyz, D, R, T, Wk, G, parity);
#else
        tlaunch(k, D.n_blocks, CNT_THREADS, st, kt.start, nullptr, d_xyz, D, R, T, Wk, G, parity);
#endif
    }
#ifdef TSDF_CNT_SPLIT
    if (!paired) tlaunch(k_resolve, D.n_blocks, RSV_THREADS, st, nullptr, kt.stop, D, R, T, Wk, G, parity);
#endif
    return hipGetLastError();
}

hipError_t launch_compact(const BatchRef& D, const Table& T, const Work& Wk, Globals* G,
                          int parity, bool fused, hipStream_t st, const KTime& kt) {
    const uint32_t nch = (uint32_t)compact_chunks(T.mask + 1);
    tlaunch(fused ? k_compact_sum<true> : k_compact_sum<false>, nch, CMP_THREADS, st, kt.start,
            nullptr, D.n_scans, T, Wk);
    k_compact_scan<<<1, CMP_SCAN_THREADS, 0, st>>>(nch, Wk, G, parity, fused ? 1 : 0);
    tlaunch(fused ? k_compact_write<true> : k_compact_write<false>, nch, CMP_THREADS, st, nullptr,
            kt.stop, D.n_scans, nch, T, Wk, G, parity);
    return hipGetLastError();
}

hipError_t launch_place(const float* d_xyz, const BatchRef& D, const RayConst& R, const Table& T,
                        const Work& Wk, Globals* G, int parity, hipStream_t st, const KTime& kt) {
    auto k = R.sem == 1 ? k_place<1> : R.sem == 3 ? k_place<3> : R.sem == 2 ? k_place<2> : k_place<0>;
    tlaunch(k, 2 * D.n_blocks, PLC_THREADS, st, kt.start, kt.stop, d_xyz, D, R, T, Wk, G, parity);
    return hipGetLastError();
}

__device__ __forceinline__ void ord_slice(uint32_t n_active, uint32_t b, uint32_t& i0,
                                          uint32_t& i1) {
    const uint32_t per = (n_active + ORD_BLOCKS - 1) / ORD_BLOCKS;
    i0 = min(n_active, b * per);
    i1 = min(n_active, i0 + per);
}

// pass 1: per-slice class histogram (LDS), written out without global atomics
__global__ __launch_bounds__(ORD_THREADS) void k_order_hist(Work Wk, Globals* G, int parity) {
    __shared__ uint32_t h[ORD_CLASSES];
    if (threadIdx.x < ORD_CLASSES) h[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t i0, i1;
    ord_slice(min(G->ctr[parity].n_active, Wk.max_active), blockIdx.x, i0, i1);
    for (uint32_t i = i0 + threadIdx.x; i < i1; i += ORD_THREADS)
        atomicAdd(&h[size_class(Wk.active[i].w)], 1u);
    __syncthreads();
    if (threadIdx.x < ORD_CLASSES) Wk.ord_hist[blockIdx.x * ORD_CLASSES + threadIdx.x] = h[threadIdx.x];
}

// pass 2 (one workgroup): slice s's first position in class k = all records of larger classes +
// class k's records in the slices before s
__global__ __launch_bounds__(ORD_BLOCKS * ORD_CLASSES / 2) void k_order_scan(Work Wk) {
    constexpr int NT = ORD_BLOCKS * ORD_CLASSES / 2;  // two (slice, class) entries per thread
    __shared__ uint32_t tot[ORD_CLASSES];
    __shared__ uint32_t cls_base[ORD_CLASSES];
    const int t = threadIdx.x;
    if (t < ORD_CLASSES) {
        uint32_t sum = 0;  // class t over all slices
        for (int b = 0; b < ORD_BLOCKS; b++) sum += Wk.ord_hist[b * ORD_CLASSES + t];
        tot[t] = sum;
    }
    __syncthreads();
    if (t < 64) {
        const uint32_t v = t < ORD_CLASSES ? tot[t] : 0u;
        const uint32_t incl = wave_incl_scan(v);
        if (t < ORD_CLASSES) cls_base[t] = incl - v;
    }
    __syncthreads();
    if (t < ORD_CLASSES) {  // running prefix over the slices of class t
        uint32_t run = cls_base[t];
        for (int b = 0; b < ORD_BLOCKS; b++) {
            const uint32_t v = Wk.ord_hist[b * ORD_CLASSES + t];
            Wk.ord_hist[b * ORD_CLASSES + t] = run;
            run += v;
        }
    }
    (void)NT;
}

// pass 3: every record to its class position (rank inside a slice's class from LDS atomics)
__global__ __launch_bounds__(ORD_THREADS) void k_order_scatter(Work Wk, Globals* G, int parity) {
    __shared__ uint32_t base[ORD_CLASSES];
    if (threadIdx.x < ORD_CLASSES) base[threadIdx.x] = Wk.ord_hist[blockIdx.x * ORD_CLASSES + threadIdx.x];
    __syncthreads();
    uint32_t i0, i1;
    ord_slice(min(G->ctr[parity].n_active, Wk.max_active), blockIdx.x, i0, i1);
    for (uint32_t i = i0 + threadIdx.x; i < i1; i += ORD_THREADS) {
        const uint4 r = Wk.active[i];
        Wk.active_ord[atomicAdd(&base[size_class(r.w)], 1u)] = r;
    }
}

hipError_t launch_order(const Work& Wk, Globals* G, int parity, hipStream_t st) {
    k_order_hist<<<ORD_BLOCKS, ORD_THREADS, 0, st>>>(Wk, G, parity);
    k_order_scan<<<1, ORD_BLOCKS * ORD_CLASSES / 2, 0, st>>>(Wk);
    k_order_scatter<<<ORD_BLOCKS, ORD_THREADS, 0, st>>>(Wk, G, parity);
    return hipGetLastError();
}

// End of a batch: fold its counters into the running totals (if it committed), keep them as the
// "last batch" snapshot and zero them for the next batch of the same parity (the same stream, so
// ordered after every reader of this batch).  A batch that raised an overflow marks the context
// failed (its id kept for the host's replay); with G->retry, it and every later batch until the
// host's check do not commit.
__global__ void k_finish(Globals* G, int parity, uint32_t batch_id) {
    constexpr int NW = sizeof(Counters) / 4;
    Counters* C = &G->ctr[parity];
    const uint32_t ovf = C->ovf, failed = G->failed;
    const bool commit = !(G->retry && (ovf || failed));
    __syncthreads();  // every lane read the flags before lane 0 updates them
    if (threadIdx.x < 8 && commit) {
        const int k = threadIdx.x;
        G->tot_rays[k] += C->n_rays[k];
        G->tot_pairs[k] += C->n_pairs[k];
        G->tot_vox[k] += C->n_vox[k];
        G->tot_dirty[k] += C->n_dirty[k];
    }
    if (threadIdx.x == 0 && ovf) {
        G->overflow |= ovf;
        if (!failed) {
            G->failed = 1u;
            G->fail_id = batch_id;
        }
    }
    if (threadIdx.x == 0) {  // the batch's metrics record
        BatchRecord r;
        r.batch_id = batch_id;
        r.n_active = C->n_active;
        r.n_new = C->n_new;
        r.ovf = ovf;
        r.committed = commit ? 1u : 0u;
        r.pool_count = G->pool_count;
        r.pad[0] = r.pad[1] = 0u;
        r.rays = r.pairs = r.vox = r.dirty = 0ull;
        for (int k = 0; k < 8; k++) {
            r.rays += C->n_rays[k];
            r.pairs += C->n_pairs[k];
            r.vox += C->n_vox[k];
            r.dirty += C->n_dirty[k];
        }
        G->ring[batch_id % METRIC_RING] = r;
    }
    __syncthreads();
    uint32_t* src = reinterpret_cast<uint32_t*>(C);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&G->last);
    for (int j = threadIdx.x; j < NW; j += blockDim.x) {
        dst[j] = src[j];
        src[j] = 0u;
    }
}

// A batch's scan records from the pinned host ring to the device ring: one small kernel reads them
// over PCIe (zero-copy) instead of a copy command, then tells the host the ring slot is free by
// storing the launch's sequence number to a pinned host word (a vector store at system scope).
// The host waits on that word to reuse a slot, so a serial batch needs no event marker in the
// stream: each marker left the GPU idle ~5 us (profiles/gap_trace.py).
__global__ void k_upload(const uint4* __restrict__ src, uint4* __restrict__ dst, uint32_t n,
                         unsigned long long* done, unsigned long long seq) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();  // every read of the host slot is complete
    if (threadIdx.x == 0)
        __hip_atomic_fetch_max(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_upload(const void* host_src, void* dst, uint32_t bytes,
                         unsigned long long* done, unsigned long long seq, hipStream_t st) {
    k_upload<<<1, 256, 0, st>>>(static_cast<const uint4*>(host_src), static_cast<uint4*>(dst),
                                bytes / 16, done, seq);
    return hipGetLastError();
}

hipError_t launch_finish(Globals* G, int parity, uint32_t batch_id, hipStream_t st) {
    k_finish<<<1, 64, 0, st>>>(G, parity, batch_id);
    return hipGetLastError();
}

// Capacity growth: the grown table is rebuilt from the pool's slot -> key map (bricks the failed
// batch inserted without a slot are dropped; the replay inserts them again).
__global__ void k_rehash(Table T, uint32_t n, Globals* G) {
    for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < n;
         slot += gridDim.x * blockDim.x) {
        const int64_t h = table_insert(T, T.brick_keys[slot], &G->overflow);
        if (h >= 0) T.slots[h] = slot;
    }
}

hipError_t launch_rehash(const Table& T, uint32_t n, Globals* G, hipStream_t st) {
    if (n) k_rehash<<<grid_for(n, 256, 4096), 256, 0, st>>>(T, n, G);
    return hipGetLastError();
}

hipError_t launch_query_dense(const Table& T, const Pool& Pl, const int64_t lo[3], const int dims[3],
                              float bg, float* d_sdf, float* d_w, hipStream_t st) {
    const uint64_t total = (uint64_t)dims[0] * dims[1] * dims[2];
    k_query_dense<<<grid_for(total, 256, 8192), 256, 0, st>>>(T, Pl, lo[0], lo[1], lo[2], dims[0],
                                                              dims[1], dims[2], bg, d_sdf, d_w);
    return hipGetLastError();
}

hipError_t launch_import(const Table& T, const Pool& Pl, const int32_t* d_coords, uint32_t n,
                         const float* d_sdf, const float* d_w, uint32_t* d_tidx, Globals* G,
                         float max_w, hipStream_t st) {
    k_import_insert<<<grid_for(n, 256, 4096), 256, 0, st>>>(T, d_coords, n, d_tidx, G);
    k_import_merge<<<grid_for((uint64_t)n * BRICK_VOX, 256, 8192), 256, 0, st>>>(T, Pl, d_tidx, n,
                                                                                 d_sdf, d_w, max_w);
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
