// tsdf_walk.hip — the single-walk front end of the batch pipeline ("one walk").
//
// The two-walk front end (k_count, then k_place, tsdf_kernels.hip) walks every ray twice: once to
// count each (brick, scan)'s samples, once to write them into per-brick segments whose positions
// only exist after the batch-wide compaction.  Here every ray is walked ONCE:
//
//   k_walk   one 512-lane workgroup per 512 consecutive rays of one scan (one ray per lane).  The
//            lane walks its DDA over the band with the sample arithmetic of k_place and keeps every
//            gated sample in registers, one slot per DDA step (static indices: NSTEP slots, NSTEP a
//            host-proven bound on the voxels a band can visit).  Its <= 4 (ray, brick) pairs go into
//            the workgroup's LDS brick hash (rank of the pair inside the workgroup's run for the
//            brick).  A block scan gives every run its offset in the workgroup's sample order; the
//            samples are staged in LDS in that order and written out LINEARLY to the workgroup's own
//            region of the sample array (full lines, no per-brick scatter).  Per distinct brick: one
//            global find-or-insert and ONE 64-bit atomic on its (brick, scan) cell, which counts
//            samples (low word) and spans (high word) and so hands the run its rank among the
//            cell's spans.  The workgroup's dense run list (table index, span rank, region offset,
//            samples, scan) goes to HBM for k_spans.
//   k_spans  after k_compact has made every cell an absolute span position: each run becomes
//            ceil(samples / SPAN) span records (region position | (count - 1) << 30) at its
//            brick's span-list position.  k_integrate then reads a brick's samples through its
//            spans — scan-ordered, SPAN-sample granules of contiguous region memory.
//
// Same semantics as the two-walk path, bit for bit: the per-voxel sums are exact and order-free,
// and the samples are computed by the same Walk<SEM>::sample_sel arithmetic (tsdf_ray.h).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

// Scan and ray range of RPB-ray block b (uniform: scalar loads of the descriptor).
__device__ __forceinline__ void walk_block_range(const BatchRef& D, uint32_t b, uint32_t& t,
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

// LDS brick hash with unbounded probing: a workgroup holds at most WLK_THREADS * 4 = HCAP distinct
// bricks, so a key always finds its slot (no global fallback path).
__device__ __forceinline__ int lds_insert_full(unsigned long long* s_key, uint64_t key) {
    uint32_t hs = (uint32_t)(mix64(key) >> 40) & (HCAP - 1);
    for (;;) {
        const unsigned long long k = s_key[hs];
        if (k == key) return (int)hs;
        if (k == EMPTY_KEY) {
            const unsigned long long old = atomicCAS(&s_key[hs], EMPTY_KEY, key);
            if (old == EMPTY_KEY || old == key) return (int)hs;
        }
        hs = (hs + 1) & (HCAP - 1);
    }
}

static_assert(WLK_THREADS * 4 <= HCAP, "a workgroup's pairs must fit its LDS brick hash");

template <int SEM, int NSTEP>
__global__ __launch_bounds__(WLK_THREADS) void k_walk(const float* __restrict__ xyz, BatchRef D,
                                                     RayConst R, Table T, Work Wk, Globals* G,
                                                     int parity) {
    constexpr int STG = WLK_THREADS * NSTEP;  // a workgroup's worst-case samples (= region size)
    static_assert(STG < 65536, "staging offsets are 16-bit");
    constexpr int SPT = HCAP / WLK_THREADS;   // LDS hash slots per thread in the block scan
    constexpr int NW = WLK_THREADS / 64;
    __shared__ unsigned long long s_key[HCAP];
    __shared__ uint32_t s_cnt[HCAP];
    __shared__ uint16_t s_off[HCAP];  // run -> its first sample in the workgroup's order
    __shared__ float st_s[STG];       // staged samples, run order
    __shared__ uint16_t st_l[STG];
    __shared__ uint32_t s_wsum[NW];
    __shared__ unsigned long long red[2][NW];
    Counters* C = &G->ctr[parity];  // zeroed by the previous batch of this parity (k_finish)
    // workgroup 2 b + half takes half of RPB-ray block b (sector sharding: block b is the
    // (w / 2)-th of k_sector_flags' list, the rest of the grid leaves at once)
    uint32_t wb = blockIdx.x;
    if (R.sec_on) {
        if ((blockIdx.x >> 1) >= C->n_act) return;
        wb = 2 * Wk.act[blockIdx.x >> 1] + (blockIdx.x & 1u);
    }
    uint32_t t, r0, r1;
    walk_block_range(D, wb >> 1, t, r0, r1);
    r0 += (wb & 1u) * WLK_THREADS;
    const uint32_t i = r0 + threadIdx.x;
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    if (i < r1) {
        const float* __restrict__ xs = scan_xyz(xyz, D, t, R);
        px = xs[3 * (size_t)i];
        py = xs[3 * (size_t)i + 1];
        pz = xs[3 * (size_t)i + 2];
    }
    for (int j = threadIdx.x; j < HCAP; j += WLK_THREADS) {
        s_key[j] = EMPTY_KEY;
        s_cnt[j] = 0u;
    }
    const float ox = D.s[t].ox, oy = D.s[t].oy, oz = D.s[t].oz;
    typename Walk<SEM>::State r{};
    const bool ok = i < r1 && Walk<SEM>::init(R, D, t, i, px, py, pz, r);
    const int bx0 = r.vx >> 3, by0 = r.vy >> 3, bz0 = r.vz >> 3;  // the ray's first brick
    // One register slot per DDA step: sv = the sample, mv = voxel | pair << 9 | rank in the pair
    // << 11 | valid << 16 (0: no sample at this step).
    float sv[NSTEP];
    uint32_t mv[NSTEP];
#pragma unroll
    for (int k = 0; k < NSTEP; k++) {
        sv[k] = 0.0f;
        mv[k] = 0u;
    }
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;  // pair brick codes
    uint32_t n0 = 0, n1 = 0, n2 = 0;          // closed pairs' sample counts
    uint32_t cur = ~0u, wv = 0;               // current pair's code and samples so far
    int pi = -1;                              // current pair
    bool live = ok;
    // Branch-free walk (lanes are at different steps of different rays): selects only.
    auto walk = [&](auto chk) {
#pragma unroll
        for (int k = 0; k < NSTEP; k++) {
            float s;
            const bool gs = Walk<SEM>::sample_sel(R, ox, oy, oz, r, s, decltype(chk)::value);
            const bool g = live && gs;
            const uint32_t bc = brick_code_of(r.vx, r.vy, r.vz);
            const bool nb = g && bc != cur;  // the ray's next pair
            const int pn = pi + (nb ? 1 : 0);
            n0 = (nb && pn == 1) ? wv : n0;
            n1 = (nb && pn == 2) ? wv : n1;
            n2 = (nb && pn == 3) ? wv : n2;
            c0 = (nb && pn == 0) ? bc : c0;
            c1 = (nb && pn == 1) ? bc : c1;
            c2 = (nb && pn == 2) ? bc : c2;
            c3 = (nb && pn == 3) ? bc : c3;
            cur = nb ? bc : cur;
            pi = pn;
            wv = nb ? 0u : wv;
            const uint32_t l = ((r.vz & 7) << 6) | ((r.vy & 7) << 3) | (r.vx & 7);
            sv[k] = s;
            mv[k] = g ? (l | ((uint32_t)(pn & 3) << 9) | (wv << 11) | 0x10000u) : 0u;
            wv += g ? 1u : 0u;
            const bool adv = Walk<SEM>::step_sel(r);  // every lane steps (a finished ray's state
            live = live && adv;                       // no longer matters): no exec-mask split
            if (k + 1 < NSTEP && !__any(live)) break;  // uniform: every ray of the wave is done
        }
    };
    // rays far from the index-domain edge (all, in practice) skip the per-voxel check
#ifdef TSDF_ABLATE_WALK_NOWALK  // diagnostic build: no walk (wrong results)
    live = false;
#endif
    if (__all(!ok || Walk<SEM>::inside(R, r))) walk(std::false_type{});
    else walk(std::true_type{});
    // a walk longer than the host's bound, or more than 4 bricks: never for eligible parameters
    if (live || pi > 3) atomicOr(&C->ovf, OVF_PAIRS);
    const uint32_t np = (uint32_t)min(pi + 1, 4);
    const uint32_t n3 = pi == 3 ? wv : 0u;
    const uint32_t nl0 = pi == 0 ? wv : n0, nl1 = pi == 1 ? wv : n1, nl2 = pi == 2 ? wv : n2;
    __syncthreads();  // LDS hash cleared
    // pairs -> LDS hash: all lanes emit pair j together (convergent); e = slot | rank << 16
    uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0;
    auto emit = [&](uint32_t code, uint32_t cnt) -> uint32_t {
        const int lid = lds_insert_full(s_key, code_key(code, bx0, by0, bz0));
        const uint32_t lr = atomicAdd(&s_cnt[lid], cnt);
        return (uint32_t)lid | (lr << 16);
    };
    if (np > 0) e0 = emit(c0, nl0);
    if (np > 1) e1 = emit(c1, nl1);
    if (np > 2) e2 = emit(c2, nl2);
    if (np > 3) e3 = emit(c3, n3);
    __syncthreads();
    // Block scan over the hash slots: each run's offset in the workgroup's sample order and its
    // index in the dense run list (SPT consecutive slots per thread).
    uint32_t cnt[SPT], packed = 0;
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        const int slot = threadIdx.x * SPT + j;
        cnt[j] = s_key[slot] != EMPTY_KEY ? s_cnt[slot] : 0u;
        packed += cnt[j] | (cnt[j] ? 1u << 16 : 0u);  // samples < 2^16, runs in the high half
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t off, idx, tot_s, tot_r;
    {
        const uint32_t incl = wave_incl_scan(packed);
        if (lane == 63) s_wsum[wid] = incl;
        __syncthreads();
        uint32_t ex = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint32_t v = s_wsum[w];
            ex += w < wid ? v : 0u;
            tot += v;
        }
        const uint32_t e = ex + incl - packed;
        off = e & 0xFFFFu;
        idx = e >> 16;
        tot_s = tot & 0xFFFFu;
        tot_r = tot >> 16;
    }
    // the thread's slots: run offsets to LDS; first-probe loads of their keys in the global table
    uint64_t key[SPT], h0[SPT], k0[SPT];
    {
        uint32_t o = off;
#pragma unroll
        for (int j = 0; j < SPT; j++) {
            const int slot = threadIdx.x * SPT + j;
            s_off[slot] = (uint16_t)o;
            o += cnt[j];
            key[j] = cnt[j] ? s_key[slot] : EMPTY_KEY;
            h0[j] = mix64(key[j]) & T.mask;
            k0[j] = key[j] != EMPTY_KEY ? T.keys[h0[j]] : EMPTY_KEY;
        }
    }
    __syncthreads();  // s_off visible
    // stage the lane's samples in run order
    {
        const uint32_t b0 = np > 0 ? s_off[e0 & 0xFFFFu] + (e0 >> 16) : 0u;
        const uint32_t b1 = np > 1 ? s_off[e1 & 0xFFFFu] + (e1 >> 16) : 0u;
        const uint32_t b2 = np > 2 ? s_off[e2 & 0xFFFFu] + (e2 >> 16) : 0u;
        const uint32_t b3 = np > 3 ? s_off[e3 & 0xFFFFu] + (e3 >> 16) : 0u;
#pragma unroll
        for (int k = 0; k < NSTEP; k++) {
            const uint32_t m = mv[k];
            if (m) {
                const uint32_t j = (m >> 9) & 3u;
                const uint32_t b = j == 0 ? b0 : (j == 1 ? b1 : (j == 2 ? b2 : b3));
                const uint32_t pos = b + ((m >> 11) & 31u);
                st_s[pos] = sv[k];
                st_l[pos] = (uint16_t)(m & 511u);
            }
        }
    }
    // global table: resolve the first probes (a hit needs nothing more), then one 64-bit cell
    // atomic per run: samples | spans << 32, whose old value ranks the run's spans in the cell
    int64_t hx[SPT];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        hx[j] = -1;
#ifdef TSDF_ABLATE_WALK_NOGLOBAL  // diagnostic build: no global table work (wrong results)
        if (key[j] != EMPTY_KEY && key[j] == 12345ull)
#else
        if (key[j] != EMPTY_KEY)
#endif
            hx[j] = k0[j] == key[j] ? (int64_t)h0[j] : table_insert(T, key[j], &C->ovf);
    }
    unsigned long long* cell64 = reinterpret_cast<unsigned long long*>(T.cell);
    unsigned long long old[SPT];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        const unsigned long long add =
            (unsigned long long)cnt[j] | ((unsigned long long)((cnt[j] + SPAN - 1) / SPAN) << 32);
        old[j] = hx[j] >= 0 ? atomicAdd(&cell64[(size_t)hx[j] * T.cell_stride + t], add) : 0ull;
    }
    // the dense run list: (table index | NO_PAIR, span rank in the cell, region offset | samples
    // << 16, scan)
    uint4* bt = Wk.blk + (size_t)blockIdx.x * HCAP;
    {
        uint32_t o = off, q = idx;
#pragma unroll
        for (int j = 0; j < SPT; j++) {
            if (cnt[j]) {
                uint32_t tx = NO_PAIR;
                if (hx[j] >= 0) {
                    tx = (uint32_t)hx[j];
                    // the brick's first run of this scan lists it for k_compact
                    if (old[j] == 0ull) T.touched[tx] = 1u;
                }
                bt[q++] = make_uint4(tx, (uint32_t)(old[j] >> 32), o | (cnt[j] << 16), t);
            }
            o += cnt[j];
        }
    }
    if (threadIdx.x == 0) Wk.blk_n[blockIdx.x] = tot_r;
    __syncthreads();  // staging complete
    // copy-out: the workgroup's samples, linear, to its region (full lines)
    const size_t region = (size_t)blockIdx.x * STG;
#ifndef TSDF_ABLATE_WALK_NOCOPY  // diagnostic build: no copy-out (wrong results)
    if (region + STG <= Wk.max_smp) {
        for (uint32_t q = threadIdx.x; q < tot_s; q += WLK_THREADS)
            Wk.smp[region + q] = make_uint2(__float_as_uint(st_s[q]), (t << 9) | st_l[q]);
    } else if (threadIdx.x == 0) {
        atomicOr(&C->ovf, OVF_SMP);  // region array too small (sector sharding): grow and replay
    }
#endif
    // stats: one atomic per block on a shard picked by block index
    unsigned long long v = wave_sum<unsigned long long>(ok ? 1ull : 0ull);
    unsigned long long q = wave_sum<unsigned long long>((unsigned long long)np);
    if (lane == 0) {
        red[0][wid] = v;
        red[1][wid] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        v = 0;
        q = 0;
        for (int w = 0; w < NW; w++) {
            v += red[0][w];
            q += red[1][w];
        }
        if (v) atomicAdd(&C->n_rays[blockIdx.x & 7], v);
        if (q) atomicAdd(&C->n_pairs[blockIdx.x & 7], q);
    }
}

// ------------------------------------------------------------------------------------------------
// k_spans: one workgroup per k_walk workgroup's run list.  A block scan over the runs' span counts
// gives every span of the list a lane; the lane finds its run by binary search in LDS and writes the
// span record at the run's position in its brick's span list (consecutive lanes, consecutive spans
// of a run: coalesced per run).

constexpr int SPN_THREADS = 256;

template <int NSTEP>
__global__ __launch_bounds__(SPN_THREADS) void k_spans(RayConst R, Table T, Work Wk, Globals* G,
                                                      int parity) {
    constexpr int STG = WLK_THREADS * NSTEP;
    constexpr int RPT = HCAP / SPN_THREADS;  // runs per thread in the scan
    __shared__ uint32_t s_pre[HCAP];  // run -> its first span in the list's span order
    __shared__ uint32_t s_dst[HCAP];  // run -> its first span's position in the span list
    __shared__ uint32_t s_src[HCAP];  // run -> its first sample's position in the sample array
    __shared__ uint16_t s_n[HCAP];    // run -> its samples
    __shared__ uint32_t s_w[SPN_THREADS / 64];
    const Counters* C = &G->ctr[parity];
    const uint32_t w = blockIdx.x;
    if (R.sec_on && (w >> 1) >= C->n_act) return;
    const uint32_t nr = Wk.blk_n[w];
    if (nr == 0) return;  // uniform
    const unsigned long long* cell64 = reinterpret_cast<const unsigned long long*>(T.cell);
    const uint4* bt = Wk.blk + (size_t)w * HCAP;
    const uint32_t region = w * STG;
    uint32_t nsp[RPT], sum = 0;
#pragma unroll
    for (int k = 0; k < RPT; k++) {
        const uint32_t j = threadIdx.x * RPT + k;
        nsp[k] = 0;
        if (j < nr) {
            const uint4 e = bt[j];
            const uint32_t n = e.z >> 16;
            s_src[j] = region + (e.z & 0xFFFFu);
            s_n[j] = (uint16_t)n;
            if (e.x != NO_PAIR) {
                nsp[k] = (n + SPAN - 1) / SPAN;
                // the cell is the absolute span position of the (brick, scan) after k_compact
                s_dst[j] = (uint32_t)(cell64[(size_t)e.x * T.cell_stride + e.w] >> 32) + e.y;
            }
        }
        sum += nsp[k];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t ex = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < SPN_THREADS / 64; k++) {
        const uint32_t v = s_w[k];
        ex += k < wid ? v : 0u;
        tot += v;
    }
    uint32_t p = ex + incl - sum;
#pragma unroll
    for (int k = 0; k < RPT; k++) {
        const uint32_t j = threadIdx.x * RPT + k;
        if (j < nr) s_pre[j] = p;
        p += nsp[k];
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < tot; q += SPN_THREADS) {
        // the run holding span q: the LAST run whose first span is <= q (runs without spans —
        // dropped pairs — share their first span with the next run, so they are never chosen)
        uint32_t lo = 0, hi = nr;  // s_pre[lo] <= q < s_pre[hi] (hi = nr: past the end)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[mid] <= q) lo = mid;
            else hi = mid;
        }
        const uint32_t k = q - s_pre[lo];
        const uint32_t rem = s_n[lo] - k * SPAN;
        const uint32_t dst = s_dst[lo] + k;
        if (dst < Wk.max_spn)
            Wk.spn[dst] = (s_src[lo] + k * SPAN) | ((min(rem, (uint32_t)SPAN) - 1u) << 30);
    }
}

hipError_t launch_walk(const float* d_xyz, const BatchRef& D, const RayConst& R, const Table& T,
                       const Work& Wk, Globals* G, int parity, int nstep, hipStream_t st) {
    const uint32_t grid = 2 * D.n_blocks;
#define TSDF_WALK_LAUNCH(S, N) \
    k_walk<S, N><<<grid, WLK_THREADS, 0, st>>>(d_xyz, D, R, T, Wk, G, parity)
    if (nstep == 16) {
        if (R.sem == 1) TSDF_WALK_LAUNCH(1, 16);
        else if (R.sem == 2) TSDF_WALK_LAUNCH(2, 16);
        else TSDF_WALK_LAUNCH(0, 16);
    } else {
        if (R.sem == 1) TSDF_WALK_LAUNCH(1, 32);
        else if (R.sem == 2) TSDF_WALK_LAUNCH(2, 32);
        else TSDF_WALK_LAUNCH(0, 32);
    }
#undef TSDF_WALK_LAUNCH
    return hipGetLastError();
}

hipError_t launch_spans(const BatchRef& D, const RayConst& R, const Table& T, const Work& Wk,
                        Globals* G, int parity, int nstep, hipStream_t st) {
    const uint32_t grid = 2 * D.n_blocks;
    if (nstep == 16) k_spans<16><<<grid, SPN_THREADS, 0, st>>>(R, T, Wk, G, parity);
    else k_spans<32><<<grid, SPN_THREADS, 0, st>>>(R, T, Wk, G, parity);
    return hipGetLastError();
}

}  // namespace tsdf
