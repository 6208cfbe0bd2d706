// tsdf_border.hip — device side of the multi-GPU border-brick reduce.
//
// Azimuth-sector shards each hold a partial field; a brick touched by rays of several sectors is
// held by several ranks.  The reduce moves each shared brick's (S, W) mass to its owner, the
// lowest rank holding it, over the caller's RCCL all-to-all:
//   k_border_owner  keys of every lower rank are looked up in this rank's table: owner[slot] =
//                   min(rank, holders below it); per-destination row counts
//   k_border_list   the bricks owned elsewhere get a row in their destination's group
//   k_border_pack   one workgroup per row: the brick's 512 S and 512 W (+ key) go into the tile,
//                   and (reset) the brick is reset to the background (its mass now travels)
//   k_border_reset  the same reset on its own: tsdf_border_reduce_local packs without resetting
//                   and resets the sent bricks only after every merge succeeded
//   k_border_merge  owner side, one workgroup per received tile, launched once per source rank in
//                   ascending order: the tsdf_import_bricks rule (weighted mean, copy where W == 0)
// Rows within a destination group are in atomic order: the owner merges each source's tiles of
// distinct bricks independently, so the merged field does not depend on it.
#include <algorithm>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

namespace {

constexpr int BRD_THREADS = 256;

__global__ __launch_bounds__(BRD_THREADS) void k_border_init(uint32_t* __restrict__ owner,
                                                             uint32_t n, uint32_t rank,
                                                             uint32_t* __restrict__ dest_n) {
    for (uint32_t i = blockIdx.x * BRD_THREADS + threadIdx.x; i < n; i += gridDim.x * BRD_THREADS)
        owner[i] = rank;
    if (blockIdx.x == 0 && threadIdx.x < MAX_WORLD) dest_n[threadIdx.x] = 0;
}

// keys of lower rank r: every one this context also holds lowers its brick's owner to r
__global__ __launch_bounds__(BRD_THREADS) void k_border_owner(Table T,
                                                              const uint64_t* __restrict__ keys,
                                                              uint64_t n, uint32_t r,
                                                              uint32_t* __restrict__ owner) {
    for (uint64_t i = blockIdx.x * (uint64_t)BRD_THREADS + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * BRD_THREADS) {
        const uint64_t key = keys[i];
        if (key == EMPTY_KEY) continue;
        const int64_t h = table_find(T, key);
        if (h < 0) continue;
        const uint32_t slot = T.slots[h];
        if (slot < T.max_bricks) atomicMin(&owner[slot], r);
    }
}

__global__ __launch_bounds__(BRD_THREADS) void k_border_count(const uint32_t* __restrict__ owner,
                                                              uint32_t n, uint32_t rank,
                                                              uint32_t* __restrict__ dest_n) {
    for (uint32_t i = blockIdx.x * BRD_THREADS + threadIdx.x; i < n; i += gridDim.x * BRD_THREADS)
        if (owner[i] != rank) atomicAdd(&dest_n[owner[i]], 1u);
}

__global__ __launch_bounds__(BRD_THREADS) void k_border_list(const uint32_t* __restrict__ owner,
                                                             uint32_t n, uint32_t rank,
                                                             uint32_t* __restrict__ cursor,
                                                             uint32_t* __restrict__ rows,
                                                             uint32_t n_rows) {
    for (uint32_t i = blockIdx.x * BRD_THREADS + threadIdx.x; i < n; i += gridDim.x * BRD_THREADS) {
        if (owner[i] == rank) continue;
        const uint32_t row = atomicAdd(&cursor[owner[i]], 1u);
        if (row < n_rows) rows[row] = i;
    }
}

// tile = [S 512][W 512][key lo, key hi, 0, 0]; 256 lanes move two voxels each as float2
__global__ __launch_bounds__(BRD_THREADS) void k_border_pack(Table T, Pool Pl, float bg,
                                                             const uint32_t* __restrict__ rows,
                                                             uint32_t* __restrict__ send, int reset) {
    const uint32_t slot = rows[blockIdx.x];
    uint32_t* tile = send + (size_t)blockIdx.x * TILE_WORDS;
    float2* S = reinterpret_cast<float2*>(Pl.sdf + (size_t)slot * BRICK_VOX);
    float2* W = reinterpret_cast<float2*>(Pl.weight + (size_t)slot * BRICK_VOX);
    const int l = threadIdx.x;
    const float2 s = S[l], w = W[l];
    reinterpret_cast<float2*>(tile)[l] = s;
    reinterpret_cast<float2*>(tile + BRICK_VOX)[l] = w;
    if (reset) {
        S[l] = make_float2(bg, bg);
        W[l] = make_float2(0.0f, 0.0f);
    }
    if (l == 0) {
        const uint64_t key = T.brick_keys[slot];
        reinterpret_cast<uint4*>(tile + 2 * BRICK_VOX)[0] =
            make_uint4((uint32_t)key, (uint32_t)(key >> 32), 0u, 0u);
    }
}

__global__ __launch_bounds__(BRD_THREADS) void k_border_reset(Pool Pl, float bg,
                                                              const uint32_t* __restrict__ rows) {
    const uint32_t slot = rows[blockIdx.x];
    float2* S = reinterpret_cast<float2*>(Pl.sdf + (size_t)slot * BRICK_VOX);
    float2* W = reinterpret_cast<float2*>(Pl.weight + (size_t)slot * BRICK_VOX);
    S[threadIdx.x] = make_float2(bg, bg);
    W[threadIdx.x] = make_float2(0.0f, 0.0f);
}

__global__ __launch_bounds__(BRD_THREADS) void k_border_merge(Table T, Pool Pl,
                                                              const uint32_t* __restrict__ recv,
                                                              Globals* G, float max_w) {
    const uint32_t* tile = recv + (size_t)blockIdx.x * TILE_WORDS;
    const uint64_t key = (uint64_t)tile[2 * BRICK_VOX] | ((uint64_t)tile[2 * BRICK_VOX + 1] << 32);
    const int64_t h = table_find(T, key);  // every lane finds the same entry (no LDS broadcast)
    const uint32_t slot = h < 0 ? UNASSIGNED : T.slots[h];
    if (slot >= T.max_bricks) {
        if (threadIdx.x == 0) atomicOr(&G->overflow, ERR_MERGE_KEY);
        return;
    }
    const float* s_in = reinterpret_cast<const float*>(tile);
    const float* w_in = reinterpret_cast<const float*>(tile + BRICK_VOX);
    for (int l = threadIdx.x; l < BRICK_VOX; l += BRD_THREADS) {
        const float wi = w_in[l];
        if (!(wi > 0.0f)) continue;
        float* S = Pl.sdf + (size_t)slot * BRICK_VOX + l;
        float* W = Pl.weight + (size_t)slot * BRICK_VOX + l;
        const float w0 = *W;
        if (w0 == 0.0f) {  // unobserved here: copy (single-holder voxels stay bit-exact)
            *S = s_in[l];
            *W = wi;
            continue;
        }
        const float nw = w0 + wi;
        *S = (*S * w0 + s_in[l] * wi) / nw;
        *W = nw > max_w ? max_w : nw;  // Voxblox: capped at max_weight (else +inf)
    }
}

int grid_of(uint64_t items) {
    const uint64_t g = (items + BRD_THREADS - 1) / BRD_THREADS;
    return (int)(g < 1 ? 1 : (g > 65535 ? 65535 : g));
}

}  // namespace

hipError_t launch_border_owner(const Table& T, uint32_t n_bricks, const uint64_t* d_all_keys,
                               const WorldCounts& counts, uint64_t stride, uint32_t rank,
                               uint32_t* d_owner, uint32_t* d_dest_n, hipStream_t st) {
    k_border_init<<<grid_of(std::max<uint64_t>(n_bricks, MAX_WORLD)), BRD_THREADS, 0, st>>>(
        d_owner, n_bricks, rank, d_dest_n);
    for (uint32_t r = 0; r < rank; r++)
        if (counts.n[r])
            k_border_owner<<<grid_of(counts.n[r]), BRD_THREADS, 0, st>>>(
                T, d_all_keys + (size_t)r * stride, counts.n[r], r, d_owner);
    if (n_bricks)
        k_border_count<<<grid_of(n_bricks), BRD_THREADS, 0, st>>>(d_owner, n_bricks, rank,
                                                                  d_dest_n);
    return hipGetLastError();
}

hipError_t launch_border_pack(const Table& T, const Pool& Pl, float bg, uint32_t n_bricks,
                              uint32_t rank, const uint32_t* d_owner, uint32_t* d_cursor,
                              uint32_t* d_rows, uint32_t n_rows, uint32_t* d_send,
                              bool reset, hipStream_t st) {
    if (!n_rows) return hipSuccess;
    k_border_list<<<grid_of(n_bricks), BRD_THREADS, 0, st>>>(d_owner, n_bricks, rank, d_cursor,
                                                             d_rows, n_rows);
    k_border_pack<<<n_rows, BRD_THREADS, 0, st>>>(T, Pl, bg, d_rows, d_send, reset ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_border_reset(const Pool& Pl, float bg, const uint32_t* d_rows, uint32_t n_rows,
                               hipStream_t st) {
    if (!n_rows) return hipSuccess;
    static_assert(BRICK_VOX == 2 * BRD_THREADS, "two voxels per lane");
    k_border_reset<<<n_rows, BRD_THREADS, 0, st>>>(Pl, bg, d_rows);
    return hipGetLastError();
}

hipError_t launch_border_merge(const Table& T, const Pool& Pl, const uint32_t* d_recv,
                               uint64_t n_rows, Globals* G, float max_w, hipStream_t st) {
    for (uint64_t r0 = 0; r0 < n_rows; r0 += (1u << 30)) {
        const uint64_t nr = std::min<uint64_t>(n_rows - r0, 1u << 30);
        k_border_merge<<<(uint32_t)nr, BRD_THREADS, 0, st>>>(T, Pl, d_recv + r0 * TILE_WORDS, G,
                                                             max_w);
    }
    return hipGetLastError();
}

}  // namespace tsdf
