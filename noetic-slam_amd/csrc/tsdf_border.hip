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
//   k_border_snapshot / k_border_restore  (ABI v9) the owner's bricks a merge will touch, copied as
//                   tiles before the merge and written back if the reduce is aborted, so a reduce
//                   that fails on any rank leaves every field as it was, bit for bit
// Mesh halo (ABI v9): after a reduce every brick's mass sits on one rank, but a
// cube on a brick's +x / +y / +z face needs voxels of its neighbour bricks, which may live on
// another rank:
//   k_brick_observed  per pool slot: does the brick hold an observed voxel (W > 0)
//   k_halo_pack       one workgroup per requested key: the brick's tile when it is observed here
//   k_halo_build      the received halo tiles as a small hash table + pool (the mesh's second
//                     lookup, tsdf_mesh.hip)
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

// the brick of every received tile, as it is before the merge: (S, W, key); a key the table lacks
// is written as EMPTY_KEY (the merge flags it; nothing to restore)
__global__ __launch_bounds__(BRD_THREADS) void k_border_snapshot(Table T, Pool Pl,
                                                                 const uint32_t* __restrict__ recv,
                                                                 uint32_t* __restrict__ bk) {
    const uint32_t* tile = recv + (size_t)blockIdx.x * TILE_WORDS;
    uint32_t* out = bk + (size_t)blockIdx.x * TILE_WORDS;
    const uint64_t key = (uint64_t)tile[2 * BRICK_VOX] | ((uint64_t)tile[2 * BRICK_VOX + 1] << 32);
    const int64_t h = table_find(T, key);
    const uint32_t slot = h < 0 ? UNASSIGNED : T.slots[h];
    const bool ok = slot < T.max_bricks;
    const int l = threadIdx.x;
    if (ok) {
        reinterpret_cast<float2*>(out)[l] =
            reinterpret_cast<const float2*>(Pl.sdf + (size_t)slot * BRICK_VOX)[l];
        reinterpret_cast<float2*>(out + BRICK_VOX)[l] =
            reinterpret_cast<const float2*>(Pl.weight + (size_t)slot * BRICK_VOX)[l];
    }
    if (l == 0) {
        const uint64_t k = ok ? key : EMPTY_KEY;
        reinterpret_cast<uint4*>(out + 2 * BRICK_VOX)[0] =
            make_uint4((uint32_t)k, (uint32_t)(k >> 32), 0u, 0u);
    }
}

// a snapshot written back (every snapshot of one brick holds the same pre-merge values)
__global__ __launch_bounds__(BRD_THREADS) void k_border_restore(Table T, Pool Pl,
                                                                const uint32_t* __restrict__ bk) {
    const uint32_t* tile = bk + (size_t)blockIdx.x * TILE_WORDS;
    const uint64_t key = (uint64_t)tile[2 * BRICK_VOX] | ((uint64_t)tile[2 * BRICK_VOX + 1] << 32);
    if (key == EMPTY_KEY) return;
    const int64_t h = table_find(T, key);
    const uint32_t slot = h < 0 ? UNASSIGNED : T.slots[h];
    if (slot >= T.max_bricks) return;
    const int l = threadIdx.x;
    reinterpret_cast<float2*>(Pl.sdf + (size_t)slot * BRICK_VOX)[l] =
        reinterpret_cast<const float2*>(tile)[l];
    reinterpret_cast<float2*>(Pl.weight + (size_t)slot * BRICK_VOX)[l] =
        reinterpret_cast<const float2*>(tile + BRICK_VOX)[l];
}

// obs[slot] = 1 when brick `slot` holds a voxel with W > 0 (one wave per brick, 8 voxels a lane)
__global__ __launch_bounds__(BRD_THREADS) void k_brick_observed(Pool Pl, uint32_t n,
                                                                uint32_t* __restrict__ obs) {
    const uint32_t b = blockIdx.x * (BRD_THREADS / 64) + (threadIdx.x >> 6);
    if (b >= n) return;  // wave-uniform
    const float* W = Pl.weight + (size_t)b * BRICK_VOX;
    bool any = false;
#pragma unroll
    for (int k = 0; k < BRICK_VOX / 64; k++) any |= W[(threadIdx.x & 63) + 64 * k] > 0.0f;
    const bool v = __any(any);
    if ((threadIdx.x & 63) == 0) obs[b] = v ? 1u : 0u;
}

// one workgroup per requested key: its tile (S, W, key) goes to the next send row when the brick
// is observed here (row order is atomic order: the receiver looks tiles up by key)
__global__ __launch_bounds__(BRD_THREADS) void k_halo_pack(Table T, Pool Pl,
                                                           const uint64_t* __restrict__ req,
                                                           uint32_t* __restrict__ send,
                                                           uint32_t cap_rows,
                                                           uint32_t* __restrict__ n_rows) {
    __shared__ uint32_t s_row;
    const uint64_t key = req[blockIdx.x];
    const int64_t h = key == EMPTY_KEY ? -1 : table_find(T, key);
    const uint32_t slot = h < 0 ? UNASSIGNED : T.slots[h];
    if (slot >= T.max_bricks) return;  // uniform
    const int l = threadIdx.x;
    const float2 s = reinterpret_cast<const float2*>(Pl.sdf + (size_t)slot * BRICK_VOX)[l];
    const float2 w = reinterpret_cast<const float2*>(Pl.weight + (size_t)slot * BRICK_VOX)[l];
    if (!__syncthreads_or(w.x > 0.0f || w.y > 0.0f)) return;  // not observed here
    if (l == 0) s_row = atomicAdd(n_rows, 1u);
    __syncthreads();
    const uint32_t row = s_row;
    if (row >= cap_rows) return;  // counted: the caller sees the overflow
    uint32_t* tile = send + (size_t)row * TILE_WORDS;
    reinterpret_cast<float2*>(tile)[l] = s;
    reinterpret_cast<float2*>(tile + BRICK_VOX)[l] = w;
    if (l == 0)
        reinterpret_cast<uint4*>(tile + 2 * BRICK_VOX)[0] =
            make_uint4((uint32_t)key, (uint32_t)(key >> 32), 0u, 0u);
}

// halo tiles -> (H, HP): row i's key inserted with slot i, its S and W unpacked to HP's planes
__global__ __launch_bounds__(BRD_THREADS) void k_halo_build(Table H, Pool HP,
                                                            const uint32_t* __restrict__ tiles,
                                                            uint32_t* __restrict__ ovf) {
    const uint32_t* tile = tiles + (size_t)blockIdx.x * TILE_WORDS;
    const int l = threadIdx.x;
    reinterpret_cast<float2*>(HP.sdf + (size_t)blockIdx.x * BRICK_VOX)[l] =
        reinterpret_cast<const float2*>(tile)[l];
    reinterpret_cast<float2*>(HP.weight + (size_t)blockIdx.x * BRICK_VOX)[l] =
        reinterpret_cast<const float2*>(tile + BRICK_VOX)[l];
    if (l == 0) {
        const uint64_t key = (uint64_t)tile[2 * BRICK_VOX] | ((uint64_t)tile[2 * BRICK_VOX + 1] << 32);
        const int64_t h = table_insert(H, key, ovf);
        if (h >= 0) H.slots[h] = blockIdx.x;
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

hipError_t launch_border_snapshot(const Table& T, const Pool& Pl, const uint32_t* d_recv,
                                  uint64_t n_rows, uint32_t* d_backup, hipStream_t st) {
    for (uint64_t r0 = 0; r0 < n_rows; r0 += (1u << 30)) {
        const uint64_t nr = std::min<uint64_t>(n_rows - r0, 1u << 30);
        k_border_snapshot<<<(uint32_t)nr, BRD_THREADS, 0, st>>>(T, Pl, d_recv + r0 * TILE_WORDS,
                                                                d_backup + r0 * TILE_WORDS);
    }
    return hipGetLastError();
}

hipError_t launch_border_restore(const Table& T, const Pool& Pl, const uint32_t* d_backup,
                                 uint64_t n_rows, hipStream_t st) {
    for (uint64_t r0 = 0; r0 < n_rows; r0 += (1u << 30)) {
        const uint64_t nr = std::min<uint64_t>(n_rows - r0, 1u << 30);
        k_border_restore<<<(uint32_t)nr, BRD_THREADS, 0, st>>>(T, Pl, d_backup + r0 * TILE_WORDS);
    }
    return hipGetLastError();
}

hipError_t launch_brick_observed(const Pool& Pl, uint32_t n_bricks, uint32_t* d_obs,
                                 hipStream_t st) {
    if (!n_bricks) return hipSuccess;
    constexpr uint32_t per = BRD_THREADS / 64;
    k_brick_observed<<<(n_bricks + per - 1) / per, BRD_THREADS, 0, st>>>(Pl, n_bricks, d_obs);
    return hipGetLastError();
}

hipError_t launch_halo_pack(const Table& T, const Pool& Pl, const uint64_t* d_req, uint32_t n_req,
                            uint32_t* d_send, uint32_t cap_rows, uint32_t* d_n_rows,
                            hipStream_t st) {
    if (!n_req) return hipSuccess;
    k_halo_pack<<<n_req, BRD_THREADS, 0, st>>>(T, Pl, d_req, d_send, cap_rows, d_n_rows);
    return hipGetLastError();
}

hipError_t launch_halo_build(const Table& H, const Pool& HP, const uint32_t* d_tiles,
                             uint32_t n_rows, uint32_t* d_ovf, hipStream_t st) {
    if (!n_rows) return hipSuccess;
    k_halo_build<<<n_rows, BRD_THREADS, 0, st>>>(H, HP, d_tiles, d_ovf);
    return hipGetLastError();
}

}  // namespace tsdf
