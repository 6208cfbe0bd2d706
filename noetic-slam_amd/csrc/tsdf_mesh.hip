// tsdf_mesh.hip — marching-cubes mesh extraction over the brick pool (SURVEY.md §8f.1;
// VDBFusion's VDBVolume::extract_triangle_mesh, restated with the oracle's semantics in
// oracle/tsdf_oracle.c tsdf_extract_mesh).
//
// One 512-lane workgroup per brick (in (z, y, x) brick order, given by the host): the brick and
// its +x / +y / +z halo — a 9^3 tile of (S, W) from up to 8 bricks, found with table lookups —
// are staged in LDS; lane l meshes the cube whose min voxel is in-brick voxel l (2 x 2 x 2 voxels,
// all observed with W >= min_weight).  Corner c is inside when S < 0; the case's triangles come
// from the generated table (tsdf_capi.cpp build_mc_table); a vertex on edge (a, b) is corner a's
// centre + t vs along the edge's axis, t = S_a / (S_a - S_b).
//   k_mesh_count  triangles per brick  -> host exclusive prefix -> offsets
//   k_mesh_emit   a block scan over the lanes' counts places every triangle: the soup is
//                 ordered by brick, then cube, then table order (the oracle's order).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsdf_device.h"
#include "tsdf_ray.h"

namespace tsdf {

__constant__ uint8_t c_mc[MC_TABLES][256][32];  // per table (TSDF_MC_*): [case][0] = triangles, then 3 edge ids each
__constant__ uint8_t c_edge[12][2];  // edge -> corners (a, b), b = a | axis bit

constexpr int MESH_THREADS = 512;
constexpr int TILE = 9;

// Stage the 9^3 tile of brick `key`: s_ok[t] = observed (W > 0, W >= min_weight).  A neighbour is
// looked up in the halo (H, HP) first -- bricks another rank owns after a border reduce, of which
// this context may hold a reset copy -- then in the context's own table; the brick itself only in
// the own table.
__device__ void mesh_tile(const Table& T, const Pool& Pl, const Table& H, const Pool& HP,
                          uint64_t key, float min_weight, float* s_S, uint8_t* s_ok,
                          uint32_t* s_slot) {
    const int bx = (int)(key & 0x1FFFFFu) - BRICK_COORD_BIAS;
    const int by = (int)((key >> 21) & 0x1FFFFFu) - BRICK_COORD_BIAS;
    const int bz = (int)((key >> 42) & 0x1FFFFFu) - BRICK_COORD_BIAS;
    if (threadIdx.x < 8) {  // the brick and its 7 +x/+y/+z neighbours
        const int dx = threadIdx.x & 1, dy = (threadIdx.x >> 1) & 1, dz = threadIdx.x >> 2;
        uint32_t slot = INVALID_SLOT, src = 0u;
        const int nx = bx + dx, ny = by + dy, nz = bz + dz;
        if (nx < BRICK_COORD_BIAS && ny < BRICK_COORD_BIAS && nz < BRICK_COORD_BIAS) {
            const uint64_t nk = pack_brick(nx, ny, nz);
            // the brick itself always from the own table: a reset copy of a brick owned elsewhere
            // is meshed by its owner (its halo copy would mesh its cubes twice)
            if (H.keys && threadIdx.x != 0) {
                const int64_t h = table_find(H, nk);
                if (h >= 0) {
                    slot = H.slots[h];
                    src = 1u << 31;
                }
            }
            if (!src) {
                const int64_t h = table_find(T, nk);
                if (h >= 0) slot = T.slots[h];
            }
        }
        // bit 31: a halo slot (slots are < 2^31 in both pools)
        s_slot[threadIdx.x] = slot < T.max_bricks || src ? slot | src : INVALID_SLOT;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < TILE * TILE * TILE; t += MESH_THREADS) {
        const int tx = t % TILE, ty = (t / TILE) % TILE, tz = t / (TILE * TILE);
        const uint32_t ss = s_slot[(tx >> 3) | ((ty >> 3) << 1) | ((tz >> 3) << 2)];
        const bool halo = ss != INVALID_SLOT && (ss >> 31);
        const uint32_t slot = ss & 0x7FFFFFFFu;
        const Pool& P = halo ? HP : Pl;
        float S = 0.0f;
        uint8_t ok = 0;
        if (ss != INVALID_SLOT && slot < (halo ? H.max_bricks : T.max_bricks)) {
            const size_t i = (size_t)slot * BRICK_VOX + ((tz & 7) << 6) + ((ty & 7) << 3) + (tx & 7);
            const float W = P.weight[i];
            S = P.sdf[i];
            ok = (W > 0.0f && W >= min_weight) ? 1 : 0;
        }
        s_S[t] = S;
        s_ok[t] = ok;
    }
    __syncthreads();
}

// The cube of in-brick voxel l: case index, or -1 when a corner is unobserved.
__device__ __forceinline__ int mesh_case(const float* s_S, const uint8_t* s_ok, int l, float S[8]) {
    const int x = l & 7, y = (l >> 3) & 7, z = l >> 6;
    int k = 0;
    for (int q = 0; q < 8; q++) {
        const int t = (x + (q & 1)) + TILE * ((y + ((q >> 1) & 1)) + TILE * (z + (q >> 2)));
        if (!s_ok[t]) return -1;
        S[q] = s_S[t];
        k |= (S[q] < 0.0f ? 1 : 0) << q;
    }
    return k;
}

__global__ __launch_bounds__(MESH_THREADS) void k_mesh_count(Table T, Pool Pl, Table H, Pool HP,
                                                            const uint64_t* __restrict__ keys,
                                                            uint32_t nb, float min_weight,
                                                            uint32_t* __restrict__ counts, int tab) {
    __shared__ float s_S[TILE * TILE * TILE];
    __shared__ uint8_t s_ok[TILE * TILE * TILE];
    __shared__ uint32_t s_slot[8];
    __shared__ uint32_t s_sum;
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        if (threadIdx.x == 0) s_sum = 0u;
        mesh_tile(T, Pl, H, HP, keys[b], min_weight, s_S, s_ok, s_slot);
        float S[8];
        const int k = mesh_case(s_S, s_ok, threadIdx.x, S);
        const uint32_t nt = k >= 0 ? c_mc[tab][k][0] : 0u;
        const uint32_t w = wave_sum<uint32_t>(nt);
        if ((threadIdx.x & 63) == 0 && w) atomicAdd(&s_sum, w);
        __syncthreads();
        if (threadIdx.x == 0) counts[b] = s_sum;
        __syncthreads();
    }
}

__global__ __launch_bounds__(MESH_THREADS) void k_mesh_emit(Table T, Pool Pl, Table H, Pool HP,
                                                           const uint64_t* __restrict__ keys,
                                                           uint32_t nb, float min_weight, float vs,
                                                           const uint64_t* __restrict__ offsets, int tab,
                                                           float* __restrict__ tri) {
    __shared__ float s_S[TILE * TILE * TILE];
    __shared__ uint8_t s_ok[TILE * TILE * TILE];
    __shared__ uint32_t s_slot[8];
    __shared__ uint32_t s_w[MESH_THREADS / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint64_t key = keys[b];
        mesh_tile(T, Pl, H, HP, key, min_weight, s_S, s_ok, s_slot);
        float S[8];
        const int l = threadIdx.x;
        const int k = mesh_case(s_S, s_ok, l, S);
        const uint32_t nt = k >= 0 ? c_mc[tab][k][0] : 0u;
        // exclusive scan of the lanes' triangle counts (cube order)
        const uint32_t incl = wave_incl_scan(nt);
        if (lane == 63) s_w[wid] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int q = 0; q < wid; q++) off += s_w[q];
        __syncthreads();  // s_w and the tile are reused by the next brick
        if (nt) {
            const int bx = (int)(key & 0x1FFFFFu) - BRICK_COORD_BIAS;
            const int by = (int)((key >> 21) & 0x1FFFFFu) - BRICK_COORD_BIAS;
            const int bz = (int)((key >> 42) & 0x1FFFFFu) - BRICK_COORD_BIAS;
            const int x = bx * 8 + (l & 7), y = by * 8 + ((l >> 3) & 7), z = bz * 8 + (l >> 6);
            float* out = tri + 9 * (offsets[b] + off + incl - nt);
            for (uint32_t t = 0; t < nt; t++) {
                for (int j = 0; j < 3; j++) {
                    const int ed = c_mc[tab][k][1 + 3 * t + j];
                    const int a = c_edge[ed][0], bb = c_edge[ed][1];
                    const int ax = (a ^ bb) == 1 ? 0 : ((a ^ bb) == 2 ? 1 : 2);
                    const float tt = S[a] / (S[a] - S[bb]);
                    float p0 = ((float)(x + (a & 1)) + 0.5f) * vs;
                    float p1 = ((float)(y + ((a >> 1) & 1)) + 0.5f) * vs;
                    float p2 = ((float)(z + ((a >> 2) & 1)) + 0.5f) * vs;
                    if (ax == 0) p0 = p0 + tt * vs;
                    else if (ax == 1) p1 = p1 + tt * vs;
                    else p2 = p2 + tt * vs;
                    out[9 * t + 3 * j] = p0;
                    out[9 * t + 3 * j + 1] = p1;
                    out[9 * t + 3 * j + 2] = p2;
                }
            }
        }
    }
}

hipError_t upload_mc_table(const uint8_t tab[MC_TABLES][256][32], const uint8_t edge[12][2]) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_mc), tab, MC_TABLES * 256 * 32);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_edge), edge, 12 * 2);
    return e;
}

hipError_t launch_mesh_count(const Table& T, const Pool& Pl, const Table& H, const Pool& HP,
                             const uint64_t* d_keys, uint32_t nb, float min_weight, int tab,
                             uint32_t* d_counts, hipStream_t st) {
    if (nb == 0) return hipSuccess;
    const uint32_t grid = nb < 4096u ? nb : 4096u;
    k_mesh_count<<<grid, MESH_THREADS, 0, st>>>(T, Pl, H, HP, d_keys, nb, min_weight, d_counts,
                                                tab);
    return hipGetLastError();
}

hipError_t launch_mesh_emit(const Table& T, const Pool& Pl, const Table& H, const Pool& HP,
                            const uint64_t* d_keys, uint32_t nb, float min_weight, int tab,
                            float vs, const uint64_t* d_offsets, float* d_tri, hipStream_t st) {
    if (nb == 0) return hipSuccess;
    const uint32_t grid = nb < 4096u ? nb : 4096u;
    k_mesh_emit<<<grid, MESH_THREADS, 0, st>>>(T, Pl, H, HP, d_keys, nb, min_weight, vs,
                                               d_offsets, tab, d_tri);
    return hipGetLastError();
}

}  // namespace tsdf
