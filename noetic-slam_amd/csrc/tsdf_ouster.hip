// tsdf_ouster.hip — Ouster lidar packets to the integrate input on the GPU:
//   k_os_decode  UDP lidar packets of one frame -> staggered field images (h x w, row-major),
//                the Ouster SDK's packet layouts (ouster_client/src/parsing.cpp:42-175) and its
//                ScanBatcher rule (ouster_client/src/lidar_scan.cpp:540-633): a column goes to its
//                measurement_id, columns with status bit 0 clear are dropped, missing ones stay 0;
//   k_os_xyz     range image + xyz LUT (lidar_scan.cpp:297-382 make_xyz_lut) -> world points,
//                xyz = r dir + off (ouster/impl/cartesian.h:55-70; r = 0 -> the sensor origin,
//                which the integrate's range filter drops), then the scan pose (fp32, 3x4).
// One lane per pixel of one packet column: the column's header is read once per lane (broadcast
// in L1), the pixel fields are byte-gathered (layouts are byte-packed, not aligned).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsdf_device.h"

namespace tsdf {

__device__ __forceinline__ uint32_t le_bytes(const uint8_t* p, uint32_t n) {
    uint32_t v = 0;
    for (uint32_t k = 0; k < n; k++) v |= (uint32_t)p[k] << (8 * k);
    return v;
}

__global__ void k_os_decode(const uint8_t* __restrict__ pk, uint32_t n_packets, OsLayout L,
                            uint32_t* __restrict__ out0, uint32_t* __restrict__ out1,
                            uint32_t* __restrict__ out2, uint32_t* __restrict__ out3) {
    const uint32_t col = blockIdx.x % L.cols_per_packet, p = blockIdx.x / L.cols_per_packet;
    if (p >= n_packets) return;
    const uint8_t* cb = pk + (size_t)p * L.packet_bytes + L.packet_header + col * L.col_bytes;
    const uint32_t m_id = le_bytes(cb + 8, 2);
    const uint32_t status = L.legacy ? le_bytes(cb + L.col_bytes - 4, 4) : le_bytes(cb + 10, 2);
    if (m_id >= L.w || !(status & 1u)) return;
    uint32_t* out[4] = {out0, out1, out2, out3};
    for (uint32_t px = threadIdx.x; px < L.h; px += blockDim.x) {
        const uint8_t* pb = cb + L.col_header + px * L.pixel_bytes;
#pragma unroll
        for (int f = 0; f < 4; f++) {
            if (!out[f] || !L.f[f].nbytes) continue;
            uint32_t v = le_bytes(pb + L.f[f].offset, L.f[f].nbytes);
            if (L.f[f].mask) v &= L.f[f].mask;
            if (L.f[f].shift > 0) v >>= L.f[f].shift;
            if (L.f[f].shift < 0) v <<= -L.f[f].shift;
            out[f][(size_t)px * L.w + m_id] = v;
        }
    }
}

__global__ void k_os_xyz(const uint32_t* __restrict__ rng, uint64_t n,
                         const float* __restrict__ dir, const float* __restrict__ off, OsPose P,
                         float* __restrict__ xyz) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = rng[i];
        float x = 0.0f, y = 0.0f, z = 0.0f;
        if (r != 0u) {
            const float rf = (float)r;
            x = rf * dir[3 * i] + off[3 * i];
            y = rf * dir[3 * i + 1] + off[3 * i + 1];
            z = rf * dir[3 * i + 2] + off[3 * i + 2];
        }
        xyz[3 * i] = P.m[0] * x + P.m[1] * y + P.m[2] * z + P.m[3];
        xyz[3 * i + 1] = P.m[4] * x + P.m[5] * y + P.m[6] * z + P.m[7];
        xyz[3 * i + 2] = P.m[8] * x + P.m[9] * y + P.m[10] * z + P.m[11];
    }
}

hipError_t launch_os_decode(const uint8_t* d_packets, uint32_t n_packets, const OsLayout& L,
                            uint32_t* const out[4], hipStream_t st) {
    if (n_packets == 0) return hipSuccess;
    const uint32_t threads = L.h >= 128 ? 128u : 64u;
    k_os_decode<<<n_packets * L.cols_per_packet, threads, 0, st>>>(d_packets, n_packets, L, out[0],
                                                                  out[1], out[2], out[3]);
    return hipGetLastError();
}

hipError_t launch_os_xyz(const uint32_t* d_range, uint64_t n, const float* d_dir,
                         const float* d_off, const OsPose& P, float* d_xyz, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t g = (n + 255) / 256;
    k_os_xyz<<<(int)(g < 8192 ? g : 8192), 256, 0, st>>>(d_range, n, d_dir, d_off, P, d_xyz);
    return hipGetLastError();
}

}  // namespace tsdf
