// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes of the TSDF
// kernels (MI355X_MICROARCH.md: FETCH_SIZE is exactly 1/2 of a 16-B/lane streaming read; other
// widths are uncalibrated).  Each kernel moves a known number of bytes of a 1 GiB buffer (far
// beyond the 256 MiB Infinity Cache) once, with one access shape; run it under
//   rocprofv3 --pmc FETCH_SIZE  -- ./fetch_calib     and     rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// and divide each kernel's counter (KiB) by the bytes it prints.  profiles/summarize_calib.py does.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint64_t BYTES = 1ull << 30;

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// reads: contiguous 4 / 8 / 12 (3 dwords, stride 12) / 16 B per lane
__global__ void rd4(const uint32_t* p, uint64_t n, uint32_t* out) {
    uint32_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 0x12345678u) out[0] = s;
}
__global__ void rd8(const uint2* p, uint64_t n, uint32_t* out) {
    uint32_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint2 v = p[i];
        s += v.x ^ v.y;
    }
    if (s == 0x12345678u) out[0] = s;
}
__global__ void rd12(const float* p, uint64_t n, uint32_t* out) {
    uint32_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        s += __float_as_uint(p[3 * i]) ^ __float_as_uint(p[3 * i + 1]) ^ __float_as_uint(p[3 * i + 2]);
    if (s == 0x12345678u) out[0] = s;
}
__global__ void rd16(const uint4* p, uint64_t n, uint32_t* out) {
    uint32_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) out[0] = s;
}
// random 4-B gathers (one per 64-B line touched: n lines of the buffer, each once)
__global__ void gather4(const uint32_t* p, uint64_t lines, uint32_t* out) {
    uint32_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t l = (hash32((uint32_t)i) % (uint32_t)lines);  // a permutation-ish spread
        s += p[l * 16];
    }
    if (s == 0x12345678u) out[0] = s;
}
// writes: contiguous 4 / 8 / 16 B per lane, and 8-B writes in runs of 12 (k_place's copy-out shape)
__global__ void wr4(uint32_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = (uint32_t)i;
}
__global__ void wr8(uint2* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = make_uint2((uint32_t)i, 1u);
}
__global__ void wr16(uint4* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
// 8-B records, lane j of a wave writes record perm(j): runs of ~12 consecutive records at
// scattered run starts (the sample runs of k_place's copy-out), every record written once
__global__ void wr8runs(uint2* p, uint64_t n) {
    const uint64_t runs = n / 12;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < runs * 12; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = i / 12, k = i % 12;
        const uint64_t rr = hash32((uint32_t)r) % (uint32_t)runs;  // scattered run order
        p[rr * 12 + k] = make_uint2((uint32_t)i, 2u);
    }
}

int main() {
    void* buf;
    uint32_t* out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, BYTES);
    const int G = 8192, T = 256;
    // 12-B reads cover 3 * n floats: n = BYTES / 12
    rd4<<<G, T>>>((const uint32_t*)buf, BYTES / 4, out);
    rd8<<<G, T>>>((const uint2*)buf, BYTES / 8, out);
    rd12<<<G, T>>>((const float*)buf, BYTES / 12, out);
    rd16<<<G, T>>>((const uint4*)buf, BYTES / 16, out);
    gather4<<<G, T>>>((const uint32_t*)buf, BYTES / 64, out);
    wr4<<<G, T>>>((uint32_t*)buf, BYTES / 4);
    wr8<<<G, T>>>((uint2*)buf, BYTES / 8);
    wr16<<<G, T>>>((uint4*)buf, BYTES / 16);
    wr8runs<<<G, T>>>((uint2*)buf, BYTES / 8);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes\": {\"rd4\": %llu, \"rd8\": %llu, \"rd12\": %llu, \"rd16\": %llu, "
           "\"gather4_lines\": %llu, \"wr4\": %llu, \"wr8\": %llu, \"wr16\": %llu, \"wr8runs\": %llu}}\n",
           (unsigned long long)BYTES, (unsigned long long)BYTES,
           (unsigned long long)(BYTES / 12 * 12), (unsigned long long)BYTES,
           (unsigned long long)(BYTES / 64), (unsigned long long)BYTES, (unsigned long long)BYTES,
           (unsigned long long)BYTES, (unsigned long long)(BYTES / 8 / 12 * 12 * 8));
    return 0;
}
