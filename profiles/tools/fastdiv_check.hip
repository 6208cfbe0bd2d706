// Exhaustive check of the range-safe fp32 division used by k_integrate's fuse chains:
//   y = rcp(d) refined by one Newton step, q0 = n * y, r = fma(-d, q0, n), q = fma(r, y, q0)
// (1) y == RN(1/d) for every mantissa of d at exponents -40..40 (Markstein's condition);
// (2) q == RN(n / d) (IEEE division) for random (n, d) pairs of both fusion rules' ranges.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float recip_rn(float d) {
    const float r = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, r, 1.0f);
    return __builtin_fmaf(r, e, r);
}
__device__ __forceinline__ float div_fast(float n, float d, float y) {
    const float q0 = n * y;
    const float r = __builtin_fmaf(-d, q0, n);
    return __builtin_fmaf(r, y, q0);
}
__global__ void k_recip(int e0, unsigned long long* bad, float* ex) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;  // 2^23 mantissas
    const int e = e0 + (int)blockIdx.y;
    const float d = __builtin_ldexpf(1.0f + (float)m * (1.0f / 8388608.0f), e);
    const float y = recip_rn(d);
    const float ref = 1.0f / d;
    if (__float_as_uint(y) != __float_as_uint(ref)) {
        if (atomicAdd(bad, 1ull) < 4) ex[0] = d;
    }
}
__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__global__ void k_div(uint32_t seed, int mode, unsigned long long* bad, float* ex) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h1 = hash(i * 2654435761u + seed), h2 = hash(h1 ^ 0x9e3779b9u), h3 = hash(h2 + i);
    float d, n;
    if (mode == 0) {  // VDBFusion: integer weights W + B in [1, 2^24], n = S W + A
        d = (float)(1u + (h1 & 0xFFFFFFu));
        const float s = ((float)(h2 & 0xFFFFFF) / 16777216.0f - 0.5f) * 0.4f;
        n = s * d + __builtin_ldexpf((float)(int)(h3 & 0x7FFFFFFF) - 1073741824.0f, -32 + (int)(h3 >> 27));
    } else {  // any normal d and n over wide exponent ranges (Voxblox weights are not integers)
        d = __builtin_ldexpf(1.0f + (float)(h1 & 0x7FFFFF) / 8388608.0f, (int)(h1 >> 23) % 40 - 20);
        n = __builtin_ldexpf(1.0f + (float)(h2 & 0x7FFFFF) / 8388608.0f, (int)(h2 >> 23) % 60 - 30);
        if (h3 & 1) n = -n;
    }
    const float q = div_fast(n, d, recip_rn(d));
    const float ref = n / d;
    if (__float_as_uint(q) != __float_as_uint(ref)) {
        if (atomicAdd(bad, 1ull) < 4) { ex[1] = n; ex[2] = d; }
    }
}
int main() {
    unsigned long long* bad; float* ex;
    hipMalloc(&bad, 8); hipMalloc(&ex, 16);
    hipMemset(bad, 0, 8);
    k_recip<<<dim3(8388608 / 256, 81), 256>>>(-40, bad, ex);
    unsigned long long h = 0; float he[4] = {0, 0, 0, 0};
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(he, ex, 16, hipMemcpyDeviceToHost);
    printf("recip: %llu mismatches of %llu (e.g. d=%a)\n", h, 8388608ull * 81, he[0]);
    for (int mode = 0; mode < 2; mode++) {
        hipMemset(bad, 0, 8);
        unsigned long long n = 0;
        for (uint32_t s = 0; s < 64; s++) {
            k_div<<<(1u << 24) / 256, 256>>>(s * 0x51ed27u + 17u, mode, bad, ex);
            n += 1u << 24;
        }
        hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(he, ex, 16, hipMemcpyDeviceToHost);
        printf("div mode %d: %llu mismatches of %llu (e.g. n=%a d=%a)\n", mode, h, n, he[1], he[2]);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
