// Accuracy of the hardware double square root (v_sqrt_f64, __builtin_amdgcn_sqrt) against the
// correctly rounded sqrt (LLVM's lowering of __builtin_sqrt), and of the float-result shortcut
// built on it (tsdf_ray.h vdb_sqrt_f): f = (float)v_sqrt_f64(x), trusted unless the residual
// x_sqrt - f lies within 2^-20 of half a float ulp (then the exact sequence runs).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o sqrt_check sqrt_check.hip
// Prints the largest |hw - ref| in double ulps, how often the shortcut deferred, and the count of
// wrong float results it did not defer (must be 0).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ inline uint64_t mix(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
    return k;
}

__global__ void k(uint64_t seed, uint64_t n, unsigned long long* out) {
    unsigned long long maxulp = 0, deferred = 0, wrong = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix(seed ^ (i * 0x9e3779b97f4a7c15ull));
        // exponent in [-80, 40], random 52-bit mantissa
        const int e = (int)(h >> 52) % 121 - 80;
        const uint64_t bits = ((uint64_t)(e + 1023) << 52) | (mix(h) & 0xFFFFFFFFFFFFFull);
        const double x = __builtin_bit_cast(double, bits);
        const double ref = __builtin_sqrt(x);
        const double hw = __builtin_amdgcn_sqrt(x);
        const int64_t d = (int64_t)__builtin_bit_cast(uint64_t, hw) - (int64_t)__builtin_bit_cast(uint64_t, ref);
        const unsigned long long ad = (unsigned long long)(d < 0 ? -d : d);
        maxulp = ad > maxulp ? ad : maxulp;
        const float f = (float)hw;
        const float res = (float)(hw - (double)f);
        const uint32_t fb = __builtin_bit_cast(uint32_t, f);
        const float hu = __builtin_bit_cast(float, (fb & 0x7F800000u) - (24u << 23));
        const bool open = !(__builtin_fabsf(res) < hu * 0.99999905f);
        deferred += open ? 1 : 0;
        wrong += (!open && f != (float)ref) ? 1 : 0;
    }
    atomicMax(&out[0], maxulp);
    atomicAdd(&out[1], deferred);
    atomicAdd(&out[2], wrong);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 24);
    hipMemset(d, 0, 24);
    const uint64_t n = 1ull << 33;
    for (int s = 0; s < 4; s++) k<<<8192, 256>>>(0x1234567ull + s * 977, n / 4, d);
    unsigned long long h[3];
    hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    printf("samples %llu max_ulp %llu deferred %llu wrong_undeferred %llu\n",
           (unsigned long long)n, h[0], h[1], h[2]);
    return h[2] ? 1 : 0;
}
