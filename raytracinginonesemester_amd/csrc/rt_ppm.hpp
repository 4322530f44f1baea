// rt_ppm.hpp — write_p6's per-sample conversion (HW1/ppm_p6_lib/src/ppm_p6.cpp:137-155),
// shared by the frame epilogue kernels (rt_frame.hip) and the render kernels' fused P6 output
// (rt_device.hip): double(sample) -> [max(0,x) -> sqrt] -> [clamp to [0,1]] -> * maxval ->
// std::lround -> clamp to [0, maxval].  HIP's double sqrt is correctly rounded, as glibc's is.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace rtp {

// std::lround as glibc computes it on x86-64: nearest integer, halves away from zero; a NaN or
// a value outside long's range converts to LONG_MIN (the x86 "integer indefinite"), which the
// caller's `rounded < 0` check turns into 0.
__host__ __device__ __forceinline__ uint32_t float_to_sample(float f, int maxval, bool clamp, bool gamma2) {
    double x = (double)f;
    if (gamma2) {
        if (x < 0.0) x = 0.0;
        x = sqrt(x);
    }
    if (clamp) {
        if (x < 0.0) x = 0.0;
        if (x > 1.0) x = 1.0;
    }
    const double s = x * (double)maxval;
    if (!(fabs(s) < 9223372036854775808.0)) return 0u;
    const double r = round(s);
    if (r < 0.0) return 0u;
    if (r > (double)maxval) return (uint32_t)maxval;
    return (uint32_t)r;
}

// write_p6's defaults (maxval 255, clamp, sqrt gamma): one byte per sample.
__host__ __device__ __forceinline__ uint8_t p6_default_sample(float f) {
    return (uint8_t)float_to_sample(f, 255, true, true);
}

}  // namespace rtp
