// rt_frame.hip — the frame epilogue on gfx950: P6 quantisation of a
// device framebuffer and the band un-permute of gathered strips, so that neither the float
// frame nor the strips have to cross PCIe before the image exists.
//
// Quantisation is write_p6's per-sample conversion (HW1/ppm_p6_lib/src/ppm_p6.cpp:137-155,
// row loop :284-299): double(sample) -> [max(0,x) -> sqrt] -> [clamp to [0,1]] -> * maxval ->
// std::lround -> clamp to [0, maxval]; one byte per sample for maxval < 256, two (big endian,
// write_sample) otherwise.  HIP's double sqrt is correctly rounded, as glibc's is, so the
// samples are the reference's bit for bit (tests/test_gpu_frame.py sweeps every rounding
// boundary of maxval 255).
//
// Both kernels are streaming copies: 12 B in, 3 B out per pixel (quantise); row_bytes in and out
// per row (un-permute).  HBM-bound; c5's 99.5 MB frame quantises in ~25 us at ~5 TB/s.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "rt_common.hpp"
#include "rt_hip_host.hpp"
#include "rt_ppm.hpp"

using rt::set_error;
using rt::hip_msg;

namespace {

constexpr int BLOCK = 256;
typedef float __attribute__((ext_vector_type(4))) vf4;
typedef uint32_t __attribute__((ext_vector_type(4))) vu4;

using rtp::float_to_sample;

struct QuantParams {
    const float* rgb;
    uint8_t* out;
    int64_t n;        // samples (rows * W * 3)
    int64_t row_len;  // samples per row (W * 3)
    int rows;
    int maxval;
    bool clamp, gamma2, flip;
};

// 16 consecutive samples per lane: four float4 loads, one 16-byte (maxval < 256) or two 16-byte
// stores.  Needs row order unchanged (no flip) and 16-byte aligned buffers; the host checks.
template <int BPS>
__global__ __launch_bounds__(BLOCK) void quantize_vec_kernel(QuantParams P) {
    const int64_t g = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const int64_t i0 = g * 16;
    if (i0 >= P.n) return;
    if (i0 + 16 > P.n) {  // ragged tail
        for (int64_t i = i0; i < P.n; ++i) {
            const uint32_t s = float_to_sample(P.rgb[i], P.maxval, P.clamp, P.gamma2);
            if (BPS == 1) P.out[i] = (uint8_t)s;
            else { P.out[2 * i] = (uint8_t)(s >> 8); P.out[2 * i + 1] = (uint8_t)(s & 0xFF); }
        }
        return;
    }
    const vf4* src = reinterpret_cast<const vf4*>(P.rgb + i0);
    float v[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const vf4 q = __builtin_nontemporal_load(src + k);
        v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
    }
    uint32_t w[BPS * 4];
#pragma unroll
    for (int k = 0; k < BPS * 4; ++k) w[k] = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t s = float_to_sample(v[k], P.maxval, P.clamp, P.gamma2);
        if (BPS == 1) {
            w[k >> 2] |= (s & 0xFFu) << (8 * (k & 3));
        } else {  // big endian pair per sample: bytes (hi, lo) at 2k, 2k+1
            const uint32_t be = ((s >> 8) & 0xFFu) | ((s & 0xFFu) << 8);
            w[k >> 1] |= be << (16 * (k & 1));
        }
    }
    vu4* dst = reinterpret_cast<vu4*>(P.out + i0 * BPS);
#pragma unroll
    for (int k = 0; k < BPS; ++k) dst[k] = (vu4){w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
}

// General case (flip_y, unaligned buffers): one sample per lane, output index order.
template <int BPS>
__global__ __launch_bounds__(BLOCK) void quantize_any_kernel(QuantParams P) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= P.n) return;
    int64_t src = i;
    if (P.flip) {
        const int64_t y = i / P.row_len;
        src = ((int64_t)P.rows - 1 - y) * P.row_len + (i - y * P.row_len);
    }
    const uint32_t s = float_to_sample(P.rgb[src], P.maxval, P.clamp, P.gamma2);
    if (BPS == 1) P.out[i] = (uint8_t)s;
    else { P.out[2 * i] = (uint8_t)(s >> 8); P.out[2 * i + 1] = (uint8_t)(s & 0xFF); }
}

// Frame row y (after the optional flip) comes from strip (band % count), row
// (band / count) * band_rows + y % band_rows of it — the strip layout rt_render_device writes
// for (band_rows, band_index, band_count).  One block per output row.
struct UnpermuteParams {
    const uint8_t* strips;
    uint8_t* frame;
    int64_t strip_stride;  // bytes between consecutive ranks' strips
    int64_t row_bytes;
    int height, band_rows, band_count;
    bool flip, vec;
};

__global__ __launch_bounds__(BLOCK) void unpermute_kernel(UnpermuteParams P) {
    const int y = (int)blockIdx.x;
    const int sy = P.flip ? P.height - 1 - y : y;
    const int band = sy / P.band_rows;
    const int rank = band % P.band_count;
    const int64_t k = (int64_t)(band / P.band_count) * P.band_rows + sy % P.band_rows;
    const uint8_t* src = P.strips + rank * P.strip_stride + k * P.row_bytes;
    uint8_t* dst = P.frame + (int64_t)y * P.row_bytes;
    if (P.vec) {
        const int64_t n16 = P.row_bytes >> 4;
        const vu4* s4 = reinterpret_cast<const vu4*>(src);
        vu4* d4 = reinterpret_cast<vu4*>(dst);
        for (int64_t j = threadIdx.x; j < n16; j += BLOCK) d4[j] = __builtin_nontemporal_load(s4 + j);
    } else {
        for (int64_t j = threadIdx.x; j < P.row_bytes; j += BLOCK) dst[j] = src[j];
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" int rt_ppm_header(int width, int height, int maxval, char* buf, size_t cap, size_t* written) {
    if (width <= 0 || height <= 0) return set_error(RT_ERR_ARG, "Image has non-positive dimensions.");
    if (maxval <= 0 || maxval > 65535) return set_error(RT_ERR_ARG, "Invalid maxval (must be 1..65535).");
    char h[64];
    const int n = std::snprintf(h, sizeof(h), "P6\n%d %d\n%d\n", width, height, maxval);
    if (written) *written = (size_t)n;
    if (!buf) return RT_OK;
    if (cap < (size_t)n) return set_error(RT_ERR_ARG, "rt_ppm_header: buffer too small");
    std::memcpy(buf, h, (size_t)n);
    return RT_OK;
}

extern "C" int rt_ppm_quantize_device(const float* rgb_dev, int width, int rows, const rt_ppm_options* opt,
                                      uint8_t* out_dev, void* hip_stream) {
    rt_ppm_options d;
    rt_ppm_options_default(&d);
    if (!opt) opt = &d;
    if (width <= 0 || rows <= 0) return set_error(RT_ERR_ARG, "Image has non-positive dimensions.");
    if (opt->maxval <= 0 || opt->maxval > 65535) return set_error(RT_ERR_ARG, "Invalid maxval (must be 1..65535).");
    if (!rgb_dev || !out_dev) return set_error(RT_ERR_ARG, "rt_ppm_quantize_device: null buffer");
    QuantParams P;
    P.rgb = rgb_dev;
    P.out = out_dev;
    P.row_len = (int64_t)width * 3;
    P.n = P.row_len * rows;
    P.rows = rows;
    P.maxval = opt->maxval;
    P.clamp = opt->clamp != 0;
    P.gamma2 = opt->gamma2 != 0;
    P.flip = opt->flip_y != 0 && rows > 1;
    const bool two = opt->maxval >= 256;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    if (!P.flip && aligned16(rgb_dev) && aligned16(out_dev)) {
        const int64_t lanes = (P.n + 15) / 16;
        const dim3 grid((unsigned)((lanes + BLOCK - 1) / BLOCK));
        if (two) hipLaunchKernelGGL(quantize_vec_kernel<2>, grid, dim3(BLOCK), 0, st, P);
        else hipLaunchKernelGGL(quantize_vec_kernel<1>, grid, dim3(BLOCK), 0, st, P);
    } else {
        const dim3 grid((unsigned)((P.n + BLOCK - 1) / BLOCK));
        if (two) hipLaunchKernelGGL(quantize_any_kernel<2>, grid, dim3(BLOCK), 0, st, P);
        else hipLaunchKernelGGL(quantize_any_kernel<1>, grid, dim3(BLOCK), 0, st, P);
    }
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

extern "C" int rt_unpermute_strips_device(const void* strips_dev, int strip_rows, size_t row_bytes, int height,
                                          int band_rows, int band_count, int flip_y, void* frame_dev,
                                          void* hip_stream) {
    if (!strips_dev || !frame_dev) return set_error(RT_ERR_ARG, "rt_unpermute_strips_device: null buffer");
    if (height <= 0 || row_bytes == 0 || band_rows <= 0 || band_count <= 0)
        return set_error(RT_ERR_ARG, "rt_unpermute_strips_device: bad shape");
    for (int r = 0; r < band_count; ++r)
        if (rt_shard_rows(height, band_rows, r, band_count) > strip_rows)
            return set_error(RT_ERR_ARG, "rt_unpermute_strips_device: strip_rows smaller than a rank's rows");
    UnpermuteParams P;
    P.strips = static_cast<const uint8_t*>(strips_dev);
    P.frame = static_cast<uint8_t*>(frame_dev);
    P.row_bytes = (int64_t)row_bytes;
    P.strip_stride = (int64_t)strip_rows * P.row_bytes;
    P.height = height;
    P.band_rows = band_rows;
    P.band_count = band_count;
    P.flip = flip_y != 0;
    P.vec = (row_bytes % 16) == 0 && aligned16(strips_dev) && aligned16(frame_dev);
    hipLaunchKernelGGL(unpermute_kernel, dim3((unsigned)height), dim3(BLOCK), 0,
                       static_cast<hipStream_t>(hip_stream), P);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}
