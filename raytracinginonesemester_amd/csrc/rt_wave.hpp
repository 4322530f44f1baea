// rt_wave.hpp — wavefront primitives (64 lanes: lane ids, ballots, readlane/writelane, DPP
// reductions) and constant-address-space loads, shared by the device translation units
// (rt_device.hip, rt_hw1.hip).  Included inside each unit's anonymous namespace, after
// <hip/hip_runtime.h>.
#pragma once

// ---- wave primitives ------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// A lane id the compiler cannot merge with any other (mbcnt of an opaque zero): one kept for a
// whole loop of items is live across all of them (and spills).
__device__ __forceinline__ uint32_t fresh_lane_id() {
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, z));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// This lane's bit of a wave-uniform mask, the inverse of ballot: one v_cndmask on the SGPR pair
// (`(m >> lane_id()) & 1` keeps a 64-bit lane bit live across the traversal loop, which the
// compiler spills to scratch and reloads at every leaf pop).
__device__ __forceinline__ bool lane_in(uint64_t m) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(r) : "s"(m));
    return r != 0;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
// v_writelane_b32 (the LLVM intrinsic; clang has no builtin for it on this toolchain): lane l
// takes v.  v and l are wave-uniform at every call.
extern "C" __device__ int rt_llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wrlane(uint32_t v, uint32_t l, uint32_t old) {
    return (uint32_t)rt_llvm_writelane((int)v, (int)l, (int)old);
}
// Wave-wide max / min of a float over all 64 lanes (callers pass the identity on lanes that do
// not take part), wave-uniform result: DPP steps within quads, half rows, rows, then the row
// broadcasts; lane 63 ends with the whole wave's.
template <bool MAX, int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_step(float x) {
    const float id = MAX ? -INFINITY : INFINITY;
    const float y =
        __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(x), CTRL, ROW_MASK, 0xF, false));
    return MAX ? fmaxf(x, y) : fminf(x, y);
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce_f(float v) {
    v = dpp_step<MAX, 0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = dpp_step<MAX, 0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = dpp_step<MAX, 0x141, 0xF>(v);  // row_half_mirror
    v = dpp_step<MAX, 0x140, 0xF>(v);  // row_mirror
    v = dpp_step<MAX, 0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v = dpp_step<MAX, 0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// ---- node accessors ---------------------------------------------------------------------
// Scene arrays are immutable while a frame renders: read them through the constant address
// space, so wave-uniform node addresses become scalar loads even inside loops that also
// store (the compiler cannot otherwise prove the stores do not clobber them).
typedef float __attribute__((ext_vector_type(4))) vf4;
typedef uint32_t __attribute__((ext_vector_type(4))) vu4;
__device__ __forceinline__ float4 ldc(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const vf4 v = *(const __attribute__((address_space(4))) vf4*)p;
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ vf4 ldc_v(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) vf4*)p;
#else
    return *reinterpret_cast<const vf4*>(p);
#endif
}
__device__ __forceinline__ uint4 ldc_u(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const vu4 v = *(const __attribute__((address_space(4))) vu4*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *reinterpret_cast<const uint4*>(p);
#endif
}

__device__ __forceinline__ uint32_t ldc_u32(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) uint32_t*)p;
#else
    return *p;
#endif
}
