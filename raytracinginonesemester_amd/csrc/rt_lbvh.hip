// rt_lbvh.hip — the reference's LBVH build on gfx950: leaf boxes ->
// scene box -> Morton keys -> sort -> Karras hierarchy -> bottom-up refit, emitting the
// reference's BVHNode / AABB arrays (2P-1 entries each, leaves at [P-1, 2P-1)) byte for byte
// as its CPU build writes them (G/include/bvh.cu:60-89 calculateAABBs, :209-317 buildBVH,
// G/include/bvh.h:131-151 and :292-406 helpers, scene box std::accumulate G/src/main.cu:296-302).
//
// Bit-exactness notes:
//  * fminf / fmaxf are the x86-64 glibc functions the reference links: x < y ? x : y (resp. >),
//    i.e. the SECOND argument wins ties (+0 vs -0) and a NaN argument loses to a number.
//    ref_fminf / ref_fmaxf restate that; v_min_f32 would not (it orders -0 < +0).
//  * The scene box is a left fold of AABB::merge from AABB() over the leaves in triangle order;
//    with "second argument wins ties" the fold's result is the minimum whose tie is broken by
//    the LAST equal element (only +-0 tie with different bits).  The parallel reduction
//    therefore reduces (value, index) keys: smallest value, then largest index, as one 64-bit
//    atomicMin per block and axis (atomicMax for the maxima); NaN leaves never win, and an
//    all-NaN axis keeps AABB()'s +-inf.
//  * Keys are (morton << 32) | triangle index, all distinct, so the sorted order is unique.  A
//    stable LSD radix sort of the 30-bit Morton code with the triangle index as value, over
//    indices in ascending order, yields exactly that order with 4 passes instead of 8.
//  * Karras range/split search and the refit follow the reference CPU code; the refit merges
//    (left, right) in that argument order, so which thread merges a node does not matter.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>
#include <cstring>

#include "rt_common.hpp"
#include "rt_hip_host.hpp"

using rt::set_error;
using rt::hip_msg;
using rt::DeviceGuard;

namespace {

constexpr int BLOCK = 256;
constexpr uint32_t NONE = 0xFFFFFFFFu;

__device__ __forceinline__ float ref_fminf(float x, float y) {
    if (y != y) return x;
    if (x != x) return y;
    return x < y ? x : y;
}
__device__ __forceinline__ float ref_fmaxf(float x, float y) {
    if (y != y) return x;
    if (x != x) return y;
    return x > y ? x : y;
}

struct Box {
    float mn[3], mx[3];
};

__device__ __forceinline__ Box merge(const Box& a, const Box& b) {  // AABB::merge (bvh.h:36-50)
    Box r;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        r.mn[k] = ref_fminf(a.mn[k], b.mn[k]);
        r.mx[k] = ref_fmaxf(a.mx[k], b.mx[k]);
    }
    return r;
}

__device__ __forceinline__ Box load_box(const rt_aabb* a, size_t i) {
    const float* p = reinterpret_cast<const float*>(a + i);
    return Box{{p[0], p[1], p[2]}, {p[3], p[4], p[5]}};
}
__device__ __forceinline__ void store_box(rt_aabb* a, size_t i, const Box& b) {
    float* p = reinterpret_cast<float*>(a + i);
    p[0] = b.mn[0]; p[1] = b.mn[1]; p[2] = b.mn[2];
    p[3] = b.mx[0]; p[4] = b.mx[1]; p[5] = b.mx[2];
}

// Orderable form of a float with +0 == -0 (ties are then broken by index); NaN -> `nan_key`.
__device__ __forceinline__ uint32_t ord(float v, uint32_t nan_key) {
    if (v != v) return nan_key;
    uint32_t u = __float_as_uint(v == 0.0f ? 0.0f : v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Scene-box reduction keys: 3 min keys ((ord << 32) | ~i, atomicMin: smallest value, last
// index) then 3 max keys ((ord << 32) | i, atomicMax).  Initial values: all-ones / zero.
struct BoundKeys {
    unsigned long long k[6];
};

__device__ __forceinline__ unsigned long long wave_min(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}
__device__ __forceinline__ unsigned long long wave_max(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

// calculateAABBs (bvh.cu:73-88, aabb_of_triangle bvh.h:54-72 with eps = 0) + the scene-box
// keys.  A triangle with an out-of-range vertex index raises *err (the host build's check).
__global__ __launch_bounds__(BLOCK) void leaf_boxes_kernel(const rt_vec3* __restrict__ pos, uint32_t nv,
                                                           const uint32_t* __restrict__ idx, uint32_t P,
                                                           rt_aabb* __restrict__ boxes, BoundKeys* keys,
                                                           int* err) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    unsigned long long kmin[3] = {~0ull, ~0ull, ~0ull}, kmax[3] = {0ull, 0ull, 0ull};
    if (i < P) {
        const uint32_t a = idx[3 * (size_t)i], b = idx[3 * (size_t)i + 1], c = idx[3 * (size_t)i + 2];
        if (a >= nv || b >= nv || c >= nv) {
            atomicOr(err, 1);
        } else {
            const rt_vec3 va = pos[a], vb = pos[b], vc = pos[c];
            const float A[3] = {va.x, va.y, va.z}, B[3] = {vb.x, vb.y, vb.z}, C[3] = {vc.x, vc.y, vc.z};
            Box bx;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                // box.minCorner -= 0.0f / maxCorner += 0.0f: x - 0 == x and x + 0 == x bit for bit
                // except -0 + 0 = +0 (round to nearest), which the max side reproduces here.
                bx.mn[k] = ref_fminf(A[k], ref_fminf(B[k], C[k])) - 0.0f;
                bx.mx[k] = ref_fmaxf(A[k], ref_fmaxf(B[k], C[k])) + 0.0f;
            }
            store_box(boxes, i, bx);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                kmin[k] = ((unsigned long long)ord(bx.mn[k], 0xFFFFFFFFu) << 32) | (uint32_t)~i;
                kmax[k] = ((unsigned long long)ord(bx.mx[k], 0u) << 32) | i;
                if (bx.mn[k] != bx.mn[k]) kmin[k] = ~0ull;
                if (bx.mx[k] != bx.mx[k]) kmax[k] = 0ull;
            }
        }
    }
    __shared__ unsigned long long red[BLOCK / 64][6];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const unsigned long long m = wave_min(kmin[k]), M = wave_max(kmax[k]);
        if (lane == 0) { red[wv][k] = m; red[wv][3 + k] = M; }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        unsigned long long v = red[0][k];
        for (int w = 1; w < BLOCK / 64; ++w) {
            const unsigned long long u = red[w][k];
            v = (k < 3) ? (u < v ? u : v) : (u > v ? u : v);
        }
        if (k < 3) { if (v != ~0ull) atomicMin(&keys->k[k], v); }
        else if (v != 0ull) atomicMax(&keys->k[k], v);
    }
}

// The scene box from the reduction keys: the winning leaf's coordinate (AABB() if none).
__device__ __forceinline__ Box scene_box(const BoundKeys& K, const rt_aabb* boxes) {
    Box s;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const unsigned long long a = K.k[k], b = K.k[3 + k];
        s.mn[k] = a == ~0ull ? INFINITY : load_box(boxes, (uint32_t)~(uint32_t)(a & 0xFFFFFFFFu)).mn[k];
        s.mx[k] = b == 0ull ? -INFINITY : load_box(boxes, (uint32_t)(b & 0xFFFFFFFFu)).mx[k];
    }
    return s;
}

__device__ __forceinline__ uint32_t bit_expansion(uint32_t v) {  // bvh.h:131-138
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// ComputeMortonCode (bvh.h:142-151) of the normalised centroid (bvh.cu:244-258): float
// (min + max) * 0.5f, (c - smin) / (smax - smin) with IEEE division, no contraction.
__global__ __launch_bounds__(BLOCK) void morton_kernel(const rt_aabb* __restrict__ boxes, uint32_t P,
                                                       const BoundKeys* keys, uint32_t* __restrict__ code,
                                                       uint32_t* __restrict__ tri) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= P) return;
    const Box s = scene_box(*keys, boxes);
    const Box b = load_box(boxes, i);
    uint32_t e[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float c = (b.mn[k] + b.mx[k]) * 0.5f;
        float n = (c - s.mn[k]) / (s.mx[k] - s.mn[k]);
        n = ref_fminf(ref_fmaxf(n * 1024.0f, 0.0f), 1024.0f - 1.0f);
        e[k] = bit_expansion((uint32_t)n);
    }
    code[i] = e[0] * 4 + e[1] * 2 + e[2];
    tri[i] = i;
}

// Leaves in key order (bvh.cu:276-291): boxes gathered, object_idx = triangle index; full
// 64-bit keys for the hierarchy; every node reset to the all-ones BVHNode.
__global__ __launch_bounds__(BLOCK) void leaves_kernel(const rt_aabb* __restrict__ boxes, uint32_t P,
                                                       const uint32_t* __restrict__ code,
                                                       const uint32_t* __restrict__ tri,
                                                       unsigned long long* __restrict__ key64,
                                                       rt_bvh_node* __restrict__ nodes, rt_aabb* __restrict__ out,
                                                       uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= P) return;
    const uint32_t t = tri[i];
    key64[i] = ((unsigned long long)code[i] << 32) | t;
    store_box(out, (size_t)(P - 1) + i, load_box(boxes, t));
    nodes[(P - 1) + i] = rt_bvh_node{NONE, NONE, NONE, t};
    if (i + 1 < P) {
        nodes[i] = rt_bvh_node{NONE, NONE, NONE, NONE};
        flags[i] = 0;
    }
}

__device__ __forceinline__ int cub(unsigned long long a, unsigned long long b) {  // common_upper_bits
    const unsigned long long d = a ^ b;
    return d == 0 ? 64 : __clzll((long long)d);
}

// One internal node per lane: determine_range (bvh.h:303-361) + find_split (:363-394); the
// node writes its own children and their parent links (each node has one parent: no races).
__global__ __launch_bounds__(BLOCK) void internal_kernel(const unsigned long long* __restrict__ key, uint32_t P,
                                                         rt_bvh_node* __restrict__ nodes, uint2* __restrict__ range) {
    const uint32_t idx = blockIdx.x * BLOCK + threadIdx.x;
    if (idx + 1 >= P) return;
    uint32_t first, last;
    if (idx == 0) {
        first = 0;
        last = P - 1;
    } else {
        const unsigned long long self = key[idx];
        const int L = cub(self, key[idx - 1]);
        const int R = cub(self, key[idx + 1]);
        const int d = (R > L) ? 1 : -1;
        const int delta_min = L < R ? L : R;
        int l_max = 2;
        int delta = -1;
        int i_tmp = (int)(idx + (uint32_t)(d * l_max));
        if (0 <= i_tmp && (uint32_t)i_tmp < P) delta = cub(self, key[i_tmp]);
        while (delta > delta_min) {
            l_max <<= 1;
            i_tmp = (int)(idx + (uint32_t)(d * l_max));
            delta = -1;
            if (0 <= i_tmp && (uint32_t)i_tmp < P) delta = cub(self, key[i_tmp]);
        }
        int l = 0;
        for (int t = l_max >> 1; t > 0; t >>= 1) {
            i_tmp = (int)(idx + (uint32_t)((l + t) * d));
            delta = -1;
            if (0 <= i_tmp && (uint32_t)i_tmp < P) delta = cub(self, key[i_tmp]);
            if (delta > delta_min) l += t;
        }
        const uint32_t jdx = idx + (uint32_t)(l * d);
        first = d < 0 ? jdx : idx;
        last = d < 0 ? idx : jdx;
    }
    uint32_t gamma;
    const unsigned long long fc = key[first], lc = key[last];
    if (fc == lc) {
        gamma = (first + last) >> 1;
    } else {
        const int delta_node = cub(fc, lc);
        int split = (int)first;
        int stride = (int)(last - first);
        do {
            stride = (stride + 1) >> 1;
            const int middle = split + stride;
            if ((uint32_t)middle < last && cub(fc, key[middle]) > delta_node) split = middle;
        } while (stride > 1);
        gamma = (uint32_t)split;
    }
    uint32_t left = gamma, right = gamma + 1;
    if (first == gamma) left += P - 1;  // min(first, last) == gamma: a leaf
    if (last == gamma + 1) right += P - 1;
    range[idx] = make_uint2(first, last);
    nodes[idx].object_idx = NONE;
    nodes[idx].left_idx = left;
    nodes[idx].right_idx = right;
    nodes[left].parent_idx = idx;
    nodes[right].parent_idx = idx;
}

// Bottom-up refit, one lane per leaf climbing while it is the second child to arrive at a
// node.  Agent-scope ordering on this chip means an L2 write-back + invalidate per fence (the
// XCDs' L2s are not coherent), so the climb is split where it needs no such fence:
//  * refit_chunk_kernel: workgroup b owns leaves [b*CHUNK, (b+1)*CHUNK) and refits every node
//    whose leaf range [first, last] lies inside its chunk — both children of such a node are
//    finished by the same workgroup, so workgroup-scope acq_rel atomics on the arrival flags
//    order the box stores (one CU, one L1).  A finished node whose parent's range crosses the
//    chunk is appended to the top list.
//  * refit_top_kernel: one workgroup climbs from the top-list entries through the nodes whose
//    ranges cross chunks (a few per chunk), again with workgroup-scope flags; phase-1 boxes
//    are visible across the kernel boundary.
// merge(left, right) has a fixed argument order, so which lane merges a node does not matter.
constexpr uint32_t CHUNK = 2048;
constexpr int TOP_BLOCK = 1024;

__device__ __forceinline__ uint32_t arrive(uint32_t* flag) {
    return __hip_atomic_fetch_add(flag, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void merge_node(const rt_bvh_node* nodes, rt_aabb* aabbs, uint32_t p) {
    const rt_bvh_node nd = nodes[p];
    store_box(aabbs, p, merge(load_box(aabbs, nd.left_idx), load_box(aabbs, nd.right_idx)));
}

__global__ __launch_bounds__(BLOCK) void refit_chunk_kernel(const rt_bvh_node* __restrict__ nodes, uint32_t P,
                                                            const uint2* __restrict__ range, rt_aabb* aabbs,
                                                            uint32_t* flags, uint32_t* top_count,
                                                            uint32_t* __restrict__ top_list) {
    const uint32_t c0 = blockIdx.x * CHUNK, c1 = min(c0 + CHUNK, P);
    for (uint32_t i = c0 + threadIdx.x; i < c1; i += BLOCK) {
        uint32_t x = (P - 1) + i;
        uint32_t p = nodes[x].parent_idx;
        while (p != NONE) {
            const uint2 rg = range[p];
            if (rg.x < c0 || rg.y >= c1) {
                top_list[atomicAdd(top_count, 1u)] = x;
                break;
            }
            if (arrive(&flags[p]) == 0) break;
            merge_node(nodes, aabbs, p);
            x = p;
            p = nodes[p].parent_idx;
        }
    }
}

__global__ __launch_bounds__(TOP_BLOCK) void refit_top_kernel(const rt_bvh_node* __restrict__ nodes,
                                                              rt_aabb* aabbs, uint32_t* flags,
                                                              const uint32_t* top_count,
                                                              const uint32_t* __restrict__ top_list) {
    const uint32_t n = *top_count;
    for (uint32_t k = threadIdx.x; k < n; k += TOP_BLOCK) {
        uint32_t p = nodes[top_list[k]].parent_idx;
        while (p != NONE) {
            if (arrive(&flags[p]) == 0) break;
            merge_node(nodes, aabbs, p);
            p = nodes[p].parent_idx;
        }
    }
}

unsigned grid_of(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

}  // namespace

extern "C" int rt_build_bvh_device(int device, const rt_vec3* positions_dev, size_t num_vertices,
                                   const uint32_t* indices_dev, size_t num_triangles, rt_bvh_node* nodes_dev,
                                   rt_aabb* aabbs_dev, void* hip_stream) {
    if (!positions_dev || !indices_dev || !nodes_dev || !aabbs_dev)
        return set_error(RT_ERR_ARG, "rt_build_bvh_device: null argument");
    const size_t P = num_triangles;
    if (P == 0) return set_error(RT_ERR_ARG, "no triangles");
    if (P > 0x7FFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "more than 2^31-1 triangles");
    if (num_vertices > 0xFFFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "more than 2^32-1 vertices");
    int rc = rt::check_device(device);
    if (rc != RT_OK) return rc;
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    const uint32_t n = (uint32_t)P;
    // One stream-ordered workspace (pooled by the runtime across builds): unsorted leaf boxes,
    // Morton codes + triangle ids (double-buffered for the sort), 64-bit keys, node ranges,
    // arrival flags, top list, reduction keys + error flag + top count, sort storage.
    size_t tmp_bytes = 0;
    HIP_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                      (uint32_t*)nullptr, (uint32_t*)nullptr, n, 0u, 30u, st));
    size_t off = 0;
    auto carve = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_box = carve(P * sizeof(rt_aabb)), o_c0 = carve(P * 4), o_t0 = carve(P * 4), o_c1 = carve(P * 4),
                 o_t1 = carve(P * 4), o_k64 = carve(P * 8), o_rng = carve(P * 8), o_fl = carve(P * 4),
                 o_top = carve(2 * P * 4), o_misc = carve(sizeof(BoundKeys) + 16), o_tmp = carve(tmp_bytes);
    void* ws = nullptr;
    HIP_TRY(hipMallocAsync(&ws, off, st));
    struct WsFree {
        void* p; hipStream_t s;
        ~WsFree() { if (p) (void)hipFreeAsync(p, s); }
    } ws_free{ws, st};
    char* W = static_cast<char*>(ws);
    auto* bx = reinterpret_cast<rt_aabb*>(W + o_box);
    auto* c0 = reinterpret_cast<uint32_t*>(W + o_c0);
    auto* t0 = reinterpret_cast<uint32_t*>(W + o_t0);
    auto* c1 = reinterpret_cast<uint32_t*>(W + o_c1);
    auto* t1 = reinterpret_cast<uint32_t*>(W + o_t1);
    auto* k64 = reinterpret_cast<unsigned long long*>(W + o_k64);
    auto* rng = reinterpret_cast<uint2*>(W + o_rng);
    auto* fl = reinterpret_cast<uint32_t*>(W + o_fl);
    auto* top = reinterpret_cast<uint32_t*>(W + o_top);
    auto* keys = reinterpret_cast<BoundKeys*>(W + o_misc);
    int* err = reinterpret_cast<int*>(W + o_misc + sizeof(BoundKeys));
    uint32_t* top_count = reinterpret_cast<uint32_t*>(W + o_misc + sizeof(BoundKeys) + 4);
    BoundKeys init;
    for (int k = 0; k < 3; ++k) { init.k[k] = ~0ull; init.k[3 + k] = 0ull; }
    HIP_TRY(hipMemcpyAsync(keys, &init, sizeof(init), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(err, 0, 8, st));  // err + top_count
    hipLaunchKernelGGL(leaf_boxes_kernel, dim3(grid_of(P)), dim3(BLOCK), 0, st, positions_dev,
                       (uint32_t)num_vertices, indices_dev, n, bx, keys, err);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(morton_kernel, dim3(grid_of(P)), dim3(BLOCK), 0, st, bx, n, keys, c0, t0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(rocprim::radix_sort_pairs(W + o_tmp, tmp_bytes, c0, c1, t0, t1, n, 0u, 30u, st));
    hipLaunchKernelGGL(leaves_kernel, dim3(grid_of(P)), dim3(BLOCK), 0, st, bx, n, c1, t1, k64, nodes_dev,
                       aabbs_dev, fl);
    HIP_TRY(hipGetLastError());
    if (P > 1) {
        hipLaunchKernelGGL(internal_kernel, dim3(grid_of(P - 1)), dim3(BLOCK), 0, st, k64, n, nodes_dev, rng);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(refit_chunk_kernel, dim3((unsigned)((P + CHUNK - 1) / CHUNK)), dim3(BLOCK), 0, st,
                           nodes_dev, n, rng, aabbs_dev, fl, top_count, top);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(refit_top_kernel, dim3(1), dim3(TOP_BLOCK), 0, st, nodes_dev, aabbs_dev, fl, top_count,
                           top);
        HIP_TRY(hipGetLastError());
    }
    int herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (herr) return set_error(RT_ERR_ARG, "triangle index out of range");
    return RT_OK;
}
