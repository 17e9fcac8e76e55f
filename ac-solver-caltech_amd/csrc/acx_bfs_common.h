// acx_bfs_common.h -- pieces shared by the single-GPU device BFS (acx_bfs.hip) and the
// owner-partitioned multi-GPU BFS (acx_sbfs.hip): packed-key compare / hash, table entry
// tags, block scans.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "acx.h"
#include "acx_moves.h"

namespace acx {
namespace bfs {

constexpr uint64_t CHUNK = 1ull << 63;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t SEEN = 0xffffffffu;  // slot index of a child whose state is already a node
constexpr int TPB = 256;


__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

template <int KWM>
struct Key {
    uint64_t w[KWM];
};

template <int KWM>
__device__ __forceinline__ Key<KWM> kload(const uint64_t* p, int kw) {
    Key<KWM> k;
#pragma unroll
    for (int i = 0; i < KWM; ++i) k.w[i] = i < kw ? p[i] : 0ull;
    return k;
}

template <int KWM>
__device__ __forceinline__ bool keq(const uint64_t* p, const Key<KWM>& k, int kw) {
    bool e = true;
#pragma unroll
    for (int i = 0; i < KWM; ++i)
        if (i < kw) e &= p[i] == k.w[i];
    return e;
}

template <int KWM>
__host__ __device__ __forceinline__ uint64_t khash(const Key<KWM>& k, int kw) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
#pragma unroll
    for (int i = 0; i < KWM; ++i)
        if (i < kw) h = fmix64(h ^ k.w[i]) + 0x632be59bd9b4e019ull;
    return fmix64(h);
}

// n bytes (n % 4 == 0) device -> pinned host memory by a kernel (no DMA-engine copy: rocprofv3's
// memory-copy tracing never receives the completion of a device-to-host engine copy on this
// stack -- profiles/r04/bfs_trace_c: one undelivered callback per copy -- so the exports below
// write host memory from a kernel instead)
static __global__ void d2h_copy_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// device -> pageable host memory on the caller's stream, through a pinned bounce buffer the
// workspace keeps (*pin, allocated on first use, BOUNCE bytes; freed with the workspace): no
// hipMemcpy on the null stream, no pageable destination, nothing freed while a copy may be
// in flight
constexpr size_t BOUNCE = 16u << 20;
static inline int copy_to_host(void* dst, const void* src, size_t n, hipStream_t st, void** pin) {
    if (n == 0) return ACX_OK;
    if (n % 4) return ACX_E_ARG;
    if (!*pin && hipHostMalloc(pin, BOUNCE, hipHostMallocDefault) != hipSuccess) {
        *pin = nullptr;
        return ACX_E_LAUNCH;
    }
    for (size_t off = 0; off < n; off += BOUNCE) {
        const size_t m = n - off < BOUNCE ? n - off : BOUNCE;
        d2h_copy_kernel<<<dim3(1024), dim3(256), 0, st>>>(static_cast<uint32_t*>(*pin),
                                                           reinterpret_cast<const uint32_t*>((const char*)src + off), m / 4);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return ACX_E_LAUNCH;
        memcpy((char*)dst + off, *pin, m);
    }
    return ACX_OK;
}

// LDS written by the wave's lanes is visible to the whole wave after this
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, WAVE));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) v += (uint32_t)__shfl_xor((int)v, o, WAVE);
    return v;
}

__device__ __forceinline__ uint64_t tload(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive prefix sum of v over the block (TPB threads); total in `tot`
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& tot) {
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
    }
    if (lane == WAVE - 1) sh[wid] = x;
    __syncthreads();
    uint32_t off = 0;
    tot = 0;
#pragma unroll
    for (int i = 0; i < TPB / WAVE; ++i) {
        off += i < wid ? sh[i] : 0u;
        tot += sh[i];
    }
    return off + x - v;
}

__device__ __forceinline__ uint32_t block_min(uint32_t v, uint32_t* sh) {
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, WAVE));
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    uint32_t m = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < TPB / WAVE; ++i) m = min(m, sh[i]);
    return m;
}

static inline int nw_for(int L) { return L <= 16 ? 1 : L <= 32 ? 2 : L <= 48 ? 3 : L <= 64 ? 4 : 8; }

template <class F>
static void by_nw(int L, F&& f) {
    switch (nw_for(L)) {
        case 1: f.template go<1>(); break;
        case 2: f.template go<2>(); break;
        case 3: f.template go<3>(); break;
        case 4: f.template go<4>(); break;
        default: f.template go<8>(); break;
    }
}

// host packing of a presentation into the key format (acx.h)
static inline void pack_key(const int32_t* pres, int L, int kw, uint64_t* out) {
    for (int k = 0; k < kw; ++k) out[k] = 0;
    int n[2] = {0, 0};
    for (int h = 0; h < 2; ++h) {
        for (int i = 0; i < L; ++i) {
            const int32_t v = pres[h * L + i];
            if (v == 0) continue;
            const uint64_t code = v == 1 ? 0 : v == -1 ? 1 : v == 2 ? 2 : 3;
            const int bit = 2 * (h * L + i);
            out[bit / 64] |= code << (bit % 64);
            ++n[h];
        }
    }
    const uint64_t lens = (uint64_t)n[0] | ((uint64_t)n[1] << 8);
    const int bit = 4 * L;
    out[bit / 64] |= lens << (bit % 64);
    if (bit % 64 > 48 && bit / 64 + 1 < kw) out[bit / 64 + 1] |= lens >> (64 - bit % 64);
}

}  // namespace bfs
}  // namespace acx
