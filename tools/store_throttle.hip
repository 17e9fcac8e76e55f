// Store-stream probe for the headline rollout's observation trajectory (K, B, 2L) int32 at
// L = 36, B = 2^20 (302 MB per step, 6 GB at K = 20), no compute.  Question: does the number of
// stores a wave keeps in flight set the write rate of the rollout's store pattern (a wave per 64
// envs writing its 18 KB slice of every step row), as against a one-shot linear fill?
//   fill_oneshot     each thread one 16-B store, blocks in address order (torch fill_'s shape)
//   fill_stride<N>   grid sized to resident capacity, grid-stride 16-B stores; N > 0: at most N
//                    stores in flight per wave (s_waitcnt vmcnt(N) after each)
//   tile<N>          the rollout's shape: wave w owns rows [64w, 64w + 64) of every step row and
//                    writes its 18 x 1 KB slice per step, K steps, spin VALU cycles between steps;
//                    N > 0 as above
//   tile_oneshot     the same slices, one wave per (step, tile), step-major (each wave one slice)
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int WAVE = 64, BLOCK = 256;

template <int N>
__device__ __forceinline__ void throttle() {
    // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt_hi[15:14]
    if constexpr (N > 0) __builtin_amdgcn_s_waitcnt((N & 0xf) | (0x7 << 4) | (0xf << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void st_nt(int4* p, int4 v) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const v4i_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(p));
}

// the same 16-B store with the gfx950 cache-policy bits through a buffer store (aux = cpol:
// sc0 = 1, nt = 2, sc1 = 16): sc1 stores do not keep the line in the XCD's L2
template <int CPOL>
__global__ __launch_bounds__(256) void tile_pol(int4* __restrict__ dst, int64_t rows, int cpr, int K, int v) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * WAVE;
    if (r0 >= rows) return;
    const int nch = WAVE * cpr;
    for (int t = 0; t < K; ++t) {
        // the wave's slice of step row t as one buffer (scalar base), lanes at their 16-B offsets
        const uint64_t b = reinterpret_cast<uint64_t>(dst + ((int64_t)t * rows + r0) * cpr);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, nch * 16, 0x00020000);
        for (int c = lane; c < nch; c += WAVE) {
            const v4i_t x = {v, t, c, lane};
            __builtin_amdgcn_raw_buffer_store_b128(x, r, (uint32_t)c * 16u, 0, CPOL);
        }
    }
}

__global__ __launch_bounds__(256) void fill_oneshot(int4* __restrict__ dst, int64_t n16, int v) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n16) st_nt(dst + i, make_int4(v, v, v, (int)i));
}

template <int N>
__global__ __launch_bounds__(256) void fill_stride(int4* __restrict__ dst, int64_t n16, int v) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n16; i += (int64_t)gridDim.x * BLOCK) {
        st_nt(dst + i, make_int4(v, v, v, (int)i));
        throttle<N>();
    }
}

// cpr 16-B chunks per row; a wave's slice of one step row = 64 * cpr chunks, contiguous
template <int N>
__global__ __launch_bounds__(256) void tile(int4* __restrict__ dst, int64_t rows, int cpr, int K, int spin, int v) {
    const int lane = threadIdx.x & 63;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * WAVE;
    if (r0 >= rows) return;
    const int nch = WAVE * cpr;
    int acc = v + lane;
    for (int t = 0; t < K; ++t) {
        int4* row = dst + ((int64_t)t * rows + r0) * cpr;
        for (int c = lane; c < nch; c += WAVE) {
            st_nt(row + c, make_int4(acc, t, c, lane));
            throttle<N>();
        }
        for (int i = 0; i < spin; ++i) acc = acc * 1664525 + 1013904223;  // the step's compute
    }
    if (acc == 0x7fffffff && lane == 64) dst[0].x = acc;  // keeps the spin
}

// the same, but wave w owns its 64 envs in groups of GE consecutive envs, group g at envs
// (g * waves + w) * GE: the resident waves writing their g-th group cover one contiguous
// (resident waves x GE x 2L x 4 B) window instead of the whole step row
template <int GE>
__global__ __launch_bounds__(256) void tile_grouped(int4* __restrict__ dst, int64_t rows, int cpr, int K, int v) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t waves = rows / WAVE;
    if (w >= waves) return;
    const int gch = GE * cpr;  // chunks per group
    for (int t = 0; t < K; ++t) {
        int4* row = dst + (int64_t)t * rows * cpr;
        for (int c = lane; c < WAVE * cpr; c += WAVE) {
            const int g = c / gch, o = c - g * gch;
            st_nt(row + ((int64_t)g * waves + w) * gch + o, make_int4(v, t, c, lane));
        }
    }
}

__global__ __launch_bounds__(256) void tile_oneshot(int4* __restrict__ dst, int64_t rows, int cpr, int v) {
    const int lane = threadIdx.x & 63;
    const int64_t tiles = rows / WAVE;
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // step-major (t, tile)
    const int64_t t = g / tiles, r0 = (g - t * tiles) * WAVE;
    int4* row = dst + (t * rows + r0) * cpr;
    for (int c = lane; c < WAVE * cpr; c += WAVE) st_nt(row + c, make_int4(v, (int)t, c, lane));
}

// the rollout's slices, but the block's 4 waves write their 4 adjacent tiles' slice of a step
// together: thread t of the block stores chunks t, t + 256, ... of the block's 256-row slice, so
// each store round covers 4 KB contiguous (as fill_oneshot's blocks do) instead of each wave
// walking its own 18 KB.  SYNC: a block barrier between steps (the rollout's LDS tiles would
// need one)
template <int SYNC>
__global__ __launch_bounds__(256) void tile_block(int4* __restrict__ dst, int64_t rows, int cpr, int K, int v) {
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    if (r0 >= rows) return;
    const int nch = 256 * cpr;
    for (int t = 0; t < K; ++t) {
        int4* row = dst + ((int64_t)t * rows + r0) * cpr;
        for (int c = threadIdx.x; c < nch; c += 256) st_nt(row + c, make_int4(v, t, c, (int)threadIdx.x));
        if (SYNC) __syncthreads();
    }
}

// tile's pattern with each wave's store sequence rotated: wave w starts its slice at chunk
// ((w * ROT) mod 64 * 64) and wraps, so the waves writing in step do not all write the same
// offset of their 18 KB slices at once (slices 18 KB apart give few distinct low-address
// classes for a given offset: a channel hot spot while the waves are in step)
__global__ __launch_bounds__(256) void tile_rot(int4* __restrict__ dst, int64_t rows, int cpr, int K, int rot, int v) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t r0 = w * WAVE;
    if (r0 >= rows) return;
    const int nch = WAVE * cpr;
    const int start = (int)((w * rot) % cpr) * WAVE;  // in chunks, a whole store instruction
    for (int t = 0; t < K; ++t) {
        int4* row = dst + ((int64_t)t * rows + r0) * cpr;
        for (int i = 0; i < nch; i += WAVE) {
            int c = start + i + lane;
            if (c >= nch) c -= nch;
            st_nt(row + c, make_int4(v, t, c, lane));
        }
    }
}

// tile's pattern with the waves out of step: wave w writes its slices of steps t0, t0 + 1, ...
// (mod K) with t0 = (w * 7) mod K, so the waves writing at a given moment spread over the K step
// rows instead of all writing the same one
__global__ __launch_bounds__(256) void tile_desync(int4* __restrict__ dst, int64_t rows, int cpr, int K, int v) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t r0 = w * WAVE;
    if (r0 >= rows) return;
    const int nch = WAVE * cpr;
    const int t0 = (int)((w * 7) % K);
    for (int i = 0; i < K; ++i) {
        const int t = t0 + i < K ? t0 + i : t0 + i - K;
        int4* row = dst + ((int64_t)t * rows + r0) * cpr;
        for (int c = lane; c < nch; c += WAVE) st_nt(row + c, make_int4(v, t, c, lane));
    }
}

// tile_block's slices written once each by short-lived blocks, step-major
__global__ __launch_bounds__(256) void tile_block_oneshot(int4* __restrict__ dst, int64_t rows, int cpr, int v) {
    const int64_t blocks_per_step = rows / 256;
    const int64_t t = blockIdx.x / blocks_per_step, r0 = (blockIdx.x - t * blocks_per_step) * 256;
    int4* row = dst + (t * rows + r0) * cpr;
    for (int c = threadIdx.x; c < 256 * cpr; c += 256) st_nt(row + c, make_int4(v, (int)t, c, (int)threadIdx.x));
}

extern "C" {
// kind: 0 fill_oneshot, 1 fill_stride, 2 tile, 3 tile_oneshot, 4 tile_grouped (n = GE: 8, 16, 32),
// 6 tile_block (n: a barrier between steps), 7 tile_block_oneshot,
// 5 tile with buffer stores of cache policy n (0 plain, 1 sc0, 2 nt, 16 sc1, 17 sc0 sc1, 18 sc1 nt); n: stores in flight per wave
// (0 = unthrottled; 1, 2, 4, 8, 16); returns a hip error code
int probe_store(int kind, int n, void* buf, int64_t rows, int L, int K, int spin, int resident_blocks, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const int cpr = 2 * L / 4;
    int4* d = (int4*)buf;
    const int64_t n16 = (int64_t)K * rows * cpr;
    const unsigned tiles = (unsigned)((rows + 255) / 256);
    if (kind == 0) {
        fill_oneshot<<<dim3((unsigned)((n16 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s>>>(d, n16, 7);
    } else if (kind == 1) {
#define F(NN) fill_stride<NN><<<dim3(resident_blocks), dim3(BLOCK), 0, s>>>(d, n16, 7)
        switch (n) { case 0: F(0); break; case 1: F(1); break; case 2: F(2); break; case 4: F(4); break;
                     case 8: F(8); break; default: F(16); }
#undef F
    } else if (kind == 2) {
#define T(NN) tile<NN><<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, spin, 7)
        switch (n) { case 0: T(0); break; case 1: T(1); break; case 2: T(2); break; case 4: T(4); break;
                     case 8: T(8); break; default: T(16); }
#undef T
    } else if (kind == 5) {
#define Q(NN) tile_pol<NN><<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, 7)
        switch (n) { case 0: Q(0); break; case 1: Q(1); break; case 2: Q(2); break; case 16: Q(16); break;
                     case 17: Q(17); break; default: Q(18); }
#undef Q
    } else if (kind == 4) {
#define G(NN) tile_grouped<NN><<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, 7)
        switch (n) { case 8: G(8); break; case 16: G(16); break; default: G(32); }
#undef G
    } else if (kind == 6) {
        if (n) tile_block<1><<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, 7);
        else tile_block<0><<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, 7);
    } else if (kind == 9) {
        tile_desync<<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, 7);
    } else if (kind == 8) {
        tile_rot<<<dim3(tiles), dim3(BLOCK), 0, s>>>(d, rows, cpr, K, n, 7);
    } else if (kind == 7) {
        tile_block_oneshot<<<dim3((unsigned)((int64_t)K * rows / 256)), dim3(BLOCK), 0, s>>>(d, rows, cpr, 7);
    } else {
        tile_oneshot<<<dim3((unsigned)((int64_t)K * rows / 256)), dim3(BLOCK), 0, s>>>(d, rows, cpr, 7);
    }
    return (int)hipGetLastError();
}
}
