// Timeline of the rollout's store pattern (tools/store_throttle.hip `tile`): every wave owns
// 64 rows of a (K, B, 2L) int32 trajectory and writes its 18 KB slice of each step row, K steps.
// Each block records its start / end on the device's constant 100 MHz clock, its XCC, and its
// wave 0's clock at the start of every step, so the host can see where a launch's time goes:
// the ramp after launch, the hand-over from the first resident round to the second, the tail.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int WAVE = 64;

__device__ __forceinline__ void st_nt(int4* p, int4 v) {
    typedef int v4i_t __attribute__((ext_vector_type(4)));
    const v4i_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(p));
}

__device__ __forceinline__ uint32_t xcc_id() {
    // HW_REG_XCC_ID (id 20), bits [3:0]
    return __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 0xf;
}

// rec: per block [start, end, xcc, 0] (uint64); steps: per block K step-start clocks of wave 0
__global__ __launch_bounds__(256) void tile_timed(int4* __restrict__ dst, int64_t rows, int cpr, int K,
                                                  uint64_t* __restrict__ rec, uint64_t* __restrict__ steps) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wid) * WAVE;
    const int nch = WAVE * cpr;
    if (r0 < rows) {
        for (int t = 0; t < K; ++t) {
            if (wid == 0 && lane == 0) steps[(int64_t)blockIdx.x * K + t] = __builtin_amdgcn_s_memrealtime();
            int4* row = dst + ((int64_t)t * rows + r0) * cpr;
            for (int c = lane; c < nch; c += WAVE) st_nt(row + c, make_int4(7, t, c, lane));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);  // the block's stores done before its end is taken
    __syncthreads();
    if (threadIdx.x == 0) {
        rec[4 * blockIdx.x + 0] = t_start;
        rec[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        rec[4 * blockIdx.x + 2] = xcc_id();
        rec[4 * blockIdx.x + 3] = 0;
    }
}

// The same slices written by persistent blocks (grid = resident blocks) that take 256-row tiles
// from a counter (DYN: atomically, one grab per tile, so blocks on faster XCDs take more tiles) or
// statically (tiles b, b + grid, ...).  rec[3] = tiles the block wrote; steps: wave 0's step
// clocks of the block's first tile.
template <bool DYN>
__global__ __launch_bounds__(256) void tile_persist(int4* __restrict__ dst, int64_t rows, int cpr, int K,
                                                    unsigned* __restrict__ ctr, uint64_t* __restrict__ rec,
                                                    uint64_t* __restrict__ steps) {
    __shared__ unsigned s_tile;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned ntiles = (unsigned)(rows / 256);
    const int nch = WAVE * cpr;
    unsigned done = 0;
    for (unsigned k = 0;; ++k) {
        unsigned tile;
        if (DYN) {
            __syncthreads();  // every wave has read the previous s_tile
            if (threadIdx.x == 0) s_tile = atomicAdd(ctr, 1u);
            __syncthreads();
            tile = s_tile;
        } else {
            tile = blockIdx.x + k * gridDim.x;
        }
        if (tile >= ntiles) break;
        const int64_t r0 = ((int64_t)tile * 4 + wid) * WAVE;
        for (int t = 0; t < K; ++t) {
            if (done == 0 && wid == 0 && lane == 0) steps[(int64_t)blockIdx.x * K + t] = __builtin_amdgcn_s_memrealtime();
            int4* row = dst + ((int64_t)t * rows + r0) * cpr;
            for (int c = lane; c < nch; c += WAVE) st_nt(row + c, make_int4(7, t, c, lane));
        }
        ++done;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        rec[4 * blockIdx.x + 0] = t_start;
        rec[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        rec[4 * blockIdx.x + 2] = xcc_id();
        rec[4 * blockIdx.x + 3] = done;
    }
}

// kind 0: one block per tile (the rollout's launch); 1: persistent blocks, dynamic tiles;
// 2: persistent blocks, static tiles.  grid: persistent blocks (rec / steps sized for the larger)
extern "C" int timeline_tile(int kind, void* buf, int64_t rows, int L, int K, int grid, void* ctr, void* rec,
                             void* steps, void* stream) {
    if (rows % 256 || K < 1 || grid < 1) return -1;
    const int cpr = 2 * L / 4;
    hipStream_t s = (hipStream_t)stream;
    if (kind == 0) {
        tile_timed<<<dim3((unsigned)(rows / 256)), dim3(256), 0, s>>>((int4*)buf, rows, cpr, K, (uint64_t*)rec,
                                                                       (uint64_t*)steps);
    } else if (kind == 1) {
        if (hipMemsetAsync(ctr, 0, 4, s) != hipSuccess) return -2;
        tile_persist<true><<<dim3(grid), dim3(256), 0, s>>>((int4*)buf, rows, cpr, K, (unsigned*)ctr,
                                                             (uint64_t*)rec, (uint64_t*)steps);
    } else {
        tile_persist<false><<<dim3(grid), dim3(256), 0, s>>>((int4*)buf, rows, cpr, K, (unsigned*)ctr,
                                                              (uint64_t*)rec, (uint64_t*)steps);
    }
    return (int)hipGetLastError();
}
