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

// One block per tile, but the tiles dealt to the XCDs unevenly: block b runs on XCC b % 8 (the
// dispatcher's round-robin, checked by kind 0's records); the even XCCs take E tiles each, the odd
// ones O (4E + 4O = tiles), each XCC a contiguous range; blocks beyond their XCC's quota exit.
__global__ __launch_bounds__(256) void tile_weighted(int4* __restrict__ dst, int64_t rows, int cpr, int K, int E,
                                                     int O, uint64_t* __restrict__ rec, uint64_t* __restrict__ steps) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int quota = (x & 1) ? O : E;
    const int64_t base = (int64_t)((x + 1) / 2) * E + (int64_t)(x / 2) * O;  // tiles of XCCs < x
    const bool work = j < quota;
    const int64_t tile = base + j;
    const int nch = WAVE * cpr;
    if (work) {
        const int64_t r0 = (tile * 4 + wid) * WAVE;
        for (int t = 0; t < K; ++t) {
            if (wid == 0 && lane == 0) steps[tile * K + t] = __builtin_amdgcn_s_memrealtime();
            int4* row = dst + ((int64_t)t * rows + r0) * cpr;
            for (int c = lane; c < nch; c += WAVE) st_nt(row + c, make_int4(7, t, c, lane));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0 && work) {
        rec[4 * tile + 0] = t_start;
        rec[4 * tile + 1] = __builtin_amdgcn_s_memrealtime();
        rec[4 * tile + 2] = xcc_id();
        rec[4 * tile + 3] = 1;
    }
}

// One block per tile, the tile taken from a ticket counter by a grid of over/100 x tiles blocks:
// an XCC that writes faster finishes its blocks sooner and its later blocks take more tickets;
// blocks that find the tickets gone exit.  ctr[0] tickets, ctr[1] blocks out (the last resets both).
__global__ __launch_bounds__(256) void tile_ticket(int4* __restrict__ dst, int64_t rows, int cpr, int K,
                                                   unsigned* __restrict__ ctr, uint64_t* __restrict__ rec,
                                                   uint64_t* __restrict__ steps) {
    __shared__ unsigned s_tile;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned ntiles = (unsigned)(rows / 256);
    if (threadIdx.x == 0) s_tile = atomicAdd(&ctr[0], 1u);
    __syncthreads();
    const unsigned tile = s_tile;
    const int nch = WAVE * cpr;
    if (tile < ntiles) {
        const int64_t r0 = ((int64_t)tile * 4 + wid) * WAVE;
        for (int t = 0; t < K; ++t) {
            if (wid == 0 && lane == 0) steps[(int64_t)tile * K + t] = __builtin_amdgcn_s_memrealtime();
            int4* row = dst + ((int64_t)t * rows + r0) * cpr;
            for (int c = lane; c < nch; c += WAVE) st_nt(row + c, make_int4(7, t, c, lane));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (tile < ntiles) {
            rec[4 * tile + 0] = t_start;
            rec[4 * tile + 1] = __builtin_amdgcn_s_memrealtime();
            rec[4 * tile + 2] = xcc_id();
            rec[4 * tile + 3] = 1;
        }
        __threadfence();
        if (atomicAdd(&ctr[1], 1u) == gridDim.x - 1) {
            atomicExch(&ctr[0], 0u);
            atomicExch(&ctr[1], 0u);
        }
    }
}

// One block per tile (kind 0), but a wave's issue priority falls with its progress (s_setprio
// 3 at the start, 0 in its last quarter of steps): the arbiter serves the waves that are behind
// first instead of the oldest, so a SIMD's waves advance together
__device__ __forceinline__ void set_prio(int q) {
    switch (q) {
        case 0: __builtin_amdgcn_s_setprio(3); break;
        case 1: __builtin_amdgcn_s_setprio(2); break;
        case 2: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
    }
}
__global__ __launch_bounds__(256) void tile_fair(int4* __restrict__ dst, int64_t rows, int cpr, int K, int mode,
                                                 uint64_t* __restrict__ rec, uint64_t* __restrict__ steps) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wid) * WAVE;
    const int nch = WAVE * cpr;
    if (r0 < rows) {
        for (int t = 0; t < K; ++t) {
            // mode 1: by progress quarter; mode 2: young waves first (3 for the whole wave's life
            // after its first step, so a new wave overtakes the old ones); mode 3: plain 0..3 by
            // block index (a fixed random-ish order)
            if (mode == 1) set_prio((4 * t) / K);
            else if (mode == 2) set_prio(t == 0 ? 3 : 0);
            else set_prio((int)(blockIdx.x * 7 % 4));
            if (wid == 0 && lane == 0) steps[(int64_t)blockIdx.x * K + t] = __builtin_amdgcn_s_memrealtime();
            int4* row = dst + ((int64_t)t * rows + r0) * cpr;
            for (int c = lane; c < nch; c += WAVE) st_nt(row + c, make_int4(7, t, c, lane));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        rec[4 * blockIdx.x + 0] = t_start;
        rec[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        rec[4 * blockIdx.x + 2] = xcc_id();
        rec[4 * blockIdx.x + 3] = 0;
    }
}

// kind 0: one block per tile (the rollout's launch); 1: persistent blocks, dynamic tiles;
// 2: persistent blocks, static tiles; 3: one block per tile, odd XCCs dealt grid/100 % of an even
// XCC's tiles (grid = that percentage here).  grid: persistent blocks (rec / steps sized for the larger)
extern "C" int timeline_tile(int kind, void* buf, int64_t rows, int L, int K, int grid, void* ctr, void* rec,
                             void* steps, void* stream) {
    if (rows % 256 || K < 1 || grid < 1) return -1;
    const int cpr = 2 * L / 4;
    hipStream_t s = (hipStream_t)stream;
    if (kind == 0) {
        tile_timed<<<dim3((unsigned)(rows / 256)), dim3(256), 0, s>>>((int4*)buf, rows, cpr, K, (uint64_t*)rec,
                                                                       (uint64_t*)steps);
    } else if (kind == 5) {
        tile_fair<<<dim3((unsigned)(rows / 256)), dim3(256), 0, s>>>((int4*)buf, rows, cpr, K, grid, (uint64_t*)rec,
                                                                     (uint64_t*)steps);
    } else if (kind == 4) {
        const unsigned tiles = (unsigned)(rows / 256);
        tile_ticket<<<dim3((unsigned)((uint64_t)tiles * grid / 100)), dim3(256), 0, s>>>(
            (int4*)buf, rows, cpr, K, (unsigned*)ctr, (uint64_t*)rec, (uint64_t*)steps);
    } else if (kind == 3) {
        const int tiles = (int)(rows / 256);
        // 4E + 4O = tiles with O = E * pct / 100
        int E = (int)((double)tiles / (4.0 * (1.0 + grid / 100.0)) + 0.5);
        int O = tiles / 4 - E;
        if (O < 0 || E < O) return -3;
        tile_weighted<<<dim3((unsigned)(8 * E)), dim3(256), 0, s>>>((int4*)buf, rows, cpr, K, E, O, (uint64_t*)rec,
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
