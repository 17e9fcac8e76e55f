// Store-pattern microbenchmark: how fast can the rollout's HBM access pattern go with no
// move compute?  Each wave owns a 64-row tile (18 KB at L=36) and, per step t, writes it to
// obs[t] as 18 coalesced 1 KB wave-stores -- exactly the acx_rollout obs pattern.  Feature
// bits add the rollout's other traffic one at a time, to find what costs bandwidth:
//   F_NT      non-temporal obs stores
//   F_SCAL    per-step reward (int32) / done / truncated (u8) stores
//   F_ACT8    per-lane int32 action loads, ACT_BLOCK = 8 steps per load batch (waits vmcnt)
//   F_ACTPF   the same loads, issued one batch ahead (prefetch; consumed 8 steps later)
//   F_LDS     obs rows staged through LDS (write 18 dwords per lane, read back per chunk)
//   F_ACT32   action loads in 32-step batches (4 groups of 8; one drain per 32 steps)
//   F_PACK8   pre-packed actions: one uint32 (8 ids x 4 bits) per lane per 8 steps
//   F_BLK     the block's 4 waves write its 4 tiles interleaved (wave k: every 4th KB) after a
//             per-step barrier: 4 KB contiguous per store instruction round instead of 1 KB
//   F_ROT     each wave starts its tile's stores at chunk (tile mod row_chunks), so waves in
//             lockstep do not all write the same offset of their tiles at the same time
// Compared with the same bytes written linearly (grid-stride, like a fill).
#include <hip/hip_runtime.h>
#include <stdint.h>

enum { F_NT = 1, F_SCAL = 2, F_ACT8 = 4, F_ACTPF = 8, F_LDS = 16, F_ACT32 = 32, F_PACK8 = 64, F_BLK = 128, F_ROT = 256 };

typedef int v4i __attribute__((ext_vector_type(4)));

template <int F>
__global__ __launch_bounds__(256, 8) void tile_pattern(int4* obs, int32_t* rew, uint8_t* dn, uint8_t* tr,
                                                       const int32_t* act, int64_t B, int T, int row_chunks) {
    __shared__ uint32_t lds[4][64 * 18];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * 4 + wid;
    if (tile * 64 >= B) return;
    const int64_t chunks_per_step = B * row_chunks;
    const int64_t env = tile * 64 + lane;
    int4 v = make_int4(lane, 1, 2, 3);
    uint32_t acc = 0, acts = 0;
    int32_t nv[8];  // prefetched raw action loads of the next batch (consumed 8 steps later)
    if (F & F_ACTPF) {
        // rows clamped to T - 1: an unguarded k < 8 read runs past the (T, B) id array when
        // T < 8 -- the round-1 rollout prefetch faulted the same way on its last batch, reading
        // rows t + 8.. >= T past the end of the allocation at full size
        for (int k = 0; k < 8; ++k) nv[k] = act[(int64_t)(k < T ? k : T - 1) * B + env];
    }
    for (int t = 0; t < T; ++t) {
        if ((F & (F_ACT8 | F_ACTPF)) && (t & 7) == 0) {
            if (F & F_ACTPF) {
                acts = 0;
                for (int k = 0; k < 8; ++k) acts |= (uint32_t)nv[k] << (4 * k);
                for (int k = 0; k < 8; ++k) {
                    const int tt = t + 8 + k < T ? t + 8 + k : T - 1;
                    nv[k] = act[(int64_t)tt * B + env];
                }
            } else {
                acts = 0;
                for (int k = 0; k < 8; ++k)
                    acts |= (t + k < T) ? (uint32_t)act[(int64_t)(t + k) * B + env] << (4 * k) : 0u;
            }
        }
        if ((F & F_ACT32) && (t & 31) == 0) {
            for (int g = 0; g < 4; ++g) {
                int32_t v8[8];
                for (int k = 0; k < 8; ++k) v8[k] = (t + 8 * g + k < T) ? act[(int64_t)(t + 8 * g + k) * B + env] : 0;
                uint32_t qg = 0;
                for (int k = 0; k < 8; ++k) qg |= (uint32_t)v8[k] << (4 * k);
                acc += qg;
            }
        }
        if ((F & F_PACK8) && (t & 7) == 0) acts = (uint32_t)act[(int64_t)(t >> 3) * B + env];
        if (F & (F_ACT8 | F_ACTPF | F_PACK8)) acc += (acts >> (4 * (t & 7))) & 15u;
        v.y += 1 + (int)acc;
        if (F & F_SCAL) {
            rew[(int64_t)t * B + env] = v.y;
            dn[(int64_t)t * B + env] = (uint8_t)v.y;
            tr[(int64_t)t * B + env] = (uint8_t)(v.y >> 8);
        }
        int4* dst = obs + t * chunks_per_step + tile * 64 * row_chunks + lane;
        if (F & F_LDS) {
            uint32_t* row = &lds[wid][lane * 18];
            for (int k = 0; k < 18; k += 2) *reinterpret_cast<uint2*>(row + k) = make_uint2(v.y + k, v.x + k);
            __builtin_amdgcn_wave_barrier();
            for (int u = 0; u < row_chunks; ++u) {
                const uint32_t p = lds[wid][lane + 64 * u];
                const v4i x = {(int)(p & 0xff), (int)((p >> 8) & 0xff), (int)((p >> 16) & 0xff), (int)(p >> 24)};
                if (F & F_NT) __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(dst + u * 64));
                else *reinterpret_cast<v4i*>(dst + u * 64) = x;
            }
            __builtin_amdgcn_wave_barrier();
        } else if (F & F_BLK) {
            __syncthreads();
            int4* bdst = obs + t * chunks_per_step + (int64_t)blockIdx.x * 4 * 64 * row_chunks + lane;
            for (int u = 0; u < row_chunks; ++u) {
                const v4i x = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(bdst + (u * 4 + wid) * 64));
            }
        } else if (F & F_ROT) {
            const int rot = (int)(tile % row_chunks);
            for (int u = 0; u < row_chunks; ++u) {
                int uu = u + rot;
                uu = uu >= row_chunks ? uu - row_chunks : uu;
                v4i x = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(dst + uu * 64));
            }
        } else {
            for (int u = 0; u < row_chunks; ++u) {
                if (F & F_NT) {
                    v4i x = {v.x, v.y, v.z, v.w};
                    __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(dst + u * 64));
                } else {
                    dst[u * 64] = v;
                }
            }
        }
    }
}

// tile_pattern<F_NT> with extra dynamic LDS per block, to cap the resident blocks per CU (and so
// the write window: resident waves x 18 KB) -- occupancy vs placement sensitivity
extern "C" int sp_tile_occ(void* obs, int64_t B, int T, int row_chunks, int lds_pad, void* stream) {
    if (B <= 0 || B % 64 != 0 || T <= 0 || row_chunks <= 0 || lds_pad < 0) return -1;
    dim3 grid((unsigned)((B + 255) / 256));
    tile_pattern<F_NT><<<grid, 256, (size_t)lds_pad, (hipStream_t)stream>>>((int4*)obs, nullptr, nullptr, nullptr,
                                                                           nullptr, B, T, row_chunks);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// each wave owns TWO 64-row tiles and writes both every step (4 waves/SIMD, so a 2^20-env batch
// is resident in one round instead of two rounds of one-tile waves)
__global__ __launch_bounds__(256, 4) void tile2_pattern(int4* obs, int64_t B, int T, int row_chunks) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int64_t pair = (int64_t)blockIdx.x * 4 + wid;
    if (pair * 128 >= B) return;
    const int64_t chunks_per_step = B * row_chunks;
    int4 v = make_int4(lane, 1, 2, 3);
    for (int t = 0; t < T; ++t) {
        v.y += 1;
        for (int h = 0; h < 2; ++h) {
            int4* dst = obs + t * chunks_per_step + (2 * pair + h) * 64 * row_chunks + lane;
            for (int u = 0; u < row_chunks; ++u) {
                v4i x = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(dst + u * 64));
            }
        }
    }
}
extern "C" int sp_tile2(void* obs, int64_t B, int T, int row_chunks, void* stream) {
    if (B <= 0 || B % 128 != 0 || T <= 0) return -1;
    tile2_pattern<<<(unsigned)((B + 511) / 512), 256, 0, (hipStream_t)stream>>>((int4*)obs, B, T, row_chunks);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

__global__ __launch_bounds__(256) void linear_fill(int4* p, int64_t n) {
    int4 v = make_int4(1, 2, 3, 4);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}

#define CASE(f)                                                                                    \
    case f:                                                                                        \
        tile_pattern<f><<<grid, 256, 0, (hipStream_t)stream>>>((int4*)obs, (int32_t*)rew, (uint8_t*)dn, \
                                                              (uint8_t*)tr, (const int32_t*)act, B, T, row_chunks); \
        break;

extern "C" int sp_tile(void* obs, void* rew, void* dn, void* tr, const void* act, int64_t B, int T, int row_chunks,
                       int flags, void* stream) {
    if (B <= 0 || B % 64 != 0 || T <= 0 || row_chunks <= 0) return -1;  // a wave writes whole 64-row tiles
    dim3 grid((unsigned)((B + 255) / 256));
    switch (flags) {
        CASE(0) CASE(1) CASE(3) CASE(5) CASE(9) CASE(7) CASE(11) CASE(17) CASE(19) CASE(23) CASE(27) CASE(33) CASE(51) CASE(65) CASE(83) CASE(129) CASE(257)
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
// each thread writes `per` consecutive 16-byte vectors (torch's elementwise launch shape)
__global__ __launch_bounds__(256) void chunk_fill(int4* p, int64_t n, int per) {
    int4 v = make_int4(1, 2, 3, 4);
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * per;
    for (int k = 0; k < per; ++k)
        if (i0 + k < n) p[i0 + k] = v;
}
extern "C" int sp_chunk(void* p, int64_t n16, int per, void* stream) {
    const int64_t threads = (n16 + per - 1) / per;
    chunk_fill<<<(unsigned)((threads + 255) / 256), 256, 0, (hipStream_t)stream>>>((int4*)p, n16, per);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
// streaming copy, one 16-byte vector per thread per iteration (grid-stride): the read+write
// ceiling the per-call step API (state in, state out) is measured against
__global__ __launch_bounds__(256) void copy16(const int4* __restrict__ src, int4* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}
// the step kernel's shape: each wave reads its whole tile (64 rows of row_chunks 16-byte chunks,
// coalesced) into registers 8 chunks at a time, then writes it out
__global__ __launch_bounds__(256) void tile_copy(const int4* __restrict__ src, int4* __restrict__ dst, int64_t B,
                                                 int row_chunks) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile * 64 >= B) return;
    const int64_t base = tile * 64 * row_chunks + lane;
    const int n = 64 * row_chunks / 64;  // chunks per lane
    for (int u0 = 0; u0 < n; u0 += 8) {
        int4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (u0 + u < n) v[u] = src[base + (int64_t)(u0 + u) * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (u0 + u < n) dst[base + (int64_t)(u0 + u) * 64] = v[u];
    }
}
extern "C" int sp_copy(const void* src, void* dst, int64_t n16, int mode, int64_t B, int row_chunks, void* stream) {
    if (mode == 0) {
        copy16<<<8192, 256, 0, (hipStream_t)stream>>>((const int4*)src, (int4*)dst, n16);
    } else {
        if (B % 64 != 0 || B * row_chunks != n16) return -1;
        tile_copy<<<(unsigned)((B / 64 + 3) / 4), 256, 0, (hipStream_t)stream>>>((const int4*)src, (int4*)dst, B,
                                                                                   row_chunks);
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
extern "C" int sp_linear(void* p, int64_t n16, int blocks, void* stream) {
    linear_fill<<<blocks, 256, 0, (hipStream_t)stream>>>((int4*)p, n16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
