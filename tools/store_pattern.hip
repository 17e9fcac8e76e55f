// Store-pattern microbenchmark: how fast can the rollout's obs-trajectory write pattern go
// with no compute?  Each wave owns a 64-row tile (18 KB at L=36) and, per step t, writes it
// to obs[t] as 18 coalesced 1 KB wave-stores -- exactly the acx_rollout pattern.  Compared
// with the same bytes written linearly (grid-stride, like a fill).
#include <hip/hip_runtime.h>
#include <stdint.h>

template <bool NT>
__global__ __launch_bounds__(256, 8) void tile_pattern(int4* obs, int64_t B, int T, int row_chunks) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile * 64 >= B) return;
    const int64_t chunks_per_step = B * row_chunks;
    int4 v = make_int4(lane, 1, 2, 3);
    for (int t = 0; t < T; ++t) {
        int4* dst = obs + t * chunks_per_step + tile * 64 * row_chunks + lane;
        for (int u = 0; u < row_chunks; ++u) {
            if (NT) {
                typedef int v4i __attribute__((ext_vector_type(4)));
                v4i x = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(dst + u * 64));
            } else {
                dst[u * 64] = v;
            }
        }
        v.y += 1;
    }
}

__global__ __launch_bounds__(256) void linear_fill(int4* p, int64_t n) {
    int4 v = make_int4(1, 2, 3, 4);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}

extern "C" int sp_tile(void* obs, int64_t B, int T, int row_chunks, int nt, void* stream) {
    dim3 grid((unsigned)((B + 255) / 256));
    if (nt) tile_pattern<true><<<grid, 256, 0, (hipStream_t)stream>>>((int4*)obs, B, T, row_chunks);
    else tile_pattern<false><<<grid, 256, 0, (hipStream_t)stream>>>((int4*)obs, B, T, row_chunks);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
extern "C" int sp_linear(void* p, int64_t n16, int blocks, void* stream) {
    linear_fill<<<blocks, 256, 0, (hipStream_t)stream>>>((int4*)p, n16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
