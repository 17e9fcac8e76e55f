// Move-kernel microbenchmark (tools only, not the product): the packed 2-bit-code move
// (acx_moves.h ac_move_clean, Word<3>) against a bit-plane prototype (move_planes_proto.h: the
// two bits of each letter in two uint64 planes, 64-bit shifts / bit reversal), lane per env,
// T cyclic moves per launch on states in registers.  Both write their final states as 2-bit
// codes so the python driver (move_probe.py) can check them equal.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx_moves.h"
#include "move_planes_proto.h"

using namespace acx;

__device__ __forceinline__ uint64_t spread(uint64_t x) {  // bit k -> bit 2k (32 low bits)
    x &= 0xffffffffull;
    x = (x | (x << 16)) & 0x0000ffff0000ffffull;
    x = (x | (x << 8)) & 0x00ff00ff00ff00ffull;
    x = (x | (x << 4)) & 0x0f0f0f0f0f0f0f0full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// codes: (B, 8) uint32: w0[3], w1[3], n0, n1 (acx Word<3> layout); actions (T) uint32 seeds
__global__ void codes_kernel(uint32_t* st, const uint32_t* acts, int T, int L, int64_t B) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= B) return;
    Word<3> w0, w1;
    int n0 = (int)st[t * 8 + 6], n1 = (int)st[t * 8 + 7];
    for (int k = 0; k < 3; ++k) { w0.w[k] = st[t * 8 + k]; w1.w[k] = st[t * 8 + 3 + k]; }
    int e = 0;
    for (int s = 0; s < T; ++s) {
        const int a = (int)((acts[s] >> (t & 15)) % 12u);
        e |= ac_move_clean<3>(w0, n0, w1, n1, a, L, true);
    }
    for (int k = 0; k < 3; ++k) { st[t * 8 + k] = w0.w[k]; st[t * 8 + 3 + k] = w1.w[k]; }
    st[t * 8 + 6] = (uint32_t)n0 | ((uint32_t)e << 16);
    st[t * 8 + 7] = (uint32_t)n1;
}

__device__ __forceinline__ pl::W to_planes(const uint32_t* w) {
    pl::W r{0, 0};
    for (int k = 0; k < 48; ++k) {
        const uint32_t c = (w[k >> 4] >> (2 * (k & 15))) & 3u;
        r.p0 |= (uint64_t)(c & 1u) << k;
        r.p1 |= (uint64_t)(c >> 1) << k;
    }
    return r;
}

__global__ void planes_kernel(uint32_t* st, const uint32_t* acts, int T, int L, int64_t B) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= B) return;
    pl::W w0 = to_planes(st + t * 8), w1 = to_planes(st + t * 8 + 3);
    int n0 = (int)st[t * 8 + 6], n1 = (int)st[t * 8 + 7];
    int e = 0;
    for (int s = 0; s < T; ++s) {
        const int a = (int)((acts[s] >> (t & 15)) % 12u);
        e |= pl::move_clean(w0, n0, w1, n1, a, L, true);
    }
    for (int h = 0; h < 2; ++h) {
        const pl::W& w = h ? w1 : w0;
        const uint64_t lo = spread(w.p0) | (spread(w.p1) << 1);
        const uint64_t hi = spread(w.p0 >> 32) | (spread(w.p1 >> 32) << 1);
        st[t * 8 + 3 * h] = (uint32_t)lo;
        st[t * 8 + 3 * h + 1] = (uint32_t)(lo >> 32);
        st[t * 8 + 3 * h + 2] = (uint32_t)hi;
    }
    st[t * 8 + 6] = (uint32_t)n0 | ((uint32_t)e << 16);
    st[t * 8 + 7] = (uint32_t)n1;
}

extern "C" {
int probe_codes(uint32_t* st, const uint32_t* acts, int T, int L, int64_t B, void* s) {
    codes_kernel<<<dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)s>>>(st, acts, T, L, B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int probe_planes(uint32_t* st, const uint32_t* acts, int T, int L, int64_t B, void* s) {
    planes_kernel<<<dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)s>>>(st, acts, T, L, B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
