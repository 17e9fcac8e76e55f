// acx_features.hip -- scoring inputs for value-guided search, computed on the GPU from
// presentations or from acx_expand12's packed child keys (so children never have to be
// materialised as int32 rows to be scored).
//
//   acx_features   the 14 hand-crafted features of value_search/feature_extraction.py:11-91
//                  (compute_features), optionally normalised (f - mean) / std as
//                  value_guided_search.py:49-66 (_score_states_mlp) does before the MLP.
//   acx_token_ids  the SequenceValueNet input of value_guided_search.py:68-84
//                  (_score_states_seq): letter + 2 as int64, padded with 2 to max_state_dim.
//
// Bit-exactness: counts are integers; length_ratio and max_min_ratio are computed as the
// reference does (Python float = double division, then rounded to float32 by np.array);
// normalisation uses IEEE float32 subtract and divide like the numpy float32 arrays.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx.h"
#include "acx_moves.h"

namespace acx {
namespace feat {

constexpr int TPB = 256;
constexpr int NF = 14;

struct Counts {
    int n[2];       // relator lengths (count_nonzero of each half)
    int c[2][4];    // per relator: count of x, x^-1, y, y^-1 among the first n letters
};

__device__ __forceinline__ void write_features(const Counts& k, float* out, const float* mean, const float* stdv) {
    const int n0 = k.n[0], n1 = k.n[1], tot = n0 + n1;
    const int ex = (k.c[0][0] - k.c[0][1]) + (k.c[1][0] - k.c[1][1]);
    const double ratio = tot > 0 ? (double)n0 / (double)tot : 0.5;
    const int mn = n0 < n1 ? n0 : n1, mx = n0 < n1 ? n1 : n0;
    const double mmr = mn > 0 ? (double)mx / (double)mn : (double)mx;
    float f[NF] = {(float)tot,       (float)n0,        (float)n1,        (float)k.c[0][0], (float)k.c[0][1],
                   (float)k.c[0][2], (float)k.c[0][3], (float)k.c[1][0], (float)k.c[1][1], (float)k.c[1][2],
                   (float)k.c[1][3], (float)ex,        (float)ratio,     (float)mmr};
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        float v = f[i];
        if (mean) v = (v - mean[i]) / stdv[i];
        out[i] = v;
    }
}

// count of 2-bit fields equal to `code` among the first n letters of w
template <int NW>
__device__ __forceinline__ int count_code(const Word<NW>& w, int n, uint32_t code) {
    const Word<NW> m = wmask<NW>(2 * n);
    const uint32_t rep = code * P55;
    int c = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t x = w.w[k] ^ rep;
        c += __popc(~(x | (x >> 1)) & P55 & m.w[k]);
    }
    return c;
}

// features from packed keys (acx.h key format), one lane per key
template <int NW>
__global__ __launch_bounds__(TPB) void features_keys_kernel(const uint64_t* keys, float* out, const float* mean,
                                                            const float* stdv, int64_t M, int L, int kw) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= M) return;
    PresRegs<NW> p;
    load_key<NW>(keys + i * kw, kw, L, p);
    Counts k;
    k.n[0] = p.n0;
    k.n[1] = p.n1;
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) {
        k.c[0][c] = count_code<NW>(p.w0, p.n0, c);
        k.c[1][c] = count_code<NW>(p.w1, p.n1, c);
    }
    write_features(k, out + i * NF, mean, stdv);
}

// features from int32 presentations (M, 2L), any int32 letters (as the reference's numpy
// code accepts them): length = count_nonzero of the half, counts over its first `length`
// entries
__global__ __launch_bounds__(TPB) void features_states_kernel(const int32_t* states, float* out, const float* mean,
                                                              const float* stdv, int64_t M, int L) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= M) return;
    const int32_t* s = states + i * 2 * L;
    Counts k;
    for (int h = 0; h < 2; ++h) {
        int n = 0;
        for (int j = 0; j < L; ++j) n += s[h * L + j] != 0;
        k.n[h] = n;
        k.c[h][0] = k.c[h][1] = k.c[h][2] = k.c[h][3] = 0;
        for (int j = 0; j < n; ++j) {
            const int32_t v = s[h * L + j];
            k.c[h][0] += v == 1;
            k.c[h][1] += v == -1;
            k.c[h][2] += v == 2;
            k.c[h][3] += v == -2;
        }
    }
    write_features(k, out + i * NF, mean, stdv);
}

// token ids, one thread per output element (coalesced int64 stores)
__global__ __launch_bounds__(TPB) void tokens_keys_kernel(const uint64_t* keys, int64_t* out, int64_t M, int L,
                                                          int kw, int D) {
    const int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (e >= M * D) return;
    const int64_t i = e / D;
    const int j = (int)(e - i * D);
    int64_t tok = 2;
    if (j < 2 * L) {
        const uint64_t* k = keys + i * kw;
        const int lb = 4 * L;
        const uint64_t lo = k[lb >> 6] >> (lb & 63);
        const uint64_t hi = (lb & 63) > 48 ? (k[(lb >> 6) + 1] << (64 - (lb & 63))) : 0ull;
        const int h = j >= L;
        const int n = (int)(((lo | hi) >> (8 * h)) & 0xffu);
        const int pos = j - h * L;
        if (pos < n) {
            const int b = 2 * j;
            const uint32_t code = (uint32_t)(k[b >> 6] >> (b & 63)) & 3u;
            tok = (int64_t)((code & 2u) ? 2 : 1) * ((code & 1u) ? -1 : 1) + 2;
        }
    }
    out[e] = tok;
}

__global__ __launch_bounds__(TPB) void tokens_states_kernel(const int32_t* states, int64_t* out, int64_t M, int L,
                                                            int D) {
    const int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (e >= M * D) return;
    const int64_t i = e / D;
    const int j = (int)(e - i * D);
    out[e] = j < 2 * L ? (int64_t)states[i * 2 * L + j] + 2 : 2;
}

static inline int nw_for(int L) { return L <= 16 ? 1 : L <= 32 ? 2 : L <= 48 ? 3 : L <= 64 ? 4 : 8; }

static inline unsigned blocks(int64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

}  // namespace feat
}  // namespace acx

using namespace acx::feat;

extern "C" {

int acx_features(const int32_t* states, const uint64_t* keys, const float* mean, const float* stdv, float* out,
                 int64_t M, int32_t L, void* stream) {
    if (M < 0 || L < 1 || L > ACX_MAX_L || (!mean != !stdv)) return ACX_E_ARG;
    if (M == 0) return ACX_OK;  // (an empty tensor's data pointer may be NULL)
    if (!out || (!states == !keys)) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (states) {
        features_states_kernel<<<dim3(blocks(M)), dim3(TPB), 0, st>>>(states, out, mean, stdv, M, L);
    } else {
        const int kw = acx_key_words(L);
        switch (nw_for(L)) {
            case 1: features_keys_kernel<1><<<dim3(blocks(M)), dim3(TPB), 0, st>>>(keys, out, mean, stdv, M, L, kw); break;
            case 2: features_keys_kernel<2><<<dim3(blocks(M)), dim3(TPB), 0, st>>>(keys, out, mean, stdv, M, L, kw); break;
            case 3: features_keys_kernel<3><<<dim3(blocks(M)), dim3(TPB), 0, st>>>(keys, out, mean, stdv, M, L, kw); break;
            case 4: features_keys_kernel<4><<<dim3(blocks(M)), dim3(TPB), 0, st>>>(keys, out, mean, stdv, M, L, kw); break;
            default: features_keys_kernel<8><<<dim3(blocks(M)), dim3(TPB), 0, st>>>(keys, out, mean, stdv, M, L, kw); break;
        }
    }
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

int acx_token_ids(const int32_t* states, const uint64_t* keys, int64_t* out, int64_t M, int32_t L,
                  int32_t max_state_dim, void* stream) {
    if (M < 0 || L < 1 || L > ACX_MAX_L || max_state_dim < 2 * L) return ACX_E_ARG;
    if (M == 0) return ACX_OK;
    if (!out || (!states == !keys)) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = M * (int64_t)max_state_dim;
    if (states) tokens_states_kernel<<<dim3(blocks(n)), dim3(TPB), 0, st>>>(states, out, M, L, max_state_dim);
    else tokens_keys_kernel<<<dim3(blocks(n)), dim3(TPB), 0, st>>>(keys, out, M, L, acx_key_words(L), max_state_dim);
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

}  // extern "C"
