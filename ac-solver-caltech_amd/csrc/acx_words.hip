// acx_words.hip -- the reference's word functions on ARBITRARY int32 letters, batched on the GPU.
//
// The fast kernels (acx_kernels.hip) pack letters +-1 / +-2 at 2 bits each; the reference's word
// functions are generator-agnostic (its unit tests use letters 3..6, tests/test_ac_env.py:17-326)
// and behave literally on inputs with zeros inside a relator.  This file restates them exactly on
// int32 letters, one lane per row, with each row staged through LDS (coalesced row loads and
// stores; odd row strides, so the lanes' per-letter accesses hit distinct banks):
//   concatenate_relators   ac_solver/envs/ac_moves.py:4-76
//   conjugate              ac_solver/envs/ac_moves.py:79-156
//   ACMove                 ac_solver/envs/ac_moves.py:159-231
//   simplify_relator       ac_solver/envs/utils.py:178-243
//   simplify_presentation  ac_solver/envs/utils.py:246-283
//   is_presentation_trivial (done)  ac_solver/envs/utils.py:57-87
// Errors are the reference's exceptions as ACX_ERR_* codes (acx.h): AssertionError ->
// ACX_ERR_INVALID, IndexError -> ACX_ERR_EMPTY_CONJ, bad move id -> ACX_ERR_ACTION, np.pad with a
// negative width (ValueError) -> ACX_ERR_PAD.  A row whose call raises keeps its input.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx.h"

namespace acx {
namespace words {

constexpr int LANES = 64;             // rows per block (one wave)
constexpr size_t LDS_BUDGET = 160 * 1024;

enum Op : int { OP_MOVE = 0, OP_CONCAT = 1, OP_CONJ = 2, OP_SIMPLIFY_PRES = 3, OP_SIMPLIFY_REL = 4 };

struct Args {
    const int32_t* in;      // (B, win)
    int32_t* out;           // (B, wout)
    const int32_t* action;  // OP_MOVE: (B) move ids
    const int32_t* lengths_in;  // OP_CONCAT / OP_CONJ: (B, 2) caller's lengths list or NULL (counts)
    int32_t* lengths_out;   // (B, 2): OP_MOVE / OP_CONCAT / OP_CONJ / OP_SIMPLIFY_PRES
    int32_t* n_out;         // OP_SIMPLIFY_REL: (B) word length
    int32_t* len_out;       // OP_SIMPLIFY_REL: (B) length of the returned array
    uint8_t* done;          // OP_MOVE: (B) strict triviality of the result (ac_env.py:99) or NULL
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int L, win, wout, stride, cyc, i, j, sign, padded;
};

__device__ __forceinline__ int nonzero_count(const int32_t* r, int n) {
    int c = 0;
    for (int k = 0; k < n; ++k) c += r[k] != 0;
    return c;
}

// utils.py:13-54 on a presentation of 2L letters
__device__ __forceinline__ bool is_valid(const int32_t* p, int L) {
    for (int h = 0; h < 2; ++h) {
        const int32_t* r = p + h * L;
        const int nz = nonzero_count(r, L);
        if (nz == 0) return false;
        for (int k = nz; k < L; ++k)
            if (r[k] != 0) return false;
    }
    return true;
}

// utils.py:57-87
__device__ __forceinline__ bool is_trivial(const int32_t* p, int L) {
    if (!is_valid(p, L)) return false;
    if (nonzero_count(p, L) != 1 || nonzero_count(p + L, L) != 1) return false;
    int a = p[0] < 0 ? -p[0] : p[0], b = p[L] < 0 ? -p[L] : p[L];
    if (a > b) { const int t = a; a = b; b = t; }
    return a == 1 && b == 2;
}

// utils.py:178-243, in place on r[0..m) (m = the array's length; np.delete shrinks it, so the
// array length `len` is tracked apart from the word length n).  The result occupies r[0..*out_len)
// (padded: exactly L entries).  Returns an ACX_ERR_* code.
__device__ int simplify_relator(int32_t* r, int m, int L, bool cyc, bool padded, int* out_len, int* n_out) {
    int len = m;
    int n = nonzero_count(r, m);
    for (int k = n; k < m; ++k)
        if (r[k] != 0) return ACX_ERR_INVALID;  // "expect all zeros to be at the right end"
    int pos = 0;
    while (pos < n - 1) {
        if (r[pos] == -r[pos + 1]) {  // np.delete(relator, [pos, pos + 1])
            for (int k = pos; k + 2 < len; ++k) r[k] = r[k + 2];
            len -= 2;
            n -= 2;
            if (pos) pos -= 1;
        } else {
            pos += 1;
        }
    }
    if (cyc && n > 0) {
        int q = 0;
        while (q < n && r[q] == -r[n - q - 1]) ++q;
        if (q) {  // np.delete of indices [0, q) and [n - q, n)
            int w = 0;
            for (int k = 0; k < len; ++k) {
                if (k < q || (k >= n - q && k < n)) continue;
                r[w++] = r[k];
            }
            len = w;
            n -= 2 * q;
        }
    }
    if (padded) {
        if (L - len < 0) return ACX_ERR_PAD;  // np.pad with a negative width raises ValueError
        for (int k = len; k < L; ++k) r[k] = 0;
        len = L;
    }
    if (L < n) return ACX_ERR_INVALID;  // "Increase max length!"
    *out_len = len;
    *n_out = n;
    return ACX_ERR_NONE;
}

// utils.py:246-283 in place on p (2L letters); tmp: >= L scratch letters
__device__ int simplify_presentation(int32_t* p, int32_t* tmp, int L, bool cyc, int* lens) {
    if (!is_valid(p, L)) return ACX_ERR_INVALID;
    for (int h = 0; h < 2; ++h) {
        for (int k = 0; k < L; ++k) tmp[k] = p[h * L + k];
        int ol = 0, n = 0;
        const int e = simplify_relator(tmp, L, L, cyc, true, &ol, &n);
        if (e != ACX_ERR_NONE) return e;
        for (int k = 0; k < L; ++k) p[h * L + k] = tmp[k];
        lens[h] = n;
    }
    return ACX_ERR_NONE;
}

// ac_moves.py:4-76 in place on p; tmp: >= 2L scratch letters.  lens[i] = new size when it fits
// (the reference writes the caller's list, :65), otherwise lens is left as given.
__device__ void concatenate(int32_t* p, int32_t* tmp, int L, int i, int j, int sign, int* lens) {
    int32_t* r1 = tmp;
    int32_t* r2 = tmp + L;
    int n1 = 0, n2 = 0;
    for (int k = 0; k < L; ++k)
        if (p[i * L + k] != 0) r1[n1++] = p[i * L + k];
    for (int k = 0; k < L; ++k) {  // sign -1: negated reversal of the padded half, then the filter
        const int32_t v = sign == 1 ? p[j * L + k] : -p[j * L + (L - 1 - k)];
        if (v != 0) r2[n2++] = v;
    }
    const int mn = n1 < n2 ? n1 : n2;
    int acc = 0;
    while (acc < mn && r1[n1 - 1 - acc] == -r2[acc]) ++acc;
    const int ns = n1 + n2 - 2 * acc;
    if (ns <= L) {
        lens[i] = ns;
        int32_t* dst = p + i * L;
        int w = 0;
        for (int k = 0; k < n1 - acc; ++k) dst[w++] = r1[k];
        for (int k = acc; k < n2; ++k) dst[w++] = r2[k];
        for (; w < L; ++w) dst[w] = 0;
    }
}

// ac_moves.py:79-156 in place on p; tmp: >= L scratch letters
__device__ int conjugate(int32_t* p, int32_t* tmp, int L, int i, int j, int sign, int* lens) {
    int n = 0;
    for (int k = 0; k < L; ++k)
        if (p[i * L + k] != 0) tmp[n++] = p[i * L + k];
    if (n == 0) return ACX_ERR_EMPTY_CONJ;  // relator_nonzero[0] raises IndexError
    const int32_t g = sign * j;
    const int sc = tmp[0] == -g, ec = tmp[n - 1] == g;
    const int ns = n + 2 - 2 * (sc + ec);
    if (ns <= L) {
        lens[i] = ns;
        const int base = i * L;
        for (int k = sc; k < n - ec; ++k) p[base + 1 - sc + (k - sc)] = tmp[k];
        if (!sc) p[base] = g;
        if (!ec) p[base + n + 1 - 2 * sc] = -g;
        if (sc && ec) {
            p[base + ns] = 0;
            p[base + ns + 1] = 0;
        }
    }
    return ACX_ERR_NONE;
}

// ac_moves.py:159-231
__device__ int ac_move(int32_t* p, int32_t* tmp, int L, int move_id, bool cyc, int* lens) {
    if (move_id < 0 || move_id > 11) return ACX_ERR_ACTION;
    const int m = move_id + 1;
    int e = ACX_ERR_NONE;
    if (move_id < 4) {
        const int i = m % 2;
        concatenate(p, tmp, L, i, 1 - i, (((m - i) / 2) % 2) ? -1 : 1, lens);
    } else {
        const int i = m % 2;
        const int jp = ((m - i) / 2) % 2;
        e = conjugate(p, tmp, L, i, jp + 1, (((m - i - 2 * jp) / 4) % 2) ? -1 : 1, lens);
    }
    if (e == ACX_ERR_NONE) e = simplify_presentation(p, tmp, L, cyc, lens);
    return e;
}

__global__ __launch_bounds__(LANES) void words_kernel(Args a, int op) {
    extern __shared__ int32_t lds[];
    const int lane = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * blockDim.x;
    const int R = (int)((a.B - r0) < (int64_t)blockDim.x ? (a.B - r0) : (int64_t)blockDim.x);
    int32_t* rows = lds;                          // blockDim rows of `stride` letters
    int32_t* tmps = lds + blockDim.x * a.stride;  // and as many scratch rows
    // coalesced load of the block's input rows
    for (int64_t idx = lane; idx < (int64_t)R * a.win; idx += blockDim.x) {
        const int r = (int)(idx / a.win);
        rows[r * a.stride + (int)(idx - (int64_t)r * a.win)] = a.in[r0 * a.win + idx];
    }
    __syncthreads();
    const int64_t row = r0 + lane;
    if (lane < R) {
        int32_t* p = rows + lane * a.stride;
        int32_t* tmp = tmps + lane * a.stride;
        const int L = a.L;
        int lens[2];
        int e = ACX_ERR_NONE;
        if (op == OP_SIMPLIFY_REL) {
            int ol = 0, n = 0;
            e = simplify_relator(p, a.win, L, a.cyc != 0, a.padded != 0, &ol, &n);
            if (e != ACX_ERR_NONE) ol = a.win;  // the row is restored from the input below
            a.len_out[row] = ol;
            if (e == ACX_ERR_NONE) a.n_out[row] = n;
            for (int k = ol; k < a.wout; ++k) p[k] = 0;  // past the returned array: zeros
        } else {
            // the caller's lengths list (concatenate / conjugate return it, updated), else counts
            for (int h = 0; h < 2; ++h)
                lens[h] = a.lengths_in ? a.lengths_in[2 * row + h] : nonzero_count(p + h * L, L);
            if (op == OP_MOVE) {
                e = ac_move(p, tmp, L, a.action[row], a.cyc != 0, lens);
            } else if (op == OP_CONCAT) {
                concatenate(p, tmp, L, a.i, a.j, a.sign, lens);
            } else if (op == OP_CONJ) {
                e = conjugate(p, tmp, L, a.i, a.j, a.sign, lens);
            } else {
                e = simplify_presentation(p, tmp, L, a.cyc != 0, lens);
            }
            if (op == OP_MOVE && a.done) a.done[row] = e == ACX_ERR_NONE && lens[0] + lens[1] == 2 && is_trivial(p, L);
        }
        if (e != ACX_ERR_NONE) {  // the reference raises: the row keeps its input
            for (int k = 0; k < a.win; ++k) p[k] = a.in[row * a.win + k];
            for (int k = a.win; k < a.wout; ++k) p[k] = 0;
            if (op != OP_SIMPLIFY_REL)
                for (int h = 0; h < 2; ++h) lens[h] = nonzero_count(p + h * L, L);
        }
        if (op != OP_SIMPLIFY_REL && a.lengths_out) {
            a.lengths_out[2 * row] = lens[0];
            a.lengths_out[2 * row + 1] = lens[1];
        }
        if (a.err) a.err[row] = (uint8_t)e;
        if (e != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    __syncthreads();
    for (int64_t idx = lane; idx < (int64_t)R * a.wout; idx += blockDim.x) {
        const int r = (int)(idx / a.wout);
        a.out[r0 * a.wout + idx] = rows[r * a.stride + (int)(idx - (int64_t)r * a.wout)];
    }
}

static int launch(Args a, int op, void* stream) {
    if (a.B < 0 || a.win < 0 || a.wout < 0) return ACX_E_ARG;
    if (a.B == 0) return ACX_OK;
    const int width = a.win > a.wout ? a.win : a.wout;
    a.stride = (width | 1);  // odd: the lanes' same-index accesses fall in distinct banks
    int lanes = LANES;
    while (lanes > 1 && (size_t)2 * lanes * a.stride * 4 > LDS_BUDGET) lanes >>= 1;
    const size_t shm = (size_t)2 * lanes * a.stride * 4;
    if (shm > LDS_BUDGET) return ACX_E_ARG;
    const unsigned grid = (unsigned)((a.B + lanes - 1) / lanes);
    words_kernel<<<dim3(grid), dim3(lanes), shm, (hipStream_t)stream>>>(a, op);
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

}  // namespace words
}  // namespace acx

using namespace acx::words;

extern "C" {

int acx_word_move(const int32_t* state_in, int32_t* state_out, const int32_t* action, int32_t* lengths_out,
                  uint8_t* done, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t cyclical,
                  void* stream) {
    if (L < 1 || !state_in || !state_out || !action) return ACX_E_ARG;
    Args a{state_in, state_out, action, nullptr, lengths_out, nullptr, nullptr, done, err, err_count,
           B, L, 2 * L, 2 * L, 0, cyclical, 0, 0, 0, 0};
    return launch(a, OP_MOVE, stream);
}

int acx_concatenate(const int32_t* state_in, int32_t* state_out, const int32_t* lengths_in, int32_t* lengths_out,
                    int64_t B, int32_t L, int32_t i, int32_t j, int32_t sign, void* stream) {
    // ac_moves.py:25-33 asserts
    if (L < 1 || !state_in || !state_out || (i != 0 && i != 1) || j != 1 - i || (sign != 1 && sign != -1))
        return ACX_E_ARG;
    Args a{state_in, state_out, nullptr, lengths_in, lengths_out, nullptr, nullptr, nullptr, nullptr, nullptr,
           B, L, 2 * L, 2 * L, 0, 0, i, j, sign, 0};
    return launch(a, OP_CONCAT, stream);
}

int acx_conjugate(const int32_t* state_in, int32_t* state_out, const int32_t* lengths_in, int32_t* lengths_out,
                  uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t i, int32_t j, int32_t sign,
                  void* stream) {
    // ac_moves.py:102-106 asserts
    if (L < 1 || !state_in || !state_out || (i != 0 && i != 1) || (j != 1 && j != 2) || (sign != 1 && sign != -1))
        return ACX_E_ARG;
    Args a{state_in, state_out, nullptr, lengths_in, lengths_out, nullptr, nullptr, nullptr, err, err_count,
           B, L, 2 * L, 2 * L, 0, 0, i, j, sign, 0};
    return launch(a, OP_CONJ, stream);
}

int acx_word_simplify_presentation(const int32_t* state_in, int32_t* state_out, int32_t* lengths_out, uint8_t* err,
                                   int32_t* err_count, int64_t B, int32_t L, int32_t cyclical, void* stream) {
    if (L < 1 || !state_in || !state_out) return ACX_E_ARG;
    Args a{state_in, state_out, nullptr, nullptr, lengths_out, nullptr, nullptr, nullptr, err, err_count,
           B, L, 2 * L, 2 * L, 0, cyclical, 0, 0, 0, 0};
    return launch(a, OP_SIMPLIFY_PRES, stream);
}

int acx_word_simplify_relator(const int32_t* relators, int32_t m, int32_t* out, int32_t* out_len, int32_t* n_out,
                              uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t cyclical,
                              int32_t padded, void* stream) {
    if (L < 0 || m < 0 || !relators || !out || !out_len || !n_out) return ACX_E_ARG;
    const int wout = m > L ? m : L;
    Args a{relators, out, nullptr, nullptr, nullptr, n_out, out_len, nullptr, err, err_count,
           B, L, m, wout, 0, cyclical, 0, 0, 0, padded};
    return launch(a, OP_SIMPLIFY_REL, stream);
}

}  // extern "C"
