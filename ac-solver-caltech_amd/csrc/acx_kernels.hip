// acx_kernels.hip -- MI355X (gfx950) kernels for the Andrews-Curtis environment hot path.
//
// Design (DESIGN.md has the full story):
//   * HBM holds presentations as (B, 2L) int32 rows (the tensor the Python host owns).
//   * One wavefront handles a tile of 64 envs, one env per lane.  The tile is staged
//     through LDS with coalesced 16-byte loads/stores (a row is 2L int32 = 288 B at
//     L = 36, so a lane reading "its" row directly would touch 64 lines per load);
//     in LDS each letter is one int8, rows padded to an odd number of dwords so the
//     per-lane row reads are bank-conflict free.
//   * Each lane then packs its two relators into registers, 2 bits per letter
//     (x=0, x^-1=1, y=2, y^-1=3, so inversion is `code ^ 1`), as little multiword
//     integers Word<NW> (NW 32-bit words, letter k at bits [2k, 2k+2)).
//   * A move is O(NW) register work, no per-letter loops:
//       concatenate r_i <- r_i r_j^{+-1}  (reference ac_moves.py:4-76): the junction
//         cancellation count is the first non-zero letter of
//         reverse(r_i) XOR r_j^{+-1} XOR 0x55..  (count-trailing-zeros), the splice is
//         mask | shift;
//       conjugate r_i <- g r_i g^-1 (ac_moves.py:79-156): first/last letter tests + splice;
//       free reduction (utils.py:211-220): a SWAR "adjacent inverse pair" mask; the loop
//         only runs when that mask is non-zero, which needs an unreduced input (moves
//         keep reduced words reduced);
//       cyclic reduction (utils.py:223-232): peel count = first non-zero letter of
//         w XOR reverse(w) XOR 0x55.. .
//   * No MFMA: the path is integer/byte work and HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx.h"

namespace acx {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
constexpr int WPB = BLOCK / WAVE;  // waves per block
constexpr uint32_t P55 = 0x55555555u;

// ---------------------------------------------------------------------------------
// multiword (2 bits per letter) helpers; every loop is over the compile-time NW
// ---------------------------------------------------------------------------------
template <int NW>
struct Word {
    uint32_t w[NW];
};

template <int NW>
__device__ __forceinline__ Word<NW> wzero() {
    Word<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = 0u;
    return r;
}

// low `nbits` bits set (nbits <= 0 -> empty, >= 32*NW -> full)
template <int NW>
__device__ __forceinline__ Word<NW> wmask(int nbits) {
    Word<NW> m;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const int b = nbits - 32 * k;
        m.w[k] = b >= 32 ? 0xffffffffu : (b <= 0 ? 0u : ((1u << b) - 1u));
    }
    return m;
}

template <int NW>
__device__ __forceinline__ Word<NW> wand(const Word<NW>& a, const Word<NW>& b) {
    Word<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = a.w[k] & b.w[k];
    return r;
}
template <int NW>
__device__ __forceinline__ Word<NW> wor(const Word<NW>& a, const Word<NW>& b) {
    Word<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = a.w[k] | b.w[k];
    return r;
}
// a ^ b ^ 0x55.. : letter k is zero iff a[k] is the inverse of b[k]
template <int NW>
__device__ __forceinline__ Word<NW> wxinv(const Word<NW>& a, const Word<NW>& b) {
    Word<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = a.w[k] ^ b.w[k] ^ P55;
    return r;
}
template <int NW>
__device__ __forceinline__ Word<NW> wsel(bool c, const Word<NW>& a, const Word<NW>& b) {
    Word<NW> r;
#pragma unroll
    for (int k = 0; k < NW; ++k) r.w[k] = c ? a.w[k] : b.w[k];
    return r;
}
template <int NW>
__device__ __forceinline__ bool wnonzero(const Word<NW>& a) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) o |= a.w[k];
    return o != 0u;
}

// logical shift right by s bits, 0 <= s (s >= 32*NW gives 0).  Word part by a
// log2(NW)-stage barrel shifter (no runtime-indexed register arrays), bit part by
// v_alignbit_b32.
template <int NW>
__device__ __forceinline__ Word<NW> wshr(const Word<NW>& a, int s) {
    const int q = s >> 5;
    const uint32_t r = (uint32_t)s & 31u;
    Word<NW> t = a;
#pragma unroll
    for (int b = 1; b < NW; b <<= 1) {
        const bool c = (q & b) != 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) t.w[k] = c ? (k + b < NW ? t.w[k + b] : 0u) : t.w[k];
    }
    Word<NW> o;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t hi = (k + 1 < NW) ? t.w[k + 1] : 0u;
        o.w[k] = __builtin_amdgcn_alignbit(hi, t.w[k], r);
    }
    if (q >= NW) o = wzero<NW>();
    return o;
}

// logical shift left by s bits, 0 <= s (s >= 32*NW gives 0)
template <int NW>
__device__ __forceinline__ Word<NW> wshl(const Word<NW>& a, int s) {
    const int q = s >> 5;
    const uint32_t r = (uint32_t)s & 31u;
    Word<NW> t = a;
#pragma unroll
    for (int b = 1; b < NW; b <<= 1) {
        const bool c = (q & b) != 0;
#pragma unroll
        for (int k = NW - 1; k >= 0; --k) t.w[k] = c ? (k - b >= 0 ? t.w[k - b] : 0u) : t.w[k];
    }
    Word<NW> o;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t lo = (k - 1 >= 0) ? t.w[k - 1] : 0u;
        o.w[k] = r ? __builtin_amdgcn_alignbit(t.w[k], lo, 32u - r) : t.w[k];
    }
    if (q >= NW) o = wzero<NW>();
    return o;
}

// reverse the order of all 16*NW letters
template <int NW>
__device__ __forceinline__ Word<NW> wrev_full(const Word<NW>& a) {
    Word<NW> o;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t x = __builtin_bitreverse32(a.w[NW - 1 - k]);
        o.w[k] = ((x >> 1) & P55) | ((x & P55) << 1);  // bit reversal swapped each pair
    }
    return o;
}

// reverse the first n letters (the word w[0..n)): result[u] = w[n-1-u]
template <int NW>
__device__ __forceinline__ Word<NW> wrev(const Word<NW>& a, int n) {
    return wshr<NW>(wrev_full<NW>(a), 32 * NW - 2 * n);
}

// index of the first non-zero letter (16*NW if none)
template <int NW>
__device__ __forceinline__ int wfirst(const Word<NW>& d) {
    int idx = 16 * NW;
#pragma unroll
    for (int k = NW - 1; k >= 0; --k)
        idx = d.w[k] ? (16 * k + (int)(__builtin_ctz(d.w[k]) >> 1)) : idx;
    return idx;
}

// code of letter k (runtime k)
template <int NW>
__device__ __forceinline__ uint32_t wletter(const Word<NW>& a, int k) {
    return wshr<NW>(a, 2 * k).w[0] & 3u;
}

// a word holding one letter `code` at position p
template <int NW>
__device__ __forceinline__ Word<NW> wsingle(uint32_t code, int p) {
    Word<NW> s = wzero<NW>();
    s.w[0] = code;
    return wshl<NW>(s, 2 * p);
}

// ---------------------------------------------------------------------------------
// word algebra
// ---------------------------------------------------------------------------------

// free reduction (utils.py:211-220).  Letters k,k+1 cancel iff w[k+1] == w[k]^1; any
// order of cancellations gives the same (unique) reduced word, so removing the first
// cancelling pair until none is left equals the reference's scan.
template <int NW>
__device__ __forceinline__ Word<NW> adjacent_pairs(const Word<NW>& w, int n) {
    const Word<NW> x = wxinv<NW>(w, wshr<NW>(w, 2));
    Word<NW> z;
#pragma unroll
    for (int k = 0; k < NW; ++k) z.w[k] = ~(x.w[k] | (x.w[k] >> 1)) & P55;
    return wand<NW>(z, wmask<NW>(2 * (n - 1)));
}

template <int NW>
__device__ __forceinline__ void free_reduce(Word<NW>& w, int& n) {
    Word<NW> z = adjacent_pairs<NW>(w, n);
    while (wnonzero<NW>(z)) {  // only for unreduced input words
        const int k = wfirst<NW>(z);
        w = wor<NW>(wand<NW>(w, wmask<NW>(2 * k)), wshl<NW>(wshr<NW>(w, 2 * k + 4), 2 * k));
        n -= 2;
        z = adjacent_pairs<NW>(w, n);
    }
}

// cyclic reduction of a freely reduced word (utils.py:223-232)
template <int NW>
__device__ __forceinline__ void cyclic_reduce(Word<NW>& w, int& n) {
    if (n <= 0) return;
    const Word<NW> d = wxinv<NW>(w, wrev<NW>(w, n));
    int p = wfirst<NW>(d);
    p = p < (n >> 1) ? p : (n >> 1);  // a reduced word never peels past its middle
    if (p > 0) {
        w = wand<NW>(wshr<NW>(w, 2 * p), wmask<NW>(2 * (n - 2 * p)));
        n -= 2 * p;
    }
}

template <int NW>
__device__ __forceinline__ void simplify(Word<NW>& w, int& n, bool cyc) {
    free_reduce<NW>(w, n);
    if (cyc) cyclic_reduce<NW>(w, n);
}

// conjugating generator code of move ids 4..11 (ac_moves.py:167-179, decode :199-206):
//   4: x^-1 (1)  5: y^-1 (3)  6: y^-1 (3)  7: x (0)  8: x (0)  9: y (2)  10: y (2)  11: x^-1 (1)
constexpr uint32_t CONJ_G = (1u << 0) | (3u << 2) | (3u << 4) | (0u << 6) | (0u << 8) | (2u << 10) |
                            (2u << 12) | (1u << 14);

// ACMove (ac_moves.py:159-231) on packed words; returns an ACX_ERR_* code, and leaves
// (w0,n0,w1,n1) unchanged on error.
//   move ids 0..3: concatenation, target i = (id+1)&1, r_j inverted for ids 1, 2.
//   move ids 4..11: conjugation of r_i, i = (id+1)&1, by CONJ_G.
template <int NW>
__device__ __forceinline__ int ac_move(Word<NW>& w0, int& n0, Word<NW>& w1, int& n1, int action, int L,
                                       bool cyc) {
    if ((unsigned)action >= 12u) return ACX_ERR_ACTION;
    const bool i1 = ((action + 1) & 1) != 0;
    const Word<NW> A = wsel<NW>(i1, w1, w0);
    const int nA = i1 ? n1 : n0;
    Word<NW> nw;
    int nn;
    bool fits;
    if (action < 4) {
        // r_i <- r_i r_j^{sign}
        const Word<NW> J = wsel<NW>(i1, w0, w1);
        const int nJ = i1 ? n0 : n1;
        const bool inv = (action == 1) || (action == 2);
        Word<NW> Bw = J;
        if (inv) {  // r_j^{-1}: reversed, every letter inverted
            Bw = wrev<NW>(J, nJ);
            const Word<NW> m = wmask<NW>(2 * nJ);
#pragma unroll
            for (int k = 0; k < NW; ++k) Bw.w[k] ^= (m.w[k] & P55);
        }
        const int mn = nA < nJ ? nA : nJ;
        int acc = wfirst<NW>(wxinv<NW>(wrev<NW>(A, nA), Bw));
        acc = acc < mn ? acc : mn;
        nn = nA + nJ - 2 * acc;
        fits = nn <= L;
        nw = wor<NW>(wand<NW>(A, wmask<NW>(2 * (nA - acc))), wshl<NW>(wshr<NW>(Bw, 2 * acc), 2 * (nA - acc)));
    } else {
        // r_i <- g r_i g^{-1}
        if (nA == 0) return ACX_ERR_EMPTY_CONJ;
        const uint32_t g = (CONJ_G >> (2 * (action - 4))) & 3u;
        const int sc = (A.w[0] & 3u) == (g ^ 1u);
        const int ec = wletter<NW>(A, nA - 1) == g;
        nn = nA + 2 - 2 * (sc + ec);
        fits = nn <= L;
        const Word<NW> mid = wand<NW>(wshr<NW>(A, 2 * sc), wmask<NW>(2 * (nA - sc - ec)));
        nw = wshl<NW>(mid, 2 * (1 - sc));
        if (!sc) nw.w[0] |= g;
        if (!ec) nw = wor<NW>(nw, wsingle<NW>(g ^ 1u, nn - 1));
    }
    // utils.py:264-266: the presentation must stay valid (both relators non-empty)
    const int m0 = (fits && !i1) ? nn : n0;
    const int m1 = (fits && i1) ? nn : n1;
    if (m0 == 0 || m1 == 0) return ACX_ERR_INVALID;
    if (fits) {
        if (i1) { w1 = nw; n1 = nn; }
        else    { w0 = nw; n0 = nn; }
    }
    simplify<NW>(w0, n0, cyc);
    simplify<NW>(w1, n1, cyc);
    return ACX_ERR_NONE;
}

// strict triviality (ac_env.py:99, utils.py:57-87): both relators one letter, one x and one y
template <int NW>
__device__ __forceinline__ bool is_trivial(const Word<NW>& w0, int n0, const Word<NW>& w1, int n1) {
    return n0 == 1 && n1 == 1 && (((w0.w[0] ^ w1.w[0]) & 2u) != 0u);
}

// ---------------------------------------------------------------------------------
// LDS staging: a wave's tile of up to 64 rows, int8 letters, padded rows
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// int32 letter -> int8; values outside {-2..2} become 0x7F and flag the row
__device__ __forceinline__ uint32_t to_i8(int32_t v, bool& bad) {
    const bool ok = (uint32_t)(v + 2) <= 4u;
    bad |= !ok;
    return ok ? ((uint32_t)v & 0xffu) : 0x7fu;
}

// Compile-time geometry when LC > 0 (L == LC), runtime L otherwise.  LMAX letters are
// scanned per relator (compile-time loop bound); rows are LROW bytes so that reading
// LMAX letters of relator 1 stays inside the row.
template <int NW, int LC>
struct Geo {
    static constexpr int LMAX = LC > 0 ? LC : 16 * NW;
    int L, twoL, rowb;
    __device__ __forceinline__ Geo(int L_) {
        L = LC > 0 ? LC : L_;
        twoL = 2 * L;
        const int bytes = (LC > 0) ? 2 * LC : (L + LMAX);
        int dw = (bytes + 3) >> 2;
        dw |= 1;  // odd dword stride: lane l's k-th dword is in bank (l*dw + k) mod 32
        rowb = dw * 4;
    }
};

// (row, pos) of the first element of chunk `c`, chunks of VEC int32 (never straddle rows)
struct ChunkIter {
    int row, pos, dq, dr, twoL;
    __device__ __forceinline__ ChunkIter(int c0, int vec, int twoL_, int stride_chunks) : twoL(twoL_) {
        const int e0 = c0 * vec;
        row = e0 / twoL;
        pos = e0 - row * twoL;
        const int de = stride_chunks * vec;
        dq = de / twoL;
        dr = de - dq * twoL;
    }
    __device__ __forceinline__ void next() {
        pos += dr;
        row += dq;
        if (pos >= twoL) { pos -= twoL; ++row; }
    }
};

constexpr int STAGE_UNROLL = 8;

// global (R rows of 2L int32, row pitch `gpitch` elements) -> LDS tile; flags[row] = 1
// for rows holding a letter outside {-2..2}.  All 64 lanes must call.
template <int VEC>
__device__ __forceinline__ void stage_in(const int32_t* __restrict__ g, int64_t gpitch, int R, int twoL,
                                         int rowb, char* lds, uint8_t* flags, int lane) {
    flags[lane] = 0;
    wave_sync();
    const int nc = (R * twoL) / VEC;
    ChunkIter it(lane, VEC, twoL, WAVE);
    for (int base = lane; base < nc; base += WAVE * STAGE_UNROLL) {
        int rows[STAGE_UNROLL], poss[STAGE_UNROLL];
        int32_t v[STAGE_UNROLL][VEC];
#pragma unroll
        for (int u = 0; u < STAGE_UNROLL; ++u) {
            rows[u] = it.row;
            poss[u] = it.pos;
            it.next();
            const int c = base + u * WAVE;
            if (c < nc) {
                const int32_t* src = g + (int64_t)rows[u] * gpitch + poss[u];
                if constexpr (VEC == 4) {
                    const int4 x = *reinterpret_cast<const int4*>(src);
                    v[u][0] = x.x; v[u][1] = x.y; v[u][2] = x.z; v[u][3] = x.w;
                } else {
                    const int2 x = *reinterpret_cast<const int2*>(src);
                    v[u][0] = x.x; v[u][1] = x.y;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < STAGE_UNROLL; ++u) {
            const int c = base + u * WAVE;
            if (c < nc) {
                bool bad = false;
                char* dst = lds + rows[u] * rowb + poss[u];
                if constexpr (VEC == 4) {
                    const uint32_t p = to_i8(v[u][0], bad) | (to_i8(v[u][1], bad) << 8) |
                                       (to_i8(v[u][2], bad) << 16) | (to_i8(v[u][3], bad) << 24);
                    *reinterpret_cast<uint32_t*>(dst) = p;
                } else {
                    const uint32_t p = to_i8(v[u][0], bad) | (to_i8(v[u][1], bad) << 8);
                    *reinterpret_cast<uint16_t*>(dst) = (uint16_t)p;
                }
                if (bad) flags[rows[u]] = 1;
            }
        }
    }
    wave_sync();
}

// LDS tile -> global (R rows, row pitch `gpitch` elements).  Rows with flags[row] set
// are copied from `fallback` (pitch `fpitch`) instead (the original int32 input of an
// env whose letters do not fit int8).  All 64 lanes must call.
template <int VEC>
__device__ __forceinline__ void stage_out(int32_t* g, int64_t gpitch, int R, int twoL, int rowb,
                                          const char* lds, const uint8_t* flags, const int32_t* fallback,
                                          int64_t fpitch, int lane) {
    const int nc = (R * twoL) / VEC;
    ChunkIter it(lane, VEC, twoL, WAVE);
    for (int c = lane; c < nc; c += WAVE) {
        const int row = it.row, pos = it.pos;
        it.next();
        int32_t* dst = g + (int64_t)row * gpitch + pos;
        const char* src = lds + row * rowb + pos;
        if (flags[row] && fallback) {
            const int32_t* f = fallback + (int64_t)row * fpitch + pos;
            if constexpr (VEC == 4) *reinterpret_cast<int4*>(dst) = *reinterpret_cast<const int4*>(f);
            else *reinterpret_cast<int2*>(dst) = *reinterpret_cast<const int2*>(f);
            continue;
        }
        if constexpr (VEC == 4) {
            const uint32_t p = *reinterpret_cast<const uint32_t*>(src);
            int4 x;
            x.x = (int32_t)(int8_t)(p & 0xffu);
            x.y = (int32_t)(int8_t)((p >> 8) & 0xffu);
            x.z = (int32_t)(int8_t)((p >> 16) & 0xffu);
            x.w = (int32_t)(int8_t)(p >> 24);
            *reinterpret_cast<int4*>(dst) = x;
        } else {
            const uint32_t p = *reinterpret_cast<const uint16_t*>(src);
            int2 x;
            x.x = (int32_t)(int8_t)(p & 0xffu);
            x.y = (int32_t)(int8_t)(p >> 8);
            *reinterpret_cast<int2*>(dst) = x;
        }
    }
}

// one relator: LDS int8 letters -> packed word; `layout_bad` if a letter follows a zero
template <int NW, int LC>
__device__ __forceinline__ void pack_relator(const int8_t* src, int L, Word<NW>& w, int& n, bool& layout_bad) {
    constexpr int LMAX = Geo<NW, LC>::LMAX;
    w = wzero<NW>();
    n = 0;
    bool zero_seen = false;
#pragma unroll
    for (int k = 0; k < LMAX; ++k) {
        int b = src[k];
        if (LC == 0) b = (k < L) ? b : 0;
        const bool nz = b != 0;
        const uint32_t code = nz ? ((((uint32_t)~b & 1u) << 1) | (((uint32_t)b >> 7) & 1u)) : 0u;
        w.w[k >> 4] |= code << (2 * (k & 15));
        n += nz;
        layout_bad |= nz && zero_seen;
        zero_seen |= !nz;
    }
}

// packed word -> LDS int8 letters (L bytes, zero padded)
template <int NW, int LC>
__device__ __forceinline__ void unpack_relator(int8_t* dst, int L, const Word<NW>& w, int n) {
    constexpr int LMAX = Geo<NW, LC>::LMAX;
#pragma unroll
    for (int k = 0; k < LMAX; ++k) {
        const uint32_t code = (w.w[k >> 4] >> (2 * (k & 15))) & 3u;
        // code 0..3 -> 1, -1, 2, -2
        const uint32_t letter = (0xFE02FF01u >> (code << 3)) & 0xffu;
        if (LC > 0 || k < L) dst[k] = (int8_t)(k < n ? letter : 0u);
    }
}

template <int NW>
struct PresRegs {
    Word<NW> w0, w1;
    int n0, n1;
};

// ---------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------
struct StepArgs {
    const int32_t* state_in;
    int32_t* state_out;
    const int32_t* action;
    const int32_t* reset_state;
    int32_t* step_count;
    int32_t* reward;
    uint8_t* done;
    uint8_t* truncated;
    int32_t* lengths_out;
    int32_t* final_obs;
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int L, horizon, cyclical;
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void step_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Geo<NW, LC> geo(a.L);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = threadIdx.x / WAVE;
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wid) * WAVE;
    if (r0 >= a.B) return;
    const int R = (int)((a.B - r0) < WAVE ? (a.B - r0) : WAVE);
    char* tile = smem + wid * (WAVE * geo.rowb + WAVE);
    uint8_t* flags = reinterpret_cast<uint8_t*>(tile + WAVE * geo.rowb);
    const int64_t env = r0 + lane;
    const bool active = lane < R;

    stage_in<VEC>(a.state_in + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags, lane);

    int e = ACX_ERR_NONE;
    if (active) {
        int8_t* row = reinterpret_cast<int8_t*>(tile + lane * geo.rowb);
        PresRegs<NW> p;
        bool layout_bad = flags[lane] != 0;
        pack_relator<NW, LC>(row, geo.L, p.w0, p.n0, layout_bad);
        pack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1, layout_bad);
        const int act = a.action[env];
        if (layout_bad) {
            e = ACX_ERR_DOMAIN;
        } else {
            e = ac_move<NW>(p.w0, p.n0, p.w1, p.n1, act, geo.L, a.cyclical != 0);
        }
        if (e == ACX_ERR_NONE) {
            unpack_relator<NW, LC>(row, geo.L, p.w0, p.n0);
            unpack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1);
        }
        const bool triv = (e == ACX_ERR_NONE) && is_trivial<NW>(p.w0, p.n0, p.w1, p.n1);
        const int total = p.n0 + p.n1;
        int cnt = 0;
        if (a.step_count) cnt = a.step_count[env] + 1;
        const bool trunc = a.step_count ? (cnt >= a.horizon) : false;
        if (a.reward) a.reward[env] = triv ? a.horizon * geo.L * 2 : -total;
        if (a.done) a.done[env] = triv;
        if (a.truncated) a.truncated[env] = trunc;
        int l0 = p.n0, l1 = p.n1;
        if ((triv || trunc) && a.reset_state && e == ACX_ERR_NONE) {
            // same-step autoreset: final_obs <- post-move state, state <- reset row
            if (a.final_obs) {
                int32_t* fo = a.final_obs + env * geo.twoL;
                for (int k = 0; k < geo.twoL; ++k) fo[k] = (int32_t)row[k];
            }
            const int32_t* rs = a.reset_state + env * geo.twoL;
            l0 = 0;
            l1 = 0;
            for (int k = 0; k < geo.twoL; ++k) {
                const int32_t v = rs[k];
                row[k] = (int8_t)v;
                if (k < geo.L) l0 += v != 0;
                else l1 += v != 0;
            }
            cnt = 0;
        }
        if (a.step_count) a.step_count[env] = cnt;
        if (a.lengths_out) {
            a.lengths_out[2 * env] = l0;
            a.lengths_out[2 * env + 1] = l1;
        }
        if (a.err) a.err[env] = (uint8_t)e;
        if (e != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    wave_sync();
    stage_out<VEC>(a.state_out + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags,
                   a.state_in + r0 * geo.twoL, geo.twoL, lane);
}

struct RolloutArgs {
    int32_t* state;
    const int32_t* actions;
    const int32_t* reset_state;
    int32_t* step_count;
    int32_t* obs_traj;
    int32_t* reward_traj;
    uint8_t* done_traj;
    uint8_t* trunc_traj;
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int T, L, horizon, cyclical;
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void rollout_kernel(RolloutArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Geo<NW, LC> geo(a.L);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = threadIdx.x / WAVE;
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wid) * WAVE;
    if (r0 >= a.B) return;
    const int R = (int)((a.B - r0) < WAVE ? (a.B - r0) : WAVE);
    char* tile = smem + wid * (WAVE * geo.rowb + WAVE);
    uint8_t* flags = reinterpret_cast<uint8_t*>(tile + WAVE * geo.rowb);
    const int64_t env = r0 + lane;
    const bool active = lane < R;
    int8_t* row = reinterpret_cast<int8_t*>(tile + lane * geo.rowb);

    // the reset (starting) state stays packed in registers for the whole rollout
    PresRegs<NW> rs;
    bool bad = false;
    stage_in<VEC>(a.reset_state + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags, lane);
    if (active) {
        bad = flags[lane] != 0;
        pack_relator<NW, LC>(row, geo.L, rs.w0, rs.n0, bad);
        pack_relator<NW, LC>(row + geo.L, geo.L, rs.w1, rs.n1, bad);
    }
    wave_sync();
    PresRegs<NW> p;
    stage_in<VEC>(a.state + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags, lane);
    int first_err = ACX_ERR_NONE;
    int cnt = 0;
    if (active) {
        bad |= flags[lane] != 0;
        pack_relator<NW, LC>(row, geo.L, p.w0, p.n0, bad);
        pack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1, bad);
        cnt = a.step_count[env];
        if (bad) first_err = ACX_ERR_DOMAIN;
    }
    const int32_t max_reward = a.horizon * geo.L * 2;
    for (int t = 0; t < a.T; ++t) {
        const int64_t ti = (int64_t)t * a.B;
        if (active) {
            const int act = a.actions[ti + env];
            int e = bad ? ACX_ERR_DOMAIN : ac_move<NW>(p.w0, p.n0, p.w1, p.n1, act, geo.L, a.cyclical != 0);
            if (first_err == ACX_ERR_NONE) first_err = e;
            const bool triv = (e == ACX_ERR_NONE) && is_trivial<NW>(p.w0, p.n0, p.w1, p.n1);
            ++cnt;
            const bool trunc = cnt >= a.horizon;
            if (a.reward_traj) a.reward_traj[ti + env] = triv ? max_reward : -(p.n0 + p.n1);
            if (a.done_traj) a.done_traj[ti + env] = triv;
            if (a.trunc_traj) a.trunc_traj[ti + env] = trunc;
            if ((triv || trunc) && !bad) {
                p = rs;
                cnt = 0;
            }
            if (a.obs_traj && !bad) {
                unpack_relator<NW, LC>(row, geo.L, p.w0, p.n0);
                unpack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1);
            }
        }
        if (a.obs_traj) {
            wave_sync();
            stage_out<VEC>(a.obs_traj + (ti + r0) * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags,
                           nullptr, 0, lane);
            wave_sync();
        }
    }
    if (active) {
        if (!bad) {
            unpack_relator<NW, LC>(row, geo.L, p.w0, p.n0);
            unpack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1);
        }
        a.step_count[env] = cnt;
        if (a.err) a.err[env] = (uint8_t)first_err;
        if (first_err != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    wave_sync();
    // rows flagged out-of-domain keep their (untouched) global contents
    stage_out<VEC>(a.state + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags,
                   a.state + r0 * geo.twoL, geo.twoL, lane);
}

// packed key: r0 letters, r1 letters, n0 (8 bits), n1 (8 bits); KW64 uint64 words
template <int NW>
__device__ __forceinline__ void store_key(uint64_t* dst, int kw64, int L, const PresRegs<NW>& p) {
    constexpr int KN = 2 * NW + 2;
    Word<KN> k0 = wzero<KN>(), k1 = wzero<KN>(), kl = wzero<KN>();
#pragma unroll
    for (int k = 0; k < NW; ++k) { k0.w[k] = p.w0.w[k]; k1.w[k] = p.w1.w[k]; }
    kl.w[0] = (uint32_t)p.n0 | ((uint32_t)p.n1 << 8);
    const Word<KN> key = wor<KN>(wor<KN>(k0, wshl<KN>(k1, 2 * L)), wshl<KN>(kl, 4 * L));
#pragma unroll
    for (int k = 0; k < KN / 2; ++k)
        if (k < kw64) dst[k] = (uint64_t)key.w[2 * k] | ((uint64_t)key.w[2 * k + 1] << 32);
}

template <int NW>
__device__ __forceinline__ void load_key(const uint64_t* src, int kw64, int L, PresRegs<NW>& p) {
    constexpr int KN = 2 * NW + 2;
    Word<KN> key = wzero<KN>();
#pragma unroll
    for (int k = 0; k < KN / 2; ++k) {
        const uint64_t v = k < kw64 ? src[k] : 0ull;
        key.w[2 * k] = (uint32_t)v;
        key.w[2 * k + 1] = (uint32_t)(v >> 32);
    }
    const Word<KN> k1 = wshr<KN>(key, 2 * L);
    const Word<KN> kl = wshr<KN>(key, 4 * L);
    const Word<KN> m = wmask<KN>(2 * L);
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        p.w0.w[k] = key.w[k] & m.w[k];
        p.w1.w[k] = k1.w[k] & m.w[k];
    }
    p.n0 = (int)(kl.w[0] & 0xffu);
    p.n1 = (int)((kl.w[0] >> 8) & 0xffu);
}

struct ExpandArgs {
    const int32_t* parents;
    int32_t* children;
    int32_t* child_len;
    uint64_t* child_key;
    uint8_t* err;
    int32_t* err_count;
    int64_t N;
    int L, cyclical, kw64;
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void expand12_kernel(ExpandArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Geo<NW, LC> geo(a.L);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = threadIdx.x / WAVE;
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wid) * WAVE;
    if (r0 >= a.N) return;
    const int R = (int)((a.N - r0) < WAVE ? (a.N - r0) : WAVE);
    char* tile = smem + wid * (WAVE * geo.rowb + WAVE);
    uint8_t* flags = reinterpret_cast<uint8_t*>(tile + WAVE * geo.rowb);
    const int64_t par = r0 + lane;
    const bool active = lane < R;
    int8_t* row = reinterpret_cast<int8_t*>(tile + lane * geo.rowb);

    stage_in<VEC>(a.parents + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags, lane);
    PresRegs<NW> p;
    bool bad = false;
    if (active) {
        bad = flags[lane] != 0;
        pack_relator<NW, LC>(row, geo.L, p.w0, p.n0, bad);
        pack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1, bad);
    }
    int nerr = 0;
    for (int act = 0; act < 12; ++act) {
        if (active) {
            PresRegs<NW> q = p;
            const int e = bad ? ACX_ERR_DOMAIN : ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, geo.L, a.cyclical != 0);
            const int64_t ci = par * 12 + act;
            nerr += e != ACX_ERR_NONE;
            if (a.err) a.err[ci] = (uint8_t)e;
            if (a.child_len) {
                a.child_len[2 * ci] = q.n0;
                a.child_len[2 * ci + 1] = q.n1;
            }
            if (a.child_key) store_key<NW>(a.child_key + ci * a.kw64, a.kw64, geo.L, q);
            if (a.children && !bad) {
                unpack_relator<NW, LC>(row, geo.L, q.w0, q.n0);
                unpack_relator<NW, LC>(row + geo.L, geo.L, q.w1, q.n1);
            }
        }
        if (a.children) {
            wave_sync();
            stage_out<VEC>(a.children + (r0 * 12 + act) * geo.twoL, (int64_t)12 * geo.twoL, R, geo.twoL, geo.rowb,
                           tile, flags, a.parents + r0 * geo.twoL, geo.twoL, lane);
            wave_sync();
        }
    }
    if (nerr && a.err_count) atomicAdd(a.err_count, nerr);
}

struct CanonArgs {
    const int32_t* state_in;
    int32_t* state_out;
    int32_t* lengths_out;
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int L, cyclical;
};

// simplify_presentation (utils.py:246-283): assert valid, then reduce both relators
template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void canon_kernel(CanonArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Geo<NW, LC> geo(a.L);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = threadIdx.x / WAVE;
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wid) * WAVE;
    if (r0 >= a.B) return;
    const int R = (int)((a.B - r0) < WAVE ? (a.B - r0) : WAVE);
    char* tile = smem + wid * (WAVE * geo.rowb + WAVE);
    uint8_t* flags = reinterpret_cast<uint8_t*>(tile + WAVE * geo.rowb);
    const int64_t env = r0 + lane;
    int8_t* row = reinterpret_cast<int8_t*>(tile + lane * geo.rowb);
    stage_in<VEC>(a.state_in + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags, lane);
    if (lane < R) {
        PresRegs<NW> p;
        bool bad = flags[lane] != 0;
        pack_relator<NW, LC>(row, geo.L, p.w0, p.n0, bad);
        pack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1, bad);
        int e = bad ? ACX_ERR_DOMAIN : ((p.n0 == 0 || p.n1 == 0) ? ACX_ERR_INVALID : ACX_ERR_NONE);
        if (e == ACX_ERR_NONE) {
            simplify<NW>(p.w0, p.n0, a.cyclical != 0);
            simplify<NW>(p.w1, p.n1, a.cyclical != 0);
            unpack_relator<NW, LC>(row, geo.L, p.w0, p.n0);
            unpack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1);
        }
        if (a.lengths_out) {
            a.lengths_out[2 * env] = p.n0;
            a.lengths_out[2 * env + 1] = p.n1;
        }
        if (a.err) a.err[env] = (uint8_t)e;
        if (e != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    wave_sync();
    stage_out<VEC>(a.state_out + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags,
                   a.state_in + r0 * geo.twoL, geo.twoL, lane);
}

struct UnpackArgs {
    const uint64_t* keys;
    int32_t* states;
    int32_t* lengths_out;
    int64_t M;
    int L, kw64;
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void unpack_keys_kernel(UnpackArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Geo<NW, LC> geo(a.L);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = threadIdx.x / WAVE;
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wid) * WAVE;
    if (r0 >= a.M) return;
    const int R = (int)((a.M - r0) < WAVE ? (a.M - r0) : WAVE);
    char* tile = smem + wid * (WAVE * geo.rowb + WAVE);
    uint8_t* flags = reinterpret_cast<uint8_t*>(tile + WAVE * geo.rowb);
    const int64_t k = r0 + lane;
    flags[lane] = 0;
    if (lane < R) {
        PresRegs<NW> p;
        load_key<NW>(a.keys + k * a.kw64, a.kw64, geo.L, p);
        int8_t* row = reinterpret_cast<int8_t*>(tile + lane * geo.rowb);
        unpack_relator<NW, LC>(row, geo.L, p.w0, p.n0);
        unpack_relator<NW, LC>(row + geo.L, geo.L, p.w1, p.n1);
        if (a.lengths_out) {
            a.lengths_out[2 * k] = p.n0;
            a.lengths_out[2 * k + 1] = p.n1;
        }
    }
    wave_sync();
    stage_out<VEC>(a.states + r0 * geo.twoL, geo.twoL, R, geo.twoL, geo.rowb, tile, flags, nullptr, 0, lane);
}

// ---------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------
static inline int nw_for(int L) {
    return L <= 16 ? 1 : L <= 32 ? 2 : L <= 48 ? 3 : L <= 64 ? 4 : 8;
}

template <int NW, int LC>
static inline size_t smem_bytes(int L) {
    const int lmax = LC > 0 ? LC : 16 * NW;
    const int bytes = (LC > 0) ? 2 * LC : (L + lmax);
    int dw = (bytes + 3) >> 2;
    dw |= 1;
    return (size_t)WPB * ((size_t)WAVE * dw * 4 + WAVE);
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// call `f.template go<NW, LC, VEC>()` for the instantiation matching L
template <class F>
static int dispatch(int L, F&& f) {
    const bool v4 = (2 * L) % 4 == 0;
    if (L == 36) return f.template go<3, 36, 4>();
    if (L == 128) return f.template go<8, 128, 4>();
    switch (nw_for(L)) {
        case 1: return v4 ? f.template go<1, 0, 4>() : f.template go<1, 0, 2>();
        case 2: return v4 ? f.template go<2, 0, 4>() : f.template go<2, 0, 2>();
        case 3: return v4 ? f.template go<3, 0, 4>() : f.template go<3, 0, 2>();
        case 4: return v4 ? f.template go<4, 0, 4>() : f.template go<4, 0, 2>();
        default: return v4 ? f.template go<8, 0, 4>() : f.template go<8, 0, 2>();
    }
}

static inline int finish_launch() {
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

static inline unsigned grid_for(int64_t rows) {
    return (unsigned)((rows + (int64_t)BLOCK - 1) / BLOCK);
}

struct StepLaunch {
    StepArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() {
        const size_t shm = smem_bytes<NW, LC>(a.L);
        step_kernel<NW, LC, VEC><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
        return finish_launch();
    }
};
struct RolloutLaunch {
    RolloutArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() {
        const size_t shm = smem_bytes<NW, LC>(a.L);
        rollout_kernel<NW, LC, VEC><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
        return finish_launch();
    }
};
struct ExpandLaunch {
    ExpandArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() {
        const size_t shm = smem_bytes<NW, LC>(a.L);
        expand12_kernel<NW, LC, VEC><<<dim3(grid_for(a.N)), dim3(BLOCK), shm, s>>>(a);
        return finish_launch();
    }
};
struct CanonLaunch {
    CanonArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() {
        const size_t shm = smem_bytes<NW, LC>(a.L);
        canon_kernel<NW, LC, VEC><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
        return finish_launch();
    }
};
struct UnpackLaunch {
    UnpackArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() {
        const size_t shm = smem_bytes<NW, LC>(a.L);
        unpack_keys_kernel<NW, LC, VEC><<<dim3(grid_for(a.M)), dim3(BLOCK), shm, s>>>(a);
        return finish_launch();
    }
};

}  // namespace acx

using namespace acx;

extern "C" {

int32_t acx_key_words(int32_t L) { return (4 * L + 16 + 63) / 64; }

const char* acx_version(void) { return "acx 0.1 gfx950"; }

int acx_step(const int32_t* state_in, int32_t* state_out, const int32_t* action, const int32_t* reset_state,
             int32_t* step_count, int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths_out,
             int32_t* final_obs, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
             int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state_in || !state_out || !action) return ACX_E_ARG;
    if (!aligned16(state_in) || !aligned16(state_out)) return ACX_E_ARG;
    if (reset_state && !step_count) return ACX_E_ARG;
    StepArgs a{state_in, state_out, action, reset_state, step_count, reward, done, truncated,
               lengths_out, final_obs, err, err_count, B, L, horizon, cyclical};
    StepLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_rollout(int32_t* state, const int32_t* actions, const int32_t* reset_state, int32_t* step_count,
                int32_t* obs_traj, int32_t* reward_traj, uint8_t* done_traj, uint8_t* trunc_traj, uint8_t* err,
                int32_t* err_count, int32_t T, int64_t B, int32_t L, int32_t horizon, int32_t cyclical,
                void* stream) {
    if (B < 0 || T < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0 || T == 0) return ACX_OK;
    if (!state || !actions || !reset_state || !step_count) return ACX_E_ARG;
    if (!aligned16(state) || !aligned16(reset_state) || (obs_traj && !aligned16(obs_traj))) return ACX_E_ARG;
    RolloutArgs a{state, actions, reset_state, step_count, obs_traj, reward_traj, done_traj, trunc_traj,
                  err, err_count, B, T, L, horizon, cyclical};
    RolloutLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_expand12(const int32_t* parents, int32_t* children, int32_t* child_len, uint64_t* child_key, uint8_t* err,
                 int32_t* err_count, int64_t N, int32_t L, int32_t cyclical, void* stream) {
    if (N < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (N == 0) return ACX_OK;
    if (!parents || !aligned16(parents) || (children && !aligned16(children))) return ACX_E_ARG;
    ExpandArgs a{parents, children, child_len, child_key, err, err_count, N, L, cyclical, acx_key_words(L)};
    ExpandLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_canonicalize(const int32_t* state_in, int32_t* state_out, int32_t* lengths_out, uint8_t* err,
                     int32_t* err_count, int64_t B, int32_t L, int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state_in || !state_out || !aligned16(state_in) || !aligned16(state_out)) return ACX_E_ARG;
    CanonArgs a{state_in, state_out, lengths_out, err, err_count, B, L, cyclical};
    CanonLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_unpack_keys(const uint64_t* keys, int32_t* states, int32_t* lengths_out, int64_t M, int32_t L,
                    void* stream) {
    if (M < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (M == 0) return ACX_OK;
    if (!keys || !states || !aligned16(states)) return ACX_E_ARG;
    UnpackArgs a{keys, states, lengths_out, M, L, acx_key_words(L)};
    UnpackLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

}  // extern "C"
