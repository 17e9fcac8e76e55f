// acx_moves.h -- per-lane Andrews-Curtis word algebra shared by the gfx950 kernels
// (acx_kernels.hip: step/rollout/expand12/canonicalize; acx_bfs.hip: device BFS).
// A relator is a little multiword integer Word<NW>, 2 bits per letter (x=0, x^-1=1,
// y=2, y^-1=3; inversion is code ^ 1); see acx_kernels.hip's header comment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx.h"

namespace acx {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
constexpr int WPB = BLOCK / WAVE;  // waves per block
constexpr uint32_t P55 = 0x55555555u;

// Minimum waves per SIMD requested from the register allocator (__launch_bounds__ 2nd
// argument).  At L = 36 the step and rollout kernels fit 64 VGPRs without spilling, so
// 8 waves/SIMD = 8 blocks of 256 per CU: 2048 resident blocks, and a 2^20-env batch
// (4096 blocks) runs in exactly two full rounds with no partially filled tail round.
template <int LC>
struct Occupancy {
    static constexpr int waves_per_simd = (LC == 36) ? 8 : 1;
};

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

// A presentation is "clean" when both relators are non-empty and reduced: freely, and
// cyclically too when `cyc`.  Every successful ac_move output is clean, and a move on a
// clean input keeps the reduced words reduced (junction/end cancellation only, SURVEY
// A.5), so a stream of moves only needs the general reduction when a state enters it.
template <int NW>
__device__ __forceinline__ bool relator_clean(const Word<NW>& w, int n, bool cyc) {
    if (n <= 0) return false;
    if (wnonzero<NW>(adjacent_pairs<NW>(w, n))) return false;
    if (cyc && n > 1 && (w.w[0] & 3u) == (wletter<NW>(w, n - 1) ^ 1u)) return false;
    return true;
}

template <int NW>
__device__ __forceinline__ bool is_clean(const Word<NW>& w0, int n0, const Word<NW>& w1, int n1, bool cyc) {
    return relator_clean<NW>(w0, n0, cyc) && relator_clean<NW>(w1, n1, cyc);
}

// ac_move for a clean input (same results as ac_move, far less work):
//   concatenation: junction cancellation + splice; when cyclical, peel the new word
//     (the untouched relator is already reduced);
//   conjugation, cyclical: g r g^-1 reduces back to r unless one end cancels, in which
//     case the result is r rotated by one letter (both ends cannot cancel in a
//     cyclically reduced r); the length gate never binds (the length is unchanged);
//   conjugation, not cyclical: splice as in ac_move (the result is freely reduced).
// The only possible error is a concatenation that empties r_i (r_i = r_j^{-sign}).
template <int NW>
__device__ __forceinline__ int ac_move_clean(Word<NW>& w0, int& n0, Word<NW>& w1, int& n1, int action, int L,
                                             bool cyc) {
    if ((unsigned)action >= 12u) return ACX_ERR_ACTION;
    const bool i1 = ((action + 1) & 1) != 0;
    Word<NW> A = wsel<NW>(i1, w1, w0);
    int nA = i1 ? n1 : n0;
    if (action < 4) {
        const Word<NW> J = wsel<NW>(i1, w0, w1);
        const int nJ = i1 ? n0 : n1;
        const bool inv = (action == 1) || (action == 2);
        Word<NW> Bw = J;
        if (inv) {
            Bw = wrev<NW>(J, nJ);
            const Word<NW> m = wmask<NW>(2 * nJ);
#pragma unroll
            for (int k = 0; k < NW; ++k) Bw.w[k] ^= (m.w[k] & P55);
        }
        const int mn = nA < nJ ? nA : nJ;
        int acc = wfirst<NW>(wxinv<NW>(wrev<NW>(A, nA), Bw));
        acc = acc < mn ? acc : mn;
        const int nn = nA + nJ - 2 * acc;
        if (nn > L) return ACX_ERR_NONE;       // gated: no-op
        if (nn == 0) return ACX_ERR_INVALID;   // r_i emptied (utils.py:264-266)
        A = wor<NW>(wand<NW>(A, wmask<NW>(2 * (nA - acc))), wshl<NW>(wshr<NW>(Bw, 2 * acc), 2 * (nA - acc)));
        nA = nn;
        if (cyc) cyclic_reduce<NW>(A, nA);
    } else {
        const uint32_t g = (CONJ_G >> (2 * (action - 4))) & 3u;
        const uint32_t first = A.w[0] & 3u;
        const uint32_t last = wletter<NW>(A, nA - 1);
        const bool sc = first == (g ^ 1u);
        const bool ec = last == g;
        if (cyc) {
            if (sc == ec) return ACX_ERR_NONE;  // no cancellation: reduces back to r_i
            if (sc) {                             // r = g^-1 v  ->  v g^-1 : rotate left
                A = wor<NW>(wshr<NW>(A, 2), wsingle<NW>(first, nA - 1));
            } else {                              // r = v g  ->  g v : rotate right
                Word<NW> t = wand<NW>(wshl<NW>(A, 2), wmask<NW>(2 * nA));
                t.w[0] |= last;
                A = t;
            }
        } else {
            const int nn = nA + 2 - 2 * ((int)sc + (int)ec);
            if (nn > L) return ACX_ERR_NONE;
            const Word<NW> mid = wand<NW>(wshr<NW>(A, 2 * (int)sc), wmask<NW>(2 * (nA - (int)sc - (int)ec)));
            Word<NW> nw = wshl<NW>(mid, 2 * (1 - (int)sc));
            if (!sc) nw.w[0] |= g;
            if (!ec) nw = wor<NW>(nw, wsingle<NW>(g ^ 1u, nn - 1));
            A = nw;
            nA = nn;
        }
    }
    if (i1) { w1 = A; n1 = nA; }
    else    { w0 = A; n0 = nA; }
    return ACX_ERR_NONE;
}

// strict triviality (ac_env.py:99, utils.py:57-87): both relators one letter, one x and one y
template <int NW>
__device__ __forceinline__ bool is_trivial(const Word<NW>& w0, int n0, const Word<NW>& w1, int n1) {
    return n0 == 1 && n1 == 1 && (((w0.w[0] ^ w1.w[0]) & 2u) != 0u);
}

template <int NW>
struct PresRegs {
    Word<NW> w0, w1;
    int n0, n1;
};

// packed key: r0 letters, r1 letters, n0 (8 bits), n1 (8 bits); KW64 uint64 words
// the packed key in registers: out[k] for k < NW + 1 (words >= kw64 are zero)
template <int NW>
__device__ __forceinline__ void make_key(int L, const PresRegs<NW>& p, uint64_t (&out)[NW + 1]) {
    constexpr int KN = 2 * NW + 2;
    Word<KN> k0 = wzero<KN>(), k1 = wzero<KN>(), kl = wzero<KN>();
#pragma unroll
    for (int k = 0; k < NW; ++k) { k0.w[k] = p.w0.w[k]; k1.w[k] = p.w1.w[k]; }
    kl.w[0] = (uint32_t)p.n0 | ((uint32_t)p.n1 << 8);
    const Word<KN> key = wor<KN>(wor<KN>(k0, wshl<KN>(k1, 2 * L)), wshl<KN>(kl, 4 * L));
#pragma unroll
    for (int k = 0; k < KN / 2; ++k) out[k] = (uint64_t)key.w[2 * k] | ((uint64_t)key.w[2 * k + 1] << 32);
}

template <int NW>
__device__ __forceinline__ void store_key(uint64_t* dst, int kw64, int L, const PresRegs<NW>& p) {
    uint64_t key[NW + 1];
    make_key<NW>(L, p, key);
#pragma unroll
    for (int k = 0; k < NW + 1; ++k)
        if (k < kw64) dst[k] = key[k];
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

}  // namespace acx
