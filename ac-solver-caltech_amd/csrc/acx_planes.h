// acx_planes.h -- the per-lane Andrews-Curtis word algebra on bit planes, for the env-step
// kernels (acx_kernels.hip: step_kernel, rollout_kernel).
//
// A relator of up to 64*PW letters is two bit planes of PW uint64 words each (letter k at bit
// k): s = "the letter is an inverse" (x^-1, y^-1), y = "the letter is y^{+-1}".  The letter's
// 2-bit code of acx_moves.h (x=0, x^-1=1, y=2, y^-1=3) is y<<1 | s; padding letters are 0 in
// both planes (only the length tells them from x).  Inversion is s ^ 1.
//
// Same semantics and results as acx_moves.h's Word<NW> functions (ac_moves.py:4-231,
// utils.py:178-283), but every word operation is a handful of 64-bit shifts / bit reversals
// on two registers per plane word instead of a per-32-bit-word barrel shifter: the cyclic
// clean move is about half the VALU instructions (tools/move_probe.py, r03).  The searches keep
// the 2-bit-code Word<NW> (their keys are that format, include/acx.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx_moves.h"

// the plane algebra is also compiled for the host: tests/planes_check.cpp checks it against the
// C oracle on the CPU
#define ACX_HD __host__ __device__

namespace acx {

template <int PW>
struct Planes {
    uint64_t s[PW], y[PW];
};

template <int PW>
struct PlaneRegs {
    Planes<PW> w0, w1;
    int n0, n1;
};

// plane words for a relator capacity of 16*NW letters (the Word<NW> instantiations)
template <int NW>
struct PlaneWords {
    static constexpr int value = (NW + 3) / 4;
};

namespace pl {

// ---------------------------------------------------------------------------------
// multiword (PW x 64-bit) bit-string helpers; loops are over the compile-time PW
// ---------------------------------------------------------------------------------
template <int PW>
struct Bits {
    uint64_t b[PW];
};

template <int PW>
ACX_HD __forceinline__ Bits<PW> bzero() {
    Bits<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) r.b[k] = 0ull;
    return r;
}

// low n bits set, 0 <= n <= 64*PW
template <int PW>
ACX_HD __forceinline__ Bits<PW> bmask(int n) {
    Bits<PW> m;
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        const int b = n - 64 * k;
        m.b[k] = b >= 64 ? ~0ull : (b <= 0 ? 0ull : ((1ull << b) - 1ull));
    }
    return m;
}

// logical shift right by s bits, 0 <= s (s >= 64*PW -> 0)
template <int PW>
ACX_HD __forceinline__ Bits<PW> bshr(const Bits<PW>& a, int s) {
    Bits<PW> r;
    if constexpr (PW == 1) {
        r.b[0] = s >= 64 ? 0ull : (a.b[0] >> s);
    } else {
        static_assert(PW == 2, "PW 1 or 2");
        const uint32_t q = (uint32_t)s >> 6, o = (uint32_t)s & 63u;
        const uint64_t lo = o ? ((a.b[0] >> o) | (a.b[1] << (64 - o))) : a.b[0];
        const uint64_t hi = a.b[1] >> o;
        r.b[0] = q == 0 ? lo : (q == 1 ? hi : 0ull);
        r.b[1] = q == 0 ? hi : 0ull;
    }
    return r;
}

// logical shift left by s bits, 0 <= s (s >= 64*PW -> 0)
template <int PW>
ACX_HD __forceinline__ Bits<PW> bshl(const Bits<PW>& a, int s) {
    Bits<PW> r;
    if constexpr (PW == 1) {
        r.b[0] = s >= 64 ? 0ull : (a.b[0] << s);
    } else {
        static_assert(PW == 2, "PW 1 or 2");
        const uint32_t q = (uint32_t)s >> 6, o = (uint32_t)s & 63u;
        const uint64_t lo = a.b[0] << o;
        const uint64_t hi = o ? ((a.b[1] << o) | (a.b[0] >> (64 - o))) : a.b[1];
        r.b[0] = q == 0 ? lo : 0ull;
        r.b[1] = q == 0 ? hi : (q == 1 ? lo : 0ull);
    }
    return r;
}

// reverse the first n bits (result bit u = a bit n-1-u), 1 <= n <= 64*PW
template <int PW>
ACX_HD __forceinline__ Bits<PW> brev(const Bits<PW>& a, int n) {
    Bits<PW> f;
#pragma unroll
    for (int k = 0; k < PW; ++k) f.b[k] = __builtin_bitreverse64(a.b[PW - 1 - k]);
    return bshr<PW>(f, 64 * PW - n);
}

// index of the lowest set bit (64*PW if none)
template <int PW>
ACX_HD __forceinline__ int bfirst(const Bits<PW>& a) {
    int idx = 64 * PW;
#pragma unroll
    for (int k = PW - 1; k >= 0; --k) idx = a.b[k] ? (64 * k + (int)__builtin_ctzll(a.b[k])) : idx;
    return idx;
}

template <int PW>
ACX_HD __forceinline__ bool bnonzero(const Bits<PW>& a) {
    uint64_t o = 0;
#pragma unroll
    for (int k = 0; k < PW; ++k) o |= a.b[k];
    return o != 0ull;
}

// ---------------------------------------------------------------------------------
// words of letters (two planes)
// ---------------------------------------------------------------------------------
template <int PW>
ACX_HD __forceinline__ Bits<PW> S(const Planes<PW>& w) {
    Bits<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) r.b[k] = w.s[k];
    return r;
}
template <int PW>
ACX_HD __forceinline__ Bits<PW> Y(const Planes<PW>& w) {
    Bits<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) r.b[k] = w.y[k];
    return r;
}
template <int PW>
ACX_HD __forceinline__ Planes<PW> make(const Bits<PW>& s, const Bits<PW>& y) {
    Planes<PW> w;
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        w.s[k] = s.b[k];
        w.y[k] = y.b[k];
    }
    return w;
}

template <int PW>
ACX_HD __forceinline__ Planes<PW> psel(bool c, const Planes<PW>& a, const Planes<PW>& b) {
    Planes<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        r.s[k] = c ? a.s[k] : b.s[k];
        r.y[k] = c ? a.y[k] : b.y[k];
    }
    return r;
}

// letters shifted down by n (letter k of the result = letter k + n)
template <int PW>
ACX_HD __forceinline__ Planes<PW> pshr(const Planes<PW>& a, int n) {
    return make<PW>(bshr<PW>(S(a), n), bshr<PW>(Y(a), n));
}
template <int PW>
ACX_HD __forceinline__ Planes<PW> pshl(const Planes<PW>& a, int n) {
    return make<PW>(bshl<PW>(S(a), n), bshl<PW>(Y(a), n));
}
// the first n letters only
template <int PW>
ACX_HD __forceinline__ Planes<PW> pkeep(const Planes<PW>& a, int n) {
    const Bits<PW> m = bmask<PW>(n);
    Planes<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        r.s[k] = a.s[k] & m.b[k];
        r.y[k] = a.y[k] & m.b[k];
    }
    return r;
}
template <int PW>
ACX_HD __forceinline__ Planes<PW> por(const Planes<PW>& a, const Planes<PW>& b) {
    Planes<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) {
        r.s[k] = a.s[k] | b.s[k];
        r.y[k] = a.y[k] | b.y[k];
    }
    return r;
}
// the first n letters reversed
template <int PW>
ACX_HD __forceinline__ Planes<PW> prev(const Planes<PW>& a, int n) {
    return make<PW>(brev<PW>(S(a), n), brev<PW>(Y(a), n));
}
// the inverse word of the first n letters: reversed, every letter inverted
template <int PW>
ACX_HD __forceinline__ Planes<PW> pinv(const Planes<PW>& a, int n) {
    Planes<PW> r = prev<PW>(a, n);
    const Bits<PW> m = bmask<PW>(n);
#pragma unroll
    for (int k = 0; k < PW; ++k) r.s[k] ^= m.b[k];
    return r;
}

// mask of the letters k where a[k] is NOT the inverse of b[k] (bits beyond the words: set)
template <int PW>
ACX_HD __forceinline__ Bits<PW> noncancel(const Planes<PW>& a, const Planes<PW>& b) {
    Bits<PW> r;
#pragma unroll
    for (int k = 0; k < PW; ++k) r.b[k] = (a.y[k] ^ b.y[k]) | ~(a.s[k] ^ b.s[k]);
    return r;
}

// code of letter k (y<<1 | s)
template <int PW>
ACX_HD __forceinline__ uint32_t pletter(const Planes<PW>& a, int k) {
    const Bits<PW> s = bshr<PW>(S(a), k), y = bshr<PW>(Y(a), k);
    return (uint32_t)(((y.b[0] & 1ull) << 1) | (s.b[0] & 1ull));
}
// a word holding the letter `code` at position p
template <int PW>
ACX_HD __forceinline__ Planes<PW> psingle(uint32_t code, int p) {
    Bits<PW> s = bzero<PW>(), y = bzero<PW>();
    s.b[0] = code & 1u;
    y.b[0] = code >> 1;
    return make<PW>(bshl<PW>(s, p), bshl<PW>(y, p));
}

// ---------------------------------------------------------------------------------
// word algebra (the Word<NW> algorithms of acx_moves.h, letter for letter)
// ---------------------------------------------------------------------------------

// letters k < n - 1 followed by their inverse
template <int PW>
ACX_HD __forceinline__ Bits<PW> adjacent_pairs(const Planes<PW>& w, int n) {
    const Planes<PW> nx = pshr<PW>(w, 1);
    Bits<PW> z = noncancel<PW>(w, nx);
    const Bits<PW> m = bmask<PW>(n - 1 > 0 ? n - 1 : 0);
#pragma unroll
    for (int k = 0; k < PW; ++k) z.b[k] = ~z.b[k] & m.b[k];
    return z;
}

// free reduction (utils.py:211-220); the loop only runs for unreduced input
template <int PW>
ACX_HD __forceinline__ void free_reduce(Planes<PW>& w, int& n) {
    Bits<PW> z = adjacent_pairs<PW>(w, n);
    while (bnonzero<PW>(z)) {
        const int k = bfirst<PW>(z);
        w = por<PW>(pkeep<PW>(w, k), pshl<PW>(pshr<PW>(w, k + 2), k));
        n -= 2;
        z = adjacent_pairs<PW>(w, n);
    }
}

// cyclic reduction of a freely reduced word (utils.py:223-232)
template <int PW>
ACX_HD __forceinline__ void cyclic_reduce(Planes<PW>& w, int& n) {
    if (n <= 0) return;
    int p = bfirst<PW>(noncancel<PW>(w, prev<PW>(w, n)));
    p = p < (n >> 1) ? p : (n >> 1);  // a reduced word never peels past its middle
    if (p > 0) {
        w = pkeep<PW>(pshr<PW>(w, p), n - 2 * p);
        n -= 2 * p;
    }
}

template <int PW>
ACX_HD __forceinline__ void simplify(Planes<PW>& w, int& n, bool cyc) {
    free_reduce<PW>(w, n);
    if (cyc) cyclic_reduce<PW>(w, n);
}

// ACMove (ac_moves.py:159-231); returns an ACX_ERR_* code and leaves the state unchanged on error
template <int PW>
ACX_HD __forceinline__ int ac_move(Planes<PW>& w0, int& n0, Planes<PW>& w1, int& n1, int action, int L, bool cyc) {
    if ((unsigned)action >= 12u) return ACX_ERR_ACTION;
    const bool i1 = ((action + 1) & 1) != 0;
    const Planes<PW> A = psel<PW>(i1, w1, w0);
    const int nA = i1 ? n1 : n0;
    Planes<PW> nw;
    int nn;
    bool fits;
    if (action < 4) {
        const Planes<PW> J = psel<PW>(i1, w0, w1);
        const int nJ = i1 ? n0 : n1;
        const bool inv = (action == 1) || (action == 2);
        const Planes<PW> Bw = inv ? pinv<PW>(J, nJ) : J;
        const int mn = nA < nJ ? nA : nJ;
        int acc = nA > 0 ? bfirst<PW>(noncancel<PW>(prev<PW>(A, nA), Bw)) : 0;
        acc = acc < mn ? acc : mn;
        nn = nA + nJ - 2 * acc;
        fits = nn <= L;
        nw = por<PW>(pkeep<PW>(A, nA - acc), pshl<PW>(pshr<PW>(Bw, acc), nA - acc));
    } else {
        if (nA == 0) return ACX_ERR_EMPTY_CONJ;
        const uint32_t g = (CONJ_G >> (2 * (action - 4))) & 3u;
        const int sc = pletter<PW>(A, 0) == (g ^ 1u);
        const int ec = pletter<PW>(A, nA - 1) == g;
        nn = nA + 2 - 2 * (sc + ec);
        fits = nn <= L;
        const Planes<PW> mid = pkeep<PW>(pshr<PW>(A, sc), nA - sc - ec);
        nw = pshl<PW>(mid, 1 - sc);
        if (!sc) nw = por<PW>(nw, psingle<PW>(g, 0));
        if (!ec) nw = por<PW>(nw, psingle<PW>(g ^ 1u, nn - 1));
    }
    // utils.py:264-266: the presentation must stay valid (both relators non-empty)
    const int m0 = (fits && !i1) ? nn : n0;
    const int m1 = (fits && i1) ? nn : n1;
    if (m0 == 0 || m1 == 0) return ACX_ERR_INVALID;
    if (fits) {
        if (i1) { w1 = nw; n1 = nn; }
        else    { w0 = nw; n0 = nn; }
    }
    simplify<PW>(w0, n0, cyc);
    simplify<PW>(w1, n1, cyc);
    return ACX_ERR_NONE;
}

// ac_move as an out-of-line call taking and returning the registers by value: the general path
// (unreduced input: starting states, resets to unreduced rows) is rare in the env-step kernels,
// and inlined next to the clean path it would set their register budget
template <int PW>
struct MoveOut {
    PlaneRegs<PW> p;
    int e;
};
template <int PW>
__device__ __noinline__ MoveOut<PW> ac_move_call(PlaneRegs<PW> p, int action, int L, bool cyc) {
    MoveOut<PW> o;
    o.e = ac_move<PW>(p.w0, p.n0, p.w1, p.n1, action, L, cyc);
    o.p = p;
    return o;
}

// both relators non-empty and reduced (freely; cyclically too when cyc) -- see is_clean
template <int PW>
ACX_HD __forceinline__ bool relator_clean(const Planes<PW>& w, int n, bool cyc) {
    if (n <= 0) return false;
    if (bnonzero<PW>(adjacent_pairs<PW>(w, n))) return false;
    if (cyc && n > 1 && pletter<PW>(w, 0) == (pletter<PW>(w, n - 1) ^ 1u)) return false;
    return true;
}
template <int PW>
ACX_HD __forceinline__ bool is_clean(const Planes<PW>& w0, int n0, const Planes<PW>& w1, int n1, bool cyc) {
    return relator_clean<PW>(w0, n0, cyc) && relator_clean<PW>(w1, n1, cyc);
}

// ac_move for a clean input (acx_moves.h ac_move_clean: same results as ac_move)
template <int PW>
ACX_HD __forceinline__ int ac_move_clean(Planes<PW>& w0, int& n0, Planes<PW>& w1, int& n1, int action, int L,
                                             bool cyc) {
    if ((unsigned)action >= 12u) return ACX_ERR_ACTION;
    const bool i1 = ((action + 1) & 1) != 0;
    Planes<PW> A = psel<PW>(i1, w1, w0);
    int nA = i1 ? n1 : n0;
    if (action < 4) {
        const Planes<PW> J = psel<PW>(i1, w0, w1);
        const int nJ = i1 ? n0 : n1;
        const bool inv = (action == 1) || (action == 2);
        const Planes<PW> Bw = inv ? pinv<PW>(J, nJ) : J;
        const int mn = nA < nJ ? nA : nJ;
        int acc = bfirst<PW>(noncancel<PW>(prev<PW>(A, nA), Bw));
        acc = acc < mn ? acc : mn;
        const int nn = nA + nJ - 2 * acc;
        if (nn > L) return ACX_ERR_NONE;      // gated: no-op
        if (nn == 0) return ACX_ERR_INVALID;  // r_i emptied (utils.py:264-266)
        A = por<PW>(pkeep<PW>(A, nA - acc), pshl<PW>(pshr<PW>(Bw, acc), nA - acc));
        nA = nn;
        if (cyc) cyclic_reduce<PW>(A, nA);
    } else {
        const uint32_t g = (CONJ_G >> (2 * (action - 4))) & 3u;
        const uint32_t first = pletter<PW>(A, 0);
        const uint32_t last = pletter<PW>(A, nA - 1);
        const bool sc = first == (g ^ 1u);
        const bool ec = last == g;
        if (cyc) {
            if (sc == ec) return ACX_ERR_NONE;  // no cancellation: reduces back to r_i
            if (sc) {                             // r = g^-1 v  ->  v g^-1 : rotate left
                A = por<PW>(pshr<PW>(A, 1), psingle<PW>(first, nA - 1));
            } else {                              // r = v g  ->  g v : rotate right
                A = por<PW>(pkeep<PW>(pshl<PW>(A, 1), nA), psingle<PW>(last, 0));
            }
        } else {
            const int nn = nA + 2 - 2 * ((int)sc + (int)ec);
            if (nn > L) return ACX_ERR_NONE;
            const Planes<PW> mid = pkeep<PW>(pshr<PW>(A, (int)sc), nA - (int)sc - (int)ec);
            Planes<PW> nw = pshl<PW>(mid, 1 - (int)sc);
            if (!sc) nw = por<PW>(nw, psingle<PW>(g, 0));
            if (!ec) nw = por<PW>(nw, psingle<PW>(g ^ 1u, nn - 1));
            A = nw;
            nA = nn;
        }
    }
    if (i1) { w1 = A; n1 = nA; }
    else    { w0 = A; n0 = nA; }
    return ACX_ERR_NONE;
}

// ac_move_clean split over the two lanes of an env (acx_kernels.hip step_pair_kernel, one lane per
// relator, PW = 1).  The lane holds relator h (w, n) and its reversal rw = prev(w, n); from its
// partner it has the other relator (pw, pn) and that one's reversal (prw).  On the lane of the
// move's target relator (ac_moves.py:167-179: i = (id + 1) & 1) it returns ac_move_clean's
// ACX_ERR_* code and the relator becomes its result; on the other lane it returns ACX_ERR_NONE
// (ACX_ERR_ACTION for a bad id) and leaves the relator as it is -- a clean move changes only its
// target -- so the caller takes the env's code from the target lane.  Same results as
// ac_move_clean:
//   r_i <- r_i r_j^{+-1}: the junction cancellation count is the first mismatch of prev(r_i) and
//     r_j^{+-1} (ac_moves.py:56-60), r_j^-1 = the partner's reversal with every letter inverted;
//     the result's reversal, for the cyclic peel (utils.py:223-232), is spliced from the two
//     reversals -- reverse(a b) = reverse(b) reverse(a) -- so each lane reverses only its own
//     relator (ac_move_clean reverses r_i, r_j and the result);
//   conjugation (ac_moves.py:79-156) reads only r_i.
ACX_HD __forceinline__ int pair_move_clean(Planes<1>& w, int& n, const Planes<1>& rw, const Planes<1>& pw, int pn,
                                           const Planes<1>& prw, int h, int action, int L, bool cyc) {
    if ((unsigned)action >= 12u) return ACX_ERR_ACTION;
    if ((((action + 1) & 1) != 0) != (h == 1)) return ACX_ERR_NONE;  // not the target relator
    if (action < 4) {
        const bool inv = (action == 1) || (action == 2);
        const int nA = n, nJ = pn;
        const uint64_t mJ = bmask<1>(nJ).b[0];
        // Bw = r_j^{+-1} and its reversal (the reversal of r_j^-1 is r_j with its letters inverted)
        Planes<1> Bw, rB;
        Bw.y[0] = inv ? prw.y[0] : pw.y[0];
        Bw.s[0] = inv ? (prw.s[0] ^ mJ) : pw.s[0];
        rB.y[0] = inv ? pw.y[0] : prw.y[0];
        rB.s[0] = inv ? (pw.s[0] ^ mJ) : prw.s[0];
        const int mn = nA < nJ ? nA : nJ;
        int acc = bfirst<1>(noncancel<1>(rw, Bw));
        acc = acc < mn ? acc : mn;
        int nn = nA + nJ - 2 * acc;
        if (nn > L) return ACX_ERR_NONE;      // gated: no-op
        if (nn == 0) return ACX_ERR_INVALID;  // r_i emptied (utils.py:264-266)
        Planes<1> A = por<1>(pkeep<1>(w, nA - acc), pshl<1>(pshr<1>(Bw, acc), nA - acc));
        if (cyc) {
            const Planes<1> rA = por<1>(pkeep<1>(rB, nJ - acc), pshl<1>(pshr<1>(rw, acc), nJ - acc));
            int p = bfirst<1>(noncancel<1>(A, rA));
            p = p < (nn >> 1) ? p : (nn >> 1);  // a reduced word never peels past its middle
            if (p > 0) {
                A = pkeep<1>(pshr<1>(A, p), nn - 2 * p);
                nn -= 2 * p;
            }
        }
        w = A;
        n = nn;
        return ACX_ERR_NONE;
    }
    // conjugation r_i <- g r_i g^-1 (ac_move_clean's branch on the lane's own relator)
    const uint32_t g = (CONJ_G >> (2 * (action - 4))) & 3u;
    const uint32_t first = pletter<1>(w, 0);
    const uint32_t last = pletter<1>(w, n - 1);
    const bool sc = first == (g ^ 1u);
    const bool ec = last == g;
    if (cyc) {
        if (sc == ec) return ACX_ERR_NONE;  // no cancellation: reduces back to r_i
        if (sc) w = por<1>(pshr<1>(w, 1), psingle<1>(first, n - 1));  // g^-1 v -> v g^-1
        else w = por<1>(pkeep<1>(pshl<1>(w, 1), n), psingle<1>(last, 0));  // v g -> g v
        return ACX_ERR_NONE;
    }
    const int nn = n + 2 - 2 * ((int)sc + (int)ec);
    if (nn > L) return ACX_ERR_NONE;
    const Planes<1> mid = pkeep<1>(pshr<1>(w, (int)sc), n - (int)sc - (int)ec);
    Planes<1> nw = pshl<1>(mid, 1 - (int)sc);
    if (!sc) nw = por<1>(nw, psingle<1>(g, 0));
    if (!ec) nw = por<1>(nw, psingle<1>(g ^ 1u, nn - 1));
    w = nw;
    n = nn;
    return ACX_ERR_NONE;
}

// strict triviality (ac_env.py:99, utils.py:57-87): both relators one letter, one x and one y
template <int PW>
ACX_HD __forceinline__ bool is_trivial(const Planes<PW>& w0, int n0, const Planes<PW>& w1, int n1) {
    return n0 == 1 && n1 == 1 && (((w0.y[0] ^ w1.y[0]) & 1ull) != 0ull);
}

// ---------------------------------------------------------------------------------
// conversions for the LDS tiles (4 letters at a time, letter j of the group at bit j)
// ---------------------------------------------------------------------------------
// 4 int8 letters (one dword of the int8 image) -> sign / y / non-zero nibbles
ACX_HD __forceinline__ void i8x4_to_nibbles(uint32_t d, uint32_t& s4, uint32_t& y4, uint32_t& nz4) {
    const uint32_t nz = (d | (d >> 1)) & 0x01010101u;  // letter != 0
    const uint32_t yb = ~d & nz;                       // |letter| == 2
    const uint32_t sb = (d >> 7) & 0x01010101u;        // letter < 0
    auto gather = [](uint32_t x) { return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xfu; };
    s4 = gather(sb);
    y4 = gather(yb);
    nz4 = gather(nz);
}

// 8 int8 letters (two dwords, letters 0-3 in d0) -> sign / y / non-zero bytes (letter j at bit j):
// bit 0 of every byte of d0 and bit 4 of every byte of d1 gathered by one shift-or chain
ACX_HD __forceinline__ void i8x8_to_bytes(uint32_t d0, uint32_t d1, uint32_t& s8, uint32_t& y8, uint32_t& z8) {
    const uint32_t nz0 = (d0 | (d0 >> 1)) & 0x01010101u, nz1 = (d1 | (d1 >> 1)) & 0x01010101u;
    const uint32_t z = nz0 | (nz1 << 4);
    const uint32_t y = (~d0 & nz0) | ((~d1 & nz1) << 4);
    const uint32_t s = ((d0 >> 7) & 0x01010101u) | (((d1 >> 7) & 0x01010101u) << 4);
    auto gather = [](uint32_t x) { return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xffu; };
    s8 = gather(s);
    y8 = gather(y);
    z8 = gather(z);
}

#ifndef ACX_PLANES_HOST_CHECK  // device-only conversions (tests/planes_check.cpp builds the rest for the host)
// bit j of a nibble -> bit 8j (byte j): one 24-bit multiply (no carries between the terms)
__device__ __forceinline__ uint32_t spread4(uint32_t n4) { return __umul24(n4, 0x00204081u) & 0x01010101u; }

// sign / y nibbles of 4 letters -> their int8 image, the first `s` bits (s = 8m, m = 0..4 letters)
// kept and the rest zero: each byte's 2-bit code selects the letter {1,-1,2,-2} from v_perm's
// first source, a byte past m selects zero from the second (acx_kernels.hip codes_to_i8x4)
__device__ __forceinline__ uint32_t nibbles_to_i8x4(uint32_t s4, uint32_t y4, uint32_t s) {
    const uint32_t sel = spread4(s4) | (spread4(y4) << 1) | (uint32_t)(0x04040404ull << s);
    return __builtin_amdgcn_perm(0u, 0xFE02FF01u, sel);
}

#endif  // ACX_PLANES_HOST_CHECK

// nibble j of a plane word (4 letters from letter 4j)
template <int PW>
__device__ __forceinline__ uint32_t nib(const uint64_t (&p)[PW], int j) {
    return (uint32_t)(p[j >> 4] >> (4 * (j & 15))) & 0xfu;
}

}  // namespace pl
}  // namespace acx
