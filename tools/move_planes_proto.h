#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace pl {
struct W { uint64_t p0, p1; };  // p0: letter < 0, p1: |letter| == 2; letter k at bit k
__device__ __forceinline__ uint64_t m64(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }
__device__ __forceinline__ W rev(const W& a, int n) {
    const int s = 64 - n;
    return {__builtin_bitreverse64(a.p0) >> s, __builtin_bitreverse64(a.p1) >> s};
}
__device__ __forceinline__ int first_noncancel(const W& a, const W& b) {  // first k with a[k] != inv(b[k])
    const uint64_t nc = (a.p1 ^ b.p1) | ~(a.p0 ^ b.p0);
    return nc ? __builtin_ctzll(nc) : 64;
}
__device__ __forceinline__ W sel(bool c, const W& a, const W& b) { return {c ? a.p0 : b.p0, c ? a.p1 : b.p1}; }
constexpr uint32_t CONJ_G = (1u << 0) | (3u << 2) | (3u << 4) | (0u << 6) | (0u << 8) | (2u << 10) | (2u << 12) | (1u << 14);
__device__ __forceinline__ int move_clean(W& w0, int& n0, W& w1, int& n1, int action, int L, bool cyc) {
    if ((unsigned)action >= 12u) return 4;
    const bool i1 = ((action + 1) & 1) != 0;
    W A = sel(i1, w1, w0);
    int nA = i1 ? n1 : n0;
    if (action < 4) {
        const W J = sel(i1, w0, w1);
        const int nJ = i1 ? n0 : n1;
        const bool inv = (action == 1) || (action == 2);
        W B = J;
        if (inv) { B = rev(J, nJ); B.p0 ^= m64(nJ); }
        const int mn = nA < nJ ? nA : nJ;
        int acc = first_noncancel(rev(A, nA), B);
        acc = acc < mn ? acc : mn;
        const int nn = nA + nJ - 2 * acc;
        if (nn > L) return 0;
        if (nn == 0) return 1;
        const uint64_t m = m64(nA - acc);
        const int sh = nA - acc;
        A.p0 = (A.p0 & m) | ((B.p0 >> acc) << sh);
        A.p1 = (A.p1 & m) | ((B.p1 >> acc) << sh);
        nA = nn;
        if (cyc) {
            int p = first_noncancel(A, rev(A, nA));
            p = p < (nA >> 1) ? p : (nA >> 1);
            const uint64_t mm = m64(nA - 2 * p);
            A.p0 = (A.p0 >> p) & mm;
            A.p1 = (A.p1 >> p) & mm;
            nA -= 2 * p;
        }
    } else {
        const uint32_t g = (CONJ_G >> (2 * (action - 4))) & 3u;
        const uint32_t g0 = g & 1u, g1 = g >> 1;
        const uint32_t f0 = (uint32_t)A.p0 & 1u, f1 = (uint32_t)A.p1 & 1u;
        const uint32_t l0 = (uint32_t)(A.p0 >> (nA - 1)) & 1u, l1 = (uint32_t)(A.p1 >> (nA - 1)) & 1u;
        const bool sc = f1 == g1 && f0 != g0;
        const bool ec = l1 == g1 && l0 == g0;
        if (cyc) {
            if (sc == ec) return 0;
            if (sc) {
                A.p0 = (A.p0 >> 1) | ((uint64_t)f0 << (nA - 1));
                A.p1 = (A.p1 >> 1) | ((uint64_t)f1 << (nA - 1));
            } else {
                const uint64_t m = m64(nA);
                A.p0 = ((A.p0 << 1) & m) | l0;
                A.p1 = ((A.p1 << 1) & m) | l1;
            }
        } else {
            const int nn = nA + 2 - 2 * ((int)sc + (int)ec);
            if (nn > L) return 0;
            const uint64_t mid = m64(nA - (int)sc - (int)ec);
            uint64_t q0 = (A.p0 >> (int)sc) & mid, q1 = (A.p1 >> (int)sc) & mid;
            q0 <<= (1 - (int)sc); q1 <<= (1 - (int)sc);
            if (!sc) { q0 |= g0; q1 |= g1; }
            if (!ec) { q0 |= (uint64_t)(g0 ^ 1u) << (nn - 1); q1 |= (uint64_t)g1 << (nn - 1); }
            A.p0 = q0; A.p1 = q1; nA = nn;
        }
    }
    if (i1) { w1 = A; n1 = nA; } else { w0 = A; n0 = nA; }
    return 0;
}
}
