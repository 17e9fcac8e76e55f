// CPU check of the bit-plane word algebra (ac-solver-caltech_amd/csrc/acx_planes.h, compiled for
// the host) against the C oracle (oracle/acx_oracle.c, pinned to the reference's fixtures):
// ac_move on arbitrary states (unreduced, empty relators, bad move ids), ac_move_clean on clean
// states, random walks of clean moves, and the int8 -> plane pack conversion.  Test
// infrastructure, built and run by tests/test_planes_host.py.
//   planes_check <cases> <seed>   -> prints "ok <n>" or the first mismatch, exit status 0 / 1
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "acx_planes.h"

extern "C" int acx_oracle_move(const int32_t* in, int32_t L, int32_t move_id, int32_t cyclical, int32_t* out,
                               int32_t* lengths);

using namespace acx;

template <int PW>
static PlaneRegs<PW> to_planes(const int32_t* row, int L) {
    PlaneRegs<PW> p;
    for (int h = 0; h < 2; ++h) {
        Planes<PW>& w = h ? p.w1 : p.w0;
        for (int j = 0; j < PW; ++j) w.s[j] = w.y[j] = 0;
        int n = 0;
        for (int k = 0; k < L; ++k) {
            const int32_t v = row[h * L + k];
            if (!v) continue;
            w.s[k >> 6] |= (uint64_t)(v < 0) << (k & 63);
            w.y[k >> 6] |= (uint64_t)(v == 2 || v == -2) << (k & 63);
            ++n;
        }
        (h ? p.n1 : p.n0) = n;
    }
    return p;
}

template <int PW>
static void from_planes(const PlaneRegs<PW>& p, int L, int32_t* row) {
    for (int h = 0; h < 2; ++h) {
        const Planes<PW>& w = h ? p.w1 : p.w0;
        const int n = h ? p.n1 : p.n0;
        for (int k = 0; k < L; ++k) {
            const int s = (w.s[k >> 6] >> (k & 63)) & 1, y = (w.y[k >> 6] >> (k & 63)) & 1;
            row[h * L + k] = k < n ? (y ? 2 : 1) * (s ? -1 : 1) : 0;
        }
    }
}

static int fail(const char* what, int L, int a, int cyc, const int32_t* in, const int32_t* want, const int32_t* got,
                int ew, int eg) {
    printf("MISMATCH %s L=%d action=%d cyc=%d err oracle=%d planes=%d\n in  :", what, L, a, cyc, ew, eg);
    for (int i = 0; i < 2 * L; ++i) printf(" %d", in[i]);
    printf("\n want:");
    for (int i = 0; i < 2 * L; ++i) printf(" %d", want[i]);
    printf("\n got :");
    for (int i = 0; i < 2 * L; ++i) printf(" %d", got[i]);
    printf("\n");
    return 1;
}

// step_pair_kernel's split of ac_move_clean (PW = 1, pl::pair_move_clean): lane h holds relator h,
// its own reversal and the partner's relator and reversal; the env's code is the target lane's,
// the other lane's relator must stay as it was.  false: the split broke that contract
static bool pair_clean(const PlaneRegs<1>& p, int a, int L, bool cyc, PlaneRegs<1>& out, int& e) {
    const Planes<1> w[2] = {p.w0, p.w1};
    const int n[2] = {p.n0, p.n1};
    const Planes<1> rv[2] = {pl::prev<1>(p.w0, p.n0), pl::prev<1>(p.w1, p.n1)};
    Planes<1> nw[2] = {w[0], w[1]};
    int nn[2] = {n[0], n[1]}, eh[2];
    for (int h = 0; h < 2; ++h) eh[h] = pl::pair_move_clean(nw[h], nn[h], rv[h], w[1 - h], n[1 - h], rv[1 - h], h, a, L, cyc);
    const bool bad_id = a < 0 || a >= 12;
    const int t = bad_id ? 0 : ((a + 1) & 1);
    e = eh[t];
    if (nw[1 - t].s[0] != w[1 - t].s[0] || nw[1 - t].y[0] != w[1 - t].y[0] || nn[1 - t] != n[1 - t]) return false;
    if (eh[1 - t] != (bad_id ? ACX_ERR_ACTION : ACX_ERR_NONE)) return false;
    out.w0 = nw[0];
    out.n0 = nn[0];
    out.w1 = nw[1];
    out.n1 = nn[1];
    return true;
}

template <int PW>
static int run(int L, int cases, std::mt19937_64& rng) {
    std::vector<int32_t> in(2 * L), out(2 * L), got(2 * L);
    int32_t lens[2];
    const int letters[4] = {1, -1, 2, -2};
    for (int c = 0; c < cases; ++c) {
        // a random (often unreduced) state; sometimes an empty relator
        for (int h = 0; h < 2; ++h) {
            const int n = (rng() % 23 == 0) ? 0 : (int)(rng() % (L + 1));
            for (int k = 0; k < L; ++k) in[h * L + k] = k < n ? letters[rng() % 4] : 0;
        }
        const int a = (int)(rng() % 14) - 1;  // includes the bad ids -1 and 12
        const int cyc = (int)(rng() & 1);
        const int ew = acx_oracle_move(in.data(), L, a, cyc, out.data(), lens);
        PlaneRegs<PW> p = to_planes<PW>(in.data(), L);
        const int eg = pl::ac_move<PW>(p.w0, p.n0, p.w1, p.n1, a, L, cyc != 0);
        from_planes<PW>(p, L, got.data());
        const int32_t* want = ew ? in.data() : out.data();
        if (ew != eg || memcmp(want, got.data(), 8 * L) != 0) return fail("ac_move", L, a, cyc, in.data(), want, got.data(), ew, eg);
        // the clean path on clean inputs: from the reduced output of the general move
        if (ew == 0 && a >= 0 && a < 12) {
            PlaneRegs<PW> q = p;
            if (pl::is_clean<PW>(q.w0, q.n0, q.w1, q.n1, cyc != 0)) {
                const int b = (int)(rng() % 12);
                std::vector<int32_t> base(got), o2(2 * L), g2(2 * L);
                const int e1 = acx_oracle_move(base.data(), L, b, cyc, o2.data(), lens);
                PlaneRegs<PW> q0 = q;
                const int e2 = pl::ac_move_clean<PW>(q.w0, q.n0, q.w1, q.n1, b, L, cyc != 0);
                from_planes<PW>(q, L, g2.data());
                const int32_t* w2 = e1 ? base.data() : o2.data();
                if (e1 != e2 || memcmp(w2, g2.data(), 8 * L) != 0)
                    return fail("ac_move_clean", L, b, cyc, base.data(), w2, g2.data(), e1, e2);
                if constexpr (PW == 1) {
                    PlaneRegs<1> r;
                    int e3;
                    const int bb = (int)(rng() % 14) - 1;  // the bad ids too
                    const int e4 = acx_oracle_move(base.data(), L, bb, cyc, o2.data(), lens);
                    if (!pair_clean(q0, bb, L, cyc != 0, r, e3)) return fail("pair contract", L, bb, cyc, base.data(), base.data(), base.data(), 0, -1);
                    from_planes<1>(r, L, g2.data());
                    const int32_t* w4 = e4 ? base.data() : o2.data();
                    if (e4 != e3 || memcmp(w4, g2.data(), 8 * L) != 0)
                        return fail("pair_move_clean", L, bb, cyc, base.data(), w4, g2.data(), e4, e3);
                }
            } else if (ew == 0 && cyc == 0) {
                // a successful move's output is reduced: freely (always) -- never unclean unless
                // a relator is empty, which the move rejects
                if (p.n0 > 0 && p.n1 > 0 && pl::bnonzero<PW>(pl::adjacent_pairs<PW>(p.w0, p.n0)))
                    return fail("reduced", L, a, cyc, in.data(), out.data(), got.data(), ew, eg);
            }
        }
        // the int8 -> plane pack conversion (8 letters at a time), on the relator words
        for (int h = 0; h < 2; ++h) {
            uint64_t s = 0, y = 0, z = 0;
            for (int k = 0; k + 8 <= L && k < 64; k += 8) {
                uint32_t d0 = 0, d1 = 0;
                for (int j = 0; j < 4; ++j) {
                    d0 |= (uint32_t)(uint8_t)(int8_t)in[h * L + k + j] << (8 * j);
                    d1 |= (uint32_t)(uint8_t)(int8_t)in[h * L + k + 4 + j] << (8 * j);
                }
                uint32_t s8, y8, z8;
                pl::i8x8_to_bytes(d0, d1, s8, y8, z8);
                s |= (uint64_t)s8 << k;
                y |= (uint64_t)y8 << k;
                z |= (uint64_t)z8 << k;
            }
            const int kmax = L < 64 ? (L / 8) * 8 : 64;
            const uint64_t m = kmax >= 64 ? ~0ull : ((1ull << kmax) - 1);
            const PlaneRegs<PW> r = to_planes<PW>(in.data(), L);
            const Planes<PW>& w = h ? r.w1 : r.w0;
            uint64_t zz = 0;
            for (int k = 0; k < kmax; ++k) zz |= (uint64_t)(in[h * L + k] != 0) << k;
            if ((s & m) != (w.s[0] & m) || (y & m) != (w.y[0] & m) || z != zz) {
                printf("MISMATCH pack L=%d h=%d\n", L, h);
                return 1;
            }
        }
    }
    // random walks of clean cyclic moves from reduced starts (the rollout's hot path)
    for (int c = 0; c < cases / 50 + 1; ++c) {
        for (int h = 0; h < 2; ++h) {
            const int n = 1 + (int)(rng() % L);
            for (int k = 0; k < L; ++k) in[h * L + k] = k < n ? letters[rng() % 4] : 0;
        }
        int32_t red[2 * 128 + 2];
        if (acx_oracle_move(in.data(), L, 4 + (int)(rng() % 8), 1, red, lens) != 0) continue;  // reduce it
        memcpy(in.data(), red, 8 * L);
        PlaneRegs<PW> p = to_planes<PW>(in.data(), L);
        for (int t = 0; t < 200; ++t) {
            if (!pl::is_clean<PW>(p.w0, p.n0, p.w1, p.n1, true)) break;
            const int a = (int)(rng() % 12);
            const int ew = acx_oracle_move(in.data(), L, a, 1, out.data(), lens);
            if constexpr (PW == 1) {
                PlaneRegs<1> r;
                int e3;
                std::vector<int32_t> g3(2 * L);
                if (!pair_clean(p, a, L, true, r, e3)) return fail("pair walk contract", L, a, 1, in.data(), in.data(), in.data(), 0, -1);
                from_planes<1>(r, L, g3.data());
                const int32_t* w3 = ew ? in.data() : out.data();
                if (ew != e3 || memcmp(w3, g3.data(), 8 * L) != 0) return fail("pair walk", L, a, 1, in.data(), w3, g3.data(), ew, e3);
            }
            const int eg = pl::ac_move_clean<PW>(p.w0, p.n0, p.w1, p.n1, a, L, true);
            from_planes<PW>(p, L, got.data());
            const int32_t* want = ew ? in.data() : out.data();
            if (ew != eg || memcmp(want, got.data(), 8 * L) != 0) return fail("walk", L, a, 1, in.data(), want, got.data(), ew, eg);
            memcpy(in.data(), want, 8 * L);
            if (pl::is_trivial<PW>(p.w0, p.n0, p.w1, p.n1) != (lens[0] + lens[1] == 2 && ew == 0 &&
                                                             (abs(want[0]) != abs(want[L])))) {
                if (ew == 0) return fail("trivial", L, a, 1, in.data(), want, got.data(), ew, eg);
            }
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
    int total = 0;
    const int Ls1[] = {1, 2, 3, 5, 7, 8, 13, 16, 17, 18, 31, 32, 33, 36, 47, 48, 63, 64};
    for (int L : Ls1) {
        if (run<1>(L, cases, rng)) return 1;
        total += cases;
    }
    const int Ls2[] = {65, 80, 100, 127, 128};
    for (int L : Ls2) {
        if (run<2>(L, cases, rng)) return 1;
        total += cases;
    }
    printf("ok %d\n", total);
    return 0;
}
