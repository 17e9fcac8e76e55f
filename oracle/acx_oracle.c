/*
 * acx_oracle.c -- CPU restatement of the reference's ACEnv step path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libacx.so, the acx package,
 * bench.py's timed region) may link, load or call this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
 *
 * It restates, array-for-array, what the reference does with numpy:
 *   concatenate_relators      ac_solver/envs/ac_moves.py:4-76
 *   conjugate                 ac_solver/envs/ac_moves.py:79-156
 *   ACMove (move decode)      ac_solver/envs/ac_moves.py:159-231
 *   is_array_valid_presentation  ac_solver/envs/utils.py:13-54
 *   is_presentation_trivial   ac_solver/envs/utils.py:57-87
 *   simplify_relator          ac_solver/envs/utils.py:178-243
 *   simplify_presentation     ac_solver/envs/utils.py:246-283
 *   ACEnv.step reward/done/truncated  ac_solver/envs/ac_env.py:91-111
 * Letters are arbitrary non-zero int32 values (the reference's word functions are
 * generator-agnostic; its unit tests use letters 3..6), zeros are padding.  Inputs with
 * zeros inside a relator are handled literally, exactly as the numpy code behaves.
 *
 * Parity of this restatement is pinned against fixtures produced by the reference
 * itself (tests/golden/make_golden.py): tests/test_oracle.py.
 *
 * Error codes (same numbering as include/acx.h):
 *   1  reference raises AssertionError (invalid presentation after the move,
 *      utils.py:264-266; bad move id, ac_moves.py:188-190 -> 4)
 *   2  reference raises IndexError (conjugating an empty relator, ac_moves.py:119)
 *   9  reference raises some other exception (np.pad with negative width)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_INVALID 1
#define ORC_EMPTY_CONJ 2
#define ORC_BAD_ACTION 4
#define ORC_OTHER 9

/* utils.py:13-54 */
int acx_oracle_is_valid(const int32_t* p, int32_t len) {
    if (len % 2 != 0) return 0;
    int32_t L = len / 2;
    for (int h = 0; h < 2; ++h) {
        const int32_t* r = p + h * L;
        int32_t nz = 0;
        for (int32_t k = 0; k < L; ++k) nz += (r[k] != 0);
        if (nz == 0) return 0;
        for (int32_t k = nz; k < L; ++k)
            if (r[k] != 0) return 0;
    }
    return 1;
}

/* utils.py:57-87 */
int acx_oracle_is_trivial(const int32_t* p, int32_t len) {
    if (!acx_oracle_is_valid(p, len)) return 0;
    int32_t L = len / 2;
    int32_t a = 0, b = 0;
    for (int h = 0; h < 2; ++h) {
        int32_t nz = 0;
        for (int32_t k = 0; k < L; ++k) nz += (p[h * L + k] != 0);
        if (nz != 1) return 0;
    }
    a = abs(p[0]);
    b = abs(p[L]);
    if (a > b) { int32_t t = a; a = b; b = t; }
    return a == 1 && b == 2;
}

/*
 * utils.py:178-243.  `rel` has m entries; the simplified word is written to `out`
 * (L entries when padded, else the un-padded remainder of length *out_len).
 * Returns an error code; *n_out receives the word length.
 */
int acx_oracle_simplify_relator(const int32_t* rel, int32_t m, int32_t L, int32_t cyclical,
                                int32_t padded, int32_t* out, int32_t* out_len, int32_t* n_out) {
    int32_t* a = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
    memcpy(a, rel, sizeof(int32_t) * (size_t)m);
    int32_t len = m; /* current array length (np.delete shrinks it) */
    int32_t n = 0;
    for (int32_t k = 0; k < m; ++k) n += (a[k] != 0);
    if (m > n) {
        for (int32_t k = n; k < m; ++k)
            if (a[k] != 0) { free(a); return ORC_INVALID; }
    }
    /* free reduction: scan, delete the cancelling pair, step back one */
    int32_t pos = 0;
    while (pos < n - 1) {
        if (a[pos] == -a[pos + 1]) {
            memmove(a + pos, a + pos + 2, sizeof(int32_t) * (size_t)(len - pos - 2));
            len -= 2;
            n -= 2;
            if (pos) pos -= 1;
        } else {
            pos += 1;
        }
    }
    /* cyclic reduction: peel inverse letters off both ends */
    if (cyclical && n > 0) {
        pos = 0;
        while (pos < n && a[pos] == -a[n - pos - 1]) pos += 1;
        if (pos) {
            /* delete indices [0,pos) and [n-pos, n) */
            int32_t* b = (int32_t*)malloc(sizeof(int32_t) * (size_t)(len > 0 ? len : 1));
            int32_t q = 0;
            for (int32_t k = 0; k < len; ++k) {
                if (k < pos || (k >= n - pos && k < n)) continue;
                b[q++] = a[k];
            }
            memcpy(a, b, sizeof(int32_t) * (size_t)q);
            free(b);
            len = q;
            n -= 2 * pos;
        }
    }
    if (padded) {
        if (L - len < 0) { free(a); return ORC_OTHER; } /* np.pad raises ValueError */
        memcpy(out, a, sizeof(int32_t) * (size_t)len);
        for (int32_t k = len; k < L; ++k) out[k] = 0;
        *out_len = L;
    } else {
        memcpy(out, a, sizeof(int32_t) * (size_t)len);
        *out_len = len;
    }
    free(a);
    if (L < n) return ORC_INVALID;
    *n_out = n;
    return ORC_OK;
}

/* utils.py:246-283 (in place on p of length 2L) */
int acx_oracle_simplify_presentation(int32_t* p, int32_t L, int32_t cyclical, int32_t* lengths) {
    if (!acx_oracle_is_valid(p, 2 * L)) return ORC_INVALID;
    int32_t tmp[4096];
    int32_t* buf = (L <= 4096) ? tmp : (int32_t*)malloc(sizeof(int32_t) * (size_t)L);
    for (int h = 0; h < 2; ++h) {
        int32_t ol = 0, n = 0;
        int e = acx_oracle_simplify_relator(p + h * L, L, L, cyclical, 1, buf, &ol, &n);
        if (e) { if (buf != tmp) free(buf); return e; }
        memcpy(p + h * L, buf, sizeof(int32_t) * (size_t)L);
        lengths[h] = n;
    }
    if (buf != tmp) free(buf);
    return ORC_OK;
}

/* ac_moves.py:4-76 (in place on p of length 2L) */
int acx_oracle_concatenate(int32_t* p, int32_t L, int32_t i, int32_t j, int32_t sign) {
    int32_t* r1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * L + 2));
    int32_t* r2 = r1 + L + 1;
    int32_t n1 = 0, n2 = 0;
    for (int32_t k = 0; k < L; ++k)
        if (p[i * L + k] != 0) r1[n1++] = p[i * L + k];
    for (int32_t k = 0; k < L; ++k) {
        /* sign = -1: negated reversal of the padded half j, then the non-zero filter */
        int32_t v = (sign == 1) ? p[j * L + k] : -p[j * L + (L - 1 - k)];
        if (v != 0) r2[n2++] = v;
    }
    int32_t acc = 0;
    int32_t mn = n1 < n2 ? n1 : n2;
    while (acc < mn && r1[n1 - 1 - acc] == -r2[acc]) acc += 1;
    int32_t new_size = n1 + n2 - 2 * acc;
    if (new_size <= L) {
        int32_t* dst = p + i * L;
        for (int32_t k = 0; k < n1 - acc; ++k) dst[k] = r1[k];
        for (int32_t k = acc; k < n2; ++k) dst[n1 - acc + (k - acc)] = r2[k];
        for (int32_t k = new_size; k < L; ++k) dst[k] = 0;
    }
    free(r1);
    return ORC_OK;
}

/* ac_moves.py:79-156 (in place on p of length 2L); j in {1,2} */
int acx_oracle_conjugate(int32_t* p, int32_t L, int32_t i, int32_t j, int32_t sign) {
    int32_t* rn = (int32_t*)malloc(sizeof(int32_t) * (size_t)(L + 1));
    int32_t n = 0;
    for (int32_t k = 0; k < L; ++k)
        if (p[i * L + k] != 0) rn[n++] = p[i * L + k];
    if (n == 0) { free(rn); return ORC_EMPTY_CONJ; } /* relator_nonzero[0] -> IndexError */
    int32_t g = sign * j;
    int32_t sc = (rn[0] == -g) ? 1 : 0;
    int32_t ec = (rn[n - 1] == g) ? 1 : 0;
    int32_t new_size = n + 2 - 2 * (sc + ec);
    if (new_size <= L) {
        int32_t base = i * L;
        /* presentation[base+1-sc : base+1+n-2sc-ec] = rn[sc : n-ec] */
        int32_t dst0 = base + 1 - sc;
        for (int32_t k = sc; k < n - ec; ++k) p[dst0 + (k - sc)] = rn[k];
        if (!sc) p[base] = g;
        if (!ec) p[base + n + 1 - 2 * sc] = -g;
        if (sc && ec) {
            p[base + new_size] = 0;
            p[base + new_size + 1] = 0;
        }
    }
    free(rn);
    return ORC_OK;
}

/* ac_moves.py:192-206: move id -> (concat?, i, j, sign) */
int acx_oracle_decode(int32_t move_id, int32_t* is_concat, int32_t* i, int32_t* j, int32_t* sign) {
    if (move_id < 0 || move_id > 11) return ORC_BAD_ACTION;
    int32_t m = move_id + 1;
    if (move_id < 4) {
        *is_concat = 1;
        *i = m % 2;
        *j = 1 - *i;
        *sign = (((m - *i) / 2) % 2) ? -1 : 1;
    } else {
        *is_concat = 0;
        *i = m % 2;
        int32_t jp = ((m - *i) / 2) % 2;
        *sign = (((m - *i - 2 * jp) / 4) % 2) ? -1 : 1;
        *j = jp + 1;
    }
    return ORC_OK;
}

/* ac_moves.py:159-231.  out may alias in.  On error, out = in, lengths = non-zero counts. */
int acx_oracle_move(const int32_t* in, int32_t L, int32_t move_id, int32_t cyclical, int32_t* out,
                    int32_t* lengths) {
    int32_t* p = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * L));
    memcpy(p, in, sizeof(int32_t) * (size_t)(2 * L));
    int32_t conc, i, j, sign;
    int e = acx_oracle_decode(move_id, &conc, &i, &j, &sign);
    if (!e) e = conc ? acx_oracle_concatenate(p, L, i, j, sign) : acx_oracle_conjugate(p, L, i, j, sign);
    if (!e) e = acx_oracle_simplify_presentation(p, L, cyclical, lengths);
    if (e) {
        memmove(out, in, sizeof(int32_t) * (size_t)(2 * L));
        for (int h = 0; h < 2; ++h) {
            int32_t nz = 0;
            for (int32_t k = 0; k < L; ++k) nz += (in[h * L + k] != 0);
            lengths[h] = nz;
        }
    } else {
        memcpy(out, p, sizeof(int32_t) * (size_t)(2 * L));
    }
    free(p);
    return e;
}

/* batched ACMove: states (B,2L), actions (B) -> out (B,2L), lengths (B,2), err (B) */
void acx_oracle_move_batch(const int32_t* states, const int32_t* actions, int64_t B, int32_t L,
                           int32_t cyclical, int32_t* out, int32_t* lengths, uint8_t* err) {
    for (int64_t b = 0; b < B; ++b)
        err[b] = (uint8_t)acx_oracle_move(states + b * 2 * L, L, actions[b], cyclical, out + b * 2 * L,
                                          lengths + 2 * b);
}

/* all 12 children of each parent: parents (N,2L) -> children (N,12,2L), lengths (N,12,2) */
void acx_oracle_expand12(const int32_t* parents, int64_t N, int32_t L, int32_t cyclical,
                         int32_t* children, int32_t* lengths, uint8_t* err) {
    for (int64_t b = 0; b < N; ++b)
        for (int a = 0; a < 12; ++a)
            err[b * 12 + a] = (uint8_t)acx_oracle_move(parents + b * 2 * L, L, a, cyclical,
                                                        children + (b * 12 + a) * 2 * L,
                                                        lengths + (b * 12 + a) * 2);
}

/*
 * ACEnv.step (ac_env.py:91-111) batched, with the same-step autoreset contract of
 * VecACEnv (reset to reset_state[b] when done or truncated; the returned obs is the
 * reset state, final_obs the pre-reset state).  reset_state may be NULL (no reset).
 * step_count is in/out.  cyclical is 1 in ACEnv.
 */
void acx_oracle_env_step(int32_t* state, const int32_t* actions, int64_t B, int32_t L, int32_t horizon,
                         int32_t cyclical, const int32_t* reset_state, int32_t* step_count,
                         int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* final_obs,
                         int32_t* lengths, uint8_t* err) {
    for (int64_t b = 0; b < B; ++b) {
        int32_t* s = state + b * 2 * L;
        int32_t lens[2];
        int e = acx_oracle_move(s, L, actions[b], cyclical, s, lens);
        err[b] = (uint8_t)e;
        int32_t tot = lens[0] + lens[1];
        int d = (tot == 2) && acx_oracle_is_trivial(s, 2 * L);
        reward[b] = d ? horizon * L * 2 : -tot;
        step_count[b] += 1;
        int t = step_count[b] >= horizon;
        done[b] = (uint8_t)d;
        truncated[b] = (uint8_t)t;
        if (final_obs) memcpy(final_obs + b * 2 * L, s, sizeof(int32_t) * (size_t)(2 * L));
        if ((d || t) && reset_state) {
            memcpy(s, reset_state + b * 2 * L, sizeof(int32_t) * (size_t)(2 * L));
            step_count[b] = 0;
            for (int h = 0; h < 2; ++h) {
                int32_t nz = 0;
                for (int32_t k = 0; k < L; ++k) nz += (s[h * L + k] != 0);
                lens[h] = nz;
            }
        }
        if (lengths) { lengths[2 * b] = lens[0]; lengths[2 * b + 1] = lens[1]; }
    }
}
