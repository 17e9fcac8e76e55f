// Sanitizer harness for the host-dedup search engine (csrc/acx_search.cpp): the engine driven
// exactly as tests/test_cpu_host.py::_drive_full drives it, with the GPU expansion replaced by
// the C oracle's (acx_oracle_expand12), so that the whole engine -- its thread pool, the
// hash-partitioned visited set and the provisional entries other threads finalise -- runs under
// ThreadSanitizer or AddressSanitizer + UBSan on the CPU (tests/test_sanitizers.py builds it).
//
// Test infrastructure only.  Reference behaviour pinned by the callers' expectations:
// breadth_first.py:15-97 / greedy.py:15-121 (kat_search_extra.json, reference runs).
//
// stdin: one case per line, "mode L cyclical budget" followed by the 2L letters of the start
// (mode 0 bfs, 1 greedy).  stdout per case: "status n_nodes path_len a0 t0 a1 t1 ...".
#include <cstdint>
#include <cstdio>
#include <vector>

#include "acx.h"

extern "C" {
int32_t acx_key_words(int32_t L) { return (4 * L + 16 + 63) / 64; }
void acx_oracle_expand12(const int32_t* parents, int64_t N, int32_t L, int32_t cyclical, int32_t* children,
                         int32_t* lengths, uint8_t* err);
}

// tests/test_cpu_host.py _pack_key / _oracle_keys: 2-bit codes r0 then r1, then the 8-bit
// letter counts at bit 4L; a child whose move raised gets both length bytes 0xFF
static void pack(const int32_t* s, int L, uint64_t* k, int kw, bool error) {
    for (int i = 0; i < kw; ++i) k[i] = 0;
    for (int h = 0; h < 2; ++h) {
        int n = 0;
        for (int i = 0; i < L; ++i) {
            const int v = s[h * L + i];
            if (!v) continue;
            ++n;
            const uint64_t c = v == 1 ? 0 : v == -1 ? 1 : v == 2 ? 2 : 3;
            const int bit = 2 * (h * L + i);
            k[bit >> 6] |= c << (bit & 63);
        }
        const uint64_t b = error ? 0xffu : (uint64_t)n;
        for (int j = 0; j < 8; ++j) {
            const int bit = 4 * L + 8 * h + j;
            k[bit >> 6] |= ((b >> j) & 1u) << (bit & 63);
        }
    }
}

static void unpack(const uint64_t* k, int L, int32_t* s) {
    static const int32_t let[4] = {1, -1, 2, -2};
    for (int h = 0; h < 2; ++h) {
        int n = 0;
        for (int j = 0; j < 8; ++j) {
            const int bit = 4 * L + 8 * h + j;
            n |= (int)((k[bit >> 6] >> (bit & 63)) & 1u) << j;
        }
        for (int i = 0; i < L; ++i) {
            const int bit = 2 * (h * L + i);
            s[h * L + i] = i < n ? let[(k[bit >> 6] >> (bit & 63)) & 3u] : 0;
        }
    }
}

int main() {
    int mode, L, cyc;
    long long budget;
    while (std::scanf("%d %d %d %lld", &mode, &L, &cyc, &budget) == 4) {
        std::vector<int32_t> start(2 * L);
        for (int i = 0; i < 2 * L; ++i)
            if (std::scanf("%d", &start[i]) != 1) return 2;
        const int kw = acx_key_words(L);
        std::vector<uint64_t> sk(kw);
        pack(start.data(), L, sk.data(), kw, false);
        void* h = acx_search_create(mode, L, sk.data(), budget);
        if (!h) return 3;
        const int64_t cap = 256;
        std::vector<uint64_t> par((size_t)cap * kw), keys((size_t)cap * 12 * kw);
        std::vector<int32_t> ps((size_t)cap * 2 * L), ch((size_t)cap * 12 * 2 * L), ln((size_t)cap * 24);
        std::vector<uint8_t> er((size_t)cap * 12);
        int st = 0;
        while (st == 0) {
            const int64_t n = acx_search_next_batch(h, par.data(), cap);
            if (n == 0) break;
            for (int64_t i = 0; i < n; ++i) unpack(&par[(size_t)i * kw], L, &ps[(size_t)i * 2 * L]);
            acx_oracle_expand12(ps.data(), n, L, cyc, ch.data(), ln.data(), er.data());
            for (int64_t c = 0; c < 12 * n; ++c) pack(&ch[(size_t)c * 2 * L], L, &keys[(size_t)c * kw], kw, er[c] != 0);
            st = acx_search_feed(h, keys.data(), n);
        }
        int64_t nn = 0;
        st = acx_search_status(h, nullptr, nullptr, &nn);
        std::vector<int32_t> acts(4096), tots(4096);
        const int64_t m = acx_search_path(h, acts.data(), tots.data(), 4096);
        std::printf("%d %lld %lld", st, (long long)nn, (long long)m);
        for (int64_t i = 0; i < m && i < 4096; ++i) std::printf(" %d %d", acts[i], tots[i]);
        std::printf("\n");
        std::fflush(stdout);
        acx_search_destroy(h);
    }
    return 0;
}
