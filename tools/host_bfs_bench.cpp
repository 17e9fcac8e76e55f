// Host-dedup BFS engine (csrc/acx_search.cpp) on the CPU alone: config 4's search (AK(3), L = 36,
// cyclical = False, 10^7 nodes) with the GPU expansion replaced by the C oracle's, cached in a
// file after the first run, so the engine's own phases can be timed and A/B'd without a GPU.
//   g++ -O3 -std=c++17 -pthread -Iinclude tools/host_bfs_bench.cpp ac-solver-caltech_amd/csrc/acx_search.cpp
//       -x c oracle/acx_oracle.c -o /tmp/host_bfs_bench && /tmp/host_bfs_bench [nodes] [cache]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "acx.h"

extern "C" {
int32_t acx_key_words(int32_t L) { return (4 * L + 16 + 63) / 64; }
void acx_oracle_expand12(const int32_t* parents, int64_t N, int32_t L, int32_t cyclical, int32_t* children,
                         int32_t* lengths, uint8_t* err);
void* acx_search_create(int32_t mode, int32_t L, const uint64_t* start_key, int64_t max_nodes);
void acx_search_destroy(void* h);
int64_t acx_search_next_batch(void* h, uint64_t* parent_keys, int64_t cap);
int32_t acx_search_feed(void* h, const uint64_t* child_keys, int64_t count);
int32_t acx_search_status(void* h, int32_t* budget_hit, int32_t* min_length, int64_t* n_nodes);
void acx_search_stats(void* h, int64_t* out);
void acx_internal_search_phases(void* h, int64_t* out);
}

static const int L = 36;

static void pack(const int32_t* s, uint64_t* k, int kw, bool error) {
    for (int i = 0; i < kw; ++i) k[i] = 0;
    int n[2] = {0, 0};
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < L; ++i) {
            const int v = s[h * L + i];
            if (!v) continue;
            n[h] = i + 1;
            const uint64_t c = v == 1 ? 0 : v == -1 ? 1 : v == 2 ? 2 : 3;
            const int bit = 2 * (h * L + i);
            k[bit >> 6] |= c << (bit & 63);
        }
    for (int h = 0; h < 2; ++h) {
        const uint64_t b = error ? 0xffu : (uint64_t)n[h];
        const int bit = 4 * L + 8 * h;
        k[bit >> 6] |= b << (bit & 63);
        if ((bit & 63) > 56) k[(bit >> 6) + 1] |= b >> (64 - (bit & 63));
    }
}
static void unpack(const uint64_t* k, int32_t* s) {
    static const int32_t let[4] = {1, -1, 2, -2};
    int n[2];
    for (int h = 0; h < 2; ++h) {
        const int bit = 4 * L + 8 * h;
        uint64_t v = k[bit >> 6] >> (bit & 63);
        if ((bit & 63) > 56) v |= k[(bit >> 6) + 1] << (64 - (bit & 63));
        n[h] = (int)(v & 0xff);
    }
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < L; ++i) {
            const int bit = 2 * (h * L + i);
            s[h * L + i] = i < n[h] ? let[(k[bit >> 6] >> (bit & 63)) & 3] : 0;
        }
}

int main(int argc, char** argv) {
    const int64_t nodes = argc > 1 ? atoll(argv[1]) : 10000000;
    const char* cache = argc > 2 ? argv[2] : "/tmp/host_bfs_children.bin";
    const int kw = acx_key_words(L);
    int32_t ak3[2 * L] = {0};
    const int r0[] = {1, 1, 1, -2, -2, -2, -2}, r1[] = {1, 2, 1, -2, -1, -2};
    for (int i = 0; i < 7; ++i) ak3[i] = r0[i];
    for (int i = 0; i < 6; ++i) ak3[L + i] = r1[i];
    std::vector<uint64_t> start(kw);
    pack(ak3, start.data(), kw, false);
    FILE* f = fopen(cache, "rb");
    std::vector<uint64_t> kids;
    if (f) {
        fseek(f, 0, SEEK_END);
        const long sz = ftell(f);
        fseek(f, 0, SEEK_SET);
        kids.resize((size_t)sz / 8);
        if (fread(kids.data(), 8, kids.size(), f) != kids.size()) return 1;
        fclose(f);
    }
    const int64_t cap = 65536;
    void* h = acx_search_create(0, L, start.data(), nodes);
    std::vector<uint64_t> par((size_t)cap * kw), ck((size_t)cap * 12 * kw);
    std::vector<int32_t> ps((size_t)cap * 2 * L), ch((size_t)cap * 12 * 2 * L), ln((size_t)cap * 24);
    std::vector<uint8_t> er((size_t)cap * 12);
    int64_t done_par = 0;
    double feed_s = 0;
    const bool have = !kids.empty();
    int st = 0;
    while (st == 0) {
        const int64_t n = acx_search_next_batch(h, par.data(), cap);
        if (n == 0) break;
        const uint64_t* src;
        if (have && (size_t)(done_par + n) * 12 * kw <= kids.size()) {
            src = &kids[(size_t)done_par * 12 * kw];
        } else {
            for (int64_t i = 0; i < n; ++i) unpack(&par[(size_t)i * kw], &ps[(size_t)i * 2 * L]);
            acx_oracle_expand12(ps.data(), n, L, 0, ch.data(), ln.data(), er.data());
            for (int64_t c = 0; c < 12 * n; ++c) pack(&ch[(size_t)c * 2 * L], &ck[(size_t)c * kw], kw, er[c] != 0);
            if (!have) kids.insert(kids.end(), ck.begin(), ck.begin() + (size_t)n * 12 * kw);
            src = ck.data();
        }
        const auto t0 = std::chrono::steady_clock::now();
        st = acx_search_feed(h, src, n);
        feed_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        done_par += n;
    }
    if (!have && (f = fopen(cache, "wb"))) {
        fwrite(kids.data(), 8, kids.size(), f);
        fclose(f);
    }
    int64_t stats[6], nn = 0;
    int32_t bud = 0, ml = 0;
    acx_search_stats(h, stats);
    int64_t ph[6];
    acx_internal_search_phases(h, ph);
    printf("phases ms: scan %.1f probe %.1f cut %.1f resize %.1f nodes %.1f entries %.1f\n", ph[0] / 1e6, ph[1] / 1e6,
           ph[2] / 1e6, ph[3] / 1e6, ph[4] / 1e6, ph[5] / 1e6);
    st = acx_search_status(h, &bud, &ml, &nn);
    printf("{\"status\": %d, \"budget\": %d, \"nodes\": %lld, \"parents\": %lld, \"rounds\": %lld, \"feed_ms\": %.2f, "
           "\"next_ms\": %.2f, \"store_ms\": %.2f, \"replay_ms\": %.2f}\n",
           st, bud, (long long)nn, (long long)stats[2], (long long)stats[0], feed_s * 1e3, stats[3] / 1e6,
           stats[4] / 1e6, stats[5] / 1e6);
    acx_search_destroy(h);
    return 0;
}
