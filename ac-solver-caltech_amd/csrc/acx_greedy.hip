// acx_greedy.hip -- greedy_search (ac_solver/search/greedy.py:15-121) with the visited set on the
// device and the expansion rounds driven from C++.
//
// The reference pops the smallest (total, path length, state tuple) node, expands it with 12
// ACMove calls, tests each child (min length, success = total 2) and pushes the unseen ones.  The
// pop order is inherently sequential; what moves to the GPU is everything around it:
//   * expansion -- every round, the smallest frontier nodes not yet expanded (a second heap of
//     the unexpanded nodes) are expanded speculatively in one launch, lane per (parent, action),
//     from their packed keys; each child's key hash is computed there too;
//   * the visited set -- the keys of all committed nodes live in HBM with a bucketed hash table
//     (as in the device BFS); the expansion kernel probes it, so every child that is already a
//     node (as of that round) comes back marked with the node's id and the host never looks it
//     up.  Nodes the host appends are committed to the device table by the next round's launch,
//     beside its expansion (one launch per round: the expansion trusts only the entries of
//     earlier launches, and the host checks the children against the nodes committed with it).
// The host replays the reference's order exactly: pops while the frontier's top has cached
// children; a child the device did not know is checked only against the nodes appended since
// its round (the in-flight conflicts), kept in a host table of the last 2^16..2^17 appended
// nodes (two generations of tagged entries); children cached before the last 2^16 appends are
// retired and their parent re-expanded with a later batch, which bounds that table.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <new>
#include <vector>

#include "acx.h"
#include "acx_moves.h"

#include "acx_bfs_common.h"

namespace acx {
namespace greedy {

using bfs::fmix64;
using bfs::Key;
using bfs::keq;
using bfs::khash;
using bfs::kload;

constexpr int ACT = 12;
constexpr int BUCKET = 8;
constexpr uint32_t FP_MASK = 0xffffffu;
constexpr int HDR = 40;  // priority-key header bits: total (9) | path length (31)
constexpr int64_t AGE = 1 << 16;  // a cached expansion stays usable while fewer nodes than this have been
                                  // appended since its probe (bounds the in-flight table: two
                                  // generations of AGE nodes, 2 x 1 MB of tagged entries, cache-
                                  // resident).  Aged caches are retired at round starts, so their
                                  // nodes are re-expanded with the next batches instead of costing
                                  // a round each at the top of the frontier (r02u: ~40k rounds)
static int64_t g_age_override = 0;  // tests only (acx_internal_greedy_age): a smaller AGE
static int64_t g_dcap_override = 0;  // tests only (acx_internal_greedy_init_cap): a smaller INIT_DCAP
constexpr int64_t INIT_DCAP = (int64_t)1 << 22;  // nodes of the first device store (doubled as needed)
constexpr int DEFAULT_BATCH = 64;  // parents per round (tools/greedy_sweep.py: 64-128 best on AK(3) /
                                   // Miller-Schupp at 10^6 nodes; larger rounds mostly expand nodes
                                   // that are never popped)

struct DevArgs {
    const uint64_t* parents;  // (n, kw) keys of the round's parents
    uint64_t* ckeys;          // (n, 12, kw) child keys (error sentinel: both length bytes 0xFF)
    uint64_t* chash;          // (n, 12) child key hashes
    int64_t* cknown;          // (n, 12) id of the node the child equals, -1 if none (as of this round)
    uint64_t* nkeys;          // (cap, kw) node keys by id
    const uint64_t* commit;   // (hi - lo, kw) keys of the nodes being committed
    uint64_t* table;          // buckets of 8: (id + 1) << 24 | fp24
    uint64_t bmask;
    int64_t lo, hi;           // commit: node ids [lo, hi)
    int n, L, kw, cyc;
    // round completion (greedy_round_kernel): blocks done so far (device word, back to 0 by the
    // last block) and the host-visible word the last block sets to `seq` -- the host sees the
    // round's outputs (pinned memory) without waiting for the stream
    uint32_t* blocks_done;
    uint32_t* done_flag;
    uint32_t seq;
};

// lane per (parent, action): one move, the child's key, its hash, its id if it is a node below
// a.lo (the nodes committed by earlier launches; greedy_round_kernel commits [lo, hi) in the same
// launch, and those entries are skipped: their keys may still be in flight, and the host checks
// every id >= lo itself)
template <int NW>
__device__ __forceinline__ void expand_lane(const DevArgs& a, int t) {
    if (t >= a.n * ACT) return;
    const int p = t / ACT, act = t - p * ACT;
    PresRegs<NW> q;
    load_key<NW>(a.parents + (int64_t)p * a.kw, a.kw, a.L, q);
    const bool cyc = a.cyc != 0;
    const int e = is_clean<NW>(q.w0, q.n0, q.w1, q.n1, cyc) ? ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, cyc)
                                                             : ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, cyc);
    if (e != ACX_ERR_NONE) {
        q.n0 = 0xff;
        q.n1 = 0xff;
    }
    uint64_t key[NW + 1];
    make_key<NW>(a.L, q, key);
    uint64_t* dst = a.ckeys + (int64_t)t * a.kw;
#pragma unroll
    for (int k = 0; k < NW + 1; ++k)
        if (k < a.kw) dst[k] = key[k];
    Key<NW + 1> kk;
#pragma unroll
    for (int k = 0; k < NW + 1; ++k) kk.w[k] = k < a.kw ? key[k] : 0ull;
    const uint64_t h = khash<NW + 1>(kk, a.kw);
    a.chash[t] = h;
    int64_t known = -1;
    if (e == ACX_ERR_NONE) {
        const uint32_t fp = (uint32_t)(h >> 40);
        uint64_t b = h & a.bmask;
        for (uint64_t it = 0; it <= a.bmask && known < 0; ++it) {
            const uint64_t* bk = a.table + b * BUCKET;
            bool empty = false;
#pragma unroll
            for (int j = 0; j < BUCKET; ++j) {
                const uint64_t v = bk[j];
                if (v == 0) {
                    empty = true;
                    break;
                }
                if (((uint32_t)v & FP_MASK) == fp) {
                    const int64_t id = (int64_t)(v >> 24) - 1;
                    if (id < a.lo && keq<NW + 1>(a.nkeys + id * a.kw, kk, a.kw)) {
                        known = id;
                        break;
                    }
                }
            }
            if (empty) break;
            b = (b + 1) & a.bmask;
        }
    }
    a.cknown[t] = known;
}

// commit the node ids [lo, hi): store their keys and enter them in the table (all distinct, new)
template <int KWM>
__device__ __forceinline__ void commit_lane(const DevArgs& a, int64_t id) {
    if (id >= a.hi) return;
    const Key<KWM> k = kload<KWM>(a.commit + (id - a.lo) * a.kw, a.kw);
#pragma unroll
    for (int i = 0; i < KWM; ++i)
        if (i < a.kw) a.nkeys[id * a.kw + i] = k.w[i];
    const uint64_t h = khash<KWM>(k, a.kw);
    const uint64_t my = ((uint64_t)(id + 1) << 24) | (uint32_t)(h >> 40);
    uint64_t b = h & a.bmask;
    for (uint64_t it = 0; it <= a.bmask; ++it) {
        uint64_t* bk = a.table + b * BUCKET;
        for (int j = 0; j < BUCKET; ++j)
            if (atomicCAS((unsigned long long*)(bk + j), 0ull, (unsigned long long)my) == 0ull) return;
        b = (b + 1) & a.bmask;
    }
}

template <int KWM>
__global__ __launch_bounds__(256) void greedy_commit_kernel(DevArgs a) {
    commit_lane<KWM>(a, a.lo + (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// one round in one launch: blocks [0, cblocks) commit the nodes [lo, hi) appended since the last
// round, the others expand the round's parents against the nodes committed before (ids < lo).
// The two halves touch disjoint key-store rows; a probe that meets a concurrent table insert
// sees the slot empty or holding an id >= lo (skipped), and either way reaches every older entry.
// Every block then releases its writes at system scope and counts itself done; the last one sets
// done_flag = seq, so the host can take the outputs (and reuse the staging buffers, which the
// commit blocks read) as soon as the last block is through, ahead of the stream's own completion.
template <int NW>
__global__ __launch_bounds__(256) void greedy_round_kernel(DevArgs a, int cblocks) {
    if ((int)blockIdx.x < cblocks)
        commit_lane<NW + 1>(a, a.lo + (int64_t)blockIdx.x * 256 + threadIdx.x);
    else
        expand_lane<NW>(a, ((int)blockIdx.x - cblocks) * 256 + threadIdx.x);
    if (a.done_flag == nullptr) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        const uint32_t old = __hip_atomic_fetch_add(a.blocks_done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1u == gridDim.x) {
            __hip_atomic_store(a.blocks_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.done_flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// host restatement of bfs::khash (the kernels' hash): the host tables index by it
static inline uint64_t host_hash(const uint64_t* k, int kw) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < kw; ++i) h = fmix64(h ^ k[i]) + 0x632be59bd9b4e019ull;
    return fmix64(h);
}

static inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct Engine {
    int L = 0, kw = 0, pk = 0, cyc = 0, dev = 0;
    int64_t max_nodes = 0, cap = 0;
    bool prio_generic = false;  // tests only (acx_internal_greedy_prio_key): the per-group priority key
    int64_t dcap = 0;  // nodes the device key store / visited set hold now (grown by doubling)
    uint64_t tsize = 0;
    int batch_cap = DEFAULT_BATCH;
    int64_t age = AGE;
    // nodes (ids in discovery order)
    std::vector<uint64_t> keys;
    std::vector<int64_t> parent;
    std::vector<int8_t> action;
    std::vector<int16_t> total;
    std::vector<int32_t> depth;
    std::vector<int32_t> cache_slot;  // -1: no cached children
    // cached children: per slot 12 keys, hashes, device-known ids, and the round of the probe
    std::vector<uint64_t> c_keys, c_hash;
    std::vector<int64_t> c_known;
    std::vector<int32_t> c_round;
    std::vector<int32_t> free_slots;
    // the recently appended nodes (the in-flight set), two generations of up to AGE ids each:
    // gen[cur] holds ids >= gen_lo[cur], gen[cur ^ 1] the AGE ids before them; open addressing
    // with entries (id + 1) << 16 | 16-bit tag, so a probe reads a node's key only on a tag hit
    std::vector<uint64_t> gen[2];
    int64_t gen_lo[2] = {0, 0};
    int cur = 0;
    uint64_t gmask = 0;
    std::vector<int64_t> n_at_round;  // round r: its kernel knew the ids below this; the host checks the rest
    int64_t committed = 0;            // ids < committed are in the device table
    int round = 0;
    // result (greedy.py:86-121)
    int status = 0;  // 0 running, 1 success, 2 failed, 3 move error
    int budget_hit = 0;
    int min_length = 0;
    std::vector<int32_t> trace;
    std::vector<int64_t> popped;
    int64_t found_parent = -1, found_explored = 0, last_popped = -1;
    int found_action = -1, last_action = -1, last_len = -1;
    uint64_t found_key[ACX_MAX_L / 16 + 2] = {0};
    int64_t st_rounds = 0, st_expanded = 0, ns_select = 0, ns_gpu = 0, ns_replay = 0, st_known = 0;
    // why each round's replay stopped: the top node was appended during that replay / was an
    // older node outside the round's batch / had children cached too long ago
    int64_t st_stop_new = 0, st_stop_old = 0, st_stop_aged = 0;
    int64_t ns_wait = 0, ns_cache = 0;
    int64_t st_retired = 0;  // cached expansions retired unused because they aged  // inside the round trip: polling for the GPU / caching children
    // staging: pinned host buffers the kernels read (parents + committed keys) and write (child
    // keys, hashes, known ids) directly, so a round is 2 launches and a completion poll -- no
    // copies, no blocking synchronisation
    hipStream_t stream = nullptr;
    DevArgs d{};
    uint64_t *h_in = nullptr, *h_out = nullptr;    // pinned, host view
    uint64_t *hd_in = nullptr, *hd_out = nullptr;  // the same memory, device view
    uint32_t *h_flag = nullptr, *hd_flag = nullptr;  // the rounds' completion word (pinned)
    uint32_t* d_blocks = nullptr;                    // the rounds' block count (device)
    uint32_t round_seq = 0;                          // the last round's completion value
    int64_t commit_cap = 0;

    // wait for the stream by polling (hipStreamSynchronize may sleep on an interrupt: tens of us
    // per round at ~1500 rounds per 10^6-node search)
    int wait() const {
        hipError_t e;
        while ((e = hipStreamQuery(stream)) == hipErrorNotReady) {
        }
        return e == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
    }
    // a round: until its last block has set the completion word (greedy_round_kernel), or the
    // stream is through (checked every 256 polls: a launch that failed never sets the word)
    int wait_round(uint32_t seq) const {
        for (uint32_t i = 1;; ++i) {
            if (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) == seq) return ACX_OK;
            if ((i & 255u) == 0u) {
                const hipError_t e = hipStreamQuery(stream);
                if (e == hipSuccess) return ACX_OK;
                if (e != hipErrorNotReady) return ACX_E_LAUNCH;
            }
        }
    }

    ~Engine() {
        if (stream) (void)hipStreamSynchronize(stream);
        void* dp[] = {d.nkeys, d.table, d_blocks};
        for (void* p : dp)
            if (p) (void)hipFree(p);
        void* hp[] = {h_in, h_out, h_flag};
        for (void* p : hp)
            if (p) (void)hipHostFree(p);
        if (stream) (void)hipStreamDestroy(stream);
    }

    bool init(int L_, int64_t max_nodes_, int cyc_, int batch) {
        L = L_;
        kw = acx_key_words(L);
        pk = (HDR + 6 * L + 63) / 64;
        frontier.init(pk, &pkeys);
        unexpanded.init(pk, &pkeys);
        cyc = cyc_;
        max_nodes = max_nodes_;
        cap = max_nodes + 12;
        batch_cap = batch > 0 ? batch : DEFAULT_BATCH;
        age = g_age_override > 0 ? g_age_override : AGE;  // a power of two
        if (hipGetDevice(&dev) != hipSuccess) return false;
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
        commit_cap = 4 * (int64_t)batch_cap * ACT + 64;
        const size_t nb = (size_t)batch_cap;
        const size_t in_words = (nb + (size_t)commit_cap) * kw, out_words = nb * ACT * (kw + 2);
        d.L = L;
        d.kw = kw;
        d.cyc = cyc;
        bool ok = hipHostMalloc((void**)&h_in, in_words * 8, hipHostMallocMapped) == hipSuccess &&
                  hipHostMalloc((void**)&h_out, out_words * 8, hipHostMallocMapped) == hipSuccess &&
                  hipHostGetDevicePointer((void**)&hd_in, h_in, 0) == hipSuccess &&
                  hipHostGetDevicePointer((void**)&hd_out, h_out, 0) == hipSuccess &&
                  hipHostMalloc((void**)&h_flag, 64, hipHostMallocMapped) == hipSuccess &&
                  hipHostGetDevicePointer((void**)&hd_flag, h_flag, 0) == hipSuccess &&
                  hipMalloc((void**)&d_blocks, 64) == hipSuccess && hipMemset(d_blocks, 0, 64) == hipSuccess;
        if (ok) *h_flag = 0u;
        // the device store starts at min(budget, INIT_DCAP) nodes and doubles as the search grows
        // (the reference's set grows with the search: a large budget on a search that ends early
        // must not fail on an up-front allocation)
        ok = ok && grow(std::min<int64_t>(cap, g_dcap_override > 0 ? g_dcap_override : INIT_DCAP));
        if (!ok) (void)hipGetLastError();
        return ok;
    }

    // (re)allocate the device key store for n >= dcap nodes and a visited set of load <= 1/2,
    // keeping the committed nodes: their keys are copied and re-entered in the new table
    bool grow(int64_t n) {
        uint64_t ts = 1024;
        while (ts < 2 * (uint64_t)n) ts <<= 1;
        uint64_t *nk = nullptr, *tb = nullptr;
        if (hipMalloc((void**)&nk, (size_t)n * kw * 8) != hipSuccess) return false;
        if (hipMalloc((void**)&tb, ts * 8) != hipSuccess) {
            (void)hipFree(nk);
            return false;
        }
        bool ok = hipMemsetAsync(tb, 0, ts * 8, stream) == hipSuccess;
        if (ok && committed > 0)
            ok = hipMemcpyAsync(nk, d.nkeys, (size_t)committed * kw * 8, hipMemcpyDeviceToDevice, stream) == hipSuccess;
        if (ok && wait() == ACX_OK) {
            if (d.nkeys) (void)hipFree(d.nkeys);
            if (d.table) (void)hipFree(d.table);
        } else {
            (void)hipFree(nk);
            (void)hipFree(tb);
            return false;
        }
        d.nkeys = nk;
        d.table = tb;
        d.bmask = ts / BUCKET - 1;
        dcap = n;
        tsize = ts;
        if (committed > 0) {  // re-enter every committed node (the commit kernel rewrites its own key)
            d.commit = d.nkeys;
            d.lo = 0;
            d.hi = committed;
            commit_launch();
            if (hipGetLastError() != hipSuccess || wait() != ACX_OK) return false;
        }
        return true;
    }
    void commit_launch();

    // ---------------------------------------------------------------- key helpers
    int len_field(const uint64_t* k, int h) const {
        const int bit = 4 * L + 8 * h;
        const uint64_t lo = k[bit >> 6] >> (bit & 63);
        const uint64_t hi = (bit & 63) > 56 ? (k[(bit >> 6) + 1] << (64 - (bit & 63))) : 0ull;
        return (int)((lo | hi) & 0xff);
    }
    int key_total(const uint64_t* k) const { return len_field(k, 0) + len_field(k, 1); }
    bool key_is_error(const uint64_t* k) const { return len_field(k, 0) == 0xff && len_field(k, 1) == 0xff; }
    uint32_t byte_at(const uint64_t* k, int bit) const {
        const uint64_t lo = k[bit >> 6] >> (bit & 63);
        const uint64_t hi = (bit & 63) > 56 ? (k[(bit >> 6) + 1] << (64 - (bit & 63))) : 0ull;
        return (uint32_t)((lo | hi) & 0xff);
    }

    // the heap key: total (9 bits) | path length (31) | every letter + 2 in 3 bits, MSB first
    // (x = 3, x^-1 = 1, y = 4, y^-1 = 0, padding = 2): unsigned word order = Python's tuple
    // order of (total, path length, state tuple) (greedy.py:55-64,104-113)
    void prio_key(const uint64_t* k, int tot, int dep, uint64_t* out) const {
        static uint16_t tbl[256];
        static bool init = false;
        if (!init) {
            static const uint32_t val[4] = {3, 1, 4, 0};
            for (int b = 0; b < 256; ++b) {
                uint32_t v = 0;
                for (int j = 0; j < 4; ++j) v = (v << 3) | val[(b >> (2 * j)) & 3];
                tbl[b] = (uint16_t)v;
            }
            init = true;
        }
        for (int i = 0; i < pk; ++i) out[i] = 0;
        out[0] = ((uint64_t)(tot & 0x1ff) << 55) | ((uint64_t)(dep & 0x7fffffff) << 24);
        int pos = HDR;
        auto put = [&](uint64_t v, int nbits) {  // append nbits (<= 61) MSB-first
            const int w = pos >> 6, o = pos & 63;
            if (o + nbits <= 64) {
                out[w] |= v << (64 - o - nbits);
            } else {
                out[w] |= v >> (o + nbits - 64);
                out[w + 1] |= v << (128 - o - nbits);
            }
            pos += nbits;
        };
        constexpr uint64_t PAD20 = 0x492492492492492ull >> 0;  // 20 x 010 (60 bits): padding letters
        if (L <= 40 && !prio_generic) {
            // a relator's 2L code bits are taken in one 128-bit shift and mapped 4 letters per
            // table lookup into two 60-bit parts (letters 0..19, 20..L-1); the padding letters'
            // fields replaced by 010s with one mask per part -- a few appends instead of one per
            // 4 letters (the general path below, which this reproduces bit for bit)
            using u128 = unsigned __int128;
            for (int h = 0; h < 2; ++h) {
                const int n = len_field(k, h);
                const int b0 = 2 * h * L, w = b0 >> 6, o = b0 & 63;
                u128 codes = ((u128)k[w] | ((u128)(w + 1 < kw ? k[w + 1] : 0ull) << 64)) >> o;
                if (o + 2 * L > 128 && w + 2 < kw) codes |= (u128)k[w + 2] << (128 - o);
                auto part = [&](int f, int cnt) -> uint64_t {  // letters [f, f + cnt), cnt <= 20
                    const int groups = (cnt + 3) / 4;
                    uint64_t v = 0;
                    for (int g = 0; g < groups; ++g) v = (v << 12) | tbl[(uint32_t)(codes >> (2 * f + 8 * g)) & 0xffu];
                    v >>= 3 * (4 * groups - cnt);  // the letters past the part in its last group
                    const int live = n - f < 0 ? 0 : (n - f > cnt ? cnt : n - f);
                    if (live < cnt) {
                        const uint64_t mask = (1ull << (3 * (cnt - live))) - 1;
                        v = (v & ~mask) | (PAD20 & mask);
                    }
                    return v;
                };
                const int c0 = L < 20 ? L : 20;
                put(part(0, c0), 3 * c0);
                if (L > 20) put(part(20, L - 20), 3 * (L - 20));
            }
            return;
        }
        for (int h = 0; h < 2; ++h) {
            const int n = len_field(k, h);
            int i = 0;
            for (; i + 4 <= n; i += 4) put(tbl[byte_at(k, 2 * (h * L + i))], 12);
            for (; i < n; ++i) {
                static const uint32_t val[4] = {3, 1, 4, 0};
                put(val[byte_at(k, 2 * (h * L + i)) & 3], 3);
            }
            for (int m = L - n; m > 0; m -= 20) {
                const int c = m < 20 ? m : 20;
                put(PAD20 >> (3 * (20 - c)), 3 * c);
            }
        }
    }

    // the nodes' heap keys (pk words per node id, prio_key), written once when a node is appended
    std::vector<uint64_t> pkeys;

    // 4-ary min-heap of node ids ordered by their heap keys.  An entry is the key's first word
    // (total | path length | the first 24 letter bits: nearly always decides) and the id, 16 bytes;
    // the rest of the key is read from pkeys only on a tie of first words.  (Round 5's entries
    // held the whole key inline, 8 + 8 * pk bytes, copied at every level of a sift.)
    struct Heap {
        struct Ent {
            uint64_t k0;
            int64_t id;
        };
        int pk = 0;
        const std::vector<uint64_t>* keys = nullptr;  // Engine::pkeys
        std::vector<Ent> e;
        bool less(const Ent& x, const Ent& y) const {
            if (x.k0 != y.k0) return x.k0 < y.k0;
            const uint64_t* a = keys->data() + (size_t)x.id * pk;
            const uint64_t* b = keys->data() + (size_t)y.id * pk;
            for (int i = 1; i < pk; ++i)
                if (a[i] != b[i]) return a[i] < b[i];
            return false;
        }
        bool empty() const { return e.empty(); }
        size_t size() const { return e.size(); }
        int64_t top() const { return e[0].id; }
        void push(uint64_t k0, int64_t v) {
            size_t i = e.size();
            e.push_back(Ent{k0, v});
            const Ent x{k0, v};
            while (i > 0) {
                const size_t par = (i - 1) / 4;
                if (!less(x, e[par])) break;
                e[i] = e[par];
                i = par;
            }
            e[i] = x;
        }
        void pop() {
            const size_t n = e.size() - 1;
            const Ent x = e[n];
            e.pop_back();
            if (n == 0) return;
            size_t i = 0;
            while (true) {
                const size_t c0 = 4 * i + 1;
                if (c0 >= n) break;
                size_t best = c0;
                const size_t ce = c0 + 4 < n ? c0 + 4 : n;
                for (size_t c = c0 + 1; c < ce; ++c)
                    if (less(e[c], e[best])) best = c;
                if (!less(e[best], x)) break;
                e[i] = e[best];
                i = best;
            }
            e[i] = x;
        }
    };
    // one heap per total (the priority key's top 9 bits): a pop sifts through the nodes of the
    // smallest total only, not the whole frontier (10^6 nodes: ~10 cold levels per pop); the order
    // is the single heap's, since the total is the key's most significant field
    struct BucketHeap {
        static constexpr int NB = 512;
        int minb = NB;  // the smallest non-empty bucket (NB: none)
        size_t n = 0;
        std::vector<Heap> b;
        void init(int pk, const std::vector<uint64_t>* keys) {
            b.assign(NB, Heap{});
            for (Heap& h : b) {
                h.pk = pk;
                h.keys = keys;
            }
            minb = NB;
            n = 0;
        }
        bool empty() const { return n == 0; }
        size_t size() const { return n; }
        void push(uint64_t k0, int64_t v) {
            const int i = (int)(k0 >> 55);
            b[(size_t)i].push(k0, v);
            if (i < minb) minb = i;
            ++n;
        }
        int64_t top() const { return b[(size_t)minb].top(); }
        void pop() {
            b[(size_t)minb].pop();
            --n;
            while (minb < NB && b[(size_t)minb].empty()) ++minb;
        }
    };
    BucketHeap frontier;  // every node not popped yet: the reference's to_explore (pop order)
    // cached expansions in round order, to retire the ones that aged (their node then counts as
    // unexpanded again and is picked up by select() with the other smallest unexpanded nodes)
    std::vector<std::pair<int32_t, int64_t>> cache_fifo;
    size_t fifo_head = 0;
    BucketHeap unexpanded;  // the frontier nodes without usable cached children (expansion order)

    // ---------------------------------------------------------------- in-flight table
    static uint64_t tag_of(uint64_t h) { return (h >> 48) & 0xffffu; }
    void recent_insert(int64_t id, uint64_t h) {
        if (id - gen_lo[cur] >= age) {  // the current generation is full: it becomes the older one
            cur ^= 1;
            std::fill(gen[cur].begin(), gen[cur].end(), 0ull);
            gen_lo[cur] = id;
        }
        std::vector<uint64_t>& g = gen[cur];
        uint64_t s = h & gmask;
        while (g[s]) s = (s + 1) & gmask;
        g[s] = ((uint64_t)(id + 1) << 16) | tag_of(h);
    }
    // a node with id >= from equal to key k, or -1 (from >= the older generation's first id:
    // usable() admits only caches probed fewer than AGE appends ago)
    int64_t recent_find(const uint64_t* k, uint64_t h, int64_t from) const {
        const uint64_t tag = tag_of(h);
        for (int i = 0; i < 2; ++i) {
            const int gi = cur ^ i;
            if (i == 1 && gen_lo[cur] <= from) break;  // every id >= from is in the current one
            const std::vector<uint64_t>& g = gen[gi];
            for (uint64_t s = h & gmask; g[s]; s = (s + 1) & gmask) {
                if ((g[s] & 0xffffu) != tag) continue;
                const int64_t id = (int64_t)(g[s] >> 16) - 1;
                if (id >= from && memcmp(&keys[(size_t)id * kw], k, 8 * kw) == 0) return id;
            }
        }
        return -1;
    }

    int64_t add_node(const uint64_t* k, uint64_t h, int64_t par, int act, int tot, int dep) {
        const int64_t id = (int64_t)parent.size();
        keys.insert(keys.end(), k, k + kw);
        parent.push_back(par);
        action.push_back((int8_t)act);
        total.push_back((int16_t)tot);
        depth.push_back(dep);
        cache_slot.push_back(-1);
        recent_insert(id, h);
        pkeys.resize(pkeys.size() + pk);
        uint64_t* pkey = &pkeys[(size_t)id * pk];
        prio_key(k, tot, dep, pkey);
        frontier.push(pkey[0], id);
        unexpanded.push(pkey[0], id);
        return id;
    }

    // A cached expansion is usable while the whole visit stays inside the in-flight table's
    // reach: the visit appends up to ACT nodes, and an append that starts a new generation
    // keeps only the `age` ids before it (recent_insert), so every id >= `from` must still be
    // there after the visit's last append: parent.size() + ACT - from <= age.
    bool usable(int64_t id) const {
        const int32_t s = cache_slot[id];
        return s >= 0 && (int64_t)parent.size() + ACT - n_at_round[c_round[s]] <= age;
    }
    void drop_cache(int64_t id) {
        const int32_t s = cache_slot[id];
        if (s >= 0) {
            free_slots.push_back(s);
            cache_slot[id] = -1;
        }
    }

    // ---------------------------------------------------------------- one popped node
    bool visit(int64_t id) {
        const int32_t s = cache_slot[id];
        const uint64_t* ck = &c_keys[(size_t)s * ACT * kw];
        const uint64_t* hs = &c_hash[(size_t)s * ACT];
        const int64_t* kn = &c_known[(size_t)s * ACT];
        const int64_t from = n_at_round[c_round[s]];
        last_popped = id;
        popped.push_back(id);
        bool ended = false;
        for (int a = 0; a < ACT; ++a) {
            const uint64_t* k = ck + (size_t)a * kw;
            if (key_is_error(k)) {  // ACMove raised (utils.py:264-266)
                status = 3;
                ended = true;
                break;
            }
            const int len = key_total(k);
            last_action = a;
            last_len = len;
            if (len < min_length) {  // greedy.py:86-89
                min_length = len;
                trace.push_back(len);
            }
            if (len == 2) {  // greedy.py:91-100
                status = 1;
                found_parent = id;
                found_action = a;
                found_explored = (int64_t)parent.size() - (int64_t)frontier.size();
                memcpy(found_key, k, 8 * kw);
                ended = true;
                break;
            }
            // greedy.py:102-113: known to the device as of the probe, or appended since
            if (kn[a] >= 0) {
                ++st_known;
                continue;
            }
            if (recent_find(k, hs[a], from) >= 0) continue;
            add_node(k, hs[a], id, a, len, depth[id] + 1);
        }
        drop_cache(id);
        if (!ended && (int64_t)parent.size() >= max_nodes) {  // greedy.py:115-119
            status = 2;
            budget_hit = 1;
            ended = true;
        }
        return ended;
    }

    // the smallest frontier nodes without usable cached children (greedy expands them next)
    void push_unexpanded(int64_t id) { unexpanded.push(pkeys[(size_t)id * pk], id); }

    // the smallest frontier nodes without usable cached children (greedy expands them next)
    void select(std::vector<int64_t>& out) {
        out.clear();
        // retire the caches that aged since the last round: their nodes are unexpanded again
        const int64_t nn = (int64_t)parent.size();
        while (fifo_head < cache_fifo.size() && nn + ACT - n_at_round[cache_fifo[fifo_head].first] > age) {
            const auto [r, id] = cache_fifo[fifo_head++];
            const int32_t sl = cache_slot[id];
            if (sl >= 0 && c_round[sl] == r) {
                ++st_retired;
                drop_cache(id);
                push_unexpanded(id);
            }
        }
        if (fifo_head > 4096 && fifo_head * 2 > cache_fifo.size()) {
            cache_fifo.erase(cache_fifo.begin(), cache_fifo.begin() + (ptrdiff_t)fifo_head);
            fifo_head = 0;
        }
        while (!unexpanded.empty() && (int)out.size() < batch_cap) {
            out.push_back(unexpanded.top());
            unexpanded.pop();
        }
    }

    int expand_round(const std::vector<int64_t>& batch);

    int run(const int32_t* pres) {
        // the root: the (unreduced) input presentation itself (greedy.py:36-68)
        uint64_t root[ACX_MAX_L / 16 + 2];
        bfs::pack_key(pres, L, kw, root);
        int tot0 = 0;
        for (int i = 0; i < 2 * L; ++i) tot0 += pres[i] != 0;
        min_length = tot0;
        keys.assign(root, root + kw);
        parent.assign(1, -1);
        action.assign(1, -1);
        total.assign(1, (int16_t)tot0);
        depth.assign(1, 0);
        cache_slot.assign(1, -1);
        // every per-node array at its final size up front (no reallocation copies mid-search)
        const size_t nres = (size_t)std::min<int64_t>(cap, 1 << 26);
        keys.reserve(nres * kw);
        for (auto* v : {&parent}) v->reserve(nres);
        action.reserve(nres);
        total.reserve(nres);
        depth.reserve(nres);
        cache_slot.reserve(nres);
        for (auto& g : gen) g.assign((size_t)2 * age, 0ull);
        gmask = 2 * age - 1;
        cur = 0;
        gen_lo[0] = gen_lo[1] = 0;
        recent_insert(0, host_hash(root, kw));
        pkeys.assign(pk, 0ull);
        pkeys.reserve(nres * pk);
        prio_key(root, tot0, 0, pkeys.data());
        frontier.push(pkeys[0], 0);
        unexpanded.push(pkeys[0], 0);
        std::vector<int64_t> batch;
        while (status == 0) {
            const int64_t t0 = now_ns();
            const int64_t n_sel = (int64_t)parent.size();
            if (frontier.empty()) {  // to_explore ran empty (greedy.py:71)
                status = 2;
                break;
            }
            select(batch);
            const int64_t t1 = now_ns();
            ns_select += t1 - t0;
            const int e = expand_round(batch);
            if (e != ACX_OK) return e;
            const int64_t t2 = now_ns();
            ns_gpu += t2 - t1;
            ++round;
            // replay: pop while the top has usable cached children (greedy.py:71-119)
            while (status == 0) {
                if (frontier.empty()) {
                    status = 2;
                    break;
                }
                const int64_t id = frontier.top();
                if (!usable(id)) {
                    if (cache_slot[id] >= 0) {  // expanded before the last AGE appends: expand again
                        ++st_stop_aged;
                        drop_cache(id);
                        push_unexpanded(id);
                    } else if (id >= n_sel) {
                        ++st_stop_new;
                    } else {
                        ++st_stop_old;
                    }
                    break;
                }
                frontier.pop();
                visit(id);
            }
            ns_replay += now_ns() - t2;
        }
        return ACX_OK;
    }
};

struct RoundLaunch {
    Engine* E;
    template <int NW>
    void go() {
        const int n = E->d.n * ACT;
        const int cb = (int)((E->d.hi - E->d.lo + 255) / 256);
        greedy_round_kernel<NW><<<dim3((unsigned)(cb + (n + 255) / 256)), dim3(256), 0, E->stream>>>(E->d, cb);
    }
};
struct CommitLaunch {
    Engine* E;
    template <int NW>
    void go() {
        const int64_t n = E->d.hi - E->d.lo;
        greedy_commit_kernel<NW + 1><<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, E->stream>>>(E->d);
    }
};

void Engine::commit_launch() {
    CommitLaunch cl{this};
    bfs::by_nw(L, cl);
}

int Engine::expand_round(const std::vector<int64_t>& batch) {
    const int n = (int)batch.size();
    const int64_t n_nodes = (int64_t)parent.size();
    if (n_nodes > dcap && !grow(std::min<int64_t>(cap, std::max<int64_t>(2 * dcap, n_nodes)))) return ACX_E_LAUNCH;
    // staging in: the batch's parent keys, then the keys of the nodes appended since the last
    // round.  The last commit_cap of those are committed by the round's own launch, beside the
    // expansion (greedy_round_kernel), which therefore knows only the ids below them: the host
    // checks the children against every node from there on (n_at_round)
    for (int i = 0; i < n; ++i) memcpy(h_in + (size_t)i * kw, &keys[(size_t)batch[i] * kw], 8 * kw);
    int64_t lo = committed;
    d.commit = hd_in + (size_t)n * kw;
    while (n_nodes - lo > commit_cap) {  // a backlog beyond one launch's staging: commit ahead
        memcpy(h_in + (size_t)n * kw, &keys[(size_t)lo * kw], (size_t)commit_cap * kw * 8);
        d.lo = lo;
        d.hi = lo + commit_cap;
        commit_launch();
        lo += commit_cap;
        if (hipGetLastError() != hipSuccess || wait() != ACX_OK) return ACX_E_LAUNCH;  // h_in is reused
    }
    if (n_nodes > lo) memcpy(h_in + (size_t)n * kw, &keys[(size_t)lo * kw], (size_t)(n_nodes - lo) * kw * 8);
    d.lo = lo;
    d.hi = n_nodes;
    committed = n_nodes;
    n_at_round.push_back(lo);
    d.n = n;
    d.parents = hd_in;
    d.ckeys = hd_out;
    d.chash = hd_out + (size_t)n * ACT * kw;
    d.cknown = reinterpret_cast<int64_t*>(d.chash + (size_t)n * ACT);
    if (n == 0 && n_nodes == lo) return ACX_OK;
    d.blocks_done = d_blocks;
    d.done_flag = hd_flag;
    d.seq = ++round_seq;
    RoundLaunch rl{this};
    bfs::by_nw(L, rl);
    if (n == 0) return hipGetLastError() == hipSuccess ? wait_round(d.seq) : ACX_E_LAUNCH;
    const int64_t tw = now_ns();
    if (hipGetLastError() != hipSuccess || wait_round(d.seq) != ACX_OK) return ACX_E_LAUNCH;
    const int64_t tc = now_ns();
    ns_wait += tc - tw;
    const uint64_t* ck = h_out;
    const uint64_t* ch = h_out + (size_t)n * ACT * kw;
    const int64_t* kn = reinterpret_cast<const int64_t*>(ch + (size_t)n * ACT);
    for (int i = 0; i < n; ++i) {
        int32_t s;
        if (!free_slots.empty()) {
            s = free_slots.back();
            free_slots.pop_back();
        } else {
            s = (int32_t)c_round.size();
            c_round.push_back(0);
            c_keys.resize(c_keys.size() + (size_t)ACT * kw);
            c_hash.resize(c_hash.size() + ACT);
            c_known.resize(c_known.size() + ACT);
        }
        memcpy(&c_keys[(size_t)s * ACT * kw], ck + (size_t)i * ACT * kw, (size_t)ACT * kw * 8);
        memcpy(&c_hash[(size_t)s * ACT], ch + (size_t)i * ACT, ACT * 8);
        memcpy(&c_known[(size_t)s * ACT], kn + (size_t)i * ACT, ACT * 8);
        c_round[s] = round;
        cache_slot[batch[i]] = s;
        cache_fifo.emplace_back(round, batch[i]);
    }
    ns_cache += now_ns() - tc;
    ++st_rounds;
    st_expanded += n;
    return ACX_OK;
}

}  // namespace greedy
}  // namespace acx

using namespace acx::greedy;

extern "C" {

int acx_greedy_run(const int32_t* presentation, int32_t L, int64_t max_nodes, int32_t cyclical, int32_t batch,
                   void** out_handle) {
    if (!presentation || !out_handle || L < 1 || L > ACX_MAX_L || max_nodes < 1 || max_nodes > (1ll << 38))
        return ACX_E_ARG;
    *out_handle = nullptr;
    Engine* E = new (std::nothrow) Engine();
    if (!E) return ACX_E_LAUNCH;
    if (!E->init(L, max_nodes, cyclical != 0, batch)) {
        delete E;
        return ACX_E_LAUNCH;
    }
    const int st = E->run(presentation);
    *out_handle = E;
    return st;
}

void acx_greedy_destroy(void* h) { delete static_cast<Engine*>(h); }

// tests only (not in acx.h): searches started afterwards use 2^log2_age as the cache age limit
// (0: the default AGE), so the retirement of aged caches is exercised harder at test sizes
void acx_internal_greedy_age(int32_t log2_age) { g_age_override = log2_age > 0 ? (int64_t)1 << log2_age : 0; }
// tests only: searches started afterwards begin with a 2^log2_cap-node device store (0: INIT_DCAP),
// so the store's regrowth mid-search is exercised at test sizes
void acx_internal_greedy_init_cap(int32_t log2_cap) { g_dcap_override = log2_cap > 0 ? (int64_t)1 << log2_cap : 0; }
// tests only (host code, no GPU): the heap priority key of a packed key at L (out: the key's
// words, (40 + 6L + 63) / 64 of them), through the fast path (generic = 0, L <= 40) or the
// per-group one; returns the number of words, -1 on bad arguments
int32_t acx_internal_greedy_prio_key(int32_t L, const uint64_t* key, int32_t total, int32_t depth, uint64_t* out,
                                     int32_t generic) {
    if (L < 1 || L > ACX_MAX_L || !key || !out) return -1;
    Engine e;
    e.L = L;
    e.kw = acx_key_words(L);
    e.pk = (HDR + 6 * L + 63) / 64;
    e.prio_generic = generic != 0;
    e.prio_key(key, total, depth, out);
    return e.pk;
}

// 0 running, 1 success, 2 failed, 3 move error; budget_hit, min_length, nodes (len(tree_nodes))
int32_t acx_greedy_status(void* h, int32_t* budget_hit, int32_t* min_length, int64_t* n_nodes) {
    Engine* E = static_cast<Engine*>(h);
    if (budget_hit) *budget_hit = E->budget_hit;
    if (min_length) *min_length = E->min_length;
    if (n_nodes) *n_nodes = (int64_t)E->parent.size();
    return E->status;
}

// the returned path: success -> the found child's; otherwise the last popped node's plus its
// last child (greedy.py:100,121).  Returns the number of (action, total) entries.
int64_t acx_greedy_path(void* h, int32_t* actions, int32_t* totals, int64_t cap) {
    Engine* E = static_cast<Engine*>(h);
    const int64_t v0 = E->status == 1 ? E->found_parent : E->last_popped;
    if (v0 < 0) return 0;
    std::vector<int64_t> chain;
    for (int64_t v = v0; v >= 0; v = E->parent[v]) chain.push_back(v);
    int64_t n = 0;
    for (auto it = chain.rbegin(); it != chain.rend(); ++it, ++n)
        if (n < cap) {
            actions[n] = E->action[*it];
            totals[n] = E->total[*it];
        }
    if (n < cap) {
        actions[n] = E->status == 1 ? E->found_action : E->last_action;
        totals[n] = E->status == 1 ? 2 : E->last_len;
    }
    return n + 1;
}

// out[0] rounds, [1] parents expanded, [2] parents popped, [3] children the device knew,
// [4..6] host ns selecting / in the GPU round trip / replaying, [7..9] replays that stopped at a
// node appended during the replay / at an older unexpanded node / at an aged cache, [10..11] ns
// of the round trips spent polling for the GPU / caching children, [12] cached expansions
// retired unused because they aged
void acx_greedy_stats(void* h, int64_t* out) {
    Engine* E = static_cast<Engine*>(h);
    out[0] = E->st_rounds;
    out[1] = E->st_expanded;
    out[2] = (int64_t)E->popped.size();
    out[3] = E->st_known;
    out[4] = E->ns_select;
    out[5] = E->ns_gpu;
    out[6] = E->ns_replay;
    out[7] = E->st_stop_new;
    out[8] = E->st_stop_old;
    out[9] = E->st_stop_aged;
    out[10] = E->ns_wait;
    out[11] = E->ns_cache;
    out[12] = E->st_retired;
}

int64_t acx_greedy_min_trace(void* h, int32_t* out, int64_t cap) {
    Engine* E = static_cast<Engine*>(h);
    const int64_t n = (int64_t)E->trace.size();
    for (int64_t i = 0; out && i < n && i < cap; ++i) out[i] = E->trace[(size_t)i];
    return n;
}

int64_t acx_greedy_popped(void* h, int64_t* ids, int64_t cap) {
    Engine* E = static_cast<Engine*>(h);
    const int64_t n = (int64_t)E->popped.size();
    for (int64_t i = 0; ids && i < n && i < cap; ++i) ids[i] = E->popped[(size_t)i];
    return n;
}

int64_t acx_greedy_node_keys(void* h, uint64_t* out, int64_t cap) {
    Engine* E = static_cast<Engine*>(h);
    const int64_t n = (int64_t)E->parent.size();
    if (out) memcpy(out, E->keys.data(), (size_t)(n < cap ? n : cap) * E->kw * 8);
    return n;
}

int32_t acx_greedy_found(void* h, int32_t* first_letters, int64_t* explored) {
    Engine* E = static_cast<Engine*>(h);
    if (E->status != 1) return 0;
    static const int32_t letter[4] = {1, -1, 2, -2};
    const int bit1 = 2 * E->L;
    if (first_letters) {
        first_letters[0] = letter[E->found_key[0] & 3u];
        first_letters[1] = letter[(E->found_key[bit1 >> 6] >> (bit1 & 63)) & 3u];
    }
    if (explored) *explored = E->found_explored;
    return 1;
}

}  // extern "C"
