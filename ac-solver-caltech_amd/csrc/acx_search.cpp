// acx_search.cpp -- host-side search engine for greedy_search / bfs over GPU expansions.
//
// The reference searches (ac_solver/search/greedy.py:15-121, breadth_first.py:15-97) pop
// one node, call ACMove 12 times, and keep a Python set of state tuples.  Here the GPU
// expands many parents per launch (acx_expand12 -> packed child keys) and this engine
// replays the reference's sequential logic exactly on those keys:
//   * BFS: FIFO queue; per popped parent, children in action order: success test
//     (n0+n1 == 2), dedup-insert, enqueue; budget test after each parent
//     (breadth_first.py:61-95).  Parents are expanded ahead in FIFO order, which cannot
//     change the result because expansion is a pure function of the state.
//   * greedy: priority order (total length, path length, state tuple) -- a total order,
//     so heapq's pop sequence equals popping a min-heap on that order (greedy.py:71-113).  The smallest not-yet-expanded nodes are expanded
//     speculatively in one launch; children are cached until their parent is popped.
// Keys are the packed states of acx_expand12 (acx.h), so set membership is a hash of
// acx_key_words(L) uint64 words.
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "acx.h"

namespace {

// A fixed set of worker threads for the BFS batch phases: run(fn) calls fn(t) for t = 0..T-1,
// t = 0 on the calling thread, and returns when all are done.
class Pool {
  public:
    explicit Pool(int n) : n_(n < 1 ? 1 : n) {
        for (int t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return n_; }
    void run(const std::function<void(int)>& fn) {
        if (n_ == 1) {
            fn(0);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            left_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
        fn_ = nullptr;
    }

  private:
    void loop(int t) {
        uint64_t seen = 0;
        while (true) {
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (quit_) return;
                fn = fn_;
            }
            (*fn)(t);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int left_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

// std::vector whose resize() leaves new trivially-constructible elements uninitialised (the BFS
// commit writes every new node's fields once; value-initialising them first was a second pass)
template <class T>
struct DefaultInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInit<U>;
    };
    DefaultInit() noexcept = default;
    template <class U>
    DefaultInit(const DefaultInit<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
template <class T>
using dvec = std::vector<T, DefaultInit<T>>;

// transparent huge pages for a large buffer (where the kernel's THP mode is "madvise"): the BFS
// node arrays and visited-set partitions are first touched by many threads at once, and 4-KB
// page faults serialise on the process's address-space lock
inline void advise_huge(const void* p, size_t bytes) {
    constexpr uintptr_t HP = (uintptr_t)2 << 20;
    const uintptr_t a = ((uintptr_t)p + HP - 1) & ~(HP - 1), b = ((uintptr_t)p + bytes) & ~(HP - 1);
    if (b > a) (void)madvise((void*)a, b - a, MADV_HUGEPAGE);
}

// host threads for the BFS engine: ACX_HOST_THREADS, else the CPUs this process may run on,
// at most 16 (the GPU box's CPU share per GPU)
int host_threads() {
    if (const char* e = std::getenv("ACX_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) return v < 64 ? v : 64;
    }
    cpu_set_t cs;
    int n = 0;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
    if (n < 1) n = (int)std::thread::hardware_concurrency();
    return n < 1 ? 1 : (n > 16 ? 16 : n);
}

constexpr int ACT = 12;
constexpr int HDR = 40;         // priority-key header bits: total (9) | depth (31)

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

struct Engine {
    int mode;  // 0 bfs, 1 greedy
    int L, kw;
    int64_t max_nodes;
    // node storage
    dvec<uint64_t> keys;  // node * kw
    dvec<int64_t> parent;
    dvec<int8_t> action;
    dvec<int16_t> total;
    dvec<int32_t> depth;  // greedy only
    // open-addressing hash set; entry = (node id + 1) << 24 | 24-bit hash tag, 0 = empty.
    // The tag filters almost every non-matching probe without touching the node's key.
    std::vector<uint64_t> table;
    uint64_t mask = 0;
    int64_t n_set = 0;
    // greedy's expansion bookkeeping (BFS: every node is queued once, when it is found, so the
    // FIFO queue is the node ids in order -- queue[i] == i -- and is not stored)
    std::vector<int64_t> queue;
    size_t head = 0, requested = 0;
    // greedy ordered frontier: the heap tuple (total, path length, state tuple) of
    // greedy.py:55-64,104-113 packed MSB-first into pk words per node -- total (9 bits: up to
    // 2L = 256), depth (31 bits), then every letter + 2 (3 bits, r0 then r1 incl. padding) --
    // so comparing the words as unsigned integers is Python's tuple order.  Two 4-ary min-heaps
    // with the keys inline (no pointer chasing per comparison): all unpopped nodes (pop
    // order) and the subset not yet sent to the GPU (speculative expansion order).
    int pk = 0;
    struct Heap {
        int pk = 0;
        std::vector<uint64_t> k;  // size() * pk key words
        std::vector<int64_t> id;
        bool empty() const { return id.empty(); }
        int64_t top() const { return id[0]; }
        bool less(const uint64_t* a, const uint64_t* b) const {
            for (int i = 0; i < pk; ++i)
                if (a[i] != b[i]) return a[i] < b[i];
            return false;
        }
        void push(const uint64_t* key, int64_t v) {
            size_t i = id.size();
            id.push_back(v);
            k.resize(k.size() + pk);
            uint64_t tmp[32];
            std::memcpy(tmp, key, sizeof(uint64_t) * pk);
            while (i > 0) {
                const size_t par = (i - 1) / 4;
                if (!less(tmp, &k[par * pk])) break;
                std::memcpy(&k[i * pk], &k[par * pk], sizeof(uint64_t) * pk);
                id[i] = id[par];
                i = par;
            }
            std::memcpy(&k[i * pk], tmp, sizeof(uint64_t) * pk);
            id[i] = v;
        }
        void pop() {
            const size_t n = id.size() - 1;
            if (n == 0) {
                id.clear();
                k.clear();
                return;
            }
            uint64_t tmp[32];
            std::memcpy(tmp, &k[n * pk], sizeof(uint64_t) * pk);
            const int64_t v = id[n];
            id.pop_back();
            k.resize(n * pk);
            size_t i = 0;
            while (true) {
                const size_t c0 = 4 * i + 1;
                if (c0 >= n) break;
                size_t best = c0;
                const size_t ce = c0 + 4 < n ? c0 + 4 : n;
                for (size_t c = c0 + 1; c < ce; ++c)
                    if (less(&k[c * pk], &k[best * pk])) best = c;
                if (!less(&k[best * pk], tmp)) break;
                std::memcpy(&k[i * pk], &k[best * pk], sizeof(uint64_t) * pk);
                id[i] = id[best];
                i = best;
            }
            std::memcpy(&k[i * pk], tmp, sizeof(uint64_t) * pk);
            id[i] = v;
        }
    };
    Heap frontier;    // pop order (all unpopped nodes)
    Heap unexpanded;  // the subset not yet sent to the GPU
    // children cache: node -> offset into cache_keys (ACT * kw words), -1 = not cached
    std::vector<int64_t> cache_pos;
    bool cached(int64_t id) const { return cache_pos[id] >= 0; }
    std::vector<uint64_t> cache_keys;
    std::vector<uint64_t> cache_hash;  // ACT hashes per slot (computed once, reused for prefetch)
    std::vector<size_t> free_slots;
    // last request (order of nodes handed to next_batch)
    std::vector<int64_t> batch;
    // result
    int status = 0;  // 0 running, 1 success, 2 failed (budget or exhausted), 3 move error
    int64_t found_parent = -1;
    int found_action = -1, found_len = -1;
    int last_action = -1, last_len = -1;
    int64_t last_popped = -1;
    int min_length = 0;
    int budget_hit = 0;
    std::vector<int32_t> trace;  // each new minimum total, in the order found (greedy.py:86-89)
    std::vector<int64_t> popped; // node ids in expansion (pop) order
    int64_t found_explored = 0;  // len(tree_nodes) - len(to_explore) at the success (greedy.py:94)
    uint64_t found_key[ACX_MAX_L / 16 + 2] = {0};
    // statistics: rounds (next_batch calls that returned parents), parents expanded, pops
    int64_t st_rounds = 0, st_expanded = 0, st_pops = 0;
    int64_t ns_next = 0, ns_store = 0, ns_visit = 0;  // host time in next_batch / caching children / replay
    static int64_t now_ns() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }

    // ---- BFS (mode 0): each fed batch of parents is processed by T threads (feed_bfs) ----
    // The visited set is partitioned by hash over T tables, one per thread, so a thread probes
    // and inserts in its own table only.  Entry: (node id + 1) << 24 | tag; while a batch is being
    // processed, a child it inserts holds a provisional entry PROV | (batch seq + 1) << 24 | tag
    // (its key is in the fed child keys) until the commit gives it its node id.
    static constexpr uint64_t PROV = 1ull << 63;
    static constexpr uint64_t ID_MASK = (1ull << 39) - 1;
    struct Part {
        dvec<uint64_t> table;
        uint64_t mask = 0;
        int64_t n = 0;
        std::vector<int64_t> own;  // the batch's children this partition owns, in sequence order
    };
    Pool* pool = nullptr;
    std::vector<Part> parts;
    std::vector<uint64_t> b_hash;  // per child of the batch
    std::vector<int16_t> b_len;    // total length, -1: the move failed
    std::vector<uint8_t> b_own, b_new;
    std::vector<uint64_t> b_slot;
    std::vector<int64_t> b_base;  // per parent: the first node id its new children get
    int n_threads = 1;
    uint64_t part_hint = 0;  // slots per partition sized once for the budget (no rehash on the way)
    int64_t ph_ns[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // feed_bfs phases (acx_internal_search_phases)

    int owner(uint64_t h) const { return (int)((((h >> 24) & 0xffffull) * (uint64_t)n_threads) >> 16); }

    Engine(int mode_, int L_, int64_t max_nodes_) : mode(mode_), L(L_), kw(acx_key_words(L_)), max_nodes(max_nodes_) {
        table.assign(1 << 12, 0);
        mask = table.size() - 1;
        pk = (HDR + 6 * L + 63) / 64;
        frontier.pk = unexpanded.pk = pk;
        if (mode == 0) {
            n_threads = host_threads();
            pool = new Pool(n_threads);
            parts.resize(n_threads);
            for (Part& P : parts) {
                P.table.assign(1 << 12, 0);
                P.mask = P.table.size() - 1;
            }
            // the node arrays and the visited set sized for the budget up front (capacity only:
            // pages are touched when written), so no reallocation copies or rehashes on the way
            const int64_t rn = std::min<int64_t>(max_nodes, (int64_t)1 << 27) + 12 * 65536;
            keys.reserve((size_t)rn * kw);
            parent.reserve((size_t)rn);
            action.reserve((size_t)rn);
            total.reserve((size_t)rn);
            advise_huge(keys.data(), keys.capacity() * sizeof(uint64_t));
            advise_huge(parent.data(), parent.capacity() * sizeof(int64_t));
            advise_huge(action.data(), action.capacity());
            advise_huge(total.data(), total.capacity() * sizeof(int16_t));
            uint64_t h = 4096;
            while (h < (uint64_t)(2.5 * (double)rn / n_threads)) h <<= 1;
            part_hint = h;
        }
    }
    ~Engine() { delete pool; }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    // partition P holds committed entries only (between batches): rehash into >= `want` slots
    void grow_part(Part& P, uint64_t want) {
        uint64_t sz = P.table.size();
        if (sz < part_hint && P.n <= 1) sz = part_hint;  // first batch: the budget's size at once
        while (sz < want) sz <<= 1;
        if (sz == P.table.size()) return;
        dvec<uint64_t> old;
        old.swap(P.table);
        P.table.reserve(sz);
        advise_huge(P.table.data(), sz * sizeof(uint64_t));
        P.table.resize(sz);
        std::memset(P.table.data(), 0, sz * sizeof(uint64_t));
        P.mask = sz - 1;
        for (uint64_t e : old)
            if (e) {
                const int64_t id = (int64_t)((e >> 24) & ID_MASK) - 1;
                const uint64_t h = hash_key(&keys[(size_t)id * kw]);
                uint64_t q = h & P.mask;
                while (P.table[q]) q = (q + 1) & P.mask;
                P.table[q] = e;
            }
    }

    uint64_t hash_key(const uint64_t* k) const {
        uint64_t h = 0x9e3779b97f4a7c15ull;
        for (int i = 0; i < kw; ++i) h = mix64(h ^ k[i]) + (uint64_t)i;
        return h;
    }
    static uint64_t entry(int64_t id, uint64_t h) { return ((uint64_t)(id + 1) << 24) | (h >> 40); }
    void grow() {
        std::vector<uint64_t> old;
        old.swap(table);
        table.assign(old.size() * 2, 0);
        mask = table.size() - 1;
        for (uint64_t e : old)
            if (e) {
                const int64_t id = (int64_t)(e >> 24) - 1;
                const uint64_t h = hash_key(&keys[(size_t)id * kw]);
                uint64_t p = h & mask;
                while (table[p]) p = (p + 1) & mask;
                table[p] = entry(id, h);
            }
    }
    // find key with hash h; returns node id or -1; *slot gets the insert position
    int64_t find(const uint64_t* k, uint64_t h, uint64_t* slot) const {
        const uint64_t tag = h >> 40;
        uint64_t p = h & mask;
        while (true) {
            const uint64_t e = table[p];
            if (!e) { *slot = p; return -1; }
            if ((e & 0xffffffull) == tag) {
                const int64_t id = (int64_t)(e >> 24) - 1;
                if (std::memcmp(&keys[(size_t)id * kw], k, sizeof(uint64_t) * kw) == 0) return id;
            }
            p = (p + 1) & mask;
        }
    }
    void prefetch_children(int64_t id) const {
        if (!cached(id)) return;
        const uint64_t* hs = &cache_hash[(size_t)cache_pos[id] / kw];
        for (int a = 0; a < ACT; ++a) __builtin_prefetch(&table[hs[a] & mask], 0, 1);
    }
    static int key_len(const uint64_t* k, int L) {
        const int bit = 4 * L;
        const uint64_t lo = k[bit >> 6] >> (bit & 63);
        const uint64_t hi = (bit & 63) > 48 ? (k[(bit >> 6) + 1] << (64 - (bit & 63))) : 0ull;
        const uint64_t v = lo | hi;
        return (int)(v & 0xff) + (int)((v >> 8) & 0xff);
    }
    // acx_expand12's key for a child whose move failed: both length bytes 0xFF
    static bool key_is_error(const uint64_t* k, int L) {
        const int bit = 4 * L;
        const uint64_t lo = k[bit >> 6] >> (bit & 63);
        const uint64_t hi = (bit & 63) > 48 ? (k[(bit >> 6) + 1] << (64 - (bit & 63))) : 0ull;
        return ((lo | hi) & 0xffffull) == 0xffffull;
    }
    // the packed priority key of a node (see Heap)
    void prio_key(const uint64_t* k, int tot, int dep, uint64_t* out) const {
        int n[2];
        {
            const int bit = 4 * L;
            const uint64_t lo = k[bit >> 6] >> (bit & 63);
            const uint64_t hi = (bit & 63) > 48 ? (k[(bit >> 6) + 1] << (64 - (bit & 63))) : 0ull;
            n[0] = (int)((lo | hi) & 0xff);
            n[1] = (int)(((lo | hi) >> 8) & 0xff);
        }
        for (int i = 0; i < pk; ++i) out[i] = 0;
        out[0] = ((uint64_t)(tot & 0x1ff) << 55) | ((uint64_t)(dep & 0x7fffffff) << 24);
        static const uint64_t val[4] = {3, 1, 4, 0};  // letter + 2 for codes x, x^-1, y, y^-1
        int pos = HDR;  // next free bit, counted from the MSB of word 0
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < L; ++i, pos += 3) {
                const int bit = 2 * (h * L + i);
                const int code = (int)((k[bit >> 6] >> (bit & 63)) & 3u);
                const uint64_t v = i < n[h] ? val[code] : 2;  // padding 0 -> 2
                // 3 bits at MSB-first position pos (may straddle two words)
                const int w = pos >> 6, o = pos & 63;
                if (o <= 61) {
                    out[w] |= v << (61 - o);
                } else {
                    out[w] |= v >> (o - 61);
                    out[w + 1] |= v << (64 - (o - 61));
                }
            }
    }
    int64_t add_node(const uint64_t* k, uint64_t h, uint64_t slot, int64_t par, int act, int tot, int dep) {
        const int64_t id = (int64_t)parent.size();
        keys.insert(keys.end(), k, k + kw);
        parent.push_back(par);
        action.push_back((int8_t)act);
        total.push_back((int16_t)tot);
        depth.push_back(dep);
        cache_pos.push_back(-1);
        table[slot] = entry(id, h);
        ++n_set;
        if ((uint64_t)n_set * 2 > table.size()) grow();
        return id;
    }

    void push_frontier(int64_t id, const uint64_t* k) {
        uint64_t key[32];
        prio_key(k, total[id], depth[id], key);
        frontier.push(key, id);
        unexpanded.push(key, id);
    }

    void start(const uint64_t* k) {
        uint64_t slot = 0;
        const uint64_t h = hash_key(k);
        const int tot = key_len(k, L);
        min_length = tot;
        if (mode == 0) {  // the root in its partition of the visited set
            Part& P = parts[owner(h)];
            keys.insert(keys.end(), k, k + kw);
            parent.push_back(-1);
            action.push_back(-1);
            total.push_back((int16_t)tot);
            depth.push_back(0);
            cache_pos.push_back(-1);
            P.table[h & P.mask] = entry(0, h);
            P.n = 1;
            n_set = 1;
            return;
        }
        find(k, h, &slot);
        const int64_t id = add_node(k, h, slot, -1, -1, tot, 0);
        push_frontier(id, k);
    }

    int64_t next_batch(uint64_t* out, int64_t cap) {
        const int64_t t0 = now_ns();
        const int64_t n = next_batch_(out, cap);
        ns_next += now_ns() - t0;
        return n;
    }
    int64_t next_batch_(uint64_t* out, int64_t cap) {
        batch.clear();
        if (status != 0) return 0;
        if (mode == 0) {  // the FIFO queue is the node ids in order
            while ((int64_t)batch.size() < cap && (int64_t)requested < n_set) batch.push_back((int64_t)requested++);
        } else {
            // the smallest unpopped nodes not expanded yet (speculative: their children are
            // cached until the node is popped in the reference's order)
            while ((int64_t)batch.size() < cap && !unexpanded.empty()) {
                batch.push_back(unexpanded.top());
                unexpanded.pop();
            }
        }
        for (size_t i = 0; i < batch.size(); ++i)
            std::memcpy(out + i * kw, &keys[(size_t)batch[i] * kw], sizeof(uint64_t) * kw);
        if (!batch.empty()) ++st_rounds;
        st_expanded += (int64_t)batch.size();
        return (int64_t)batch.size();
    }

    void store_children(int64_t id, const uint64_t* ck) {
        size_t off;
        if (!free_slots.empty()) {
            off = free_slots.back();
            free_slots.pop_back();
        } else {
            off = cache_keys.size();
            cache_keys.resize(off + (size_t)ACT * kw);
            cache_hash.resize(cache_hash.size() + ACT);
        }
        std::memcpy(&cache_keys[off], ck, sizeof(uint64_t) * ACT * kw);
        for (int a = 0; a < ACT; ++a) cache_hash[off / kw + a] = hash_key(ck + (size_t)a * kw);
        cache_pos[id] = (int64_t)off;
    }

    // expand one popped node from its cached children; returns true when the search ends
    bool visit(int64_t id) {
        const size_t off = (size_t)cache_pos[id];
        const uint64_t* ck = &cache_keys[off];
        const uint64_t* hs = &cache_hash[off / kw];
        last_popped = id;
        ++st_pops;
        popped.push_back(id);
        bool ended = false;
        for (int a = 0; a < ACT && !ended; ++a) {
            const uint64_t* k = ck + (size_t)a * kw;
            if (key_is_error(k, L)) {  // ACMove raised (utils.py:264-266) before any test
                status = 3;
                ended = true;
                break;
            }
            const int len = key_len(k, L);
            last_action = a;
            last_len = len;
            if (len < min_length) {
                min_length = len;
                trace.push_back(len);
            }
            if (len == 2) {  // greedy.py:91, breadth_first.py:84
                status = 1;
                found_parent = id;
                found_action = a;
                found_len = len;
                found_explored = n_set - (int64_t)frontier.id.size();
                std::memcpy(found_key, k, sizeof(uint64_t) * kw);
                ended = true;
                break;
            }
            uint64_t slot = 0;
            if (find(k, hs[a], &slot) < 0) {
                const int64_t nid = add_node(k, hs[a], slot, id, a, len, depth[id] + 1);
                if (mode == 0) queue.push_back(nid);
                else {
                    push_frontier(nid, k);
                }
            }
        }
        cache_pos[id] = -1;
        free_slots.push_back(off);
        if (!ended && n_set >= max_nodes) {  // greedy.py:115, breadth_first.py:91
            status = 2;
            budget_hit = 1;
            ended = true;
        }
        return ended;
    }

    // BFS: the fed batch = the parents queue[head, head + P) in FIFO order, their children (P, 12,
    // kw) in the reference's order (parent, then action: sequence number c = 12 g + a).  Same
    // result as visiting them one by one (visit()):
    //   1. (threads, by child) hash, total length / move error, owner partition;
    //   2. (one thread) the first move error and the first success in sequence order, and the
    //      new minimum totals up to there (breadth_first.py:76-89);
    //   3. (threads, by partition) every child before that point, in sequence order within the
    //      partition: probe, and insert the ones not seen -- the first occurrence in sequence order
    //      wins, as the reference's sequential `in tree_nodes` test;
    //   4. (one thread, per parent) node ids in FIFO order and the budget cut after the first parent
    //      that brings len(tree_nodes) to max_nodes (breadth_first.py:91);
    //   5. (threads, by parent) the new nodes written at their ids; (by partition) their entries.
    int feed_bfs(const uint64_t* ck, int64_t P) {
        const int64_t t0 = now_ns();
        const int T = n_threads;
        const int64_t C = P * ACT;
        b_hash.resize((size_t)C);
        b_len.resize((size_t)C);
        b_own.resize((size_t)C);
        b_new.assign((size_t)C, 0);
        b_slot.resize((size_t)C);
        b_base.resize((size_t)P + 1);
        pool->run([&](int t) {
            const int64_t c0 = C * t / T, c1 = C * (t + 1) / T;
            for (int64_t c = c0; c < c1; ++c) {
                const uint64_t* k = ck + (size_t)c * kw;
                const uint64_t h = hash_key(k);
                b_hash[(size_t)c] = h;
                b_len[(size_t)c] = key_is_error(k, L) ? (int16_t)-1 : (int16_t)key_len(k, L);
                b_own[(size_t)c] = (uint8_t)owner(h);
            }
        });
        const int64_t t1 = now_ns();
        ns_store += t1 - t0;
        // 2. the reference's per-child order: move error (utils.py:264-266, before any test), new
        // minimum (breadth_first.py:79-82), success (:84-88), then the dedup insert -- the first
        // error or success ends the search there (if the budget has not ended it before)
        int64_t end = C, succ = -1, err_c = -1;
        for (int64_t c = 0; c < C; ++c) {
            const int len = b_len[(size_t)c];
            if (len < 0 || len == 2) {
                (len < 0 ? err_c : succ) = c;
                end = c;
                break;
            }
        }
        const int64_t t2 = now_ns();
        ph_ns[0] += t2 - t1;
        // 3. probe / insert by partition
        pool->run([&](int t) {
            Part& Pt = parts[t];
            Pt.own.clear();
            for (int64_t c = 0; c < end; ++c)
                if (b_own[(size_t)c] == t) Pt.own.push_back(c);
            grow_part(Pt, 2 * (uint64_t)(Pt.n + (int64_t)Pt.own.size()) + 2);
            const size_t m = Pt.own.size();
            for (size_t i = 0; i < m; ++i) {
                // two prefetch stages: the table line 16 children ahead, and 8 ahead (that line is
                // in cache by then) the stored key of a tag match, which a duplicate is compared with
                if (i + 16 < m) __builtin_prefetch(&Pt.table[b_hash[(size_t)Pt.own[i + 16]] & Pt.mask], 0, 1);
                if (i + 8 < m) {
                    const uint64_t hh = b_hash[(size_t)Pt.own[i + 8]];
                    const uint64_t e = Pt.table[hh & Pt.mask];
                    if (e && !(e & PROV) && (e & 0xffffffull) == (hh >> 40))
                        __builtin_prefetch(&keys[(size_t)(((e >> 24) & ID_MASK) - 1) * kw], 0, 1);
                }
                const int64_t c = Pt.own[i];
                const uint64_t h = b_hash[(size_t)c];
                const uint64_t* k = ck + (size_t)c * kw;
                const uint64_t tag = h >> 40;
                uint64_t q = h & Pt.mask;
                bool seen = false;
                while (true) {
                    const uint64_t e = Pt.table[q];
                    if (!e) break;
                    if ((e & 0xffffffull) == tag) {
                        const int64_t v = (int64_t)((e >> 24) & ID_MASK) - 1;
                        const uint64_t* o = (e & PROV) ? ck + (size_t)v * kw : &keys[(size_t)v * kw];
                        if (std::memcmp(o, k, sizeof(uint64_t) * kw) == 0) {
                            seen = true;
                            break;
                        }
                    }
                    q = (q + 1) & Pt.mask;
                }
                if (!seen) {
                    Pt.table[q] = PROV | ((uint64_t)(c + 1) << 24) | tag;
                    b_slot[(size_t)c] = q;
                    b_new[(size_t)c] = 1;
                    ++Pt.n;
                }
            }
        });
        const int64_t t3 = now_ns();
        ph_ns[1] += t3 - t2;
        // 4. ids in FIFO order; where the batch stops (an error / success inside parent g, or the
        // budget after parent g)
        int64_t n = n_set, stop = P - 1;
        bool budget = false;
        for (int64_t g = 0; g < P; ++g) {
            b_base[(size_t)g] = n;
            const int64_t c0 = g * ACT, c1 = c0 + ACT < end ? c0 + ACT : end;
            for (int64_t c = c0; c < c1; ++c) n += b_new[(size_t)c];
            if (end < c0 + ACT) {
                stop = g;
                break;
            }
            if (n >= max_nodes) {
                stop = g;
                budget = true;
                break;
            }
        }
        const int64_t limit = std::min<int64_t>(end, (stop + 1) * ACT);  // children committed: c < limit
        const bool ended_here = end < (stop + 1) * ACT;  // the error / success is inside the last visited parent
        // the new minimum totals over the children the reference tests, in order (the successful
        // child included, the failing one not)
        const int64_t trace_end = ended_here && succ >= 0 ? succ + 1 : limit;
        for (int64_t c = 0; c < trace_end; ++c) {
            const int len = b_len[(size_t)c];
            if (len < min_length) {
                min_length = len;
                trace.push_back(len);
            }
        }
        const int64_t t4 = now_ns();
        ph_ns[2] += t4 - t3;
        // 5. commit
        const int64_t n0 = n_set;
        keys.resize((size_t)n * kw);
        parent.resize((size_t)n);
        action.resize((size_t)n);
        total.resize((size_t)n);
        const int64_t qh = (int64_t)head;
        const int64_t t5 = now_ns();
        ph_ns[3] += t5 - t4;
        pool->run([&](int t) {
            const int64_t g0 = (stop + 1) * t / T, g1 = (stop + 1) * (t + 1) / T;
            for (int64_t g = g0; g < g1; ++g) {
                const int64_t par = qh + g;
                int64_t id = b_base[(size_t)g];
                const int64_t c0 = g * ACT, c1 = c0 + ACT < limit ? c0 + ACT : limit;
                for (int64_t c = c0; c < c1; ++c) {
                    if (!b_new[(size_t)c]) continue;
                    std::memcpy(&keys[(size_t)id * kw], ck + (size_t)c * kw, sizeof(uint64_t) * kw);
                    parent[(size_t)id] = par;
                    action[(size_t)id] = (int8_t)(c - c0);
                    total[(size_t)id] = b_len[(size_t)c];
                    b_slot[(size_t)c] |= (uint64_t)id << 32;  // slot < 2^32 (a partition's size)
                    ++id;
                }
            }
        });
        const int64_t t6 = now_ns();
        ph_ns[4] += t6 - t5;
        pool->run([&](int t) {
            Part& Pt = parts[t];
            for (const int64_t c : Pt.own) {
                if (!b_new[(size_t)c]) continue;
                const uint64_t q = b_slot[(size_t)c] & 0xffffffffull;
                // a child past the cut keeps its provisional entry: the search ends with this batch
                if (c < limit) Pt.table[q] = entry((int64_t)(b_slot[(size_t)c] >> 32), b_hash[(size_t)c]);
            }
        });
        ph_ns[5] += now_ns() - t6;
        n_set = n;
        (void)n0;
        // bookkeeping as visit() leaves it
        const int64_t visited = stop + 1;  // parents qh .. qh + stop popped (acx_search_popped: ids 0 .. st_pops - 1)
        st_pops += visited;
        last_popped = qh + stop;
        head += (size_t)visited;
        const int64_t last_c = ended_here ? (err_c >= 0 ? err_c - 1 : succ) : limit - 1;
        if (last_c >= 0) {
            last_action = (int)(last_c % ACT);
            last_len = b_len[(size_t)last_c];
        }
        if (ended_here && err_c >= 0) {
            status = 3;
        } else if (ended_here) {
            status = 1;
            const int64_t g = succ / ACT;
            found_parent = qh + g;
            found_action = (int)(succ % ACT);
            found_len = 2;
            found_explored = qh + g + 1;  // n_set - (len(queue) - head) with every node queued once
            std::memcpy(found_key, ck + (size_t)succ * kw, sizeof(uint64_t) * kw);
        } else if (budget) {
            status = 2;
            budget_hit = 1;
        } else if ((int64_t)head >= n_set) {
            status = 2;  // the queue ran out (breadth_first.py:97)
        }
        ns_visit += now_ns() - t1;
        return status;
    }

    int feed(const uint64_t* child_keys, int64_t count) {
        if (mode == 0) {
            if (count != (int64_t)batch.size() || (int64_t)head + count != (int64_t)requested) return -1;
            if (status != 0) return status;
            batch.clear();
            return count > 0 ? feed_bfs(child_keys, count) : status;
        }
        const int64_t t0 = now_ns();
        for (int64_t i = 0; i < count && i < (int64_t)batch.size(); ++i)
            store_children(batch[i], child_keys + (size_t)i * ACT * kw);
        batch.clear();
        const int64_t t1 = now_ns();
        ns_store += t1 - t0;
        const int st = replay();
        ns_visit += now_ns() - t1;
        return st;
    }
    int replay() {  // greedy: pop as far as the cached children allow
        while (status == 0) {
            if (frontier.empty()) {
                status = 2;
                break;
            }
            const int64_t id = frontier.top();
            if (!cached(id)) return 0;
            frontier.pop();
            if (visit(id)) break;
        }
        return status;
    }

    // path of node `id` as (action, total) pairs from the root (root = (-1, total))
    int64_t path(int64_t id, int32_t* acts, int32_t* lens, int64_t cap, bool append_found) const {
        std::vector<int64_t> chain;
        for (int64_t v = id; v >= 0; v = parent[v]) chain.push_back(v);
        int64_t n = 0;
        for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
            if (n < cap) {
                acts[n] = action[*it];
                lens[n] = total[*it];
            }
            ++n;
        }
        if (append_found) {
            if (n < cap) {
                acts[n] = found_action >= 0 ? found_action : last_action;
                lens[n] = found_action >= 0 ? found_len : last_len;
            }
            ++n;
        }
        return n;
    }
};

}  // namespace

extern "C" {

void* acx_search_create(int32_t mode, int32_t L, const uint64_t* start_key, int64_t max_nodes) {
    if ((mode != 0 && mode != 1) || L < 1 || L > ACX_MAX_L || !start_key) return nullptr;
    Engine* e = new Engine(mode, L, max_nodes);
    e->start(start_key);
    return e;
}

void acx_search_destroy(void* h) { delete static_cast<Engine*>(h); }

int64_t acx_search_next_batch(void* h, uint64_t* parent_keys, int64_t cap) {
    return static_cast<Engine*>(h)->next_batch(parent_keys, cap);
}

int32_t acx_search_feed(void* h, const uint64_t* child_keys, int64_t count) {
    return static_cast<Engine*>(h)->feed(child_keys, count);
}

// 0 running, 1 success, 2 failed, 3 move error; *budget_hit = 1 when the node budget ended
// the search
int32_t acx_search_status(void* h, int32_t* budget_hit, int32_t* min_length, int64_t* n_nodes) {
    Engine* e = static_cast<Engine*>(h);
    if (budget_hit) *budget_hit = e->budget_hit;
    if (min_length) *min_length = e->min_length;
    if (n_nodes) *n_nodes = e->n_set;
    return e->status;
}

// success: path of the found child; failure (greedy): path of the last popped node plus its
// last child (greedy.py:121).  Returns the number of (action, total) entries.
int64_t acx_search_path(void* h, int32_t* actions, int32_t* totals, int64_t cap) {
    Engine* e = static_cast<Engine*>(h);
    if (e->status == 1) return e->path(e->found_parent, actions, totals, cap, true);
    if (e->last_popped < 0) return 0;
    return e->path(e->last_popped, actions, totals, cap, true);
}

// BFS batch phases (tools/host_bfs_bench.cpp; not in the public header): ns in 2 (scan), 3
// (probe / insert), 4 (ids / cut), resize, 5 (node arrays), 5 (table entries)
void acx_internal_search_phases(void* h, int64_t* out) {
    Engine* e = static_cast<Engine*>(h);
    for (int i = 0; i < 6; ++i) out[i] = e->ph_ns[i];
}

// statistics: out[0] = rounds, out[1] = parents expanded on the GPU, out[2] = parents popped,
// out[3..5] = host nanoseconds in next_batch / caching fed children / the replay
void acx_search_stats(void* h, int64_t* out) {
    Engine* e = static_cast<Engine*>(h);
    out[0] = e->st_rounds;
    out[1] = e->st_expanded;
    out[2] = e->st_pops;
    out[3] = e->ns_next;
    out[4] = e->ns_store;
    out[5] = e->ns_visit;
}

// ids of the expanded (popped) nodes in the reference's expansion order; returns the count
int64_t acx_search_popped(void* h, int64_t* ids, int64_t cap) {
    Engine* e = static_cast<Engine*>(h);
    if (e->mode == 0) {  // BFS pops the node ids in order
        for (int64_t i = 0; ids && i < e->st_pops && i < cap; ++i) ids[i] = i;
        return e->st_pops;
    }
    const int64_t n = (int64_t)e->popped.size();
    for (int64_t i = 0; ids && i < n && i < cap; ++i) ids[i] = e->popped[(size_t)i];
    return n;
}

// the new minimum totals in the order found (the verbose "New minimal length found" lines)
int64_t acx_search_min_trace(void* h, int32_t* out, int64_t cap) {
    Engine* e = static_cast<Engine*>(h);
    const int64_t n = (int64_t)e->trace.size();
    for (int64_t i = 0; out && i < n && i < cap; ++i) out[i] = e->trace[(size_t)i];
    return n;
}

// after a success: the first letters of both relators of the found child (each of length 1) and
// len(tree_nodes) - len(to_explore) at that moment (greedy.py:92-95); returns 1, else 0
int32_t acx_search_found(void* h, int32_t* first_letters, int64_t* explored) {
    Engine* e = static_cast<Engine*>(h);
    if (e->status != 1) return 0;
    static const int32_t letter[4] = {1, -1, 2, -2};
    const int bit1 = 2 * e->L;
    if (first_letters) {
        first_letters[0] = letter[e->found_key[0] & 3u];
        first_letters[1] = letter[(e->found_key[bit1 >> 6] >> (bit1 & 63)) & 3u];
    }
    if (explored) *explored = e->found_explored;
    return 1;
}

// copy the packed keys of the first min(cap, n_nodes) discovered nodes (discovery order)
int64_t acx_search_node_keys(void* h, uint64_t* out, int64_t cap) {
    Engine* e = static_cast<Engine*>(h);
    const int64_t n = e->n_set < cap ? e->n_set : cap;
    if (out && n > 0) std::memcpy(out, e->keys.data(), sizeof(uint64_t) * (size_t)n * e->kw);
    return e->n_set;
}

}  // extern "C"
