// acx_bfs.hip -- breadth-first search over the AC graph with the whole search on the GPU:
// FIFO queue, visited set (bucketed open-addressing hash table in HBM), 12-way expansion,
// dedup and budget accounting as kernels.  The host launches one round of kernels per chunk
// of parents and reads back a small control block.
//
// Reference: ac_solver/search/breadth_first.py:15-97.  Semantics kept exactly:
//   * the queue is processed parent by parent in FIFO order, actions 0..11 per parent;
//   * a child with total length 2 ends the search (checked before the visited test,
//     breadth_first.py:84-85), path = parent's path + (action, 2);
//   * a child is appended iff its state was never seen (breadth_first.py:87-89); within a
//     chunk "seen" includes earlier children (in (parent, action) order) of the same chunk;
//   * after each parent, len(tree_nodes) >= max_nodes ends the search (:91-95);
//   * an ACMove that empties a relator raises in the reference (utils.py:264-266): status
//     ACX_BFS_MOVE_ERROR when it happens before the search would have ended;
//   * min_length and the verbose "New minimal length found" sequence (:79-82) are the prefix
//     minima of the child totals in sequential order (bfs_close_kernel).
//
// Layout.  Child (g, a) -- move a of the g-th node in FIFO order -- has the global sequence
// number s = 12 g + a, its position in the reference's sequential order.  Every child key the
// expansion produces stays where it was written: the child store is laid out in tiles of 64
// parents (one wave), action-major inside a tile, so a wave writes each action's 64 keys as
// one contiguous run.  A node is named by its code (1 = root, s + 2 = child s); the FIFO queue
// holds codes, and a node's parent is queue[(code - 2) / 12] -- no compaction copy of keys, no
// parent / move arrays.  The visited set maps a state to the code of its first occurrence:
// entry = code << 24 | 24-bit fingerprint, buckets of 8 entries (one 64-B line per probe).
// Within a chunk the first occurrence wins by atomicMin on the entry (codes order as the
// reference does); the child whose entry is replaced is told so by the replacing child
// (`lost`), so survivors are known without re-reading the table.
//
// Kernels per chunk of P parents (FIFO indices [head, head + P)):
//   1. bfs_expand_kernel  block per tile: parent keys (via queue), 3 moves per lane (wave w:
//                         actions 3w..3w+2), child keys staged through LDS and written
//                         coalesced; first success / move-error seq, per-parent min child total;
//   2. bfs_insert_kernel  lane per child (up to the search's last child): probe / claim /
//                         join the state's table entry;
//   3. bfs_count_kernel   wave per tile: survivors per tile;
//   4. bfs_scan_kernel    exclusive scan of the tile counts;
//   5. bfs_commit_kernel  wave per tile: survivors' codes appended to the queue in (parent,
//                         action) order (LDS-staged, coalesced), the node-budget cut;
//   6. bfs_close_kernel   one block: the reference's decision for the chunk, the min_length
//                         trace, the next chunk's parameters (Live, on the device) and a copy
//                         of the state in pinned host memory.
// The host never sits between chunks: it keeps one chunk enqueued beyond the one whose outcome
// it is reading (grids sized for an upper bound, parameters read from Live), so a chunk's
// kernels follow the previous chunk's back to back (round 3: 10^7 nodes had 8 host round trips
// of ~20 us plus a D2H copy and a reset kernel per chunk, a quarter of the search's time).
// Cross-XCD visibility: every value a kernel compares against (child keys, queue codes) was
// written by an earlier kernel; within bfs_insert_kernel an entry only goes 0 -> one state's
// code -> a smaller code of the same state, so stale plain reads are harmless (a stale 0 is
// corrected by the CAS, a stale entry names the same state).
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

// visited-set sizing: the table has >= 100/ACX_BFS_TABLE_LOAD_PCT entries per bound entry (every
// node plus every claimed chunk entry), power of two; see acx_bfs_create
#ifndef ACX_BFS_TABLE_LOAD_PCT
#define ACX_BFS_TABLE_LOAD_PCT 50
#endif

namespace acx {
namespace bfs {

constexpr int TILE = 64;                // parents per tile (one wave)
constexpr int TILE_CH = 12 * TILE;      // children per tile
constexpr int BUCKET = 8;               // table entries per bucket (64 B)
constexpr int TRACE_CAP = 1024;         // new-minimum records per trace walk (<= 2L + 1 ever)
constexpr uint32_t FP_MASK = 0xffffffu;
// 8-entry table: entry = epoch << 58 | code << 24 | fp; codes < 12 (2^30 + 12) + 14 < 2^34.  An
// entry of another epoch (an earlier search on this workspace) is an empty slot, so a search
// does not clear the table (it did: a 512 MB memset per 10^7-node search); the table is
// cleared only when the 6-bit epoch wraps.
constexpr int EP_SHIFT = 58;
constexpr uint64_t CODE_MASK = (1ull << 34) - 1;

// store index (in keys) of the node with code c
__host__ __device__ __forceinline__ int64_t store_index(uint64_t c) {
    if (c <= 1) return 0;
    const uint64_t s = c - 2, g = s / 12, a = s - 12 * g;
    return 1 + (int64_t)((g >> 6) * TILE_CH + a * TILE + (g & 63));
}

struct Ctl {
    uint32_t succ;      // min chunk-local seq (12 p + a) of a child with n0 + n1 == 2
    uint32_t err;       // min chunk-local seq of a child whose move raised
    uint32_t cut_p;     // chunk-local parent after which len(tree_nodes) >= max_nodes
    uint32_t overflow;  // a probe walked the whole table (cannot happen at load <= 1/2)
    uint32_t min_len;   // min total over the chunk's (non-error) children
    uint32_t ntrace;    // trace walk: new minima recorded
    uint64_t total_new;     // nodes appended by the chunk
    uint64_t nodes_at_cut;  // len(tree_nodes) after parent cut_p
    uint32_t trace_min;     // trace walk: running minimum after the walk
    uint32_t pad;
};

// The search's state across chunks, kept on the device (bfs_close_kernel advances it), so the
// host can enqueue several chunks ahead without reading anything back; every chunk kernel takes
// its chunk's parameters from here and does nothing once `stop` is set.
struct Live {
    int64_t head;       // FIFO index of the next chunk's first parent
    int64_t n_nodes;    // len(tree_nodes)
    int64_t parents;    // parents the reference has expanded
    int64_t chunks;     // chunks run
    int64_t max_nodes, pmax;
    int64_t tile0;      // next chunk: head / 64
    int64_t succ_node, succ_act;
    int32_t P, ntiles;  // next chunk: parents, tiles
    uint32_t stop;      // the search has ended: later chunks do nothing
    int32_t status;     // ACX_BFS_* once stopped; -1 table overflow
    uint32_t running;   // min_length so far (breadth_first.py:79-82)
    uint32_t ntrace;    // "New minimal length" records so far
};

struct Args {
    Live* live;        // per-chunk parameters below are loaded from here (chunk_args)
    uint64_t* store;   // (scap, kw) node / child keys, store_index layout
    uint64_t* queue;   // (qcap) node codes in FIFO order
    uint8_t* cand;     // (ntiles * 768) child holds its state's entry after its own probe
    uint8_t* lost;     // (ntiles * 768) another child of the chunk replaced its entry (zeroed per chunk)
    uint16_t* pmin;    // (pmax) min child total per parent, 0xffff when every move raised
    uint32_t* tsum;    // (tiles) survivors per tile -> exclusive offsets
    uint32_t* tmin;    // (tiles) min child total per tile
    uint64_t* table;   // (buckets * 8) visited set
    Ctl* ctl;
    uint16_t* trace;   // (TRACE_CAP) the trace walk's new minima
    uint64_t bmask;    // buckets - 1
    int64_t head;      // FIFO index of the chunk's first parent
    int64_t tile0;     // head / 64
    int64_t n_before;  // len(tree_nodes) before the chunk
    int64_t need;      // max_nodes - n_before
    int64_t qcap;
    int P, L, kw, cyc, ntiles;
    int kt;            // key-in-table layout (bfs_insert_kt_kernel)
    uint64_t ep;       // this search's epoch << EP_SHIFT (8-entry table)
};

// this chunk's parameters from the device-side state; false once the search has ended (the
// chunk was enqueued speculatively and has nothing to do)
__device__ __forceinline__ bool chunk_args(Args& a) {
    const Live* lv = a.live;
    if (lv->stop) return false;
    a.head = lv->head;
    a.P = lv->P;
    a.tile0 = lv->tile0;
    a.ntiles = lv->ntiles;
    a.n_before = lv->n_nodes;
    a.need = lv->max_nodes - lv->n_nodes;
    return true;
}

// (1) expand: one block per tile of 64 parents; wave w makes the children of actions 3w..3w+2
// (4x the lanes of a lane-per-parent loop: the move chain is latency-bound, and a 2^19-parent
// chunk is only ~8 waves per SIMD that way); keys staged through LDS, written coalesced
constexpr int APW = 12 / (TPB / WAVE);  // actions per wave (3)
template <int NW>
__global__ __launch_bounds__(TPB, NW <= 4 ? 8 : 4) void bfs_expand_kernel(Args a) {
    __shared__ uint64_t kst[TPB / WAVE][TILE * (NW + 1)];
    __shared__ uint32_t smin[TILE];
    if (!chunk_args(a)) return;
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    const int t = blockIdx.x;  // one tile per block (the grid is an upper bound on the tiles)
    if (t >= a.ntiles) return;
    const int64_t gt = (a.tile0 + t) * TILE;  // FIFO index of the tile's parent 0
    const int64_t g = gt + lane;
    const bool active = g >= a.head && g < a.head + a.P;
    const bool full = __ballot(active) == ~0ull;
    const int kw = a.kw;
    if (wid == 0) smin[lane] = 0xffffu;
    PresRegs<NW> pr;
    bool clean = false;
    if (active) {
        load_key<NW>(a.store + store_index(a.queue[g]) * kw, kw, a.L, pr);
        clean = is_clean<NW>(pr.w0, pr.n0, pr.w1, pr.n1, a.cyc != 0);
    }
    __syncthreads();
    const uint32_t p = (uint32_t)(g - a.head);
    uint32_t succ = NONE, err = NONE, mn = 0xffffu;
    uint64_t* out = a.store + (1 + (a.tile0 + t) * TILE_CH) * kw;
    uint64_t* st = kst[wid];
#pragma unroll 1
    for (int j = 0; j < APW; ++j) {
        const int act = wid * APW + j;
        if (active) {
            PresRegs<NW> q = pr;
            const int e = clean ? ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, a.cyc != 0)
                                : ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, a.cyc != 0);
            const uint32_t s = p * 12u + (uint32_t)act;
            if (e != ACX_ERR_NONE) {
                err = min(err, s);
            } else {
                const uint32_t tot = (uint32_t)(q.n0 + q.n1);
                if (tot == 2) succ = min(succ, s);
                mn = min(mn, tot);
            }
            uint64_t key[NW + 1];
            make_key<NW>(a.L, q, key);
#pragma unroll
            for (int k = 0; k < NW + 1; ++k)
                if (k < kw) st[lane * kw + k] = key[k];
        }
        wsync();
        uint64_t* o = out + (int64_t)act * TILE * kw;
        if (full) {
            for (int i = lane; i < TILE * kw; i += WAVE) o[i] = st[i];
        } else {  // a tile at a chunk edge: the other chunk's parents' slots are not ours
            for (int i = lane; i < TILE * kw; i += WAVE) {
                const int64_t gi = gt + i / kw;
                if (gi >= a.head && gi < a.head + a.P) o[i] = st[i];
            }
        }
        wsync();
    }
    if (active) atomicMin(&smin[lane], mn);
    // success / move error are rare: one global atomic per wave that has one; the chunk's min
    // child total goes through a per-tile value the scan kernel reduces (a same-address atomic
    // from every wave of a chunk serialises: 4x the waves made it cost 90 us per chunk)
    succ = wave_min(succ);
    err = wave_min(err);
    if (lane == 0) {
        if (succ != NONE) atomicMin(&a.ctl->succ, succ);
        if (err != NONE) atomicMin(&a.ctl->err, err);
    }
    __syncthreads();
    if (wid == 0) {
        const uint32_t m = smin[lane];
        if (active) a.pmin[p] = (uint16_t)m;
        const uint32_t tm = wave_min(m);
        if (lane == 0) a.tmin[t] = tm;
    }
}

// chunk-local position (in cand / lost) of the child with code c of this chunk
__device__ __forceinline__ int64_t local_pos(const Args& a, uint64_t c) {
    const uint64_t s = c - 2, g = s / 12, act = s - 12 * g;
    return (int64_t)(((int64_t)(g >> 6) - a.tile0) * TILE_CH + act * TILE + (g & 63));
}

// Key-in-table layout (L <= KT_MAX_L: the 4L + 16 key bits fit 3 x 63): an entry is 4 words,
// [code << 24 | fp, g0, g1, g2], two entries per 64-B bucket; g_j = (bits [63j, 63j + 63) of the
// key) << 1 | 1.  The claimer CASes the first word, then stores g0..g2, so a reader sees each g_j
// either as written (guard bit 1: the entry's state's key bits, exactly) or still 0: an entry
// whose three guards are set decides equality from the bucket line alone; otherwise the state's
// key is read from the store, as in the 8-entry layout.
constexpr int KT_MAX_L = 43;
constexpr int KT_ENT = 4;  // words per entry
__host__ __device__ __forceinline__ void kt_guarded(const uint64_t* k, int kw, uint64_t (&g)[3]) {
    const uint64_t k0 = k[0], k1 = kw > 1 ? k[1] : 0ull, k2 = kw > 2 ? k[2] : 0ull;
    const uint64_t M = (1ull << 63) - 1;
    g[0] = ((k0 & M) << 1) | 1ull;
    g[1] = ((((k0 >> 63) | (k1 << 1)) & M) << 1) | 1ull;
    g[2] = (((k1 >> 62) | (k2 << 2)) << 1) | 1ull;
}

// (2') key-in-table insert: a duplicate of a committed node costs one random line (its bucket)
template <int KWM>
__global__ __launch_bounds__(TPB, 8) void bfs_insert_kt_kernel(Args a) {
    if (!chunk_args(a)) return;
    const int64_t c = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (c >= (int64_t)a.ntiles * TILE_CH) return;
    const int t = (int)(c / TILE_CH);
    const int r = (int)(c - (int64_t)t * TILE_CH);
    const int act = r / TILE, lane = r - act * TILE;
    const int64_t g = (a.tile0 + t) * TILE + lane;
    uint8_t res = 0;
    if (g >= a.head && g < a.head + a.P) {
        const uint32_t s = (uint32_t)(g - a.head) * 12u + (uint32_t)act;
        const uint32_t end = min(a.ctl->succ, a.ctl->err);
        if (s < end) {
            const int kw = a.kw;
            const uint64_t code = (uint64_t)g * 12 + act + 2;
            const Key<KWM> key = kload<KWM>(a.store + (1 + (a.tile0 + t) * TILE_CH + r) * kw, kw);
            const uint64_t h = khash<KWM>(key, kw);
            const uint32_t fp = (uint32_t)(h >> 40);
            const uint64_t my = (code << 24) | fp;
            uint64_t gd[3];
            kt_guarded(key.w, kw, gd);
            uint64_t b = h & a.bmask;
            for (uint64_t it = 0;; ++it) {
                if (it > a.bmask) {
                    atomicOr(&a.ctl->overflow, 1u);
                    break;
                }
                uint64_t* bk = a.table + b * BUCKET;
                uint64_t e[BUCKET];
#pragma unroll
                for (int j = 0; j < BUCKET; j += 2) {
                    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(bk + j);
                    e[j] = v.x;
                    e[j + 1] = v.y;
                }
                int done = 0;  // 1 seen / lost, 2 holds the entry
#pragma unroll
                for (int j = 0; j < BUCKET / KT_ENT && !done; ++j) {
                    uint64_t* ent = bk + KT_ENT * j;
                    uint64_t v = e[KT_ENT * j];
                    bool fresh = true;  // e[] holds this entry's words as read with v
                    if (v == 0) {
                        const uint64_t old = atomicCAS((unsigned long long*)ent, 0ull, (unsigned long long)my);
                        if (old == 0) {
                            ent[1] = gd[0];
                            ent[2] = gd[1];
                            ent[3] = gd[2];
                            done = 2;
                            break;
                        }
                        v = old;
                        fresh = false;
                    }
                    if (((uint32_t)v & FP_MASK) != fp) continue;
                    const uint64_t e1 = e[KT_ENT * j + 1], e2 = e[KT_ENT * j + 2], e3 = e[KT_ENT * j + 3];
                    bool eq;
                    if (fresh && (e1 & e2 & e3 & 1ull)) eq = e1 == gd[0] && e2 == gd[1] && e3 == gd[2];
                    else eq = keq<KWM>(a.store + store_index(v >> 24) * kw, key, kw);
                    if (!eq) continue;
                    const uint64_t vc = v >> 24;
                    if (vc < code) {
                        done = 1;
                        break;
                    }
                    const uint64_t old = atomicMin((unsigned long long*)ent, (unsigned long long)my);
                    if (old < my) {
                        done = 1;
                    } else {
                        a.lost[local_pos(a, old >> 24)] = 1;
                        done = 2;
                    }
                }
                if (done) {
                    res = done == 2;
                    break;
                }
                b = (b + 1) & a.bmask;
            }
        }
    }
    a.cand[c] = res;
}

// (2) lane per child: probe the visited set; claim an empty slot or join the state's entry
template <int KWM>
__global__ __launch_bounds__(TPB, 8) void bfs_insert_kernel(Args a) {  // 8 waves/SIMD: latency-bound, SGPRs capped at 96
    if (!chunk_args(a)) return;
    const int64_t c = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (c >= (int64_t)a.ntiles * TILE_CH) return;
    const int t = (int)(c / TILE_CH);
    const int r = (int)(c - (int64_t)t * TILE_CH);
    const int act = r / TILE, lane = r - act * TILE;
    const int64_t g = (a.tile0 + t) * TILE + lane;
    uint8_t res = 0;
    if (g >= a.head && g < a.head + a.P) {
        const uint32_t s = (uint32_t)(g - a.head) * 12u + (uint32_t)act;
        const uint32_t end = min(a.ctl->succ, a.ctl->err);  // the success / raising child ends the search
        if (s < end) {
            const int kw = a.kw;
            const uint64_t code = (uint64_t)g * 12 + act + 2;
            const Key<KWM> key = kload<KWM>(a.store + (1 + (a.tile0 + t) * TILE_CH + r) * kw, kw);
            const uint64_t h = khash<KWM>(key, kw);
            const uint32_t fp = (uint32_t)(h >> 40);
            const uint64_t my = a.ep | (code << 24) | fp;
            uint64_t b = h & a.bmask;
            for (uint64_t it = 0;; ++it) {
                if (it > a.bmask) {
                    atomicOr(&a.ctl->overflow, 1u);
                    break;
                }
                uint64_t* bk = a.table + b * BUCKET;
                uint64_t e[BUCKET];
#pragma unroll
                for (int j = 0; j < BUCKET; j += 2) {
                    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(bk + j);
                    e[j] = v.x;
                    e[j + 1] = v.y;
                }
                int done = 0;  // 1 seen / lost, 2 holds the entry
#pragma unroll
                for (int j = 0; j < BUCKET && !done; ++j) {
                    uint64_t v = e[j];
                    if ((v >> EP_SHIFT) != (a.ep >> EP_SHIFT)) {  // empty in this search
                        const uint64_t old = atomicCAS((unsigned long long*)(bk + j), (unsigned long long)v,
                                                       (unsigned long long)my);
                        if (old == v) {
                            done = 2;
                            break;
                        }
                        v = old;  // claimed meanwhile: a value of this search
                    }
                    if (((uint32_t)v & FP_MASK) != fp) continue;
                    const uint64_t vc = (v >> 24) & CODE_MASK;
                    if (!keq<KWM>(a.store + store_index(vc) * kw, key, kw)) continue;
                    if (vc < code) {  // an earlier occurrence (a node, or an earlier child of the chunk)
                        done = 1;
                        break;
                    }
                    const uint64_t old = atomicMin((unsigned long long*)(bk + j), (unsigned long long)my);
                    if (old < my) {
                        done = 1;
                    } else {  // replaced a later child of the chunk: it learns it lost
                        a.lost[local_pos(a, (old >> 24) & CODE_MASK)] = 1;
                        done = 2;
                    }
                }
                if (done) {
                    res = done == 2;
                    break;
                }
                b = (b + 1) & a.bmask;
            }
        }
    }
    a.cand[c] = res;
}

// survivor mask of this lane's parent (bit a: child (g, a) is appended)
__device__ __forceinline__ uint32_t survivors(const Args& a, int t, int lane, bool clear) {
    uint32_t m = 0;
    const int64_t base = (int64_t)t * TILE_CH + lane;
#pragma unroll
    for (int act = 0; act < 12; ++act) {
        const int64_t c = base + act * TILE;
        const bool lo = a.lost[c] != 0;
        if (a.cand[c] && !lo) m |= 1u << act;
        if (clear && lo) a.lost[c] = 0;
    }
    return m;
}

// (3) survivors per tile
__global__ __launch_bounds__(TPB) void bfs_count_kernel(Args a) {
    if (!chunk_args(a)) return;
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    const int t = blockIdx.x * (TPB / WAVE) + wid;
    if (t >= a.ntiles) return;
    const uint32_t n = wave_sum(__popc(survivors(a, t, lane, false)));
    if (lane == 0) a.tsum[t] = n;
}

// (4) exclusive scan of the tile counts (one block of 1024 threads)
__global__ __launch_bounds__(1024) void bfs_scan_kernel(Args a) {
    __shared__ uint32_t sh[1024 / WAVE];
    if (!chunk_args(a)) return;
    const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
    const int nb = a.ntiles;
    const int per = (nb + 1023) / 1024;
    const int b0 = t * per, b1 = min(nb, b0 + per);
    uint32_t loc = 0, mn = 0xffffffffu;
    for (int i = b0; i < b1; ++i) {
        loc += a.tsum[i];
        mn = min(mn, a.tmin[i]);
    }
    mn = wave_min(mn);
    if (lane == 0) atomicMin(&a.ctl->min_len, mn);  // 16 per chunk
    uint32_t x = loc;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
    }
    if (lane == WAVE - 1) sh[wid] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < 1024 / WAVE; ++i) {
        off += i < wid ? sh[i] : 0u;
        tot += sh[i];
    }
    uint32_t run = off + x - loc;
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = a.tsum[i];
        a.tsum[i] = run;
        run += c;
    }
    if (t == 0) a.ctl->total_new = tot;
}

// (5) append the survivors' codes in (parent, action) order; the node-budget cut
__global__ __launch_bounds__(TPB) void bfs_commit_kernel(Args a) {
    __shared__ uint64_t stage[TPB / WAVE][TILE_CH];
    if (!chunk_args(a)) return;
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    const int t = blockIdx.x * (TPB / WAVE) + wid;
    if (t >= a.ntiles) return;
    const int64_t g = (a.tile0 + t) * TILE + lane;
    const bool active = g >= a.head && g < a.head + a.P;
    const uint32_t m = survivors(a, t, lane, true);  // (0 for inactive lanes: cand is 0)
    const uint32_t c = __popc(m);
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
    }
    const uint32_t excl = x - c;
    const uint32_t wtot = __shfl(x, WAVE - 1, WAVE);
    const int64_t base = (int64_t)a.tsum[t] + excl;  // survivors of the chunk before this parent
    if (active) {
        // cut = first parent with n_before + (nodes appended through it) >= max_nodes
        const int64_t incl = base + c;
        const int64_t p = g - a.head;
        if (incl >= a.need && (base < a.need || p == 0)) {
            a.ctl->cut_p = (uint32_t)p;
            a.ctl->nodes_at_cut = (uint64_t)(a.n_before + incl);
        }
    }
    uint64_t* st = stage[wid];
    uint32_t mm = m, k = excl;
    while (mm) {
        const int act = __builtin_ctz(mm);
        mm &= mm - 1;
        st[k++] = (uint64_t)g * 12 + act + 2;
    }
    wsync();
    const int64_t n0 = a.n_before + a.tsum[t];
    for (uint32_t i = lane; i < wtot; i += WAVE)
        if (n0 + i < a.qcap) a.queue[n0 + i] = st[i];
}

// the root's packed key, passed by value (no host-to-device copy of host memory per search)
struct RootKey {
    uint64_t w[ACX_MAX_L / 16 + 2];
};

// root: node 0 (code 1), its key in the store and its table entry
template <int KWM>
__global__ void bfs_root_kernel(Args a, RootKey rk) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int k = 0; k < a.kw; ++k) a.store[k] = rk.w[k];
    const Key<KWM> key = kload<KWM>(a.store, a.kw);
    const uint64_t h = khash<KWM>(key, a.kw);
    uint64_t* ent = a.table + (h & a.bmask) * BUCKET;
    ent[0] = a.ep | (1ull << 24) | (uint32_t)(h >> 40);  // (a.ep is 0 in the key-in-table layout)
    if (a.kt) {
        uint64_t gd[3];
        kt_guarded(key.w, a.kw, gd);
        ent[1] = gd[0];
        ent[2] = gd[1];
        ent[3] = gd[2];
    }
    a.queue[0] = 1;
}

// the control block to its initial values (before each chunk)
__device__ __forceinline__ void ctl_reset(Ctl* c) {
    Ctl z;
    memset(&z, 0, sizeof(z));
    z.succ = z.err = z.cut_p = z.min_len = NONE;
    *c = z;
}

// the search's state before its first chunk (one thread)
__global__ void bfs_init_kernel(Args a, int64_t max_nodes, int64_t pmax, uint32_t total0) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    Live* lv = a.live;
    Live z;
    memset(&z, 0, sizeof(z));
    z.n_nodes = 1;
    z.max_nodes = max_nodes;
    z.pmax = pmax;
    z.P = 1;
    z.ntiles = 1;
    z.status = ACX_BFS_EXHAUSTED;
    z.running = total0;
    *lv = z;
    ctl_reset(a.ctl);
}

// what the host reads after each chunk (pinned host memory, one slot per chunk in flight)
struct LiveMirror {
    Live s;
    uint64_t seq;  // chunk number + 1 once the slot holds that chunk's state
};
constexpr int RING = 4;

// (6) close the chunk (one block, after commit), in the reference's order: a raising child
// before the first success and not after the budget cut -> AssertionError; else a success not
// after the cut -> the path; else the cut -> the budget message; else the next chunk; an empty
// queue -> (False, None).  Then min_length: when the chunk's minimum child total beats the
// running minimum, the parents whose minimum does are found with a prefix-min scan and walked
// move by move, appending the reference's "New minimal length found" values
// (breadth_first.py:79-82).  Then the state for the next chunk, the control block reset, and
// the state published to the host's slot for chunk `k` (also when the search had already ended
// before this speculatively enqueued chunk).
template <int NW>
__global__ __launch_bounds__(256) void bfs_close_kernel(Args a, int64_t k, LiveMirror* mirror, uint16_t* trace_host) {
    __shared__ uint32_t lmin[256];
    __shared__ uint32_t list[TRACE_CAP];
    __shared__ uint32_t nlist, s_end, s_trace;
    const int t = threadIdx.x;
    Live* lv = a.live;
    const bool run = chunk_args(a);
    bool ends = false, err_first = false, succ_first = false;
    int64_t cut = INT64_MAX, err_p = INT64_MAX, suc_p = INT64_MAX;
    Ctl c;
    if (run && t == 0) {
        c = *a.ctl;
        cut = c.cut_p == NONE ? INT64_MAX : (int64_t)c.cut_p;
        err_p = c.err == NONE ? INT64_MAX : (int64_t)(c.err / 12);
        suc_p = c.succ == NONE ? INT64_MAX : (int64_t)(c.succ / 12);
        err_first = c.err != NONE && c.err < c.succ && err_p <= cut;
        succ_first = !err_first && c.succ != NONE && suc_p <= cut;
        ends = err_first || succ_first || cut != INT64_MAX;
        // children the reference looks at in this chunk, in order: up to and including the
        // success child, up to (not including) the raising child, through the cut parent
        s_end = err_first ? c.err : succ_first ? c.succ + 1 : cut != INT64_MAX ? (uint32_t)((cut + 1) * 12)
                                                                                : (uint32_t)a.P * 12u;
        s_trace = !c.overflow && c.min_len < lv->running;
        nlist = 0;
    }
    __syncthreads();
    if (run && s_trace) {
        const uint32_t end = s_end, running = lv->running;
        const int64_t np = ((int64_t)end + 11) / 12;  // parents with children before `end`
        const int64_t per = (np + 255) / 256;
        const int64_t p0 = t * per, p1 = min<int64_t>(np, p0 + per);
        uint32_t m = 0xffffffffu;
        for (int64_t p = p0; p < p1; ++p) m = min(m, (uint32_t)a.pmin[p]);
        lmin[t] = m;
        __syncthreads();
        uint32_t r = running;
        for (int i = 0; i < t; ++i) r = min(r, lmin[i]);
        for (int64_t p = p0; p < p1; ++p) {
            const uint32_t v = a.pmin[p];
            if (v < r) {
                const uint32_t q = atomicAdd(&nlist, 1u);
                if (q < TRACE_CAP) list[q] = (uint32_t)p;
                r = v;
            }
        }
        __syncthreads();
        if (t == 0) {
            const uint32_t n = min(nlist, (uint32_t)TRACE_CAP);
            for (uint32_t i = 1; i < n; ++i) {  // insertion sort: the parents in order (few)
                const uint32_t v = list[i];
                uint32_t j = i;
                for (; j > 0 && list[j - 1] > v; --j) list[j] = list[j - 1];
                list[j] = v;
            }
            uint32_t cur = running, nt = lv->ntrace;
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t p = list[i];
                PresRegs<NW> pr;
                load_key<NW>(a.store + store_index(a.queue[a.head + p]) * a.kw, a.kw, a.L, pr);
                for (int act = 0; act < 12 && p * 12u + act < end; ++act) {
                    PresRegs<NW> q = pr;
                    if (ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, a.cyc != 0) != ACX_ERR_NONE) continue;
                    const uint32_t tot = (uint32_t)(q.n0 + q.n1);
                    if (tot < cur) {
                        cur = tot;
                        if (nt < TRACE_CAP) trace_host[nt] = (uint16_t)tot;  // pinned host memory
                        ++nt;
                    }
                }
            }
            lv->ntrace = nt;
            lv->running = cur;
        }
    }
    if (t != 0) return;
    if (run) {
        if (c.overflow) {
            lv->status = -1;
            lv->stop = 1;
        } else if (ends) {
            const int64_t last = err_first ? err_p : succ_first ? suc_p : cut;
            lv->parents += last + 1;
            if (err_first) {
                lv->status = ACX_BFS_MOVE_ERROR;
            } else if (succ_first) {
                lv->status = ACX_BFS_FOUND;
                lv->succ_node = a.head + suc_p;
                lv->succ_act = c.succ % 12;
            } else {
                lv->status = ACX_BFS_BUDGET;
                lv->n_nodes = (int64_t)c.nodes_at_cut;
            }
            lv->stop = 1;
        } else {
            lv->parents += a.P;
            lv->n_nodes += (int64_t)c.total_new;
            lv->head += a.P;
            if (lv->head >= lv->n_nodes) {  // the queue ran dry: (False, None)
                lv->status = ACX_BFS_EXHAUSTED;
                lv->stop = 1;
            } else {
                const int64_t avail = lv->n_nodes - lv->head;
                lv->P = (int32_t)(avail < lv->pmax ? avail : lv->pmax);
                lv->tile0 = lv->head / TILE;
                lv->ntiles = (int32_t)((lv->head + lv->P - 1) / TILE - lv->tile0 + 1);
            }
        }
        lv->chunks += 1;
        ctl_reset(a.ctl);
    }
    LiveMirror* m = mirror + (k % RING);
    m->s = *lv;
    __threadfence_system();
    __hip_atomic_store(&m->seq, (uint64_t)(k + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// path root -> node (FIFO index v): (action, total length) per edge into out[0..2*depth)
template <int NW>
__global__ void bfs_path_kernel(Args a, int64_t v, int32_t* out, int64_t cap, int64_t* out_n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t d = 0;
    for (uint64_t c = a.queue[v]; c > 1; c = a.queue[(c - 2) / 12]) ++d;
    *out_n = d;
    if (d > cap) return;
    int64_t i = d;
    for (uint64_t c = a.queue[v]; c > 1; c = a.queue[(c - 2) / 12]) {
        PresRegs<NW> pr;
        load_key<NW>(a.store + store_index(c) * a.kw, a.kw, a.L, pr);
        --i;
        out[2 * i] = (int32_t)((c - 2) % 12);
        out[2 * i + 1] = pr.n0 + pr.n1;
    }
}

// keys of FIFO nodes [0, n) -> out (n, kw)
__global__ __launch_bounds__(TPB) void bfs_gather_kernel(Args a, int64_t n, uint64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const uint64_t* src = a.store + store_index(a.queue[i]) * a.kw;
    for (int k = 0; k < a.kw; ++k) out[i * a.kw + k] = src[k];
}

struct Search {
    int dev = 0, L = 0, kw = 0, cyc = 0;
    int64_t max_nodes = 0, qcap = 0, pmax = 0, scap = 0, tiles_max = 0;
    int64_t last_nodes = 0;  // len(tree_nodes) at the end of the last run (<= qcap)
    uint64_t tsize = 0;
    Args a{};
    LiveMirror* mirror = nullptr;  // pinned host memory, RING slots (bfs_close_kernel publishes)
    hipEvent_t fin = nullptr;      // after a search's last (speculative) chunk: the next search
                                   // and the destructor wait for it (any stream)
    bool fin_pending = false;
    int64_t kbase = 0;             // chunks enqueued by earlier searches
    int epoch = 0;                 // 8-entry table: the last search's epoch (0: table all zero)
    uint16_t* trace_host = nullptr;
    int32_t* path_dev = nullptr;    // pinned, coherent host memory: bfs_path_kernel writes the path
    int64_t* path_n_dev = nullptr;  // there directly (no device-to-host copy)
    std::vector<int32_t> trace;  // new minima of the last run, in order
    uint64_t* gather = nullptr;  // acx_bfs_node_keys: the keys in FIFO order (grown on demand)
    int64_t gather_cap = 0;
    void* bounce = nullptr;      // pinned (copy_to_host)

    ~Search() {
        if (fin_pending) (void)hipEventSynchronize(fin);
        void* ptrs[] = {a.store, a.queue, a.cand, a.lost, a.pmin, a.tsum, a.tmin, a.table, a.ctl, a.trace, a.live};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        if (gather) (void)hipFree(gather);
        void* hptrs[] = {mirror, trace_host, path_dev, path_n_dev, bounce};
        for (void* p : hptrs)
            if (p) (void)hipHostFree(p);
        if (fin) (void)hipEventDestroy(fin);
    }
};

static constexpr int64_t PATH_CAP = 1 << 16;
// a chunk (<= 2^20 parents, ~0.15 ms) that has not published its state after this long is a
// kernel that does not finish: acx_bfs_run returns ACX_E_LAUNCH instead of polling forever
#ifndef ACX_BFS_CHUNK_DEADLINE_S
#define ACX_BFS_CHUNK_DEADLINE_S 30.0
#endif
static constexpr int ACX_E_TIMEOUT = -100;  // internal to acx_bfs_run (returned as ACX_E_LAUNCH)
static int g_bfs_layout = 0;  // 0 default (8-entry table), 2 key-in-table where L allows (tests, A/B)

template <class T>
static bool dalloc(T*& p, size_t n) {
    return hipMalloc((void**)&p, n * sizeof(T) + 64) == hipSuccess;
}

// launches of one chunk (number k), templated on the key-word bound; the grids cover `ntiles`
// tiles, an upper bound on the chunk's real tile count (the kernels read the real one, Live)
struct ChunkLaunch {
    Search* S;
    hipStream_t st;
    int64_t k;
    int ntiles;
    template <int NW>
    void go() {
        Args& a = S->a;
        const unsigned wb = (unsigned)((ntiles + TPB / WAVE - 1) / (TPB / WAVE));
        const int64_t nc = (int64_t)ntiles * TILE_CH;
        bfs_expand_kernel<NW><<<dim3((unsigned)ntiles), dim3(TPB), 0, st>>>(a);
        bool kt_done = false;
        if constexpr (NW <= 3) {  // L <= KT_MAX_L
            if (a.kt) {
                bfs_insert_kt_kernel<NW + 1><<<dim3((unsigned)((nc + TPB - 1) / TPB)), dim3(TPB), 0, st>>>(a);
                kt_done = true;
            }
        }
        if (!kt_done) bfs_insert_kernel<NW + 1><<<dim3((unsigned)((nc + TPB - 1) / TPB)), dim3(TPB), 0, st>>>(a);
        bfs_count_kernel<<<dim3(wb), dim3(TPB), 0, st>>>(a);
        bfs_scan_kernel<<<dim3(1), dim3(1024), 0, st>>>(a);
        bfs_commit_kernel<<<dim3(wb), dim3(TPB), 0, st>>>(a);
        bfs_close_kernel<NW><<<dim3(1), dim3(256), 0, st>>>(a, k, S->mirror, S->trace_host);
    }
};
struct RootLaunch {
    Search* S;
    hipStream_t st;
    RootKey rk;
    template <int NW>
    void go() { bfs_root_kernel<NW + 1><<<dim3(1), dim3(64), 0, st>>>(S->a, rk); }
};
struct PathLaunch {
    Search* S;
    hipStream_t st;
    int64_t node;
    template <int NW>
    void go() { bfs_path_kernel<NW><<<dim3(1), dim3(64), 0, st>>>(S->a, node, S->path_dev, PATH_CAP, S->path_n_dev); }
};
}  // namespace bfs
}  // namespace acx

using namespace acx::bfs;

extern "C" {

void* acx_bfs_create(int32_t L, int64_t max_nodes, int64_t chunk_parents, int32_t cyclical) {
    if (L < 1 || L > ACX_MAX_L || max_nodes < 1 || max_nodes > (1ll << 30)) return nullptr;
    Search* S = new (std::nothrow) Search();
    if (!S) return nullptr;
    if (hipGetDevice(&S->dev) != hipSuccess) { delete S; return nullptr; }
    S->L = L;
    S->kw = acx_key_words(L);
    S->cyc = cyclical != 0;
    S->max_nodes = max_nodes;
    S->qcap = max_nodes + 12;
    if (chunk_parents <= 0) chunk_parents = 1 << 20;  // tools/bfs_chunk_probe.py (r02ak): 2^20 fastest at 10^7 / 10^8 nodes
    S->pmax = chunk_parents < S->qcap ? chunk_parents : S->qcap;
    S->tiles_max = S->pmax / TILE + 2;
    // every parent that can be expanded (< qcap) has its 12 child slots; one spare tile
    S->scap = 1 + ((S->qcap + TILE - 1) / TILE + 1) * TILE_CH;
    // every node and every claimed chunk entry at load <= 1/2, buckets of 8 (one 64-B line per
    // probe).  Other sizes, A/B on the final pipeline (profiles/r03/r03x_bfs_table_load.json):
    // half the entries 1.52 vs 1.47 ms at 10^7 and (load <= 1) 16.0 vs 13.7 ms at 10^8; twice
    // the entries within 1 % at 10^7 and 14.5 vs 13.4 ms at 10^8.
    // Key-in-table (L <= KT_MAX_L, opt-in): 4 words per entry, entries >= 1.25x the same bound
    // (2 per bucket; the bound counts a whole last chunk's children as new: the real load stays
    // lower).  Measured slower than the 8-entry table (r03i: 2.11 vs 1.68 ms at 10^7 nodes, 20.0
    // vs 14.2 ms at 10^8): the saved node-key reads cost less than the table's doubled footprint.
    const bool kt = L <= KT_MAX_L && g_bfs_layout == 2;
    uint64_t ts = 1024;
    const uint64_t bound = (uint64_t)(S->qcap + 12 * S->pmax);
    while (kt ? ts < 5 * bound : ts * ACX_BFS_TABLE_LOAD_PCT < 100 * bound) ts <<= 1;
    S->tsize = ts;
    Args& a = S->a;
    bool ok = dalloc(a.store, (size_t)(S->scap * S->kw)) && dalloc(a.queue, (size_t)S->qcap) &&
              dalloc(a.cand, (size_t)(S->tiles_max * TILE_CH)) && dalloc(a.lost, (size_t)(S->tiles_max * TILE_CH)) &&
              dalloc(a.pmin, (size_t)S->pmax) && dalloc(a.tsum, (size_t)S->tiles_max) &&
              dalloc(a.tmin, (size_t)S->tiles_max) && dalloc(a.table, (size_t)ts) &&
              dalloc(a.ctl, 1) && dalloc(a.trace, (size_t)TRACE_CAP) && dalloc(a.live, 1) &&
              hipHostMalloc((void**)&S->path_dev, sizeof(int32_t) * 2 * PATH_CAP, hipHostMallocCoherent) == hipSuccess &&
              hipHostMalloc((void**)&S->path_n_dev, sizeof(int64_t), hipHostMallocCoherent) == hipSuccess &&
              hipHostMalloc((void**)&S->mirror, sizeof(LiveMirror) * RING, hipHostMallocCoherent) == hipSuccess &&
              hipHostMalloc((void**)&S->trace_host, sizeof(uint16_t) * TRACE_CAP, hipHostMallocCoherent) == hipSuccess &&
              hipMemset(a.lost, 0, (size_t)(S->tiles_max * TILE_CH)) == hipSuccess &&
              hipMemset(a.table, 0, (size_t)ts * 8) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&S->fin, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        delete S;
        return nullptr;
    }
    a.bmask = ts / BUCKET - 1;
    a.kt = kt ? 1 : 0;
    a.qcap = S->qcap;
    a.L = L;
    a.kw = S->kw;
    a.cyc = S->cyc;
    return S;
}

// test / A-B hook: 2 selects the key-in-table layout (L <= 43) for searches created afterwards,
// 0 the default 8-entry table
void acx_internal_bfs_layout(int32_t layout) { g_bfs_layout = layout; }

void acx_bfs_destroy(void* h) { delete static_cast<Search*>(h); }

int acx_bfs_run(void* h, const int32_t* presentation, int64_t max_nodes, int32_t* path_actions,
                int32_t* path_totals, int64_t path_cap, int64_t* stats, void* stream) {
    Search* S = static_cast<Search*>(h);
    if (!S || !presentation || !stats) return ACX_E_ARG;
    if (max_nodes < 1 || max_nodes > S->max_nodes) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    Args& a = S->a;
    const int L = S->L, kw = S->kw;
    RootLaunch rl{S, st, {}};
    pack_key(presentation, L, kw, rl.rk.w);
    int total0 = 0;
    for (int i = 0; i < 2 * L; ++i) total0 += presentation[i] != 0;

    // a previous search that ended on an error may have left work in flight (on another stream, too)
    if (S->fin_pending) {
        if (hipStreamWaitEvent(st, S->fin, 0) != hipSuccess) return ACX_E_LAUNCH;
        S->fin_pending = false;
    }
    if (a.kt) {  // key-in-table entries have no epoch: cleared per search
        if (hipMemsetAsync(a.table, 0, S->tsize * 8, st) != hipSuccess) return ACX_E_LAUNCH;
        a.ep = 0;
    } else {
        if (++S->epoch == 64) {  // the epoch wraps: clear once every 63 searches
            if (hipMemsetAsync(a.table, 0, S->tsize * 8, st) != hipSuccess) return ACX_E_LAUNCH;
            S->epoch = 1;
        }
        a.ep = (uint64_t)S->epoch << EP_SHIFT;
    }
    by_nw(L, rl);
    bfs_init_kernel<<<dim3(1), dim3(64), 0, st>>>(a, max_nodes, S->pmax, (uint32_t)total0);

    // Chunks are enqueued one ahead of the one the host waits for: chunk k + 1 is in the stream
    // before the host reads chunk k's outcome, so no chunk waits for a host round trip.  Its
    // grids are sized for an upper bound on its parents -- after chunk k the queue holds at most
    // avail_k - P_k + 12 P_k unexpanded nodes -- and its kernels take the real parameters from
    // the device state; once the search has ended they do nothing.
    S->trace.clear();
    // chunk numbers run on across searches (S->kbase), so a slot never holds a stale match
    int64_t enqueued = 0;  // chunk numbers this search has used
    auto enqueue = [&](int64_t k, int64_t avail_ub) -> int {
        const int64_t pub = avail_ub < S->pmax ? avail_ub : S->pmax;
        ChunkLaunch cl{S, st, S->kbase + k, (int)((pub - 1) / TILE + 2)};
        by_nw(L, cl);
        enqueued = k + 1;
        return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
    };
    // poll the slot's sequence number (written last, system scope, by the chunk's close kernel);
    // no per-chunk event (an event marker held the next chunk back ~5 us).  Every 4096 polls
    // the stream is queried so that a failed launch cannot leave the host spinning, and a chunk
    // that has not published within ACX_BFS_CHUNK_DEADLINE_S seconds (a hung kernel) is an error.
    auto wait_chunk = [&](int64_t k) -> int {
        const int64_t K = S->kbase + k;
        const uint64_t* seq = &S->mirror[K % RING].seq;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t it = 1;; ++it) {
            if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) == (uint64_t)(K + 1)) return ACX_OK;
            if ((it & 4095) == 0) {
                const hipError_t e = hipStreamQuery(st);
                if (e == hipSuccess)  // idle: the slot is final now
                    return __atomic_load_n(seq, __ATOMIC_ACQUIRE) == (uint64_t)(K + 1) ? ACX_OK : ACX_E_LAUNCH;
                if (e != hipErrorNotReady) return ACX_E_LAUNCH;
                if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(ACX_BFS_CHUNK_DEADLINE_S))
                    return ACX_E_TIMEOUT;
            }
        }
    };
    // every exit after the first enqueue: the chunk numbers used advance kbase, and the chunks
    // still in the stream (the speculative one after the search's end) are retired before the
    // search returns -- on success the stream is idle when acx_bfs_run returns.  After a
    // timeout (a kernel that does not finish) nothing is waited for here: `fin` makes the next
    // search and the destructor wait instead.
    auto finish = [&](int rc) -> int {
        S->kbase += enqueued;
        const bool rec = hipEventRecord(S->fin, st) == hipSuccess;
        S->fin_pending = rec;
        if (rc == ACX_E_TIMEOUT) return ACX_E_LAUNCH;
        if (!rec || hipStreamSynchronize(st) != hipSuccess) return ACX_E_LAUNCH;
        S->fin_pending = false;
        return rc;
    };
    const int64_t qcap = S->qcap;
    auto grow = [&](int64_t avail) -> int64_t {  // bound on the next chunk's available parents
        const int64_t p = avail < S->pmax ? avail : S->pmax;
        const int64_t ub = avail + 11 * p;
        return ub < qcap ? ub : qcap;
    };
    int64_t next_ub = grow(1);  // chunk 1's bound (chunk 0 expands the root alone)
    if (enqueue(0, 1) != ACX_OK || enqueue(1, next_ub) != ACX_OK) return finish(ACX_E_LAUNCH);
    Live lv{};
    int64_t k = 0;
    for (;; ++k) {
        const int w = wait_chunk(k);
        if (w != ACX_OK) return finish(w);
        lv = S->mirror[(S->kbase + k) % RING].s;
        if (lv.stop) break;
        // exact state after chunk k = chunk k + 1's parameters: bound chunk k + 2
        const int64_t avail = lv.n_nodes - lv.head;
        if (enqueue(k + 2, grow(avail)) != ACX_OK) return finish(ACX_E_LAUNCH);
    }
    // chunk k + 1 is in the stream (it does nothing): retired here, with the path kernel below
    if (lv.status < 0) return finish(ACX_E_LAUNCH);  // table overflow (cannot happen at load <= 1/2)
    const int status = lv.status;
    const int64_t n_nodes = lv.n_nodes, parents = lv.parents, chunks = lv.chunks;
    const int64_t min_len = lv.running;
    const int64_t succ_node = lv.succ_node, succ_act = lv.succ_act;
    int64_t path_len = 0;
    // the close kernels wrote the trace straight into pinned host memory before publishing
    const uint32_t nt = lv.ntrace < (uint32_t)TRACE_CAP ? lv.ntrace : TRACE_CAP;
    for (uint32_t i = 0; i < nt; ++i) S->trace.push_back(S->trace_host[i]);
    if (status == ACX_BFS_FOUND) {
        PathLaunch pl{S, st, succ_node};
        by_nw(L, pl);
        if (hipGetLastError() != hipSuccess) return finish(ACX_E_LAUNCH);
    }
    const int fin_rc = finish(ACX_OK);  // the stream is idle from here on
    if (fin_rc != ACX_OK) return fin_rc;
    if (status == ACX_BFS_FOUND) {
        const int64_t d = *(volatile int64_t*)S->path_n_dev;
        if (d > PATH_CAP) return ACX_E_ARG;
        std::vector<int32_t> buf((size_t)(2 * d + 2));
        for (int64_t i = 0; i < 2 * d; ++i) buf[(size_t)i] = ((volatile int32_t*)S->path_dev)[i];
        buf[2 * d] = (int32_t)succ_act;
        buf[2 * d + 1] = 2;
        // reference path: [(-1, total0)] + edges + (succ action, 2)
        path_len = d + 2;
        if (path_actions && path_totals) {
            for (int64_t i = 0; i < path_len && i < path_cap; ++i) {
                path_actions[i] = i == 0 ? -1 : buf[2 * (i - 1)];
                path_totals[i] = i == 0 ? total0 : buf[2 * (i - 1) + 1];
            }
        }
    }
    S->last_nodes = n_nodes < S->qcap ? n_nodes : S->qcap;
    stats[0] = n_nodes;
    stats[1] = parents;
    stats[2] = chunks;
    stats[3] = min_len;
    stats[4] = path_len;
    return status;
}

int64_t acx_bfs_node_keys(void* h, uint64_t* out, int64_t cap, void* stream) {
    Search* S = static_cast<Search*>(h);
    if (!S) return ACX_E_ARG;
    const int64_t n = S->last_nodes < cap ? S->last_nodes : cap;
    if (out && n > 0) {
        hipStream_t st = (hipStream_t)stream;
        if (n > S->gather_cap) {
            if (S->gather && hipFree(S->gather) != hipSuccess) return ACX_E_LAUNCH;
            S->gather = nullptr;
            S->gather_cap = 0;
            if (hipMalloc((void**)&S->gather, (size_t)(n * S->kw) * 8) != hipSuccess) return ACX_E_LAUNCH;
            S->gather_cap = n;
        }
        bfs_gather_kernel<<<dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, st>>>(S->a, n, S->gather);
        if (hipGetLastError() != hipSuccess ||
            copy_to_host(out, S->gather, (size_t)(n * S->kw) * 8, st, &S->bounce) != ACX_OK)
            return ACX_E_LAUNCH;
    }
    return S->last_nodes;
}

int64_t acx_bfs_min_trace(void* h, int32_t* out, int64_t cap) {
    Search* S = static_cast<Search*>(h);
    if (!S) return ACX_E_ARG;
    const int64_t n = (int64_t)S->trace.size();
    for (int64_t i = 0; out && i < n && i < cap; ++i) out[i] = S->trace[(size_t)i];
    return n;
}

}  // extern "C"
