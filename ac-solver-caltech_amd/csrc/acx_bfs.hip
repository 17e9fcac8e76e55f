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
//     minima of the child totals in sequential order (bfs_trace_kernel).
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
//                         action) order (LDS-staged, coalesced), the node-budget cut.
// Cross-XCD visibility: every value a kernel compares against (child keys, queue codes) was
// written by an earlier kernel; within bfs_insert_kernel an entry only goes 0 -> one state's
// code -> a smaller code of the same state, so stale plain reads are harmless (a stale 0 is
// corrected by the CAS, a stale entry names the same state).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "acx.h"
#include "acx_moves.h"

#include "acx_bfs_common.h"

namespace acx {
namespace bfs {

constexpr int TILE = 64;                // parents per tile (one wave)
constexpr int TILE_CH = 12 * TILE;      // children per tile
constexpr int BUCKET = 8;               // table entries per bucket (64 B)
constexpr int TRACE_CAP = 1024;         // new-minimum records per trace walk (<= 2L + 1 ever)
constexpr uint32_t FP_MASK = 0xffffffu;

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

struct Args {
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
};

// (1) expand: one block per tile of 64 parents; wave w makes the children of actions 3w..3w+2
// (4x the lanes of a lane-per-parent loop: the move chain is latency-bound, and a 2^19-parent
// chunk is only ~8 waves per SIMD that way); keys staged through LDS, written coalesced
constexpr int APW = 12 / (TPB / WAVE);  // actions per wave (3)
template <int NW>
__global__ __launch_bounds__(TPB, NW <= 4 ? 8 : 4) void bfs_expand_kernel(Args a) {
    __shared__ uint64_t kst[TPB / WAVE][TILE * (NW + 1)];
    __shared__ uint32_t smin[TILE];
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    const int t = blockIdx.x;  // one tile per block
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
            const uint64_t my = (code << 24) | fp;
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
                    if (v == 0) {
                        const uint64_t old = atomicCAS((unsigned long long*)(bk + j), 0ull, (unsigned long long)my);
                        if (old == 0) {
                            done = 2;
                            break;
                        }
                        v = old;
                    }
                    if (((uint32_t)v & FP_MASK) != fp) continue;
                    const uint64_t vc = v >> 24;
                    if (!keq<KWM>(a.store + store_index(vc) * kw, key, kw)) continue;
                    if (vc < code) {  // an earlier occurrence (a node, or an earlier child of the chunk)
                        done = 1;
                        break;
                    }
                    const uint64_t old = atomicMin((unsigned long long*)(bk + j), (unsigned long long)my);
                    if (old < my) {
                        done = 1;
                    } else {  // replaced a later child of the chunk: it learns it lost
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
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    const int t = blockIdx.x * (TPB / WAVE) + wid;
    if (t >= a.ntiles) return;
    const uint32_t n = wave_sum(__popc(survivors(a, t, lane, false)));
    if (lane == 0) a.tsum[t] = n;
}

// (4) exclusive scan of the tile counts (one block of 1024 threads)
__global__ __launch_bounds__(1024) void bfs_scan_kernel(Args a) {
    __shared__ uint32_t sh[1024 / WAVE];
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

// the chunk's control block to its initial values (a kernel, so the reset is asynchronous on
// the stream: a host-to-device copy from pageable memory blocks the host for its duration)
__global__ void bfs_ctl_reset_kernel(Ctl* c) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    Ctl z;
    memset(&z, 0, sizeof(z));
    z.succ = z.err = z.cut_p = z.min_len = NONE;
    *c = z;
}

// wait for the stream by polling (hipStreamSynchronize may sleep and wake late: one wait per
// chunk is on the search's critical path)
static int stream_wait(hipStream_t st) {
    hipError_t e;
    while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
    }
    return e == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

// root: node 0 (code 1) and its table entry
template <int KWM>
__global__ void bfs_root_kernel(Args a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const Key<KWM> key = kload<KWM>(a.store, a.kw);
    const uint64_t h = khash<KWM>(key, a.kw);
    uint64_t* ent = a.table + (h & a.bmask) * BUCKET;
    ent[0] = (1ull << 24) | (uint32_t)(h >> 40);
    if (a.kt) {
        uint64_t gd[3];
        kt_guarded(key.w, a.kw, gd);
        ent[1] = gd[0];
        ent[2] = gd[1];
        ent[3] = gd[2];
    }
    a.queue[0] = 1;
}

// min_length trace over the chunk's children in sequential order up to (exclusive) seq `end`
// (one block): parents whose min child total beats the running minimum are found with a
// prefix-min scan; those few are re-expanded and walked move by move (breadth_first.py:79-82)
template <int NW>
__global__ __launch_bounds__(256) void bfs_trace_kernel(Args a, uint32_t end, uint32_t running) {
    __shared__ uint32_t lmin[256];
    __shared__ uint32_t list[TRACE_CAP];
    __shared__ uint32_t nlist;
    const int t = threadIdx.x;
    const int64_t np = ((int64_t)end + 11) / 12;  // parents with children before `end`
    const int64_t per = (np + 255) / 256;
    const int64_t p0 = t * per, p1 = min<int64_t>(np, p0 + per);
    uint32_t m = 0xffffffffu;
    for (int64_t p = p0; p < p1; ++p) m = min(m, (uint32_t)a.pmin[p]);
    lmin[t] = m;
    if (t == 0) nlist = 0;
    __syncthreads();
    uint32_t r = running;
    for (int i = 0; i < t; ++i) r = min(r, lmin[i]);
    for (int64_t p = p0; p < p1; ++p) {
        const uint32_t v = a.pmin[p];
        if (v < r) {
            const uint32_t k = atomicAdd(&nlist, 1u);
            if (k < TRACE_CAP) list[k] = (uint32_t)p;
            r = v;
        }
    }
    __syncthreads();
    if (t != 0) return;
    const uint32_t n = min(nlist, (uint32_t)TRACE_CAP);
    for (uint32_t i = 1; i < n; ++i) {  // insertion sort: the parents in order (few)
        const uint32_t v = list[i];
        uint32_t j = i;
        for (; j > 0 && list[j - 1] > v; --j) list[j] = list[j - 1];
        list[j] = v;
    }
    uint32_t cur = running, nt = 0;
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
                if (nt < TRACE_CAP) a.trace[nt] = (uint16_t)tot;
                ++nt;
            }
        }
    }
    a.ctl->ntrace = nt;
    a.ctl->trace_min = cur;
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
    Ctl* ctl_host = nullptr;
    uint16_t* trace_host = nullptr;
    int32_t* path_dev = nullptr;
    int64_t* path_n_dev = nullptr;
    std::vector<int32_t> trace;  // new minima of the last run, in order

    ~Search() {
        void* ptrs[] = {a.store, a.queue, a.cand, a.lost, a.pmin, a.tsum, a.tmin, a.table, a.ctl, a.trace, path_dev,
                        path_n_dev};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        if (ctl_host) (void)hipHostFree(ctl_host);
        if (trace_host) (void)hipHostFree(trace_host);
    }
};

static constexpr int64_t PATH_CAP = 1 << 16;
static int g_bfs_layout = 0;  // 0 default (8-entry table), 2 key-in-table where L allows (tests, A/B)

template <class T>
static bool dalloc(T*& p, size_t n) {
    return hipMalloc((void**)&p, n * sizeof(T) + 64) == hipSuccess;
}

// launches of one chunk, templated on the key-word bound
struct ChunkLaunch {
    Search* S;
    hipStream_t st;
    template <int NW>
    void go() {
        Args& a = S->a;
        const unsigned wb = (unsigned)((a.ntiles + TPB / WAVE - 1) / (TPB / WAVE));
        const int64_t nc = (int64_t)a.ntiles * TILE_CH;
        bfs_expand_kernel<NW><<<dim3((unsigned)a.ntiles), dim3(TPB), 0, st>>>(a);
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
    }
};
struct RootLaunch {
    Search* S;
    hipStream_t st;
    template <int NW>
    void go() { bfs_root_kernel<NW + 1><<<dim3(1), dim3(64), 0, st>>>(S->a); }
};
struct PathLaunch {
    Search* S;
    hipStream_t st;
    int64_t node;
    template <int NW>
    void go() { bfs_path_kernel<NW><<<dim3(1), dim3(64), 0, st>>>(S->a, node, S->path_dev, PATH_CAP, S->path_n_dev); }
};
struct TraceLaunch {
    Search* S;
    hipStream_t st;
    uint32_t end, running;
    template <int NW>
    void go() { bfs_trace_kernel<NW><<<dim3(1), dim3(256), 0, st>>>(S->a, end, running); }
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
    // probe).  (Half that -- load <= 1, 134 MB at 10^7 nodes, inside the 256 MB MALL -- measured
    // 1.83 vs 1.93 ms at 10^7 but 18.4 vs 17.0 ms at 10^8 nodes: not taken.)
    // Key-in-table (L <= KT_MAX_L, opt-in): 4 words per entry, entries >= 1.25x the same bound
    // (2 per bucket; the bound counts a whole last chunk's children as new: the real load stays
    // lower).  Measured slower than the 8-entry table (r03i: 2.11 vs 1.68 ms at 10^7 nodes, 20.0
    // vs 14.2 ms at 10^8): the saved node-key reads cost less than the table's doubled footprint.
    const bool kt = L <= KT_MAX_L && g_bfs_layout == 2;
    uint64_t ts = 1024;
    const uint64_t bound = (uint64_t)(S->qcap + 12 * S->pmax);
    while (kt ? ts < 5 * bound : ts < 2 * bound) ts <<= 1;
    S->tsize = ts;
    Args& a = S->a;
    bool ok = dalloc(a.store, (size_t)(S->scap * S->kw)) && dalloc(a.queue, (size_t)S->qcap) &&
              dalloc(a.cand, (size_t)(S->tiles_max * TILE_CH)) && dalloc(a.lost, (size_t)(S->tiles_max * TILE_CH)) &&
              dalloc(a.pmin, (size_t)S->pmax) && dalloc(a.tsum, (size_t)S->tiles_max) &&
              dalloc(a.tmin, (size_t)S->tiles_max) && dalloc(a.table, (size_t)ts) &&
              dalloc(a.ctl, 1) && dalloc(a.trace, (size_t)TRACE_CAP) && dalloc(S->path_dev, (size_t)(2 * PATH_CAP)) &&
              dalloc(S->path_n_dev, 1) &&
              hipHostMalloc((void**)&S->ctl_host, sizeof(Ctl), hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc((void**)&S->trace_host, sizeof(uint16_t) * TRACE_CAP, hipHostMallocDefault) == hipSuccess &&
              hipMemset(a.lost, 0, (size_t)(S->tiles_max * TILE_CH)) == hipSuccess;
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
    uint64_t root[ACX_MAX_L / 16 + 2];
    pack_key(presentation, L, kw, root);
    int total0 = 0;
    for (int i = 0; i < 2 * L; ++i) total0 += presentation[i] != 0;

    if (hipMemcpyAsync(a.store, root, (size_t)kw * 8, hipMemcpyHostToDevice, st) != hipSuccess) return ACX_E_LAUNCH;
    if (hipMemsetAsync(a.table, 0, S->tsize * 8, st) != hipSuccess) return ACX_E_LAUNCH;
    RootLaunch rl{S, st};
    by_nw(L, rl);

    S->trace.clear();
    int64_t n_nodes = 1, head = 0, parents = 0, chunks = 0;
    int64_t min_len = total0, path_len = 0;
    int status = ACX_BFS_EXHAUSTED;
    int64_t succ_node = -1, succ_act = -1;
    while (head < n_nodes) {
        const int64_t avail = n_nodes - head;
        const int P = (int)(avail < S->pmax ? avail : S->pmax);
        a.P = P;
        a.head = head;
        a.tile0 = head / TILE;
        a.ntiles = (int)((head + P - 1) / TILE - a.tile0 + 1);
        a.n_before = n_nodes;
        a.need = max_nodes - n_nodes;
        bfs_ctl_reset_kernel<<<dim3(1), dim3(64), 0, st>>>(a.ctl);
        ChunkLaunch cl{S, st};
        by_nw(L, cl);
        if (hipGetLastError() != hipSuccess) return ACX_E_LAUNCH;
        if (hipMemcpyAsync(S->ctl_host, a.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st) != hipSuccess)
            return ACX_E_LAUNCH;
        if (stream_wait(st) != ACX_OK) return ACX_E_LAUNCH;
        const Ctl c = *S->ctl_host;
        ++chunks;
        if (c.overflow) return ACX_E_LAUNCH;
        const int64_t cut = c.cut_p == NONE ? INT64_MAX : (int64_t)c.cut_p;
        const int64_t err_p = c.err == NONE ? INT64_MAX : (int64_t)(c.err / 12);
        const int64_t suc_p = c.succ == NONE ? INT64_MAX : (int64_t)(c.succ / 12);
        const bool err_first = c.err != NONE && c.err < c.succ && err_p <= cut;
        const bool succ_first = !err_first && c.succ != NONE && suc_p <= cut;
        const bool ends = err_first || succ_first || cut != INT64_MAX;
        // children the reference looks at in this chunk, in order: up to and including the
        // success child, up to (not including) the raising child, through the cut parent
        const uint32_t end = err_first ? c.err : succ_first ? c.succ + 1
                           : cut != INT64_MAX ? (uint32_t)((cut + 1) * 12) : (uint32_t)P * 12u;
        if (c.min_len < (uint32_t)min_len) {  // a new minimum somewhere in the chunk: walk it
            TraceLaunch tl{S, st, end, (uint32_t)min_len};
            by_nw(L, tl);
            if (hipGetLastError() != hipSuccess) return ACX_E_LAUNCH;
            if (hipMemcpyAsync(S->ctl_host, a.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(S->trace_host, a.trace, sizeof(uint16_t) * TRACE_CAP, hipMemcpyDeviceToHost, st) !=
                    hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return ACX_E_LAUNCH;
            const uint32_t nt = S->ctl_host->ntrace < (uint32_t)TRACE_CAP ? S->ctl_host->ntrace : TRACE_CAP;
            for (uint32_t i = 0; i < nt; ++i) S->trace.push_back(S->trace_host[i]);
            min_len = S->ctl_host->trace_min;
        }
        if (ends) {
            const int64_t last = err_first ? err_p : succ_first ? suc_p : cut;
            parents += last + 1;
            if (err_first) {
                status = ACX_BFS_MOVE_ERROR;
            } else if (succ_first) {
                status = ACX_BFS_FOUND;
                succ_node = head + suc_p;
                succ_act = c.succ % 12;
            } else {
                status = ACX_BFS_BUDGET;
                n_nodes = (int64_t)c.nodes_at_cut;
            }
            break;
        }
        parents += P;
        n_nodes += (int64_t)c.total_new;
        head += P;
    }
    if (status == ACX_BFS_FOUND) {
        PathLaunch pl{S, st, succ_node};
        by_nw(L, pl);
        int64_t d = 0;
        if (hipMemcpyAsync(&d, S->path_n_dev, 8, hipMemcpyDeviceToHost, st) != hipSuccess) return ACX_E_LAUNCH;
        if (hipStreamSynchronize(st) != hipSuccess) return ACX_E_LAUNCH;
        if (d > PATH_CAP) return ACX_E_ARG;
        std::vector<int32_t> buf((size_t)(2 * d + 2));
        if (d && hipMemcpy(buf.data(), S->path_dev, (size_t)(2 * d) * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return ACX_E_LAUNCH;
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

int64_t acx_bfs_node_keys(void* h, uint64_t* out, int64_t cap) {
    Search* S = static_cast<Search*>(h);
    if (!S) return ACX_E_ARG;
    const int64_t n = S->last_nodes < cap ? S->last_nodes : cap;
    if (out && n > 0) {
        uint64_t* tmp = nullptr;
        if (hipMalloc((void**)&tmp, (size_t)(n * S->kw) * 8) != hipSuccess) return ACX_E_LAUNCH;
        bfs_gather_kernel<<<dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB)>>>(S->a, n, tmp);
        const bool ok = hipGetLastError() == hipSuccess &&
                        hipMemcpy(out, tmp, (size_t)(n * S->kw) * 8, hipMemcpyDeviceToHost) == hipSuccess;
        (void)hipFree(tmp);
        if (!ok) return ACX_E_LAUNCH;
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
