// acx_bfs.hip -- breadth-first search over the AC graph with the whole search on the GPU:
// FIFO queue of packed node keys, visited set as an open-addressing hash table in HBM,
// 12-way expansion, dedup and budget accounting as kernels.  The host only launches one
// round of kernels per chunk of parents and reads back a 40-byte control block.
//
// Reference: ac_solver/search/breadth_first.py:15-97.  Semantics kept exactly:
//   * the queue is processed parent by parent in FIFO order, actions 0..11 per parent;
//   * a child with total length 2 ends the search (checked before the visited test,
//     breadth_first.py:84-85), path = parent's path + (action, 2);
//   * a child is appended iff its state was never seen (breadth_first.py:87-89); within a
//     chunk "seen" includes earlier children (in (parent, action) order) of the same chunk;
//   * after each parent, len(tree_nodes) >= max_nodes ends the search (:91-95);
//   * an ACMove that empties a relator raises in the reference (utils.py:264-266): status
//     ACX_BFS_MOVE_ERROR when it happens before the search would have ended.
// A chunk of P parents is expanded at once; child seq s = 12 p + action is its position in
// the reference's sequential order.  First occurrence wins: every unseen child claims or
// joins the hash slot of its state with atomicMin on s, so exactly the child the
// reference would have appended survives; survivors are ranked by a prefix sum over
// parents, which also yields the parent at which the node budget is reached.
//
// Table entry (uint64, 0 = empty):  node entry  (node+1) << 32 | fp
//                                   chunk entry 1 << 63 | seq << 32 | fp
// fp = high 32 bits of the key hash, slot = low bits.  Keys are compared in full
// (qkeys / ckeys), never by hash alone.  Within a kernel a slot only changes 0 -> entry of
// one state -> smaller seq of the same state, so plain (possibly stale) reads are safe:
// a stale 0 is corrected by the CAS, a stale entry names the same state.  Writes that a
// later phase compares against (child keys, node keys, node entries) are made one kernel
// earlier, so they are visible across XCDs (kernel boundaries write back / invalidate L2).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <new>

#include "acx.h"
#include "acx_moves.h"

#include "acx_bfs_common.h"

namespace acx {
namespace bfs {

struct Ctl {
    uint32_t succ_seq;  // min seq of a child with n0 + n1 == 2
    uint32_t err_seq;   // min seq of a child whose move raised in the reference
    uint32_t cut_p;     // parent after which len(tree_nodes) >= max_nodes
    uint32_t overflow;  // a probe walked the whole table (cannot happen at load <= 1/2)
    uint32_t min_len;   // min total length over all children of the chunk
    uint32_t pad;
    uint64_t total_new;     // nodes appended by the chunk
    uint64_t nodes_at_cut;  // len(tree_nodes) after parent cut_p
};

struct Args {
    uint64_t* qkeys;     // (qcap, kw) node keys in FIFO order
    int32_t* qparent;    // (qcap) parent node, -1 for the root
    uint8_t* qact;       // (qcap) move id that produced the node
    uint64_t* ckeys;     // (12, P) x kw child keys of the chunk, action-major
    uint32_t* slot;      // (12, P) hash slot claimed/joined by the child, SEEN if known
    uint16_t* masks;     // (P) bit a: child (p, a) is appended
    uint8_t* pmin;       // (P) min child total length per parent
    uint32_t* bsum;      // (nblocks) per-block new-node counts -> exclusive offsets
    uint32_t* bmin;      // (nblocks) per-block min child length
    uint64_t* table;     // (mask + 1) hash table
    Ctl* ctl;
    uint64_t mask;       // table size - 1
    int64_t head;        // queue index of the chunk's first parent
    int64_t n_before;    // len(tree_nodes) before the chunk
    int64_t need;        // max_nodes - n_before (>= 1)
    int64_t qcap;
    int P, L, kw, cyc;
};

// (1) expand: one lane per parent, 12 child keys
template <int NW>
__global__ __launch_bounds__(TPB) void bfs_expand_kernel(Args a) {
    const int p = blockIdx.x * TPB + threadIdx.x;
    if (p >= a.P) return;
    PresRegs<NW> pr;
    load_key<NW>(a.qkeys + (a.head + p) * a.kw, a.kw, a.L, pr);
    const bool cyc = a.cyc != 0;
    const bool clean = is_clean<NW>(pr.w0, pr.n0, pr.w1, pr.n1, cyc);
    uint32_t succ = NONE, err = NONE;
    int mn = 255;
    for (int act = 0; act < 12; ++act) {
        PresRegs<NW> q = pr;
        const int e = clean ? ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, cyc)
                            : ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, cyc);
        const uint32_t s = (uint32_t)p * 12u + (uint32_t)act;
        const int tot = q.n0 + q.n1;
        if (e != ACX_ERR_NONE) {
            if (err == NONE) err = s;
        } else {
            if (tot == 2 && succ == NONE) succ = s;
            mn = tot < mn ? tot : mn;
        }
        store_key<NW>(a.ckeys + ((int64_t)act * a.P + p) * a.kw, a.kw, a.L, q);
    }
    a.pmin[p] = (uint8_t)mn;
    if (succ != NONE) atomicMin(&a.ctl->succ_seq, succ);
    if (err != NONE) atomicMin(&a.ctl->err_seq, err);
}

// (2) probe the visited set / claim or join the child's slot, one lane per child
template <int KWM>
__global__ __launch_bounds__(TPB) void bfs_insert_kernel(Args a) {
    const int64_t ci = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (ci >= 12ll * a.P) return;
    const uint32_t act = (uint32_t)(ci / a.P);
    const uint32_t p = (uint32_t)(ci - (int64_t)act * a.P);
    const uint32_t s = p * 12u + act;
    const uint32_t end = min(a.ctl->succ_seq, a.ctl->err_seq);
    if (s > end) {  // after the search's last child: never looked at
        a.slot[ci] = SEEN;
        return;
    }
    const Key<KWM> key = kload<KWM>(a.ckeys + ci * a.kw, a.kw);
    const uint64_t h = khash<KWM>(key, a.kw);
    const uint32_t fp = (uint32_t)(h >> 32);
    uint64_t idx = h & a.mask;
    const uint64_t my = CHUNK | ((uint64_t)s << 32) | fp;
    uint32_t res = SEEN;
    for (uint64_t it = 0;; ++it) {
        if (it > a.mask) {
            atomicOr(&a.ctl->overflow, 1u);
            break;
        }
        uint64_t v = tload(a.table + idx);
        if (v == 0) {
            const uint64_t old = atomicCAS((unsigned long long*)(a.table + idx), 0ull, (unsigned long long)my);
            if (old == 0) {
                res = (uint32_t)idx;
                break;
            }
            v = old;
        }
        if ((uint32_t)v == fp) {
            const uint32_t hi = (uint32_t)(v >> 32);
            if (v & CHUNK) {
                const uint32_t s2 = hi & 0x7fffffffu;
                const int64_t ci2 = (int64_t)(s2 % 12u) * a.P + s2 / 12u;
                if (keq<KWM>(a.ckeys + ci2 * a.kw, key, a.kw)) {
                    atomicMin((unsigned long long*)(a.table + idx), (unsigned long long)my);
                    res = (uint32_t)idx;
                    break;
                }
            } else if (keq<KWM>(a.qkeys + (int64_t)(hi - 1) * a.kw, key, a.kw)) {
                break;  // already a node
            }
        }
        idx = (idx + 1) & a.mask;
    }
    a.slot[ci] = res;
}

// (3) which children survived (first occurrence), per-block counts and min lengths
__global__ __launch_bounds__(TPB) void bfs_mark_kernel(Args a) {
    __shared__ uint32_t sh[TPB / WAVE];
    const int p = blockIdx.x * TPB + threadIdx.x;
    uint32_t m = 0, mn = 0xffffffffu;
    if (p < a.P) {
        for (int act = 0; act < 12; ++act) {
            const int64_t ci = (int64_t)act * a.P + p;
            const uint32_t si = a.slot[ci];
            if (si == SEEN) continue;
            const uint64_t want = (CHUNK >> 32) | ((uint64_t)p * 12u + act);
            if ((a.table[si] >> 32) == want) m |= 1u << act;
        }
        a.masks[p] = (uint16_t)m;
        mn = a.pmin[p];
    }
    uint32_t tot;
    block_excl_scan(__popc(m), sh, tot);
    __syncthreads();
    const uint32_t bm = block_min(mn, sh);
    if (threadIdx.x == 0) {
        a.bsum[blockIdx.x] = tot;
        a.bmin[blockIdx.x] = bm;
    }
}

// (4) exclusive scan of the block counts (one block of 1024 threads)
__global__ __launch_bounds__(1024) void bfs_scan_kernel(Args a, int nb) {
    __shared__ uint32_t sh[1024 / WAVE];
    __shared__ uint32_t shm[1024 / WAVE];
    const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
    const int per = (nb + 1023) / 1024;
    const int b0 = t * per, b1 = min(nb, b0 + per);
    uint32_t loc = 0, mn = 0xffffffffu;
    for (int i = b0; i < b1; ++i) {
        loc += a.bsum[i];
        mn = min(mn, a.bmin[i]);
    }
    uint32_t x = loc;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, WAVE));
    }
    if (lane == WAVE - 1) sh[wid] = x;
    if (lane == 0) shm[wid] = mn;
    __syncthreads();
    uint32_t off = 0, tot = 0, bm = 0xffffffffu;
    for (int i = 0; i < 1024 / WAVE; ++i) {
        off += i < wid ? sh[i] : 0u;
        tot += sh[i];
        bm = min(bm, shm[i]);
    }
    uint32_t run = off + x - loc;
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = a.bsum[i];
        a.bsum[i] = run;
        run += c;
    }
    if (t == 0) {
        a.ctl->total_new = tot;
        a.ctl->min_len = bm;
    }
}

// (5) append the survivors in (parent, action) order; the node budget cut
__global__ __launch_bounds__(TPB) void bfs_commit_kernel(Args a) {
    __shared__ uint32_t sh[TPB / WAVE];
    const int p = blockIdx.x * TPB + threadIdx.x;
    const uint32_t m = p < a.P ? a.masks[p] : 0u;
    const uint32_t c = __popc(m);
    uint32_t tot;
    const int64_t base = (int64_t)a.bsum[blockIdx.x] + block_excl_scan(c, sh, tot);
    if (p >= a.P) return;
    // cut = first parent with n_before + (nodes appended through it) >= max_nodes
    const int64_t incl = base + c;
    if (incl >= a.need && (base < a.need || p == 0)) {
        a.ctl->cut_p = (uint32_t)p;
        a.ctl->nodes_at_cut = (uint64_t)(a.n_before + incl);
    }
    if (c == 0) return;
    int64_t node = a.n_before + base;
    uint32_t mm = m;
    while (mm) {
        const int act = __builtin_ctz(mm);
        mm &= mm - 1;
        if (node < a.qcap) {
            const int64_t ci = (int64_t)act * a.P + p;
            for (int k = 0; k < a.kw; ++k) a.qkeys[node * a.kw + k] = a.ckeys[ci * a.kw + k];
            a.qparent[node] = (int32_t)(a.head + p);
            a.qact[node] = (uint8_t)act;
            const uint32_t si = a.slot[ci];
            const uint64_t v = a.table[si];
            a.table[si] = ((uint64_t)(node + 1) << 32) | (uint32_t)v;
        }
        ++node;
    }
}

// root: node 0 and its table entry
template <int KWM>
__global__ void bfs_root_kernel(Args a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const Key<KWM> key = kload<KWM>(a.qkeys, a.kw);
    const uint64_t h = khash<KWM>(key, a.kw);
    a.table[h & a.mask] = (1ull << 32) | (uint32_t)(h >> 32);
    a.qparent[0] = -1;
    a.qact[0] = 0xff;
}

// path root -> node: (action, total length) per edge, into out[0..2*depth), depth in out_n
template <int NW>
__global__ void bfs_path_kernel(Args a, int64_t node, int32_t* out, int64_t cap, int64_t* out_n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t d = 0;
    for (int64_t v = node; v > 0; v = a.qparent[v]) ++d;
    *out_n = d;
    if (d > cap) return;
    int64_t i = d;
    for (int64_t v = node; v > 0; v = a.qparent[v]) {
        PresRegs<NW> pr;
        load_key<NW>(a.qkeys + v * a.kw, a.kw, a.L, pr);
        --i;
        out[2 * i] = a.qact[v];
        out[2 * i + 1] = pr.n0 + pr.n1;
    }
}


struct Search {
    int dev = 0, L = 0, kw = 0, cyc = 0;
    int64_t max_nodes = 0, qcap = 0, pmax = 0;
    int64_t last_nodes = 0;  // len(tree_nodes) at the end of the last run
    uint64_t tsize = 0;
    Args a{};
    Ctl* ctl_host = nullptr;
    int32_t* path_dev = nullptr;
    int64_t* path_n_dev = nullptr;
    bool ok = false;

    ~Search() {
        void* ptrs[] = {a.qkeys, a.qparent, a.qact, a.ckeys, a.slot, a.masks, a.pmin,
                        a.bsum,  a.bmin,    a.table, a.ctl,  path_dev, path_n_dev};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        if (ctl_host) (void)hipHostFree(ctl_host);
    }
};

static constexpr int64_t PATH_CAP = 1 << 16;

template <class T>
static bool dalloc(T*& p, size_t n) {
    return hipMalloc((void**)&p, n * sizeof(T) + 16) == hipSuccess;
}

// launches of one chunk, templated on the key-word bound
struct ChunkLaunch {
    Search* S;
    hipStream_t st;
    int nb;
    template <int NW>
    void go() {
        Args& a = S->a;
        const int64_t nc = 12ll * a.P;
        bfs_expand_kernel<NW><<<dim3(nb), dim3(TPB), 0, st>>>(a);
        bfs_insert_kernel<NW + 1><<<dim3((unsigned)((nc + TPB - 1) / TPB)), dim3(TPB), 0, st>>>(a);
        bfs_mark_kernel<<<dim3(nb), dim3(TPB), 0, st>>>(a);
        bfs_scan_kernel<<<dim3(1), dim3(1024), 0, st>>>(a, nb);
        bfs_commit_kernel<<<dim3(nb), dim3(TPB), 0, st>>>(a);
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
    if (chunk_parents <= 0) chunk_parents = 1 << 19;  // tools/bfs_chunk_probe.py: 2^19-2^20 fastest
    S->pmax = chunk_parents < S->qcap ? chunk_parents : S->qcap;
    // every node and every claimed chunk slot at load <= 1/2
    uint64_t ts = 1024;
    while (ts < 2 * (uint64_t)(S->qcap + 12 * S->pmax)) ts <<= 1;
    if (ts > (1ull << 31)) { delete S; return nullptr; }
    S->tsize = ts;
    Args& a = S->a;
    const int64_t nb = (S->pmax + TPB - 1) / TPB;
    bool ok = dalloc(a.qkeys, (size_t)(S->qcap * S->kw)) && dalloc(a.qparent, (size_t)S->qcap) &&
              dalloc(a.qact, (size_t)S->qcap) && dalloc(a.ckeys, (size_t)(12 * S->pmax * S->kw)) &&
              dalloc(a.slot, (size_t)(12 * S->pmax)) && dalloc(a.masks, (size_t)S->pmax) &&
              dalloc(a.pmin, (size_t)S->pmax) && dalloc(a.bsum, (size_t)nb) && dalloc(a.bmin, (size_t)nb) &&
              dalloc(a.table, (size_t)ts) && dalloc(a.ctl, 1) && dalloc(S->path_dev, (size_t)(2 * PATH_CAP)) &&
              dalloc(S->path_n_dev, 1) &&
              hipHostMalloc((void**)&S->ctl_host, sizeof(Ctl), hipHostMallocDefault) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        delete S;
        return nullptr;
    }
    a.mask = ts - 1;
    a.qcap = S->qcap;
    a.L = L;
    a.kw = S->kw;
    a.cyc = S->cyc;
    return S;
}

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

    if (hipMemcpyAsync(a.qkeys, root, (size_t)kw * 8, hipMemcpyHostToDevice, st) != hipSuccess) return ACX_E_LAUNCH;
    if (hipMemsetAsync(a.table, 0, S->tsize * 8, st) != hipSuccess) return ACX_E_LAUNCH;
    RootLaunch rl{S, st};
    by_nw(L, rl);

    int64_t n_nodes = 1, head = 0, parents = 0, chunks = 0;
    int64_t min_len = total0, path_len = 0;
    int status = ACX_BFS_EXHAUSTED;
    int64_t succ_node = -1, succ_act = -1;
    Ctl init;
    memset(&init, 0xff, sizeof(init));
    init.overflow = 0;
    init.total_new = 0;
    init.nodes_at_cut = 0;
    while (head < n_nodes) {
        const int64_t avail = n_nodes - head;
        const int P = (int)(avail < S->pmax ? avail : S->pmax);
        a.P = P;
        a.head = head;
        a.n_before = n_nodes;
        a.need = max_nodes - n_nodes;
        if (hipMemcpyAsync(a.ctl, &init, sizeof(Ctl), hipMemcpyHostToDevice, st) != hipSuccess) return ACX_E_LAUNCH;
        ChunkLaunch cl{S, st, (P + TPB - 1) / TPB};
        by_nw(L, cl);
        if (hipGetLastError() != hipSuccess) return ACX_E_LAUNCH;
        if (hipMemcpyAsync(S->ctl_host, a.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st) != hipSuccess)
            return ACX_E_LAUNCH;
        if (hipStreamSynchronize(st) != hipSuccess) return ACX_E_LAUNCH;
        const Ctl c = *S->ctl_host;
        ++chunks;
        if (c.overflow) return ACX_E_LAUNCH;
        const int64_t cut = c.cut_p == NONE ? INT64_MAX : (int64_t)c.cut_p;
        const int64_t err_p = c.err_seq == NONE ? INT64_MAX : (int64_t)(c.err_seq / 12);
        const int64_t suc_p = c.succ_seq == NONE ? INT64_MAX : (int64_t)(c.succ_seq / 12);
        const bool err_first = c.err_seq != NONE && c.err_seq < c.succ_seq && err_p <= cut;
        const bool succ_first = !err_first && c.succ_seq != NONE && suc_p <= cut;
        if (err_first || succ_first || cut != INT64_MAX) {
            // the search ends in this chunk: min over the parents it reached (verbose only)
            const int64_t last = err_first ? err_p : succ_first ? suc_p : cut;
            if (succ_first) {
                min_len = 2;
            } else {
                uint8_t* pm = new (std::nothrow) uint8_t[last + 1];
                if (!pm) return ACX_E_LAUNCH;
                if (hipMemcpy(pm, a.pmin, (size_t)(last + 1), hipMemcpyDeviceToHost) != hipSuccess) {
                    delete[] pm;
                    return ACX_E_LAUNCH;
                }
                for (int64_t i = 0; i <= last; ++i) min_len = pm[i] < min_len ? pm[i] : min_len;
                delete[] pm;
            }
            parents += last + 1;
            if (err_first) {
                status = ACX_BFS_MOVE_ERROR;
            } else if (succ_first) {
                status = ACX_BFS_FOUND;
                succ_node = head + suc_p;
                succ_act = c.succ_seq % 12;
            } else {
                status = ACX_BFS_BUDGET;
                n_nodes = (int64_t)c.nodes_at_cut;
            }
            break;
        }
        min_len = (int64_t)c.min_len < min_len ? (int64_t)c.min_len : min_len;
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
        int32_t* buf = new (std::nothrow) int32_t[2 * d + 2];
        if (!buf) return ACX_E_LAUNCH;
        if (d && hipMemcpy(buf, S->path_dev, (size_t)(2 * d) * 4, hipMemcpyDeviceToHost) != hipSuccess) {
            delete[] buf;
            return ACX_E_LAUNCH;
        }
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
        delete[] buf;
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
    if (out && n > 0 &&
        hipMemcpy(out, S->a.qkeys, (size_t)(n * S->kw) * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return ACX_E_LAUNCH;
    return S->last_nodes;
}

}  // extern "C"
