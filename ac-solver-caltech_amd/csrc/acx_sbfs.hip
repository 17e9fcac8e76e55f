// acx_sbfs.hip -- breadth-first search with the node store and the visited set partitioned
// over G GPUs by key owner (SURVEY §8e "GPU-side dedup", §8f item 1).  One process per GPU;
// the host (acx/search/_sharded_bfs.py) runs the same chunk loop on every rank and does the
// three exchanges of a chunk with torch.distributed (RCCL over xGMI on the GPU node):
//   1. all_gather of a small vector per rank (success / move-error seqs, min length, the
//      number of children this rank sends to each owner);
//   2. all_to_all of child records (packed key + chunk seq) to their owners;
//   3. all_reduce (sum) of the per-parent survivor masks (P x int32; bits are disjoint).
//
// Reference: ac_solver/search/breadth_first.py:15-97; results (path, budget cut, node order)
// equal the single-GPU device BFS (acx_bfs.hip) and the reference.  The FIFO queue is global
// and implicit: node g (its position in the reference's `to_explore` / `tree_nodes` order)
// lives on rank owner(key(g)), which stores it in ascending g.  A chunk is the global parent
// range [head, head + P); each rank expands the parents it owns in that range (a contiguous
// run of its store), so child seq s = 12 (g - head) + action is the child's position in the
// reference's sequential order, exactly as on one GPU.
//
// Per chunk on rank r:
//   expand  -- its parents' 12 children (keys action-major), owner per child, per-owner counts;
//   pack    -- children owned by other ranks into the send buffer grouped by owner: record =
//              kw key words + seq (the rank's own children stay where the expansion wrote them);
//   insert  -- its own children in place and the received records: probe / claim / join the
//              owner's hash table with atomicMin on (seq, record) (first occurrence wins, as in
//              acx_bfs.hip; a displaced child is marked lost); survivors -> bit (s % 12) of
//              mask[s / 12];
//   commit  -- after the mask all-reduce every rank knows all survivors: a prefix sum over
//              parents gives each survivor's global id g and the node-budget cut (identical on
//              all ranks); a second prefix sum over the survivors this rank owns gives their
//              slots in its store, where they are appended (ascending g).
// Keys live in an append-only arena of records: the expansion writes a chunk's children straight
// into it (12 per local parent, seq order), a received child that survives is copied in after
// them, and a table entry names its record's arena position from the moment it is claimed.  So a
// node's key is never copied and its entry never rewritten (round 4's commit copied every
// survivor's key into a compact store and rewrote its entry: 0.63 of the search's 2.5 ms at one
// rank); the store holds, per node, its arena position.  The arena grows by reallocation between
// chunks (entries hold positions, not addresses).
// Owner of a key = (fp * G) >> 32 with fp the high hash bits (table slot = low bits).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <new>

#include "acx.h"
#include "acx_bfs_common.h"

namespace acx {
namespace sbfs {

using namespace acx::bfs;

constexpr int MAXW = 64;  // max ranks

struct Ctl {
    uint32_t succ_seq;   // expand: min seq of a local child with n0 + n1 == 2
    uint32_t err_seq;    // expand: min seq of a local child whose move raised
    uint32_t min_len;    // expand: min child total over the local parents
    uint32_t npar;       // expand: local parents in the chunk
    uint32_t overflow;   // a probe walked the whole table / the node store is full
    uint32_t cut_p;      // commit: parent after which len(tree_nodes) >= max_nodes (all ranks)
    uint64_t total_new;  // commit: nodes appended by the chunk over all ranks
    uint64_t local_new;  // commit: nodes appended to this rank's store
    uint64_t nodes_at_cut;
    uint32_t stored;     // commit: nodes stored here (appends before max_nodes + 12)
    uint32_t pad2;
    uint32_t cnt[MAXW];  // expand: children sent to each owner
    uint32_t cur[MAXW];  // pack cursors
};

__device__ __forceinline__ void ctl_init(Ctl* c) {
    Ctl z;
    memset(&z, 0, sizeof(z));
    z.succ_seq = z.err_seq = z.min_len = z.cut_p = NONE;
    *c = z;
}

struct Args {
    uint64_t* arena;  // (acap, kw) records: every chunk's expanded children, received survivors
    int64_t* lapos;   // (lcap) owned nodes, ascending global id: arena position of the key
    int64_t* lgid;    // (lcap) global node id
    int64_t* lpar;    // (lcap) global id of the parent, -1 for the root
    uint8_t* lact;    // (lcap) move id that produced the node
    uint64_t* ckeys;  // = arena + abase * kw: (Pr, 12) keys of the local parents' children,
                      // parent-major (seq order); the chunk's received survivors follow
    uint8_t* cown;    // (Pr, 12) owner of each child, 0xff: parent not in the chunk
    uint16_t* pmin;   // (Pr) min child total per local parent (totals reach 2L = 256)
    uint32_t* sslot;  // (12 P) per chunk seq: table slot its child claimed / joined as the first
                      // occurrence, SEEN if none (a known state, past the end, or not owned here)
    uint32_t* srec;   // (12 P) per chunk seq: the child's record (arena position - abase)
    uint8_t* lost;    // (12 P) per chunk seq: a smaller seq of the same state took its entry
    uint32_t* mine;   // (P) this rank's survivors per parent (bits by action)
    uint32_t* bsum;   // (nb) all survivors per block of parents -> exclusive offsets
    uint32_t* lbsum;  // (nb) own survivors per block -> exclusive offsets
    uint64_t* table;  // (mask + 1)
    Ctl* ctl;
    const uint64_t* recv;  // (nrecv, kw + 1) received records
    uint64_t* send;        // (nsend, kw + 1) records grouped by owner
    uint32_t* gmask;       // (P) survivor masks (this rank's, then all-reduced)
    int64_t* look;         // lookup result
    uint32_t* xblk;        // (expand blocks, 2 + world) per-block min child total, parents, owner counts
    uint64_t mask;
    int64_t head, n_before, need, lcap, nloc, lo, nrecv, abase;
    int P, Pr, L, kw, cyc, world, rank;
    uint32_t end;
    int end_from_ctl;
};

// Table entries: (arena position + 1) << 24 | 24-bit fingerprint, final from the claim on.  An
// entry at or past the chunk's arena base is a child of the running chunk; a probe that meets
// an equal child there compares sequence numbers (the record's) and takes the entry with a CAS
// when it comes first -- the reference's first occurrence -- marking the holder lost.
// Records of the running chunk: r < 12 Pr is this rank's own child (r = 12 * local parent +
// action, in the arena already), others are received records r - 12 Pr (read from the receive
// buffer; the commit copies the survivors among them to arena position abase + r).  Chunks are
// <= 2^19 parents: seq < 12 * 2^19 < 2^23.
constexpr int POS_SHIFT = 24;
constexpr uint64_t FP_MASK = (1ull << POS_SHIFT) - 1;
constexpr int64_t MAX_CHUNK = 1 << 19;
constexpr int64_t MAX_ARENA = (1ll << (64 - POS_SHIFT)) - 2;  // positions the entry can name
static int64_t g_arena_override = 0;  // tests only (acx_internal_sbfs_arena_cap): a smaller first arena
__device__ __forceinline__ uint64_t entry_of(int64_t pos, uint64_t h) {
    return ((uint64_t)(pos + 1) << POS_SHIFT) | ((h >> 32) & FP_MASK);
}
__device__ __forceinline__ int64_t entry_pos(uint64_t v) { return (int64_t)(v >> POS_SHIFT) - 1; }
__device__ __forceinline__ const uint64_t* rec_key(const Args& a, uint32_t r) {
    const uint32_t n_own = 12u * (uint32_t)a.Pr;
    return r < n_own ? a.ckeys + (int64_t)r * a.kw : a.recv + (int64_t)(r - n_own) * (a.kw + 1);
}
// the chunk seq of record r (its parent's position in the chunk * 12 + action)
__device__ __forceinline__ uint32_t rec_seq(const Args& a, uint32_t r) {
    const uint32_t n_own = 12u * (uint32_t)a.Pr;
    if (r < n_own) return (uint32_t)(a.lgid[a.lo + r / 12u] - a.head) * 12u + r % 12u;
    return (uint32_t)a.recv[(int64_t)(r - n_own) * (a.kw + 1) + a.kw];
}

__device__ __forceinline__ uint32_t owner_of(uint64_t h, int world) {
    return (uint32_t)(((h >> 32) * (uint64_t)world) >> 32);
}

// (1) block per tile of 64 candidate local parents lo + j (j < Pr = min(P, nloc - lo); the
// parents of the chunk are the prefix with gid < head + P); wave w makes the children of actions
// 3w..3w+2 of the same 64 parents (as acx_bfs.hip's bfs_expand_kernel: 4x the lanes of a
// lane-per-parent loop over 12 serial moves), owners counted by ballots.  The block's 64 x 12
// child keys and owners are staged in LDS and written parent-major (the chunk's sequence order)
// as one contiguous run, so the insert and the commit read them in order; for NW > 4 (L > 64,
// 55 KB of keys per block) each lane writes its children directly
constexpr int STILE = 64;
constexpr int SAPW = 12 / (TPB / WAVE);  // actions per wave (3)
template <int NW>
struct ExpandStage {
    static constexpr bool LDS = NW <= 4;
    static constexpr int WORDS = LDS ? STILE * 12 * (NW + 1) : 1;
};
template <int NW>
__global__ __launch_bounds__(TPB, NW <= 4 ? 6 : 4) void sbfs_expand_kernel(Args a) {
    __shared__ uint64_t kst[ExpandStage<NW>::WORDS];
    __shared__ uint8_t cst[STILE * 12];
    __shared__ uint32_t hist[MAXW];
    __shared__ uint32_t smin[STILE];
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    for (int i = threadIdx.x; i < a.world; i += TPB) hist[i] = 0;
    if (wid == 0) smin[lane] = 0xffffu;
    const int j0 = blockIdx.x * STILE;
    const int j = j0 + lane;
    const int64_t gid = j < a.Pr ? a.lgid[a.lo + j] : INT64_MAX;
    const bool live = gid < a.head + a.P;
    const int kw = a.kw;
    const bool cyc = a.cyc != 0;
    PresRegs<NW> pr;
    bool clean = false;
    if (live) {
        load_key<NW>(a.arena + a.lapos[a.lo + j] * kw, kw, a.L, pr);
        clean = is_clean<NW>(pr.w0, pr.n0, pr.w1, pr.n1, cyc);
    }
    __syncthreads();
    const uint32_t p = live ? (uint32_t)(gid - a.head) : 0u;
    uint32_t succ = NONE, err = NONE, mn = 0xffffu;
    uint32_t ownp = 0xffffffu;  // owner byte of action 3w + jj at bits 8 jj (a runtime-indexed
                                // array here would live in scratch: the loop is not unrolled)
    const int nrow = min(STILE, a.Pr - j0);  // the tile's lanes with a local parent slot
#pragma unroll 1
    for (int jj = 0; jj < SAPW; ++jj) {
        const int act = wid * SAPW + jj;
        uint32_t own = 0xff;
        if (live) {
            PresRegs<NW> q = pr;
            const int e = clean ? ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, cyc)
                                : ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, a.L, cyc);
            const uint32_t s = p * 12u + (uint32_t)act;
            if (e != ACX_ERR_NONE) {
                err = min(err, s);
            } else {
                const uint32_t tot = (uint32_t)(q.n0 + q.n1);
                if (tot == 2) succ = min(succ, s);
                mn = min(mn, tot);
            }
            Key<NW + 1> key;
            make_key<NW>(a.L, q, key.w);
            own = owner_of(khash<NW + 1>(key, kw), a.world);
            ownp = (ownp & ~(0xffu << (8 * jj))) | (own << (8 * jj));
            if constexpr (ExpandStage<NW>::LDS) {
#pragma unroll
                for (int k = 0; k < NW + 1; ++k)
                    if (k < kw) kst[(lane * 12 + act) * kw + k] = key.w[k];
            } else {
#pragma unroll
                for (int k = 0; k < NW + 1; ++k)
                    if (k < kw) a.ckeys[((int64_t)j * 12 + act) * kw + k] = key.w[k];
            }
        }
        // a lane whose parent is past the chunk (or has no slot) leaves a stale key; its owner
        // byte 0xff tells pack and insert to skip it
        if constexpr (ExpandStage<NW>::LDS) cst[lane * 12 + act] = (uint8_t)own;
        else if (j < a.Pr) a.cown[(int64_t)j * 12 + act] = (uint8_t)own;
    }
    if constexpr (ExpandStage<NW>::LDS) {
        __syncthreads();
        // the block's children in sequence order: one contiguous run of keys and of owners
        uint64_t* o = a.ckeys + (int64_t)j0 * 12 * kw;
        for (int i = threadIdx.x; i < nrow * 12 * kw; i += TPB) o[i] = kst[i];
        uint8_t* oc = a.cown + (int64_t)j0 * 12;
        for (int i = threadIdx.x; i < nrow * 12; i += TPB) oc[i] = cst[i];
    }
    // per-owner counts: one ballot per (action, owner) and one LDS add per wave
    for (int o = 0; o < a.world; ++o) {
        uint32_t c = 0;
#pragma unroll
        for (int jj = 0; jj < SAPW; ++jj) c += __popcll(__ballot(((ownp >> (8 * jj)) & 0xffu) == (uint32_t)o));
        if (lane == 0 && c) atomicAdd(&hist[o], c);  // LDS
    }
    if (live) atomicMin(&smin[lane], mn);
    succ = wave_min(succ);
    err = wave_min(err);
    if (lane == 0) {  // rare: one global atomic per wave that has one
        if (succ != NONE) atomicMin(&a.ctl->succ_seq, succ);
        if (err != NONE) atomicMin(&a.ctl->err_seq, err);
    }
    __syncthreads();
    // the block's min child total, parent count and owner counts go to its own record, reduced
    // by sbfs_expand_reduce_kernel: a same-address atomic per block serialises in L2 (3 of them
    // per block over the 8,192 blocks of a 2^19-parent chunk cost ~80 us)
    uint32_t* x = a.xblk + (size_t)blockIdx.x * (2 + a.world);
    if (wid == 0) {
        const uint32_t m = smin[lane];
        if (live) a.pmin[j] = (uint16_t)m;
        const uint32_t bmin = wave_min(live ? m : NONE);
        const uint32_t bpar = wave_min(live ? NONE - (uint32_t)(j + 1) : NONE);
        if (lane == 0) {
            x[0] = bmin;
            x[1] = NONE - bpar;  // 1 + last live lane's j, 0 if none
        }
    }
    for (int i = threadIdx.x; i < a.world; i += TPB) x[2 + i] = hist[i];
}

// exclusive scan over a 1024-thread block (sh: 16 words)
__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t* sh, uint32_t& tot) {
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
    }
    if (lane == WAVE - 1) sh[wid] = x;
    __syncthreads();
    uint32_t off = 0;
    tot = 0;
#pragma unroll
    for (int i = 0; i < 1024 / WAVE; ++i) {
        off += i < wid ? sh[i] : 0u;
        tot += sh[i];
    }
    return off + x - v;
}

// (1b) the expand blocks' records -> the chunk's min child total, local parent count and
// children per owner (one block); each block's per-owner count is replaced by its exclusive
// prefix over the blocks, and ctl->cur[o] set to owner o's first send slot, so pack places
// every record without a global atomic
__global__ __launch_bounds__(1024) void sbfs_expand_reduce_kernel(Args a, int nblk) {
    __shared__ uint32_t red[2][1024 / WAVE];
    __shared__ uint32_t tot[MAXW];
    const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
    const int rw = 2 + a.world;
    uint32_t mn = NONE, np = 0;
    for (int b = t; b < nblk; b += 1024) {
        mn = min(mn, a.xblk[(size_t)b * rw]);
        np = max(np, a.xblk[(size_t)b * rw + 1]);
    }
    mn = wave_min(mn);
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) np = max(np, (uint32_t)__shfl_xor((int)np, o, WAVE));
    if (lane == 0) {
        red[0][wid] = mn;
        red[1][wid] = np;
    }
    __syncthreads();
    if (t == 0) {
        for (int w = 1; w < 1024 / WAVE; ++w) {
            mn = min(mn, red[0][w]);
            np = max(np, red[1][w]);
        }
        if (mn != NONE) a.ctl->min_len = min(a.ctl->min_len, mn);
        a.ctl->npar = np;
    }
    // per owner: thread t scans blocks [b0, b1) of a contiguous split
    const int per = (nblk + 1023) / 1024;
    const int b0 = min(nblk, t * per), b1 = min(nblk, b0 + per);
    for (int o = 0; o < a.world; ++o) {
        uint32_t loc = 0;
        for (int b = b0; b < b1; ++b) loc += a.xblk[(size_t)b * rw + 2 + o];
        __syncthreads();  // red reuse
        uint32_t total;
        uint32_t run = block_excl_scan_1024(loc, &red[0][0], total);
        for (int b = b0; b < b1; ++b) {
            uint32_t* x = a.xblk + (size_t)b * rw + 2 + o;
            const uint32_t c = *x;
            *x = run;
            run += c;
        }
        if (t == 0) tot[o] = total;
    }
    __syncthreads();
    if (t == 0) {
        // the rank's own children are inserted where the expansion wrote them: no send group
        uint32_t run = 0;
        for (int o = 0; o < a.world; ++o) {
            const uint32_t c = o == a.rank ? 0u : tot[o];
            a.ctl->cnt[o] = c;
            a.ctl->cur[o] = run;
            run += c;
        }
    }
}

// (2) records into the send buffer, grouped by owner (order within a group is arbitrary:
// the owner indexes records by seq).  Same tiling as the expansion (block per 64 local parents,
// wave w: actions 3w..3w+2): the block's run for owner o starts at cur[o] + its prefix (1b);
// inside the block, per (action, owner) a ballot ranks the lanes and lane 0 reserves the wave's
// run with one LDS add.
__global__ __launch_bounds__(TPB) void sbfs_pack_kernel(Args a) {
    __shared__ uint32_t hist[MAXW];
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    for (int i = threadIdx.x; i < a.world; i += TPB) hist[i] = 0;
    __syncthreads();
    const int j = blockIdx.x * STILE + lane;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t* x = a.xblk + (size_t)blockIdx.x * (2 + a.world) + 2;
    const uint32_t p = j < a.Pr ? (uint32_t)(a.lgid[a.lo + j] - a.head) : 0u;
    const int rw = a.kw + 1;
#pragma unroll 1
    for (int jj = 0; jj < SAPW; ++jj) {
        const int act = wid * SAPW + jj;
        uint32_t o = j < a.Pr ? a.cown[(int64_t)j * 12 + act] : 0xffu;
        if (o == (uint32_t)a.rank) o = 0xffu;  // inserted in place, not sent
        uint32_t pos = 0;
        for (uint32_t w = 0; w < (uint32_t)a.world; ++w) {
            if (w == (uint32_t)a.rank) continue;
            const uint64_t m = __ballot(o == w);
            if (!m) continue;
            uint32_t b = lane == 0 ? atomicAdd(&hist[w], (uint32_t)__popcll(m)) : 0u;  // LDS
            b = (uint32_t)__shfl((int)b, 0, WAVE);
            if (o == w) pos = a.ctl->cur[w] + x[w] + b + (uint32_t)__popcll(m & below);
        }
        if (o == 0xffu) continue;
        const uint64_t* src = a.ckeys + ((int64_t)j * 12 + act) * a.kw;
        uint64_t* dst = a.send + (int64_t)pos * rw;
        for (int k = 0; k < a.kw; ++k) dst[k] = src[k];
        dst[a.kw] = (uint64_t)(p * 12u + (uint32_t)act);
    }
}

// (3a) probe / claim / join, one lane per child this rank owns: its own children in place
// (records r < 12 Pr, ckeys) and the received ones; as acx_bfs.hip's bfs_insert_kernel, the first
// occurrence of a state within the chunk keeps the entry (atomicMin), a child it displaces is
// marked lost
template <int KWM>
__global__ __launch_bounds__(TPB, 8) void sbfs_insert_kernel(Args a) {  // 8 waves/SIMD (latency-bound)
    const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
    const int64_t n_own = 12 * (int64_t)a.Pr;
    if (t >= n_own + a.nrecv) return;
    uint32_t s;
    int64_t r = t;  // the record
    const uint64_t* kp;
    if (t < n_own) {
        // own children in (parent, action) order: consecutive lanes read consecutive keys and
        // write consecutive seqs (sslot, srec)
        const int j = (int)(t / 12);
        const int act = (int)(t - 12 * (int64_t)j);
        if (a.cown[r] != (uint8_t)a.rank) return;  // another rank's child, or a parent past the chunk
        s = (uint32_t)(a.lgid[a.lo + j] - a.head) * 12u + (uint32_t)act;
        kp = a.ckeys + r * a.kw;
    } else {
        kp = a.recv + (r - n_own) * (a.kw + 1);
        s = (uint32_t)kp[a.kw];
    }
    // after the search's last child (its sslot stays SEEN); end_from_ctl: this rank's own first
    // success / move error is the chunk's (one rank: no exchange, no read-back before the insert)
    const uint32_t end = a.end_from_ctl ? min(a.ctl->succ_seq, a.ctl->err_seq) : a.end;
    if (s > end) return;
    const Key<KWM> key = kload<KWM>(kp, a.kw);
    const uint64_t h = khash<KWM>(key, a.kw);
    const uint64_t fp = (h >> 32) & FP_MASK;
    uint64_t idx = h & a.mask;
    const uint64_t my = entry_of(a.abase + r, h);
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
        if ((v & FP_MASK) == fp) {
            const int64_t pos = entry_pos(v);
            if (pos >= a.abase) {  // a child of this chunk
                if (keq<KWM>(rec_key(a, (uint32_t)(pos - a.abase)), key, a.kw)) {
                    // the same state: the smaller seq keeps the entry.  A CAS that fails found
                    // another equal child's entry (only equal states join this slot): compare again
                    while (true) {
                        const uint32_t hs = rec_seq(a, (uint32_t)(entry_pos(v) - a.abase));
                        if (hs < s) break;  // an earlier occurrence holds it
                        const uint64_t old = atomicCAS((unsigned long long*)(a.table + idx), (unsigned long long)v,
                                                       (unsigned long long)my);
                        if (old == v) {  // the previous holder lost
                            a.lost[hs] = 1;
                            res = (uint32_t)idx;
                            break;
                        }
                        v = old;
                    }
                    break;
                }
            } else if (keq<KWM>(a.arena + pos * a.kw, key, a.kw)) {
                break;  // already a node
            }
        }
        idx = (idx + 1) & a.mask;
    }
    a.sslot[s] = res;
    a.srec[s] = (uint32_t)r;
}

// (3b) this rank's survivors per parent -> mask bits (gmask, all-reduced next; mine, kept):
// a child survives if it holds its entry and was not displaced by a smaller seq
__device__ __forceinline__ uint32_t survivor_bits(const Args& a, int p) {
    uint32_t bits = 0;
#pragma unroll
    for (int act = 0; act < 12; ++act) {
        const uint32_t s = (uint32_t)p * 12u + (uint32_t)act;
        if (a.sslot[s] != SEEN && !a.lost[s]) bits |= 1u << act;
    }
    return bits;
}
__global__ __launch_bounds__(TPB) void sbfs_mask_kernel(Args a) {
    const int p = blockIdx.x * TPB + threadIdx.x;
    if (p >= a.P) return;
    const uint32_t bits = survivor_bits(a, p);
    a.gmask[p] = bits;
    a.mine[p] = bits;
}

// (4a) per-block counts of all survivors and of this rank's.  FOLD (one rank, no exchange: the
// mask is this rank's own): the survivor bits are made here, the mask pass is not launched
template <bool FOLD>
__global__ __launch_bounds__(TPB) void sbfs_count_kernel(Args a) {
    __shared__ uint32_t sh[TPB / WAVE];
    const int p = blockIdx.x * TPB + threadIdx.x;
    uint32_t m = 0, mine = 0;
    if (p < a.P) {
        if constexpr (FOLD) {
            m = mine = survivor_bits(a, p);
            a.gmask[p] = m;
            a.mine[p] = m;
        } else {
            m = a.gmask[p];
            mine = a.mine[p];
        }
    }
    uint32_t tot, ltot;
    block_excl_scan(__popc(m), sh, tot);
    __syncthreads();
    block_excl_scan(__popc(mine), sh, ltot);
    if (threadIdx.x == 0) {
        a.bsum[blockIdx.x] = tot;
        a.lbsum[blockIdx.x] = ltot;
    }
}

// (4b) exclusive scans of x[0..nb) and y[0..nb) in place, one block of 1024 (both arrays in one
// launch); the totals into *tx, *ty
__device__ __forceinline__ void scan_1024(uint32_t* x, int nb, uint64_t* total, uint32_t* sh) {
    const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
    const int per = (nb + 1023) / 1024;
    const int b0 = t * per, b1 = min(nb, b0 + per);
    uint32_t loc = 0;
    for (int i = b0; i < b1; ++i) loc += x[i];
    uint32_t v = loc;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, WAVE);
        if (lane >= o) v += y;
    }
    if (lane == WAVE - 1) sh[wid] = v;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < 1024 / WAVE; ++i) {
        off += i < wid ? sh[i] : 0u;
        tot += sh[i];
    }
    uint32_t run = off + v - loc;
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = x[i];
        x[i] = run;
        run += c;
    }
    if (t == 0) *total = tot;
    __syncthreads();  // sh reuse
}
__global__ __launch_bounds__(1024) void sbfs_scan_kernel(uint32_t* x, uint32_t* y, int nb, uint64_t* tx, uint64_t* ty) {
    __shared__ uint32_t sh[1024 / WAVE];
    scan_1024(x, nb, tx, sh);
    scan_1024(y, nb, ty, sh);
}

// (4c) global ids, the budget cut, and the appends to this rank's store.  A block's own
// survivors take consecutive store slots (their global ids ascend with the slot), so each lane
// stages its survivors in LDS at their block-local rank and the block then writes the slot range
// cooperatively as coalesced arrays (ids, parents, moves, arena positions).  Keys stay where they
// are (own children) or are copied from the receive buffer into the arena (received survivors);
// table entries already name them.
constexpr int CMAX = TPB * 12;  // own survivors a block can stage
__global__ __launch_bounds__(TPB) void sbfs_commit_kernel(Args a) {
    __shared__ uint32_t sh[TPB / WAVE];
    __shared__ uint32_t srec[CMAX];  // record of the k-th own survivor
    __shared__ uint32_t sinf[CMAX];  // parent within the block (8 bits) | move (4) | id offset (12)
    const int p = blockIdx.x * TPB + threadIdx.x;
    const uint32_t m = p < a.P ? a.gmask[p] : 0u;
    const uint32_t mine = p < a.P ? a.mine[p] : 0u;
    uint32_t tot;
    const uint32_t bex = block_excl_scan(__popc(m), sh, tot);  // survivors of the block before p
    const int64_t base = (int64_t)a.bsum[blockIdx.x] + bex;
    __syncthreads();
    uint32_t ltot;
    const uint32_t lrank = block_excl_scan(__popc(mine), sh, ltot);
    if (p < a.P) {
        const int64_t incl = base + __popc(m);
        if (incl >= a.need && (base < a.need || p == 0)) {
            a.ctl->cut_p = (uint32_t)p;
            a.ctl->nodes_at_cut = (uint64_t)(a.n_before + incl);
        }
    }
    uint32_t mm = mine, k = lrank;
    while (mm) {
        const int act = __builtin_ctz(mm);
        mm &= mm - 1;
        srec[k] = a.srec[(uint32_t)p * 12u + act];
        sinf[k] = (uint32_t)threadIdx.x << 16 | (uint32_t)act << 12 | (bex + __popc(m & ((1u << act) - 1u)));
        ++k;
    }
    __syncthreads();
    // a node at or past max_nodes + 12 comes after the budget cut and is never used (the
    // single-GPU queue drops it too): the stored ones are a prefix of the slot range
    const int64_t g0 = a.n_before + (int64_t)a.bsum[blockIdx.x];  // id of the block's first survivor
    const int64_t keep_below = a.n_before + a.need + 12;
    const int64_t li0 = a.nloc + (int64_t)a.lbsum[blockIdx.x];
    uint32_t stored = 0;
    for (uint32_t i = threadIdx.x; i < ltot; i += TPB) {
        const uint32_t inf = sinf[i];
        const int64_t gid = g0 + (inf & 0xfffu);
        const int64_t li = li0 + i;
        if (gid >= keep_below) continue;
        if (li >= a.lcap) {
            atomicOr(&a.ctl->overflow, 2u);
            continue;
        }
        ++stored;
        const int64_t pp = (int64_t)blockIdx.x * TPB + (inf >> 16);
        const uint32_t act = (inf >> 12) & 0xfu;
        a.lgid[li] = gid;
        a.lpar[li] = a.head + pp;
        a.lact[li] = (uint8_t)act;
        a.lapos[li] = a.abase + srec[i];
    }
    // received survivors' keys into the arena after the chunk's own children: word w of the
    // block's survivors comes from word w % kw of record srec[w / kw] (own ones: already there)
    const uint32_t n_own = 12u * (uint32_t)a.Pr;
    for (uint32_t w = threadIdx.x; w < ltot * (uint32_t)a.kw; w += TPB) {
        const uint32_t i = w / (uint32_t)a.kw, c = w - i * (uint32_t)a.kw;
        const uint32_t r = srec[i];
        if (r < n_own) continue;
        a.arena[(a.abase + r) * a.kw + c] = a.recv[(int64_t)(r - n_own) * (a.kw + 1) + c];
    }
    uint32_t bs;
    block_excl_scan(stored, sh, bs);  // (its barrier: every read of the block's sslot / srec is done)
    if (threadIdx.x == 0 && bs) atomicAdd(&a.ctl->stored, bs);
    // the block's seqs back to SEEN / not lost for the next chunk (no per-chunk memset);
    // consecutive threads on consecutive seqs
    const uint32_t s0 = (uint32_t)blockIdx.x * TPB * 12u;
    const uint32_t s1 = min((uint32_t)a.P * 12u, s0 + TPB * 12u);
    for (uint32_t sq = s0 + threadIdx.x; sq < s1; sq += TPB) {
        a.sslot[sq] = SEEN;
        a.lost[sq] = 0;
    }
}

// min child total over the local parents of the chunk with p <= last
__global__ __launch_bounds__(TPB) void sbfs_minlen_kernel(Args a, int64_t last, int npar) {
    __shared__ uint32_t sh[TPB / WAVE];
    const int j = blockIdx.x * TPB + threadIdx.x;
    uint32_t v = NONE;
    if (j < npar && a.lgid[a.lo + j] - a.head <= last) v = a.pmin[j];
    v = block_min(v, sh);
    if (threadIdx.x == 0 && v != NONE) atomicMin(&a.ctl->min_len, v);
}

// the total length stored in a packed child key (n0 at bit 4L, n1 at bit 4L + 8)
__device__ __forceinline__ uint32_t key_total(const uint64_t* k, int L) {
    uint32_t t = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int bit = 4 * L + 8 * h, w = bit >> 6, o = bit & 63;
        uint64_t v = k[w] >> o;
        if (o > 56) v |= k[w + 1] << (64 - o);
        t += (uint32_t)(v & 0xffu);
    }
    return t;
}

// verbose trace (breadth_first.py:79-82): this rank's chunk children with seq < end whose total
// is below every earlier child of this rank and below `running` -- the rank's prefix minima, a
// superset of the global new minima that lie on this rank (<= 2L of them).  One block: a min
// scan over contiguous parent ranges (pmin, or the children below `end` for the boundary
// parent), then every range whose running min drops walks its parents' children in order.
constexpr int TRACE_MAX = 512;
__global__ __launch_bounds__(1024) void sbfs_trace_kernel(Args a, int npar, uint32_t running, uint32_t end,
                                                          int64_t* out, int32_t* n_out) {
    __shared__ uint32_t red[1024 / WAVE];
    __shared__ uint32_t cnt;
    const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
    if (t == 0) cnt = 0;
    const int per = (npar + 1023) / 1024;
    const int j0 = min(npar, t * per), j1 = min(npar, j0 + per);
    auto child_total = [&](int j, int act) -> uint32_t {
        return key_total(a.ckeys + ((int64_t)j * 12 + act) * a.kw, a.L);
    };
    auto parent_seq = [&](int j) -> uint32_t { return (uint32_t)(a.lgid[a.lo + j] - a.head) * 12u; };
    uint32_t mn = NONE;
    for (int j = j0; j < j1; ++j) {
        const uint32_t s0 = parent_seq(j);
        if (s0 >= end) break;
        if (s0 + 12u <= end) {
            mn = min(mn, (uint32_t)a.pmin[j]);
        } else {
            for (int act = 0; s0 + act < end; ++act) mn = min(mn, child_total(j, act));
        }
    }
    // exclusive prefix min over the threads' ranges (in parent order = seq order)
    uint32_t x = mn;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, WAVE);
        if (lane >= o) x = min(x, y);
    }
    if (lane == WAVE - 1) red[wid] = x;
    __syncthreads();
    uint32_t before = running;
    for (int i = 0; i < wid; ++i) before = min(before, red[i]);
    const uint32_t xe = (uint32_t)__shfl_up((int)x, 1, WAVE);
    if (lane > 0) before = min(before, xe);
    if (mn < before) {  // this range holds prefix minima: walk it in order
        uint32_t run = before;
        for (int j = j0; j < j1; ++j) {
            const uint32_t s0 = parent_seq(j);
            if (s0 >= end) break;
            if (s0 + 12u <= end && (uint32_t)a.pmin[j] >= run) continue;
            for (int act = 0; act < 12 && s0 + act < end; ++act) {
                const uint32_t tt = child_total(j, act);
                if (tt < run) {
                    run = tt;
                    const uint32_t k = atomicAdd(&cnt, 1u);  // LDS
                    if (k < TRACE_MAX) {
                        out[2 * k] = (int64_t)(s0 + act);
                        out[2 * k + 1] = (int64_t)tt;
                    }
                }
            }
        }
    }
    __syncthreads();
    if (t == 0) *n_out = (int32_t)cnt;
}

// the stored node with global id g: found, parent id, action, total length
template <int NW>
__global__ void sbfs_lookup_kernel(Args a, int64_t g) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t lo = 0, hi = a.nloc;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (a.lgid[mid] < g) lo = mid + 1; else hi = mid;
    }
    a.look[0] = 0;
    if (lo < a.nloc && a.lgid[lo] == g) {
        PresRegs<NW> pr;
        load_key<NW>(a.arena + a.lapos[lo] * a.kw, a.kw, a.L, pr);
        a.look[0] = 1;
        a.look[1] = a.lpar[lo];
        a.look[2] = a.lact[lo];
        a.look[3] = pr.n0 + pr.n1;
    }
}

struct RootKey {
    uint64_t w[ACX_MAX_L / 16 + 2];
};

template <int KWM>
__global__ void sbfs_root_kernel(Args a, RootKey rk) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int k = 0; k < a.kw; ++k) a.arena[k] = rk.w[k];  // passed by value: no host copy
    const Key<KWM> key = kload<KWM>(a.arena, a.kw);
    const uint64_t h = khash<KWM>(key, a.kw);
    a.table[h & a.mask] = entry_of(0, h);
    a.lapos[0] = 0;
    a.lgid[0] = 0;
    a.lpar[0] = -1;
    a.lact[0] = 0xff;
}

// the first n stored nodes' keys, ascending id, into out ((n, kw))
__global__ void sbfs_gather_keys_kernel(Args a, int64_t n, uint64_t* out) {
    const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (t >= n * a.kw) return;
    const int64_t i = t / a.kw, c = t - i * a.kw;
    out[t] = a.arena[a.lapos[i] * a.kw + c];
}

struct Pub {
    Ctl c;
    uint64_t seq;  // the read-back number once c holds that read-back's control block
};

struct Shard {
    int dev = 0, L = 0, kw = 0, cyc = 0, rank = 0, world = 1;
    int64_t lcap = 0, pmax = 0, rcap = 0, nloc = 0, lo = 0;
    int64_t acap = 0, abase = 0;  // arena records allocated / used
    bool fold_mask = false;       // the last insert left the survivor bits to the commit's count
    int P = 0, Pr = 0;
    int64_t head = 0, nrecv = 0;
    uint64_t tsize = 0;
    Args a{};
    Ctl* ctl_host = nullptr;  // the last read-back (host copy)
    Pub* pub = nullptr;       // pinned, coherent: sbfs_publish_kernel writes it
    uint64_t pub_seq = 0;
    int chunk_npar = 0;       // local parents of the last committed chunk
    int64_t* look_host = nullptr;
    void* bounce = nullptr;  // pinned (copy_to_host)
    // a read-back that timed out (sync_ctl) left its kernels on the stream: `fence` is recorded
    // behind them, the shard refuses work (`stalled`) until acx_sbfs_reset has waited for it, and
    // the destructor waits for it before freeing anything those kernels may still use
    hipEvent_t fence = nullptr;
    bool stalled = false;

    ~Shard() {
        if (fence) {
            (void)hipEventSynchronize(fence);
            (void)hipEventDestroy(fence);
        }
        void* ptrs[] = {a.arena, a.lapos, a.lgid, a.lpar, a.lact, a.cown, a.pmin, a.sslot, a.srec,
                        a.lost, a.mine, a.bsum, a.lbsum, a.table, a.ctl, a.look, a.xblk};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        delete ctl_host;
        if (pub) (void)hipHostFree(pub);
        if (look_host) (void)hipHostFree(look_host);
        if (bounce) (void)hipHostFree(bounce);
    }
};

template <class T>
static bool dalloc(T*& p, size_t n) {
    return hipMalloc((void**)&p, n * sizeof(T) + 16) == hipSuccess;
}

static inline int nblocks(int64_t n) { return (int)((n + TPB - 1) / TPB); }

struct ExpandLaunch {
    Shard* S;
    hipStream_t st;
    template <int NW>
    void go() { sbfs_expand_kernel<NW><<<dim3((unsigned)((S->Pr + STILE - 1) / STILE)), dim3(TPB), 0, st>>>(S->a); }
};
struct InsertLaunch {
    Shard* S;
    hipStream_t st;
    template <int NW>
    void go() { sbfs_insert_kernel<NW + 1><<<dim3(nblocks(12 * (int64_t)S->Pr + S->nrecv)), dim3(TPB), 0, st>>>(S->a); }
};
struct RootLaunch {
    Shard* S;
    hipStream_t st;
    RootKey rk;
    template <int NW>
    void go() { sbfs_root_kernel<NW + 1><<<dim3(1), dim3(64), 0, st>>>(S->a, rk); }
};

// the chunk's control block to its initial values (no host copy): at a search's start, and
// after every chunk's commit read-back (sbfs_publish_kernel)
__global__ void sbfs_ctl_init_kernel(Ctl* c) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    ctl_init(c);
}
struct LookupLaunch {
    Shard* S;
    hipStream_t st;
    int64_t g;
    template <int NW>
    void go() { sbfs_lookup_kernel<NW><<<dim3(1), dim3(64), 0, st>>>(S->a, g); }
};

// the control block published to pinned, coherent host memory by a one-wave kernel (the
// sequence number written last, system scope) -- a hipMemcpyAsync of it was a ~9 us blit per
// read-back, two per chunk -- and read by the host's poll
__global__ void sbfs_publish_kernel(Ctl* c, Pub* host, uint64_t seq, int reset) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(c);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&host->c);
    for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += WAVE) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&host->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (reset) ctl_init(c);  // after a chunk's commit: the next chunk's initial values
    }
}

// every read-back: publish, then poll the sequence number (hipStreamSynchronize may sleep and
// wake late; two waits per chunk are on the search's critical path).  Every 4096 polls the
// stream is queried (a failed launch), and a control block not published within 30 s (a kernel
// that does not finish) is an error.
static int sync_ctl(Shard* S, hipStream_t st, int reset = 0) {
    if (S->stalled || hipGetLastError() != hipSuccess) return ACX_E_LAUNCH;
    const uint64_t want = ++S->pub_seq;
    sbfs_publish_kernel<<<dim3(1), dim3(WAVE), 0, st>>>(S->a.ctl, S->pub, want, reset);
    if (hipGetLastError() != hipSuccess) return ACX_E_LAUNCH;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t it = 1;; ++it) {
        if (__atomic_load_n(&S->pub->seq, __ATOMIC_ACQUIRE) == want) break;
        if ((it & 4095) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {  // idle: the slot is final now
                if (__atomic_load_n(&S->pub->seq, __ATOMIC_ACQUIRE) == want) break;
                return ACX_E_LAUNCH;
            }
            if (e != hipErrorNotReady) return ACX_E_LAUNCH;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
                // the kernels are still queued or running: fence them (see Shard::fence)
                if (!S->fence) (void)hipEventCreateWithFlags(&S->fence, hipEventDisableTiming);
                if (S->fence) (void)hipEventRecord(S->fence, st);
                S->stalled = true;
                return ACX_E_LAUNCH;
            }
        }
    }
    memcpy(S->ctl_host, (const void*)&S->pub->c, sizeof(Ctl));
    return ACX_OK;
}

// the arena to at least `need` records (doubling): a copy of the used records into a new
// allocation between chunks; entries hold positions, so nothing else changes
static int grow_arena(Shard* S, int64_t need, hipStream_t st) {
    if (need <= S->acap) return ACX_OK;
    if (need > MAX_ARENA) return ACX_E_ARG;
    int64_t cap = 2 * S->acap > need ? 2 * S->acap : need;
    if (cap > MAX_ARENA) cap = MAX_ARENA;
    uint64_t* p = nullptr;
    if (!dalloc(p, (size_t)(cap * S->kw))) {
        (void)hipGetLastError();
        cap = need;
        if (!dalloc(p, (size_t)(cap * S->kw))) {
            (void)hipGetLastError();
            return ACX_E_LAUNCH;
        }
    }
    if ((S->abase > 0 &&
         hipMemcpyAsync(p, S->a.arena, (size_t)(S->abase * S->kw) * 8, hipMemcpyDeviceToDevice, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess) {  // the old arena's readers are done too
        (void)hipFree(p);
        return ACX_E_LAUNCH;
    }
    (void)hipFree(S->a.arena);
    S->a.arena = p;
    S->acap = cap;
    return ACX_OK;
}

}  // namespace sbfs
}  // namespace acx

using namespace acx::sbfs;

extern "C" {

void* acx_sbfs_create(int32_t L, int64_t local_cap, int64_t chunk_parents, int32_t cyclical, int32_t rank,
                      int32_t world) {
    if (L < 1 || L > ACX_MAX_L || local_cap < 1 || local_cap > (1ll << 30)) return nullptr;
    if (world < 1 || world > MAXW || rank < 0 || rank >= world) return nullptr;
    Shard* S = new (std::nothrow) Shard();
    if (!S) return nullptr;
    if (hipGetDevice(&S->dev) != hipSuccess) { delete S; return nullptr; }
    S->L = L;
    S->kw = acx_key_words(L);
    S->cyc = cyclical != 0;
    S->rank = rank;
    S->world = world;
    S->lcap = local_cap;
    if (chunk_parents <= 0) chunk_parents = MAX_CHUNK;  // tools/bfs_chunk_probe.py: 2^19-2^20 fastest
    if (chunk_parents > MAX_CHUNK) { delete S; return nullptr; }  // seqs < 12 * 2^19 (the per-seq arrays)
    S->pmax = chunk_parents;
    S->rcap = 12 * S->pmax;  // every child of a chunk may have this owner
    uint64_t ts = 1024;
    while (ts < 2 * (uint64_t)(S->lcap + S->rcap)) ts <<= 1;
    if (ts > (1ull << 31)) { delete S; return nullptr; }
    S->tsize = ts;
    Args& a = S->a;
    const int64_t nb = nblocks(S->pmax);
    const int64_t pl = S->pmax < S->lcap ? S->pmax : S->lcap;  // local parents per chunk
    // the arena's first size: 12 records per expanded parent, which is ~2 per node in an AK(n)
    // search (BASELINE config 4: 1.59M parents for 10^7 nodes), plus received records at G > 1,
    // and room for one full chunk; it doubles when a chunk would not fit (grow_arena)
    S->acap = g_arena_override > 0 ? g_arena_override : 1 + 3 * S->lcap + 24 * pl;
    if (S->acap > MAX_ARENA) S->acap = MAX_ARENA;
    bool ok = dalloc(a.arena, (size_t)(S->acap * S->kw)) && dalloc(a.lapos, (size_t)S->lcap) &&
              dalloc(a.lgid, (size_t)S->lcap) && dalloc(a.lpar, (size_t)S->lcap) && dalloc(a.lact, (size_t)S->lcap) &&
              dalloc(a.cown, (size_t)(12 * pl)) &&
              dalloc(a.pmin, (size_t)pl) && dalloc(a.sslot, (size_t)(12 * S->pmax)) &&
              dalloc(a.srec, (size_t)(12 * S->pmax)) && dalloc(a.lost, (size_t)(12 * S->pmax)) &&
              dalloc(a.mine, (size_t)S->pmax) &&
              dalloc(a.bsum, (size_t)nb) && dalloc(a.lbsum, (size_t)nb) && dalloc(a.table, (size_t)ts) &&
              dalloc(a.ctl, 1) && dalloc(a.look, 4) &&
              dalloc(a.xblk, (size_t)((pl + STILE - 1) / STILE + 1) * (2 + world)) &&
              (S->ctl_host = new (std::nothrow) Ctl()) != nullptr &&
              hipHostMalloc((void**)&S->pub, sizeof(Pub), hipHostMallocCoherent) == hipSuccess &&
              hipHostMalloc((void**)&S->look_host, 4 * sizeof(int64_t), hipHostMallocDefault) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        delete S;
        return nullptr;
    }
    memset((void*)S->pub, 0, sizeof(Pub));
    a.mask = ts - 1;
    a.lcap = S->lcap;
    a.L = L;
    a.kw = S->kw;
    a.cyc = S->cyc;
    a.world = world;
    a.rank = rank;
    return S;
}

void acx_sbfs_destroy(void* h) { delete static_cast<Shard*>(h); }

// tests only: the first arena of workspaces created from now on holds 2^log2_cap records
// (0: the normal size), so a search regrows it (grow_arena) many times
void acx_internal_sbfs_arena_cap(int32_t log2_cap) {
    g_arena_override = log2_cap > 0 ? (int64_t)1 << log2_cap : 0;
}

int64_t acx_sbfs_max_records(void* h) {
    Shard* S = static_cast<Shard*>(h);
    return S ? S->rcap : ACX_E_ARG;
}

int32_t acx_sbfs_owner(const int32_t* presentation, int32_t L, int32_t world) {
    if (!presentation || L < 1 || L > ACX_MAX_L || world < 1 || world > MAXW) return ACX_E_ARG;
    constexpr int KM = ACX_MAX_L / 16 + 2;
    const int kw = acx_key_words(L);
    Key<KM> k{};
    pack_key(presentation, L, kw, k.w);
    const uint64_t hv = khash<KM>(k, kw);
    return (int32_t)(((hv >> 32) * (uint64_t)world) >> 32);
}

int acx_sbfs_reset(void* h, const int32_t* presentation, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (!S || !presentation) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (S->stalled) {  // a timed-out read-back: its kernels must be done before the buffers are reused
        if (hipEventSynchronize(S->fence) != hipSuccess) return ACX_E_LAUNCH;
        S->stalled = false;
    }
    const int own = acx_sbfs_owner(presentation, S->L, S->world);
    if (own < 0) return own;
    S->nloc = 0;
    S->lo = 0;
    S->abase = 0;
    S->a.nloc = 0;
    if (hipMemsetAsync(S->a.table, 0, S->tsize * 8, st) != hipSuccess) return ACX_E_LAUNCH;
    // the per-seq arrays are clean between chunks (each commit resets what its chunk used); a
    // search that ended on an error may not have got there
    if (hipMemsetAsync(S->a.sslot, 0xff, (size_t)12 * S->pmax * 4, st) != hipSuccess ||
        hipMemsetAsync(S->a.lost, 0, (size_t)12 * S->pmax, st) != hipSuccess)
        return ACX_E_LAUNCH;
    sbfs_ctl_init_kernel<<<dim3(1), dim3(64), 0, st>>>(S->a.ctl);
    if (own == S->rank) {
        RootLaunch rl{S, st, {}};
        pack_key(presentation, S->L, S->kw, rl.rk.w);
        by_nw(S->L, rl);
        S->nloc = 1;
        S->abase = 1;  // the root's record
    }
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return ACX_E_LAUNCH;
    return own;
}

// out (int64[5 + world]): succ_seq, err_seq, min_len, local parents, overflow, send counts
int acx_sbfs_expand(void* h, int64_t head, int32_t P, int64_t* out, int32_t read_back, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (S && S->stalled) return ACX_E_LAUNCH;  // see Shard::fence
    if (!S || (read_back && !out) || P < 1 || P > S->pmax || head < 0) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    Args& a = S->a;
    S->head = head;
    S->P = P;
    const int64_t avail = S->nloc - S->lo;
    S->Pr = (int)(avail < P ? avail : P);
    a.head = head;
    a.P = P;
    a.Pr = S->Pr;
    a.lo = S->lo;
    a.nloc = S->nloc;
    // the chunk's records: its own children, then (G > 1) up to rcap received ones
    const int r0 = grow_arena(S, S->abase + 12 * (int64_t)S->Pr + (S->world > 1 ? S->rcap : 0), st);
    if (r0 != ACX_OK) return r0;
    a.abase = S->abase;
    a.ckeys = a.arena + S->abase * S->kw;
    // the control block holds its initial values (the search's reset, or the previous chunk's
    // commit read-back re-initialised it)
    if (S->Pr > 0) {
        ExpandLaunch el{S, st};
        by_nw(S->L, el);
        sbfs_expand_reduce_kernel<<<dim3(1), dim3(1024), 0, st>>>(a, (S->Pr + STILE - 1) / STILE);
    }
    if (!read_back) return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
    const int r = sync_ctl(S, st);
    if (r != ACX_OK) return r;
    const Ctl& c = *S->ctl_host;
    out[0] = c.succ_seq;
    out[1] = c.err_seq;
    out[2] = c.min_len;
    out[3] = c.npar;
    out[4] = c.overflow;
    for (int i = 0; i < S->world; ++i) out[5 + i] = c.cnt[i];
    return ACX_OK;
}

// the expanded children into `send` ((sum of counts, kw + 1) uint64), grouped by owner rank
int acx_sbfs_pack(void* h, uint64_t* send, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (S && S->stalled) return ACX_E_LAUNCH;  // see Shard::fence
    if (!S || !send) return ACX_E_ARG;
    uint64_t nsend = 0;  // the counts acx_sbfs_expand read back (the rank's own group is empty)
    for (int o = 0; o < S->world; ++o) nsend += S->ctl_host->cnt[o];
    if (S->Pr == 0 || nsend == 0) return ACX_OK;
    S->a.send = send;
    sbfs_pack_kernel<<<dim3((unsigned)((S->Pr + STILE - 1) / STILE)), dim3(TPB), 0, (hipStream_t)stream>>>(S->a);
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

// this rank's own children (in place) and the received records ((nrecv, kw + 1) uint64) ->
// probe / insert; this rank's survivors as bits of gmask ((P) int32, written here).  end = min(success seq, move-error seq) over all ranks.
int acx_sbfs_insert(void* h, const uint64_t* recv, int64_t nrecv, int64_t end, uint32_t* gmask, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (S && S->stalled) return ACX_E_LAUNCH;  // see Shard::fence
    if (!S || !gmask || nrecv < 0 || nrecv > S->rcap || (nrecv > 0 && !recv)) return ACX_E_ARG;
    if (S->abase + 12 * (int64_t)S->Pr + nrecv > S->acap) return ACX_E_ARG;  // reserved by acx_sbfs_expand
    hipStream_t st = (hipStream_t)stream;
    Args& a = S->a;
    a.recv = recv;
    a.nrecv = nrecv;
    a.gmask = gmask;
    a.end_from_ctl = end < 0;
    a.end = end < 0 || end > (int64_t)NONE ? NONE : (uint32_t)end;
    S->nrecv = nrecv;
    // sslot / lost are SEEN / 0 here: the previous chunk's commit (or the search's reset) cleared them
    if (12 * (int64_t)S->Pr + nrecv > 0) {
        InsertLaunch il{S, st};
        by_nw(S->L, il);
    }
    // one rank with no exchange (end < 0): nobody reads gmask before the commit, whose count pass
    // makes the survivor bits itself (sbfs_count_kernel<true>)
    S->fold_mask = end < 0 && S->world == 1;
    if (!S->fold_mask) sbfs_mask_kernel<<<dim3(nblocks(S->P)), dim3(TPB), 0, st>>>(a);
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

// gmask = the all-reduced survivor masks.  out (int64[5]): nodes appended by the chunk (all
// ranks), cut parent (-1: none), len(tree_nodes) after the cut parent, nodes appended here,
// overflow flags
int acx_sbfs_commit(void* h, const uint32_t* gmask, int64_t n_before, int64_t need, int64_t* out, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (S && S->stalled) return ACX_E_LAUNCH;  // see Shard::fence
    if (!S || !gmask || !out) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    Args& a = S->a;
    a.gmask = (uint32_t*)gmask;
    a.n_before = n_before;
    a.need = need;
    a.nloc = S->nloc;
    const int nb = nblocks(S->P);
    if (S->fold_mask) sbfs_count_kernel<true><<<dim3(nb), dim3(TPB), 0, st>>>(a);
    else sbfs_count_kernel<false><<<dim3(nb), dim3(TPB), 0, st>>>(a);
    S->fold_mask = false;
    sbfs_scan_kernel<<<dim3(1), dim3(1024), 0, st>>>(a.bsum, a.lbsum, nb, &a.ctl->total_new, &a.ctl->local_new);
    sbfs_commit_kernel<<<dim3(nb), dim3(TPB), 0, st>>>(a);
    const int r = sync_ctl(S, st, 1);  // and re-initialise the control block for the next chunk
    if (r != ACX_OK) return r;
    const Ctl& c = *S->ctl_host;
    out[0] = (int64_t)c.total_new;
    out[1] = c.cut_p == NONE ? -1 : (int64_t)c.cut_p;
    out[2] = (int64_t)c.nodes_at_cut;
    out[3] = (int64_t)c.local_new;
    out[4] = c.overflow;
    out[5] = c.succ_seq;  // the chunk's expansion, as acx_sbfs_expand reads it back
    out[6] = c.err_seq;
    out[7] = c.min_len;
    out[8] = c.npar;
    S->nloc += c.stored;
    S->lo += c.npar;
    S->abase += 12 * (int64_t)S->Pr + S->nrecv;  // the chunk's records stay (entries name them)
    S->chunk_npar = (int)c.npar;
    return ACX_OK;
}

// min child total over this rank's parents of the last chunk with chunk index <= last (255: none)
int64_t acx_sbfs_min_len(void* h, int64_t last, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (!S) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(&S->a.ctl->min_len, 0xff, 4, st) != hipSuccess) return ACX_E_LAUNCH;  // NONE
    // lo was advanced by commit past the chunk's local parents
    Args a = S->a;
    a.lo = S->lo - S->chunk_npar;
    if (S->Pr > 0) sbfs_minlen_kernel<<<dim3(nblocks(S->Pr)), dim3(TPB), 0, st>>>(a, last, S->chunk_npar);
    const int r = sync_ctl(S, st);
    if (r != ACX_OK) return r;
    return S->ctl_host->min_len == NONE ? 255 : (int64_t)S->ctl_host->min_len;
}

// verbose trace of the last chunk (call after acx_sbfs_commit): this rank's children with seq <
// end whose total is below `running` and below every earlier child of this rank, as (seq, total)
// int64 pairs into out (HOST, 2 * cap); returns their count (<= 2L + 1 in practice)
int64_t acx_sbfs_trace(void* h, int64_t running, int64_t end, int64_t* out, int64_t cap, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (!S || !out || cap < 0) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    Args a = S->a;
    const int npar = S->chunk_npar;
    a.lo = S->lo - npar;  // commit advanced lo past the chunk's local parents
    if (npar == 0) return 0;
    int64_t* d_out = nullptr;
    int32_t* d_n = nullptr;
    if (hipMalloc((void**)&d_out, 2 * TRACE_MAX * sizeof(int64_t)) != hipSuccess) return ACX_E_LAUNCH;
    if (hipMalloc((void**)&d_n, sizeof(int32_t)) != hipSuccess) {
        (void)hipFree(d_out);
        return ACX_E_LAUNCH;
    }
    const uint32_t run = running < 0 ? 0u : running > (int64_t)NONE ? NONE : (uint32_t)running;
    const uint32_t e = end < 0 ? 0u : end > (int64_t)NONE ? NONE : (uint32_t)end;
    sbfs_trace_kernel<<<dim3(1), dim3(1024), 0, st>>>(a, npar, run, e, d_out, d_n);
    int32_t n = 0;
    int64_t res = ACX_E_LAUNCH;
    if (hipGetLastError() == hipSuccess && copy_to_host(&n, d_n, 4, st, &S->bounce) == ACX_OK) {
        const int64_t m = n < cap ? n : cap;
        const int64_t mm = m < TRACE_MAX ? m : TRACE_MAX;
        if (mm == 0 || copy_to_host(out, d_out, (size_t)(2 * mm) * sizeof(int64_t), st, &S->bounce) == ACX_OK)
            res = n;
    }
    (void)hipFree(d_out);
    (void)hipFree(d_n);
    return res;
}

// node with global id g if this rank stores it: out (int64[4]) = found, parent id, action, total
int acx_sbfs_lookup(void* h, int64_t g, int64_t* out, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (!S || !out) return ACX_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    S->a.nloc = S->nloc;
    LookupLaunch ll{S, st, g};
    by_nw(S->L, ll);
    if (hipGetLastError() != hipSuccess) return ACX_E_LAUNCH;
    if (hipMemcpyAsync(S->look_host, S->a.look, 32, hipMemcpyDeviceToHost, st) != hipSuccess) return ACX_E_LAUNCH;
    if (hipStreamSynchronize(st) != hipSuccess) return ACX_E_LAUNCH;
    for (int i = 0; i < 4; ++i) out[i] = S->look_host[i];
    return ACX_OK;
}

// this rank's stored nodes: keys (cap, kw) and global ids (cap), ascending id; returns the count
int64_t acx_sbfs_node_keys(void* h, uint64_t* keys, int64_t* gids, int64_t cap, void* stream) {
    Shard* S = static_cast<Shard*>(h);
    if (!S) return ACX_E_ARG;
    const int64_t n = S->nloc < cap ? S->nloc : cap;
    hipStream_t st = (hipStream_t)stream;
    if (n > 0 && keys) {
        uint64_t* d = nullptr;
        if (!dalloc(d, (size_t)(n * S->kw))) {
            (void)hipGetLastError();
            return ACX_E_LAUNCH;
        }
        Args a = S->a;
        sbfs_gather_keys_kernel<<<dim3(nblocks(n * S->kw)), dim3(TPB), 0, st>>>(a, n, d);
        const int r = hipGetLastError() == hipSuccess ? copy_to_host(keys, d, (size_t)(n * S->kw) * 8, st, &S->bounce)
                                                      : ACX_E_LAUNCH;
        (void)hipFree(d);
        if (r != ACX_OK) return ACX_E_LAUNCH;
    }
    if (n > 0 && gids && copy_to_host(gids, S->a.lgid, (size_t)n * 8, st, &S->bounce) != ACX_OK)
        return ACX_E_LAUNCH;
    return S->nloc;
}

}  // extern "C"
