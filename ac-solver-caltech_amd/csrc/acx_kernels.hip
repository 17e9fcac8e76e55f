// acx_kernels.hip -- MI355X (gfx950) kernels for the Andrews-Curtis environment hot path.
//
// Design (DESIGN.md has the full story):
//   * HBM holds presentations as (B, 2L) int32 rows (the tensor the Python host owns).
//   * One wavefront handles a tile of 64 envs, one env per lane.  The tile is staged
//     through LDS with coalesced 16-byte loads/stores (a row is 2L int32 = 288 B at
//     L = 36, so a lane reading "its" row directly would touch 64 lines per load);
//     in LDS each letter is one int8, rows padded to an odd number of dwords so the
//     per-lane row reads are bank-conflict free.
//   * Each lane then packs its two relators into registers, 2 bits per letter
//     (x=0, x^-1=1, y=2, y^-1=3, so inversion is `code ^ 1`), as little multiword
//     integers Word<NW> (NW 32-bit words, letter k at bits [2k, 2k+2)).
//   * A move is O(NW) register work, no per-letter loops:
//       concatenate r_i <- r_i r_j^{+-1}  (reference ac_moves.py:4-76): the junction
//         cancellation count is the first non-zero letter of
//         reverse(r_i) XOR r_j^{+-1} XOR 0x55..  (count-trailing-zeros), the splice is
//         mask | shift;
//       conjugate r_i <- g r_i g^-1 (ac_moves.py:79-156): first/last letter tests + splice;
//       free reduction (utils.py:211-220): a SWAR "adjacent inverse pair" mask; the loop
//         only runs when that mask is non-zero, which needs an unreduced input (moves
//         keep reduced words reduced);
//       cyclic reduction (utils.py:223-232): peel count = first non-zero letter of
//         w XOR reverse(w) XOR 0x55.. .
//   * No MFMA: the path is integer/byte work and HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <new>

#include <type_traits>

#include "acx.h"

#include "acx_moves.h"
#include "acx_planes.h"

namespace acx {

// ---------------------------------------------------------------------------------
// LDS staging.  A wave owns a tile of up to 64 consecutive envs.  The tile is moved
// HBM <-> LDS with coalesced 16-byte (or 8-byte) accesses by all 64 lanes, as int8
// letters; then each lane packs / unpacks its own row.  Two implementations with one
// interface:
//   FastTile   compile-time L with L % 4 == 0 (the L = 36 and L = 128 configs): the LDS
//              tile is the int8 image of the global tile, row stride S dwords with
//              S = 2 mod 4 so each lane's 8-byte row reads/writes hit distinct bank
//              pairs; addresses are affine in the chunk index; pack/unpack are SWAR over
//              4 letters per dword.
//   GenericTile  runtime L (parity tests at any L <= 128): per-letter pack/unpack.
// Rows holding a value outside {-2..2} are flagged (flags[row]) at load time.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// int32 letter -> int8; values outside {-2..2} become 0x7F and set `bad`
__device__ __forceinline__ uint32_t to_i8(int32_t v, bool& bad) {
    const bool ok = (uint32_t)(v + 2) <= 4u;
    bad |= !ok;
    return ok ? ((uint32_t)v & 0xffu) : 0x7fu;
}

__device__ __forceinline__ int4 widen4(uint32_t p) {
    int4 x;
    x.x = (int32_t)(int8_t)(p & 0xffu);
    x.y = (int32_t)(int8_t)((p >> 8) & 0xffu);
    x.z = (int32_t)(int8_t)((p >> 16) & 0xffu);
    x.w = (int32_t)(int8_t)(p >> 24);
    return x;
}


constexpr int STAGE_UNROLL = 8;
// Cache-policy choices, each settled by an interleaved A/B on one buffer set (the measurements
// are cited where each is used; the losing variants live in commit history, not here):
//   * the rollout's write-once trajectory: non-temporal / sc1 stores (1.4 % faster at T = 200);
//     its reward/done/truncated stay plain (non-temporal cost 0.4 %);
//   * the in-place step's write-back of changed relators: non-temporal (L = 36) or an sc1
//     buffer store (L = 128); whole output rows stay plain;
//   * tile loads: non-temporal for the L = 128 step and the rollout's state in, plain for the
//     L = 36 step; expand12's parent loads and key stores non-temporal.
constexpr bool NT_OBS = true;

typedef int v4i_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ void st16(int4* p, const int4& v) {
    if constexpr (NT) {
        const v4i_t x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(p));
    } else {
        *p = v;
    }
}
// 16 bytes of a row: int32 letters, or (F32) the same letters as float32 (the PPO learner's
// observation buffer, training.py:151-153)
template <bool NT, bool F32>
__device__ __forceinline__ void out16(int4* p, const int4& v) {
    if constexpr (F32) {
        typedef float v4f_t __attribute__((ext_vector_type(4)));
        const v4f_t f = {(float)v.x, (float)v.y, (float)v.z, (float)v.w};
        if constexpr (NT) __builtin_nontemporal_store(f, reinterpret_cast<v4f_t*>(p));
        else *reinterpret_cast<v4f_t*>(p) = f;
    } else {
        st16<NT>(p, v);
    }
}
template <bool F32>
__device__ __forceinline__ void out8(int2* p, const int2& v) {
    if constexpr (F32) {
        float2 f;
        f.x = (float)v.x;
        f.y = (float)v.y;
        *reinterpret_cast<float2*>(p) = f;
    } else {
        *p = v;
    }
}
template <bool NT, class T>
__device__ __forceinline__ void st_scalar(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// 4 int8 letters (one dword) -> 8-bit code field (2 bits per letter, x=0 X=1 y=2 Y=3, zero
// letters -> 0) and a 4-bit non-zero mask.  A letter's low 3 bits index an 8-entry byte table
// (v_perm_b32: 0 -> 0, 1 (x), 2 (y), 6 (Y = -2), 7 (X = -1)), and v_dot4_u32_u8 folds the four
// per-byte results into their fields (weights 1, 4, 16, 64 for the codes, 1, 2, 4, 8 for the
// mask): 6 VALU where a shift-and-mask SWAR took ~16.  Bytes outside {0, +-1, +-2} give
// arbitrary codes (their rows are flagged and never decoded from the tile); 0x7F, to_i8's
// out-of-domain byte, counts as non-zero.
__device__ __forceinline__ void pack4_codes(uint32_t d, uint32_t& c8, uint32_t& nz4) {
    const uint32_t m = d & 0x07070707u;
    const uint32_t codes = __builtin_amdgcn_perm(0x01030000u, 0x00020000u, m);
    const uint32_t nz = __builtin_amdgcn_perm(0x01010101u, 0x01010100u, m);
    c8 = __builtin_amdgcn_udot4(codes, 0x40100401u, 0u, false);
    nz4 = __builtin_amdgcn_udot4(nz, 0x08040201u, 0u, false);
}

// Non-temporal stores for the in-place step's write-back of changed relators: nothing reads
// those lines again inside the launch, and plain stores kept them in L2 beside the tile loads
// (same buffers: L = 128 0.2727 -> 0.2581 ms, lengths-carrying 0.2302 -> 0.2102, L = 36
// 0.0742 -> 0.0697; profiles/r04/r04z_ab_nt*.json).  Whole output rows (the out-of-place step,
// the rollout's final state, canonicalized rows, expanded children) stay plain: non-temporal
// made the rollout slower (K = 20 int32 1.332 -> 1.351 ms, int8 0.447 -> 0.477; its next launch
// reads that state) and expand12's children no faster (0.778 -> 0.772 ms).
constexpr bool NT_WRITEBACK = true;
constexpr bool NT_STATE = false;
// Buffer-instruction cache policies (gfx950 cpol bits: sc0 1, nt 2, sc1 16).
// The L = 128 in-place step's write-back (CodeTile): sc1, same buffers: lengths-carrying 0.1993 ->
// 0.1791 ms, acx_step 0.2423 -> 0.2182 against nt; nt + sc1 0.1989 (profiles/r04/r04s_ab_wb_cpol.json).
// FastTile (L = 36) keeps the global non-temporal write-back: sc1 measured 0.0757 vs nt 0.0698 ms
// per 2^20-env step (r04s_ab_wb36_cpol.json).
constexpr int WB_CPOL = 16;
// The rollout's int32 trajectory stores (full tiles): sc1 (the line is not kept in the XCD's L2):
// same buffers, K = 20 on Samsung boxes 1.2377 -> 1.2059 and 1.3241 -> 1.3027 ms against nt,
// plain 1.2267 / 1.3195; K = 200 within 0.3 % (profiles/r04/r04s_ab_obs_cpol*.json).  The int8
// trajectory keeps global non-temporal stores: K = 20 0.4626 ms vs sc1 0.4862, plain 0.494
// (r04s_ab_obs8_cpol.json).
constexpr int OBS_CPOL = 16;
// expand12's parent loads and packed-key stores non-temporal (keys as 16-B stores): same buffers,
// 4M parents (profiles/r04/r04z_ab_keys.json): 0.4246 ms (0.71 of 8 TB/s) -> 0.380 ms (0.79) with
// both; the loads alone 0.4085, the stores alone 0.5101 (slower); the children kernel unchanged
constexpr bool NT_EXPAND_LOADS = true;
constexpr bool NT_KEYS = true;
// Non-temporal tile loads (NTL): the state rows are read once per launch.  Taken where it
// measured faster (same buffers, profiles/r04/r04z_ab_ld*.json): the L = 128 step (CodeTile:
// 0.2587 -> 0.2432 ms, lengths-carrying 0.2105 -> 0.1991) and the rollout's state in (int8
// trajectory 0.4635 -> 0.4402 ms, int32 1.3235 -> 1.3131); not the L = 36 step, whose write-back
// of relators that are not sector-aligned (288-B rows) then went 0.0699 -> 0.0944 ms.
template <bool NT>
__device__ __forceinline__ int4 ld_tile(const int4* p) {
    if constexpr (NT) {
        const v4i_t x = __builtin_nontemporal_load(reinterpret_cast<const v4i_t*>(p));
        return make_int4(x[0], x[1], x[2], x[3]);
    } else {
        return *p;
    }
}
constexpr int tile_cpol(bool nt) { return nt ? 2 : 0; }  // buffer-load cache policy: nt (gfx94x/950 bits)
// 16 bytes of a row (4 int32 letters) -> the dword of their low bytes (2 v_perm_b32 + or);
// bad = a letter outside {-2..2} (max / min of the four).  A bad chunk's bytes are arbitrary:
// its row is flagged and never decoded from the tile.
__device__ __forceinline__ uint32_t chunk_i8(const int4& v, bool& bad) {
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v.y, (uint32_t)v.x, 0x0c0c0400u);  // x.b0, y.b0
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v.w, (uint32_t)v.z, 0x04000c0cu);  // z.b0, w.b0
    const int mx = max(max(v.x, v.y), max(v.z, v.w));
    const int mn = min(min(v.x, v.y), min(v.z, v.w));
    bad = mx > 2 || mn < -2;
    return lo | hi;
}

// chunk_i8 with the range test folded into a running max / min of the letters (two v_max3 and
// two v_min3 per chunk, no compare): some letter is outside {-2..2} <=> mx > 2 or mn < -2
__device__ __forceinline__ uint32_t chunk_i8_acc(const int4& v, int& mx, int& mn) {
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)v.y, (uint32_t)v.x, 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)v.w, (uint32_t)v.z, 0x04000c0cu);
    mx = max(max(mx, v.x), v.y);
    mx = max(max(mx, v.z), v.w);
    mn = min(min(mn, v.x), v.y);
    mn = min(min(mn, v.z), v.w);
    return lo | hi;
}

// 8-bit code field -> 4 int8 letters, the first s/8 kept (s = 8m, m = 0..4), the rest zero.
// The four 2-bit codes are spread to one per byte (two shift-or-mask rounds); a byte past m
// gets selector bit 2 set, so one v_perm_b32 reads either the letter table {1,-1,2,-2}
// (src1 bytes 0..3) or zero (src0 bytes 4..7).  ~7 full-rate VALU ops per 4 letters.
__device__ __forceinline__ uint32_t codes_to_i8x4(uint32_t c8, uint32_t s) {
    uint32_t x = (c8 | (c8 << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    const uint32_t z = (uint32_t)(0x04040404ull << s);  // 0x04 in bytes >= m (s = 32 -> none)
    return __builtin_amdgcn_perm(0u, 0xFE02FF01u, x | z);
}
__device__ __forceinline__ uint32_t clamp_bits(int s) { return (uint32_t)(s < 0 ? 0 : (s > 32 ? 32 : s)); }

// Rows outside the packed domain (a letter not in {-2..2}, a zero inside a relator) cannot be
// held in the LDS image; the stores copy their exact int32 values from a fallback row instead,
// chosen per row by its code in the tile's flags[]:
//   FB_IN     the row the kernel loaded (state_in / the rollout's input state)
//   FB_RESET  the env's starting row (reset_state): an autoreset to an out-of-domain row
constexpr uint32_t FB_IN = 1u, FB_RESET = 2u;
__device__ __forceinline__ const int32_t* fb_src(uint32_t code, const int32_t* fb_in, const int32_t* fb_reset) {
    return code == FB_RESET ? fb_reset : fb_in;
}

template <int NW, int LC>
struct FastTile {
    static_assert(LC > 0 && LC % 4 == 0, "FastTile needs a compile-time L multiple of 4");
    static constexpr int L = LC;
    static constexpr int twoL = 2 * LC;
    static constexpr int CPR = LC / 2;  // 16-byte chunks (4 letters) per row
    static constexpr int S = (CPR % 4 == 2) ? CPR : CPR + 2;  // LDS row stride (dwords), = 2 mod 4
    static constexpr int HALF = CPR / 2;  // dwords per relator
    static_assert(S % 4 == 2, "row stride must be 2 mod 4 dwords");
    static constexpr int LOAD_BATCH = 6;

    uint32_t* lds;
    uint8_t* flags;
    uint8_t* dirty;         // per row: bit h = relator h differs from the loaded row (store_dirty)
    uint8_t* lim;           // per row and relator, lengths-carrying step: live 16-byte chunks (lim[2r + h])
    bool tile_bad = false;  // wave-uniform: some row of the last load was flagged

    static __host__ __device__ constexpr size_t wave_bytes(int) { return (size_t)WAVE * S * 4 + 4 * WAVE; }
    // per-row fallback codes (FB_* below) replacing whatever the loads left in flags[]; the
    // flagged rows of store<true> / store_dirty / store_rows_i8_fb copy their fallback row
    __device__ __forceinline__ void restore_flags(int lane, uint32_t code) {
        flags[lane] = (uint8_t)code;
        tile_bad = __any(code != 0u);
        wave_sync();
    }
    // additionally flag the rows of lanes with code != 0
    __device__ __forceinline__ void flag_rows(int lane, uint32_t code) {
        if (code) flags[lane] = (uint8_t)code;
        tile_bad = tile_bad || __any(code != 0u);
    }
    // int8 letter k of row r of the LDS image (the rare fallback stores)
    __device__ __forceinline__ int32_t letter(int r, int k) const { return row(r)[k]; }
    __device__ __forceinline__ FastTile(char* base, int) {
        lds = reinterpret_cast<uint32_t*>(base);
        flags = reinterpret_cast<uint8_t*>(base + WAVE * S * 4);
        dirty = flags + WAVE;
        lim = flags + 2 * WAVE;
    }
    // lengths-carrying step: row `lane` has relators of n0 / n1 letters -> its live chunk counts
    __device__ __forceinline__ void set_lim(int lane, int n0, int n1) const {
        lim[2 * lane] = (uint8_t)live_chunks(n0);
        lim[2 * lane + 1] = (uint8_t)live_chunks(n1);
    }
    __device__ __forceinline__ static int live_chunks(int n) { return n <= 0 ? 0 : n >= L ? HALF : (n + 3) >> 2; }
    // before the store: the live chunks of the row's old (set_lim) or new letters n0 / n1
    __device__ __forceinline__ void widen_lim(int lane, int n0, int n1) const {
        const int a = live_chunks(n0), b = live_chunks(n1);
        if (a > lim[2 * lane]) lim[2 * lane] = (uint8_t)a;
        if (b > lim[2 * lane + 1]) lim[2 * lane + 1] = (uint8_t)b;
    }
    // chunk k (< CPR) of row r is live (inside its relator's letters)
    __device__ __forceinline__ bool live(int r, int k) const {
        const int h = k >= HALF ? 1 : 0;
        return k - h * HALF < lim[2 * r + h];
    }
    __device__ __forceinline__ int Lr() const { return L; }
    __device__ __forceinline__ int8_t* row(int r) const { return reinterpret_cast<int8_t*>(lds + r * S); }

    // LDS dword index of chunk c = lane + 64u (compile-time u)
    __device__ __forceinline__ static int lds_index(int ln, int u) {
        if constexpr (S == CPR) return ln + WAVE * u;           // unpadded: LDS image is flat
        else if constexpr (CPR == WAVE) return u * S + ln;      // one row per wave-instruction
        else {
            const int c = ln + WAVE * u;
            const int r = c / CPR;
            return r * S + (c - r * CPR);
        }
    }

    // global rows (contiguous, 2L int32 each) -> LDS (PIPE: see CodeTile::load; this full-tile
    // loop is unrolled already).  LIVE (the lengths-carrying step; lim[] set for every row): only
    // the chunks inside each relator's letters are read, the rest of the image is zero (the rows
    // are canonical: letters, then zero padding)
    template <bool PIPE = false, bool LIVE = false, bool NTL = false, int BATCH = 0>
    __device__ __forceinline__ void load(const int32_t* __restrict__ g, int R, int lane) {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // keep the address math here (no hoisting into the caller)
        flags[ln] = 0;
        wave_sync();
        const int nc = R * CPR;
        const int4* src = reinterpret_cast<const int4*>(g) + ln;
        bool any_bad = false;
        if (R == WAVE) {  // full tile (wave-uniform): unguarded, LOAD_BATCH loads in flight
            // LIVE: loads through a buffer descriptor over the tile's rows, a dead chunk at an
            // out-of-range offset (zeros, nothing read): no load under a branch (see CodeTile::load)
            const uint64_t gb = reinterpret_cast<uint64_t>(g);
            const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)gb);
            const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32));
            const __amdgpu_buffer_rsrc_t rows = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<void*>(((uint64_t)ghi << 32) | glo), (short)0, WAVE * CPR * 16, 0x00020000);
            // BATCH (the small-batch step instance): loads in flight per batch, up to the whole
            // tile row (CPR: one round trip); LOAD_BATCH otherwise (the 8-wave/SIMD VGPR budget)
            constexpr int LB = BATCH > 0 ? BATCH : LOAD_BATCH;
#pragma unroll
            for (int u0 = 0; u0 < CPR; u0 += LB) {
                int4 v[LB];
                bool lv[LB];
#pragma unroll
                for (int u = 0; u < LB; ++u) {
                    if (u0 + u >= CPR) continue;
                    const int c = ln + (u0 + u) * WAVE;
                    lv[u] = true;
                    if constexpr (LIVE) {
                        const uint32_t off = live(c / CPR, c % CPR) ? (uint32_t)c * 16u : 0x80000000u;
                        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rows, off, 0, tile_cpol(NTL));
                        v[u] = make_int4((int)x[0], (int)x[1], (int)x[2], (int)x[3]);
                    } else {
                        v[u] = ld_tile<NTL>(src + (u0 + u) * WAVE);
                    }
                }
#pragma unroll
                for (int u = 0; u < LB; ++u) {
                    if (u0 + u >= CPR) continue;
                    bool bad = false;
                    uint32_t p = 0;
                    if (lv[u]) p = chunk_i8(v[u], bad);
                    lds[lds_index(ln, u0 + u)] = p;
                    if (bad) flags[(ln + (u0 + u) * WAVE) / CPR] = 1;
                    any_bad |= bad;
                }
            }
        } else {
            for (int u = 0; u < CPR; ++u) {
                const int c = ln + u * WAVE;
                if (c < nc) {
                    const int r = c / CPR;
                    bool bad = false;
                    uint32_t p = 0;
                    if (!LIVE || live(r, c - r * CPR)) {
                        const int4 v = ld_tile<NTL>(src + u * WAVE);
                        p = to_i8(v.x, bad) | (to_i8(v.y, bad) << 8) | (to_i8(v.z, bad) << 16) | (to_i8(v.w, bad) << 24);
                    }
                    lds[r * S + (c - r * CPR)] = p;
                    if (bad) flags[r] = 1;
                    any_bad |= bad;
                }
            }
        }
        tile_bad = __any(any_bad);
        wave_sync();
        if (tile_bad) {
            // rare (wave-uniform): chunk_i8 left arbitrary bytes in the flagged rows; their image
            // is rebuilt with to_i8 (an out-of-domain letter -> 0x7f), so the letter counts the
            // contract reports for them (reward, lengths) are those of the input row
            if (ln < R && flags[ln]) {
                const int4* row = reinterpret_cast<const int4*>(g) + (int64_t)ln * CPR;
                for (int k = 0; k < CPR; ++k) {
                    if (LIVE && !live(ln, k)) continue;
                    const int4 v = row[k];
                    bool b = false;
                    lds[ln * S + k] = to_i8(v.x, b) | (to_i8(v.y, b) << 8) | (to_i8(v.z, b) << 16) | (to_i8(v.w, b) << 24);
                }
            }
            wave_sync();
        }
    }

    // all BLOCK threads load R rows into this tile (the block's one): consecutive threads on
    // consecutive 16-byte chunks, every load issued before any conversion; flags as load().
    // Block-wide barriers before and after (the expand kernels' shared parent tile: a quarter of
    // the per-lane round trips of one wave loading all 64 rows while three wait).
    __device__ __forceinline__ void load_block(const int32_t* __restrict__ g, int R) {
        constexpr int U = (WAVE * CPR + BLOCK - 1) / BLOCK;
        if (threadIdx.x < WAVE) flags[threadIdx.x] = 0;
        __syncthreads();
        const int nc = R * CPR;
        const int4* src = reinterpret_cast<const int4*>(g);
        int4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = (int)threadIdx.x + u * BLOCK;
            if (c < nc) v[u] = ld_tile<NT_EXPAND_LOADS>(src + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = (int)threadIdx.x + u * BLOCK;
            if (c >= nc) continue;
            bool bad = false;
            const uint32_t q = to_i8(v[u].x, bad) | (to_i8(v[u].y, bad) << 8) | (to_i8(v[u].z, bad) << 16) |
                               (to_i8(v[u].w, bad) << 24);
            const int r = c / CPR;
            lds[r * S + (c - r * CPR)] = q;
            if (bad) flags[r] = 1;
        }
        __syncthreads();
    }

    // the rows of the lanes in the wave-uniform mask `rows` only (a few resetting envs),
    // cooperatively: lane l loads 16-byte chunk l % CPR of the (l / CPR)-th selected row, so a
    // wave-instruction fetches 64 / CPR whole rows (3 at L = 36) with one round trip per group
    __device__ __forceinline__ void load_rows(const int32_t* __restrict__ g, uint64_t rows, int R, int lane) {
        load_rows_from([&](int r) { return g + (int64_t)r * twoL; }, rows, R, lane);
    }
    // rp(r): row r's source (called by every lane of the wave: it may read across lanes)
    template <class RowPtr>
    __device__ __forceinline__ void load_rows_from(RowPtr rp, uint64_t rows, int, int lane) {
        constexpr int RPI = WAVE / CPR;
        static_assert(RPI >= 1, "a row must fit one wave-instruction");
        const int s = lane / CPR, c = lane - s * CPR;
        const int n = __popcll(rows);
        if ((rows >> lane) & 1ull) flags[lane] = 0;
        wave_sync();
        bool any_bad = false;
        for (int k0 = 0; k0 < n; k0 += RPI) {
            const int k = k0 + s;
            const bool on = s < RPI && k < n;
            uint64_t m = rows;
            for (int i = 0; i < (on ? k : 0); ++i) m &= m - 1;
            const int r = __builtin_ctzll(m);
            const int32_t* row_src = rp(r);
            if (on) {
                const int4 v = reinterpret_cast<const int4*>(row_src)[c];
                bool bad = false;
                lds[r * S + c] = to_i8(v.x, bad) | (to_i8(v.y, bad) << 8) | (to_i8(v.z, bad) << 16) |
                                 (to_i8(v.w, bad) << 24);
                if (bad) flags[r] = 1;
                any_bad |= bad;
            }
        }
        tile_bad = tile_bad || __any(any_bad);
        wave_sync();
    }

    // load_rows in two halves, for rows known before they are needed (an env step's truncations:
    // step_count + 1 >= horizon before the move): fetch_rows issues the loads of the rows in the
    // wave-uniform mask `rows` (at most RPI of them: one wave-instruction) and returns each lane's
    // chunk; put_rows later writes the rows in `apply` (a subset) into the tile, as load_rows does
    static constexpr bool PREFETCH_OK = true;
    static constexpr bool LIVE_ROWS = true;  // set_lim selects the chunks a live load reads
    static constexpr int RPI = WAVE / CPR;  // rows per wave-instruction
    __device__ __forceinline__ int4 fetch_rows(const int32_t* __restrict__ g, uint64_t rows, int lane) const {
        const int s = lane / CPR, c = lane - s * CPR;
        uint64_t m = rows;
        for (int i = 0; i < (s < RPI ? s : 0); ++i) m &= m - 1;
        int4 v = {0, 0, 0, 0};
        if (s < RPI && m) v = reinterpret_cast<const int4*>(g + (int64_t)__builtin_ctzll(m) * twoL)[c];
        return v;
    }
    __device__ __forceinline__ void put_rows(const int4& v, uint64_t rows, uint64_t apply, int lane) {
        const int s = lane / CPR, c = lane - s * CPR;
        uint64_t m = rows;
        for (int i = 0; i < (s < RPI ? s : 0); ++i) m &= m - 1;
        if ((apply >> lane) & 1ull) flags[lane] = 0;
        wave_sync();
        bool bad = false;
        if (s < RPI && m) {
            const int r = __builtin_ctzll(m);
            if ((apply >> r) & 1ull) {
                lds[r * S + c] = to_i8(v.x, bad) | (to_i8(v.y, bad) << 8) | (to_i8(v.z, bad) << 16) |
                                 (to_i8(v.w, bad) << 24);
                if (bad) flags[r] = 1;
            }
        }
        tile_bad = tile_bad || __any(bad);
        wave_sync();
    }

    template <bool NT, bool F32, bool FULL, int UB = 0, int UE = CPR>
    __device__ __forceinline__ void store_flat(int4* dst, int ln, int nc) const {
#pragma unroll
        for (int u0 = UB; u0 < UE; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u)
                if (u0 + u < UE && (FULL || ln + (u0 + u) * WAVE < nc)) p[u] = lds[lds_index(ln, u0 + u)];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u)
                if (u0 + u < UE && (FULL || ln + (u0 + u) * WAVE < nc))
                    out16<NT, F32>(dst + (u0 + u) * WAVE, widen4(p[u]));
        }
    }

    // LDS -> R contiguous global rows, EXACTLY CPR store instructions on every path (a partial
    // tile's spare lanes re-store its last chunk, same data to the same address), so the
    // compiler's waitcnt pass can count them (rollout_kernel's one-step-ahead action load).
    // [UB, UE): a range of the lane's chunk slots only (the rollout's split obs store)
    static constexpr bool NT_STEP_LOADS = false;  // see ld_tile
    template <bool NT, int UB = 0, int UE = CPR>
    __device__ __forceinline__ void store_rows(int32_t* g, int R, int lane) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        int4* dst = reinterpret_cast<int4*>(g);
        const int nc = R * CPR;
        if (R == WAVE) {
            if constexpr (NT) {  // the trajectory store with an explicit cache policy (OBS_CPOL)
                const uint64_t b = reinterpret_cast<uint64_t>(g);
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
                const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, WAVE * CPR * 16, 0x00020000);
#pragma unroll
                for (int u0 = UB; u0 < UE; u0 += STAGE_UNROLL) {
                    uint32_t p[STAGE_UNROLL];
#pragma unroll
                    for (int u = 0; u < STAGE_UNROLL; ++u)
                        if (u0 + u < UE) p[u] = lds[lds_index(ln, u0 + u)];
#pragma unroll
                    for (int u = 0; u < STAGE_UNROLL; ++u)
                        if (u0 + u < UE) {
                            const int4 v = widen4(p[u]);
                            const v4i_t x = {v.x, v.y, v.z, v.w};
                            __builtin_amdgcn_raw_buffer_store_b128(x, rs, (uint32_t)(ln + (u0 + u) * WAVE) * 16u, 0,
                                                                   OBS_CPOL);
                        }
                }
                return;
            }
            store_flat<NT, false, true, UB, UE>(dst + ln, ln, nc);
            return;
        }
#pragma unroll
        for (int u0 = UB; u0 < UE; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
            int cc[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                if (u0 + u >= UE) continue;
                const int c0 = ln + (u0 + u) * WAVE;
                const int c = c0 < nc ? c0 : nc - 1;
                const int r = c / CPR;
                cc[u] = c;
                p[u] = lds[r * S + (c - r * CPR)];
            }
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u)
                if (u0 + u < UE) out16<NT, false>(dst + cc[u], widen4(p[u]));
        }
    }

    // LDS -> R contiguous global rows as int8 letters (the observation_space dtype,
    // ac_env.py:64-70): the tile's LDS image IS the int8 tile, so a 16-byte LDS read is a
    // 16-byte global store; 2L bytes per row, (R * 2L) / 16 stores per wave (4.5 per lane at L = 36)
    template <bool NT>
    __device__ __forceinline__ void store_rows_i8(int8_t* g, int R, int lane) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nd = R * CPR;  // dwords of the int8 tile
        uint32_t* dst = reinterpret_cast<uint32_t*>(g);
        // rows are 2L = 8m bytes: a tile starts 16-byte aligned unless m and the row index are
        // both odd (L = 36 with an odd batch), then dword stores (wave-uniform branch)
        const bool al = (reinterpret_cast<uintptr_t>(g) & 15u) == 0;
        if constexpr (S == CPR) {
            if (R == WAVE && al) {
                // full aligned tile (wave-uniform; every step of a full batch): one 16-byte LDS
                // read and one 16-byte store per lane and chunk, no per-dword guards (the general
                // loop below costs ~150 VALU per wave-step at L = 36)
                constexpr int ND = WAVE * CPR;
#pragma unroll
                for (int u = 0; u < (ND + 4 * WAVE - 1) / (4 * WAVE); ++u) {
                    const int d0 = 4 * (ln + u * WAVE);
                    if ((u + 1) * 4 * WAVE > ND && d0 >= ND) continue;  // the last, partial chunk row
                    const v4i_t x = *reinterpret_cast<const v4i_t*>(lds + d0);
                    if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(dst + d0));
                    else *reinterpret_cast<v4i_t*>(dst + d0) = x;
                }
                return;
            }
        }
#pragma unroll
        for (int u = 0; u < (WAVE * CPR + 4 * WAVE - 1) / (4 * WAVE); ++u) {
            const int d0 = 4 * (ln + u * WAVE);
            if (d0 >= nd) continue;
            uint32_t v[4];
            if constexpr (S == CPR) {
                // flat image: one 16-byte LDS read per lane, consecutive lanes consecutive
                // 16 bytes (per-dword reads at a 16-byte lane stride were 8-way bank conflicts)
                if (d0 + 4 <= nd) {
                    const uint4 x = *reinterpret_cast<const uint4*>(lds + d0);
                    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = lds[d0 + j < nd ? d0 + j : d0];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int d = d0 + j < nd ? d0 + j : d0;
                    const int r = d / CPR;
                    v[j] = lds[r * S + (d - r * CPR)];
                }
            }
            if (al && d0 + 4 <= nd) {
                const v4i_t x = {(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
                if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(dst + d0));
                else *reinterpret_cast<v4i_t*>(dst + d0) = x;
            } else {
                for (int j = 0; j < 4 && d0 + j < nd; ++j) dst[d0 + j] = v[j];
            }
        }
    }

    // LDS -> global rows with row pitch `gpitch` int32; FB: flagged rows copied from their
    // fallback row (fb_src: `fallback`, or `fallback2` for FB_RESET rows; both pitch fpitch)
    // skip (wave-uniform): rows left unwritten (the learner's finished envs when the curriculum
    // table surely lasts the launch: their copy writes them, step_body)
    template <bool FB, bool NT = false, bool F32 = false>
    __device__ __forceinline__ void store(int32_t* g, int64_t gpitch, int R, const int32_t* fallback,
                                          int64_t fpitch, int lane, const int32_t* fallback2 = nullptr,
                                          uint64_t skip = 0) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nc = R * CPR;
        if (gpitch == twoL && !(FB && tile_bad)) {
            // contiguous rows, nothing flagged: chunk c goes to g + 4c (immediate offsets); a
            // full tile (wave-uniform) needs no per-chunk guards
            int4* dst = reinterpret_cast<int4*>(g) + ln;
            if (skip) {  // the row of chunk c is c / CPR: one test against the scalar mask per chunk
#pragma unroll
                for (int u0 = 0; u0 < CPR; u0 += STAGE_UNROLL) {
                    uint32_t p[STAGE_UNROLL];
#pragma unroll
                    for (int u = 0; u < STAGE_UNROLL; ++u)
                        if (u0 + u < CPR && ln + (u0 + u) * WAVE < nc) p[u] = lds[lds_index(ln, u0 + u)];
#pragma unroll
                    for (int u = 0; u < STAGE_UNROLL; ++u) {
                        const int c = ln + (u0 + u) * WAVE;
                        if (u0 + u < CPR && c < nc && !((skip >> (c / CPR)) & 1ull))
                            out16<NT, F32>(dst + (u0 + u) * WAVE, widen4(p[u]));
                    }
                }
            } else if (R == WAVE) {
                store_flat<NT, F32, true>(dst, ln, nc);
            } else {
                store_flat<NT, F32, false>(dst, ln, nc);
            }
            return;
        }
#pragma unroll
        for (int u0 = 0; u0 < CPR; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u)
                if (u0 + u < CPR && ln + (u0 + u) * WAVE < nc) p[u] = lds[lds_index(ln, u0 + u)];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                const int c = ln + (u0 + u) * WAVE;
                if (u0 + u < CPR && c < nc && !((skip >> (c / CPR)) & 1ull)) {
                    const int r = c / CPR;
                    const int pos = 4 * (c - r * CPR);
                    int4* dst = reinterpret_cast<int4*>(g + (int64_t)r * gpitch + pos);
                    const uint32_t fc = FB ? flags[r] : 0u;
                    if (fc) out16<false, F32>(dst, *reinterpret_cast<const int4*>(fb_src(fc, fallback, fallback2) + (int64_t)r * fpitch + pos));
                    else out16<NT, F32>(dst, widen4(p[u]));
                }
            }
        }
    }

    // ---- bit-plane registers (acx_planes.h; the env-step kernels) ----
    static constexpr int PW = PlaneWords<NW>::value;

    // lane's row -> bit planes; returns true if the row is outside the domain.  Streams the row
    // 8 letters (two dwords) at a time through one gather per plane (pl::i8x8_to_bytes), so few
    // values are live at once: this pack sets the env-step kernels' register peak
    template <bool LIVE = false>  // LIVE: CodeTile only (see there)
    __device__ __forceinline__ bool pack(int lane, PlaneRegs<PW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t* src = lds + ln * S;
        bool bad = flags[ln] != 0;
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {  // one relator at a time (register peak)
            Planes<PW> w;
            uint64_t nz[PW];
#pragma unroll
            for (int j = 0; j < PW; ++j) w.s[j] = w.y[j] = nz[j] = 0ull;
#pragma unroll
            for (int k = 0; k < HALF; k += 2) {
                const uint32_t d0 = src[h * HALF + k];
                const uint32_t d1 = k + 1 < HALF ? src[h * HALF + k + 1] : 0u;
                uint32_t s8, y8, z8;
                pl::i8x8_to_bytes(d0, d1, s8, y8, z8);
                const int sh = 4 * (k & 15);
                w.s[k >> 4] |= (uint64_t)s8 << sh;
                w.y[k >> 4] |= (uint64_t)y8 << sh;
                nz[k >> 4] |= (uint64_t)z8 << sh;
            }
            int n = 0;
#pragma unroll
            for (int j = 0; j < PW; ++j) n += __builtin_popcountll(nz[j]);
            const pl::Bits<PW> e = pl::bmask<PW>(n);  // zeros only as right padding <=> mask == low n bits
#pragma unroll
            for (int j = 0; j < PW; ++j) bad |= nz[j] != e.b[j];
            if (h == 0) { p.w0 = w; p.n0 = n; }
            else        { p.w1 = w; p.n1 = n; }
        }
        return bad;
    }
    __device__ __forceinline__ void unpack(int lane, const PlaneRegs<PW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        uint32_t d[CPR];
        image(p, d);
#pragma unroll
        for (int k = 0; k < CPR; k += 2) *reinterpret_cast<uint2*>(dst + k) = make_uint2(d[k], d[k + 1]);
    }
    template <bool LIVE = false>  // LIVE: CodeTile only (see there)
    __device__ __forceinline__ uint32_t unpack_dirty(int lane, const PlaneRegs<PW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        uint32_t d[CPR];
        image(p, d);
        uint32_t x0 = 0, x1 = 0;
#pragma unroll
        for (int k = 0; k < CPR; k += 2) {
            const uint2 o = *reinterpret_cast<const uint2*>(dst + k);
            if (k < HALF) x0 |= o.x ^ d[k];
            else x1 |= o.x ^ d[k];
            if (k + 1 < HALF) x0 |= o.y ^ d[k + 1];
            else x1 |= o.y ^ d[k + 1];
            *reinterpret_cast<uint2*>(dst + k) = make_uint2(d[k], d[k + 1]);
        }
        return (x0 != 0u ? 1u : 0u) | (x1 != 0u ? 2u : 0u);
    }
    __device__ __forceinline__ void unpack_half(int lane, const PlaneRegs<PW>& p, bool h1) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const Planes<PW> w = pl::psel<PW>(h1, p.w1, p.w0);
        const int n8 = 8 * (h1 ? p.n1 : p.n0);
        uint32_t* dst = lds + ln * S + (h1 ? HALF : 0);
#pragma unroll
        for (int k = 0; k < HALF; ++k) dst[k] = pl::nibbles_to_i8x4(pl::nib<PW>(w.s, k), pl::nib<PW>(w.y, k), clamp_bits(n8 - 32 * k));
    }
    __device__ __forceinline__ static void image(const PlaneRegs<PW>& p, uint32_t (&d)[CPR]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const Planes<PW>& w = h ? p.w1 : p.w0;
            const int n8 = 8 * (h ? p.n1 : p.n0);
#pragma unroll
            for (int k = 0; k < HALF; ++k)
                d[h * HALF + k] = pl::nibbles_to_i8x4(pl::nib<PW>(w.s, k), pl::nib<PW>(w.y, k), clamp_bits(n8 - 32 * k));
        }
    }

    // lane's row -> packed registers; returns true if the row is outside the domain
    __device__ __forceinline__ bool pack(int lane, PresRegs<NW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t* src = lds + ln * S;
        uint32_t d[CPR];
#pragma unroll
        for (int k = 0; k < CPR; k += 2) {
            const uint2 x = *reinterpret_cast<const uint2*>(src + k);
            d[k] = x.x;
            d[k + 1] = x.y;
        }
        bool bad = flags[ln] != 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            Word<NW> w = wzero<NW>();
            uint64_t mlo = 0, mhi = 0;
#pragma unroll
            for (int k = 0; k < HALF; ++k) {
                uint32_t c8, nz4;
                pack4_codes(d[h * HALF + k], c8, nz4);
                w.w[k >> 2] |= c8 << (8 * (k & 3));
                if (k < 16) mlo |= (uint64_t)nz4 << (4 * k);
                else mhi |= (uint64_t)nz4 << (4 * (k - 16));
            }
            const int n = __builtin_popcountll(mlo) + __builtin_popcountll(mhi);
            // zeros only as right padding <=> mask == low n bits
            const uint64_t elo = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
            const uint64_t ehi = n <= 64 ? 0ull : (n >= 128 ? ~0ull : ((1ull << (n - 64)) - 1ull));
            bad |= (mlo != elo) || (mhi != ehi);
            if (h == 0) { p.w0 = w; p.n0 = n; }
            else        { p.w1 = w; p.n1 = n; }
        }
        return bad;
    }

    // packed registers -> lane's row
    __device__ __forceinline__ void unpack(int lane, const PresRegs<NW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        uint32_t d[CPR];
        image(p, d);
#pragma unroll
        for (int k = 0; k < CPR; k += 2) *reinterpret_cast<uint2*>(dst + k) = make_uint2(d[k], d[k + 1]);
    }

    // unpack, and return which relators differ from the row it overwrites (bit h = relator h):
    // the int8 image is canonical (zero letters past the length), so equal relators compare equal
    __device__ __forceinline__ uint32_t unpack_dirty(int lane, const PresRegs<NW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        uint32_t d[CPR];
        image(p, d);
        uint32_t x0 = 0, x1 = 0;
#pragma unroll
        for (int k = 0; k < CPR; k += 2) {
            const uint2 o = *reinterpret_cast<const uint2*>(dst + k);
            if (k < HALF) x0 |= o.x ^ d[k];
            else x1 |= o.x ^ d[k];
            if (k + 1 < HALF) x0 |= o.y ^ d[k + 1];
            else x1 |= o.y ^ d[k + 1];
            *reinterpret_cast<uint2*>(dst + k) = make_uint2(d[k], d[k + 1]);
        }
        return (x0 != 0u ? 1u : 0u) | (x1 != 0u ? 2u : 0u);
    }

    // relator h1 of the lane's row only: a clean move changes just its target relator, so the
    // rollout keeps the LDS tile as the int8 image of the current states and re-images one half
    // per step (the trajectory store then reads the whole tile)
    __device__ __forceinline__ void unpack_half(int lane, const PresRegs<NW>& p, bool h1) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const Word<NW> w = wsel<NW>(h1, p.w1, p.w0);
        const int n8 = 8 * (h1 ? p.n1 : p.n0);
        uint32_t* dst = lds + ln * S + (h1 ? HALF : 0);
#pragma unroll
        for (int k = 0; k < HALF; ++k)
            dst[k] = codes_to_i8x4((w.w[k >> 2] >> (8 * (k & 3))) & 0xffu, clamp_bits(n8 - 32 * k));
    }

    __device__ __forceinline__ void set_dirty(int lane, uint32_t m) const { dirty[lane] = (uint8_t)m; }

    // In-place state store (g is the row block the tile was loaded from): only the 16-byte
    // chunks of relators marked in dirty[] are written; every other chunk already holds its
    // value in HBM (a gated move, an unchanged relator, a failed env).  Needs set_dirty for every
    // row of the tile and a wave_sync after it.  Dirty rows flagged FB_RESET (an autoreset to an
    // out-of-domain starting row) are copied from fallback2 (same row pitch).
    // LIVE: a dirty relator's chunks past lim[] (the live chunks of its old and new letters, set
    // by the caller) already hold zero padding in HBM and are not written
    template <bool NT, bool LIVE = false>
    __device__ __forceinline__ void store_dirty(int32_t* g, int R, int lane, const int32_t* fallback2 = nullptr) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nc = R * CPR;
        int4* dst = reinterpret_cast<int4*>(g);
        if (tile_bad) {  // rare (wave-uniform): per-chunk fallback test
            for (int c = ln; c < nc; c += WAVE) {
                const int r = c / CPR;
                const int k = c - r * CPR;
                if (!((dirty[r] >> (k >= HALF ? 1 : 0)) & 1u)) continue;
                if (flags[r] == FB_RESET) dst[c] = reinterpret_cast<const int4*>(fallback2)[c];
                else if (!LIVE || live(r, k)) dst[c] = widen4(lds[r * S + k]);
            }
            return;
        }
#pragma unroll
        for (int u0 = 0; u0 < CPR; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
            bool wr[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                wr[u] = false;
                const int c = ln + (u0 + u) * WAVE;
                if (u0 + u < CPR && c < nc) {
                    const int r = c / CPR;
                    const int k = c - r * CPR;
                    wr[u] = ((dirty[r] >> (k >= HALF ? 1 : 0)) & 1u) && (!LIVE || live(r, k));
                    if (wr[u]) p[u] = lds[r * S + k];
                }
            }
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                if (!wr[u]) continue;
                out16<NT, false>(dst + ln + (u0 + u) * WAVE, widen4(p[u]));
            }
        }
    }

  private:
    __device__ __forceinline__ static void image(const PresRegs<NW>& p, uint32_t (&d)[CPR]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const Word<NW>& w = h ? p.w1 : p.w0;
            const int n = h ? p.n1 : p.n0;
            const int n8 = 8 * n;
#pragma unroll
            for (int k = 0; k < HALF; ++k)
                d[h * HALF + k] = codes_to_i8x4((w.w[k >> 2] >> (8 * (k & 3))) & 0xffu, clamp_bits(n8 - 32 * k));
        }
    }
};

// CodeTile: compile-time L % 8 == 0, large L (128).  LDS holds, per 4-letter chunk, one
// 16-bit slot = 8-bit code field | 4-bit non-zero mask << 8 (half the bytes of an int8
// image: 8.5 KB per wave at L = 128, so LDS no longer caps occupancy); the SWAR
// conversion happens in the cooperative load/store, and a lane's pack/unpack is plain
// field assembly.  Row stride S dwords, S = 2 mod 4 (conflict-free 8-byte lane accesses).
template <int NW, int LC>
struct CodeTile {
    static_assert(LC > 0 && LC % 8 == 0, "CodeTile needs a compile-time L multiple of 8");
    static constexpr int L = LC;
    static constexpr int twoL = 2 * LC;
    static constexpr int CPR = LC / 2;   // 4-letter chunks per row (16-bit slots)
    static constexpr int RDW = CPR / 2;  // dwords per row
    static constexpr int S = (RDW % 4 == 2) ? RDW : RDW + ((6 - RDW % 4) % 4);
    static constexpr int HALF = CPR / 2;  // chunks per relator
    static_assert(S % 4 == 2 && RDW % 2 == 0, "row layout");
    static constexpr int LOAD_BATCH = 8;

    uint32_t* lds;
    uint8_t* flags;
    uint8_t* dirty;  // see FastTile
    uint8_t* lim;    // see FastTile
    uint32_t limv = 0;  // this lane's row's live chunk counts, lim0 | lim1 << 8 (set_lim)
    uint32_t dirtyv = 0;  // this lane's row's dirty bits (set_dirty)
    bool tile_bad = false;

    static __host__ __device__ constexpr size_t wave_bytes(int) { return (size_t)WAVE * S * 4 + 4 * WAVE; }
    static constexpr bool PREFETCH_OK = false;  // fetch_rows / put_rows: FastTile only
    static constexpr bool LIVE_ROWS = true;  // see FastTile
    static constexpr int RPI = 1;
    __device__ __forceinline__ int4 fetch_rows(const int32_t*, uint64_t, int) const { return int4{0, 0, 0, 0}; }
    __device__ __forceinline__ void put_rows(const int4&, uint64_t, uint64_t, int) {}
    static constexpr bool NT_STEP_LOADS = true;  // see ld_tile
    __device__ __forceinline__ void restore_flags(int lane, uint32_t code) {
        flags[lane] = (uint8_t)code;
        tile_bad = __any(code != 0u);
        wave_sync();
    }
    __device__ __forceinline__ void flag_rows(int lane, uint32_t code) {
        if (code) flags[lane] = (uint8_t)code;
        tile_bad = tile_bad || __any(code != 0u);
    }
    __device__ __forceinline__ int32_t letter(int r, int k) const {
        const uint32_t sl = slots(r)[k >> 2];
        const uint32_t d = codes_to_i8x4(sl & 0xffu, 8u * __builtin_popcount((sl >> 8) & 0xfu));
        return (int32_t)(int8_t)(d >> (8 * (k & 3)));
    }
    __device__ __forceinline__ CodeTile(char* base, int) {
        lds = reinterpret_cast<uint32_t*>(base);
        flags = reinterpret_cast<uint8_t*>(base + WAVE * S * 4);
        dirty = flags + WAVE;
        lim = flags + 2 * WAVE;
    }
    // see FastTile::set_lim / live (chunks of 4 letters; HALF chunks per relator)
    __device__ __forceinline__ void set_lim(int lane, int n0, int n1) {
        lim[2 * lane] = (uint8_t)live_chunks(n0);
        lim[2 * lane + 1] = (uint8_t)live_chunks(n1);
        limv = (uint32_t)live_chunks(n0) | ((uint32_t)live_chunks(n1) << 8);
    }
    // see FastTile::widen_lim; rounded up to whole 64-byte sectors (4 chunks; relators start on a
    // sector at L % 32 == 0): the chunks past the letters in the last sector hold zero padding in
    // HBM and in the tile, and a partly written sector was a read-modify-write in HBM
    __device__ __forceinline__ void widen_lim(int lane, int n0, int n1) {
        int a = max((int)(limv & 0xffu), live_chunks(n0)), b = max((int)(limv >> 8), live_chunks(n1));
        if constexpr (L % 32 == 0) {
            a = min(HALF, (a + 3) & ~3);
            b = min(HALF, (b + 3) & ~3);
        }
        lim[2 * lane] = (uint8_t)a;
        lim[2 * lane + 1] = (uint8_t)b;
        limv = (uint32_t)a | ((uint32_t)b << 8);
    }
    // CPR == WAVE (one row per wave-instruction): chunk ln of row u is live, row u's counts read
    // from lane u's register (a scalar per compile-time u; no LDS read, no per-u VGPR)
    __device__ __forceinline__ bool live_lane(int u, int ln) const {
        const int lu = __builtin_amdgcn_readlane((int)limv, u);
        const int l0 = lu & 0xff, l1 = (lu >> 8) & 0xff;  // scalars
        return ln < l0 || (ln >= HALF && ln < HALF + l1);  // l0 <= HALF
    }
    __device__ __forceinline__ static int live_chunks(int n) { return n <= 0 ? 0 : n >= L ? HALF : (n + 3) >> 2; }
    __device__ __forceinline__ bool live(int r, int k) const {
        const int h = k >= HALF ? 1 : 0;
        return k - h * HALF < lim[2 * r + h];
    }
    __device__ __forceinline__ int Lr() const { return L; }
    __device__ __forceinline__ uint16_t* slots(int r) const { return reinterpret_cast<uint16_t*>(lds + r * S); }

    __device__ __forceinline__ void put(int c, uint32_t slot) const {
        const int r = c / CPR;
        slots(r)[c - r * CPR] = (uint16_t)slot;
    }
    __device__ __forceinline__ uint32_t get(int c) const {
        const int r = c / CPR;
        return slots(r)[c - r * CPR];
    }

    // PIPE (the step kernel; the rollout keeps the plain loop, whose register budget the
    // in-flight batch pair would exceed): full tiles software-pipelined, see below
    template <bool PIPE = false, bool LIVE = false, bool NTL = false, int BATCH = 0>
    __device__ __forceinline__ void load(const int32_t* __restrict__ g, int R, int lane) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        flags[ln] = 0;
        wave_sync();
        const int nc = R * CPR;
        const int4* src = reinterpret_cast<const int4*>(g) + ln;
        bool any_bad = false;
        if constexpr (CPR == WAVE) {
            if (PIPE && R == WAVE) {
                // full tile, one row per wave-instruction (row u, lane ln = its chunk ln):
                // software-pipelined as below; each chunk is converted by chunk_i8 and stored at
                // the lane's fixed slot address (row u at a compile-time offset).  Rows with a
                // letter outside {-2..2} (error inputs only) are found afterwards, when some
                // chunk was bad: each lane rescans its own row's loaded chunks
                // LIVE: every chunk is loaded through a buffer descriptor over the tile's rows, a
                // dead chunk at an out-of-range offset -- the hardware returns zeros and reads
                // nothing -- so no load sits under a branch (a conditional load made the
                // compiler wait for all of them, vmcnt(0), before each conversion) and a dead
                // chunk converts to an empty slot like any zero padding
                int4 va[LOAD_BATCH], vb[LOAD_BATCH];
                uint16_t* mine = reinterpret_cast<uint16_t*>(lds) + ln;
                const uint64_t gb = reinterpret_cast<uint64_t>(g);
                const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)gb);
                const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32));
                const __amdgpu_buffer_rsrc_t rows = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<void*>(((uint64_t)ghi << 32) | glo), (short)0, WAVE * CPR * 16, 0x00020000);
                const uint32_t lane_off = (uint32_t)ln * 16u;
                const uint32_t oob = 0x80000000u;
                auto issue = [&](int4* v, int u0) {
#pragma unroll
                    for (int u = 0; u < LOAD_BATCH; ++u) {
                        if constexpr (LIVE) {
                            // row u's live lanes as a 64-bit scalar mask (its counts read from lane
                            // u: one readlane, the rest scalar), then one v_cndmask on it picks the
                            // lane's offset or the out-of-range one; the row's base is the scalar
                            // offset (in range on either reading of the bounds check)
                            const uint32_t lu = (uint32_t)__builtin_amdgcn_readlane((int)limv, u0 + u);
                            const uint32_t l0 = lu & 0xffu, l1 = (lu >> 8) & 0xffu;
                            const uint64_t m = ((1ull << l0) - 1ull) | (((1ull << l1) - 1ull) << 32);
                            uint32_t off;
                            asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(off) : "v"(oob), "v"(lane_off), "s"(m));
                            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rows, off, (u0 + u) * WAVE * 16, tile_cpol(NTL));
                            v[u] = make_int4((int)x[0], (int)x[1], (int)x[2], (int)x[3]);
                        } else {
                            v[u] = ld_tile<NTL>(src + (u0 + u) * WAVE);
                        }
                    }
                };
                int mx = 0, mn = 0;  // running max / min of every loaded letter (dead chunks load 0)
                auto convert = [&](const int4* v, int u0) {
#pragma unroll
                    for (int u = 0; u < LOAD_BATCH; ++u) {
                        uint32_t c8, nz4;
                        pack4_codes(chunk_i8_acc(v[u], mx, mn), c8, nz4);
                        mine[(u0 + u) * 2 * S] = (uint16_t)(c8 | (nz4 << 8));
                    }
                };
                static_assert(CPR % (2 * LOAD_BATCH) == 0, "pipelined tile load: whole batch pairs");
                issue(va, 0);
#pragma unroll
                for (int u0 = 0; u0 < CPR; u0 += 2 * LOAD_BATCH) {
                    issue(vb, u0 + LOAD_BATCH);
                    convert(va, u0);
                    if (u0 + 2 * LOAD_BATCH < CPR) issue(va, u0 + 2 * LOAD_BATCH);
                    convert(vb, u0 + LOAD_BATCH);
                }
                any_bad = mx > 2 || mn < -2;
                tile_bad = __any(any_bad);
                if (tile_bad) {  // rare (wave-uniform)
                    bool rb = false;
                    const int32_t* row = g + (int64_t)ln * twoL;
                    for (int k = 0; k < CPR; ++k) {
                        bool in = true;
                        if constexpr (LIVE) in = live(ln, k);
                        if (!in) continue;
                        const int4 v = reinterpret_cast<const int4*>(row)[k];
                        bool b = false;
                        chunk_i8(v, b);
                        rb |= b;
                    }
                    flags[ln] = rb ? 1 : 0;
                    // a flagged row's slots are rebuilt with to_i8 (an out-of-domain letter ->
                    // 0x7f, non-zero), so the letter counts reported for it are the input row's
                    if (rb) {
                        for (int k = 0; k < CPR; ++k) {
                            bool in = true;
                            if constexpr (LIVE) in = live(ln, k);
                            if (!in) continue;
                            const int4 v = reinterpret_cast<const int4*>(row)[k];
                            bool b = false;
                            const uint32_t d = to_i8(v.x, b) | (to_i8(v.y, b) << 8) | (to_i8(v.z, b) << 16) |
                                               (to_i8(v.w, b) << 24);
                            uint32_t c8, nz4;
                            pack4_codes(d, c8, nz4);
                            slots(ln)[k] = (uint16_t)(c8 | (nz4 << 8) | ((uint32_t)b << 12));
                        }
                    }
                }
                wave_sync();
                return;
            }
        }
        if (PIPE && R == WAVE) {
            // full tile (wave-uniform): software-pipelined, batch b + 1's loads are issued before
            // batch b is converted, so LOAD_BATCH..2*LOAD_BATCH loads stay in flight through the
            // whole 64 KB tile (L = 128) instead of draining to zero between batches
            // LIVE: a wave-instruction u covers row u (CPR == WAVE), lane ln its chunk ln
            int4 va[LOAD_BATCH], vb[LOAD_BATCH];
            auto lv = [&](int u) {
                if constexpr (!LIVE) return true;
                else if constexpr (CPR == WAVE) return live_lane(u, ln);
                else return live((ln + u * WAVE) / CPR, (ln + u * WAVE) % CPR);
            };
            auto issue = [&](int4* v, int u0) {
#pragma unroll
                for (int u = 0; u < LOAD_BATCH; ++u)
                    if (lv(u0 + u)) v[u] = ld_tile<NTL>(src + (u0 + u) * WAVE);
            };
            auto convert = [&](const int4* v, int u0) {
#pragma unroll
                for (int u = 0; u < LOAD_BATCH; ++u) {
                    const int c = ln + (u0 + u) * WAVE;
                    bool bad = false;
                    uint32_t slot = 0;
                    if (lv(u0 + u)) {
                        const uint32_t d = to_i8(v[u].x, bad) | (to_i8(v[u].y, bad) << 8) |
                                           (to_i8(v[u].z, bad) << 16) | (to_i8(v[u].w, bad) << 24);
                        uint32_t c8, nz4;
                        pack4_codes(d, c8, nz4);
                        slot = c8 | (nz4 << 8) | ((uint32_t)bad << 12);
                    }
                    put(c, slot);
                    if (bad) flags[c / CPR] = 1;
                    any_bad |= bad;
                }
            };
            static_assert(CPR % (2 * LOAD_BATCH) == 0, "pipelined tile load: whole batch pairs");
            issue(va, 0);
#pragma unroll
            for (int u0 = 0; u0 < CPR; u0 += 2 * LOAD_BATCH) {
                issue(vb, u0 + LOAD_BATCH);
                convert(va, u0);
                if (u0 + 2 * LOAD_BATCH < CPR) issue(va, u0 + 2 * LOAD_BATCH);
                convert(vb, u0 + LOAD_BATCH);
            }
            tile_bad = __any(any_bad);
            wave_sync();
            return;
        }
        for (int u0 = 0; u0 < CPR; u0 += LOAD_BATCH) {
            int4 v[LOAD_BATCH];
            bool lv[LOAD_BATCH];
#pragma unroll
            for (int u = 0; u < LOAD_BATCH; ++u) {
                const int c = ln + (u0 + u) * WAVE;
                lv[u] = c < nc && (!LIVE || live(c / CPR, c % CPR));
                if (lv[u]) v[u] = ld_tile<NTL>(src + (u0 + u) * WAVE);
            }
#pragma unroll
            for (int u = 0; u < LOAD_BATCH; ++u) {
                const int c = ln + (u0 + u) * WAVE;
                if (c < nc) {
                    bool bad = false;
                    uint32_t slot = 0;
                    if (lv[u]) {
                        const uint32_t d = to_i8(v[u].x, bad) | (to_i8(v[u].y, bad) << 8) |
                                           (to_i8(v[u].z, bad) << 16) | (to_i8(v[u].w, bad) << 24);
                        uint32_t c8, nz4;
                        pack4_codes(d, c8, nz4);
                        slot = c8 | (nz4 << 8) | ((uint32_t)bad << 12);
                    }
                    put(c, slot);
                    if (bad) flags[c / CPR] = 1;
                    any_bad |= bad;
                }
            }
        }
        tile_bad = __any(any_bad);
        wave_sync();
    }

    // see FastTile::load_block
    __device__ __forceinline__ void load_block(const int32_t* __restrict__ g, int R) {
        constexpr int U = (WAVE * CPR + BLOCK - 1) / BLOCK;
        if (threadIdx.x < WAVE) flags[threadIdx.x] = 0;
        __syncthreads();
        const int nc = R * CPR;
        const int4* src = reinterpret_cast<const int4*>(g);
        int4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = (int)threadIdx.x + u * BLOCK;
            if (c < nc) v[u] = ld_tile<NT_EXPAND_LOADS>(src + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = (int)threadIdx.x + u * BLOCK;
            if (c >= nc) continue;
            bool bad = false;
            const uint32_t d = to_i8(v[u].x, bad) | (to_i8(v[u].y, bad) << 8) | (to_i8(v[u].z, bad) << 16) |
                               (to_i8(v[u].w, bad) << 24);
            uint32_t c8, nz4;
            pack4_codes(d, c8, nz4);
            put(c, c8 | (nz4 << 8) | ((uint32_t)bad << 12));
            if (bad) flags[c / CPR] = 1;
        }
        __syncthreads();
    }

    // the rows of the lanes in `rows` only (see FastTile::load_rows); a row is >= one
    // wave-instruction here (CPR >= 16 chunks), so row by row, lanes over its chunks
    __device__ __forceinline__ void load_rows(const int32_t* __restrict__ g, uint64_t rows, int R, int lane) {
        load_rows_from([&](int r) { return g + (int64_t)r * twoL; }, rows, R, lane);
    }
    template <class RowPtr>
    __device__ __forceinline__ void load_rows_from(RowPtr rp, uint64_t rows, int, int lane) {
        if ((rows >> lane) & 1ull) flags[lane] = 0;
        wave_sync();
        bool any_bad = false;
        for (uint64_t m = rows; m; m &= m - 1) {
            const int r = __builtin_ctzll(m);
            const int32_t* row_src = rp(r);
            for (int c = lane; c < CPR; c += WAVE) {
                const int4 v = reinterpret_cast<const int4*>(row_src)[c];
                bool bad = false;
                const uint32_t d = to_i8(v.x, bad) | (to_i8(v.y, bad) << 8) | (to_i8(v.z, bad) << 16) |
                                   (to_i8(v.w, bad) << 24);
                uint32_t c8, nz4;
                pack4_codes(d, c8, nz4);
                slots(r)[c] = (uint16_t)(c8 | (nz4 << 8) | ((uint32_t)bad << 12));
                if (bad) flags[r] = 1;
                any_bad |= bad;
            }
        }
        tile_bad = tile_bad || __any(any_bad);
        wave_sync();
    }

    // LDS -> R contiguous global rows, exactly CPR store instructions on every path (see
    // FastTile::store_rows)
    template <bool NT>
    __device__ __forceinline__ void store_rows(int32_t* g, int R, int lane) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nc = R * CPR;
        int4* dst = reinterpret_cast<int4*>(g);
        for (int u0 = 0; u0 < CPR; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
            int cc[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                const int c0 = ln + (u0 + u) * WAVE;
                cc[u] = c0 < nc ? c0 : nc - 1;
                p[u] = get(cc[u]);
            }
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                const uint32_t nz4 = (p[u] >> 8) & 0xfu;
                out16<NT, false>(dst + cc[u], widen4(codes_to_i8x4(p[u] & 0xffu, 8u * __builtin_popcount(nz4))));
            }
        }
    }

    // see FastTile::store_rows_i8: slot c of the tile is int8 dword c of the global tile
    template <bool NT>
    __device__ __forceinline__ void store_rows_i8(int8_t* g, int R, int lane) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nc = R * CPR;
        uint32_t* dst = reinterpret_cast<uint32_t*>(g);
#pragma unroll
        for (int u = 0; u < (WAVE * CPR) / (4 * WAVE); ++u) {
            const int c0 = 4 * (ln + u * WAVE);
            if (c0 >= nc) continue;  // nc is a multiple of 4 (CPR % 4 == 0)
            // 4 slots of one row (CPR % 4 == 0): one 8-byte LDS read
            const int r = c0 / CPR;
            const uint2 q = *reinterpret_cast<const uint2*>(slots(r) + (c0 - r * CPR));
            const uint32_t sl[4] = {q.x & 0xffffu, q.x >> 16, q.y & 0xffffu, q.y >> 16};
            int x[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                x[j] = (int)codes_to_i8x4(sl[j] & 0xffu, 8u * __builtin_popcount((sl[j] >> 8) & 0xfu));
            const v4i_t v = {x[0], x[1], x[2], x[3]};
            if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4i_t*>(dst + c0));
            else *reinterpret_cast<v4i_t*>(dst + c0) = v;
        }
    }

    template <bool FB, bool NT = false, bool F32 = false>
    __device__ __forceinline__ void store(int32_t* g, int64_t gpitch, int R, const int32_t* fallback,
                                          int64_t fpitch, int lane, const int32_t* fallback2 = nullptr,
                                          uint64_t skip = 0) const {  // skip: see FastTile::store
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nc = R * CPR;
        for (int u0 = 0; u0 < CPR; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u)
                if (ln + (u0 + u) * WAVE < nc) p[u] = get(ln + (u0 + u) * WAVE);
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                const int c = ln + (u0 + u) * WAVE;
                if (c >= nc) continue;
                const int r = c / CPR;
                if ((skip >> r) & 1ull) continue;
                const int pos = 4 * (c - r * CPR);
                int4* dst = reinterpret_cast<int4*>(g + (int64_t)r * gpitch + pos);
                if (FB && tile_bad && flags[r]) {
                    out16<false, F32>(dst, *reinterpret_cast<const int4*>(fb_src(flags[r], fallback, fallback2) +
                                                                          (int64_t)r * fpitch + pos));
                } else {
                    const uint32_t nz4 = (p[u] >> 8) & 0xfu;
                    out16<NT, F32>(dst, widen4(codes_to_i8x4(p[u] & 0xffu, 8u * __builtin_popcount(nz4))));
                }
            }
        }
    }

    // ---- bit-plane registers (acx_planes.h; the env-step kernels) ----
    // 4 slots (16 letters) per 8-byte LDS access: their code fields -> 32 bits of 2-bit codes ->
    // the even / odd bits compressed into the s / y planes (and back the same way)
    static constexpr int PW = PlaneWords<NW>::value;
    __device__ __forceinline__ static uint32_t compress_even(uint32_t x) {
        x &= 0x55555555u;
        x = (x | (x >> 1)) & 0x33333333u;
        x = (x | (x >> 2)) & 0x0F0F0F0Fu;
        x = (x | (x >> 4)) & 0x00FF00FFu;
        return (x | (x >> 8)) & 0x0000FFFFu;
    }
    __device__ __forceinline__ static uint32_t spread_even(uint32_t x) {
        x = (x | (x << 8)) & 0x00FF00FFu;
        x = (x | (x << 4)) & 0x0F0F0F0Fu;
        x = (x | (x << 2)) & 0x33333333u;
        return (x | (x << 1)) & 0x55555555u;
    }
    template <bool LIVE = false>  // LIVE: CodeTile only (see there)
    __device__ __forceinline__ bool pack(int lane, PlaneRegs<PW>& p) const {
        static_assert(HALF % 4 == 0, "16-letter groups per relator");
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t* src = lds + ln * S;
        bool bad = flags[ln] != 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            Planes<PW> w;
            uint64_t nz[PW];
#pragma unroll
            for (int j = 0; j < PW; ++j) w.s[j] = w.y[j] = nz[j] = 0ull;
            const int lim_h = (int)((limv >> (8 * h)) & 0xffu);
#pragma unroll
            for (int g = 0; g < HALF / 4; ++g) {  // 16 letters
                // LIVE (the first pack after a live load): a group past every row's live chunks
                // holds zero slots -- skipped when no lane of the wave has one (wave-uniform)
                if (LIVE && !__any(lim_h > 4 * g)) continue;
                const uint2 x = *reinterpret_cast<const uint2*>(src + (h * HALF + 4 * g) / 2);
                const uint32_t codes = __builtin_amdgcn_perm(x.y, x.x, 0x06040200u);
                uint32_t nzb = __builtin_amdgcn_perm(x.y, x.x, 0x07050301u) & 0x0F0F0F0Fu;
                nzb = (nzb | (nzb >> 4)) & 0x00FF00FFu;
                nzb = (nzb | (nzb >> 8)) & 0x0000FFFFu;
                const int sh = 16 * (g & 3);
                w.s[g >> 2] |= (uint64_t)compress_even(codes) << sh;
                w.y[g >> 2] |= (uint64_t)compress_even(codes >> 1) << sh;
                nz[g >> 2] |= (uint64_t)nzb << sh;
            }
            int n = 0;
#pragma unroll
            for (int j = 0; j < PW; ++j) n += __builtin_popcountll(nz[j]);
            const pl::Bits<PW> e = pl::bmask<PW>(n);
#pragma unroll
            for (int j = 0; j < PW; ++j) bad |= nz[j] != e.b[j];
            if (h == 0) { p.w0 = w; p.n0 = n; }
            else        { p.w1 = w; p.n1 = n; }
        }
        return bad;
    }
    // relator h of the lane's row from planes (canonical slots: codes and nz of absent letters 0)
    // glim >= 0: the slots past chunk glim are zero both in the tile and in the new image (a
    // live-loaded relator: max of its old and new live chunks); groups past every lane's glim
    // are neither compared nor written
    __device__ __forceinline__ uint32_t put_relator(uint32_t* dst, const Planes<PW>& w, int n, bool cmp,
                                                    int glim = -1) const {
        const pl::Bits<PW> m = pl::bmask<PW>(n);
        uint32_t x = 0;
#pragma unroll
        for (int g = 0; g < HALF / 4; ++g) {
            if (glim >= 0 && !__any(glim > 4 * g)) continue;
            const int sh = 16 * (g & 3);
            const uint32_t s16 = (uint32_t)(w.s[g >> 2] >> sh) & 0xffffu;
            const uint32_t y16 = (uint32_t)(w.y[g >> 2] >> sh) & 0xffffu;
            const uint32_t codes = spread_even(s16) | (spread_even(y16) << 1);
            uint32_t nzb = (uint32_t)(m.b[g >> 2] >> sh) & 0xffffu;
            nzb = (nzb | (nzb << 8)) & 0x00FF00FFu;
            nzb = (nzb | (nzb << 4)) & 0x0F0F0F0Fu;
            const uint2 v = make_uint2(__builtin_amdgcn_perm(nzb, codes, 0x05010400u),
                                       __builtin_amdgcn_perm(nzb, codes, 0x07030602u));
            uint2* q = reinterpret_cast<uint2*>(dst + 2 * g);
            if (cmp) {
                const uint2 o = *q;
                x |= (o.x ^ v.x) | (o.y ^ v.y);
            }
            *q = v;
        }
        return x;
    }
    __device__ __forceinline__ void unpack(int lane, const PlaneRegs<PW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        put_relator(dst, p.w0, p.n0, false);
        put_relator(dst + HALF / 2, p.w1, p.n1, false);
    }
    template <bool LIVE = false>  // LIVE: CodeTile only (see there)
    __device__ __forceinline__ uint32_t unpack_dirty(int lane, const PlaneRegs<PW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        int g0 = -1, g1 = -1;
        if constexpr (LIVE) {
            g0 = max((int)(limv & 0xffu), live_chunks(p.n0));
            g1 = max((int)((limv >> 8) & 0xffu), live_chunks(p.n1));
        }
        const uint32_t x0 = put_relator(dst, p.w0, p.n0, true, g0);
        const uint32_t x1 = put_relator(dst + HALF / 2, p.w1, p.n1, true, g1);
        return (x0 != 0u ? 1u : 0u) | (x1 != 0u ? 2u : 0u);
    }
    __device__ __forceinline__ void unpack_half(int lane, const PlaneRegs<PW>& p, bool h1) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        put_relator(lds + ln * S + (h1 ? HALF / 2 : 0), pl::psel<PW>(h1, p.w1, p.w0), h1 ? p.n1 : p.n0, false);
    }

    __device__ __forceinline__ bool pack(int lane, PresRegs<NW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t* src = lds + ln * S;
        bool bad = flags[ln] != 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            Word<NW> w = wzero<NW>();
            uint64_t mlo = 0, mhi = 0;
#pragma unroll
            for (int k = 0; k < HALF; k += 4) {  // 4 slots = one 8-byte LDS read
                const uint2 x = *reinterpret_cast<const uint2*>(src + (h * HALF + k) / 2);
                const uint32_t sl[4] = {x.x & 0xffffu, x.x >> 16, x.y & 0xffffu, x.y >> 16};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int kk = k + j;
                    w.w[kk >> 2] |= (sl[j] & 0xffu) << (8 * (kk & 3));
                    const uint64_t nz4 = (sl[j] >> 8) & 0xfu;
                    if (kk < 16) mlo |= nz4 << (4 * kk);
                    else mhi |= nz4 << (4 * (kk - 16));
                }
            }
            const int n = __builtin_popcountll(mlo) + __builtin_popcountll(mhi);
            const uint64_t elo = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
            const uint64_t ehi = n <= 64 ? 0ull : (n >= 128 ? ~0ull : ((1ull << (n - 64)) - 1ull));
            bad |= (mlo != elo) || (mhi != ehi);
            if (h == 0) { p.w0 = w; p.n0 = n; }
            else        { p.w1 = w; p.n1 = n; }
        }
        return bad;
    }

    __device__ __forceinline__ void unpack(int lane, const PresRegs<NW>& p) const { unpack_impl<false>(lane, p); }
    // see FastTile::unpack_half
    __device__ __forceinline__ void unpack_half(int lane, const PresRegs<NW>& p, bool h1) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const Word<NW> w = wsel<NW>(h1, p.w1, p.w0);
        const int n = h1 ? p.n1 : p.n0;
        uint32_t* dst = lds + ln * S + (h1 ? HALF / 2 : 0);
#pragma unroll
        for (int k = 0; k < HALF; k += 4) {
            uint32_t sl[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kk = k + j;
                const int nin = n - 4 * kk;
                const uint32_t nz4 = nin >= 4 ? 0xfu : (nin <= 0 ? 0u : ((1u << nin) - 1u));
                sl[j] = ((w.w[kk >> 2] >> (8 * (kk & 3))) & 0xffu) | (nz4 << 8);
            }
            *reinterpret_cast<uint2*>(dst + k / 2) = make_uint2(sl[0] | (sl[1] << 16), sl[2] | (sl[3] << 16));
        }
    }
    // see FastTile::unpack_dirty; the slots compared are canonical (codes of absent letters
    // masked to 0, as load writes them)
    __device__ __forceinline__ uint32_t unpack_dirty(int lane, const PresRegs<NW>& p) const {
        return unpack_impl<true>(lane, p);
    }
    __device__ __forceinline__ void set_dirty(int lane, uint32_t m) {
        dirty[lane] = (uint8_t)m;
        dirtyv = m;
    }

    // see FastTile::store_dirty
    template <bool NT, bool LIVE = false>
    __device__ __forceinline__ void store_dirty(int32_t* g, int R, int lane, const int32_t* fallback2 = nullptr) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int nc = R * CPR;
        int4* dst = reinterpret_cast<int4*>(g);
        if (tile_bad) {  // rare (wave-uniform): per-chunk fallback test
            for (int c = ln; c < nc; c += WAVE) {
                const int r = c / CPR;
                const int k = c - r * CPR;
                if (!((dirty[r] >> (k >= HALF ? 1 : 0)) & 1u)) continue;
                if (flags[r] == FB_RESET) {
                    dst[c] = reinterpret_cast<const int4*>(fallback2)[c];
                } else if (!LIVE || live(r, k)) {
                    const uint32_t sl = slots(r)[k];
                    dst[c] = widen4(codes_to_i8x4(sl & 0xffu, 8u * __builtin_popcount((sl >> 8) & 0xfu)));
                }
            }
            return;
        }
        if constexpr (CPR == WAVE) {
            // one row per wave-instruction (row r, lane ln = its chunk ln): the lane's fixed slot
            // address, row r's dirty bits and live counts read from lane r's registers (scalars)
            const uint16_t* mine = reinterpret_cast<const uint16_t*>(lds) + ln;
            const int hs = ln >= HALF ? 1 : 0;
            const uint64_t gb = reinterpret_cast<uint64_t>(g);
            const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)gb);
            const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<void*>(((uint64_t)ghi << 32) | glo), (short)0, WAVE * CPR * 16, 0x00020000);
            for (int r0 = 0; r0 < R; r0 += STAGE_UNROLL) {
                uint32_t p[STAGE_UNROLL];
                bool wr[STAGE_UNROLL];
#pragma unroll
                for (int u = 0; u < STAGE_UNROLL; ++u) {
                    const int r = r0 + u;
                    const uint32_t dr = (uint32_t)__builtin_amdgcn_readlane((int)dirtyv, r);
                    bool lv = true;
                    if constexpr (LIVE) lv = live_lane(r, ln);
                    wr[u] = r < R && ((dr >> hs) & 1u) && lv;
                    if (wr[u]) p[u] = mine[r * 2 * S];
                }
#pragma unroll
                for (int u = 0; u < STAGE_UNROLL; ++u) {
                    if (!wr[u]) continue;
                    const uint32_t nz4 = (p[u] >> 8) & 0xfu;
                    const int4 v = widen4(codes_to_i8x4(p[u] & 0xffu, 8u * __builtin_popcount(nz4)));
                    const v4i_t x = {v.x, v.y, v.z, v.w};
                    __builtin_amdgcn_raw_buffer_store_b128(x, rs, (uint32_t)(ln + (r0 + u) * WAVE) * 16u, 0, WB_CPOL);
                }
            }
            return;
        }
        for (int u0 = 0; u0 < CPR; u0 += STAGE_UNROLL) {
            uint32_t p[STAGE_UNROLL];
            bool wr[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                wr[u] = false;
                const int c = ln + (u0 + u) * WAVE;
                if (c < nc) {
                    const int r = c / CPR;
                    const int k = c - r * CPR;
                    bool lv = true;
                    if constexpr (LIVE) lv = (CPR == WAVE) ? live_lane(u0 + u, ln) : live(r, k);
                    wr[u] = ((dirty[r] >> (k >= HALF ? 1 : 0)) & 1u) && lv;
                    if (wr[u]) p[u] = slots(r)[k];
                }
            }
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                if (!wr[u]) continue;
                const uint32_t nz4 = (p[u] >> 8) & 0xfu;
                out16<NT, false>(dst + ln + (u0 + u) * WAVE,
                                 widen4(codes_to_i8x4(p[u] & 0xffu, 8u * __builtin_popcount(nz4))));
            }
        }
    }

  private:
    template <bool CMP>
    __device__ __forceinline__ uint32_t unpack_impl(int lane, const PresRegs<NW>& p) const {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        uint32_t* dst = lds + ln * S;
        uint32_t x[2] = {0u, 0u};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const Word<NW>& w = h ? p.w1 : p.w0;
            const int n = h ? p.n1 : p.n0;
#pragma unroll
            for (int k = 0; k < HALF; k += 4) {
                uint32_t sl[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int kk = k + j;
                    const int nin = n - 4 * kk;
                    const uint32_t nz4 = nin >= 4 ? 0xfu : (nin <= 0 ? 0u : ((1u << nin) - 1u));
                    uint32_t c8 = (w.w[kk >> 2] >> (8 * (kk & 3))) & 0xffu;
                    if constexpr (CMP) c8 &= nin >= 4 ? 0xffu : (nin <= 0 ? 0u : ((1u << (2 * nin)) - 1u));
                    sl[j] = c8 | (nz4 << 8);
                }
                uint2* q = reinterpret_cast<uint2*>(dst + (h * HALF + k) / 2);
                const uint2 v = make_uint2(sl[0] | (sl[1] << 16), sl[2] | (sl[3] << 16));
                if constexpr (CMP) {
                    const uint2 o = *q;
                    x[h] |= (o.x ^ v.x) | (o.y ^ v.y);
                }
                *q = v;
            }
        }
        return (x[0] != 0u ? 1u : 0u) | (x[1] != 0u ? 2u : 0u);
    }
};

template <int NW, int LC, int VEC>
struct GenericTile {
    static constexpr bool PREFETCH_OK = false;  // fetch_rows / put_rows: FastTile only
    static constexpr bool LIVE_ROWS = false;  // whole rows: set_lim is a no-op
    static constexpr int RPI = 1;
    __device__ __forceinline__ int4 fetch_rows(const int32_t*, uint64_t, int) const { return int4{0, 0, 0, 0}; }
    __device__ __forceinline__ void put_rows(const int4&, uint64_t, uint64_t, int) {}
    static constexpr bool NT_STEP_LOADS = false;  // see ld_tile
    static constexpr int LMAX = LC > 0 ? LC : 16 * NW;
    int L, twoL, rowb;
    char* base;
    uint8_t* flags;

    static __host__ __device__ int row_bytes(int L_) {
        const int bytes = (LC > 0) ? 2 * LC : (L_ + LMAX);
        return (((bytes + 3) >> 2) | 1) * 4;  // odd dword stride: conflict-free per-lane reads
    }
    static __host__ __device__ size_t wave_bytes(int L_) { return (size_t)WAVE * row_bytes(L_) + WAVE; }
    __device__ __forceinline__ GenericTile(char* b, int L_) {
        L = LC > 0 ? LC : L_;
        twoL = 2 * L;
        rowb = row_bytes(L);
        base = b;
        flags = reinterpret_cast<uint8_t*>(b + WAVE * rowb);
    }
    __device__ __forceinline__ int Lr() const { return L; }
    // contiguous rows
    template <bool NT>
    __device__ __forceinline__ void store_rows(int32_t* g, int R, int lane) const {
        store<false, NT>(g, 2 * L, R, nullptr, 0, lane);
    }
    // int8 rows, byte by byte (parity instantiations)
    template <bool NT>
    __device__ __forceinline__ void store_rows_i8(int8_t* g, int R, int lane) const {
        for (int i = lane; i < R * twoL; i += WAVE) g[i] = row(i / twoL)[i % twoL];
    }
    __device__ __forceinline__ void restore_flags(int lane, uint32_t code) {
        flags[lane] = (uint8_t)code;
        wave_sync();
    }
    __device__ __forceinline__ void flag_rows(int lane, uint32_t code) {
        if (code) flags[lane] = (uint8_t)code;
    }
    __device__ __forceinline__ int32_t letter(int r, int k) const { return row(r)[k]; }
    // the rows of the lanes in `rows` only, row by row (the generic-L instantiations serve
    // parity, not speed)
    __device__ __forceinline__ void load_rows(const int32_t* __restrict__ g, uint64_t rows, int R, int lane) {
        load_rows_from([&](int r) { return g + (int64_t)r * twoL; }, rows, R, lane);
    }
    template <class RowPtr>
    __device__ __forceinline__ void load_rows_from(RowPtr rp, uint64_t rows, int, int lane) {
        if ((rows >> lane) & 1ull) flags[lane] = 0;
        wave_sync();
        for (uint64_t m = rows; m; m &= m - 1) {
            const int r = __builtin_ctzll(m);
            const int32_t* row_src = rp(r);
            bool bad = false;
            for (int k = lane; k < twoL; k += WAVE)
                row(r)[k] = (int8_t)to_i8(row_src[k], bad);
            if (__any(bad) && lane == 0) flags[r] = 1;
        }
        wave_sync();
    }
    __device__ __forceinline__ int8_t* row(int r) const { return reinterpret_cast<int8_t*>(base + r * rowb); }

    // (row, pos) of a chunk of VEC int32; chunks never straddle rows (2L % VEC == 0)
    struct It {
        int row, pos, dq, dr, twoL;
        __device__ __forceinline__ It(int c0, int twoL_) : twoL(twoL_) {
            const int e0 = c0 * VEC;
            row = e0 / twoL;
            pos = e0 - row * twoL;
            dq = (WAVE * VEC) / twoL;
            dr = WAVE * VEC - dq * twoL;
        }
        __device__ __forceinline__ void next() {
            pos += dr;
            row += dq;
            if (pos >= twoL) { pos -= twoL; ++row; }
        }
    };

    // PIPE, LIVE: see CodeTile::load (the runtime-L path reads and writes whole rows)
    template <bool PIPE = false, bool LIVE = false, bool NTL = false, int BATCH = 0>
    __device__ __forceinline__ void load(const int32_t* __restrict__ g, int R, int lane) {
        flags[lane] = 0;
        wave_sync();
        const int nc = (R * twoL) / VEC;
        It it(lane, twoL);
        for (int b0 = lane; b0 < nc; b0 += WAVE * STAGE_UNROLL) {
            int rows[STAGE_UNROLL], poss[STAGE_UNROLL];
            int32_t v[STAGE_UNROLL][VEC];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                rows[u] = it.row;
                poss[u] = it.pos;
                it.next();
                if (b0 + u * WAVE < nc) {
                    const int32_t* src = g + (int64_t)rows[u] * twoL + poss[u];
                    if constexpr (VEC == 4) {
                        const int4 x = *reinterpret_cast<const int4*>(src);
                        v[u][0] = x.x; v[u][1] = x.y; v[u][2] = x.z; v[u][3] = x.w;
                    } else {
                        const int2 x = *reinterpret_cast<const int2*>(src);
                        v[u][0] = x.x; v[u][1] = x.y;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                if (b0 + u * WAVE < nc) {
                    bool bad = false;
                    char* dst = base + rows[u] * rowb + poss[u];
                    if constexpr (VEC == 4) {
                        *reinterpret_cast<uint32_t*>(dst) = to_i8(v[u][0], bad) | (to_i8(v[u][1], bad) << 8) |
                                                            (to_i8(v[u][2], bad) << 16) | (to_i8(v[u][3], bad) << 24);
                    } else {
                        *reinterpret_cast<uint16_t*>(dst) = (uint16_t)(to_i8(v[u][0], bad) | (to_i8(v[u][1], bad) << 8));
                    }
                    if (bad) flags[rows[u]] = 1;
                }
            }
        }
        wave_sync();
    }

    template <bool FB, bool NT = false, bool F32 = false>
    __device__ __forceinline__ void store(int32_t* g, int64_t gpitch, int R, const int32_t* fallback,
                                          int64_t fpitch, int lane, const int32_t* fallback2 = nullptr,
                                          uint64_t skip = 0) const {  // skip: see FastTile::store
        const int nc = (R * twoL) / VEC;
        It it(lane, twoL);
        for (int b0 = lane; b0 < nc; b0 += WAVE * STAGE_UNROLL) {
            int rows[STAGE_UNROLL], poss[STAGE_UNROLL];
            uint32_t p[STAGE_UNROLL];
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                rows[u] = it.row;
                poss[u] = it.pos;
                it.next();
                p[u] = 0;
                if (b0 + u * WAVE < nc) {
                    const char* src = base + rows[u] * rowb + poss[u];
                    if constexpr (VEC == 4) p[u] = *reinterpret_cast<const uint32_t*>(src);
                    else p[u] = *reinterpret_cast<const uint16_t*>(src);
                }
            }
#pragma unroll
            for (int u = 0; u < STAGE_UNROLL; ++u) {
                if (b0 + u * WAVE >= nc || ((skip >> rows[u]) & 1ull)) continue;
                int32_t* dst = g + (int64_t)rows[u] * gpitch + poss[u];
                const uint32_t fc = FB ? flags[rows[u]] : 0u;
                const bool fb = fc != 0u;
                const int32_t* f = fb_src(fc, fallback, fallback2) + (int64_t)rows[u] * fpitch + poss[u];
                if constexpr (VEC == 4) {
                    out16<false, F32>(reinterpret_cast<int4*>(dst), fb ? *reinterpret_cast<const int4*>(f) : widen4(p[u]));
                } else {
                    int2 x;
                    x.x = (int32_t)(int8_t)(p[u] & 0xffu);
                    x.y = (int32_t)(int8_t)((p[u] >> 8) & 0xffu);
                    out8<F32>(reinterpret_cast<int2*>(dst), fb ? *reinterpret_cast<const int2*>(f) : x);
                }
            }
        }
    }

    // ---- bit-plane registers (acx_planes.h; the env-step kernels), letter by letter ----
    static constexpr int PW = PlaneWords<NW>::value;
    __device__ __forceinline__ void pack_relator(const int8_t* src, Planes<PW>& w, int& n, bool& bad) const {
#pragma unroll
        for (int j = 0; j < PW; ++j) w.s[j] = w.y[j] = 0ull;
        n = 0;
        bool zero_seen = false;
#pragma unroll
        for (int k = 0; k < LMAX; ++k) {
            int b = src[k];
            if (LC == 0) b = (k < L) ? b : 0;
            const bool nz = b != 0;
            w.s[k >> 6] |= (uint64_t)(nz && b < 0) << (k & 63);
            w.y[k >> 6] |= (uint64_t)(nz && (b & 1) == 0) << (k & 63);
            n += nz;
            bad |= nz && zero_seen;
            zero_seen |= !nz;
        }
    }
    template <bool LIVE = false>  // LIVE: CodeTile only (see there)
    __device__ __forceinline__ bool pack(int lane, PlaneRegs<PW>& p) const {
        const int8_t* r = row(lane);
        bool bad = flags[lane] != 0;
        pack_relator(r, p.w0, p.n0, bad);
        pack_relator(r + L, p.w1, p.n1, bad);
        return bad;
    }
    __device__ __forceinline__ void unpack_relator(int8_t* dst, const Planes<PW>& w, int n) const {
#pragma unroll
        for (int k = 0; k < LMAX; ++k) {
            const uint32_t code = (uint32_t)(((w.y[k >> 6] >> (k & 63)) & 1ull) << 1 | ((w.s[k >> 6] >> (k & 63)) & 1ull));
            const uint32_t letter = (0xFE02FF01u >> (code << 3)) & 0xffu;  // code -> 1, -1, 2, -2
            if (LC > 0 || k < L) dst[k] = (int8_t)(k < n ? letter : 0u);
        }
    }
    __device__ __forceinline__ void unpack(int lane, const PlaneRegs<PW>& p) const {
        int8_t* r = row(lane);
        unpack_relator(r, p.w0, p.n0);
        unpack_relator(r + L, p.w1, p.n1);
    }
    __device__ __forceinline__ void unpack_half(int lane, const PlaneRegs<PW>& p, bool h1) const {
        unpack_relator(row(lane) + (h1 ? L : 0), pl::psel<PW>(h1, p.w1, p.w0), h1 ? p.n1 : p.n0);
    }
    template <bool LIVE = false>  // LIVE: CodeTile only (see there)
    __device__ __forceinline__ uint32_t unpack_dirty(int lane, const PlaneRegs<PW>& p) const {
        unpack(lane, p);
        return 3u;
    }

    __device__ __forceinline__ void pack_relator(const int8_t* src, Word<NW>& w, int& n, bool& bad) const {
        w = wzero<NW>();
        n = 0;
        bool zero_seen = false;
#pragma unroll
        for (int k = 0; k < LMAX; ++k) {
            int b = src[k];
            if (LC == 0) b = (k < L) ? b : 0;
            const bool nz = b != 0;
            const uint32_t code = nz ? ((((uint32_t)~b & 1u) << 1) | (((uint32_t)b >> 7) & 1u)) : 0u;
            w.w[k >> 4] |= code << (2 * (k & 15));
            n += nz;
            bad |= nz && zero_seen;
            zero_seen |= !nz;
        }
    }
    __device__ __forceinline__ bool pack(int lane, PresRegs<NW>& p) const {
        const int8_t* r = row(lane);
        bool bad = flags[lane] != 0;
        pack_relator(r, p.w0, p.n0, bad);
        pack_relator(r + L, p.w1, p.n1, bad);
        return bad;
    }
    __device__ __forceinline__ void unpack_relator(int8_t* dst, const Word<NW>& w, int n) const {
#pragma unroll
        for (int k = 0; k < LMAX; ++k) {
            const uint32_t code = (w.w[k >> 4] >> (2 * (k & 15))) & 3u;
            const uint32_t letter = (0xFE02FF01u >> (code << 3)) & 0xffu;  // code -> 1, -1, 2, -2
            if (LC > 0 || k < L) dst[k] = (int8_t)(k < n ? letter : 0u);
        }
    }
    __device__ __forceinline__ void unpack(int lane, const PresRegs<NW>& p) const {
        int8_t* r = row(lane);
        unpack_relator(r, p.w0, p.n0);
        unpack_relator(r + L, p.w1, p.n1);
    }
    // relator h1 of the lane's row only (the rollout's clean moves change one relator)
    __device__ __forceinline__ void unpack_half(int lane, const PresRegs<NW>& p, bool h1) const {
        unpack_relator(row(lane) + (h1 ? L : 0), wsel<NW>(h1, p.w1, p.w0), h1 ? p.n1 : p.n0);
    }
    // runtime-L tiles (parity tests at any L) track no dirty relators: every row is written
    __device__ __forceinline__ uint32_t unpack_dirty(int lane, const PresRegs<NW>& p) const {
        unpack(lane, p);
        return 3u;
    }
    __device__ __forceinline__ void set_dirty(int, uint32_t) const {}
    __device__ __forceinline__ void set_lim(int, int, int) const {}  // whole rows (see FastTile)
    __device__ __forceinline__ void widen_lim(int, int, int) const {}
    template <bool NT, bool LIVE = false>
    __device__ __forceinline__ void store_dirty(int32_t* g, int R, int lane, const int32_t* fallback2 = nullptr) const {
        store<true, NT>(g, twoL, R, g, twoL, lane, fallback2);
    }
};

// The int8 trajectory rows of a tile with flagged rows (rare, wave-uniform branch): byte by byte,
// flagged rows as the int8 values of their fallback row (numpy's astype(int8) wrap)
template <class Tile>
__device__ __forceinline__ void store_rows_i8_fb(const Tile& t, int8_t* g, int R, int twoL, int lane,
                                              const int32_t* fb_in, const int32_t* fb_reset) {
    for (int i = lane; i < R * twoL; i += WAVE) {
        const int r = i / twoL, k = i - r * twoL;
        const uint32_t fc = t.flags[r];
        g[i] = (int8_t)(fc ? fb_src(fc, fb_in, fb_reset)[(int64_t)r * twoL + k] : t.letter(r, k));
    }
}

template <int NW, int LC, int VEC>
using TileFor = typename std::conditional<
    (LC >= 64 && LC % 8 == 0), CodeTile<NW, LC>,
    typename std::conditional<(LC > 0 && LC % 4 == 0), FastTile<NW, LC>, GenericTile<NW, LC, VEC>>::type>::type;

// Per-lane registers -> row in HBM directly (uncoalesced; only for final_obs on the rare
// same-step-autoreset path of the step kernel).
template <int NW>
__device__ __forceinline__ void regs_to_global(int32_t* dst, const PresRegs<NW>& p, int L) {
    for (int h = 0; h < 2; ++h) {
        const Word<NW> w = h ? p.w1 : p.w0;
        const int n = h ? p.n1 : p.n0;
#pragma unroll 1
        for (int k = 0; k < L; ++k) {
            const uint32_t code = wletter<NW>(w, k);
            const int32_t v = (int32_t)(int8_t)((0xFE02FF01u >> (code << 3)) & 0xffu);
            dst[h * L + k] = k < n ? v : 0;
        }
    }
}

template <int PW>
__device__ __forceinline__ void regs_to_global(int32_t* dst, const PlaneRegs<PW>& p, int L) {
    for (int h = 0; h < 2; ++h) {
        const Planes<PW> w = h ? p.w1 : p.w0;
        const int n = h ? p.n1 : p.n0;
#pragma unroll 1
        for (int k = 0; k < L; ++k) {
            const uint32_t code = pl::pletter<PW>(w, k);
            const int32_t v = (int32_t)(int8_t)((0xFE02FF01u >> (code << 3)) & 0xffu);
            dst[h * L + k] = k < n ? v : 0;
        }
    }
}

// A wave reloads its whole tile of starting states (one coalesced pass) when more than this
// many of its lanes reset on the same step (a synchronised truncation); for fewer resetting
// lanes the wave loads just their rows (tile.load_rows), so scattered resets cost their rows.
constexpr int RESET_TILE_MIN = 24;

// common per-wave prologue: tile index, rows in the tile, LDS slice
struct WaveCtx {
    int lane, wid;
    int64_t r0;
    int R;
    bool active;
};
__device__ __forceinline__ bool wave_ctx(int64_t rows, WaveCtx& w) {
    w.lane = threadIdx.x & (WAVE - 1);
    // wave-uniform (SGPR): the tile base, its row count and the addresses derived from them
    w.wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    w.r0 = ((int64_t)blockIdx.x * WPB + w.wid) * WAVE;
    if (w.r0 >= rows) return false;
    w.R = (int)((rows - w.r0) < WAVE ? (rows - w.r0) : WAVE);
    w.active = w.lane < w.R;
    return true;
}

// ---------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------
struct StepArgs {
    const int32_t* state_in;
    int32_t* state_out;
    const int32_t* action;
    const int32_t* reset_state;
    int32_t* step_count;
    int32_t* reward;
    uint8_t* done;
    uint8_t* truncated;
    int32_t* lengths_out;
    int32_t* final_obs;
    uint8_t* err;
    int32_t* err_count;
    // learner-side outputs (acx_step_learner; all NULL for acx_step)
    const int64_t* action64;
    float* obs_f32;
    float* reward_f32;
    float* done_f32;
    uint8_t* action_hist;
    int32_t* episode_len;
    int64_t B;
    int L, horizon, cyclical, hist_cap;
    // acx_learner_step: the round-1 curriculum fused into the step (training.py:319-352).
    // cur_ws NULL: none.  cur_ws (uint64 words): [0] launch sequence number, [1, 2] reserved,
    // then the tiles' counts, the groups' totals and arrival words (cur_publish, cur_prefix)
    uint64_t* cur_ws;
    const int32_t* cur_states;  // (n_states, 2L) initial states
    int64_t n_states;
    int32_t* cur_next;          // [1] max(states_processed) + 1
    int32_t* curr_index;        // (B)
    uint8_t* needs_host;        // (B)
    // state_out == state_in (set by the launcher): the state store writes changed relators only
    int in_place;
    // next-step autoreset (acx_step_next; NULL: same-step): per env, its episode ended on the
    // previous call -- this call resets it instead of stepping, and records whether it ends now
    uint8_t* pending;
    // lengths-carrying step (acx_step_lengths): lengths_out holds the rows' relator lengths on
    // entry (canonical rows), so only their letters are read and written
    int live;
    // move-history ring (NULL: move k of an episode at row k): per env, the row of its current
    // episode's move 0; an episode's first move sets it to hist_t mod hist_cap (hist_t: the
    // caller's step counter), so envs whose episodes are out of phase still write this step's
    // moves to one row -- coalesced -- instead of one cache line per lane
    int32_t* hist_base;
    int64_t hist_t;
    // tests only (acx_internal_learner_ranking_fails): ranking waits give up at once, as one that
    // polled 2^20 times would (1: every wait, needs_host = 3; 2: only the last tile's total)
    int cur_fail;
    // acx_step_lengths_reduced (live steps only; NULL: none): per env, bit 0 = both relators are
    // non-empty and freely reduced, bit 1 = and cyclically reduced, as the previous step left them.
    // A conjugation of such a row reads only its target relator (step_body).  Written every call.
    uint8_t* reduced;
};

// ---------------------------------------------------------------------------------
// The curriculum's ranking inside the step kernel (acx_learner_step, one launch).  Finished envs
// (done | truncated) take the initial states next_index, next_index + 1, ... in env order
// (training.py:329-336), so an env needs the number of finished envs before it -- a prefix count
// over the whole batch -- and the last tile needs the total (the new next_index).  Two levels,
// no chain: a tile is one wave's 64 envs, a group is 64 consecutive tiles.
//   * every tile publishes its count (a seq-tagged status word) and adds (1, count) to its
//     group's arrival word with one 64-bit atomic; the add that completes the group publishes the
//     group's total and clears the arrival word for the next launch (64 adds per address at most:
//     MI355X_MICROARCH "dequeue" -- one word saturates at ~88 adds per us);
//   * tile 0 publishes next_index as the scan's base;
//   * a tile that needs its prefix -- one with finished envs -- polls the base, the totals of the
//     groups before its own and the counts of the tiles before it in its group, until all are
//     there (no propagation through intermediate tiles: it waits only for earlier tiles to have
//     published once); the last tile polls every group total, writes next_index and advances the
//     launch's sequence number;
//   * words are written and polled with agent-scope atomics (each word is the whole hand-off:
//     "8-B agent atomics both sides"); a word of an earlier launch carries another sequence number
//     and reads as not there.  Every wave reads the sequence number before it publishes, so once
//     every group is complete no wave of the launch reads it again and the last tile may advance it;
//   * HIP promises no dispatch order: a tile that polls too long (2^20 polls, ~seconds -- an
//     earlier tile never scheduled) gives up and flags its finished envs needs_host = 3
//     (CurriculumRecord.process raises), so the launch always ends.  Any give-up -- a tile's
//     prefix, or the last tile's total, after which next_index is stale -- also sets the sticky
//     word [2]: every later launch then ranks nothing (its finished envs get needs_host = 3) until
//     the host re-zeroes the workspace (LearnerEnv.reset_workspace, which also restores
//     next_index from curr_index), since a give-up can leave a group's arrival word incomplete;
//     CurriculumRecord.process raises on the word.  Concurrent launches on one workspace are not
//     supported (they would overwrite each other's words; nothing detects it).
// cur_ws (uint64 words): [0] sequence number, [1] base, [2] sticky failure word, [3, 3 + T) tile
// counts, [3 + T, 3 + T + G) group totals, [3 + T + G, 3 + T + 2G) group arrival words (T tiles,
// G groups).
// ---------------------------------------------------------------------------------
constexpr uint64_t CUR_SET = 1ull << 62;
constexpr uint32_t CUR_FAIL = 0xffffffffu;
constexpr uint32_t CUR_SEQ_MASK = (1u << 30) - 1u;

__device__ __forceinline__ uint64_t cur_word(uint32_t seq, uint32_t v) {
    return CUR_SET | ((uint64_t)(seq & CUR_SEQ_MASK) << 32) | v;
}
__device__ __forceinline__ bool cur_is(uint64_t w, uint32_t seq) {
    return (w >> 62) == 1 && ((uint32_t)(w >> 32) & CUR_SEQ_MASK) == (seq & CUR_SEQ_MASK);
}
__device__ __forceinline__ uint64_t cur_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void cur_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// uint64 words between two groups' arrival words, the launch's only same-address atomics (64
// tiles add to each): 256 bytes apart, one per channel-interleave unit, the step is 6 % faster
// than with the words packed (fresh episodes 0.1257 vs 0.1345 ms, steady state 0.159 vs 0.165,
// profiles/r05/r05x_learner_probe_stride.json; spacing the tile count words too changed nothing).
// acx_curriculum_workspace (acx_curriculum.hip) sizes the workspace with the same value
#define ACX_CUR_ARRIVE_STRIDE 32
struct CurLayout {
    int64_t tiles, groups;
    uint64_t *base, *tile, *group, *arrive;
    __device__ __forceinline__ CurLayout(const StepArgs& a) {
        tiles = (a.B + WAVE - 1) / WAVE;
        groups = (tiles + WAVE - 1) / WAVE;
        base = a.cur_ws + 1;
        tile = a.cur_ws + 3;
        group = tile + tiles;
        arrive = group + groups;
    }
};

// this tile's count, its group arrival, and (tile 0) the base.  Returns the arrival word before
// this tile's add (lane 0), for cur_publish_end right after: deferring that to the tile's tail
// (so the add's return trip overlaps the stores) made the step slower, fresh episodes 0.143 vs
// 0.140 ms and steady state 0.21 vs 0.172 (same buffers, r05v), as later tiles then wait longer
// for the group total
// cnext: next_index as this wave read it, before publishing -- the last tile overwrites it once
// every tile has published, so the read must complete first: the published word takes an opaque
// dependency on it, both words being relaxed agent-scope atomics
__device__ __forceinline__ uint64_t cur_publish(const StepArgs& a, const WaveCtx& w, uint32_t seq, uint32_t cnt,
                                                int64_t cnext) {
    if (w.lane != 0) return 0;
    const CurLayout c(a);
    const int64_t t = w.r0 / WAVE, g = t / WAVE;
    if (t == 0) cur_store(c.base, cur_word(seq, (uint32_t)*a.cur_next));
    uint64_t word = cur_word(seq, cnt);
    asm volatile("" : "+v"(word) : "s"((uint32_t)cnext));
    cur_store(c.tile + t, word);
    return __hip_atomic_fetch_add(c.arrive + g * ACX_CUR_ARRIVE_STRIDE, (1ull << 32) | cnt, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}
// the sticky failure word (cur_ws[2], see above)
__device__ __forceinline__ void cur_set_failed(const StepArgs& a) { cur_store(a.cur_ws + 2, 1ull); }

// the add that completed its group publishes the group's total and clears the arrival word for
// the next launch
__device__ __forceinline__ void cur_publish_end(const StepArgs& a, const WaveCtx& w, uint32_t seq, uint32_t cnt,
                                                uint64_t old) {
    if (w.lane != 0) return;
    const CurLayout c(a);
    const int64_t t = w.r0 / WAVE, g = t / WAVE;
    const int64_t gsize = (c.tiles - g * WAVE) < WAVE ? (c.tiles - g * WAVE) : WAVE;
    if ((int64_t)(old >> 32) + 1 == gsize) {
        cur_store(c.group + g, cur_word(seq, (uint32_t)old + cnt));
        cur_store(c.arrive + g * ACX_CUR_ARRIVE_STRIDE, 0ull);
    }
}

// base + the counts of every tile before this one (all_groups: + every group's total instead: the
// last tile's next_index), or CUR_FAIL.  Wave-uniform control flow.  A word, once seen with this
// launch's seq, is final: each lane re-reads only the words it has not seen yet (`pend`), so the
// polls of the waiting tiles thin out as the prefix fills in (re-reading every word on every poll
// put ~4k waiting waves on the same few dozen lines).  Group totals are taken 4 per lane, 256 per
// round; the base (lane 0) and the own group's earlier tile counts (a lane each) with the first.
// (s_sleep 8 between polls instead: the same, r05v)
__device__ __forceinline__ uint32_t cur_prefix(const StepArgs& a, const WaveCtx& w, uint32_t seq, bool all_groups) {
    if (a.cur_fail == 1 || (a.cur_fail == 2 && all_groups)) return CUR_FAIL;  // test hook
    const CurLayout c(a);
    const int64_t t = w.r0 / WAVE, g = t / WAVE;
    const int64_t ng = all_groups ? c.groups : g;  // whole groups summed
    auto group_bits = [&](int64_t k0) {
        uint32_t b = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) b |= (k0 + 4 * w.lane + i < ng) ? 1u << i : 0u;
        return b;
    };
    uint32_t pend = group_bits(0);
    if (w.lane == 0) pend |= 1u << 5;                            // the base
    if (!all_groups && g * WAVE + w.lane < t) pend |= 1u << 4;  // a tile before this one in its group
    uint32_t x = 0, polls = 0;
    int64_t k0 = 0;
    while (true) {
        uint64_t v[6];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (pend >> i) & 1u ? cur_load(c.group + k0 + 4 * w.lane + i) : 0ull;
        v[4] = (pend >> 4) & 1u ? cur_load(c.tile + g * WAVE + w.lane) : 0ull;
        v[5] = (pend >> 5) & 1u ? cur_load(c.base) : 0ull;
#pragma unroll
        for (int i = 0; i < 6; ++i)
            if (((pend >> i) & 1u) && cur_is(v[i], seq)) {
                x += (uint32_t)v[i];
                pend &= ~(1u << i);
            }
        if (__all(pend == 0u)) {
            k0 += 4 * WAVE;
            if (k0 >= ng) break;
            pend = group_bits(k0);
            continue;
        }
        if (++polls > (1u << 20)) return CUR_FAIL;
        __builtin_amdgcn_s_sleep(2);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, WAVE);
    return x;
}

// the rows of the tile in the wave-uniform mask `rows` <- src(q, r) (q: the row's ordinal in the
// mask, r: its row in the tile), written to state_out, obs_f32 (as float) and, with to_reset,
// reset_state: the whole wave copies, 16-byte chunks spread over the lanes (a lane copying its
// own row issued 4 x 2L/4 instructions for the wave per finished env)
template <class Src>
__device__ __forceinline__ void copy_rows(const StepArgs& a, const WaveCtx& w, uint64_t rows, int twoL, Src src,
                                          bool to_reset) {
    const int n = __popcll(rows);
    if (n == 0) return;
    const bool full = rows == ~0ull;
    int32_t* st = a.state_out + w.r0 * twoL;
    float* of = a.obs_f32 ? a.obs_f32 + w.r0 * twoL : nullptr;
    int32_t* rs = to_reset ? const_cast<int32_t*>(a.reset_state) + w.r0 * twoL : nullptr;  // learner: writable
    auto row_of = [&](int q) {
        if (full) return q;
        uint64_t m = rows;
        for (int j = 0; j < q; ++j) m &= m - 1;
        return (int)__builtin_ctzll(m);
    };
    if ((twoL & 3) == 0) {
        const int cpr = twoL >> 2;
        for (int i = w.lane; i < n * cpr; i += WAVE) {
            const int q = i / cpr, c = i - q * cpr, r = row_of(q);
            const int4 v = reinterpret_cast<const int4*>(src(q, r))[c];
            reinterpret_cast<int4*>(st + (int64_t)r * twoL)[c] = v;
            if (rs) reinterpret_cast<int4*>(rs + (int64_t)r * twoL)[c] = v;
            if (of) reinterpret_cast<float4*>(of + (int64_t)r * twoL)[c] = make_float4((float)v.x, (float)v.y, (float)v.z,
                                                                                       (float)v.w);
        }
    } else {
        for (int i = w.lane; i < n * twoL; i += WAVE) {
            const int q = i / twoL, c = i - q * twoL, r = row_of(q);
            const int32_t v = src(q, r)[c];
            st[(int64_t)r * twoL + c] = v;
            if (rs) rs[(int64_t)r * twoL + c] = v;
            if (of) of[(int64_t)r * twoL + c] = (float)v;
        }
    }
}

// LEARN: acx_step_learner's extra inputs/outputs (compiled out of the plain acx_step path);
// LIVE: the lengths-carrying step (its own kernel, so the plain step's registers stay its own)
template <int NW, int LC, int VEC, bool LEARN, bool LIVE, int BATCH = 0>
__device__ __forceinline__ void step_body(const StepArgs& a) {
    using Tile = TileFor<NW, LC, VEC>;
        extern __shared__ __attribute__((aligned(16))) char smem[];
    WaveCtx w;
    // acx_learner_step: the curriculum fused in (cur_publish / cur_prefix)
    const bool cur = LEARN && a.cur_ws != nullptr;  // kernel argument: uniform
    if (!wave_ctx(a.B, w)) return;
    // the launch's sequence number, read before this tile publishes (cur_publish)
    const uint32_t cseq = cur ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)cur_load(a.cur_ws)) : 0u;
    // next_index as this launch found it (the last tile replaces it only after every tile has
    // published, i.e. read it).  exhausted (round 1 complete): no finished env gets a state from
    // the table, so no tile waits for its ranking; the host draws for every finished env.
    // (Leaving a finished env's rows out of the tile's stores when the table surely lasts the
    // launch, so that its copy needs no drain, was slower: the tile's obs store then takes its
    // per-chunk flagged path, 0.164 vs 0.150 ms per steady-state step, r05zg.)
    const int64_t cnext = cur ? (int64_t)__builtin_amdgcn_readfirstlane(
                                    __hip_atomic_load(a.cur_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              : 0;
    const bool exhausted = cur && cnext >= a.n_states;
    // a give-up in an earlier launch (cur_set_failed) left the workspace unusable until the host
    // re-zeroes it: this launch ranks nothing
    const bool broken = cur && __builtin_amdgcn_readfirstlane((int)(uint32_t)cur_load(a.cur_ws + 2)) != 0;
    // the table surely lasts the launch (every finished env gets an initial state from it): a
    // finished env is not autoreset here -- its rows are left out of the tile's stores and written
    // once, by the curriculum copy, which then needs no drain of the tile's stores (below)
    const bool sure = cur && !broken && !exhausted && a.n_states - cnext >= a.B;
    Tile tile(smem + w.wid * Tile::wave_bytes(a.L), a.L);
    const int L = tile.Lr(), twoL = 2 * L;
    const int64_t env = w.r0 + w.lane;

    // the env's move id and step count: issued ahead of the tile so their latency hides under it
    int act_in = 0, cnt_in = 0;
    const bool pend = w.active && a.pending && a.pending[env] != 0;  // next-step autoreset: reset now
    if (w.active) {
        if (LEARN && a.action64) {  // policy samples (int64); out of range -> ACX_ERR_ACTION
            const int64_t v = a.action64[env];
            act_in = (v >= 0 && v < 12) ? (int)v : -1;
        } else {
            act_in = a.action[env];
        }
        cnt_in = a.step_count ? a.step_count[env] : 0;
    }
    int hb = 0;  // the move-history ring's row of this env's episode move 0
    if (LEARN && w.active && a.hist_base) hb = a.hist_base[env];
    // Relator skip (acx_step_lengths_reduced): a conjugation (ids 4..11, ac_moves.py:79-156)
    // reads and writes only its target r_i, and simplify_presentation (utils.py:246-283) leaves a
    // reduced r_j as it is -- so when the previous step left both relators reduced (a.reduced) the
    // untouched relator is not read at all; its length comes from the carried lengths.  Not
    // skipped: an r_j of one letter (the triviality test, utils.py:57-87, needs it), a step that
    // truncates (final_obs holds the whole row) and next-step resets.  The lane then holds r_j as
    // empty (n = 0, no live chunks), which the move, the dirty image and the write-back leave alone.
    bool skip = false;
    int skip_h = 0, n_skip = 0;  // the relator left unread and its length
    if constexpr (LIVE) {
        int n_in0 = 0, n_in1 = 0;  // the rows' relator lengths on entry
        if (w.active) {
            n_in0 = a.lengths_out[2 * env];
            n_in1 = a.lengths_out[2 * env + 1];
        }
        if constexpr (Tile::LIVE_ROWS) {
            if (a.reduced && w.active) {
                const uint32_t rf = a.reduced[env];
                skip_h = act_in & 1;  // ids 4..11: the move's target is r_{(id + 1) & 1}
                n_skip = skip_h ? n_in1 : n_in0;
                skip = ((rf >> (a.cyclical ? 1 : 0)) & 1u) != 0u && act_in >= 4 && act_in < 12 && !pend &&
                       n_skip >= 2 && n_skip <= L && !(a.step_count && cnt_in + 1 >= a.horizon);
            }
        }
        tile.set_lim(w.lane, (skip && skip_h == 0) ? 0 : n_in0, (skip && skip_h == 1) ? 0 : n_in1);
        wave_sync();
        tile.template load<true, true, Tile::NT_STEP_LOADS>(a.state_in + w.r0 * twoL, w.R, w.lane);
    } else {
        tile.template load<true, false, Tile::NT_STEP_LOADS, BATCH>(a.state_in + w.r0 * twoL, w.R, w.lane);
    }

    // Truncations are known before the move (step_count + 1 >= horizon, unless the move fails):
    // their starting rows are fetched now, under the pack and the move, and put into the tile
    // before this step's stores -- loaded after the move instead, behind those stores, they were
    // a second dependent round trip that doubled the life of every wave holding one (a learner
    // step with episodes out of phase, ~B/H truncations per step: +44 us on a 124 us step)
    constexpr bool PREF = !LIVE && Tile::PREFETCH_OK;
    uint64_t pre = 0;  // wave-uniform: the rows fetched
    int4 pv = {0, 0, 0, 0};
    if constexpr (PREF) {
        if (a.reset_state && a.step_count && !a.pending) {  // kernel arguments: uniform
            pre = __ballot(w.active && cnt_in + 1 >= a.horizon);
            if (__popcll(pre) > Tile::RPI || sure) pre = 0;  // more (a synchronised truncation): the tile reload below
            if (pre) pv = tile.fetch_rows(a.reset_state + w.r0 * twoL, pre, w.lane);
        }
    }

    bool fin = false;    // done | truncated (the curriculum's "finished")
    bool reset = false;  // same-step autoreset of this env
    bool keep = false;   // the env's row is left as loaded (out of domain, or its move failed)
    constexpr int PW = Tile::PW;
    PlaneRegs<PW> p;
    int cnt0 = 0, cnt = 0, e = ACX_ERR_NONE;
    uint32_t dm = 0;     // relators of the row that differ from state_in (in-place store)
    int act = 0;
    bool triv = false, trunc = false;
    int32_t rwd = 0;
    bool bad = false, clean = false;
    const bool cyc = a.cyclical != 0;
    if (w.active) {
        act = act_in;
        cnt0 = cnt_in;
        cnt = a.step_count ? cnt0 + 1 : 0;
        bad = tile.template pack<LIVE>(w.lane, p);
        clean = !bad && !skip && pl::is_clean<PW>(p.w0, p.n0, p.w1, p.n1, cyc);
    }
    // the curriculum (acx_learner_step, training.py:319-336): every tile publishes its finished
    // count as soon as it is known; the ranking itself waits until the tile's stores are issued
    // (the tail below).  Usually that is before the move: a truncating env finishes unless its move
    // fails, which on a reduced row only an emptying concatenation (n_i == n_j) can; any other env
    // finishes only if the move makes it trivial, which needs the relator it leaves alone at one
    // letter.  A tile with an env outside those cases publishes after the move.
    uint64_t fm = 0;
    bool early = false;  // wave-uniform: published before the move
    uint32_t early_cnt = 0;
    if (cur && !broken) {
        bool unc = false, f0 = false;
        if (w.active && !pend && !bad && act_in >= 0 && act_in < 12) {
            const bool i1 = ((act_in + 1) & 1) != 0;  // the move's target relator (ac_moves.py:192-206)
            const int nt = i1 ? p.n1 : p.n0, nu = i1 ? p.n0 : p.n1;
            const bool tr = a.step_count && cnt0 + 1 >= a.horizon;
            if (!clean) unc = true;  // the general path reduces both relators: anything can happen
            else if (tr) { unc = act_in < 4 && nt == nu; f0 = true; }
            else unc = nu <= 1;
        }
        if (!__any(unc)) {
            early = true;
            early_cnt = (uint32_t)__popcll(__ballot(f0));
            cur_publish_end(a, w, cseq, early_cnt, cur_publish(a, w, cseq, early_cnt, cnext));
        }
    }
    if (w.active) {
        if (pend) e = ACX_ERR_NONE;  // no move: the env resets (gymnasium >= 1.0 NEXT_STEP autoreset)
        else if (bad) e = ACX_ERR_DOMAIN;
        else if (skip) e = pl::ac_move_clean<PW>(p.w0, p.n0, p.w1, p.n1, act, L, cyc);  // reduced: see above
        else if (clean) e = pl::ac_move_clean<PW>(p.w0, p.n0, p.w1, p.n1, act, L, cyc);
        else {
                const pl::MoveOut<PW> mo = pl::ac_move_call<PW>(p, act, L, cyc);
                p = mo.p;
                e = mo.e;
            }
        keep = e != ACX_ERR_NONE;
        if (keep) cnt = cnt0;  // the reference raises before count_steps += 1 (ac_env.py:93-102)
        if (!keep) dm = tile.template unpack_dirty<LIVE>(w.lane, p);
        // (a skipped relator is held as n = 0 in p and has >= 2 letters: never trivial)
        triv = !pend && !keep && pl::is_trivial<PW>(p.w0, p.n0, p.w1, p.n1);
        trunc = !pend && !keep && a.step_count && cnt >= a.horizon;
        // a resetting step (next-step autoreset) returns reward 0, as the vector env's reset does
        rwd = pend ? 0 : triv ? a.horizon * L * 2 : -(p.n0 + p.n1 + n_skip * (int)skip);
        fin = triv || trunc;
        // same-step autoreset: an env that ends resets now; next-step: a pending env resets now and
        // an env that ends is reset by the next call
        reset = a.pending ? pend : (fin && a.reset_state && !keep && !sure);
    }
    if (cur) {
        fm = __ballot(fin);
        const uint32_t cnt = (uint32_t)__popcll(fm);
        if (!broken) {
            if (!early) cur_publish_end(a, w, cseq, cnt, cur_publish(a, w, cseq, cnt, cnext));
            else if (cnt != early_cnt && w.lane == 0) cur_set_failed(a);  // cannot happen: made loud
        }
    }
    if constexpr (PREF) {
        if (pre) tile.put_rows(pv, pre, pre & __ballot(reset), w.lane);
    }
    if (w.active) {
        // info["actions"] (ac_env.py:96,105): the episode's moves, one byte each, move k of env i
        // at row k, or with the ring at row (hist_base[i] + k) mod hist_cap -- envs at the same
        // episode position (ring: every env whose episode had no failed move) write one
        // coalesced row segment (an (env, k) layout made every lane's byte its own cache line:
        // 90 us of a 300 us step; (k, env) with episodes out of phase, 26 us of a 196 us one)
        if (LEARN && a.action_hist && !pend && cnt0 < a.hist_cap) {
            int row = cnt0;
            if (a.hist_base) {
                if (cnt0 == 0) {
                    hb = (int)(a.hist_t % a.hist_cap);
                    a.hist_base[env] = hb;
                }
                row = hb + cnt0 < a.hist_cap ? hb + cnt0 : hb + cnt0 - a.hist_cap;
            }
            a.action_hist[(int64_t)row * a.B + env] = (uint8_t)act;
        }
        if (a.reward) st_scalar<false, int32_t>(a.reward + env, rwd);
        if (a.done) st_scalar<false, uint8_t>(a.done + env, (uint8_t)triv);
        if (a.truncated) st_scalar<false, uint8_t>(a.truncated + env, (uint8_t)trunc);
        if constexpr (LEARN) {
            if (a.reward_f32) a.reward_f32[env] = (float)rwd;
            if (a.done_f32) a.done_f32[env] = triv ? 1.0f : 0.0f;
            if (a.episode_len) a.episode_len[env] = (triv || trunc) ? cnt : 0;
        }
        if (a.pending) a.pending[env] = fin ? 1 : 0;
        // final_obs <- post-move state (per lane: rare, and only with final_obs)
        if (reset && a.final_obs) regs_to_global<PW>(a.final_obs + env * twoL, p, L);
    }
    // out-of-domain rows the load did not flag (a zero inside a relator: CodeTile's slots cannot
    // hold it) are stored from their input row too
    tile.flag_rows(w.lane, (w.active && e == ACX_ERR_DOMAIN) ? FB_IN : 0u);
    const uint64_t rb = __ballot(reset);
    if (rb) {
        // same-step autoreset to the env's starting state.  An out-of-domain starting row is
        // taken as it is, like the reference's reset (ac_env.py:113-129, no validation): the
        // env's row becomes that row's exact values (copied from reset_state, FB_RESET), its
        // step count 0 and its err ACX_ERR_DOMAIN; from then on it is an out-of-domain row.
        bool rbad = false;
        if (__popcll(rb) > RESET_TILE_MIN) {
            // many lanes (a synchronised truncation): one coalesced load of the tile's starting
            // states (per-lane reads of every row cost ~1 ms on a whole-batch truncation step);
            // the other lanes re-stage their state, rows left as loaded copy state_in
            wave_sync();
            tile.load(a.reset_state + w.r0 * twoL, w.R, w.lane);
            if (reset) rbad = tile.pack(w.lane, p);
            wave_sync();
            if (w.active && !keep && !rbad) tile.unpack(w.lane, p);
            dm = (w.active && !keep) ? 3u : 0u;  // the tile now holds starting rows: write every kept-moving row
            tile.restore_flags(w.lane, (w.active && keep) ? FB_IN : (rbad ? FB_RESET : 0u));
        } else {
            // a few lanes: the wave loads just their rows (scattered resets cost their rows only),
            // those it has not fetched before the move
            const uint64_t late = rb & ~pre;
            if (late) tile.load_rows(a.reset_state + w.r0 * twoL, late, w.R, w.lane);
            if (reset) {
                // the tile row already holds the starting row's image (what unpack would write
                // for a row in the domain; a row outside it is stored from its fallback): pack
                // only checks it and sets the lengths
                rbad = tile.pack(w.lane, p);
                dm = 3u;
            }
            tile.flag_rows(w.lane, rbad ? FB_RESET : 0u);
        }
        if (rbad) e = ACX_ERR_DOMAIN;  // lengths_out: the non-zero counts of the starting row
        if (reset) cnt = 0;
    }
    if (sure && fin) {  // the curriculum copy writes the row (no autoreset above: rb has none of them)
        cnt = 0;
        dm = 0u;
    }
    if (w.active) {
        if (a.step_count) st_scalar<false, int32_t>(a.step_count + env, cnt);
        if (a.lengths_out) {
            // lengths-carrying step: an out-of-domain row is read whole on the next call (L, L)
            const bool whole = LIVE && e == ACX_ERR_DOMAIN;
            st_scalar<false, int32_t>(a.lengths_out + 2 * env, whole ? L : (skip && skip_h == 0) ? n_skip : p.n0);
            st_scalar<false, int32_t>(a.lengths_out + 2 * env + 1, whole ? L : (skip && skip_h == 1) ? n_skip : p.n1);
        }
        // a moved row is reduced: freely, and cyclically too when cyclical (simplify_presentation,
        // utils.py:246-283) -- but may hold an empty relator (validity is asserted before the
        // reduction, :264-266: an unreduced y^-1 y empties); a failed, reset or out-of-domain row
        // is read whole next time
        if (LIVE && a.reduced) {
            const bool full = (p.n0 > 0 || (skip && skip_h == 0)) && (p.n1 > 0 || (skip && skip_h == 1));
            st_scalar<false, uint8_t>(
                a.reduced + env,
                (uint8_t)((!keep && !reset && !pend && e == ACX_ERR_NONE && full) ? (a.cyclical ? 3 : 1) : 0));
        }
        if (a.err) st_scalar<false, uint8_t>(a.err + env, (uint8_t)e);
        if (e != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    if (a.in_place) {
        // state_out == state_in: write only the relators that changed (a gated move, a
        // cyclic conjugation that is a no-op and a failed env leave their row as it is in HBM);
        // lengths-carrying: of those, only the chunks inside the old or the new letters
        tile.set_dirty(w.lane, dm);
        if constexpr (LIVE) tile.widen_lim(w.lane, p.n0, p.n1);
        wave_sync();
        if (__ballot(dm != 0u)) {
            if constexpr (LIVE)
                tile.template store_dirty<NT_WRITEBACK, true>(a.state_out + w.r0 * twoL, w.R, w.lane,
                                                       a.reset_state + w.r0 * twoL);
            else
                tile.template store_dirty<NT_WRITEBACK>(a.state_out + w.r0 * twoL, w.R, w.lane, a.reset_state + w.r0 * twoL);
        }
    } else {
        wave_sync();
        tile.template store<true, NT_STATE>(a.state_out + w.r0 * twoL, twoL, w.R, a.state_in + w.r0 * twoL,
                                                     twoL, w.lane,
                                  a.reset_state + w.r0 * twoL);
    }
    if (LEARN && a.obs_f32)  // the same rows as float32, straight into the learner's buffer
        tile.template store<true, NT_OBS, true>(reinterpret_cast<int32_t*>(a.obs_f32) + w.r0 * twoL, twoL, w.R,
                                               a.state_in + w.r0 * twoL, twoL, w.lane, a.reset_state + w.r0 * twoL,
                                               sure ? fm : 0ull);
    if (cur) {
        // The curriculum's tail (training.py:329-336, 349-352).  A finished env was reset to its own
        // starting row above like any env; now -- every store of the tile issued, so the memory
        // system stays busy while a tile waits -- a tile with finished envs waits for its prefix
        // and each finished env with index k = prefix + (finished envs before it in the tile) <
        // n_states takes initial state k: its state, obs_f32 and reset_state rows are overwritten
        // with that row as it is (acx_curriculum_assign's copy; a row outside the packed domain
        // is then reported with err 3 by the next step) and curr_index = k; past the table's end
        // (round 1 complete) needs_host = 1 and the host draws.  The last tile waits for the total
        // (the new next_index).  The copies are made by the whole wave, 16-byte chunks over the
        // lanes (copy_rows): one lane copying its own row made the steady-state step 0.165 ms
        // instead of 0.150 (r05zg).
        const uint32_t first = broken ? CUR_FAIL : (fm && !exhausted) ? cur_prefix(a, w, cseq, false) : 0u;
        if (!broken && w.r0 + w.R == a.B) {
            const uint32_t tot = cur_prefix(a, w, cseq, true);
            if (w.lane == 0) {
                // every group is complete: no wave of this launch reads next_index or the sequence
                // number again -- advance both for the next one.  A total that never arrived leaves
                // next_index stale: the workspace is marked failed (the host restores both)
                if (tot != CUR_FAIL) {
                    *a.cur_next = (int32_t)((int64_t)tot < a.n_states ? (int64_t)tot : a.n_states);
                    cur_store(a.cur_ws, (uint64_t)((cseq + 1u) & CUR_SEQ_MASK));
                } else {
                    cur_set_failed(a);
                }
            }
        }
        const bool failed = first == CUR_FAIL;  // wave-uniform
        if (failed && !broken && w.lane == 0) cur_set_failed(a);
        // finished envs with index k = first + (finished envs before it in the tile) < n_states
        uint64_t take = 0;
        if (fm && !exhausted && !failed) {
            const int64_t nq = a.n_states - (int64_t)first;  // how many of the tile's finished envs get a state
            take = fm;
            while (take && (int64_t)__popcll(take) > nq) take &= ~(1ull << (63 - __builtin_clzll(take)));
        }
        if (take) {
            // the rows were autoreset above (a failed ranking leaves them so): the tile's own
            // stores of them complete first -- unless `sure`: the tile left them out
            if (!sure) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            copy_rows(a, w, take, twoL, [&](int q, int) { return a.cur_states + ((int64_t)first + q) * twoL; }, true);
        }
        // `sure` and a finished env without a state (a failed ranking): its own starting row, as the
        // autoreset would have left it
        const uint64_t own = sure ? (fm & ~take) : 0ull;
        if (own) copy_rows(a, w, own, twoL, [&](int, int r) { return a.reset_state + (w.r0 + r) * twoL; }, false);
        if (w.active) {
            uint8_t nh = 0;
            if (fin) {
                if (failed) nh = 3;
                else if ((take >> w.lane) & 1ull) a.curr_index[env] = (int32_t)((int64_t)first + __popcll(fm & ((1ull << w.lane) - 1ull)));
                else nh = 1;
            }
            a.needs_host[env] = nh;
        }
    }
}

template <int NW, int LC, int VEC, bool LEARN>
__global__ __launch_bounds__(BLOCK, Occupancy<LC>::waves_per_simd) void step_kernel(StepArgs a) {
    step_body<NW, LC, VEC, LEARN, false>(a);
}
// ---------------------------------------------------------------------------------
// Small batches: two lanes per env (BASELINE configs[1]: 65,536 envs at L = 36).
//
// With one lane per env, 65,536 envs are 1,024 waves -- one per SIMD: nothing hides a wave's
// load -> pack -> move -> unpack -> store chain, and a lone wave issues a VALU instruction every
// 4 cycles instead of every 2 (MI355X_MICROARCH.md, "vector-instruction ISSUE cost").
// step_pair_kernel gives each env two lanes of a 32-env tile, lane 2e + h holding relator h of
// env e, so the same batch is 2,048 waves and the per-relator work is split between the lanes:
//   * the tile (32 rows, 18 16-byte chunks each) is read with 9 coalesced loads per lane into an
//     int8 image in LDS; relator q of the tile (q = 2e + h) is chunks [9q, 9q + 9) -- lane q's;
//   * lane q packs ITS relator into bit planes (pl::, one 64-bit word per plane at L <= 64) and
//     takes its partner's planes and length with four DPP quad-permutes (quad_perm [1,0,3,2]);
//   * the move is split over the pair (pl::pair_move_clean: the target lane moves its relator,
//     the junction cancellation count and the cyclic peel are the first set bit of a mismatch
//     mask, the splice is shifts of the planes); an unreduced env runs the general move on both;
//   * lane q decides on the planes whether its relator changed; in the common case (in place, full
//     tile, no out-of-domain reset) it writes that relator's 9 chunks straight from its planes.
//     Otherwise the moved relators are re-imaged into the tile and the "changed" bits, the rows'
//     fallback codes and the error flags -- wave ballots, one bit per relator, bit q <-> chunks
//     [9q, 9q + 9) -- steer a coalesced write-back that tests chunk c against bit c / 9.
// Results are those of step_body<..., LEARN = false, LIVE = false> (the same pack, move,
// image and error contract; tests/test_gpu_*: every acx_step test at L = 36 and B <= 131,072 runs
// here); only the instruction schedule differs.  launch_step takes it for B <= SMALL_STEP_MAX_B.
// ---------------------------------------------------------------------------------
constexpr int64_t SMALL_STEP_MAX_B = (int64_t)2 * 4 * 256 * WAVE;  // <= 4 pair-waves per SIMD on 256 CUs
template <int NW, int LC, int VEC>
constexpr bool small_step_ok() {
    return std::is_same<TileFor<NW, LC, VEC>, FastTile<NW, LC>>::value && LC <= 64;
}

// partner lane's value (lane ^ 1): DPP quad_perm [1,0,3,2], full-rate VALU, no LDS
__device__ __forceinline__ uint32_t pair_xchg(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t pair_xchg64(uint64_t v) {
    return (uint64_t)pair_xchg((uint32_t)v) | ((uint64_t)pair_xchg((uint32_t)(v >> 32)) << 32);
}

template <int LC>
struct PairLayout {
    static constexpr int CPR = LC / 2;          // 16-byte chunks per row
    static constexpr int HALF = CPR / 2;        // chunks (= image dwords) per relator
    static constexpr int ENVS = WAVE / 2;       // envs per wave
    static constexpr int NCH = ENVS * CPR;      // chunks per full tile
    static constexpr int U = NCH / WAVE;        // chunk loads per lane (full tile)
    static_assert(LC % 4 == 0 && LC <= 64 && HALF * 2 == CPR && U * WAVE == NCH, "pair tile layout");
    static constexpr size_t wave_bytes = (size_t)NCH * 4 + WAVE;  // int8 image + one flag byte per relator
};

// relator image (HALF dwords of int8 letters, zero padding) -> its planes and length; true if
// outside the domain (a zero inside the relator): FastTile::pack on one relator
template <int HALF>
__device__ __forceinline__ bool pair_pack(const uint32_t* src, Planes<1>& w, int& n) {
    uint64_t s = 0, y = 0, nz = 0;
#pragma unroll
    for (int k = 0; k < HALF; k += 2) {
        const uint32_t d0 = src[k];
        const uint32_t d1 = k + 1 < HALF ? src[k + 1] : 0u;
        uint32_t s8, y8, z8;
        pl::i8x8_to_bytes(d0, d1, s8, y8, z8);
        s |= (uint64_t)s8 << (4 * k);
        y |= (uint64_t)y8 << (4 * k);
        nz |= (uint64_t)z8 << (4 * k);
    }
    w.s[0] = s;
    w.y[0] = y;
    n = __builtin_popcountll(nz);
    return nz != pl::bmask<1>(n).b[0];  // zeros only as right padding <=> mask == low n bits
}

// planes -> the relator's int8 image in dst; returns true if it differs from what dst held
template <int HALF>
__device__ __forceinline__ bool pair_image(uint32_t* dst, const Planes<1>& w, int n) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
        const uint32_t d = pl::nibbles_to_i8x4(pl::nib<1>(w.s, k), pl::nib<1>(w.y, k), clamp_bits(8 * n - 32 * k));
        x |= dst[k] ^ d;
        dst[k] = d;
    }
    return x != 0u;
}

// a relator's int32 letters (HALF chunks from src) -> its int8 image in dst; true if a letter is
// outside {-2..2} (the image then holds 0x7f there, as FastTile::load_rows)
template <int HALF>
__device__ __forceinline__ bool pair_load_relator(uint32_t* dst, const int32_t* src) {
    int4 v[HALF];
#pragma unroll
    for (int k = 0; k < HALF; ++k) v[k] = reinterpret_cast<const int4*>(src)[k];
    bool bad = false;
#pragma unroll
    for (int k = 0; k < HALF; ++k)
        dst[k] = to_i8(v[k].x, bad) | (to_i8(v[k].y, bad) << 8) | (to_i8(v[k].z, bad) << 16) | (to_i8(v[k].w, bad) << 24);
    return bad;
}

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK, 4) void step_pair_kernel(StepArgs a) {
    using PT = PairLayout<LC>;
    constexpr int L = LC, twoL = 2 * LC, CPR = PT::CPR, HALF = PT::HALF, ENVS = PT::ENVS;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wid) * ENVS;  // wave-uniform
    if (r0 >= a.B) return;
    const int R = (int)((a.B - r0) < ENVS ? (a.B - r0) : ENVS);
    const int er = lane >> 1, h = lane & 1;  // env (tile row) and relator of this lane
    const bool active = er < R;
    const int64_t env = r0 + er;
    uint32_t* img = reinterpret_cast<uint32_t*>(smem + wid * PT::wave_bytes);
    uint8_t* rflag = reinterpret_cast<uint8_t*>(img + PT::NCH);  // per relator: a bad chunk at load (rare path)
    uint32_t* mine = img + lane * HALF;                          // this lane's relator image

    // scalars first: their latency hides under the tile's loads (both lanes of an env read the
    // same words; the second is a cache hit)
    int act = 0, cnt0 = 0;
    bool pend = false;
    if (active) {
        act = a.action[env];
        cnt0 = a.step_count ? a.step_count[env] : 0;
        pend = a.pending && a.pending[env] != 0;  // next-step autoreset: reset now
    }
    // the tile: chunk c = lane + 64u of the tile's rows (coalesced), relator c / HALF
    bool flagged = false;  // this lane's relator has a chunk with a letter outside {-2..2}
    {
        const int4* src = reinterpret_cast<const int4*>(a.state_in + r0 * twoL) + lane;
        uint32_t badm = 0;  // bit u: chunk lane + 64u
        if (R == ENVS) {  // full tile (wave-uniform): every load in flight at once
            int4 v[PT::U];
#pragma unroll
            for (int u = 0; u < PT::U; ++u) v[u] = src[u * WAVE];
#pragma unroll
            for (int u = 0; u < PT::U; ++u) {
                bool bad;
                img[lane + u * WAVE] = chunk_i8(v[u], bad);
                badm |= (uint32_t)bad << u;
            }
        } else {
            const int nc = R * CPR;
#pragma unroll
            for (int u = 0; u < PT::U; ++u) {
                const int c = lane + u * WAVE;
                if (c < nc) {
                    bool bad;
                    img[c] = chunk_i8(src[u * WAVE], bad);
                    badm |= (uint32_t)bad << u;
                }
            }
        }
        if (__any(badm != 0u)) {
            // rare (wave-uniform): the flagged relators are found through LDS, and chunk_i8's
            // arbitrary bytes in them re-imaged letter by letter (an out-of-domain letter ->
            // 0x7f), so the letter counts the contract reports for the row (reward, lengths) are
            // those of the input row
            rflag[lane] = 0;
            wave_sync();
#pragma unroll
            for (int u = 0; u < PT::U; ++u)
                if ((badm >> u) & 1u) rflag[(lane + u * WAVE) / HALF] = 1;
            wave_sync();
            flagged = rflag[lane] != 0;
            if (active && flagged) pair_load_relator<HALF>(mine, a.state_in + env * twoL + h * L);
        }
        wave_sync();
    }

    // this lane's relator -> planes and its reversal; the partner's by DPP
    const bool cyc = a.cyclical != 0;
    Planes<1> w;
    int n;
    bool bad = pair_pack<HALF>(mine, w, n) || flagged;
    const Planes<1> w_in = w;  // the relator as loaded: "changed" is decided on the planes
    const int n_in = n;
    const Planes<1> rw = pl::prev<1>(w, n);
    bool clean = pl::relator_clean<1>(w, n, cyc);
    Planes<1> pw, prw;
    int pn;
    {
        pw.s[0] = pair_xchg64(w.s[0]);
        pw.y[0] = pair_xchg64(w.y[0]);
        prw.s[0] = pair_xchg64(rw.s[0]);
        prw.y[0] = pair_xchg64(rw.y[0]);
        const uint32_t x = pair_xchg((uint32_t)n | (bad ? 0x100u : 0u) | (clean ? 0x200u : 0u));
        pn = (int)(x & 0xffu);
        bad = bad || (x & 0x100u) != 0u;
        clean = clean && (x & 0x200u) != 0u;
    }

    // the env's move: on a clean env (both relators reduced) each lane runs its relator's part of
    // it (pl::pair_move_clean: the target lane moves, its partner keeps its relator); otherwise
    // (an unreduced start: rare) both lanes run the general move on the whole env
    int e = ACX_ERR_NONE;
    bool general = false;
    if (active) {
        if (pend) e = ACX_ERR_NONE;  // no move: the env resets (gymnasium >= 1.0 NEXT_STEP autoreset)
        else if (bad) e = ACX_ERR_DOMAIN;
        else if (clean) e = pl::pair_move_clean(w, n, rw, pw, pn, prw, h, act, L, cyc);
        else general = true;
    }
    if (general) {
        PlaneRegs<1> q;
        q.w0 = h ? pw : w;
        q.w1 = h ? w : pw;
        q.n0 = h ? pn : n;
        q.n1 = h ? n : pn;
        const pl::MoveOut<1> mo = pl::ac_move_call<1>(q, act, L, cyc);
        e = mo.e;
        w = h ? mo.p.w1 : mo.p.w0;
        n = h ? mo.p.n1 : mo.p.n0;
    }
    // the env's code is its target lane's (ac_moves.py:167-179: relator (id + 1) & 1; every other
    // outcome is the same on both lanes); the partner's new length and letter-0 y bit
    bool xy = false;  // the relators' first letters: one x^{+-1} and one y^{+-1}
    {
        const uint32_t x = pair_xchg((uint32_t)e | ((uint32_t)n << 8) | ((uint32_t)(w.y[0] & 1u) << 16));
        if (h != ((act + 1) & 1)) e = (int)(x & 0xffu);
        pn = (int)((x >> 8) & 0xffu);
        xy = ((x >> 16) & 1u) != (uint32_t)(w.y[0] & 1u);
    }
    const int n0 = h ? pn : n, n1 = h ? n : pn;
    int cnt = 0;
    bool keep = false, triv = false, trunc = false, fin = false, reset = false;
    int32_t rwd = 0;
    if (active) {
        cnt = a.step_count ? cnt0 + 1 : 0;
        keep = e != ACX_ERR_NONE;
        if (keep) cnt = cnt0;  // the reference raises before count_steps += 1 (ac_env.py:93-102)
        // strict triviality (pl::is_trivial): both relators one letter, one x and one y
        triv = !pend && !keep && n0 == 1 && n1 == 1 && xy;
        trunc = !pend && !keep && a.step_count && cnt >= a.horizon;
        rwd = pend ? 0 : triv ? a.horizon * L * 2 : -(n0 + n1);
        fin = triv || trunc;
        reset = a.pending ? pend : (fin && a.reset_state && !keep);
    }
    // this lane's relator changed (a failed env keeps its row): compared on the planes (canonical:
    // no bits past the letters), so the common store below needs no re-imaged tile
    bool chg = false;
    if (active && !keep) {
        const uint64_t m = pl::bmask<1>(n).b[0];
        chg = n != n_in || (((w.s[0] ^ w_in.s[0]) | (w.y[0] ^ w_in.y[0])) & m) != 0ull;
    }
    // same-step autoreset (or a pending env's reset): the lane loads its relator of the starting
    // row into the image (FastTile::load_rows' result; an out-of-domain starting row is taken as it
    // is and stored from reset_state, FB_RESET)
    bool rbad = false;
    int rn = n;
    if (active && reset) {
        if (a.final_obs) {  // final_obs <- the post-move state (rare): each lane its relator
            int32_t* fo = a.final_obs + env * twoL + h * L;
#pragma unroll 1
            for (int k = 0; k < L; ++k) {
                const uint32_t code = pl::pletter<1>(w, k);
                fo[k] = k < n ? (int32_t)(int8_t)((0xFE02FF01u >> (code << 3)) & 0xffu) : 0;
            }
        }
        rbad = pair_load_relator<HALF>(mine, a.reset_state + env * twoL + h * L);
        Planes<1> rw2;
        rbad = pair_pack<HALF>(mine, rw2, rn) || rbad;
        chg = true;  // dm = 3: the whole row is written
    }
    // the partner's starting-row length and domain flag (every lane takes part in the DPP)
    int ln0 = n0, ln1 = n1;  // lengths_out
    {
        const uint32_t x = pair_xchg((uint32_t)rn | (rbad ? 0x100u : 0u));
        if (reset) {
            rbad = rbad || (x & 0x100u) != 0u;
            ln0 = h ? (int)(x & 0xffu) : rn;
            ln1 = h ? rn : (int)(x & 0xffu);
        }
    }
    if (rbad) e = ACX_ERR_DOMAIN;  // lengths_out: the non-zero counts of the starting row
    if (reset) cnt = 0;
    // per-env outputs: lane 0 of the pair the env's scalars, lane 1 the lengths
    if (active) {
        if (h == 0) {
            if (a.reward) a.reward[env] = rwd;
            if (a.done) a.done[env] = (uint8_t)triv;
            if (a.truncated) a.truncated[env] = (uint8_t)trunc;
            if (a.pending) a.pending[env] = fin ? 1 : 0;
            if (a.step_count) a.step_count[env] = cnt;
            if (a.err) a.err[env] = (uint8_t)e;
            if (e != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
        } else if (a.lengths_out) {
            a.lengths_out[2 * env] = ln0;
            a.lengths_out[2 * env + 1] = ln1;
        }
    }

    // the state store.  Relator masks, bit q = relator q of the tile (chunks [9q, 9q + 9)):
    //   fb_in    rows stored from their input row (out of domain, not reset: FB_IN)
    //   fb_rst   rows stored from their starting row (reset to an out-of-domain row: FB_RESET)
    //   dirty    relators that differ from state_in (in place: the only chunks written)
    const uint64_t fb_rst = __ballot(active && reset && rbad);
    const uint64_t fb_in = __ballot(active && !reset && e == ACX_ERR_DOMAIN);
    const uint64_t dirty = __ballot(active && chg);
    if (a.in_place && fb_rst == 0ull && R == ENVS) {
        // the common case (wave-uniform): each lane writes its own changed relator, 9 contiguous
        // 16-byte chunks, straight from its planes (or, reset, from the starting row it loaded
        // into its image) -- no re-imaged tile, no tile-wide LDS pass
        if (dirty == 0ull) return;
        if (chg) {
            int4* d = reinterpret_cast<int4*>(a.state_out + env * twoL + h * L);
            if (reset) {
#pragma unroll
                for (int k = 0; k < HALF; ++k) out16<NT_WRITEBACK, false>(d + k, widen4(mine[k]));
            } else {
#pragma unroll
                for (int k = 0; k < HALF; ++k)
                    out16<NT_WRITEBACK, false>(
                        d + k, widen4(pl::nibbles_to_i8x4(pl::nib<1>(w.s, k), pl::nib<1>(w.y, k), clamp_bits(8 * n - 32 * k))));
            }
        }
        return;
    }
    // otherwise the tile's image (moved relators re-imaged) and the coalesced stores below
    if (active && !keep && !reset) pair_image<HALF>(mine, w, n);
    wave_sync();
    const int nc = R * CPR;
    int4* dst = reinterpret_cast<int4*>(a.state_out + r0 * twoL);
    const int4* fin_row = reinterpret_cast<const int4*>(a.state_in + r0 * twoL);
    const int4* frs_row = reinterpret_cast<const int4*>(a.reset_state ? a.reset_state + r0 * twoL : a.state_in);
    if (a.in_place) {
        if (dirty == 0ull) return;
        // dirty and fb_in never share a relator (a failed env is not dirty)
        if (fb_rst == 0ull && R == ENVS) {
            // the common case (wave-uniform): every image dword read first (one LDS wait, not one
            // per chunk), then the dirty chunks stored
            uint32_t v[PT::U];
#pragma unroll
            for (int u = 0; u < PT::U; ++u) v[u] = img[lane + u * WAVE];
#pragma unroll
            for (int u = 0; u < PT::U; ++u) {
                const int c = lane + u * WAVE;
                if ((dirty >> (c / HALF)) & 1ull) out16<NT_WRITEBACK, false>(dst + c, widen4(v[u]));
            }
            return;
        }
#pragma unroll
        for (int u = 0; u < PT::U; ++u) {
            const int c = lane + u * WAVE;
            if (c >= nc) continue;
            const int q = c / HALF;
            if (!((dirty >> q) & 1ull)) continue;
            if ((fb_rst >> q) & 1ull) dst[c] = frs_row[c];
            else out16<NT_WRITEBACK, false>(dst + c, widen4(img[c]));
        }
    } else {
#pragma unroll
        for (int u = 0; u < PT::U; ++u) {
            const int c = lane + u * WAVE;
            if (c >= nc) continue;
            const int q = c / HALF;
            if ((fb_rst >> q) & 1ull) dst[c] = frs_row[c];
            else if ((fb_in >> q) & 1ull) dst[c] = fin_row[c];
            else dst[c] = widen4(img[c]);
        }
    }
}

// acx_step_lengths (in place, lengths in and out).  At L = 128 the tile's LDS allows 4 waves per
// SIMD; the live-chunk predicates took the register count just past 128 VGPRs (3 waves), so
// the allocator is held to 4
template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK, LC == 128 ? 4 : Occupancy<LC>::waves_per_simd) void step_lengths_kernel(StepArgs a) {
    step_body<NW, LC, VEC, false, true>(a);
}

struct RolloutArgs {
    int32_t* state;
    const int32_t* actions;
    const uint32_t* packed;  // or: move ids pre-packed by pack_actions_kernel (actions unused)
    const int32_t* reset_state;
    int32_t* step_count;
    int32_t* obs_traj;
    int32_t* reward_traj;
    uint8_t* done_traj;
    uint8_t* trunc_traj;
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int T, L, horizon, cyclical;
    int8_t* obs_traj8;  // acx_rollout_obs8: the trajectory as int8 letters (obs_traj unused)
};

// OBS: 0 no trajectory, 1 int32 obs trajectory (obs_traj), 2 int8 obs trajectory (obs_traj8)
template <int NW, int LC, int VEC, int OBS>
__global__ __launch_bounds__(BLOCK, Occupancy<LC>::waves_per_simd) void rollout_kernel(RolloutArgs a) {
    using Tile = TileFor<NW, LC, VEC>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    WaveCtx w;
    if (!wave_ctx(a.B, w)) return;
    Tile tile(smem + w.wid * Tile::wave_bytes(a.L), a.L);
    const int L = tile.Lr(), twoL = 2 * L;
    const int64_t env = w.r0 + w.lane;

    // starting states are read only when an episode ends (not kept in registers, which are
    // the rollout's occupancy limit): by the resetting lane alone, or by a coalesced reload of
    // the tile when many lanes of the wave reset together.
    // Errors follow acx_step exactly, so T launches of acx_step give the same trajectory: a
    // failed move (err 1, 2, 4) leaves the state and the step count as they are for that step
    // (done = truncated = 0, reward = -(n0+n1)); an out-of-domain row (err 3: the input row, or
    // a starting row an autoreset loaded -- then held as that row, count 0) never moves and
    // never counts; its observations are its exact int32 values (fallback rows, FB_*).
    bool bad = false;
    bool bad_reset = false;  // the out-of-domain row is the env's starting row (FB_RESET)
    constexpr int PW = Tile::PW;
    PlaneRegs<PW> p;
    tile.template load<false, false, true>(a.state + w.r0 * twoL, w.R, w.lane);
    int first_err = ACX_ERR_NONE;
    int cnt = 0;
    const bool cyc = a.cyclical != 0;
    bool clean = false;
    if (w.active) {
        bad = tile.pack(w.lane, p);
        cnt = a.step_count[env];
        if (bad) first_err = ACX_ERR_DOMAIN;
        clean = pl::is_clean<PW>(p.w0, p.n0, p.w1, p.n1, cyc);
    }
    const int32_t max_reward = a.horizon * L * 2;
    // Drain the prologue's loads here: otherwise the waitcnt pass carries the pending
    // step_count load around the loop back-edge and waits vmcnt(0) (= for every store of
    // the previous step) at each use of `cnt`.
    __builtin_amdgcn_s_waitcnt(0);
    const int32_t* act_tile = a.actions + w.r0;  // wave-uniform

    // One env step of the wave: move, reward/done/truncated, autoreset, obs rows.
    auto step = [&](int t, uint32_t id) {
        const int64_t ti = (int64_t)t * a.B;
        // opaque per step: keeps uniform-base + lane addressing in the loop (hoisted 64-bit
        // per-lane pointers are what the register allocator spills)
        // the lane index recomputed per step (v_mbcnt), not held across the loop: a live copy
        // was what the register allocator spilled, and its reload put a vmcnt(0) -- a drain of
        // the previous step's stores -- at the top of every step
        const int lane = (int)__lane_id();
        int ln = lane;
        asm volatile("" : "+v"(ln));
        bool reset = false;
        bool both = false;  // the LDS image needs both relators (general move: both reduced)
        bool h1 = false;    // the moved relator (ac_moves.py:167-179: i = (id + 1) & 1)
        if (w.active) {
            const int act = (int)id;
            int e;
            both = !clean;
            h1 = ((act + 1) & 1) != 0;
            if (bad) e = ACX_ERR_DOMAIN;
            else if (clean) e = pl::ac_move_clean<PW>(p.w0, p.n0, p.w1, p.n1, act, L, cyc);
            else {
                const pl::MoveOut<PW> mo = pl::ac_move_call<PW>(p, act, L, cyc);
                p = mo.p;
                e = mo.e;
            }
            const bool ok = e == ACX_ERR_NONE;
            // a successful general move leaves both relators reduced -- clean unless the
            // reduction emptied one (an unreduced input like [y^-1 y]: the reference keeps going
            // with the empty relator, utils.py:264-266 checks only before the reduction)
            clean = clean || (ok && p.n0 > 0 && p.n1 > 0);
            if (first_err == ACX_ERR_NONE) first_err = e;
            const bool triv = ok && pl::is_trivial<PW>(p.w0, p.n0, p.w1, p.n1);
            cnt += ok ? 1 : 0;  // the reference raises before count_steps += 1 (ac_env.py:93-102)
            const bool trunc = ok && cnt >= a.horizon;
            if (a.reward_traj) st_scalar<false, int32_t>(a.reward_traj + ti + w.r0 + ln, triv ? max_reward : -(p.n0 + p.n1));
            if (a.done_traj) st_scalar<false, uint8_t>(a.done_traj + ti + w.r0 + ln, (uint8_t)triv);
            if (a.trunc_traj) st_scalar<false, uint8_t>(a.trunc_traj + ti + w.r0 + ln, (uint8_t)trunc);
            reset = triv || trunc;
            if (reset) cnt = 0;
        }
        const uint64_t rb = __ballot(reset);
        bool reloaded = false;  // wave-uniform: the whole tile now holds starting rows
        if (rb) {  // same-step autoreset to the starting states
            bool rbad = false;
            if (__popcll(rb) > RESET_TILE_MIN) {  // many lanes: one coalesced tile reload
                tile.load(a.reset_state + w.r0 * twoL, w.R, lane);
                if (reset) rbad = tile.pack(lane, p);
                wave_sync();
                reloaded = true;
            } else {  // a few lanes: the wave loads just their rows
                tile.load_rows(a.reset_state + w.r0 * twoL, rb, w.R, lane);
                if (reset) rbad = tile.pack(lane, p);
            }
            if (reset) {
                clean = pl::is_clean<PW>(p.w0, p.n0, p.w1, p.n1, cyc);
                bad = rbad;
                bad_reset = rbad;
                if (rbad && first_err == ACX_ERR_NONE) first_err = ACX_ERR_DOMAIN;
            }
        }
        if constexpr (OBS != 0) {
            // the LDS tile stays the int8 image of the current states: a clean move re-images
            // its target relator, a general move both; a row reset by load_rows already holds its
            // starting row; after a whole-tile reload every row is re-imaged
            if (w.active && !bad) {
                if (reloaded || both) tile.unpack(lane, p);
                else if (!reset) tile.unpack_half(lane, p, h1);
            }
            if (__ballot(w.active && bad)) {
                // rare: out-of-domain rows as their exact values from their fallback rows
                tile.restore_flags(lane, (w.active && bad) ? (bad_reset ? FB_RESET : FB_IN) : 0u);
                if constexpr (OBS == 1)
                    tile.template store<true>(a.obs_traj + (ti + w.r0) * twoL, twoL, w.R, a.state + w.r0 * twoL, twoL,
                                              lane, a.reset_state + w.r0 * twoL);
                else
                    store_rows_i8_fb(tile, a.obs_traj8 + (ti + w.r0) * twoL, w.R, twoL, lane, a.state + w.r0 * twoL,
                                     a.reset_state + w.r0 * twoL);
                wave_sync();
                return;
            }
            wave_sync();
            if constexpr (OBS == 1) {
                tile.template store_rows<NT_OBS>(a.obs_traj + (ti + w.r0) * twoL, w.R, lane);
            } else {
                tile.template store_rows_i8<NT_OBS>(a.obs_traj8 + (ti + w.r0) * twoL, w.R, lane);
            }
            wave_sync();
        }
    };
    // ids outside [0,12) -> 15 (ACX_ERR_ACTION in ac_move)
    auto decode = [](int32_t v) { return (uint32_t)v < 12u ? (uint32_t)v : 15u; };

    // Move ids are loaded ACT_BLOCK steps at a time and kept packed, 4 bits each, in
    // ACT_BLOCK/8 registers.  The wait for a load issued after trajectory stores covers those
    // stores too (loads and stores pending on vmcnt may complete out of order, so the
    // compiler waits vmcnt(0)): a drain of the wave's write queue.  8-step batches cost 8 %
    // of the rollout in drains (tools/store_pattern.py, ACT8 vs none); with obs stores the
    // batch is 32 steps, loaded as four groups of 8 (only the first wait finds stores).
    constexpr int ACT_BLOCK = OBS != 0 ? 32 : 8;
    constexpr int ACT_GROUP = 8;
    constexpr int QW = ACT_BLOCK / 8;
    uint32_t q[QW];
#pragma unroll
    for (int k = 0; k < QW; ++k) q[k] = 0;
    for (int t = 0; t < a.T; ++t) {
        if ((t & (ACT_BLOCK - 1)) == 0) {
            // recomputed (v_mbcnt), not kept live across the loop
            int lc = (int)__lane_id();
            lc = lc < w.R ? lc : 0;
            if (a.packed) {  // one uint32 per 8 steps (acx_pack_actions)
                const uint32_t* pk = a.packed + (int64_t)(t >> 3) * a.B + w.r0;
#pragma unroll
                for (int g = 0; g < QW; ++g) q[g] = t + 8 * g < a.T ? (pk + (int64_t)g * a.B)[lc] : 0u;
            } else {
#pragma unroll
            for (int g = 0; g < ACT_BLOCK / ACT_GROUP; ++g) {
                int32_t v[ACT_GROUP];
#pragma unroll
                for (int k = 0; k < ACT_GROUP; ++k) {
                    const int tk = t + g * ACT_GROUP + k;
                    v[k] = tk < a.T ? (act_tile + (int64_t)tk * a.B)[lc] : 0;
                }
                uint32_t qg = 0;
#pragma unroll
                for (int k = 0; k < ACT_GROUP; ++k) qg |= decode(v[k]) << (4 * k);
                q[g] = qg;
            }
            }
            // consume the loaded words here: otherwise the waitcnt pass sees them pending where
            // this block rejoins the step and puts a vmcnt(0) on the first use of the move id in
            // EVERY step (a drain of the wave's previous trajectory stores per step)
#pragma unroll
            for (int k = 0; k < QW; ++k) asm volatile("" ::"v"(q[k]));
        }
        const uint32_t id = q[0] & 15u;
#pragma unroll
        for (int k = 0; k < QW; ++k) q[k] = (q[k] >> 4) | (k + 1 < QW ? q[k + 1] << 28 : 0u);
        step(t, id);
    }
    if (w.active) {
        if (!bad) tile.unpack(w.lane, p);
        a.step_count[env] = cnt;
        if (a.err) a.err[env] = (uint8_t)first_err;
        if (first_err != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    // out-of-domain rows: their input row (untouched in HBM), or the starting row they reset to
    tile.restore_flags(w.lane, (w.active && bad) ? (bad_reset ? FB_RESET : FB_IN) : 0u);
    tile.template store<true, NT_STATE>(a.state + w.r0 * twoL, twoL, w.R, a.state + w.r0 * twoL, twoL,
                                                 w.lane, a.reset_state + w.r0 * twoL);
}

// Move ids (T, B) int32 -> (ceil(T/8), B) uint32, 8 consecutive steps of one env per word,
// 4 bits each (ids outside [0,12) -> 15, ACX_ERR_ACTION).  The rollout then reads 0.5 B per
// env-step instead of 4: its action reads are small scattered requests between trajectory
// write bursts, and at 4 B they cost 7 % of the rollout (tools/store_pattern.py ACT8 vs
// PACK8); this pass streams them once.
__device__ __forceinline__ uint32_t pack_id(int32_t v) { return (uint32_t)v < 12u ? (uint32_t)v : 15u; }

// VEC4: four consecutive envs per thread with 16-byte loads/stores (B % 4 == 0, aligned)
template <bool VEC4>
__global__ __launch_bounds__(256) void pack_actions_kernel(const int32_t* __restrict__ actions,
                                                           uint32_t* __restrict__ packed, int T, int64_t B) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int t0 = (int)blockIdx.y * 8;
    if constexpr (VEC4) {
        if (4 * i >= B) return;
        const int4* src = reinterpret_cast<const int4*>(actions) + i;
        const int64_t row4 = B / 4;
        int4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = t0 + k < T ? src[(int64_t)(t0 + k) * row4] : make_int4(0, 0, 0, 0);
        uint4 q = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (t0 + k >= T) continue;
            q.x |= pack_id(v[k].x) << (4 * k);
            q.y |= pack_id(v[k].y) << (4 * k);
            q.z |= pack_id(v[k].z) << (4 * k);
            q.w |= pack_id(v[k].w) << (4 * k);
        }
        reinterpret_cast<uint4*>(packed + (int64_t)blockIdx.y * B)[i] = q;
    } else {
        if (i >= B) return;
        int32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = t0 + k < T ? actions[(int64_t)(t0 + k) * B + i] : 0;
        uint32_t q = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) q |= (t0 + k < T ? pack_id(v[k]) : 0u) << (4 * k);
        packed[(int64_t)blockIdx.y * B + i] = q;
    }
}


constexpr int KEY_GROUP = 3;  // actions per staged key group in expand12 (12 % KEY_GROUP == 0)

// expand12's per-wave LDS: the tile, or the staged keys of one group, whichever is larger
template <int NW, int LC, int VEC>
struct ExpandLaunchSmem {
    static __host__ __device__ size_t wave_bytes(int L) {
        const size_t t = TileFor<NW, LC, VEC>::wave_bytes(L);
        const size_t k = (size_t)WAVE * KEY_GROUP * (size_t)((4 * L + 16 + 63) / 64) * 8;
        return ((t > k ? t : k) + 15) & ~(size_t)15;
    }
};

struct ExpandArgs {
    const int32_t* parents;
    int32_t* children;
    int32_t* child_len;
    uint64_t* child_key;
    uint8_t* err;
    int32_t* err_count;
    int64_t N;
    int L, cyclical, kw64;
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK, Occupancy<LC>::waves_per_simd) void expand12_kernel(ExpandArgs a) {
    using Tile = TileFor<NW, LC, VEC>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    WaveCtx w;
    if (!wave_ctx(a.N, w)) return;
    Tile tile(smem + w.wid * ExpandLaunchSmem<NW, LC, VEC>::wave_bytes(a.L), a.L);
    const int L = tile.Lr(), twoL = 2 * L;
    const int64_t par = w.r0 + w.lane;

    tile.load(a.parents + w.r0 * twoL, w.R, w.lane);
    PresRegs<NW> p;
    bool bad = false, clean = false;
    const bool cyc = a.cyclical != 0;
    if (w.active) {
        bad = tile.pack(w.lane, p);
        clean = !bad && is_clean<NW>(p.w0, p.n0, p.w1, p.n1, cyc);
    }
    tile.flag_rows(w.lane, bad ? FB_IN : 0u);  // children of out-of-domain parents copy the parent row
    int nerr = 0;
    // keys only (the search path): stage each group of KEY_GROUP actions' keys in LDS
    // (the parents' rows are no longer needed once packed) and write them out as
    // contiguous KEY_GROUP*kw64*8-byte segments instead of per-lane 8-byte pieces
    const bool stage_keys = a.child_key != nullptr && a.children == nullptr;
    uint64_t* kst = reinterpret_cast<uint64_t*>(smem + w.wid * ExpandLaunchSmem<NW, LC, VEC>::wave_bytes(a.L));
    for (int act = 0; act < 12; ++act) {
        if (w.active) {
            PresRegs<NW> q = p;
            int e;
            if (bad) e = ACX_ERR_DOMAIN;
            else if (clean) e = ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            else e = ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            const int64_t ci = par * 12 + act;
            nerr += e != ACX_ERR_NONE;
            if (a.err) a.err[ci] = (uint8_t)e;
            if (a.child_len) {
                a.child_len[2 * ci] = q.n0;
                a.child_len[2 * ci + 1] = q.n1;
            }
            if (a.child_key) {
                // an errored child's key is the sentinel with both length bytes 0xFF (acx.h)
                PresRegs<NW> kq = q;
                if (e != ACX_ERR_NONE) {
                    kq.n0 = 0xff;
                    kq.n1 = 0xff;
                }
                if (stage_keys) store_key<NW>(kst + (w.lane * KEY_GROUP + act % KEY_GROUP) * a.kw64, a.kw64, L, kq);
                else store_key<NW>(a.child_key + ci * a.kw64, a.kw64, L, kq);
            }
            if (a.children && !bad) tile.unpack(w.lane, q);
        }
        if (a.children) {
            wave_sync();
            tile.template store<true, NT_STATE>(a.children + (w.r0 * 12 + act) * twoL, (int64_t)12 * twoL, w.R,
                                      a.parents + w.r0 * twoL, twoL, w.lane);
            wave_sync();
        }
        if (stage_keys && act % KEY_GROUP == KEY_GROUP - 1) {
            wave_sync();
            const int kw = LC > 0 ? (4 * LC + 16 + 63) / 64 : a.kw64;
            const int seg = KEY_GROUP * kw;  // u64 words per parent in this group
            const int n = w.R * seg;
            uint64_t* gbase = a.child_key + (w.r0 * 12 + (act - (KEY_GROUP - 1))) * kw;
            for (int i = w.lane; i < n; i += WAVE) {
                const int pp = i / seg;
                gbase[(int64_t)pp * 12 * kw + (i - pp * seg)] = kst[i];
            }
            wave_sync();
        }
    }
    if (nerr && a.err_count) atomicAdd(a.err_count, nerr);
}

// expand12 without int32 children (the search path: packed child keys, optional lengths/err):
// one block of 4 waves per tile of 64 parents; wave 0 stages and packs the tile, every wave then
// makes the children of 3 actions (wave w: 3w..3w+2) -- 4x the lanes of a lane-per-parent loop
// over 12 moves, whose dependent VALU chain left most issue slots empty -- and the block's
// 12 * 64 keys are staged in LDS (parent-major, as in HBM) and written as one contiguous run.
constexpr int KEYS_APW = 12 / WPB;  // actions per wave (3)

template <int NW>
__host__ __device__ constexpr int packed_words() { return 2 * NW + 2; }

template <int NW, int LC, int VEC>
struct ExpandKeysSmem {
    static __host__ __device__ size_t region_a(int L) {
        const size_t t = TileFor<NW, LC, VEC>::wave_bytes(L);
        const size_t k = (size_t)WAVE * 12 * (size_t)((4 * L + 16 + 63) / 64) * 8;
        return ((t > k ? t : k) + 15) & ~(size_t)15;
    }
    static __host__ __device__ size_t bytes(int L) { return region_a(L) + (size_t)WAVE * packed_words<NW>() * 4; }
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void expand12_keys_kernel(ExpandArgs a) {
    using Tile = TileFor<NW, LC, VEC>;
    using Smem = ExpandKeysSmem<NW, LC, VEC>;
    constexpr int PW = packed_words<NW>();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int64_t r0 = (int64_t)blockIdx.x * WAVE;
    if (r0 >= a.N) return;  // block-uniform
    const int R = (int)((a.N - r0) < WAVE ? (a.N - r0) : WAVE);
    const int L = LC > 0 ? LC : a.L;
    const int kw = LC > 0 ? (4 * LC + 16 + 63) / 64 : a.kw64;
    char* region = smem;
    uint32_t* packed = reinterpret_cast<uint32_t*>(smem + Smem::region_a(a.L));
    const bool cyc = a.cyclical != 0;
    Tile tile(region, a.L);
    if constexpr (LC > 0 && LC % 4 == 0) tile.load_block(a.parents + r0 * 2 * L, R);
    else if (wid == 0) tile.load(a.parents + r0 * 2 * L, R, lane);
    if (wid == 0) {
        if (lane < R) {
            PresRegs<NW> p;
            const bool bad = tile.pack(lane, p);
            const bool clean = !bad && is_clean<NW>(p.w0, p.n0, p.w1, p.n1, cyc);
            uint32_t* d = packed + lane * PW;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                d[k] = p.w0.w[k];
                d[NW + k] = p.w1.w[k];
            }
            d[2 * NW] = (uint32_t)p.n0 | ((uint32_t)p.n1 << 8);
            d[2 * NW + 1] = (uint32_t)bad | ((uint32_t)clean << 1);
        }
    }
    __syncthreads();
    uint64_t* kst = reinterpret_cast<uint64_t*>(region);
    int nerr = 0;
    if (lane < R) {
        PresRegs<NW> p;
        const uint32_t* d = packed + lane * PW;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            p.w0.w[k] = d[k];
            p.w1.w[k] = d[NW + k];
        }
        p.n0 = (int)(d[2 * NW] & 0xffu);
        p.n1 = (int)((d[2 * NW] >> 8) & 0xffu);
        const bool bad = (d[2 * NW + 1] & 1u) != 0, clean = (d[2 * NW + 1] & 2u) != 0;
        const int64_t par = r0 + lane;
#pragma unroll 1
        for (int j = 0; j < KEYS_APW; ++j) {
            const int act = wid * KEYS_APW + j;
            PresRegs<NW> q = p;
            int e;
            if (bad) e = ACX_ERR_DOMAIN;
            else if (clean) e = ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            else e = ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            const int64_t ci = par * 12 + act;
            nerr += e != ACX_ERR_NONE;
            if (a.err) a.err[ci] = (uint8_t)e;
            if (a.child_len) {
                a.child_len[2 * ci] = q.n0;
                a.child_len[2 * ci + 1] = q.n1;
            }
            if (e != ACX_ERR_NONE) {  // the error sentinel: both length bytes 0xFF (acx.h)
                q.n0 = 0xff;
                q.n1 = 0xff;
            }
            uint64_t key[NW + 1];
            make_key<NW>(L, q, key);
#pragma unroll
            for (int k = 0; k < NW + 1; ++k)
                if (k < kw) kst[(lane * 12 + act) * kw + k] = key[k];
        }
    }
    __syncthreads();
    uint64_t* dst = a.child_key + r0 * 12 * kw;
    if constexpr (NT_KEYS) {
        // 16-B non-temporal stores (dst is 16-B aligned: r0 is a multiple of 64), odd tail word apart
        const int nw = R * 12 * kw;
        for (int i = threadIdx.x; 2 * i + 1 < nw; i += BLOCK) {
            typedef unsigned long long v2u_t __attribute__((ext_vector_type(2)));
            const v2u_t x = {kst[2 * i], kst[2 * i + 1]};
            __builtin_nontemporal_store(x, reinterpret_cast<v2u_t*>(dst) + i);
        }
        if ((nw & 1) && threadIdx.x == 0) dst[nw - 1] = kst[nw - 1];
    } else {
        for (int i = threadIdx.x; i < R * 12 * kw; i += BLOCK) dst[i] = kst[i];
    }
    if (nerr && a.err_count) atomicAdd(a.err_count, nerr);
}

// expand12 with int32 children (acx_expand12 children != NULL): one block of 4 waves per tile
// of 64 parents, as expand12_keys_kernel -- every wave stages and packs the parents, wave w
// makes the children of actions 3w..3w+2, one action at a time: unpack into its own LDS tile,
// then a tile store with row pitch 12 * 2L (child (p, a) is row 12p + a).  The block's 64 x 12
// child rows are one contiguous 221 KB region at L = 36, written as 3-row runs per parent and
// wave (the lane-per-parent loop it replaces made 12 serial moves per lane and wrote each child
// row as its own 288-byte run).  Lengths and error codes go through LDS and out as one
// contiguous run per block.  Out-of-domain parents' children are copies of the parent row (the
// fallback rows of the tile store), as in expand12_kernel.
template <int NW, int LC, int VEC>
struct ExpandChildrenSmem {
    static __host__ __device__ size_t tile_bytes(int L) {
        return (TileFor<NW, LC, VEC>::wave_bytes(L) + 15) & ~(size_t)15;
    }
    static __host__ __device__ size_t lens_off(int L) { return WPB * tile_bytes(L); }
    static __host__ __device__ size_t err_off(int L) { return lens_off(L) + (size_t)WAVE * 12 * 2 * 4; }
    static __host__ __device__ size_t bytes(int L) { return err_off(L) + (size_t)WAVE * 12; }
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void expand12_children_kernel(ExpandArgs a) {
    using Tile = TileFor<NW, LC, VEC>;
    using Smem = ExpandChildrenSmem<NW, LC, VEC>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int64_t r0 = (int64_t)blockIdx.x * WAVE;
    if (r0 >= a.N) return;  // block-uniform
    const int R = (int)((a.N - r0) < WAVE ? (a.N - r0) : WAVE);
    const bool active = lane < R;
    Tile tile(smem + wid * Smem::tile_bytes(a.L), a.L);
    const int L = tile.Lr(), twoL = 2 * L;
    int32_t* lens_st = reinterpret_cast<int32_t*>(smem + Smem::lens_off(a.L));
    uint8_t* err_st = reinterpret_cast<uint8_t*>(smem + Smem::err_off(a.L));
    const bool cyc = a.cyclical != 0;
    // every wave stages and packs the parent tile itself (the block's other three reads of the
    // 18 KB tile are L2 hits): no block-wide wait on one wave's load before the moves start;
    // the tile's flags mark the out-of-domain rows, whose children copy the parent row
    tile.load(a.parents + r0 * twoL, R, lane);
    PresRegs<NW> p;
    bool bad = false, clean = false;
    if (active) {
        bad = tile.pack(lane, p);
        clean = !bad && is_clean<NW>(p.w0, p.n0, p.w1, p.n1, cyc);
    }
    tile.flag_rows(lane, bad ? FB_IN : 0u);  // incl. a zero inside a relator (not flagged by the load)

    int nerr = 0;
    const int64_t par = r0 + lane;
#pragma unroll 1
    for (int j = 0; j < KEYS_APW; ++j) {
        const int act = wid * KEYS_APW + j;
        if (active) {
            PresRegs<NW> q = p;
            int e;
            if (bad) e = ACX_ERR_DOMAIN;
            else if (clean) e = ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            else e = ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            nerr += e != ACX_ERR_NONE;
            err_st[lane * 12 + act] = (uint8_t)e;
            lens_st[(lane * 12 + act) * 2] = q.n0;
            lens_st[(lane * 12 + act) * 2 + 1] = q.n1;
            if (a.child_key) {  // keys as well (not the search path): per lane, unstaged
                PresRegs<NW> kq = q;
                if (e != ACX_ERR_NONE) {
                    kq.n0 = 0xff;
                    kq.n1 = 0xff;
                }
                store_key<NW>(a.child_key + (par * 12 + act) * a.kw64, a.kw64, L, kq);
            }
            if (!bad) tile.unpack(lane, q);
        }
        wave_sync();
        tile.template store<true, NT_STATE>(a.children + (r0 * 12 + act) * twoL, (int64_t)12 * twoL, R,
                                  a.parents + r0 * twoL, twoL, lane);
        wave_sync();
    }
    __syncthreads();
    if (a.child_len) {
        int32_t* dst = a.child_len + r0 * 24;
        for (int i = threadIdx.x; i < R * 24; i += BLOCK) dst[i] = lens_st[i];
    }
    if (a.err) {
        uint8_t* dst = a.err + r0 * 12;
        for (int i = threadIdx.x; i < R * 12; i += BLOCK) dst[i] = err_st[i];
    }
    if (nerr && a.err_count) atomicAdd(a.err_count, nerr);
}

// expand12 with int32 children for compile-time L % 4 == 0 (L = 36 and 128): the block makes its
// 64 x 12 children exactly as expand12_keys_kernel (wave 0 packs the parents, wave w the actions
// 3w..3w+2), stages each child in LDS as packed words (both relators' 2-bit codes and the two
// lengths: 2 NW + 1 dwords), then all 256 threads expand the staged children into the block's
// contiguous 64 x 12 x 2L int32 region with 16-byte stores, consecutive threads on consecutive
// chunks -- the whole 221 KB (L = 36) as one linear stream per block.  Out-of-domain parents'
// children are copies of the parent row; lengths come from the staged words, error codes from LDS.
template <int NW, int LC, int VEC>
struct ExpandRowsSmem {
    static constexpr int SW = 2 * NW + 1;  // staged dwords per child
    static __host__ __device__ size_t region_a(int L) {
        const size_t t = TileFor<NW, LC, VEC>::wave_bytes(L);
        const size_t k = (size_t)WAVE * 12 * SW * 4;
        return ((t > k ? t : k) + 15) & ~(size_t)15;
    }
    static __host__ __device__ size_t err_off(int L) { return region_a(L) + (size_t)WAVE * packed_words<NW>() * 4; }
    static __host__ __device__ size_t bytes(int L) { return err_off(L) + (size_t)WAVE * 12; }
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void expand12_rows_kernel(ExpandArgs a) {
    static_assert(LC > 0 && LC % 4 == 0, "compile-time L, whole 16-byte chunks per relator");
    using Tile = TileFor<NW, LC, VEC>;
    using Smem = ExpandRowsSmem<NW, LC, VEC>;
    constexpr int PW = packed_words<NW>();
    constexpr int SW = Smem::SW;
    constexpr int L = LC, CPR = LC / 2, HC = LC / 4;  // 16-byte chunks per row / per relator
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int64_t r0 = (int64_t)blockIdx.x * WAVE;
    if (r0 >= a.N) return;  // block-uniform
    const int R = (int)((a.N - r0) < WAVE ? (a.N - r0) : WAVE);
    uint32_t* packed = reinterpret_cast<uint32_t*>(smem + Smem::region_a(a.L));
    uint8_t* err_st = reinterpret_cast<uint8_t*>(smem + Smem::err_off(a.L));
    const bool cyc = a.cyclical != 0;
    Tile tile(smem, a.L);
    tile.load_block(a.parents + r0 * 2 * L, R);
    if (wid == 0) {
        if (lane < R) {
            PresRegs<NW> p;
            const bool bad = tile.pack(lane, p);
            const bool clean = !bad && is_clean<NW>(p.w0, p.n0, p.w1, p.n1, cyc);
            uint32_t* d = packed + lane * PW;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                d[k] = p.w0.w[k];
                d[NW + k] = p.w1.w[k];
            }
            d[2 * NW] = (uint32_t)p.n0 | ((uint32_t)p.n1 << 8);
            d[2 * NW + 1] = (uint32_t)bad | ((uint32_t)clean << 1);
        }
    }
    __syncthreads();  // the tile is dead from here: region a holds the staged children
    uint32_t* stw = reinterpret_cast<uint32_t*>(smem);
    int nerr = 0;
    if (lane < R) {
        PresRegs<NW> p;
        const uint32_t* d = packed + lane * PW;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            p.w0.w[k] = d[k];
            p.w1.w[k] = d[NW + k];
        }
        p.n0 = (int)(d[2 * NW] & 0xffu);
        p.n1 = (int)((d[2 * NW] >> 8) & 0xffu);
        const bool bad = (d[2 * NW + 1] & 1u) != 0, clean = (d[2 * NW + 1] & 2u) != 0;
        const int64_t par = r0 + lane;
#pragma unroll 1
        for (int j = 0; j < KEYS_APW; ++j) {
            const int act = wid * KEYS_APW + j;
            PresRegs<NW> q = p;
            int e;
            if (bad) e = ACX_ERR_DOMAIN;
            else if (clean) e = ac_move_clean<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            else e = ac_move<NW>(q.w0, q.n0, q.w1, q.n1, act, L, cyc);
            nerr += e != ACX_ERR_NONE;
            err_st[lane * 12 + act] = (uint8_t)e;
            if (a.child_key) {  // keys as well (not the search path): per lane, unstaged
                PresRegs<NW> kq = q;
                if (e != ACX_ERR_NONE) {
                    kq.n0 = 0xff;
                    kq.n1 = 0xff;
                }
                store_key<NW>(a.child_key + (par * 12 + act) * a.kw64, a.kw64, L, kq);
            }
            uint32_t* c = stw + (lane * 12 + act) * SW;  // odd stride: conflict-free
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                c[k] = q.w0.w[k];
                c[NW + k] = q.w1.w[k];
            }
            c[2 * NW] = (uint32_t)q.n0 | ((uint32_t)q.n1 << 8);
        }
    }
    __syncthreads();
    int4* dst = reinterpret_cast<int4*>(a.children + r0 * 12 * 2 * L);
    const int nch = R * 12 * CPR;
    for (int i = threadIdx.x; i < nch; i += BLOCK) {
        const int ci = i / CPR, k = i - ci * CPR;  // child (parent-major), 16-byte chunk of its row
        const int pp = ci / 12;
        int4 v;
        if (packed[pp * PW + 2 * NW + 1] & 1u) {  // out-of-domain parent: its row, as is
            v = reinterpret_cast<const int4*>(a.parents + (r0 + pp) * 2 * L)[k];
        } else {
            const uint32_t* c = stw + ci * SW;
            const int h = k >= HC ? 1 : 0, m = k - h * HC;
            const uint32_t c8 = (c[h * NW + (m >> 2)] >> (8 * (m & 3))) & 0xffu;
            const int n = (int)((c[2 * NW] >> (8 * h)) & 0xffu);
            v = widen4(codes_to_i8x4(c8, clamp_bits(8 * n - 32 * m)));
        }
        dst[i] = v;
    }
    if (a.child_len) {
        int32_t* ld = a.child_len + r0 * 24;
        for (int i = threadIdx.x; i < R * 24; i += BLOCK) ld[i] = (int32_t)((stw[(i >> 1) * SW + 2 * NW] >> (8 * (i & 1))) & 0xffu);
    }
    if (a.err) {
        uint8_t* ed = a.err + r0 * 12;
        for (int i = threadIdx.x; i < R * 12; i += BLOCK) ed[i] = err_st[i];
    }
    if (nerr && a.err_count) atomicAdd(a.err_count, nerr);
}

struct CanonArgs {
    const int32_t* state_in;
    int32_t* state_out;
    int32_t* lengths_out;
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int L, cyclical;
};

// simplify_presentation (utils.py:246-283): assert valid, then reduce both relators
template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void canon_kernel(CanonArgs a) {
    using Tile = TileFor<NW, LC, VEC>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    WaveCtx w;
    if (!wave_ctx(a.B, w)) return;
    Tile tile(smem + w.wid * Tile::wave_bytes(a.L), a.L);
    const int L = tile.Lr(), twoL = 2 * L;
    const int64_t env = w.r0 + w.lane;
    tile.load(a.state_in + w.r0 * twoL, w.R, w.lane);
    bool bad = false;
    if (w.active) {
        PresRegs<NW> p;
        bad = tile.pack(w.lane, p);
        const int e = bad ? ACX_ERR_DOMAIN : ((p.n0 == 0 || p.n1 == 0) ? ACX_ERR_INVALID : ACX_ERR_NONE);
        if (e == ACX_ERR_NONE) {
            simplify<NW>(p.w0, p.n0, a.cyclical != 0);
            simplify<NW>(p.w1, p.n1, a.cyclical != 0);
            tile.unpack(w.lane, p);
        }
        if (a.lengths_out) {
            a.lengths_out[2 * env] = p.n0;
            a.lengths_out[2 * env + 1] = p.n1;
        }
        if (a.err) a.err[env] = (uint8_t)e;
        if (e != ACX_ERR_NONE && a.err_count) atomicAdd(a.err_count, 1);
    }
    tile.flag_rows(w.lane, bad ? FB_IN : 0u);  // incl. a zero inside a relator (not flagged by the load)
    wave_sync();
    tile.template store<true, NT_STATE>(a.state_out + w.r0 * twoL, twoL, w.R, a.state_in + w.r0 * twoL, twoL,
                                                 w.lane);
}

struct UnpackArgs {
    const uint64_t* keys;
    int32_t* states;
    int32_t* lengths_out;
    int64_t M;
    int L, kw64;
};

template <int NW, int LC, int VEC>
__global__ __launch_bounds__(BLOCK) void unpack_keys_kernel(UnpackArgs a) {
    using Tile = TileFor<NW, LC, VEC>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    WaveCtx w;
    if (!wave_ctx(a.M, w)) return;
    Tile tile(smem + w.wid * Tile::wave_bytes(a.L), a.L);
    const int L = tile.Lr(), twoL = 2 * L;
    const int64_t k = w.r0 + w.lane;
    if (w.active) {
        PresRegs<NW> p;
        load_key<NW>(a.keys + k * a.kw64, a.kw64, L, p);
        tile.unpack(w.lane, p);
        if (a.lengths_out) {
            a.lengths_out[2 * k] = p.n0;
            a.lengths_out[2 * k + 1] = p.n1;
        }
    }
    wave_sync();
    tile.template store<false>(a.states + w.r0 * twoL, twoL, w.R, nullptr, 0, w.lane);
}

// ---------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------
static inline int nw_for(int L) {
    return L <= 16 ? 1 : L <= 32 ? 2 : L <= 48 ? 3 : L <= 64 ? 4 : 8;
}

template <int NW, int LC, int VEC>
static inline size_t smem_bytes(int L) {
    return (size_t)WPB * TileFor<NW, LC, VEC>::wave_bytes(L);
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// call `f.template go<NW, LC, VEC>()` for the instantiation matching L
template <class F>
static int dispatch(int L, F&& f) {
    const bool v4 = (2 * L) % 4 == 0;
#if defined(ACX_ISA_L128_ONLY)  // faster builds for ISA inspection only
    (void)v4;
    return L == 128 ? f.template go<8, 128, 4>() : ACX_E_ARG;
#elif defined(ACX_ISA_L36_ONLY)  // faster builds for ISA inspection only
    (void)v4;
    return L == 36 ? f.template go<3, 36, 4>() : ACX_E_ARG;
#else
    if (L == 36) return f.template go<3, 36, 4>();
    if (L == 128) return f.template go<8, 128, 4>();
    switch (nw_for(L)) {
        case 1: return v4 ? f.template go<1, 0, 4>() : f.template go<1, 0, 2>();
        case 2: return v4 ? f.template go<2, 0, 4>() : f.template go<2, 0, 2>();
        case 3: return v4 ? f.template go<3, 0, 4>() : f.template go<3, 0, 2>();
        case 4: return v4 ? f.template go<4, 0, 4>() : f.template go<4, 0, 2>();
        default: return v4 ? f.template go<8, 0, 4>() : f.template go<8, 0, 2>();
    }
#endif
}

static inline int finish_launch() {
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

static inline unsigned grid_for(int64_t rows) {
    return (unsigned)((rows + (int64_t)BLOCK - 1) / BLOCK);
}

// One launcher per kernel family and instantiation.  They are plain (non-static) function
// templates so that the slow-to-compile L = 128 instantiations can be explicitly instantiated in
// separate objects built from this same file (-DACX_PART=n, compiled in parallel by build.py)
// while the main object declares them `extern template` below.
template <int NW, int LC, int VEC, bool LEARN>
int launch_step(StepArgs a, hipStream_t s) {
    const size_t shm = smem_bytes<NW, LC, VEC>(a.L);
    if (!LEARN && a.live) {
        step_lengths_kernel<NW, LC, VEC><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
        return finish_launch();
    }
    if constexpr (!LEARN && small_step_ok<NW, LC, VEC>()) {
        if (a.B <= SMALL_STEP_MAX_B) {
            constexpr int per_block = WPB * PairLayout<LC>::ENVS;
            step_pair_kernel<NW, LC, VEC><<<dim3((unsigned)((a.B + per_block - 1) / per_block)), dim3(BLOCK),
                                            WPB * PairLayout<LC>::wave_bytes, s>>>(a);
            return finish_launch();
        }
    }
    step_kernel<NW, LC, VEC, LEARN><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
    return finish_launch();
}
template <int NW, int LC, int VEC, int OBS>
int launch_rollout(RolloutArgs a, hipStream_t s) {
    const size_t shm = smem_bytes<NW, LC, VEC>(a.L);
    rollout_kernel<NW, LC, VEC, OBS><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
    return finish_launch();
}
template <int NW, int LC, int VEC>
int launch_expand(ExpandArgs a, hipStream_t s) {
    if constexpr (LC > 0 && LC % 4 == 0) {
        const size_t rshm = ExpandRowsSmem<NW, LC, VEC>::bytes(a.L);
        if (a.children && rshm <= 64 * 1024) {
            expand12_rows_kernel<NW, LC, VEC><<<dim3((unsigned)((a.N + WAVE - 1) / WAVE)), dim3(BLOCK), rshm, s>>>(a);
            return finish_launch();
        }
    }
    const size_t cshm = ExpandChildrenSmem<NW, LC, VEC>::bytes(a.L);
    if (a.children && cshm <= 64 * 1024) {
        expand12_children_kernel<NW, LC, VEC><<<dim3((unsigned)((a.N + WAVE - 1) / WAVE)), dim3(BLOCK), cshm, s>>>(a);
        return finish_launch();
    }
    const size_t kshm = ExpandKeysSmem<NW, LC, VEC>::bytes(a.L);
    if (!a.children && a.child_key && kshm <= 40 * 1024) {  // the search path
        expand12_keys_kernel<NW, LC, VEC><<<dim3((unsigned)((a.N + WAVE - 1) / WAVE)), dim3(BLOCK), kshm, s>>>(a);
        return finish_launch();
    }
    const size_t shm = (size_t)WPB * ExpandLaunchSmem<NW, LC, VEC>::wave_bytes(a.L);
    expand12_kernel<NW, LC, VEC><<<dim3(grid_for(a.N)), dim3(BLOCK), shm, s>>>(a);
    return finish_launch();
}
template <int NW, int LC, int VEC>
int launch_canon(CanonArgs a, hipStream_t s) {
    const size_t shm = smem_bytes<NW, LC, VEC>(a.L);
    canon_kernel<NW, LC, VEC><<<dim3(grid_for(a.B)), dim3(BLOCK), shm, s>>>(a);
    return finish_launch();
}
template <int NW, int LC, int VEC>
int launch_unpack(UnpackArgs a, hipStream_t s) {
    const size_t shm = smem_bytes<NW, LC, VEC>(a.L);
    unpack_keys_kernel<NW, LC, VEC><<<dim3(grid_for(a.M)), dim3(BLOCK), shm, s>>>(a);
    return finish_launch();
}

// Each kernel instantiation set compiles in an object of its own, built from this same file with
// -DACX_PART=n (build.py compiles them in parallel with the main object, which holds L = 36):
// the runtime-L generic sets (fully unrolled per-letter loops up to 16*NW letters) took ~7 of the
// ~7.5 minutes of one object.  The main object declares them `extern template`.
#define ACX_INST_STEP(EXT, NW, LC, VEC)                                   \
    EXT template int launch_step<NW, LC, VEC, false>(StepArgs, hipStream_t); \
    EXT template int launch_step<NW, LC, VEC, true>(StepArgs, hipStream_t);
#define ACX_INST_ROLL(EXT, NW, LC, VEC, OBS) EXT template int launch_rollout<NW, LC, VEC, OBS>(RolloutArgs, hipStream_t);
#define ACX_INST_SEARCH(EXT, NW, LC, VEC)                                 \
    EXT template int launch_expand<NW, LC, VEC>(ExpandArgs, hipStream_t);  \
    EXT template int launch_canon<NW, LC, VEC>(CanonArgs, hipStream_t);    \
    EXT template int launch_unpack<NW, LC, VEC>(UnpackArgs, hipStream_t);
#define ACX_INST_ALL(EXT, NW, LC, VEC) \
    ACX_INST_STEP(EXT, NW, LC, VEC)    \
    ACX_INST_ROLL(EXT, NW, LC, VEC, 0) \
    ACX_INST_ROLL(EXT, NW, LC, VEC, 1) \
    ACX_INST_ROLL(EXT, NW, LC, VEC, 2) \
    ACX_INST_SEARCH(EXT, NW, LC, VEC)
// part n: 1-3 the L = 128 rollout (int32 obs / int8 obs / none), 4 the L = 128 step, 5 the L = 128
// expand / canonicalize / unpack, 6-10 the generic (runtime-L) sets; build.py's KERNEL_PARTS = 10
#if !defined(ACX_PART)
#if !defined(ACX_ISA_L36_ONLY) && !defined(ACX_ISA_L128_ONLY)
ACX_INST_ROLL(extern, 8, 128, 4, 1)
ACX_INST_ROLL(extern, 8, 128, 4, 2)
ACX_INST_ROLL(extern, 8, 128, 4, 0)
ACX_INST_STEP(extern, 8, 128, 4)
ACX_INST_SEARCH(extern, 8, 128, 4)
ACX_INST_ALL(extern, 8, 0, 4)
ACX_INST_ALL(extern, 8, 0, 2)
ACX_INST_ALL(extern, 4, 0, 4)
ACX_INST_ALL(extern, 4, 0, 2)
ACX_INST_ALL(extern, 3, 0, 4)
ACX_INST_ALL(extern, 3, 0, 2)
ACX_INST_ALL(extern, 2, 0, 4)
ACX_INST_ALL(extern, 2, 0, 2)
ACX_INST_ALL(extern, 1, 0, 4)
ACX_INST_ALL(extern, 1, 0, 2)
#endif
#elif ACX_PART == 1
ACX_INST_ROLL(, 8, 128, 4, 1)
#elif ACX_PART == 2
ACX_INST_ROLL(, 8, 128, 4, 2)
#elif ACX_PART == 3
ACX_INST_ROLL(, 8, 128, 4, 0)
#elif ACX_PART == 4
ACX_INST_STEP(, 8, 128, 4)
#elif ACX_PART == 5
ACX_INST_SEARCH(, 8, 128, 4)
#elif ACX_PART == 6
ACX_INST_ALL(, 8, 0, 4)
#elif ACX_PART == 7
ACX_INST_ALL(, 8, 0, 2)
#elif ACX_PART == 8
ACX_INST_ALL(, 4, 0, 4)
ACX_INST_ALL(, 4, 0, 2)
#elif ACX_PART == 9
ACX_INST_ALL(, 3, 0, 4)
ACX_INST_ALL(, 3, 0, 2)
#elif ACX_PART == 10
ACX_INST_ALL(, 2, 0, 4)
ACX_INST_ALL(, 2, 0, 2)
ACX_INST_ALL(, 1, 0, 4)
ACX_INST_ALL(, 1, 0, 2)
#endif

struct StepLaunch {
    StepArgs a;
    hipStream_t s;
    bool learn;
    template <int NW, int LC, int VEC>
    int go() {
        a.in_place = a.state_in == a.state_out;
        return learn ? launch_step<NW, LC, VEC, true>(a, s) : launch_step<NW, LC, VEC, false>(a, s);
    }
};
struct RolloutLaunch {
    RolloutArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() {
        if (a.obs_traj8) return launch_rollout<NW, LC, VEC, 2>(a, s);
        if (a.obs_traj) return launch_rollout<NW, LC, VEC, 1>(a, s);
        return launch_rollout<NW, LC, VEC, 0>(a, s);
    }
};
struct ExpandLaunch {
    ExpandArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() { return launch_expand<NW, LC, VEC>(a, s); }
};
struct CanonLaunch {
    CanonArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() { return launch_canon<NW, LC, VEC>(a, s); }
};
struct UnpackLaunch {
    UnpackArgs a;
    hipStream_t s;
    template <int NW, int LC, int VEC>
    int go() { return launch_unpack<NW, LC, VEC>(a, s); }
};

}  // namespace acx

#ifndef ACX_PART  // the C-ABI lives in the main object only
using namespace acx;

extern "C" {

int32_t acx_key_words(int32_t L) { return (4 * L + 16 + 63) / 64; }

// build provenance: build.py passes the sha256 of the sources this library is compiled from
#ifndef ACX_SOURCE_HASH
#define ACX_SOURCE_HASH "unknown"
#endif
const char* acx_version(void) { return "acx 0.3 gfx950 acx-src-sha256:" ACX_SOURCE_HASH; }

int acx_step(const int32_t* state_in, int32_t* state_out, const int32_t* action, const int32_t* reset_state,
             int32_t* step_count, int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths_out,
             int32_t* final_obs, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
             int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state_in || !state_out || !action) return ACX_E_ARG;
    if (!aligned16(state_in) || !aligned16(state_out)) return ACX_E_ARG;
    if (reset_state && !step_count) return ACX_E_ARG;
    StepArgs a{state_in, state_out, action, reset_state, step_count, reward, done, truncated,
               lengths_out, final_obs, err, err_count, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
               B, L, horizon, cyclical, 0};
    StepLaunch f{a, (hipStream_t)stream, false};
    return dispatch(L, f);
}

int acx_step_lengths(int32_t* state, const int32_t* action, const int32_t* reset_state, int32_t* step_count,
                     int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths, int32_t* final_obs,
                     uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon, int32_t cyclical,
                     void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state || !action || !lengths) return ACX_E_ARG;
    if (!aligned16(state)) return ACX_E_ARG;
    if (reset_state && !step_count) return ACX_E_ARG;
    StepArgs a{state, state, action, reset_state, step_count, reward, done, truncated, lengths, final_obs, err,
               err_count, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, B, L, horizon, cyclical, 0};
    a.live = 1;
    StepLaunch f{a, (hipStream_t)stream, false};
    return dispatch(L, f);
}

int acx_step_lengths_reduced(int32_t* state, const int32_t* action, const int32_t* reset_state, int32_t* step_count,
                             int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths, uint8_t* reduced,
                             int32_t* final_obs, uint8_t* err, int32_t* err_count, int64_t B, int32_t L,
                             int32_t horizon, int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state || !action || !lengths || !reduced) return ACX_E_ARG;
    if (!aligned16(state)) return ACX_E_ARG;
    if (reset_state && !step_count) return ACX_E_ARG;
    StepArgs a{state, state, action, reset_state, step_count, reward, done, truncated, lengths, final_obs, err,
               err_count, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, B, L, horizon, cyclical, 0};
    a.live = 1;
    a.reduced = reduced;
    StepLaunch f{a, (hipStream_t)stream, false};
    return dispatch(L, f);
}

// a per-call step with everything but the move ids resolved once (acx.h): the launch is then a
// three-argument call -- at 65,536 envs a caller's ctypes call with 17 arguments took as long as
// half the kernel, and the host, not the GPU, set the eager rate
struct acx_step_plan {
    int32_t kind;
    const int32_t* state_in;
    int32_t* state_out;
    const int32_t* reset_state;
    int32_t* step_count;
    int32_t* reward;
    uint8_t* done;
    uint8_t* truncated;
    int32_t* lengths;
    uint8_t* reduced;
    int32_t* final_obs;
    uint8_t* err;
    int32_t* err_count;
    int64_t B;
    int32_t L, horizon, cyclical;
};

acx_step_plan* acx_step_plan_create(int32_t kind, const int32_t* state_in, int32_t* state_out,
                                    const int32_t* reset_state, int32_t* step_count, int32_t* reward, uint8_t* done,
                                    uint8_t* truncated, int32_t* lengths, uint8_t* reduced, int32_t* final_obs,
                                    uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
                                    int32_t cyclical) {
    // the checks of the entry the plan calls (acx_step / acx_step_lengths / _reduced), made once
    if (kind < ACX_STEP_PLAN_STEP || kind > ACX_STEP_PLAN_LENGTHS_REDUCED) return nullptr;
    if (B < 0 || L < 1 || L > ACX_MAX_L) return nullptr;
    if (B > 0) {
        if (!state_in || !state_out || !aligned16(state_in) || !aligned16(state_out)) return nullptr;
        if (reset_state && !step_count) return nullptr;
        if (kind != ACX_STEP_PLAN_STEP && (state_out != state_in || !lengths)) return nullptr;
        if (kind == ACX_STEP_PLAN_LENGTHS_REDUCED && !reduced) return nullptr;
    }
    if (kind != ACX_STEP_PLAN_LENGTHS_REDUCED && reduced) return nullptr;
    return new (std::nothrow) acx_step_plan{kind, state_in, state_out, reset_state, step_count, reward, done, truncated,
                                            lengths, reduced, final_obs, err, err_count, B, L, horizon, cyclical};
}

int acx_step_plan_launch(const acx_step_plan* p, const int32_t* action, void* stream) {
    if (!p) return ACX_E_ARG;
    switch (p->kind) {
    case ACX_STEP_PLAN_STEP:
        return acx_step(p->state_in, p->state_out, action, p->reset_state, p->step_count, p->reward, p->done,
                        p->truncated, p->lengths, p->final_obs, p->err, p->err_count, p->B, p->L, p->horizon,
                        p->cyclical, stream);
    case ACX_STEP_PLAN_LENGTHS:
        return acx_step_lengths(p->state_out, action, p->reset_state, p->step_count, p->reward, p->done, p->truncated,
                                p->lengths, p->final_obs, p->err, p->err_count, p->B, p->L, p->horizon, p->cyclical,
                                stream);
    default:
        return acx_step_lengths_reduced(p->state_out, action, p->reset_state, p->step_count, p->reward, p->done,
                                        p->truncated, p->lengths, p->reduced, p->final_obs, p->err, p->err_count,
                                        p->B, p->L, p->horizon, p->cyclical, stream);
    }
}

void acx_step_plan_destroy(acx_step_plan* p) { delete p; }

int acx_step_next(const int32_t* state_in, int32_t* state_out, const int32_t* action, const int32_t* reset_state,
                  int32_t* step_count, int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths_out,
                  uint8_t* pending, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                  int32_t* episode_len, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
                  int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L || hist_cap < 0 || hist_t < 0 || (hist_base && !action_hist)) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state_in || !state_out || !action || !reset_state || !step_count || !pending) return ACX_E_ARG;
    if ((action_hist != nullptr) != (hist_cap > 0) || (episode_len && !action_hist)) return ACX_E_ARG;
    if (!aligned16(state_in) || !aligned16(state_out)) return ACX_E_ARG;
    StepArgs a{state_in, state_out, action, reset_state, step_count, reward, done, truncated, lengths_out, nullptr,
               err, err_count, nullptr, nullptr, nullptr, nullptr, action_hist, episode_len, B, L, horizon, cyclical,
               hist_cap};
    a.pending = pending;
    a.hist_base = hist_base;
    a.hist_t = hist_t;
    // with a move history: the learner instantiation (it compiles the history writes)
    StepLaunch f{a, (hipStream_t)stream, action_hist != nullptr};
    return dispatch(L, f);
}

int acx_step_learner(int32_t* state, const int32_t* action, const int64_t* action_i64, const int32_t* reset_state,
                     int32_t* step_count, float* obs_f32, float* reward_f32, float* done_f32, uint8_t* done,
                     uint8_t* truncated, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                     int32_t* episode_len, int32_t* final_obs, uint8_t* err, int32_t* err_count, int64_t B, int32_t L,
                     int32_t horizon, int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L || hist_cap < 0 || hist_t < 0 || (hist_base && !action_hist)) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state || !step_count || (!action == !action_i64) || (action_hist && hist_cap == 0)) return ACX_E_ARG;
    if (!aligned16(state) || (obs_f32 && !aligned16(obs_f32))) return ACX_E_ARG;
    StepArgs a{state, state, action, reset_state, step_count, nullptr, done, truncated, nullptr, final_obs, err,
               err_count, action_i64, obs_f32, reward_f32, done_f32, action_hist, episode_len, B, L, horizon,
               cyclical, hist_cap};
    a.hist_base = hist_base;
    a.hist_t = hist_t;
    StepLaunch f{a, (hipStream_t)stream, true};
    return dispatch(L, f);
}

int acx_step_record(const int32_t* state_in, int32_t* state_out, const int32_t* action, const int32_t* reset_state,
                    int32_t* step_count, int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths_out,
                    int32_t* final_obs, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                    int32_t* episode_len, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
                    int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L || hist_cap < 0 || hist_t < 0) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state_in || !state_out || !action || !step_count || !action_hist || hist_cap == 0) return ACX_E_ARG;
    if (!aligned16(state_in) || !aligned16(state_out)) return ACX_E_ARG;
    // the learner instantiation (it compiles the history writes) with the plain step's outputs
    StepArgs a{state_in, state_out, action, reset_state, step_count, reward, done, truncated, lengths_out, final_obs,
               err, err_count, nullptr, nullptr, nullptr, nullptr, action_hist, episode_len, B, L, horizon, cyclical,
               hist_cap};
    a.hist_base = hist_base;
    a.hist_t = hist_t;
    StepLaunch f{a, (hipStream_t)stream, true};
    return dispatch(L, f);
}

// acx_curriculum.hip: where acx_learner_step's part of the shared workspace starts (int32 words)
int64_t acx_internal_curriculum_fused_offset(int64_t B);

int64_t acx_learner_failure_word(int64_t B) { return acx_internal_curriculum_fused_offset(B) + 4; }  // cur_ws[2]

static int g_learner_fail = 0;  // tests only
// tests only: acx_learner_step's ranking polls give up at once: 1 every one, 2 only the last tile's
// total (next_index), 0 none
void acx_internal_learner_ranking_fails(int32_t on) { g_learner_fail = on; }

int acx_learner_step(int32_t* state, const int32_t* action, const int64_t* action_i64, int32_t* reset_state,
                     int32_t* step_count, float* obs_f32, float* reward_f32, float* done_f32, uint8_t* done,
                     uint8_t* truncated, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                     int32_t* episode_len, uint8_t* err, int32_t* err_count, const int32_t* curriculum_states,
                     int64_t n_states, int32_t* next_index, int32_t* curr_index, uint8_t* needs_host,
                     int32_t* workspace, int64_t B, int32_t L, int32_t horizon, int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L || hist_cap < 0 || n_states < 0 || n_states > INT32_MAX) return ACX_E_ARG;
    if (hist_t < 0 || (hist_base && !action_hist)) return ACX_E_ARG;
    if (B >= (1ll << 31)) return ACX_E_ARG;  // the look-back's 32-bit prefixes (next_index + finished envs)
    if (B == 0) return ACX_OK;
    if (!state || !step_count || (!action == !action_i64) || (action_hist && hist_cap == 0)) return ACX_E_ARG;
    if (!done || !truncated || !reset_state || !curriculum_states || !next_index || !curr_index || !needs_host ||
        !workspace)
        return ACX_E_ARG;
    if (!aligned16(state) || (obs_f32 && !aligned16(obs_f32))) return ACX_E_ARG;
    if ((L % 2) == 0 && (!aligned16(reset_state) || !aligned16(curriculum_states))) return ACX_E_ARG;  // int4 row copies
    // one launch: the step kernel ranks the finished envs itself (cur_publish / cur_prefix) in its part of the
    // workspace (acx_curriculum_workspace(B) int32 words, zeroed before the first call, 8-byte aligned)
    int32_t* ws = workspace + acx_internal_curriculum_fused_offset(B);
    if ((reinterpret_cast<uintptr_t>(ws) & 7u) != 0) return ACX_E_ARG;
    StepArgs a{state, state, action, reset_state, step_count, nullptr, done, truncated, nullptr, nullptr, err,
               err_count, action_i64, obs_f32, reward_f32, done_f32, action_hist, episode_len, B, L, horizon,
               cyclical, hist_cap, reinterpret_cast<uint64_t*>(ws), curriculum_states, n_states, next_index,
               curr_index, needs_host};
    a.hist_base = hist_base;
    a.hist_t = hist_t;
    a.cur_fail = g_learner_fail;
    StepLaunch f{a, (hipStream_t)stream, true};
    return dispatch(L, f);
}

int acx_rollout(int32_t* state, const int32_t* actions, const int32_t* reset_state, int32_t* step_count,
                int32_t* obs_traj, int32_t* reward_traj, uint8_t* done_traj, uint8_t* trunc_traj, uint8_t* err,
                int32_t* err_count, int32_t T, int64_t B, int32_t L, int32_t horizon, int32_t cyclical,
                void* stream) {
    if (B < 0 || T < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0 || T == 0) return ACX_OK;
    if (!state || !actions || !reset_state || !step_count) return ACX_E_ARG;
    if (!aligned16(state) || !aligned16(reset_state) || (obs_traj && !aligned16(obs_traj))) return ACX_E_ARG;
    RolloutArgs a{state, actions, nullptr, reset_state, step_count, obs_traj, reward_traj, done_traj, trunc_traj,
                  err, err_count, B, T, L, horizon, cyclical};
    RolloutLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int64_t acx_packed_actions_words(int32_t T, int64_t B) { return T <= 0 || B <= 0 ? 0 : (int64_t)((T + 7) / 8) * B; }

int acx_pack_actions(const int32_t* actions, uint32_t* packed, int32_t T, int64_t B, void* stream) {
    if (B < 0 || T < 0) return ACX_E_ARG;
    if (B == 0 || T == 0) return ACX_OK;
    if (!actions || !packed || (T + 7) / 8 > 65535) return ACX_E_ARG;
    if (B % 4 == 0 && aligned16(actions) && aligned16(packed)) {
        const dim3 grid((unsigned)((B / 4 + 255) / 256), (unsigned)((T + 7) / 8));
        pack_actions_kernel<true><<<grid, dim3(256), 0, (hipStream_t)stream>>>(actions, packed, T, B);
    } else {
        const dim3 grid((unsigned)((B + 255) / 256), (unsigned)((T + 7) / 8));
        pack_actions_kernel<false><<<grid, dim3(256), 0, (hipStream_t)stream>>>(actions, packed, T, B);
    }
    return finish_launch();
}

int acx_rollout_packed(int32_t* state, const uint32_t* packed_actions, const int32_t* reset_state,
                       int32_t* step_count, int32_t* obs_traj, int32_t* reward_traj, uint8_t* done_traj,
                       uint8_t* trunc_traj, uint8_t* err, int32_t* err_count, int32_t T, int64_t B, int32_t L,
                       int32_t horizon, int32_t cyclical, void* stream) {
    if (B < 0 || T < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0 || T == 0) return ACX_OK;
    if (!state || !packed_actions || !reset_state || !step_count) return ACX_E_ARG;
    if (!aligned16(state) || !aligned16(reset_state) || (obs_traj && !aligned16(obs_traj))) return ACX_E_ARG;
    RolloutArgs a{state, nullptr, packed_actions, reset_state, step_count, obs_traj, reward_traj, done_traj,
                  trunc_traj, err, err_count, B, T, L, horizon, cyclical};
    RolloutLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_rollout_obs8(int32_t* state, const int32_t* actions, const uint32_t* packed_actions, const int32_t* reset_state,
                     int32_t* step_count, int8_t* obs_traj8, int32_t* reward_traj, uint8_t* done_traj,
                     uint8_t* trunc_traj, uint8_t* err, int32_t* err_count, int32_t T, int64_t B, int32_t L,
                     int32_t horizon, int32_t cyclical, void* stream) {
    if (B < 0 || T < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0 || T == 0) return ACX_OK;
    if (!state || !reset_state || !step_count || !obs_traj8 || (!actions == !packed_actions)) return ACX_E_ARG;
    if (!aligned16(state) || !aligned16(reset_state) || !aligned16(obs_traj8)) return ACX_E_ARG;
    RolloutArgs a{state, actions, packed_actions, reset_state, step_count, nullptr, reward_traj, done_traj,
                  trunc_traj, err, err_count, B, T, L, horizon, cyclical, obs_traj8};
    RolloutLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_expand12(const int32_t* parents, int32_t* children, int32_t* child_len, uint64_t* child_key, uint8_t* err,
                 int32_t* err_count, int64_t N, int32_t L, int32_t cyclical, void* stream) {
    if (N < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (N == 0) return ACX_OK;
    if (!parents || !aligned16(parents) || (children && !aligned16(children))) return ACX_E_ARG;
    ExpandArgs a{parents, children, child_len, child_key, err, err_count, N, L, cyclical, acx_key_words(L)};
    ExpandLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_canonicalize(const int32_t* state_in, int32_t* state_out, int32_t* lengths_out, uint8_t* err,
                     int32_t* err_count, int64_t B, int32_t L, int32_t cyclical, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if (!state_in || !state_out || !aligned16(state_in) || !aligned16(state_out)) return ACX_E_ARG;
    CanonArgs a{state_in, state_out, lengths_out, err, err_count, B, L, cyclical};
    CanonLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

int acx_unpack_keys(const uint64_t* keys, int32_t* states, int32_t* lengths_out, int64_t M, int32_t L,
                    void* stream) {
    if (M < 0 || L < 1 || L > ACX_MAX_L) return ACX_E_ARG;
    if (M == 0) return ACX_OK;
    if (!keys || !states || !aligned16(states)) return ACX_E_ARG;
    UnpackArgs a{keys, states, lengths_out, M, L, acx_key_words(L)};
    UnpackLaunch f{a, (hipStream_t)stream};
    return dispatch(L, f);
}

}  // extern "C"
#endif  // ACX_PART
