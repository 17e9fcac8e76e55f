// acx_curriculum.hip -- the PPO trainer's start-state curriculum on the GPU.
//
// Reference: ac_solver/agents/training.py:319-352.  After every env step, each env whose
// episode ended (done or truncated), in env-index order, takes the next start state:
// while "round 1" is not complete the next unprocessed initial state,
// max(states_processed) + 1 (:329-336); afterwards a random solved/unsolved state
// (:337-346, Python `random`, left to the host).  The env's observation and its reset
// state become initial_states[idx] (:349-352).
// Here `next_index` holds max(states_processed) + 1; finished envs are ranked by a prefix
// sum in env order, so env i gets next_index + (number of finished envs before i) --
// exactly the sequence of the reference's loop.  Envs whose index would reach n_states
// (round 1 complete) are flagged in needs_host and left for the host to place.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acx.h"

namespace acx {
namespace cur {

constexpr int TPB = 256;
constexpr int WAVE = 64;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& tot) {
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
    for (int i = 0; i < TPB / WAVE; ++i) {
        off += i < wid ? sh[i] : 0u;
        tot += sh[i];
    }
    return off + x - v;
}

struct Args {
    const uint8_t* done;
    const uint8_t* truncated;
    const int32_t* states;  // (n_states, 2L) curriculum table
    int64_t n_states;
    int32_t* next_index;    // [1] max(states_processed) + 1
    int32_t* curr_index;    // (B)
    uint8_t* needs_host;    // (B)
    int32_t* state;         // (B, 2L)
    int32_t* reset_state;   // (B, 2L) or NULL
    float* obs_f32;         // (B, 2L) or NULL
    uint32_t* bsum;         // (nblocks) workspace
    int32_t* base;          // [1] workspace: next_index before this call
    int64_t B;
    int L;
};

__device__ __forceinline__ bool finished(const Args& a, int64_t i) {
    return i < a.B && ((a.done && a.done[i]) || (a.truncated && a.truncated[i]));
}

__global__ __launch_bounds__(TPB) void count_kernel(Args a) {
    __shared__ uint32_t sh[TPB / WAVE];
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    uint32_t tot;
    block_excl_scan(finished(a, i) ? 1u : 0u, sh, tot);
    if (threadIdx.x == 0) a.bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void scan_kernel(Args a, int nb) {
    __shared__ uint32_t sh[1024 / WAVE];
    const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
    const int per = (nb + 1023) / 1024;
    const int b0 = t * per, b1 = min(nb, b0 + per);
    uint32_t loc = 0;
    for (int i = b0; i < b1; ++i) loc += a.bsum[i];
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
    const int32_t nxt = *a.next_index;
    uint32_t run = off + x - loc;
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = a.bsum[i];
        a.bsum[i] = run;
        run += c;
    }
    __syncthreads();
    if (t == 0) {
        *a.base = nxt;
        const int64_t n = (int64_t)nxt + tot;
        *a.next_index = (int32_t)(n < a.n_states ? n : a.n_states);
    }
}

// each finished env of the block takes its state; the block's copies are made by all its threads,
// 16-byte chunks spread over them (a thread copying its own env's row element by element took
// 24-35 us per 2^20-env step with ~B/H envs finishing)
__global__ __launch_bounds__(TPB) void assign_kernel(Args a) {
    __shared__ uint32_t sh[TPB / WAVE];
    __shared__ int64_t sidx[TPB];  // the block's finished envs with a state, in env order: their table row
    __shared__ int32_t senv[TPB];  //   ... and their env index within the block
    __shared__ uint32_t scnt;
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    const bool f = finished(a, i);
    uint32_t tot;
    const uint32_t r = block_excl_scan(f ? 1u : 0u, sh, tot);
    if (threadIdx.x == 0) scnt = 0;
    __syncthreads();
    if (i < a.B) {
        uint8_t nh = 0;
        if (f) {
            const int64_t idx = (int64_t)*a.base + a.bsum[blockIdx.x] + r;
            if (idx >= a.n_states) {  // round 1 complete (training.py:329-333): the host picks
                nh = 1;
            } else {
                a.curr_index[i] = (int32_t)idx;
                // the finished envs that take a state are a prefix of the block's finished envs
                // (idx grows with r), so r is also their position in the copy list
                sidx[r] = idx;
                senv[r] = (int32_t)threadIdx.x;
                atomicAdd(&scnt, 1u);  // LDS
            }
        }
        a.needs_host[i] = nh;
    }
    __syncthreads();
    const int n = (int)scnt;
    const int twoL = 2 * a.L;
    const int64_t row0 = (int64_t)blockIdx.x * TPB;
    if ((twoL & 3) == 0) {
        const int cpr = twoL >> 2;
        for (int t = threadIdx.x; t < n * cpr; t += TPB) {
            const int q = t / cpr, c = t - q * cpr;
            const int64_t e = row0 + senv[q];
            const int4 v = reinterpret_cast<const int4*>(a.states + sidx[q] * twoL)[c];
            reinterpret_cast<int4*>(a.state + e * twoL)[c] = v;
            if (a.reset_state) reinterpret_cast<int4*>(a.reset_state + e * twoL)[c] = v;
            if (a.obs_f32)
                reinterpret_cast<float4*>(a.obs_f32 + e * twoL)[c] = make_float4((float)v.x, (float)v.y, (float)v.z,
                                                                                 (float)v.w);
        }
    } else {
        for (int t = threadIdx.x; t < n * twoL; t += TPB) {
            const int q = t / twoL, c = t - q * twoL;
            const int64_t e = row0 + senv[q];
            const int32_t v = a.states[sidx[q] * twoL + c];
            a.state[e * twoL + c] = v;
            if (a.reset_state) a.reset_state[e * twoL + c] = v;
            if (a.obs_f32) a.obs_f32[e * twoL + c] = (float)v;
        }
    }
}

}  // namespace cur
}  // namespace acx

using namespace acx::cur;

extern "C" {

int64_t acx_internal_curriculum_fused_offset(int64_t B);
#define ACX_CUR_ARRIVE_STRIDE 32  // as acx_kernels.hip's CurLayout
int64_t acx_curriculum_workspace(int64_t B) {
    if (B < 0) return 0;
    const int64_t tiles = (B + WAVE - 1) / WAVE, groups = (tiles + WAVE - 1) / WAVE;
    // acx_learner_step's part: [0] sequence number, [1, 2] base, tile counts, group totals, and
    // the groups' arrival words ACX_CUR_ARRIVE_STRIDE apart (acx_kernels.hip, CurLayout)
    return acx_internal_curriculum_fused_offset(B) + 2 * (3 + tiles + groups + groups * ACX_CUR_ARRIVE_STRIDE);
}

int acx_curriculum_assign(const uint8_t* done, const uint8_t* truncated, const int32_t* curriculum_states,
                          int64_t n_states, int32_t* next_index, int32_t* curr_index, uint8_t* needs_host,
                          int32_t* state, int32_t* reset_state, float* obs_f32, int32_t* workspace, int64_t B,
                          int32_t L, void* stream) {
    if (B < 0 || L < 1 || L > ACX_MAX_L || n_states < 0 || n_states > INT32_MAX) return ACX_E_ARG;
    if (B == 0) return ACX_OK;
    if ((!done && !truncated) || !curriculum_states || !next_index || !curr_index || !needs_host || !state ||
        !workspace)
        return ACX_E_ARG;
    auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
    if ((L % 2) == 0 && (!a16(curriculum_states) || !a16(state) || (reset_state && !a16(reset_state)) ||
                         (obs_f32 && !a16(obs_f32))))
        return ACX_E_ARG;  // the copies move 16-byte chunks
    const int nb = (int)((B + TPB - 1) / TPB);
    Args a{done, truncated, curriculum_states, n_states, next_index, curr_index, needs_host, state, reset_state,
           obs_f32, reinterpret_cast<uint32_t*>(workspace) + 1, workspace, B, L};
    hipStream_t st = (hipStream_t)stream;
    count_kernel<<<dim3(nb), dim3(TPB), 0, st>>>(a);
    scan_kernel<<<dim3(1), dim3(1024), 0, st>>>(a, nb);
    assign_kernel<<<dim3(nb), dim3(TPB), 0, st>>>(a);
    return hipGetLastError() == hipSuccess ? ACX_OK : ACX_E_LAUNCH;
}

// acx_learner_step (acx_kernels.hip) ranks the finished envs inside its step kernel with a
// look-back over per-64-env-tile status words; its part of the workspace starts after this
// file's (next_index copy + per-block counts), so either call may use one workspace:
// uint64 words from off: the launch sequence number, the base, one reserved word, one count per
// 64-env tile, then per group of 64 tiles its total and its arrival word (acx_kernels.hip
// cur_publish / cur_prefix).
int64_t acx_internal_curriculum_fused_offset(int64_t B) {
    const int64_t own = (B + TPB - 1) / TPB + 2;
    return (own + 1) & ~(int64_t)1;  // 8-byte aligned
}

}  // extern "C"
