// Calibration of the read side of rocprofv3's FETCH_SIZE for partial-line reads (config 5's
// lengths-carrying step reads each relator's live 16-B chunks: its last 128-B line is usually
// read in part).  read_lines<P, OFF>: every 128-B line of a buffer is read P x 16 B, starting
// OFF x 16 B into the line (P = 8: the whole line; P = 4: one 64-B sector; P = 1: one chunk),
// one 16-B load per lane, grid-stride, one dword out per block (never taken).  Timed against the
// full-line read of the same lines and run under rocprofv3 --pmc (tools/line_probe.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int P, int OFF>
__global__ __launch_bounds__(256) void read_lines(const int4* __restrict__ src, int64_t lines, int* out) {
    constexpr int LPI = 64 / P;  // lines per wave-instruction
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
    int acc = 0;
    for (int64_t l0 = wave * LPI; l0 < lines; l0 += nw * LPI) {
        const int64_t line = l0 + lane / P;
        if (line < lines) {
            const int4 v = src[line * 8 + OFF + lane % P];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x7fffffff) out[blockIdx.x] = acc;
}

extern "C" int line_probe_run(int kind, const void* buf, int64_t lines, void* out, void* stream) {
    const dim3 grid(256 * 8), block(256);
    hipStream_t s = (hipStream_t)stream;
    const int4* src = (const int4*)buf;
    int* o = (int*)out;
    switch (kind) {
        case 0: read_lines<8, 0><<<grid, block, 0, s>>>(src, lines, o); break;  // whole line
        case 1: read_lines<4, 0><<<grid, block, 0, s>>>(src, lines, o); break;  // first sector
        case 2: read_lines<4, 4><<<grid, block, 0, s>>>(src, lines, o); break;  // second sector
        case 3: read_lines<1, 0><<<grid, block, 0, s>>>(src, lines, o); break;  // one chunk
        case 4: read_lines<2, 3><<<grid, block, 0, s>>>(src, lines, o); break;  // 32 B across the sector boundary
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
