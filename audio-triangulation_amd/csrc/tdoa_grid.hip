// tdoa_grid.hip -- the grid solve of vga_draw_heatmap's max pass
// (src/components/vga/vga_heatmap.h:99-108) as its own kernel:
//   L(cell) = sum_p weighted_p[LUT_p(cell)],  max L,  first row-major argmax,
// evaluated over the distinct lag tuples of the grid (tuples are in
// first-cell order, so the first maximal tuple carries the first argmax cell).
//
// One 256-thread workgroup scores F = 8 frames per tuple: the tuple table
// (U words) and the 8 frames' weighted scores, transposed to [p][k][frame],
// sit in LDS, so one tuple costs P vector gathers for all 8 frames.
// Running it apart from the FFT / xcorr kernels lets it run at full
// occupancy; it reads B*P*K weighted scores (1.1 KiB/frame fp32) back from L2/HBM.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cmath>

#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {


template <typename T> __device__ __forceinline__ T lowest_t();
template <> __device__ __forceinline__ int64_t lowest_t<int64_t>() { return INT64_MIN; }
template <> __device__ __forceinline__ float lowest_t<float>() { return -INFINITY; }

template <typename T>
__device__ __forceinline__ void better_t(T &bv, int &bu, T ov, int ou)
{
    if (ov > bv || (ov == bv && ou < bu)) {
        bv = ov;
        bu = ou;
    }
}

template <typename T>
__device__ __forceinline__ void store_max_t(const tdoa_kout &o, int64_t i, T v);
template <>
__device__ __forceinline__ void store_max_t<int64_t>(const tdoa_kout &o, int64_t i, int64_t v)
{
    if (o.max_L)
        o.max_L[i] = v;
}
template <>
__device__ __forceinline__ void store_max_t<float>(const tdoa_kout &o, int64_t i, float v)
{
    if (o.max_Lf)
        o.max_Lf[i] = v;
}

// GF frames per workgroup (8; 1 for 8-mic grids whose scores fill LDS);
// the tuple table is staged in LDS when it fits, else read from L2.
template <typename T, int TWC, int GF>
__global__ void __launch_bounds__(256) k_grid(tdoa_kparams kp, tdoa_kout out,
                                              const T *__restrict__ weighted, int64_t B,
                                              int stage_tuples)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int P = kp.P, K = kp.K, U = kp.U, TW = kp.TW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *tups = stage_tuples ? (uint32_t *)smem : (uint32_t *)kp.tuples;  // [U * TW]
    const size_t toff = stage_tuples ? ((((size_t)U * TW * 4) + 15) & ~(size_t)15) : 0;
    T *W = (T *)(smem + toff);                                        // [P][K][GF]
    T *redv = W + (size_t)P * K * GF;                                 // [4][GF]
    int *redi = (int *)(redv + 4 * GF);                               // [4][GF]

    const int64_t f0 = (int64_t)blockIdx.x * GF;
    const int nf = (B - f0) < GF ? (int)(B - f0) : GF;
    if (stage_tuples)
        for (int e = tid; e < U * TW; e += 256)
            tups[e] = kp.tuples[e];
    // transpose the frames' [P][K] score rows to [p][k][frame]; absent frames
    // score the lowest value so they never matter
    const int PK = P * K;
    for (int e = tid; e < GF * PK; e += 256) {
        const int f = e / PK, r = e - f * PK;
        W[r * GF + f] = f < nf ? weighted[(f0 + f) * PK + r] : lowest_t<T>();
    }
    __syncthreads();

    T bv[GF];
    int bu[GF];
#pragma unroll
    for (int f = 0; f < GF; f++) {
        bv[f] = lowest_t<T>();
        bu[f] = INT_MAX;
    }
    for (int u = tid; u < U; u += 256) {  // increasing u per thread: strict '>' keeps the first
        T L[GF];
#pragma unroll
        for (int f = 0; f < GF; f++)
            L[f] = 0;
#pragma unroll
        for (int tw = 0; tw < TWC; tw++) {
            if (tw < TW) {
                const uint32_t word = tups[u * TW + tw];
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int p = 4 * tw + b;
                    if (p < P) {
                        const T *src = W + (size_t)(p * K + ((word >> (8 * b)) & 0xFFu)) * GF;
#pragma unroll
                        for (int f = 0; f < GF; f++)
                            L[f] += src[f];
                    }
                }
            }
        }
#pragma unroll
        for (int f = 0; f < GF; f++)
            if (L[f] > bv[f]) {
                bv[f] = L[f];
                bu[f] = u;
            }
    }
#pragma unroll
    for (int f = 0; f < GF; f++) {
        for (int m = 32; m >= 1; m >>= 1)
            better_t(bv[f], bu[f], __shfl_xor(bv[f], m, 64), __shfl_xor(bu[f], m, 64));
        if (lane == 0) {
            redv[wave * GF + f] = bv[f];
            redi[wave * GF + f] = bu[f];
        }
    }
    __syncthreads();
    if (tid < nf) {
        const int f = tid;
        T v = redv[f];
        int ui = redi[f];
        for (int w = 1; w < 4; w++)
            better_t(v, ui, redv[w * GF + f], redi[w * GF + f]);
        if (ui < 0 || ui >= U)  // only if every L compared false (NaN scores)
            ui = 0;
        const int cell = kp.tuple_cell[ui];
        const int64_t fi = f0 + f;
        if (out.cell)
            out.cell[fi] = cell;
        store_max_t<T>(out, fi, v);
        if (out.xy) {
            const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
            out.xy[2 * fi] = (float)(cx - kp.half_w) / kp.grid_scale;
            out.xy[2 * fi + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
        }
    }
}

int hip_fail(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

template <typename T>
int launch(const tdoa_kparams &kp, const tdoa_kout &out, const T *weighted, int64_t B,
           void *stream)
{
    const size_t tbytes = (((size_t)kp.U * kp.TW * 4) + 15) & ~(size_t)15;
    const size_t per_frame = (size_t)kp.P * kp.K * sizeof(T);
    const int gf = per_frame * 8 <= 48 * 1024 ? 8 : 1;
    const size_t red = 4 * (size_t)gf * (sizeof(T) + sizeof(int));
    const int stage = tbytes + per_frame * gf + red <= 96 * 1024 ? 1 : 0;
    const size_t lds = (stage ? tbytes : 0) + per_frame * gf + red;
    if (lds > 160 * 1024)
        return tdoa_set_error(-1, "grid: scores of one frame exceed 160 KiB LDS");
    const int64_t grid = (B + gf - 1) / gf;
    if (grid > INT_MAX)
        return tdoa_set_error(-1, "grid: batch too large for one launch");
    hipStream_t st = (hipStream_t)stream;
    constexpr int TWX = (TDOA_MAX_PAIRS + 3) / 4;
    if (kp.TW == 1 && gf == 8)
        hipLaunchKernelGGL((k_grid<T, 1, 8>), dim3((unsigned)grid), dim3(256), lds, st, kp, out,
                           weighted, B, stage);
    else if (kp.TW == 1)
        hipLaunchKernelGGL((k_grid<T, 1, 1>), dim3((unsigned)grid), dim3(256), lds, st, kp, out,
                           weighted, B, stage);
    else if (gf == 8)
        hipLaunchKernelGGL((k_grid<T, TWX, 8>), dim3((unsigned)grid), dim3(256), lds, st, kp,
                           out, weighted, B, stage);
    else
        hipLaunchKernelGGL((k_grid<T, TWX, 1>), dim3((unsigned)grid), dim3(256), lds, st, kp,
                           out, weighted, B, stage);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "k_grid launch");
}

}  // namespace

int tdoa_launch_grid(const tdoa_kparams &kp, const tdoa_kout &out, const void *weighted,
                     bool is_float, int64_t B, void *stream)
{
    if (B <= 0 || (!out.cell && !out.xy && !out.max_L && !out.max_Lf))
        return 0;
    return is_float ? launch<float>(kp, out, (const float *)weighted, B, stream)
                    : launch<int64_t>(kp, out, (const int64_t *)weighted, B, stream);
}
