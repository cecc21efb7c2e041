// tdoa_grid.hip -- the grid solve of vga_draw_heatmap's max pass
// (src/components/vga/vga_heatmap.h:99-108) as its own kernel:
//   L(cell) = sum_p weighted_p[LUT_p(cell)],  max L,  first row-major argmax,
// evaluated over the distinct lag tuples of the grid (tuples are in
// first-cell order, so the first maximal tuple carries the first argmax cell).
//
// One workgroup scores GF = 8 frames per tuple (4 or 1 when their scores
// would not fit): the tuple table (U x TW words, in chunks when large) and the
// frames' weighted scores, transposed to [p][k][frame], sit in LDS, so one
// tuple costs P vector gathers for all GF frames.
// Running it apart from the FFT / xcorr kernels lets it run at full
// occupancy; it reads B*P*K weighted scores (1.1 KiB/frame fp32) back from L2/HBM.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cmath>
#include <cstdlib>

#include <type_traits>

#include "tdoa_internal.h"
#include "tdoa_grid_bb.h"

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

// GF frames per workgroup (8, 4 or 1: as many as the [P][K][GF] score block
// allows); the tuple table passes through LDS in chunks of CH tuples (one
// chunk for 3-4 mic grids, several for the 28-pair grid of config 4).
template <typename T, int TWC, int GF>
__global__ void __launch_bounds__(1024) k_grid(tdoa_kparams kp, tdoa_kout out,
                                               const T *__restrict__ weighted, int64_t B, int CH)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int P = kp.P, K = kp.K, U = kp.U, TW = kp.TW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nth = blockDim.x;
    const int nwaves = nth >> 6;
    uint32_t *tups = (uint32_t *)smem;                                      // [CH * TW]
    T *W = (T *)(smem + ((((size_t)CH * TW * 4) + 15) & ~(size_t)15));      // [P][K][GF]
    T *redv = W + (size_t)P * K * GF;                                       // [nwaves][GF]
    int *redi = (int *)(redv + (size_t)nwaves * GF);                        // [nwaves][GF]

    const int64_t f0 = (int64_t)blockIdx.x * GF;
    const int nf = (B - f0) < GF ? (int)(B - f0) : GF;
    // transpose the frames' [P][K] score rows to [p][k][frame]; absent frames
    // score the lowest value so they never matter
    const int PK = P * K;
    for (int e = tid; e < GF * PK; e += nth) {
        const int f = e / PK, r = e - f * PK;
        W[r * GF + f] = f < nf ? weighted[(f0 + f) * PK + r] : lowest_t<T>();
    }

    T bv[GF];
    int bu[GF];
#pragma unroll
    for (int f = 0; f < GF; f++) {
        bv[f] = lowest_t<T>();
        bu[f] = INT_MAX;
    }
    for (int c0 = 0; c0 < U; c0 += CH) {
        const int n = (U - c0) < CH ? U - c0 : CH;
        __syncthreads();  // previous chunk consumed (and, first time, W written)
        for (int e = tid; e < n * TW; e += nth)
            tups[e] = kp.tuples[(size_t)c0 * TW + e];
        __syncthreads();
        // increasing u per thread across chunks: strict '>' keeps the first
        for (int u = tid; u < n; u += nth) {
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
                    bu[f] = c0 + u;
                }
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
        for (int w = 1; w < nwaves; w++)
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

#ifdef TDOA_DIAG
__device__ unsigned long long g_diag_bb[8192 * 8];  // per-wave phase cycles (tdoa_grid_bb.h)
#endif

// ---------------------------------------------------------------------------
// k_grid_bb: the same solve (max L, first argmax tuple) by exact branch and
// bound, one wave per frame (tdoa_grid_bb.h).
// at most 10 waves (640 threads) for the many-pair tables (TWC > 4, more than 8
// pairs: config 4's LDS holds 10 frames), so the solve gets up to 168 VGPRs
// instead of 128
template <int TWC> constexpr int bb_max_threads() { return TWC > 4 ? 640 : 1024; }
#ifndef BB_WPE
#define BB_WPE
#endif
template <typename T, int TWC, int JT>
__global__ void __launch_bounds__(bb_max_threads<TWC>()) BB_WPE k_grid_bb(tdoa_kparams kp, tdoa_kout out,
                                                  const T *__restrict__ weighted, int64_t B)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int P = kp.P, K = kp.K, NT = kp.bb_NT, PK = P * K, KS = tdoa_bb::bb_ks(P, K);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = blockDim.x >> 6;
    const int32_t *tiles = kp.bb_tile;  // [NT][2], read by entry (wave-uniform)
    uint16_t *qt = (uint16_t *)smem;    // [NT][P]
    // per wave: the frame's scores Wl [P][K], then the solve's sparse-table
    // levels (tdoa_bb::bb_scratch), 16-B aligned
    const size_t per_wave =
        ((size_t)(tdoa_bb::bb_pk(P, K) + tdoa_bb::bb_scratch(P, K)) * sizeof(T) + 15) & ~(size_t)15;
    T *Wl = (T *)(smem + (((size_t)NT * 2 * P) + 15 & ~(size_t)15) + (size_t)wave * per_wave);
    for (int e = tid; e < NT * P; e += blockDim.x)
        qt[e] = kp.bb_q[e];
    __syncthreads();

    unsigned long long bbacc[8] = {};
    if constexpr (std::is_same<T, float>::value)
        if (out.weighted_c)  // compact scratch: the unused lags of Wl stay defined (never read)
            for (int e = lane; e < tdoa_bb::bb_pk(P, K); e += 64)
                Wl[e] = (T)0;
    for (int64_t f = (int64_t)blockIdx.x * NW + wave; f < B; f += (int64_t)gridDim.x * NW) {
#ifdef TDOA_DIAG
        const unsigned long long t_load = __builtin_amdgcn_s_memtime();
#endif
        wave_lds_sync();  // the previous frame's reads of Wl come first
        {
            // the frame's P x K scores (10.4 KB at config 4): 16-B loads, eight per
            // lane in flight before their LDS stores (one element per load and
            // iteration waited on every load in turn: ~40 HBM round trips a frame);
            // nontemporal, so the streamed scores do not evict the entry tables'
            // tuples from L2 (every evaluation reads them)
            bool compact = false;
            if constexpr (std::is_same<T, float>::value)
                compact = out.weighted_c != nullptr;
            if (compact) {
                // compact scratch: 16-B chunks of the used lags, expanded to
                // Wl[p][KS] (lags no tuple uses are never read)
                typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
                const v4u_t *s4 = reinterpret_cast<const v4u_t *>(out.weighted_c + f * kp.wc_CK);
                const int nch = kp.wc_nch;
                for (int b = 0; b < nch; b += 4 * 64) {
                    v4u_t t[4];
                    uint32_t dsc[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {  // clamped: unconditional loads
                        const int c = b + i * 64 + lane;
                        const int cc = c < nch ? c : nch - 1;
                        t[i] = __builtin_nontemporal_load(&s4[cc]);
                        dsc[i] = kp.wc_chunks[cc];
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int c = b + i * 64 + lane;
                        if (c < nch && P > 8) {
                            // many pairs: 16-B aligned chunks (rows KS apart, chunk
                            // starts multiples of 4, tdoa_capi.cpp): one store; a
                            // last chunk's extra lags lie past every tuple's lag
                            *reinterpret_cast<v4u_t *>(reinterpret_cast<float *>(Wl) + (dsc[i] & 0xFFFFu)) = t[i];
                        } else if (c < nch) {
                            float *d = reinterpret_cast<float *>(Wl) + (dsc[i] & 0xFFFFu);
                            const int n = (int)(dsc[i] >> 16);
                            // scalar copies first: __builtin_bit_cast of an
                            // ext_vector element reads element 0 with this compiler
                            const unsigned u0 = t[i].x, u1 = t[i].y, u2 = t[i].z, u3 = t[i].w;
                            d[0] = __uint_as_float(u0);
                            if (n > 1)
                                d[1] = __uint_as_float(u1);
                            if (n > 2)
                                d[2] = __uint_as_float(u2);
                            if (n > 3)
                                d[3] = __uint_as_float(u3);
                        }
                    }
                }
            } else if (KS != K) {
                // full [P][K] scores into rows KS apart
                const T *src = weighted + f * PK;
                for (int e = lane; e < PK; e += 64)
                    Wl[e + (e / K) * (KS - K)] = __builtin_nontemporal_load(&src[e]);
            } else {
            const T *src = weighted + f * PK;
            const int nv = (int)(((size_t)PK * sizeof(T)) / 16);
            const bool vec = nv > 0 && (((uintptr_t)src | (uintptr_t)Wl) & 15) == 0;
            int e0 = 0;
            if (vec) {
                const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
                uint4 *d4 = reinterpret_cast<uint4 *>(Wl);
                for (int b = 0; b < nv; b += 8 * 64) {
                    uint4 t[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) {  // clamped: unconditional loads
                        const int e = b + i * 64 + lane;
                        typedef unsigned v4u __attribute__((ext_vector_type(4)));
                        const v4u x = __builtin_nontemporal_load(
                            reinterpret_cast<const v4u *>(&s4[e < nv ? e : nv - 1]));
                        t[i] = make_uint4(x.x, x.y, x.z, x.w);
                    }
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int e = b + i * 64 + lane;
                        if (e < nv)
                            d4[e] = t[i];
                    }
                }
                e0 = nv * (int)(16 / sizeof(T));
            }
            for (int e = e0 + lane; e < PK; e += 64)
                Wl[e] = src[e];
            }
        }
        wave_lds_sync();  // a wave's LDS operations complete in order
#ifdef TDOA_DIAG
        {
            // the loads' data reaches LDS (and so the clock) once the stores are issued
            __builtin_amdgcn_s_waitcnt(0);
            bbacc[0] += __builtin_amdgcn_s_memtime() - t_load;
            bbacc[5] += 1;
        }
#endif
        T best;
        int bu;
        tdoa_bb::solve_wave<T, TWC, JT>(kp, Wl, tiles, qt, lane, best, bu, bbacc);
        if (lane == 0) {
            const int ui = (bu < 0 || bu >= kp.U) ? 0 : bu;  // every L compared false: tuple 0
            const int cell = kp.tuple_cell[ui];
            if (out.cell)
                out.cell[f] = cell;
            store_max_t<T>(out, f, best);
            if (out.xy) {
                const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
                out.xy[2 * f] = (float)(cx - kp.half_w) / kp.grid_scale;
                out.xy[2 * f + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
            }
        }
    }
#ifdef TDOA_DIAG
    {
        const int gw = blockIdx.x * NW + wave;
        if (lane == 0 && gw < 8192)
            for (int i = 0; i < 8; i++)
                g_diag_bb[gw * 8 + i] = bbacc[i];
    }
#endif
}


constexpr size_t BB_LDS = 160 * 1024;  // k_grid_bb's LDS: the entry table + per-wave scratch and scores

template <typename T, int TWC, int JT>
int launch_bb(const tdoa_kparams &kp, const tdoa_kout &out, const T *weighted, int64_t B,
              hipStream_t st)
{
    const size_t table = ((size_t)kp.bb_NT * 2 * kp.P + 15) & ~(size_t)15;  // the queries
    const size_t per_wave =
        (((size_t)tdoa_bb::bb_pk(kp.P, kp.K) + tdoa_bb::bb_scratch(kp.P, kp.K)) * sizeof(T) + 15) & ~(size_t)15;
    int nw = (int)((BB_LDS - table) / per_wave);
    nw = nw > bb_max_threads<TWC>() / 64 ? bb_max_threads<TWC>() / 64 : nw;
    const size_t lds = table + (size_t)nw * per_wave;
    const void *kern = (const void *)k_grid_bb<T, TWC, JT>;
    const int res = tdoa_resident_blocks(kern, nw * 64, lds);
    int64_t grid = (B + nw - 1) / nw;
    if (res > 0 && grid > res)
        grid = res;
    hipLaunchKernelGGL((k_grid_bb<T, TWC, JT>), dim3((unsigned)grid), dim3(nw * 64), lds, st, kp, out,
                       weighted, B);
    return 0;
}

template <typename T, int TWC>
int launch_bb_jt(const tdoa_kparams &kp, const tdoa_kout &out, const T *weighted, int64_t B,
                 hipStream_t st)
{
    switch ((kp.bb_NT + 63) / 64) {
    case 1: return launch_bb<T, TWC, 1>(kp, out, weighted, B, st);
    case 2: return launch_bb<T, TWC, 2>(kp, out, weighted, B, st);
    case 3: return launch_bb<T, TWC, 3>(kp, out, weighted, B, st);
    default: return launch_bb<T, TWC, 4>(kp, out, weighted, B, st);
    }
}

// k_grid_bb applies: tables built, at most 256 entries, and room for the
// entry table plus one frame's scores
template <typename T>
bool bb_fits(const tdoa_kparams &kp)
{
    if (kp.bb_NT <= 0 || kp.bb_NT > 256 || !kp.bb_tile || !kp.bb_q || kp.bb_wide)
        return false;
    const size_t table = ((size_t)kp.bb_NT * 2 * kp.P + 15) & ~(size_t)15;  // the queries
    return kp.K <= 127 &&
           table + ((size_t)tdoa_bb::bb_pk(kp.P, kp.K) + tdoa_bb::bb_scratch(kp.P, kp.K)) * sizeof(T) + 16 <= BB_LDS;
}

}  // namespace
// k_grid_bb solves the float grid and can read the compact scratch
bool tdoa_grid_bb_compact(const tdoa_kparams &kp)
{
    return bb_fits<float>(kp) && kp.wc_chunks != nullptr && kp.wc_CK > 0 && kp.wc_nch > 0;
}
namespace {
int hip_fail(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

template <typename T, int TWC>
void launch_gf(int gf, dim3 grid, dim3 block, size_t lds, hipStream_t st, const tdoa_kparams &kp,
               const tdoa_kout &out, const T *weighted, int64_t B, int CH)
{
    if (gf == 8)
        hipLaunchKernelGGL((k_grid<T, TWC, 8>), grid, block, lds, st, kp, out, weighted, B, CH);
    else if (gf == 4)
        hipLaunchKernelGGL((k_grid<T, TWC, 4>), grid, block, lds, st, kp, out, weighted, B, CH);
    else
        hipLaunchKernelGGL((k_grid<T, TWC, 1>), grid, block, lds, st, kp, out, weighted, B, CH);
}

template <typename T>
int launch(const tdoa_kparams &kp, const tdoa_kout &out, const T *weighted, int64_t B,
           void *stream)
{
    // frames per workgroup: the [P][K][GF] score block within 96 KiB
    const size_t per_frame = (size_t)kp.P * kp.K * sizeof(T);
    int gf = 8;
    while (gf > 1 && per_frame * gf > 96 * 1024)
        gf /= 2;
    if (gf == 2)
        gf = 1;
    // small grids (3-4 mics): 256 threads, several workgroups per CU; the
    // 28-pair grid: one big workgroup per CU sharing one score block
    const int threads = per_frame * gf > 32 * 1024 ? 1024 : 256;
    const size_t red = (size_t)(threads / 64) * gf * (sizeof(T) + sizeof(int));
    const size_t wbytes = per_frame * gf;
    // tuple chunk: the whole table if it fits beside the scores, else what does
    const size_t budget = 150 * 1024;
    if (wbytes + red + 16 + (size_t)kp.TW * 4 * threads > budget)
        return tdoa_set_error(-1, "grid: scores of one frame exceed the LDS budget");
    size_t ch = (budget - wbytes - red - 16) / ((size_t)kp.TW * 4);
    if (ch >= (size_t)kp.U)
        ch = (size_t)kp.U;
    else
        ch = ch / threads * threads;
    const int CH = (int)ch;
    const size_t lds = ((((size_t)CH * kp.TW * 4) + 15) & ~(size_t)15) + wbytes + red;
    const int64_t grid = (B + gf - 1) / gf;
    if (grid > INT_MAX)
        return tdoa_set_error(-1, "grid: batch too large for one launch");
    hipStream_t st = (hipStream_t)stream;
    constexpr int TWX = (TDOA_MAX_PAIRS + 3) / 4;
    if (bb_fits<T>(kp)) {
        if (kp.TW == 1)
            launch_bb_jt<T, 1>(kp, out, weighted, B, st);
        else if (kp.TW == 2)  // 5-8 pairs: up to 16 waves per workgroup
            launch_bb_jt<T, 2>(kp, out, weighted, B, st);
        else
            launch_bb_jt<T, TWX>(kp, out, weighted, B, st);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : hip_fail(e, "k_grid_bb launch");
    }
    if (kp.TW == 1)
        launch_gf<T, 1>(gf, dim3((unsigned)grid), dim3(threads), lds, st, kp, out, weighted, B, CH);
    else
        launch_gf<T, TWX>(gf, dim3((unsigned)grid), dim3(threads), lds, st, kp, out, weighted, B,
                          CH);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "k_grid launch");
}

// vga_heatmap.h:110-130 colouring pass as classes: 4 white (L >= 63/64 max),
// 3 green (31/32), 2 red (15/16), 1 blue (7/8), 0 black; thresholds are the
// reference's int64 (max * n) >> b; for float scores max * n / 2^b.
__device__ __forceinline__ int64_t thr_t(int64_t mx, int n, int b) { return (mx * n) >> b; }
__device__ __forceinline__ float thr_t(float mx, int n, int b) { return mx * ((float)n / (float)(1 << b)); }

template <typename T>
__global__ void __launch_bounds__(256) k_heatmap(tdoa_kparams kp, const T *__restrict__ weighted,
                                                 const T *__restrict__ max_L,
                                                 uint8_t *__restrict__ classes)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T *W = (T *)smem;  // [P][K]
    const int64_t f = blockIdx.y;
    const int P = kp.P, K = kp.K, G = kp.G, tid = threadIdx.x;
    for (int e = tid; e < P * K; e += blockDim.x)
        W[e] = weighted[(size_t)f * P * K + e];
    __syncthreads();
    const T mx = max_L[f];
    const T tw = thr_t(mx, 63, 6), tg = thr_t(mx, 31, 5), tr = thr_t(mx, 15, 4), tb = thr_t(mx, 7, 3);
    const int c = blockIdx.x * blockDim.x + tid;
    if (c >= G)
        return;
    T L = 0;
    for (int p = 0; p < P; p++)
        L += W[p * K + kp.lut[(size_t)p * G + c]];
    classes[(size_t)f * G + c] = L >= tw ? 4 : L >= tg ? 3 : L >= tr ? 2 : L >= tb ? 1 : 0;
}

}  // namespace

int tdoa_launch_heatmap(const tdoa_kparams &kp, const void *weighted, const void *max_L,
                        bool is_float, int64_t B, uint8_t *classes, void *stream)
{
    if (B <= 0)
        return 0;
    if (B > 65535)
        return tdoa_set_error(-1, "heatmap: at most 65535 frames per call");
    const dim3 grid((unsigned)((kp.G + 255) / 256), (unsigned)B);
    const size_t lds = (size_t)kp.P * kp.K * (is_float ? 4 : 8);
    hipStream_t st = (hipStream_t)stream;
    if (is_float)
        hipLaunchKernelGGL(k_heatmap<float>, grid, dim3(256), lds, st, kp, (const float *)weighted,
                           (const float *)max_L, classes);
    else
        hipLaunchKernelGGL(k_heatmap<int64_t>, grid, dim3(256), lds, st, kp,
                           (const int64_t *)weighted, (const int64_t *)max_L, classes);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "k_heatmap launch");
}

int tdoa_launch_grid(const tdoa_kparams &kp, const tdoa_kout &out, const void *weighted,
                     bool is_float, int64_t B, void *stream)
{
    if (B <= 0 || (!out.cell && !out.xy && !out.max_L && !out.max_Lf))
        return 0;
    return is_float ? launch<float>(kp, out, (const float *)weighted, B, stream)
                    : launch<int64_t>(kp, out, (const int64_t *)weighted, B, stream);
}

#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch_bb(unsigned long long *host, int n)
{
    if (n > 8192 * 8)
        n = 8192 * 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_bb), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
