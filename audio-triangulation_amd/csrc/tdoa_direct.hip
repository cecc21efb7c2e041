// tdoa_kernels.hip -- gfx950 kernels of the TDOA hot path.
//
// k_direct: one launch runs, for F frames per workgroup,
//   stage      coalesced 16-B loads of int16 [M][N] rows into LDS, per-row
//              floor-mean DC removal (rolling_buffer.c:64-66), <<8 int16 wrap
//              (buffer.c:13-16), Q15 window (buffer.c:4-11), in place
//   xcorr      exact int64 cross-correlation for every pair and lag
//              (correlations.c:9-18) with packed v_dot2_i32_i16: one operand
//              is split into a signed high byte and an unsigned low byte so
//              every int32 partial is exact; partials widen to int64 once
//   argmax     first strictly-greater lag (correlations.c:20-23), wave shuffle
//   prior      (int64)((float)score * scale[|s-best|]) (correlations.c:26-33)
//   gate       sum_p best^2 > 4 (sample_compute.h:124-134)
//   grid       L = sum_p corr_p[LUT_p] max pass (vga_heatmap.h:99-108) over
//              the distinct lag tuples of the grid, first row-major argmax
// k_average: the EMA of correlations.c:38-63 for S independent streams.
//
// Built with -ffp-contract=off: the float steps must round exactly as the
// reference's IEEE host build does.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

#include "tdoa_internal.h"
#include "tdoa_device.h"

int tdoa_set_error(int code, const char *msg);

#ifdef TDOA_DIAG
// Diagnostic build only (libtdoa_diag.so): per-workgroup phase stamps.
#define TDOA_DIAG_SLOTS 8
__device__ unsigned long long g_diag[1 << 20];
#define DIAG_STAMP(i)                                                   \
    do {                                                                \
        if (threadIdx.x == 0)                                           \
            g_diag[(size_t)blockIdx.x * TDOA_DIAG_SLOTS + (i)] =        \
                __builtin_amdgcn_s_memtime();                           \
    } while (0)
#else
#define DIAG_STAMP(i) \
    do {              \
    } while (0)
#endif

namespace {

template <bool PREPARED, int TWC>
__global__ void __launch_bounds__(1024) k_direct(tdoa_kparams kp, tdoa_kout out,
                                                 const int16_t *__restrict__ frames, int64_t B,
                                                 const int32_t *__restrict__ count)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Smem sm = carve(smem, kp, blockDim.x >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * kp.F;
    if (count) {  // batch size known on the device only (streaming pipeline)
        const int64_t c = *count;
        B = c < B ? c : B;
        if (f0 >= B)
            return;
    }
    const int nf = (int)((B - f0) < kp.F ? (B - f0) : kp.F);
    DIAG_STAMP(0);
    stage_frames<PREPARED>(kp, sm, frames, f0, nf);
    DIAG_STAMP(1);
    xcorr_phase(kp, sm, nf);
    DIAG_STAMP(2);
    argmax_prior_phase<int64_t>(kp, sm.scores, sm.best, out, f0, nf);
    DIAG_STAMP(3);
    DIAG_STAMP(4);  // grid solve runs in k_grid (tdoa_grid.hip)
}

// --------------------------------------------------------------- EMA
// correlations.c:38-63 for stream s (one workgroup per stream):
//   est = (int64)((float)est + (float)(fresh - est) * decay); best = first max
__global__ void __launch_bounds__(256) k_average(tdoa_kparams kp, int64_t *__restrict__ est,
                                                 const int64_t *__restrict__ fresh,
                                                 const float *__restrict__ decay,
                                                 int32_t *__restrict__ best, tdoa_kout out,
                                                 int do_grid)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int64_t *W = (int64_t *)smem;                   // [P][K]
    int64_t *redv = W + kp.P * kp.K;                // [4]
    int *redi = (int *)(redv + 4);                  // [4]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
    const int64_t s = blockIdx.x;
    const int K = kp.K, P = kp.P;
    const float dec = decay[s];
    for (int p = wave; p < P; p += nwaves) {
        int64_t *e = est + ((size_t)s * P + p) * K;
        const int64_t *fr = fresh + ((size_t)s * P + p) * K;
        int64_t bv = INT64_MIN;
        int bk = INT_MAX;
        for (int k = lane; k < 128; k += 64) {
            if (k < K) {
                const int64_t ev = e[k];
                const float delta = (float)(fr[k] - ev) * dec;
                const float sum = (float)ev + delta;
                const int64_t nv = (int64_t)sum;
                e[k] = nv;
                W[p * K + k] = nv;
                if (nv > bv) {
                    bv = nv;
                    bk = k;
                }
            }
        }
        for (int m = 32; m >= 1; m >>= 1) {
            const int64_t ov = __shfl_xor(bv, m, 64);
            const int ok = __shfl_xor(bk, m, 64);
            if (ov > bv || (ov == bv && ok < bk)) {
                bv = ov;
                bk = ok;
            }
        }
        if (lane == 0)
            best[s * P + p] = bk - kp.S;
    }
    __syncthreads();
    if (!do_grid)
        return;
    int64_t bv = INT64_MIN;
    int bu = INT_MAX;
    for (int u = tid; u < kp.U; u += blockDim.x) {
        int64_t L = 0;
        for (int tw = 0; tw < kp.TW; tw++) {
            const uint32_t word = kp.tuples[u * kp.TW + tw];
            for (int b = 0; b < 4; b++) {
                const int p = 4 * tw + b;
                if (p < P)
                    L += W[p * K + ((word >> (8 * b)) & 0xFFu)];
            }
        }
        if (L > bv) {
            bv = L;
            bu = u;
        }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const int64_t ov = __shfl_xor(bv, m, 64);
        const int ou = __shfl_xor(bu, m, 64);
        if (ov > bv || (ov == bv && ou < bu)) {
            bv = ov;
            bu = ou;
        }
    }
    if (lane == 0) {
        redv[wave] = bv;
        redi[wave] = bu;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < nwaves; w++)
            if (redv[w] > bv || (redv[w] == bv && redi[w] < bu)) {
                bv = redv[w];
                bu = redi[w];
            }
        if (bu < 0 || bu >= kp.U)
            bu = 0;
        const int cell = kp.tuple_cell[bu];
        if (out.cell)
            out.cell[s] = cell;
        if (out.max_L)
            out.max_L[s] = bv;
        if (out.xy) {
            out.xy[2 * s] = (float)(cell % kp.grid_W - kp.half_w) / kp.grid_scale;
            out.xy[2 * s + 1] = (float)(kp.half_h - cell / kp.grid_W) / kp.grid_scale;
        }
    }
}

// ------------------------------------------------ per-frame reference ops
// op 0: rolling_buffer.c:43-71  linearise ring from head, floor-mean DC, power
// op 1: buffer.c:13-18          x <<= 8 (int16 wrap)
// op 2: buffer.c:4-11           x = (int16)((int32)x * W[i] >> 15)
__global__ void __launch_bounds__(256) k_ref_buffer(int op, int16_t *__restrict__ buf,
                                                    const int16_t *__restrict__ ring, int head,
                                                    int64_t *__restrict__ power,
                                                    const int16_t *__restrict__ window, int n,
                                                    int log2n)
{
    __shared__ int tot;
    __shared__ unsigned long long pw;
    const int tid = threadIdx.x;
    if (op == 0) {
        if (tid == 0) {
            tot = 0;
            pw = 0;
        }
        __syncthreads();
        int s = 0;
        for (int i = tid; i < n; i += blockDim.x)
            s += ring[(head + i) & (n - 1)];
        atomicAdd(&tot, s);
        __syncthreads();
        const uint32_t off16 = (uint32_t)(tot >> log2n) & 0xFFFFu;
        long long p = 0;
        for (int i = tid; i < n; i += blockDim.x) {
            const uint32_t x = (uint32_t)(uint16_t)ring[(head + i) & (n - 1)];
            const int16_t y = (int16_t)(uint16_t)((x - off16) & 0xFFFFu);
            buf[i] = y;
            p += (long long)y * y;
        }
        atomicAdd(&pw, (unsigned long long)p);
        __syncthreads();
        if (tid == 0)
            *power = (int64_t)pw;
    } else if (op == 1) {
        for (int i = tid; i < n; i += blockDim.x)
            buf[i] = (int16_t)(uint16_t)(((uint32_t)(uint16_t)buf[i] << 8) & 0xFFFFu);
    } else {
        for (int i = tid; i < n; i += blockDim.x) {
            const int32_t t = (int32_t)buf[i] * (int32_t)window[i];
            buf[i] = (int16_t)(uint16_t)((uint32_t)(t >> 15) & 0xFFFFu);
        }
    }
}


int hip_fail(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

}  // namespace

// Frames per workgroup and threads: F*items rounded to whole waves, chosen
// to waste the fewest lanes (cfg2: 144 items/frame -> F = 4, 576 threads).
static void direct_geometry(tdoa_kparams &kp, int &threads)
{
    const int items = kp.P * kp.T * kp.NSEG;
    int bestF = 1;
    double bestEff = -1.0;
    for (int F = 1; F <= 8; F++) {
        const int th = ((F * items + 63) / 64) * 64;
        if (th > 1024 && F > 1)
            break;
        kp.F = F;
        if (smem_bytes(kp, (th > 1024 ? 1024 : th) / 64) > 64 * 1024 && F > 1)
            break;
        const double eff = th > 1024 ? 1.0 : (double)(F * items) / th;
        if (eff > bestEff + 1e-9) {
            bestEff = eff;
            bestF = F;
        }
    }
    kp.F = bestF;
    threads = ((bestF * items + 63) / 64) * 64;
    if (threads > 1024)
        threads = 1024;
}

int tdoa_launch_direct(const tdoa_kparams &kp_in, const tdoa_kout &out, const int16_t *frames,
                       int64_t B, bool prepared, void *stream, int *lds_bytes_out,
                       const int32_t *count_dev)
{
    if (((uintptr_t)frames & 15) != 0)
        return tdoa_set_error(-1, "frames must be 16-byte aligned");
    tdoa_kparams kp = kp_in;
    int threads = 0;
    direct_geometry(kp, threads);
    const size_t lds = smem_bytes(kp, threads / 64);
    if (lds > 160 * 1024)
        return tdoa_set_error(-1, "DIRECT: shape needs more than 160 KiB LDS per workgroup");
    if (lds_bytes_out)
        *lds_bytes_out = (int)lds;
    const int64_t grid = (B + kp.F - 1) / kp.F;
    if (grid > INT_MAX)
        return tdoa_set_error(-1, "DIRECT: batch too large for one launch");
    hipStream_t st = (hipStream_t)stream;
#define TDOA_LAUNCH_DIRECT(PREP, TWC)                                                       \
    hipLaunchKernelGGL((k_direct<PREP, TWC>), dim3((unsigned)grid), dim3(threads), lds, st, kp, \
                       out, frames, B, count_dev)
    if (kp.TW == 1) {
        if (prepared)
            TDOA_LAUNCH_DIRECT(true, 1);
        else
            TDOA_LAUNCH_DIRECT(false, 1);
    } else {
        if (prepared)
            TDOA_LAUNCH_DIRECT(true, 7);
        else
            TDOA_LAUNCH_DIRECT(false, 7);
    }
#undef TDOA_LAUNCH_DIRECT
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_direct launch");
    return 0;
}

int tdoa_launch_average(const tdoa_kparams &kp, int64_t S, int64_t *est, const int64_t *fresh,
                        const float *decay, int32_t *best, const tdoa_kout *solve, void *stream)
{
    if (S > INT_MAX)
        return tdoa_set_error(-1, "average: too many streams for one launch");
    tdoa_kout o{};
    if (solve)
        o = *solve;
    const size_t lds = (size_t)kp.P * kp.K * 8 + 4 * 8 + 4 * 4;
    hipLaunchKernelGGL(k_average, dim3((unsigned)S), dim3(256), lds, (hipStream_t)stream, kp,
                       est, fresh, decay, best, o, solve ? 1 : 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_average launch");
    return 0;
}

int tdoa_launch_ref_buffer(int op, int16_t *buf, const int16_t *ring, int head, int64_t *power,
                           const int16_t *window, int n, void *stream)
{
    int log2n = 0;
    while ((1 << log2n) < n)
        log2n++;
    hipLaunchKernelGGL(k_ref_buffer, dim3(1), dim3(256), 0, (hipStream_t)stream, op, buf, ring,
                       head, power, window, n, log2n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return hip_fail(e, "k_ref_buffer launch");
    return 0;
}

#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch(unsigned long long *host, int n)
{
    if (n > (1 << 20))
        n = 1 << 20;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
