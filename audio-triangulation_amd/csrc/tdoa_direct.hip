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
#include <cstdlib>

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

// ------------------------------------------------ exact xcorr on the matrix cores
// k_direct_mfma: the same stage / argmax / prior / gate as k_direct, with the
// int64 cross-correlation (correlations.c:9-18) on v_mfma_i32_16x16x64_i8.
//   Offset byte limbs: every int16 x is stored as z = x ^ 0x0080, whose high
//   byte h = x >> 8 and low byte l = (x & 255) - 128 are int8 with
//   x' = x - 128 = 256 h + l.  a'.b' = 65536 ah.bh + 256 (ah.bl + al.bh)
//   + al.bl; each limb product accumulates exactly in int32 (<= 2 (N+64) 128^2).
//   Lag s = 16 (n - n0) + w is C[w][n] of a Toeplitz product summed over
//   NB 64-sample blocks beta:  A[w][k] = a[64 beta + k - w],  B[k][n] =
//   b[64 beta + k + 16 (n - n0)]  (every i = 64 beta + k - w once), over a
//   window of L = 64 NB indices that holds the whole a-row and b[16 (n - n0)..N).
//   Padding (x = 0) is z = 0x0080, so over the window
//   sum a b = sum a'b' + 128 (sum a + sum_window b) - 128^2 L  exactly.
// Lane l holds A row w = l & 15, B column n = l & 15, k = 16 (l >> 4) + j in
// byte j of its 16-byte operands (A and B pair byte for byte), and C rows
// 4 (l >> 4) + e of column l & 15.
constexpr int MF_PADW = 96;  // zero words each side of a staged row (b reads reach N + 175 samples)

typedef int v4i_mf __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i_mf mf_limbs(const uint32_t (&w)[8], uint32_t sel)
{
    v4i_mf r;
#pragma unroll
    for (int d = 0; d < 4; d++)
        r[d] = (int)__builtin_amdgcn_perm(w[2 * d + 1], w[2 * d], sel);
    return r;
}

template <bool PREPARED, int TWC>
__global__ void __launch_bounds__(1024) k_direct_mfma(tdoa_kparams kp, tdoa_kout out,
                                                      const int16_t *__restrict__ frames, int64_t B,
                                                      const int32_t *__restrict__ count, int n0, int nq,
                                                      int rsum_off)
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
    stage_frames<PREPARED>(kp, sm, frames, f0, nf);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const int RS = kp.RS, rows = nf * kp.M, words = rows * RS;
    // per row: sum of the row and of its first 16 / 32 / 48 samples (one wave a row)
    int *rsum = reinterpret_cast<int *>(smem + rsum_off);
    for (int row = wave; row < rows; row += nwaves) {
        const uint32_t *x = sm.X + row * RS + kp.PADW;
        const int v0 = sum_word(x[lane]);
        int t = v0;
        for (int i = lane + 64; i < kp.N / 2; i += 64)
            t += sum_word(x[i]);
        int p16 = lane < 8 ? v0 : 0, p32 = lane < 16 ? v0 : 0, p48 = lane < 24 ? v0 : 0;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            t += __shfl_xor(t, m, 64);
            p16 += __shfl_xor(p16, m, 64);
            p32 += __shfl_xor(p32, m, 64);
            p48 += __shfl_xor(p48, m, 64);
        }
        if (lane == 0) {
            rsum[4 * row + 0] = t;
            rsum[4 * row + 1] = p16;
            rsum[4 * row + 2] = p32;
            rsum[4 * row + 3] = p48;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += blockDim.x)
        sm.X[i] ^= 0x00800080u;
    __syncthreads();

    const int g = lane >> 4, r = lane & 15, rr = r < nq ? r : nq - 1;
    const int K = kp.K, S = kp.S, P = kp.P, NB = kp.N / 64 + 1;
    for (int it = wave; it < nf * P; it += nwaves) {
        const int f = it / P, p = it - f * P;
        const int rowa = f * kp.M + kp.pair_i[p], rowb = f * kp.M + kp.pair_j[p];
        const uint32_t *ra = sm.X + rowa * RS + kp.PADW;  // word of sample 0
        const uint32_t *rb = sm.X + rowb * RS + kp.PADW;
        v4i_mf hh = {0, 0, 0, 0}, xx = {0, 0, 0, 0}, ll = {0, 0, 0, 0};
        for (int beta = 0; beta < NB; beta++) {
            // A: samples q0 .. q0 + 15, q0 = 64 beta + 16 g - w (w = r; may be odd / negative)
            const int q0 = 64 * beta + 16 * g - r;
            const int wa = q0 >> 1;
            const uint32_t sh = (uint32_t)(q0 & 1) * 2u;
            uint32_t u[9], aw[8], bw[8];
#pragma unroll
            for (int m = 0; m < 9; m++)
                u[m] = ra[wa + m];
#pragma unroll
            for (int m = 0; m < 8; m++)
                aw[m] = __builtin_amdgcn_alignbyte(u[m + 1], u[m], sh);
            // B: samples 64 beta + 16 (g + n - n0) .. + 15 (even start)
            const int wb = 32 * beta + 8 * (g + rr - n0);
#pragma unroll
            for (int m = 0; m < 8; m++)
                bw[m] = rb[wb + m];
            const v4i_mf ah = mf_limbs(aw, 0x07050301u), al = mf_limbs(aw, 0x06040200u);
            const v4i_mf bh = mf_limbs(bw, 0x07050301u), bl = mf_limbs(bw, 0x06040200u);
            hh = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bh, hh, 0, 0, 0);
            xx = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bl, xx, 0, 0, 0);
            xx = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bh, xx, 0, 0, 0);
            ll = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bl, ll, 0, 0, 0);
        }
        if (r < nq) {
            // 128 (sum a + sum_window b) - 128^2 L; the b window starts at 16 (r - n0)
            const int d = r - n0;
            const int sb = rsum[4 * rowb] - (d > 0 ? rsum[4 * rowb + d] : 0);
            const int64_t corr = 128 * ((int64_t)rsum[4 * rowa] + sb) - (int64_t)16384 * 64 * NB;
            int64_t *dst = sm.scores + (size_t)(f * P + p) * K + S;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int sl = 16 * (r - n0) + 4 * g + e;
                if (sl >= -S && sl <= S)
                    dst[sl] = (int64_t)hh[e] * 65536 + (int64_t)xx[e] * 256 + (int64_t)ll[e] + corr;
            }
        }
    }
    __syncthreads();
    argmax_prior_phase<int64_t>(kp, sm.scores, sm.best, out, f0, nf);
    // grid solve (vga_heatmap.h:99-108) on the weighted scores still in LDS:
    // no [B][P][K] round trip through HBM and no second launch
    if (out.cell || out.xy || out.max_L)
        grid_phase_t<int64_t, 4, TWC>(kp, sm.scores, sm.redv, sm.redi, out, f0, nf);
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

static int direct_use_mfma()
{
    // matrix-core path (k_direct_mfma): TDOA_DIRECT_MFMA=0 keeps the VALU kernel (A/B)
    static const int v = [] {
        const char *s = getenv("TDOA_DIRECT_MFMA");
        return s ? atoi(s) : 1;
    }();
    return v;
}

// the matrix-core kernel (config 2..4 shapes) runs the grid solve itself
bool tdoa_direct_fused_grid(const tdoa_kparams &kp)
{
    return direct_use_mfma() && kp.N % 64 == 0 && kp.N >= 64 && kp.S <= 63;
}

int tdoa_launch_direct(const tdoa_kparams &kp_in, const tdoa_kout &out, const int16_t *frames,
                       int64_t B, bool prepared, void *stream, int *lds_bytes_out,
                       const int32_t *count_dev)
{
    if (((uintptr_t)frames & 15) != 0)
        return tdoa_set_error(-1, "frames must be 16-byte aligned");
    tdoa_kparams kp = kp_in;
    int threads = 0;
    if (tdoa_direct_fused_grid(kp)) {
        const int n0 = (kp.S + 15) / 16, nq = n0 + (kp.S + 1 + 15) / 16;  // lag columns -16 n0 .. 16 (nq - n0) - 1
        kp.PADW = MF_PADW;
        kp.RS = kp.N / 2 + 2 * MF_PADW;
        kp.F = kp.P >= 16 ? 1 : 16 / kp.P > 4 ? 4 : 16 / kp.P;  // frames per workgroup: one wave per (frame, pair) up to 16
        threads = 64 * (kp.F * kp.P < 16 ? kp.F * kp.P : 16);
        const size_t rsum_off = smem_bytes(kp, threads / 64);
        const size_t lds = rsum_off + (size_t)16 * kp.F * kp.M;
        if (lds > 160 * 1024)
            return tdoa_set_error(-1, "DIRECT: shape needs more than 160 KiB LDS per workgroup");
        if (lds_bytes_out)
            *lds_bytes_out = (int)lds;
        const int64_t grid = (B + kp.F - 1) / kp.F;
        if (grid > INT_MAX)
            return tdoa_set_error(-1, "DIRECT: batch too large for one launch");
        hipStream_t st = (hipStream_t)stream;
        constexpr int TWX = (TDOA_MAX_PAIRS + 3) / 4;
#define TDOA_LAUNCH_MF(PREP, TWC)                                                                 \
    hipLaunchKernelGGL((k_direct_mfma<PREP, TWC>), dim3((unsigned)grid), dim3(threads), lds, st, kp, \
                       out, frames, B, count_dev, n0, nq, (int)rsum_off)
        if (kp.TW == 1) {
            if (prepared)
                TDOA_LAUNCH_MF(true, 1);
            else
                TDOA_LAUNCH_MF(false, 1);
        } else {
            if (prepared)
                TDOA_LAUNCH_MF(true, TWX);
            else
                TDOA_LAUNCH_MF(false, TWX);
        }
#undef TDOA_LAUNCH_MF
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : hip_fail(e, "k_direct_mfma launch");
    }
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
