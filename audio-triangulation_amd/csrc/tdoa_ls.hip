// tdoa_ls.hip -- least-squares refinement of the grid argmax (north-star
// extension a15, absent in the reference; definition in oracle/tdoa_oracle.h):
// one thread per frame, double precision (MI355X FP64 vector is 1/2 the FP32
// rate and this is a few thousand flops per frame).
//   tau_p  = best_p + parabolic vertex of the raw scores around best_p
//   pred_p = (d_j - d_i) fs / c on the LUT's hemisphere geometry
//            (vga_heatmap.h:55-65), (u, v) in grid metres
//   10 Levenberg-Marquardt steps from the argmax cell, clamped to the grid.
// Built with -ffp-contract=off so it rounds like the C oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {

template <typename T>
__device__ __forceinline__ double ls_tau(const T *s, int K, int best)
{
    const int S = K / 2, kb = best + S;
    const bool inside = kb > 0 && kb < K - 1;
    return inside ? ls_tau3((double)s[kb - 1], (double)s[kb], (double)s[kb + 1], best, true)
                  : ls_tau3(0.0, 0.0, 0.0, best, false);
}

// MM: the mic count at compile time, so the per-frame arrays (P sub-sample
// lags, M distances and their derivatives) are registers, not scratch
template <typename T, int MM>
__global__ void __launch_bounds__(128) k_ls(tdoa_kparams kp, const T *__restrict__ scores,
                                            const float *__restrict__ peak3,
                                            const int32_t *__restrict__ lags,
                                            const int32_t *__restrict__ cells,
                                            float *__restrict__ xy_ls, float *__restrict__ rms_out,
                                            int64_t B, int iters)
{
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B)
        return;
    constexpr int M = MM, P = MM * (MM - 1) / 2;
    const int K = kp.K;
    double tau[P];
    if (peak3) {
        // the sub-sample lags from the peaks' scores: every lag and peak word
        // loaded before the first use (the branch inside the loop made each
        // pair's loads a round trip of their own)
        int best[P];
        float y[3 * P];
#pragma unroll
        for (int p = 0; p < P; p++)
            best[p] = lags[f * P + p];
#pragma unroll
        for (int e = 0; e < 3 * P; e++)
            y[e] = peak3[(size_t)f * P * 3 + e];
#pragma unroll
        for (int p = 0; p < P; p++) {
            const bool inside = best[p] + K / 2 > 0 && best[p] + K / 2 < K - 1;
            tau[p] = inside ? ls_tau3((double)y[3 * p], (double)y[3 * p + 1], (double)y[3 * p + 2], best[p], true)
                            : ls_tau3(0.0, 0.0, 0.0, best[p], false);
        }
    } else {
#pragma unroll
        for (int p = 0; p < P; p++)  // ... or from the raw scores
            tau[p] = ls_tau(scores + ((size_t)f * P + p) * K, K, lags[f * P + p]);
    }
    int cell = cells[f];
    cell = cell < 0 ? 0 : (cell >= kp.G ? kp.G - 1 : cell);
    const double sc = (double)kp.grid_scale;
    double u = (double)(cell % kp.grid_W - kp.half_w) / sc;
    double v = (double)(kp.half_h - cell / kp.grid_W) / sc;
    const double lu = (double)kp.half_w / sc, lv = (double)kp.half_h / sc;
    const double h = (double)kp.height, kf = (double)kp.fs / (double)kp.c;
    double ss = 0.0;
    for (int it = 0; it <= iters; it++) {
        const double n2 = u * u + v * v + h * h, n = sqrt(n2), n3 = n2 * n;
        const double k = h / n;
        const double px = k * u, py = k * v, pz = k * h;
        const double dxu = h * (1.0 / n - u * u / n3), dyu = h * (-v * u / n3),
                     dzu = h * (-h * u / n3);
        const double dxv = h * (-u * v / n3), dyv = h * (1.0 / n - v * v / n3),
                     dzv = h * (-h * v / n3);
        double d[M], du[M], dv[M];
#pragma unroll
        for (int m = 0; m < M; m++) {
            const double ex = px - (double)kp.mic_xy[2 * m], ey = py - (double)kp.mic_xy[2 * m + 1],
                         ez = pz;
            d[m] = sqrt(ex * ex + ey * ey + ez * ez);
            du[m] = (ex * dxu + ey * dyu + ez * dzu) / d[m];
            dv[m] = (ex * dxv + ey * dyv + ez * dzv) / d[m];
        }
        double a11 = 0.0, a12 = 0.0, a22 = 0.0, g1 = 0.0, g2 = 0.0;
        ss = 0.0;
        int p = 0;  // pairs (i, j), i < j, in the context's (lexicographic) order
#pragma unroll
        for (int i = 0; i < M; i++)
#pragma unroll
            for (int j = i + 1; j < M; j++, p++) {
                const double r = (d[j] - d[i]) * kf - tau[p];
                const double ju = (du[j] - du[i]) * kf, jv = (dv[j] - dv[i]) * kf;
                a11 += ju * ju;
                a12 += ju * jv;
                a22 += jv * jv;
                g1 += ju * r;
                g2 += jv * r;
                ss += r * r;
            }
        if (it == iters)
            break;
        const double lam = 1e-3 * (a11 + a22) + 1e-12;
        const double b11 = a11 + lam, b22 = a22 + lam;
        const double det = b11 * b22 - a12 * a12;
        u -= (b22 * g1 - a12 * g2) / det;
        v -= (b11 * g2 - a12 * g1) / det;
        u = u < -lu ? -lu : (u > lu ? lu : u);
        v = v < -lv ? -lv : (v > lv ? lv : v);
    }
    if (xy_ls) {
        xy_ls[2 * f] = (float)u;
        xy_ls[2 * f + 1] = (float)v;
    }
    if (rms_out)
        rms_out[f] = (float)sqrt(ss / (double)P);
}

}  // namespace

int tdoa_launch_ls(const tdoa_kparams &kp, const void *scores, bool is_float, const float *peak3,
                   const int32_t *lags, const int32_t *cells, float *xy_ls, float *rms,
                   int64_t B, void *stream)
{
    if (B <= 0)
        return 0;
    const int64_t grid = (B + 127) / 128;
    if (grid > 0x7fffffff)
        return tdoa_set_error(-1, "ls: batch too large for one launch");
    if (!peak3 && !scores)
        return tdoa_set_error(-1, "ls: neither peak scores nor raw scores");
    hipStream_t st = (hipStream_t)stream;
    const bool flt = is_float || peak3;
#define TDOA_LS_M(MM)                                                                                   \
    case MM:                                                                                            \
        if (flt)                                                                                        \
            hipLaunchKernelGGL((k_ls<float, MM>), dim3((unsigned)grid), dim3(128), 0, st, kp,          \
                               (const float *)scores, peak3, lags, cells, xy_ls, rms, B, TDOA_LS_ITERS); \
        else                                                                                            \
            hipLaunchKernelGGL((k_ls<int64_t, MM>), dim3((unsigned)grid), dim3(128), 0, st, kp,        \
                               (const int64_t *)scores, peak3, lags, cells, xy_ls, rms, B,              \
                               TDOA_LS_ITERS);                                                          \
        break
    switch (kp.M) {
        TDOA_LS_M(2);
        TDOA_LS_M(3);
        TDOA_LS_M(4);
        TDOA_LS_M(5);
        TDOA_LS_M(6);
        TDOA_LS_M(7);
        TDOA_LS_M(8);
    default:
        return tdoa_set_error(-1, "ls: num_mics outside 2..8");
    }
#undef TDOA_LS_M
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char buf[256];
        snprintf(buf, sizeof buf, "k_ls launch: %s", hipGetErrorString(e));
        return tdoa_set_error(-2, buf);
    }
    return 0;
}
