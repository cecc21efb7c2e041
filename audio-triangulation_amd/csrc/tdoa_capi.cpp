// tdoa_capi.cpp -- host side of libtdoa: configuration, one-time tables and
// the batched entry points declared in include/tdoa.h.
//
// The one-time tables reproduce the reference's float arithmetic exactly and
// are therefore built on the host (this file is compiled with
// -ffp-contract=off, no fast-math):
//   microphones_init      src/components/microphones.c:9-33
//   per-cell lag LUT      src/components/vga/vga_heatmap.h:48-93
//   Gaussian lag prior    src/components/correlations.c:26-33 (exp in libm)
//   DPSS(N, 2) Q15 window window.ipynb cells 2-4 (scipy dpss procedure)
// Everything per frame runs in the gfx950 kernels (tdoa_kernels.hip).

#include "../../include/tdoa.h"
#include "tdoa_internal.h"

#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess)                                                  \
            return fail(TDOA_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

int ilog2(int n)
{
    int b = 0;
    while ((1 << b) < n)
        b++;
    return b;
}

// ---------------------------------------------------------------- DPSS
// First Slepian taper of length n and time-bandwidth nw: the eigenvector of
// the largest eigenvalue of the symmetric tridiagonal matrix
//   diag_i = ((n-1-2i)/2)^2 cos(2 pi nw/n),  off_i = i(n-i)/2
// (Percival & Walden 1993, the system scipy.signal.windows.dpss solves).
// Largest eigenvalue by Sturm-count bisection, vector by inverse iteration
// with a partially pivoted tridiagonal LU.
int sturm_count_below(const std::vector<double> &d, const std::vector<double> &e2, double x)
{
    int cnt = 0;
    double q = d[0] - x;
    if (q < 0)
        cnt++;
    for (size_t i = 1; i < d.size(); i++) {
        if (q == 0.0)
            q = 1e-300;
        q = d[i] - x - e2[i] / q;
        if (q < 0)
            cnt++;
    }
    return cnt;
}

void tridiag_solve_pivoted(const std::vector<double> &d, const std::vector<double> &e,
                           double lam, std::vector<double> &b)
{
    // Solve (T - lam I) x = b in place; e[i] couples rows i-1 and i (e[0] unused).
    const int n = (int)d.size();
    std::vector<double> a(n), c(n), u2(n, 0.0), l(n, 0.0), dd(n);
    std::vector<int> piv(n, 0);
    // rows: sub a_i = e[i] (i>=1), diag dd_i = d_i - lam, super c_i = e[i+1]
    for (int i = 0; i < n; i++) {
        dd[i] = d[i] - lam;
        a[i] = i > 0 ? e[i] : 0.0;
        c[i] = i + 1 < n ? e[i + 1] : 0.0;
    }
    // Gaussian elimination with partial pivoting (LAPACK dgttrf style)
    for (int i = 0; i < n - 1; i++) {
        if (std::fabs(dd[i]) >= std::fabs(a[i + 1])) {
            double f = dd[i] != 0.0 ? a[i + 1] / dd[i] : 0.0;
            if (dd[i] == 0.0)
                dd[i] = 1e-300;
            l[i] = f;
            dd[i + 1] -= f * c[i];
            b[i + 1] -= f * b[i];
            u2[i] = 0.0;
            piv[i] = 0;
        } else {
            double f = dd[i] / a[i + 1];
            l[i] = f;
            // swap rows i and i+1
            double t_d = a[i + 1], t_c = dd[i + 1], t_u2 = i + 2 < n ? c[i + 1] : 0.0;
            double nd1 = c[i] - f * t_c;
            double nu2 = -f * t_u2;
            dd[i] = t_d;
            c[i] = t_c;
            u2[i] = t_u2;
            dd[i + 1] = nd1;
            if (i + 2 < n)
                c[i + 1] = nu2;
            double tb = b[i];
            b[i] = b[i + 1];
            b[i + 1] = tb - f * b[i];
            piv[i] = 1;
        }
    }
    if (dd[n - 1] == 0.0)
        dd[n - 1] = 1e-300;
    // back substitution
    b[n - 1] /= dd[n - 1];
    if (n > 1)
        b[n - 2] = (b[n - 2] - c[n - 2] * b[n - 1]) / dd[n - 2];
    for (int i = n - 3; i >= 0; i--)
        b[i] = (b[i] - c[i] * b[i + 1] - u2[i] * b[i + 2]) / dd[i];
}

}  // namespace

extern "C" int tdoa_dpss_q15(int32_t n, double nw, int32_t *out)
{
    if (n < 4 || !out || !(nw > 0))
        return fail(TDOA_ERR_INVALID, "tdoa_dpss_q15: bad arguments");
    const double W = nw / n, cw = std::cos(2.0 * M_PI * W);
    std::vector<double> d(n), e(n, 0.0), e2(n, 0.0);
    for (int i = 0; i < n; i++) {
        const double t = (n - 1 - 2.0 * i) / 2.0;
        d[i] = t * t * cw;
    }
    for (int i = 1; i < n; i++) {
        e[i] = i * (double)(n - i) / 2.0;
        e2[i] = e[i] * e[i];
    }
    // Gershgorin bounds
    double lo = 1e300, hi = -1e300;
    for (int i = 0; i < n; i++) {
        double r = std::fabs(e[i]) + (i + 1 < n ? std::fabs(e[i + 1]) : 0.0);
        lo = std::min(lo, d[i] - r);
        hi = std::max(hi, d[i] + r);
    }
    // largest eigenvalue: smallest x with count_below(x) == n
    for (int it = 0; it < 200; it++) {
        double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi)
            break;
        if (sturm_count_below(d, e2, mid) >= n)
            hi = mid;
        else
            lo = mid;
    }
    const double lam = 0.5 * (lo + hi);
    std::vector<double> v(n, 1.0);
    for (int it = 0; it < 4; it++) {
        tridiag_solve_pivoted(d, e, lam, v);
        double nrm = 0;
        for (double x : v)
            nrm += x * x;
        nrm = std::sqrt(nrm);
        for (double &x : v)
            x /= nrm;
    }
    double s = 0, mx = 0;
    for (double x : v)
        s += x;
    if (s < 0)
        for (double &x : v)
            x = -x;
    for (double x : v)
        mx = std::max(mx, std::fabs(x));
    for (int i = 0; i < n; i++)
        out[i] = (int32_t)std::nearbyint(v[i] / mx * 32767.0);
    return TDOA_OK;
}

// ------------------------------------------------------------ context
struct tdoa_ctx {
    tdoa_config cfg;
    int device;
    int M, N, P, K, S, G, W, H, U, TW;
    std::vector<float> mic;     // [M][2]
    std::vector<int32_t> win;   // [N]
    std::vector<float> prior;   // [K]
    std::vector<uint8_t> lut;   // [P][G]
    std::vector<uint32_t> tuples;
    std::vector<int32_t> tuple_cell;
    // device
    int16_t *d_window = nullptr;
    float *d_prior = nullptr;
    uint32_t *d_tuples = nullptr;
    int32_t *d_tuple_cell = nullptr;
    float *d_tw = nullptr;  // GCC_PHAT twiddles: [N] e^{-2 pi i k/N}, then [N+1] e^{-2 pi i k/2N}
    void *d_p1k_img = nullptr;  // LDS table image of the config-2 GCC_PHAT kernel
    void *d_w64_img = nullptr;  // ... and of its one-frame-per-wave form
    // weighted-score scratch for the grid kernel when the caller did not ask
    // for weighted scores ([B][P][K] int64 or float); grows on demand
    void *d_wscratch = nullptr;
    size_t wscratch_bytes = 0;
    // raw-score and cell scratch for the least-squares refinement
    void *d_rscratch = nullptr;
    size_t rscratch_bytes = 0;
    void *d_cscratch = nullptr;
    size_t cscratch_bytes = 0;
    void *d_tscratch = nullptr;  // [B][P][3] float peak scores (least squares)
    size_t tscratch_bytes = 0;
    std::vector<uint8_t> bb_img;  // k_grid_bb tables: tiles | ranges | tuples | uidx | queries
    std::vector<uint16_t> bb_rng; // [NT][P] lo | hi << 8 (host copy)
    void *d_fgq = nullptr;        // kp.fg_q
    int bb_wide = 0;              // a range wider than the queries encode: no k_grid_bb
    void *d_bb = nullptr;
    void *d_wc = nullptr;         // compact weighted-score chunk table (kp.wc_chunks)
    std::vector<uint32_t> wc_chunks;
    int bb_NT = 0;
    float *d_mic = nullptr;  // [M][2]
    uint8_t *d_lut = nullptr;  // [P][G]
    // GCC_PHAT spectrum scratch for the two-pass shapes (M > 3 or N > 2048):
    // a fixed chunk of frames' spectra that stays in L2 / MALL between passes
    void *d_spec = nullptr;
    size_t spec_bytes = 0;
    tdoa_kparams kp;
};

namespace {

// microphones.c:9-33 (constants.h:17-19: AB .132, BC .15, CA .20; MIRROR on)
void reference_triangle(float *xy)
{
    const float dAB = 0.132f, dBC = 0.15f, dCA = 0.20f;
    const float xC = (dAB * dAB + dCA * dCA - dBC * dBC) / (2.0f * dAB);
    const float yC = sqrtf(fmaxf(0.0f, dCA * dCA - xC * xC));
    const float pAx = 0.0f, pAy = 0.0f, pBx = dAB, pBy = 0.0f;
    const float pCx = xC, pCy = yC * -1.0f;
    const float cx = (pAx + pBx + pCx) / 3.0f;
    const float cy = (pAy + pBy + pCy) / 3.0f;
    xy[0] = pAx - cx;
    xy[1] = pAy - cy;
    xy[2] = pBx - cx;
    xy[3] = pBy - cy;
    xy[4] = pCx - cx;
    xy[5] = pCy - cy;
}

inline float hypot3(float x, float y, float z) { return sqrtf(x * x + y * y + z * z); }

void build_bb_tiles(tdoa_ctx *c);

// vga_heatmap.h:48-93, generalised to lexicographic pairs of M mics.
void build_lut(tdoa_ctx *c)
{
    const int W = c->W, H = c->H, G = c->G;
    const float scale = c->cfg.grid_scale, hgt = c->cfg.height_offset;
    const float sos = c->cfg.speed_of_sound;
    const int fs = c->cfg.sample_rate_hz;
    c->lut.assign((size_t)c->P * G, 0);
    std::vector<float> d(c->M);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float xm = (float)(x - c->cfg.grid_half_w) / scale;
            float ym = (float)(c->cfg.grid_half_h - y) / scale;
            float zm = hgt;
            const float k = hgt / hypot3(zm, xm, ym);
            xm *= k;
            ym *= k;
            zm *= k;
            for (int m = 0; m < c->M; m++)
                d[m] = hypot3(zm, xm - c->mic[2 * m], ym - c->mic[2 * m + 1]);
            int p = 0;
            for (int i = 0; i < c->M; i++)
                for (int j = i + 1; j < c->M; j++, p++) {
                    const float dt = (d[j] - d[i]) / sos;
                    int s = (int)roundf(dt * (float)fs);
                    s = std::min(std::max(s, -c->S), c->S);
                    c->lut[(size_t)p * G + (size_t)y * W + x] = (uint8_t)(s + c->S);
                }
        }
    // Distinct lag tuples in order of their first (row-major) cell: the max
    // over cells equals the max over tuples, and the first argmax tuple
    // carries the first argmax cell (tuple first-cells are increasing).
    std::map<std::vector<uint8_t>, int> seen;
    c->tuples.clear();
    c->tuple_cell.clear();
    std::vector<uint8_t> key(c->P);
    for (int cell = 0; cell < G; cell++) {
        for (int p = 0; p < c->P; p++)
            key[p] = c->lut[(size_t)p * G + cell];
        if (seen.emplace(key, (int)c->tuple_cell.size()).second) {
            c->tuple_cell.push_back(cell);
            for (int w = 0; w < c->TW; w++) {
                uint32_t v = 0;
                for (int b = 0; b < 4; b++) {
                    int p = 4 * w + b;
                    if (p < c->P)
                        v |= (uint32_t)key[p] << (8 * b);
                }
                c->tuples.push_back(v);
            }
        }
    }
    c->U = (int)c->tuple_cell.size();
    build_bb_tiles(c);
}

// An entry's range [lo, hi] of pair p as k_grid_bb's sparse-table query
// (tdoa_grid_bb.h): the LDS element offset o1 of the level-j window
// max w[lo .. lo + 2^j - 1] (2^j <= n = hi - lo + 1 < 2^(j+1)) from the wave's
// scores, and the distance d = n - 2^j of the second window, as o1 | d << 13;
// ranges wider than 15 are marked wide (o1 = 0x1FFF: the kernel loops)
uint16_t bb_query(int P, int K, int p, int lo, int hi)
{
    const int n = hi - lo + 1;
    if (n > 15)
        return 0x1FFF;  // wide: the table is not used (kp.bb_wide)
    // The query's two windows [lo, lo + 2^lv) and [hi + 1 - 2^lv, hi + 1) lie
    // inside [lo, hi] (2^lv <= n), and k_grid_bb's level build reads lags past
    // K - 1 (unclamped 16-B reads, tdoa_grid_bb.h): those level elements are
    // never queried only while every range stays inside the lag range.  A
    // range that does not is encoded wide (the exhaustive k_grid runs instead).
    if (lo < 0 || hi >= K || n < 1)
        return 0x1FFF;
    const int lv = n >= 8 ? 3 : (n >= 4 ? 2 : (n >= 2 ? 1 : 0));
    const int KS = P > 8 ? (K + 3) & ~3 : K;  // bb_ks (tdoa_grid_bb.h): score row stride
    const int PKp = (P * KS + 3) & ~3, RW = K <= 96 ? 96 : 128;
    int o1;
    if (lv == 0)
        o1 = p * KS + lo;  // the scores themselves
    else if (P <= 8)
        o1 = lv * PKp + p * K + lo;  // levels [3][P][K] after the scores
    else
        o1 = PKp + (lv - 1) * 4 * RW + (p & 3) * RW + lo;  // [3][4][RW]: four pairs a group
    if (o1 < 0 || o1 >= 0x1FFF)
        return 0x1FFF;  // the offset does not fit 13 bits: wide (exhaustive k_grid)
    return (uint16_t)(o1 | ((n - (1 << lv)) << 13));
}

// Tables of the exact branch-and-bound grid solve (k_grid_bb, tdoa_grid.hip):
// the distinct tuples regrouped by the TILE x TILE block of grid cells their
// first cell lies in (entries of at most 64 tuples, one per lane), and for
// every entry and pair the range of lag indices its tuples use.  The bound of
// an entry is the sum over pairs of the weighted-score maximum over that range.
void build_bb_tiles(tdoa_ctx *c)
{
    constexpr int TILE = 8, CAP = 64;
    const int P = c->P, TW = c->TW, U = c->U;
    const int tx = (c->W + TILE - 1) / TILE, ty = (c->H + TILE - 1) / TILE;
    std::vector<std::vector<int>> members((size_t)tx * ty);
    for (int u = 0; u < U; u++) {
        const int cell = c->tuple_cell[u];
        const int x = cell % c->W, y = cell / c->W;
        members[(size_t)(y / TILE) * tx + x / TILE].push_back(u);
    }
    std::vector<int32_t> tile;
    std::vector<uint16_t> rng, qry;
    std::vector<uint32_t> tup;
    std::vector<int32_t> uidx;
    for (const auto &m : members)
        for (size_t c0 = 0; c0 < m.size(); c0 += CAP) {
            const size_t n = std::min(m.size() - c0, (size_t)CAP);
            tile.push_back((int32_t)uidx.size());
            tile.push_back((int32_t)n);
            std::vector<int> lo(P, 255), hi(P, 0);
            for (size_t i = 0; i < n; i++) {
                const int u = m[c0 + i];
                uidx.push_back(u);
                for (int w = 0; w < TW; w++)
                    tup.push_back(c->tuples[(size_t)u * TW + w]);
                for (int p = 0; p < P; p++) {
                    const int l = (c->tuples[(size_t)u * TW + p / 4] >> (8 * (p & 3))) & 0xFF;
                    lo[p] = std::min(lo[p], l);
                    hi[p] = std::max(hi[p], l);
                }
            }
            for (int p = 0; p < P; p++) {
                rng.push_back((uint16_t)(lo[p] | (hi[p] << 8)));
                qry.push_back(bb_query(P, c->K, p, lo[p], hi[p]));
            }
        }
    const int NT = (int)tile.size() / 2;
    c->bb_NT = NT;
    c->bb_rng = rng;
    c->bb_wide = 0;
    for (const uint16_t q : qry)
        c->bb_wide |= (q & 0x1FFF) == 0x1FFF;
    auto put = [&](const void *src, size_t bytes) {
        const size_t at = c->bb_img.size();
        c->bb_img.resize(at + ((bytes + 15) & ~(size_t)15), 0);
        memcpy(c->bb_img.data() + at, src, bytes);
        return at;
    };
    c->bb_img.clear();
    put(tile.data(), tile.size() * 4);
    put(rng.data(), rng.size() * 2);
    put(tup.data(), tup.size() * 4);
    put(uidx.data(), uidx.size() * 4);
    put(qry.data(), qry.size() * 2);
}

void free_device(tdoa_ctx *c)
{
    (void)hipFree(c->d_window);
    (void)hipFree(c->d_prior);
    (void)hipFree(c->d_tuples);
    (void)hipFree(c->d_tuple_cell);
    (void)hipFree(c->d_bb);
    (void)hipFree(c->d_wc);
    c->d_wc = nullptr;
    (void)hipFree(c->d_fgq);
    c->d_fgq = nullptr;
    (void)hipFree(c->d_tw);
    (void)hipFree(c->d_p1k_img);
    c->d_p1k_img = nullptr;
    (void)hipFree(c->d_w64_img);
    c->d_w64_img = nullptr;
    (void)hipFree(c->d_wscratch);
    (void)hipFree(c->d_rscratch);
    (void)hipFree(c->d_cscratch);
    (void)hipFree(c->d_tscratch);
    (void)hipFree(c->d_mic);
    (void)hipFree(c->d_lut);
    c->d_lut = nullptr;
    c->d_rscratch = c->d_cscratch = nullptr;
    c->rscratch_bytes = c->cscratch_bytes = 0;
    c->d_tscratch = nullptr;
    c->tscratch_bytes = 0;
    c->d_mic = nullptr;
    (void)hipFree(c->d_spec);
    c->d_spec = nullptr;
    c->spec_bytes = 0;
    c->d_wscratch = nullptr;
    c->wscratch_bytes = 0;
    c->d_tw = nullptr;
    c->d_window = nullptr;
    c->d_prior = nullptr;
    c->d_tuples = nullptr;
    c->d_tuple_cell = nullptr;
}

}  // namespace

extern "C" int tdoa_config_default(tdoa_config *cfg)
{
    if (!cfg)
        return fail(TDOA_ERR_INVALID, "tdoa_config_default: NULL");
    std::memset(cfg, 0, sizeof *cfg);
    cfg->num_mics = 3;
    cfg->frame_len = 1024;
    cfg->sample_rate_hz = 50000;
    cfg->max_shift = 0;
    cfg->speed_of_sound = 343.0f;
    cfg->engine = TDOA_ENGINE_DIRECT;
    cfg->mic_xy = nullptr;
    cfg->grid_half_w = 50;
    cfg->grid_half_h = 50;
    cfg->grid_scale = 24.0f;
    cfg->height_offset = 1.2f;
    cfg->window_q15 = nullptr;
    cfg->phat_eps = 1e-12f;
    return TDOA_OK;
}

extern "C" int tdoa_create(const tdoa_config *cfg, int device, tdoa_ctx **out)
{
    if (!cfg || !out)
        return fail(TDOA_ERR_INVALID, "tdoa_create: NULL argument");
    *out = nullptr;
    const int M = cfg->num_mics, N = cfg->frame_len;
    if (M < 2 || M > TDOA_MAX_MICS)
        return fail(TDOA_ERR_INVALID, "num_mics %d outside [2,%d]", M, TDOA_MAX_MICS);
    if (N < 256 || N > 4096 || (N & (N - 1)))
        return fail(TDOA_ERR_INVALID, "frame_len %d must be a power of two in [256,4096]", N);
    if (cfg->sample_rate_hz <= 0 || !(cfg->speed_of_sound > 0))
        return fail(TDOA_ERR_INVALID, "sample_rate_hz / speed_of_sound must be positive");
    // constants.h:12 -- SAMPLE_RATE_HZ * 32 / 34300 (integer division)
    const int S = cfg->max_shift > 0 ? cfg->max_shift
                                     : (int)((int64_t)cfg->sample_rate_hz * 32 / 34300);
    if (S < 1 || S > 63)
        return fail(TDOA_ERR_INVALID, "max_shift %d outside [1,63]", S);
    if (cfg->engine != TDOA_ENGINE_DIRECT && cfg->engine != TDOA_ENGINE_GCC_PHAT)
        return fail(TDOA_ERR_INVALID, "unknown engine %d", cfg->engine);
    if (cfg->grid_half_w < 0 || cfg->grid_half_h < 0 || cfg->grid_half_w > 1000 ||
        cfg->grid_half_h > 1000 || !(cfg->grid_scale > 0) || !(cfg->height_offset > 0))
        return fail(TDOA_ERR_INVALID, "bad grid geometry");
    if (M != 3 && !cfg->mic_xy)
        return fail(TDOA_ERR_INVALID, "mic_xy is required unless num_mics == 3");

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(TDOA_ERR_NO_DEVICE, "no HIP device visible (libtdoa has no CPU path)");
    if (device < 0 || device >= ndev)
        return fail(TDOA_ERR_INVALID, "device %d out of range (%d visible)", device, ndev);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(TDOA_ERR_NO_DEVICE, "device %d is %s; libtdoa is built for gfx950 only",
                    device, prop.gcnArchName);

    tdoa_ctx *c = new tdoa_ctx();
    c->cfg = *cfg;
    c->cfg.mic_xy = nullptr;
    c->cfg.window_q15 = nullptr;
    c->cfg.max_shift = S;
    c->device = device;
    c->M = M;
    c->N = N;
    c->P = M * (M - 1) / 2;
    c->S = S;
    c->K = 2 * S + 1;
    c->W = 2 * cfg->grid_half_w + 1;
    c->H = 2 * cfg->grid_half_h + 1;
    c->G = c->W * c->H;
    c->TW = (c->P + 3) / 4;

    c->mic.resize(2 * M);
    if (cfg->mic_xy)
        std::memcpy(c->mic.data(), cfg->mic_xy, sizeof(float) * 2 * M);
    else
        reference_triangle(c->mic.data());

    c->win.resize(N);
    if (cfg->window_q15) {
        for (int i = 0; i < N; i++) {
            if (cfg->window_q15[i] < 0 || cfg->window_q15[i] > 32767) {
                delete c;
                return fail(TDOA_ERR_INVALID, "window_q15[%d] outside [0,32767]", i);
            }
            c->win[i] = cfg->window_q15[i];
        }
    } else if (N < 1024 && 1024 % N == 0) {
        // buffer.c:8 indexes WINDOW_FUNCTION[i << (10 - BUFFER_SIZE_BITS)]: a
        // shorter frame subsamples the 1024-point Q15 table
        std::vector<int32_t> w1k(1024);
        int rc = tdoa_dpss_q15(1024, 2.0, w1k.data());
        if (rc) {
            delete c;
            return rc;
        }
        for (int i = 0; i < N; i++)
            c->win[i] = w1k[(size_t)i * (1024 / N)];
    } else {
        // N > 1024 (where buffer.c:8 is undefined): DPSS(N, NW=2) by the
        // window.ipynb procedure
        int rc = tdoa_dpss_q15(N, 2.0, c->win.data());
        if (rc) {
            delete c;
            return rc;
        }
    }

    // correlations.c:27-30: scale = (float)exp((double)((float)(-d^2) / 36.f))
    c->prior.resize(c->K);
    for (int d = 0; d < c->K; d++) {
        const float arg = (float)(-(d * d)) / 36.f;
        c->prior[d] = (float)std::exp((double)arg);
    }

    build_lut(c);

    // kernel parameters
    tdoa_kparams &kp = c->kp;
    std::memset(&kp, 0, sizeof kp);
    kp.M = M;
    kp.N = N;
    kp.log2N = ilog2(N);
    kp.P = c->P;
    kp.K = c->K;
    kp.S = S;
    kp.G = c->G;
    kp.U = c->U;
    kp.grid_W = c->W;
    kp.half_w = cfg->grid_half_w;
    kp.half_h = cfg->grid_half_h;
    kp.grid_scale = cfg->grid_scale;
    kp.sbase = (S % 2 == 0) ? -S : -S - 1;
    kp.T = (S - kp.sbase + 1 + TDOA_LT - 1) / TDOA_LT;
    kp.NSEG = (N / 2) / TDOA_SEGW;
    // rows are read at word offsets [h, h + SEGW*NSEG + LT2 + 1) with
    // h in [sbase/2, sbase/2 + LT2*(T-1)]
    const int need_left = -kp.sbase / 2;
    const int need_right = kp.sbase / 2 + TDOA_LT2 * (kp.T - 1) + TDOA_LT2 + 2;
    kp.PADW = ((std::max(need_left, need_right) + 3) / 4) * 4;
    kp.RS = N / 2 + 2 * kp.PADW;
    kp.TW = c->TW;
    {
        int p = 0;
        for (int i = 0; i < M; i++)
            for (int j = i + 1; j < M; j++, p++) {
                kp.pair_i[p] = (uint8_t)i;
                kp.pair_j[p] = (uint8_t)j;
            }
    }

    // upload
    HIP_TRY(hipSetDevice(device));
    std::vector<int16_t> w16(N);
    for (int i = 0; i < N; i++)
        w16[i] = (int16_t)c->win[i];
    if (hipMalloc(&c->d_window, sizeof(int16_t) * N) != hipSuccess ||
        hipMalloc(&c->d_prior, sizeof(float) * c->K) != hipSuccess ||
        hipMalloc(&c->d_tuples, sizeof(uint32_t) * c->tuples.size()) != hipSuccess ||
        hipMalloc(&c->d_tuple_cell, sizeof(int32_t) * c->U) != hipSuccess ||
        hipMalloc(&c->d_mic, sizeof(float) * 2 * M) != hipSuccess ||
        hipMalloc(&c->d_lut, c->lut.size()) != hipSuccess) {
        free_device(c);
        delete c;
        return fail(TDOA_ERR_NOMEM, "hipMalloc of context tables failed");
    }
    hipError_t e = hipMemcpy(c->d_window, w16.data(), sizeof(int16_t) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(c->d_mic, c->mic.data(), sizeof(float) * 2 * M, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(c->d_lut, c->lut.data(), c->lut.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(c->d_prior, c->prior.data(), sizeof(float) * c->K, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(c->d_tuples, c->tuples.data(), sizeof(uint32_t) * c->tuples.size(),
                      hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(c->d_tuple_cell, c->tuple_cell.data(), sizeof(int32_t) * c->U,
                      hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        free_device(c);
        delete c;
        return fail(TDOA_ERR_HIP, "uploading context tables: %s", hipGetErrorString(e));
    }
    {
        // GCC_PHAT twiddles, in double then rounded once
        std::vector<float> tw(2 * N + 2 * (N + 1) + 2 * 3 * 256);
        for (int k = 0; k < N; k++) {
            const double a = -2.0 * M_PI * k / N;
            tw[2 * k] = (float)std::cos(a);
            tw[2 * k + 1] = (float)std::sin(a);
        }
        for (int k = 0; k <= N; k++) {
            const double a = -2.0 * M_PI * k / (2.0 * N);
            tw[2 * N + 2 * k] = (float)std::cos(a);
            tw[2 * N + 2 * k + 1] = (float)std::sin(a);
        }
        // coalesced twiddle tables of the long-frame kernels (tdoa_phat_r16.hip):
        // [r][k] W_N^{(N/256) r k}; [r][l] W_N^{r l}; [r][h] W_N^{16 r h}  (r, k, l, h < 16)
        {
            float *t = tw.data() + 2 * N + 2 * (N + 1);
            const int R1 = N >= 256 ? N / 256 : 1;
            const int mul[3] = {R1, 1, 16};
            for (int s = 0; s < 3; s++)
                for (int r = 0; r < 16; r++)
                    for (int k = 0; k < 16; k++) {
                        const long e = ((long)mul[s] * r * k) % N;
                        const double a = -2.0 * M_PI * (double)e / N;
                        t[2 * (256 * s + 16 * r + k)] = (float)std::cos(a);
                        t[2 * (256 * s + 16 * r + k) + 1] = (float)std::sin(a);
                    }
        }
        if (hipMalloc(&c->d_tw, sizeof(float) * tw.size()) != hipSuccess ||
            hipMemcpy(c->d_tw, tw.data(), sizeof(float) * tw.size(), hipMemcpyHostToDevice) !=
                hipSuccess) {
            free_device(c);
            delete c;
            return fail(TDOA_ERR_NOMEM, "uploading twiddle tables failed");
        }
        kp.tw = c->d_tw;
        kp.tw2 = c->d_tw + 2 * N;
        kp.r16_tw = c->d_tw + 2 * N + 2 * (N + 1);
        std::vector<uint8_t> img;
        tdoa_phat1024_image(M, N, c->K, c->U, tw.data(), c->win.data(), c->prior.data(),
                            c->tuples.data(), c->tuple_cell.data(), img);
        if (!img.empty()) {
            if (hipMalloc(&c->d_p1k_img, img.size()) != hipSuccess ||
                hipMemcpy(c->d_p1k_img, img.data(), img.size(), hipMemcpyHostToDevice) !=
                    hipSuccess) {
                free_device(c);
                delete c;
                return fail(TDOA_ERR_NOMEM, "uploading the GCC_PHAT table image failed");
            }
            kp.p1k_img = c->d_p1k_img;
            kp.p1k_img_bytes = (int32_t)img.size();
        }
#if TDOA_AB
        // the one-frame-per-wave A/B kernel's image (tdoa/libtdoa_ab.so only)
        tdoa_p1k_w64_image(M, N, c->K, c->U, c->win.data(), c->prior.data(), c->tuples.data(), img);
        if (!img.empty()) {
            if (hipMalloc(&c->d_w64_img, img.size()) != hipSuccess ||
                hipMemcpy(c->d_w64_img, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess) {
                free_device(c);
                delete c;
                return fail(TDOA_ERR_NOMEM, "uploading the GCC_PHAT (w64) table image failed");
            }
            kp.w64_img = c->d_w64_img;
            kp.w64_img_bytes = (int32_t)img.size();
        }
#endif
        if (tdoa_gcc_phat_needs_split(M, N)) {
            const size_t want = (size_t)128 << 20;
            if (hipMalloc(&c->d_spec, want) != hipSuccess) {
                free_device(c);
                delete c;
                return fail(TDOA_ERR_NOMEM, "GCC_PHAT spectrum scratch of %zu bytes", want);
            }
            c->spec_bytes = want;
        }
    }
    kp.window = c->d_window;
    kp.prior = c->d_prior;
    kp.mic_xy = c->d_mic;
    kp.lut = c->d_lut;
    kp.fs = (float)cfg->sample_rate_hz;
    kp.c = cfg->speed_of_sound;
    kp.height = cfg->height_offset;
    kp.tuples = c->d_tuples;
    kp.tuple_cell = c->d_tuple_cell;
    kp.bb_NT = c->bb_NT;
    kp.bb_wide = c->bb_wide;
    if (kp.bb_NT > 0) {
        if (hipMalloc(&c->d_bb, c->bb_img.size()) != hipSuccess ||
            hipMemcpy(c->d_bb, c->bb_img.data(), c->bb_img.size(), hipMemcpyHostToDevice) !=
                hipSuccess) {
            free_device(c);
            delete c;
            return fail(TDOA_ERR_NOMEM, "uploading the grid tile tables failed");
        }
        const char *b = (const char *)c->d_bb;
        const size_t a1 = ((size_t)kp.bb_NT * 8 + 15) & ~(size_t)15;
        const size_t a2 = a1 + ((((size_t)kp.bb_NT * c->P * 2) + 15) & ~(size_t)15);
        const size_t a3 = a2 + ((((size_t)c->U * c->TW * 4) + 15) & ~(size_t)15);
        kp.bb_tile = (const int32_t *)b;
        kp.bb_rng = (const uint16_t *)(b + a1);
        kp.bb_tuples = (const uint32_t *)(b + a2);
        kp.bb_uidx = (const int32_t *)(b + a3);
        kp.bb_q = (const uint16_t *)(b + a3 + ((((size_t)c->U * 4) + 15) & ~(size_t)15));
        // compact weighted-score layout: per pair the lag range the tuples use
        // (vga_heatmap.h:68-93: the LUT clamps lags to it), padded to 4 floats
        std::vector<int> lo(c->P, 255), hi(c->P, -1);
        for (int u = 0; u < c->U; u++)
            for (int p = 0; p < c->P; p++) {
                const int l = (c->tuples[(size_t)u * c->TW + p / 4] >> (8 * (p & 3))) & 0xFF;
                lo[p] = std::min(lo[p], l);
                hi[p] = std::max(hi[p], l);
            }
        int off = 0;
        bool ok = c->P <= TDOA_MAX_PAIRS;
        c->wc_chunks.clear();
        // many pairs (P > 8): k_grid_bb's score rows are KS = bb_ks apart and a
        // range starts at a multiple of 4 lags, so every chunk lands 16-B aligned
        const int KS = c->P > 8 ? (c->K + 3) & ~3 : c->K;
        for (int p = 0; ok && p < c->P; p++) {
            if (c->P > 8 && hi[p] >= lo[p])
                lo[p] &= ~3;
            const int w = hi[p] - lo[p] + 1;
            ok = w > 0 && off < 65536;
            if (!ok)
                break;
            kp.wc_lo[p] = (uint8_t)lo[p];
            kp.wc_w[p] = (uint8_t)w;
            kp.wc_off[p] = (uint16_t)off;
            for (int j = 0; j < w; j += 4)
                c->wc_chunks.push_back((uint32_t)(p * KS + lo[p] + j) | ((uint32_t)std::min(4, w - j) << 16));
            off += (w + 3) & ~3;
        }
        if (ok && hipMalloc(&c->d_wc, c->wc_chunks.size() * 4) == hipSuccess &&
            hipMemcpy(c->d_wc, c->wc_chunks.data(), c->wc_chunks.size() * 4, hipMemcpyHostToDevice) ==
                hipSuccess) {
            kp.wc_CK = off;
            kp.wc_nch = (int32_t)c->wc_chunks.size();
            kp.wc_chunks = (const uint32_t *)c->d_wc;
#if TDOA_AB
            // the fused k_frame16 grid's queries (tdoa_internal.h, kp.fg_q): an
            // A/B path, built only into tdoa/libtdoa_ab.so (every
            // context paid O(U P) host work and a device table for it)
            std::vector<uint16_t> fq((size_t)kp.bb_NT * 32, 0);
            bool fok = off <= 2048 && kp.bb_NT <= 256 && c->P <= 32;
            for (int t = 0; fok && t < kp.bb_NT; t++)
                for (int p = 0; p < c->P; p++) {
                    const int lo = c->bb_rng[(size_t)t * c->P + p] & 0xFF, hi = c->bb_rng[(size_t)t * c->P + p] >> 8;
                    const int n = hi - lo + 1;
                    if (n < 1 || n > 15 || lo < kp.wc_lo[p] || hi >= kp.wc_lo[p] + kp.wc_w[p]) {
                        fok = false;
                        break;
                    }
                    const int lv = n >= 8 ? 3 : (n >= 4 ? 2 : (n >= 2 ? 1 : 0));
                    const int e = kp.wc_off[p] + lo - kp.wc_lo[p];
                    fq[(size_t)t * 32 + p] = (uint16_t)(e | (lv << 11) | ((n - (1 << lv)) << 13));
                }
            // ... and the regrouped tuples (bb order) as compact element indices,
            // so a tuple's gathers need no per-pair offsets: [U][32] u16
            const size_t qbytes = fq.size() * 2;
            if (fok) {
                const uint32_t *bt = (const uint32_t *)(c->bb_img.data() + (((size_t)kp.bb_NT * 8 + 15) & ~(size_t)15) +
                                                        ((((size_t)kp.bb_NT * c->P * 2) + 15) & ~(size_t)15));
                for (int u = 0; u < c->U; u++)
                    for (int p = 0; p < c->P; p++) {
                        const int lag = (bt[(size_t)u * c->TW + p / 4] >> (8 * (p & 3))) & 0xFF;
                        fq.push_back((uint16_t)(kp.wc_off[p] + lag - kp.wc_lo[p]));
                    }
                fq.resize((size_t)kp.bb_NT * 32 + (size_t)c->U * 32, 0);
                // (rows of 32: the pushes above are P per tuple; re-lay them out)
                std::vector<uint16_t> tup((size_t)c->U * 32, 0);
                for (int u = 0; u < c->U; u++)
                    for (int p = 0; p < c->P; p++)
                        tup[(size_t)u * 32 + p] = fq[(size_t)kp.bb_NT * 32 + (size_t)u * c->P + p];
                std::copy(tup.begin(), tup.end(), fq.begin() + (size_t)kp.bb_NT * 32);
            }
            if (fok && hipMalloc(&c->d_fgq, fq.size() * 2) == hipSuccess &&
                hipMemcpy(c->d_fgq, fq.data(), fq.size() * 2, hipMemcpyHostToDevice) == hipSuccess) {
                kp.fg_q = (const uint16_t *)c->d_fgq;
                kp.fg_tup = (const uint16_t *)((const char *)c->d_fgq + qbytes);
                kp.fg_ok = 1;
            }
#endif
        }
    }
    *out = c;
    return TDOA_OK;
}

extern "C" int tdoa_destroy(tdoa_ctx *ctx)
{
    if (!ctx)
        return TDOA_OK;
    (void)hipSetDevice(ctx->device);
    free_device(ctx);
    delete ctx;
    return TDOA_OK;
}

extern "C" int tdoa_get_dims(const tdoa_ctx *c, int32_t *M, int32_t *N, int32_t *P,
                             int32_t *K, int32_t *G)
{
    if (!c)
        return fail(TDOA_ERR_INVALID, "tdoa_get_dims: NULL ctx");
    if (M)
        *M = c->M;
    if (N)
        *N = c->N;
    if (P)
        *P = c->P;
    if (K)
        *K = c->K;
    if (G)
        *G = c->G;
    return TDOA_OK;
}

static tdoa_kout to_kout(const tdoa_outputs *o)
{
    tdoa_kout k{};
    k.lags = o->lags;
    k.gate = o->gate;
    k.cell = o->cell;
    k.xy = o->xy;
    k.max_L = o->max_L;
    k.max_Lf = o->max_Lf;
    k.scores = o->scores;
    k.weighted = o->weighted;
    k.scores_f = o->scores_f;
    k.weighted_f = o->weighted_f;
    return k;
}

// device scratch that grows on demand (synchronises the stream before a resize)
static int grow(void **p, size_t *have, size_t need, void *stream, const char *what)
{
    if (need <= *have)
        return TDOA_OK;
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipMalloc(p, need) != hipSuccess)
        return fail(TDOA_ERR_NOMEM, "%s scratch of %zu bytes", what, need);
    *have = need;
    return TDOA_OK;
}

int tdoa_resident_blocks(const void *kernel, int threads, size_t lds)
{
    static std::mutex mu;
    static std::map<std::tuple<int, const void *, int, size_t>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(dev, kernel, threads, lds);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end())
        return it->second;
    int per_cu = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds);
    const int r = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 256);
    cache[key] = r;
    return r;
}

// A/B switch of the environment: set and not "0"
static bool env_flag(const char *name)
{
    const char *e = getenv(name);
    return e && *e && strcmp(e, "0") != 0;
}

// frames per k_frame16 -> k_grid_bb chunk in the compact mode: TDOA_F16_CHUNK
// (A/B switch; default 0, the whole batch in one launch pair).  Measured at
// config 4 (same box, ms per 1e6 frames): chunks of 16384 / 32768 frames 87.4 /
// 86.5 vs 85.8 unchunked -- and the counter traffic does not drop: the compact
// scores still leave and re-enter the L2 (k_frame16 writes 7.5 GB, k_grid_bb
// reads 7.1 GB per 1e6 frames, FETCH_SIZE / WRITE_SIZE count L2 <-> fabric
// requests whether the MALL serves them or HBM does), and each chunk adds two
// launch tails (DESIGN.md, round-6 negative results)
static int64_t compact_chunk(int64_t B)
{
    static const int64_t chunk = [] {
        const char *e = getenv("TDOA_F16_CHUNK");
        return e ? (int64_t)atoll(e) : (int64_t)0;
    }();
    return chunk > 0 && chunk < B ? chunk : B;
}

// the outputs of frames [c0, ...) of a batch (per-frame arrays advanced; the
// compact scratch, reused per chunk, is not)
static tdoa_kout offset_kout(const tdoa_kout &k, int64_t c0, int P, int K)
{
    tdoa_kout o = k;
    auto adv = [&](auto *&ptr, int64_t per) {
        if (ptr)
            ptr += c0 * per;
    };
    adv(o.lags, P);
    adv(o.gate, 1);
    adv(o.cell, 1);
    adv(o.xy, 2);
    adv(o.max_L, 1);
    adv(o.max_Lf, 1);
    adv(o.scores, (int64_t)P * K);
    adv(o.weighted, (int64_t)P * K);
    adv(o.scores_f, (int64_t)P * K);
    adv(o.weighted_f, (int64_t)P * K);
    adv(o.peak3, (int64_t)P * 3);
    return o;
}

static int run_batch(tdoa_ctx *ctx, const int16_t *frames, int64_t B, const tdoa_outputs *out,
                     void *stream, bool prepared)
{
    if (!ctx || !out)
        return fail(TDOA_ERR_INVALID, "localize: NULL argument");
    if (B < 0)
        return fail(TDOA_ERR_INVALID, "localize: negative batch");
    if (B == 0)
        return TDOA_OK;
    if (!frames)
        return fail(TDOA_ERR_INVALID, "localize: NULL frames");
    if (!out->lags)
        return fail(TDOA_ERR_INVALID, "localize: outputs.lags is required");
    HIP_TRY(hipSetDevice(ctx->device));
    const bool phat = ctx->cfg.engine == TDOA_ENGINE_GCC_PHAT && !prepared;
    tdoa_kout k = to_kout(out);
    const bool ls = out->xy_ls || out->ls_rms;
    const bool grid =
        ls || out->cell || out->xy || (phat ? out->max_Lf != nullptr : out->max_L != nullptr);
    const size_t sz = phat ? sizeof(float) : sizeof(int64_t);
    const size_t pk = (size_t)B * ctx->P * ctx->K * sz;
    const void *weighted = phat ? (const void *)out->weighted_f : (const void *)out->weighted;
    const bool fused_grid = phat ? tdoa_gcc_phat_grid_in_kernel(ctx->kp) : tdoa_direct_fused_grid(ctx->kp);
    // the per-frame long-frame kernel (k_frame16) can write only the lags the
    // grid reads, compacted, when k_grid_bb solves the grid (configs 3, 4)
    const bool compact = grid && !weighted && !fused_grid && phat && tdoa_gcc_phat_peak3(ctx->kp) &&
                         tdoa_grid_bb_compact(ctx->kp) && !env_flag("TDOA_NO_COMPACT");
    const int64_t chunk = compact ? compact_chunk(B) : B;
    if (compact) {
        int rc = grow(&ctx->d_wscratch, &ctx->wscratch_bytes, (size_t)chunk * ctx->kp.wc_CK * sizeof(float), stream,
                      "weighted-score");
        if (rc)
            return rc;
        k.weighted_c = (float *)ctx->d_wscratch;
        weighted = ctx->d_wscratch;
    } else if (grid && !weighted && !fused_grid) {
        // the grid kernel reads the weighted scores back: keep them in scratch
        int rc = grow(&ctx->d_wscratch, &ctx->wscratch_bytes, pk, stream, "weighted-score");
        if (rc)
            return rc;
        weighted = ctx->d_wscratch;
        if (phat)
            k.weighted_f = (float *)ctx->d_wscratch;
        else
            k.weighted = (int64_t *)ctx->d_wscratch;
    }
    const void *raw = phat ? (const void *)out->scores_f : (const void *)out->scores;
    // the refinement's peak scores: from the kernel (it keeps the scores on
    // chip) or from the raw scores around each peak
    const bool peak_k = ls && phat && tdoa_gcc_phat_peak3(ctx->kp);
    if (peak_k) {
        int rc = grow(&ctx->d_tscratch, &ctx->tscratch_bytes, (size_t)B * ctx->P * 3 * sizeof(float), stream,
                      "peak-score");
        if (rc)
            return rc;
        k.peak3 = (float *)ctx->d_tscratch;
    }
    if (ls && !raw && !peak_k) {  // the refinement reads the raw scores around each peak
        int rc = grow(&ctx->d_rscratch, &ctx->rscratch_bytes, pk, stream, "raw-score");
        if (rc)
            return rc;
        raw = ctx->d_rscratch;
        if (phat)
            k.scores_f = (float *)ctx->d_rscratch;
        else
            k.scores = (int64_t *)ctx->d_rscratch;
    }
    if (ls && !out->cell) {
        int rc = grow(&ctx->d_cscratch, &ctx->cscratch_bytes, (size_t)B * 4, stream, "cell");
        if (rc)
            return rc;
        k.cell = (int32_t *)ctx->d_cscratch;
    }
    int rc = 0;
    if (compact && chunk < B) {
        // (TDOA_F16_CHUNK, A/B) the compact scratch of one chunk of frames at a
        // time, reused: k_frame16 writes it and k_grid_bb reads it back while it
        // can still sit in the 256 MB MALL (16384 x 7.3 KB at config 4)
        const int64_t M = ctx->kp.M, N = ctx->kp.N;
        for (int64_t c0 = 0; rc == 0 && c0 < B; c0 += chunk) {
            const int64_t n = B - c0 < chunk ? B - c0 : chunk;
            const tdoa_kout kc = offset_kout(k, c0, ctx->P, ctx->K);
            rc = tdoa_launch_gcc_phat(ctx->kp, kc, frames + c0 * M * N, n, ctx->cfg.phat_eps, ctx->d_spec,
                                      ctx->spec_bytes, stream);
            if (rc == 0)
                rc = tdoa_launch_grid(ctx->kp, kc, weighted, phat, n, stream);
        }
    } else {
        rc = phat ? tdoa_launch_gcc_phat(ctx->kp, k, frames, B, ctx->cfg.phat_eps, ctx->d_spec, ctx->spec_bytes,
                                         stream)
                  : tdoa_launch_direct(ctx->kp, k, frames, B, prepared, stream, nullptr);
        if (rc != 0 || !grid)
            return rc;
        if (!fused_grid)
            rc = tdoa_launch_grid(ctx->kp, k, weighted, phat, B, stream);
    }
    if (rc != 0 || !ls)
        return rc;
    return tdoa_launch_ls(ctx->kp, raw, phat, k.peak3, k.lags, k.cell, out->xy_ls, out->ls_rms, B, stream);
}

extern "C" int tdoa_heatmap(tdoa_ctx *ctx, const void *weighted, const void *max_L, int is_float,
                            int64_t B, uint8_t *classes, void *stream)
{
    if (!ctx || !weighted || !max_L || !classes)
        return fail(TDOA_ERR_INVALID, "tdoa_heatmap: NULL argument");
    if (B < 0)
        return fail(TDOA_ERR_INVALID, "tdoa_heatmap: negative batch");
    HIP_TRY(hipSetDevice(ctx->device));
    return tdoa_launch_heatmap(ctx->kp, weighted, max_L, is_float != 0, B, classes, stream);
}

// accessors for the streaming pipeline (tdoa_stream.cpp)
const tdoa_kparams *tdoa_ctx_kparams(const tdoa_ctx *c) { return &c->kp; }
int tdoa_ctx_device(const tdoa_ctx *c) { return c->device; }
int tdoa_ctx_engine(const tdoa_ctx *c) { return c->cfg.engine; }
int tdoa_ctx_rate(const tdoa_ctx *c) { return c->cfg.sample_rate_hz; }

extern "C" int tdoa_localize_batch(tdoa_ctx *ctx, const int16_t *frames, int64_t B,
                                   const tdoa_outputs *out, void *stream)
{
    return run_batch(ctx, frames, B, out, stream, false);
}

extern "C" int tdoa_correlate_prepared(tdoa_ctx *ctx, const int16_t *prepared, int64_t B,
                                       const tdoa_outputs *out, void *stream)
{
    return run_batch(ctx, prepared, B, out, stream, true);
}

extern "C" int tdoa_average_batch(tdoa_ctx *ctx, int64_t S, int64_t *est, const int64_t *fresh,
                                  const float *decay, int32_t *best, const tdoa_outputs *solve,
                                  void *stream)
{
    if (!ctx || !est || !fresh || !decay || !best)
        return fail(TDOA_ERR_INVALID, "tdoa_average_batch: NULL argument");
    if (S < 0)
        return fail(TDOA_ERR_INVALID, "tdoa_average_batch: negative stream count");
    if (S == 0)
        return TDOA_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    tdoa_kout k;
    const tdoa_kout *kptr = nullptr;
    if (solve) {
        k = to_kout(solve);
        kptr = &k;
    }
    return tdoa_launch_average(ctx->kp, S, est, fresh, decay, best, kptr, stream);
}

// correlations.c:40-43
extern "C" float tdoa_decay_us(uint64_t now_us, uint64_t last_us)
{
    const float dt = (float)(now_us - last_us) / 1e6f;
    const float arg = -dt / 0.5f;
    return (float)(1.0 - std::exp((double)arg));
}

extern "C" int tdoa_get_window(const tdoa_ctx *c, int32_t *w)
{
    if (!c || !w)
        return fail(TDOA_ERR_INVALID, "NULL");
    std::memcpy(w, c->win.data(), sizeof(int32_t) * c->N);
    return TDOA_OK;
}

extern "C" int tdoa_get_mics(const tdoa_ctx *c, float *xy)
{
    if (!c || !xy)
        return fail(TDOA_ERR_INVALID, "NULL");
    std::memcpy(xy, c->mic.data(), sizeof(float) * 2 * c->M);
    return TDOA_OK;
}

extern "C" int tdoa_get_lut(const tdoa_ctx *c, uint8_t *lut)
{
    if (!c || !lut)
        return fail(TDOA_ERR_INVALID, "NULL");
    std::memcpy(lut, c->lut.data(), c->lut.size());
    return TDOA_OK;
}

extern "C" int tdoa_get_prior(const tdoa_ctx *c, float *scale)
{
    if (!c || !scale)
        return fail(TDOA_ERR_INVALID, "NULL");
    std::memcpy(scale, c->prior.data(), sizeof(float) * c->K);
    return TDOA_OK;
}

extern "C" const char *tdoa_last_error(void) { return g_err.c_str(); }

extern "C" const char *tdoa_batch_kernel(const tdoa_ctx *ctx)
{
    if (!ctx)
        return "";
    if (ctx->cfg.engine == TDOA_ENGINE_GCC_PHAT)
        return tdoa_gcc_phat_kernel_name(ctx->kp);
    return tdoa_direct_fused_grid(ctx->kp) ? "k_direct_mfma" : "k_direct";
}

extern "C" int tdoa_batch_grid_fused(const tdoa_ctx *ctx)
{
    if (!ctx)
        return 0;
    return (ctx->cfg.engine == TDOA_ENGINE_GCC_PHAT ? tdoa_gcc_phat_grid_in_kernel(ctx->kp)
                                                    : tdoa_direct_fused_grid(ctx->kp))
               ? 1
               : 0;
}

extern "C" int tdoa_abi_version(void) { return TDOA_ABI_VERSION; }

// used by tdoa_kernels.hip launchers
int tdoa_set_error(int code, const char *msg)
{
    g_err = msg;
    return code;
}
