// tdoa_p1k_w64.hip -- GCC-PHAT metric kernel for BASELINE config 2 (3 mics x
// 1024-sample frames, L = 2048) at ONE FRAME PER 64-LANE WAVE, see DESIGN.md
// "k_p1k_w64".
//
// Why: k_p1k_lean (tdoa_phat1024.hip) runs a frame per 32-lane half-wave, so a
// 4096-frame batch is 2048 waves = two waves per SIMD for the launch's whole
// life, and the kernel time is one wave's latency chain (SQ: the SIMD's VALU
// idle about a third of the time).  Here a batch is 4096 waves: four per SIMD,
// 16-wave workgroups of 16 frames, one per CU, with the same LDS per frame.
//
// Per mic row (rolling_buffer.c:64-66, buffer.c:4-18 front end, as k_p1k_lean):
//   z[n] = x[2n] + i x[2n+1] (n < 512; n >= 512 is the 2N zero padding),
//   lane L loads z[L + 64 t], t < 8 (one 256-B segment per load).
//   Z = FFT_1024(z), n = a + 16 b, b = bh + 4 bl (a, bl < 16, bh < 4):
//     pass 1  DFT-16 over bl in registers (half zero)          -> rho_lo
//     pass 2  DFT-4 over bh = lane bits 4-5: v_permlane32/16_swap move those
//             lane bits into registers (one instruction per dword pair), the
//             W_64^{bh rho_lo} twiddles, then four register DFT-4 -> rho_hi
//     transpose through the wave's LDS tile [a][rho] (520-B rows; the column
//             of rho is a bit permutation, bank-conflict free both ways)
//     pass 3  W_1024^{a rho} twiddles, DFT-16 over a in registers -> j
//   Lane L ends with Z[res(L) + 64 j], j < 16.  res() pairs lanes (2i, 2i+1)
//   with partner residues (r, 64 - r), so the real-FFT split (bins b, N - b)
//   is in-lane after a DPP swap of the upper eight registers (lane 0: residue
//   0, a one-register rotation; lane 1: residue 32, self-paired).
//   PHAT per mic: U = X / max(|X|, sqrt(e)) (as k_p1k_lean).
// Per pair (0,1), (0,2), (1,2) (sample_compute.h:120-122 order):
//   Y[b] = (R[b] + R*[N-b]) + i (R[b] - R*[N-b]) W_2048^{-b}, R = conj(U_i) U_j,
//   y = IFFT_1024(Y) pruned to n in [0, 32) u [992, 1024) (lags -64..63):
//     pass A  DFT-16 over t in registers, W_1024^{-k1 l}, transpose [k1][l]
//     pass B  DFT-16 over l1 (l = l0 + 4 l1) pruned to outputs 0, 1, 14, 15
//     pass C  sum over l0 = lane bits 4-5 with its factors, as a reduce-
//             scatter by two permlane swaps: one complex output per lane
//   argmax + lag prior (correlations.c:20-33 on float scores), gate
//   (sample_compute.h:124-134), grid solve of vga_heatmap.h:99-108 for the
//   wave's frame (lanes split the distinct lag tuples).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "tdoa_cplx.h"
#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {

constexpr int W64_NW = 16;                 // waves (frames) per workgroup
constexpr int W64_ROW = 520;               // tile row stride: 64 f2 + 8 B
constexpr int W64_TILE = 16 * W64_ROW;     // 8320 B per wave
constexpr int W64_KPAD = 128;              // lag slots per pair in the grid table
constexpr int W64_GB = 8;                  // grid tuples per lane per loop trip
// LDS table image (byte offsets from its start)
constexpr int IMG_TW = 0;                  // [16 a][64 L] f2  W_1024^{a res(L)}
constexpr int IMG_TW2 = IMG_TW + 16 * 64 * 8;    // [8 k][64 L] f2  W_2048^{res(L) + 64 k}
constexpr int IMG_WIN = IMG_TW2 + 8 * 64 * 8;    // [8 t][64 L] f2  window / 128 of word L + 64 t
constexpr int IMG_T1 = IMG_WIN + 8 * 64 * 8;     // [4 g][3 b][4 q] f2  W_64^{b (g + 4 q)}
constexpr int IMG_FI = IMG_T1 + 48 * 8;          // [3][4 l0] f2  W_64^{-l0}, W_64^{2 l0}, W_64^{l0}
constexpr int IMG_PRIOR = IMG_FI + 12 * 8;       // [128] f32
constexpr int IMG_LANE = IMG_PRIOR + 128 * 4;    // [64] u32x2 per-lane tile offsets (w64_lane_info)
constexpr int IMG_FIXED = IMG_LANE + 64 * 8;     // tuples follow: [Upad] u32
static_assert(IMG_FIXED % 16 == 0, "tuple table must stay 16-B aligned");
// The image sits at the start of LDS, so every table read is a lane base plus
// an instruction offset (< 64 KiB); the tiles follow at W64_TILES.
constexpr int W64_UMAX = 2560;                    // padded tuple count the layout holds
// LDS: [0, HDR) the small per-wave words (balance, pair flags, exchange) and
// bin-512 slots, addressed by instruction offsets; then the image; then tiles
constexpr int W64_WORDS = W64_NW * 6;
constexpr int W64_B512 = 512;                     // [16 waves][2] f2
constexpr int W64_HDR = 1024;
static_assert(W64_WORDS * 4 <= W64_B512 && W64_B512 + W64_NW * 16 <= W64_HDR, "LDS header overflow");
constexpr int W64_TILES = W64_HDR + IMG_FIXED + W64_UMAX * 4;
// + words: [16] balance, [16] pair flags, [16][4] pair exchange; then bin 512
constexpr int W64_LDS_BYTES = W64_TILES + W64_NW * W64_TILE;
static_assert(W64_LDS_BYTES <= 160 * 1024, "k_p1k_w64 exceeds the CU's LDS");

// residue column held by lane L (0..63): lane pairs (2i, 2i+1) hold partner
// residues (r, 64 - r); the four 16-lane groups take r = 4i + {0, 2, 1, 3}, so
// every group holds one residue of each class r >> 2 (the inverse transpose's
// writes are conflict-free) and each 32-lane half holds the even (odd)
// residues (the forward transpose's reads are conflict-free).  Lane 0:
// residue 0, lane 1: residue 32 (both self-paired).
__host__ __device__ constexpr int w64_res(int L)
{
    const int g = L >> 4, i = (L & 15) >> 1;
    const int r = 4 * i + (((g & 1) << 1) | (g >> 1));
    return (L & 1) ? (L == 1 ? 32 : 64 - r) : r;
}
// forward tile column of residue rho: rho bit 0 -> column bit 5
__host__ __device__ constexpr int w64_colf(int rho) { return (rho >> 1) + 32 * (rho & 1); }
// inverse tile column of residue l = l0 + 4 l1: l1 + 16 l0
__host__ __device__ constexpr int w64_coli(int l) { return (l >> 2) + 16 * (l & 3); }

__device__ __forceinline__ f2 lds_f2(const char *base, int off) { return *reinterpret_cast<const f2 *>(base + off); }
__device__ __forceinline__ void sts_f2(char *base, int off, f2 v) { *reinterpret_cast<f2 *>(base + off) = v; }
__device__ __forceinline__ void pin(f2 &x) { asm volatile("" : "+v"(x)); }
// volatile LDS words through an LDS-address-space pointer (ds_read / ds_write;
// a generic volatile pointer gives flat accesses, whose waits drain vmcnt too)
typedef volatile __attribute__((address_space(3))) int vlds_int;
typedef short v2s_t __attribute__((ext_vector_type(2)));

// the lane id through an opaque move: lane-dependent values derived from it
// are recomputed where they are used instead of being held across phases
__device__ __forceinline__ int fresh_lane()
{
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t & 63;
}

__host__ __device__ constexpr int brev4(int k) { return ((k & 1) << 3) | ((k & 2) << 1) | ((k & 4) >> 1) | ((k & 8) >> 3); }

// Radix-2 DIT DFT-16 with the FMA butterflies of tdoa_cplx.h (W_16^q = W_32^2q),
// natural order in and out.  HALF_ZERO: inputs 8..15 are zero, so the first
// stage would copy; the second stage's groups are then DFT-4s of (x0, x1, 0, 0)
// built from their two inputs directly (no copies)
template <bool INV, bool HALF_ZERO>
__device__ __forceinline__ void fft16d(f2 (&x)[16])
{
    f2 v[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
        v[i] = x[brev4(i)];
    if (HALF_ZERO) {
#pragma unroll
        for (int g = 0; g < 16; g += 4) {
            const f2 a = v[g], b = v[g + 2];  // x[brev(g)], x[brev(g + 2)]
            v[g] = a + b;
            v[g + 2] = a - b;
            v[g + 1] = INV ? c_add_i(a, b) : c_add_mi(a, b);
            v[g + 3] = INV ? c_add_mi(a, b) : c_add_i(a, b);
        }
    } else {
#pragma unroll
        for (int g = 0; g < 16; g += 2)
            bfly_dit<INV>(v[g], v[g + 1], 0);
#pragma unroll
        for (int g = 0; g < 16; g += 4)
#pragma unroll
            for (int j = 0; j < 2; j++)
                bfly_dit<INV>(v[g + j], v[g + j + 2], j * 8);
    }
#pragma unroll
    for (int m = 8; m <= 16; m *= 2)
#pragma unroll
        for (int g = 0; g < 16; g += m)
#pragma unroll
            for (int j = 0; j < m / 2; j++)
                bfly_dit<INV>(v[g + j], v[g + j + m / 2], j * (32 / m));
#pragma unroll
    for (int k = 0; k < 16; k++)
        x[k] = v[k];
}

// pswap32 / pswap16: tdoa_cplx.h

// Partner swap of the upper eight bins (registers 8..15) between lanes 2i and
// 2i+1 (DPP quad_perm [1,0,3,2]) for every lane but 0 and 1; lane 0 (residue 0,
// pairs j <-> 16 - j) rotates its upper half by one register instead (FWD:
// V[j] <- V[j+1], V[15] <- V[0]; !FWD: V[j] <- V[j-1], V[8] <- E); lane 1
// keeps its registers.  Wait states as in tdoa_phat1024.hip.
#define W64_X(i) "%" #i
#define W64_DPP(i) "v_mov_b32_dpp " W64_X(i) ", " W64_X(i) " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define W64_MOV(d, s) "v_mov_b64 " W64_X(d) ", " W64_X(s) "\n\t"
template <bool FWD>
__device__ __forceinline__ void w64_swap_upper(f2 (&V)[16], f2 E)
{
    float x[16];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        x[2 * j] = V[8 + j].x;
        x[2 * j + 1] = V[8 + j].y;
    }
    uint64_t sv;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_and_b64 exec, exec, %[m1]\n\t"
                 "s_nop 4\n\t" W64_DPP(0) W64_DPP(1) W64_DPP(2) W64_DPP(3) W64_DPP(4) W64_DPP(5) W64_DPP(6)
                     W64_DPP(7) W64_DPP(8) W64_DPP(9) W64_DPP(10) W64_DPP(11) W64_DPP(12) W64_DPP(13)
                         W64_DPP(14) W64_DPP(15) "s_mov_b64 exec, %[sv]\n\t"
                 "s_nop 4"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                   "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                   "+v"(x[14]), "+v"(x[15]), [sv] "=&s"(sv)
                 : [m1] "s"(0xFFFFFFFFFFFFFFFCull));
    f2 y[8];
#pragma unroll
    for (int j = 0; j < 8; j++)
        y[j] = f2{x[2 * j], x[2 * j + 1]};
    const f2 e = FWD ? V[0] : E;
#define W64_ROT_ASM(ROT)                                                                          \
    asm volatile("s_mov_b64 %[sv], exec\n\t"                                                      \
                 "s_and_b64 exec, exec, %[m2]\n\t"                                                \
                 "s_nop 4\n\t" ROT "s_mov_b64 exec, %[sv]\n\t"                                   \
                 "s_nop 4"                                                                         \
                 : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]),         \
                   "+v"(y[6]), "+v"(y[7]), [sv] "=&s"(sv)                                          \
                 : [m2] "s"(0x1ull), [e] "v"(e))
    if constexpr (FWD)
        W64_ROT_ASM(W64_MOV(0, 1) W64_MOV(1, 2) W64_MOV(2, 3) W64_MOV(3, 4) W64_MOV(4, 5) W64_MOV(5, 6)
                        W64_MOV(6, 7) "v_mov_b64 %7, %[e]\n\t");
    else
        W64_ROT_ASM(W64_MOV(7, 6) W64_MOV(6, 5) W64_MOV(5, 4) W64_MOV(4, 3) W64_MOV(3, 2) W64_MOV(2, 1)
                        W64_MOV(1, 0) "v_mov_b64 %0, %[e]\n\t");
#undef W64_ROT_ASM
#pragma unroll
    for (int j = 0; j < 8; j++)
        V[8 + j] = y[j];
}

// sum over the 64 lanes, VALU only: row all-reduce by DPP, row_bcast:15 and
// row_bcast:31, then lane 63 (a scalar for the whole wave)
__device__ __forceinline__ int wsum64(int s)
{
    s += __builtin_amdgcn_mov_dpp(s, 0xB1, 0xF, 0xF, false);   // xor 1
    s += __builtin_amdgcn_mov_dpp(s, 0x4E, 0xF, 0xF, false);   // xor 2
    s += __builtin_amdgcn_mov_dpp(s, 0x141, 0xF, 0xF, false);  // half-row mirror
    s += __builtin_amdgcn_mov_dpp(s, 0x140, 0xF, 0xF, false);  // row mirror
    s += __builtin_amdgcn_update_dpp(0, s, 0x142, 0xA, 0xF, false);  // row_bcast:15
    s += __builtin_amdgcn_update_dpp(0, s, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return __builtin_amdgcn_readlane(s, 63);
}

// per-lane tile offsets (bytes), staged with the image:
//   x: forward read column 8 colf(res) | inverse write column 8 coli(res) << 16
//   y: forward write (L & 15) * ROW + 16 (L >> 4) | inverse read (L & 15) * ROW + 128 (L >> 4) << 16
__host__ __device__ constexpr uint32_t w64_lane_info(int L, int w)
{
    return w == 0 ? (uint32_t)(8 * w64_colf(w64_res(L))) | ((uint32_t)(8 * w64_coli(w64_res(L))) << 16)
                  : (uint32_t)((L & 15) * W64_ROW + 16 * (L >> 4)) |
                        ((uint32_t)((L & 15) * W64_ROW + 128 * (L >> 4)) << 16);
}

#ifndef W64_PAIR
#define W64_PAIR 0  // 1: grid solve of two frames per gather (waves w, w ^ 1; measured slower)
#endif
#ifndef W64_BAL
#define W64_BAL 1  // issue balance: 0 none, 1 at phase boundaries, 2 also inside the transforms
#endif

struct W64Lane {
    int *prog;            // balance words [SIMD group][4] (see the kernel)
    int pslot, pgroup;    // this wave's word, its group's first word
    mutable int phase;    // phase boundaries passed
    char *tile;       // this wave's transpose tile (wave-uniform)
    const char *img;  // the table image
    f2 *b512;         // this wave's unit spectra at bin 512 ([0] mic 0 / U0, [1] mic 1 / U1):
                      // lane 0's values (residue 0), kept in LDS instead of a 17th register pair
    int L8;           // 8 * lane: the lane's offset in every [..][64] f2 table
};

// issue balance between the four waves of a SIMD (waves w, w + 4, w + 8,
// w + 12).  The SIMD issues oldest-first, so without this the waves finish
// one after another (measured: 22, 28, 34, 40 us by age) and the last one
// runs alone -- and packed fp32 issues at half rate below four waves per SIMD
// (tools/probe/valu_rate.hip); here a wave that has passed more balance points
// than the slowest wave of its SIMD drops to the low priority until it catches up
__device__ __forceinline__ void w64_balance(const W64Lane &W)
{
    vlds_int *pv = (vlds_int *)W.prog;
    const int ph = ++W.phase;
    if ((W.L8 >> 3) == 0)
        pv[W.pslot] = ph;
    const int g0 = pv[W.pgroup], g1 = pv[W.pgroup + 1], g2 = pv[W.pgroup + 2], g3 = pv[W.pgroup + 3];
    int mn = g0 < g1 ? g0 : g1;
    mn = mn < g2 ? mn : g2;
    mn = mn < g3 ? mn : g3;
    mn = __builtin_amdgcn_readfirstlane(mn);
    if (ph > mn)
        __builtin_amdgcn_s_setprio(0);
    else
        __builtin_amdgcn_s_setprio(2);
}
__device__ __forceinline__ void w64_bal_fine(const W64Lane &W)
{
    if (W64_BAL >= 2)
        w64_balance(W);
}

// front end of one mic row (16 samples per lane): floor-mean DC (whole wave),
// low byte of x - off, floor(s W / 128); v[t] = z[L + 64 t], t < 8
__device__ __forceinline__ void w64_front(const W64Lane &W, const uint32_t (&w)[8], f2 (&v)[16])
{
    int s = 0;
#pragma unroll
    for (int t = 0; t < 8; t++)
        s = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s_t, w[t]), v2s_t{1, 1}, s, false);
    s = wsum64(s);
    const uint32_t off = (uint32_t)(s >> 10) & 0xFFu;
    const uint32_t off2 = off | (off << 16);
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const f2 wf = lds_f2(W.img, IMG_WIN + 512 * t + W.L8);
        const uint32_t d = (w[t] | 0x01000100u) - off2;
        const float s0 = (float)(int8_t)(d & 0xFFu);
        const float s1 = (float)(int8_t)((d >> 16) & 0xFFu);
        const f2 pr = f2{s0, s1} * wf;
        v[t] = f2{floorf(pr.x), floorf(pr.y)};
    }
}

// forward FFT_1024 of z[L + 64 t] (t < 8, upper half zero) in v ->
// v[j] = Z[res(L) + 64 j]
__device__ __forceinline__ void w64_fft_fwd(const W64Lane &W, f2 (&v)[16])
{
    fft16d<false, true>(v);  // pass 1: v[rho_lo], lane = (a, bh)
    // pass 2: lane bits 5, 4 (bh bits 1, 0) <-> register bits 3, 2
#pragma unroll
    for (int r = 0; r < 8; r++)
        pswap32(v[r], v[r + 8]);
#pragma unroll
    for (int r = 0; r < 16; r++)
        if (!(r & 4))
            pswap16(v[r], v[r + 4]);
    // now lane = (a, rho_lo bits 2-3 = q), register g + 4 bh (g = rho_lo bits 0-1)
    {
        const int q8 = (W.L8 >> 4) & ~7;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            f2 x[4];
            x[0] = v[g];
#pragma unroll
            for (int b = 1; b < 4; b++)
                x[b] = c_mul(v[g + 4 * b], lds_f2(W.img, IMG_T1 + 32 * (3 * g + b - 1) + q8));
            const f2 a0 = x[0] + x[2], b0 = x[0] - x[2], c0 = x[1] + x[3], d0 = x[1] - x[3];
            v[g] = a0 + c0;
            v[g + 8] = a0 - c0;
            v[g + 4] = c_add_mi(b0, d0);
            v[g + 12] = c_add_i(b0, d0);
        }
    }
    w64_bal_fine(W);
    // transpose: X_a[rho], rho = g + 4 q + 16 rh -> tile[a][colf(rho)]
    const uint2 li = *reinterpret_cast<const uint2 *>(W.img + IMG_LANE + W.L8);
    wave_lds_sync();  // after the tile's previous readers
    {
        char *wb = W.tile + (li.y & 0xFFFFu);
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int rh = 0; rh < 4; rh++)
                sts_f2(wb, 8 * ((g >> 1) + 8 * rh + 32 * (g & 1)), v[g + 4 * rh]);
    }
    wave_lds_sync();
    {
        const char *rb = W.tile + (li.x & 0xFFFFu);
#pragma unroll
        for (int a = 0; a < 16; a++)
            v[a] = lds_f2(rb, W64_ROW * a);
#pragma unroll
        for (int a = 1; a < 16; a++)
            v[a] = c_mul(v[a], lds_f2(W.img, IMG_TW + 512 * a + W.L8));
    }
    w64_bal_fine(W);
    fft16d<false, false>(v);  // pass 3: v[j] = Z[res + 64 j]
}

// real-FFT split of pair k (bins b = res + 64 k and N - b) + unit normalisation
__device__ __forceinline__ void w64_split(const W64Lane &W, f2 A, f2 Bv, int k, float e2, f2 &ub, f2 &un)
{
    const f2 wk = lds_f2(W.img, IMG_TW2 + 512 * k + W.L8);
    const f2 e = c_addconj(A, Bv);
    const f2 od = c_mul(c_subconj(A, Bv), wk);
    ub = c_unit(c_add_mi(e, od), e2);
    un = c_unit(c_conj_add_i(e, od), e2);
}

// unit spectrum of one mic row in the paired layout: U[k], U[15 - k] hold
// bins b, N - b (k < 8); returns unit X[512] (meaningful on lane 0)
template <typename Hook>
__device__ __forceinline__ f2 w64_spectrum(const W64Lane &W, const uint32_t (&w)[8], f2 (&V)[16], float e2,
                                           Hook after_front)
{
    w64_front(W, w, V);
    after_front();
    w64_fft_fwd(W, V);
    const f2 x512 = c_unit(conjf2(V[8]), e2);  // bin 512 (lane 0, residue 0)
    w64_swap_upper<true>(V, f2{0.0f, 0.0f});
    return x512;
}

struct NoHook {
    __device__ void operator()() const {}
};

template <typename Hook = NoHook>
__device__ __forceinline__ void w64_forward(const W64Lane &W, const uint32_t (&w)[8], f2 (&U)[16], int slot,
                                            float e2, Hook after_front = Hook())
{
    const f2 x512 = w64_spectrum(W, w, U, e2, after_front);
    if ((W.L8 >> 3) == 0)
        W.b512[slot] = x512;
#pragma unroll
    for (int k = 0; k < 8; k++)
        w64_split(W, U[k], U[15 - k], k, e2, U[k], U[15 - k]);
}

// mic 2: its unit spectrum V consumed bin pair by bin pair into
// A <- conj(A) V, B <- conj(B) V
__device__ __forceinline__ void w64_forward_cross(const W64Lane &W, const uint32_t (&w)[8], f2 (&A)[16],
                                                  f2 (&Bs)[16], float e2)
{
    f2 V[16];
    const f2 x512 = w64_spectrum(W, w, V, e2, NoHook());
    if ((W.L8 >> 3) == 0) {
        W.b512[0] = c_conjmul(W.b512[0], x512);
        W.b512[1] = c_conjmul(W.b512[1], x512);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        f2 ub, un;
        w64_split(W, V[k], V[15 - k], k, e2, ub, un);
        A[k] = c_conjmul(A[k], ub);
        A[15 - k] = c_conjmul(A[15 - k], un);
        Bs[k] = c_conjmul(Bs[k], ub);
        Bs[15 - k] = c_conjmul(Bs[15 - k], un);
    }
}

// packed inverse input of the cross spectrum R (R = conj(A) B when CROSS,
// else A), back in the residue layout v[t] = Y[res + 64 t]
template <bool CROSS>
__device__ __forceinline__ void w64_pretwiddle(const W64Lane &W, const f2 (&A)[16], const f2 (&Bs)[16], int slot,
                                               f2 (&v)[16])
{
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const f2 Rk = CROSS ? c_conjmul(A[k], Bs[k]) : A[k];
        const f2 Rn = CROSS ? c_conjmul(A[15 - k], Bs[15 - k]) : A[15 - k];
        const f2 wk = lds_f2(W.img, IMG_TW2 + 512 * k + W.L8);
        const f2 s = c_addconj(Rk, Rn);
        const f2 q = c_mulconj(c_subconj(Rk, Rn), wk);
        v[k] = c_add_i(s, q);
        v[15 - k] = c_conj_add_mi(s, q);
    }
    const f2 R16 = CROSS ? c_conjmul(W.b512[0], W.b512[1]) : W.b512[slot];  // (lane 0's)
    const f2 Ye = f2{2.0f * R16.x, -2.0f * R16.y};  // Y[512] = 2 conj(R[512])
    w64_swap_upper<false>(v, Ye);
}

// pruned inverse: v[t] = Y[res + 64 t] -> this lane's complex output y[n],
// n = k1 + {0, 16, 992, 1008}[lane bits 4, 5]
__device__ __forceinline__ f2 w64_fft_inv(const W64Lane &W, f2 (&v)[16])
{
    fft16d<true, false>(v);  // pass A: v[k1]
    const uint2 li = *reinterpret_cast<const uint2 *>(W.img + IMG_LANE + W.L8);
#pragma unroll
    for (int k = 1; k < 16; k++)
        v[k] = c_mulconj(v[k], lds_f2(W.img, IMG_TW + 512 * k + W.L8));
    wave_lds_sync();  // after the tile's previous readers
    {
        char *wb = W.tile + (li.x >> 16);
#pragma unroll
        for (int k = 0; k < 16; k++)
            sts_f2(wb, W64_ROW * k, v[k]);
    }
    wave_lds_sync();
    f2 x[16];
    {
        const char *rb = W.tile + (li.y >> 16);
#pragma unroll
        for (int l1 = 0; l1 < 16; l1++)
            x[l1] = lds_f2(rb, 8 * l1);
    }
    w64_bal_fine(W);
    // pass B, outputs m0 = 0, 1, 14, 15 of sum_l1 x W_16^{-m0 l1}
    f2 a[8], d[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        a[j] = x[j] + x[j + 8];
        d[j] = x[j] - x[j + 8];
    }
    // X0 = sum a
    f2 X0;
    {
        f2 s0 = (a[0] + a[1]) + (a[2] + a[3]);
        f2 s1 = (a[4] + a[5]) + (a[6] + a[7]);
        X0 = s0 + s1;
    }
    // X14 = sum a_j W_8^j: (a0 - a4) - i (a2 - a6) + sqrt(1/2) [(u - w) - i (u + w)],
    // u = a1 - a5, w = a3 - a7
    f2 X14;
    {
        const f2 e0 = a[0] - a[4], e2v = a[2] - a[6];
        const f2 ev = c_add_mi(e0, e2v);
        const f2 u = a[1] - a[5], w = a[3] - a[7];
        const f2 od = c_add_mi(u - w, u + w);
        const float h = 0.70710678118654752f;
        X14 = v_fma(od, f2{h, h}, ev);
    }
    // X1 = sum d_j e^{+i pi j/8}, X15 = sum d_j e^{-i pi j/8}: with
    // P = sum d_j cos_j and Q = sum swap(d_j) sin_j, X1 = (P.x - Q.x, P.y + Q.y),
    // X15 = (P.x + Q.x, P.y - Q.y)
    f2 X1, X15;
    {
        f2 P = d[0], Q = v_sw(d[4]);
#pragma unroll
        for (int j = 1; j < 8; j++) {
            if (j == 4)
                continue;
            const float c = (float)COS32D[2 * j], s = (float)COS32D[8 - 2 * j < 0 ? 2 * j - 8 : 8 - 2 * j];
            P = v_fma(d[j], f2{c, c}, P);
            Q = v_fma(v_sw(d[j]), f2{s, s}, Q);
        }
        X1 = f2{P.x - Q.x, P.y + Q.y};
        X15 = f2{P.x + Q.x, P.y - Q.y};
    }
    // pass C factors W_64^{-l0}, W_64^{2 l0}, W_64^{l0} (the last two carry W_4^{-3 l0})
    {
        const int l08 = (W.L8 >> 4) & ~7;
        X1 = c_mul(X1, lds_f2(W.img, IMG_FI + l08));
        X14 = c_mul(X14, lds_f2(W.img, IMG_FI + 32 + l08));
        X15 = c_mul(X15, lds_f2(W.img, IMG_FI + 64 + l08));
    }
    // reduce-scatter over lane bits 5, 4
    pswap32(X0, X1);
    pswap32(X14, X15);
    f2 Sa = X0 + X1, Sb = X14 + X15;
    pswap16(Sa, Sb);
    return Sa + Sb;
}

}  // namespace

#ifdef TDOA_DIAG
__device__ unsigned long long g_diag_w64[1 << 16];
#endif

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_p1k_w64(tdoa_kparams kp, tdoa_kout out, const int16_t *__restrict__ frames,
                                                  int64_t B, float e2)
{
    constexpr int N = 1024, P = 3, NT = W64_NW * 64;
    // static LDS (the whole 160 KiB budget): addresses are compile-time
    // constants that fold into the instruction offsets (the dynamic segment's
    // base is a link-time relocation, materialised by an add at every use)
    __shared__ __attribute__((aligned(16))) char smem[W64_LDS_BYTES];
    char *img = smem + W64_HDR;                      // table image
    char *tiles = smem + W64_TILES;                  // [NW][TILE]
    const float *prior = (const float *)(img + IMG_PRIOR);
    const uint32_t *tups = (const uint32_t *)(img + IMG_FIXED);

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
#ifdef TDOA_DIAG
    unsigned long long stamp[16] = {};
    int nst = 0;
#define W64_MARK()                                       \
    do {                                                 \
        if (nst < 13)                                    \
            stamp[nst++] = __builtin_amdgcn_s_memtime(); \
    } while (0)
    stamp[nst++] = __builtin_amdgcn_s_memtime();
    stamp[14] = __builtin_amdgcn_s_memrealtime();
#else
#define W64_MARK() \
    do {           \
    } while (0)
#endif
    int *prog = (int *)smem;  // [SIMD group][4] balance, [16] pair flags, [16][4] exchange
    if (lane == 0) {
        prog[(wave & 3) * 4 + (wave >> 2)] = 0;
        prog[W64_NW + wave] = 0;  // pair flag (read after the staging barrier)
    }
    __builtin_amdgcn_s_setprio(2);
    W64Lane W;
    W.prog = prog;
    W.pslot = (wave & 3) * 4 + (wave >> 2);
    W.pgroup = (wave & 3) * 4;
    W.phase = 0;
    W.tile = tiles + __builtin_amdgcn_readfirstlane(wave) * W64_TILE;
    W.img = img;
    W.L8 = 8 * lane;
    W.b512 = (f2 *)(smem + W64_B512) + 2 * __builtin_amdgcn_readfirstlane(wave);
    auto balance = [&]() {
        if (W64_BAL >= 1)
            w64_balance(W);
    };

    const int K = kp.K, S = kp.S;
    const bool do_grid = out.cell || out.xy || out.max_Lf;
    const int Upad = (kp.U + W64_GB * 64 - 1) / (W64_GB * 64) * (W64_GB * 64);
    const int64_t f = (int64_t)blockIdx.x * W64_NW + wave;
    const bool live = f < B;
    const int64_t fc = live ? f : B - 1;

    auto fetch = [&](uint32_t(&w)[8], int m) {
        const uint32_t *row = reinterpret_cast<const uint32_t *>(frames + (fc * 3 + m) * (int64_t)N) + (W.L8 >> 3);
#pragma unroll
        for (int t = 0; t < 8; t++)
            w[t] = __builtin_nontemporal_load(row + 64 * t);
    };
    // table image: its loads first (L2 hits), then the first row (HBM), then
    // the image's LDS writes
    uint32_t w0[8], w1[8], w2[8];
    {
        const uint4 *src = (const uint4 *)kp.w64_img;
        uint4 *dst = (uint4 *)img;
        const int n16 = do_grid ? kp.w64_img_bytes / 16 : IMG_FIXED / 16;
        // image <= 2 * NT * 16 B = 32 KiB (tdoa_p1k_w64_fits); two named
        // units (an array of them was put in scratch)
        const int i0 = tid < n16 ? tid : n16 - 1, i1 = tid + NT < n16 ? tid + NT : n16 - 1;
        const uint4 im0 = src[i0], im1 = src[i1];
        fetch(w0, 0);
        dst[i0] = im0;
        dst[i1] = im1;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 8; t++)
        asm volatile("" : "+v"(w0[t]));

    const float invL = 1.0f / 2048.0f;
    float wv[3][2];
    int best[3];
    // argmax + lag prior of pair p from this lane's output y (lags lg, lg + 1)
    auto finish_pair = [&](int p, f2 y) {
        const int L = W.L8 >> 3;
        const int q = L >> 4;
        const int lg = 2 * (L & 15) + ((q & 1) ? -64 : 0) + ((q & 2) ? 32 : 0);
        const int ck[2] = {lg + S, lg + 1 + S};
        const bool ok[2] = {lg >= -S && lg <= S, lg + 1 >= -S && lg + 1 <= S};
        const float cv[2] = {y.x * invL, y.y * invL};
        int bkey = INT_MIN, bk = INT_MAX;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int kc = fkey(cv[c]);
            if (ok[c] && kc > bkey) {
                bkey = kc;
                bk = ck[c];
            }
        }
        wave_argmax_key(bkey, bk);
        bk = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);
        best[p] = bk - S;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int dd = ck[c] > bk ? ck[c] - bk : bk - ck[c];
            wv[p][c] = ok[c] ? cv[c] * prior[ok[c] ? dd : 0] : 0.0f;
        }
        if (out.scores_f || out.weighted_f) {  // debug / parity outputs (uniform branch)
            float *sr = out.scores_f ? out.scores_f + (size_t)(f * P + p) * K : nullptr;
            float *wr = out.weighted_f ? out.weighted_f + (size_t)(f * P + p) * K : nullptr;
#pragma unroll
            for (int c = 0; c < 2; c++)
                if (live && ok[c]) {
                    if (sr)
                        sr[ck[c]] = cv[c];
                    if (wr)
                        wr[ck[c]] = wv[p][c];
                }
        }
        if (live && L == 0)
            out.lags[f * P + p] = bk - S;
    };

    f2 U0[16], U1[16];
    W64_MARK();
    w64_forward(W, w0, U0, 0, e2, [&] {
        fetch(w1, 1);
        balance();
    });
    W64_MARK();
    balance();
    w64_forward(W, w1, U1, 1, e2, [&] { balance(); });
    W64_MARK();
    balance();
    {
        f2 v[16];
        w64_pretwiddle<true>(W, U0, U1, 0, v);  // pair 0: (0, 1)
        fetch(w2, 2);
        const f2 y = w64_fft_inv(W, v);
        finish_pair(0, y);
    }
    W64_MARK();
    balance();
    w64_forward_cross(W, w2, U0, U1, e2);  // pairs 1: (0, 2), 2: (1, 2)
    W64_MARK();
    balance();
    {
        f2 v[16];
        w64_pretwiddle<false>(W, U0, U0, 0, v);
        const f2 y = w64_fft_inv(W, v);
        finish_pair(1, y);
    }
    W64_MARK();
    balance();
    {
        f2 v[16];
        w64_pretwiddle<false>(W, U1, U1, 1, v);
        const f2 y = w64_fft_inv(W, v);
        finish_pair(2, y);
    }
    W64_MARK();
    balance();
    if (live && lane == 0 && out.gate)
        out.gate[f] = best[0] * best[0] + best[1] * best[1] + best[2] * best[2] > 4 ? 1 : 0;

    if (do_grid) {
#if W64_PAIR
        // ---- grid solve (vga_heatmap.h:99-108), two frames at once: the waves
        // w and w ^ 1 share one [p][KPAD] f2 table of their weighted scores
        // (frame of the even wave in .x, of the odd wave in .y) in the even
        // wave's tile, each gathers half of the distinct lag tuples for both
        // frames (alternate 256-tuple steps), then they swap partial maxima.
        // Hand-offs through LDS words of the pair (same CU: in-order DS, no
        // fence); the odd wave writes only after the even wave has finished
        // reading its tile.
        const int odd = wave & 1;
        vlds_int *flag = (vlds_int *)(prog + W64_NW + (wave & ~1));  // [pair][2]: 1 table half written, 2 partials
        const int toff = (W64_TILES + __builtin_amdgcn_readfirstlane(wave & ~1) * W64_TILE + 1023) & ~1023;
        float *wsc = (float *)(smem + toff);  // [p][KPAD][2]
        auto wait_flag = [&](vlds_int *fp, int v) {
            while (__builtin_amdgcn_readfirstlane(*fp) < v)
                __builtin_amdgcn_s_sleep(1);
        };
        wave_lds_sync();  // after the last pair's reads of this wave's tile
        if (odd)
            wait_flag(flag, 1);  // the even wave is done with its tile
        {
            const int L = W.L8 >> 3;
            const int q = L >> 4;
            const int lg = 2 * (L & 15) + ((q & 1) ? -64 : 0) + ((q & 2) ? 32 : 0);
#pragma unroll
            for (int c = 0; c < 2; c++)
                if (lg + c >= -S && lg + c <= S)
#pragma unroll
                    for (int p = 0; p < P; p++)
                        wsc[(p * W64_KPAD + lg + c + S) * 2 + odd] = wv[p][c];
            if (L < 3)  // lag slot 127 of every pair: the padding tuple
                wsc[(L * W64_KPAD + W64_KPAD - 1) * 2 + odd] = -INFINITY;
        }
        wave_lds_sync();
        if (lane == 0)
            flag[odd] = 1;
        wait_flag(flag + (odd ^ 1), 1);  // the partner's half of the table is written
        W64_MARK();
        f2 gv = f2{-INFINITY, -INFINITY};
        int gs0 = INT_MAX - 64, gs1 = INT_MAX - 64;  // (tuple index - lane) of the lane's best, per frame
        const char *lds = smem;
        auto gather = [&](const uint32_t (&qq)[4], f2 (&g)[4][3]) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                g[i][0] = *reinterpret_cast<const f2 *>(lds + ((qq[i] & 0x3FFu) | toff));
                g[i][1] = *reinterpret_cast<const f2 *>(lds + (((qq[i] >> 10) & 0x3FFu) | toff) + W64_KPAD * 8);
                g[i][2] = *reinterpret_cast<const f2 *>(lds + ((qq[i] >> 20) | toff) + 2 * W64_KPAD * 8);
            }
        };
        auto consume = [&](const f2 (&gg)[4][3], int ub) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const f2 Lg = (gg[i][0] + gg[i][1]) + gg[i][2];
                if (Lg.x > gv.x) {
                    gv.x = Lg.x;
                    gs0 = ub + 64 * i;
                }
                if (Lg.y > gv.y) {
                    gv.y = Lg.y;
                    gs1 = ub + 64 * i;
                }
            }
        };
        // this wave's steps: u = 256 (2 j + odd), pipelined by one step
        uint32_t qa[4];
        f2 ga[4][3];
        const int nstep = Upad / 256;
#pragma unroll
        for (int i = 0; i < 4; i++)
            qa[i] = tups[256 * odd + 64 * i + lane];
        gather(qa, ga);
        for (int st = odd; st < nstep; st += 2) {
            const int sn = st + 2 < nstep ? st + 2 : st;  // (a harmless re-read)
            uint32_t qn[4];
#pragma unroll
            for (int i = 0; i < 4; i++)
                qn[i] = tups[256 * sn + 64 * i + lane];
            f2 gn[4][3];
            gather(qn, gn);
            consume(ga, 256 * st);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                qa[i] = qn[i];
#pragma unroll
                for (int p = 0; p < 3; p++)
                    ga[i][p] = gn[i][p];
            }
        }
        W64_MARK();
        // (max L, first tuple) per frame over the wave, each lane's candidate
        // cell requested before the reductions
        int gu[2] = {gs0 + lane, gs1 + lane}, cell2[2];
        float mv[2] = {gv.x, gv.y};
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int myu = gu[j];
            const int mycell = kp.tuple_cell[(myu < 0 || myu >= kp.U) ? 0 : myu];
            int gk = fkey(mv[j]);
            wave_argmax_key(gk, gu[j]);
            mv[j] = fkey_value(gk);
            const uint64_t wm = __ballot(myu == gu[j] && gu[j] >= 0 && gu[j] < kp.U);
            cell2[j] = wm ? __builtin_amdgcn_readlane(mycell, __builtin_ctzll(wm)) : kp.tuple_cell[0];
        }
        // swap partials: each wave needs the partner's result for its own frame
        int *xch = prog + 2 * W64_NW + 4 * wave;  // [wave][3]: key, index, cell for the partner's frame
        if (lane == 0) {
            xch[0] = fkey(mv[odd ^ 1]);
            xch[1] = gu[odd ^ 1];
            xch[2] = cell2[odd ^ 1];
        }
        wave_lds_sync();
        if (lane == 0)
            flag[odd] = 2;
        wait_flag(flag + (odd ^ 1), 2);
        const vlds_int *px = (const vlds_int *)(prog + 2 * W64_NW + 4 * (wave ^ 1));
        const int ok_ = __builtin_amdgcn_readfirstlane(px[0]), oi = __builtin_amdgcn_readfirstlane(px[1]),
                  oc = __builtin_amdgcn_readfirstlane(px[2]);
        int mk = fkey(mv[odd]), mi = gu[odd], cell = cell2[odd];
        if (ok_ > mk || (ok_ == mk && oi < mi)) {
            mk = ok_;
            mi = oi;
            cell = oc;
        }
        const float gvf = fkey_value(mk);
        if (live && lane == 0) {
            if (out.cell)
                out.cell[f] = cell;
            if (out.max_Lf)
                out.max_Lf[f] = gvf;
            if (out.xy) {
                const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
                out.xy[2 * f] = (float)(cx - kp.half_w) / kp.grid_scale;
                out.xy[2 * f + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
            }
        }
        W64_MARK();
#else
        // ---- grid solve (vga_heatmap.h:99-108) of the wave's frame: weighted
        // scores [p][KPAD] f32 in the wave's tile, lanes split the distinct lag
        // tuples (lane-strided, ascending per lane: a strict '>' keeps the
        // first maximum)
        wave_lds_sync();  // after the last pair's reads of this tile
        // the table at a 1 KiB-aligned LDS address inside the tile: a gather
        // address is then (field | base), one v_and_or for pair 0
        const int toff = (W64_TILES + __builtin_amdgcn_readfirstlane(wave) * W64_TILE + 1023) & ~1023;
        float *wsc = (float *)(smem + toff);
        {
            const int L = W.L8 >> 3;
            const int q = L >> 4;
            const int lg = 2 * (L & 15) + ((q & 1) ? -64 : 0) + ((q & 2) ? 32 : 0);
            if (!(S & 1)) {  // lg + S even: one 8-B store (the second slot may be K: unused)
                if (lg >= -S && lg <= S)
#pragma unroll
                    for (int p = 0; p < P; p++)
                        *reinterpret_cast<f2 *>(wsc + p * W64_KPAD + lg + S) = f2{wv[p][0], wv[p][1]};
            } else {
#pragma unroll
                for (int c = 0; c < 2; c++)
                    if (lg + c >= -S && lg + c <= S)
#pragma unroll
                        for (int p = 0; p < P; p++)
                            wsc[p * W64_KPAD + lg + c + S] = wv[p][c];
            }
            if (L < 3)  // lag slot 127 of every pair: the padding tuple
                wsc[L * W64_KPAD + W64_KPAD - 1] = -INFINITY;
        }
        wave_lds_sync();
        W64_MARK();
        float gv = -INFINITY;
        int gs = INT_MAX - 64;  // (tuple index - lane) of the lane's best: wave-uniform
                                // candidates, selected from scalar registers
        const char *lds = smem;
        auto gather = [&](const uint32_t (&qq)[4], float (&g)[4][3]) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                g[i][0] = *reinterpret_cast<const float *>(lds + ((qq[i] & 0x3FFu) | toff));
                g[i][1] = *reinterpret_cast<const float *>(lds + (((qq[i] >> 10) & 0x3FFu) | toff) + W64_KPAD * 4);
                g[i][2] = *reinterpret_cast<const float *>(lds + ((qq[i] >> 20) | toff) + 2 * W64_KPAD * 4);
            }
        };
        auto consume = [&](const float (&gg)[4][3], int ub) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float Lg = (gg[i][0] + gg[i][1]) + gg[i][2];
                if (Lg > gv) {
                    gv = Lg;
                    gs = ub + 64 * i;
                }
            }
        };
        uint32_t qa[4];
        float ga[4][3];
#pragma unroll
        for (int i = 0; i < 4; i++)
            qa[i] = tups[64 * i + lane];
        gather(qa, ga);
        for (int u0 = 0; u0 < Upad; u0 += 512) {
            uint32_t qn[4];
#pragma unroll
            for (int i = 0; i < 4; i++)
                qn[i] = tups[u0 + 256 + 64 * i + lane];
            float gn[4][3];
            gather(qn, gn);
            consume(ga, u0);
            const int un = u0 + 512 < Upad ? u0 + 512 : u0 + 256;  // (a harmless re-read)
#pragma unroll
            for (int i = 0; i < 4; i++)
                qa[i] = tups[un + 64 * i + lane];
            gather(qa, ga);
            consume(gn, u0 + 256);
        }
        int gu = gs + lane;
        W64_MARK();
        const int myu = gu;
        const int mycell = kp.tuple_cell[(gu < 0 || gu >= kp.U) ? 0 : gu];
        int gk = fkey(gv);
        wave_argmax_key(gk, gu);
        gv = fkey_value(gk);
        const uint64_t wm = __ballot(myu == gu && gu >= 0 && gu < kp.U);
        const int cell = wm ? __builtin_amdgcn_readlane(mycell, __builtin_ctzll(wm)) : kp.tuple_cell[0];
        if (live && lane == 0) {
            if (out.cell)
                out.cell[f] = cell;
            if (out.max_Lf)
                out.max_Lf[f] = gv;
            if (out.xy) {
                const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
                out.xy[2 * f] = (float)(cx - kp.half_w) / kp.grid_scale;
                out.xy[2 * f + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
            }
        }
        W64_MARK();
    #endif
    }
#ifdef TDOA_DIAG
    stamp[13] = __builtin_amdgcn_s_memtime();
    stamp[15] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && (blockIdx.x * W64_NW + wave) < 4096)
        for (int i = 0; i < 16; i++)
            g_diag_w64[(blockIdx.x * W64_NW + wave) * 16 + i] = stamp[i];
#endif
#undef W64_MARK
}

#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch_w64(unsigned long long *host, int n)
{
    if (n > (1 << 16))
        n = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_w64), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif

// --------------------------------------------------------------- host side
namespace {
constexpr size_t w64_lds(int U)
{
    return (void)U, (size_t)W64_LDS_BYTES;
}
}  // namespace

// LDS table image of k_p1k_w64 (layout of the kernel's shared memory after the
// tiles); twiddles rounded once from double
void tdoa_p1k_w64_image(int M, int N, int K, int U, const int32_t *win, const float *prior, const uint32_t *tuples,
                        std::vector<uint8_t> &img)
{
    img.clear();
    if (M != 3 || N != 1024 || K > W64_KPAD - 1)
        return;
    const int Upad = (U + W64_GB * 64 - 1) / (W64_GB * 64) * (W64_GB * 64);
    img.resize((size_t)IMG_FIXED + (size_t)Upad * 4, 0);
    auto put = [&](int off, int idx, double re, double im) {
        float *p = (float *)(img.data() + off) + 2 * idx;
        p[0] = (float)re;
        p[1] = (float)im;
    };
    auto w = [](long num, long den, double &re, double &im) {  // e^{-2 pi i num / den}
        const long e = ((num % den) + den) % den;
        const double a = -2.0 * M_PI * (double)e / (double)den;
        re = std::cos(a);
        im = std::sin(a);
    };
    double re, im;
    for (int a = 0; a < 16; a++)
        for (int L = 0; L < 64; L++) {
            w((long)a * w64_res(L), 1024, re, im);
            put(IMG_TW, 64 * a + L, re, im);
        }
    for (int k = 0; k < 8; k++)
        for (int L = 0; L < 64; L++) {
            w(w64_res(L) + 64 * k, 2048, re, im);
            put(IMG_TW2, 64 * k + L, re, im);
        }
    for (int t = 0; t < 8; t++)
        for (int L = 0; L < 64; L++) {
            const int wd = L + 64 * t;
            put(IMG_WIN, 64 * t + L, (double)((float)win[2 * wd] * (1.0f / 128.0f)),
                (double)((float)win[2 * wd + 1] * (1.0f / 128.0f)));
        }
    for (int g = 0; g < 4; g++)
        for (int b = 1; b < 4; b++)
            for (int q = 0; q < 4; q++) {
                w((long)b * (g + 4 * q), 64, re, im);
                put(IMG_T1, 4 * (3 * g + b - 1) + q, re, im);
            }
    for (int l0 = 0; l0 < 4; l0++) {
        w(-l0, 64, re, im);
        put(IMG_FI, l0, re, im);
        w(2 * l0, 64, re, im);
        put(IMG_FI, 4 + l0, re, im);
        w(l0, 64, re, im);
        put(IMG_FI, 8 + l0, re, im);
    }
    float *pr = (float *)(img.data() + IMG_PRIOR);
    for (int k = 0; k < 128; k++)
        pr[k] = k < K ? prior[k] : 0.0f;
    uint32_t *li = (uint32_t *)(img.data() + IMG_LANE);
    for (int L = 0; L < 64; L++) {
        li[2 * L] = w64_lane_info(L, 0);
        li[2 * L + 1] = w64_lane_info(L, 1);
    }
    uint32_t *t = (uint32_t *)(img.data() + IMG_FIXED);
    // tuples as byte offsets into a wave's [p][KPAD] f32 table, 10 bits per
    // pair; padding tuple (127, 127, 127) scores -inf
    for (int e = 0; e < Upad; e++) {
        const uint32_t wd = e < U ? tuples[e] : 0x007F7F7Fu;
        const int sh = W64_PAIR ? 3 : 2;  // byte offsets of f2 (paired) / f32 slots
        t[e] = ((wd & 0xFFu) << sh) | (((wd >> 8) & 0xFFu) << (10 + sh)) | (((wd >> 16) & 0xFFu) << (20 + sh));
    }
}

bool tdoa_p1k_w64_fits(const tdoa_kparams &kp)
{
    if (kp.M != 3 || kp.N != 1024 || kp.S > 63 || kp.TW != 1 || !kp.w64_img)
        return false;
    static_assert(3 * W64_KPAD * 4 <= W64_TILE, "grid scores exceed the wave's tile");
    const int Upad = (kp.U + W64_GB * 64 - 1) / (W64_GB * 64) * (W64_GB * 64);
    return Upad <= W64_UMAX && w64_lds(kp.U) <= 160 * 1024 && kp.w64_img_bytes <= 2 * W64_NW * 64 * 16;
}

int tdoa_launch_p1k_w64(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames, int64_t B,
                        float phat_eps, void *stream)
{
    float e2 = phat_eps * 4294967296.0f;  // as tdoa_launch_phat1024
    if (!(e2 >= 1e-30f))
        e2 = 1e-30f;
    if (B <= 0)
        return 0;
    const int64_t grid = (B + W64_NW - 1) / W64_NW;
    if (grid > 0x7FFFFFFF)
        return tdoa_set_error(-1, "k_p1k_w64: batch too large for one launch");
    hipLaunchKernelGGL(k_p1k_w64, dim3((unsigned)grid), dim3(W64_NW * 64), 0, (hipStream_t)stream, kp,
                       out, frames, B, e2);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char buf[256];
        snprintf(buf, sizeof buf, "k_p1k_w64 launch: %s", hipGetErrorString(e));
        return tdoa_set_error(-2, buf);
    }
    return 0;
}
