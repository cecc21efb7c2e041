// tdoa_phat1024.hip -- GCC-PHAT metric kernel for BASELINE config 2
// (3 mics x 1024-sample frames, L = 2048), see DESIGN.md "k_phat1024".
//
// One frame per 32-lane half-wave; the three mics of the frame run in the same
// lanes, so no spectrum ever crosses a wave and the kernel has no workgroup
// barrier after the table staging.  The work of a frame is issued as two
// independent FFT streams at a time (mic 0 | mic 1, pair (0,1) inverse | mic 2
// forward, pair (0,2) | pair (1,2)), each with its own transpose tile, so one
// wave per SIMD has the instruction-level parallelism to cover LDS latency.
//
// Per mic m (rolling_buffer.c:64-66, buffer.c:13-16, buffer.c:4-11 front end):
//   z[n] = x[2n] + i x[2n+1]  (n < 512; the upper half is the zero padding)
//   Z = FFT_1024(z) as 32 x 32: DFT-32 over n1 in registers (lane = residue
//       column n2 = res(lane)), twiddle W_1024^{n2 k1}, transpose through a
//       private padded LDS tile (row stride 264 B, residues 16 and 24 in
//       swapped slots: b64 writes and reads bank-conflict free), DFT-32 over n2.
//       Lane l then holds Z[res + 32 k2], k2 = 0..31.
//   Real-FFT split X[b] (b <-> N - b): lanes l, l^1 hold the partner residues
//       res, 32 - res; they swap their upper 16 registers by DPP so that the
//       partner of register k is register 31 - k in the same lane (lane 0 --
//       residue 0, self-paired with two fixed points 0 and 512 -- rotates its
//       upper half instead and keeps bin 512 in a 33rd register; lane 1 --
//       residue 16, self-paired -- keeps its registers).
//   PHAT factored per mic: U_m = X_m / max(|X_m|, sqrt(e)), so
//       R_ij = conj(U_i) U_j is the unit cross-spectrum.  Equal to the oracle's
//       R / max(|R|, eps) whenever |X_i|, |X_j| >= sqrt(eps) (every nonzero bin
//       of an integer frame in practice; an all-zero bin gives 0 either way).
// Per pair (0,1), (0,2), (1,2) (sample_compute.h:120-122 order):
//   Y[b] = (R[b] + R*[N-b]) + i (R[b] - R*[N-b]) W_2048^{-b}   (in-lane pairs)
//   swap back to residue columns, y = IFFT_1024(Y) pruned to the outputs
//   n = n1 (+992) that hold lags -S..S, argmax + lag prior (correlations.c:20-33
//   semantics on float scores), gate (sample_compute.h:124-134).
// Per wave and two iterations: the grid solve of vga_heatmap.h:99-108 for its
// four frames at once (lanes split the distinct lag tuples, one b128 gather per
// pair reads the four frames' weighted scores).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <type_traits>
#include <vector>

#include "tdoa_cplx.h"
#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);

namespace {

constexpr int P1K_ROW = 264;              // tile row stride, bytes (32 complex + 8 B pad)
constexpr int P1K_TILE = 32 * P1K_ROW;    // 8448 B: one transpose of one half-wave
constexpr int P1K_KPAD = 128;             // lag slots per pair in the grid score table
constexpr int P1K_WAVE_LDS = 2 * P1K_TILE;  // a wave's two transpose tiles (one per half-wave)
[[maybe_unused]] constexpr int P1K_GB = 8;               // grid tuples per lane per batch
// LDS table image: twm [32][32] f2 | tw2 [16][32] f2 | win [512] f2 | prior [128] | tuples
constexpr int P1K_IMG_FIXED = 32 * 32 * 8 + 16 * 32 * 8 + 512 * 8 + 128 * 4;

// Tile row / column and table column of residue (or DFT index) x: 16 and 24
// swap places, so the residues of every 16-lane group of a half-wave --
// {0, 16, 1, 31, .., 7, 25} and {8, 24, 9, 23, .., 15, 17} -- fall on distinct
// 8-B bank slots mod 16: the transposes' ds_write_b64 / ds_read2_b64 and the
// table reads (bank = dword mod 32) are conflict-free (plain order: 2-way).
__host__ __device__ constexpr int slot(int x) { return x == 16 ? 24 : (x == 24 ? 16 : x); }

// residue column held by lane l of a half-wave: lanes (2j, 2j+1) hold the
// partner residues (j, 32 - j); lanes 0, 1 the self-paired residues 0, 16
__device__ __forceinline__ int lane_res(int l)
{
    return l < 2 ? l * 16 : ((l & 1) ? 32 - (l >> 1) : (l >> 1));
}

__device__ __forceinline__ float dpp_xor1(float v)
{
    return __builtin_bit_cast(
        float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ f2 dpp_xor1(f2 v) { return f2{dpp_xor1(v.x), dpp_xor1(v.y)}; }
typedef short v2s_t __attribute__((ext_vector_type(2)));

// Partner swap of the upper 16 bins (registers 16..31), exec-masked instead of
// two selects per dword: lanes other than 0, 1 (of each half-wave) take their
// DPP partner's register in place (one instruction per dword); lane 0 then
// shifts its own upper half by one register (FWD: V[j] <- V[j+1], V[31] <- V[0];
// !FWD: V[j] <- V[j-1], V[16] <- E) in 64-bit moves; lane 1 keeps its registers.
// Wait states inside the strings: 2 before a DPP reads a VGPR a VALU wrote
// (s_nop 1; the compiler pads only its own boundary), and a conservative
// s_nop 4 after each EXEC write ahead of a DPP / VALU.
#define P1K_X(i) "%" #i
#define P1K_DPP(i) "v_mov_b32_dpp " P1K_X(i) ", " P1K_X(i) " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define P1K_MOV(d, s) "v_mov_b64 " P1K_X(d) ", " P1K_X(s) "\n\t"
template <bool FWD, int NV>
__device__ __forceinline__ void swap_upper_exec(f2 (&V)[NV], f2 E)
{
    float x[32];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        x[2 * j] = V[16 + j].x;
        x[2 * j + 1] = V[16 + j].y;
    }
    uint64_t sv;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_and_b64 exec, exec, %[m1]\n\t"
                 "s_nop 4\n\t" P1K_DPP(0) P1K_DPP(1) P1K_DPP(2) P1K_DPP(3) P1K_DPP(4) P1K_DPP(5)
                     P1K_DPP(6) P1K_DPP(7) P1K_DPP(8) P1K_DPP(9) P1K_DPP(10) P1K_DPP(11) P1K_DPP(12)
                         P1K_DPP(13) P1K_DPP(14) P1K_DPP(15) P1K_DPP(16) P1K_DPP(17) P1K_DPP(18)
                             P1K_DPP(19) P1K_DPP(20) P1K_DPP(21) P1K_DPP(22) P1K_DPP(23) P1K_DPP(24)
                                 P1K_DPP(25) P1K_DPP(26) P1K_DPP(27) P1K_DPP(28) P1K_DPP(29)
                                     P1K_DPP(30) P1K_DPP(31) "s_mov_b64 exec, %[sv]\n\t"
                 "s_nop 4"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                   "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]),
                   "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]), "+v"(x[16]), "+v"(x[17]),
                   "+v"(x[18]), "+v"(x[19]), "+v"(x[20]), "+v"(x[21]), "+v"(x[22]), "+v"(x[23]),
                   "+v"(x[24]), "+v"(x[25]), "+v"(x[26]), "+v"(x[27]), "+v"(x[28]), "+v"(x[29]),
                   "+v"(x[30]), "+v"(x[31]), [sv] "=&s"(sv)
                 : [m1] "s"(0xFFFFFFFCFFFFFFFCull));
    f2 y[16];
#pragma unroll
    for (int j = 0; j < 16; j++)
        y[j] = f2{x[2 * j], x[2 * j + 1]};
    const f2 e = FWD ? V[0] : E;
#define P1K_ROT_ASM(ROT)                                                                            \
    asm volatile("s_mov_b64 %[sv], exec\n\t"                                                        \
                 "s_and_b64 exec, exec, %[m2]\n\t"                                                  \
                 "s_nop 4\n\t" ROT "s_mov_b64 exec, %[sv]\n\t"                                     \
                 "s_nop 4"                                                                           \
                 : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]),           \
                   "+v"(y[6]), "+v"(y[7]), "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]),         \
                   "+v"(y[12]), "+v"(y[13]), "+v"(y[14]), "+v"(y[15]), [sv] "=&s"(sv)                \
                 : [m2] "s"(0x0000000100000001ull), [e] "v"(e))
    if constexpr (FWD)
        P1K_ROT_ASM(P1K_MOV(0, 1) P1K_MOV(1, 2) P1K_MOV(2, 3) P1K_MOV(3, 4) P1K_MOV(4, 5) P1K_MOV(5, 6)
                        P1K_MOV(6, 7) P1K_MOV(7, 8) P1K_MOV(8, 9) P1K_MOV(9, 10) P1K_MOV(10, 11)
                            P1K_MOV(11, 12) P1K_MOV(12, 13) P1K_MOV(13, 14) P1K_MOV(14, 15)
                                "v_mov_b64 %15, %[e]\n\t");
    else
        P1K_ROT_ASM(P1K_MOV(15, 14) P1K_MOV(14, 13) P1K_MOV(13, 12) P1K_MOV(12, 11) P1K_MOV(11, 10)
                        P1K_MOV(10, 9) P1K_MOV(9, 8) P1K_MOV(8, 7) P1K_MOV(7, 6) P1K_MOV(6, 5)
                            P1K_MOV(5, 4) P1K_MOV(4, 3) P1K_MOV(3, 2) P1K_MOV(2, 1) P1K_MOV(1, 0)
                                "v_mov_b64 %0, %[e]\n\t");
#undef P1K_ROT_ASM
#pragma unroll
    for (int j = 0; j < 16; j++)
        V[16 + j] = y[j];
}

// sum over the 32 lanes of each half-wave, VALU only (no LDS queue): row
// all-reduce by DPP, row_bcast:15 into rows 1 and 3, then lanes 31 / 63
__device__ __forceinline__ int hsum32(int s, int hw)
{
    s += __builtin_amdgcn_mov_dpp(s, 0xB1, 0xF, 0xF, false);   // xor 1
    s += __builtin_amdgcn_mov_dpp(s, 0x4E, 0xF, 0xF, false);   // xor 2
    s += __builtin_amdgcn_mov_dpp(s, 0x141, 0xF, 0xF, false);  // half-row mirror
    s += __builtin_amdgcn_mov_dpp(s, 0x140, 0xF, 0xF, false);  // row mirror
    s += __builtin_amdgcn_update_dpp(0, s, 0x142, 0xA, 0xF, false);  // row_bcast:15
    const int s0 = __builtin_amdgcn_readlane(s, 31), s1 = __builtin_amdgcn_readlane(s, 63);
    return hw ? s1 : s0;
}

// LDS reads: volatile ds_read_b64 unless P1K_VLDS=0 (the backend otherwise
// merges neighbours into ds_read2_b64, twice the LDS cycles of two b64 reads)
#ifndef P1K_VLDS
#define P1K_VLDS 1
#endif
__device__ __forceinline__ f2 lds_f2(const char *base, int off)
{
#if P1K_VLDS
    return lds_rd(reinterpret_cast<const f2 *>(base + off));
#else
    return *reinterpret_cast<const f2 *>(base + off);
#endif
}
// the grid over tuples grouped by their first two lags (see the grid solve;
// A/B variant, not the default: 25 % fewer LDS instructions per wave, but the
// phase is latency-bound and the group's cell resolution adds ~1.9 k cycles,
// 31.0 vs 30.4 us per 4096 frames -- DESIGN.md "Measured negative results")
#ifndef P1K_GROUPS
#define P1K_GROUPS 0
#endif
// the winner's first cell from LDS (tuple words carry it; see the grid end).
// A/B variant, not the default: neutral (30.3 vs 30.35 us per 4096 frames) once
// the lag / gate stores moved behind the grid, and it needs every 32-tuple row
// to span < 2048 cells
#ifndef P1K_CELL_LDS
#define P1K_CELL_LDS 0
#endif
// the SIMD issue balance (s_setprio by phase progress; see the kernel).
// Without it (P1K_BALANCE=0): 31.8 vs 29.1 us per 4096 frames
#ifndef P1K_BALANCE
#define P1K_BALANCE 1
#endif
// mic 2's words requested inside mic 1's forward (as mic 1's inside mic 0's).
// A/B variant, not the default: 29.9 vs 29.1 us (the column pass of pair
// (0,1) then runs with 16 more live registers)
#ifndef P1K_W2_EARLY
#define P1K_W2_EARLY 0
#endif
// the frame's lag / gate stores after the grid (see store_frame)
#ifndef P1K_LATE_STORES
#define P1K_LATE_STORES 1
#endif
// plain LDS read (the grid's gathers: data-dependent addresses, never merged,
// and free to be scheduled around the other reads of the software pipeline)
__device__ __forceinline__ f2 lds_f2_plain(const char *base, int off)
{
    return *reinterpret_cast<const f2 *>(base + off);
}
// LDS read at a 32-bit LDS byte address
__device__ __forceinline__ f2 lds_at(uint32_t addr)
{
    return *(const __attribute__((address_space(3))) f2 *)(uintptr_t)addr;
}
__device__ __forceinline__ void sts_f2(char *base, int off, f2 v)
{
    *reinterpret_cast<f2 *>(base + off) = v;
}

// an empty asm that needs the value: it must be computed here (keeps IR
// passes from sinking a finished partial sum past later phases)
__device__ __forceinline__ void pin(f2 &x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ f2 unit(f2 x, float e2)
{
    return x * __builtin_amdgcn_rsqf(fmaxf(x.x * x.x + x.y * x.y, e2));
}


struct Lane {
    int hw;           // half-wave of the wave
    int lane;         // 0..31 within the half-wave
    int res;          // residue column
    int cs;           // its tile / table slot, slot(res)
    bool is0, is1;    // the self-paired lanes
    char *tileA;      // this half-wave's transpose tile
    const char *twm;  // [k][r] W_1024^{r k}
    const char *tw2;  // [k][r] W_2048^{r + 32 k}, k < 16
    const char *win;  // [w] (W[2w], W[2w+1]) / 128
};

// first half of a 32 x 32 FFT_1024 on a residue column: DFT-32 in registers,
// twiddle W_1024^{-+res k}, column write into the tile
// ... with the twiddles read from LDS in groups of 8 ahead of their writes
// (register-lean form for two waves per SIMD)
template <bool INV, bool HALF_ZERO>
__device__ __forceinline__ void fft_col_lds(const Lane &L, f2 (&v)[32], char *tile)
{
    fft32d<INV, HALF_ZERO>(v);
    wave_lds_sync();  // after the previous pass's row reads of this tile
    const int wo = 8 * L.cs;
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 8) {
        f2 tw[8];
#pragma unroll
        for (int i = 0; i < 8; i++)
            tw[i] = lds_f2(L.twm, wo + 256 * (k0 + i));
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int k = k0 + i;
            f2 x = v[k];
            if (k)
                x = INV ? c_mulconj(x, tw[i]) : c_mul(x, tw[i]);
            sts_f2(tile, wo + P1K_ROW * slot(k), x);
        }
    }
    wave_lds_sync();  // before the row reads of other lanes' columns
}
// second half: row read (row res) + forward DFT-32 -> V[k2] = Z[res + 32 k2]
__device__ __forceinline__ void fft_row_fwd(const Lane &L, const char *tile, f2 (&V)[33])
{
    f2 v[32];
    const int ro = P1K_ROW * L.cs;
#pragma unroll
    for (int n = 0; n < 32; n++)
        v[n] = lds_f2(tile, ro + 8 * slot(n));
    fft32d<false, false>(v);
#pragma unroll
    for (int k = 0; k < 32; k++)
        V[k] = v[k];
}
}  // namespace

#ifdef TDOA_DIAG
// diagnostic build only: per-wave phase stamps of k_p1k_lean
__device__ unsigned long long g_diag_p1k[1 << 16];
#endif

// ---------------------------------------------------------------------------
// k_p1k_lean: the same per-frame algorithm at TWO waves per SIMD (8 waves per
// workgroup, one workgroup per CU, <= 256 registers per lane).  One frame per
// half-wave and one FFT stream; the register plan keeps at most two unit
// spectra plus one working column live:
//   mic 0 -> U0, mic 1 -> U1, pair (0,1) built straight into the inverse's
//   column (no third spectrum), mic 2 -> V, U0 <- conj(U0) V, U1 <- conj(U1) V,
//   pairs (0,2), (1,2).
// Table values (window, twiddles) are read from LDS next to their use instead
// of as whole per-phase arrays.  The grid solve runs per iteration on the
// wave's two frames (b64 gathers of an [p][k] f2 score table).  The partner
// wave of the SIMD hides the LDS round trips that bound the one-wave kernel.
namespace {

// front end + forward FFT_1024 of one mic row, then the partner swap: V[k],
// V[31 - k] hold Z[b], Z[N - b] (paired layout); V[32] = unit X[512] (lane 0)
struct NoHook {
    __device__ void operator()() const {}
};

template <typename Hook = NoHook>
__device__ __forceinline__ void lean_spectrum(const Lane &L, const uint32_t (&w)[16], f2 (&V)[33],
                                              float e2, Hook after_front = Hook())
{
    f2 v[32];
    {
        int s = 0;
#pragma unroll
        for (int t = 0; t < 16; t++)
            s = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s_t, w[t]), v2s_t{1, 1}, s, false);
        s = hsum32(s, L.hw);
        const uint32_t off = (uint32_t)(s >> 10) & 0xFFu;
        const uint32_t off2 = off | (off << 16);
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const f2 wf = lds_f2(L.win, 8 * L.cs + 256 * t);
            const uint32_t d = (w[t] | 0x01000100u) - off2;
            const float s0 = (float)(int8_t)(d & 0xFFu);
            const float s1 = (float)(int8_t)((d >> 16) & 0xFFu);
            const f2 pr = f2{s0, s1} * wf;  // one packed multiply
            v[t] = f2{floorf(pr.x), floorf(pr.y)};
        }
    }
    after_front();  // the row's words are consumed
    fft_col_lds<false, true>(L, v, L.tileA);
    fft_row_fwd(L, L.tileA, V);
    V[32] = c_unit(conjf2(V[16]), e2);
    swap_upper_exec<true>(V, f2{0.0f, 0.0f});
}

// real-FFT split of the partner pair k + unit normalisation: the unit
// spectrum at bins b and N - b (the W_2048^b twiddle read next to its use)
__device__ __forceinline__ void lean_split_w(f2 A, f2 Bv, f2 wk, float e2, f2 &ub, f2 &un)
{
    const f2 e = c_addconj(A, Bv);
    const f2 od = c_mul(c_subconj(A, Bv), wk);
    ub = c_unit(c_add_mi(e, od), e2);
    un = c_unit(c_conj_add_i(e, od), e2);
}
// the W_2048^b twiddle of pair k (P1K_TWPF: requested one pair ahead of its
// use, so its LDS round trip overlaps the previous pair's arithmetic; read
// next to its use, each was a round trip of its own -- the inline-asm packed
// operations keep the backend from hoisting it)
#ifndef P1K_TWPF
#define P1K_TWPF 5  // bit 0: lean_forward, 1: lean_forward_cross, 2: lean_pretwiddle
#endif
__device__ __forceinline__ f2 lean_tw2(const Lane &L, int k) { return lds_f2(L.tw2, 8 * L.cs + 256 * k); }
__device__ __forceinline__ void lean_split(const Lane &L, f2 A, f2 Bv, int k, float e2, f2 &ub,
                                           f2 &un)
{
    lean_split_w(A, Bv, lean_tw2(L, k), e2, ub, un);
}

// unit spectrum of one mic row, in place (paired layout)
template <typename Hook = NoHook>
__device__ __forceinline__ void lean_forward(const Lane &L, const uint32_t (&w)[16], f2 (&U)[33],
                                             float e2, Hook after_front = Hook())
{
    lean_spectrum(L, w, U, e2, after_front);
#if P1K_TWPF & 1
    f2 wn = lean_tw2(L, 0);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const f2 wk = wn;
        if (k < 15)
            wn = lean_tw2(L, k + 1);
        lean_split_w(U[k], U[31 - k], wk, e2, U[k], U[31 - k]);
    }
#else
#pragma unroll
    for (int k = 0; k < 16; k++)
        lean_split(L, U[k], U[31 - k], k, e2, U[k], U[31 - k]);
#endif
}

// unit spectrum V of one mic row consumed bin pair by bin pair as it is
// produced: A <- conj(A) V, B <- conj(B) V (V is never whole after the split)
__device__ __forceinline__ void lean_forward_cross(const Lane &L, const uint32_t (&w)[16],
                                                   f2 (&A)[33], f2 (&Bs)[33], float e2)
{
    f2 V[33];
    lean_spectrum(L, w, V, e2);
    A[32] = c_conjmul(A[32], V[32]);
    Bs[32] = c_conjmul(Bs[32], V[32]);
#if P1K_TWPF & 2
    f2 wn = lean_tw2(L, 0);
#endif
#pragma unroll
    for (int k = 0; k < 16; k++) {
        f2 ub, un;
#if P1K_TWPF & 2
        const f2 wk = wn;
        if (k < 15)
            wn = lean_tw2(L, k + 1);
        lean_split_w(V[k], V[31 - k], wk, e2, ub, un);
#else
        lean_split(L, V[k], V[31 - k], k, e2, ub, un);
#endif
        A[k] = c_conjmul(A[k], ub);
        A[31 - k] = c_conjmul(A[31 - k], un);
        Bs[k] = c_conjmul(Bs[k], ub);
        Bs[31 - k] = c_conjmul(Bs[31 - k], un);
    }
}

// acc + d W_32^k (forward W), k compile-time after unrolling: two chained
// packed FMAs (one packed add for W = 1, -i)
__device__ __forceinline__ f2 cmac_fwd(f2 acc, f2 d, int k)
{
    if (k == 0)
        return acc + d;
    if (k == 8)
        return c_add_mi(acc, d);
    const f2 w = f2{(float)COS32D[k], -(float)COS32D[k < 8 ? 8 - k : k - 8]};
    return v_fma(v_yy(d), f2{-w.y, w.x}, v_fma(v_xx(d), w, acc));
}

// second half of the pruned inverse (fft_row_inv) in two groups of 8 residue
// pairs, so at most half a row of tile values is in registers at a time:
// y0 = sum of the row, y31 = sum_i (v_i - v_{i+16}) W_32^i accumulated by
// FMA in two chains per group
__device__ __forceinline__ void lean_row_inv(const Lane &L, const char *tile, f2 &y0, f2 &y31)
{
    const int ro = P1K_ROW * L.cs;
    f2 ga[2], gd[2];
#pragma unroll
    for (int g = 0; g < 2; g++) {
        f2 a[8], c[2];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const f2 v = lds_f2(tile, ro + 8 * slot(8 * g + i));
            const f2 u = lds_f2(tile, ro + 8 * slot(8 * g + i + 16));
            a[i] = v + u;
            const f2 d = v - u;
            c[i & 1] = i < 2 ? tw_only<false>(d, 8 * g + i) : cmac_fwd(c[i & 1], d, 8 * g + i);
        }
#pragma unroll
        for (int h = 4; h >= 1; h >>= 1)
#pragma unroll
            for (int r = 0; r < h; r++)
                a[r] = a[r] + a[r + h];
        ga[g] = a[0];
        gd[g] = c[0] + c[1];
        pin(ga[g]);
        pin(gd[g]);
    }
    y0 = ga[0] + ga[1];
    y31 = gd[0] + gd[1];
}

// residue of lane l (lane_res) in plain arithmetic (no divergent branch)
__device__ __forceinline__ int lane_res_sel(int l)
{
    const int h = l >> 1, o = l & 1;
    return h + o * (32 - 2 * h) - ((l == 1) << 4);
}


// the lane id through an opaque move: lane-dependent values derived from it
// are computed where they are used instead of being hoisted to the kernel's
// start and held in registers across every phase
__device__ __forceinline__ int fresh_tid()
{
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// packed inverse input of the cross spectrum R (paired layout; R[k] =
// conj(A[k]) B[k] when B is given, else R = A), back in residue columns
template <bool CROSS>
__device__ __forceinline__ void lean_pretwiddle(const Lane &L, const f2 (&A)[33], const f2 (&Bs)[33],
                                                f2 (&v)[32])
{
#if P1K_TWPF & 4
    f2 wn = lean_tw2(L, 0);
#endif
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const f2 Rk = CROSS ? c_conjmul(A[k], Bs[k]) : A[k];
        const f2 Rn = CROSS ? c_conjmul(A[31 - k], Bs[31 - k]) : A[31 - k];
#if P1K_TWPF & 4
        const f2 wk = wn;
        if (k < 15)
            wn = lean_tw2(L, k + 1);
#else
        const f2 wk = lean_tw2(L, k);
#endif
        const f2 s = c_addconj(Rk, Rn);
        const f2 q = c_mulconj(c_subconj(Rk, Rn), wk);
        v[k] = c_add_i(s, q);
        v[31 - k] = c_conj_add_mi(s, q);
    }
    const f2 R32 = CROSS ? c_conjmul(A[32], Bs[32]) : A[32];
    const f2 Ye = f2{2.0f * R32.x, -2.0f * R32.y};  // Y[512] = 2 conj(R[512])
    swap_upper_exec<false>(v, Ye);
}

}  // namespace

__global__ void __launch_bounds__(512, 2) k_p1k_lean(tdoa_kparams kp, tdoa_kout out,
                                                     const int16_t *__restrict__ frames, int64_t B,
                                                     float e2)
{
    constexpr int N = 1024, P = 3, NW = 8, NF = 2 * NW, NT = NW * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *tiles = smem;                               // [NW][2][TILE]
    char *twm = tiles + NW * 2 * P1K_TILE;            // [32][32] f2
    char *tw2 = twm + 32 * 32 * 8;                    // [16][32] f2
    char *win = tw2 + 16 * 32 * 8;                    // [512] f2
    const float *prior = (const float *)(win + 512 * 8);  // [128]
    const uint32_t *tups = (const uint32_t *)(prior + 128);

    const int tid = threadIdx.x, wave = tid >> 6, hw = (tid >> 5) & 1, lane64 = tid & 63;
#ifdef TDOA_DIAG
    // diagnostic build only: absolute s_memtime per phase of the first iteration
    unsigned long long stamp[16] = {};
    int nst = 0;
#define LEAN_MARK()                                               \
    do {                                                          \
        if (nst < 16)                                             \
            stamp[nst++] = __builtin_amdgcn_s_memtime();          \
    } while (0)
    stamp[nst++] = __builtin_amdgcn_s_memtime();
    stamp[14] = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
#else
#define LEAN_MARK() \
    do {            \
    } while (0)
#endif
    // issue balance between the two waves of a SIMD (waves w and w ^ 4: a
    // workgroup's waves are dealt to the CU's four SIMDs in turn).  The SIMD
    // issues oldest-first, so without this wave w runs ahead and wave w ^ 4
    // finishes its last ~9 us alone, with nothing to hide its latencies; here
    // a wave that has passed more phase boundaries than its partner drops to
    // the low priority until the partner catches up
    __shared__ int prog[NW];
    if (lane64 == 0)
        prog[wave] = 0;
    __builtin_amdgcn_s_setprio(2);
    int phase = 0;
    auto balance = [&]() {
        // through an LDS-address-space pointer: ds_write / ds_read.  A generic
        // volatile pointer made them flat accesses, and the flat load's wait
        // (vmcnt(0) lgkmcnt(0)) also waited for the next mic's words in flight
#if P1K_BALANCE
        volatile __attribute__((address_space(3))) int *pv = (volatile __attribute__((address_space(3))) int *)prog;
        ++phase;
        if (lane64 == 0)
            pv[wave] = phase;
        const int other = __builtin_amdgcn_readfirstlane(pv[wave ^ 4]);
        if (phase > other)
            __builtin_amdgcn_s_setprio(0);
        else
            __builtin_amdgcn_s_setprio(2);
#endif
    };
    Lane L;
    L.hw = hw;
    L.lane = tid & 31;
    L.res = lane_res(L.lane);
    L.cs = slot(L.res);
    L.is0 = L.lane == 0;
    L.is1 = L.lane == 1;
    char *wtiles = tiles + wave * 2 * P1K_TILE;
    L.tileA = wtiles + hw * P1K_TILE;
    L.twm = twm;
    L.tw2 = tw2;
    L.win = win;

    const int K = kp.K, S = kp.S;
    const bool do_grid = out.cell || out.xy || out.max_Lf;
#if !P1K_GROUPS
    const int Upad = (kp.U + P1K_GB * 64 - 1) / (P1K_GB * 64) * (P1K_GB * 64);
#endif

    auto fetch = [&](uint32_t(&w)[16], int64_t fr, int m) {
        const uint32_t *row = reinterpret_cast<const uint32_t *>(
            frames + ((fr < B ? fr : B - 1) * 3 + m) * (int64_t)N) + L.res;
#pragma unroll
        for (int t = 0; t < 16; t++)
            w[t] = __builtin_nontemporal_load(row + 32 * t);
    };
    // table image: its loads first (L2 hits), then the first frames' words
    // (HBM), then the image's LDS writes -- the frames' latency overlaps the
    // staging instead of following it
    uint32_t w0[16], w1[16];
    {
        const uint4 *src = (const uint4 *)kp.p1k_img;
        uint4 *dst = (uint4 *)twm;
        const int n16 = do_grid ? kp.p1k_img_bytes / 16 : P1K_IMG_FIXED / 16;
        constexpr int SR = 4;  // image <= SR * NT * 16 B = 32 KiB (tdoa_phat1024_fits)
        uint4 img[SR];
#pragma unroll
        for (int r = 0; r < SR; r++)  // unconditional (clamped) loads: straight-line
            img[r] = src[tid + r * NT < n16 ? tid + r * NT : n16 - 1];  // code, counted waits
        const int64_t f = (int64_t)blockIdx.x * NF + 2 * wave + hw;
        fetch(w0, f, 0);
#pragma unroll
        for (int r = 0; r < SR; r++)  // unconditional too (a clamped index rewrites
            dst[tid + r * NT < n16 ? tid + r * NT : n16 - 1] = img[r];  // the last unit)
    }
    __syncthreads();
    // keep the first row's use (and its wait) below the barrier: hoisted above
    // it, every wave of the workgroup would wait for the latest wave's row
#pragma unroll
    for (int t = 0; t < 16; t++)
        asm volatile("" : "+v"(w0[t]));

    const float invL = 1.0f / 2048.0f;

    // one iteration per workgroup (grid = ceil(B / 16)): no value lives across
    // a loop back-edge, which the register allocator answered with spills
    {
        const int64_t base = (int64_t)blockIdx.x * NF;
        const int64_t f = base + 2 * wave + hw;
        const bool live = f < B;
        uint32_t w2[16];
        LEAN_MARK();
        float wv[3][4];
        int best[3];
        auto finish_pair = [&](int p, f2 y0, f2 y31) {
            // this lane's four candidate lags (recomputed here, see fresh_tid)
            const int ft = fresh_tid();
            const int fres = lane_res_sel(ft & 31), fhw = (ft >> 5) & 1;
            const int la = 2 * fres, lb = 2 * fres - 64;
            const int ck[4] = {lb + S, lb + 1 + S, la + S, la + 1 + S};
            const bool ok[4] = {lb >= -S, lb + 1 >= -S, la <= S, la + 1 <= S};
            const float cv[4] = {y31.x * invL, y31.y * invL, y0.x * invL, y0.y * invL};
            // the lane's first maximum of its candidates (ascending lags), then
            // the half-wave's (correlations.c:20-23 first max) by keys
            int bkey = INT_MIN, bk = INT_MAX;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int kc = fkey(cv[c]);
                if (ok[c] && kc > bkey) {
                    bkey = kc;
                    bk = ck[c];
                }
            }
            half_argmax_key(bkey, bk);  // every lane of the half-wave
            bk = bk < 0 ? 0 : (bk >= K ? K - 1 : bk);
            best[p] = bk - S;
            const int64_t ff = base + 2 * ((ft >> 6) & 7) + fhw;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int d = ck[c] > bk ? ck[c] - bk : bk - ck[c];
                wv[p][c] = ok[c] ? cv[c] * prior[ok[c] ? d : 0] : 0.0f;
            }
            if (out.scores_f || out.weighted_f) {  // debug / parity outputs (uniform branch)
                float *sr = out.scores_f ? out.scores_f + (size_t)(ff * P + p) * K : nullptr;
                float *wr = out.weighted_f ? out.weighted_f + (size_t)(ff * P + p) * K : nullptr;
#pragma unroll
                for (int c = 0; c < 4; c++)
                    if (ff < B && ok[c]) {
                        if (sr)
                            sr[ck[c]] = cv[c];
                        if (wr)
                            wr[ck[c]] = wv[p][c];
                    }
            }
#if !P1K_LATE_STORES
            if (ff < B && (ft & 31) == 0)
                out.lags[ff * P + p] = bk - S;
#endif
        };

        f2 U0[33], U1[33], y0, y31;
        // the mics' rows are requested one at a time, each after the previous
        // one's front end: at the kernel's start the memory system serves every
        // wave's first row (8 MB) instead of all rows at once
        lean_forward(L, w0, U0, e2, [&] {
            fetch(w1, f, 1);
            balance();
        });
        LEAN_MARK();
        balance();
#if P1K_W2_EARLY
        lean_forward(L, w1, U1, e2, [&] {
            fetch(w2, f, 2);
            balance();
        });
#else
        lean_forward(L, w1, U1, e2, [&] { balance(); });
#endif
        LEAN_MARK();
        balance();
        {
            f2 v[32];
            lean_pretwiddle<true>(L, U0, U1, v);  // pair 0: (0, 1)
            fft_col_lds<true, false>(L, v, L.tileA);
#if !P1K_W2_EARLY
            // mic 2's words: fetched after the pair's column pass, the kernel's
            // register peak (two unit spectra + a working column)
            fetch(w2, f, 2);
#endif
            lean_row_inv(L, L.tileA, y0, y31);
        }
        finish_pair(0, y0, y31);
        LEAN_MARK();
        balance();
        lean_forward_cross(L, w2, U0, U1, e2);  // pairs 1: (0, 2), 2: (1, 2)
        LEAN_MARK();
        balance();
        {
            f2 v[32];
            lean_pretwiddle<false>(L, U0, U0, v);
            fft_col_lds<true, false>(L, v, L.tileA);
            lean_row_inv(L, L.tileA, y0, y31);
        }
        finish_pair(1, y0, y31);
        LEAN_MARK();
        balance();
        {
            f2 v[32];
            lean_pretwiddle<false>(L, U1, U1, v);
            fft_col_lds<true, false>(L, v, L.tileA);
            lean_row_inv(L, L.tileA, y0, y31);
        }
        finish_pair(2, y0, y31);
        LEAN_MARK();
        balance();
        // the frame's lags and gate (sample_compute.h:124-134): stored last
        // unless P1K_LATE_STORES=0.  gfx9's vmcnt counts stores too, and the
        // grid's one global load (the winner's first cell) waits in issue
        // order: behind these stores it waited for their HBM write acks
        auto store_frame = [&]() {
            if (live && L.lane == 0) {
#pragma unroll
                for (int p = 0; p < 3; p++)
                    out.lags[f * P + p] = best[p];
                if (out.gate)
                    out.gate[f] = best[0] * best[0] + best[1] * best[1] + best[2] * best[2] > 4 ? 1 : 0;
            }
        };
#if !P1K_LATE_STORES
        store_frame();
#endif
        if (!do_grid) {
#if P1K_LATE_STORES
            store_frame();
#endif
            return;
        }
        // ---- grid solve (vga_heatmap.h:99-108) of the wave's two frames:
        // weighted scores [p][KPAD] f2 (frame hw in component hw) in the wave's
        // tile space, lanes split the distinct lag tuples (4 consecutive per
        // lane and step, ascending: a strict '>' keeps the first maximum)
        wave_lds_sync();  // after the last pair's row reads of these tiles
#if P1K_CELL_LDS && !P1K_GROUPS
        // [P][KPAD][2], 1 KiB-aligned in the wave's tiles: a gather address is
        // then one and-or of a tuple field with the table base
        float *wsc = (float *)(((uintptr_t)wtiles + 1023) & ~(uintptr_t)1023);
#else
        float *wsc = (float *)wtiles;  // [P][KPAD][2]
#endif
        const int gres = lane_res_sel(fresh_tid() & 31);
        const int gla = 2 * gres, glb = 2 * gres - 64;
        const int ck[4] = {glb + S, glb + 1 + S, gla + S, gla + 1 + S};
        const bool ok[4] = {glb >= -S, glb + 1 >= -S, gla <= S, gla + 1 <= S};
#pragma unroll
        for (int p = 0; p < P; p++)
#pragma unroll
            for (int c = 0; c < 4; c++)
                if (ok[c])
                    wsc[(p * P1K_KPAD + ck[c]) * 2 + hw] = wv[p][c];
        {
            const int ft = fresh_tid();  // (lane, half-wave) not held across the phases
            if ((ft & 31) < 3)  // lag slot 127 of every pair: the padding tuple
                wsc[((ft & 31) * P1K_KPAD + P1K_KPAD - 1) * 2 + ((ft >> 5) & 1)] = -INFINITY;
        }
        wave_lds_sync();  // the gathers read other lanes' score slots
        LEAN_MARK();
#if P1K_GROUPS
        // Tuples grouped by their first two lags (tdoa_phat1024_image): a
        // group word holds the LDS offsets of lags l0, l1 and the first of n
        // consecutive l2 (n = 3, 2, 1 by bucket), so a group costs 2 + n score
        // gathers for its n tuples instead of 3 n, and (w0 + w1) is formed once
        // -- the same association as ((w0 + w1) + w2), so the same floats.
        // A lane keeps per frame the largest group maximum and its slot (strict
        // '>', one compare per group instead of per tuple) and flags a tie with
        // its running maximum.  At the end each lane re-reads its best group
        // and takes the smallest first cell among the members equal to the
        // maximum; the wave reduces (L, cell) -- the smallest cell among maxima
        // is the first tuple (tuples are in first-cell order).  A lane whose
        // maximum tied another of its groups rescans everything (rare: flat or
        // equal scores).  Bucket sizes and tuple 0's cell: the image header,
        // read as scalars from the global image.
        const int *ghdr = reinterpret_cast<const int *>(static_cast<const char *>(kp.p1k_img) + P1K_IMG_FIXED);
        const int gn3 = ghdr[0], gn2 = ghdr[1], gn1 = ghdr[2], gcell0 = ghdr[3];
        const uint32_t *gw = tups + 4;
        const uint16_t *gcl = reinterpret_cast<const uint16_t *>(gw + gn3 + gn2 + gn1);
        const int gcb2 = 3 * gn3, gcb1 = gcb2 + 2 * gn2, gend = gn3 + gn2 + gn1;
        // per frame: the largest group maximum, the first slot that reached it
        // (strict '>') and the last slot that matched it ('>='); they differ
        // exactly when a later group tied the maximum
        float gv[2] = {-INFINITY, -INFINITY};
        int gs[2] = {0, 0}, gsl[2] = {0, 0};
        const char *ws = (const char *)wsc;
        constexpr int R1 = P1K_KPAD * 8, R2 = 2 * P1K_KPAD * 8;
        // volatile LDS reads: issued in program order, so the pipeline below is
        // the one the hardware sees (the scheduler otherwise sank each step's
        // word read to just before its gathers, and waited on it there)
        auto gat = [&](auto nm, uint32_t w, f2 &a, f2 &b, f2 (&c)[decltype(nm)::value]) {
            a = lds_rd(reinterpret_cast<const f2 *>(ws + (w & 0x3FFu)));
            b = lds_rd(reinterpret_cast<const f2 *>(ws + R1 + ((w >> 10) & 0x3FFu)));
#pragma unroll
            for (int j = 0; j < decltype(nm)::value; j++)
                c[j] = lds_rd(reinterpret_cast<const f2 *>(ws + R2 + (w >> 20) + 8 * j));
        };
        // one bucket of groups of NM tuples: slots [s0, s1), an even number of
        // 64-slot rows, taken two rows (a unit) at a time.  Software-pipelined
        // over two register sets (no copies, which would wait for the loads):
        // while unit u is compared, unit u+1's 2 (2 + NM) gathers are in flight,
        // and every word is read before the gathers issued ahead of its own, so
        // that waiting for it (LDS returns in order) never waits for those
        auto bucket = [&](auto nm, int s0, int s1) {
            constexpr int NM = decltype(nm)::value;
            if (s0 >= s1)
                return;
            const int last = s1 - 64;  // (clamped units past the end: harmless re-reads)
            const int nu = (s1 - s0) / 128;
            auto words = [&](uint32_t (&w)[2], int u) {
                w[0] = lds_rd_u32(gw + imin(s0 + 128 * u, last) + lane64);
                w[1] = lds_rd_u32(gw + imin(s0 + 128 * u + 64, last) + lane64);
            };
            auto gather = [&](const uint32_t (&w)[2], f2 (&a)[2], f2 (&b)[2], f2 (&c)[2][NM]) {
                gat(nm, w[0], a[0], b[0], c[0]);
                gat(nm, w[1], a[1], b[1], c[1]);
            };
            auto consume = [&](const f2 (&a)[2], const f2 (&b)[2], const f2 (&c)[2][NM], int u) {
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    const f2 part = a[r] + b[r];
                    f2 L[NM];
#pragma unroll
                    for (int j = 0; j < NM; j++)
                        L[j] = part + c[r][j];
                    float m[2] = {L[0].x, L[0].y};
#pragma unroll
                    for (int j = 1; j < NM; j++) {
                        m[0] = fmaxf(m[0], L[j].x);
                        m[1] = fmaxf(m[1], L[j].y);
                    }
                    const int sl = s0 + 128 * u + 64 * r + lane64;
#pragma unroll
                    for (int f = 0; f < 2; f++) {
                        const bool gt = m[f] > gv[f];
                        gsl[f] = m[f] >= gv[f] ? sl : gsl[f];
                        gs[f] = gt ? sl : gs[f];
                        gv[f] = gt ? m[f] : gv[f];
                    }
                }
            };
            f2 a0[2], b0[2], c0[2][NM], a1[2], b1[2], c1[2][NM];
            uint32_t w2[2], w3[2];
            // (the prologue leaves the loads in the loop's own order -- unit 0,
            // then the words of unit 2, then unit 1 -- so the wait counts at the
            // loop head are the steady state's, not a full drain)
            words(w2, 0);
            gather(w2, a0, b0, c0);
            words(w3, 1);
            words(w2, 2);
            gather(w3, a1, b1, c1);
            // whole pairs of units whose loads stay inside the bucket, in a
            // branch-free body (a branch inside made the wait-count pass drain
            // every load at the loop head; scheduling barriers: the scheduler
            // hoisted unit u+1's sums above unit u+2's gathers, the same drain)
            int u = 0;
            for (; u + 3 < nu; u += 2) {
                consume(a0, b0, c0, u);
                words(w3, u + 3);
                gather(w2, a0, b0, c0);
                __builtin_amdgcn_sched_barrier(0);
                consume(a1, b1, c1, u + 1);
                words(w2, u + 4);
                gather(w3, a1, b1, c1);
                __builtin_amdgcn_sched_barrier(0);
            }
            // the last one to three units, none loaded past the end
            consume(a0, b0, c0, u);
            if (u + 2 < nu)
                gather(w2, a0, b0, c0);
            if (u + 1 < nu)
                consume(a1, b1, c1, u + 1);
            if (u + 2 < nu)
                consume(a0, b0, c0, u + 2);
        };
        bucket(std::integral_constant<int, 3>{}, 0, gn3);
        bucket(std::integral_constant<int, 2>{}, gn3, gn3 + gn2);
        bucket(std::integral_constant<int, 1>{}, gn3 + gn2, gend);
        LEAN_MARK();
        // smallest first cell among the members of group slot sl whose L (frame
        // f) equals v; INT_MAX if none (the rare full rescan)
        auto group_cell = [&](int sl, int f, float v) {
            const int nm = sl < gn3 ? 3 : (sl < gn3 + gn2 ? 2 : 1);
            const int cb = sl < gn3 ? 3 * sl : (sl < gn3 + gn2 ? gcb2 + 2 * (sl - gn3) : gcb1 + (sl - gn3 - gn2));
            const uint32_t w = gw[sl];
            const f2 part = lds_f2_plain(ws, (int)(w & 0x3FFu)) + lds_f2_plain(ws, R1 + (int)((w >> 10) & 0x3FFu));
            int mc = INT_MAX;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                if (j < nm) {
                    const f2 Lg = part + lds_f2_plain(ws, R2 + (int)(w >> 20) + 8 * j);
                    if ((f ? Lg.y : Lg.x) == v)
                        mc = imin(mc, (int)gcl[cb + j]);
                }
            }
            return mc;
        };
        // each lane's candidate per frame: its best group's members equal to
        // the maximum, both frames' words and cells read together, then the
        // gathers (two LDS round trips)
        int cand[2];
        {
            uint32_t bw[2];
            int bnm[2], bc[2][3];
#pragma unroll
            for (int f = 0; f < 2; f++) {
                const int sl = gs[f];
                bnm[f] = sl < gn3 ? 3 : (sl < gn3 + gn2 ? 2 : 1);
                const int cb = sl < gn3 ? 3 * sl : (sl < gn3 + gn2 ? gcb2 + 2 * (sl - gn3) : gcb1 + (sl - gn3 - gn2));
                bw[f] = gw[sl];
#pragma unroll
                for (int j = 0; j < 3; j++)
                    bc[f][j] = gcl[cb + imin(j, bnm[f] - 1)];
            }
#pragma unroll
            for (int f = 0; f < 2; f++) {
                const uint32_t w = bw[f];
                const f2 part = lds_f2_plain(ws, (int)(w & 0x3FFu)) + lds_f2_plain(ws, R1 + (int)((w >> 10) & 0x3FFu));
                int mc = INT_MAX;
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    const f2 Lg = part + lds_f2_plain(ws, R2 + (int)(w >> 20) + 8 * j);
                    if (j < bnm[f] && (f ? Lg.y : Lg.x) == gv[f])
                        mc = imin(mc, bc[f][j]);
                }
                cand[f] = gv[f] > -INFINITY ? mc : INT_MAX;
            }
        }
        int wcell[2];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            int ci = cand[j];
            int gk = fkey(gv[j]);
            wave_argmax_key(gk, ci);
            const float V = fkey_value(gk);
            if (__ballot(gsl[j] != gs[j] && gv[j] == V && V > -INFINITY)) {
                // rare: some lane's maximum tied another of its groups -- the
                // smallest first cell of every member whose L equals it
                int mc = INT_MAX;
                for (int sl = lane64; sl < gend; sl += 64)
                    mc = imin(mc, group_cell(sl, j, V));
                ci = wave_reduce<false>(mc);
            }
            wcell[j] = ci == INT_MAX ? gcell0 : ci;  // no maximum (NaN scores): tuple 0
            gv[j] = V;
        }
        LEAN_MARK();
#else
        float gv[2] = {-INFINITY, -INFINITY};
        int gu[2] = {INT_MAX, INT_MAX};
        const char *ws = (const char *)wsc;
        // lane-strided: the 32 lanes of a gather read 32 consecutive tuples
        // (first-cell order: neighbouring cells, so equal or adjacent lag slots
        // -- broadcasts and distinct banks instead of 4-way conflicts).
        // Software-pipelined by one step: the next step's tuple words and 12
        // gathers are in flight while this step's sums and compares run (the
        // loop is bound by LDS latency, not by its few VALU operations).
#if P1K_CELL_LDS
        const uint32_t wsb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)ws;
#endif
        auto gather = [&](const uint32_t (&qq)[4], f2 (&g)[4][3]) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
#if P1K_CELL_LDS
                // tuple fields: the lag slots' byte offsets (slot << 3) in bits
                // 3-9, 10-16 (>> 7), 17-23 (>> 14); the 1 KiB-aligned base
                // goes in by an or.  The first cell's offset from its row's
                // is in bits 24-31 and 0-2
                g[i][0] = lds_at((qq[i] & 0x3F8u) | wsb);
                g[i][1] = lds_at((((qq[i] >> 7) & 0x3F8u) | wsb) + P1K_KPAD * 8);
                g[i][2] = lds_at((((qq[i] >> 14) & 0x3F8u) | wsb) + 2 * P1K_KPAD * 8);
#else
                // tuple fields are byte offsets of f2 slots in [p][KPAD]
                g[i][0] = lds_f2_plain(ws, (int)(qq[i] & 0x3FFu));
                g[i][1] = lds_f2_plain(ws, P1K_KPAD * 8 + (int)((qq[i] >> 10) & 0x3FFu));
                g[i][2] = lds_f2_plain(ws, 2 * P1K_KPAD * 8 + (int)(qq[i] >> 20));
#endif
            }
        };
        uint32_t q[4];
        f2 g[4][3];
#pragma unroll
        for (int i = 0; i < 4; i++)
            q[i] = tups[64 * i + lane64];
        gather(q, g);
        auto consume = [&](const f2 (&gg)[4][3], int ub) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const f2 Lg = (gg[i][0] + gg[i][1]) + gg[i][2];
                const int u = ub + 64 * i + lane64;  // ascending per lane
                if (Lg.x > gv[0]) {
                    gv[0] = Lg.x;
                    gu[0] = u;
                }
                if (Lg.y > gv[1]) {
                    gv[1] = Lg.y;
                    gu[1] = u;
                }
            }
        };
        // two steps per trip (Upad is a multiple of 512): the step buffers
        // alternate instead of being copied back (24 moves a step)
        for (int u0 = 0; u0 < Upad; u0 += 512) {
            uint32_t qn[4];
#pragma unroll
            for (int i = 0; i < 4; i++)
                qn[i] = tups[u0 + 256 + 64 * i + lane64];
            f2 gn[4][3];
            gather(qn, gn);
            consume(g, u0);
            const int un = u0 + 512 < Upad ? u0 + 512 : u0 + 256;  // (a harmless re-read)
#pragma unroll
            for (int i = 0; i < 4; i++)
                q[i] = tups[un + 64 * i + lane64];
            gather(q, g);
            consume(gn, u0 + 256);
        }
        LEAN_MARK();
        // each lane looks up the first cell of its own candidate before the
        // wave reduction: the winner's comes back by a lane read, not by a
        // dependent load after it
        int mycell[2], myu[2];
#if P1K_CELL_LDS
        // from LDS: the tuple word's cell offset plus its 32-tuple row's first
        // cell (two LDS reads).  No global load may be pending here: gfx9's
        // vmcnt counts stores too, and every wait for such a load behind the
        // outputs below waited for their HBM write acks (~2.5 k cycles)
        const int *rowcell = reinterpret_cast<const int *>(tups + Upad);
#pragma unroll
        for (int j = 0; j < 2; j++) {
            myu[j] = gu[j];
            const int uc = (gu[j] < 0 || gu[j] >= kp.U) ? 0 : gu[j];
            const uint32_t tw = tups[uc];
            mycell[j] = rowcell[uc >> 5] + (int)((tw >> 24) | ((tw & 7u) << 8));
        }
#else
#pragma unroll
        for (int j = 0; j < 2; j++) {
            myu[j] = gu[j];
            mycell[j] = kp.tuple_cell[(gu[j] < 0 || gu[j] >= kp.U) ? 0 : gu[j]];
        }
#endif
        // (max L, first tuple) over the wave by keys (gv is -inf, never NaN,
        // where a lane had no L above it: those lanes keep gu = INT_MAX)
        int gk[2];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            gk[j] = fkey(gv[j]);
            wave_argmax_key(gk[j], gu[j]);
            gv[j] = fkey_value(gk[j]);
        }
        LEAN_MARK();
        int wcell[2];
#if P1K_CELL_LDS
        const int tuple_cell0 = rowcell[0];  // (offset 0)
#else
        const int tuple_cell0 = kp.tuple_cell[0];
#endif
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int fu = gu[j];
            const uint64_t wm = __ballot(myu[j] == fu && fu >= 0 && fu < kp.U);
            wcell[j] = wm ? __builtin_amdgcn_readlane(mycell[j], __builtin_ctzll(wm)) : tuple_cell0;
        }
#endif
        if (lane64 == 63) {
            const int cells[2] = {wcell[0], wcell[1]};  // no winner (NaN scores): tuple 0
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int64_t fs = base + 2 * wave + j;
                if (fs < B) {
                    if (out.cell)
                        out.cell[fs] = cells[j];
                    if (out.max_Lf)
                        out.max_Lf[fs] = gv[j];
                    if (out.xy) {
                        const int cx = cells[j] % kp.grid_W, cy = cells[j] / kp.grid_W;
                        out.xy[2 * fs] = (float)(cx - kp.half_w) / kp.grid_scale;
                        out.xy[2 * fs + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
                    }
                }
            }
        }
#if P1K_LATE_STORES
        store_frame();
#endif
        LEAN_MARK();
    }
#ifdef TDOA_DIAG
    stamp[13] = __builtin_amdgcn_s_memtime();
    stamp[15] = __builtin_amdgcn_s_memrealtime();
    if (lane64 == 0 && (blockIdx.x * NW + wave) < 4096)
        for (int i = 0; i < 16; i++)
            g_diag_p1k[(blockIdx.x * NW + wave) * 16 + i] = stamp[i];
#endif
#undef LEAN_MARK
}

#ifdef TDOA_DIAG
extern "C" int tdoa_diag_fetch_p1k(unsigned long long *host, int n)
{
    if (n > (1 << 16))
        n = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_p1k), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif

// --------------------------------------------------------------- host side
namespace {
constexpr int P1K_NW = 8;  // waves per workgroup (two per SIMD)

// dynamic LDS of a launch: the waves' tiles and the whole table image
constexpr size_t p1k_lds(int img_bytes) { return (size_t)P1K_NW * P1K_WAVE_LDS + (size_t)img_bytes; }
}  // namespace

// LDS table image of k_phat1024 (layout of the kernel's shared memory from twm on)
void tdoa_phat1024_image(int M, int N, int K, int U, const float *tw, const int32_t *win,
                         const float *prior, const uint32_t *tuples, const int32_t *tuple_cell,
                         std::vector<uint8_t> &img)
{
    img.clear();
    if (M != 3 || N != 1024 || K > P1K_KPAD - 1)
        return;
#if P1K_GROUPS
    // groups: tuples of equal (l0, l1) whose l2 are consecutive, at most 3 per
    // group (config 2: 1121 groups of 3 / 2 / 1 for 2469 tuples), bucketed by
    // size, each bucket in the order of its groups' first tuples (neighbouring
    // lanes, neighbouring cells and lag slots) and padded to whole waves
    struct Grp {
        int l0, l1, l2, n, u0;
        int cell[3];
    };
    std::map<std::pair<int, int>, std::vector<std::pair<int, int>>> by;  // (l0, l1) -> (l2, u)
    for (int u = 0; u < U; u++)
        by[{(int)(tuples[u] & 0xFFu), (int)((tuples[u] >> 8) & 0xFFu)}].push_back({(int)((tuples[u] >> 16) & 0xFFu), u});
    std::vector<Grp> bk[4];
    for (auto &kv : by) {
        auto &v = kv.second;
        std::sort(v.begin(), v.end());
        for (size_t i = 0; i < v.size();) {
            Grp g{kv.first.first, kv.first.second, v[i].first, 0, INT_MAX, {0, 0, 0}};
            while (i < v.size() && g.n < 3 && v[i].first == g.l2 + g.n) {
                if (tuple_cell[v[i].second] < 0 || tuple_cell[v[i].second] >= 0xFFFF)
                    return;  // cells are 16-bit in the table
                g.cell[g.n++] = tuple_cell[v[i].second];
                g.u0 = std::min(g.u0, v[i].second);
                i++;
            }
            bk[g.n].push_back(g);
        }
    }
    int nslot[4];
    for (int n = 1; n <= 3; n++) {
        std::sort(bk[n].begin(), bk[n].end(), [](const Grp &x, const Grp &y) { return x.u0 < y.u0; });
        nslot[n] = ((int)bk[n].size() + 127) / 128 * 128;  // whole pairs of 64-slot steps
    }
    const int ncell = 3 * nslot[3] + 2 * nslot[2] + nslot[1];
    const size_t bytes = (size_t)P1K_IMG_FIXED + 16 + 4 * (size_t)(nslot[3] + nslot[2] + nslot[1]) + 2 * (size_t)ncell;
    img.resize((bytes + 15) / 16 * 16);
#else
    const int Upad = (U + P1K_GB * 64 - 1) / (P1K_GB * 64) * (P1K_GB * 64);
#if P1K_CELL_LDS
    img.resize((size_t)P1K_IMG_FIXED + (size_t)Upad * 4 + (size_t)(Upad / 32) * 4);  // + the row cells
#else
    (void)tuple_cell;
    img.resize((size_t)P1K_IMG_FIXED + (size_t)Upad * 4);
#endif
#endif
    float *f = (float *)img.data();
    const float *tw2 = tw + 2 * N;
    for (int k = 0; k < 32; k++)  // twm [k][r] = W_1024^{r k}
        for (int r = 0; r < 32; r++) {
            const int i = (k * r) & (N - 1);
            f[2 * (32 * k + slot(r))] = tw[2 * i];
            f[2 * (32 * k + slot(r)) + 1] = tw[2 * i + 1];
        }
    f += 2 * 1024;
    for (int k = 0; k < 16; k++)  // tw2 [k][r] = W_2048^{r + 32 k}
        for (int r = 0; r < 32; r++) {
            const int b = r + 32 * k;
            f[2 * (32 * k + slot(r))] = tw2[2 * b];
            f[2 * (32 * k + slot(r)) + 1] = tw2[2 * b + 1];
        }
    f += 2 * 512;
    for (int e = 0; e < 512; e++) {  // (W[2e], W[2e+1]) / 128, word e = 32 t + r at slot(r)
        const int d = (e & ~31) + slot(e & 31);
        f[2 * d] = (float)win[2 * e] * (1.0f / 128.0f);
        f[2 * d + 1] = (float)win[2 * e + 1] * (1.0f / 128.0f);
    }
    f += 2 * 512;
    for (int k = 0; k < 128; k++)
        f[k] = k < K ? prior[k] : 0.0f;
    uint32_t *t = (uint32_t *)(f + 128);
#if P1K_GROUPS
    // header: slots per bucket (n = 3, 2, 1), tuple 0's cell; then the group
    // words (LDS byte offsets of l0, l1 and the first l2 in a wave's [p][KPAD]
    // f2 score table, 10 bits each; padding groups start at slot 127 of every
    // pair, -inf) and the member cells (u16, bucket n: [slot][n])
    int32_t *hdr = (int32_t *)t;
    hdr[0] = nslot[3];
    hdr[1] = nslot[2];
    hdr[2] = nslot[1];
    hdr[3] = U > 0 ? tuple_cell[0] : 0;
    t += 4;
    uint16_t *cl = (uint16_t *)(t + nslot[3] + nslot[2] + nslot[1]);
    for (int n = 3; n >= 1; n--) {
        for (int e = 0; e < nslot[n]; e++) {
            const bool real = e < (int)bk[n].size();
            const Grp g = real ? bk[n][e] : Grp{127, 127, 128 - n, n, 0, {0xFFFF, 0xFFFF, 0xFFFF}};
            *t++ = ((uint32_t)g.l0 << 3) | ((uint32_t)g.l1 << 13) | ((uint32_t)g.l2 << 23);
            for (int j = 0; j < n; j++)
                *cl++ = (uint16_t)g.cell[j];
        }
    }
#else
    // tuples as LDS byte offsets into a wave's [p][KPAD] f2 score table, 10 bits
    // per pair; padding tuple (127, 127, 127) scores -inf
#if P1K_CELL_LDS
    // (lag slots 7 bits each, then the first cell minus its 32-tuple row's
    // first cell in 11 bits; a table with a row that spans more has no image:
    // the generic kernel runs it)
    int32_t *rowcell = (int32_t *)(t + Upad);
    for (int r = 0; r < Upad / 32; r++) {
        const int e0 = 32 * r, e1 = std::min(U, e0 + 32) - 1;
        rowcell[r] = e0 >= U ? 0 : tuple_cell[e0];
        if (e0 < U && tuple_cell[e1] - tuple_cell[e0] >= 2048) {
            img.clear();
            return;
        }
    }
    for (int e = 0; e < Upad; e++) {
        const uint32_t wd = e < U ? tuples[e] : 0x007F7F7Fu;
        const uint32_t dc = e < U ? (uint32_t)(tuple_cell[e] - rowcell[e >> 5]) : 0u;
        t[e] = ((wd & 0x7Fu) << 3) | (((wd >> 8) & 0x7Fu) << 10) | (((wd >> 16) & 0x7Fu) << 17) |
               ((dc & 0xFFu) << 24) | (dc >> 8);
    }
#else
    for (int e = 0; e < Upad; e++) {
        const uint32_t wd = e < U ? tuples[e] : 0x007F7F7Fu;
        t[e] = ((wd & 0xFFu) << 3) | (((wd >> 8) & 0xFFu) << 13) | (((wd >> 16) & 0xFFu) << 23);
    }
#endif
#endif
}

// config-2 shape (M = 3, N = 1024, S <= 63) with a tuple table that fits the tail
bool tdoa_phat1024_fits(const tdoa_kparams &kp)
{
    if (kp.M != 3 || kp.N != 1024 || kp.S > 63 || kp.TW != 1 || !kp.p1k_img)
        return false;
    // grid scores of a wave's two frames live in its tiles: [3][KPAD] float2 = 3 KiB
    static_assert(3 * P1K_KPAD * 8 <= P1K_WAVE_LDS, "grid scores exceed the wave's tiles");
    // the image loads as at most 4 units of 16 B per thread (k_p1k_lean's staging)
    return kp.p1k_img_bytes <= 4 * P1K_NW * 64 * 16 && p1k_lds(kp.p1k_img_bytes) + 64 <= 160 * 1024;  // + the static progress words
}

int tdoa_launch_phat1024(const tdoa_kparams &kp, const tdoa_kout &out, const int16_t *frames,
                         int64_t B, float phat_eps, void *stream)
{
    // per-mic clamp: |X_m| >= sqrt(eps) in the oracle's units (x / 2^15, X / 2),
    // i.e. |X|^2 >= eps * 2^32 in the kernel's int16 units with the split's factor 2
    float e2 = phat_eps * 4294967296.0f;
    if (!(e2 >= 1e-30f))
        e2 = 1e-30f;
    if (B <= 0)
        return 0;
    // one workgroup of 16 frames (8 waves, one frame per half-wave) per group
    constexpr int NF = 2 * P1K_NW;
    const int64_t grid = (B + NF - 1) / NF;
    if (grid > 0x7FFFFFFF)
        return tdoa_set_error(-1, "k_p1k_lean: batch too large for one launch");
    hipLaunchKernelGGL(k_p1k_lean, dim3((unsigned)grid), dim3(P1K_NW * 64), p1k_lds(kp.p1k_img_bytes), (hipStream_t)stream,
                       kp, out, frames, B, e2);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char buf[256];
        snprintf(buf, sizeof buf, "k_p1k_lean launch: %s", hipGetErrorString(e));
        return tdoa_set_error(-2, buf);
    }
    return 0;
}
