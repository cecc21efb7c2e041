// tdoa_stream.hip -- the streaming loop of sample_compute.h:53-146 for S
// independent mic-array streams, one hop of H samples per step (BASELINE
// config 5).  Three kernels per step (plus k_direct on the triggered frames):
//
//   k_stream_trigger  one workgroup per stream: reads the hop's 8-bit ADC
//                     bytes (dma_sampler.c:17-23, round-robin per mic, read
//                     as sample_t at sample_compute.h:67-73) and the N-1
//                     samples before it from the capture ring, evaluates the
//                     trigger of sample_compute.h:75-91 after every sample of
//                     the hop -- half powers of rolling_buffer.c:73-85 from
//                     LDS prefix sums -- and takes the first firing sample
//                     at least N samples after the stream's last trigger
//                     (the rings restart empty after a trigger,
//                     sample_compute.h:55-57).  A firing stream appends its
//                     frame (the ring oldest..newest) to a compact batch.
//   k_direct          (tdoa_direct.hip) on the compact batch, its size read
//                     from device memory: write_out, normalize, window,
//                     xcorr, prior, gate.
//   k_stream_update   one workgroup per compact slot: for gated frames the
//                     EMA of correlations.c:38-63 on the stream's state
//                     (clock now_us = end * 1e6 / fs) and the grid solve on
//                     the EMA scores (vga_heatmap.h:99-108 runs on corr_*);
//                     advances the device sample clock by H.
//
// Built with -ffp-contract=off: the EMA's float steps round as the
// reference's IEEE host build does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cstdlib>

#include "tdoa_internal.h"
#include "tdoa_keys.h"

int tdoa_set_error(int code, const char *msg);

namespace {

constexpr int TPB = 256;
constexpr int MAX_CAND = 16;  // hop <= 4096 candidates, TPB per pass

// inclusive block scan of per-thread totals (int32 and int64 together)
__device__ __forceinline__ void block_exclusive_scan(int &v1, long long &v2, int *s1,
                                                     long long *s2)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int x1 = v1;
    long long x2 = v2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y1 = __shfl_up(x1, o, 64);
        const long long y2 = __shfl_up(x2, o, 64);
        if (lane >= o) {
            x1 += y1;
            x2 += y2;
        }
    }
    if (lane == 63) {
        s1[wave] = x1;
        s2[wave] = x2;
    }
    __syncthreads();
    int b1 = 0;
    long long b2 = 0;
    for (int w = 0; w < wave; w++) {
        b1 += s1[w];
        b2 += s2[w];
    }
    v1 = b1 + x1 - v1;  // exclusive
    v2 = b2 + x2 - v2;
    __syncthreads();
}

__global__ void __launch_bounds__(TPB) k_stream_trigger(tdoa_stream_params sp)
{
    if (blockIdx.x == 0 && threadIdx.x == 0 && sp.count_next)
        *sp.count_next = 0;  // the next hop's counter (last read by the previous hop)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int M = sp.M, N = sp.N, H = sp.H, L = N + H - 1, tid = threadIdx.x;
    int16_t *xs = (int16_t *)smem;                                   // [M][L]
    size_t o = (((size_t)M * L * 2) + 15) & ~(size_t)15;
    int *Q1 = (int *)(smem + o);                                      // [L + 1]
    o += (((size_t)(L + 1) * 4) + 15) & ~(size_t)15;
    long long *Q2 = (long long *)(smem + o);                          // [L + 1]
    __shared__ int sc1[TPB / 64];
    __shared__ long long sc2[TPB / 64];
    __shared__ int first, slot;

    const int64_t s = blockIdx.x;
    const int64_t pos = *sp.pos;           // samples consumed before this hop
    const int64_t base = pos + 1 - N;      // stream index of local sample 0
    const uint8_t *cap = sp.capture + (size_t)s * sp.capture_len * M;
    // local samples l = 0..L-1 <-> stream index base + l (zero before the stream starts)
    {
        int64_t j0 = base % sp.capture_len;
        if (j0 < 0)
            j0 += sp.capture_len;
        for (int i = tid; i < L * M; i += TPB) {
            const int l = i / M, m = i - l * M;
            int64_t j = j0 + l;
            if (j >= sp.capture_len)
                j -= sp.capture_len;
            xs[m * L + l] = base + l < 0 ? (int16_t)0 : (int16_t)cap[(size_t)j * M + m];
        }
    }
    if (tid == 0)
        first = INT_MAX;
    __syncthreads();

    // per candidate a (frame = local [a, a + N), end = pos + 1 + a): sum over
    // mics of the outgoing (older half) and incoming (newer half) powers
    const int hb = sp.log2N - 1;
    long long pout[MAX_CAND], pin[MAX_CAND];
#pragma unroll
    for (int c = 0; c < MAX_CAND; c++)
        pout[c] = pin[c] = 0;
    const int per = (L + 1 + TPB - 1) / TPB;  // prefix entries per thread
    for (int m = 0; m < M; m++) {
        const int16_t *x = xs + m * L;
        // Q[l] = sum_{l' < l} x, Q2 the same of x^2 (rolling_buffer.c:22-32 totals)
        int t1 = 0;
        long long t2 = 0;
        const int l0 = tid * per;
        for (int k = 0; k < per; k++) {
            const int l = l0 + k;
            if (l < L) {
                const int v = x[l];
                t1 += v;
                t2 += (long long)v * v;
            }
        }
        int e1 = t1;
        long long e2 = t2;
        block_exclusive_scan(e1, e2, sc1, sc2);
        for (int k = 0; k <= per; k++) {
            const int l = l0 + k;
            if (l <= L && (k < per || l == L)) {
                Q1[l] = e1;
                Q2[l] = e2;
            }
            if (k < per && l < L) {
                const int v = x[l];
                e1 += v;
                e2 += (long long)v * v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < MAX_CAND; c++) {
            const int a = tid + TPB * c;
            if (a < H) {
                const int h = N >> 1;
                const long long so1 = Q1[a + h] - Q1[a], so2 = Q2[a + h] - Q2[a];
                const long long si1 = Q1[a + N] - Q1[a + h], si2 = Q2[a + N] - Q2[a + h];
                pout[c] += (long long)((unsigned long long)so2 << hb) - so1 * so1;
                pin[c] += (long long)((unsigned long long)si2 << hb) - si1 * si1;
            }
        }
        __syncthreads();
    }
    const long long thr = (long long)2 << (2 * hb);  // POWER_THRESHOLD, sample_compute.h:21
    const int64_t rs = sp.ring_start[s];
    // full ring: at least N samples since the last trigger
    const int64_t amin = rs + N - pos - 1;
#pragma unroll
    for (int c = 0; c < MAX_CAND; c++) {
        const int a = tid + TPB * c;
        if (a < H && a >= amin && pout[c] > thr + pin[c]) {
            atomicMin(&first, a);
            break;  // candidates grow with c: this thread's first is its best
        }
    }
    __syncthreads();
    const int a = first;
    if (a == INT_MAX)
        return;
    if (tid == 0) {
        slot = atomicAdd(sp.count, 1);
        const int64_t end = pos + 1 + a;
        if (slot < (int)gridDim.x) {  // one slot per stream (see k_stream_trigger_p)
            sp.ids[slot] = (int32_t)s;
            sp.end[slot] = end;
        }
        sp.ring_start[s] = end;
    }
    __syncthreads();
    if (slot >= (int)gridDim.x)
        return;
    // the frame as 8-bit samples (the capture's values; DIRECT widens them,
    // kp.frames_u8), four per dword store
    uint32_t *dst = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(sp.frames) + (size_t)slot * M * N);
    for (int i = tid; i < M * N / 4; i += TPB) {
        const int m = (4 * i) / N, n = 4 * i - m * N;
        const int16_t *x = xs + m * L + a + n;
        dst[i] = (uint32_t)(uint8_t)x[0] | (uint32_t)(uint8_t)x[1] << 8 | (uint32_t)(uint8_t)x[2] << 16 |
                 (uint32_t)(uint8_t)x[3] << 24;
    }
}

// ------------------------------------------- register trigger scan (N = 2H)
// One wave per stream, four streams per workgroup, no LDS.  Lane k holds, for
// rows r = 0, 1, 2, the G = H/64 local samples l = rH + Gk + i (i < G) of every
// mic: candidate a = Gk + i needs the prefix sums at a, a + N/2 = a + H and
// a + N = a + 2H, i.e. at position i of the lane's own three chunks.  The chunk
// totals are wave-scanned (DPP), the rest is a running sum in registers.  Same
// trigger as k_stream_trigger (sample_compute.h:75-91, rolling_buffer.c:73-85).

// inclusive wave scan (rows by row_shr, then row_bcast:15 / :31)
__device__ __forceinline__ int wave_scan_incl(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// the same over several independent values, stage by stage: the values
// interleave, so no DPP read follows the write of its own source (each such
// pair costs an s_nop 1)
template <int NV>
__device__ __forceinline__ void wave_scan_incl_n(int (&v)[NV])
{
#pragma unroll
    for (int j = 0; j < NV; j++)
        v[j] += __builtin_amdgcn_update_dpp(0, v[j], 0x111, 0xF, 0xF, false);  // row_shr:1
#pragma unroll
    for (int j = 0; j < NV; j++)
        v[j] += __builtin_amdgcn_update_dpp(0, v[j], 0x112, 0xF, 0xF, false);  // row_shr:2
#pragma unroll
    for (int j = 0; j < NV; j++)
        v[j] += __builtin_amdgcn_update_dpp(0, v[j], 0x114, 0xF, 0xF, false);  // row_shr:4
#pragma unroll
    for (int j = 0; j < NV; j++)
        v[j] += __builtin_amdgcn_update_dpp(0, v[j], 0x118, 0xF, 0xF, false);  // row_shr:8
#pragma unroll
    for (int j = 0; j < NV; j++)
        v[j] += __builtin_amdgcn_update_dpp(0, v[j], 0x142, 0xA, 0xF, false);  // row_bcast:15
#pragma unroll
    for (int j = 0; j < NV; j++)
        v[j] += __builtin_amdgcn_update_dpp(0, v[j], 0x143, 0xC, 0xF, false);  // row_bcast:31
}

// Persistent: each wave walks streams gw, gw + GW, ... with the NEXT stream's
// capture words and ring start already requested while it scans the current one
// (a one-stream-per-wave form waited on its loads at the start of every wave:
// 68 % of wave cycles in SQ_WAIT_ANY).  A firing stream is only listed (stream,
// end, ring index of the frame's first sample): DIRECT stages the frame from
// the capture ring itself (kp.frame_ring), so no copy of it is written and
// read back (10.7 MB per config-5 hop as 8-bit copies).
constexpr int TRIG_NWB = 4;  // waves per workgroup: occupancy in steps of one wave per SIMD
template <int G, int M>
__global__ void __launch_bounds__(64 * TRIG_NWB) k_stream_trigger_p(tdoa_stream_params sp, int64_t S)
{
    constexpr int H = 64 * G, N = 2 * H, CB = G * M, CW = CB / 4;
    static_assert(CB % 4 == 0, "a lane's chunk is whole words");
    constexpr int NWB = TRIG_NWB;  // waves per workgroup
    extern __shared__ __attribute__((aligned(16))) uint32_t stage_all[];  // [NWB waves][3 H M / 4]
    __shared__ int nfired[NWB], slot_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (blockIdx.x == 0 && threadIdx.x == 0 && sp.count_next)
        *sp.count_next = 0;  // the next hop's counter (last read by the previous hop)
    uint32_t *stage = stage_all + wv * (3 * H * M / 4);
    const int64_t GW = (int64_t)gridDim.x * NWB;
    const int64_t s0 = (int64_t)blockIdx.x * NWB;  // the workgroup's first stream of an iteration
    int64_t s = s0 + wv;
    const int64_t pos = *sp.pos;
    const int64_t base = pos + 1 - N;
    const int64_t cl = sp.capture_len;
    int64_t j0 = base % cl;
    if (j0 < 0)
        j0 += cl;
    // ring positions of the lane's three chunks: the same for every stream
    int64_t jr[3];
    bool fast[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const int64_t l0 = base + r * H + G * lane;
        int64_t j = j0 + r * H + G * lane;
        if (j >= cl)
            j -= cl;
        jr[r] = j;
        fast[r] = l0 >= 0 && (j + G) * M + 7 <= cl * M;
    }
    // aligned words of the fast rows (the word pointer and the byte shift from
    // the absolute address: a ring need not start 4-byte aligned)
    auto fetch = [&](int64_t st, uint32_t (&w)[3][CW + 1], uint32_t (&sh)[3]) {
        const uint8_t *cap = sp.capture + (size_t)st * cl * M;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            // (pointer arithmetic, not an integer-to-pointer cast: that made
            // these flat loads, whose waits also drain the LDS counter)
            const uint8_t *pb = cap + (size_t)(fast[r] ? jr[r] : 0) * M;
            sh[r] = (uint32_t)((uintptr_t)pb & 3u);
            const uint32_t *wp = reinterpret_cast<const uint32_t *>(pb - sh[r]);
#pragma unroll
            for (int k = 0; k <= CW; k++)
                w[r][k] = fast[r] ? wp[k] : 0u;
        }
    };
    uint32_t wc[3][CW + 1], shc[3];
    int64_t rs = 0;
    // this wave's triggered streams: lane i holds the i-th (stream, end)
    int my_n = 0;
    int my_id = 0;
    int64_t my_end = 0, my_at = 0;
    if (s < S) {
        fetch(s, wc, shc);
        rs = sp.ring_start[s];
    }
    constexpr int hb = __builtin_ctz(N) - 1;
    const long long thr = (long long)2 << (2 * hb);  // POWER_THRESHOLD, sample_compute.h:21
    for (int64_t sb = s0; sb < S; sb += GW, s += GW) {
        const bool have = s < S;
        // a stream that fired during the previous hop cannot fire in this one
        // (its ring holds fewer than N samples for every candidate: a >= amin
        // >= H); ~1 in 5 streams at config 5: no scan
        const bool skip = __builtin_amdgcn_readfirstlane((int)(!have || rs + N - pos - 1 >= H)) != 0;
        const uint8_t *cap = sp.capture + (size_t)(have ? s : 0) * cl * M;
        uint32_t x[3][CW];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            if (fast[r]) {
#pragma unroll
                for (int k = 0; k < CW; k++)
                    x[r][k] = __builtin_amdgcn_alignbyte(wc[r][k + 1], wc[r][k], shc[r]);
            } else {  // stream start (zeros) or the ring's end: byte by byte through
                // the wave's stage (a compact loop: this rare path must not set
                // the kernel's register count)
                const int64_t l0 = base + r * H + G * lane;
                uint8_t *sb8 = reinterpret_cast<uint8_t *>(stage) + r * H * M + lane * CB;
                wave_lds_sync();  // the previous stream's stage reads come first
#pragma unroll 1
                for (int b = 0; b < CB; b++) {
                    const int i = b / M, m = b - i * M;
                    int64_t ji = jr[r] + i;
                    if (ji >= cl)
                        ji -= cl;
                    sb8[b] = l0 + i < 0 ? (uint8_t)0 : cap[(size_t)ji * M + m];
                }
                wave_lds_sync();
#pragma unroll
                for (int k = 0; k < CW; k++)
                    x[r][k] = stage[r * (H * M / 4) + lane * CW + k];
            }
        }
        // the next stream's words into the same registers, in flight while
        // this stream is scanned
        const int64_t sn = s + GW;
        int64_t rsn = 0;
        if (sn < S) {
            fetch(sn, wc, shc);
            rsn = sp.ring_start[sn];
        }
        if (skip) {
            rs = rsn;
            continue;
        }
        auto smp = [&](int r, int i, int m) -> int {
            const int b = i * M + m;
            return (int)((x[r][b >> 2] >> (8 * (b & 3))) & 0xFFu);
        };
        // exclusive prefix sums over the lanes' chunks of each row: per mic the
        // samples (v_dot4 of the chunk's words with a 0/1 byte mask of that
        // mic's bytes), over all mics their squares (v_dot4 of a word with itself)
        int q1[3][M], q2[3];
        {
            int tot1[M], tot2 = 0;
#pragma unroll
            for (int m = 0; m < M; m++)
                tot1[m] = 0;
            // (the row's M + 1 dot chains and scans interleaved: a dot or DPP
            // read right after the write of its own source waits in s_nops)
#pragma unroll
            for (int r = 0; r < 3; r++) {
                uint32_t c[M + 1] = {};  // [0, M): mic m's samples, [M]: all squares
#pragma unroll
                for (int k = 0; k < CW; k++) {
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        uint32_t mask = 0;  // bytes 4k + j of the chunk that are mic m's
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            mask |= ((4 * k + j) % M == m ? 1u : 0u) << (8 * j);
                        c[m] = __builtin_amdgcn_udot4(x[r][k], mask, c[m], false);
                    }
                    c[M] = __builtin_amdgcn_udot4(x[r][k], x[r][k], c[M], false);
                }
                int inc[M + 1];
#pragma unroll
                for (int j = 0; j <= M; j++)
                    inc[j] = (int)c[j];
                wave_scan_incl_n(inc);
#pragma unroll
                for (int m = 0; m < M; m++) {
                    q1[r][m] = tot1[m] + inc[m] - (int)c[m];
                    tot1[m] += __builtin_amdgcn_readlane(inc[m], 63);
                }
                q2[r] = tot2 + inc[M] - (int)c[M];
                tot2 += __builtin_amdgcn_readlane(inc[M], 63);
            }
        }
        // the words re-enter here opaque: the scan re-extracts the samples
        // instead of keeping the prefix pass's extracted bytes live
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int k = 0; k < CW; k++)
                asm volatile("" : "+v"(x[r][k]));
        const int64_t amin = rs + N - pos - 1;  // full ring: >= N samples since the last trigger
        // (clamped to the candidates' range: a 32-bit compare per candidate)
        const int amin32 = (int)(amin < 0 ? 0 : (amin > H ? H : amin));
        // the trigger of sample_compute.h:75-91 in difference form: with the
        // older / newer half-window sums so, si per mic and D2 = (q2[1] - q2[0])
        // - (q2[2] - q2[1]) of the squares, pout - pin = (D2 << hb) -
        // sum_m (so - si)(so + si) -- pout > thr + pin exactly as the
        // reference's int64 powers (rolling_buffer.c:73-85), one 64-bit
        // multiply-add per mic instead of two squares
        int so[M], si[M];
#pragma unroll
        for (int m = 0; m < M; m++) {
            so[m] = q1[1][m] - q1[0][m];
            si[m] = q1[2][m] - q1[1][m];
        }
        int D2 = (q2[1] - q2[0]) - (q2[2] - q2[1]);
        int fi = -1;
#pragma unroll
        for (int i = 0; i < G; i++) {
            // sample i's words re-enter opaque: their bytes are extracted here,
            // not hoisted for every i at once (registers: occupancy)
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int k = (i * M) >> 2; k <= (i * M + M - 1) >> 2; k++)
                    asm volatile("" : "+v"(x[r][k]));
            const int a = G * lane + i;
            // (accumulated by 64-bit multiply-adds from the squares' term: no
            // 64-bit subtract and its carry chain)
            long long T = (long long)D2 << hb;
#pragma unroll
            for (int m = 0; m < M; m++)
                T += (long long)(si[m] - so[m]) * (long long)(so[m] + si[m]);
            if (fi < 0 && a >= amin32 && T > thr)
                fi = i;
#pragma unroll
            for (int m = 0; m < M; m++) {
                const int v0 = smp(0, i, m), v1 = smp(1, i, m), v2 = smp(2, i, m);
                so[m] += v1 - v0;
                si[m] += v2 - v1;
            }
            // sample i's squares summed over the mics, per row: its M bytes
            // gathered into one word (v_perm, zeros above) and dotted with
            // themselves -- two instructions a row (the compiler's form was a
            // 24-bit multiply, a perm and a dot)
            int w[3];
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const int b = i * M, k = b >> 2, sh = b & 3;
                uint32_t sel = 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    sel |= (uint32_t)(j < M ? sh + j : 0x0C) << (8 * j);
                const uint32_t hi = sh + M - 1 > 3 ? x[r][k + 1 < CW ? k + 1 : k] : x[r][k];
                const uint32_t p = M == 4 ? x[r][k] : __builtin_amdgcn_perm(hi, x[r][k], sel);
                w[r] = (int)__builtin_amdgcn_udot4(p, p, 0u, false);
            }
            D2 += (w[1] - w[0]) - (w[2] - w[1]);
        }
        const uint64_t fire = have ? __ballot(fi >= 0) : 0;
        if (fire != 0) {
            const int fl = __builtin_ctzll(fire);  // lowest lane = lowest candidates
            const int a = G * fl + __builtin_amdgcn_readlane(fi, fl);
            const int64_t end = pos + 1 + a;
            // the frame is local samples a .. a + N - 1 (rolling_buffer.c:48-62
            // order): DIRECT reads them from the ring (kp.frame_ring), no copy
            if (lane == my_n) {
                my_id = (int)s;
                my_end = end;
                my_at = j0 + a >= cl ? j0 + a - cl : j0 + a;
            }
            ++my_n;
            if (lane == 0)
                sp.ring_start[s] = end;
        }
        rs = rsn;
    }
    // the workgroup's triggered streams into the compact list: one atomic
    if ((threadIdx.x & 63) == 0)
        nfired[wv] = my_n;
    __syncthreads();
    if (threadIdx.x == 0) {
        int n = 0;
        for (int w = 0; w < NWB; w++)
            n += nfired[w];
        slot_base = n ? atomicAdd(sp.count, n) : 0;
    }
    __syncthreads();
    int o = slot_base;
    for (int w = 0; w < wv; w++)
        o += nfired[w];
    // o + lane < S always holds while the hop's slot started at 0 (one slot per
    // firing stream); the clamp keeps a corrupted counter from writing past S
    if (lane < my_n && o + lane < S) {
        sp.ids[o + lane] = my_id;
        sp.end[o + lane] = my_end;
        sp.ring_at[o + lane] = my_at;
    }
}

// correlations.c:40-43 in the reference's float/double steps
__device__ __forceinline__ float decay_us(uint64_t now, uint64_t last) { return tdoa_decay_dev(now, last); }

__global__ void __launch_bounds__(TPB) k_stream_update(tdoa_stream_params sp, tdoa_kparams kp,
                                                       tdoa_stream_kout out, int nstreams)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int64_t *W = (int64_t *)smem;     // [P][K] EMA scores
    __shared__ int64_t redv[TPB / 64];
    __shared__ int redi[TPB / 64];
    __shared__ uint64_t redk[TPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = TPB / 64;
    const int K = kp.K, P = kp.P;
    // at most one slot per stream: a corrupted counter cannot index past [S]
    const int cnt_raw = *sp.count;
    const int cnt = cnt_raw < 0 ? 0 : (cnt_raw > nstreams ? nstreams : cnt_raw);
    if (blockIdx.x == 0) {
        // gated frames of this hop: block 0 sums the batch's gate bytes (a
        // per-slot atomic on one counter serialises in L2)
        int g = 0;
        for (int i = tid; i < cnt; i += TPB)
            g += sp.fresh_gate[i];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
            g += __shfl_xor(g, o, 64);
        if (lane == 0)
            redi[wave] = g;
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < nwaves; w++)
                g += redi[w];
            *sp.pos += sp.H;  // every block of k_stream_trigger has read it
            sp.stats[0] += cnt;
            sp.stats[1] += g;
            if (out.count)
                *out.count = cnt;
        }
    }
    // persistent over the compact batch (its size is only known on the device)
    for (int slot = blockIdx.x; slot < cnt; slot += gridDim.x) {
    __syncthreads();  // the previous slot's W and reductions are consumed
        const int s = sp.ids[slot];
        if (out.lags) {
            for (int p = tid; p < P; p += TPB)
                out.lags[(size_t)slot * P + p] = sp.fresh_lags[(size_t)slot * P + p];
        }
        if (tid == 0) {
            if (out.stream_id)
                out.stream_id[slot] = s;
            if (out.end)
                out.end[slot] = sp.end[slot];
            if (out.gate)
                out.gate[slot] = sp.fresh_gate[slot];
        }
        if (!sp.fresh_gate[slot]) {  // sample_compute.h:134: only gated frames update
            if (tid == 0) {
                if (out.cell)
                    out.cell[slot] = -1;
            }
            continue;
        }
        const uint64_t now = (uint64_t)sp.end[slot] * 1000000u / (uint64_t)sp.fs;
        const float dec = decay_us(now, sp.last[s]);
        int64_t *est = sp.est + (size_t)s * P * K;
        const int64_t *fr = sp.fresh + (size_t)slot * P * K;
        for (int p = wave; p < P; p += nwaves) {
            // EMA of correlations.c:38-63, then the first maximum as a DPP key
            // reduction (tdoa_keys.h: |EMA| <= 2^42 < 2^47)
            uint64_t key = 0;
            for (int k = lane; k < 128; k += 64) {
                if (k < K) {
                    const int64_t ev = est[p * K + k];
                    const float delta = (float)(fr[p * K + k] - ev) * dec;
                    const float sum = (float)ev + delta;
                    const int64_t nv = (int64_t)sum;
                    est[p * K + k] = nv;
                    W[p * K + k] = nv;
                    const uint64_t kk = vkey<7>(nv, k);
                    key = kk > key ? kk : key;
                }
            }
            const int bk = key_index<7>(lane63_u64(wave_umax_dpp(key)));
            if (lane == 0 && out.ema_best)
                out.ema_best[(size_t)slot * P + p] = bk - kp.S;
        }
        __syncthreads();
        if (tid == 0)
            sp.last[s] = now;
        // grid solve on the EMA scores over the distinct lag tuples
        int64_t bv = INT64_MIN;
        int bu = INT_MAX;
        if (kp.TW == 1) {
            // 3-4 mic grids: a thread's tuple words are loaded 8 at a time ahead of
            // their gathers (one L2 round trip per 8 tuples, not per tuple)
            for (int u0 = tid; u0 < kp.U; u0 += 8 * TPB) {
                uint32_t wd[8];
    #pragma unroll
                for (int t = 0; t < 8; t++) {
                    const int u = u0 + t * TPB;
                    wd[t] = u < kp.U ? kp.tuples[u] : 0u;
                }
    #pragma unroll
                for (int t = 0; t < 8; t++) {
                    const int u = u0 + t * TPB;
                    if (u < kp.U) {
                        int64_t Lv = 0;
                        for (int p = 0; p < P; p++)
                            Lv += W[p * K + ((wd[t] >> (8 * p)) & 0xFFu)];
                        if (Lv > bv) {  // ascending u per thread: strict '>' keeps the first
                            bv = Lv;
                            bu = u;
                        }
                    }
                }
            }
        } else {
            for (int u = tid; u < kp.U; u += TPB) {
                int64_t Lv = 0;
                for (int tw = 0; tw < kp.TW; tw++) {
                    const uint32_t word = kp.tuples[u * kp.TW + tw];
                    for (int b = 0; b < 4; b++) {
                        const int p = 4 * tw + b;
                        if (p < P)
                            Lv += W[p * K + ((word >> (8 * b)) & 0xFFu)];
                    }
                }
                if (Lv > bv) {
                    bv = Lv;
                    bu = u;
                }
            }
        }
        if (kp.U < 65536) {
            // (L, first tuple) as one key (tdoa_keys.h, 16 index bits): DPP over
            // the wave, LDS over the waves.  A thread without tuples keeps key 0.
            uint64_t key = bu < kp.U ? vkey<16>(bv, bu) : 0;
            key = wave_umax_dpp(key);
            if (lane == 63)
                redk[wave] = key;
        } else {
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
        }
        __syncthreads();
        if (tid == 0) {
            if (kp.U < 65536) {
                uint64_t key = 0;
                for (int w = 0; w < nwaves; w++)
                    key = redk[w] > key ? redk[w] : key;
                bv = key_value<16>(key);
                bu = key_index<16>(key);
            } else {
                for (int w = 1; w < nwaves; w++)
                    if (redv[w] > bv || (redv[w] == bv && redi[w] < bu)) {
                        bv = redv[w];
                        bu = redi[w];
                    }
            }
            if (bu < 0 || bu >= kp.U)
                bu = 0;
            const int cell = kp.tuple_cell[bu];
            if (out.cell)
                out.cell[slot] = cell;
            if (out.max_L)
                out.max_L[slot] = bv;
            if (out.xy) {
                const int cx = cell % kp.grid_W, cy = cell / kp.grid_W;
                out.xy[2 * slot] = (float)(cx - kp.half_w) / kp.grid_scale;
                out.xy[2 * slot + 1] = (float)(kp.half_h - cy) / kp.grid_scale;
            }
        }
    }
}

int fail_hip(hipError_t e, const char *what)
{
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return tdoa_set_error(-2, buf);
}

}  // namespace

size_t tdoa_stream_trigger_lds(int M, int N, int H)
{
    const size_t L = (size_t)N + H - 1;
    return ((M * L * 2 + 15) & ~(size_t)15) + (((L + 1) * 4 + 15) & ~(size_t)15) + (L + 1) * 8;
}

// the persistent register scan applies (N = 2H, config 5: N 1024, hop 512;
// aligned capture); it writes each frame at its stream's index
static bool trigger_p_applies(const tdoa_stream_params &sp)
{
    return sp.N == 2 * sp.H && ((uintptr_t)sp.capture & 3) == 0 &&
           sp.capture_len >= (int64_t)sp.N + 2 * sp.H && (sp.H == 256 || sp.H == 512 || sp.H == 1024) &&
           sp.M >= 2 && sp.M <= 4;
}

template <int G, int M>
static void launch_trigger_p(const tdoa_stream_params &sp, int64_t S, hipStream_t st)
{
    constexpr int NWB = TRIG_NWB;
    const size_t lds = (size_t)NWB * 3 * 64 * G * M;
    const int res = tdoa_resident_blocks((const void *)k_stream_trigger_p<G, M>, 64 * NWB, lds);
    int64_t grid = (S + NWB - 1) / NWB;
    if (res > 0 && grid > res)
        grid = res;
    // a wave lists at most 64 triggered streams (one per lane): <= 64 per wave
    const int64_t min_grid = (S + NWB * 64 - 1) / (NWB * 64);
    if (grid < min_grid)
        grid = min_grid;
    hipLaunchKernelGGL((k_stream_trigger_p<G, M>), dim3((unsigned)grid), dim3(64 * NWB), lds, st, sp, S);
}

template <int G>
static void launch_trigger_m(const tdoa_stream_params &sp, int64_t S, hipStream_t st)
{
    if (sp.M == 2)
        launch_trigger_p<G, 2>(sp, S, st);
    else if (sp.M == 3)
        launch_trigger_p<G, 3>(sp, S, st);
    else
        launch_trigger_p<G, 4>(sp, S, st);
}

int tdoa_launch_stream_trigger(const tdoa_stream_params &sp, int64_t S, void *stream, bool *by_id)
{
    hipStream_t st = (hipStream_t)stream;
    if (trigger_p_applies(sp)) {
        if (sp.H == 256)
            launch_trigger_m<4>(sp, S, st);
        else if (sp.H == 512)
            launch_trigger_m<8>(sp, S, st);
        else
            launch_trigger_m<16>(sp, S, st);
        *by_id = true;  // firing streams listed only: DIRECT reads their frames from the ring
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : fail_hip(e, "k_stream_trigger_p launch");
    }
    *by_id = false;  // frames in compact slots
    if (sp.H > TPB * MAX_CAND)
        return tdoa_set_error(-1, "stream: hop too large");
    const size_t lds = tdoa_stream_trigger_lds(sp.M, sp.N, sp.H);
    if (lds > 150 * 1024)
        return tdoa_set_error(-1, "stream: (frame_len + hop) x mics exceeds the LDS budget");
    hipLaunchKernelGGL(k_stream_trigger, dim3((unsigned)S), dim3(TPB), lds, st, sp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail_hip(e, "k_stream_trigger launch");
}

int tdoa_launch_stream_update(const tdoa_stream_params &sp, const tdoa_kparams &kp,
                              const tdoa_stream_kout &out, int64_t S, void *stream)
{
    const size_t lds = (size_t)kp.P * kp.K * 8;
    const int64_t grid = S < 2048 ? S : 2048;  // persistent: up to 8 workgroups per CU
    hipLaunchKernelGGL(k_stream_update, dim3((unsigned)(grid > 0 ? grid : 1)), dim3(TPB), lds, (hipStream_t)stream, sp,
                       kp, out, (int)S);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail_hip(e, "k_stream_update launch");
}
