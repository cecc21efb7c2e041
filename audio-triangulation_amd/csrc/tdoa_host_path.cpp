// tdoa_host_path.cpp -- libtdoa's own host-CPU implementation of the
// reference's per-frame hot-path symbols, selected with tdoa_ref_set_device(-1)
// (BASELINE config 1: "2-mic, 1024-sample frames ... on host CPU, no GPU").
// Plain C++ (built with g++ -ffp-contract=off: the lag prior and the EMA must
// round exactly as the reference's IEEE host build does); no HIP
// call is made on this path.
//
//   host_write_out    rolling_buffer.c:43-71   linearise, floor-mean DC, power
//   host_normalize    buffer.c:13-18           x <<= 8 (int16 wrap)
//   host_window       buffer.c:4-11            (int16)((x * W[i]) >> 15)
//   host_correlate    correlations.c:4-33      int64 xcorr, first max, prior
//   host_average      correlations.c:38-63     float EMA, first max
//
// The cross-correlation is the cost (93 lags x 1024 MACs per pair): each lag
// is a 1024-term dot product against a zero-padded copy of b, so every lag has
// the same trip count; AVX2 vpmaddwd forms pairs of int16 products (each
// |x| <= 32767 after the window, so a pair sum stays below 2^31) that are
// widened to int64 before they are summed -- exact for every input.

#include <immintrin.h>

#include <cstdint>
#include <cstring>

namespace tdoa_host {

constexpr int N = 1024, S = 46, K = 2 * S + 1;

void write_out(const int16_t *ring, int head, int16_t *dst, int64_t *power)
{
    int64_t total = 0;
    int i = 0;
    for (int j = head; j < N; i++, j++) {
        dst[i] = ring[j];
        total += ring[j];
    }
    for (int j = 0; j < head; i++, j++) {
        dst[i] = ring[j];
        total += ring[j];
    }
    const int16_t off = (int16_t)(total >> 10);  // arithmetic shift: floor
    int64_t p = 0;
    for (i = 0; i < N; i++) {
        dst[i] = (int16_t)(dst[i] - off);  // wraps, as the int16 compound assignment
        p += (int64_t)dst[i] * dst[i];
    }
    *power = p;
}

void normalize(int16_t *buf)
{
    // buffer.c:16 `buf->buffer[i] <<= 8`: only the low byte survives
    for (int i = 0; i < N; i++)
        buf[i] = (int16_t)(uint16_t)((uint32_t)(uint16_t)buf[i] << 8);
}

void window(int16_t *buf, const int16_t *w)
{
    for (int i = 0; i < N; i++)
        buf[i] = (int16_t)(((int32_t)buf[i] * (int32_t)w[i]) >> 15);
}

namespace {

void scores_scalar(const int16_t *a, const int16_t *bpad, int64_t *score)
{
    for (int k = 0; k < K; k++) {
        const int16_t *q = bpad + k;
        int64_t s = 0;
        for (int i = 0; i < N; i++)
            s += (int32_t)a[i] * (int32_t)q[i];
        score[k] = s;
    }
}

__attribute__((target("avx2"))) inline __m256i widen_add(__m256i acc, __m256i m)
{
    // 8 int32 pair sums -> two 4 x int64 halves, both added to acc (4 x int64)
    const __m256i lo = _mm256_cvtepi32_epi64(_mm256_castsi256_si128(m));
    const __m256i hi = _mm256_cvtepi32_epi64(_mm256_extracti128_si256(m, 1));
    return _mm256_add_epi64(acc, _mm256_add_epi64(lo, hi));
}

__attribute__((target("avx2"))) inline int64_t hsum64(__m256i v)
{
    alignas(32) int64_t t[4];
    _mm256_store_si256((__m256i *)t, v);
    return t[0] + t[1] + t[2] + t[3];
}

// four lags per pass share each 16-sample load of a
__attribute__((target("avx2"))) void scores_avx2(const int16_t *a, const int16_t *bpad, int64_t *score)
{
    int k = 0;
    for (; k + 4 <= K; k += 4) {
        __m256i c0 = _mm256_setzero_si256(), c1 = c0, c2 = c0, c3 = c0;
        const int16_t *q = bpad + k;
        for (int i = 0; i < N; i += 16) {
            const __m256i va = _mm256_loadu_si256((const __m256i *)(a + i));
            c0 = widen_add(c0, _mm256_madd_epi16(va, _mm256_loadu_si256((const __m256i *)(q + i))));
            c1 = widen_add(c1, _mm256_madd_epi16(va, _mm256_loadu_si256((const __m256i *)(q + i + 1))));
            c2 = widen_add(c2, _mm256_madd_epi16(va, _mm256_loadu_si256((const __m256i *)(q + i + 2))));
            c3 = widen_add(c3, _mm256_madd_epi16(va, _mm256_loadu_si256((const __m256i *)(q + i + 3))));
        }
        score[k] = hsum64(c0);
        score[k + 1] = hsum64(c1);
        score[k + 2] = hsum64(c2);
        score[k + 3] = hsum64(c3);
    }
    for (; k < K; k++) {
        __m256i c = _mm256_setzero_si256();
        const int16_t *q = bpad + k;
        for (int i = 0; i < N; i += 16)
            c = widen_add(c, _mm256_madd_epi16(_mm256_loadu_si256((const __m256i *)(a + i)),
                                               _mm256_loadu_si256((const __m256i *)(q + i))));
        score[k] = hsum64(c);
    }
}

bool have_avx2()
{
    static const bool yes = __builtin_cpu_supports("avx2");
    return yes;
}

// vpmaddwd's pair sum wraps only for (-32768)^2 + (-32768)^2: `a` without an
// INT16_MIN keeps every lane below 2^31
bool has_int16_min(const int16_t *a)
{
    int any = 0;
    for (int i = 0; i < N; i++)
        any |= a[i] == INT16_MIN;
    return any != 0;
}

}  // namespace

// correlations.c:7-33.  score[s + S] = sum_i a[i + max(0, -s)] * b[i + max(0, s)]
// over N - |s| terms, which is sum_{i < N} a[i] * bpad[S + s + i] for b placed at
// bpad[S] between zeros.  prior[d] = (float)exp((double)((float)(-d^2) / 36.f)).
void correlate(const int16_t *a, const int16_t *b, const float *prior, int64_t *corr, int *best)
{
    alignas(32) int16_t bpad[S + N + S + 16];
    std::memset(bpad, 0, sizeof bpad);
    std::memcpy(bpad + S, b, sizeof(int16_t) * N);
    if (have_avx2() && !has_int16_min(a))
        scores_avx2(a, bpad, corr);
    else
        scores_scalar(a, bpad, corr);
    int64_t bs = INT64_MIN;
    int bi = 0;
    for (int k = 0; k < K; k++)
        if (corr[k] > bs) {  // strict: the first (most negative) lag wins ties
            bs = corr[k];
            bi = k;
        }
    *best = bi - S;
    for (int k = 0; k < K; k++) {
        const int d = k > bi ? k - bi : bi - k;
        corr[k] = (int64_t)((float)corr[k] * prior[d]);  // RN to float, RN product, truncation
    }
}

// correlations.c:44-62: est += (float)(new - est) * decay in float (no FMA),
// truncated, then the first maximum
void average(int64_t *est, const int64_t *fresh, float decay, int *best)
{
    for (int k = 0; k < K; k++) {
        const float inc = (float)(fresh[k] - est[k]) * decay;
        est[k] = (int64_t)((float)est[k] + inc);
    }
    int64_t bs = INT64_MIN;
    for (int k = 0; k < K; k++)
        if (est[k] > bs) {
            bs = est[k];
            *best = k - S;
        }
}

}  // namespace tdoa_host
