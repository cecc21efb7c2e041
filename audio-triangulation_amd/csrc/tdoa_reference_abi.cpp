// tdoa_reference_abi.cpp -- the reference's per-frame component symbols
// (include/tdoa_reference_abi.h) on top of libtdoa.
//
// GPU-backed (one-frame launches, synchronous, abort on HIP failure):
//   rolling_buffer_write_out  rolling_buffer.c:43-71 (its launch also computes
//                             the next two ops on its output, see buffer_op)
//   buffer_normalize_range    buffer.c:13-18
//   buffer_window             buffer.c:4-11
//   correlations_init         correlations.c:4-36   (via tdoa_correlate_prepared)
//   correlations_average      correlations.c:38-63  (via tdoa_average_batch)
// Host (capture ring / one-time geometry):
//   rolling_buffer_init/push/get_*_power  rolling_buffer.c:3-41,73-85
//   microphones_init                      microphones.c:9-33
// tdoa_ref_set_device(-1) runs the GPU-backed five on libtdoa's own host-CPU
// implementation instead (tdoa_host_path.cpp; BASELINE config 1 "on host CPU,
// no GPU"): same results bit for bit, and no HIP call at all.

#include "../../include/tdoa_reference_abi.h"
#include "../../include/tdoa.h"
#include "tdoa_internal.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <time.h>

namespace tdoa_host {
void write_out(const int16_t *ring, int head, int16_t *dst, int64_t *power);
void normalize(int16_t *buf);
void window(int16_t *buf, const int16_t *w);
void correlate(const int16_t *a, const int16_t *b, const float *prior, int64_t *corr, int *best);
void average(int64_t *est, const int64_t *fresh, float decay, int *best);
}  // namespace tdoa_host

int tdoa_ctx_device(const tdoa_ctx *c);
int tdoa_launch_ref_buffer(int op, int16_t *buf, const int16_t *ring, int head, int64_t *power,
                           const int16_t *window, int n, void *stream, int16_t *s1, int16_t *s2);

point2d_t mic_a_location;
point2d_t mic_b_location;
point2d_t mic_c_location;

static_assert(sizeof(struct buffer_t) == 2056, "buffer_t layout (x86-64)");
static_assert(sizeof(struct correlations_t) == 760, "correlations_t layout (x86-64)");
static_assert(sizeof(struct rolling_buffer_t) == 2096, "rolling_buffer_t layout (x86-64)");
static_assert(offsetof(struct rolling_buffer_t, buffer) == 42, "rolling_buffer_t.buffer offset");

namespace {

absolute_time_t default_clock()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (absolute_time_t)ts.tv_sec * 1000000u + (absolute_time_t)(ts.tv_nsec / 1000);
}

absolute_time_t (*g_clock)(void) = default_clock;
std::atomic<int> g_device{0};  // < 0: the host-CPU path (tdoa_host_path.cpp)

bool host_mode() { return g_device.load(std::memory_order_relaxed) < 0; }

// the host path's tables: the Q15 DPSS(1024, 2) window (window_function.h) and
// the lag prior of correlations.c:27-30, built once with libm on the host
struct HostTables {
    int16_t window[TDOA_REF_BUFFER_SIZE];
    float prior[TDOA_REF_CORR_SIZE];
};
const HostTables &host_tables()
{
    static const HostTables t = [] {
        HostTables h;
        int32_t w[TDOA_REF_BUFFER_SIZE];
        if (tdoa_dpss_q15(TDOA_REF_BUFFER_SIZE, 2.0, w) != TDOA_OK) {
            std::fprintf(stderr, "libtdoa reference shim: tdoa_dpss_q15 failed\n");
            std::abort();
        }
        for (int i = 0; i < TDOA_REF_BUFFER_SIZE; i++)
            h.window[i] = (int16_t)w[i];
        for (int d = 0; d < TDOA_REF_CORR_SIZE; d++)
            h.prior[d] = (float)std::exp((double)((float)(-(d * d)) / 36.f));
        return h;
    }();
    return t;
}

// One lazily created 2-mic context (pair = (buf_a, buf_b)), its stream and
// one block of pinned, device-mapped host memory the per-frame kernels read
// and write directly: a call is a host copy in, one launch, one stream
// synchronisation and a host copy out (no hipMemcpy round trips).  The
// reference's functions are single-threaded; guard anyway.
struct HostIO {
    int16_t frames[2][TDOA_REF_BUFFER_SIZE];  // buffers a, b (16-B aligned rows)
    int16_t ring[TDOA_REF_BUFFER_SIZE];
    int16_t chain[2][TDOA_REF_BUFFER_SIZE];   // write_out's output normalised, then windowed
    int64_t i64[4 * 128];                     // weighted / est / fresh
    int64_t power;
    int32_t i32[64];                          // best lags
    float f32[64];                            // decay
};
struct RefState {
    std::mutex mu;
    std::atomic<bool> ready{false};  // published after the state below (double-checked init)
    tdoa_ctx *ctx = nullptr;
    hipStream_t st = nullptr;
    HostIO *io = nullptr;          // pinned, mapped: host and kernels address it alike
    int16_t *d_window = nullptr;   // Q15 DPSS(1024, 2)
} g_ref;

[[noreturn]] void die(const char *what)
{
    std::fprintf(stderr, "libtdoa reference shim: %s: %s\n", what, tdoa_last_error());
    std::abort();
}

void check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        std::fprintf(stderr, "libtdoa reference shim: %s: %s\n", what, hipGetErrorString(e));
        std::abort();
    }
}

RefState &ref()
{
    if (g_ref.ready.load(std::memory_order_acquire))
        return g_ref;
    std::lock_guard<std::mutex> lk(g_ref.mu);
    if (g_ref.ready.load(std::memory_order_relaxed))
        return g_ref;
    tdoa_config cfg;
    tdoa_config_default(&cfg);
    cfg.num_mics = 2;
    const float two_mics[4] = {-0.066f, 0.0f, 0.066f, 0.0f};  // grid unused here
    cfg.mic_xy = two_mics;
    cfg.grid_half_w = 0;
    cfg.grid_half_h = 0;
    if (tdoa_create(&cfg, g_device.load(), &g_ref.ctx) != TDOA_OK)
        die("tdoa_create");
    check(hipSetDevice(g_device.load()), "hipSetDevice");
    check(hipStreamCreateWithFlags(&g_ref.st, hipStreamNonBlocking), "hipStreamCreate");
    check(hipHostMalloc(reinterpret_cast<void **>(&g_ref.io), sizeof(HostIO),
                        hipHostMallocMapped | hipHostMallocCoherent),
          "hipHostMalloc");
    check(hipMalloc(&g_ref.d_window, 1024 * sizeof(int16_t)), "hipMalloc");
    int32_t w[1024];
    tdoa_get_window(g_ref.ctx, w);
    int16_t w16[1024];
    for (int i = 0; i < 1024; i++)
        w16[i] = (int16_t)w[i];
    check(hipMemcpy(g_ref.d_window, w16, sizeof w16, hipMemcpyHostToDevice), "hipMemcpy");
    g_ref.ready.store(true, std::memory_order_release);
    return g_ref;
}

// The frame path's ops after write_out (sample_compute.h:105-118 order:
// buffer_normalize_range, then buffer_window) are computed by write_out's own
// launch on its output and kept as (input -> output) records.  A later
// normalize / window call on a buffer holding exactly a recorded input returns
// the recorded output -- the GPU's result for that very input -- instead of a
// launch of its own; any other buffer takes its own launch.  Per frame of two
// mics: three GPU round trips (two write_outs, correlations_init) instead of seven.
struct Memo {
    bool valid = false;
    int16_t in[TDOA_REF_BUFFER_SIZE];
    int16_t out[TDOA_REF_BUFFER_SIZE];
};
constexpr int MEMO_SLOTS = 4;  // a few buffers in flight (two mics interleave)
struct Memos {
    std::mutex mu;
    Memo norm[MEMO_SLOTS], win[MEMO_SLOTS];
    int next = 0;
} g_memo;

bool memo_hit(Memo (&m)[MEMO_SLOTS], int16_t *buf)
{
    for (Memo &e : m)
        if (e.valid && std::memcmp(e.in, buf, sizeof e.in) == 0) {
            std::memcpy(buf, e.out, sizeof e.out);
            return true;
        }
    return false;
}

// One op of k_ref_buffer on a single 1024-sample buffer, in place in the
// mapped host block
void buffer_op(int op, struct buffer_t *dst, const struct rolling_buffer_t *ring)
{
    RefState &R = ref();
    if (op != 0) {
        std::lock_guard<std::mutex> lk(g_memo.mu);
        if (memo_hit(op == 1 ? g_memo.norm : g_memo.win, dst->buffer))
            return;
    }
    check(hipSetDevice(g_device.load()), "hipSetDevice");
    HostIO &io = *R.io;
    int16_t *buf = io.frames[0];
    if (ring)
        std::memcpy(io.ring, ring->buffer, sizeof ring->buffer);
    else
        std::memcpy(buf, dst->buffer, sizeof dst->buffer);
    if (tdoa_launch_ref_buffer(op, buf, io.ring, ring ? ring->head : 0, &io.power, R.d_window,
                               TDOA_REF_BUFFER_SIZE, R.st, op == 0 ? io.chain[0] : nullptr,
                               op == 0 ? io.chain[1] : nullptr) != 0)
        die("k_ref_buffer");
    check(hipStreamSynchronize(R.st), "hipStreamSynchronize");
    std::memcpy(dst->buffer, buf, sizeof dst->buffer);
    if (op == 0) {
        dst->power = io.power;
        std::lock_guard<std::mutex> lk(g_memo.mu);
        const int k = g_memo.next;
        g_memo.next = (k + 1) % MEMO_SLOTS;
        Memo &n = g_memo.norm[k], &w = g_memo.win[k];
        std::memcpy(n.in, buf, sizeof n.in);
        std::memcpy(n.out, io.chain[0], sizeof n.out);
        std::memcpy(w.in, io.chain[0], sizeof w.in);
        std::memcpy(w.out, io.chain[1], sizeof w.out);
        n.valid = w.valid = true;
    }
}

}  // namespace

extern "C" void tdoa_ref_set_clock(absolute_time_t (*now_us)(void))
{
    g_clock = now_us ? now_us : default_clock;
}

extern "C" int tdoa_ref_set_device(int device)
{
    // -1 (any negative): the host-CPU path, selectable at any time; a GPU
    // device only before the first GPU-backed call (its context is bound to it),
    // or the device already in use
    if (device >= 0 && g_ref.ready.load(std::memory_order_acquire) && g_ref.ctx &&
        device != tdoa_ctx_device(g_ref.ctx))
        return TDOA_ERR_INVALID;
    g_device = device < 0 ? -1 : device;
    return TDOA_OK;
}

// ------------------------------------------------------------ microphones
// microphones.c:9-33 (MIRROR_MICROPHONES true, ROTATE_MICROPHONES false)
extern "C" void microphones_init(void)
{
    const float dAB = 0.132f, dBC = 0.15f, dCA = 0.20f;
    const float xC = (dAB * dAB + dCA * dCA - dBC * dBC) / (2.0f * dAB);
    const float yC = sqrtf(fmaxf(0.0f, dCA * dCA - xC * xC));
    const point2d_t pA = {0.0f, 0.0f}, pB = {dAB, 0.0f}, pC = {xC, yC * -1.0f};
    const float cx = (pA.x + pB.x + pC.x) / 3.0f;
    const float cy = (pA.y + pB.y + pC.y) / 3.0f;
    mic_a_location = {pA.x - cx, pA.y - cy};
    mic_b_location = {pB.x - cx, pB.y - cy};
    mic_c_location = {pC.x - cx, pC.y - cy};
}

// ------------------------------------------------------ capture ring (host)
extern "C" void rolling_buffer_init(struct rolling_buffer_t *b)
{
    b->head = 0;
    b->incoming_power = b->incoming_total = 0;
    b->outgoing_power = b->outgoing_total = 0;
    b->is_full = false;
    std::memset(b->buffer, 0, sizeof b->buffer);
}

// rolling_buffer.c:16-41: the sample at head-N/2 crosses from the newer half
// to the older half; the sample at head leaves the older half.
extern "C" void rolling_buffer_push(struct rolling_buffer_t *b, sample_t sample)
{
    const int n = TDOA_REF_BUFFER_SIZE;
    int mid = b->head - n / 2;
    if (mid < 0)
        mid += n;
    const int64_t m = b->buffer[mid], o = b->buffer[b->head], s = sample;
    b->outgoing_total += m - o;
    b->outgoing_power += m * m - o * o;
    b->incoming_total += s - m;
    b->incoming_power += s * s - m * m;
    b->buffer[b->head] = sample;
    if (++b->head >= n) {
        b->head = 0;
        b->is_full = true;
    }
}

// rolling_buffer.c:73-85 with BUFFER_HALF_SIZE_BITS = 9
extern "C" power_t rolling_buffer_get_incoming_power(const struct rolling_buffer_t *b)
{
    return (power_t)((uint64_t)b->incoming_power << 9) - b->incoming_total * b->incoming_total;
}

extern "C" power_t rolling_buffer_get_outgoing_power(const struct rolling_buffer_t *b)
{
    return (power_t)((uint64_t)b->outgoing_power << 9) - b->outgoing_total * b->outgoing_total;
}

// ------------------------------------------------------------- GPU-backed
extern "C" void rolling_buffer_write_out(const struct rolling_buffer_t *b, struct buffer_t *dst)
{
    if (host_mode()) {
        tdoa_host::write_out(b->buffer, b->head, dst->buffer, &dst->power);
        return;
    }
    buffer_op(0, dst, b);
}

extern "C" void buffer_normalize_range(struct buffer_t *buf)
{
    if (host_mode()) {
        tdoa_host::normalize(buf->buffer);
        return;
    }
    buffer_op(1, buf, nullptr);
}

extern "C" void buffer_window(struct buffer_t *buf)
{
    if (host_mode()) {
        tdoa_host::window(buf->buffer, host_tables().window);
        return;
    }
    buffer_op(2, buf, nullptr);
}

extern "C" void correlations_init(struct correlations_t *corr, const struct buffer_t *a,
                                  const struct buffer_t *b)
{
    if (host_mode()) {
        tdoa_host::correlate(a->buffer, b->buffer, host_tables().prior, corr->correlations, &corr->best_shift);
        corr->last_update = g_clock();
        return;
    }
    RefState &R = ref();
    check(hipSetDevice(g_device.load()), "hipSetDevice");
    HostIO &io = *R.io;
    std::memcpy(io.frames[0], a->buffer, sizeof a->buffer);
    std::memcpy(io.frames[1], b->buffer, sizeof b->buffer);
    tdoa_outputs o;
    std::memset(&o, 0, sizeof o);
    o.lags = io.i32;
    o.weighted = io.i64;
    if (tdoa_correlate_prepared(R.ctx, &io.frames[0][0], 1, &o, R.st) != TDOA_OK)
        die("correlations_init");
    check(hipStreamSynchronize(R.st), "hipStreamSynchronize");
    std::memcpy(corr->correlations, io.i64, sizeof corr->correlations);
    corr->best_shift = io.i32[0];
    corr->last_update = g_clock();
}

extern "C" void correlations_average(struct correlations_t *est, struct correlations_t *fresh)
{
    if (host_mode()) {
        const absolute_time_t now = g_clock();
        tdoa_host::average(est->correlations, fresh->correlations, tdoa_decay_us(now, est->last_update),
                           &est->best_shift);
        est->last_update = now;
        return;
    }
    RefState &R = ref();
    check(hipSetDevice(g_device.load()), "hipSetDevice");
    HostIO &io = *R.io;
    const absolute_time_t now = g_clock();
    int64_t *h_est = io.i64, *h_new = io.i64 + 128;
    std::memcpy(h_est, est->correlations, sizeof est->correlations);
    std::memcpy(h_new, fresh->correlations, sizeof fresh->correlations);
    io.f32[0] = tdoa_decay_us(now, est->last_update);
    if (tdoa_average_batch(R.ctx, 1, h_est, h_new, io.f32, io.i32, nullptr, R.st) != TDOA_OK)
        die("correlations_average");
    check(hipStreamSynchronize(R.st), "hipStreamSynchronize");
    std::memcpy(est->correlations, h_est, sizeof est->correlations);
    est->best_shift = io.i32[0];
    est->last_update = now;
}
