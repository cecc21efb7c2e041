// tdoa_stream.cpp -- host side of the streaming pipeline (include/tdoa.h,
// kernels in tdoa_stream.hip): device state, the per-hop kernel sequence
//   k_stream_trigger -> k_direct_mfma (device-sized batch, EMA + grid on the
//   EMA scores fused) -- or, for shapes that kernel does not solve, k_direct ->
//   k_stream_update -- and its hipGraph capture / replay.  The hop's trigger
//   counter alternates between two slots by hop parity: the trigger zeroes the
//   other slot for the next hop (a memset node cost 3.9 us per hop), so the
//   two parities are two captured graphs.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "../../include/tdoa.h"
#include "tdoa_internal.h"

int tdoa_set_error(int code, const char *msg);
const tdoa_kparams *tdoa_ctx_kparams(const tdoa_ctx *c);
int tdoa_ctx_device(const tdoa_ctx *c);
int tdoa_ctx_engine(const tdoa_ctx *c);
int tdoa_ctx_rate(const tdoa_ctx *c);

struct tdoa_stream {
    tdoa_ctx *ctx;
    int device;
    int64_t S;
    tdoa_kparams kp;
    tdoa_stream_params sp;
    void *mem = nullptr;  // one allocation for all state
    size_t mem_bytes = 0;
    int use_graph;
    int64_t hop = 0;  // steps enqueued since create / reset: the counter slot's parity
    // captured step graphs (one per counter parity) and what they were captured for
    hipGraphExec_t exec[2] = {nullptr, nullptr};
    hipGraph_t graph[2] = {nullptr, nullptr};
    tdoa_stream_outputs g_out[2]{};
    hipStream_t g_stream[2] = {nullptr, nullptr};
};

namespace {

int sfail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return tdoa_set_error(code, buf);
}

#define S_TRY(expr)                                                            \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess)                                                  \
            return sfail(TDOA_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

tdoa_stream_kout to_kout(const tdoa_stream_outputs *o)
{
    tdoa_stream_kout k{};
    if (o) {
        k.count = o->count;
        k.stream_id = o->stream_id;
        k.end = o->end;
        k.lags = o->lags;
        k.gate = o->gate;
        k.ema_best = o->ema_best;
        k.cell = o->cell;
        k.xy = o->xy;
        k.max_L = o->max_L;
    }
    return k;
}

// the per-hop kernel sequence; par: the hop's counter slot
int enqueue_step(tdoa_stream *st, const tdoa_stream_outputs *out, hipStream_t s, int par)
{
    tdoa_stream_params sp = st->sp;
    sp.count = st->sp.count + par;
    sp.count_next = st->sp.count + (1 - par);
    bool by_id = false;  // where DIRECT finds the frames: the capture ring or compact copies
    int rc = tdoa_launch_stream_trigger(sp, st->S, s, &by_id);
    if (rc)
        return rc;
    tdoa_kparams kp = st->kp;
    if (by_id) {  // listed only: DIRECT stages each frame from its stream's ring
        kp.frame_ids = sp.ids;
        kp.frame_ring = sp.capture;
        kp.ring_len = sp.capture_len;
        kp.frame_end = sp.end;
        kp.frame_ring_at = sp.ring_at;
    }
    kp.frames_u8 = 1;  // k_stream_trigger's compact copies are 8-bit
    if (tdoa_direct_ema_fits(kp)) {
        // k_direct_mfma runs the EMA and the grid on the EMA scores itself:
        // results straight into the caller's slots, no fresh-score round trip
        tdoa_stream_fuse ef{};
        ef.sp = sp;
        ef.so = to_kout(out);
        tdoa_kout ko{};
        ko.lags = ef.so.lags ? ef.so.lags : sp.fresh_lags;
        ko.gate = ef.so.gate;
        ko.cell = ef.so.cell;
        ko.xy = ef.so.xy;
        ko.max_L = ef.so.max_L;
        return tdoa_launch_direct(kp, ko, sp.frames, st->S, false, s, nullptr, sp.count, &ef);
    }
    tdoa_kout ko{};
    ko.lags = sp.fresh_lags;
    ko.gate = sp.fresh_gate;
    ko.weighted = sp.fresh;
    rc = tdoa_launch_direct(kp, ko, sp.frames, st->S, false, s, nullptr, sp.count);
    if (rc)
        return rc;
    return tdoa_launch_stream_update(sp, st->kp, to_kout(out), st->S, s);
}

void drop_graph(tdoa_stream *st, int par)
{
    if (st->exec[par])
        (void)hipGraphExecDestroy(st->exec[par]);
    if (st->graph[par])
        (void)hipGraphDestroy(st->graph[par]);
    st->exec[par] = nullptr;
    st->graph[par] = nullptr;
}

}  // namespace

extern "C" int tdoa_stream_create(tdoa_ctx *ctx, int32_t num_streams, int32_t hop,
                                  const uint8_t *capture, int64_t capture_len, int use_graph,
                                  tdoa_stream **out)
{
    if (!ctx || !out || !capture)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_create: NULL argument");
    *out = nullptr;
    if (tdoa_ctx_engine(ctx) != TDOA_ENGINE_DIRECT)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_create: needs a DIRECT context");
    const tdoa_kparams &kp = *tdoa_ctx_kparams(ctx);
    const int M = kp.M, N = kp.N, P = kp.P, K = kp.K;
    if (num_streams < 1)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_create: num_streams %d < 1", num_streams);
    if (hop < 1 || hop > N || hop > 4096)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_create: hop %d outside [1, frame_len]", hop);
    if (capture_len < (int64_t)N + 2 * hop)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_create: capture_len %lld < frame_len + 2 hop",
                     (long long)capture_len);
    if (tdoa_stream_trigger_lds(M, N, hop) > 150 * 1024)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_create: (frame_len + hop) x mics too large");
    const int dev = tdoa_ctx_device(ctx);
    S_TRY(hipSetDevice(dev));

    tdoa_stream *st = new tdoa_stream();
    st->ctx = ctx;
    st->device = dev;
    st->S = num_streams;
    st->kp = kp;
    st->use_graph = use_graph;
    const size_t S = (size_t)num_streams;
    // carve: 256-B aligned sub-buffers of one allocation
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_pos = take(8), o_count = take(8), o_rs = take(S * 8), o_ids = take(S * 4),
                 o_end = take(S * 8), o_at = take(S * 8), o_frames = take(S * M * N), o_fresh = take(S * P * K * 8),
                 o_fl = take(S * P * 4), o_fg = take(S), o_est = take(S * P * K * 8),
                 o_last = take(S * 8), o_stats = take(16);
    if (hipMalloc(&st->mem, off) != hipSuccess) {
        delete st;
        return sfail(TDOA_ERR_NOMEM, "tdoa_stream_create: %zu bytes of stream state", off);
    }
    st->mem_bytes = off;
    char *b = (char *)st->mem;
    tdoa_stream_params &sp = st->sp;
    sp.M = M;
    sp.N = N;
    sp.H = hop;
    sp.log2N = kp.log2N;
    sp.fs = tdoa_ctx_rate(ctx);
    sp.capture_len = capture_len;
    sp.capture = capture;
    sp.pos = (int64_t *)(b + o_pos);
    sp.count = (int32_t *)(b + o_count);
    sp.ring_start = (int64_t *)(b + o_rs);
    sp.ids = (int32_t *)(b + o_ids);
    sp.end = (int64_t *)(b + o_end);
    sp.ring_at = (int64_t *)(b + o_at);
    sp.frames = (int16_t *)(b + o_frames);
    sp.fresh = (int64_t *)(b + o_fresh);
    sp.fresh_lags = (int32_t *)(b + o_fl);
    sp.fresh_gate = (uint8_t *)(b + o_fg);
    sp.est = (int64_t *)(b + o_est);
    sp.last = (uint64_t *)(b + o_last);
    sp.stats = (int64_t *)(b + o_stats);
    if (hipMemset(st->mem, 0, off) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(st->mem);
        delete st;
        return sfail(TDOA_ERR_HIP, "tdoa_stream_create: clearing state failed");
    }
    *out = st;
    return TDOA_OK;
}

extern "C" int tdoa_stream_step(tdoa_stream *st, const tdoa_stream_outputs *out, void *stream)
{
    if (!st)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_step: NULL stream");
    S_TRY(hipSetDevice(st->device));
    hipStream_t s = (hipStream_t)stream;
    const int par = (int)(st->hop & 1);
    if (!st->use_graph || !s) {
        const int rc = enqueue_step(st, out, s, par);
        if (!rc) {
            st->hop++;
        } else {
            // a launch after the trigger failed: the trigger may have counted
            // into this hop's slot without the hop advancing; both slots are
            // zeroed so the next hop's slot base starts at 0 again
            (void)hipMemsetAsync(st->sp.count, 0, 2 * sizeof(int32_t), s);
        }
        return rc;
    }
    const tdoa_stream_outputs want = out ? *out : tdoa_stream_outputs{};
    if (!st->exec[par] || st->g_stream[par] != s || std::memcmp(&want, &st->g_out[par], sizeof want) != 0) {
        drop_graph(st, par);
        S_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        const int rc = enqueue_step(st, out, s, par);
        hipGraph_t g = nullptr;
        const hipError_t ec = hipStreamEndCapture(s, &g);
        if (rc) {
            if (g)
                (void)hipGraphDestroy(g);
            return rc;
        }
        if (ec != hipSuccess)
            return sfail(TDOA_ERR_HIP, "hipStreamEndCapture: %s", hipGetErrorString(ec));
        st->graph[par] = g;
        S_TRY(hipGraphInstantiate(&st->exec[par], g, nullptr, nullptr, 0));
        st->g_out[par] = want;
        st->g_stream[par] = s;
    }
    const hipError_t el = hipGraphLaunch(st->exec[par], s);
    if (el != hipSuccess) {
        // as in the eager path: a partly run hop may have counted into its
        // slot; both slots are zeroed so the next hop starts from slot 0
        (void)hipMemsetAsync(st->sp.count, 0, 2 * sizeof(int32_t), s);
        return sfail(TDOA_ERR_HIP, "hipGraphLaunch: %s", hipGetErrorString(el));
    }
    st->hop++;
    return TDOA_OK;
}

extern "C" int tdoa_stream_reset(tdoa_stream *st, void *stream)
{
    if (!st)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_reset: NULL stream");
    S_TRY(hipSetDevice(st->device));
    S_TRY(hipMemsetAsync(st->mem, 0, st->mem_bytes, (hipStream_t)stream));
    st->hop = 0;  // both counter slots are zero again
    return TDOA_OK;
}

extern "C" int tdoa_stream_state(tdoa_stream *st, int64_t *pos, int64_t *est, uint64_t *last,
                                 int64_t *stats)
{
    if (!st)
        return sfail(TDOA_ERR_INVALID, "tdoa_stream_state: NULL stream");
    S_TRY(hipSetDevice(st->device));
    S_TRY(hipDeviceSynchronize());
    const size_t S = (size_t)st->S;
    if (pos)
        S_TRY(hipMemcpy(pos, st->sp.pos, sizeof(int64_t), hipMemcpyDeviceToHost));
    if (est)
        S_TRY(hipMemcpy(est, st->sp.est, S * st->kp.P * st->kp.K * sizeof(int64_t),
                        hipMemcpyDeviceToHost));
    if (last)
        S_TRY(hipMemcpy(last, st->sp.last, S * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (stats)
        S_TRY(hipMemcpy(stats, st->sp.stats, 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
    return TDOA_OK;
}

extern "C" int tdoa_stream_destroy(tdoa_stream *st)
{
    if (!st)
        return TDOA_OK;
    (void)hipSetDevice(st->device);
    (void)hipDeviceSynchronize();
    drop_graph(st, 0);
    drop_graph(st, 1);
    (void)hipFree(st->mem);
    delete st;
    return TDOA_OK;
}
