// engine.cpp -- C ABI of the MI355X SDA engine (include/sda_engine.h).
//
// Host-side responsibilities only: argument validation with the reference's error behaviour
// (Err strings of client/src/crypto/sharing/*.rs -> status 1..6, assert!/panic -> PRECONDITION),
// staging of host buffers to HBM, kernel launches (kernels.h) and copying results back.  No
// arithmetic on the data happens here and there is no CPU fallback: if the device path fails
// the call fails.
#include "../../include/sda_engine.h"

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"

struct sda_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    void* work = nullptr;
    size_t work_bytes = 0;
    void* stage = nullptr;        // staging for host-path inputs/outputs
    size_t stage_bytes = 0;
    sda::DeviceTable gen_tab;     // packed-Shamir twiddles (per scheme)
    void* gen_log = nullptr;      // packed-Shamir generic fix-up log (sda::packed_gen_log_bytes())
    size_t gen_log_bytes = 0;
    void* codec_work = nullptr;   // varint codec plan / scan workspace
    size_t codec_work_bytes = 0;
    void* codec_mat = nullptr;    // decoded [N][len] matrix of the clerk decode+combine path
    size_t codec_mat_bytes = 0;
    void* pipe = nullptr;         // recipient / participant pipeline scratch (mask, masked, compacted shares)
    size_t pipe_bytes = 0;
    sda::DeviceTable rev_tab;     // packed-Shamir Newton/Lagrange tables (per scheme + clerk set)
    void* snap = nullptr;         // snapshot transposition copy plan
    size_t snap_bytes = 0;
    // The scratch buffers above are shared by every call on the handle.  A call on another stream
    // than the previous one first waits (on the device) for the work queued on that stream.
    hipStream_t last_stream = nullptr;
    hipEvent_t order_ev = nullptr;
    bool order_ok = true;         // order_ev was recorded when the last call ended (else: host sync)
    unsigned long long* rej_host = nullptr;   // pinned: the ChaCha rejection count of a pipeline's mask
};

namespace {

thread_local std::string g_last_error;

// The handle and stream of the call in progress on this thread (set by pick()): when the call returns,
// its stream records the handle's order event, so the NEXT call -- on whatever stream -- only waits on
// that event and never touches this call's stream again (the caller may destroy it in between).
thread_local sda_engine* t_call_h = nullptr;
thread_local hipStream_t t_call_s = nullptr;

void end_call() {
    if (t_call_h) {
        t_call_h->order_ok = hipEventRecord(t_call_h->order_ev, t_call_s) == hipSuccess;
        t_call_h = nullptr;
    }
}

// Every extern "C" entry point opens a CallScope (SDA_ENTRY) as its first statement; the outermost scope
// ends the call's ordering scope (end_call) on every return path, after everything the call queued.
// Internal helpers -- and entry points called from entry points -- may return ok()/fail() freely.
thread_local int t_depth = 0;
struct CallScope {
    CallScope() { ++t_depth; }
    ~CallScope() {
        if (--t_depth == 0) end_call();
    }
    CallScope(const CallScope&) = delete;
    CallScope& operator=(const CallScope&) = delete;
};
#define SDA_ENTRY CallScope sda_call_scope_

sda_status fail(sda_status st, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return st;
}

sda_status ok() {
    g_last_error.clear();
    return SDA_OK;
}

// A failed HIP call also sets the thread's sticky last-error, which the caller's own runtime checks (torch's
// hipGetLastError after each launch) would then report against their next, unrelated op: the status we
// return carries the error, so the sticky copy is cleared.
#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            (void)hipGetLastError();                                                               \
            return fail(_e == hipErrorOutOfMemory ? SDA_ERR_OUT_OF_MEMORY : SDA_ERR_DEVICE,        \
                        "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
        }                                                                                          \
    } while (0)

sda_status ensure(void** buf, size_t* have, size_t need) {
    if (need <= *have) return SDA_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    size_t want = need + need / 4 + 4096;
    HIP_TRY(hipMalloc(buf, want));
    *have = want;
    return SDA_OK;
}

// `_dev` entry points run on the caller's stream; NULL is the HIP null (default) stream, which is
// also what torch's default stream reports -- so work stays ordered with the caller's own ops.
// Switching streams orders the new stream after the previous call (event wait, no host sync), so a
// call never reuses a scratch buffer that work queued on another stream may still be reading.  The
// event was recorded on the previous call's stream when that call returned (end_call), so the previous
// stream itself is never touched here and may have been destroyed since.
hipStream_t pick(sda_engine* h, void* stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (s != h->last_stream) {
        // a failed record leaves a stale event: order from the host instead (the previous stream may be
        // gone, so the whole device)
        if (!h->order_ok || hipStreamWaitEvent(s, h->order_ev, 0) != hipSuccess) (void)hipDeviceSynchronize();
        h->last_stream = s;
    }
    t_call_h = h;
    t_call_s = s;
    return s;
}

bool is_pow(uint64_t x, uint64_t b) {
    if (x < 1) return false;
    while (x % b == 0) x /= b;
    return x == 1;
}

// Rust `x % m` with m < 0 equals `x % |m|`; m == 0 panics.
sda_status modulus_abs(int64_t m, int64_t* out) {
    if (m == 0) return fail(SDA_ERR_PRECONDITION, "attempt to calculate the remainder with a divisor of zero");
    if (m == INT64_MIN) return fail(SDA_ERR_UNSUPPORTED, "modulus i64::MIN is outside the engine's domain");
    *out = m < 0 ? -m : m;
    return SDA_OK;
}

// Packed-Shamir parameter domain of the engine (DESIGN.md "Domain").
sda_status check_packed(const sda_sharing_scheme* s) {
    const uint64_t k = s->secret_count, t = s->privacy_threshold, n = s->share_count;
    const int64_t p = s->modulus;
    if (k == 0) return fail(SDA_ERR_UNSUPPORTED, "secret_count must be >= 1");
    if (n + 1 < k + t + 1)   // tss: vec![0; share_count - reconstruct_limit()] underflows
        return fail(SDA_ERR_PRECONDITION, "share_count (%llu) < secret_count + privacy_threshold (%llu)",
                    (unsigned long long)n, (unsigned long long)(k + t));
    if (!is_pow(k + t + 1, 2) || k + t + 1 > sda::kWideMaxL)
        return fail(SDA_ERR_UNSUPPORTED, "secret_count + privacy_threshold + 1 = %llu must be a power of 2 <= %u",
                    (unsigned long long)(k + t + 1), sda::kWideMaxL);
    if (!is_pow(n + 1, 3) || n + 1 > sda::kWideMaxN3)
        return fail(SDA_ERR_UNSUPPORTED, "share_count + 1 = %llu must be a power of 3 <= %u",
                    (unsigned long long)(n + 1), sda::kWideMaxN3);
    if (p < 3 || p % 2 == 0 || p >= ((int64_t)1 << 31))
        return fail(SDA_ERR_UNSUPPORTED, "prime_modulus %lld must be odd and < 2^31 (tss i64 headroom)",
                    (long long)p);
    if (s->omega_secrets <= 0 || s->omega_secrets >= p || s->omega_shares <= 0 || s->omega_shares >= p)
        return fail(SDA_ERR_UNSUPPORTED, "omega_secrets / omega_shares must lie in (0, p)");
    return SDA_OK;
}

// upload n rows of `len` elements each into a dense [n][len] device buffer
sda_status upload_rows(sda_engine* h, int64_t* dst, const int64_t* const* rows, uint64_t n, uint64_t len) {
    uint64_t i = 0;
    while (i < n) {
        uint64_t j = i + 1;   // coalesce rows that are contiguous in host memory
        while (j < n && rows[j] == rows[j - 1] + len) ++j;
        if (len) HIP_TRY(hipMemcpyAsync(dst + i * len, rows[i], (j - i) * len * 8, hipMemcpyHostToDevice, h->stream));
        i = j;
    }
    return SDA_OK;
}

struct DevArena {   // bump allocator over the engine's staging buffer
    char* base;
    size_t off = 0;
    template <typename T> T* take(size_t count) {
        T* p = reinterpret_cast<T*>(base + off);
        off += (count * sizeof(T) + 255) & ~(size_t)255;
        return p;
    }
};

sda_status stage(sda_engine* h, size_t bytes, DevArena* a) {
    (void)pick(h, h->stream);                  // host entry points run on the engine's own stream
    sda_status st = ensure(&h->stage, &h->stage_bytes, bytes + 4096);
    if (st) return st;
    a->base = static_cast<char*>(h->stage);
    a->off = 0;
    return SDA_OK;
}

size_t rup(size_t b) { return (b + 255) & ~(size_t)255; }

// chacha.rs:57-76: combine of n seed streams ([n][w] u32 words on the device) into out (device, D
// values).  The fast counter-mode kernel where its rejection log suffices; otherwise (moduli above
// 2^62, high rejection rates, or a log overflow) the exact stream path.
sda_status chacha_combine(sda_engine* h, int64_t m, uint64_t D, const uint32_t* seeds, uint32_t w, uint64_t n,
                          int64_t* out, hipStream_t st) {
    if (D == 0) return SDA_OK;
    // SDA_CHACHA_PATH=stream: test hook forcing the stream path (both paths are exact; the tests
    // compare them at sizes the oracle cannot finish)
    const char* force = getenv("SDA_CHACHA_PATH");
    if (!sda::chacha_needs_stream_path(m) && !(force && strcmp(force, "stream") == 0)) {
        if (sda_status e = ensure(&h->work, &h->work_bytes, sda::chacha_work_bytes(D, n))) return e;
        bool overflow = false;
        int fixups = 0;
        HIP_TRY(sda::launch_chacha_mask_combine(m, D, seeds, w, n, out, h->work, st, &overflow, &fixups));
        if (!overflow) return SDA_OK;
    }
    if (sda_status e = ensure(&h->work, &h->work_bytes, sda::chacha_stream_work_bytes(D, n, m))) return e;
    HIP_TRY(sda::launch_chacha_streams_combine(m, D, seeds, w, n, out, h->work, st));
    return SDA_OK;
}

// chacha_combine for a pipeline that keeps queueing work behind the mask: the rejection count is copied
// to the handle's pinned word instead of being waited for, and chacha_combine_end -- called after the
// pipeline's own final stream sync -- applies the fix-ups (each draw is rejected with probability
// < 2^-28 on this path, so a call rarely has any).  *changed tells the caller to redo what it queued on
// `out`.  Moduli that need the stream path run it synchronously in _begin, as chacha_combine does.
struct PendingChacha {
    bool pending = false;
    int64_t m = 0;
    uint64_t D = 0, n = 0;
    const uint32_t* seeds = nullptr;
    uint32_t w = 0;
    int64_t* out = nullptr;
};
sda_status chacha_combine_begin(sda_engine* h, int64_t m, uint64_t D, const uint32_t* seeds, uint32_t w, uint64_t n,
                                int64_t* out, hipStream_t st, PendingChacha* pc) {
    *pc = PendingChacha{};
    if (D == 0) return SDA_OK;
    const char* force = getenv("SDA_CHACHA_PATH");
    if (sda::chacha_needs_stream_path(m) || (force && strcmp(force, "stream") == 0) || n == 0)
        return chacha_combine(h, m, D, seeds, w, n, out, st);
    if (sda_status e = ensure(&h->work, &h->work_bytes, sda::chacha_work_bytes(D, n))) return e;
    HIP_TRY(sda::launch_chacha_mask_combine_async(m, D, seeds, w, n, out, h->work, st, h->rej_host));
    *pc = PendingChacha{true, m, D, n, seeds, w, out};
    return SDA_OK;
}
sda_status chacha_combine_end(sda_engine* h, const PendingChacha& pc, hipStream_t st, bool* changed) {
    *changed = false;
    if (!pc.pending || *h->rej_host == 0) return SDA_OK;
    *changed = true;
    bool overflow = false;
    HIP_TRY(sda::resolve_chacha_mask_combine(pc.m, pc.D, pc.seeds, pc.w, pc.n, pc.out, h->work, st, *h->rej_host,
                                             &overflow, nullptr));
    if (!overflow) return SDA_OK;
    if (sda_status e = ensure(&h->work, &h->work_bytes, sda::chacha_stream_work_bytes(pc.D, pc.n, pc.m))) return e;
    HIP_TRY(sda::launch_chacha_streams_combine(pc.m, pc.D, pc.seeds, pc.w, pc.n, pc.out, h->work, st));
    return SDA_OK;
}

// chacha.rs:36-45: masked = (secrets + draw) % m for one seed (host words); mask = scratch of D values
sda_status chacha_mask(sda_engine* h, int64_t m, const uint32_t* seed_host, uint32_t w, const int64_t* secrets,
                       uint64_t D, int64_t* mask, uint32_t* seed_dev, int64_t* masked, hipStream_t st) {
    if (D == 0) return SDA_OK;
    if (w) HIP_TRY(hipMemcpyAsync(seed_dev, seed_host, w * 4, hipMemcpyHostToDevice, st));
    if (sda_status e = chacha_combine(h, m, D, seed_dev, w, 1, mask, st)) return e;   // one stream == its draws
    HIP_TRY(sda::launch_addsub_trem(secrets, mask, +1, D, masked, m, st));
    return SDA_OK;
}

sda_status finish(sda_engine* h) {
    HIP_TRY(hipStreamSynchronize(h->stream));
    return ok();
}

}  // namespace

extern "C" {

int sda_abi_version(void) { return SDA_ENGINE_ABI_VERSION; }

const char* sda_last_error_message(void) { return g_last_error.c_str(); }

const char* sda_status_string(int st) {
    SDA_ENTRY;
    switch (st) {
        case SDA_OK: return "ok";
        case SDA_ERR_BATCH_INPUT_WRONG_LENGTH: return "Batch input wrong length";
        case SDA_ERR_PACKED_SHARING_FAILED: return "Sharing failed for packed secret sharing scheme";
        case SDA_ERR_WRONG_DIMENSION: return "Wrong dimension";
        case SDA_ERR_MISMATCHING_DIMENSION: return "Mismatching dimension";
        case SDA_ERR_INPUTS_MUST_HAVE_SAME_LENGTH: return "Inputs must have same length";
        case SDA_ERR_NOT_ENOUGH_SHARES: return "Not enough shares to reconstruct";
        case SDA_ERR_PRECONDITION: return "precondition violated (the reference panics here)";
        case SDA_ERR_INVALID_ARGUMENT: return "invalid argument";
        case SDA_ERR_UNSUPPORTED: return "unsupported parameters";
        case SDA_ERR_DEVICE: return "device error";
        case SDA_ERR_OUT_OF_MEMORY: return "out of device memory";
    }
    return "unknown status";
}

sda_status sda_engine_create(int device_ordinal, sda_engine** out) {
    SDA_ENTRY;
    if (!out) return fail(SDA_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device_ordinal < 0 || device_ordinal >= n)
        return fail(SDA_ERR_INVALID_ARGUMENT, "device %d out of range (%d devices)", device_ordinal, n);
    HIP_TRY(hipSetDevice(device_ordinal));
    sda_engine* h = new sda_engine();
    h->device = device_ordinal;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&h->rej_host), 64, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        if (h->order_ev) (void)hipEventDestroy(h->order_ev);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        return fail(SDA_ERR_DEVICE, "hipStreamCreate/hipEventCreate: %s", hipGetErrorString(e));
    }
    h->last_stream = h->stream;
    *out = h;
    return ok();
}

void sda_engine_destroy(sda_engine* h) {
    SDA_ENTRY;
    if (!h) return;
    if (t_call_h == h) t_call_h = nullptr;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();            // _dev work may still be queued on callers' streams
    if (h->work) (void)hipFree(h->work);
    if (h->gen_log) (void)hipFree(h->gen_log);
    if (h->codec_work) (void)hipFree(h->codec_work);
    if (h->codec_mat) (void)hipFree(h->codec_mat);
    if (h->pipe) (void)hipFree(h->pipe);
    if (h->snap) (void)hipFree(h->snap);
    if (h->stage) (void)hipFree(h->stage);
    sda::free_table(h->gen_tab);
    sda::free_table(h->rev_tab);
    if (h->rej_host) (void)hipHostFree(h->rej_host);
    if (h->order_ev) (void)hipEventDestroy(h->order_ev);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

sda_status sda_engine_synchronize(sda_engine* h) {
    SDA_ENTRY;
    if (!h) return fail(SDA_ERR_INVALID_ARGUMENT, "engine handle is NULL");
    HIP_TRY(hipDeviceSynchronize());
    return ok();
}

// ---------------- protocol/src/crypto.rs:117-155 ----------------
uint64_t sda_scheme_input_size(const sda_sharing_scheme* s) {
    SDA_ENTRY;
    return s->kind == SDA_SHARING_ADDITIVE ? 1 : s->secret_count;
}
uint64_t sda_scheme_output_size(const sda_sharing_scheme* s) { return s->share_count; }
uint64_t sda_scheme_privacy_threshold(const sda_sharing_scheme* s) {
    SDA_ENTRY;
    return s->kind == SDA_SHARING_ADDITIVE ? s->share_count - 1 : s->privacy_threshold;
}
uint64_t sda_scheme_reconstruction_threshold(const sda_sharing_scheme* s) {
    SDA_ENTRY;
    return s->kind == SDA_SHARING_ADDITIVE ? s->share_count : s->privacy_threshold + s->secret_count;
}
uint64_t sda_share_length(const sda_sharing_scheme* s, uint64_t dimension) {
    SDA_ENTRY;
    const uint64_t k = sda_scheme_input_size(s);
    return k ? (dimension + k - 1) / k : 0;
}

// ---------------- ShareGenerator::generate ----------------
sda_status sda_share_generate(sda_engine* h, const sda_sharing_scheme* s, const int64_t* secrets, uint64_t D,
                              const int64_t* draws, uint64_t n_draws, int64_t* out, uint64_t out_cap) {
    SDA_ENTRY;
    if (!h || !s) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL handle or scheme");
    if ((D && !secrets) || (n_draws && !draws)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL input buffer");
    HIP_TRY(hipSetDevice(h->device));
    if (s->kind == SDA_SHARING_ADDITIVE) {
        const uint64_t n = s->share_count;
        if (n == 0) return fail(SDA_ERR_PRECONDITION, "share_count - 1 underflows (additive.rs:42)");
        if (s->modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
        if (n_draws != D * (n - 1))
            return fail(SDA_ERR_INVALID_ARGUMENT, "expected %llu draws (dimension * (share_count - 1)), got %llu",
                        (unsigned long long)(D * (n - 1)), (unsigned long long)n_draws);
        if (out_cap < n * D) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
        if (D == 0) return ok();
        DevArena a;
        if (sda_status st = stage(h, rup(D * 8) + rup(n_draws * 8) + rup(n * D * 8), &a)) return st;
        int64_t* dsec = a.take<int64_t>(D);
        int64_t* ddr = a.take<int64_t>(n_draws);
        int64_t* dout = a.take<int64_t>(n * D);
        HIP_TRY(hipMemcpyAsync(dsec, secrets, D * 8, hipMemcpyHostToDevice, h->stream));
        if (n_draws) HIP_TRY(hipMemcpyAsync(ddr, draws, n_draws * 8, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(sda::launch_additive_generate(dsec, D, ddr, n, dout, s->modulus, h->stream));
        HIP_TRY(hipMemcpyAsync(out, dout, n * D * 8, hipMemcpyDeviceToHost, h->stream));
        return finish(h);
    }
    if (s->kind != SDA_SHARING_PACKED_SHAMIR) return fail(SDA_ERR_INVALID_ARGUMENT, "unknown sharing scheme kind");
    if (sda_status st = check_packed(s)) return st;
    const uint64_t k = s->secret_count, t = s->privacy_threshold, n = s->share_count;
    const uint64_t B = (D + k - 1) / k;
    if (n_draws != B * t)
        return fail(SDA_ERR_INVALID_ARGUMENT, "expected %llu draws (batches * privacy_threshold), got %llu",
                    (unsigned long long)(B * t), (unsigned long long)n_draws);
    if (out_cap < n * B) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (B == 0) return ok();
    DevArena a;
    if (sda_status st = stage(h, rup(D * 8) + rup(n_draws * 8) + rup(n * B * 8), &a)) return st;
    int64_t* dsec = a.take<int64_t>(D);
    int64_t* ddr = a.take<int64_t>(n_draws);
    int64_t* dout = a.take<int64_t>(n * B);
    HIP_TRY(hipMemcpyAsync(dsec, secrets, D * 8, hipMemcpyHostToDevice, h->stream));
    if (n_draws) HIP_TRY(hipMemcpyAsync(ddr, draws, n_draws * 8, hipMemcpyHostToDevice, h->stream));
    sda::PackedGenArgs ga{dsec, D, 1, ddr, dout};
    if (sda_status st = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return st;
    HIP_TRY(sda::launch_packed_generate(ga, (uint32_t)k, (uint32_t)t, (uint32_t)n, (uint32_t)s->modulus,
                                        (uint32_t)s->omega_secrets, (uint32_t)s->omega_shares, h->gen_tab,
                                        h->gen_log, h->stream));
    HIP_TRY(hipMemcpyAsync(out, dout, n * B * 8, hipMemcpyDeviceToHost, h->stream));
    return finish(h);
}

// ---------------- ShareCombiner::combine ----------------
static sda_status combine_rows(sda_engine* h, int64_t modulus, const int64_t* const* rows, const uint64_t* lens,
                               uint64_t n_rows, int64_t* out, uint64_t out_cap, uint64_t* out_len,
                               sda_status dim_err, const char* dim_msg) {
    if (!h || (n_rows && (!rows || !lens)) || !out_len) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    HIP_TRY(hipSetDevice(h->device));
    const uint64_t dim = n_rows ? lens[0] : 0;              // combiner.rs:17
    *out_len = 0;
    int64_t m;
    // combiner.rs:20-25 / additive.rs:62-67: row 0 (of length dim) is folded -- `%= 0` panics there --
    // before row 1's length is checked
    if (dim && modulus == 0) return modulus_abs(modulus, &m);
    for (uint64_t i = 0; i < n_rows; ++i)
        if (lens[i] != dim) return fail(dim_err, "%s (row %llu has %llu elements, expected %llu)", dim_msg,
                                        (unsigned long long)i, (unsigned long long)lens[i],
                                        (unsigned long long)dim);
    if (dim && n_rows) {
        if (sda_status st = modulus_abs(modulus, &m)) return st;
    } else {
        m = 1;
    }
    if (out_cap < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    *out_len = dim;
    if (dim == 0) return ok();
    for (uint64_t i = 0; i < n_rows; ++i)
        if (!rows[i]) return fail(SDA_ERR_INVALID_ARGUMENT, "row %llu is NULL", (unsigned long long)i);
    DevArena a;
    if (sda_status st = stage(h, rup(n_rows * dim * 8) + rup(dim * 8), &a)) return st;
    int64_t* din = a.take<int64_t>(n_rows * dim);
    int64_t* dout = a.take<int64_t>(dim);
    if (sda_status st = upload_rows(h, din, rows, n_rows, dim)) return st;
    HIP_TRY(sda::launch_combine_exact(din, n_rows, dim, dim, dout, m, h->stream));
    HIP_TRY(hipMemcpyAsync(out, dout, dim * 8, hipMemcpyDeviceToHost, h->stream));
    return finish(h);
}

sda_status sda_share_combine(sda_engine* h, const sda_sharing_scheme* s, const int64_t* const* rows,
                             const uint64_t* lens, uint64_t n_rows, int64_t* out, uint64_t out_cap,
                             uint64_t* out_len) {
    SDA_ENTRY;
    if (!s) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL scheme");
    // sharing/mod.rs:61-69: Additive -> modulus, PackedShamir -> prime_modulus (same field here)
    return combine_rows(h, s->modulus, rows, lens, n_rows, out, out_cap, out_len, SDA_ERR_WRONG_DIMENSION,
                        "Wrong dimension");
}

// ---------------- SecretReconstructor::reconstruct ----------------
sda_status sda_secret_reconstruct(sda_engine* h, const sda_sharing_scheme* s, uint64_t dimension,
                                  const uint64_t* indices, const int64_t* const* rows, const uint64_t* lens,
                                  uint64_t n_rows, int64_t* out, uint64_t out_cap, uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !s || !out_len) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (s->kind == SDA_SHARING_ADDITIVE) {
        // additive.rs:56-72: dimension = first row's length; indices are ignored
        return combine_rows(h, s->modulus, rows, lens, n_rows, out, out_cap, out_len,
                            SDA_ERR_MISMATCHING_DIMENSION, "Mismatching dimension");
    }
    if (s->kind != SDA_SHARING_PACKED_SHAMIR) return fail(SDA_ERR_INVALID_ARGUMENT, "unknown sharing scheme kind");
    if (sda_status st = check_packed(s)) return st;
    HIP_TRY(hipSetDevice(h->device));
    const uint64_t k = s->secret_count;
    const uint64_t B = (dimension + k - 1) / k;             // batched.rs:77
    *out_len = 0;
    if (out_cap < dimension) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (B == 0) { *out_len = 0; return ok(); }              // no batch => no error checks run
    if (n_rows && (!rows || !lens || !indices)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    // batched.rs:82-86: batch 0 gathers [clerk][0] (a panic on an empty row), then
    // packed_shamir.rs:75 may fail; any later batch b panics on a row shorter than b + 1
    const bool enough = n_rows >= s->privacy_threshold + k;
    for (uint64_t i = 0; i < n_rows; ++i)
        if (lens[i] < (enough ? B : 1))
            return fail(SDA_ERR_PRECONDITION, "index out of bounds: row %llu has %llu < %llu batches",
                        (unsigned long long)i, (unsigned long long)lens[i], (unsigned long long)(enough ? B : 1));
    if (!enough)
        return fail(SDA_ERR_NOT_ENOUGH_SHARES, "Not enough shares to reconstruct (%llu < %llu)",
                    (unsigned long long)n_rows, (unsigned long long)(s->privacy_threshold + k));
    if (n_rows > sda::kRevealMaxShares)
        return fail(SDA_ERR_UNSUPPORTED, "more than %u clerk shares per batch", sda::kRevealMaxShares);
    DevArena a;
    if (sda_status st = stage(h, rup(n_rows * B * 8) + rup(dimension * 8), &a)) return st;
    int64_t* din = a.take<int64_t>(n_rows * B);
    int64_t* dout = a.take<int64_t>(dimension);
    for (uint64_t i = 0; i < n_rows; ++i)
        HIP_TRY(hipMemcpyAsync(din + i * B, rows[i], B * 8, hipMemcpyHostToDevice, h->stream));
    if (sda_status st = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return st;
    sda::PackedRevealArgs ra{din, dimension, 1, dout};
    HIP_TRY(sda::launch_packed_reveal(ra, indices, (uint32_t)n_rows, (uint32_t)k, (uint32_t)s->modulus,
                                      (uint32_t)s->omega_secrets, (uint32_t)s->omega_shares, SDA_REVEAL_EXACT,
                                      h->rev_tab, h->gen_log, h->stream));
    HIP_TRY(hipMemcpyAsync(out, dout, dimension * 8, hipMemcpyDeviceToHost, h->stream));
    *out_len = dimension;
    return finish(h);
}

// ---------------- masking ----------------
sda_status sda_secret_mask(sda_engine* h, const sda_masking_scheme* s, const int64_t* secrets, uint64_t D,
                           const uint32_t* seed, uint64_t seed_words, const int64_t* full_masks, int64_t* mask_out,
                           uint64_t mask_cap, uint64_t* mask_len, int64_t* masked_out) {
    SDA_ENTRY;
    if (!h || !s || !mask_len || (D && (!secrets || !masked_out)))
        return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    HIP_TRY(hipSetDevice(h->device));
    *mask_len = 0;
    if (s->kind == SDA_MASKING_NONE) {                      // none.rs:14-19
        if (D) memcpy(masked_out, secrets, D * 8);
        return ok();
    }
    if (s->modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
    if (s->kind == SDA_MASKING_FULL) {                      // full.rs:22-35
        if (D && !full_masks) return fail(SDA_ERR_INVALID_ARGUMENT, "Full masking needs the drawn masks");
        if (mask_cap < D) return fail(SDA_ERR_INVALID_ARGUMENT, "mask buffer too small");
        if (D == 0) return ok();
        DevArena a;
        if (sda_status st = stage(h, 3 * rup(D * 8), &a)) return st;
        int64_t* ds = a.take<int64_t>(D);
        int64_t* dm = a.take<int64_t>(D);
        int64_t* dout = a.take<int64_t>(D);
        HIP_TRY(hipMemcpyAsync(ds, secrets, D * 8, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(dm, full_masks, D * 8, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(sda::launch_addsub_trem(ds, dm, +1, D, dout, s->modulus, h->stream));
        HIP_TRY(hipMemcpyAsync(masked_out, dout, D * 8, hipMemcpyDeviceToHost, h->stream));
        memcpy(mask_out, full_masks, D * 8);
        *mask_len = D;
        return finish(h);
    }
    if (s->kind != SDA_MASKING_CHACHA) return fail(SDA_ERR_INVALID_ARGUMENT, "unknown masking scheme kind");
    // chacha.rs:26 assert_eq!(self.dimension, secrets.len())
    if (s->dimension != D) return fail(SDA_ERR_PRECONDITION, "assertion failed: dimension == secrets.len()");
    const uint64_t want_words = (s->seed_bitsize + 31) / 32;   // chacha.rs:30
    if (seed_words != want_words || (seed_words && !seed))
        return fail(SDA_ERR_PRECONDITION, "expected %llu seed words for seed_bitsize %llu",
                    (unsigned long long)want_words, (unsigned long long)s->seed_bitsize);
    if (mask_cap < seed_words) return fail(SDA_ERR_INVALID_ARGUMENT, "mask buffer too small");
    for (uint64_t i = 0; i < seed_words; ++i) mask_out[i] = (int64_t)seed[i];   // chacha.rs:48-50
    *mask_len = seed_words;
    if (D == 0) return ok();
    const uint32_t w = (uint32_t)(seed_words < 8 ? seed_words : 8);           // key holds 8 words
    DevArena a;
    if (sda_status st = stage(h, 3 * rup(D * 8) + rup(64), &a)) return st;
    int64_t* ds = a.take<int64_t>(D);
    int64_t* dmask = a.take<int64_t>(D);
    int64_t* dout = a.take<int64_t>(D);
    uint32_t* dseed = a.take<uint32_t>(16);
    HIP_TRY(hipMemcpyAsync(ds, secrets, D * 8, hipMemcpyHostToDevice, h->stream));
    if (sda_status st = chacha_mask(h, s->modulus, seed, w, ds, D, dmask, dseed, dout, h->stream)) return st;
    HIP_TRY(hipMemcpyAsync(masked_out, dout, D * 8, hipMemcpyDeviceToHost, h->stream));
    return finish(h);
}

sda_status sda_mask_combine(sda_engine* h, const sda_masking_scheme* s, const int64_t* const* rows,
                            const uint64_t* lens, uint64_t n_rows, int64_t* out, uint64_t out_cap,
                            uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !s || !out_len || (n_rows && (!rows || !lens))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    *out_len = 0;
    if (s->kind == SDA_MASKING_NONE) {                      // none.rs:22-25
        for (uint64_t i = 0; i < n_rows; ++i)
            if (lens[i]) return fail(SDA_ERR_PRECONDITION, "assertion failed: masks.iter().all(|mask| mask.len() == 0)");
        return ok();
    }
    if (s->kind == SDA_MASKING_FULL) {                      // full.rs:38-50 (panics on mismatch)
        const uint64_t dim = n_rows ? lens[0] : 0;
        for (uint64_t i = 0; i < n_rows; ++i)
            if (lens[i] != dim) return fail(SDA_ERR_PRECONDITION, "assertion failed: mask.len() == dimension");
        return combine_rows(h, s->modulus, rows, lens, n_rows, out, out_cap, out_len, SDA_ERR_PRECONDITION,
                            "assertion failed");
    }
    if (s->kind != SDA_MASKING_CHACHA) return fail(SDA_ERR_INVALID_ARGUMENT, "unknown masking scheme kind");
    HIP_TRY(hipSetDevice(h->device));
    const uint64_t D = s->dimension;                        // chacha.rs:58 vec![0; self.dimension]
    if (out_cap < D) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (D && s->modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
    uint64_t w = 0;
    for (uint64_t i = 0; i < n_rows; ++i) w = lens[i] > w ? lens[i] : w;
    if (w > 8) w = 8;                                       // ChaChaRng key = first 8 seed words
    if (w == 0) w = 1;                                      // empty seeds == all-zero key
    std::vector<uint32_t> seeds(n_rows * w, 0u);            // shorter seeds pad with zero key words
    for (uint64_t i = 0; i < n_rows; ++i)
        for (uint64_t j = 0; j < lens[i] && j < w; ++j) seeds[i * w + j] = (uint32_t)rows[i][j];   // chacha.rs:62-64
    *out_len = D;
    if (D == 0) return ok();
    DevArena a;
    if (sda_status st = stage(h, rup(seeds.size() * 4 + 4) + rup(D * 8), &a)) return st;
    uint32_t* dseeds = a.take<uint32_t>(seeds.size() + 1);
    int64_t* dout = a.take<int64_t>(D);
    if (!seeds.empty())
        HIP_TRY(hipMemcpyAsync(dseeds, seeds.data(), seeds.size() * 4, hipMemcpyHostToDevice, h->stream));
    if (sda_status st = chacha_combine(h, s->modulus, D, dseeds, (uint32_t)w, n_rows, dout, h->stream)) return st;
    HIP_TRY(hipMemcpyAsync(out, dout, D * 8, hipMemcpyDeviceToHost, h->stream));
    return finish(h);
}

sda_status sda_secret_unmask(sda_engine* h, const sda_masking_scheme* s, const int64_t* mask, uint64_t mask_len,
                             const int64_t* masked, uint64_t masked_len, int64_t* out, uint64_t out_cap,
                             uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !s || !out_len || (masked_len && (!masked || !out))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    *out_len = 0;
    if (out_cap < masked_len) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (s->kind == SDA_MASKING_NONE) {                      // none.rs:28-32
        if (mask_len != 0) return fail(SDA_ERR_PRECONDITION, "assertion failed: values.0.len() == 0");
        if (masked_len) memcpy(out, masked, masked_len * 8);
        *out_len = masked_len;
        return ok();
    }
    if (s->kind != SDA_MASKING_FULL && s->kind != SDA_MASKING_CHACHA)
        return fail(SDA_ERR_INVALID_ARGUMENT, "unknown masking scheme kind");
    if (mask_len != masked_len) return fail(SDA_ERR_PRECONDITION, "assertion failed: mask.len() == masked_secrets.len()");
    *out_len = masked_len;
    if (masked_len == 0) return ok();
    int64_t m;
    if (sda_status st = modulus_abs(s->modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    const uint64_t D = masked_len;
    DevArena a;
    if (sda_status st = stage(h, 3 * rup(D * 8), &a)) return st;
    int64_t* dm = a.take<int64_t>(D);
    int64_t* dms = a.take<int64_t>(D);
    int64_t* dout = a.take<int64_t>(D);
    HIP_TRY(hipMemcpyAsync(dm, mask, D * 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipMemcpyAsync(dms, masked, D * 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(sda::launch_addsub_trem(dms, dm, -1, D, dout, m, h->stream));      // (ms - m) % q
    HIP_TRY(hipMemcpyAsync(out, dout, D * 8, hipMemcpyDeviceToHost, h->stream));
    return finish(h);
}

sda_status sda_recipient_positive(sda_engine* h, int64_t modulus, const int64_t* values, uint64_t n, int64_t* out) {
    SDA_ENTRY;
    if (!h || (n && (!values || !out))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n == 0) return ok();
    HIP_TRY(hipSetDevice(h->device));
    DevArena a;
    if (sda_status st = stage(h, 2 * rup(n * 8), &a)) return st;
    int64_t* dv = a.take<int64_t>(n);
    int64_t* dout = a.take<int64_t>(n);
    HIP_TRY(hipMemcpyAsync(dv, values, n * 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(sda::launch_positive(dv, n, dout, modulus, h->stream));
    HIP_TRY(hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, h->stream));
    return finish(h);
}

// ---------------- device-resident entry points ----------------
sda_status sda_combine_dev(sda_engine* h, int64_t modulus, const int64_t* shares, uint64_t n, uint64_t dim,
                           uint64_t row_stride, int64_t* out, void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!out || (n && !shares)))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n > 1 && row_stride < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "row_stride < dim");
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_combine_exact(shares, n, dim, n > 1 ? row_stride : dim, out, m, pick(h, stream)));
    return ok();
}

sda_status sda_combine_accumulate_dev(sda_engine* h, int64_t modulus, const int64_t* shares, uint64_t n,
                                      uint64_t dim, uint64_t row_stride, int64_t* inout, void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!inout || (n && !shares)))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n > 1 && row_stride < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "row_stride < dim");
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    if (n == 0) return ok();
    HIP_TRY(sda::launch_combine_exact(shares, n, dim, n > 1 ? row_stride : dim, inout, m, pick(h, stream), true));
    return ok();
}

sda_status sda_combine_finalize_dev(sda_engine* h, int64_t modulus, const int64_t* sums, uint64_t dim, int64_t* out,
                                    void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!sums || !out))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_mod_canonical(sums, dim, out, m, pick(h, stream)));
    return ok();
}

sda_status sda_combine_split_dev(sda_engine* h, int64_t modulus, const int64_t* shares, uint64_t n, uint64_t dim,
                                 uint64_t row_stride, int64_t* inout, int64_t* flags, void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!inout || !flags || (n && !shares)))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n > 1 && row_stride < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "row_stride < dim");
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_combine_split(shares, n, dim, n > 1 ? row_stride : dim, inout, m, flags, pick(h, stream)));
    return ok();
}

sda_status sda_combine_split_prefix_dev(sda_engine* h, int64_t modulus, const int64_t* gathered, uint64_t world,
                                        uint64_t rank, uint64_t dim, int64_t* c_in, int64_t* total, int32_t* code,
                                        void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!gathered || !c_in || !total || !code))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (rank >= world || world > (1u << 29)) return fail(SDA_ERR_INVALID_ARGUMENT, "rank %llu of world %llu",
                                                         (unsigned long long)rank, (unsigned long long)world);
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    if ((unsigned __int128)world * (uint64_t)(m - 1) > (unsigned __int128)INT64_MAX)
        return fail(SDA_ERR_INVALID_ARGUMENT, "world * (m - 1) exceeds 2^63 - 1");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_split_prefix(gathered, world, rank, dim, c_in, total, code, m, pick(h, stream)));
    return ok();
}

sda_status sda_combine_split_replay_dev(sda_engine* h, int64_t modulus, const int64_t* shares, uint64_t n,
                                        uint64_t dim, uint64_t row_stride, uint64_t rank, int64_t* state,
                                        int32_t* code, void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!state || !code || (n && !shares)))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n > 1 && row_stride < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "row_stride < dim");
    if (rank > (1u << 29)) return fail(SDA_ERR_INVALID_ARGUMENT, "rank %llu too large", (unsigned long long)rank);
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_combine_replay(shares, n, dim, n > 1 ? row_stride : dim, state, code, (int32_t)(2 * rank + 1),
                                       m, pick(h, stream)));
    return ok();
}

sda_status sda_combine_split_resolve_dev(sda_engine* h, int64_t modulus, const int64_t* total, const int32_t* code,
                                         uint64_t dim, int64_t* out, void* stream) {
    SDA_ENTRY;
    if (!h || (dim && (!total || !code || !out))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    int64_t m;
    if (sda_status st = modulus_abs(modulus, &m)) return st;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_split_resolve(total, code, dim, out, m, pick(h, stream)));
    return ok();
}

sda_status sda_packed_generate_dev(sda_engine* h, const sda_sharing_scheme* s, const int64_t* secrets,
                                   uint64_t dimension, uint64_t n_vectors, const int64_t* draws, int64_t* out,
                                   void* stream) {
    SDA_ENTRY;
    if (!h || !s || s->kind != SDA_SHARING_PACKED_SHAMIR) return fail(SDA_ERR_INVALID_ARGUMENT, "need a PackedShamir scheme");
    if (sda_status st = check_packed(s)) return st;
    if (n_vectors > 65535) return fail(SDA_ERR_UNSUPPORTED, "at most 65535 vectors per launch");
    HIP_TRY(hipSetDevice(h->device));
    sda::PackedGenArgs ga{secrets, dimension, n_vectors, draws, out};
    if (sda_status st = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return st;
    HIP_TRY(sda::launch_packed_generate(ga, (uint32_t)s->secret_count, (uint32_t)s->privacy_threshold,
                                        (uint32_t)s->share_count, (uint32_t)s->modulus, (uint32_t)s->omega_secrets,
                                        (uint32_t)s->omega_shares, h->gen_tab, h->gen_log, pick(h, stream)));
    return ok();
}

sda_status sda_packed_generate_mode_dev(sda_engine* h, const sda_sharing_scheme* s, const int64_t* secrets,
                                        uint64_t dimension, uint64_t n_vectors, const int64_t* draws, int64_t* out,
                                        int32_t mode, void* stream) {
    SDA_ENTRY;
    if (!h || !s || s->kind != SDA_SHARING_PACKED_SHAMIR) return fail(SDA_ERR_INVALID_ARGUMENT, "need a PackedShamir scheme");
    if (mode != SDA_REVEAL_EXACT && mode != SDA_REVEAL_CANONICAL) return fail(SDA_ERR_INVALID_ARGUMENT, "bad mode");
    if (sda_status st = check_packed(s)) return st;
    if (n_vectors > 65535) return fail(SDA_ERR_UNSUPPORTED, "at most 65535 vectors per launch");
    HIP_TRY(hipSetDevice(h->device));
    sda::PackedGenArgs ga{secrets, dimension, n_vectors, draws, out, mode == SDA_REVEAL_CANONICAL};
    if (sda_status st = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return st;
    HIP_TRY(sda::launch_packed_generate(ga, (uint32_t)s->secret_count, (uint32_t)s->privacy_threshold,
                                        (uint32_t)s->share_count, (uint32_t)s->modulus, (uint32_t)s->omega_secrets,
                                        (uint32_t)s->omega_shares, h->gen_tab, h->gen_log, pick(h, stream)));
    return ok();
}

sda_status sda_packed_reconstruct_dev(sda_engine* h, const sda_sharing_scheme* s, uint64_t dimension,
                                      const uint64_t* indices, uint64_t n_idx, uint64_t n_vectors,
                                      const int64_t* shares, int64_t* out, int32_t mode, void* stream) {
    SDA_ENTRY;
    if (!h || !s || s->kind != SDA_SHARING_PACKED_SHAMIR) return fail(SDA_ERR_INVALID_ARGUMENT, "need a PackedShamir scheme");
    if (sda_status st = check_packed(s)) return st;
    if (mode != SDA_REVEAL_EXACT && mode != SDA_REVEAL_CANONICAL) return fail(SDA_ERR_INVALID_ARGUMENT, "bad mode");
    if (dimension == 0) return ok();                        // batched.rs:77-81: no batch, no check
    if (n_idx < s->privacy_threshold + s->secret_count)
        return fail(SDA_ERR_NOT_ENOUGH_SHARES, "Not enough shares to reconstruct");
    if (n_idx > sda::kRevealMaxShares)
        return fail(SDA_ERR_UNSUPPORTED, "more than %u clerk shares per batch", sda::kRevealMaxShares);
    if (n_vectors > 65535) return fail(SDA_ERR_UNSUPPORTED, "at most 65535 vectors per launch");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = pick(h, stream);
    if (sda_status e = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return e;
    sda::PackedRevealArgs ra{shares, dimension, n_vectors, out};
    hipError_t e = sda::launch_packed_reveal(ra, indices, (uint32_t)n_idx, (uint32_t)s->secret_count,
                                             (uint32_t)s->modulus, (uint32_t)s->omega_secrets,
                                             (uint32_t)s->omega_shares, mode, h->rev_tab, h->gen_log, st);
    if (e == hipErrorInvalidValue && mode == SDA_REVEAL_CANONICAL)
        return fail(SDA_ERR_UNSUPPORTED, "canonical reveal needs distinct clerk indices");
    HIP_TRY(e);
    return ok();
}

sda_status sda_additive_generate_dev(sda_engine* h, int64_t modulus, uint64_t share_count, const int64_t* secrets,
                                     uint64_t dimension, const int64_t* draws, int64_t* out, void* stream) {
    SDA_ENTRY;
    if (!h) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL handle");
    if (share_count == 0) return fail(SDA_ERR_PRECONDITION, "share_count - 1 underflows (additive.rs:42)");
    if (modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_additive_generate(secrets, dimension, draws, share_count, out, modulus, pick(h, stream)));
    return ok();
}

sda_status sda_chacha_mask_combine_dev(sda_engine* h, int64_t modulus, uint64_t dimension, const uint32_t* seeds,
                                       uint64_t w, uint64_t n_seeds, int64_t* out, void* stream) {
    SDA_ENTRY;
    if (!h || (dimension && !out) || (n_seeds && w && !seeds)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (dimension && modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
    if (w == 0 || w > 8) return fail(SDA_ERR_INVALID_ARGUMENT, "seed width must be 1..8 words");
    HIP_TRY(hipSetDevice(h->device));
    if (sda_status st = chacha_combine(h, modulus, dimension, seeds, (uint32_t)w, n_seeds, out, pick(h, stream)))
        return st;
    return ok();
}

sda_status sda_synth_fill_dev(sda_engine* h, int64_t* dst, uint64_t rows, uint64_t cols, uint64_t seed, int64_t lo,
                              int64_t hi, void* stream) {
    SDA_ENTRY;
    if (!h || (rows * cols && !dst)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (hi <= lo) return fail(SDA_ERR_INVALID_ARGUMENT, "need hi > lo");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(sda::launch_synth_fill(dst, rows, cols, seed, lo, hi, pick(h, stream)));
    return ok();
}

}  // extern "C"

// ---------------- HBM buffers built from fixed-size physical chunks ----------------
// A plain hipMalloc of tens of GB takes whatever physical blocks the driver's VRAM manager has free; on a
// box whose VRAM earlier processes left fragmented, that backing can cost share-gen 15 % (the same kernel,
// the same buffer size: 6.45 vs 7.4-7.65 ms, profiles/r04p and r04r).  Buffers mapped from physical
// chunks of a fixed size (hipMemCreate, SDA_HBM_CHUNK_MB, default 64 MiB) ran at the fast rate in every
// case measured, whatever the chunk size (2 MiB - 1 GiB) and whether the chunks were mapped in order or
// shuffled (profiles/r04r).  sda_hbm_alloc / sda_hbm_free give the resident hot-path buffers that backing.
//
// A freed buffer stays mapped, in a per-process pool that later allocations reuse (best fit, at most twice
// the size asked for).  Unmapping and releasing a buffer, then letting the runtime hand its virtual range to
// other allocations, corrupted data in the GPU suite (profiles/r04y: reads of a torch temporary returned a
// different count each time), so no range is ever unmapped while the process runs.
namespace {

struct HbmBuffer {
    int device = 0;
    size_t bytes = 0;                                   // reserved (a whole number of chunks)
    std::vector<hipMemGenericAllocationHandle_t> chunks;
};
std::mutex g_hbm_mu;
std::map<uintptr_t, HbmBuffer> g_hbm;                   // handed out
std::map<uintptr_t, HbmBuffer> g_hbm_pool;              // freed, still mapped

size_t hbm_chunk_bytes() {
    const char* e = getenv("SDA_HBM_CHUNK_MB");
    const long mb = e ? atol(e) : 64;
    return (size_t)(mb > 0 ? mb : 64) << 20;
}

// unmap and release what a partly built buffer holds (the failure path of sda_hbm_alloc only)
void hbm_release(void* ptr, HbmBuffer& b, size_t mapped_chunks, size_t chunk) {
    for (size_t i = 0; i < mapped_chunks; ++i) (void)hipMemUnmap(static_cast<char*>(ptr) + i * chunk, chunk);
    for (auto& c : b.chunks) (void)hipMemRelease(c);
    if (ptr) (void)hipMemAddressFree(ptr, b.bytes);
}

}  // namespace

extern "C" {

// The caller's current device is left as it was (the HBM calls take a device, not a handle).
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

sda_status sda_hbm_alloc(int device, uint64_t bytes, void** out) {
    SDA_ENTRY;
    if (!out) return fail(SDA_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    if (bytes == 0) return fail(SDA_ERR_INVALID_ARGUMENT, "bytes must be > 0");
    DeviceGuard dg;
    HIP_TRY(hipSetDevice(device));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    if (gran == 0) gran = 4096;
    const size_t chunk = (hbm_chunk_bytes() + gran - 1) / gran * gran;
    const size_t n = (size_t)((bytes + chunk - 1) / chunk);
    {   // a pooled buffer of this device that fits, the smallest one (at most twice the size)
        std::lock_guard<std::mutex> lk(g_hbm_mu);
        auto best = g_hbm_pool.end();
        for (auto it = g_hbm_pool.begin(); it != g_hbm_pool.end(); ++it) {
            const HbmBuffer& c = it->second;
            if (c.device == device && c.bytes >= bytes && c.bytes <= 2 * n * chunk &&
                (best == g_hbm_pool.end() || c.bytes < best->second.bytes))
                best = it;
        }
        if (best != g_hbm_pool.end()) {
            *out = reinterpret_cast<void*>(best->first);
            g_hbm[best->first] = std::move(best->second);
            g_hbm_pool.erase(best);
            return ok();
        }
    }
    HbmBuffer b;
    b.device = device;
    b.bytes = n * chunk;
    void* ptr = nullptr;
    HIP_TRY(hipMemAddressReserve(&ptr, b.bytes, chunk, nullptr, 0));
    b.chunks.reserve(n);
    size_t mapped = 0;
    hipError_t e = hipSuccess;
    for (size_t i = 0; i < n && e == hipSuccess; ++i) {
        hipMemGenericAllocationHandle_t c;
        e = hipMemCreate(&c, chunk, &prop, 0);
        if (e != hipSuccess) break;
        b.chunks.push_back(c);
        e = hipMemMap(static_cast<char*>(ptr) + i * chunk, chunk, 0, c, 0);
        if (e == hipSuccess) ++mapped;
    }
    if (e == hipSuccess) {
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(ptr, b.bytes, &acc, 1);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        hbm_release(ptr, b, mapped, chunk);
        return fail(e == hipErrorOutOfMemory ? SDA_ERR_OUT_OF_MEMORY : SDA_ERR_DEVICE,
                    "sda_hbm_alloc(%llu bytes in %zu MiB chunks): %s", (unsigned long long)bytes, chunk >> 20,
                    hipGetErrorString(e));
    }
    {
        std::lock_guard<std::mutex> lk(g_hbm_mu);
        g_hbm[reinterpret_cast<uintptr_t>(ptr)] = std::move(b);
    }
    *out = ptr;
    return ok();
}

sda_status sda_hbm_free(void* ptr) {
    SDA_ENTRY;
    if (!ptr) return ok();
    int device = 0;
    {
        std::lock_guard<std::mutex> lk(g_hbm_mu);
        auto it = g_hbm.find(reinterpret_cast<uintptr_t>(ptr));
        if (it == g_hbm.end()) return fail(SDA_ERR_INVALID_ARGUMENT, "%p was not returned by sda_hbm_alloc", ptr);
        device = it->second.device;
    }
    // work queued on any stream may still use the buffer: it returns to the pool once the device is idle
    DeviceGuard dg;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipDeviceSynchronize());
    std::lock_guard<std::mutex> lk(g_hbm_mu);
    auto it = g_hbm.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == g_hbm.end()) return fail(SDA_ERR_INVALID_ARGUMENT, "%p was freed twice", ptr);
    g_hbm_pool[it->first] = std::move(it->second);
    g_hbm.erase(it);
    return ok();
}

}  // extern "C"

// ---------------- share payload codec (sodium.rs:36-41 / :82-88) ----------------
namespace {

// Plan + count N device-resident blobs; counts[n] on the host.
sda_status codec_count(sda_engine* h, const uint8_t* bytes, const uint64_t* blob_off, uint64_t n_blobs,
                       sda::VarintPlan* plan, uint64_t* counts, bool* irregular, hipStream_t st,
                       bool sub_counts = false, bool* long_any = nullptr) {
    if (((uintptr_t)bytes & 15) != 0) return fail(SDA_ERR_INVALID_ARGUMENT, "byte buffer must be 16-byte aligned");
    for (uint64_t b = 0; b < n_blobs; ++b)
        if (blob_off[b + 1] < blob_off[b]) return fail(SDA_ERR_INVALID_ARGUMENT, "blob offsets must be non-decreasing");
    sda::varint_plan(blob_off, n_blobs, plan);
    if (sda_status e = ensure(&h->codec_work, &h->codec_work_bytes,
                              sda::varint_decode_work_bytes(plan->regions, n_blobs)))
        return e;
    HIP_TRY(sda::launch_varint_count(bytes, blob_off, n_blobs, *plan, h->codec_work, counts, irregular, st,
                                     sub_counts, long_any));
    return SDA_OK;
}

// decode + combiner.rs:16-28 over device-resident blobs; out (device) gets out_len = count of blob 0
sda_status decode_combine(sda_engine* h, int64_t m, const uint8_t* bytes, const uint64_t* blob_off, uint64_t n_blobs,
                          int64_t* out, uint64_t out_cap, uint64_t* out_len, hipStream_t st) {
    *out_len = 0;
    if (n_blobs == 0) return ok();                                  // combiner.rs:17: empty input
    // SDA_CODEC_PATH=fused (A/B and test knob) runs the column-tile decode+combine, which reads the payload
    // once instead of writing and re-reading an int32 matrix but measured slower (VALU-bound: 3.4 ms per
    // 1000 x 1M launch vs 2.2 + 0.7 ms, profiles/r02d/ab_codec_fused.txt); the default is the matrix path.
    const char* path = getenv("SDA_CODEC_PATH");
    const bool force_fused = path && strcmp(path, "fused") == 0, force_matrix = !force_fused;
    const char* env = getenv("SDA_CODEC_NARROW");                    // "0": A/B and test knob
    const bool narrow_ok = !(env && atoi(env) == 0);
    sda::VarintPlan plan;
    std::vector<uint64_t> counts(n_blobs);
    // Default: decode once into int32 slots per 16 KiB region (no count pass), then the exact combine
    // over the slots.  SDA_CODEC_PATH=matrix (A/B and test knob) takes the count pass + dense int32
    // matrix path; any element longer than 5 bytes or outside int32 (malformed or raw i64 payloads)
    // falls back to it as well.
    if (narrow_ok && !force_fused && !(path && strcmp(path, "matrix") == 0)) {
        if (((uintptr_t)bytes & 15) != 0) return fail(SDA_ERR_INVALID_ARGUMENT, "byte buffer must be 16-byte aligned");
        for (uint64_t b = 0; b < n_blobs; ++b)
            if (blob_off[b + 1] < blob_off[b]) return fail(SDA_ERR_INVALID_ARGUMENT, "blob offsets must be non-decreasing");
        sda::varint_plan(blob_off, n_blobs, &plan);
        if (sda_status e = ensure(&h->codec_work, &h->codec_work_bytes,
                                  sda::varint_decode_work_bytes(plan.regions, n_blobs)))
            return e;
        // the slots are sized by the bytes, the tile plan by the dimension (<= the bytes of blob 0)
        const uint64_t dim_max = blob_off[1] - blob_off[0];
        if (sda_status e = ensure(&h->codec_mat, &h->codec_mat_bytes, sda::varint_slot_bytes(plan, n_blobs, dim_max)))
            return e;
        // everything is queued before the host sees a count: the combine itself exits when a flag is set
        // or blob 0's count exceeds out_cap, and the checks below then report it in the reference's order
        const bool m_ok = m != 0 && m != INT64_MIN;
        uint32_t flags = 0;
        HIP_TRY(sda::launch_varint_decode_slots_combine(bytes, blob_off, n_blobs, plan, h->codec_work, h->codec_mat,
                                                        out, out_cap, m_ok ? (m < 0 ? -m : m) : 0, counts.data(),
                                                        &flags, st));
        if (!(flags & 1u)) {
            const uint64_t dim = counts[0];
            int64_t mm = 1;
            if (dim && m == 0) return modulus_abs(m, &mm);     // blob 0 is folded first (combiner.rs:20-25)
            for (uint64_t i = 1; i < n_blobs; ++i)
                if (counts[i] != dim)
                    return fail(SDA_ERR_WRONG_DIMENSION,
                                "Wrong dimension (participation %llu decodes to %llu shares, expected %llu)",
                                (unsigned long long)i, (unsigned long long)counts[i], (unsigned long long)dim);
            if (dim) {
                if (sda_status e = modulus_abs(m, &mm)) return e;
            }
            if (out_cap < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
            *out_len = dim;
            return SDA_OK;
        }
    }
    bool irregular = false, long_elems = false;
    if (sda_status e = codec_count(h, bytes, blob_off, n_blobs, &plan, counts.data(), &irregular, st, !force_matrix,
                                   &long_elems))
        return e;
    const uint64_t dim = counts[0];
    int64_t mm;
    if (dim && m == 0) return modulus_abs(m, &mm);             // blob 0 is folded first (combiner.rs:20-25)
    for (uint64_t i = 1; i < n_blobs; ++i)
        if (counts[i] != dim)
            return fail(SDA_ERR_WRONG_DIMENSION, "Wrong dimension (participation %llu decodes to %llu shares, expected %llu)",
                        (unsigned long long)i, (unsigned long long)counts[i], (unsigned long long)dim);
    if (dim) {
        if (sda_status e = modulus_abs(m, &mm)) return e;
    }
    if (out_cap < dim) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    *out_len = dim;
    if (dim == 0) return ok();
    if (!irregular && force_fused) {
        // one pass over the payload: no [N][dim] matrix (the matrix buffer holds the tile plan)
        if (sda_status e = ensure(&h->codec_mat, &h->codec_mat_bytes, sda::varint_tile_plan_bytes(n_blobs, dim)))
            return e;
        HIP_TRY(sda::launch_varint_decode_combine(bytes, n_blobs, plan, h->codec_work,
                                                  static_cast<uint64_t*>(h->codec_mat), dim, out, mm, long_elems, st));
        return SDA_OK;
    }
    if (sda_status e = ensure(&h->codec_mat, &h->codec_mat_bytes, n_blobs * dim * 8)) return e;
    // Decoded field shares fit in int32 (|share| < m <= 2^31 for every field the reference uses): the
    // [N][dim] matrix between the decode and the combine is stored narrowed, which halves its write and
    // its read.  Any value that does not fit (or a malformed blob) takes the int64 matrix instead.
    if (narrow_ok && !irregular) {
        bool wide = false;
        int32_t* mat32 = static_cast<int32_t*>(h->codec_mat);
        HIP_TRY(sda::launch_varint_decode_narrow(bytes, n_blobs, plan, h->codec_work, mat32, dim, &wide, st));
        if (!wide) {
            HIP_TRY(sda::launch_combine_exact32(mat32, n_blobs, dim, dim, out, mm, st));
            return SDA_OK;
        }
    }
    int64_t* mat = static_cast<int64_t*>(h->codec_mat);
    HIP_TRY(sda::launch_varint_decode(bytes, n_blobs, plan, h->codec_work, mat, dim, dim, irregular, st));
    HIP_TRY(sda::launch_combine_exact(mat, n_blobs, dim, dim, out, mm, st));
    return SDA_OK;
}

// concatenate host blobs into a 16-byte aligned, padded device buffer
sda_status upload_blobs(sda_engine* h, const uint8_t* const* blobs, const uint64_t* lens, uint64_t n,
                        DevArena* a, uint8_t** dev, std::vector<uint64_t>* off) {
    off->assign(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
        if (lens[i] && !blobs[i]) return fail(SDA_ERR_INVALID_ARGUMENT, "blob %llu is NULL", (unsigned long long)i);
        (*off)[i + 1] = (*off)[i] + lens[i];
    }
    const uint64_t total = (*off)[n];
    std::vector<uint8_t> host(total + 32, 0);
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i]) memcpy(host.data() + (*off)[i], blobs[i], lens[i]);
    *dev = a->take<uint8_t>(total + 32);
    HIP_TRY(hipMemcpyAsync(*dev, host.data(), total + 32, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));       // `host` goes out of scope
    return SDA_OK;
}

}  // namespace

extern "C" {

sda_status sda_varint_encode(sda_engine* h, const int64_t* vals, uint64_t n, uint8_t* out, uint64_t out_cap,
                             uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !out_len || (n && !vals)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    *out_len = 0;
    if (n == 0) return ok();
    HIP_TRY(hipSetDevice(h->device));
    DevArena a;
    if (sda_status st = stage(h, rup(n * 8) + rup(n * 10 + 16), &a)) return st;
    int64_t* dv = a.take<int64_t>(n);
    uint8_t* db = a.take<uint8_t>(n * 10 + 16);
    HIP_TRY(hipMemcpyAsync(dv, vals, n * 8, hipMemcpyHostToDevice, h->stream));
    if (sda_status st = ensure(&h->codec_work, &h->codec_work_bytes, sda::varint_encode_work_bytes(1, n))) return st;
    uint64_t bytes = 0;
    HIP_TRY(sda::launch_varint_encode(dv, 1, n, n, db, n * 10 + 16, h->codec_work, &bytes, h->stream));
    if (bytes > out_cap) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small (%llu bytes needed)",
                                     (unsigned long long)bytes);
    HIP_TRY(hipMemcpyAsync(out, db, bytes, hipMemcpyDeviceToHost, h->stream));
    *out_len = bytes;
    return finish(h);
}

sda_status sda_varint_decode(sda_engine* h, const uint8_t* bytes, uint64_t n_bytes, int64_t* out, uint64_t out_cap,
                             uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !out_len || (n_bytes && !bytes)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    *out_len = 0;
    HIP_TRY(hipSetDevice(h->device));
    DevArena a;
    if (sda_status st = stage(h, rup(n_bytes + 32) + rup(n_bytes * 8 + 8), &a)) return st;
    uint8_t* db;
    std::vector<uint64_t> off;
    const uint8_t* const blobs[1] = {bytes};
    if (sda_status st = upload_blobs(h, blobs, &n_bytes, 1, &a, &db, &off)) return st;
    int64_t* dv = a.take<int64_t>(n_bytes + 1);
    sda::VarintPlan plan;
    uint64_t count = 0;
    bool irregular = false;
    if (sda_status st = codec_count(h, db, off.data(), 1, &plan, &count, &irregular, h->stream)) return st;
    if (count > out_cap) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small (%llu values)",
                                     (unsigned long long)count);
    HIP_TRY(sda::launch_varint_decode(db, 1, plan, h->codec_work, dv, count, count, irregular, h->stream));
    if (count) HIP_TRY(hipMemcpyAsync(out, dv, count * 8, hipMemcpyDeviceToHost, h->stream));
    *out_len = count;
    return finish(h);
}

sda_status sda_clerk_decode_combine(sda_engine* h, const sda_sharing_scheme* s, const uint8_t* const* blobs,
                                    const uint64_t* blob_lens, uint64_t n_blobs, int64_t* out, uint64_t out_cap,
                                    uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !s || !out_len || (n_blobs && (!blobs || !blob_lens))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    *out_len = 0;
    HIP_TRY(hipSetDevice(h->device));
    uint64_t total = 0;
    for (uint64_t i = 0; i < n_blobs; ++i) total += blob_lens[i];
    DevArena a;
    if (sda_status st = stage(h, rup(total + 32) + rup(total * 8 + 8), &a)) return st;
    uint8_t* db;
    std::vector<uint64_t> off;
    if (sda_status st = upload_blobs(h, blobs, blob_lens, n_blobs, &a, &db, &off)) return st;
    int64_t* dout = a.take<int64_t>(total + 1);
    uint64_t len = 0;
    if (sda_status st = decode_combine(h, s->modulus, db, off.data(), n_blobs, dout, (uint64_t)-1, &len, h->stream))
        return st;
    if (out_cap < len) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (len) HIP_TRY(hipMemcpyAsync(out, dout, len * 8, hipMemcpyDeviceToHost, h->stream));
    *out_len = len;
    return finish(h);
}

sda_status sda_varint_decode_dev(sda_engine* h, const uint8_t* bytes, const uint64_t* blob_off, uint64_t n_blobs,
                                 int64_t* out, uint64_t out_stride, uint64_t* counts, void* stream) {
    SDA_ENTRY;
    if (!h || !blob_off || !counts || (n_blobs && (!bytes || !out))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = pick(h, stream);
    if (n_blobs == 0) return ok();
    if (((uintptr_t)bytes & 15) != 0) return fail(SDA_ERR_INVALID_ARGUMENT, "byte buffer must be 16-byte aligned");
    for (uint64_t b = 0; b < n_blobs; ++b)
        if (blob_off[b + 1] < blob_off[b]) return fail(SDA_ERR_INVALID_ARGUMENT, "blob offsets must be non-decreasing");
    sda::VarintPlan plan;
    sda::varint_plan(blob_off, n_blobs, &plan);
    if (sda_status e = ensure(&h->codec_work, &h->codec_work_bytes, sda::varint_decode_work_bytes(plan.regions, n_blobs)))
        return e;
    // count, check the capacity and decode without a host wait in between: a blob longer than out_stride
    // stops every write on the device and is reported here (nothing written)
    bool too_long = false;
    HIP_TRY(sda::launch_varint_decode_one_wait(bytes, blob_off, n_blobs, plan, h->codec_work, out, out_stride, counts,
                                               &too_long, st));
    if (too_long)
        for (uint64_t i = 0; i < n_blobs; ++i)
            if (counts[i] > out_stride)
                return fail(SDA_ERR_INVALID_ARGUMENT, "blob %llu decodes to %llu values > out_stride",
                            (unsigned long long)i, (unsigned long long)counts[i]);
    return ok();
}

sda_status sda_clerk_decode_combine_dev(sda_engine* h, int64_t modulus, const uint8_t* bytes, const uint64_t* blob_off,
                                        uint64_t n_blobs, int64_t* out, uint64_t out_cap, uint64_t* out_len,
                                        void* stream) {
    SDA_ENTRY;
    if (!h || !blob_off || !out_len || (n_blobs && !bytes)) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    HIP_TRY(hipSetDevice(h->device));
    if (sda_status e = decode_combine(h, modulus, bytes, blob_off, n_blobs, out, out_cap, out_len, pick(h, stream)))
        return e;
    return ok();
}

sda_status sda_varint_encode_dev(sda_engine* h, const int64_t* vals, uint64_t rows, uint64_t len, uint64_t stride,
                                 uint8_t* dst, uint64_t dst_cap, uint64_t* row_bytes, void* stream) {
    SDA_ENTRY;
    if (!h || !row_bytes || (rows && len && (!vals || !dst))) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (rows > 65535) return fail(SDA_ERR_UNSUPPORTED, "at most 65535 rows per call");
    if (stride < len) return fail(SDA_ERR_INVALID_ARGUMENT, "stride < len");
    HIP_TRY(hipSetDevice(h->device));
    if (sda_status e = ensure(&h->codec_work, &h->codec_work_bytes, sda::varint_encode_work_bytes(rows, len))) return e;
    hipError_t e = sda::launch_varint_encode(vals, rows, len, stride, dst, dst_cap, h->codec_work, row_bytes,
                                             pick(h, stream));
    if (e == hipErrorInvalidValue) return fail(SDA_ERR_INVALID_ARGUMENT, "dst_cap too small");
    HIP_TRY(e);
    return ok();
}

// ---------------- snapshot transposition (stores.rs:86-101) ----------------
// Offsets are a host-side plan (like the codec's blob_off); the bytes move on the device.
sda_status sda_snapshot_transpose_dev(sda_engine* h, const uint8_t* src, const uint64_t* part_off,
                                      uint64_t n_participations, uint64_t n_clerks, uint8_t* dst, uint64_t dst_cap,
                                      uint64_t* dst_len, uint64_t* clerk_base, uint64_t* clerk_off, void* stream) {
    SDA_ENTRY;
    if (!h || !part_off || !dst_len || (n_clerks && (!clerk_base || !clerk_off)))
        return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    const uint64_t P = n_participations, n = n_clerks, nb = P * n;
    if (n && P > ((uint64_t)1 << 32) / n) return fail(SDA_ERR_UNSUPPORTED, "at most 2^32 blobs per snapshot");
    for (uint64_t b = 0; b < nb; ++b)
        if (part_off[b + 1] < part_off[b]) return fail(SDA_ERR_INVALID_ARGUMENT, "blob offsets must be non-decreasing");
    // clerk c's job: its P blobs back to back in snapshot order, the job 16-byte aligned and followed
    // by 16 readable bytes (what sda_clerk_decode_combine_dev takes)
    uint64_t total = 0;
    for (uint64_t c = 0; c < n; ++c) {
        clerk_base[c] = total;
        uint64_t* off = clerk_off + c * (P + 1);
        off[0] = 0;
        for (uint64_t p = 0; p < P; ++p) off[p + 1] = off[p] + (part_off[p * n + c + 1] - part_off[p * n + c]);
        total += ((off[P] + 15) & ~(uint64_t)15) + 16;
    }
    *dst_len = total;
    if (!dst) return ok();                                          // sizing query
    if (dst_cap < total) return fail(SDA_ERR_INVALID_ARGUMENT, "dst_cap %llu < %llu bytes needed",
                                     (unsigned long long)dst_cap, (unsigned long long)total);
    if (nb && !src) return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    if (((uintptr_t)src & 15) || ((uintptr_t)dst & 15))
        return fail(SDA_ERR_INVALID_ARGUMENT, "src and dst must be 16-byte aligned");
    const uint64_t chunk = sda::snapshot_chunk_bytes();
    std::vector<sda::SnapshotCopy> blobs;                          // clerk-major, non-empty blobs only
    std::vector<uint64_t> cstart(1, 0);
    blobs.reserve(nb);
    cstart.reserve(nb + 1);
    for (uint64_t c = 0; c < n; ++c)
        for (uint64_t p = 0; p < P; ++p) {
            const uint64_t len = part_off[p * n + c + 1] - part_off[p * n + c];
            if (!len) continue;
            blobs.push_back({part_off[p * n + c], clerk_base[c] + clerk_off[c * (P + 1) + p], len});
            cstart.push_back(cstart.back() + (len + chunk - 1) / chunk);
        }
    if (blobs.empty()) return ok();
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = pick(h, stream);
    const size_t b0 = rup(blobs.size() * sizeof(sda::SnapshotCopy));
    if (sda_status e = ensure(&h->snap, &h->snap_bytes, b0 + rup(cstart.size() * 8))) return e;
    char* plan = static_cast<char*>(h->snap);
    HIP_TRY(hipMemcpyAsync(plan, blobs.data(), blobs.size() * sizeof(sda::SnapshotCopy), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(plan + b0, cstart.data(), cstart.size() * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(sda::launch_snapshot_transpose(src, dst, reinterpret_cast<const sda::SnapshotCopy*>(plan),
                                           reinterpret_cast<const uint64_t*>(plan + b0), blobs.size(),
                                           cstart.back(), st));
    HIP_TRY(hipStreamSynchronize(st));                             // the host plan vectors go out of scope
    return ok();
}

}  // extern "C"

// ---------------- fused role pipelines ----------------
namespace {

// receive.rs:80-157 + :14-20 on device-resident inputs (see sda_recipient_reveal_dev).
sda_status recipient_pipeline(sda_engine* h, const sda_masking_scheme* ms, const void* mask_in, uint64_t n_masks,
                              uint64_t mask_width, const sda_sharing_scheme* ss, uint64_t dimension,
                              const uint64_t* indices, const int64_t* shares, uint64_t n_idx, uint64_t share_len,
                              int64_t output_modulus, int32_t mode, int64_t* out, uint64_t out_cap,
                              uint64_t* out_len, hipStream_t st) {
    *out_len = 0;
    // Checks in the reference's order: mask combine (receive.rs:101-117), reconstruct (:120-146),
    // unmask (:149-152).
    // ---- 1. mask combine: its length and panics ----
    uint64_t mask_len = 0;
    if (ms->kind == SDA_MASKING_NONE) {
        if (n_masks && mask_width) return fail(SDA_ERR_PRECONDITION, "assertion failed: masks.iter().all(|mask| mask.len() == 0)");
    } else if (ms->kind == SDA_MASKING_FULL) {
        mask_len = n_masks ? mask_width : 0;                // full.rs:38-40
        if (mask_len) {                                     // full.rs:45 `%= modulus`
            int64_t q0;
            if (sda_status e = modulus_abs(ms->modulus, &q0)) return e;
        }
    } else if (ms->kind == SDA_MASKING_CHACHA) {
        mask_len = ms->dimension;                           // chacha.rs:58
        if (mask_width == 0 || mask_width > 8) return fail(SDA_ERR_UNSUPPORTED, "device seeds must be 1..8 words");
        if (mask_len && n_masks && ms->modulus <= 0)        // chacha.rs:69 gen_range(0, m)
            return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
    } else {
        return fail(SDA_ERR_INVALID_ARGUMENT, "unknown masking scheme kind");
    }
    // ---- 2. reconstruct: masked output length and errors ----
    uint64_t D;
    if (ss->kind == SDA_SHARING_ADDITIVE) {
        D = n_idx ? share_len : 0;                           // additive.rs:56-60
        if (D) {                                             // additive.rs:67 `%= modulus`
            int64_t m0;
            if (sda_status e = modulus_abs(ss->modulus, &m0)) return e;
        }
    } else if (ss->kind == SDA_SHARING_PACKED_SHAMIR) {
        if (sda_status e = check_packed(ss)) return e;
        if (mode != SDA_REVEAL_EXACT && mode != SDA_REVEAL_CANONICAL) return fail(SDA_ERR_INVALID_ARGUMENT, "bad mode");
        const uint64_t B = (dimension + ss->secret_count - 1) / ss->secret_count;
        if (B) {                                             // batched.rs:77-81: no batch => no check
            const bool enough = n_idx >= ss->privacy_threshold + ss->secret_count;
            if (n_idx && share_len < (enough ? B : 1))      // batched.rs:84 indexes [batch_index]
                return fail(SDA_ERR_PRECONDITION, "index out of bounds: clerk vector shorter than the batch count");
            if (!enough) return fail(SDA_ERR_NOT_ENOUGH_SHARES, "Not enough shares to reconstruct");  // packed_shamir.rs:75
            if (n_idx > sda::kRevealMaxShares)
                return fail(SDA_ERR_UNSUPPORTED, "more than %u clerk shares per batch", sda::kRevealMaxShares);
        }
        D = dimension;
    } else {
        return fail(SDA_ERR_INVALID_ARGUMENT, "unknown sharing scheme kind");
    }
    // ---- 3. unmask ----
    if (ms->kind != SDA_MASKING_NONE && mask_len != D)     // chacha.rs:83 / full.rs:58 assert_eq!
        return fail(SDA_ERR_PRECONDITION, "assertion failed: mask.len() == masked_secrets.len() (%llu vs %llu)",
                    (unsigned long long)mask_len, (unsigned long long)D);
    if (out_cap < D) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (D == 0) return ok();
    int64_t q = 1;
    if (ms->kind != SDA_MASKING_NONE)
        if (sda_status e = modulus_abs(ms->modulus, &q)) return e;
    const bool packed = ss->kind == SDA_SHARING_PACKED_SHAMIR;
    const uint64_t B = packed ? (dimension + ss->secret_count - 1) / ss->secret_count : 0;
    const bool compact = packed && share_len != B;
    if (sda_status e = ensure(&h->pipe, &h->pipe_bytes, 2 * rup(D * 8) + (compact ? rup(n_idx * B * 8) : 0) + 256))
        return e;
    int64_t* dmask = static_cast<int64_t*>(h->pipe);
    int64_t* dmasked = dmask + rup(D * 8) / 8;
    // 1. masks (receive.rs:101-117)
    if (ms->kind == SDA_MASKING_FULL) {
        if (sda_status e = modulus_abs(ms->modulus, &q)) return e;
        HIP_TRY(sda::launch_combine_exact(static_cast<const int64_t*>(mask_in), n_masks, D, mask_width, dmask, q, st));
    }
    PendingChacha pc;                                       // ChaCha: its rejection count is checked at the end
    if (ms->kind == SDA_MASKING_CHACHA) {
        if (sda_status e = chacha_combine_begin(h, ms->modulus, D, static_cast<const uint32_t*>(mask_in),
                                                (uint32_t)mask_width, n_masks, dmask, st, &pc))
            return e;
    }
    // 2. reconstruct (receive.rs:120-146)
    if (!packed) {
        int64_t m;
        if (sda_status e = modulus_abs(ss->modulus, &m)) return e;
        HIP_TRY(sda::launch_combine_exact(shares, n_idx, D, share_len, dmasked, m, st));
    } else {
        const int64_t* src = shares;
        if (compact) {                                      // batched.rs:83-85 reads [clerk][0..B)
            int64_t* c = dmasked + rup(D * 8) / 8;
            HIP_TRY(hipMemcpy2DAsync(c, B * 8, shares, share_len * 8, B * 8, n_idx, hipMemcpyDeviceToDevice, st));
            src = c;
        }
        if (sda_status e = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return e;
        sda::PackedRevealArgs ra{src, dimension, 1, dmasked};
        hipError_t e = sda::launch_packed_reveal(ra, indices, (uint32_t)n_idx, (uint32_t)ss->secret_count,
                                                 (uint32_t)ss->modulus, (uint32_t)ss->omega_secrets,
                                                 (uint32_t)ss->omega_shares, mode, h->rev_tab, h->gen_log, st);
        if (e == hipErrorInvalidValue && mode == SDA_REVEAL_CANONICAL)
            return fail(SDA_ERR_UNSUPPORTED, "canonical reveal needs distinct clerk indices");
        HIP_TRY(e);
    }
    // 3. unmask (receive.rs:149-152) + RecipientOutput::positive (:14-20), one pass
    HIP_TRY(sda::launch_unmask_positive(dmasked, ms->kind == SDA_MASKING_NONE ? nullptr : dmask, D, q,
                                        output_modulus, out, st));
    if (pc.pending) {            // the mask's rejection count: fix the mask and unmask again if it had any
        HIP_TRY(hipStreamSynchronize(st));
        bool changed = false;
        if (sda_status e = chacha_combine_end(h, pc, st, &changed)) return e;
        if (changed)
            HIP_TRY(sda::launch_unmask_positive(dmasked, dmask, D, q, output_modulus, out, st));
    }
    *out_len = D;
    return SDA_OK;
}

}  // namespace

extern "C" {

sda_status sda_recipient_reveal_dev(sda_engine* h, const sda_masking_scheme* ms, const void* mask_in, uint64_t n_masks,
                                    uint64_t mask_width, const sda_sharing_scheme* ss, uint64_t dimension,
                                    const uint64_t* indices, const int64_t* shares, uint64_t n_idx,
                                    uint64_t share_len, int64_t output_modulus, int32_t mode, int64_t* out,
                                    uint64_t out_cap, uint64_t* out_len, void* stream) {
    SDA_ENTRY;
    if (!h || !ms || !ss || !out_len || (n_idx && (!shares || !indices)) || (n_masks && mask_width && !mask_in))
        return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    HIP_TRY(hipSetDevice(h->device));
    if (sda_status e = recipient_pipeline(h, ms, mask_in, n_masks, mask_width, ss, dimension, indices, shares, n_idx,
                                          share_len, output_modulus, mode, out, out_cap, out_len, pick(h, stream)))
        return e;
    return ok();
}

sda_status sda_recipient_reveal(sda_engine* h, const sda_masking_scheme* ms, const int64_t* const* mask_rows,
                                const uint64_t* mask_lens, uint64_t n_masks, const sda_sharing_scheme* ss,
                                uint64_t dimension, const uint64_t* indices, const int64_t* const* share_rows,
                                const uint64_t* share_lens, uint64_t n_idx, int64_t output_modulus, int32_t mode,
                                int64_t* out, uint64_t out_cap, uint64_t* out_len) {
    SDA_ENTRY;
    if (!h || !ms || !ss || !out_len || (n_masks && (!mask_rows || !mask_lens)) ||
        (n_idx && (!share_rows || !share_lens || !indices)))
        return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    *out_len = 0;
    HIP_TRY(hipSetDevice(h->device));
    // host-side shape checks in the reference's order, then one upload
    uint64_t share_len = n_idx ? share_lens[0] : 0;
    for (uint64_t i = 0; i < n_idx; ++i) {
        if (share_lens[i] == share_len) continue;
        if (ss->kind == SDA_SHARING_ADDITIVE) return fail(SDA_ERR_MISMATCHING_DIMENSION, "Mismatching dimension");
        share_len = share_lens[i] < share_len ? share_lens[i] : share_len;   // packed: reads [0, B) of each
    }
    uint64_t width = 0;
    std::vector<uint32_t> seeds;
    if (ms->kind == SDA_MASKING_FULL) {
        width = n_masks ? mask_lens[0] : 0;
        for (uint64_t i = 0; i < n_masks; ++i)
            if (mask_lens[i] != width) return fail(SDA_ERR_PRECONDITION, "assertion failed: mask.len() == dimension");
    } else if (ms->kind == SDA_MASKING_CHACHA) {
        for (uint64_t i = 0; i < n_masks; ++i) width = mask_lens[i] > width ? mask_lens[i] : width;
        width = width > 8 ? 8 : (width == 0 ? 1 : width);    // key = first 8 words, zero padded
        seeds.assign(n_masks * width, 0u);
        for (uint64_t i = 0; i < n_masks; ++i)
            for (uint64_t j = 0; j < mask_lens[i] && j < width; ++j) seeds[i * width + j] = (uint32_t)mask_rows[i][j];
    } else {
        for (uint64_t i = 0; i < n_masks; ++i)
            if (mask_lens[i]) return fail(SDA_ERR_PRECONDITION, "assertion failed: masks.iter().all(|mask| mask.len() == 0)");
    }
    const uint64_t outn = ss->kind == SDA_SHARING_ADDITIVE ? share_len : dimension;
    DevArena a;
    if (sda_status e = stage(h, rup(n_idx * share_len * 8 + 8) + rup(n_masks * width * 8 + 8) + rup(outn * 8 + 8), &a))
        return e;
    int64_t* dsh = a.take<int64_t>(n_idx * share_len + 1);
    void* dmask = a.take<int64_t>(n_masks * width + 1);
    int64_t* dout = a.take<int64_t>(outn + 1);
    for (uint64_t i = 0; i < n_idx; ++i)
        if (share_len) HIP_TRY(hipMemcpyAsync(dsh + i * share_len, share_rows[i], share_len * 8, hipMemcpyHostToDevice, h->stream));
    if (ms->kind == SDA_MASKING_FULL)
        for (uint64_t i = 0; i < n_masks; ++i)
            if (width) HIP_TRY(hipMemcpyAsync(static_cast<int64_t*>(dmask) + i * width, mask_rows[i], width * 8,
                                              hipMemcpyHostToDevice, h->stream));
    if (ms->kind == SDA_MASKING_CHACHA && !seeds.empty())
        HIP_TRY(hipMemcpyAsync(dmask, seeds.data(), seeds.size() * 4, hipMemcpyHostToDevice, h->stream));
    uint64_t len = 0;
    if (sda_status e = recipient_pipeline(h, ms, dmask, n_masks, ms->kind == SDA_MASKING_NONE ? 0 : width, ss,
                                          dimension, indices, dsh, n_idx, share_len, output_modulus, mode, dout,
                                          (uint64_t)-1, &len, h->stream))
        return e;
    if (out_cap < len) return fail(SDA_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (len) HIP_TRY(hipMemcpyAsync(out, dout, len * 8, hipMemcpyDeviceToHost, h->stream));
    *out_len = len;
    return finish(h);
}

// participate.rs:53-76 (+ the encoding step of Encryptor::encrypt, sodium.rs:36-41) on device.
sda_status sda_participant_share_dev(sda_engine* h, const sda_masking_scheme* ms, const uint32_t* seed,
                                     uint64_t seed_words, const int64_t* full_masks, const sda_sharing_scheme* ss,
                                     const int64_t* secrets, uint64_t dimension, const int64_t* draws,
                                     int32_t mode, int64_t* shares_out, uint8_t* payload, uint64_t payload_cap,
                                     uint64_t* payload_row_bytes, void* stream) {
    SDA_ENTRY;
    if (!h || !ms || !ss || (dimension && (!secrets || !shares_out)) || (payload && !payload_row_bytes))
        return fail(SDA_ERR_INVALID_ARGUMENT, "NULL argument");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = pick(h, stream);
    const uint64_t D = dimension;
    const bool packed = ss->kind == SDA_SHARING_PACKED_SHAMIR;
    if (!packed && ss->kind != SDA_SHARING_ADDITIVE) return fail(SDA_ERR_INVALID_ARGUMENT, "unknown sharing scheme kind");
    if (mode != SDA_REVEAL_EXACT && mode != SDA_REVEAL_CANONICAL) return fail(SDA_ERR_INVALID_ARGUMENT, "bad mode");
    if (packed) {
        if (sda_status e = check_packed(ss)) return e;
    } else {
        if (ss->share_count == 0) return fail(SDA_ERR_PRECONDITION, "share_count - 1 underflows (additive.rs:42)");
        if (ss->modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
    }
    // 1. SecretMasker::mask (participate.rs:53-54)
    const int64_t* masked = secrets;
    // ChaCha on the fast path: the masked secrets come straight out of the ChaCha kernel and its rejection
    // count is checked at the end of the call (a nonzero count -- probability < 2^-28 per draw -- redoes
    // the mask exactly, then every later step)
    bool mask_pending = false;
    int64_t* cmask = nullptr;
    uint32_t* cseed = nullptr;
    uint32_t cw = 0;
    if (ms->kind != SDA_MASKING_NONE && D) {
        if (ms->modulus <= 0) return fail(SDA_ERR_PRECONDITION, "Rng.gen_range called with low >= high");
        if (sda_status e = ensure(&h->pipe, &h->pipe_bytes, 2 * rup(D * 8) + 256)) return e;
        int64_t* dm = static_cast<int64_t*>(h->pipe);
        if (ms->kind == SDA_MASKING_FULL) {
            if (!full_masks) return fail(SDA_ERR_INVALID_ARGUMENT, "Full masking needs the drawn masks");
            HIP_TRY(sda::launch_addsub_trem(secrets, full_masks, +1, D, dm, ms->modulus, st));      // full.rs:28-31
        } else if (ms->kind == SDA_MASKING_CHACHA) {
            if (ms->dimension != D) return fail(SDA_ERR_PRECONDITION, "assertion failed: dimension == secrets.len()");
            const uint64_t want = (ms->seed_bitsize + 31) / 32;
            if (seed_words != want || (seed_words && !seed))
                return fail(SDA_ERR_PRECONDITION, "expected %llu seed words", (unsigned long long)want);
            int64_t* dmask = dm + rup(D * 8) / 8;
            uint32_t* dseed = reinterpret_cast<uint32_t*>(dmask + rup(D * 8) / 8);
            const uint32_t w = (uint32_t)(seed_words < 8 ? seed_words : 8);
            if (w) HIP_TRY(hipMemcpyAsync(dseed, seed, w * 4, hipMemcpyHostToDevice, st));
            // chacha.rs:36-45: masked = (secrets + draw) % m over one stream
            const char* force = getenv("SDA_CHACHA_PATH");
            if (!sda::chacha_needs_stream_path(ms->modulus) && !(force && strcmp(force, "stream") == 0)) {
                if (sda_status e = ensure(&h->work, &h->work_bytes, sda::chacha_work_bytes(D, 0))) return e;
                HIP_TRY(sda::launch_chacha_mask_add_async(ms->modulus, D, dseed, w, secrets, dm, h->work, st,
                                                          h->rej_host));
                mask_pending = true;
            } else {
                if (sda_status e = chacha_combine(h, ms->modulus, D, dseed, w, 1, dmask, st)) return e;
                HIP_TRY(sda::launch_addsub_trem(secrets, dmask, +1, D, dm, ms->modulus, st));
            }
            cmask = dmask;
            cseed = dseed;
            cw = w;
        } else {
            return fail(SDA_ERR_INVALID_ARGUMENT, "unknown masking scheme kind");
        }
        masked = dm;
    }
    // 2. ShareGenerator::generate (participate.rs:75-76): shares [n][B]
    const uint64_t n = ss->share_count;
    const uint64_t B = packed ? (D + ss->secret_count - 1) / ss->secret_count : D;
    if (B && !draws) return fail(SDA_ERR_INVALID_ARGUMENT, "need the randomness draws");
    if (payload && n > 65535) return fail(SDA_ERR_UNSUPPORTED, "at most 65535 clerks");
    auto share_and_encode = [&]() -> sda_status {
        if (B) {
            if (packed) {
                if (sda_status e = ensure(&h->gen_log, &h->gen_log_bytes, sda::packed_gen_log_bytes())) return e;
                sda::PackedGenArgs ga{masked, D, 1, draws, shares_out, mode == SDA_REVEAL_CANONICAL};
                HIP_TRY(sda::launch_packed_generate(ga, (uint32_t)ss->secret_count, (uint32_t)ss->privacy_threshold,
                                                    (uint32_t)n, (uint32_t)ss->modulus, (uint32_t)ss->omega_secrets,
                                                    (uint32_t)ss->omega_shares, h->gen_tab, h->gen_log, st));
            } else {
                HIP_TRY(sda::launch_additive_generate(masked, D, draws, n, shares_out, ss->modulus, st));
            }
        }
        // 3. per-clerk payload encoding (participate.rs:79-98 -> sodium.rs:36-41); sealing stays on the host
        if (payload) {
            if (sda_status e = ensure(&h->codec_work, &h->codec_work_bytes, sda::varint_encode_work_bytes(n, B)))
                return e;
            hipError_t e = sda::launch_varint_encode(shares_out, n, B, B, payload, payload_cap, h->codec_work,
                                                     payload_row_bytes, st);
            if (e == hipErrorInvalidValue) return fail(SDA_ERR_INVALID_ARGUMENT, "payload_cap too small");
            HIP_TRY(e);
        }
        return SDA_OK;
    };
    if (sda_status e = share_and_encode()) return e;
    if (mask_pending) {          // the mask's rejection count: redo the mask exactly, and every later step
        HIP_TRY(hipStreamSynchronize(st));
        if (*h->rej_host) {
            if (sda_status e = chacha_combine(h, ms->modulus, D, cseed, cw, 1, cmask, st)) return e;
            HIP_TRY(sda::launch_addsub_trem(secrets, cmask, +1, D, const_cast<int64_t*>(masked), ms->modulus, st));
            if (sda_status e = share_and_encode()) return e;
        }
    }
    return ok();
}

}  // extern "C"
