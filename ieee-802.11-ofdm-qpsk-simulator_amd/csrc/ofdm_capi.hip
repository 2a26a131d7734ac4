// ofdm_capi.hip -- the extern "C" boundary (include/ofdm_mi355x.h): contexts, streams, device
// buffers, kernel timing and the symbol-mode sweep driver.  Host code only (the kernels are in
// ofdm_symbol.hip / ofdm_frame.hip).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <complex>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include "ofdm_internal.h"
#include "ofdm_ctx.h"

using namespace ofdm;

namespace ofdm {

thread_local std::string g_last_error;

int set_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

// ------------------------------------------------------------------ host-side frame constants
// Long training symbol T = ifft(Lf) (Preamble_Generator, OFDM.c:368-399) in double, per
// convention; Lf = [0 x6, L_k (53), 0 x5] (OFDM.c:494).
static void host_ltf_time(int conv, std::vector<float2> &out) {
    std::complex<double> X[64], Xs[64], v[64];
    for (int i = 0; i < 64; ++i) X[i] = (double)ltf_sign(i);
    for (int i = 0; i < 64; ++i) Xs[i] = X[(i + 32) & 63];                    // ifftshift
    const double tp = 6.283185307179586476925286766559;
    for (int n = 0; n < 64; ++n) {
        std::complex<double> acc = 0;
        for (int m = 0; m < 64; ++m) acc += Xs[m] * std::polar(1.0, tp * ((m * n) & 63) / 64.0);
        v[n] = acc / 64.0;
    }
    out.resize(64);
    for (int n = 0; n < 64; ++n) {
        const std::complex<double> y = (conv == OFDM_CONV_C) ? v[(n + 32) & 63] : v[n];   // fftshift (C)
        out[n] = make_float2((float)y.real(), (float)y.imag());
    }
}

// payload words: reference message (Data_Generator, OFDM.c:435-465) or MATLAB Tester (Tester.m:50-51)
int payload_table(int payload, const std::string &message, uint32_t table[3 * MSG_MAX_FRAMES]) {
    unsigned char bytes[MSG_MAX_CHARS];
    int frames;
    if (payload == OFDM_PAYLOAD_TESTER) {                       // 'A' x 11 + ' ' per 96 bits (Tester.m:50-51)
        frames = 2;
        for (int f = 0; f < 2; ++f)
            for (int c = 0; c < 12; ++c) bytes[12 * f + c] = c < 11 ? 0x41 : 0x20;
    } else {
        const int len = (int)message.size();
        frames = (8 * len + 95) / 96;                           // ceil(8 len / 96) (OFDM.c:439)
        for (int c = 0; c < 12 * frames; ++c) bytes[c] = c < len ? (unsigned char)message[c] : ' ';
    }
    for (int w = 0; w < 3 * frames; ++w)
        table[w] = ((uint32_t)bytes[4 * w] << 24) | ((uint32_t)bytes[4 * w + 1] << 16) |
                   ((uint32_t)bytes[4 * w + 2] << 8) | (uint32_t)bytes[4 * w + 3];
    for (int w = 3 * frames; w < 3 * MSG_MAX_FRAMES; ++w) table[w] = 0u;
    return frames;
}

int check_cfg(const ofdm_cfg *c) {
    if (!c) return set_error(OFDM_E_ARG, "cfg is NULL");
    if (c->conv != OFDM_CONV_C && c->conv != OFDM_CONV_MATLAB) return set_error(OFDM_E_ARG, "bad conv %d", c->conv);
    if (c->payload < 0 || c->payload > 2) return set_error(OFDM_E_ARG, "bad payload %d", c->payload);
    if (c->est != OFDM_EST_LS && c->est != OFDM_EST_IDEAL) return set_error(OFDM_E_ARG, "bad est %d", c->est);
    if (c->noise < 0 || c->noise > 2) return set_error(OFDM_E_ARG, "bad noise %d", c->noise);
    if (c->channel != OFDM_CHAN_AWGN && c->channel != OFDM_CHAN_RAYLEIGH4)
        return set_error(OFDM_E_ARG, "bad channel %d", c->channel);
    if (c->data_per_frame != 2) return set_error(OFDM_E_ARG, "data_per_frame must be 2 (got %d)", c->data_per_frame);
    if (!(c->kappa > 0) || !(c->p_ref > 0)) return set_error(OFDM_E_ARG, "kappa and p_ref must be > 0");
    return OFDM_OK;
}

// ------------------------------------------------------------------ timing
void Ctx::tic(int k) {
    if (!timing) return;
    Ev e;
    e.kernel = k;
    if (!pool.empty()) { e.a = pool.back(); pool.pop_back(); } else hipEventCreate(&e.a);
    if (!pool.empty()) { e.b = pool.back(); pool.pop_back(); } else hipEventCreate(&e.b);
    hipEventRecord(e.a, stream);
    open.push_back(e);
}
void Ctx::toc() {
    if (!timing || open.empty()) return;
    hipEventRecord(open.back().b, stream);
    done.push_back(open.back());
    open.pop_back();
}
void Ctx::resolve() {
    for (auto &e : done) {
        float ms = 0.f;
        hipEventSynchronize(e.b);
        hipEventElapsedTime(&ms, e.a, e.b);
        acc_ms[e.kernel] += ms;
        launches[e.kernel] += 1;
        pool.push_back(e.a);
        pool.push_back(e.b);
    }
    done.clear();
}

// OFDM_DEVICE_ALLOC_CAP=<bytes>: a scratch allocation above it fails as if hipMalloc had (OFDM_E_NOMEM) -- the
// test hook of the frame sweep's chunk-halving path (tests/test_gpu_frame.py::test_frame_sweep_nomem_halving_*)
static size_t alloc_cap() {
    const char *s = getenv("OFDM_DEVICE_ALLOC_CAP");
    return s && *s ? (size_t)strtoull(s, nullptr, 10) : SIZE_MAX;
}

int Ctx::ensure(void **p, size_t *cap, size_t bytes) {
    if (*cap >= bytes) return OFDM_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (bytes > alloc_cap()) return set_error(OFDM_E_NOMEM, "allocation of %zu bytes above OFDM_DEVICE_ALLOC_CAP", bytes);
    if (hipMalloc(p, bytes) != hipSuccess) {
        *p = nullptr;
        return set_error(OFDM_E_NOMEM, "hipMalloc(%zu) failed", bytes);
    }
    *cap = bytes;
    return OFDM_OK;
}

int Ctx::read_counters(void *out, size_t bytes) {
    if (cap_h_cnt < bytes) {
        if (h_cnt) hipHostFree(h_cnt);
        h_cnt = nullptr;
        cap_h_cnt = 0;
        if (hipHostMalloc(&h_cnt, bytes, hipHostMallocDefault) != hipSuccess) {
            h_cnt = nullptr;
            return set_error(OFDM_E_NOMEM, "hipHostMalloc(%zu) failed", bytes);
        }
        cap_h_cnt = bytes;
    }
    hipError_t e = hipMemcpyAsync(h_cnt, d_cnt, bytes, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return set_error(OFDM_E_HIP, "counter read-back: %s", hipGetErrorString(e));
    std::memcpy(out, h_cnt, bytes);
    return OFDM_OK;
}

}  // namespace ofdm

#define HIPOK(expr)                                                                             \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return set_error(OFDM_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

extern "C" {

int ofdm_abi_version(void) { return OFDM_ABI_VERSION; }
const char *ofdm_last_error(void) { return g_last_error.c_str(); }

int ofdm_device_count(int *count) {
    if (!count) return set_error(OFDM_E_ARG, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return OFDM_OK;
}

int ofdm_ctx_create(int device, ofdm_ctx **out) {
    if (!out) return set_error(OFDM_E_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_error(OFDM_E_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return set_error(OFDM_E_ARG, "device %d out of range [0,%d)", device, n);
    HIPOK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPOK(hipGetDeviceProperties(&prop, device));
    if (!strstr(prop.gcnArchName, "gfx950"))
        return set_error(OFDM_E_NODEV, "device %d is %s; this library is built for gfx950 only", device, prop.gcnArchName);
    Ctx *c = new Ctx();
    c->device = device;
    c->cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_error(OFDM_E_HIP, "hipStreamCreate failed");
    }
    c->stream = c->own;
    for (int conv = 0; conv < 2; ++conv) {
        std::vector<float2> t;
        host_ltf_time(conv, t);
        // 2T by staged row for the LS receiver: row r of a group holds window sample n = r - 4
        // (rows start 3+1 samples into the CP for the 4-tap channel), cyclic in T
        std::vector<float2> t2(68 * 2);
        for (int r = 0; r < 68; ++r) {
            const float2 v = t[(r - 4 + 64) & 63];
            t2[2 * r] = t2[2 * r + 1] = make_float2(2.0f * v.x, 2.0f * v.y);
        }
        if (hipMalloc(&c->d_ltf[conv], 64 * sizeof(float2)) != hipSuccess ||
            hipMemcpy(c->d_ltf[conv], t.data(), 64 * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
            hipMalloc(&c->d_ltf2_rows[conv], t2.size() * sizeof(float2)) != hipSuccess ||
            hipMemcpy(c->d_ltf2_rows[conv], t2.data(), t2.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
            ofdm_ctx_destroy(reinterpret_cast<ofdm_ctx *>(c));
            return set_error(OFDM_E_NOMEM, "LTF table upload failed");
        }
    }
    *out = reinterpret_cast<ofdm_ctx *>(c);
    return OFDM_OK;
}

int ofdm_ctx_destroy(ofdm_ctx *ctx) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return OFDM_OK;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    for (auto &e : c->done) { hipEventDestroy(e.a); hipEventDestroy(e.b); }
    for (auto &e : c->open) { hipEventDestroy(e.a); hipEventDestroy(e.b); }
    for (auto ev : c->pool) hipEventDestroy(ev);
    if (c->tx_stream) hipStreamSynchronize(c->tx_stream);
    for (void *p : {(void *)c->d_ltf[0], (void *)c->d_ltf[1], (void *)c->d_ltf2_rows[0], (void *)c->d_ltf2_rows[1], c->d_tx, c->d_bits, c->d_cnt, c->d_scratch,
                    c->d_scratch2, c->d_wave, c->d_tx2, c->d_bits2, c->d_work})
        if (p) hipFree(p);
    for (hipEvent_t ev : {c->ev_start, c->ev_tx[0], c->ev_tx[1], c->ev_rx[0], c->ev_rx[1]})
        if (ev) hipEventDestroy(ev);
    if (c->h_cnt) hipHostFree(c->h_cnt);
    if (c->tx_stream) hipStreamDestroy(c->tx_stream);
    if (c->own) hipStreamDestroy(c->own);
    delete c;
    return OFDM_OK;
}

int ofdm_ctx_trim(ofdm_ctx *ctx, int64_t *released) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    HIPOK(hipSetDevice(c->device));
    // every launch that may still read or write the scratch has finished (both of the context's streams)
    HIPOK(hipStreamSynchronize(c->stream));
    if (c->tx_stream) HIPOK(hipStreamSynchronize(c->tx_stream));
    int64_t n = 0;
    struct { void **p; size_t *cap; } bufs[] = {{&c->d_tx, &c->cap_tx}, {&c->d_bits, &c->cap_bits}, {&c->d_tx2, &c->cap_tx2},
                                                {&c->d_bits2, &c->cap_bits2}, {&c->d_cnt, &c->cap_cnt},
                                                {&c->d_scratch, &c->cap_scratch}, {&c->d_scratch2, &c->cap_scratch2}};
    for (auto &b : bufs) {
        if (*b.p) {
            HIPOK(hipFree(*b.p));
            n += (int64_t)*b.cap;
        }
        *b.p = nullptr;
        *b.cap = 0;
    }
    if (released) *released = n;
    return OFDM_OK;
}

int ofdm_ctx_scratch_bytes(ofdm_ctx *ctx, int64_t *bytes) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || !bytes) return set_error(OFDM_E_ARG, "bad scratch_bytes arguments");
    *bytes = (int64_t)(c->cap_tx + c->cap_bits + c->cap_tx2 + c->cap_bits2 + c->cap_cnt + c->cap_scratch + c->cap_scratch2);
    return OFDM_OK;
}

int ofdm_ctx_set_stream(ofdm_ctx *ctx, void *stream) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    c->stream = reinterpret_cast<hipStream_t>(stream);   // NULL = null stream, ordered with it
    return OFDM_OK;
}

int ofdm_ctx_synchronize(ofdm_ctx *ctx) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipStreamSynchronize(c->stream));
    return OFDM_OK;
}

int ofdm_set_message(ofdm_ctx *ctx, const char *msg, int32_t len, int32_t *frames) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || (len && !msg)) return set_error(OFDM_E_ARG, "bad message arguments");
    if (len < 1 || len > MSG_MAX_CHARS)
        return set_error(OFDM_E_ARG, "message length %d outside [1, %d] (at most %d data symbols per frame)", len,
                         MSG_MAX_CHARS, MSG_MAX_FRAMES);
    c->message.assign(msg, (size_t)len);
    c->wave_key = -1;                                          // the frame waveform depends on it
    if (frames) *frames = (8 * len + 95) / 96;
    return OFDM_OK;
}

int ofdm_payload_frames(ofdm_ctx *ctx, int payload, int32_t *frames) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || !frames) return set_error(OFDM_E_ARG, "bad arguments");
    if (payload != OFDM_PAYLOAD_MESSAGE && payload != OFDM_PAYLOAD_TESTER)
        return set_error(OFDM_E_ARG, "payload %d has no fixed frame structure", payload);
    uint32_t t[3 * MSG_MAX_FRAMES];
    *frames = payload_table(payload, c->message, t);
    return OFDM_OK;
}

int ofdm_timing_enable(ofdm_ctx *ctx, int enable) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    c->timing = enable != 0;
    return OFDM_OK;
}

int ofdm_timing_query(ofdm_ctx *ctx, int kernel, double *ms_total, int64_t *launches) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || kernel < 0 || kernel >= Ctx::NK) return set_error(OFDM_E_ARG, "bad ctx/kernel");
    hipSetDevice(c->device);
    c->resolve();
    if (ms_total) *ms_total = c->acc_ms[kernel];
    if (launches) *launches = c->launches[kernel];
    return OFDM_OK;
}

int ofdm_timing_reset(ofdm_ctx *ctx) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    hipSetDevice(c->device);
    c->resolve();
    for (int k = 0; k < Ctx::NK; ++k) { c->acc_ms[k] = 0; c->launches[k] = 0; }
    return OFDM_OK;
}

int ofdm_fft64(ofdm_ctx *ctx, const void *d_in, void *d_out, int64_t n, int inverse, int conv) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || (!d_in && n) || (!d_out && n) || n < 0) return set_error(OFDM_E_ARG, "bad fft64 arguments");
    if (conv != OFDM_CONV_C && conv != OFDM_CONV_MATLAB) return set_error(OFDM_E_ARG, "bad conv %d", conv);
    if (n == 0) return OFDM_OK;
    HIPOK(hipSetDevice(c->device));
    c->tic(Ctx::K_FFT);
    launch_fft64(c->stream, (const float2 *)d_in, (float2 *)d_out, n, inverse, conv);
    c->toc();
    HIPOK(hipGetLastError());
    return OFDM_OK;
}

int ofdm_tx_bytes(int64_t n_frames, int64_t *tx_bytes, int64_t *bits_bytes) {
    if (n_frames < 0 || n_frames > MAX_BATCH_FRAMES)
        return set_error(OFDM_E_ARG, "n_frames %lld outside [0, %lld]", (long long)n_frames, (long long)MAX_BATCH_FRAMES);
    const int64_t p = sym_pitch(n_frames);
    if (tx_bytes) *tx_bytes = SYM_SAMPLES * p * (int64_t)sizeof(float2);
    if (bits_bytes) *bits_bytes = TX_BIT_ROWS * p * (int64_t)sizeof(uint32_t);
    return OFDM_OK;
}

static int check_tx(Ctx *c, const ofdm_cfg *cfg, int64_t n_frames, const void *d_tx, const void *d_bits) {
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (n_frames < 0 || (n_frames && (!d_tx || !d_bits))) return set_error(OFDM_E_ARG, "bad tx buffers");
    if (n_frames > MAX_BATCH_FRAMES) return set_error(OFDM_E_ARG, "n_frames > %lld per batch", (long long)MAX_BATCH_FRAMES);
    return OFDM_OK;
}

static TxArgs tx_args(Ctx *c, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames, void *d_tx, void *d_bits) {
    TxArgs a{};
    a.tx = (float2 *)d_tx;
    a.bits = (uint32_t *)d_bits;
    a.first_symbol = 2 * first_frame;
    a.pitch = sym_pitch(n_frames);
    a.n_sym = (2 * n_frames + 63) / 64 * 64;
    a.k0 = (uint32_t)cfg->seed;
    a.k1 = (uint32_t)(cfg->seed >> 32);
    a.payload = cfg->payload;
    a.table_frames = payload_table(cfg->payload, c->message, a.table);
    return a;
}

int ofdm_tx_frames(ofdm_ctx *ctx, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames, void *d_tx,
                   void *d_bits) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    int rc = check_tx(c, cfg, n_frames, d_tx, d_bits);
    if (rc) return rc;
    if (n_frames == 0) return OFDM_OK;
    HIPOK(hipSetDevice(c->device));
    const TxArgs a = tx_args(c, cfg, first_frame, n_frames, d_tx, d_bits);
    c->tic(Ctx::K_TX);
    launch_tx(c->stream, a, cfg->conv);
    c->toc();
    HIPOK(hipGetLastError());
    return OFDM_OK;
}

int ofdm_set_next_tx(ofdm_ctx *ctx, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames, void *d_tx,
                     void *d_bits) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    int rc = check_tx(c, cfg, n_frames, d_tx, d_bits);
    if (rc) return rc;
    c->nx_pending = n_frames > 0;
    c->nx_cfg = *cfg;
    c->nx_first = first_frame;
    c->nx_n = n_frames;
    c->nx_tx = d_tx;
    c->nx_bits = d_bits;
    return OFDM_OK;
}

// [a, a + na) and [b, b + nb) share a byte
static bool overlaps(const void *a, int64_t na, const void *b, int64_t nb) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return na > 0 && nb > 0 && x < y + (uintptr_t)nb && y < x + (uintptr_t)na;
}

// own_tx: the call also builds the batch it reads (ofdm_txrx_frames), d_tx / d_bits then being writable
static int rx_common(Ctx *c, const ofdm_cfg *cfg, const void *d_tx, const void *d_bits, uint64_t first_frame,
                     int64_t n_frames, const double *snr_db, int n_snr, void *d_counters, void *d_eq, void *d_dbits,
                     bool own_tx = false) {
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    // every argument check first: a call that fails them returns with a pending ofdm_set_next_tx batch still
    // pending (nothing consumed, nothing launched)
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (n_snr < 0 || (n_snr && !snr_db) || !d_counters) return set_error(OFDM_E_ARG, "bad snr/counters");
    if (n_frames < 0 || (n_frames && (!d_tx || !d_bits))) return set_error(OFDM_E_ARG, "bad rx buffers");
    if (n_frames > MAX_BATCH_FRAMES) return set_error(OFDM_E_ARG, "n_frames > %lld per batch", (long long)MAX_BATCH_FRAMES);
    const bool dump = d_eq || d_dbits;
    if (dump && (!d_eq || !d_dbits)) return set_error(OFDM_E_ARG, "dump needs both d_eq and d_dbits");
    // a pending next batch is written while this call reads (or, fused, builds) its own: the two must not share a
    // byte (groups of one launch would race on it)
    if (c->nx_pending && n_frames > 0) {
        int64_t otx, obits, ntx, nbits;
        ofdm_tx_bytes(n_frames, &otx, &obits);
        ofdm_tx_bytes(c->nx_n, &ntx, &nbits);
        const void *own[2] = {d_tx, d_bits}, *nx[2] = {c->nx_tx, c->nx_bits};
        const int64_t osz[2] = {otx, obits}, nsz[2] = {ntx, nbits};
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                if (overlaps(own[i], osz[i], nx[j], nsz[j]))
                    return set_error(OFDM_E_ARG, "the pending ofdm_set_next_tx batch overlaps this call's batch");
    }
    // a pending ofdm_set_next_tx batch: fused into the packed receiver's group prologues when this call
    // launches it, otherwise built by the Tx kernel right here (same stream, so it is ready in either case
    // once this call's work is)
    bool fuse_nx = false;
    const bool packed = !dump && n_frames > 0 && n_snr > 0 && rx_pack_applies(*cfg);
    if (c->nx_pending) {
        c->nx_pending = false;
        fuse_nx = packed;
        if (!fuse_nx) {
            const int rt = ofdm_tx_frames(reinterpret_cast<ofdm_ctx *>(c), &c->nx_cfg, c->nx_first, c->nx_n,
                                          c->nx_tx, c->nx_bits);
            if (rt) return rt;
        }
    }
    // the call's own batch: built in the packed receiver's group prologues, otherwise by the Tx kernel first
    const bool fuse_own = own_tx && packed;
    if (own_tx && !fuse_own) {
        const int rt = ofdm_tx_frames(reinterpret_cast<ofdm_ctx *>(c), cfg, first_frame, n_frames,
                                      const_cast<void *>(d_tx), const_cast<void *>(d_bits));
        if (rt) return rt;
    }
    if (n_frames == 0 || n_snr == 0) return OFDM_OK;
    HIPOK(hipSetDevice(c->device));
    const unsigned grid = (unsigned)rx_grid(*cfg, n_frames, c->device);
    for (int q0 = 0; q0 < n_snr; q0 += OFDM_MAX_SNR) {
        RxArgs a{};
        a.tx = (const float2 *)d_tx;
        a.bits = (const uint32_t *)d_bits;
        a.ltf = c->d_ltf[cfg->conv];
        a.ltf2_rows = c->d_ltf2_rows[cfg->conv];
        a.first_frame = first_frame;
        a.n_frames = n_frames;
        a.pitch = sym_pitch(n_frames);
        a.k0 = (uint32_t)cfg->seed;
        a.k1 = (uint32_t)(cfg->seed >> 32);
        a.n_snr = std::min(OFDM_MAX_SNR, n_snr - q0);
        a.q_base = q0;
        a.counters = (unsigned long long *)d_counters + (size_t)q0 * OFDM_NCOUNTERS;
        a.dump_frames = n_frames;
        if (dump) {
            a.dump_eq = (float2 *)d_eq + (size_t)q0 * n_frames * 2 * 48;
            a.dump_bits = (uint32_t *)d_dbits + (size_t)q0 * n_frames * 2 * 3;
        }
        for (int q = 0; q < a.n_snr; ++q) {
            const double s2 = cfg->kappa * cfg->p_ref / std::pow(10.0, snr_db[q0 + q] / 10.0);
            a.sigma[q] = (float)std::sqrt(s2);
        }
        if (fuse_nx && q0 == 0) {
            a.nx = tx_args(c, &c->nx_cfg, c->nx_first, c->nx_n, c->nx_tx, c->nx_bits);
            a.nx_conv = c->nx_cfg.conv;
        }
        if (fuse_own && q0 == 0) {       // later SNR slices read the batch the first launch built
            a.own = tx_args(c, cfg, first_frame, n_frames, const_cast<void *>(d_tx), const_cast<void *>(d_bits));
            a.own_conv = cfg->conv;
        }
        if (!c->d_work) HIPOK(hipMalloc(&c->d_work, 256));
        a.work = (unsigned long long *)c->d_work;
        HIPOK(hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        c->tic(Ctx::K_RX);
        launch_rx(c->stream, a, *cfg, dump, grid);
        c->toc();
        HIPOK(hipGetLastError());
    }
    return OFDM_OK;
}

int ofdm_rx_frames(ofdm_ctx *ctx, const ofdm_cfg *cfg, const void *d_tx, const void *d_bits, uint64_t first_frame,
                   int64_t n_frames, const double *snr_db, int n_snr, void *d_counters) {
    return rx_common(reinterpret_cast<Ctx *>(ctx), cfg, d_tx, d_bits, first_frame, n_frames, snr_db, n_snr,
                     d_counters, nullptr, nullptr);
}

int ofdm_rx_frames_dump(ofdm_ctx *ctx, const ofdm_cfg *cfg, const void *d_tx, const void *d_bits,
                        uint64_t first_frame, int64_t n_frames, const double *snr_db, int n_snr, void *d_counters,
                        void *d_eq, void *d_dbits) {
    return rx_common(reinterpret_cast<Ctx *>(ctx), cfg, d_tx, d_bits, first_frame, n_frames, snr_db, n_snr,
                     d_counters, d_eq, d_dbits);
}

int ofdm_txrx_frames(ofdm_ctx *ctx, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames, void *d_tx,
                     void *d_bits, const double *snr_db, int n_snr, void *d_counters) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    int rc = check_tx(c, cfg, n_frames, d_tx, d_bits);
    if (rc) return rc;
    return rx_common(c, cfg, d_tx, d_bits, first_frame, n_frames, snr_db, n_snr, d_counters, nullptr, nullptr, true);
}

int ofdm_symbol_sweep(ofdm_ctx *ctx, const ofdm_cfg *cfg, const double *snr_db, int n_snr, uint64_t first_frame,
                      int64_t n_frames, int64_t chunk_frames, int64_t *counters) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (n_snr < 0 || (n_snr && (!snr_db || !counters)) || n_frames < 0) return set_error(OFDM_E_ARG, "bad sweep args");
    if (n_snr == 0) return OFDM_OK;
    HIPOK(hipSetDevice(c->device));
    if (c->nx_pending) {             // a batch queued by the caller: built now, before the sweep's own batches
        c->nx_pending = false;
        if ((rc = ofdm_tx_frames(ctx, &c->nx_cfg, c->nx_first, c->nx_n, c->nx_tx, c->nx_bits))) return rc;
    }
    const size_t cbytes = (size_t)n_snr * OFDM_NCOUNTERS * sizeof(int64_t);
    if ((rc = c->ensure(&c->d_cnt, &c->cap_cnt, cbytes))) return rc;
    HIPOK(hipMemsetAsync(c->d_cnt, 0, cbytes, c->stream));
    if (chunk_frames <= 0) {
        // 8.4M symbols (~5.4 GB) per chunk, and at least SWEEP_PIPE chunks of >= 2^18 frames, so that the
        // HBM-bound Tx of chunk k+1 runs on the context's second stream under the VALU-bound receiver of
        // chunk k (double-buffered batches; the counters do not depend on the chunking)
        chunk_frames = int64_t(1) << 22;
        constexpr int64_t SWEEP_PIPE = 4, MIN_PIPE = int64_t(1) << 18;
        if (n_frames >= SWEEP_PIPE * MIN_PIPE) chunk_frames = std::min(chunk_frames, (n_frames + SWEEP_PIPE - 1) / SWEEP_PIPE);
    }
    chunk_frames = std::min(chunk_frames, MAX_BATCH_FRAMES);
    const int64_t cf = std::min<int64_t>(chunk_frames, std::max<int64_t>(n_frames, 1));
    const int64_t n_chunks = (n_frames + cf - 1) / cf;
    int64_t txb = 0, bb = 0;
    ofdm_tx_bytes(cf, &txb, &bb);
    if ((rc = c->ensure(&c->d_tx, &c->cap_tx, (size_t)txb))) return rc;
    if ((rc = c->ensure(&c->d_bits, &c->cap_bits, (size_t)bb))) return rc;
    if (n_chunks > 1) {
        if ((rc = c->ensure(&c->d_tx2, &c->cap_tx2, (size_t)txb))) return rc;
        if ((rc = c->ensure(&c->d_bits2, &c->cap_bits2, (size_t)bb))) return rc;
        if (!c->tx_stream) HIPOK(hipStreamCreateWithFlags(&c->tx_stream, hipStreamNonBlocking));
        for (hipEvent_t *ev : {&c->ev_start, &c->ev_tx[0], &c->ev_tx[1], &c->ev_rx[0], &c->ev_rx[1]})
            if (!*ev) HIPOK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        HIPOK(hipEventRecord(c->ev_start, c->stream));          // the Tx stream starts after the memset
        HIPOK(hipStreamWaitEvent(c->tx_stream, c->ev_start, 0));
    }
    float2 *txbuf[2] = {(float2 *)c->d_tx, (float2 *)c->d_tx2};
    uint32_t *bitbuf[2] = {(uint32_t *)c->d_bits, (uint32_t *)c->d_bits2};
    hipStream_t main_stream = c->stream;
    auto chunk_of = [&](int64_t k, int64_t *first, int64_t *nf) { *first = first_frame + k * cf; *nf = std::min(cf, n_frames - k * cf); };
    int64_t f0, n0;
    chunk_of(0, &f0, &n0);
    if (rx_pack_applies(*cfg)) {
        // the packed receivers build the Tx batches themselves, one stream: chunk 0's receiver its own batch
        // (ofdm_txrx_frames) and the receiver of chunk k chunk k+1's batch (ofdm_set_next_tx) in their group
        // prologues; the batch a receiver overwrites was last read by receiver k-1
        for (int64_t k = 0; k < n_chunks; ++k) {
            if (k + 1 < n_chunks) {
                int64_t f1, n1;
                chunk_of(k + 1, &f1, &n1);
                if ((rc = ofdm_set_next_tx(ctx, cfg, f1, n1, txbuf[(k + 1) & 1], bitbuf[(k + 1) & 1]))) return rc;
            }
            int64_t fk, nk;
            chunk_of(k, &fk, &nk);
            rc = k == 0 ? ofdm_txrx_frames(ctx, cfg, fk, nk, txbuf[0], bitbuf[0], snr_db, n_snr, c->d_cnt)
                        : ofdm_rx_frames(ctx, cfg, txbuf[k & 1], bitbuf[k & 1], fk, nk, snr_db, n_snr, c->d_cnt);
            if (rc) return rc;
        }
        return c->read_counters(counters, cbytes);
    }
    if ((rc = ofdm_tx_frames(ctx, cfg, f0, n0, txbuf[0], bitbuf[0]))) return rc;
    for (int64_t k = 0; k < n_chunks; ++k) {
        if (k + 1 < n_chunks) {                                  // Tx of chunk k+1 into the other batch
            if (k >= 1) HIPOK(hipStreamWaitEvent(c->tx_stream, c->ev_rx[(k - 1) & 1], 0));   // chunk k-1 read it
            int64_t f1, n1;
            chunk_of(k + 1, &f1, &n1);
            c->stream = c->tx_stream;
            rc = ofdm_tx_frames(ctx, cfg, f1, n1, txbuf[(k + 1) & 1], bitbuf[(k + 1) & 1]);
            c->stream = main_stream;
            if (rc) return rc;
            HIPOK(hipEventRecord(c->ev_tx[(k + 1) & 1], c->tx_stream));
        }
        if (k >= 1) HIPOK(hipStreamWaitEvent(main_stream, c->ev_tx[k & 1], 0));
        int64_t fk, nk;
        chunk_of(k, &fk, &nk);
        if ((rc = ofdm_rx_frames(ctx, cfg, txbuf[k & 1], bitbuf[k & 1], fk, nk, snr_db, n_snr, c->d_cnt))) return rc;
        if (n_chunks > 1) HIPOK(hipEventRecord(c->ev_rx[k & 1], main_stream));
    }
    return c->read_counters(counters, cbytes);
}

}  // extern "C"
