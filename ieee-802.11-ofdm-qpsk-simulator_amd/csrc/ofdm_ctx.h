// ofdm_ctx.h -- the opaque ofdm_ctx behind the C ABI (host-side state of one GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <string>
#include <vector>
#include "ofdm_mi355x.h"

namespace ofdm {

int set_error(int code, const char *fmt, ...);
int check_cfg(const ofdm_cfg *c);

constexpr int MSG_MAX_FRAMES = 8;           // data symbols per frame-mode frame (LDS budget)
constexpr int MSG_MAX_CHARS = 12 * MSG_MAX_FRAMES;
// payload words (MSB-first bits, 3 per data symbol) of the TESTER pattern or `message` padded with
// ' ' to whole symbols (Data_Generator, OFDM.c:435-465); returns the data symbols per frame
int payload_table(int payload, const std::string &message, uint32_t table[3 * MSG_MAX_FRAMES]);

struct Ctx {
    enum { K_FFT = 0, K_TX = 1, K_RX = 2, K_FRAME = 3, NK = 4 };
    int device = 0;
    int cus = 256;
    hipStream_t own = nullptr;       // created by the context
    hipStream_t stream = nullptr;    // where work is enqueued (own or external)
    float2 *d_ltf[2] = {nullptr, nullptr};
    float2 *d_ltf2_rows[2] = {nullptr, nullptr};   // LS staging column: [68][2] 2T[(r - 4) mod 64]
    std::string message = "Hey! I am Vivaswan";   // MESSAGE payload (OFDM.c:20), ofdm_set_message
    // sweep scratch (grown on demand, freed with the context)
    void *d_tx = nullptr, *d_bits = nullptr, *d_cnt = nullptr, *d_scratch = nullptr, *d_scratch2 = nullptr;
    // ofdm_symbol_sweep's pipeline: the second Tx batch and the stream the next chunk's Tx runs on
    void *d_tx2 = nullptr, *d_bits2 = nullptr;
    size_t cap_tx2 = 0, cap_bits2 = 0;
    hipStream_t tx_stream = nullptr;
    // ofdm_set_next_tx: a Tx batch the next ofdm_rx_frames call builds (fused into the packed receiver)
    bool nx_pending = false;
    ofdm_cfg nx_cfg{};
    uint64_t nx_first = 0;
    int64_t nx_n = 0;
    void *nx_tx = nullptr, *nx_bits = nullptr;
    hipEvent_t ev_start = nullptr, ev_tx[2] = {nullptr, nullptr}, ev_rx[2] = {nullptr, nullptr};
    void *d_wave = nullptr;
    void *d_work = nullptr;          // K3c's work-item counter (one receiver launch in flight per context)
    // pinned host staging for the sweeps' counter read-back (a pageable destination costs HIP a staging copy kernel
    // and a host round trip per call); grown on demand, freed with the context
    void *h_cnt = nullptr;
    size_t cap_h_cnt = 0;
    size_t cap_tx = 0, cap_bits = 0, cap_cnt = 0, cap_scratch = 0, cap_scratch2 = 0, cap_wave = 0;
    // frame-mode waveform cache (per conv/payload/message)
    int wave_key = -1;
    int wave_frames = 0;
    int32_t wave_len = 0;
    double wave_power = 0.0;
    // kernel timing
    struct Ev { hipEvent_t a, b; int kernel; };
    bool timing = false;
    std::vector<Ev> open, done;
    std::vector<hipEvent_t> pool;
    double acc_ms[NK] = {0, 0, 0, 0};
    int64_t launches[NK] = {0, 0, 0, 0};

    void tic(int k);
    void toc();
    void resolve();
    int ensure(void **p, size_t *cap, size_t bytes);
    // d_cnt[0, bytes) -> host `out` on `stream` through the pinned staging buffer; returns after the copy has landed
    int read_counters(void *out, size_t bytes);
};

}  // namespace ofdm
