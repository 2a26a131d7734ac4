// ofdm_internal.h -- kernel argument blocks and launcher declarations shared by the HIP
// translation units of libofdm_mi355x.so.  Not part of the public ABI (include/ofdm_mi355x.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ofdm_mi355x.h"
#include "ofdm_device.h"

namespace ofdm {

constexpr int OFDM_MAX_SNR = 64;       // SNR points per launch (the host splits larger grids)
constexpr int TILE_SYMBOLS = 32;       // data symbols per Tx tile (16 frames x D = 2)
constexpr int TILE_FRAMES = 16;
constexpr int SYM_SAMPLES = 80;        // 64 + 16-sample cyclic prefix (OFDM.c:559-565)

// tiles for n frames, rounded up to an even count so a 64-lane wave can always read 2 tiles
inline int64_t tiles_for(int64_t n_frames) {
    int64_t t = (n_frames + TILE_FRAMES - 1) / TILE_FRAMES;
    return (t + 1) & ~int64_t(1);
}

struct TxArgs {
    float2 *tx;
    uint32_t *bits;
    uint64_t first_symbol;
    int64_t n_sym;                     // symbols to build (tiles * 32)
    uint32_t k0, k1;
    int32_t payload;
    uint32_t table[6];                 // MESSAGE / TESTER payload words (2 symbols x 3 words)
};

struct RxArgs {
    const float2 *tx;
    const uint32_t *bits;
    const float2 *ltf;                 // 64 time samples of one long training symbol (conv-specific)
    uint64_t first_frame;
    int64_t n_frames;
    int64_t n_tiles;
    uint32_t k0, k1;
    int32_t n_snr;
    int32_t q_base;                    // global SNR index of sigma[0] (Philox stream id)
    unsigned long long *counters;      // [n_snr][OFDM_NCOUNTERS] (already offset by q_base)
    float2 *dump_eq;                   // optional parity dumps
    uint32_t *dump_bits;
    int64_t dump_frames;               // leading dimension of the dumps (frames)
    float sigma[OFDM_MAX_SNR];
};

void launch_fft64(hipStream_t st, const float2 *in, float2 *out, int64_t n, int inverse, int conv);
void launch_tx(hipStream_t st, const TxArgs &a, int conv);
void launch_rx(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid);
int rx_grid(const ofdm_cfg &cfg, int64_t n_tiles, int device);

}  // namespace ofdm
