// ofdm_internal.h -- kernel argument blocks and launcher declarations shared by the HIP
// translation units of libofdm_mi355x.so.  Not part of the public ABI (include/ofdm_mi355x.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ofdm_mi355x.h"
#include "ofdm_device.h"

namespace ofdm {

constexpr int OFDM_MAX_SNR = 64;       // SNR points per launch (the host splits larger grids)
constexpr int SYM_SAMPLES = 80;        // 64 + 16-sample cyclic prefix (OFDM.c:559-565)

// Tx batch layout, rows of symbols ("structure of arrays" over the batch):
//   tx  [n * pitch + s] = time sample n (0..79, CP first) of data symbol s = 2 * frame + d
//   bits[k * pitch + s] = payload word k (MSB-first bits 32k..32k+31) of symbol s, k = 0..2;
//                         rows k = 3..6: demap word k - 3 (ofdm_rxcommon.h demap_word)
//                         rows k = 7..9: pair-order word k - 7 (ofdm_rxcommon.h pair_words)
// pitch = symbols rounded up to a whole wave plus one guard wave, so whole-wave reads and the
// receivers' groups (LS: 42 symbols, packed: 128 symbols) stay inside the buffer.
inline int64_t sym_pitch(int64_t n_frames) { return (2 * n_frames + 63) / 64 * 64 + 64; }
constexpr int TX_BIT_ROWS = 10;
constexpr int64_t MAX_BATCH_FRAMES = int64_t(1) << 23;   // 80 * pitch fits int32 element offsets

// LS receiver grouping: 21 frames per wave, lanes {E, D0, D1} x 21 + 1 idle
constexpr int LS_GROUP_FRAMES = 21;
constexpr int LS_GROUP_SYMS = 42;
constexpr int LS_ROW_F2 = 44;          // staged LDS row: 42 data symbols + 2T sample (x2, one 16-B chunk)

struct TxArgs {
    float2 *tx;
    uint32_t *bits;
    uint64_t first_symbol;
    int64_t n_sym;                     // symbols to build (whole waves, < pitch)
    int64_t pitch;
    uint32_t k0, k1;
    int32_t payload;
    int32_t table_frames;              // MESSAGE / TESTER: symbols in the payload table
    uint32_t table[24];                // MESSAGE / TESTER payload words (3 per symbol; symbol s uses s % frames)
};

struct RxArgs {
    const float2 *tx;
    const uint32_t *bits;
    const float2 *ltf;                 // 64 time samples of one long training symbol (conv-specific)
    uint64_t first_frame;
    int64_t n_frames;
    int64_t pitch;
    const float2 *ltf2_rows;           // LS: [row][2] 2T[(row + R0 - 16) mod 64], row pitch 16 B
    uint32_t k0, k1;
    int32_t n_snr;
    int32_t q_base;                    // global SNR index of sigma[0] (Philox stream id)
    unsigned long long *counters;      // [n_snr][OFDM_NCOUNTERS] (already offset by q_base)
    float2 *dump_eq;                   // optional parity dumps
    uint32_t *dump_bits;
    int64_t dump_frames;               // leading dimension of the dumps (frames)
    unsigned long long *stamps;        // OFDM_RX_STAMPS builds: cycles per receiver phase [5]
    unsigned long long *work;          // K3c: work items handed out past the first gridDim.x (zeroed per launch)
    TxArgs nx;                         // K3c: the NEXT chunk's Tx batch, built in the group prologues (n_sym 0: none)
    int32_t nx_conv;                   // its ifft convention
    TxArgs own;                        // K3c: THIS launch's Tx batch (ofdm_txrx_frames), each group built by the
    int32_t own_conv;                  // items that read it, before its clean spectra (n_sym 0: none)
    float sigma[OFDM_MAX_SNR];
};

void launch_fft64(hipStream_t st, const float2 *in, float2 *out, int64_t n, int inverse, int conv);
void launch_tx(hipStream_t st, const TxArgs &a, int conv);
void launch_rx(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid);
int rx_grid(const ofdm_cfg &cfg, int64_t n_frames, int device);
// K3c (ofdm_rxpack.hip): real-noise AWGN receivers, one frame per lane, two noise windows per FFT
bool rx_pack_applies(const ofdm_cfg &cfg);
void launch_rx_pack(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid);
int rx_pack_grid(const ofdm_cfg &cfg, int64_t n_frames, int device);
// K3c's ideal-CSI instantiations (ofdm_rxpack_ideal.hip)
void launch_rx_pack_ideal(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid);
int rx_pack_ideal_grid(int64_t n_frames, int device);

}  // namespace ofdm
