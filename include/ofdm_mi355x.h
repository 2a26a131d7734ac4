/*
 * ofdm_mi355x.h -- C ABI of the MI355X-native 802.11a OFDM-QPSK Monte-Carlo engine
 * (libofdm_mi355x.so, built from ieee-802.11-ofdm-qpsk-simulator_amd/csrc/).
 *
 * The reference (Unalome81/IEEE-802.11-OFDM-QPSK-Simulator, src/OFDM.c) has no library API: its
 * hot path is three internal functions driven by main() and its only external surface is the
 * data/Output_*.txt files (OFDM.c:1228-1231).  The entry points below replace those functions;
 * each cites the reference interface it stands in for.  The Python host
 * (ieee-802.11-ofdm-qpsk-simulator_amd/abi.py, engine.py, sweep.py) binds them with ctypes and writes
 * the same files.
 *
 * Conventions: plain pointers and sizes only.  "d_" pointers are device (HBM) pointers, all
 * others are host pointers.  Complex samples are interleaved fp32 (re, im).  Every function
 * returns 0 on success or a negative OFDM_E_* code; ofdm_last_error() describes the last failure
 * on the calling thread.  Nothing here ever calls exit() (contrast OFDM.c:150-153).
 * A context is bound to one GPU; use one context per process/GPU (reentrant per context).
 */
#ifndef OFDM_MI355X_H
#define OFDM_MI355X_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFDM_ABI_VERSION 1

/* ---- error codes ---- */
#define OFDM_OK 0
#define OFDM_E_ARG (-1)     /* invalid argument */
#define OFDM_E_HIP (-2)     /* HIP runtime failure */
#define OFDM_E_NODEV (-3)   /* no usable gfx950 device */
#define OFDM_E_NOMEM (-4)   /* device allocation failed */

/* ---- configuration enums ---- */
#define OFDM_CONV_C 0          /* OFDM.c ifft(): fftshift(IDFT(ifftshift(X)))  (OFDM.c:320-339) */
#define OFDM_CONV_MATLAB 1     /* MATLAB ifft(ifftshift(X))  (IEEE_802_11_a_Code_Tester.m:92-93) */
#define OFDM_PAYLOAD_RANDOM 0  /* Philox i.i.d. bits per data symbol */
#define OFDM_PAYLOAD_MESSAGE 1 /* "Hey! I am Vivaswan" padded to 2 symbols (OFDM.c:20,435-465) */
#define OFDM_PAYLOAD_TESTER 2  /* MATLAB Tester payload (IEEE_802_11_a_Code_Tester.m:50-51) */
#define OFDM_EST_LS 0          /* LTF least-squares channel estimate (OFDM.c:830-850) */
#define OFDM_EST_IDEAL 1       /* perfect channel knowledge (config C2) */
#define OFDM_NOISE_REAL 0      /* real-only AWGN, var sigma^2 -- what OFDM.c:651 actually does (D7) */
#define OFDM_NOISE_COMPLEX 1   /* circular complex AWGN, E|n|^2 = sigma^2 */
#define OFDM_NOISE_NONE 2      /* noiseless (MATLAB Tester, Tester.m:146) */
#define OFDM_CHAN_AWGN 0       /* OFDM.c:635-655 */
#define OFDM_CHAN_RAYLEIGH4 1  /* 4-tap i.i.d. CN(0,1/4) block fading per frame (config C5) */

/* ---- per-SNR counters: int64[OFDM_NCOUNTERS]; all sums are exact integers (shard-invariant) ---- */
#define OFDM_NCOUNTERS 16
#define OFDM_C_FRAMES 0            /* frames (= trials in frame mode) */
#define OFDM_C_SYMBOLS 1           /* data OFDM symbols */
#define OFDM_C_BITS 2              /* payload bits compared */
#define OFDM_C_BIT_ERR 3           /* bit errors (OFDM.c:1154-1161) */
#define OFDM_C_FRAME_ERR 4         /* frames with >= 1 bit error */
#define OFDM_C_SYNC_FAIL 5         /* frame mode: Packet_Selection fell back to 0 (OFDM.c:752) */
#define OFDM_C_EVM_TERMS 6         /* equalised data subcarriers (48 per symbol) */
#define OFDM_C_EVM_PRE_Q 7         /* sum |z - d|^2 before the slicer, fixed point 2^-20, per frame */
#define OFDM_C_EVM_POST_AXIS 8     /* slicer axis errors; sum |s - d|^2 = 2 * this (OFDM.c:1128-1150) */
#define OFDM_C_EVMDB_PRE_Q 9       /* sum over frames of per-frame EVM_dB (OFDM.c:1126), 2^-20 */
#define OFDM_C_EVMDB_POST_Q 10     /* sum over frames with finite post-slicer EVM_dB, 2^-20 */
#define OFDM_C_EVMDB_POST_FINITE 11
#define OFDM_C_OOB 12              /* frame mode: down-sampler ran past the capture (ref reads garbage) */
/* frame mode with ofdm_rx_opts.word_stats = 1: Word_Optimization_Analysis (OFDM.c:38-73) of every
 * trial's RRC-filtered capture, aggregated per SNR point.  NOT sums: extremes over trials. */
#define OFDM_C_WL_MIN_Q 13         /* min over trials of min(Re, Im), fixed point 2^-20 */
#define OFDM_C_WL_MAX_Q 14         /* max over trials of max(Re, Im), fixed point 2^-20 */
#define OFDM_C_WL_BITS 15          /* integer bits for max(|min|, |max|): 1 if < 1, else ceil(log2) + 1 */
#define OFDM_EVM_Q_SCALE 1048576.0 /* 2^20 */

typedef struct {
    uint64_t seed;          /* Philox key; default 0x80211A */
    int32_t conv;           /* OFDM_CONV_* */
    int32_t payload;        /* OFDM_PAYLOAD_* */
    int32_t est;            /* OFDM_EST_* */
    int32_t noise;          /* OFDM_NOISE_* */
    int32_t channel;        /* OFDM_CHAN_* */
    int32_t data_per_frame; /* D, data symbols per frame; must be 2 (OFDM.c:439 gives 2) */
    double kappa;           /* symbol mode: sigma^2 = kappa * p_ref / 10^(snr/10) */
    double p_ref;           /* symbol mode reference power, default 52/4096 */
} ofdm_cfg;

typedef struct {
    int32_t cap_len;        /* capture length: 0 = int(0.307 x waveform length) (OFDM.c:945; 3008 for the
                               reference message) or e.g. 3000 (Tester.m:151) */
    int32_t float_cfo;      /* 1: CFO estimates rounded to float as OFDM.c:798,821 */
    int32_t matlab_slicer;  /* 1: MATLAB zero handling in slicer/demod (Tester.m:338-411) */
    int32_t float_taps;     /* 1: fp32 RRC taps (OFDM.c:32) -- 0: double rcosdesign taps */
    int32_t fixed_start;    /* >=0: capture offset for every trial (Tester.m:152); -1: Philox draw (OFDM.c:949) */
    int32_t word_stats;     /* 1: word-length analysis per trial into OFDM_C_WL_* (frame sweeps) */
    int32_t reserved[2];
} ofdm_rx_opts;

typedef struct ofdm_ctx ofdm_ctx;

/* ---- context / runtime ---- */
int ofdm_abi_version(void);
const char *ofdm_last_error(void);
int ofdm_device_count(int *count);
int ofdm_ctx_create(int device, ofdm_ctx **out);
int ofdm_ctx_destroy(ofdm_ctx *ctx);
/* Enqueue all work of this context on hip_stream from now on (e.g. PyTorch's current stream).
 * NULL selects the HIP null (default) stream.  A new context uses its own non-blocking stream. */
int ofdm_ctx_set_stream(ofdm_ctx *ctx, void *hip_stream);
int ofdm_ctx_synchronize(ofdm_ctx *ctx);
/* Release the context's sweep scratch (Tx batches of ofdm_symbol_sweep, the frame sweep's sync -> symbol
 * hand-off buffer of up to 12 GiB, counters, capture staging) after waiting for the context's streams; the
 * waveform cache and LTF tables stay.  Later calls grow the scratch again on demand.  `released` (optional)
 * receives the bytes freed.  (The reference holds no device memory; its buffers are stack/heap arrays freed
 * when Receiver() returns, OFDM.c:941-1165.) */
int ofdm_ctx_trim(ofdm_ctx *ctx, int64_t *released);
/* bytes of sweep scratch the context holds now (what ofdm_ctx_trim would release) */
int ofdm_ctx_scratch_bytes(ofdm_ctx *ctx, int64_t *bytes);
/* kernel timing: when enabled, every launch of the named kernel is bracketed by HIP events on the
 * launch stream; query returns the summed device time (ms) and launch count since the last reset.
 * kernel ids: 0 = fft64, 1 = tx_symbols, 2 = rx_symbols, 3 = frame_rx */
int ofdm_timing_enable(ofdm_ctx *ctx, int enable);
int ofdm_timing_query(ofdm_ctx *ctx, int kernel, double *ms_total, int64_t *launches);
int ofdm_timing_reset(ofdm_ctx *ctx);

/* ---- K1: batched 64-point transforms on device buffers ----
 * in/out: n transforms of 64 complex fp32, contiguous.  inverse=0: fft() = fftshift(DFT(x))
 * (OFDM.c:314-318).  inverse=1: ifft() in the given convention, 1/64 scaled (OFDM.c:320-339). */
int ofdm_fft64(ofdm_ctx *ctx, const void *d_in, void *d_out, int64_t n, int inverse, int conv);

/* ---- symbol-mode Monte Carlo (the per-symbol chain) ----
 * Tx batch ("Transmitter()", OFDM.c:467-618, for data symbols): frames [first_frame,
 * first_frame + n_frames) with D = 2 data symbols each (symbol s = 2 * frame + d).  Row-major
 * layout: d_tx[n * pitch + s] = sample n (0..79, CP first) as float2, d_bits[k * pitch
 * + s] = payload word k (MSB-first bits, k = 0..2) as uint32, rows k = 3..6 the receivers' demap words
 * (truth signs in FFT sub-block order), rows k = 7..9 the packed receivers' truth words (Hermitian bin
 * pair order), pitch = tx_bytes / (80 * 8).  Buffer sizes:
 * ofdm_tx_bytes(n_frames, &tx_bytes, &bits_bytes); at most 2^23 frames per batch. */
int ofdm_tx_bytes(int64_t n_frames, int64_t *tx_bytes, int64_t *bits_bytes);
int ofdm_tx_frames(ofdm_ctx *ctx, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames,
                   void *d_tx, void *d_bits);
/* Rx pass ("Transmission_Over_Air" + "Receiver" symbol chain, OFDM.c:635-655, 1018-1165) over a Tx
 * batch for n_snr SNR points: ADDS into d_counters (int64 [n_snr][OFDM_NCOUNTERS], device).
 * snr_db is a host array. */
int ofdm_rx_frames(ofdm_ctx *ctx, const ofdm_cfg *cfg, const void *d_tx, const void *d_bits,
                   uint64_t first_frame, int64_t n_frames, const double *snr_db, int n_snr,
                   void *d_counters);
/* Pipelining: the NEXT ofdm_rx_frames / ofdm_rx_frames_dump call on ctx also builds this Tx batch
 * (exactly what ofdm_tx_frames with the same arguments writes).  The packed real-noise receivers build it
 * in their group prologues on the block's otherwise idle waves; any other call launches ofdm_tx_frames on
 * the context's stream first.  The batch must not be the one that call reads.  One batch is pending at a
 * time (a second call replaces it).  An rx call that fails its argument checks leaves the batch pending;
 * ofdm_symbol_sweep builds a pending batch (Tx kernel, context stream) before its own work. */
int ofdm_set_next_tx(ofdm_ctx *ctx, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames,
                     void *d_tx, void *d_bits);
/* Tx + Rx of one batch in one call: writes exactly what ofdm_tx_frames(cfg, first_frame, n_frames, d_tx,
 * d_bits) writes and adds exactly what ofdm_rx_frames on that batch adds.  The packed real-noise receivers
 * build each group's symbols in their group prologue and read them back (one launch); the others launch
 * the Tx kernel first.  A pending ofdm_set_next_tx batch is built as by ofdm_rx_frames. */
int ofdm_txrx_frames(ofdm_ctx *ctx, const ofdm_cfg *cfg, uint64_t first_frame, int64_t n_frames, void *d_tx,
                     void *d_bits, const double *snr_db, int n_snr, void *d_counters);
/* Per-symbol dump for parity tests: equalised data subcarriers d_eq [n_snr][n_frames][2][48] float2
 * and demodulated bits d_dbits [n_snr][n_frames][2][3] uint32 (MSB-first). */
int ofdm_rx_frames_dump(ofdm_ctx *ctx, const ofdm_cfg *cfg, const void *d_tx, const void *d_bits,
                        uint64_t first_frame, int64_t n_frames, const double *snr_db, int n_snr,
                        void *d_counters, void *d_eq, void *d_dbits);
/* Whole sweep ("main()" SNR loop, OFDM.c:1187-1222): Tx + Rx in device-resident chunks of at most
 * chunk_frames frames (0: 2^22, and at least 4 chunks when n_frames >= 2^20); writes host counters
 * [n_snr][OFDM_NCOUNTERS].  Real-noise sweeps on the packed receivers build every batch inside the
 * receivers: chunk 0's its own (ofdm_txrx_frames), chunk k's the batch of chunk k+1 (ofdm_set_next_tx,
 * double-buffered).  The others run the Tx of chunk k+1 on a second stream owned by the context, ordered by
 * events against the context's stream, under the receiver of chunk k.  The counters do not depend on the
 * chunking. */
int ofdm_symbol_sweep(ofdm_ctx *ctx, const ofdm_cfg *cfg, const double *snr_db, int n_snr,
                      uint64_t first_frame, int64_t n_frames, int64_t chunk_frames,
                      int64_t *counters);

/* ---- payload text (SURVEY §8(f) message mode) ----
 * MESSAGE payload = `msg` (default "Hey! I am Vivaswan", OFDM.c:20), MSB-first bytes padded with ' '
 * to ceil(8 len / 96) data symbols per frame (Data_Generator, OFDM.c:435-465); 1 <= len <= 96 (frame
 * mode carries at most 8 data symbols).  Symbol mode uses message symbol s mod frames for data
 * symbol s.  `frames` (optional) receives the data symbols per frame. */
int ofdm_set_message(ofdm_ctx *ctx, const char *msg, int32_t len, int32_t *frames);
/* data symbols per frame of a fixed payload: MESSAGE (current message) or TESTER (2) */
int ofdm_payload_frames(ofdm_ctx *ctx, int payload, int32_t *frames);

/* ---- frame mode: the reference's own trial (preambles, RRC, packet sync, CFO), SURVEY §8 F1-F7 ----
 * "Transmitter()" (OFDM.c:467-618): writes the repeated RRC-filtered frame waveform (host,
 * interleaved, capacity max_complex) and its length 10 (2 (320 + 80 D) + 20) for D data symbols
 * (9800 for the reference message); payload MESSAGE or TESTER. */
int ofdm_transmitter(ofdm_ctx *ctx, int conv, int payload, int float_taps, float *tx_out,
                     int32_t max_complex, int32_t *len_out);
/* "Transmission_Over_Air" (OFDM.c:635-655): real-only AWGN with var mean|tx|^2/10^(snr/10), Philox
 * stream (seed, trial, snr_index); host buffers of len complex samples. */
int ofdm_transmission_over_air(ofdm_ctx *ctx, const float *tx, float *ota, int32_t len, double snr_db,
                               uint64_t seed, uint64_t trial, int32_t snr_index);
/* "Receiver" (OFDM.c:941-1165) on one host capture already offset (cap_len samples; cap_len 0 =
 * int(0.307 x waveform length), OFDM.c:945): returns res3 = {EVM_dB, EVM_AGC_dB, BER},
 * ints4 = {packet_idx, sync_fail, oob, D}, and optionally the demodulated bits (int32 [D*96]) and
 * equalised subcarriers (float2 [D*48]), D = ofdm_payload_frames(payload). */
int ofdm_receiver(ofdm_ctx *ctx, const float *capture, const ofdm_rx_opts *opts, int payload,
                  float *res3, int32_t *ints4, int32_t *bits_out, float *eq_out);
/* "Word_Optimization_Analysis(Rx_filter_signal, len)" (OFDM.c:38-73, called at :967): the RRC
 * matched filter of a capture (full convolution, cap_len + 20 outputs, OFDM.c:962-965), then
 * out3 = {min, max, max |.|} over real and imaginary parts and the integer bits it needs. */
int ofdm_word_length_report(ofdm_ctx *ctx, const float *capture, int32_t cap_len, float *out3, int32_t *bits);
/* Batched frame-mode sweep: n_trials reference trials per SNR point (capture offset + noise from
 * Philox); host counters [n_snr][OFDM_NCOUNTERS]; optional per-trial packet_idx
 * [n_snr][n_trials]. */
int ofdm_frame_sweep(ofdm_ctx *ctx, const ofdm_cfg *cfg, const ofdm_rx_opts *opts,
                     const double *snr_db, int n_snr, uint64_t first_trial, int64_t n_trials,
                     int64_t *counters, int32_t *packet_idx);

#ifdef __cplusplus
}
#endif
#endif
