/*
 * oracle/ofdm_oracle.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference hot path.
 *
 * This is NOT product code.  It is the checker the HIP path is compared against (tests/,
 * __graft_entry__.smoke(), and bench.py's cpu_baseline "port" leg are its only users).  It is
 * our own restatement, in double precision, of the algorithm in /root/reference/src/OFDM.c
 * and "MATLAB Reference/IEEE_802_11_a_Code_Tester.m"; each function cites the lines it follows.
 *
 * Parity of this oracle is pinned (tests/test_oracle.py) against
 *   - the compiled reference itself (oracle/_ref/libofdm_ref.so, built from the unmodified
 *     OFDM.c) -> committed fixtures in tests/golden/ (FFT vectors, Tx waveform, per-stage
 *     receiver dumps with injected noise), and
 *   - data/Matlab_Output.txt (the MATLAB Tester known-answer vector, 96 bits).
 *
 * Complex arrays are interleaved (re, im) doubles.  The Monte-Carlo spec (Philox streams,
 * counter layout, frame timeline) is the one in DESIGN.md §3 and is shared with the HIP path.
 */
#ifndef OFDM_ORACLE_H
#define OFDM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_CONV_C = 0, ORC_CONV_MATLAB = 1 };
enum { ORC_PAYLOAD_RANDOM = 0, ORC_PAYLOAD_MESSAGE = 1, ORC_PAYLOAD_TESTER = 2 };
enum { ORC_EST_LS = 0, ORC_EST_IDEAL = 1 };
enum { ORC_NOISE_REAL = 0, ORC_NOISE_COMPLEX = 1, ORC_NOISE_NONE = 2 };
enum { ORC_CHAN_AWGN = 0, ORC_CHAN_RAYLEIGH4 = 1 };

/* counters per SNR point (int64 x 16); layout identical to include/ofdm_mi355x.h */
enum {
    ORC_C_FRAMES = 0, ORC_C_SYMBOLS, ORC_C_BITS, ORC_C_BIT_ERR, ORC_C_FRAME_ERR, ORC_C_SYNC_FAIL,
    ORC_C_EVM_TERMS, ORC_C_EVM_PRE_Q, ORC_C_EVM_POST_AXIS, ORC_C_EVMDB_PRE_Q, ORC_C_EVMDB_POST_Q,
    ORC_C_EVMDB_POST_FINITE, ORC_C_OOB, ORC_C_RSV13, ORC_C_RSV14, ORC_C_RSV15, ORC_NCOUNTERS
};

typedef struct {
    uint64_t seed;
    int conv;      /* ORC_CONV_* : Tx IFFT convention (D5) */
    int payload;   /* ORC_PAYLOAD_* */
    int est;       /* ORC_EST_* */
    int noise;     /* ORC_NOISE_* */
    int channel;   /* ORC_CHAN_* */
    int data_per_frame; /* D, must be 2 */
    double kappa;  /* sigma^2 = kappa * p_ref / 10^(snr/10) */
    double p_ref;
} orc_cfg;

/* ---- RNG spec ---- */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* four standard normals of one Philox block; u1/u2 quantised exactly as the HIP path */
void orc_gauss4(const uint32_t ctr[4], const uint32_t key[2], double z[4]);

/* ---- transforms: OFDM.c:314-339 ---- */
void orc_fft64(const double *in, double *out);              /* fft(): fftshift(DFT(x)) */
void orc_ifft64(const double *in, double *out, int conv);   /* ifft() (C) / ifft(ifftshift()) (MATLAB) */

/* ---- transmitter primitives ---- */
int  orc_message_bits(const unsigned char *msg, int len, int *bits_out);  /* returns frames */
int  orc_set_message(const unsigned char *msg, int len);   /* MESSAGE payload text; returns frames */
void orc_tester_bits(int *bits192);                                       /* Tester.m:50-51 */
void orc_qpsk_map(const int *bits96, double *sym48);                      /* OFDM.c:415-433 */
void orc_subcarrier_map(const double *sym48, double *X64);                /* OFDM.c:523-548 */
void orc_preambles(int conv, double *stf160, double *ltf160, double *lf64);
void orc_data_symbol(const int *bits96, int conv, double *time80);        /* map+ifft+CP */
void orc_rrc_taps(int float_rounded, double *h21);                        /* OFDM.c:32 */
int  orc_word_length(const double *capture, int n, int float_taps, double *min_max_abs3);  /* OFDM.c:38-73 */
/* whole reference waveform: preambles + nf data symbols, 2x zero-stuff, RRC, x reps */
int  orc_frame_waveform(const int *bits, int nf, int conv, int float_taps, int reps, double *out);

/* ---- receiver restatement (frame mode, OFDM.c:941-1165 / Tester.m:150-469) ---- */
typedef struct {
    int cap_len;        /* 3008 (C: floor(0.307*len)) or 3000 (Tester) */
    int float_cfo;      /* 1: round CFO estimates to float as OFDM.c:798,821 do */
    int matlab_slicer;  /* 1: MATLAB zero handling in slicer/demod (Tester.m:338-411) */
    int float_taps;     /* 1: float-rounded RRC taps (OFDM.c:32) */
} orc_rx_opts;

typedef struct {
    int packet_idx, len_corr, sync_fail, oob;
    double res[3];      /* EVM_dB pre, EVM_dB post, BER (OFDM.c:1163-1165) */
    double cfo[2];
} orc_rx_info;

/* capture = caller-provided samples (already offset), all dumps optional (NULL) */
void orc_receiver_frame(const double *capture, const orc_rx_opts *o, const int *truth_bits, int nf,
                        double *corr, double *rxframe, double *coarse, double *fine, double *H,
                        double *Yf, double *nopilot, int *bits_out, orc_rx_info *info);

/* ---- Monte-Carlo twins of the HIP sweeps (small sizes only) ---- */
void orc_symbol_sweep(const orc_cfg *cfg, const double *snr_db, int n_snr,
                      uint64_t first_frame, uint64_t n_frames, int64_t *counters,
                      double *dump_eq /* [n_snr][n_frames][D][48][2] or NULL */,
                      int *dump_bits  /* [n_snr][n_frames][D][96] or NULL */);

/* frame mode with Philox capture offsets + noise over a fixed-payload reference waveform */
void orc_frame_sweep(const orc_cfg *cfg, const orc_rx_opts *o, const double *snr_db, int n_snr,
                     uint64_t first_trial, uint64_t n_trials, int64_t *counters,
                     int *dump_packet_idx /* [n_snr][n_trials] or NULL */);

/* timing helper for the CPU baseline: returns seconds for one symbol sweep */
double orc_time_symbol_sweep(const orc_cfg *cfg, const double *snr_db, int n_snr,
                             uint64_t n_frames, int64_t *counters);

#ifdef __cplusplus
}
#endif
#endif
