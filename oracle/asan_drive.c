/*
 * oracle/asan_drive.c -- TEST INFRASTRUCTURE ONLY: drives the oracle (default) or the reference harness
 * (-DDRIVE_REF, linked with ref_harness.c) through every entry point the tests use, small sizes, so that an
 * AddressSanitizer / UBSan / LeakSanitizer build reports on them from a plain C process (no Python allocator in
 * the leak report).  SURVEY §5 "host side under ASan/UBSan"; run by tools/sanitize.py (make -C oracle asan).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#ifndef DRIVE_REF
#include "ofdm_oracle.h"

int main(void)
{
    double x[128], y[128];
    for (int i = 0; i < 128; ++i) x[i] = (double)((i * 37) % 11) - 5.0;
    orc_fft64(x, y);
    orc_ifft64(y, x, ORC_CONV_C);
    orc_ifft64(y, x, ORC_CONV_MATLAB);

    const double snr[3] = {0.0, 10.0, 30.0};
    int64_t cnt[3 * ORC_NCOUNTERS];
    const int nfr = 12;
    double *eq = malloc(sizeof(double) * 3 * nfr * 2 * 48 * 2);
    int *bits = malloc(sizeof(int) * 3 * nfr * 2 * 96);
    /* every configuration the GPU sweeps run (est x noise x channel x conv x payload) */
    for (int est = 0; est < 2; ++est)
        for (int noise = 0; noise < 3; ++noise)
            for (int chan = 0; chan < 2; ++chan)
                for (int conv = 0; conv < 2; ++conv)
                    for (int pay = 0; pay < 3; ++pay) {
                        orc_cfg c = {0x80211AULL, conv, pay, est, noise, chan, 2, 0.4980, 52.0 / 4096.0};
                        memset(cnt, 0, sizeof cnt);
                        orc_symbol_sweep(&c, snr, 3, 7, nfr, cnt, (est + noise + chan) & 1 ? eq : NULL,
                                         (est + noise + chan) & 1 ? bits : NULL);
                    }
    free(eq);
    free(bits);

    /* frame mode: the reference message's waveform, sync + CFO + LS receiver over Philox captures */
    const unsigned char msg[] = "Hello MI355X OFDM QPSK 802.11a!";
    orc_set_message(msg, (int)sizeof msg - 1);
    for (int mode = 0; mode < 2; ++mode) {
        orc_cfg c = {0x80211AULL, mode, ORC_PAYLOAD_MESSAGE, ORC_EST_LS, ORC_NOISE_REAL, ORC_CHAN_AWGN, 2, 0.4980,
                     52.0 / 4096.0};
        orc_rx_opts o = {mode ? 3000 : 3008, !mode, mode, !mode};
        int pidx[3 * 6];
        memset(cnt, 0, sizeof cnt);
        orc_frame_sweep(&c, &o, snr, 3, 0, 6, cnt, pidx);
    }
    int wbits[96 * 8];                                    // up to 8 frames (96-character messages)
    int nf = orc_message_bits(msg, (int)sizeof msg - 1, wbits);
    double *wave = calloc((size_t)2 * (2 * (320 + 80 * nf) + 20) * 10, sizeof(double));
    int n = orc_frame_waveform(wbits, nf, ORC_CONV_C, 1, 10, wave);
    double mm[3];
    orc_word_length(wave, n < 3000 ? n : 3000, 1, mm);
    free(wave);
    printf("drive_oracle done\n");
    return 0;
}

#else
/* the reference harness's entry points (oracle/ref_harness.c) */
int ref_init(void);
int ref_tx_copy(float *out, int max_complex);
void ref_globals(float *bits, float *payload_mod, float *ltf_freq, int *dims);
void ref_fft(const float *in, float *out, int n);
void ref_ifft(const float *in, float *out, int n);
double ref_time_fft(const float *in, int n_vectors, int n_transforms, int inverse, double *check);
void ref_convolution(const float *in, int n, float *out);
void ref_trial(float snr_db, float *res3);
double ref_mc_trials(float snr_db, int n_trials, double *acc8);
void ref_receiver_stages(const float *ota_in, int len_Tx_Signal, int rx_start, float *corr, float *rxf,
                         float *coarse, float *fine, float *H, float *Yf, float *nopilot, float *bits, float *res3,
                         int *ints);
void ref_channel_estimation(const float *frame480, float *H64);
void ref_gaussian_noise(int n, float *out);
double ref_time_symbol_chain(const float *snr_db, int n_snr, int n_frames, int flags, double *acc3);
void ref_toa(const float *tx, float *out, float snr_db, int len);

int main(void)
{
    int n = ref_init();
    float *tx = malloc(sizeof(float) * 2 * (size_t)n), *ota = malloc(sizeof(float) * 2 * (size_t)n);
    ref_tx_copy(tx, n);
    float bits[192], pm[192], lf[128];
    int dims[3];
    ref_globals(bits, pm, lf, dims);
    float a[128], b[128], chk_in[128 * 4];
    for (int i = 0; i < 128; ++i) a[i] = (float)((i * 13) % 7) - 3.0f;
    for (int i = 0; i < 128 * 4; ++i) chk_in[i] = (float)(i % 5);
    ref_fft(a, b, 64);
    ref_ifft(b, a, 64);
    double chk;
    ref_time_fft(chk_in, 4, 16, 0, &chk);
    ref_time_fft(chk_in, 4, 16, 1, &chk);
    float *conv = malloc(sizeof(float) * 2 * (size_t)(n + 20));
    ref_convolution(tx, n / 4, conv);
    free(conv);
    float res[3];
    ref_trial(10.0f, res);
    double acc8[8];
    ref_mc_trials(6.0f, 3, acc8);
    ref_toa(tx, ota, 20.0f, n);
    /* the stage-by-stage receiver at an in-range capture offset */
    const int len_rx = (int)(n * 0.307);
    float *corr = malloc(sizeof(float) * (size_t)len_rx), fr[960], co[960], fi[960], H[128], Yf[256], np_[192],
          db[192];
    int ints[4];
    ref_receiver_stages(ota, n, 1000, corr, fr, co, fi, H, Yf, np_, db, res, ints);
    free(corr);
    ref_channel_estimation(fr, H);
    float g[64];
    ref_gaussian_noise(64, g);
    const float snr[2] = {0.0f, 12.0f};
    double acc5[5] = {0, 0, 0, 0, 0};
    for (int flags = 0; flags < 8; ++flags) ref_time_symbol_chain(snr, 2, 3, flags, acc5);
    free(tx);
    free(ota);
    printf("drive_ref done\n");
    return 0;
}
#endif
