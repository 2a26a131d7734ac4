/*
 * ofdm_caller.c -- a C program calling the engine through include/ofdm_mi355x.h only: what the reference's
 * main() (src/OFDM.c:1187-1236) becomes when its three calls go through libofdm_mi355x.so
 * (INTEGRATION.md §2):
 *   float complex* Transmitter(void)                               OFDM.c:467  -> ofdm_transmitter
 *   Transmission_Over_Air(TX_signal, TX_OTA_signal, snr, len)      OFDM.c:635  -> ofdm_transmission_over_air
 *   Receiver(Tx_OTA_signal, len, data_frames_number, Res)          OFDM.c:941  -> ofdm_receiver
 * over the reference's SNR grid 6..40 dB (OFDM.c:1197).  Test infrastructure (tests/test_c_caller.py):
 * gcc compiles it against the header with the struct layout of the ctypes binding asserted
 * (abi_expect.h, generated from ofdm_amd.abi), links it against the library, and on a GPU runs it.
 *
 * usage: ofdm_caller OUT_DIR
 *   OUT_DIR/caller.txt     one line per SNR point: snr rx_start EVM_dB EVM_AGC_dB BER packet_idx sync_fail
 *                          oob D bits[0..96 D) (the reference's Res = {EVM_dB, EVM_AGC_dB, BER}, OFDM.c:1163-1165)
 *   OUT_DIR/capture_I.bin  the capture Receiver() got at SNR point I (interleaved fp32)
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ofdm_mi355x.h"
#include "abi_expect.h"   /* ABI_FIELDS(X): X(type, field, offset) per field, ABI_SIZEOF_<type> */

/* the layout the Python binding (abi.py Cfg / RxOpts) assumes, checked by the C compiler */
#define CHECK_FIELD(T, f, off) _Static_assert(offsetof(T, f) == (off), #T "." #f ": offset differs from the ctypes binding");
ABI_FIELDS(CHECK_FIELD)
_Static_assert(sizeof(ofdm_cfg) == ABI_SIZEOF_ofdm_cfg, "sizeof(ofdm_cfg) differs from the ctypes binding");
_Static_assert(sizeof(ofdm_rx_opts) == ABI_SIZEOF_ofdm_rx_opts, "sizeof(ofdm_rx_opts) differs from the ctypes binding");

/* every entry point the header declares: the link fails if the library does not export one */
typedef void (*entry_fn)(void);
static const volatile entry_fn k_entry_points[] = {   /* volatile: kept at -O2 */
    (entry_fn)ofdm_abi_version,     (entry_fn)ofdm_last_error,        (entry_fn)ofdm_device_count,
    (entry_fn)ofdm_ctx_create,      (entry_fn)ofdm_ctx_destroy,       (entry_fn)ofdm_ctx_set_stream,
    (entry_fn)ofdm_ctx_synchronize, (entry_fn)ofdm_ctx_trim,          (entry_fn)ofdm_ctx_scratch_bytes,
    (entry_fn)ofdm_timing_enable,   (entry_fn)ofdm_timing_query,
    (entry_fn)ofdm_timing_reset,    (entry_fn)ofdm_fft64,             (entry_fn)ofdm_tx_bytes,
    (entry_fn)ofdm_tx_frames,       (entry_fn)ofdm_rx_frames,         (entry_fn)ofdm_set_next_tx,
    (entry_fn)ofdm_txrx_frames,     (entry_fn)ofdm_rx_frames_dump,    (entry_fn)ofdm_symbol_sweep,
    (entry_fn)ofdm_set_message,     (entry_fn)ofdm_payload_frames,    (entry_fn)ofdm_transmitter,
    (entry_fn)ofdm_transmission_over_air, (entry_fn)ofdm_receiver,    (entry_fn)ofdm_word_length_report,
    (entry_fn)ofdm_frame_sweep,
};

#define WAVE_MAX 9800   /* Transmitter() length for the reference message (OFDM.c:607-612) */
#define CAP_LEN 3008    /* int(0.307 x 9800) (OFDM.c:945) */

static int fail(const char *what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, ofdm_last_error());
    return 1;
}

int main(int argc, char **argv) {
    const char *out = argc > 1 ? argv[1] : ".";
    char path[4096];
    if (ofdm_abi_version() != OFDM_ABI_VERSION) return fail("ofdm_abi_version", ofdm_abi_version());
    for (size_t k = 0; k < sizeof k_entry_points / sizeof k_entry_points[0]; ++k)
        if (!k_entry_points[k]) return fail("entry point table", (int)k);
    ofdm_ctx *ctx = NULL;
    int rc = ofdm_ctx_create(0, &ctx);
    if (rc) return fail("ofdm_ctx_create", rc);

    /* Transmitter() (OFDM.c:467): caller-owned buffers instead of a malloc'd return value */
    static float tx[2 * WAVE_MAX], ota[2 * WAVE_MAX];
    int32_t len = 0, nd = 0;
    if ((rc = ofdm_transmitter(ctx, OFDM_CONV_C, OFDM_PAYLOAD_MESSAGE, 1, tx, WAVE_MAX, &len)))
        return fail("ofdm_transmitter", rc);
    if ((rc = ofdm_payload_frames(ctx, OFDM_PAYLOAD_MESSAGE, &nd))) return fail("ofdm_payload_frames", rc);

    snprintf(path, sizeof path, "%s/caller.txt", out);
    FILE *f = fopen(path, "w");
    if (!f) { perror(path); return 1; }
    /* the C receiver: capture int(0.307 len), fp32 CFO, C slicer, fp32 taps, Philox capture offset */
    const ofdm_rx_opts opts = {0, 1, 0, 1, -1, 0, {0, 0}};
    int last_rs = 0;
    float last_res[3] = {0, 0, 0};
    int32_t last_ints[4] = {0, 0, 0, 0};
    for (int i = 0; i < 35; ++i) {                          /* SNR_i = 6 + i (OFDM.c:1197) */
        const double snr = 6.0 + i;
        /* Transmission_Over_Air(tx, ota, snr, len) (OFDM.c:635) */
        if ((rc = ofdm_transmission_over_air(ctx, tx, ota, len, snr, 0x80211A, 0, i)))
            return fail("ofdm_transmission_over_air", rc);
        /* rx_start = rand() % (len - 3008) (OFDM.c:949): any offset; a fixed walk here */
        const int rs = (1234 + 977 * i) % (len - CAP_LEN);
        /* Receiver(ota + rx_start, 3008, frames, Res) (OFDM.c:941) */
        float res[3];
        int32_t ints[4], bits[96 * 8];
        if ((rc = ofdm_receiver(ctx, ota + 2 * rs, &opts, OFDM_PAYLOAD_MESSAGE, res, ints, bits, NULL)))
            return fail("ofdm_receiver", rc);
        fprintf(f, "%.1f %d %.9g %.9g %.9g %d %d %d %d", snr, rs, res[0], res[1], res[2], ints[0], ints[1], ints[2],
                ints[3]);
        for (int b = 0; b < 96 * ints[3]; ++b) fprintf(f, " %d", bits[b]);
        last_rs = rs;
        for (int k = 0; k < 3; ++k) last_res[k] = res[k];
        for (int k = 0; k < 4; ++k) last_ints[k] = ints[k];
        fputc('\n', f);
        snprintf(path, sizeof path, "%s/capture_%d.bin", out, i);
        FILE *c = fopen(path, "wb");
        if (!c || fwrite(ota + 2 * rs, sizeof(float), 2 * CAP_LEN, c) != 2 * CAP_LEN) { perror(path); return 1; }
        fclose(c);
    }
    fclose(f);
    /* the receiver's staging scratch is held by the context until ofdm_ctx_trim releases it */
    int64_t held = 0, released = -1, after = -1;
    if ((rc = ofdm_ctx_scratch_bytes(ctx, &held))) return fail("ofdm_ctx_scratch_bytes", rc);
    if ((rc = ofdm_ctx_trim(ctx, &released))) return fail("ofdm_ctx_trim", rc);
    if ((rc = ofdm_ctx_scratch_bytes(ctx, &after))) return fail("ofdm_ctx_scratch_bytes", rc);
    if (held <= 0 || released != held || after != 0) {
        fprintf(stderr, "ofdm_ctx_trim: held %lld, released %lld, after %lld\n", (long long)held, (long long)released,
                (long long)after);
        return 1;
    }
    /* the context stays usable: the next Receiver() call grows its scratch again and repeats the last result */
    {
        float res[3];
        int32_t ints[4];
        if ((rc = ofdm_receiver(ctx, ota + 2 * last_rs, &opts, OFDM_PAYLOAD_MESSAGE, res, ints, NULL, NULL)))
            return fail("ofdm_receiver after trim", rc);
        if (ints[0] != last_ints[0] || ints[1] != last_ints[1] || res[0] != last_res[0] || res[2] != last_res[2]) {
            fprintf(stderr, "receiver after trim differs from the same call before it\n");
            return 1;
        }
    }
    if ((rc = ofdm_ctx_destroy(ctx))) return fail("ofdm_ctx_destroy", rc);
    return nd == 2 ? 0 : 1;
}
