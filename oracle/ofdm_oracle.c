/*
 * oracle/ofdm_oracle.c -- TEST INFRASTRUCTURE ONLY (see ofdm_oracle.h).
 *
 * CPU restatement, in double precision, of the reference's per-symbol chain and of its frame
 * receiver.  Own code; every block cites the reference lines it restates.  Never linked into,
 * or called by, the product library.
 */
#include "ofdm_oracle.h"
#include <complex.h>
#include <math.h>
#include <string.h>
#include <stdlib.h>
#include <time.h>

typedef double complex cplx;
#define NFFT 64
static const double TWO_PI = 6.283185307179586476925286766559;
static const double PI_D = 3.14159265358979323846;

/* ===================================================================== RNG spec */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0, p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* u1 = fma((float)x, 2^-32, 2^-33) in (0,1]; u2 = (float)x * 2^-32 in revolutions. */
static void bm_pair(uint32_t x1, uint32_t x2, double *za, double *zb)
{
    float u1 = fmaf((float)x1, 0x1p-32f, 0x1p-33f);
    float u2 = (float)x2 * 0x1p-32f;
    double r = sqrt(-2.0 * log((double)u1));
    *za = r * cos(TWO_PI * (double)u2);
    *zb = r * sin(TWO_PI * (double)u2);
}

void orc_gauss4(const uint32_t ctr[4], const uint32_t key[2], double z[4])
{
    uint32_t o[4];
    orc_philox4x32_10(ctr, key, o);
    bm_pair(o[0], o[1], &z[0], &z[1]);
    bm_pair(o[2], o[3], &z[2], &z[3]);
}

#define STREAM_BITS   0xB1750000u
#define STREAM_NOISE  0x5A000000u
#define STREAM_CHAN   0xC4A00000u
#define STREAM_START  0x5B000000u

static void key_of(uint64_t seed, uint32_t key[2]) { key[0] = (uint32_t)seed; key[1] = (uint32_t)(seed >> 32); }

/* Gaussian g of frame f at SNR index q (one block per 4 Gaussians, cached). */
typedef struct { uint64_t f; uint32_t q, blk; int valid; double z[4]; uint32_t key[2]; } gcache;
static double gauss_at(gcache *gc, uint64_t f, uint32_t q, uint32_t g)
{
    uint32_t blk = g >> 2;
    if (!gc->valid || gc->f != f || gc->q != q || gc->blk != blk) {
        uint32_t ctr[4] = { (uint32_t)f, (uint32_t)(f >> 32), blk, STREAM_NOISE | q };
        orc_gauss4(ctr, gc->key, gc->z);
        gc->f = f; gc->q = q; gc->blk = blk; gc->valid = 1;
    }
    return gc->z[g & 3];
}

/* ===================================================================== transforms */
static cplx W64[NFFT];  /* e^{-j 2 pi k / 64} */
static int g_tw_init = 0;
static void tw_init(void)
{
    if (g_tw_init) return;
    for (int k = 0; k < NFFT; ++k) W64[k] = cos(TWO_PI * k / NFFT) - I * sin(TWO_PI * k / NFFT);
    g_tw_init = 1;
}

/* fft() = fft_Cooley then fft_shift (OFDM.c:282-318): out[i] = DFT(x)[(i+32) mod 64] */
static void fft64c(const cplx *x, cplx *y)
{
    tw_init();
    for (int i = 0; i < NFFT; ++i) {
        int k = (i + 32) & 63;
        cplx acc = 0;
        for (int n = 0; n < NFFT; ++n) acc += x[n] * W64[(k * n) & 63];
        y[i] = acc;
    }
}

/* IDFT with 1/64 (OFDM.c:331-334 computes it as conj(fft(conj))/sz) */
static void idft64(const cplx *X, cplx *v)
{
    tw_init();
    for (int n = 0; n < NFFT; ++n) {
        cplx acc = 0;
        for (int m = 0; m < NFFT; ++m) acc += X[m] * conj(W64[(m * n) & 63]);
        v[n] = acc / NFFT;
    }
}

/* C: ifft() = ifft_shift, conj-fft-conj, i.e. fftshift(IDFT(ifftshift(X))) (OFDM.c:320-339, D5).
 * MATLAB: ifft(ifftshift(X)) (IEEE_802_11_a_Code_Tester.m:29,37,92-93). */
static void ifft64c(const cplx *X, cplx *y, int conv)
{
    cplx Xs[NFFT], v[NFFT];
    for (int i = 0; i < NFFT; ++i) Xs[i] = X[(i + 32) & 63];          /* ifft_shift OFDM.c:208-223 */
    idft64(Xs, v);
    if (conv == ORC_CONV_MATLAB) { memcpy(y, v, sizeof(v)); return; }
    for (int i = 0; i < NFFT; ++i) y[(i + 32) & 63] = v[i];           /* fft_shift OFDM.c:227-244 */
}

void orc_fft64(const double *in, double *out) { fft64c((const cplx *)in, (cplx *)out); }
void orc_ifft64(const double *in, double *out, int conv) { ifft64c((const cplx *)in, (cplx *)out, conv); }

/* ===================================================================== transmitter */
/* Data_Generator + Decimal_To_Binary (OFDM.c:401-413, 435-465): MSB first, pad with ' ' */
int orc_message_bits(const unsigned char *msg, int len, int *bits)
{
    int nf = (8 * len + 95) / 96;
    int nchar = nf * 96 / 8;
    for (int c = 0; c < nchar; ++c) {
        int v = c < len ? msg[c] : ' ';
        for (int b = 0; b < 8; ++b) bits[c * 8 + b] = (v >> (7 - b)) & 1;
    }
    return nf;
}

/* IEEE_802_11_a_Code_Tester.m:50-51: eleven 'A' (0x41) bytes then 0x20 -- both payloads equal */
void orc_tester_bits(int *bits192)
{
    for (int f = 0; f < 2; ++f)
        for (int c = 0; c < 12; ++c) {
            int v = c < 11 ? 0x41 : 0x20;
            for (int b = 0; b < 8; ++b) bits192[f * 96 + c * 8 + b] = (v >> (7 - b)) & 1;
        }
}

/* QPSK_Modulator (OFDM.c:415-433): 00->(1+j), 01->(-1+j), 10->(-1-j), 11->(1-j), /sqrt(2) (D10) */
static cplx qpsk(int a, int b)
{
    const double s = 1.0 / sqrt(2.0);
    if (!a && !b) return s + I * s;
    if (!a && b) return -s + I * s;
    if (a && !b) return -s - I * s;
    return s - I * s;
}
void orc_qpsk_map(const int *bits96, double *sym48)
{
    cplx *o = (cplx *)sym48;
    for (int j = 0; j < 48; ++j) o[j] = qpsk(bits96[2 * j], bits96[2 * j + 1]);
}

/* fftshifted data-bin map, Transmitter() OFDM.c:528-547 and Receiver() OFDM.c:1063-1068 */
static const int DATA_BINS[48] = {
    6, 7, 8, 9, 10, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 26, 27, 28, 29, 30, 31,
    33, 34, 35, 36, 37, 38, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 54, 55, 56, 57, 58};

void orc_subcarrier_map(const double *sym48, double *X64)
{
    const cplx *d = (const cplx *)sym48;
    cplx *X = (cplx *)X64;
    for (int i = 0; i < NFFT; ++i) X[i] = 0;
    for (int j = 0; j < 48; ++j) X[DATA_BINS[j]] = d[j];
    X[11] = 1; X[25] = 1; X[39] = 1; X[53] = -1;                 /* pilot[] = {1,1,1,-1} OFDM.c:523 */
}

/* S_k, L_k: IEEE 802.11a preamble tones (OFDM.c:483-494; Tester.m:26,34) */
static void preamble_tones(cplx *S53, double *L53)
{
    static const signed char s_pat[53] = {0,0,1,0,0,0,-1,0,0,0,1,0,0,0,-1,0,0,0,-1,0,0,0,1,0,0,0,0,0,0,0,
                                           -1,0,0,0,-1,0,0,0,1,0,0,0,1,0,0,0,1,0,0,0,1,0,0};
    static const signed char l_pat[53] = {1,1,-1,-1,1,1,-1,1,-1,1,1,1,1,1,1,-1,-1,1,1,-1,1,-1,1,1,1,1,0,
                                           1,-1,-1,1,1,-1,1,-1,1,-1,-1,-1,-1,-1,1,1,-1,-1,1,-1,1,-1,1,1,1,1};
    for (int i = 0; i < 53; ++i) { S53[i] = s_pat[i] * (1.0 + I); L53[i] = l_pat[i]; }
}

/* Preamble_Generator (OFDM.c:368-399): tones at bins 6..58, short = first 16 samples x10,
 * long = [T(32:64), T, T].  The short scale sqrt(13/6) is a float in OFDM.c:479. */
void orc_preambles(int conv, double *stf160, double *ltf160, double *lf64)
{
    cplx S[53]; double L[53];
    preamble_tones(S, L);
    const double sc = (conv == ORC_CONV_C) ? (double)(float)sqrt(13.0 / 6.0) : sqrt(13.0 / 6.0);
    cplx fs[NFFT] = {0}, fl[NFFT] = {0}, ts[NFFT], tl[NFFT];
    for (int i = 0; i < 53; ++i) { fs[6 + i] = S[i] * sc; fl[6 + i] = L[i]; }
    ifft64c(fs, ts, conv);
    ifft64c(fl, tl, conv);
    cplx *s = (cplx *)stf160, *l = (cplx *)ltf160;
    if (s) for (int i = 0; i < 160; ++i) s[i] = ts[i % 16];
    if (l) for (int i = 0; i < 160; ++i) l[i] = tl[(i + 32) & 63];
    if (lf64) memcpy(lf64, fl, sizeof(fl));
}

/* one data OFDM symbol: map + pilots + ifft + CP [x48..63, x0..63] (OFDM.c:526-565) */
void orc_data_symbol(const int *bits96, int conv, double *time80)
{
    double d[96], X[128];
    cplx x[NFFT];
    orc_qpsk_map(bits96, d);
    orc_subcarrier_map(d, X);
    ifft64c((const cplx *)X, x, conv);
    cplx *o = (cplx *)time80;
    for (int i = 0; i < 16; ++i) o[i] = x[48 + i];
    for (int i = 0; i < 64; ++i) o[16 + i] = x[i];
}

/* rcosdesign(0.5, 10, 2, 'sqrt') (Tester.m:112, OFDM.c:32 holds its values, D-F1) */
void orc_rrc_taps(int float_rounded, double *h)
{
    const double beta = 0.5, sps = 2.0;
    double e = 0;
    for (int i = 0; i < 21; ++i) {
        double t = (i - 10) / sps, b;
        if (t == 0) b = -1.0 / (PI_D * sps) * (PI_D * (beta - 1) - 4 * beta);
        else if (fabs(fabs(4 * beta * t) - 1.0) < 1e-12)
            b = 1.0 / (2 * PI_D * sps) * (PI_D * (beta + 1) * sin(PI_D * (beta + 1) / (4 * beta))
                                         - 4 * beta * sin(PI_D * (beta - 1) / (4 * beta))
                                         + PI_D * (beta - 1) * cos(PI_D * (beta - 1) / (4 * beta)));
        else
            b = -4 * beta / sps * (cos((1 + beta) * PI_D * t) + sin((1 - beta) * PI_D * t) / (4 * beta * t))
                / (PI_D * ((4 * beta * t) * (4 * beta * t) - 1));
        h[i] = b; e += b * b;
    }
    for (int i = 0; i < 21; ++i) {
        h[i] /= sqrt(e);
        if (float_rounded) h[i] = (double)(float)h[i];
    }
}

/* Transmitter() frame assembly, 2x zero-stuffing, RRC Convolution, x10 repeat (OFDM.c:569-612) */
int orc_frame_waveform(const int *bits, int nf, int conv, int float_taps, int reps, double *out)
{
    int fsz = 320 + 80 * nf;
    cplx *fr = calloc(fsz, sizeof(cplx));
    orc_preambles(conv, (double *)fr, (double *)(fr + 160), NULL);
    for (int d = 0; d < nf; ++d) orc_data_symbol(bits + 96 * d, conv, (double *)(fr + 320 + 80 * d));
    int nos = 2 * fsz, nout = nos + 20;
    double h[21];
    orc_rrc_taps(float_taps, h);
    cplx *o = (cplx *)out;
    for (int n = 0; n < nout; ++n) {
        cplx acc = 0;
        for (int j = 0; j < 21; ++j) {
            int m = n - j;
            if (m >= 0 && m < nos && !(m & 1)) acc += fr[m >> 1] * h[j];
        }
        o[n] = acc;
    }
    for (int r = 1; r < reps; ++r) memcpy(o + r * nout, o, nout * sizeof(cplx));
    free(fr);
    return nout * reps;
}

/* ===================================================================== receiver (frame mode) */
static int packet_selection(const double *M, int len)
{
    /* Packet_Selection (OFDM.c:685-771; Tester.m:205-248) */
    int *idx = malloc(sizeof(int) * (len + 1));
    int cnt = 0;
    for (int i = 0; i < len; ++i) if (M[i] > 0.75) idx[cnt++] = i;
    int *front = malloc(sizeof(int) * (cnt + 1));
    int nfront = 0;
    for (int i = 0; i <= cnt; ++i) {
        int a = i < cnt ? idx[i] : -1;
        int b = i >= 1 ? idx[i - 1] : -1;
        if (a - b > 300) front[nfront++] = idx[i];
    }
    int p = 0;
    for (int x = 0; x < nfront - 1; ++x)
        if (M[front[x] + 230] > 0.75) { p = front[x] + 10 + 1; break; }   /* len_RRC_rx + 1 */
    free(idx); free(front);
    return p;
}

void orc_receiver_frame(const double *capture, const orc_rx_opts *o, const int *truth_bits, int nf,
                        double *corr, double *rxframe, double *coarse, double *fine, double *Hout,
                        double *Yf, double *nopilot, int *bits_out, orc_rx_info *info)
{
    const cplx *r = (const cplx *)capture;
    const int L = o->cap_len, LF = L + 20;
    const int fsz = 320 + 80 * nf;
    double h[21];
    orc_rrc_taps(o->float_taps, h);

    /* Packet_Detection on the UNFILTERED capture, no conjugate (OFDM.c:659-683) */
    int lc = L - 16 + 1 - 32;
    double *M = malloc(sizeof(double) * lc);
    for (int i = 0; i < lc; ++i) {
        cplx c = 0; double p = 0;
        for (int k = 0; k < 32; ++k) {
            c += r[i + k] * r[i + k + 16];
            double a = cabs(r[i + k + 16]);
            p += a * a;
        }
        double ac = cabs(c);
        M[i] = (ac * ac) / (p * p);
    }
    if (corr) memcpy(corr, M, sizeof(double) * lc);
    int pidx = packet_selection(M, lc);
    free(M);

    /* matched filter (Convolution, OFDM.c:965) evaluated at the down-sampled taps (OFDM.c:992) */
    cplx *fr = calloc(fsz, sizeof(cplx));
    int oob = 0;
    for (int i = 0; i < fsz; ++i) {
        int n = pidx + 2 * i;
        if (n >= LF) { oob = 1; fr[i] = 0; continue; }
        cplx acc = 0;
        for (int j = 0; j < 21; ++j) { int m = n - j; if (m >= 0 && m < L) acc += r[m] * h[j]; }
        fr[i] = acc;
    }
    if (rxframe) memcpy(rxframe, fr, sizeof(cplx) * fsz);

    /* Coarse_CFO_Estimation (OFDM.c:773-804) */
    const double ts = 1.0 / 20e6;
    cplx pc = 0;
    for (int i = 0; i < 16; ++i) pc += fr[80 + i] * conj(fr[96 + i]);
    double fc = (-1.0 / (2 * PI_D * 16 * ts)) * atan2(cimag(pc), creal(pc));
    if (o->float_cfo) fc = (double)(float)fc;
    for (int i = 0; i < fsz; ++i) fr[i] *= cexp(-I * 2 * PI_D * fc * ts * i);
    if (coarse) memcpy(coarse, fr, sizeof(cplx) * fsz);

    /* Fine_CFO_Estimation (OFDM.c:806-828) */
    cplx pf = 0;
    for (int i = 0; i < 64; ++i) pf += fr[192 + i] * conj(fr[256 + i]);
    double ff = (-1.0 / (2 * PI_D * 64 * ts)) * atan2(cimag(pf), creal(pf));
    if (o->float_cfo) ff = (double)(float)ff;
    for (int i = 0; i < fsz; ++i) fr[i] *= cexp(-1.0 * I * 2 * PI_D * ff * ts * i);
    if (fine) memcpy(fine, fr, sizeof(cplx) * fsz);

    /* Channel_Estimation (OFDM.c:830-850): H = 0.5(FFT(L1)+FFT(L2)) conj(Lf) */
    double lf[128];
    orc_preambles(ORC_CONV_C, NULL, NULL, lf);     /* Lf does not depend on the convention */
    const cplx *Lf = (const cplx *)lf;
    cplx F1[NFFT], F2[NFFT], H[NFFT];
    fft64c(fr + 192, F1);
    fft64c(fr + 256, F2);
    for (int k = 0; k < NFFT; ++k) H[k] = 0.5 * (F1[k] + F2[k]) * conj(Lf[k]);
    if (Hout) memcpy(Hout, H, sizeof(H));

    double epre = 0, epost = 0, dsum = 0;
    int nerr = 0;
    const double s2 = 1.0 / sqrt(2.0);
    for (int d = 0; d < nf; ++d) {
        cplx Y[NFFT];
        fft64c(fr + 320 + 80 * d + 16, Y);                 /* CP strip + fft (OFDM.c:1024-1040) */
        if (Yf) memcpy(Yf + 128 * d, Y, sizeof(Y));
        cplx ref48[48];
        orc_qpsk_map(truth_bits + 96 * d, (double *)ref48);
        for (int j = 0; j < 48; ++j) {
            int k = DATA_BINS[j];
            cplx z = Y[k] / H[k];                          /* one-tap ZF (OFDM.c:1044-1052) */
            if (nopilot) { nopilot[(48 * d + j) * 2] = creal(z); nopilot[(48 * d + j) * 2 + 1] = cimag(z); }
            /* AGC_Receiver slicer (OFDM.c:852-871; MATLAB: zero stays zero, Tester.m:338-349) */
            double sr, si;
            if (o->matlab_slicer) {
                sr = creal(z) > 0 ? s2 : (creal(z) < 0 ? -s2 : 0);
                si = cimag(z) > 0 ? s2 : (cimag(z) < 0 ? -s2 : 0);
            } else {
                sr = creal(z) > 0 ? s2 : -s2;
                si = cimag(z) > 0 ? s2 : -s2;
            }
            /* QPSK_Demodulator (OFDM.c:873-908; MATLAB leaves [0 0] if no branch matches) */
            int c = 1, e = 1;
            if (sr > 0 && si > 0) { c = 0; e = 0; }
            else if (sr < 0 && si > 0) { c = 0; e = 1; }
            else if (sr < 0 && si < 0) { c = 1; e = 0; }
            else if (sr > 0 && si < 0) { c = 1; e = 1; }
            else if (o->matlab_slicer) { c = 0; e = 0; }
            if (bits_out) { bits_out[96 * d + 2 * j] = c; bits_out[96 * d + 2 * j + 1] = e; }
            nerr += (c != truth_bits[96 * d + 2 * j]) + (e != truth_bits[96 * d + 2 * j + 1]);
            double ae = cabs(z - ref48[j]);
            epre += ae * ae;
            double ap = cabs((sr + I * si) - ref48[j]);
            epost += ap * ap;
            double ad = cabs(ref48[j]);
            dsum += ad * ad;
        }
    }
    free(fr);
    if (info) {
        info->packet_idx = pidx;
        info->len_corr = lc;
        info->sync_fail = (pidx == 0);
        info->oob = oob;
        int N = nf * 48;
        info->res[0] = 20 * log10(sqrt(epre / N) / sqrt(dsum / N));  /* OFDM.c:1124-1126 */
        info->res[1] = 20 * log10(sqrt(epost / N) / sqrt(dsum / N)); /* OFDM.c:1148-1150 */
        info->res[2] = (double)nerr / (nf * 96);                     /* OFDM.c:1154-1161 */
        info->cfo[0] = fc; info->cfo[1] = ff;
    }
}

/* ===================================================================== Monte-Carlo twins */
/* MESSAGE payload text: OFDM.c:20 by default, orc_set_message for message-mode tests */
static unsigned char g_msg[97] = "Hey! I am Vivaswan";
static int g_msg_len = 18;

int orc_set_message(const unsigned char *msg, int len)
{
    if (len < 1 || len > 96) return -1;
    memcpy(g_msg, msg, (size_t)len);
    g_msg_len = len;
    return (8 * len + 95) / 96;
}

/* bits of the fixed payloads: returns the data symbols per frame */
static int fixed_payload_bits(int payload, int *bits)
{
    if (payload == ORC_PAYLOAD_TESTER) { orc_tester_bits(bits); return 2; }
    return orc_message_bits(g_msg, g_msg_len, bits);
}

static void payload_bits(const orc_cfg *cfg, uint64_t s, int *bits96)
{
    if (cfg->payload == ORC_PAYLOAD_RANDOM) {
        uint32_t key[2], o[4];
        key_of(cfg->seed, key);
        uint32_t ctr[4] = { (uint32_t)s, (uint32_t)(s >> 32), 0, STREAM_BITS };
        orc_philox4x32_10(ctr, key, o);
        for (int b = 0; b < 96; ++b) bits96[b] = (o[b >> 5] >> (31 - (b & 31))) & 1;
    } else {
        int all[96 * 8];
        const int nf = fixed_payload_bits(cfg->payload, all);   /* data symbol s carries message symbol s mod nf */
        memcpy(bits96, all + 96 * (int)(s % (uint64_t)nf), sizeof(int) * 96);
    }
}

static void channel_taps(const orc_cfg *cfg, uint64_t f, cplx h[4])
{
    if (cfg->channel != ORC_CHAN_RAYLEIGH4) { h[0] = 1; h[1] = h[2] = h[3] = 0; return; }
    uint32_t key[2];
    key_of(cfg->seed, key);
    double z[8];
    for (uint32_t b = 0; b < 2; ++b) {
        uint32_t ctr[4] = { (uint32_t)f, (uint32_t)(f >> 32), b, STREAM_CHAN };
        orc_gauss4(ctr, key, z + 4 * b);
    }
    const double a = sqrt(1.0 / 8.0);      /* CN(0, 1/4) per tap */
    for (int l = 0; l < 4; ++l) h[l] = a * (z[2 * l] + I * z[2 * l + 1]);
}

static inline int64_t q20(double v) { return (int64_t)llrint(v * 1048576.0); }

void orc_symbol_sweep(const orc_cfg *cfg, const double *snr_db, int n_snr,
                      uint64_t first_frame, uint64_t n_frames, int64_t *counters,
                      double *dump_eq, int *dump_bits)
{
    const int D = 2;
    double lf[128], ltf[320];
    orc_preambles(cfg->conv, NULL, ltf, lf);
    const cplx *Lf = (const cplx *)lf, *LP = (const cplx *)ltf;
    const double s2 = 1.0 / sqrt(2.0);
    gcache gc; memset(&gc, 0, sizeof(gc)); key_of(cfg->seed, gc.key);

    for (int q = 0; q < n_snr; ++q) {
        int64_t *C = counters + (size_t)q * ORC_NCOUNTERS;
        memset(C, 0, sizeof(int64_t) * ORC_NCOUNTERS);
        const float sigma = (float)sqrt(cfg->kappa * cfg->p_ref / pow(10.0, snr_db[q] / 10.0));
        for (uint64_t fi = 0; fi < n_frames; ++fi) {
            const uint64_t f = first_frame + fi;
            /* clean frame timeline: [0,160) STF (unused), [160,320) LTF, data at 320+80d */
            cplx x[320 + 80 * 2];
            int bits[2][96];
            memset(x, 0, sizeof(x));
            for (int k = 0; k < 160; ++k) x[160 + k] = LP[k];
            for (int d = 0; d < D; ++d) {
                payload_bits(cfg, f * D + d, bits[d]);
                orc_data_symbol(bits[d], cfg->conv, (double *)(x + 320 + 80 * d));
            }
            cplx h[4];
            channel_taps(cfg, f, h);
            /* received sample t = sum_l h_l x[t-l] + noise(t)  (channel + AWGN, OFDM.c:635-655) */
            #define RX_AT(t, out) do { \
                cplx acc_ = 0; \
                for (int l_ = 0; l_ < 4; ++l_) if ((t) - l_ >= 0) acc_ += h[l_] * x[(t) - l_]; \
                if (cfg->noise == ORC_NOISE_REAL) acc_ += sigma * gauss_at(&gc, f, q, (uint32_t)(t)); \
                else if (cfg->noise == ORC_NOISE_COMPLEX) \
                    acc_ += (sigma * s2) * (gauss_at(&gc, f, q, 2u * (t)) + I * gauss_at(&gc, f, q, 2u * (t) + 1)); \
                (out) = acc_; } while (0)

            cplx H[NFFT];
            if (cfg->est == ORC_EST_LS) {
                /* H = 0.5 (F1 + F2) conj(Lf) (OFDM.c:830-850) = 0.5 FFT(r1 + r2) conj(Lf).  The LTF
                 * windows [192,256) and [256,320) carry the same clean samples (cyclic T, the channel
                 * reaches back into T's tail either way), so r1 + r2 = 2 clean(192 + n) + (n1 + n2);
                 * symbol mode draws the pair noise n1 + n2 once: sqrt(2) x the LTF1-slot Gaussians
                 * (identical law). */
                cplx e[NFFT], E[NFFT];
                for (int n = 0; n < NFFT; ++n) {
                    const int t = 192 + n;
                    cplx acc = 0;
                    for (int l = 0; l < 4; ++l) acc += h[l] * x[t - l];
                    acc *= 2.0;
                    if (cfg->noise == ORC_NOISE_REAL) acc += M_SQRT2 * sigma * gauss_at(&gc, f, q, (uint32_t)t);
                    else if (cfg->noise == ORC_NOISE_COMPLEX)
                        acc += sigma * (gauss_at(&gc, f, q, 2u * t) + I * gauss_at(&gc, f, q, 2u * t + 1));
                    e[n] = acc;
                }
                fft64c(e, E);
                for (int k = 0; k < NFFT; ++k) H[k] = 0.5 * E[k] * conj(Lf[k]);
            } else {
                /* perfect channel knowledge: H[i] = c_i sum_l h_l e^{-j2pi(i-32)l/64},
                 * c_i = (-1)^i for the C ifft convention (D5), 1 for MATLAB */
                for (int i = 0; i < NFFT; ++i) {
                    cplx acc = 0;
                    for (int l = 0; l < 4; ++l) acc += h[l] * cexp(-I * TWO_PI * (i - 32) * l / NFFT);
                    H[i] = (cfg->conv == ORC_CONV_C && (i & 1)) ? -acc : acc;
                }
            }
            double fe_pre = 0; int64_t fe_axis = 0, ferr = 0;
            for (int d = 0; d < D; ++d) {
                cplx y[NFFT], Y[NFFT], ref48[48];
                for (int n = 0; n < NFFT; ++n) RX_AT(336 + 80 * d + n, y[n]);
                fft64c(y, Y);
                orc_qpsk_map(bits[d], (double *)ref48);
                for (int j = 0; j < 48; ++j) {
                    int k = DATA_BINS[j];
                    cplx z = Y[k] / H[k];
                    size_t di = (((size_t)q * n_frames + fi) * D + d) * 48 + j;
                    if (dump_eq) { dump_eq[2 * di] = creal(z); dump_eq[2 * di + 1] = cimag(z); }
                    int pr = creal(z) > 0, pi = cimag(z) > 0;
                    int b0 = !pi, b1 = (pr != pi);                  /* OFDM.c:860-905 */
                    if (dump_bits) {
                        size_t bi = (((size_t)q * n_frames + fi) * D + d) * 96 + 2 * j;
                        dump_bits[bi] = b0; dump_bits[bi + 1] = b1;
                    }
                    ferr += (b0 != bits[d][2 * j]) + (b1 != bits[d][2 * j + 1]);
                    double ae = cabs(z - ref48[j]);
                    fe_pre += ae * ae;
                    fe_axis += (pr != (creal(ref48[j]) > 0)) + (pi != (cimag(ref48[j]) > 0));
                }
            }
            #undef RX_AT
            const double N = 48.0 * D;
            C[ORC_C_FRAMES] += 1;
            C[ORC_C_SYMBOLS] += D;
            C[ORC_C_BITS] += 96 * D;
            C[ORC_C_BIT_ERR] += ferr;
            C[ORC_C_FRAME_ERR] += ferr > 0;
            C[ORC_C_EVM_TERMS] += 48 * D;
            C[ORC_C_EVM_PRE_Q] += q20(fe_pre);
            C[ORC_C_EVM_POST_AXIS] += fe_axis;
            C[ORC_C_EVMDB_PRE_Q] += q20(10.0 * log10(fe_pre / N));
            if (fe_axis > 0) {
                C[ORC_C_EVMDB_POST_Q] += q20(10.0 * log10(2.0 * fe_axis / N));
                C[ORC_C_EVMDB_POST_FINITE] += 1;
            }
        }
    }
}

void orc_frame_sweep(const orc_cfg *cfg, const orc_rx_opts *o, const double *snr_db, int n_snr,
                     uint64_t first_trial, uint64_t n_trials, int64_t *counters, int *dump_pidx)
{
    int bits[96 * 8];
    const int nf = fixed_payload_bits(cfg->payload, bits), reps = 10;
    const int len = (2 * (320 + 80 * nf) + 20) * reps;
    double *wf = malloc(sizeof(double) * 2 * len);
    orc_frame_waveform(bits, nf, cfg->conv, o->float_taps, reps, wf);
    /* the HIP path streams the fp32 waveform; use the same samples */
    for (int i = 0; i < 2 * len; ++i) wf[i] = (double)(float)wf[i];
    double P = 0;
    for (int i = 0; i < len; ++i) P += wf[2 * i] * wf[2 * i] + wf[2 * i + 1] * wf[2 * i + 1];
    P /= len;                                                   /* OFDM.c:637-643 */
    uint32_t key[2];
    key_of(cfg->seed, key);
    gcache gc; memset(&gc, 0, sizeof(gc)); memcpy(gc.key, key, sizeof(key));
    const int L = o->cap_len;
    double *cap = malloc(sizeof(double) * 2 * L);
    for (int q = 0; q < n_snr; ++q) {
        int64_t *C = counters + (size_t)q * ORC_NCOUNTERS;
        memset(C, 0, sizeof(int64_t) * ORC_NCOUNTERS);
        const float sigma = (float)sqrt(P / pow(10.0, snr_db[q] / 10.0));     /* OFDM.c:645-651 */
        for (uint64_t ti = 0; ti < n_trials; ++ti) {
            uint64_t t = first_trial + ti;
            uint32_t ctr[4] = { (uint32_t)t, (uint32_t)(t >> 32), 0, STREAM_START | (uint32_t)q }, ro[4];
            orc_philox4x32_10(ctr, key, ro);
            int rx_start = (int)(ro[0] % (uint32_t)(len - L));          /* OFDM.c:949 */
            for (int n = 0; n < L; ++n) {
                int k = rx_start + n;
                double nz = (cfg->noise == ORC_NOISE_NONE) ? 0.0 : sigma * gauss_at(&gc, t, q, (uint32_t)k);
                cap[2 * n] = wf[2 * k] + nz;                             /* real-only noise (D7) */
                cap[2 * n + 1] = wf[2 * k + 1];
            }
            orc_rx_info info;
            int rb[96 * 8];
            orc_receiver_frame(cap, o, bits, nf, NULL, NULL, NULL, NULL, NULL, NULL, NULL, rb, &info);
            if (dump_pidx) dump_pidx[(size_t)q * n_trials + ti] = info.packet_idx;
            int ferr = 0;
            for (int b = 0; b < 96 * nf; ++b) ferr += rb[b] != bits[b];
            C[ORC_C_FRAMES] += 1;
            C[ORC_C_SYMBOLS] += nf;
            C[ORC_C_BITS] += 96 * nf;
            C[ORC_C_BIT_ERR] += ferr;
            C[ORC_C_FRAME_ERR] += ferr > 0;
            C[ORC_C_SYNC_FAIL] += info.sync_fail;
            C[ORC_C_OOB] += info.oob;
            C[ORC_C_EVM_TERMS] += 48 * nf;
            double N = 48.0 * nf;
            double epre = pow(10.0, info.res[0] / 10.0) * N;
            C[ORC_C_EVM_PRE_Q] += q20(epre);
            C[ORC_C_EVMDB_PRE_Q] += q20(info.res[0]);
            if (isfinite(info.res[1])) {
                double epost = pow(10.0, info.res[1] / 10.0) * N;
                C[ORC_C_EVM_POST_AXIS] += llrint(epost / 2.0);
                C[ORC_C_EVMDB_POST_Q] += q20(info.res[1]);
                C[ORC_C_EVMDB_POST_FINITE] += 1;
            }
        }
    }
    free(cap); free(wf);
}

double orc_time_symbol_sweep(const orc_cfg *cfg, const double *snr_db, int n_snr,
                             uint64_t n_frames, int64_t *counters)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    orc_symbol_sweep(cfg, snr_db, n_snr, 0, n_frames, counters, NULL, NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* Word_Optimization_Analysis (OFDM.c:38-73) of Convolution(capture, RRC) (OFDM.c:342-364, 962-967):
 * min / max over the real and imaginary parts of all n + 20 outputs, max |.|, integer bits. */
int orc_word_length(const double *capture, int n, int float_taps, double *min_max_abs3)
{
    double h[21];
    orc_rrc_taps(float_taps, h);
    const cplx *x = (const cplx *)capture;
    double mn = 1e9, mx = -1e9;
    for (int k = 0; k < n + 20; ++k) {
        cplx acc = 0;
        for (int j = 0; j < 21; ++j) if (k - j >= 0 && k - j < n) acc += x[k - j] * h[j];
        if (creal(acc) < mn) mn = creal(acc);
        if (creal(acc) > mx) mx = creal(acc);
        if (cimag(acc) < mn) mn = cimag(acc);
        if (cimag(acc) > mx) mx = cimag(acc);
    }
    const double ma = fmax(fabs(mn), fabs(mx));
    min_max_abs3[0] = mn; min_max_abs3[1] = mx; min_max_abs3[2] = ma;
    return ma < 1.0 ? 1 : (int)ceil(log2(ma)) + 1;
}
