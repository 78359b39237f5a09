/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product library.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * CPU restatement of the reference iSTFT:
 *   istft_cache ctor  : /root/reference/src/istft.cpp:7-32   (float twiddles, periodic Hann)
 *   irfft             : /root/reference/src/istft.cpp:43-66  (direct DFT synthesis, Im(DC)/Im(Nyq) ignored)
 *   istft             : /root/reference/src/istft.cpp:68-108 (OLA, /sum w^2 where > 1e-8, "same" trim)
 * Parity pinned against the reference istft.cpp compiled in this container
 * (oracle/Makefile target ref -> oracle/_ref/libmioref.so) and against the
 * committed fixtures tests/golden/istft_*.npz made by tests/golden/make_golden.py.
 */
#include "mio_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* istft.cpp:7-32 — same float expressions, same order. */
void mo_istft_tables(int n_fft, int win_length, float *cos_tbl, float *sin_tbl,
                     float *nyq, float *hann) {
    const int n_freq = n_fft / 2 + 1;
    const int n_mid = n_freq - 2 > 0 ? n_freq - 2 : 0;
    const float two_pi_over_n = 2.0f * (float)M_PI / (float)n_fft;
    for (int n = 0; n < n_fft; n++) {
        nyq[n] = (n & 1) ? -1.0f : 1.0f;
        for (int k = 1; k <= n_mid; k++) {
            const float w = two_pi_over_n * (float)k * (float)n;
            const size_t idx = (size_t)n * n_mid + (size_t)(k - 1);
            cos_tbl[idx] = cosf(w);
            sin_tbl[idx] = sinf(w);
        }
    }
    for (int i = 0; i < win_length; i++) {
        hann[i] = 0.5f * (1.0f - cosf(2.0f * (float)M_PI * i / win_length));
    }
}

/* istft.cpp:43-66 */
static void irfft(const float *spec, int n_fft, const float *cos_tbl, const float *sin_tbl,
                  const float *nyq, float *out) {
    const int n_freq = n_fft / 2 + 1;
    const int n_mid = n_freq - 2 > 0 ? n_freq - 2 : 0;
    const float inv_n = 1.0f / (float)n_fft;
    for (int n = 0; n < n_fft; n++) {
        float sum = spec[0];
        sum += spec[(n_freq - 1) * 2] * nyq[n];
        const size_t row = (size_t)n * n_mid;
        for (int k = 1; k <= n_mid; k++) {
            const float re = spec[k * 2 + 0];
            const float im = spec[k * 2 + 1];
            const size_t idx = row + (size_t)(k - 1);
            sum += 2.0f * (re * cos_tbl[idx] - im * sin_tbl[idx]);
        }
        out[n] = sum * inv_n;
    }
}

/* istft.cpp:68-108. Returns the trimmed length written to out (may be 0);
 * out must hold n_frames*hop floats at least. */
int mo_istft(const float *spec, int n_frames, int n_fft, int win_length, int hop_length,
             float *out) {
    const int n_freq = n_fft / 2 + 1;
    const int n_mid = n_freq - 2 > 0 ? n_freq - 2 : 0;
    const int n_pad = (win_length - hop_length) / 2;
    const int n_out = (n_frames - 1) * hop_length + win_length;
    if (n_out <= 0) return 0;

    float *cos_tbl = (float *)malloc(sizeof(float) * (size_t)n_fft * (n_mid ? n_mid : 1));
    float *sin_tbl = (float *)malloc(sizeof(float) * (size_t)n_fft * (n_mid ? n_mid : 1));
    float *nyq = (float *)malloc(sizeof(float) * n_fft);
    float *hann = (float *)malloc(sizeof(float) * win_length);
    float *audio = (float *)calloc((size_t)n_out, sizeof(float));
    float *wsum = (float *)calloc((size_t)n_out, sizeof(float));
    float *tbuf = (float *)malloc(sizeof(float) * n_fft);
    mo_istft_tables(n_fft, win_length, cos_tbl, sin_tbl, nyq, hann);

    for (int t = 0; t < n_frames; t++) {
        irfft(spec + (size_t)t * n_freq * 2, n_fft, cos_tbl, sin_tbl, nyq, tbuf);
        const int offset = t * hop_length;
        for (int j = 0; j < win_length; j++) {
            audio[offset + j] += tbuf[j] * hann[j];
            wsum[offset + j] += hann[j] * hann[j];
        }
    }
    for (int i = 0; i < n_out; i++) {
        if (wsum[i] > 1e-8f) audio[i] /= wsum[i];
    }
    int n_ret = 0;
    const int trim_start = n_pad, trim_end = n_out - n_pad;
    if (trim_end > trim_start) {
        n_ret = trim_end - trim_start;
        memcpy(out, audio + trim_start, sizeof(float) * (size_t)n_ret);
    }
    free(cos_tbl); free(sin_tbl); free(nyq); free(hann);
    free(audio); free(wsum); free(tbuf);
    return n_ret;
}
