/* stream_ref.c — TEST INFRASTRUCTURE ONLY (oracle/; never linked by the product).
 *
 * C restatement of what TestToSpeech::synthesize_stream_profiled emits through its callback
 * (reference src/test-to-speech.cpp):
 *   - check cadence :496, :597-602   every `check_interval` generated tokens, plus a final
 *                                    check after generation (:606-608);
 *   - maybe_emit :503-571            target = all codes (final) or all but `holdback`; nothing
 *                                    unless target > committed and (final or the step is at
 *                                    least `min_commit` codes); a full re-decode of every
 *                                    code so far without peak normalisation (:534-544,
 *                                    decode_codes_to_audio :248-300); committed positions
 *                                    mapped to samples with llround(codes * len/n) (:555-563);
 *   - emit_range :367-417            chunk_samples pieces; the first piece of every call is
 *                                    crossfaded with the last min(30 ms, 4096) samples kept
 *                                    from the previous piece (weights (j+1)/(xf+1)); the tail
 *                                    is refreshed after every piece.
 * Speech-only generation (the harness of the GPU tests): every generated token is one code,
 * so the check after token n sees codes[0, n). The decode is the oracle codec + iSTFT.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "mio_oracle.h"

typedef struct {
    float *out;
    long cap, n;
    long long *chunks;
    long chunk_cap, n_chunks;
    float *tail;
    long tail_n, xfade, chunk_samples;
    int overflow;
} emitter;

static long min_l(long a, long b) { return a < b ? a : b; }

/* emit_range (test-to-speech.cpp:367-417) for samples [begin, end) of audio */
static void emit_range(emitter *e, const float *audio, long begin, long end) {
    int first = 1;
    for (long i = begin; i < end;) {
        const long n = min_l(e->chunk_samples, end - i);
        if (e->n + n > e->cap || e->n_chunks >= e->chunk_cap) {
            e->overflow = 1;
            return;
        }
        float *chunk = e->out + e->n;
        memcpy(chunk, audio + i, (size_t)n * sizeof(float));
        if (first && e->tail_n > 0) {
            const long xf = min_l(e->tail_n, n);
            for (long j = 0; j < xf; ++j) {
                const float a = (float)(j + 1) / (float)(xf + 1);
                const float b = 1.0f - a;
                chunk[j] = b * e->tail[j] + a * chunk[j];
            }
        }
        if (n >= e->xfade) {
            memcpy(e->tail, chunk + n - e->xfade, (size_t)e->xfade * sizeof(float));
            e->tail_n = e->xfade;
        } else {
            memcpy(e->tail, chunk, (size_t)n * sizeof(float));
            e->tail_n = n;
        }
        e->chunks[e->n_chunks++] = n;
        e->n += n;
        i += n;
        first = 0;
    }
}

/* Emitted stream for the generated codes[0, n_codes). Returns the number of samples written
 * to out (chunk sizes in chunks[], their count in *n_chunks, full decodes in *n_decodes), or
 * -1 on a decode failure / overflow. */
long mo_stream_emit(mo_codec *c, const float *emb, const int *codes, int n_codes, int check_interval,
                    int holdback, int min_commit, long chunk_samples, float *out, long out_cap,
                    long long *chunks, long chunk_cap, long *n_chunks, int *n_decodes) {
    int info[8];
    mo_codec_info(c, info);
    const int sample_rate = info[0], n_fft = info[1], hop = info[2], spt = info[3], n_freq = info[4];
    const int frames_per_code = info[6];
    emitter e;
    memset(&e, 0, sizeof(e));
    e.out = out, e.cap = out_cap, e.chunks = chunks, e.chunk_cap = chunk_cap;
    e.chunk_samples = chunk_samples > 0 ? chunk_samples : 4096;
    e.xfade = min_l((long)(sample_rate * 3 / 100), 4096);
    e.tail = (float *)malloc((size_t)e.xfade * sizeof(float));
    float *spec = (float *)malloc((size_t)n_codes * frames_per_code * n_freq * 2 * sizeof(float) + 16);
    float *audio = (float *)malloc((size_t)n_codes * spt * sizeof(float) + (size_t)n_fft * sizeof(float) + 16);
    long committed = 0;
    int decodes = 0, rc = 0;
    if (!e.tail || !spec || !audio) rc = -1;
    for (int n = 1; !rc && n <= n_codes + 1; ++n) {
        const int is_final = n == n_codes + 1;
        const int have = is_final ? n_codes : n;
        if (!is_final && (check_interval <= 0 || n % check_interval != 0)) continue;
        if (have == 0) continue;
        const long target = is_final ? have : (have > holdback ? have - holdback : 0);
        if (target <= committed) continue;
        if (!is_final && target - committed < min_commit) continue;
        const int frames = mo_codec_decode(c, codes, have, emb, spec);
        if (frames < 0) {
            rc = -1;
            break;
        }
        const int len = mo_istft(spec, frames, n_fft, n_fft, hop, audio);
        if (len < 0) {
            rc = -1;
            break;
        }
        ++decodes;
        const double per_code = (double)len / (double)have;
        const long b = (long)llround((double)committed * per_code);
        const long end = (long)llround((double)target * per_code);
        const long safe_end = min_l(end, (long)len);
        if (b >= safe_end) continue;
        committed = target;
        emit_range(&e, audio, b, safe_end);
        if (e.overflow) rc = -1;
    }
    free(e.tail);
    free(spec);
    free(audio);
    if (n_chunks) *n_chunks = e.n_chunks;
    if (n_decodes) *n_decodes = decodes;
    return rc ? -1 : e.n;
}
