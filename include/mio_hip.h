/*
 * mio_hip.h — thin C-ABI over the MI355X (gfx950) MioTTS hot path.
 *
 * Plain pointers and sizes only; no HIP or torch types in any signature
 * (streams are passed as `void *` = hipStream_t, NULL = the handle's own stream).
 * Every function returns an int status (MIO_OK = 0) unless noted; the text of the
 * last failure on the calling thread is in mio_hip_last_error().
 *
 * Buffers are caller-owned. Pointer arguments are HOST memory unless the matching
 * MIO_*_DEVICE flag says they are device memory of the handle's GPU.
 * One handle per device; a handle is used from one host thread at a time
 * (the reference TestToSpeech is single-threaded per instance, test-to-speech.h:26).
 *
 * Which reference interface each entry point replaces is cited per function.
 */
#ifndef MIO_HIP_H
#define MIO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIO_OK 0
#define MIO_ERR_INVALID (-1)
#define MIO_ERR_HIP (-2)
#define MIO_ERR_IO (-3)
#define MIO_ERR_FORMAT (-4)
#define MIO_ERR_OOM (-5)
#define MIO_ERR_UNSUPPORTED (-6)

/* buffer-location flags */
#define MIO_IN_DEVICE 1u
#define MIO_OUT_DEVICE 2u

typedef struct mio_hip_device mio_hip_device;
typedef struct mio_hip_istft mio_hip_istft;

/* ---------------- device / memory ---------------- */
const char *mio_hip_last_error(void);
int mio_hip_device_count(int *n);
/* Opens GPU `dev` and creates its default stream. */
int mio_hip_device_open(int dev, mio_hip_device **out);
void mio_hip_device_close(mio_hip_device *d);
int mio_hip_device_sync(mio_hip_device *d);
/* Number of compute units of the opened device (256 on MI355X). */
int mio_hip_device_cu_count(const mio_hip_device *d, int *n_cu);
int mio_hip_malloc(mio_hip_device *d, size_t bytes, void **dptr);
int mio_hip_free(mio_hip_device *d, void *dptr);
int mio_hip_memcpy_h2d(mio_hip_device *d, void *dst, const void *src, size_t bytes);
int mio_hip_memcpy_d2h(mio_hip_device *d, void *dst, const void *src, size_t bytes);
int mio_hip_memset(mio_hip_device *d, void *dst, int value, size_t bytes);

/* Event timer on the handle's stream (or `stream`): returns ms between two marks.
 * mio_hip_timer_mark(d, stream, slot) records event `slot` (0..15). */
int mio_hip_timer_mark(mio_hip_device *d, void *stream, int slot);
int mio_hip_timer_elapsed(mio_hip_device *d, int slot_a, int slot_b, float *ms);

/* ---------------- iSTFT ----------------
 * Replaces istft_cache(n_fft, win_length) (istft.h:6-30, istft.cpp:7-32) and
 * istft(spec, n_frames, hop, cache) (istft.h:38-42, istft.cpp:68-108).
 * spec: [n_frames][n_fft/2+1][2] f32 (re, im) — the layout miocodec_decode returns
 * (miocodec.cpp:801-808). out: (n_frames-1)*hop + win - 2*((win-hop)/2) samples
 * (= hop*n_frames when win-hop is even); *out_len receives that count (0 if empty,
 * like the reference's empty vector). */
int mio_hip_istft_create(mio_hip_device *d, int n_fft, int win_length, mio_hip_istft **out);
void mio_hip_istft_destroy(mio_hip_istft *h);
int mio_hip_istft_out_len(const mio_hip_istft *h, int n_frames, int hop_length, int *out_len);
int mio_hip_istft_run(mio_hip_istft *h, const float *spec, int n_frames, int hop_length,
                      float *out, int *out_len, unsigned flags, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MIO_HIP_H */
