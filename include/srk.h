/*
 * srk.h — the C ABI of libsrk.so, the MI355X (gfx950 / CDNA4) native hot path of
 * remit0/SpeechRecognitionProject: feature extraction -> acoustic model train step.
 *
 * Conventions (SURVEY.md §8b "C-ABI the build must export"):
 *  - every tensor pointer is a caller-owned DEVICE pointer (e.g. a torch tensor's data_ptr());
 *  - every call only ENQUEUES work on the caller's stream (`void* stream` = hipStream_t,
 *    nullptr = the legacy default stream) and returns 0 on success or a negative srk_status;
 *  - srk_last_error() returns a thread-local description of the last failure;
 *  - no call allocates device memory in steady state: scratch comes from the caller, sized by
 *    the matching *_workspace_bytes() query.  Constant tables are uploaded once per device
 *    by srk_init() (idempotent, thread-safe; called implicitly on first use);
 *  - layouts are row-major, innermost dimension last, fp32 unless the name says otherwise.
 *
 * Each entry point cites the reference function whose arithmetic it replaces
 * (paths relative to the reference repository).
 */
#ifndef SRK_H_
#define SRK_H_

#include <stdint.h>

#define SRK_ABI_VERSION 1

#ifdef __cplusplus
extern "C" {
#endif

enum srk_status {
  SRK_OK = 0,
  SRK_ERR_INVALID = -1,   /* bad argument (shape, null pointer, unsupported option) */
  SRK_ERR_HIP = -2,       /* a HIP runtime call failed */
  SRK_ERR_INTERNAL = -3,  /* anything else (host exception) */
};

/* ---------------------------------------------------------------- library / device */
int srk_version(void);                 /* ABI version, bumped on any signature change */
const char* srk_last_error(void);      /* thread-local, never NULL */
int srk_init(int device);              /* build + upload constant tables on `device` */

/* ---------------------------------------------------------------- feature extraction
 * pcm: float32 [n_clips, 16000], int16-valued (NOT scaled to +-1), exactly what
 * dataset.py:89-122 returns per item and DataLoader collates (training.py:77).        */

/* K2: log-mel filter banks, models/model_fbanks_cnn.py:15-66 (`filter_banks`).
 * out: [n_clips, 98, 120] (time x mel), dB.                                            */
int srk_fbank_fwd(const float* pcm, int64_t n_clips, float* out, void* stream);

/* K1: MFCC + delta + delta-delta, models/model_mfcc_bgru.py:11-19 (`compute_mfcc`, librosa
 * mfcc(n_mfcc=13, n_fft=640, hop=320) + np.gradient x2).
 * layout 0: out [n_clips, 39, 51] (the reference's compute_mfcc layout);
 * layout 1: out [n_clips, 51, 39] (time-major, = the transpose at model_mfcc_bgru.py:34). */
int srk_mfcc_fwd(const float* pcm, int64_t n_clips, float* out, int layout, void* stream);

/* K3: log spectrogram, models/model_spec_bgru.py:11-17 (`compute_spec`, scipy.signal.spectrogram
 * nperseg=640, noverlap=320, Tukey(0.25), PSD density, log(S + 1e-10)).
 * transposed 0: out [n_clips, 321, 49] (freq x time, model_spec_bgru.py);
 * transposed 1: out [n_clips, 49, 321] (time x freq, models/model_spec_cnn.py:14).     */
int srk_spec_fwd(const float* pcm, int64_t n_clips, float* out, int transposed, void* stream);

/* K4: uniform noise mix, dataset.py:183-193 (`add_noise_uniform`) with the random draws made
 * explicit: out[b, i] = (float) int16_trunc( (double)pcm[b, i] + gain[b] * (double)
 *                        bank[file_idx[b] * bank_len + offset[b] + i] ).
 * pcm: int16 [n_clips, 16000]; bank: int16 [n_files, bank_len]; out: float32 [n_clips, 16000].
 * The caller guarantees 0 <= offset[b] <= bank_len - 16000 and 0 <= file_idx[b] < n_files. */
int srk_noise_mix(const int16_t* pcm, const int16_t* bank, int64_t n_files, int64_t bank_len,
                  const int64_t* file_idx, const int64_t* offset, const double* gain,
                  int64_t n_clips, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SRK_H_ */
