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

#define SRK_ABI_VERSION 2

#ifdef __cplusplus
extern "C" {
#endif

enum srk_status {
  SRK_OK = 0,
  SRK_ERR_INVALID = -1,   /* bad argument (shape, null pointer, unsupported option) */
  SRK_ERR_HIP = -2,       /* a HIP runtime call failed */
  SRK_ERR_INTERNAL = -3,  /* anything else (host exception) */
  SRK_ERR_TIMEOUT = -4,   /* a persistent kernel's bounded spin-wait gave up: results are invalid */
};

/* ---------------------------------------------------------------- library / device */
int srk_version(void);                 /* ABI version, bumped on any signature change */
/* First 16 hex digits of the sha256 over the library's sources (the csrc .hip / .h / .cpp files and this
 * header, in name order) as built: profiling records (profiles/pmc_*.json) carry the stamp of the
 * library they measured, and bench.py attaches them only to a run of the same build.              */
const char* srk_source_stamp(void);
const char* srk_last_error(void);      /* thread-local, never NULL */
int srk_init(int device);              /* build + upload constant tables on `device` */
/* Opt-in kernel timing: while enabled, instrumented launches record a HIP event pair on their
 * stream; srk_prof_read sums, over every launch named `name` ("mfcc", "fbank", "spec",
 * "noise_mix", "gemm_f32", "gru_fwd_step", "gru_bwd_step", "adam", ...), the elapsed time and
 * the launches' ALGORITHMIC work (flops for matrix kernels, bytes for streaming kernels).
 * srk_prof_enable synchronizes the device and clears previous records.                     */
/* Generation of the library's grow-only scratch buffers (split-K slabs, conv / BatchNorm partials):
 * it changes whenever one is reallocated, which invalidates any HIP graph captured before.         */
int64_t srk_scratch_generation(void);
int srk_prof_enable(int on);
int srk_prof_read(const char* name, int64_t* count, double* total_ms, double* total_work);
/* Every record since srk_prof_enable grouped by (name, launch detail: kernel template + shape), one
 * "name\tdetail\tcount\ttotal_ms\ttotal_work\ttotal_bytes\n" line each, NUL-terminated into buf
 * (truncated at cap bytes); *needed = the full size.  total_bytes = the launches' ALGORITHMIC HBM
 * bytes where the launch site states them (matrix kernels: operands once + the output; 0 elsewhere).
 * bench.py names the largest single kernel with it and prices PMC traffic against the bytes. */
int srk_prof_kernels(char* buf, int64_t cap, int64_t* needed);
/* Runtime options: "gru_persistent" (default 1) = run each GRU layer's recurrence as ONE
 * persistent launch with W_hh resident in LDS (0 = one launch per time step);
 * "matmul_precision" (default 0) = operand precision of the matrix-core kernels (GEMM, GRU
 * recurrence): 0 fp32 (exact, the reference's arithmetic), 1 bf16, 2 fp16 — operands rounded to
 * nearest-even on chip, fp32 accumulation, fp32 tensors in and out (BASELINE.json cfg2 / cfg5);
 * "gemm16_kernel" (default 0 = by shape) = the 16-bit-operand GEMM kernel: 1 register-staged,
 * 2 LDS-DMA ping-pong (same results up to fp32 summation order; for A/B measurements and tests);
 * "gemm32_kernel" (default 0 = by shape) = the same choice for the fp32 GEMM;
 * "conv16_sources" (default 1) = bf16 / fp16 convolutions gather from one pre-rounded 16-bit copy
 * of their operands (0 = round at LDS-store time; bit-identical results either way);
 * "conv_ring" (default 0x77) = the LDS-DMA ring implicit-GEMM convolutions where the shape
 * qualifies (bits 0-2 fp32 fwd / dgrad / wgrad, 4-6 the same in 16 bit, 7 also the pooled forward
 * and the fp32 forward at K < 3072); "conv_unpool16" (default 1) = the 16-bit pooled-conv backward
 * writes the dense dY straight as its 16-bit operand copy; "gru_dwhh_fused" (default 1) = the 16-bit
 * BiGRU backward accumulates dW_hh inside the recurrence kernel (0 = a GEMM over dgh16 / y16; bits
 * 1 / 2 of a non-zero value: timing variants, bitwise bit 0's results) — results equal up to fp32
 * summation order (A/B measurements and tests). */
int srk_set_option(const char* name, int64_t value);
/* Number of bounded spin-waits of the persistent kernels that gave up (synchronizes the
 * device; must stay 0 — a non-zero value means a co-residency assumption failed).  -1 on error. */
int64_t srk_spin_timeouts(void);
/* Fatal-timeout check: SRK_OK, or SRK_ERR_TIMEOUT (sticky until srk_health_reset) once any
 * persistent-kernel spin-wait has given up.  Reads a host-pinned word the kernels raise, so with
 * sync = 0 it costs no device synchronization (it sees timeouts of work the GPU has reached);
 * sync = 1 synchronizes the device first.  Option "gru_spin_limit" (test hook) shortens the wait. */
int srk_health_check(int sync);
/* Host-side audit of the persistent GRU's step-ordering words for a batch of B rows at the given
 * precision (0 fp32, 1 bf16, 2 fp16): *max_word = largest counter / flag word any workgroup of the
 * planned launches touches, *chunks = launches, *census = first word of the XCD census (must exceed
 * *max_word).  No GPU needed.                                                                     */
int srk_gru_audit_words(int64_t B, int precision, int backward, int64_t* max_word, int64_t* chunks, int64_t* census);
int srk_health_reset(void);

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

/* K1 / K2 / K3 on int16 PCM [n_clips, 16000] (4-byte aligned): the samples the WAV holds, widened to
 * float32 in the kernels' load stage — the same values as the float32 entry points above (the
 * reference's float32 PCM is int16-valued, dataset.py:117), at half the bytes to upload and read. */
int srk_fbank_fwd_i16(const int16_t* pcm, int64_t n_clips, float* out, void* stream);
int srk_mfcc_fwd_i16(const int16_t* pcm, int64_t n_clips, float* out, int layout, void* stream);
int srk_spec_fwd_i16(const int16_t* pcm, int64_t n_clips, float* out, int transposed, void* stream);

/* K4: uniform noise mix, dataset.py:183-193 (`add_noise_uniform`) with the random draws made
 * explicit: out[b, i] = (float) int16_trunc( (double)pcm[b, i] + gain[b] * (double)
 *                        bank[file_idx[b] * bank_len + offset[b] + i] ).
 * pcm: int16 [n_clips, 16000]; bank: int16 [n_files, bank_len]; out: float32 [n_clips, 16000].
 * The caller guarantees 0 <= offset[b] <= bank_len - 16000 and 0 <= file_idx[b] < n_files. */
int srk_noise_mix(const int16_t* pcm, const int16_t* bank, int64_t n_files, int64_t bank_len,
                  const int64_t* file_idx, const int64_t* offset, const double* gain,
                  int64_t n_clips, float* out, void* stream);

/* K4 fused into K3's load stage (model_spec_bgru on noise-augmented clips, dataset.py:183-193 then
 * models/model_spec_bgru.py:11-17): out = srk_spec_fwd of srk_noise_mix(pcm, bank, ...) — the same
 * values bit for bit — without the mixed fp32 PCM going through HBM (int16 clip + int16 noise window
 * in, the spectrogram out).  Arguments as srk_noise_mix (bank 4-byte aligned) and srk_spec_fwd. */
int srk_spec_noise_fwd(const int16_t* pcm, const int16_t* bank, int64_t n_files, int64_t bank_len,
                       const int64_t* file_idx, const int64_t* offset, const double* gain, int64_t n_clips,
                       float* out, int transposed, void* stream);

/* K10: batched training-mode augmentation, dataset.py:103-118 and its helpers :148-223, with the
 * random draws made explicit (one op per clip; the Python `Dataset.__getitem__` draws them per
 * item, srk_augment applies a whole batch in one launch).  op[b]:
 *   SRK_AUG_NONE      out = pcm
 *   SRK_AUG_SPEED     speed_tuning (:206-223): cv2 INTER_LINEAR resample to iparam[b] =
 *                     int(16000 * rate) samples, then centre cut, or random pad when shorter
 *   SRK_AUG_SHIFT     time_stretching (:195-204): shift by iparam[b] in (-16000, 16000)
 *   SRK_AUG_NOISE     add_noise_uniform (:183-193): int16(pcm + dparam[b] * noise)
 *   SRK_AUG_NOISE_SNR add_noise_snr (:163-181): dparam[b] = 10 ** (snr_dB / 10)
 *   SRK_AUG_SILENCE   generate_silence_sample (:148-161): float32(noise * dparam[b]); pcm unused;
 *                     noise_pos[b] < 0 gives the all-zero sample
 *   SRK_AUG_PITCH     pitch_shifting (:225-235): out = pcm here; srk_pitch_shift (K12) then
 *                     overwrites the clip with its shifted version (iparam[b] = n_steps)
 * noise = bank[noise_pos[b] .. + 16000) of the flat int16 noise bank (ragged files concatenated);
 * ops without noise ignore noise_pos.  The pad samples the reference draws with
 * np.random.randint(-32, 32, k) come from a counter hash of (seed, b, output position)
 * (oracle/augment.py aug_fill).  pcm: int16 [n_clips, 16000] (zero padded as dataset.py:100-102),
 * out: float32 [n_clips, 16000]; both 16-byte aligned.  op/iparam/noise_pos/dparam: device arrays
 * of n_clips entries, validated by the caller (out-of-range noise windows read as silence). */
/* ---------------------------------------------------------------- evaluation callers
 * K11: softmax ensemble, predictions.py:56-69 / models/model_analyst.py:22-53: logits float32
 * [K, B, C] (model-major) -> per clip the softmax of each model's logits; probs_cat [B, K*C] their
 * concatenation (the analyst's input, nullable), mean [B, C] = (p_1 + ... + p_K) / K (nullable),
 * pred int64 [B] = first arg-max of the mean (nullable).  1 <= K <= 8, 1 <= C <= 64.          */
int srk_softmax_ensemble(const float* logits, int64_t K, int64_t B, int64_t C, float* probs_cat, float* mean,
                         int64_t* pred, void* stream);

/* ---------------------------------------------------------------- input pipeline (host)
 * Batched WAV decode, dataset.py:98-102 (scipy.io.wavfile.read + zero pad to 16000): n files
 * (NUL-terminated paths) decoded by up to min(n_threads, 16) host threads (n_threads <= 0: all
 * hardware threads, capped at 16) into out int16 [n, 16000] (HOST memory, e.g. pinned): the first
 * min(len, 16000) samples, zero padded.  lengths[b] = the file's sample count (a count > 16000
 * is reported as is — dataset.py:104-106 then fails on that item), or a negative SRK_WAV_ERR_*
 * with out[b] all zero.  PCM16 mono RIFF/WAVE only (tag 1 or WAVE_FORMAT_EXTENSIBLE/PCM); other
 * chunks skipped.  Returns SRK_OK unless the arguments are invalid: per-file errors are data,
 * as __getitem__'s except branch (dataset.py:124-128) makes them.  Touches no GPU state.      */
enum { SRK_WAV_ERR_OPEN = -1, SRK_WAV_ERR_FORMAT = -2, SRK_WAV_ERR_UNSUPPORTED = -3 };
int srk_wav_read_batch(const char* const* paths, int64_t n, int16_t* out, int64_t* lengths, int n_threads);

enum { SRK_AUG_NONE = 0, SRK_AUG_SPEED = 1, SRK_AUG_SHIFT = 2, SRK_AUG_NOISE = 3, SRK_AUG_NOISE_SNR = 4,
       SRK_AUG_SILENCE = 5, SRK_AUG_PITCH = 6 /* srk_augment copies the clip; srk_pitch_shift shifts it */ };
int srk_augment(const int16_t* pcm, int64_t n_clips, const int16_t* bank, int64_t bank_len, const int32_t* op,
                const int64_t* iparam, const int64_t* noise_pos, const double* dparam, uint64_t seed, float* out,
                void* stream);

/* K12: batched pitch_shifting, dataset.py:225-235 — np.int16(librosa.effects.pitch_shift(
 * sample.astype(float), 16000, n_steps)) for n_steps in {-2, -1, 1, 2} (the reference's level None
 * leaves the clip as is): librosa 0.6's time_stretch (STFT 2048 / 512, phase vocoder, inverse STFT)
 * then resampy's kaiser_best resample from 16000 / rate to 16000 Hz, rate = 2^(-n_steps / 12)
 * (algorithm and dtypes: oracle/pitch.py; parity unpinned — librosa / resampy are absent).
 * For s < n_shift: out[clip_idx[s]] = the shifted pcm[clip_idx[s]] as int16-valued float32,
 * level_idx[s] in 0..3 = n_steps -2, -1, 1, 2.  pcm: int16 [n_clips, 16000]; out: float32
 * [n_clips, 16000] (rows not listed untouched); clip_idx / level_idx: device int32 [n_shift],
 * validated by the caller.  One launch for the whole batch (one workgroup per shifted clip).
 * workspace: device scratch of srk_pitch_workspace_bytes(n_shift) bytes, 16-byte aligned.     */
int64_t srk_pitch_workspace_bytes(int64_t n_shift);
int srk_pitch_shift(const int16_t* pcm, int64_t n_clips, const int32_t* clip_idx, const int32_t* level_idx,
                    int64_t n_shift, float* out, void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- dense algebra (fp32 MFMA)
 * C[M,N] = alpha * op(A) op(B) + beta * C (+ bias), row-major.  op(A) = A [M,K] (lda) or, with
 * trans_a, A stored [K,M]; op(B) = B [K,N] (ldb) or, with trans_b, B stored [N,K].
 * bias_mode: 0 none, 1 bias[N] per column, 2 bias[M] per row.  Replaces the cuBLAS/CPU GEMMs of
 * nn.Linear (model_mfcc_bgru.py:26,36; model_fbanks_cnn.py:80-81,99-100).                  */
int srk_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                 int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                 const float* bias, int bias_mode, void* stream);
/* The same GEMM (alpha, beta, no bias) that also writes rowsum[m] = beta * rowsum[m] +
 * sum_k op(A)[m, k]: the weight and bias gradients of a Linear in one pass (dW = dY^T X,
 * db = sum over the batch of dY); beta = 1 accumulates both into existing .grad buffers.     */
int srk_gemm_rowsum_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                        int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                        float* rowsum, void* stream);
/* The same GEMM on 16-bit operands already in memory (bf16 or fp16 as set by matmul_precision,
 * which must not be fp32): A / B hold raw 16-bit values, leading dimensions in elements; fp32
 * accumulation, C / bias fp32.  Needs 16-B aligned rows whose lengths are multiples of 8.      */
int srk_gemm_16(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const uint16_t* A,
                int64_t lda, const uint16_t* B, int64_t ldb, float beta, float* C, int64_t ldc,
                const float* bias, int bias_mode, void* stream);
/* Batched form of srk_gemm_16 (no bias): for z < batch, C + z sC = alpha op(A + z sA) op(B + z sB)
 * + beta (C + z sC); strides in elements, multiples of 8 (sC of 4).  The BiGRU backward's two
 * recurrent weight gradients (nn.GRU weight_hh_l{k}{,_reverse}.grad, models/model_mfcc_bgru.py:25)
 * run as one batch-2 launch.                                                                  */
int srk_gemm_16_batched(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                        const uint16_t* A, int64_t lda, int64_t sA, const uint16_t* B, int64_t ldb,
                        int64_t sB, float beta, float* C, int64_t ldc, int64_t sC, int batch, void* stream);
/* out[n] = beta * out[n] + sum_m X[m, n]  (bias gradients).                                 */
int srk_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, void* stream);

/* ---------------------------------------------------------------- K5: bidirectional GRU layer
 * nn.GRU(in, H, bidirectional=True, batch_first=True), one layer, PyTorch gate order [r; z; n],
 * h0 = 0 (model_mfcc_bgru.py:25,35; model_spec_bgru.py:23,33; model_resnet_bgru.py:130,135).
 * x [B, T, in]; y [B, T, 2H] (forward direction in [..., :H], reverse in [..., H:]).
 * Weights are direction-stacked: w_ih [2][3H][in] (= weight_ih_lK ; weight_ih_lK_reverse),
 * w_hh [2][3H][H], b_ih [2][3H], b_hh [2][3H].  H must be a multiple of 128.
 * ws (fwd, kept until the backward): srk_gru_workspace_floats(.., backward=0) floats;
 * ws (bwd scratch): srk_gru_workspace_floats(.., backward=1) floats.
 * Backward writes dx [B, T, in] (NULL when the input needs no gradient) and OVERWRITES
 * (accumulate = 0) or ADDS TO (accumulate = 1: autograd's .grad accumulation, done in the GEMM
 * epilogues) dw_ih, dw_hh, db_ih, db_hh (same stacked layouts).  The backward must run at the
 * matmul_precision of its forward (with bf16 / fp16 the forward workspace carries the 16-bit
 * operands of the backward's GEMMs; a layer with the fused input projection, in <= 64, leaves the
 * 16-bit W_ih slot to the backward, which fills it there only when dx is requested).          */
int64_t srk_gru_workspace_floats(int64_t B, int64_t T, int64_t in, int64_t H, int backward);
int srk_gru_layer_fwd(const float* x, int64_t B, int64_t T, int64_t in, int64_t H, const float* w_ih,
                      const float* w_hh, const float* b_ih, const float* b_hh, float* y, float* ws,
                      void* stream);
int srk_gru_layer_bwd(const float* x, int64_t B, int64_t T, int64_t in, int64_t H, const float* w_ih,
                      const float* w_hh, const float* y, const float* ws_fwd, const float* dy, float* dx,
                      float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate, float* ws,
                      void* stream);
/* The same pair taking x's ready 16-bit copy x16 ([B*T][in] bf16 / fp16 at the current precision,
 * in % 8 == 0, 16-B aligned; nullable = the plain pair) instead of rounding x: a 2-layer BiGRU's
 * second layer reads the first layer's own 16-bit h copy, which srk_gru_y16_offset locates in that
 * layer's forward workspace (in floats; -1 when the layer does not take the 16-bit path).  The
 * backward must get the forward's x16.  Bitwise the results of the plain pair (the kernels round h
 * exactly as the conversion of x would).                                                          */
int64_t srk_gru_y16_offset(int64_t B, int64_t T, int64_t in, int64_t H);
int srk_gru_layer_fwd_x16(const float* x, const void* x16, int64_t B, int64_t T, int64_t in, int64_t H,
                          const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* y,
                          float* ws, void* stream);
int srk_gru_layer_bwd_x16(const float* x, const void* x16, int64_t B, int64_t T, int64_t in, int64_t H,
                          const float* w_ih, const float* w_hh, const float* y, const float* ws_fwd, const float* dy,
                          float* dx, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate,
                          float* ws, void* stream);

/* ---------------------------------------------------------------- K6: convolution / pooling
 * nn.Conv2d / nn.Conv1d (zero padding ph/pw, stride sh/sw, no dilation/groups) as implicit GEMM
 * on CHANNELS-LAST activations: x [N][H][W][Ci], y [N][Ho][Wo][Co], Ho = (H + 2ph - KH)/sh + 1.
 * Weights stay in torch layout w [Co][Ci][KH][KW] (the state_dict tensor), bias [Co] (nullable).
 * ws: srk_conv2d_workspace_floats() floats (re-laid-out weights).  The 1-D convolutions of
 * model_resnet_bgru.py are H = 1, KH = 1.  Replaces model_fbanks_cnn.py:72-75,89-94.
 * Backward writes dw [Co][Ci][KH][KW] (overwrite), db (nullable) and dx (nullable).          */
int64_t srk_conv2d_workspace_floats(int64_t Ci, int64_t Co, int64_t KH, int64_t KW);
int srk_conv2d_nhwc_fwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                        const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh,
                        int64_t sw, float* y, float* ws, void* stream);
int srk_conv2d_nhwc_bwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                        int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw, const float* dy,
                        float* dx, float* dw, float* db, float* ws, void* stream);
/* The same pair with the forward's 16-bit copy of x kept for the backward (bf16 / fp16 matmul
 * precision, Ci and Co multiples of 8, 16-B aligned tensors: the 16-bit operand path).  fwd16
 * rounds x into x16 (N*H*W*Ci 16-bit elements, 16-B aligned, caller storage) and sets
 * *x16_written = 1 when that path ran, else 0 (x16 untouched); bwd16 gathers from that copy instead
 * of rounding x again (x16 null: as srk_conv2d_nhwc_bwd).  The backward must run at the forward's
 * precision.  Bitwise the results of the plain pair.  *x16_written = 2 on entry declares that x16
 * already holds x's copy at this precision (srk_batchnorm_fwd16's y16): fwd16 then reads it instead
 * of rounding x.  bwd16_dy16 also takes dY's ready copy dy16 (srk_batchnorm_bwd16's dx16; nullable;
 * used wherever the 16-bit path would round dy, dy itself still required).                   */
int srk_conv2d_nhwc_fwd16(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                          const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh,
                          int64_t sw, float* y, float* ws, void* x16, int* x16_written, void* stream);
int srk_conv2d_nhwc_bwd16(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                          int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw, const float* dy,
                          float* dx, float* dw, float* db, float* ws, const void* x16, void* stream);
int srk_conv2d_nhwc_bwd16_dy16(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                               int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw,
                               const float* dy, const void* dy16, float* dx, float* dw, float* db, float* ws,
                               const void* x16, void* stream);
/* The same with dw_accumulate = 1: dw is the parameter's existing .grad and the weight gradient is ADDED
 * to it (autograd's accumulation of a returned gradient, fused into the layout kernel that writes it). */
int srk_conv2d_nhwc_bwd16_acc(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                              int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw,
                              const float* dy, const void* dy16, float* dx, float* dw, float* db, float* ws,
                              const void* x16, int dw_accumulate, void* stream);
/* Conv2d (stride 1) + bias + MaxPool2d((1, 4)) fused (model_fbanks_cnn.py:74-75,91-92: conv2 then
 * maxpool2): the implicit GEMM's epilogue pools its own output, so only the pooled activation y
 * [N][Ho][Wo/4][Co] and the uint8 window argmax [N][Ho][Wo/4][Co] (first maximum, NaN wins: the
 * maxpool rule) are written.  Needs pool_w = 4 dividing Wo.  x16 / x16_written as fwd16.  The
 * backward takes the POOLED gradient and the argmax (the dense gradient exists only in library
 * scratch) and gives what srk_conv2d_nhwc_bwd16 gives for the unpooled gradient.               */
int srk_conv2d_nhwc_fwd_pool(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                             const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw,
                             int64_t pool_w, float* y, uint8_t* argmax, float* ws, void* x16, int* x16_written,
                             void* stream);
int srk_conv2d_nhwc_bwd_pool(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                             int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool_w, const float* dy_pooled,
                             const uint8_t* argmax, float* dx, float* dw, float* db, float* ws, const void* x16,
                             void* stream);
/* Max pooling, window = stride = (kh, kw), floor mode, channels-last (nn.MaxPool2d((1,3)),
 * ((1,4)) and nn.MaxPool1d(98), model_fbanks_cnn.py:73,75,78).  Backward routes each gradient to
 * the first maximum of its window, as PyTorch does.                                          */
/* Fused first layer of model_fbanks_cnn (models/model_fbanks_cnn.py:72-73,89-90): Conv2d(1, 64,
 * (7,3), padding (3,1)) + bias + MaxPool2d((1,3)) in one pass.  x: [N, H, W] (one input channel);
 * y: pooled [N, H, W/3, 64] (NHWC); argmax: uint8 [N, H, W/3, 64] = position (0..2) of each window's
 * first maximum (PyTorch's rule, NaN wins).  Only that geometry is accepted (SRK_ERR_INVALID else).
 * The backward gives dW [64,1,7,3] and db [64] (db may be NULL) from the POOLED gradient dy and
 * argmax (the unpooled gradient is never formed); ws: srk_conv1_pool_workspace_floats() floats. */
int64_t srk_conv1_pool_workspace_floats(int64_t Co, int64_t KH, int64_t KW);
int srk_conv1_pool_fwd(const float* x, int64_t N, int64_t H, int64_t W, const float* w, const float* bias,
                       int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool, float* y,
                       uint8_t* argmax, void* stream);
/* As srk_conv1_pool_fwd, and in the 16-bit matmul modes also the pooled activation's bf16 / fp16 operand copy
 * (y16: N*H*(W/pool)*Co 16-bit elements, 8-byte aligned, or null), the one srk_conv2d_nhwc_fwd_pool accepts as
 * ready (x16_written = 2) instead of converting y again; *y16_written = 1 when it was written.  *y16_written = 3
 * on entry: the caller consumes only the copy, and y is left unwritten when the copy is written. */
int srk_conv1_pool_fwd16(const float* x, int64_t N, int64_t H, int64_t W, const float* w, const float* bias,
                         int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool, float* y,
                         uint8_t* argmax, void* y16, int* y16_written, void* stream);
int srk_conv1_pool_wgrad(const float* x, int64_t N, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                         int64_t ph, int64_t pw, int64_t pool, const float* dy, const uint8_t* argmax, float* dw,
                         float* db, float* ws, void* stream);
int srk_maxpool_nhwc_fwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t kh, int64_t kw,
                         float* y, void* stream);
int srk_maxpool_nhwc_bwd(const float* x, const float* dy, int64_t N, int64_t H, int64_t W, int64_t C, int64_t kh,
                         int64_t kw, float* dx, void* stream);

/* ---------------------------------------------------------------- K9: batch norm (+ residual, ReLU)
 * nn.BatchNorm1d on channels-last x [M][C] (M = N * L), fused with an optional residual add and
 * ReLU: y = act((x - mean) * invstd * gamma + beta [+ residual]) (model_resnet_bgru.py:20-39,49).
 * training = 1: batch statistics (biased variance), running stats updated in place with
 * `momentum` (unbiased variance), as nn.BatchNorm1d; training = 0: running statistics.
 * save_mean / save_invstd [C] are written for the backward.  Backward takes the forward's y (for
 * the ReLU mask) and writes dx (nullable), dgamma, dbeta and dresidual (nullable).            */
int srk_batchnorm_fwd(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                      float momentum, int training, float* running_mean, float* running_var, const float* residual,
                      int relu, float* y, float* save_mean, float* save_invstd, void* stream);
int srk_batchnorm_bwd(const float* x, const float* y, const float* dy, int64_t M, int64_t C, const float* gamma,
                      const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                      float* dgamma, float* dbeta, float* dresidual, void* stream);
/* The same pair emitting the 16-bit operand copy of their output for the convolution that consumes it
 * (model_resnet_bgru.py: every conv reads a BatchNorm output, and every BatchNorm's dx is a conv's dY).
 * fwd16 writes y16 = y rounded to the bf16 / fp16 matmul precision (M*C 16-bit elements, 16-B aligned,
 * caller storage) beside y; bwd16 writes dx16 = dx rounded likewise; *_written = 1 when the copy was
 * written, else 0 (fp32 precision, null or misaligned pointer; dx16 also needs dx).  The rounding is
 * the convolutions' own (round to nearest even), so srk_conv2d_nhwc_fwd16 (x16_written = 2 on entry)
 * and srk_conv2d_nhwc_bwd16_dy16 use the copies bitwise as if they had made them.               */
int srk_batchnorm_fwd16(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                        float momentum, int training, float* running_mean, float* running_var, const float* residual,
                        int relu, float* y, void* y16, int* y16_written, float* save_mean, float* save_invstd,
                        void* stream);
int srk_batchnorm_bwd16(const float* x, const float* y, const float* dy, int64_t M, int64_t C, const float* gamma,
                        const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                        void* dx16, int* dx16_written, float* dgamma, float* dbeta, float* dresidual, void* stream);
/* The same, and dgamma_acc / dbeta_acc (nullable: the parameters' existing .grad) += dgamma / dbeta
 * (autograd's accumulation fused into the kernel that forms the sums; dgamma / dbeta stay outputs). */
int srk_batchnorm_bwd16_acc(const float* x, const float* y, const float* dy, int64_t M, int64_t C,
                            const float* gamma, const float* save_mean, const float* save_invstd, int training,
                            int relu, float* dx, void* dx16, int* dx16_written, float* dgamma, float* dbeta,
                            float* dresidual, float* dgamma_acc, float* dbeta_acc, void* stream);
/* The ReLU as bits: with relu set, fwd16_mask also writes relu_mask (M*C/4 bytes; byte i holds bit e = y[4i+e] > 0,
 * nullable), and bwd16_mask takes that mask in place of y (y may then be null) — the backward's two reads of the
 * ReLU pattern are 1/16 of y's bytes.  Otherwise as fwd16 / bwd16_acc, whose results they equal bit for bit. */
int srk_batchnorm_fwd16_mask(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                             float momentum, int training, float* running_mean, float* running_var,
                             const float* residual, int relu, float* y, void* y16, int* y16_written,
                             uint8_t* relu_mask, float* save_mean, float* save_invstd, void* stream);
int srk_batchnorm_bwd16_mask(const float* x, const float* y, const uint8_t* relu_mask, const float* dy, int64_t M,
                             int64_t C, const float* gamma, const float* save_mean, const float* save_invstd,
                             int training, int relu, float* dx, void* dx16, int* dx16_written, float* dgamma,
                             float* dbeta, float* dresidual, float* dgamma_acc, float* dbeta_acc, void* stream);
/* SyncBatchNorm pieces (torch.nn.SyncBatchNorm semantics: training statistics over the global
 * batch of all data-parallel ranks; model_resnet_bgru.py's BatchNorm1d layers under DP).  Forward:
 * srk_batchnorm_stats (this rank's count, mean, M2 per channel -> stats [3][C]), the caller gathers
 * every rank's triple ([world][3][C], rank order), srk_batchnorm_combine (Chan's combination in rank
 * order: identical on every rank; running stats with the global unbiased variance; total_count [1]
 * = the global row count, nullable), then
 * srk_batchnorm_apply.  Backward: srk_batchnorm_bwd_reduce (this rank's sums [2][C] = sum g,
 * sum g * xhat, g = dy * act'(y): also its dbeta / dgamma contributions), the caller sums them over
 * ranks, srk_batchnorm_bwd_dx with the combine's total_count (device).  The C-ABI replaces the fused
 * srk_batchnorm_fwd / _bwd statistics step only; layouts as srk_batchnorm_fwd.                    */
int srk_batchnorm_stats(const float* x, int64_t M, int64_t C, float* stats, void* stream);
int srk_batchnorm_combine(const float* stats_all, int world, int64_t C, float eps, float momentum,
                          float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                          float* total_count, void* stream);
int srk_batchnorm_apply(const float* x, int64_t M, int64_t C, const float* save_mean, const float* save_invstd,
                        const float* gamma, const float* beta, const float* residual, int relu, float* y,
                        void* stream);
int srk_batchnorm_bwd_reduce(const float* x, const float* y, const float* dy, int64_t M, int64_t C,
                             const float* save_mean, const float* save_invstd, int relu, float* sums, void* stream);
int srk_batchnorm_bwd_dx(const float* x, const float* y, const float* dy, int64_t M, int64_t C,
                         const float* total_count, const float* gamma, const float* save_mean,
                         const float* save_invstd, const float* sums, int relu, float* dx, float* dresidual,
                         void* stream);

/* ---------------------------------------------------------------- K7/K8: step ops
 * Cross-entropy, mean over the batch (nn.CrossEntropyLoss, training.py:73,87):
 * loss[0] = mean_b(logsumexp(logits_b) - logits_b[label_b]); dlogits (nullable) =
 * (softmax - onehot) / B.  ws: B + 1 floats.  An out-of-range label makes the loss NaN.     */
int srk_cross_entropy(const float* logits, const int64_t* labels, int64_t B, int64_t C, float* loss,
                      float* dlogits, float* ws, void* stream);
/* torch.optim.Adam step (no weight decay / amsgrad) over n contiguous floats (training.py:74,91);
 * step is the 1-based step count after increment; grad is multiplied by grad_scale first.   */
int srk_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                  float beta1, float beta2, float eps, int64_t step, float grad_scale, void* stream);
/* The same step with its per-step values on the device, so a captured HIP graph can replay it:
 * state is a 4-int64 (32-B) device buffer — int64 step, then floats bc1, sqrt(bc2), lr, 0.  The
 * caller writes lr (float, byte offset 16); the call advances the step and derives the bias
 * corrections on the device (double precision, as srk_adam_step's host side).                    */
int srk_adam_step_state(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float beta1,
                        float beta2, float eps, int64_t* state, float grad_scale, void* stream);
/* Loss scaling for 16-bit training (torch.cuda.amp.GradScaler semantics, on the device so a
 * captured step replays it).  scaler: 8 x 32-bit device words {float scale, float 1/scale, float
 * growth, float backoff, int found_inf, int good_steps, int growth_interval, int overflows};
 * growth_interval 0 = static scale.  The caller multiplies the loss by scale (word 0) before
 * backward.  No reference counterpart: the reference trains fp32 only (training.py:85-91).       */
int srk_grad_scaler_init(int32_t* scaler, float init_scale, float growth_factor, float backoff_factor,
                         int growth_interval, void* stream);
/* srk_adam_step_state on loss-scaled gradients: one pass flags any non-finite gradient element;
 * if one is found the step is SKIPPED (parameters, moments and the step count unchanged), the
 * overflow counter (word 7) advances and a dynamic scale backs off; otherwise the gradients are
 * multiplied by grad_scale / scale inside the update and a dynamic scale grows after
 * growth_interval clean steps.                                                                    */
int srk_adam_step_scaled(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float beta1,
                         float beta2, float eps, int64_t* state, float grad_scale, int32_t* scaler, void* stream);
/* nn.Dropout(p) training forward: keep[i] = Bernoulli(1-p) from a counter-based hash of
 * (seed, i) (not torch's RNG stream), y = keep ? x / (1-p) : 0.                              */
int srk_dropout_fwd(const float* x, int64_t n, float p, uint64_t seed, float* y, uint8_t* keep, void* stream);
/* srk_dropout_fwd with its seed on the device: state = uint64[2] {base, counter}; the mask hashes
 * base + counter * odd constant, then the call advances state[1] (graph-replayable; nn.Dropout,
 * model_fbanks_cnn.py:79,98).                                                                    */
int srk_dropout_fwd_state(const float* x, int64_t n, float p, uint64_t* state, float* y, uint8_t* keep,
                          void* stream);
/* y = keep ? x * scale : 0 (dropout with an explicit keep-mask; also its backward).          */
int srk_dropout_apply(const float* x, const uint8_t* keep, int64_t n, float scale, float* y, void* stream);

/* ---------------------------------------------------------------- diagnostics (tests only)
 * Directed checks of two instruction patterns (csrc/diag.hip; tests/test_diag_gpu.py):
 * srk_diag_acc_store: the row-staged data gradient's epilogue (raw buffer stores of 32x32 MFMA
 *   accumulators, its descriptor, offsets and drop value) into dx [rows][40][64] fp32 (rows % 8 == 0):
 *   tile g's first 32 pixels get 1 + 64 p + c + 2048 g; variant 0 = the product form, 1 = the round-5
 *   source form (a bit cast of a vector-component lvalue, miscompiled to component 0).
 * srk_diag_tr16_read: ds_read_b64_tr_b16 B fragments of a [32 k][cols] 16-bit matrix m staged as the
 *   64-column (cols = 64) or the 128-column TR image: out[(fragment * 64 + lane) * 4 + d], fragments
 *   (r0 = 0, 32, ...) x (kk = 0, 16). */
int srk_diag_acc_store(float* dx, int64_t rows, int variant, void* stream);
int srk_diag_tr16_read(const uint16_t* m, int64_t cols, uint32_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SRK_H_ */
