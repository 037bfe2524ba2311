/* whisper_mi355.h — C-ABI of the MI355X (gfx950) Whisper engine, libwhisper_mi355.so.
 *
 * The drop-in boundary is faster-whisper's `WhisperModel(...).transcribe(...)` as the vlog transcription
 * worker calls it (reference `worker/transcription.py:78-111`).  Below that call, faster-whisper drives
 * CTranslate2's C++ `models.Whisper` (encode / generate / detect_language / align) [FW↑]; this library
 * replaces that C++ seam, plus faster-whisper's numpy log-mel.  The Python host (vlog_amd/) mirrors the
 * faster-whisper surface on top of these entry points and owns all input/output device buffers
 * (PyTorch-ROCm tensors); the engine owns the weights, the KV caches and its scratch.
 *
 * Conventions: every function returns 0 on success and -1 on failure (never aborts); the message is
 * available from wm_last_error() (thread-local).  Every call sets the engine's device itself, so calls may
 * come from any thread (the worker runs `transcribe` on a ThreadPoolExecutor thread,
 * worker/transcription.py:361-369); calls on one engine are serialised by an internal lock.  Pointers
 * named d_* are device pointers; h_* are host pointers.  `stream` is a hipStream_t (NULL = null stream).
 */
#ifndef WHISPER_MI355_H
#define WHISPER_MI355_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wm_engine wm_engine;

typedef struct wm_model_dims {
  int32_t n_mels, n_state, n_head, n_enc_layer, n_dec_layer, n_vocab, n_audio_ctx, n_text_ctx;
  int32_t eot, sot, no_speech, no_timestamps, timestamp_begin, blank;
} wm_model_dims;

/* Replaces ctranslate2.models.Whisper(model_path, device, compute_type) as constructed by
 * faster_whisper.WhisperModel.__init__ [FW↑] (called at worker/transcription.py:81-85). */
int wm_create(const wm_model_dims* dims, int32_t device, wm_engine** out);
void wm_destroy(wm_engine* e);
const char* wm_last_error(void);
int32_t wm_abi_version(void);

/* Weight upload into the engine's packed layout (names and layouts: see INTEGRATION.md §Weights).
 * d_src must hold exactly nbytes (bf16 matrices, f32 vectors). */
int wm_set_weight(wm_engine* e, const char* name, const void* d_src, int64_t nbytes, void* stream);
/* 1 when every weight has been set. */
int32_t wm_weights_complete(wm_engine* e);
/* The weights wm_set_weight expects, in layout order (for bindings that do not carry this table, e.g. a C or
 * Go host): name (owned by the engine), size in bytes, element bytes (2 = bf16 matrix, 4 = f32). */
int32_t wm_weight_count(wm_engine* e);
int wm_weight_info(wm_engine* e, int32_t i, const char** name, int64_t* nbytes, int32_t* elem_bytes);

/* Log-mel, replacing faster-whisper FeatureExtractor.__call__ [FW↑] (reached from
 * worker/transcription.py:105).  Computes frames [frame0, frame0+n_frames) of the WHOLE-FILE spectrogram
 * (file of n_samples samples; d_pcm[i] is file sample pcm_offset+i) as log10(max(mel, 1e-10)) into
 * d_mel[m*ld + f], and folds their maximum into *d_gmax (order-preserving uint32, zero-initialised by the
 * caller).  frame0 must be even: frames are transformed in (even, odd) pairs, so any split of a file into
 * even-aligned frame ranges gives bit-identical frames.  wm_logmel_finalize applies max(x, gmax-8), (x+4)/4
 * in place; gmax is taken from h_gmax when non-NULL (cross-shard max), else from d_gmax. */
int wm_logmel(wm_engine* e, const float* d_pcm, int64_t pcm_offset, int64_t n_samples, int64_t frame0,
              int32_t n_frames, float* d_mel, int64_t ld, uint32_t* d_gmax, void* stream);
int wm_logmel_finalize(wm_engine* e, float* d_mel, int64_t n_frames, int64_t ld, const uint32_t* d_gmax,
                       const float* h_gmax, float* h_gmax_out, void* stream);

/* Streaming ingest: n s16le samples (the worker's ffmpeg output, received through a pipe into a pinned
 * buffer and copied to the device) -> f32 x / 32768, faster-whisper decode_audio's conversion.  The caller
 * then runs wm_logmel on the frames whose window lies inside the samples received so far (vlog_amd/ingest.py). */
int wm_pcm_from_s16(wm_engine* e, const int16_t* d_src, int64_t n, float* d_dst, void* stream);

/* Per-frame log energy (dB) of ceil(n_samples / frame) frames, the speech-probability input of the VAD
 * stand-in (faster-whisper's Silero VAD [FW↑], reached via vad_filter=True at worker/transcription.py:110). */
int wm_frame_energy(wm_engine* e, const float* d_pcm, int64_t n_samples, int32_t frame, float* d_db, void* stream);

/* The fp8 cross memory's quantisation (wm_set_option "cross_fp8"), exposed for tests: rows of n_state bf16
 * values -> OCP e4m3 codes of x * 448 / amax_row (round to nearest even) and scale amax_row / 448 per row
 * (an all-zero row: zeros, scale 0).  wm_cross_kv applies it to the window slots when cross_fp8 is on. */
int wm_cross_fp8_quantize(wm_engine* e, const void* d_enc, int64_t rows, uint8_t* d_codes, float* d_scale, void* stream);

/* Silero VAD v5 (16 kHz) network weights, f32 device pointers in PyTorch layouts: STFT basis [258][256],
 * encoder convs conv_w[i] [out][in][3] with (in, out) = (129,128), (128,64), (64,64), (64,128) and biases
 * [out], LSTMCell w_ih/w_hh [512][128] (gate order i, f, g, o) and b_ih/b_hh [512], head conv1x1 [128] + [1]. */
typedef struct wm_vad_weights {
  const float* stft_basis;
  const float* conv_w[4];
  const float* conv_b[4];
  const float* w_ih;
  const float* w_hh;
  const float* b_ih;
  const float* b_hh;
  const float* head_w;
  const float* head_b;
} wm_vad_weights;

/* Speech probability of each 512-sample window of d_pcm (n_samples a multiple of 512; the caller pads as
 * faster-whisper's get_speech_timestamps does), replacing faster-whisper 1.1 SileroVADModel.__call__ [FW↑
 * vad.py] — its batched encoder (each window prefixed with the previous window's last 64 samples, zeros for
 * the first) and its sequential LSTM decoder with h, c starting at zero.  d_work: 512 * n_samples/512 floats
 * of scratch; d_probs: n_samples/512 floats. */
int wm_vad_probs(wm_engine* e, const wm_vad_weights* w, const float* d_pcm, int64_t n_samples, float* d_work,
                 float* d_probs, void* stream);

/* Encoder, replacing ctranslate2 Whisper.encode(features) [FW↑] (faster-whisper generate_segments).
 * Window b reads mel frames [h_seek[b], h_seek[b]+h_nframes[b]) of d_mel (ld = frames per mel row) and
 * zero-pads to 3000 frames (faster-whisper pad_or_trim).  Output bf16 [B][1500][n_state]. */
int wm_encode(wm_engine* e, const float* d_mel, int64_t ld, const int32_t* h_seek, const int32_t* h_nframes,
              int32_t B, void* d_enc_out, void* stream);

/* Capacity of the decoder state: n_slots windows (encoder outputs, or cross-KV panels with cross_mode 0),
 * n_hyp hypotheses of self-KV. */
int wm_reserve(wm_engine* e, int32_t n_slots, int32_t n_hyp, void* stream);

/* Makes B encoder outputs the cross-attention memory of slots [slot0, slot0+B) (CTranslate2 projects them
 * to K/V inside generate [FW↑]).  Default (factored cross-attention): the slot keeps the encoder output
 * itself and the decoder attends over it (q' = Wk_h^T q, u = P E, Wv after the merge).  cross_mode 0: the
 * K/V projection of all decoder layers is computed here. */
int wm_cross_kv(wm_engine* e, const void* d_enc, int32_t B, int32_t slot0, void* stream);

/* ctranslate2 Whisper.generate(encoder_output, prompts, ...) [FW↑] as faster-whisper
 * generate_with_fallback calls it: all windows share one prompt length; greedy (beam_size 1,
 * temperature 0), beam search (beam_size > 1, patience, length_penalty) or sampling (temperature > 0,
 * num_hypotheses = best_of).  Logit rules, log-softmax and selection run on the device. */
typedef struct wm_generate_args {
  int32_t n_windows;
  const int32_t* h_slots;        /* [n_windows] cross-KV slot of each window */
  int32_t prompt_len;
  const int32_t* h_prompts;      /* [n_windows][prompt_len] */
  int32_t sot_index;             /* position of <|startoftranscript|> in the prompt; -1: no no_speech_prob */
  int32_t beam_size;
  float patience;
  float length_penalty;
  int32_t max_length;            /* total decoder length including the prompt (<= n_text_ctx) */
  float temperature;             /* > 0: sampling */
  int32_t num_hypotheses;        /* sampling: best_of */
  uint64_t seed;
  const int32_t* h_suppress;     /* suppressed token ids */
  int32_t n_suppress;
  int32_t suppress_blank;
  int32_t max_initial_timestamp_index;   /* < 0: none */
  int32_t with_timestamps;
  int32_t check_every;           /* steps between host checks for completion (>= 1) */
  /* outputs (host) */
  int32_t* h_tokens;             /* [n_windows][max_length] generated tokens (no prompt, no <|endoftext|>) */
  int32_t* h_lengths;            /* [n_windows] */
  float* h_scores;               /* [n_windows] cum_logprob / len^length_penalty (CTranslate2 score) */
  float* h_cum_logprob;          /* [n_windows] */
  float* h_no_speech;            /* [n_windows] */
  int32_t* h_steps;              /* [1] decoder steps run (incl. prefill) */
  /* ---- ABI 2 (wm_abi_version() >= 2) */
  /* Row-set decode (greedy, or sampling with num_hypotheses 1): at most max_rows windows decode at once (0: all);
   * when one ends, its row takes the next window in h_slots order at the next host check (the new window's prompt
   * is prefilled inside that step's decoder pass), so the step count follows the total work instead of the longest
   * window.  Order the windows longest-expected first (vlog_amd/shard.py expected_tokens).  compact = 1: once no
   * window is waiting, finished rows are dropped from the passes when the live rows fall to 7/8 of the pass (the
   * step graph is re-captured for the new row count).  Each window's result is the same computation either way;
   * the GEMM / attention routes follow the pass's row count, so results agree to f32 rounding, not bit for bit.
   * Beam search: max_rows (a multiple of beam_size is used: max_rows / beam_size windows in flight) refills a
   * finished window's group of beam_size rows with the next window (no per-step records in this form); compact = 1
   * drops the hypotheses of finished windows from the passes once nothing waits (when the live hypotheses fall to
   * 7/8 of the pass). */
  int32_t max_rows;
  int32_t compact;
  /* Optional per-step records, [n_windows][max_length] (NULL: off): the log-prob (after the logit rules) of the
   * token chosen at each generated step, the final <|endoftext|> included (h_lengths[w] + 1 entries when the window
   * ended on it, else h_lengths[w]); and, greedy / sampling, the best log-prob among the other allowed tokens at that
   * step.  Beam search records the chosen hypothesis' path. */
  float* h_token_logprobs;
  float* h_token_logprobs_other;
  /* Optional statistics [4] (NULL: off): decoder passes, sum over decode passes of the rows in the pass, windows
   * started after the first pass (refills), step graphs captured. */
  int64_t* h_stats;
} wm_generate_args;
/* Failure contract: a NaN / inf logits row or a row whose rules allow no token, detected on the device, fails the
 * call (-1, wm_last_error names the window and step) instead of emitting a token. */
int wm_generate(wm_engine* e, const wm_generate_args* a, void* stream);

/* Teacher-forced decoder forward over n_seq sequences of seq_len tokens (one window slot each): logits for
 * every position (d_logits f32 [n_seq*seq_len][n_vocab]) or only the last (last_only: [n_seq][n_vocab]).
 * Optional cross-attention capture for word alignment (ctranslate2 Whisper.align [FW↑]): for each of
 * n_align (layer, head) pairs in h_align_heads, softmax weights are written to
 * d_attn[((s*seq_len + p)*n_align + a)*1500 + t].  Also serves detect_language ([sot], last_only). */
int wm_forward(wm_engine* e, int32_t n_seq, const int32_t* h_slots, int32_t seq_len, const int32_t* h_tokens,
               float* d_logits, int32_t last_only, const int32_t* h_align_heads, int32_t n_align, float* d_attn,
               void* stream);

/* ctranslate2 Whisper.detect_language(encoder_output) [FW↑] (faster-whisper detect_language, reached from
 * worker/transcription.py:105-111 with language=None): one decoder step from <|startoftranscript|> for each of n
 * windows (slots h_slots), softmax over the n_langs language tokens starting at lang_begin, on the device.
 * h_probs [n][n_langs], in language-token order. */
int wm_detect_language(wm_engine* e, int32_t n, const int32_t* h_slots, int32_t lang_begin, int32_t n_langs,
                       float* h_probs, void* stream);

/* ctranslate2 Whisper.align(encoder_output, start_sequence, text_tokens, num_frames, median_filter_width)
 * [FW↑] for ONE window (faster-whisper find_alignment, word_timestamps=True): teacher-forced decoder pass over
 * h_sot + <|notimestamps|> + h_text + <|endoftext|> with the n_heads (layer, head) alignment heads'
 * cross-attention captured, text-token probabilities, z-score + median filter + head mean, DTW on the
 * device.  Outputs: h_probs[n_text], the DTW path (h_text_idx, h_time_idx) of *h_path_len entries
 * (capacity n_text + 1 + num_frames/2). */
int wm_align(wm_engine* e, int32_t slot, int32_t sot_len, const int32_t* h_sot, int32_t n_text, const int32_t* h_text,
             int32_t num_frames, const int32_t* h_heads, int32_t n_heads, int32_t median_filter_width, float* h_probs,
             int32_t* h_text_idx, int32_t* h_time_idx, int32_t* h_path_len, void* stream);
/* wm_align over a batch of windows (faster-whisper add_word_timestamps over a batch of segments, as the
 * batched pipeline runs it; one teacher-forced decoder pass per chunk of windows and one batched DTW launch
 * instead of one wm_align per window).  Item i: window slot h_slots[i], text tokens
 * h_text[h_text_off[i] .. h_text_off[i+1]), h_num_frames[i] mel frames.  Outputs: probabilities at
 * h_probs[h_text_off[i] + k]; DTW path of item i at h_text_idx / h_time_idx + h_path_off[i] (capacity
 * n_text_i + 1 + num_frames_i / 2), length h_path_len[i]. */
int wm_align_batch(wm_engine* e, int32_t n, const int32_t* h_slots, int32_t sot_len, const int32_t* h_sot,
                   const int32_t* h_text_off, const int32_t* h_text, const int32_t* h_num_frames, const int32_t* h_heads,
                   int32_t n_heads, int32_t median_filter_width, float* h_probs, const int64_t* h_path_off,
                   int32_t* h_text_idx, int32_t* h_time_idx, int32_t* h_path_len, void* stream);
/* DTW alone on a device cost matrix d_cost[n][m] (openai dtw semantics); path as for wm_align. */
int wm_dtw(wm_engine* e, const float* d_cost, int32_t n, int32_t m, int32_t* h_text_idx, int32_t* h_time_idx,
           int32_t* h_path_len, void* stream);

/* Encoder self-attention kernel alone (diagnostics / parity tests; wm_encode runs it per layer):
 * d_qkv bf16 [B][T][3 n_state] (q | k | v, head h at columns h*64), d_out bf16 [B][T][n_state]. */
int wm_encoder_attention(wm_engine* e, const void* d_qkv, void* d_out, int32_t B, int32_t T, void* stream);

/* Bytes of device memory held by the engine (weights + caches + scratch). */
int64_t wm_device_bytes(wm_engine* e);

/* Built-in kernel profiler (used by bench.py for the live roofline numbers): when enabled, every launch
 * of a kernel class is bracketed by HIP events on its own stream, and the class accumulates its
 * algorithmic FLOPs and bytes (the decoder attention kernels count the K/V bytes they actually read).
 * wm_profile(e, 1) resets and enables, wm_profile(e, 0) disables; wm_profile_read returns launches,
 * summed event time, FLOPs and bytes of one class. */
int32_t wm_profile_classes(void);
const char* wm_profile_name(int32_t cls);
int wm_profile(wm_engine* e, int32_t enable);
/* Engine options (no reference counterpart: scheduling knobs of this build only).
 *   "cross_mode" (default 1): 1 = factored cross-attention over the encoder output (attn_xenc.hip),
 *   0 = projected cross-KV panels (attn_dec.hip).  Switching re-allocates the window slots (their content is
 *   dropped: call wm_cross_kv again).  The two forms agree to bf16 rounding (not bit-identical).
 *   "decode_split" (default 0): decode steps with >= 32 rows run as two row slices on two streams, one
 *   slice's weight GEMMs overlapping the other's cross-attention.  Results are bit-identical
 *   either way; off by default because the overlap measured slower on MI355X (the GEMM blocks queue behind
 *   the cross-attention blocks).
 *   "decode_graph" (default 1): after one eager decode step, wm_generate captures a step (decoder pass +
 *   token selection) as a HIP graph and replays it for the remaining steps (every per-step quantity lives in
 *   device memory).  Bit-identical either way; off while the event profiler is on or with "decode_split".
 *   "decode_gemv" (default 1): passes of <= 32 decoder rows (one window's beam, a few windows) run every
 *   projection on the small-M weight-streaming GEMM (gemm_dec.hip gemv_dec_kernel); it agrees with the other
 *   routes to f32 rounding.  "decode_gemv_ln" (default 1): passes of <= 16 rows compute the LayerNorms after the
 *   out and cout projections inside the cq / fc1 GEMMs (from the residual and the per-tile row sums and sums of
 *   squares about the tile means that the producers write: a two-pass-equivalent variance) instead of two combine
 *   launches per layer; agrees with the unfused form to f32 rounding.  "decode_gemv_ln_fc2" (default 0): 1 = also
 *   fc2 writes the residual and its row statistics without split-K (16-wave blocks over K = 4 d) and the next layer's
 *   qkv GEMM applies ln1 to its operand (one combine launch fewer per layer; measured ~5 % slower per decoder pass).
 *   "decode_ring_gemm" (default 1): 0 disables the all-rows ring GEMM (plan value 0 below falls back to the
 *   split-K skinny GEMM).
 *   "decode_gemm_plan" (default 1): preset routing of the six decoder projections (qkv, out, cq, cout, fc1, fc2)
 *   for passes of <= 1024 rows; 0 = round-1 routing (ring for qkv/fc1, skinny split-K for the rest), 1 = the
 *   per-projection fastest at 150 rows (tools/dec_gemm_bench; fc1 and fc2 as 64 x 64 ring tiles).  "decode_gemm.<proj>" sets one projection:
 *   > 0 ring GEMM with the rows in groups of that many, 0 all-rows ring, -1 skinny split-K, -2 one-shot GEMM.
 *   Routes differ in K summation order (results agree to f32 rounding, not bit for bit).
 *   "decode_gemm_cols.<proj>" (preset 1: 64 for fc1 and fc2, else 32): output columns per ring-GEMM block, 32 or 64 (64
 *   takes row groups of at most 64; other routes ignore it).  Bit-identical either way.  decode_gemm_plan also
 *   resets these to its preset.
 *   "decode_gemm_big_rows" (default 161): passes of at least this many rows (<= 1024; beam groups of many windows)
 *   route every projection to 64-row ring groups over its whole K (64 columns for qkv / fc1 / fc2, and for all from
 *   512 rows; 0 disables).  Results agree to f32 rounding.
 *   "decode_gemm_big128" (default 512; 0 = never): passes of at least this many rows on that route take the 8-wave
 *   plan: qkv, fc1 and fc2 as 128-row x 128-column blocks, the d x d projections as 64 x 64 (one block of 8 waves per
 *   CU).  Bit-identical to the 4-wave route (same K order per row) except fc2's K ranges below.
 *   "decode_gemm_big_fc2_kr" (default 1280): fc2's K range per block on the 8-wave plan (0 = the whole K, bit-identical
 *   to the 4-wave route; a split sums its slabs in the residual + LayerNorm combine: f32 rounding).
 *   "decode_gemm_big_lds" (default 72): LDS budget in KiB of the qkv / fc1 / fc2 ring blocks on that route, 72 (two
 *   resident blocks per CU) or 144 (one; the d x d projections always take 144).  Bit-identical either way.
 *   "decode_ln_fold" (default 0; measured slower, kept for A/B): passes of 33..1024 rows whose projections all take the ring route fold each
 *   pre-LayerNorm into its consumer: the residual producer writes bf16(x * gamma) and row sums, the consumer's
 *   epilogue applies rstd * acc - rstd * mean * (W gamma) + (W beta + bias), so no LayerNorm launch follows out and
 *   cout.  Results agree with 0 to the bf16 rounding of a different operand (not bit for bit).
 *   "align_fused" (default 1, process-wide): word alignment's z-score + median filter as one statistics kernel and
 *   one wave-per-row-segment median kernel that recomputes z from the attention (never stored); 0 runs the two-kernel
 *   form that writes z.  Bit-identical.
 *   "gemm_persistent" (default 0, process-wide): 1 runs large encoder GEMMs as one persistent block per CU
 *   walking its tiles, the next tile's first K-tiles loaded during the current tile's last K-steps and epilogue
 *   (measured no faster than one block per tile).  Bit-identical.
 *   "cross_attn_keep" (default 0): the factored cross-attention loads the encoder output of the first that many
 *   windows with the default cache policy and the rest non-temporally (an Infinity Cache residency experiment;
 *   measured no gain).  Bit-identical.
 *   "cross_attn_snake" (default 0): odd decoder layers walk the factored cross-attention's items in reverse, so
 *   the encoder output read last by one layer is read first by the next (Infinity Cache reuse).  Bit-identical.
 *   "cross_attn_dma" (default 0): 1 = at n_state 1280 with bf16 cross memory, the factored cross-attention streams the
 *   encoder output straight into LDS (LDS-DMA, two tiles ahead); 0 runs the register-staged form.  Bit-identical on
 *   key-split items; measured slower in the bench step.
 *   "cross_attn_chunks" (default 0): 1 = at n_state 1280, greedy passes cut their (window, 32-position tile) units into
 *   one contiguous chunk per CU (stream-K) instead of per-window key splits (the register form runs a chunk's
 *   segments as work items, the LDS-DMA form walks a chunk per workgroup; the two give the same bits); the pieces
 *   of a window are merged like key splits, so results agree with the key-split cut to f32 rounding, not bit for
 *   bit.  Measured slower at the headline's 150 windows.
 *   "cross_attn_blocks" (default 0): grid cap of the cross-attention kernel, which walks its
 *   (window, head, key split) items with a grid stride; 0 launches one block per item.
 *   "cross_attn_fuse" (default 1): bit 0 folds the cq projection's split-K combine into the cross-attention
 *   kernel's q load (the q' kernel's, in the factored form); bit 1 combines the key splits in-kernel (last-arriving split) instead of a combine
 *   launch.  Every setting of these three knobs gives bit-identical results.
 *   "encode_chunk" (default 160): windows per encoder pass inside wm_encode (~52 MB of activation scratch
 *   per large-v3 window).
 *   "cross_fp8" (default 0): opt-in fp8 (OCP e4m3) cross memory in the factored form (changes numerics).
 *   "cross_tf" (default 1): the teacher-forced passes of wm_align / wm_align_batch (projected form) run the
 *   cross-attention on the matrix cores (bf16 MFMA, f32 scores and captured probabilities; the attention weights
 *   enter the V product as bf16); 0 = the f32 VALU kernels of the decode path.
 *   "cross_mfma" (default 1): projected form, decode passes whose windows have 2..32 rows (beam hypotheses, prompt
 *   prefill) run the cross-attention on the same matrix-core kernel, the keys split over blocks to fill the chip and
 *   merged by the split-combine kernel; 0 = the f32 VALU group kernel.  Changes numerics at bf16-rounding level.
 *   "cross_mfma_fuse" (default 0): 1 = that merge done inside the kernel by the last-arriving key split (same
 *   arithmetic and order, bit-identical output; measured ~6 % slower per cross-attention than the separate kernel).
 *   "debug_nan_row" (default -1, TEST ONLY): >= 0 overwrites logits row r of every decode pass of wm_generate with
 *   NaN before token selection (exercises the failure contract of wm_generate).
 *   "debug_nan_count" (default 1, TEST ONLY): the number of consecutive rows from "debug_nan_row" (a whole beam group
 *   gives that window no live candidate). */
int wm_set_option(wm_engine* e, const char* key, int64_t value);
/* The engine's current value of an option (every key wm_set_option accepts, incl. environment overrides). */
int wm_get_option(wm_engine* e, const char* key, int64_t* value);
/* As wm_profile(e, 1) but only the classes whose bit is set in class_mask are timed (0 disables), so a
 * timed run can keep events on the dominant kernel alone. */
int wm_profile_select(wm_engine* e, uint32_t class_mask);
int wm_profile_read(wm_engine* e, int32_t cls, int64_t* launches, double* ms, double* flops, double* bytes);

#ifdef __cplusplus
}
#endif
#endif
