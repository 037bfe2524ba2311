/* C-level smoke test of libwhisper_mi355 through its C-ABI only (include/whisper_mi355.h), as a non-Python host
 * (cgo / JNI / plain C) would bind it.  Built twice by tools/capi/Makefile: against the normal library, and with
 * host-side AddressSanitizer + UndefinedBehaviorSanitizer on the library's host C++ and on this program
 * (hipcc -Xarch_host -fsanitize=...; device code is not instrumented).
 *
 * Without a GPU it checks the error contract (-1 + wm_last_error, never an abort).  With a GPU it builds a
 * tiny-dims engine, enumerates and uploads every weight (wm_weight_count / wm_weight_info) with small
 * deterministic values, then runs log-mel -> encode -> cross-KV -> greedy generate -> forward -> align and
 * checks return codes and output ranges.  Exit 0 = pass. */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/whisper_mi355.h"

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    if ((x) != 0) {                                                                                \
      fprintf(stderr, "FAIL %s:%d %s: %s\n", __FILE__, __LINE__, #x, wm_last_error());            \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)
#define HCHECK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "FAIL %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

static uint32_t rng_state = 12345u;
static float frand(void) {            /* xorshift32 in [-1, 1) */
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 17;
  rng_state ^= rng_state << 5;
  return (float)(rng_state >> 8) / 8388608.0f - 1.0f;
}
static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

int main(void) {
  /* the error contract, no GPU needed */
  wm_model_dims bad;
  memset(&bad, 0, sizeof(bad));
  wm_engine* e = NULL;
  if (wm_create(&bad, 0, &e) == 0 || e != NULL || strlen(wm_last_error()) == 0) {
    fprintf(stderr, "FAIL: wm_create accepted zero dims\n");
    return 1;
  }
  if (wm_set_weight(NULL, "x", NULL, 0, NULL) == 0 || wm_weight_count(NULL) != 0) {
    fprintf(stderr, "FAIL: NULL engine accepted\n");
    return 1;
  }
  wm_destroy(NULL);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    printf("capi_smoke: error contract ok; no GPU, device part skipped\n");
    return 0;
  }

  /* tiny: 80 mels, d 384, 6 heads, 4 + 4 layers, multilingual vocabulary */
  wm_model_dims d = {80, 384, 6, 4, 4, 51865, 1500, 448, 50257, 50258, 50362, 50363, 50364, 220};
  CHECK(wm_create(&d, 0, &e));
  const int32_t nw = wm_weight_count(e);
  for (int32_t i = 0; i < nw; ++i) {
    const char* name = NULL;
    int64_t nbytes = 0;
    int32_t elem = 0;
    CHECK(wm_weight_info(e, i, &name, &nbytes, &elem));
    void* host = malloc((size_t)nbytes);
    const int ln_gain = strstr(name, "ln") && name[strlen(name) - 1] == 'w';
    if (elem == 2) {
      uint16_t* h = (uint16_t*)host;
      for (int64_t k = 0; k < nbytes / 2; ++k) h[k] = f2bf(0.02f * frand());
    } else {
      float* h = (float*)host;
      for (int64_t k = 0; k < nbytes / 4; ++k) h[k] = ln_gain ? 1.0f : 0.02f * frand();
    }
    void* dev = NULL;
    HCHECK(hipMalloc(&dev, (size_t)nbytes));
    HCHECK(hipMemcpy(dev, host, (size_t)nbytes, hipMemcpyHostToDevice));
    CHECK(wm_set_weight(e, name, dev, nbytes, NULL));
    HCHECK(hipDeviceSynchronize());
    HCHECK(hipFree(dev));
    free(host);
  }
  if (!wm_weights_complete(e)) {
    fprintf(stderr, "FAIL: weights incomplete after uploading %d\n", nw);
    return 1;
  }
  if (wm_set_weight(e, "no.such.weight", NULL, 4, NULL) == 0) {
    fprintf(stderr, "FAIL: unknown weight accepted\n");
    return 1;
  }

  /* 12 s of a synthetic signal -> log-mel of the whole file */
  const int64_t n = 16000 * 12;
  float* hp = (float*)malloc(n * 4);
  for (int64_t i = 0; i < n; ++i) hp[i] = 0.1f * sinf(2.0f * 3.14159265f * 220.0f * (float)i / 16000.0f) + 0.01f * frand();
  float *dp, *dmel;
  uint32_t* dg;
  const int32_t frames = (int32_t)(n / 160 + 1);
  HCHECK(hipMalloc((void**)&dp, n * 4));
  HCHECK(hipMalloc((void**)&dmel, (size_t)d.n_mels * frames * 4));
  HCHECK(hipMalloc((void**)&dg, 4));
  HCHECK(hipMemset(dg, 0, 4));
  HCHECK(hipMemcpy(dp, hp, n * 4, hipMemcpyHostToDevice));
  CHECK(wm_logmel(e, dp, 0, n, 0, frames, dmel, frames, dg, NULL));
  float gmax = 0.f;
  CHECK(wm_logmel_finalize(e, dmel, frames, frames, dg, NULL, &gmax, NULL));

  /* encode one window (pad_or_trim to 3000 frames) and make it slot 0 */
  void* denc;
  HCHECK(hipMalloc(&denc, (size_t)1500 * d.n_state * 2));
  const int32_t seek = 0, nf = frames - 1;
  CHECK(wm_encode(e, dmel, frames, &seek, &nf, 1, denc, NULL));
  CHECK(wm_reserve(e, 1, 5, NULL));
  CHECK(wm_cross_kv(e, denc, 1, 0, NULL));

  /* greedy generate, 32 tokens max */
  const int32_t prompt[3] = {d.sot, 50259, 50359};
  const int32_t sup[2] = {50359, 50358};
  int32_t toks[32], len = 0, steps = 0, slot = 0;
  float score = 0.f, cum = 0.f, nsp = 0.f;
  wm_generate_args g;
  memset(&g, 0, sizeof(g));
  g.n_windows = 1; g.h_slots = &slot; g.prompt_len = 3; g.h_prompts = prompt; g.sot_index = 0; g.beam_size = 1;
  g.patience = 1.f; g.length_penalty = 1.f; g.max_length = 32; g.temperature = 0.f; g.num_hypotheses = 1;
  g.h_suppress = sup; g.n_suppress = 2; g.suppress_blank = 1; g.max_initial_timestamp_index = 50;
  g.with_timestamps = 1; g.check_every = 4; g.h_tokens = toks; g.h_lengths = &len; g.h_scores = &score;
  g.h_cum_logprob = &cum; g.h_no_speech = &nsp; g.h_steps = &steps;
  CHECK(wm_generate(e, &g, NULL));
  if (len < 0 || len > 32 || !(nsp >= 0.f && nsp <= 1.f) || !isfinite(score)) {
    fprintf(stderr, "FAIL: generate output len %d no_speech %f score %f\n", len, nsp, score);
    return 1;
  }
  for (int i = 0; i < len; ++i)
    if (toks[i] < 0 || toks[i] >= d.n_vocab) {
      fprintf(stderr, "FAIL: token %d out of range\n", toks[i]);
      return 1;
    }

  /* beam 5 on the same slot */
  g.beam_size = 5;
  CHECK(wm_generate(e, &g, NULL));

  /* teacher-forced logits of the prompt */
  float* dl;
  HCHECK(hipMalloc((void**)&dl, (size_t)3 * d.n_vocab * 4));
  CHECK(wm_forward(e, 1, &slot, 3, prompt, dl, 0, NULL, 0, NULL, NULL));

  /* alignment of a few text tokens against the window */
  const int32_t text[4] = {1000, 2000, 3000, 4000}, heads[4] = {2, 0, 3, 1};
  float probs[4];
  int32_t ti[1600], tj[1600], plen = 0;
  const int32_t sot3[3] = {d.sot, 50259, 50359};
  CHECK(wm_align(e, 0, 3, sot3, 4, text, 1200, heads, 2, 7, probs, ti, tj, &plen, NULL));
  if (plen <= 0 || plen > 1600) {
    fprintf(stderr, "FAIL: align path length %d\n", plen);
    return 1;
  }
  HCHECK(hipDeviceSynchronize());
  HCHECK(hipFree(dl));
  HCHECK(hipFree(denc));
  HCHECK(hipFree(dp));
  HCHECK(hipFree(dmel));
  HCHECK(hipFree(dg));
  free(hp);
  wm_destroy(e);
  printf("capi_smoke: ok (%d weights, %d tokens, %d steps, gmax %.3f, align path %d)\n", nw, len, steps, gmax, plen);
  return 0;
}
