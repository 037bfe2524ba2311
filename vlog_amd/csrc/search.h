#pragma once
#include "common.h"

#define SEARCH_SB 1024           // threads per logits row (logits_select_kernel)
#define SEARCH_PER 52            // ids per thread: vocab <= SEARCH_SB * SEARCH_PER = 53248

struct SearchParams {
  const float* logits;   // [rows][V] f32, row r belongs to hypothesis r
  long long ldl;
  int V;
  int* tokens;           // [n_hyp][n_ctx] full sequences (prompt + generated)
  int n_ctx;
  int* seq_len;          // [n_hyp]
  int sample_begin;      // prompt length
  // suppressed ids as per-thread bit words: bit k of word t <=> id t + k * SEARCH_SB is suppressed (or >= V); one
  // 8-B load per thread instead of one dependent byte load per element (search_suppress_bits builds it)
  const unsigned long long* suppress_bits;   // [SEARCH_SB]
  int suppress_blank, blank, eot, no_timestamps, ts_begin, max_initial;   // max_initial < 0: none
  int with_ts;
  int* done;             // [n_hyp]
  int mode;              // 0 greedy, 1 beam candidates, 2 sampling
  int topk;              // beam: beam_size + 1
  float inv_temperature;
  unsigned long long seed;
  int step;
  int max_length;
  int abl;               // diagnostics (VLOG_AMD_SEL_ABL): bit 1 = beam top-k by K rounds over the row
  // greedy / sampling state (updated in place)
  float* cum;            // [n_hyp]
  int* row_tok; int* row_pos;      // next step's decoder input per hypothesis
  int* n_active;         // decremented when a hypothesis finishes
  // beam outputs
  int* cand_tok; float* cand_lp;   // [n_hyp][topk]
};

struct BeamParams {
  int beam, max_cand, n_ctx, sample_begin, max_length, eot;
  const int* cand_tok; const float* cand_lp;
  int* tokens; int* lin; int* seq_len; float* cum; int* done;
  int* row_tok; int* row_pos;
  int* fin_tok;          // [n_win][max_cand][n_ctx]  (generated tokens only)
  int* fin_len; float* fin_cum; int* n_fin;   // [n_win][max_cand], [n_win]
  int* n_active;
};

void launch_logits_select(const SearchParams& p, int n_hyp, hipStream_t st);
// host: the suppress_bits words for a vocabulary of V ids (sup[i] != 0: suppressed)
void search_suppress_bits(const unsigned char* sup, int V, unsigned long long* bits /* [SEARCH_SB] */);
void launch_beam_select(const BeamParams& p, int n_win, hipStream_t st);
void launch_no_speech(const float* logits, long long ldl, int V, int rows, int no_speech, float* out, hipStream_t st);
