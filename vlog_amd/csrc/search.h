#pragma once
#include "common.h"

struct SearchParams {
  const float* logits;   // [rows][V] f32, row r belongs to hypothesis r
  long long ldl;
  int V;
  int* tokens;           // [n_hyp][n_ctx] full sequences (prompt + generated)
  int n_ctx;
  int* seq_len;          // [n_hyp]
  int sample_begin;      // prompt length
  const unsigned char* suppress;   // [V] 1 = suppressed
  int suppress_blank, blank, eot, no_timestamps, ts_begin, max_initial;   // max_initial < 0: none
  int with_ts;
  int* done;             // [n_hyp]
  int mode;              // 0 greedy, 1 beam candidates, 2 sampling
  int topk;              // beam: beam_size + 1
  float inv_temperature;
  unsigned long long seed;
  int step;
  int max_length;
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
void launch_beam_select(const BeamParams& p, int n_win, hipStream_t st);
void launch_no_speech(const float* logits, long long ldl, int V, int rows, int no_speech, float* out, hipStream_t st);
