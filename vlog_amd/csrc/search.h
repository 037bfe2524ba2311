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
  // compacted row set (nullptr: row r is hypothesis r): block r reads logits row r and decodes hypothesis
  // row_hyp[r]; row_tok / row_pos are written per ROW (the next pass's inputs), the rest per hypothesis
  const int* row_hyp;
  // device error word (nullptr: none): [0] code (1 non-finite logits row, 2 no legal token), [1] hypothesis,
  // [2] tokens sampled before the failing step; the first failure wins (wm_report_error)
  int* err;
  // optional per-step records [n_hyp][n_ctx] (nullptr: off): log-prob of the token chosen at sequence position
  // len (the final <|endoftext|> included) and, greedy / sampling, the best log-prob among the other allowed tokens
  float* tok_lp;
  float* tok_lp_other;
  // results of finished hypotheses by OUTPUT id (greedy / sampling: the row-set decode, whose hypothesis slots are
  // reused; nullptr: the host reads the hypothesis tables): written by the block that ends the hypothesis
  const int* hyp_out;              // [n_hyp] output id of the hypothesis in each slot
  int* res_tok; int* res_len; float* res_cum;   // [n_out][n_ctx] generated tokens (no prompt), [n_out], [n_out]
  float* res_lp;                   // [n_out][n_ctx] per-step records (with tok_lp; nullptr: none)
  float* res_lp_other;
};

struct BeamParams {
  int beam, max_cand, n_ctx, sample_begin, max_length, eot;
  const int* cand_tok; const float* cand_lp;
  int* tokens; int* lin; int* seq_len; float* cum; int* done;
  int* row_tok; int* row_pos;
  int* fin_tok;          // [n_win][max_cand][n_ctx]  (generated tokens only)
  int* fin_len; float* fin_cum; int* n_fin;   // [n_win][max_cand], [n_win]
  int* n_active;
  // optional per-step records (nullptr: off): tok_lp [n_hyp][n_ctx] log-prob of the token at each position (copied
  // along the lineage like the tokens), fin_lp [n_win][max_cand][n_ctx] a finished hypothesis' records (generated
  // tokens, then its <|endoftext|>)
  float* tok_lp;
  float* fin_lp;
};

// Row-set decode bookkeeping (engine.cpp generate_rows).  Start hypotheses: slot hs[i] takes window ws[i] (prompt
// win_prompt[ws[i]][0..P) into tokens, seq_len P, live, cum 0, its cross slot and output id).
void launch_hyp_start(int n, const int* hs, const int* ws, const int* win_prompt, int P, const int* win_slot, int n_ctx,
                      int* tokens, int* seq_len, int* done, float* cum, int* hyp_slot, int* hyp_out, hipStream_t st);
// Pass rows whose token / position live on the device: row i with src[i] >= 0 takes (row_tok, row_pos)[src[i]].
void launch_rows_fill(int n, const int* src, int* tok, int* pos, const int* row_tok, const int* row_pos, hipStream_t st);
void launch_beam_start(int n, const int* gs, const int* ws, int K, const int* win_prompt, int P, const int* win_slot,
                       int n_ctx, int* tokens, int* lin, int* seq_len, int* done, float* cum, int* hyp_slot, int* n_fin,
                       hipStream_t st);

// one block per row (n_rows = hypotheses, or the compacted row set's rows with p.row_hyp)
void launch_logits_select(const SearchParams& p, int n_rows, hipStream_t st);
// host: the suppress_bits words for a vocabulary of V ids (sup[i] != 0: suppressed)
void search_suppress_bits(const unsigned char* sup, int V, unsigned long long* bits /* [SEARCH_SB] */);
void launch_beam_select(const BeamParams& p, int n_win, hipStream_t st);
// out[r][j] = softmax(logits row r restricted to [lang_begin, lang_begin + n_langs))[j]
void launch_lang_probs(const float* logits, long long ldl, int rows, int lang_begin, int n_langs, float* out, hipStream_t st);
// out[out_idx ? out_idx[r] : r] = softmax(logits row r)[no_speech]
void launch_no_speech(const float* logits, long long ldl, int V, int rows, int no_speech, float* out, hipStream_t st,
                      const int* out_idx = nullptr);
