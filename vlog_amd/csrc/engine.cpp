// libwhisper_mi355 engine: C-ABI (include/whisper_mi355.h) over the gfx950 kernels.
//
// Owns: the packed bf16/f32 weight arena, the encoder scratch, the decoder state (cross-KV slots, self-KV
// cache, token/lineage tables) and the decode loop.  Orchestration mirrors what CTranslate2's
// models::Whisper does below faster-whisper [FW↑] (encode -> generate with logit rules -> results), but the
// loop keeps everything on the device: per step one decoder pass (embed, L x {LN, QKV GEMM -> KV cache,
// self-attn, O GEMM+residual, LN, Q GEMM, cross-attn, O GEMM+residual, LN, FC1+GELU, FC2+residual}, final
// LN, tied-embedding logits GEMM) and one selection kernel; the host only polls an "active hypotheses"
// counter every `check_every` steps.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/whisper_mi355.h"
#include "gemm.h"
#include "search.h"
#include "vad.h"

// ---- launchers defined in the .hip files
void launch_logmel(const float*, long long, long long, long long, long long, int, const float*, const float*,
                   const float*, const float*, const int*, const int*, int, float*, long long, unsigned int*, hipStream_t);
void launch_logmel_clamp(float*, long long, long long, long long, const unsigned int*, const float*, hipStream_t);
void launch_ordered_to_float(const unsigned int*, float*, hipStream_t);
void launch_frame_energy(const float*, long long, int, int, float*, hipStream_t);
void launch_pcm_s16(const short*, long long, float*, hipStream_t);
void launch_layernorm(const float*, long long, const int*, int, int, const float*, const float*, bf16*, long long, hipStream_t);
void launch_embed(const int*, const int*, const bf16*, const float*, float*, int, int, int, int, hipStream_t, int*);
void launch_im2col_conv1(const float*, long long, const int*, const int*, int, int, int, bf16*, hipStream_t);
void launch_zero_pad_rows(bf16*, int, long long, int, hipStream_t);
void launch_attn_enc(const bf16*, bf16*, int, int, int, int, hipStream_t);
void launch_self_attn(const bf16*, long long, const bf16*, const bf16*, const int*, const int*, const int*, const int*,
                      bf16*, long long, int, int, int, unsigned long long*, hipStream_t, hipEvent_t, hipEvent_t, int, int);
void launch_cross_attn(const bf16*, long long, const bf16*, const bf16*, int, const int*, const int*, const int*, bf16*,
                       long long, int, int, int, float*, float*, float*, float*, const int*, int, int, int,
                       const CrossFuse&, unsigned long long*, hipStream_t, hipEvent_t, hipEvent_t);

// factored cross-attention over the encoder output (attn_xenc.hip)
void launch_xpack(const bf16*, bf16*, bf16*, int, int, int, hipStream_t);
void launch_xq(const bf16*, long long, const CrossFuse&, const bf16*, bf16*, int, int, int, hipStream_t);
int xattn_splits(int, int, int, int, int);
XPlan xattn_plan(int, int, int, int, int, bool);
void launch_xquant8(const bf16*, long long, int, unsigned char*, float*, hipStream_t);
long long xblock_slot_elems(int T, int d);
void launch_xblock(const bf16* src, int B, int T, int d, bf16* dst, bool to_blocked, hipStream_t st);
void launch_xattn(const bf16*, const void*, const float*, const int*, const int*, const int*, int, long long, int, int, int, int,
                  const XPlan&, int, int, int, int, bf16*, float*, float*, const int*, int, unsigned long long*, hipStream_t, hipEvent_t, hipEvent_t);
void launch_xcomb_vo(const bf16*, const float*, const XPlan&, int, long long, const bf16*, const float*, const int*, const int*,
                     bf16*, long long, int, int, int, int, int, float*, const int*, int, hipStream_t);

void launch_token_probs(const float*, int, int, int, const int*, float*, hipStream_t);
void launch_align_matrix(const float*, int, int, int, int, int, int, int, float*, float*, float*, hipStream_t);
void launch_align_matrix_batch(const float*, int, int, int, int, int, int, int, int, const int*, const int*, const int*,
                               const long long*, float*, double*, float*, hipStream_t);
void align_set_fused(int on);
int align_get_fused();
void launch_dtw(const float*, int, int, float*, signed char*, int*, int*, int*, hipStream_t);
void launch_dtw_batch(const float*, const long long*, const int*, const int*, float*, signed char*, const long long*,
                      int*, int*, const long long*, int*, int, hipStream_t);

// Kernel classes timed by the built-in profiler (wm_profile / wm_profile_read).
enum ProfClass {
  P_LOGMEL = 0, P_ENC_GEMM, P_ENC_ATTN, P_ENC_OTHER, P_CROSSKV_GEMM, P_DEC_GEMM, P_SELF_ATTN, P_CROSS_ATTN,
  P_LOGITS_GEMM, P_SELECT, P_DEC_OTHER, P_CROSS_COMB, P_N
};
static const char* kProfNames[P_N] = {"logmel", "enc_gemm", "enc_attn", "enc_other", "crosskv_gemm", "dec_gemm",
                                      "self_attn", "cross_attn", "logits_gemm", "select", "dec_other", "cross_comb"};

namespace {

thread_local std::string g_err;

#define HIP_OK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e__ = (x);                                                                          \
    if (e__ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e__)); \
  } while (0)

// Bumped whenever a device buffer moves: a captured step graph holds raw pointers, so a decode loop that
// captured one re-captures it when this changed (e.g. a refill pass that grew a scratch buffer).  The counter is
// PER ENGINE: `guarded` points t_realloc at the engine whose entry point runs on this thread (under its lock), so
// another engine's allocations neither force a re-capture nor fail a capture in progress.  Allocations outside an
// entry point (wm_create) count on a fallback no graph reads.
// Greedy row-set compaction threshold in eighths of the pass (VLOG_AMD_COMPACT_8THS, default 7): the live rows are
// packed once they fall to this many eighths of the pass's rows (a step-graph re-capture per compaction).  Variable
// workload, arms alternating on one box: 4/8 2605, 5/8 2644-2645, 6/8 2660-2672, 7/8 2680 RTFx, the same tokens
// (profiles/ab_r05_compact.txt): the cross-attention's items track the live windows more closely, and a re-capture
// costs less than the passes over finished rows it saves.
static int row_compact_8ths() {
  static const int v = [] {
    const char* e = std::getenv("VLOG_AMD_COMPACT_8THS");
    const int x = e ? std::atoi(e) : 7;
    return x >= 1 && x <= 7 ? x : 7;
  }();
  return v;
}

thread_local long long* t_realloc = nullptr;
long long g_realloc_none = 0;
inline long long& realloc_gen() { return t_realloc ? *t_realloc : g_realloc_none; }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) HIP_OK(hipFree(p));
    p = nullptr;
    bytes = 0;
    HIP_OK(hipMalloc(&p, b));
    bytes = b;
    ++realloc_gen();
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T* as() const { return (T*)p; }
};

struct Slot {
  size_t off, bytes;
  bool set = false;
  int elem = 2;              // element bytes: 2 = bf16 matrix, 4 = f32 vector / table
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// Decoder projections (index of wm_engine::dec_plan)
enum DecProj { DEC_QKV = 0, DEC_OUT, DEC_CQ, DEC_COUT, DEC_FC1, DEC_FC2, DEC_NPROJ };
static const char* kDecProjNames[DEC_NPROJ] = {"qkv", "out", "cq", "cout", "fc1", "fc2"};
// preset 1 (default): per-projection fastest at 150 rows (tools/dec_gemm_bench, then bench.py A/B).  Round 2:
// fc1 as 64-row x 64-column ring tiles (240 blocks of 320 KB instead of 160 of 480 KB: 12.4 -> 9.0 us) and fc2
// likewise (K split in 4 ranges of 1280, slabs summed by the residual+LayerNorm combine: 16.1 -> 13.8 us with the
// combine); bench.py on one box: dec_gemm 372 -> 352 (fc1) -> 341-343 ms/step (fc2).
static const int kDecPlanPresets[2][DEC_NPROJ] = {{0, -1, -1, -1, 0, -1}, {96, 32, 32, 32, 64, 64}};
static const int kDecColsPresets[2][DEC_NPROJ] = {{32, 32, 32, 32, 32, 32}, {32, 32, 32, 32, 64, 64}};

// Decoder weight pointers per layer (resolved once: the arena layout is fixed at wm_create).
struct DecLayerW {
  const bf16 *qkv_w, *out_w, *cq_w, *cout_w, *fc1_w, *fc2_w;
  const float *qkv_b, *out_b, *cq_b, *cout_b, *fc1_b, *fc2_b, *ln1_w, *ln1_b, *ln2_w, *ln2_b, *ln3_w, *ln3_b;
};

struct wm_engine {
  wm_model_dims dm;
  int device;
  std::mutex mu;
  bool weights_ok = false;     // every weight slot set (cached by require_weights)
  long long realloc_gen = 0;   // this engine's buffer generation (t_realloc while one of its entry points runs)
  // weights
  std::map<std::string, Slot> slots;
  std::vector<std::string> slot_order;   // weight names in layout order (wm_weight_info)
  DevBuf arena;
  int k1p;  // padded conv1 K
  // frontend constants
  DevBuf fe_window, fe_cos, fe_sin, fe_filt, fe_lo, fe_hi;
  // encoder scratch
  DevBuf e_cols, e_h1, e_x, e_hb, e_qkv, e_ao, e_ff, e_seek, e_len;
  int enc_cap = 0;
  int enc_chunk = 160;       // windows per encoder pass (activation scratch ~52 MB per large-v3 window; bigger
                             // passes cut the GEMM tail rounds: 16 -> 150 measured +1.2 % end to end)
  // decoder state
  int n_slots = 0, n_hyp_cap = 0;
  DevBuf ckv, skv;
  DevBuf d_tokens, d_lin, d_seq_len, d_done, d_cum, d_row_tok, d_row_pos, d_row_hyp, d_hyp_slot, d_n_active;
  DevBuf d_suppress, d_cand_tok, d_cand_lp, d_fin_tok, d_fin_len, d_fin_cum, d_n_fin, d_ns, d_logit_rows;
  DevBuf d_prow_tok, d_prow_pos, d_prow_hyp, d_head_map;
  // d_n_active holds [0] the live-hypothesis counter and [1..3] the decode's device error word (common.h
  // wm_report_error), so one poll copy reads both
  // per-step records (wm_generate_args h_token_logprobs): per hypothesis, per finished beam candidate
  DevBuf d_tok_lp, d_tok_lp_o, d_fin_lp;
  // row-set decode (generate_rows): per-window prompts / slots, slot -> output id, output tables by window, and
  // the event upload (pass rows, row set, logit rows, starts)
  DevBuf d_win_prompt, d_win_slot, d_hyp_out, d_res_tok, d_res_len, d_res_cum, d_res_ns, d_res_lp, d_res_lp_o, d_ev;
  std::vector<int> h_ev;     // host image of d_ev (kept alive until the next poll syncs the stream)
  int dbg_nan_row = -1;      // TEST ONLY (wm_set_option "debug_nan_row"): NaN logits row before every selection
  int dbg_nan_count = 1;     // TEST ONLY ("debug_nan_count"): rows [debug_nan_row, + count) (a whole beam group: nlive 0)
  // step activations
  DevBuf s_x, s_hb, s_q, s_ao, s_ff, s_logits, s_pm, s_pl, s_po;
  // profiler: per class, HIP event pairs recorded on the launch stream + algorithmic flops / bytes
  bool prof_on = false;
  unsigned prof_mask = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev[P_N];
  std::vector<hipEvent_t> ev_pool;
  double prof_flops[P_N] = {0}, prof_bytes[P_N] = {0};
  DevBuf gemm_ws, gemm_ws2;  // split-K partial slabs (per decoder slice stream)
  // two-slice decode (decoder_pass): second stream + fork/phase/join events
  bool dec_ring = true;      // ring-pipelined decoder GEMMs for the wide K <= 1280 projections (gemm_dec.hip)
  // Decoder projection plan, per projection (DEC_QKV .. DEC_FC2), for passes of <= 1024 rows:
  //   > 0  ring GEMM with the rows in groups of that many (one block per 32-column tile x row group x K split)
  //     0  ring GEMM, all rows in one block (passes of <= 160 rows; wide projections only)
  //    -1  skinny split-K GEMM (gemm.hip launch_gemm)
  //    -2  one-shot GEMM (gemm_dec.hip launch_dec_oneshot)
  // Preset 1 (default) is the fastest per projection measured at 150 rows (tools/dec_gemm_bench);
  // preset 0 is round 1's routing.
  int dec_plan[6] = {96, 32, 32, 32, 64, 64};
  int dec_cols[6] = {32, 32, 32, 32, 64, 64};   // ring GEMM output columns per block (32 or 64)
  int dec_kr[6] = {0, 0, 0, 0, 0, 0};           // ring GEMM K range per block (0: the whole K up to 1280)
  bool dec_split = false;    // two-stream row slices (see decoder_pass)
  int dec_graph = 1;         // decode steps replayed from one captured HIP graph (see generate)
  int dec_gemv = 1;          // passes of <= 32 rows: the small-M weight-streaming GEMM (gemm_dec.hip gemv)
  int dec_gemv_ln = 1;       // passes of <= 16 rows: the LayerNorms after out / cout computed inside cq / fc1
  int dec_gemv_ln_fc2 = 0;   // ... and the one after fc2 inside the next layer's qkv (fc2 a 16-wave residual producer):
                             // measured slower (fc2 on 80 blocks 11.5 us alone, as slab + combine; qkv +2.4 us)
  DevBuf d_lnstat;           // their per-(tile, row) partial row sums, one region per decode slice
  hipStream_t gst = nullptr; // the capture / replay stream (a graph cannot be captured on the legacy null stream)
  hipEvent_t ev_g0 = nullptr, ev_g1 = nullptr;
  int cross_fuse = 1;        // bit 0: cq split-K combine, bit 1: key-split combine (last arriver), folded into
                             // the cross-attention kernel; bit 1 measured slower (per-item hand-off latency)
  DevBuf d_cross_cnt;        // its per-(row, head) arrival counters (zeroed at allocation, reset in-kernel)
  // cross-attention form: 1 = factored (attention over the encoder output, attn_xenc.hip: a window's slot
  // holds its encoder output, 3.84 MB for large-v3), 0 = projected cross-KV panels (attn_dec.hip: 245.8 MB
  // per large-v3 window, projected by wm_cross_kv)
  int cross_mode = 1;
  int cross_tf = 1;          // teacher-forced passes (alignment) run the projected form's cross-attention on MFMA
  int cross_mfma = 1;        // projected form, decode passes with 2..32 rows per window (beam groups): MFMA kernel
  int cross_mfma_fuse = 0;   // ... its key-split combine done by the last-arriving split (d_cross_cnt), not a kernel:
                             // measured slower (16.3 vs 15.3 us per layer at 1 window, beam 5: the L2 hand-off
                             // costs ~3 round trips, more than the combine kernel behind it in the stream)
  int dec_big_rows = 161;    // passes of >= this many rows (beam groups of many windows): 64-row ring groups, the
                             // whole K per block (decoder_layer); 320 before the two-blocks-per-CU tiles below
  int dec_big128 = 512;      // ... from this many rows the 8-wave ring plan (0: never; VLOG_AMD_DEC_BIG128): qkv, fc1
                             // and fc2 as 128 x 128 tiles (fc2's K of 4d in ranges of dec_big_fc2_kr), the d x d
                             // projections as 64 x 64 tiles, one block of 8 waves per CU.  Config 5 (750 rows): dec_gemm
                             // 568 -> 504-506 ms per step, same tokens (profiles/ab_r06_c5_plan*.txt).  Below 512 rows
                             // the 4-wave 64-row groups stay (tools/dec_gemm_bench at 384 rows, profiles/dgb_r06_*).
  int dec_big_fc2_kr = 1280; // ... fc2's K range per block on that plan (0: the whole K; 1280: four ranges, 240 blocks,
                             // slabs summed by its residual + LayerNorm combine; whole K = 60 blocks, 50 us in the step)
  int dec_ln_fold = 0;       // ring passes (33..1024 rows): LayerNorms folded into their consumers (no combine launch
                             // after out / cout; fc2's combine writes stats instead of the LayerNorm).  Off: the
                             // consumers' epilogue costs more than the two launches it removes (dec_gemm 336 vs 319
                             // ms per step at 150 rows, 656 vs 568 at 750; profiles/ab_r05_ln_fold_v2.txt)
  int dec_big_lds = 72;      // ... qkv / fc1 / fc2 with this LDS budget per ring block (KiB): 72 = two resident blocks
                             // per CU (tools/dec_gemm_bench at 750 rows: qkv 24.7 -> 18.8 us, fc1 31.3 -> 21.4, fc2
                             // 41.6 -> 33.1 against 144; at 256 rows qkv+fc1+fc2 45.6 -> 35.7 us per layer against the
                             // 150-row plan; bit-identical: the ring depth never changes a row's K order)
  int xkeep = 0;             // factored cross-attention: window groups whose encoder output is loaded with the default
                             // cache policy (the rest non-temporal), to keep them in the Infinity Cache across layers
  bool xsnake = false;       // factored cross-attention: odd layers walk each XCD's items in reverse (Infinity Cache reuse)
  int xdma = 0;              // factored cross-attention, bf16 at n_state 1280: 1 = the LDS-DMA form, 0 = the
                             // register-staged form (default; same bits on key-split items; attn_xenc.hip).  Headline
                             // A/B on one box (profiles/ab_r06_xattn_forms.jsonl): register 3773, LDS-DMA chunks 3752,
                             // LDS-DMA key-split items 3711 RTFx
  int xchunks = 0;           // ... greedy passes at n_state 1280: 1 = the stream-K chunk cut (register form: its
                             // segments as items; LDS-DMA form: a chunk per workgroup), 0 = key-split items (default:
                             // the chunk cut loses at 150 windows, profiles/xattn_bench_r06_chunk_items.txt)
  DevBuf xenc;               // factored: [n_slots][T][d] bf16 encoder outputs (cross_fp8: OCP e4m3 bytes)
  DevBuf xscale;             // cross_fp8: [n_slots][T] f32 per-position scales
  int cross_fp8 = 0;         // opt-in fp8 cross memory (factored form only; changes numerics, never the default)
  DevBuf xwkt;               // factored: Wk^T per layer and head [L][H][d][64] bf16, packed from dec.ckv.w
  DevBuf xwvb;               // factored: Wv per layer and head in 16-column blocks [L][H][d/16][64][16]
  bool xwkt_ready = false;
  // folded LayerNorm (decode_ln_fold): per decoder layer s = W g and c = W b + bias of qkv (ln1), cq (ln2), fc1 (ln3),
  // [L][qkv_s 3d | qkv_c 3d | cq_s d | cq_c d | fc1_s 4d | fc1_c 4d] f32, computed once per weight upload
  DevBuf fold_vec;
  bool fold_ready = false;
  DevBuf fold_stat[2];       // producer row sums per decode slice: [d/16][rows][2]
  DevBuf s_qp, s_pu, s_pml;  // factored step scratch: q' [rows][H][d], split partials u/l and (m, l)
  int cross_cap = 0;         // cross-attention grid cap (0: one block per item; >0: persistent grid-stride form,
                             // 2 blocks/CU measured ~2 % faster alone but slower with the fused q combine)
  hipStream_t st2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_mid = nullptr, ev_join = nullptr;
  std::vector<DecLayerW> dec_w;
  // factored form, teacher-forced alignment pass: the pass's windows' encoder outputs gathered contiguously, and one
  // layer's projected K/V panels of them [2][tf_nwin][H][T][64] (re-projected per layer on MFMA)
  DevBuf a_enc, a_kv;
  int tf_nwin = 0;
  DevBuf a_logits, a_attn, a_next, a_probs, a_rowsum, a_z, a_mat, a_cost, a_trace, a_pi, a_pj, a_plen, a_meta;
  DevBuf prof_dbytes;        // device counters (attention kernels add the bytes they actually read)
  hipEvent_t ev_get() {
    if (ev_pool.empty()) {
      hipEvent_t ev;
      HIP_OK(hipEventCreate(&ev));
      return ev;
    }
    hipEvent_t ev = ev_pool.back();
    ev_pool.pop_back();
    return ev;
  }
  unsigned long long* dstat(int cls) { return (prof_on && ((prof_mask >> cls) & 1u)) ? prof_dbytes.as<unsigned long long>() + (size_t)cls * STAT_SLOTS : nullptr; }

  const Slot& slot(const std::string& n) const {
    auto it = slots.find(n);
    if (it == slots.end()) throw std::runtime_error("unknown weight " + n);
    return it->second;
  }
  template <class T> T* W(const std::string& n) const { return (T*)((char*)arena.p + slot(n).off); }
  const bf16* Wb(const std::string& n) const { return W<bf16>(n); }
  const float* Wf(const std::string& n) const { return W<float>(n); }

  size_t device_bytes() const {
    size_t t = arena.bytes;
    for (const DevBuf* b : {&e_cols, &e_h1, &e_x, &e_hb, &e_qkv, &e_ao, &e_ff, &ckv, &xenc, &xscale, &xwkt, &xwvb, &s_qp, &s_pu, &skv, &s_x, &s_hb, &s_q, &s_ao,
                            &s_ff, &s_logits, &s_pm, &s_pl, &s_po, &d_tokens, &d_lin, &d_fin_tok})
      t += b->bytes;
    return t;
  }
};

namespace {

void add_slot(wm_engine* e, size_t& off, const std::string& name, size_t count, int elem) {
  e->slots[name] = Slot{off, count * elem, false, elem};
  e->slot_order.push_back(name);
  off += align256(count * elem);
}

void build_layout(wm_engine* e) {
  const auto& m = e->dm;
  const size_t d = m.n_state, f = 4 * d, b2 = 2, f4 = 4;
  e->k1p = ((3 * m.n_mels + 63) / 64) * 64;
  size_t off = 0;
  add_slot(e, off, "enc.conv1.w", d * e->k1p, 2);
  add_slot(e, off, "enc.conv1.b", d, 4);
  add_slot(e, off, "enc.conv2.w", d * 3 * d, 2);
  add_slot(e, off, "enc.conv2.b", d, 4);
  add_slot(e, off, "enc.pos", (size_t)m.n_audio_ctx * d, 4);
  for (int l = 0; l < m.n_enc_layer; ++l) {
    const std::string p = "enc." + std::to_string(l) + ".";
    add_slot(e, off, p + "ln1.w", d, 4); add_slot(e, off, p + "ln1.b", d, 4);
    add_slot(e, off, p + "qkv.w", 3 * d * d, 2); add_slot(e, off, p + "qkv.b", 3 * d, 4);
    add_slot(e, off, p + "out.w", d * d, 2); add_slot(e, off, p + "out.b", d, 4);
    add_slot(e, off, p + "ln2.w", d, 4); add_slot(e, off, p + "ln2.b", d, 4);
    add_slot(e, off, p + "fc1.w", f * d, 2); add_slot(e, off, p + "fc1.b", f, 4);
    add_slot(e, off, p + "fc2.w", d * f, 2); add_slot(e, off, p + "fc2.b", d, 4);
  }
  add_slot(e, off, "enc.ln.w", d, 4); add_slot(e, off, "enc.ln.b", d, 4);
  add_slot(e, off, "dec.embed", (size_t)m.n_vocab * d, 2);
  add_slot(e, off, "dec.pos", (size_t)m.n_text_ctx * d, 4);
  for (int l = 0; l < m.n_dec_layer; ++l) {
    const std::string p = "dec." + std::to_string(l) + ".";
    add_slot(e, off, p + "ln1.w", d, 4); add_slot(e, off, p + "ln1.b", d, 4);
    add_slot(e, off, p + "qkv.w", 3 * d * d, 2); add_slot(e, off, p + "qkv.b", 3 * d, 4);
    add_slot(e, off, p + "out.w", d * d, 2); add_slot(e, off, p + "out.b", d, 4);
    add_slot(e, off, p + "ln2.w", d, 4); add_slot(e, off, p + "ln2.b", d, 4);
    add_slot(e, off, p + "cq.w", d * d, 2); add_slot(e, off, p + "cq.b", d, 4);
    add_slot(e, off, p + "cout.w", d * d, 2); add_slot(e, off, p + "cout.b", d, 4);
    add_slot(e, off, p + "ln3.w", d, 4); add_slot(e, off, p + "ln3.b", d, 4);
    add_slot(e, off, p + "fc1.w", f * d, 2); add_slot(e, off, p + "fc1.b", f, 4);
    add_slot(e, off, p + "fc2.w", d * f, 2); add_slot(e, off, p + "fc2.b", d, 4);
  }
  add_slot(e, off, "dec.ckv.w", (size_t)m.n_dec_layer * 2 * d * d, 2);
  add_slot(e, off, "dec.ckv.b", (size_t)m.n_dec_layer * 2 * d, 4);
  add_slot(e, off, "dec.ln.w", d, 4); add_slot(e, off, "dec.ln.b", d, 4);
  e->arena.ensure(off);
}

// slaney mel filterbank (faster-whisper get_mel_filters), periodic Hann, DFT twiddles — host f64 -> f32
void build_frontend(wm_engine* e, hipStream_t st) {
  const int nm = e->dm.n_mels, nb = 201, nfft = 400, sr = 16000;
  std::vector<float> win(nfft), c(nfft), s(nfft);
  for (int n = 0; n < nfft; ++n) {
    win[n] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * n / nfft));
    c[n] = (float)std::cos(2.0 * M_PI * n / nfft);
    s[n] = (float)std::sin(2.0 * M_PI * n / nfft);
  }
  std::vector<double> mels(nm + 2), freqs(nm + 2), fft(nb);
  const double max_mel = 45.245640471924965, f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  for (int i = 0; i < nm + 2; ++i) {
    mels[i] = max_mel * i / (nm + 1);
    freqs[i] = mels[i] >= min_log_mel ? min_log_hz * std::exp(logstep * (mels[i] - min_log_mel)) : f_sp * mels[i];
  }
  for (int k = 0; k < nb; ++k) fft[k] = (double)k * sr / nfft;
  std::vector<float> filt((size_t)nm * nb, 0.f);
  std::vector<int> lo(nm, nb), hi(nm, 0);
  for (int m = 0; m < nm; ++m) {
    const double enorm = 2.0 / (freqs[m + 2] - freqs[m]);
    for (int k = 0; k < nb; ++k) {
      const double lower = -(freqs[m] - fft[k]) / (freqs[m + 1] - freqs[m]);
      const double upper = (freqs[m + 2] - fft[k]) / (freqs[m + 2] - freqs[m + 1]);
      const double w = std::max(0.0, std::min(lower, upper)) * enorm;
      filt[(size_t)m * nb + k] = (float)w;
      if (w > 0) { lo[m] = std::min(lo[m], k); hi[m] = std::max(hi[m], k + 1); }
    }
    if (lo[m] >= hi[m]) { lo[m] = 0; hi[m] = 0; }
  }
  auto up = [&](DevBuf& b, const void* src, size_t bytes) {
    b.ensure(bytes);
    HIP_OK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, st));
  };
  up(e->fe_window, win.data(), nfft * 4);
  up(e->fe_cos, c.data(), nfft * 4);
  up(e->fe_sin, s.data(), nfft * 4);
  up(e->fe_filt, filt.data(), filt.size() * 4);
  up(e->fe_lo, lo.data(), nm * 4);
  up(e->fe_hi, hi.data(), nm * 4);
  HIP_OK(hipStreamSynchronize(st));
}

GemmEpi epi_of(int kind, void* out, long long ldc, const float* bias) {
  GemmEpi p;
  std::memset(&p, 0, sizeof(p));
  p.kind = kind;
  p.out = out;
  p.ldc = ldc;
  p.bias = bias;
  return p;
}
GemmA amat(const bf16* ptr, long long ld) { return GemmA{ptr, ld, 0, 0}; }

// Times one kernel class.  Plain mode records events around the launches; `attached` mode hands the two
// events to a launcher that attaches them to the dispatch itself (hipExtLaunchKernelGGL), which times the
// kernel alone (what rocprofv3 reports) instead of kernel + event-record overhead.
struct ProfScope {
  wm_engine* e;
  int cls;
  hipStream_t st;
  bool attached;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(wm_engine* e_, int cls_, hipStream_t st_, double flops = 0, double bytes = 0, bool attached_ = false)
      : e(e_), cls(cls_), st(st_), attached(attached_) {
    if (!e->prof_on || !((e->prof_mask >> cls) & 1u)) return;
    a = e->ev_get();
    b = e->ev_get();
    if (!attached) HIP_OK(hipEventRecord(a, st));
    e->prof_flops[cls] += flops;
    e->prof_bytes[cls] += bytes;
  }
  ~ProfScope() {
    if (!a) return;
    if (!attached) (void)hipEventRecord(b, st);
    e->prof_ev[cls].push_back({a, b});
  }
};

// algorithmic bytes of a GEMM: A (M x K bf16) + W (N x K bf16) + output
double gemm_bytes(double M, double N, double K, double out_bytes) { return 2 * M * K + 2 * N * K + out_bytes * M * N; }

void gemm_p(wm_engine* e, int cls, const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& ep,
            hipStream_t st) {
  const double ob = (ep.kind == EPI_RESID_F32) ? 8 : (ep.kind == EPI_RESID_LN) ? 10 : (ep.kind == EPI_F32 || ep.kind == EPI_GELU_POS_F32) ? 4 : 2;
  ProfScope ps(e, cls, st, 2.0 * M * N * K, gemm_bytes(M, N, K, ob));
  // split-K only where the grid is too small to fill the chip (decoder rows); 64 MB slab scratch
  const size_t wsb = 64ull << 20;
  e->gemm_ws.ensure(wsb);
  launch_gemm(a, w, ldw, M, N, K, ep, e->gemm_ws.as<float>(), wsb, st);
}

// ------------------------------------------------------------------------------------------ encoder
void encode_chunk(wm_engine* e, const float* mel, long long ld, const int* h_seek, const int* h_len, int B, bf16* out,
                  hipStream_t st) {
  const auto& m = e->dm;
  const int d = m.n_state, T = m.n_audio_ctx, L = m.n_enc_layer, H = m.n_head;
  const long long M = (long long)B * T;
  if (B > e->enc_cap) {
    e->e_cols.ensure((size_t)B * 3000 * e->k1p * 2);
    e->e_h1.ensure((size_t)B * 3001 * d * 2);
    e->e_x.ensure((size_t)M * d * 4);
    e->e_hb.ensure((size_t)M * d * 2);
    e->e_qkv.ensure((size_t)M * 3 * d * 2);
    e->e_ao.ensure((size_t)M * d * 2);
    e->e_ff.ensure((size_t)M * 4 * d * 2);
    e->e_seek.ensure(B * 4);
    e->e_len.ensure(B * 4);
    e->enc_cap = B;
  }
  HIP_OK(hipMemcpyAsync(e->e_seek.p, h_seek, B * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->e_len.p, h_len, B * 4, hipMemcpyHostToDevice, st));
  bf16* cols = e->e_cols.as<bf16>();
  bf16* h1 = e->e_h1.as<bf16>();
  float* x = e->e_x.as<float>();
  bf16* hb = e->e_hb.as<bf16>();
  bf16* qkv = e->e_qkv.as<bf16>();
  bf16* ao = e->e_ao.as<bf16>();
  bf16* ff = e->e_ff.as<bf16>();
  // conv1 (implicit GEMM over the window-sliced mel) + GELU -> h1 rows 1..3000 of each [3001][d] block
  {
    ProfScope ps(e, P_ENC_OTHER, st);
    launch_im2col_conv1(mel, ld, e->e_seek.as<int>(), e->e_len.as<int>(), B, m.n_mels, e->k1p, cols, st);
    launch_zero_pad_rows(h1, B, 3001LL * d, d, st);
  }
  {
    GemmEpi ep = epi_of(EPI_BF16, h1, d, e->Wf("enc.conv1.b"));
    ep.act = 1; ep.rpb = 3000; ep.bstride = 3001LL * d; ep.roff = 1;
    gemm_p(e, P_ENC_GEMM, amat(cols, e->k1p), e->Wb("enc.conv1.w"), e->k1p, B * 3000, d, e->k1p, ep, st);
  }
  // conv2 (k3, s2): row t of window b reads h1 rows 2t-1, 2t, 2t+1 = 3d contiguous elements starting at
  // block row 2t (the zero row 0 is the left padding); + GELU + positional embedding -> residual x
  {
    GemmA a{h1, 2LL * d, T, 3001LL * d};
    GemmEpi ep = epi_of(EPI_GELU_POS_F32, x, d, e->Wf("enc.conv2.b"));
    ep.rpb = T; ep.pos = e->Wf("enc.pos");
    gemm_p(e, P_ENC_GEMM, a, e->Wb("enc.conv2.w"), 3LL * d, (int)M, d, 3 * d, ep, st);
  }
  for (int l = 0; l < L; ++l) {
    const std::string p = "enc." + std::to_string(l) + ".";
    {
      ProfScope ps(e, P_ENC_OTHER, st);
      launch_layernorm(x, d, nullptr, (int)M, d, e->Wf(p + "ln1.w"), e->Wf(p + "ln1.b"), hb, d, st);
    }
    gemm_p(e, P_ENC_GEMM, amat(hb, d), e->Wb(p + "qkv.w"), d, (int)M, 3 * d, d, epi_of(EPI_BF16, qkv, 3LL * d, e->Wf(p + "qkv.b")), st);
    {
      ProfScope ps(e, P_ENC_ATTN, st, 4.0 * B * (double)T * T * d, 2.0 * 4 * M * d);
      launch_attn_enc(qkv, ao, B, T, d, H, st);
    }
    gemm_p(e, P_ENC_GEMM, amat(ao, d), e->Wb(p + "out.w"), d, (int)M, d, d, epi_of(EPI_RESID_F32, x, d, e->Wf(p + "out.b")), st);
    {
      ProfScope ps(e, P_ENC_OTHER, st);
      launch_layernorm(x, d, nullptr, (int)M, d, e->Wf(p + "ln2.w"), e->Wf(p + "ln2.b"), hb, d, st);
    }
    {
      GemmEpi ep = epi_of(EPI_BF16, ff, 4LL * d, e->Wf(p + "fc1.b"));
      ep.act = 1;
      gemm_p(e, P_ENC_GEMM, amat(hb, d), e->Wb(p + "fc1.w"), d, (int)M, 4 * d, d, ep, st);
    }
    gemm_p(e, P_ENC_GEMM, amat(ff, 4LL * d), e->Wb(p + "fc2.w"), 4LL * d, (int)M, d, 4 * d, epi_of(EPI_RESID_F32, x, d, e->Wf(p + "fc2.b")), st);
  }
  ProfScope ps(e, P_ENC_OTHER, st);
  launch_layernorm(x, d, nullptr, (int)M, d, e->Wf("enc.ln.w"), e->Wf("enc.ln.b"), out, d, st);
}

// ------------------------------------------------------------------------------------------ decoder
void ensure_step(wm_engine* e, int rows, int logit_rows) {
  const int d = e->dm.n_state, H = e->dm.n_head;
  e->s_x.ensure((size_t)rows * d * 4);
  e->s_hb.ensure((size_t)rows * d * 2);
  e->s_q.ensure((size_t)rows * d * 2);
  e->s_ao.ensure((size_t)rows * d * 2);
  e->s_ff.ensure((size_t)rows * 4 * d * 2);
  e->s_logits.ensure((size_t)logit_rows * e->dm.n_vocab * 4);
  e->s_pm.ensure((size_t)rows * H * 16 * 4);
  e->s_pl.ensure((size_t)rows * H * 16 * 4);
  e->s_po.ensure((size_t)rows * H * 16 * 64 * 4);
  if (e->d_cross_cnt.bytes < (size_t)rows * H * 4) {
    e->d_cross_cnt.ensure((size_t)rows * H * 4);
    HIP_OK(hipMemset(e->d_cross_cnt.p, 0, e->d_cross_cnt.bytes));
  }
  e->d_prow_tok.ensure((size_t)rows * 4);
  e->d_prow_pos.ensure((size_t)rows * 4);
  e->d_prow_hyp.ensure((size_t)rows * 4);
  e->d_logit_rows.ensure((size_t)logit_rows * 4);
}

const std::vector<DecLayerW>& dec_weights(wm_engine* e) {
  if ((int)e->dec_w.size() == e->dm.n_dec_layer) return e->dec_w;
  e->dec_w.clear();
  for (int l = 0; l < e->dm.n_dec_layer; ++l) {
    const std::string p = "dec." + std::to_string(l) + ".";
    DecLayerW w;
    w.qkv_w = e->Wb(p + "qkv.w"); w.out_w = e->Wb(p + "out.w"); w.cq_w = e->Wb(p + "cq.w");
    w.cout_w = e->Wb(p + "cout.w"); w.fc1_w = e->Wb(p + "fc1.w"); w.fc2_w = e->Wb(p + "fc2.w");
    w.qkv_b = e->Wf(p + "qkv.b"); w.out_b = e->Wf(p + "out.b"); w.cq_b = e->Wf(p + "cq.b");
    w.cout_b = e->Wf(p + "cout.b"); w.fc1_b = e->Wf(p + "fc1.b"); w.fc2_b = e->Wf(p + "fc2.b");
    w.ln1_w = e->Wf(p + "ln1.w"); w.ln1_b = e->Wf(p + "ln1.b"); w.ln2_w = e->Wf(p + "ln2.w");
    w.ln2_b = e->Wf(p + "ln2.b"); w.ln3_w = e->Wf(p + "ln3.w"); w.ln3_b = e->Wf(p + "ln3.b");
    e->dec_w.push_back(w);
  }
  return e->dec_w;
}

// A contiguous range of decoder rows [r0, r0 + rows) of a pass over total_rows, issued on its own stream
// with its own split-K scratch.
struct DecSlice {
  int r0, rows, total_rows;
  hipStream_t st;
  DevBuf* ws;
};

// Issues decoder layer l for one slice.  `mid` (optional) is recorded on the slice's stream right before its
// cross-attention, which is where the second slice starts (see decoder_pass).
// The factored cross-attention may cut a greedy pass into stream-K chunks (attn_xenc.hip xattn_plan): bf16 cross
// memory, no cache-policy or walk-order experiment on
static bool xattn_chunks_ok(const wm_engine* e) {
  return e->xchunks && !e->cross_fp8 && e->xkeep == 0 && !e->xsnake;
}

void decoder_layer(wm_engine* e, const DecSlice& sl, int l, const int* row_pos, const int* row_hyp, const int* done,
                   const int* lin, const std::vector<std::vector<int>>* align_map, int n_align, float* attn,
                   int cross_group, hipEvent_t mid) {
  const auto& m = e->dm;
  const int d = m.n_state, H = m.n_head, L = m.n_dec_layer, T = m.n_audio_ctx, C = m.n_text_ctx;
  const int r0 = sl.r0, rows = sl.rows;
  hipStream_t st = sl.st;
  float* x = e->s_x.as<float>() + (size_t)r0 * d;
  bf16* hb = e->s_hb.as<bf16>() + (size_t)r0 * d;
  bf16* q = e->s_q.as<bf16>() + (size_t)r0 * d;
  bf16* ao = e->s_ao.as<bf16>() + (size_t)r0 * d;
  bf16* ff = e->s_ff.as<bf16>() + (size_t)r0 * 4 * d;
  row_pos += r0;
  row_hyp += r0;
  const size_t skv_layer = (size_t)e->n_hyp_cap * H * C * 64;      // elements per (layer, k|v)
  const size_t ckv_layer = (size_t)e->n_slots * H * T * 64;
  bf16* skv = e->skv.as<bf16>();
  bf16* ckv = e->ckv.as<bf16>();
  const auto& W = dec_weights(e)[l];
  const size_t wsb = 64ull << 20;
  sl.ws->ensure(wsb);
  float* ws = sl.ws->as<float>();
  // The route of each projection follows the whole pass's rows (sl.total_rows), so slicing a pass never changes
  // a row's arithmetic.  Long prefills (> 1024 rows) keep the large-tile GEMMs.
  auto plan_of = [&](int proj) -> int { return sl.total_rows > 1024 ? -1 : e->dec_plan[proj]; };
  auto gemm = [&](int proj, const GemmA& a, const bf16* w, long long ldw, int N, int K, const GemmEpi& ep) {
    const double ob = (ep.kind == EPI_RESID_F32) ? 8 : (ep.kind == EPI_RESID_LN) ? 10 : 2;
    ProfScope ps(e, P_DEC_GEMM, st, 2.0 * rows * N * K, gemm_bytes(rows, N, K, ob));
    // one window's beam (or a handful of rows): the weight-streaming small-M kernel
    if (sl.total_rows <= 32 && e->dec_gemv && launch_dec_gemv(a, w, ldw, rows, N, K, ep, ws, wsb, st)) return;
    if (a.lnx || (ep.stat_out && !ep.xg_out)) throw std::runtime_error("decoder: fused LayerNorm operand off the small-M path");
    // passes of >= dec_big_rows rows (beam groups of many windows; tools/dec_gemm_bench at 384 and 750 rows): 64-row
    // ring groups; 64 columns for qkv and fc1, and for every projection from 512 rows; fc2's whole K per block
    // (384 rows: 76 vs 86 us per layer for the 150-row plan; 750 rows: 114 vs 159 us)
    const int tr = sl.total_rows;
    const bool big = e->dec_big_rows > 0 && tr >= e->dec_big_rows && tr <= 1024;
    // (dec_big128 from round 6: the 8-wave plan below; round 4's form, qkv / fc1 / fc2 in 4-wave 128-row groups,
    // two blocks per CU at 750 rows: 17.2 / 18.4 / 25.6 us against
    // 18.9 / 21.0 / 32.8 for 64-row groups in tools/dec_gemm_bench, yet slower inside the decode step)
    const bool sq = proj == DEC_OUT || proj == DEC_CQ || proj == DEC_COUT;
    const bool b128 = big && e->dec_big128 > 0 && tr >= e->dec_big128;
    int p = big ? 64 : plan_of(proj);
    // the three d x d projections keep 32-column tiles below 512 rows and one block per CU (144 KiB); qkv / fc1 / fc2
    // take 64 x 64 tiles, two blocks per CU (dec_big_lds; tools/dec_gemm_bench at 256 / 384 / 750 rows,
    // profiles/dec_gemm_bench_r04_*rows_lds*.txt)
    int cols = big ? ((tr >= 512 || !sq) ? 64 : 32) : e->dec_cols[proj];
    int lds = big ? (sq ? 144 : e->dec_big_lds) : 0;
    int waves = 4;
    int kr_big = 0;
    if (b128) {                            // the 8-wave plan (dec_big128)
      if (sq) { p = 64; cols = 64; lds = 144; waves = 8; }
      else { p = 128; cols = 128; lds = 144; waves = 8; }
      // fc2 (K = 4d) in K ranges of dec_big_fc2_kr: as 128 x 128 tiles over the whole K (60 blocks) it took 50 us per
      // launch in the step against 27.5 for the 4-wave 64 x 64 tiles (rocprof, config 5), though 25 us in
      // tools/dec_gemm_bench: a block streams its 1.3 MB activation panel from the MALL at the per-CU rate, so few
      // blocks lose in the step.  Qkv 128 x 64 (two blocks per CU) / fc1 128 x 64 / fc2 128 x 64 in two K ranges
      // measured 5 / 2 / 10 ms per step slower (profiles/ab_r06_c5_plan2.txt)
      if (proj == DEC_FC2) kr_big = e->dec_big_fc2_kr;
      // VLOG_AMD_DEC_BIG_<QKV|SQ|FC1|FC2>="rows,cols,lds,kr,waves" overrides a projection's plan (A/B only)
      static const int* const ov = [] {
        static int v[4][5] = {};
        const char* names[4] = {"VLOG_AMD_DEC_BIG_QKV", "VLOG_AMD_DEC_BIG_SQ", "VLOG_AMD_DEC_BIG_FC1", "VLOG_AMD_DEC_BIG_FC2"};
        for (int i = 0; i < 4; ++i)
          if (const char* ev = std::getenv(names[i]))
            if (std::sscanf(ev, "%d,%d,%d,%d,%d", &v[i][0], &v[i][1], &v[i][2], &v[i][3], &v[i][4]) != 5) v[i][0] = 0;
        return &v[0][0];
      }();
      const int* o = ov + 5 * (sq ? 1 : proj == DEC_QKV ? 0 : proj == DEC_FC1 ? 2 : 3);
      if (o[0] > 0) { p = o[0]; cols = o[1]; lds = o[2]; kr_big = o[3]; waves = o[4]; }
    }
    if (p == -2 && launch_dec_oneshot(a, w, ldw, rows, N, K, ep, ws, wsb, N >= 3 * K ? 4 : 2, st)) return;
    // ring: one pass over each 1280-deep K range, epilogue in place (K > 1280: slabs summed by the combine)
    const int kr = kr_big > 0 ? std::min(kr_big, K) : e->dec_kr[proj] > 0 ? std::min(e->dec_kr[proj], K) : (K <= 1280 || big ? K : 1280);
    if (p > 0 && launch_dec_ring(a, w, ldw, rows, N, K, ep, ws, wsb, kr, st, p, cols, lds, waves)) return;
    if (p == 0 && e->dec_ring && K <= 1280 && sl.total_rows <= 160 && launch_dec_ring(a, w, ldw, rows, N, K, ep, ws, wsb, 0, st))
      return;
    if (a.fold_stat || ep.xg_out) throw std::runtime_error("decoder: a folded-LayerNorm projection left the ring path");
    launch_gemm(a, w, ldw, rows, N, K, ep, ws, wsb, st);
  };
  // residual-producing GEMMs also apply the LayerNorm that consumes the residual (EPI_RESID_LN: fused into
  // the split-K combine on the skinny path): out -> ln2, cout -> ln3, fc2 -> next layer's ln1
  auto resid_ln = [&](const float* g, const float* b, const float* bias) {
    GemmEpi ep = epi_of(EPI_RESID_LN, x, d, bias);
    ep.ln_g = g; ep.ln_b = b; ep.ln_out = hb; ep.ln_ld = d;
    return ep;
  };
  // <= 16 rows: the LayerNorms after out and cout run inside their consumers (cq, fc1), from the residual and
  // the per-(16-column tile, row) sums their producers write (two combine launches fewer per layer)
  const bool ln_fuse = sl.total_rows <= 16 && e->dec_gemv && e->dec_gemv_ln && gemv_ln_fusable(rows, d, d, d);
  float* lnstat = nullptr;
  if (ln_fuse) {
    e->d_lnstat.ensure(2 * 128 * 16 * 2 * 4);
    lnstat = e->d_lnstat.as<float>() + (r0 == 0 ? 0 : 128 * 16 * 2);
  }
  auto resid_stat = [&](const float* bias) {
    GemmEpi ep = epi_of(EPI_RESID_F32, x, d, bias);
    ep.stat_out = lnstat;
    return ep;
  };
  auto ln_operand = [&](const float* g, const float* b) {
    GemmA a = amat(nullptr, d);
    a.lnx = x; a.ln_g = g; a.ln_b = b; a.ln_stat = lnstat; a.ln_tiles = d / 16;
    return a;
  };
  // fc2 -> the next layer's ln1 the same way: fc2 (K = 4d) writes the residual and its statistics without split-K,
  // the next layer's qkv normalises its operand (the same for every layer of a pass, so layer l > 0's qkv knows)
  const bool fc2_fuse = ln_fuse && e->dec_gemv_ln_fc2 && gemv_ln_fusable(rows, d, 4 * d, d);
  // Folded LayerNorms (ring passes): the residual producers (out, cout, fc2) write x, bf16(x * g) into hb and row
  // sums; the consumers (cq, fc1, next qkv) multiply hb and finish the LayerNorm in their epilogue (gemm.h GemmA
  // fold_*), so out and cout need no combine launch and fc2's combine writes sums instead of the LayerNorm.  Only
  // where every projection of the layer takes the ring path with the consumers' whole K per block.
  const int trows = sl.total_rows;
  const bool big_route = e->dec_big_rows > 0 && trows >= e->dec_big_rows && trows <= 1024;
  auto ring_route = [&](int proj, int K) {
    if (trows <= 32 && e->dec_gemv) return false;
    if (big_route) return true;
    const int p = plan_of(proj);
    return p > 0 || (p == 0 && e->dec_ring && K <= 1280 && trows <= 160);
  };
  const bool b128_route = big_route && e->dec_big128 > 0 && trows >= e->dec_big128;   // 8-wave tiles take no fold
  const bool fold = e->dec_ln_fold && e->fold_ready && !ln_fuse && trows > 32 && trows <= 1024 && !(attn && align_map) && !b128_route &&
                    ring_route(DEC_QKV, d) && ring_route(DEC_OUT, d) && ring_route(DEC_CQ, d) && ring_route(DEC_COUT, d) &&
                    ring_route(DEC_FC1, d) && ring_route(DEC_FC2, 4 * d) && e->dec_kr[DEC_QKV] == 0 &&
                    e->dec_kr[DEC_CQ] == 0 && e->dec_kr[DEC_FC1] == 0 && d % 16 == 0;
  float* fstat = nullptr;
  const float* fv = nullptr;
  if (fold) {
    DevBuf& fb = e->fold_stat[r0 == 0 ? 0 : 1];
    fb.ensure((size_t)(d / 16) * rows * 2 * 4);
    fstat = fb.as<float>();
    fv = e->fold_vec.as<float>() + (size_t)l * 16 * d;
  }
  auto fold_producer = [&](const float* bias, const float* g_next) {
    GemmEpi ep = epi_of(EPI_RESID_F32, x, d, bias);
    ep.stat_out = fstat; ep.xg_out = hb; ep.xg_g = g_next; ep.xg_ld = d;
    return ep;
  };
  auto fold_operand = [&](int tiles) {
    GemmA a = amat(hb, d);
    a.fold_stat = fstat; a.fold_tiles = tiles; a.fold_rows = rows;
    return a;
  };
  auto fold_epi = [&](GemmEpi ep, size_t off, int N) {
    ep.bias = nullptr;
    ep.fold_s = fv + off; ep.fold_c = fv + off + N;
    return ep;
  };
  // fc2's K ranges as the gemm route picks them (the same for every layer of the pass): split-K slabs -> its combine
  // writes one whole-row tile of sums; one range -> the ring epilogue writes d / 16 tiles (read by the next qkv)
  const int fc2_kr = e->dec_kr[DEC_FC2] > 0 ? std::min(e->dec_kr[DEC_FC2], 4 * d) : (4 * d <= 1280 || big_route ? 4 * d : 1280);
  const int fc2_tiles = (4 * d + fc2_kr - 1) / fc2_kr > 1 ? 1 : d / 16;
  const bool fold_qkv = fold && l > 0;
  bf16* kc = skv + (size_t)(2 * l) * skv_layer;
  bf16* vc = skv + (size_t)(2 * l + 1) * skv_layer;
  {
    GemmEpi ep = epi_of(EPI_DEC_QKV, q, d, W.qkv_b);
    ep.kcache = kc; ep.vcache = vc; ep.row_hyp = row_hyp; ep.row_pos = row_pos;
    ep.d = d; ep.n_head = H; ep.head_dim = 64; ep.n_ctx = C;
    if (fold_qkv) gemm(DEC_QKV, fold_operand(fc2_tiles), W.qkv_w, d, 3 * d, d, fold_epi(ep, 0, 3 * d));
    else gemm(DEC_QKV, (fc2_fuse && l > 0) ? ln_operand(W.ln1_w, W.ln1_b) : amat(hb, d), W.qkv_w, d, 3 * d, d, ep);
  }
  {
    ProfScope ps(e, P_SELF_ATTN, st, 0, 0, true);
    launch_self_attn(q, d, kc, vc, lin, row_hyp, row_pos, done, ao, d, rows, H, C, e->dstat(P_SELF_ATTN), st, ps.a, ps.b,
                     sl.total_rows, cross_group);
  }
  gemm(DEC_OUT, amat(ao, d), W.out_w, d, d, d,
       fold ? fold_producer(W.out_b, W.ln2_w) : ln_fuse ? resid_stat(W.out_b) : resid_ln(W.ln2_w, W.ln2_b, W.out_b));
  // cq: when the skinny split-K path runs it and no attention is captured, its slabs stay in the scratch and
  // the cross-attention kernel sums them while loading q (no combine launch)
  CrossFuse fz;
  {
    GemmEpi ep = epi_of(EPI_BF16, q, d, W.cq_b);
    const int pcq = plan_of(DEC_CQ);
    const int gsk = (sl.total_rows <= 32 && e->dec_gemv) ? gemv_splits(rows, d, d, nullptr) : 0;
    const int sk = gsk > 0 ? gsk
                 : pcq == -1 ? skinny_splits(rows, d, d, wsb)
                             : (pcq > 0 && e->dec_kr[DEC_CQ] > 0 ? (d + e->dec_kr[DEC_CQ] - 1) / e->dec_kr[DEC_CQ] : 1);
    if ((e->cross_fuse & 1) && !(attn && align_map) && sk > 1) {
      ep.defer_combine = 1;
      fz.q_part = ws; fz.q_splits = sk; fz.q_rows = rows; fz.q_bias = W.cq_b;
    }
    if (fold) gemm(DEC_CQ, fold_operand(d / 16), W.cq_w, d, d, d, fold_epi(ep, 6 * (size_t)d, d));
    else gemm(DEC_CQ, ln_fuse ? ln_operand(W.ln2_w, W.ln2_b) : amat(hb, d), W.cq_w, d, d, d, ep);
  }
  if ((e->cross_fuse & 2) && e->cross_mode == 0) fz.cnt = e->d_cross_cnt.as<int>() + (size_t)r0 * H;
  fz.tf = (attn && align_map && e->cross_tf) ? 1 : 0;
  fz.mfma = e->cross_mfma;
  if (e->cross_mfma_fuse && e->cross_mode == 0) fz.tf_cnt = e->d_cross_cnt.as<int>() + (size_t)r0 * H;
  float* probs = nullptr;
  const int* hmap = nullptr;
  if (attn && align_map) {
    const auto& mp = (*align_map)[l];
    bool any = false;
    for (int v : mp) any |= v >= 0;
    if (any) {
      HIP_OK(hipMemcpyAsync(e->d_head_map.p, mp.data(), H * 4, hipMemcpyHostToDevice, st));
      probs = attn + (size_t)r0 * n_align * T;
      hmap = e->d_head_map.as<int>();
    }
  }
  if (mid) HIP_OK(hipEventRecord(mid, st));
  if (e->cross_mode == 1 && e->tf_nwin > 0 && attn && align_map) {
    // factored form, alignment pass: this layer's K/V panels of the pass's windows projected on MFMA (the wm_cross_kv
    // GEMM restricted to one layer: 2 x d x d x T flops per window), then the projected form's teacher-forced kernel
    // over them (window = hypothesis index of the pass).  ~2.5x fewer flops than the factored attention at ~100
    // rows per window, and all of it on the matrix cores.
    const int nw = e->tf_nwin;
    GemmEpi ep = epi_of(EPI_CROSS_KV, e->a_kv.p, 0, e->Wf("dec.ckv.b") + (size_t)l * 2 * d);
    ep.rpb = T; ep.d = d; ep.head_dim = 64; ep.n_head = H; ep.n_slots = nw; ep.slot0 = 0;
    gemm_p(e, P_CROSSKV_GEMM, amat(e->a_enc.as<bf16>(), d), e->Wb("dec.ckv.w") + (size_t)l * 2 * d * d, d, nw * T, 2 * d, d,
           ep, st);
    const bf16* kv = e->a_kv.as<bf16>();
    const size_t po = (size_t)r0 * H * 16;
    ProfScope ps(e, P_CROSS_ATTN, st, 0, 0, true);
    launch_cross_attn(q, d, kv, kv + (size_t)nw * H * T * 64, T, nullptr, row_hyp, done, ao, d, rows, H, cross_group,
                      e->s_pm.as<float>() + po, e->s_pl.as<float>() + po, e->s_po.as<float>() + po * 64, probs, hmap,
                      n_align, sl.total_rows, e->cross_cap, fz, e->dstat(P_CROSS_ATTN), st, ps.a, ps.b);
  } else if (e->cross_mode == 1) {
    // factored: q' = Wk_h^T q_h, attention over the encoder output, split merge + Wv_h (attn_xenc.hip)
    const XPlan plan = xattn_plan(sl.total_rows, cross_group, H, T, d, xattn_chunks_ok(e));
    const int splits = plan.slabs;
    const size_t prow = (size_t)H * d;
    bf16* qp = e->s_qp.as<bf16>() + (size_t)r0 * prow;
    bf16* pu = e->s_pu.as<bf16>() + (size_t)r0 * 16;         // blocked layout: rows are 16-element records
    float* pml = e->s_pml.as<float>() + (size_t)r0 * H * 2;
    const bf16* wkt = e->xwkt.as<bf16>() + (size_t)l * H * d * 64;
    const bf16* wv = e->xwvb.as<bf16>() + (size_t)l * H * d * 64;
    const float* bv = e->Wf("dec.ckv.b") + (size_t)l * 2 * d + d;
    {
      ProfScope ps(e, P_DEC_GEMM, st, 2.0 * rows * H * d * 64, 2.0 * H * d * 64 + 2.0 * rows * d + 2.0 * rows * prow);
      launch_xq(q, d, fz, wkt, qp, rows, H, d, st);
    }
    {
      ProfScope ps(e, P_CROSS_ATTN, st, 0, 0, true);
      launch_xattn(qp, e->xenc.p, e->cross_fp8 ? e->xscale.as<float>() : nullptr, e->d_hyp_slot.as<int>(), row_hyp, done, rows, sl.total_rows, cross_group, H, T,
                   d, plan, e->xsnake ? (l & 1) : 0, e->xkeep, e->xdma, r0 / cross_group, pu, pml, probs, hmap, n_align, e->dstat(P_CROSS_ATTN), st, ps.a, ps.b);
    }
    {
      ProfScope ps(e, P_CROSS_COMB, st, 2.0 * rows * d * d, 2.0 * d * d + 2.0 * splits * rows * prow + 2.0 * rows * d);
      launch_xcomb_vo(pu, pml, plan, r0 / cross_group, sl.total_rows, wv, bv, row_hyp, done, ao, d, rows, cross_group, H, d, T, probs, hmap,
                      n_align, st);
    }
  } else {
    const size_t po = (size_t)r0 * H * 16;
    ProfScope ps(e, P_CROSS_ATTN, st, 0, 0, true);
    launch_cross_attn(q, d, ckv + (size_t)(2 * l) * ckv_layer, ckv + (size_t)(2 * l + 1) * ckv_layer, T,
                      e->d_hyp_slot.as<int>(), row_hyp, done, ao, d, rows, H, cross_group, e->s_pm.as<float>() + po,
                      e->s_pl.as<float>() + po, e->s_po.as<float>() + po * 64, probs, hmap, n_align, sl.total_rows,
                      e->cross_cap, fz, e->dstat(P_CROSS_ATTN), st, ps.a, ps.b);
  }
  if (probs) HIP_OK(hipStreamSynchronize(st));   // the head map buffer is reused by the next layer
  gemm(DEC_COUT, amat(ao, d), W.cout_w, d, d, d,
       fold ? fold_producer(W.cout_b, W.ln3_w) : ln_fuse ? resid_stat(W.cout_b) : resid_ln(W.ln3_w, W.ln3_b, W.cout_b));
  {
    GemmEpi ep = epi_of(EPI_BF16, ff, 4LL * d, W.fc1_b);
    ep.act = 1;
    if (fold) gemm(DEC_FC1, fold_operand(d / 16), W.fc1_w, d, 4 * d, d, fold_epi(ep, 8 * (size_t)d, 4 * d));
    else gemm(DEC_FC1, ln_fuse ? ln_operand(W.ln3_w, W.ln3_b) : amat(hb, d), W.fc1_w, d, 4 * d, d, ep);
  }
  if (l + 1 < L) {
    const auto& Wn = dec_weights(e)[l + 1];
    if (fold) {
      gemm(DEC_FC2, amat(ff, 4LL * d), W.fc2_w, 4LL * d, d, 4 * d, fold_producer(W.fc2_b, Wn.ln1_w));
    } else {
      gemm(DEC_FC2, amat(ff, 4LL * d), W.fc2_w, 4LL * d, d, 4 * d,
           fc2_fuse ? resid_stat(W.fc2_b) : resid_ln(Wn.ln1_w, Wn.ln1_b, W.fc2_b));
    }
  } else {
    gemm(DEC_FC2, amat(ff, 4LL * d), W.fc2_w, 4LL * d, d, 4 * d, epi_of(EPI_RESID_F32, x, d, W.fc2_b));
  }
}

// One decoder pass over `rows` rows; logits for the n_logit rows listed in logit_rows (device; nullptr =
// rows 0..n_logit-1) go to `logits`.  Optional cross-attention capture (align): head_map per layer computed
// by caller.
//
// Decode steps (logit_rows == nullptr, n_logit == rows, no capture) with enough rows split the rows into two
// slices on two streams, the second started when the first reaches its layer-0 cross-attention.  Each
// slice then alternates a latency-bound chain of skinny weight GEMMs with an HBM-bound cross-attention,
// and the two slices run in opposite phase: one slice's GEMM chain executes while the other streams its
// cross-KV, so the step costs ~max(chain, cross) per layer instead of their sum.  The weights are read once
// per slice (46 MB per layer for large-v3, against 1.15 GB of cross-KV), and every row sees exactly the
// same arithmetic as in a one-slice pass.
void decoder_pass(wm_engine* e, int rows, const int* row_tok, const int* row_pos, const int* row_hyp, const int* done,
                  const int* lin, const int* logit_rows, int n_logit, float* logits,
                  const std::vector<std::vector<int>>* align_map, int n_align, float* attn, int cross_group,
                  hipStream_t st, int* err = nullptr) {
  const auto& m = e->dm;
  const int d = m.n_state, L = m.n_dec_layer;
  const auto& W0 = dec_weights(e)[0];
  // host-side check of the row buffers against what the launches below index (rows of the pass, and the
  // final LayerNorm's gathered logit rows)
  if ((size_t)rows * d * 4 > e->s_x.bytes || (size_t)std::max(rows, n_logit) * d * 2 > e->s_hb.bytes)
    throw std::runtime_error("decoder_pass: row buffers smaller than the pass (" + std::to_string(rows) + " rows, " +
                             std::to_string(n_logit) + " logit rows)");
  if (e->cross_mode == 1) {
    // factored cross-attention scratch for the whole pass (slices index it by absolute row), and the
    // per-head Wk^T layout (packed once per upload of dec.ckv.w)
    const int H = m.n_head, T = m.n_audio_ctx;
    const size_t prow = (size_t)H * d;
    const int splits = xattn_plan(rows, cross_group, H, T, d, xattn_chunks_ok(e)).slabs;
    e->s_qp.ensure((size_t)rows * prow * 2);
    e->s_pu.ensure((size_t)splits * rows * prow * 2);
    e->s_pml.ensure((size_t)splits * rows * H * 2 * 4);
    if (!e->xwkt_ready) {
      e->xwkt.ensure((size_t)L * H * d * 64 * 2);
      e->xwvb.ensure((size_t)L * H * d * 64 * 2);
      launch_xpack(e->Wb("dec.ckv.w"), e->xwkt.as<bf16>(), e->xwvb.as<bf16>(), L, H, d, st);
      e->xwkt_ready = true;
    }
    if (!e->xenc.p) throw std::runtime_error("decoder: no encoder slots (wm_reserve + wm_cross_kv first)");
  }
  if (e->dec_ln_fold && !e->fold_ready) {
    const int L2 = m.n_dec_layer;
    e->fold_vec.ensure((size_t)L2 * 16 * d * 4);
    for (int l = 0; l < L2; ++l) {
      const auto& W = dec_weights(e)[l];
      float* f = e->fold_vec.as<float>() + (size_t)l * 16 * d;
      launch_fold_vectors(W.qkv_w, 3 * d, d, W.ln1_w, W.ln1_b, W.qkv_b, f, f + 3 * d, st);
      launch_fold_vectors(W.cq_w, d, d, W.ln2_w, W.ln2_b, W.cq_b, f + 6 * d, f + 7 * d, st);
      launch_fold_vectors(W.fc1_w, 4 * d, d, W.ln3_w, W.ln3_b, W.fc1_b, f + 8 * d, f + 12 * d, st);
    }
    e->fold_ready = true;
  }
  int h0 = (rows / 2 / cross_group) * cross_group;
  const bool split = e->dec_split && logit_rows == nullptr && n_logit == rows && attn == nullptr && h0 >= 16 &&
                     rows - h0 >= 16;
  std::vector<DecSlice> sl;
  if (split) {
    if (!e->st2) {
      int lo = 0, hi = 0;
      HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_OK(hipStreamCreateWithPriority(&e->st2, hipStreamNonBlocking, hi));
      HIP_OK(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&e->ev_mid, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
    }
    sl.push_back({0, h0, rows, st, &e->gemm_ws});
    sl.push_back({h0, rows - h0, rows, e->st2, &e->gemm_ws2});
    HIP_OK(hipEventRecord(e->ev_fork, st));
    HIP_OK(hipStreamWaitEvent(e->st2, e->ev_fork, 0));
  } else {
    sl.push_back({0, rows, rows, st, &e->gemm_ws});
  }
  for (const auto& s : sl) {
    ProfScope ps(e, P_DEC_OTHER, s.st);
    float* x = e->s_x.as<float>() + (size_t)s.r0 * d;
    launch_embed(row_tok + s.r0, row_pos + s.r0, e->Wb("dec.embed"), e->Wf("dec.pos"), x, s.rows, d, m.n_vocab, m.n_text_ctx,
                 s.st, err);
    launch_layernorm(x, d, nullptr, s.rows, d, W0.ln1_w, W0.ln1_b, e->s_hb.as<bf16>() + (size_t)s.r0 * d, d, s.st);
  }
  for (int l = 0; l < L; ++l) {
    for (size_t i = 0; i < sl.size(); ++i) {
      if (split && l == 0 && i == 1) HIP_OK(hipStreamWaitEvent(e->st2, e->ev_mid, 0));
      decoder_layer(e, sl[i], l, row_pos, row_hyp, done, lin, align_map, n_align, attn, cross_group,
                    (split && l == 0 && i == 0) ? e->ev_mid : nullptr);
    }
  }
  for (const auto& s : sl) {
    const int nl = split ? s.rows : n_logit;
    const int* lr = split ? nullptr : logit_rows;
    {
      ProfScope ps(e, P_DEC_OTHER, s.st);
      launch_layernorm(e->s_x.as<float>() + (size_t)s.r0 * d, d, lr, nl, d, e->Wf("dec.ln.w"), e->Wf("dec.ln.b"),
                       e->s_hb.as<bf16>() + (size_t)s.r0 * d, d, s.st);
    }
    const size_t wsb = 64ull << 20;
    s.ws->ensure(wsb);
    ProfScope ps(e, P_LOGITS_GEMM, s.st, 2.0 * nl * m.n_vocab * d, gemm_bytes(nl, m.n_vocab, d, 4));
    launch_gemm(amat(e->s_hb.as<bf16>() + (size_t)s.r0 * d, d), e->Wb("dec.embed"), d, nl, m.n_vocab, d,
                epi_of(EPI_F32, logits + (size_t)s.r0 * m.n_vocab, m.n_vocab, nullptr), s.ws->as<float>(), wsb, s.st);
  }
  if (split) {
    HIP_OK(hipEventRecord(e->ev_join, e->st2));
    HIP_OK(hipStreamWaitEvent(st, e->ev_join, 0));
  }
}

void check_weights(wm_engine* e) {
  for (auto& kv : e->slots)
    if (!kv.second.set) throw std::runtime_error("weight not set: " + kv.first);
}

void reserve(wm_engine* e, int n_slots, int n_hyp) {
  const auto& m = e->dm;
  const int H = m.n_head, C = m.n_text_ctx, T = m.n_audio_ctx, L = m.n_dec_layer;
  if (n_slots > e->n_slots) {
    // factored mode keeps each window's encoder output (T x d bf16); projected mode its L x 2 K/V panels
    e->ckv.release();
    e->xenc.release();
    e->xscale.release();
    if (e->cross_mode == 1) {
      // bf16: tile-blocked slots (attn_xenc.hip xblock_kernel), T padded to whole 32-row tiles
      e->xenc.ensure(e->cross_fp8 ? (size_t)n_slots * T * m.n_state : (size_t)n_slots * xblock_slot_elems(T, m.n_state) * 2);
      if (e->cross_fp8) e->xscale.ensure((size_t)n_slots * T * 4);
    } else {
      e->ckv.ensure((size_t)L * 2 * n_slots * H * T * 64 * 2);
    }
    e->n_slots = n_slots;
  }
  if (n_hyp > e->n_hyp_cap) {
    e->skv.release();
    e->skv.ensure((size_t)L * 2 * n_hyp * H * C * 64 * 2);
    e->n_hyp_cap = n_hyp;
    const size_t nh = n_hyp;
    e->d_tokens.ensure(nh * C * 4);
    e->d_lin.ensure(nh * C * 4);
    e->d_seq_len.ensure(nh * 4);
    e->d_done.ensure(nh * 4);
    e->d_cum.ensure(nh * 4);
    e->d_row_tok.ensure(nh * 4);
    e->d_row_pos.ensure(nh * 4);
    e->d_row_hyp.ensure(nh * 4);
    e->d_hyp_slot.ensure(nh * 4);
    e->d_cand_tok.ensure(nh * 9 * 4);
    e->d_cand_lp.ensure(nh * 9 * 4);
    e->d_ns.ensure(nh * 4);
    e->d_fin_tok.ensure(nh * 16 * C * 4);
    e->d_fin_len.ensure(nh * 16 * 4);
    e->d_fin_cum.ensure(nh * 16 * 4);
    e->d_n_fin.ensure(nh * 4);
  }
  e->d_n_active.ensure(8 * 4);
  e->d_suppress.ensure((size_t)SEARCH_SB * 8);
  e->d_head_map.ensure((size_t)H * 4);
}

// The decode's device error word (d_n_active[1..3]) -> exception (wm_generate returns -1 with this text).
void check_decode_error(const int* w) {
  if (w[0] == 0) return;
  std::string what;
  if (w[0] == WM_ERR_TOKEN_RANGE)
    what = "decoder input token " + std::to_string(w[1]) + " at position " + std::to_string(w[2]) + " outside its table";
  else
    what = std::string(w[0] == WM_ERR_NONFINITE ? "non-finite (NaN / inf) logits" : "no token allowed by the logit rules") +
           " for hypothesis " + std::to_string(w[1]) + " after " + std::to_string(w[2]) + " generated tokens";
  throw std::runtime_error("generate: " + what + "; the decode was stopped");
}

// Search parameters shared by both decode loops (per-call fields: mode, tables, records)
SearchParams search_params(wm_engine* e, const wm_generate_args* a, float* logits, int P) {
  const auto& m = e->dm;
  SearchParams sp;
  std::memset(&sp, 0, sizeof(sp));
  sp.logits = logits; sp.ldl = m.n_vocab; sp.V = m.n_vocab;
  sp.tokens = e->d_tokens.as<int>(); sp.n_ctx = m.n_text_ctx; sp.seq_len = e->d_seq_len.as<int>(); sp.sample_begin = P;
  sp.suppress_bits = e->d_suppress.as<unsigned long long>();
  static const int sel_abl = [] {
    const char* v = std::getenv("VLOG_AMD_SEL_ABL");
    return v ? std::atoi(v) : 0;
  }();
  sp.abl = sel_abl;
  sp.suppress_blank = a->suppress_blank; sp.blank = m.blank;
  sp.eot = m.eot; sp.no_timestamps = m.no_timestamps; sp.ts_begin = m.timestamp_begin;
  sp.max_initial = a->max_initial_timestamp_index; sp.with_ts = a->with_timestamps; sp.done = e->d_done.as<int>();
  sp.seed = a->seed; sp.max_length = a->max_length;
  sp.inv_temperature = a->temperature > 0.f ? 1.0f / a->temperature : 1.0f;
  sp.cum = e->d_cum.as<float>(); sp.row_tok = e->d_row_tok.as<int>(); sp.row_pos = e->d_row_pos.as<int>();
  sp.n_active = e->d_n_active.as<int>(); sp.cand_tok = e->d_cand_tok.as<int>(); sp.cand_lp = e->d_cand_lp.as<float>();
  sp.err = e->d_n_active.as<int>() + 1;
  return sp;
}

void upload_suppress(wm_engine* e, const wm_generate_args* a, hipStream_t st) {
  const int V = e->dm.n_vocab;
  std::vector<unsigned char> sup(V, 0);
  for (int i = 0; i < a->n_suppress; ++i)
    if (a->h_suppress[i] >= 0 && a->h_suppress[i] < V) sup[a->h_suppress[i]] = 1;
  std::vector<unsigned long long> supbits(SEARCH_SB);
  search_suppress_bits(sup.data(), V, supbits.data());
  HIP_OK(hipMemcpyAsync(e->d_suppress.p, supbits.data(), SEARCH_SB * 8, hipMemcpyHostToDevice, st));
  HIP_OK(hipStreamSynchronize(st));
}

// TEST ONLY (options debug_nan_row / debug_nan_count): NaN into logits rows before selection (bytes 0xFF are a NaN)
void debug_nan(wm_engine* e, float* logits, int rows, hipStream_t s) {
  if (e->dbg_nan_row >= 0 && e->dbg_nan_row < rows) {
    const int n = std::min(e->dbg_nan_count, rows - e->dbg_nan_row);
    HIP_OK(hipMemsetAsync(logits + (size_t)e->dbg_nan_row * e->dm.n_vocab, 0xFF, (size_t)n * e->dm.n_vocab * 4, s));
  }
}

// One graph-replayed decode loop's capture state (see generate)
struct StepGraph {
  hipGraphExec_t exec = nullptr;
  bool capturing = false;
  long long gen = -1;                       // realloc_gen() at capture
  void drop() {
    if (exec) (void)hipGraphExecDestroy(exec);
    exec = nullptr;
  }
  // false: buffers moved since the capture (the caller runs an eager step, which re-sizes, then captures again)
  bool valid() const { return !exec || gen == realloc_gen(); }
  template <class F> void run(hipStream_t ds, F&& step) {
    if (!exec) {
      hipGraph_t g = nullptr;
      gen = realloc_gen();
      HIP_OK(hipStreamBeginCapture(ds, hipStreamCaptureModeThreadLocal));
      capturing = true;
      step();
      capturing = false;
      HIP_OK(hipStreamEndCapture(ds, &g));
      const hipError_t ie = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIP_OK(ie);
      if (gen != realloc_gen()) throw std::runtime_error("decode step graph: a buffer moved during capture");
    }
    HIP_OK(hipGraphLaunch(exec, ds));
  }
  void abort(hipStream_t ds) {            // leave the stream out of capture mode before reporting an error
    if (capturing) {
      hipGraph_t g = nullptr;
      if (hipStreamEndCapture(ds, &g) == hipSuccess && g) (void)hipGraphDestroy(g);
      capturing = false;
    }
    drop();
  }
};

void generate_rows(wm_engine* e, const wm_generate_args* a, hipStream_t st);
void generate_rows_beam(wm_engine* e, const wm_generate_args* a, hipStream_t st);

void generate(wm_engine* e, const wm_generate_args* a, hipStream_t st) {
  check_weights(e);
  const auto& m = e->dm;
  const int C = m.n_text_ctx, V = m.n_vocab;
  const int W = a->n_windows, P = a->prompt_len;
  if (W <= 0) return;
  if (P <= 0 || P >= a->max_length || a->max_length > C) throw std::runtime_error("generate: bad prompt_len/max_length");
  if (a->sot_index >= P) throw std::runtime_error("generate: sot_index outside the prompt");
  const bool beam = a->beam_size > 1 && a->temperature <= 0.f;
  const bool sampling = a->temperature > 0.f;
  const int per = beam ? a->beam_size : (sampling ? std::max(1, a->num_hypotheses) : 1);
  const int NH = W * per;
  if (beam && a->beam_size > 8) throw std::runtime_error("generate: beam_size <= 8 supported");
  for (int w = 0; w < W; ++w)
    if (a->h_slots[w] < 0 || a->h_slots[w] >= e->n_slots) throw std::runtime_error("generate: slot out of range");
  for (int i = 0; i < W * P; ++i)
    if (a->h_prompts[i] < 0 || a->h_prompts[i] >= V) throw std::runtime_error("generate: prompt token out of the vocabulary");
  if (a->max_rows < 0) throw std::runtime_error("generate: max_rows must be >= 0");
  if (per == 1 && !beam && ((a->max_rows > 0 && a->max_rows < W) || a->compact)) {
    generate_rows(e, a, st);
    return;
  }
  if (beam && a->max_rows > 0 && a->max_rows < NH) {
    if (a->max_rows < per) throw std::runtime_error("generate: max_rows must hold one window's beam");
    generate_rows_beam(e, a, st);
    return;
  }
  if (a->max_rows > 0 && a->max_rows < W) throw std::runtime_error("generate: max_rows needs greedy, beam search or num_hypotheses 1");
  reserve(e, e->n_slots, NH);
  const bool rec = a->h_token_logprobs != nullptr;
  const int max_cand = beam ? std::max(1, (int)std::lround(a->beam_size * a->patience)) : 0;
  if (max_cand > 16) throw std::runtime_error("generate: beam_size * patience must be <= 16");

  // ---- host-side init of the state tables
  std::vector<int> tokens((size_t)NH * C, 0), lin((size_t)NH * C, 0), seq_len(NH, P), zeros(NH, 0), hyp_slot(NH);
  std::vector<float> cum(NH, 0.f);
  // Beam search: the hypotheses of a window share its prompt, so the prompt is prefilled once per window (into
  // the first hypothesis' self-KV rows) and every hypothesis' lineage points its prompt positions there (the
  // lineage is what beam reordering copies; the cache itself is never copied).  Greedy / sampling keep one
  // prefill per hypothesis: their self-attention reads each row's own cache (no lineage table).
  for (int h = 0; h < NH; ++h) {
    const int w = h / per;
    hyp_slot[h] = a->h_slots[w];
    for (int p = 0; p < P; ++p) tokens[(size_t)h * C + p] = a->h_prompts[(size_t)w * P + p];
    for (int p = 0; p < C; ++p) lin[(size_t)h * C + p] = (beam && p < P) ? w * per : h;
    if (beam && (h % per) != 0) cum[h] = -INFINITY;
  }
  HIP_OK(hipMemcpyAsync(e->d_tokens.p, tokens.data(), tokens.size() * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_lin.p, lin.data(), lin.size() * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_seq_len.p, seq_len.data(), NH * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_done.p, zeros.data(), NH * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_n_fin.p, zeros.data(), NH * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_cum.p, cum.data(), NH * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_hyp_slot.p, hyp_slot.data(), NH * 4, hipMemcpyHostToDevice, st));
  upload_suppress(e, a, st);
  const int counter0[4] = {NH, 0, 0, 0};          // live hypotheses; error word cleared
  HIP_OK(hipMemcpyAsync(e->d_n_active.p, counter0, sizeof(counter0), hipMemcpyHostToDevice, st));
  if (rec) {
    e->d_tok_lp.ensure((size_t)NH * C * 4);
    if (!beam) e->d_tok_lp_o.ensure((size_t)NH * C * 4);
    else e->d_fin_lp.ensure((size_t)W * max_cand * C * 4);
  }

  // ---- prefill: rows (h, p) for every prompt position of every prefilled hypothesis (beam: one per window)
  const int pf_per = beam ? per : 1;                 // hypotheses per prefilled row set
  const int n_pf = NH / pf_per;
  const int rows = n_pf * P;
  const int nlog = a->sot_index >= 0 ? 2 * NH : NH;
  // the pass's final LayerNorm gathers its nlog logit rows into s_hb rows [0, nlog): with the beam's shared
  // prefill (rows = W * P) that can exceed the pass rows, so the row buffers hold max(rows, NH, nlog)
  ensure_step(e, std::max(std::max(rows, NH), nlog), std::max(nlog, NH));
  {
    std::vector<int> rt(rows), rp(rows), rh(rows), lr(nlog);
    for (int i = 0; i < n_pf; ++i)
      for (int p = 0; p < P; ++p) {
        const int r = i * P + p, h = i * pf_per;
        rt[r] = tokens[(size_t)h * C + p]; rp[r] = p; rh[r] = h;
      }
    for (int h = 0; h < NH; ++h) {            // a hypothesis' logits come from its row set's last prompt row
      const int i = h / pf_per;
      lr[h] = i * P + P - 1;
      if (a->sot_index >= 0) lr[NH + h] = i * P + a->sot_index;
    }
    HIP_OK(hipMemcpyAsync(e->d_prow_tok.p, rt.data(), rows * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(e->d_prow_pos.p, rp.data(), rows * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(e->d_prow_hyp.p, rh.data(), rows * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(e->d_logit_rows.p, lr.data(), nlog * 4, hipMemcpyHostToDevice, st));
    std::vector<int> ident(NH);
    for (int h = 0; h < NH; ++h) ident[h] = h;
    HIP_OK(hipMemcpyAsync(e->d_row_hyp.p, ident.data(), NH * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));   // host vectors above go out of scope
  }
  float* logits = e->s_logits.as<float>();
  int* err = e->d_n_active.as<int>() + 1;
  decoder_pass(e, rows, e->d_prow_tok.as<int>(), e->d_prow_pos.as<int>(), e->d_prow_hyp.as<int>(), nullptr,
               e->d_lin.as<int>(), e->d_logit_rows.as<int>(), nlog, logits, nullptr, 0, nullptr, (per / pf_per) * P, st, err);
  if (a->sot_index >= 0) launch_no_speech(logits + (size_t)NH * V, V, V, NH, m.no_speech, e->d_ns.as<float>(), st);

  SearchParams sp = search_params(e, a, logits, P);
  sp.mode = beam ? 1 : (sampling ? 2 : 0); sp.topk = beam ? a->beam_size + 1 : 1;
  if (rec) {
    sp.tok_lp = e->d_tok_lp.as<float>();
    if (!beam) sp.tok_lp_other = e->d_tok_lp_o.as<float>();
  }
  BeamParams bp;
  std::memset(&bp, 0, sizeof(bp));
  bp.beam = a->beam_size; bp.max_cand = max_cand; bp.n_ctx = C; bp.sample_begin = P; bp.max_length = a->max_length;
  bp.eot = m.eot; bp.cand_tok = sp.cand_tok; bp.cand_lp = sp.cand_lp; bp.tokens = sp.tokens; bp.lin = e->d_lin.as<int>();
  bp.seq_len = sp.seq_len; bp.cum = sp.cum; bp.done = sp.done; bp.row_tok = sp.row_tok; bp.row_pos = sp.row_pos;
  bp.fin_tok = e->d_fin_tok.as<int>(); bp.fin_len = e->d_fin_len.as<int>(); bp.fin_cum = e->d_fin_cum.as<float>();
  bp.n_fin = e->d_n_fin.as<int>(); bp.n_active = sp.n_active;
  if (rec && beam) {
    bp.tok_lp = e->d_tok_lp.as<float>();
    bp.fin_lp = e->d_fin_lp.as<float>();
  }

  auto select = [&](int step) {
    sp.step = step;
    debug_nan(e, logits, NH, st);
    ProfScope ps(e, P_SELECT, st);
    launch_logits_select(sp, NH, st);
    if (beam) launch_beam_select(bp, W, st);
  };
  select(0);
  int steps = 1;
  long long row_steps = NH;                      // the prefill pass selects every hypothesis' first token
  int captures = 0;
  const int max_steps = a->max_length - P;      // generated tokens (incl. the final one) <= max_length - P
  const int check = std::max(1, a->check_every);
  // A decode step's launches are identical from step to step: every per-step quantity (tokens, positions,
  // lineage, done flags, sequence lengths) lives in device memory and is advanced by the select kernels, so
  // after one eager step (which sizes every scratch buffer) the step is captured once as a HIP graph and
  // replayed: one graph launch per step instead of ~11 kernel launches per layer.  Not with the event profiler
  // (its events are per launch) or the two-stream split.  The replay stream is joined to `st` before every
  // host poll and at the end.
  const bool use_graph = e->dec_graph && !e->prof_on && !e->dec_split;
  hipGraphExec_t gexec = nullptr;
  bool capturing = false;
  hipStream_t ds = st;
  if (use_graph) {
    if (!e->gst) {
      HIP_OK(hipStreamCreateWithFlags(&e->gst, hipStreamNonBlocking));
      HIP_OK(hipEventCreateWithFlags(&e->ev_g0, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&e->ev_g1, hipEventDisableTiming));
    }
    HIP_OK(hipEventRecord(e->ev_g0, st));
    HIP_OK(hipStreamWaitEvent(e->gst, e->ev_g0, 0));
    ds = e->gst;
  }
  // Beam compaction (a->compact): once the live windows' hypotheses fill <= 7/8 of the pass, the pass keeps only
  // them (row r -> hypothesis row_hyp[r], window groups stay contiguous); the beam state stays where it is, per
  // hypothesis (KV cache, lineage, tokens), so the rows' tokens / positions are gathered per pass (rows_fill) and
  // the selection reads its logits row by row.  Finished windows then stop costing GEMM rows in the tail.
  int nrows = NH;
  const bool bcompact = beam && a->compact;
  std::vector<int> h_rows(NH), h_bdone;
  for (int h = 0; h < NH; ++h) h_rows[h] = h;
  auto step_eager = [&](int step, hipStream_t s) {
    // logits rows of a decode step are the hypotheses themselves
    // greedy / sampling never reorder hypotheses: the lineage table is the identity and self-attention
    // reads each row's own cache directly (no dependent lineage load per key block)
    if (nrows < NH) {
      launch_rows_fill(nrows, e->d_row_hyp.as<int>(), e->d_prow_tok.as<int>(), e->d_prow_pos.as<int>(),
                       e->d_row_tok.as<int>(), e->d_row_pos.as<int>(), s);
      decoder_pass(e, nrows, e->d_prow_tok.as<int>(), e->d_prow_pos.as<int>(), e->d_row_hyp.as<int>(), e->d_done.as<int>(),
                   e->d_lin.as<int>(), nullptr, nrows, logits, nullptr, 0, nullptr, per, s, err);
    } else {
      decoder_pass(e, NH, e->d_row_tok.as<int>(), e->d_row_pos.as<int>(), e->d_row_hyp.as<int>(), e->d_done.as<int>(),
                   beam ? e->d_lin.as<int>() : nullptr, nullptr, NH, logits, nullptr, 0, nullptr, per, s, err);
    }
    sp.step = step;
    debug_nan(e, logits, nrows, s);
    ProfScope ps(e, P_SELECT, s);
    launch_logits_select(sp, nrows, s);
    if (beam) launch_beam_select(bp, W, s);
  };
  StepGraph graph;
  int poll[4] = {0, 0, 0, 0};                   // live count + error word
  bool eager_next = false;                      // the pass after a compaction runs eagerly (sizes scratch), then captures
  if (bcompact) h_bdone.resize(NH);
  try {
    for (int step = 1; step < max_steps; ++step) {
      if ((step - 1) % check == 0) {
        HIP_OK(hipMemcpyAsync(poll, e->d_n_active.p, sizeof(poll), hipMemcpyDeviceToHost, ds));
        if (bcompact) HIP_OK(hipMemcpyAsync(h_bdone.data(), e->d_done.p, (size_t)NH * 4, hipMemcpyDeviceToHost, ds));
        HIP_OK(hipStreamSynchronize(ds));
        check_decode_error(poll + 1);
        if (poll[0] <= 0) break;
        // (beam passes are GEMM-row-bound at hundreds of rows, unlike the latency-bound greedy passes: compact at 7/8)
        if (bcompact && poll[0] * 8 <= nrows * 7) {
          // a finished window's hypotheses are all done (beam_select); keep the live windows' groups in order
          int n = 0;
          for (int r = 0; r < nrows; r += per) {
            const int h0 = h_rows[r];
            if (h_bdone[h0]) continue;
            for (int b = 0; b < per; ++b) h_rows[n + b] = h0 + b;
            n += per;
          }
          if (n > 0 && n < nrows) {
            nrows = n;
            HIP_OK(hipMemcpyAsync(e->d_row_hyp.p, h_rows.data(), (size_t)nrows * 4, hipMemcpyHostToDevice, ds));
            HIP_OK(hipStreamSynchronize(ds));
            sp.row_hyp = e->d_row_hyp.as<int>();
            graph.drop();
            eager_next = true;
          }
        }
      }
      if (!graph.valid()) {                     // a buffer moved since the capture: one eager pass re-sizes
        graph.drop();
        eager_next = true;
      }
      if (!use_graph || step == 1 || eager_next) {
        eager_next = false;
        step_eager(step, use_graph ? ds : st);
      } else {
        if (!graph.exec) ++captures;
        graph.run(ds, [&] { step_eager(step, ds); });
      }
      ++steps;
      row_steps += nrows;
    }
  } catch (...) {
    graph.abort(ds);
    throw;
  }
  if (use_graph) {
    HIP_OK(hipEventRecord(e->ev_g1, ds));
    HIP_OK(hipStreamWaitEvent(st, e->ev_g1, 0));
  }
  if (graph.exec) {
    HIP_OK(hipStreamSynchronize(ds));          // the graph's last replay has completed before it is destroyed
    graph.drop();
  }

  // ---- results
  std::vector<int> out_tok((size_t)NH * C), out_len(NH);
  std::vector<float> out_cum(NH), ns(NH, 0.f), out_lp, out_lpo, fin_lp;
  HIP_OK(hipMemcpyAsync(out_tok.data(), e->d_tokens.p, out_tok.size() * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(out_len.data(), e->d_seq_len.p, NH * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(out_cum.data(), e->d_cum.p, NH * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(poll, e->d_n_active.p, sizeof(poll), hipMemcpyDeviceToHost, st));
  if (a->sot_index >= 0) HIP_OK(hipMemcpyAsync(ns.data(), e->d_ns.p, NH * 4, hipMemcpyDeviceToHost, st));
  if (rec) {
    out_lp.resize((size_t)NH * C);
    HIP_OK(hipMemcpyAsync(out_lp.data(), e->d_tok_lp.p, out_lp.size() * 4, hipMemcpyDeviceToHost, st));
    if (!beam) {
      out_lpo.resize((size_t)NH * C);
      HIP_OK(hipMemcpyAsync(out_lpo.data(), e->d_tok_lp_o.p, out_lpo.size() * 4, hipMemcpyDeviceToHost, st));
    }
  }
  std::vector<int> fin_tok, fin_len, n_fin;
  std::vector<float> fin_cum;
  if (beam) {
    fin_tok.resize((size_t)W * max_cand * C); fin_len.resize((size_t)W * max_cand); fin_cum.resize((size_t)W * max_cand);
    n_fin.resize(W);
    HIP_OK(hipMemcpyAsync(fin_tok.data(), e->d_fin_tok.p, fin_tok.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(fin_len.data(), e->d_fin_len.p, fin_len.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(fin_cum.data(), e->d_fin_cum.p, fin_cum.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(n_fin.data(), e->d_n_fin.p, W * 4, hipMemcpyDeviceToHost, st));
    if (rec) {
      fin_lp.resize((size_t)W * max_cand * C);
      HIP_OK(hipMemcpyAsync(fin_lp.data(), e->d_fin_lp.p, fin_lp.size() * 4, hipMemcpyDeviceToHost, st));
    }
  }
  HIP_OK(hipStreamSynchronize(st));
  check_decode_error(poll + 1);
  const float lp = a->length_penalty;
  auto norm = [&](float c, int n) { return c / std::pow((float)std::max(n, 1), lp); };
  const int ML = a->max_length;
  for (int w = 0; w < W; ++w) {
    int best_len = 0;
    float best_cum = 0.f, best_score = -INFINITY;
    const int* best_ptr = nullptr;
    const float *best_lp = nullptr, *best_lpo = nullptr;   // records of the chosen hypothesis (first generated step)
    if (beam) {
      struct C2 { const int* t; int n; float c; const float* r; };
      std::vector<C2> cands;
      for (int i = 0; i < n_fin[w]; ++i) {
        const size_t f = (size_t)w * max_cand + i;
        cands.push_back({&fin_tok[f * C], fin_len[f], fin_cum[f], rec ? &fin_lp[f * C] : nullptr});
      }
      if ((int)cands.size() < a->beam_size) {       // openai finalize: add unfinished beams by sum_logprob
        std::vector<int> order;
        for (int b = 0; b < per; ++b)
          if (out_cum[w * per + b] > -INFINITY) order.push_back(b);
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return out_cum[w * per + x] > out_cum[w * per + y]; });
        for (int b : order) {
          if ((int)cands.size() >= a->beam_size) break;
          const int h = w * per + b;
          cands.push_back({&out_tok[(size_t)h * C + P], out_len[h] - P, out_cum[h], rec ? &out_lp[(size_t)h * C + P] : nullptr});
        }
      }
      for (const auto& c : cands) {
        const float s = norm(c.c, c.n);
        if (s > best_score) { best_score = s; best_len = c.n; best_cum = c.c; best_ptr = c.t; best_lp = c.r; }
      }
    } else {
      for (int j = 0; j < per; ++j) {
        const int h = w * per + j;
        const int n = out_len[h] - P;
        const float s = norm(out_cum[h], n);
        if (s > best_score) {
          best_score = s; best_len = n; best_cum = out_cum[h]; best_ptr = &out_tok[(size_t)h * C + P];
          if (rec) { best_lp = &out_lp[(size_t)h * C + P]; best_lpo = &out_lpo[(size_t)h * C + P]; }
        }
      }
    }
    for (int i = 0; i < best_len && i < ML; ++i) a->h_tokens[(size_t)w * ML + i] = best_ptr[i];
    a->h_lengths[w] = best_len;
    a->h_scores[w] = best_score;
    if (a->h_cum_logprob) a->h_cum_logprob[w] = best_cum;
    if (a->h_no_speech) a->h_no_speech[w] = ns[w * per];
    if (rec) {
      // one record per generated token, plus the final <|endoftext|> when the window ended on it
      const int nr = std::min(ML, best_len + (P + best_len < ML ? 1 : 0));
      for (int i = 0; i < nr; ++i) {
        a->h_token_logprobs[(size_t)w * ML + i] = best_lp ? best_lp[i] : NAN;
        if (a->h_token_logprobs_other) a->h_token_logprobs_other[(size_t)w * ML + i] = best_lpo ? best_lpo[i] : NAN;
      }
    }
  }
  if (a->h_stats) {
    a->h_stats[0] = steps;
    a->h_stats[1] = row_steps;
    a->h_stats[2] = 0;
    a->h_stats[3] = captures;
  }
  if (a->h_steps) a->h_steps[0] = steps;
}

// Row-set decode: greedy (or sampling with one hypothesis) over W windows with at most R = max_rows in flight.
//
// A batch of 30 s windows ends when its LONGEST window does (speech density varies: a few tokens for silence, 200+
// for dense speech), and every decode step pays the weight-streaming GEMM chain however many rows are still live.
// Here the decode keeps a ROW SET: hypothesis slot h of row r holds one window; when the host check finds rows
// whose window ended, it starts the next windows (in h_slots order, which the host sorts longest-expected first)
// in those rows.  The new windows' prompts are prefilled INSIDE that step's decoder pass (pass rows = one decode
// row per live hypothesis + P prompt rows per new one; the final LayerNorm gathers one logits row per row-set row
// in row order), so a refill costs no extra pass.  Rows stay in place while windows wait, so the captured step
// graph stays valid; once the queue is empty and compaction is on, the live rows are packed densely when they
// fall to 7/8 of the pass (row_compact_8ths; re-capture for the new count).  A finished hypothesis' tokens are copied to the
// per-window output tables by the block that ends it (search.hip), since its slot is then reused.
void generate_rows(wm_engine* e, const wm_generate_args* a, hipStream_t st) {
  const auto& m = e->dm;
  const int C = m.n_text_ctx, V = m.n_vocab;
  const int W = a->n_windows, P = a->prompt_len;
  const int R = a->max_rows > 0 ? std::min(a->max_rows, W) : W;
  const bool rec = a->h_token_logprobs != nullptr;
  const int ML = a->max_length;
  reserve(e, e->n_slots, R);
  // per-window inputs and outputs
  e->d_win_prompt.ensure((size_t)W * P * 4);
  e->d_win_slot.ensure((size_t)W * 4);
  e->d_hyp_out.ensure((size_t)R * 4);
  e->d_res_tok.ensure((size_t)W * C * 4);
  e->d_res_len.ensure((size_t)W * 4);
  e->d_res_cum.ensure((size_t)W * 4);
  e->d_res_ns.ensure((size_t)W * 4);
  if (rec) {
    e->d_tok_lp.ensure((size_t)R * C * 4);
    e->d_tok_lp_o.ensure((size_t)R * C * 4);
    e->d_res_lp.ensure((size_t)W * C * 4);
    e->d_res_lp_o.ensure((size_t)W * C * 4);
  }
  HIP_OK(hipMemcpyAsync(e->d_win_prompt.p, a->h_prompts, (size_t)W * P * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_win_slot.p, a->h_slots, (size_t)W * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemsetAsync(e->d_res_ns.p, 0, (size_t)W * 4, st));
  HIP_OK(hipMemsetAsync(e->d_n_active.p, 0, 4 * 4, st));      // live counter, error word
  {
    std::vector<int> ones(R, 1);               // every slot starts ended (no hypothesis)
    HIP_OK(hipMemcpyAsync(e->d_done.p, ones.data(), (size_t)R * 4, hipMemcpyHostToDevice, st));
    upload_suppress(e, a, st);                 // (synchronises: `ones` goes out of scope)
  }
  // pass rows: R decode rows + P prompt rows per starting window; logits rows: R + one sot row per start
  ensure_step(e, R * (1 + P), 2 * R);
  float* logits = e->s_logits.as<float>();
  int* counters = e->d_n_active.as<int>();     // [0] live hypotheses, [1..3] error word
  int* err = counters + 1;
  SearchParams sp = search_params(e, a, logits, P);
  sp.mode = a->temperature > 0.f ? 2 : 0;
  sp.topk = 1;
  sp.row_hyp = e->d_row_hyp.as<int>();
  sp.hyp_out = e->d_hyp_out.as<int>();
  sp.res_tok = e->d_res_tok.as<int>(); sp.res_len = e->d_res_len.as<int>(); sp.res_cum = e->d_res_cum.as<float>();
  if (rec) {
    sp.tok_lp = e->d_tok_lp.as<float>(); sp.tok_lp_other = e->d_tok_lp_o.as<float>();
    sp.res_lp = e->d_res_lp.as<float>(); sp.res_lp_other = e->d_res_lp_o.as<float>();
  }

  // host view: row r holds hypothesis slot row_hyp[r]; slot h decodes window hyp_win[h] while live[h]
  std::vector<int> row_hyp(R), hyp_win(R, -1);
  std::vector<char> live(R, 0);
  for (int r = 0; r < R; ++r) row_hyp[r] = r;
  int nrows = R, next = 0;
  long long passes = 0, row_steps = 0, refills = 0;
  int captures = 0;

  // One event pass.  `carry` per new row: the old row index of a carried live row, -1 for a row whose slot starts
  // a window (`starts`, in row order), -2 for an idle row (its slot ended; the selection skips it).
  std::vector<int> carry, new_row_hyp;
  std::vector<std::pair<int, int>> starts;      // (slot, window)
  auto event = [&](hipStream_t s) {
    const int nr = (int)new_row_hyp.size(), nst = (int)starts.size();
    const int nsot = a->sot_index >= 0 ? nst : 0;
    int np = 0, n_live = 0;
    for (int c : carry) {
      np += c >= 0 ? 1 : (c == -1 ? P : 0);
      n_live += c >= -1;
    }
    // upload: ptok, ppos, phyp, psrc [np] | row set [nr] | logits rows [nr + nsot] | start slots, windows [nst] | live
    std::vector<int>& u = e->h_ev;
    u.assign((size_t)4 * np + 2 * nr + nsot + 2 * nst + 1, 0);
    int* ptok = u.data(); int* ppos = ptok + np; int* phyp = ppos + np; int* psrc = phyp + np;
    int* rh = psrc + np; int* lr = rh + nr; int* hs = lr + nr + nsot; int* ws = hs + nst;
    ws[nst] = n_live;
    int i = 0, k = 0;
    for (int r = 0; r < nr; ++r) {
      rh[r] = new_row_hyp[r];
      if (carry[r] >= 0) {
        phyp[i] = new_row_hyp[r]; psrc[i] = carry[r];
        lr[r] = i++;
      } else if (carry[r] == -1) {
        const int h = starts[k].first, w = starts[k].second;
        for (int p = 0; p < P; ++p, ++i) {
          ptok[i] = a->h_prompts[(size_t)w * P + p]; ppos[i] = p; phyp[i] = h; psrc[i] = -1;
          if (p == a->sot_index) lr[nr + k] = i;
        }
        lr[r] = i - 1;                          // the last prompt position predicts the first token
        hs[k] = h; ws[k] = w;
        ++k;
      } else {
        lr[r] = 0;
      }
    }
    e->d_ev.ensure(u.size() * 4);
    int* du = e->d_ev.as<int>();
    HIP_OK(hipMemcpyAsync(du, u.data(), u.size() * 4, hipMemcpyHostToDevice, s));
    int* dptok = du; int* dppos = du + np; int* dphyp = du + 2 * np; int* dpsrc = du + 3 * np;
    int* drh = du + 4 * np; int* dlr = drh + nr; int* dhs = dlr + nr + nsot; int* dws = dhs + nst;
    // carried rows read token / position from the last selection's (old) row order before it is overwritten
    launch_rows_fill(np, dpsrc, dptok, dppos, e->d_row_tok.as<int>(), e->d_row_pos.as<int>(), s);
    launch_hyp_start(nst, dhs, dws, e->d_win_prompt.as<int>(), P, e->d_win_slot.as<int>(), C, e->d_tokens.as<int>(),
                     e->d_seq_len.as<int>(), e->d_done.as<int>(), e->d_cum.as<float>(), e->d_hyp_slot.as<int>(),
                     e->d_hyp_out.as<int>(), s);
    HIP_OK(hipMemcpyAsync(e->d_row_hyp.p, drh, (size_t)nr * 4, hipMemcpyDeviceToDevice, s));
    HIP_OK(hipMemcpyAsync(counters, dws + nst, 4, hipMemcpyDeviceToDevice, s));
    decoder_pass(e, np, dptok, dppos, dphyp, e->d_done.as<int>(), nullptr, dlr, nr + nsot, logits, nullptr, 0, nullptr, 1, s,
                 err);
    if (nsot) launch_no_speech(logits + (size_t)nr * V, V, V, nsot, m.no_speech, e->d_res_ns.as<float>(), s, dws);
    debug_nan(e, logits, nr, s);
    {
      ProfScope ps(e, P_SELECT, s);
      launch_logits_select(sp, nr, s);
    }
    // host view of the new row set
    for (int r = 0; r < nr; ++r) row_hyp[r] = new_row_hyp[r];
    for (const auto& sw : starts) { hyp_win[sw.first] = sw.second; live[sw.first] = 1; }
    nrows = nr;
    ++passes;
    row_steps += nr;
  };

  const bool use_graph = e->dec_graph && !e->prof_on && !e->dec_split;
  hipStream_t ds = st;
  if (use_graph) {
    if (!e->gst) {
      HIP_OK(hipStreamCreateWithFlags(&e->gst, hipStreamNonBlocking));
      HIP_OK(hipEventCreateWithFlags(&e->ev_g0, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&e->ev_g1, hipEventDisableTiming));
    }
    HIP_OK(hipEventRecord(e->ev_g0, st));
    HIP_OK(hipStreamWaitEvent(e->gst, e->ev_g0, 0));
    ds = e->gst;
  }
  auto step_eager = [&](hipStream_t s) {
    decoder_pass(e, nrows, e->d_row_tok.as<int>(), e->d_row_pos.as<int>(), e->d_row_hyp.as<int>(), e->d_done.as<int>(),
                 nullptr, nullptr, nrows, logits, nullptr, 0, nullptr, 1, s, err);
    debug_nan(e, logits, nrows, s);
    ProfScope ps(e, P_SELECT, s);
    launch_logits_select(sp, nrows, s);
  };

  StepGraph graph;
  bool graph_rows_changed = true;               // the next decode step runs eagerly (sizes scratch), then captures
  const int check = std::max(1, a->check_every);
  const int refill_min = std::max(1, R / 16);   // a refill pass runs eagerly: batch the starts
  std::vector<int> h_done(R);
  int h_cnt[4] = {0, 0, 0, 0};
  // every window's tokens need at most max_length - P steps; a generous bound against a stuck loop
  const long long pass_limit = (long long)(W / std::max(1, R) + 2) * (ML - P + check + 2) + 16;
  try {
    // first pass: the first R windows start
    carry.assign(R, -1);
    new_row_hyp.resize(R);
    starts.clear();
    for (int r = 0; r < R; ++r) {
      new_row_hyp[r] = r;
      starts.push_back({r, next++});
    }
    event(ds);
    int k = 1;                                  // decode passes since the last host check
    for (;;) {
      if (k >= check) {
        k = 0;
        HIP_OK(hipMemcpyAsync(h_cnt, counters, sizeof(h_cnt), hipMemcpyDeviceToHost, ds));
        HIP_OK(hipMemcpyAsync(h_done.data(), e->d_done.p, (size_t)R * 4, hipMemcpyDeviceToHost, ds));
        HIP_OK(hipStreamSynchronize(ds));
        check_decode_error(h_cnt + 1);
        int n_live = 0, n_free = 0;
        for (int r = 0; r < nrows; ++r) {
          const int h = row_hyp[r];
          if (live[h] && h_done[h]) live[h] = 0;
          n_live += live[h];
        }
        n_free = nrows - n_live;
        if (n_live == 0 && next >= W) break;
        const bool refill = next < W && (n_free >= refill_min || n_live == 0);
        const bool compact = next >= W && a->compact && n_live * 8 <= nrows * row_compact_8ths();
        if (refill || compact) {
          carry.clear(); new_row_hyp.clear(); starts.clear();
          for (int r = 0; r < nrows; ++r) {
            const int h = row_hyp[r];
            if (live[h]) {
              carry.push_back(r); new_row_hyp.push_back(h);
            } else if (refill) {
              if (next < W) {
                carry.push_back(-1); new_row_hyp.push_back(h); starts.push_back({h, next++});
                ++refills;
              } else {
                carry.push_back(-2); new_row_hyp.push_back(h);
              }
            }                                   // compact: ended rows leave the row set
          }
          const int before = nrows;
          event(ds);
          if (nrows != before) {
            graph.drop();
            graph_rows_changed = true;
          }
          k = 1;
          continue;
        }
      }
      if (!graph.valid()) {                     // an event pass grew a buffer the captured graph points into
        graph.drop();
        graph_rows_changed = true;
      }
      if (!use_graph || graph_rows_changed) {
        step_eager(ds);
        graph_rows_changed = false;
      } else {
        if (!graph.exec) ++captures;
        graph.run(ds, [&] { step_eager(ds); });
      }
      ++passes;
      row_steps += nrows;
      ++k;
      if (passes > pass_limit) throw std::runtime_error("generate: decode did not terminate");
    }
  } catch (...) {
    graph.abort(ds);
    throw;
  }
  if (use_graph) {
    HIP_OK(hipEventRecord(e->ev_g1, ds));
    HIP_OK(hipStreamWaitEvent(st, e->ev_g1, 0));
  }
  if (graph.exec) {
    HIP_OK(hipStreamSynchronize(ds));
    graph.drop();
  }

  // ---- results, by window
  std::vector<int> res_tok((size_t)W * C), res_len(W);
  std::vector<float> res_cum(W), res_ns(W), res_lp, res_lpo;
  HIP_OK(hipMemcpyAsync(res_tok.data(), e->d_res_tok.p, res_tok.size() * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(res_len.data(), e->d_res_len.p, (size_t)W * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(res_cum.data(), e->d_res_cum.p, (size_t)W * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(res_ns.data(), e->d_res_ns.p, (size_t)W * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(h_cnt, counters, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
  if (rec) {
    res_lp.resize((size_t)W * C);
    res_lpo.resize((size_t)W * C);
    HIP_OK(hipMemcpyAsync(res_lp.data(), e->d_res_lp.p, res_lp.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(res_lpo.data(), e->d_res_lp_o.p, res_lpo.size() * 4, hipMemcpyDeviceToHost, st));
  }
  HIP_OK(hipStreamSynchronize(st));
  check_decode_error(h_cnt + 1);
  const float lp = a->length_penalty;
  for (int w = 0; w < W; ++w) {
    const int n = res_len[w];
    if (n < 0 || n > ML) throw std::runtime_error("generate: window " + std::to_string(w) + " has no result");
    for (int i = 0; i < n; ++i) a->h_tokens[(size_t)w * ML + i] = res_tok[(size_t)w * C + i];
    a->h_lengths[w] = n;
    a->h_scores[w] = res_cum[w] / std::pow((float)std::max(n, 1), lp);
    if (a->h_cum_logprob) a->h_cum_logprob[w] = res_cum[w];
    if (a->h_no_speech) a->h_no_speech[w] = res_ns[w];
    if (rec) {
      const int nr = std::min(ML, n + (P + n < ML ? 1 : 0));
      for (int i = 0; i < nr; ++i) {
        a->h_token_logprobs[(size_t)w * ML + i] = res_lp[(size_t)w * C + i];
        if (a->h_token_logprobs_other) a->h_token_logprobs_other[(size_t)w * ML + i] = res_lpo[(size_t)w * C + i];
      }
    }
  }
  if (a->h_steps) a->h_steps[0] = (int)passes;
  if (a->h_stats) {
    a->h_stats[0] = passes;
    a->h_stats[1] = row_steps;
    a->h_stats[2] = refills;
    a->h_stats[3] = captures;
  }
}

// logit_rows (optional): the pass rows whose logits are wanted, in output order (overrides last_only)
void forward(wm_engine* e, int n_seq, const int* h_slots, int S, const int* h_tokens, float* d_logits, int last_only,
             const int* h_align, int n_align, float* d_attn, hipStream_t st, const std::vector<int>* logit_rows = nullptr) {
  check_weights(e);
  const auto& m = e->dm;
  const int C = m.n_text_ctx, H = m.n_head;
  if (S <= 0 || S > C) throw std::runtime_error("forward: bad seq_len");
  reserve(e, e->n_slots, n_seq);
  const int rows = n_seq * S;
  const int nlog = logit_rows ? (int)logit_rows->size() : last_only ? n_seq : rows;
  ensure_step(e, rows, 1);
  std::vector<int> rt(rows), rp(rows), rh(rows), lr(nlog), hs(n_seq), lin((size_t)n_seq * C);
  for (int s = 0; s < n_seq; ++s) {
    if (h_slots[s] < 0 || h_slots[s] >= e->n_slots) throw std::runtime_error("forward: slot out of range");
    hs[s] = h_slots[s];
    for (int p = 0; p < S; ++p) {
      const int r = s * S + p;
      rt[r] = h_tokens[r]; rp[r] = p; rh[r] = s;
    }
    for (int p = 0; p < C; ++p) lin[(size_t)s * C + p] = s;
  }
  for (int i = 0; i < nlog; ++i) lr[i] = logit_rows ? (*logit_rows)[i] : last_only ? i * S + S - 1 : i;
  std::vector<std::vector<int>> amap(m.n_dec_layer, std::vector<int>(H, -1));
  for (int i = 0; i < n_align; ++i) {
    const int l = h_align[2 * i], h = h_align[2 * i + 1];
    if (l < 0 || l >= m.n_dec_layer || h < 0 || h >= H) throw std::runtime_error("forward: bad alignment head");
    amap[l][h] = i;
  }
  e->d_logit_rows.ensure((size_t)nlog * 4);
  HIP_OK(hipMemcpyAsync(e->d_prow_tok.p, rt.data(), rows * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_prow_pos.p, rp.data(), rows * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_prow_hyp.p, rh.data(), rows * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_logit_rows.p, lr.data(), nlog * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_hyp_slot.p, hs.data(), n_seq * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_lin.p, lin.data(), lin.size() * 4, hipMemcpyHostToDevice, st));
  // factored form with capture (alignment): gather the windows' encoder outputs for the per-layer K/V projection
  // (decoder_layer); the rows of a window must reach the teacher-forced kernel (S >= 16, launch_cross_attn)
  e->tf_nwin = 0;
  if (n_align && e->cross_mode == 1 && e->cross_tf && !e->cross_fp8 && S >= 16) {
    const int T = m.n_audio_ctx, d = m.n_state;
    const size_t per = (size_t)T * d;
    e->a_enc.ensure((size_t)n_seq * per * 2);
    e->a_kv.ensure((size_t)2 * n_seq * per * 2);
    const size_t bper = (size_t)xblock_slot_elems(T, d);
    for (int s = 0; s < n_seq; ++s)
      launch_xblock(e->xenc.as<bf16>() + (size_t)hs[s] * bper, 1, T, d, e->a_enc.as<bf16>() + (size_t)s * per, false, st);
    e->tf_nwin = n_seq;
  }
  struct TfReset { wm_engine* e; ~TfReset() { e->tf_nwin = 0; } } tf_reset{e};
  decoder_pass(e, rows, e->d_prow_tok.as<int>(), e->d_prow_pos.as<int>(), e->d_prow_hyp.as<int>(), nullptr,
               e->d_lin.as<int>(), e->d_logit_rows.as<int>(), nlog, d_logits, n_align ? &amap : nullptr, n_align,
               n_align ? d_attn : nullptr, S, st);
  HIP_OK(hipStreamSynchronize(st));
}

void dtw_run(wm_engine* e, const float* d_x, int N, int M, int* h_i, int* h_j, int* h_len, hipStream_t st) {
  e->a_cost.ensure((size_t)(N + 1) * (M + 1) * 4);
  e->a_trace.ensure((size_t)(N + 1) * (M + 1));
  e->a_pi.ensure((size_t)(N + M + 2) * 4);
  e->a_pj.ensure((size_t)(N + M + 2) * 4);
  e->a_plen.ensure(4);
  launch_dtw(d_x, N, M, e->a_cost.as<float>(), e->a_trace.as<signed char>(), e->a_pi.as<int>(), e->a_pj.as<int>(),
             e->a_plen.as<int>(), st);
  int n = 0;
  HIP_OK(hipMemcpyAsync(&n, e->a_plen.p, 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipMemcpyAsync(h_i, e->a_pi.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(h_j, e->a_pj.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  *h_len = n;
}

// Beam row-set decode: beam search over W windows with at most G = max_rows / K windows (groups of K hypothesis
// slots) in flight.  A group decodes one window; when beam_select ends it (max_cand finished, max_length, or no live
// beam), the host check reads the group's finished list and beams, finalises the window (openai's ranking, as
// generate()) and starts the next window in the group: the event pass prefills the new window's prompt into the
// group's first slot (P rows) beside the other groups' decode rows, and beam_start_kernel resets the group's state.
// The K rows of a group stay together (its window's cross panels are read once for them), the row set keeps its
// groups in place while windows wait (the step graph stays valid), and once nothing waits the finished groups'
// rows are dropped at 7/8 (beam passes are GEMM-row-bound).  No per-step records in this form.
void generate_rows_beam(wm_engine* e, const wm_generate_args* a, hipStream_t st) {
  const auto& m = e->dm;
  const int C = m.n_text_ctx, V = m.n_vocab;
  const int W = a->n_windows, P = a->prompt_len, K = a->beam_size;
  const int G = std::max(1, std::min(a->max_rows / K, W));
  const int NH = G * K;
  const int ML = a->max_length;
  const int max_cand = std::max(1, (int)std::lround(a->beam_size * a->patience));
  if (max_cand > 16) throw std::runtime_error("generate: beam_size * patience must be <= 16");
  if (a->h_token_logprobs) throw std::runtime_error("generate: per-step records need max_rows 0 with beam search");
  reserve(e, e->n_slots, NH);
  e->d_win_prompt.ensure((size_t)W * P * 4);
  e->d_win_slot.ensure((size_t)W * 4);
  e->d_res_ns.ensure((size_t)W * 4);
  HIP_OK(hipMemcpyAsync(e->d_win_prompt.p, a->h_prompts, (size_t)W * P * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(e->d_win_slot.p, a->h_slots, (size_t)W * 4, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemsetAsync(e->d_res_ns.p, 0, (size_t)W * 4, st));
  HIP_OK(hipMemsetAsync(e->d_n_active.p, 0, 4 * 4, st));
  {
    std::vector<int> ones(NH, 1);              // every group starts ended (no window)
    HIP_OK(hipMemcpyAsync(e->d_done.p, ones.data(), (size_t)NH * 4, hipMemcpyHostToDevice, st));
    upload_suppress(e, a, st);                 // (synchronises: `ones` goes out of scope)
  }
  // pass rows: every hypothesis row + P prompt rows per starting group; logits rows: one per hypothesis row + one
  // sot row per start
  ensure_step(e, NH + G * std::max(P, K), NH + G);
  float* logits = e->s_logits.as<float>();
  int* counters = e->d_n_active.as<int>();
  int* err = counters + 1;
  SearchParams sp = search_params(e, a, logits, P);
  sp.mode = 1; sp.topk = K + 1;
  sp.row_hyp = e->d_row_hyp.as<int>();
  BeamParams bp;
  std::memset(&bp, 0, sizeof(bp));
  bp.beam = K; bp.max_cand = max_cand; bp.n_ctx = C; bp.sample_begin = P; bp.max_length = ML;
  bp.eot = m.eot; bp.cand_tok = sp.cand_tok; bp.cand_lp = sp.cand_lp; bp.tokens = sp.tokens; bp.lin = e->d_lin.as<int>();
  bp.seq_len = sp.seq_len; bp.cum = sp.cum; bp.done = sp.done; bp.row_tok = sp.row_tok; bp.row_pos = sp.row_pos;
  bp.fin_tok = e->d_fin_tok.as<int>(); bp.fin_len = e->d_fin_len.as<int>(); bp.fin_cum = e->d_fin_cum.as<float>();
  bp.n_fin = e->d_n_fin.as<int>(); bp.n_active = sp.n_active;

  // host view: the row set is a list of groups (K rows each, in order); group g decodes window gwin[g] while glive[g]
  std::vector<int> set(G), gwin(G, -1);
  std::vector<char> glive(G, 0), wdone(W, 0);
  for (int g = 0; g < G; ++g) set[g] = g;
  int next = 0, nfinal = 0;
  long long passes = 0, row_steps = 0, refills = 0;
  int captures = 0;
  const float lp = a->length_penalty;
  auto norm = [&](float c, int n) { return c / std::pow((float)std::max(n, 1), lp); };
  // the finished groups' lists and beams -> their windows' results (openai finalize, as generate())
  std::vector<int> f_tok, f_len, f_n, o_tok, o_len;
  std::vector<float> f_cum, o_cum;
  auto finalize = [&](const std::vector<int>& gs, hipStream_t s) {
    if (gs.empty()) return;
    f_tok.resize((size_t)G * max_cand * C); f_len.resize((size_t)G * max_cand); f_cum.resize((size_t)G * max_cand);
    f_n.resize(G); o_tok.resize((size_t)NH * C); o_len.resize(NH); o_cum.resize(NH);
    HIP_OK(hipMemcpyAsync(f_tok.data(), e->d_fin_tok.p, f_tok.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(f_len.data(), e->d_fin_len.p, f_len.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(f_cum.data(), e->d_fin_cum.p, f_cum.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(f_n.data(), e->d_n_fin.p, (size_t)G * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(o_tok.data(), e->d_tokens.p, o_tok.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(o_len.data(), e->d_seq_len.p, (size_t)NH * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(o_cum.data(), e->d_cum.p, (size_t)NH * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    for (int g : gs) {
      const int w = gwin[g];
      struct C2 { const int* t; int n; float c; };
      std::vector<C2> cands;
      for (int i = 0; i < std::min(f_n[g], max_cand); ++i) {
        const size_t f = (size_t)g * max_cand + i;
        cands.push_back({&f_tok[f * C], f_len[f], f_cum[f]});
      }
      if ((int)cands.size() < K) {
        std::vector<int> order;
        for (int b = 0; b < K; ++b)
          if (o_cum[g * K + b] > -INFINITY) order.push_back(b);
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return o_cum[g * K + x] > o_cum[g * K + y]; });
        for (int b : order) {
          if ((int)cands.size() >= K) break;
          const int h = g * K + b;
          cands.push_back({&o_tok[(size_t)h * C + P], o_len[h] - P, o_cum[h]});
        }
      }
      int best_len = 0;
      float best_cum = 0.f, best_score = -INFINITY;
      const int* best_ptr = nullptr;
      for (const auto& c : cands) {
        const float sc = norm(c.c, c.n);
        if (sc > best_score) { best_score = sc; best_len = c.n; best_cum = c.c; best_ptr = c.t; }
      }
      if (best_len < 0 || best_len > ML) throw std::runtime_error("generate: window " + std::to_string(w) + " has no result");
      for (int i = 0; i < best_len; ++i) a->h_tokens[(size_t)w * ML + i] = best_ptr[i];
      a->h_lengths[w] = best_len;
      a->h_scores[w] = best_score;
      if (a->h_cum_logprob) a->h_cum_logprob[w] = best_cum;
      wdone[w] = 1;
      ++nfinal;
      glive[g] = 0;
      gwin[g] = -1;
    }
  };

  // One event pass: `starts` (group, window) begin in place; `nset` is the new row set (compaction drops groups).
  std::vector<int> nset;
  std::vector<std::pair<int, int>> starts;
  int nrows = NH;
  // A starting group's P prompt rows are padded to K with copies of its last prompt row (same hypothesis, position
  // and token: identical self-KV writes), so every group of the pass holds K rows of one window and the
  // cross-attention keeps its per-window grouping (prompts longer than K rows: ungrouped rows).
  const int PR = std::max(P, K);
  const int ev_group = P <= K ? K : 1;
  auto event = [&](hipStream_t s) {
    const int ng = (int)nset.size(), nr = ng * K, nst = (int)starts.size();
    const int nsot = a->sot_index >= 0 ? nst : 0;
    std::vector<int> start_of(G, -1);
    for (int k = 0; k < nst; ++k) start_of[starts[k].first] = k;
    int np = 0, n_live = 0;
    for (int g : nset) {
      np += start_of[g] >= 0 ? (ev_group > 1 ? PR : P) : K;
      n_live += (start_of[g] >= 0 || glive[g]) ? K : 0;
    }
    std::vector<int>& u = e->h_ev;
    u.assign((size_t)4 * np + 2 * nr + nsot + 2 * nst + 1, 0);
    int* ptok = u.data(); int* ppos = ptok + np; int* phyp = ppos + np; int* psrc = phyp + np;
    int* rh = psrc + np; int* lr = rh + nr; int* gsd = lr + nr + nsot; int* wsd = gsd + nst;
    wsd[nst] = n_live;
    int i = 0, r = 0;
    for (int g : nset) {
      const int h0 = g * K, k = start_of[g];
      if (k >= 0) {
        const int w = starts[k].second;
        int last = 0;
        for (int p = 0; p < P; ++p, ++i) {
          ptok[i] = a->h_prompts[(size_t)w * P + p]; ppos[i] = p; phyp[i] = h0; psrc[i] = -1;
          if (p == a->sot_index) lr[nr + k] = i;
          last = i;
        }
        for (int p = P; ev_group > 1 && p < PR; ++p, ++i) {
          ptok[i] = a->h_prompts[(size_t)w * P + P - 1]; ppos[i] = P - 1; phyp[i] = h0; psrc[i] = -1;
        }
        for (int b = 0; b < K; ++b, ++r) { rh[r] = h0 + b; lr[r] = last; }
        gsd[k] = g; wsd[k] = w;
      } else {
        for (int b = 0; b < K; ++b, ++i, ++r) {
          phyp[i] = h0 + b; psrc[i] = h0 + b;
          rh[r] = h0 + b; lr[r] = i;
        }
      }
    }
    e->d_ev.ensure(u.size() * 4);
    int* du = e->d_ev.as<int>();
    HIP_OK(hipMemcpyAsync(du, u.data(), u.size() * 4, hipMemcpyHostToDevice, s));
    int* dptok = du; int* dppos = du + np; int* dphyp = du + 2 * np; int* dpsrc = du + 3 * np;
    int* drh = du + 4 * np; int* dlr = drh + nr; int* dgs = dlr + nr + nsot; int* dws = dgs + nst;
    // carried rows: token / position of their hypothesis from the last beam selection (hypothesis-indexed)
    launch_rows_fill(np, dpsrc, dptok, dppos, e->d_row_tok.as<int>(), e->d_row_pos.as<int>(), s);
    launch_beam_start(nst, dgs, dws, K, e->d_win_prompt.as<int>(), P, e->d_win_slot.as<int>(), C, e->d_tokens.as<int>(),
                      e->d_lin.as<int>(), e->d_seq_len.as<int>(), e->d_done.as<int>(), e->d_cum.as<float>(),
                      e->d_hyp_slot.as<int>(), e->d_n_fin.as<int>(), s);
    HIP_OK(hipMemcpyAsync(e->d_row_hyp.p, drh, (size_t)nr * 4, hipMemcpyDeviceToDevice, s));
    HIP_OK(hipMemcpyAsync(counters, dws + nst, 4, hipMemcpyDeviceToDevice, s));
    decoder_pass(e, np, dptok, dppos, dphyp, e->d_done.as<int>(), e->d_lin.as<int>(), dlr, nr + nsot, logits, nullptr, 0,
                 nullptr, ev_group, s, err);
    if (nsot) launch_no_speech(logits + (size_t)nr * V, V, V, nsot, m.no_speech, e->d_res_ns.as<float>(), s, dws);
    debug_nan(e, logits, nr, s);
    {
      ProfScope ps(e, P_SELECT, s);
      launch_logits_select(sp, nr, s);
      launch_beam_select(bp, G, s);
    }
    for (const auto& gw : starts) { gwin[gw.first] = gw.second; glive[gw.first] = 1; }
    set = nset;
    nrows = nr;
    ++passes;
    row_steps += nr;
  };

  const bool use_graph = e->dec_graph && !e->prof_on && !e->dec_split;
  hipStream_t ds = st;
  if (use_graph) {
    if (!e->gst) {
      HIP_OK(hipStreamCreateWithFlags(&e->gst, hipStreamNonBlocking));
      HIP_OK(hipEventCreateWithFlags(&e->ev_g0, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&e->ev_g1, hipEventDisableTiming));
    }
    HIP_OK(hipEventRecord(e->ev_g0, st));
    HIP_OK(hipStreamWaitEvent(e->gst, e->ev_g0, 0));
    ds = e->gst;
  }
  auto step_eager = [&](hipStream_t s) {
    launch_rows_fill(nrows, e->d_row_hyp.as<int>(), e->d_prow_tok.as<int>(), e->d_prow_pos.as<int>(),
                     e->d_row_tok.as<int>(), e->d_row_pos.as<int>(), s);
    decoder_pass(e, nrows, e->d_prow_tok.as<int>(), e->d_prow_pos.as<int>(), e->d_row_hyp.as<int>(), e->d_done.as<int>(),
                 e->d_lin.as<int>(), nullptr, nrows, logits, nullptr, 0, nullptr, K, s, err);
    debug_nan(e, logits, nrows, s);
    ProfScope ps(e, P_SELECT, s);
    launch_logits_select(sp, nrows, s);
    launch_beam_select(bp, G, s);
  };

  StepGraph graph;
  bool graph_rows_changed = true;
  const int check = std::max(1, a->check_every);
  const int refill_min = std::max(1, G / 16);
  std::vector<int> h_done(NH);
  int h_cnt[4] = {0, 0, 0, 0};
  const long long pass_limit = (long long)(W / G + 2) * (ML - P + check + 2) + 16;
  try {
    nset = set;
    starts.clear();
    for (int g = 0; g < G; ++g) starts.push_back({g, next++});
    event(ds);
    int k = 1;
    for (;;) {
      if (k >= check) {
        k = 0;
        HIP_OK(hipMemcpyAsync(h_cnt, counters, sizeof(h_cnt), hipMemcpyDeviceToHost, ds));
        HIP_OK(hipMemcpyAsync(h_done.data(), e->d_done.p, (size_t)NH * 4, hipMemcpyDeviceToHost, ds));
        HIP_OK(hipStreamSynchronize(ds));
        check_decode_error(h_cnt + 1);
        std::vector<int> ended;
        for (int g = 0; g < G; ++g)
          if (glive[g] && h_done[g * K]) ended.push_back(g);
        finalize(ended, ds);
        int n_live = 0, n_free = 0;
        for (int g : set) { n_live += glive[g]; n_free += !glive[g]; }
        if (n_live == 0 && next >= W) break;
        const bool refill = next < W && (n_free >= refill_min || n_live == 0);
        const bool compact = a->compact && next >= W && n_live * 8 <= (int)set.size() * 7;   // opt-in, as the header says
        if (refill || compact) {
          nset.clear(); starts.clear();
          for (int g : set) {
            if (glive[g]) nset.push_back(g);
            else if (refill && next < W) { nset.push_back(g); starts.push_back({g, next++}); ++refills; }
            else if (refill) nset.push_back(g);       // idle until compaction (rows stay in place)
          }
          const int before = nrows;
          event(ds);
          if (nrows != before) {
            graph.drop();
            graph_rows_changed = true;
          }
          k = 1;
          continue;
        }
      }
      if (!graph.valid()) {
        graph.drop();
        graph_rows_changed = true;
      }
      if (!use_graph || graph_rows_changed) {
        step_eager(ds);
        graph_rows_changed = false;
      } else {
        if (!graph.exec) ++captures;
        graph.run(ds, [&] { step_eager(ds); });
      }
      ++passes;
      row_steps += nrows;
      ++k;
      if (passes > pass_limit) throw std::runtime_error("generate: decode did not terminate");
    }
  } catch (...) {
    graph.abort(ds);
    throw;
  }
  if (use_graph) {
    HIP_OK(hipEventRecord(e->ev_g1, ds));
    HIP_OK(hipStreamWaitEvent(st, e->ev_g1, 0));
  }
  if (graph.exec) {
    HIP_OK(hipStreamSynchronize(ds));
    graph.drop();
  }
  std::vector<float> res_ns(W);
  HIP_OK(hipMemcpyAsync(res_ns.data(), e->d_res_ns.p, (size_t)W * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(h_cnt, counters, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  check_decode_error(h_cnt + 1);
  if (nfinal != W) throw std::runtime_error("generate: beam row-set finished " + std::to_string(nfinal) + " of " +
                                            std::to_string(W) + " windows");
  for (int w = 0; w < W; ++w)
    if (a->h_no_speech) a->h_no_speech[w] = res_ns[w];
  if (a->h_steps) a->h_steps[0] = (int)passes;
  if (a->h_stats) {
    a->h_stats[0] = passes;
    a->h_stats[1] = row_steps;
    a->h_stats[2] = refills;
    a->h_stats[3] = captures;
  }
}

void align(wm_engine* e, int slot, int sot_len, const int* h_sot, int n_text, const int* h_text, int num_frames,
           const int* h_heads, int n_heads, int medw, float* h_probs, int* h_ti, int* h_tj, int* h_len, hipStream_t st) {
  const auto& m = e->dm;
  const int T = m.n_audio_ctx, V = m.n_vocab;
  const int S = sot_len + 1 + n_text + 1;
  if (n_text <= 0 || S > m.n_text_ctx) throw std::runtime_error("wm_align: bad token count");
  const int F = num_frames / 2;
  if (F <= 0 || F > T) throw std::runtime_error("wm_align: bad num_frames");
  std::vector<int> toks(S), next(n_text);
  for (int i = 0; i < sot_len; ++i) toks[i] = h_sot[i];
  toks[sot_len] = m.no_timestamps;
  for (int i = 0; i < n_text; ++i) toks[sot_len + 1 + i] = next[i] = h_text[i];
  toks[S - 1] = m.eot;
  e->a_logits.ensure((size_t)S * V * 4);
  e->a_attn.ensure((size_t)S * n_heads * T * 4);
  forward(e, 1, &slot, S, toks.data(), e->a_logits.as<float>(), 0, h_heads, n_heads, e->a_attn.as<float>(), st);
  // text token probabilities: position sot_len + k predicts text token k
  e->a_next.ensure((size_t)n_text * 4);
  e->a_probs.ensure((size_t)n_text * 4);
  HIP_OK(hipMemcpyAsync(e->a_next.p, next.data(), n_text * 4, hipMemcpyHostToDevice, st));
  launch_token_probs(e->a_logits.as<float>() + (size_t)sot_len * V, n_text, V, m.eot, e->a_next.as<int>(),
                     e->a_probs.as<float>(), st);
  // DTW input matrix rows sot_len .. S-2 (n_text + 1 rows)
  const int nrows = n_text + 1;
  e->a_rowsum.ensure((size_t)S * n_heads * 4);
  e->a_z.ensure((size_t)n_heads * S * F * 4);
  e->a_mat.ensure((size_t)nrows * F * 4);
  launch_align_matrix(e->a_attn.as<float>(), S, n_heads, T, F, medw, sot_len, nrows, e->a_rowsum.as<float>(),
                      e->a_z.as<float>(), e->a_mat.as<float>(), st);
  HIP_OK(hipMemcpyAsync(h_probs, e->a_probs.p, n_text * 4, hipMemcpyDeviceToHost, st));
  dtw_run(e, e->a_mat.as<float>(), nrows, F, h_ti, h_tj, h_len, st);
}

// Batched word alignment (ctranslate2 Whisper.align over a batch of windows [FW↑]): items are chunked so the
// captured attention (S x heads x 1500 f32 per item) and the text-row logits stay under ~1.5 GB; per chunk ONE
// teacher-forced decoder pass over every item (sequences padded with <|endoftext|> to the chunk's longest: the
// pass is causal, so padding never changes a real position), then per item the probabilities and the
// alignment matrix, and one batched DTW launch for the whole chunk.
void align_batch(wm_engine* e, int n, const int* h_slots, int sot_len, const int* h_sot, const int* h_text_off,
                 const int* h_text, const int* h_num_frames, const int* h_heads, int n_heads, int medw, float* h_probs,
                 const long long* h_path_off, int* h_pi, int* h_pj, int* h_plen, hipStream_t st) {
  const auto& m = e->dm;
  const int T = m.n_audio_ctx, V = m.n_vocab;
  if (n <= 0) return;
  if (n_heads <= 0) throw std::runtime_error("wm_align_batch: no alignment heads");
  std::vector<int> S(n), nt(n), F(n);
  for (int i = 0; i < n; ++i) {
    nt[i] = h_text_off[i + 1] - h_text_off[i];
    S[i] = sot_len + 1 + nt[i] + 1;
    F[i] = h_num_frames[i] / 2;
    if (nt[i] <= 0 || S[i] > m.n_text_ctx) throw std::runtime_error("wm_align_batch: bad token count");
    if (F[i] <= 0 || F[i] > T) throw std::runtime_error("wm_align_batch: bad num_frames");
  }
  // The capture buffer (S x heads x 1500 f32 per item: ~230 MB for a large-v3 window with the default 320 heads)
  // may take half of the free device memory (at most 48 GB): a batch of 150 large-v3 windows then aligns in ONE
  // teacher-forced pass instead of ~25 passes of 6 windows under a fixed 1.5 GB budget (round 3: 0.89 s per
  // 150-window step, most of it those passes).
  size_t free_b = 0, total_b = 0;
  HIP_OK(hipMemGetInfo(&free_b, &total_b));
  // the factored form's alignment pass also gathers each item's encoder output and its per-layer K/V projection
  // (a_enc + a_kv, 3 x T x d bf16 per item, forward()): counted per item below
  const bool tf_gather = e->cross_mode == 1 && e->cross_tf && !e->cross_fp8;
  const double per_item_kv = tf_gather ? 3.0 * (double)T * m.n_state * 2 : 0.0;
  const double reusable = (double)e->a_attn.bytes + (double)e->a_logits.bytes +
                          (tf_gather ? (double)e->a_enc.bytes + (double)e->a_kv.bytes : 0.0);
  const double budget = std::max(1.5e9, std::min(48e9, 0.5 * (double)free_b + reusable));
  static const bool align_log = [] {
    const char* v = std::getenv("VLOG_AMD_ALIGN_LOG");
    return v && v[0] == '1';
  }();
  if (align_log) std::fprintf(stderr, "[align_batch] %d items, free %.1f GB, budget %.1f GB\n", n, free_b / 1e9, budget / 1e9);
  // Items longest-first, chunked so padding (every sequence of a chunk padded to its longest) stays under a
  // quarter of the chunk's rows: with transcripts of 5 to 220 tokens one padded pass would run ~2x the rows.
  std::vector<int> ord(n);
  for (int i = 0; i < n; ++i) ord[i] = i;
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return S[x] > S[y]; });
  int i0 = 0;
  while (i0 < n) {
    int i1 = i0, smax = 0;
    long long ntext = 0, sum_s = 0;
    while (i1 < n) {
      const int it = ord[i1];
      const int s2 = std::max(smax, S[it]);
      // per item: its attention capture, the factored form's K/V gather, and the fused alignment's f64 statistics
      // (n_heads x F x 2 doubles, F <= T: the buffer is c x n_heads x fmax x 16 bytes)
      const double bytes = (double)(i1 - i0 + 1) * (s2 * n_heads * T * 4 + per_item_kv + (double)n_heads * T * 16) +
                           (double)(ntext + nt[it]) * V * 4;
      if (i1 > i0 && (bytes > budget || (double)(i1 - i0 + 1) * s2 > 1.25 * (double)(sum_s + S[it]))) break;
      smax = s2;
      ntext += nt[it];
      sum_s += S[it];
      ++i1;
    }
    const int c = i1 - i0;
    std::vector<int> toks((size_t)c * smax, m.eot), slots(c), lrows, next;
    for (int k = 0; k < c; ++k) {
      const int i = ord[i0 + k];
      int* t = &toks[(size_t)k * smax];
      for (int j = 0; j < sot_len; ++j) t[j] = h_sot[j];
      t[sot_len] = m.no_timestamps;
      for (int j = 0; j < nt[i]; ++j) {
        t[sot_len + 1 + j] = h_text[h_text_off[i] + j];
        lrows.push_back(k * smax + sot_len + j);         // position sot_len + j predicts text token j
        next.push_back(h_text[h_text_off[i] + j]);
      }
      slots[k] = h_slots[i];
    }
    e->a_logits.ensure((size_t)ntext * V * 4);
    e->a_attn.ensure((size_t)c * smax * n_heads * T * 4);
    forward(e, c, slots.data(), smax, toks.data(), e->a_logits.as<float>(), 0, h_heads, n_heads, e->a_attn.as<float>(), st,
            &lrows);
    e->a_next.ensure((size_t)ntext * 4);
    e->a_probs.ensure((size_t)ntext * 4);
    HIP_OK(hipMemcpyAsync(e->a_next.p, next.data(), ntext * 4, hipMemcpyHostToDevice, st));
    launch_token_probs(e->a_logits.as<float>(), (int)ntext, V, m.eot, e->a_next.as<int>(), e->a_probs.as<float>(), st);
    // alignment matrices of the chunk, packed; DTW scratch and path offsets
    std::vector<long long> xo(c), co(c), po(c);
    std::vector<int> Ns(c), Ms(c);
    long long xt = 0, ct = 0, pt = 0;
    for (int k = 0; k < c; ++k) {
      const int i = ord[i0 + k];
      Ns[k] = nt[i] + 1; Ms[k] = F[i];
      xo[k] = xt; co[k] = ct; po[k] = pt;
      xt += (long long)Ns[k] * Ms[k];
      ct += (long long)(Ns[k] + 1) * (Ms[k] + 1);
      pt += Ns[k] + Ms[k];
    }
    e->a_mat.ensure((size_t)xt * 4);
    e->a_meta.ensure((size_t)c * (3 * 8 + 3 * 4));
    char* meta = (char*)e->a_meta.p;
    long long* d_xo = (long long*)meta;
    long long* d_co = d_xo + c;
    long long* d_po = d_co + c;
    int* d_N = (int*)(d_po + c);
    int* d_M = d_N + c;
    int* d_S = d_M + c;
    std::vector<int> Ss(c);
    int fmax = 0, nmax = 0;
    for (int k = 0; k < c; ++k) {
      Ss[k] = S[ord[i0 + k]];
      fmax = std::max(fmax, Ms[k]);
      nmax = std::max(nmax, Ns[k]);
    }
    HIP_OK(hipMemcpyAsync(d_xo, xo.data(), c * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_co, co.data(), c * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_po, po.data(), c * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_N, Ns.data(), c * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_M, Ms.data(), c * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_S, Ss.data(), c * 4, hipMemcpyHostToDevice, st));
    if (align_get_fused()) {
      // the whole chunk in three launches (rows of window k: its text + <|endoftext|>, from row sot_len)
      e->a_rowsum.ensure((size_t)c * smax * n_heads * 4);
      e->a_z.ensure((size_t)c * n_heads * fmax * 16);
      launch_align_matrix_batch(e->a_attn.as<float>(), c, smax, n_heads, T, fmax, nmax, medw, sot_len, d_S, d_M, d_N, d_xo,
                                e->a_rowsum.as<float>(), (double*)e->a_z.p, e->a_mat.as<float>(), st);
    } else {
      e->a_rowsum.ensure((size_t)smax * n_heads * 4);
      e->a_z.ensure((size_t)n_heads * smax * T * 4);
      for (int k = 0; k < c; ++k) {
        const int i = ord[i0 + k];
        launch_align_matrix(e->a_attn.as<float>() + (size_t)k * smax * n_heads * T, S[i], n_heads, T, F[i], medw, sot_len,
                            nt[i] + 1, e->a_rowsum.as<float>(), e->a_z.as<float>(), e->a_mat.as<float>() + xo[k], st);
      }
    }
    e->a_cost.ensure((size_t)ct * 4);
    e->a_trace.ensure((size_t)ct);
    e->a_pi.ensure((size_t)pt * 4);
    e->a_pj.ensure((size_t)pt * 4);
    e->a_plen.ensure((size_t)c * 4);
    launch_dtw_batch(e->a_mat.as<float>(), d_xo, d_N, d_M, e->a_cost.as<float>(), e->a_trace.as<signed char>(), d_co,
                     e->a_pi.as<int>(), e->a_pj.as<int>(), d_po, e->a_plen.as<int>(), c, st);
    std::vector<int> pi(pt), pj(pt), plen(c);
    std::vector<float> probs(ntext);                // in chunk order: item k's text tokens after item k-1's
    HIP_OK(hipMemcpyAsync(probs.data(), e->a_probs.p, ntext * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(pi.data(), e->a_pi.p, pt * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(pj.data(), e->a_pj.p, pt * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(plen.data(), e->a_plen.p, c * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (int k = 0, pos = 0; k < c; ++k) {
      const int i = ord[i0 + k];
      for (int j = 0; j < nt[i]; ++j) h_probs[h_text_off[i] + j] = probs[pos + j];
      pos += nt[i];
      h_plen[i] = plen[k];
      for (int q = 0; q < plen[k]; ++q) {
        h_pi[h_path_off[i] + q] = pi[po[k] + q];
        h_pj[h_path_off[i] + q] = pj[po[k] + q];
      }
    }
    i0 = i1;
  }
}

template <class F>
int guarded(wm_engine* e, F&& f) {
  try {
    if (!e) throw std::runtime_error("null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    struct GenScope {                     // restored on every exit, exceptions included
      long long* prev;
      explicit GenScope(long long* g) : prev(t_realloc) { t_realloc = g; }
      ~GenScope() { t_realloc = prev; }
    } gs(&e->realloc_gen);
    HIP_OK(hipSetDevice(e->device));
    f();
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// The model entry points need every weight slot set (an engine made for the front end alone has none)
void require_weights(wm_engine* e) {
  if (e->weights_ok) return;
  for (auto& kv : e->slots)
    if (!kv.second.set) throw std::runtime_error("engine weights incomplete (front-end-only engine?): " + kv.first);
  e->weights_ok = true;
}

}  // namespace

extern "C" {

const char* wm_last_error(void) { return g_err.c_str(); }
int32_t wm_abi_version(void) { return 2; }

int wm_create(const wm_model_dims* dims, int32_t device, wm_engine** out) {
  try {
    if (!dims || !out) throw std::runtime_error("wm_create: null argument");
    *out = nullptr;
    if (dims->n_head <= 0 || dims->n_state <= 0 || dims->n_mels <= 0 || dims->n_enc_layer <= 0 ||
        dims->n_dec_layer <= 0 || dims->n_vocab <= 0 || dims->n_text_ctx <= 0 || dims->n_text_ctx > 448)
      throw std::runtime_error("wm_create: dimensions must be positive (n_text_ctx <= 448)");
    for (int32_t t : {dims->eot, dims->sot, dims->no_speech, dims->no_timestamps, dims->timestamp_begin, dims->blank})
      if (t < 0 || t >= dims->n_vocab) throw std::runtime_error("wm_create: special token id out of the vocabulary");
    if (dims->n_state % 64 != 0 || dims->n_state / dims->n_head != 64)
      throw std::runtime_error("wm_create: head_dim must be 64 and n_state a multiple of 64");
    if (dims->n_audio_ctx != 1500) throw std::runtime_error("wm_create: n_audio_ctx must be 1500");
    HIP_OK(hipSetDevice(device));
    auto* e = new wm_engine();
    e->dm = *dims;
    e->device = device;
    if (const char* v = std::getenv("VLOG_AMD_DEC_SPLIT")) e->dec_split = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_GRAPH")) e->dec_graph = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_GEMV")) e->dec_gemv = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_GEMV_LN")) e->dec_gemv_ln = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_RING")) e->dec_ring = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_LN_FOLD")) e->dec_ln_fold = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_PLAN")) {
      const int p = std::atoi(v) != 0;
      for (int i = 0; i < DEC_NPROJ; ++i) e->dec_plan[i] = kDecPlanPresets[p][i], e->dec_cols[i] = kDecColsPresets[p][i];
    }
    // per projection, e.g. VLOG_AMD_DEC_GEMM="qkv=32,fc2=64" (rows per block), VLOG_AMD_DEC_COLS="fc1=64"
    auto per_proj = [](const char* v, int* dst) {
      std::string spec(v);
      size_t pos = 0;
      while (pos < spec.size()) {
        const size_t end = std::min(spec.find(',', pos), spec.size());
        const std::string item = spec.substr(pos, end - pos);
        const size_t eq = item.find('=');
        if (eq != std::string::npos)
          for (int i = 0; i < DEC_NPROJ; ++i)
            if (item.substr(0, eq) == kDecProjNames[i]) dst[i] = std::atoi(item.c_str() + eq + 1);
        pos = end + 1;
      }
    };
    if (const char* v = std::getenv("VLOG_AMD_DEC_GEMM")) per_proj(v, e->dec_plan);
    if (const char* v = std::getenv("VLOG_AMD_DEC_COLS")) per_proj(v, e->dec_cols);
    if (const char* v = std::getenv("VLOG_AMD_DEC_KR")) per_proj(v, e->dec_kr);
    if (const char* v = std::getenv("VLOG_AMD_CROSS_BLOCKS")) e->cross_cap = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("VLOG_AMD_CROSS_FUSE")) e->cross_fuse = std::atoi(v) & 3;
    if (const char* v = std::getenv("VLOG_AMD_ENC_CHUNK")) e->enc_chunk = std::max(1, std::atoi(v));
    if (const char* v = std::getenv("VLOG_AMD_CROSS_MODE")) e->cross_mode = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_XSNAKE")) e->xsnake = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_XKEEP")) e->xkeep = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("VLOG_AMD_XDMA")) e->xdma = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_XCHUNKS")) e->xchunks = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_CROSS_FP8")) e->cross_fp8 = std::atoi(v) != 0;
    if (const char* v = std::getenv("VLOG_AMD_DEC_BIG_LDS")) e->dec_big_lds = std::atoi(v) == 144 ? 144 : 72;
    if (const char* v = std::getenv("VLOG_AMD_DEC_BIG_ROWS")) e->dec_big_rows = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("VLOG_AMD_DEC_BIG128")) e->dec_big128 = std::max(0, std::atoi(v));
    try {
      build_layout(e);
      build_frontend(e, nullptr);
    } catch (...) {
      delete e;
      throw;
    }
    *out = e;
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

void wm_destroy(wm_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  for (DevBuf* b : {&e->arena, &e->fe_window, &e->fe_cos, &e->fe_sin, &e->fe_filt, &e->fe_lo, &e->fe_hi, &e->e_cols,
                    &e->e_h1, &e->e_x, &e->e_hb, &e->e_qkv, &e->e_ao, &e->e_ff, &e->e_seek, &e->e_len, &e->ckv,
                    &e->skv, &e->d_tokens, &e->d_lin, &e->d_seq_len, &e->d_done, &e->d_cum, &e->d_row_tok,
                    &e->d_row_pos, &e->d_row_hyp, &e->d_hyp_slot, &e->d_n_active, &e->d_suppress, &e->d_cand_tok,
                    &e->d_cand_lp, &e->d_fin_tok, &e->d_fin_len, &e->d_fin_cum, &e->d_n_fin, &e->d_ns,
                    &e->d_logit_rows, &e->d_prow_tok, &e->d_prow_pos, &e->d_prow_hyp, &e->d_head_map, &e->s_x,
                    &e->s_hb, &e->s_q, &e->s_ao, &e->s_ff, &e->s_logits, &e->s_pm, &e->s_pl, &e->s_po, &e->gemm_ws, &e->gemm_ws2, &e->prof_dbytes, &e->d_cross_cnt, &e->d_lnstat,
                    &e->xenc, &e->xscale, &e->xwkt, &e->xwvb, &e->s_qp, &e->s_pu, &e->s_pml, &e->a_logits, &e->a_attn,
                    &e->a_next, &e->a_probs, &e->a_rowsum, &e->a_z, &e->a_mat, &e->a_cost, &e->a_trace, &e->a_pi,
                    &e->a_pj, &e->a_plen, &e->a_meta, &e->a_enc, &e->a_kv, &e->d_tok_lp, &e->d_tok_lp_o, &e->d_fin_lp, &e->d_win_prompt,
                    &e->d_win_slot, &e->d_hyp_out, &e->d_res_tok, &e->d_res_len, &e->d_res_cum, &e->d_res_ns, &e->d_res_lp,
                    &e->d_res_lp_o, &e->d_ev})
    b->release();
  if (e->st2) (void)hipStreamDestroy(e->st2);
  if (e->gst) (void)hipStreamDestroy(e->gst);
  if (e->ev_g0) (void)hipEventDestroy(e->ev_g0);
  if (e->ev_g1) (void)hipEventDestroy(e->ev_g1);
  for (hipEvent_t ev : {e->ev_fork, e->ev_mid, e->ev_join})
    if (ev) (void)hipEventDestroy(ev);
  delete e;
}

int wm_set_weight(wm_engine* e, const char* name, const void* d_src, int64_t nbytes, void* stream) {
  return guarded(e, [&] {
    auto it = e->slots.find(name);
    if (it == e->slots.end()) throw std::runtime_error(std::string("wm_set_weight: unknown weight ") + name);
    if ((size_t)nbytes != it->second.bytes)
      throw std::runtime_error(std::string("wm_set_weight: ") + name + " expects " + std::to_string(it->second.bytes) +
                               " bytes, got " + std::to_string(nbytes));
    HIP_OK(hipMemcpyAsync((char*)e->arena.p + it->second.off, d_src, nbytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    it->second.set = true;
    if (it->first == "dec.ckv.w") e->xwkt_ready = false;
    e->fold_ready = false;
  });
}

int32_t wm_weight_count(wm_engine* e) { return e ? (int32_t)e->slot_order.size() : 0; }

int wm_weight_info(wm_engine* e, int32_t i, const char** name, int64_t* nbytes, int32_t* elem_bytes) {
  return guarded(e, [&] {
    if (i < 0 || i >= (int32_t)e->slot_order.size()) throw std::runtime_error("wm_weight_info: index out of range");
    const auto& nm = e->slot_order[i];
    const Slot& s = e->slots.at(nm);
    if (name) *name = nm.c_str();
    if (nbytes) *nbytes = (int64_t)s.bytes;
    if (elem_bytes) *elem_bytes = s.elem;
  });
}

int32_t wm_weights_complete(wm_engine* e) {
  if (!e) return 0;
  for (auto& kv : e->slots)
    if (!kv.second.set) return 0;
  return 1;
}

int wm_logmel(wm_engine* e, const float* d_pcm, int64_t pcm_offset, int64_t n_samples, int64_t frame0, int32_t n_frames,
              float* d_mel, int64_t ld, uint32_t* d_gmax, void* stream) {
  return guarded(e, [&] {
    if (frame0 % 2) throw std::runtime_error("wm_logmel: frame0 must be even (frames are transformed in pairs)");
    const long long n_padded = n_samples + 160;
    ProfScope ps(e, P_LOGMEL, (hipStream_t)stream, 2.0 * 201 * 400 * 2 * n_frames, 4.0 * 160 * n_frames + 4.0 * e->dm.n_mels * n_frames);
    launch_logmel(d_pcm, pcm_offset, n_samples, n_padded, frame0, n_frames, e->fe_window.as<float>(), e->fe_cos.as<float>(),
                  e->fe_sin.as<float>(), e->fe_filt.as<float>(), e->fe_lo.as<int>(), e->fe_hi.as<int>(), e->dm.n_mels,
                  d_mel, ld, d_gmax, (hipStream_t)stream);
  });
}

int wm_logmel_finalize(wm_engine* e, float* d_mel, int64_t n_frames, int64_t ld, const uint32_t* d_gmax, const float* h_gmax,
                       float* h_gmax_out, void* stream) {
  return guarded(e, [&] {
    hipStream_t st = (hipStream_t)stream;
    e->s_pm.ensure(64);
    float* gm = e->s_pm.as<float>();
    if (h_gmax) HIP_OK(hipMemcpyAsync(gm, h_gmax, 4, hipMemcpyHostToDevice, st));
    else launch_ordered_to_float(d_gmax, gm, st);
    if (h_gmax_out) {
      HIP_OK(hipMemcpyAsync(h_gmax_out, gm, 4, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
    }
    launch_logmel_clamp(d_mel, e->dm.n_mels, n_frames, ld, nullptr, gm, st);
    if (h_gmax) HIP_OK(hipStreamSynchronize(st));
  });
}

int wm_encode(wm_engine* e, const float* d_mel, int64_t ld, const int32_t* h_seek, const int32_t* h_nframes, int32_t B,
              void* d_enc_out, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    check_weights(e);
    hipStream_t st = (hipStream_t)stream;
    const int chunk = std::max(1, e->enc_chunk);
    const size_t per = (size_t)e->dm.n_audio_ctx * e->dm.n_state;
    for (int b0 = 0; b0 < B; b0 += chunk) {
      const int nb = std::min(chunk, B - b0);
      for (int i = 0; i < nb; ++i)
        if (h_nframes[b0 + i] < 0 || h_nframes[b0 + i] > 3000 || h_seek[b0 + i] < 0 || h_seek[b0 + i] + h_nframes[b0 + i] > ld)
          throw std::runtime_error("wm_encode: window outside the mel buffer");
      encode_chunk(e, d_mel, ld, h_seek + b0, h_nframes + b0, nb, (bf16*)d_enc_out + (size_t)b0 * per, st);
      HIP_OK(hipStreamSynchronize(st));   // seek/len staging buffers are reused by the next chunk
    }
  });
}

int wm_reserve(wm_engine* e, int32_t n_slots, int32_t n_hyp, void* stream) {
  return guarded(e, [&] {
    (void)stream;
    reserve(e, n_slots, n_hyp);
  });
}

int wm_cross_kv(wm_engine* e, const void* d_enc, int32_t B, int32_t slot0, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    check_weights(e);
    if (slot0 < 0 || slot0 + B > e->n_slots) throw std::runtime_error("wm_cross_kv: slots out of range (wm_reserve first)");
    const auto& m = e->dm;
    const int d = m.n_state, T = m.n_audio_ctx;
    if (e->cross_mode == 1 && e->cross_fp8) {   // factored, fp8: e4m3 image + per-position scales
      const size_t per = (size_t)T * d;
      ProfScope ps(e, P_CROSSKV_GEMM, (hipStream_t)stream, 0, 3.0 * B * per + 4.0 * B * T);
      launch_xquant8((const bf16*)d_enc, (long long)B * T, d, e->xenc.as<unsigned char>() + (size_t)slot0 * per,
                     e->xscale.as<float>() + (size_t)slot0 * T, (hipStream_t)stream);
      return;
    }
    if (e->cross_mode == 1) {   // factored: the slot holds the encoder output itself, tile-blocked
      const size_t per = (size_t)T * d;
      ProfScope ps(e, P_CROSSKV_GEMM, (hipStream_t)stream, 0, 2.0 * 2 * B * per);
      launch_xblock((const bf16*)d_enc, B, T, d, e->xenc.as<bf16>() + (size_t)slot0 * xblock_slot_elems(T, d), true,
                    (hipStream_t)stream);
      return;
    }
    GemmEpi ep = epi_of(EPI_CROSS_KV, e->ckv.p, 0, e->Wf("dec.ckv.b"));
    ep.rpb = T; ep.d = d; ep.head_dim = 64; ep.n_head = m.n_head; ep.n_slots = e->n_slots; ep.slot0 = slot0;
    gemm_p(e, P_CROSSKV_GEMM, amat((const bf16*)d_enc, d), e->Wb("dec.ckv.w"), d, B * T, m.n_dec_layer * 2 * d, d, ep,
           (hipStream_t)stream);
  });
}

int wm_generate(wm_engine* e, const wm_generate_args* a, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    generate(e, a, (hipStream_t)stream);
  });
}

int wm_forward(wm_engine* e, int32_t n_seq, const int32_t* h_slots, int32_t seq_len, const int32_t* h_tokens, float* d_logits,
               int32_t last_only, const int32_t* h_align_heads, int32_t n_align, float* d_attn, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    forward(e, n_seq, h_slots, seq_len, h_tokens, d_logits, last_only, h_align_heads, n_align, d_attn, (hipStream_t)stream);
  });
}

int wm_detect_language(wm_engine* e, int32_t n, const int32_t* h_slots, int32_t lang_begin, int32_t n_langs,
                       float* h_probs, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    if (n <= 0) return;
    if (lang_begin < 0 || n_langs <= 0 || lang_begin + n_langs > e->dm.n_vocab)
      throw std::runtime_error("wm_detect_language: language tokens outside the vocabulary");
    hipStream_t st = (hipStream_t)stream;
    const int V = e->dm.n_vocab;
    std::vector<int> toks(n, e->dm.sot);
    e->a_logits.ensure((size_t)n * V * 4);
    forward(e, n, h_slots, 1, toks.data(), e->a_logits.as<float>(), 1, nullptr, 0, nullptr, st);
    e->a_probs.ensure((size_t)n * n_langs * 4);
    launch_lang_probs(e->a_logits.as<float>(), V, n, lang_begin, n_langs, e->a_probs.as<float>(), st);
    HIP_OK(hipMemcpyAsync(h_probs, e->a_probs.p, (size_t)n * n_langs * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  });
}

int64_t wm_device_bytes(wm_engine* e) { return e ? (int64_t)e->device_bytes() : 0; }

int wm_frame_energy(wm_engine* e, const float* d_pcm, int64_t n_samples, int32_t frame, float* d_db, void* stream) {
  return guarded(e, [&] {
    if (frame <= 0) throw std::runtime_error("wm_frame_energy: bad frame size");
    const int frames = (int)((n_samples + frame - 1) / frame);
    launch_frame_energy(d_pcm, n_samples, frame, frames, d_db, (hipStream_t)stream);
  });
}

int wm_pcm_from_s16(wm_engine* e, const int16_t* d_src, int64_t n, float* d_dst, void* stream) {
  return guarded(e, [&] {
    if (n < 0) throw std::runtime_error("wm_pcm_from_s16: negative length");
    launch_pcm_s16((const short*)d_src, n, d_dst, (hipStream_t)stream);
  });
}

int wm_cross_fp8_quantize(wm_engine* e, const void* d_enc, int64_t rows, uint8_t* d_codes, float* d_scale, void* stream) {
  return guarded(e, [&] {
    launch_xquant8((const bf16*)d_enc, rows, e->dm.n_state, d_codes, d_scale, (hipStream_t)stream);
  });
}

int wm_vad_probs(wm_engine* e, const wm_vad_weights* w, const float* d_pcm, int64_t n_samples, float* d_work,
                 float* d_probs, void* stream) {
  return guarded(e, [&] {
    if (!w || !w->stft_basis || !w->w_ih || !w->w_hh || !w->b_ih || !w->b_hh || !w->head_w || !w->head_b)
      throw std::runtime_error("wm_vad_probs: missing weight");
    if (n_samples < 0 || n_samples % 512) throw std::runtime_error("wm_vad_probs: n_samples must be a multiple of 512");
    VadW vw;
    vw.basis = w->stft_basis;
    for (int i = 0; i < 4; ++i) {
      if (!w->conv_w[i] || !w->conv_b[i]) throw std::runtime_error("wm_vad_probs: missing conv weight");
      vw.cw[i] = w->conv_w[i];
      vw.cb[i] = w->conv_b[i];
    }
    vw.w_ih = w->w_ih; vw.w_hh = w->w_hh; vw.b_ih = w->b_ih; vw.b_hh = w->b_hh;
    vw.dec_w = w->head_w; vw.dec_b = w->head_b;
    launch_vad(vw, d_pcm, n_samples / 512, d_work, d_probs, (hipStream_t)stream);
  });
}

int wm_align(wm_engine* e, int32_t slot, int32_t sot_len, const int32_t* h_sot, int32_t n_text, const int32_t* h_text,
             int32_t num_frames, const int32_t* h_heads, int32_t n_heads, int32_t median_filter_width, float* h_probs,
             int32_t* h_text_idx, int32_t* h_time_idx, int32_t* h_path_len, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    check_weights(e);
    align(e, slot, sot_len, h_sot, n_text, h_text, num_frames, h_heads, n_heads, median_filter_width, h_probs, h_text_idx,
          h_time_idx, h_path_len, (hipStream_t)stream);
  });
}

int wm_align_batch(wm_engine* e, int32_t n, const int32_t* h_slots, int32_t sot_len, const int32_t* h_sot,
                   const int32_t* h_text_off, const int32_t* h_text, const int32_t* h_num_frames, const int32_t* h_heads,
                   int32_t n_heads, int32_t median_filter_width, float* h_probs, const int64_t* h_path_off,
                   int32_t* h_text_idx, int32_t* h_time_idx, int32_t* h_path_len, void* stream) {
  return guarded(e, [&] {
    require_weights(e);
    check_weights(e);
    for (int i = 0; i < n; ++i)
      if (h_slots[i] < 0 || h_slots[i] >= e->n_slots) throw std::runtime_error("wm_align_batch: slot out of range");
    align_batch(e, n, h_slots, sot_len, h_sot, h_text_off, h_text, h_num_frames, h_heads, n_heads, median_filter_width,
                h_probs, (const long long*)h_path_off, h_text_idx, h_time_idx, h_path_len, (hipStream_t)stream);
  });
}

int wm_dtw(wm_engine* e, const float* d_cost, int32_t n, int32_t m, int32_t* h_text_idx, int32_t* h_time_idx,
           int32_t* h_path_len, void* stream) {
  return guarded(e, [&] { dtw_run(e, d_cost, n, m, h_text_idx, h_time_idx, h_path_len, (hipStream_t)stream); });
}

int wm_encoder_attention(wm_engine* e, const void* d_qkv, void* d_out, int32_t B, int32_t T, void* stream) {
  return guarded(e, [&] {
    if (B <= 0 || T <= 0) throw std::runtime_error("wm_encoder_attention: bad B/T");
    launch_attn_enc((const bf16*)d_qkv, (bf16*)d_out, B, T, e->dm.n_state, e->dm.n_head, (hipStream_t)stream);
  });
}

int wm_set_option(wm_engine* e, const char* key, int64_t value) {
  return guarded(e, [&] {
    if (!key) throw std::runtime_error("wm_set_option: null key");
    const std::string k(key);
    if (k == "decode_split") e->dec_split = value != 0;
    else if (k == "decode_graph") e->dec_graph = value != 0;
    else if (k == "decode_gemv") e->dec_gemv = value != 0;
    else if (k == "decode_gemv_ln") e->dec_gemv_ln = value != 0;
    else if (k == "decode_gemv_ln_fc2") e->dec_gemv_ln_fc2 = value != 0;
    else if (k == "decode_ring_gemm") e->dec_ring = value != 0;
    else if (k == "decode_gemm_plan") {
      if (value != 0 && value != 1) throw std::runtime_error("wm_set_option: decode_gemm_plan is 0 or 1");
      for (int i = 0; i < DEC_NPROJ; ++i) e->dec_plan[i] = kDecPlanPresets[value][i], e->dec_cols[i] = kDecColsPresets[value][i];
    } else if (k.rfind("decode_gemm.", 0) == 0) {
      const std::string pj = k.substr(12);
      int i = 0;
      while (i < DEC_NPROJ && pj != kDecProjNames[i]) ++i;
      if (i == DEC_NPROJ) throw std::runtime_error("wm_set_option: unknown projection " + pj);
      if (value < -2 || value > 160) throw std::runtime_error("wm_set_option: decode_gemm.<proj> in [-2, 160]");
      e->dec_plan[i] = (int)value;
    } else if (k.rfind("decode_gemm_cols.", 0) == 0) {
      const std::string pj = k.substr(17);
      int i = 0;
      while (i < DEC_NPROJ && pj != kDecProjNames[i]) ++i;
      if (i == DEC_NPROJ) throw std::runtime_error("wm_set_option: unknown projection " + pj);
      if (value != 32 && value != 64) throw std::runtime_error("wm_set_option: decode_gemm_cols.<proj> is 32 or 64");
      e->dec_cols[i] = (int)value;
    }
    else if (k == "cross_attn_blocks") e->cross_cap = (int)std::max<int64_t>(0, value);
    else if (k == "cross_attn_fuse") e->cross_fuse = (int)(value & 3);
    else if (k == "cross_attn_snake") e->xsnake = value != 0;
    else if (k == "cross_attn_keep") e->xkeep = (int)std::max<int64_t>(0, std::min<int64_t>(value, 1 << 20));
    else if (k == "cross_attn_dma") e->xdma = value != 0;
    else if (k == "cross_attn_chunks") e->xchunks = value != 0;
    else if (k == "gemm_persistent") gemm_8p_set_persistent((int)value);
    else if (k == "align_fused") align_set_fused((int)value);
    else if (k == "encode_chunk") e->enc_chunk = (int)std::max<int64_t>(1, std::min<int64_t>(value, 4096));
    else if (k == "cross_fp8") {
      // fp8 (OCP e4m3) cross memory in the factored form; switching re-allocates the window slots (their
      // contents are dropped: run wm_cross_kv again)
      const int v = value ? 1 : 0;
      if (v != e->cross_fp8) {
        HIP_OK(hipDeviceSynchronize());
        e->cross_fp8 = v;
        const int n = e->n_slots;
        e->n_slots = 0;
        if (n > 0) reserve(e, n, e->n_hyp_cap);
        else { e->xenc.release(); e->xscale.release(); }
      }
    }
    else if (k == "cross_mode") {
      // switching re-allocates the window slots in the new form (their contents are dropped: run
      // wm_cross_kv again)
      const int v = value ? 1 : 0;
      if (v != e->cross_mode) {
        HIP_OK(hipDeviceSynchronize());
        e->cross_mode = v;
        const int n = e->n_slots;
        e->n_slots = 0;
        if (n > 0) reserve(e, n, e->n_hyp_cap);
        else { e->ckv.release(); e->xenc.release(); }
      }
    }
    else if (k == "debug_nan_row") e->dbg_nan_row = (int)std::max<int64_t>(-1, std::min<int64_t>(value, 1 << 30));
    else if (k == "debug_nan_count") e->dbg_nan_count = (int)std::max<int64_t>(1, std::min<int64_t>(value, 1 << 20));
    else if (k == "cross_tf") e->cross_tf = value ? 1 : 0;
    else if (k == "cross_mfma") e->cross_mfma = value ? 1 : 0;
    else if (k == "cross_mfma_fuse") e->cross_mfma_fuse = value ? 1 : 0;
    else if (k == "decode_gemm_big_rows") e->dec_big_rows = (int)std::max<int64_t>(0, std::min<int64_t>(value, 1 << 20));
    else if (k == "decode_gemm_big128") e->dec_big128 = (int)std::max<int64_t>(0, std::min<int64_t>(value, 1 << 20));
    else if (k == "decode_gemm_big_fc2_kr") {
      if (value != 0 && (value < 64 || value % 64 != 0)) throw std::runtime_error("decode_gemm_big_fc2_kr: 0 or a multiple of 64");
      e->dec_big_fc2_kr = (int)std::min<int64_t>(value, 1 << 20);
    }
    else if (k == "decode_ln_fold") e->dec_ln_fold = value ? 1 : 0;
    else if (k == "decode_gemm_big_lds") {
      if (value != 72 && value != 144) throw std::runtime_error("decode_gemm_big_lds: 72 or 144");
      e->dec_big_lds = (int)value;
    }
    else throw std::runtime_error("wm_set_option: unknown option " + k);
  });
}

int wm_get_option(wm_engine* e, const char* key, int64_t* value) {
  return guarded(e, [&] {
    if (!key || !value) throw std::runtime_error("wm_get_option: null argument");
    const std::string k(key);
    auto proj = [&](size_t n) {
      const std::string pj = k.substr(n);
      for (int i = 0; i < DEC_NPROJ; ++i)
        if (pj == kDecProjNames[i]) return i;
      throw std::runtime_error("wm_get_option: unknown projection " + pj);
    };
    if (k == "decode_split") *value = e->dec_split;
    else if (k == "decode_graph") *value = e->dec_graph;
    else if (k == "decode_gemv") *value = e->dec_gemv;
    else if (k == "decode_gemv_ln") *value = e->dec_gemv_ln;
    else if (k == "decode_gemv_ln_fc2") *value = e->dec_gemv_ln_fc2;
    else if (k == "decode_ring_gemm") *value = e->dec_ring;
    else if (k == "decode_gemm_plan") {
      int p = -1;
      for (int q = 0; q < 2 && p < 0; ++q) {
        bool eq = true;
        for (int i = 0; i < DEC_NPROJ; ++i) eq &= e->dec_plan[i] == kDecPlanPresets[q][i] && e->dec_cols[i] == kDecColsPresets[q][i];
        if (eq) p = q;
      }
      *value = p;                               // -1: a per-projection setting departs from both presets
    } else if (k.rfind("decode_gemm.", 0) == 0) *value = e->dec_plan[proj(12)];
    else if (k.rfind("decode_gemm_cols.", 0) == 0) *value = e->dec_cols[proj(17)];
    else if (k == "cross_attn_blocks") *value = e->cross_cap;
    else if (k == "cross_attn_fuse") *value = e->cross_fuse;
    else if (k == "cross_attn_snake") *value = e->xsnake;
    else if (k == "cross_attn_keep") *value = e->xkeep;
    else if (k == "cross_attn_dma") *value = e->xdma;
    else if (k == "cross_attn_chunks") *value = e->xchunks;
    else if (k == "gemm_persistent") *value = gemm_8p_get_persistent();
    else if (k == "align_fused") *value = align_get_fused();
    else if (k == "encode_chunk") *value = e->enc_chunk;
    else if (k == "cross_fp8") *value = e->cross_fp8;
    else if (k == "cross_mode") *value = e->cross_mode;
    else if (k == "debug_nan_row") *value = e->dbg_nan_row;
    else if (k == "debug_nan_count") *value = e->dbg_nan_count;
    else if (k == "cross_tf") *value = e->cross_tf;
    else if (k == "cross_mfma") *value = e->cross_mfma;
    else if (k == "cross_mfma_fuse") *value = e->cross_mfma_fuse;
    else if (k == "decode_gemm_big_rows") *value = e->dec_big_rows;
    else if (k == "decode_gemm_big128") *value = e->dec_big128;
    else if (k == "decode_gemm_big_fc2_kr") *value = e->dec_big_fc2_kr;
    else if (k == "decode_ln_fold") *value = e->dec_ln_fold;
    else if (k == "decode_gemm_big_lds") *value = e->dec_big_lds;
    else throw std::runtime_error("wm_get_option: unknown option " + k);
  });
}

int32_t wm_profile_classes(void) { return P_N; }
const char* wm_profile_name(int32_t cls) { return (cls >= 0 && cls < P_N) ? kProfNames[cls] : ""; }

int wm_profile_select(wm_engine* e, uint32_t class_mask) {
  return guarded(e, [&] {
    HIP_OK(hipDeviceSynchronize());
    if (!class_mask) {        // stop recording; keep what was recorded for wm_profile_read
      e->prof_on = false;
      return;
    }
    for (int c = 0; c < P_N; ++c) {
      for (auto& pr : e->prof_ev[c]) { e->ev_pool.push_back(pr.first); e->ev_pool.push_back(pr.second); }
      e->prof_ev[c].clear();
      e->prof_flops[c] = 0;
      e->prof_bytes[c] = 0;
    }
    e->prof_dbytes.ensure((size_t)P_N * STAT_SLOTS * sizeof(unsigned long long));
    HIP_OK(hipMemset(e->prof_dbytes.p, 0, (size_t)P_N * STAT_SLOTS * sizeof(unsigned long long)));
    e->prof_mask = class_mask;
    e->prof_on = true;
  });
}

int wm_profile(wm_engine* e, int32_t enable) { return wm_profile_select(e, enable ? ((1u << P_N) - 1u) : 0u); }

int wm_profile_read(wm_engine* e, int32_t cls, int64_t* launches, double* ms, double* flops, double* bytes) {
  return guarded(e, [&] {
    if (cls < 0 || cls >= P_N) throw std::runtime_error("wm_profile_read: bad class");
    HIP_OK(hipDeviceSynchronize());
    double t = 0;
    for (auto& pr : e->prof_ev[cls]) {
      float x = 0;
      HIP_OK(hipEventElapsedTime(&x, pr.first, pr.second));
      t += x;
    }
    std::vector<unsigned long long> slots(STAT_SLOTS, 0);
    if (e->prof_dbytes.p)
      HIP_OK(hipMemcpy(slots.data(), e->prof_dbytes.as<unsigned long long>() + (size_t)cls * STAT_SLOTS,
                       STAT_SLOTS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double dbytes = 0;
    for (auto v : slots) dbytes += (double)v;
    *launches = (int64_t)e->prof_ev[cls].size();
    *ms = t;
    *flops = e->prof_flops[cls];
    *bytes = e->prof_bytes[cls] + dbytes;
  });
}

}  // extern "C"
