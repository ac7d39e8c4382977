// mz_learner.h — launchers of the learner / trainer kernels (mz_stem, mz_optim, mz_qnet,
// mz_trainer, mz_ppo, mz_qact), used by the C ABI (mz_api.hip).
#pragma once
#include "mz_kernels.h"

int mz_stem_chunks(int n);
hipError_t mz_launch_stem_fwd(const uint32_t* bits, const float* obs6, int n, const float* w,
                              const float* b, float drop_p, const uint64_t* rng, uint32_t salt,
                              float* feat, int ld, uint8_t* code, hipStream_t s);
hipError_t mz_launch_stem_bwd(const uint32_t* bits, const uint8_t* code, const float* g, int ld,
                              int n, float drop_p, float* partial, float* dw, float* db,
                              hipStream_t s, uint64_t* advance = nullptr);
#define MZ_OPT_MAX_SEGS 16

hipError_t mz_launch_adamw(float* p, float* m, float* v, const float* const* grads,
                           const int64_t* seg_len, int nseg, const float* lr, float* step, double b1,
                           double b2, double eps, double wd, float clamp, float gscale,
                           int write_grad, hipStream_t s);
hipError_t mz_launch_pair_surrogate(const float* lp_new, const float* lp_old, const float* adv,
                                    int b, float clip, float* part, float* dsum, hipStream_t s);
hipError_t mz_launch_leaky_bf16(uint16_t* x, int64_t n, float slope, hipStream_t s);
hipError_t mz_launch_colsum(const float* g, int n, int m, int ld, float* out, hipStream_t s);
hipError_t mz_launch_replay_gather(const int64_t* idx, int b, int64_t cap, const float* s6,
                                   const uint32_t* sw, const int64_t* a, const float* r,
                                   const float* s6n, const uint32_t* swn, float* o6, uint32_t* ow,
                                   int64_t* oa, float* orw, hipStream_t s);

// ---- trainer bookkeeping (mz_trainer.hip)
struct MzHeadBf16 {  // acting head: f32 Linear weights / biases -> bf16 (fc1 permuted + padded)
  const float* w[3];
  const float* b[3];
  uint16_t* dw[3];
  uint16_t* db[3];
  int out[3], in[3];
  int ld0, conv_out, conv_ch;
};
struct MzReplayPush {  // ring rows ptr .. ptr + n - 1 <- n source rows, per array (NULL src: skip)
  const void* src[6];  // obs6, bits, action (int32 -> int64), reward, next obs6, next bits
  void* dst[6];
  int words[6];        // 32-bit words per row
  int n;
  int64_t cap, ptr;
};
hipError_t mz_launch_greedy_list(const MzAct& ap, int n, const int32_t* blk, int32_t* rows,
                                 int32_t* count, int32_t* count_host, hipStream_t s);
hipError_t mz_launch_tick(const uint8_t* term, const uint8_t* trunc, float* steps_done,
                          float eps_final, float eps_span, float inv_decay, float* eps_out,
                          unsigned long long* wins, unsigned long long* episodes, uint64_t seed,
                          uint64_t counter, int n, int32_t* scratch, int32_t* rows, int32_t* count,
                          hipStream_t s);
hipError_t mz_launch_greedy_scatter(const uint16_t* q, int ldq, const int32_t* rows,
                                    const int32_t* count, int m, int64_t* greedy, hipStream_t s);
hipError_t mz_launch_head_bf16(const MzHeadBf16& h, hipStream_t s);
hipError_t mz_launch_replay_push(const MzReplayPush& p, hipStream_t s);
hipError_t mz_launch_replay_idx(uint64_t seed, uint64_t counter, int64_t newest, int64_t n_avail,
                                int64_t cap, int64_t* out, int n, hipStream_t s);
hipError_t mz_launch_q_loss(const float* q, int ldq, const float* qn, int ldn, const float* qt,
                            int ldt, const int64_t* action, const float* reward, float gamma, int b,
                            float* loss, float* diff, hipStream_t s);
hipError_t mz_launch_q_loss_bwd(const float* g, const float* diff, const int64_t* action, int b,
                                int rows, float norm, float* dq, hipStream_t s);
// the Q head (act(z2) -> fc3) of the source's and the target's rows + the loss (mz_trainer.hip)
struct MzHeadLoss {
  const float *z2s, *w3s, *b3s, *z2t, *w3t, *b3t;
  int lds, ldt, dbl, b, H, act;
  const int64_t* action;
  const float* reward;
  float gamma;
  float* part;      // [mz_head_loss_blocks(b)]
  unsigned* ticket; // unused since round 5 (the partials are summed by a second launch)
  float *loss, *diff;
};
int mz_head_loss_blocks(int b);
int mz_head_loss_bwd_blocks(int b);
hipError_t mz_launch_head_loss(const MzHeadLoss& p, hipStream_t s);
hipError_t mz_launch_head_loss_bwd(const float* g, const float* diff, const int64_t* action, int b,
                                   float norm, const float* z2s, int lds, const float* w3s, int H,
                                   int act, float* dz2, int ldd, float* part, hipStream_t s);
hipError_t mz_launch_adamw_groups(float* p, float* m, float* v, const float* const* grads,
                                  const int64_t* seg_len, const int32_t* seg_group, int nseg,
                                  const float* lr, float* step, double b1, double b2, double eps,
                                  double wd, float max_norm, float* scratch, hipStream_t s);

// ---- PPO rollout (mz_ppo.hip) ------------------------------------------------------------
struct MzPpoAct {
  const float* logits; int ldl;     // actor logits [B][ldl >= 4], f32
  const float* value; int ldv;      // critic values [B] (stride ldv)
  const float* obs6; const uint32_t* bits;
  int B, L;                         // instances, episode buffer length
  uint64_t seed, counter;
  const int32_t* t;                 // per-instance step index
  float* b_s6; uint32_t* b_w; int64_t* b_a; float* b_lp; float* b_v;  // [B][L] records
  int32_t* act_out;                 // [B] actions for mz_step
};
struct MzPpoScan {
  const double* reward64; const uint8_t* term; const uint8_t* trunc;
  int B, L;
  int32_t* t; double* b_r;
  int32_t* fin_id; int64_t* fin_off; int32_t* fin_len; int32_t* fin_count;
  int64_t* pool_fill; int64_t* pool_total; long long* stats;
};
struct MzPpoFinish {
  const double* b_r; const float* b_s6; const uint32_t* b_w; const int64_t* b_a; const float* b_lp;
  const float* b_v; int L;
  const int32_t* fin_id; const int64_t* fin_off; const int32_t* fin_len; const int32_t* fin_count;
  double gamma; int64_t cap;
  float* p_s6; uint32_t* p_w; int64_t* p_a; float* p_lp; float* p_adv; float* p_ret;
};
hipError_t mz_launch_ppo_act(const MzPpoAct& q, hipStream_t s);
hipError_t mz_launch_ppo_scan(const MzPpoScan& q, hipStream_t s);
hipError_t mz_launch_ppo_finish(const MzPpoFinish& q, int max_episodes, hipStream_t s);
struct MzPpoHead {  // fused loss of one minibatch (4 actions)
  const float* logits; int ldl; const float* value; int ldv;
  const int64_t* action; const float* lp_old; const float* adv; const float* ret;
  const float* coef; int b;
  float* lp_new; float* ent; float* p; float* dent; float* part; float* dsum;  // scratch
  float* loss; float* dlogits; int ldg; float* dvalue; int ldvg;
};
hipError_t mz_launch_ppo_head(const MzPpoHead& q, float clip, hipStream_t s);

// ---- f32-accurate acting forward on the bf16 MFMA (mz_qact.hip) ------------------------------
struct MzQAct {
  const uint32_t* bits; const float* obs6;   // [B][22], [B][6] (instance rows)
  const int32_t* rows; const int32_t* count; int n;  // rows[i] (i < min(n, *count)) or row i
  const float* conv_w; const float* conv_b;  // [32][27], [32]
  const uint16_t* w1h; const uint16_t* w1l; const float* b1;  // prepared [1024][1600] bf16, [1024]
  const uint16_t* w2h; const uint16_t* w2l; const float* b2;  // prepared [512][1024] bf16, [512]
  const float* w3; const float* b3;          // [4][512], [4]
  uint32_t drop_thresh; float drop_scale; uint32_t key;
  float* h1;                                 // workspace [n][1024] f32
  int64_t* greedy; float* q_out;             // greedy[inst] = argmax; q_out [n][4] (nullable)
};
int mz_qact_row_tiles(int n);
int64_t mz_qact_ws_floats(int n);
hipError_t mz_launch_qact(const MzQAct& q, int relu, hipStream_t s);
hipError_t mz_launch_qact_prepare(const float* w1, const float* w2, uint16_t* w1h, uint16_t* w1l,
                                  uint16_t* w2h, uint16_t* w2l, hipStream_t s);

