// mz_kernels.h — launchers of the env-side device kernels (mz_env.hip, mz_metrics.hip), used by
// the C ABI (mz_api.hip). The learner kernels' launchers are in mz_learner.h: this header is part
// of k_step's source hash (bench.py KSTEP_SOURCES), which decides whether the committed PMC
// traffic record still describes the k_step being benchmarked.
#pragma once
#include "mz_common.h"
#include "mz_screen.h"

size_t mz_build_lds_size(int P);
hipError_t mz_launch_build(const MzDev& d, const int32_t* env_ids, int32_t n, bool generate,
                           const uint8_t* algo_list, int32_t algo_all, int32_t dim, uint64_t seed,
                           const uint8_t* grids, const int32_t* start_goal, int pymode,
                           uint32_t* py_state, hipStream_t s);
hipError_t mz_launch_regen(const MzDev& d, const int32_t* idx, const int32_t* count,
                           int32_t n_static, uint64_t seed, uint32_t epoch, hipStream_t s);
hipError_t mz_launch_step(const MzDev& d, const int32_t* act, const MzAct* ap, bool autoreset,
                          const MzOut& o, hipStream_t s);
hipError_t mz_launch_reset_list(const MzDev& d, const int32_t* idx, int32_t* count,
                                int32_t n_static, const MzOut& o, hipStream_t s);
hipError_t mz_launch_meta(const MzDev& d, int32_t* out, hipStream_t s);
hipError_t mz_launch_returns(const double* rew, int ld, const int32_t* rows, const int32_t* lens,
                             int n, double gamma, float* out, int ldo, hipStream_t s);
hipError_t mz_launch_reset_done(const MzDev& d, int regen, uint64_t seed, uint32_t epoch,
                                const MzOut& o, hipStream_t s);
hipError_t mz_launch_mask(const MzDev& d, int probs, float* out4, hipStream_t s);
hipError_t mz_launch_act(const MzDev& d, const MzAct& ap, hipStream_t s);
hipError_t mz_launch_greedy_rows(const MzAct& ap, int n, int32_t* blk, int32_t* rows,
                                 int32_t* count, int32_t* count_host, hipStream_t s);
hipError_t mz_launch_expand(const uint32_t* bits, float* out, int n, hipStream_t s);
hipError_t mz_launch_qfront(const uint32_t* bits, const float* obs6, const int32_t* rows,
                            const int32_t* count, int n, const float* w, const float* b,
                            float drop_p, uint64_t seed, uint64_t counter, uint16_t* out, int ld,
                            hipStream_t s);
// candidate builds / best-of-C selection (maze bank refills with C > 1, mz_generate_best; the
// compact candidates and the screen: mz_screen.h)
hipError_t mz_launch_cand_build(const MzDev& cd, const int32_t* ids, int base, const int* count, int n,
                                int C, const uint8_t* algo_list, int algo_all, int dim,
                                uint64_t seed, uint32_t epoch, hipStream_t s, int dbg = 0);
hipError_t mz_launch_cand_compact(const MzCompact& cc, int P, const int32_t* ids, int base,
                                  const int* count, int n, int C, const uint8_t* algo_list,
                                  int algo_all, int dim, uint64_t seed, uint32_t epoch, hipStream_t s,
                                  int dbg);
hipError_t mz_launch_cand_pick(const int* count, int n, int C, const double* score,
                               const int32_t* status, int32_t* pick, int32_t* xlist, int* xcount,
                               int xcap, int* stats, hipStream_t s, int dbg);
hipError_t mz_launch_cand_expand(const MzCompact& cc, const MzDev& dst, const int32_t* dst_ids,
                                 int base, const int* count, int n, int C, const int32_t* pick,
                                 const uint8_t* algo_list, int algo_all, hipStream_t s);
hipError_t mz_launch_cand_rebuild(const MzDev& cd, const int32_t* xlist, const int* xcount, int xcap,
                                  const int32_t* ids, int base, int C, const uint8_t* algo_list,
                                  int algo_all, int dim, uint64_t seed, uint32_t epoch, hipStream_t s,
                                  int dbg);
hipError_t mz_launch_cand_gather(const MzDev& cd, const int* count, int n, int C,
                                 const int32_t* status, int32_t* hmap, uint8_t* hgrid,
                                 int32_t* hinfo, int* hcount, int hcap, int gstride, hipStream_t s,
                                 int dbg);
hipError_t mz_launch_compact_from_handle(const MzDev& d, const int32_t* ids, int n, const MzCompact& cc,
                                        hipStream_t s);
hipError_t mz_launch_cand_select(const MzDev& cd, const MzDev& dst, const int32_t* dst_ids,
                                 int base, const int* count, int n, int C, const double* score,
                                 const int32_t* status, int* stats, hipStream_t s,
                                 const int32_t* xlist = nullptr, const int32_t* hmap = nullptr,
                                 const double* hprod = nullptr, const int32_t* hok = nullptr,
                                 int hcap = 0, int count_groups = 1, int dbg = 0);
size_t mz_metrics_lds_bytes(int P);
hipError_t mz_launch_metrics(const MzDev& d, const int32_t* env_ids, int32_t n, double* out,
                             hipStream_t s);

// Instances per workgroup of the greedy-row list (k_greedy_count / k_greedy_list, mz_env.hip) and
// of the trainer tick's per-block counts (k_tick_count, mz_trainer.hip): the tick writes the
// per-block counts the list kernel then reads as its block prefix sums, so both must use this.
constexpr int MZ_GR_BLOCK = 1024;
