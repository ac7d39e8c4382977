"""ctypes binding of libmazerl.so (include/mazerl.h). This is the product's only compute path.

If the library is missing or fails to load, every env constructor raises immediately — there is
no CPU fallback.
"""
import ctypes as C
import os

from . import _build

c_i32p = C.POINTER(C.c_int32)


class Config(C.Structure):
    _fields_ = [("num_envs", C.c_int32), ("max_dim", C.c_int32), ("toroidal", C.c_int32),
                ("enrich", C.c_int32), ("device", C.c_int32), ("reserved", C.c_int32 * 7)]


class StepOut(C.Structure):
    _fields_ = [("reward", C.c_void_p), ("reward64", C.c_void_p), ("terminated", C.c_void_p),
                ("truncated", C.c_void_p), ("pos", C.c_void_p), ("best_dir", C.c_void_p),
                ("obs6", C.c_void_p), ("window_bits", C.c_void_p), ("window", C.c_void_p),
                ("done_idx", C.c_void_p), ("done_count", C.c_void_p)]


class EnvInfo(C.Structure):
    _fields_ = [(k, C.c_int32) for k in ("n", "start_r", "start_c", "goal_r", "goal_c",
                                         "max_steps", "r", "c", "steps", "invalid_streak",
                                         "nmoves", "last_action", "done")]


MZ_STEP_COUNT_ZEROED = 1
MZ_STEP_AUTORESET = 2
MZ_RNG_PHILOX, MZ_RNG_CPYTHON = 0, 1
MZ_ERRORS = {-1: ValueError, -2: ValueError, -3: RuntimeError, -4: MemoryError, -5: ValueError}

EXPORTS = ["mz_last_error", "mz_device_count", "mz_create", "mz_destroy", "mz_load_mazes",
           "mz_generate", "mz_generate_ex", "mz_generate_state", "mz_reset_all", "mz_reset_list", "mz_reset_done", "mz_step", "mz_step_ex", "mz_direction_mask",
           "mz_act", "mz_step_act", "mz_expand_window", "mz_set_algorithm", "mz_query", "mz_get_grid",
           "mz_difficulty", "mz_maze_complexity", "mz_maze_metrics", "mz_difficulty_batch", "mz_get_meta", "mz_discounted_returns", "mz_q_front",
           "mz_bank_create", "mz_bank_create_dims", "mz_bank_create_ex", "mz_bank_fill", "mz_bank_use",
           "mz_bank_slot_grid", "mz_generate_best", "mz_select_stats", "mz_select_stats_ex",
           "mz_set_debug", "mz_screen_batch", "mz_set_regen_dims",
           "mz_bank_consumed", "mz_state_bytes", "mz_state_save", "mz_state_load",
           "mz_stem_forward", "mz_stem_backward", "mz_stem_backward_ex", "mz_stem_workspace_floats", "mz_adamw_flat",
           "mz_pair_surrogate", "mz_leaky_relu_bf16", "mz_colsum_f32",
           "mz_replay_gather", "mz_host_alloc", "mz_host_free", "mz_q_front_rows", "mz_greedy_rows",
           "mz_trainer_tick", "mz_greedy_scatter", "mz_head_bf16", "mz_replay_push",
           "mz_replay_sample_idx", "mz_q_loss", "mz_q_loss_backward", "mz_head_loss",
           "mz_head_loss_backward", "mz_head_loss_workspace_floats",
           "mz_head_loss_backward_workspace_floats", "mz_adamw_groups",
           "mz_ppo_act", "mz_ppo_scan", "mz_ppo_finish", "mz_ppo_head_loss", "mz_qact_prepare", "mz_qact",
           "mz_qact_workspace_floats"]

_lib = None


def lib_path():
    return _build.LIB


def load(build_if_missing=True):
    """Load libmazerl.so (building it with hipcc if absent and allowed)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("MZ_LIB_OVERRIDE") or _build.LIB  # an alternative build (experiments)
    if not os.path.exists(path):
        if not build_if_missing:
            raise RuntimeError(f"libmazerl.so not built ({path}); run mazerl._build.build()")
        _build.build()
    L = C.CDLL(path)
    vp = C.c_void_p
    L.mz_last_error.restype = C.c_char_p
    L.mz_device_count.argtypes = [c_i32p]
    L.mz_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
    L.mz_destroy.argtypes = [vp]
    L.mz_load_mazes.argtypes = [vp, vp, C.c_int32, vp, vp, C.c_int32, vp]
    L.mz_generate.argtypes = [vp, vp, C.c_int32, vp, C.c_int32, C.c_int32, C.c_uint64, vp]
    L.mz_generate_ex.argtypes = [vp, vp, C.c_int32, vp, C.c_int32, C.c_int32, C.c_uint64,
                                 C.c_int32, vp]
    L.mz_generate_state.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, vp]
    L.mz_reset_all.argtypes = [vp, C.POINTER(StepOut), vp]
    L.mz_reset_list.argtypes = [vp, vp, vp, C.c_int32, C.c_int32, C.c_uint64, C.c_uint32,
                                C.POINTER(StepOut), vp]
    L.mz_reset_done.argtypes = [vp, C.c_int32, C.c_uint64, C.c_uint32, C.POINTER(StepOut), vp]
    L.mz_step.argtypes = [vp, vp, C.POINTER(StepOut), vp]
    L.mz_step_ex.argtypes = [vp, vp, C.POINTER(StepOut), C.c_int32, vp]
    L.mz_direction_mask.argtypes = [vp, C.c_int32, vp, vp]
    L.mz_act.argtypes = [vp, vp, C.c_float, vp, C.c_uint64, C.c_uint64, vp, vp]
    L.mz_step_act.argtypes = [vp, vp, C.c_float, vp, C.c_uint64, C.c_uint64, vp,
                              C.POINTER(StepOut), C.c_int32, vp]
    L.mz_expand_window.argtypes = [vp, vp, C.c_int32, vp]
    L.mz_set_algorithm.argtypes = [vp, vp, C.c_int32, vp]
    L.mz_query.argtypes = [vp, C.c_int32, C.POINTER(EnvInfo)]
    L.mz_get_grid.argtypes = [vp, C.c_int32, vp]
    L.mz_get_meta.argtypes = [vp, vp, vp]
    L.mz_discounted_returns.argtypes = [vp, C.c_int32, vp, vp, C.c_int32, C.c_double, vp,
                                        C.c_int32, vp]
    L.mz_difficulty.argtypes = [vp] + [C.c_int32] * 6 + [C.POINTER(C.c_double)]
    L.mz_maze_complexity.argtypes = [vp] + [C.c_int32] * 6 + [C.POINTER(C.c_double)] * 2
    L.mz_maze_metrics.argtypes = [vp, vp, C.c_int32, vp, vp]
    L.mz_difficulty_batch.argtypes = [vp, vp, C.c_int32, vp, vp, vp]
    L.mz_bank_create.argtypes = [vp, C.c_int32, C.c_int32, C.c_uint32]
    L.mz_bank_create_dims.argtypes = [vp, C.c_int32, vp, C.c_int32, C.c_uint32]
    L.mz_bank_create_ex.argtypes = [vp, C.c_int32, vp, C.c_int32, C.c_uint32, C.c_int32]
    L.mz_bank_fill.argtypes = [vp, C.c_int32, C.c_uint64, vp]
    L.mz_bank_slot_grid.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, vp]
    L.mz_generate_best.argtypes = [vp, vp, C.c_int32, vp, C.c_int32, C.c_int32, C.c_uint64,
                                   C.c_int32, vp]
    L.mz_select_stats.argtypes = [vp, vp, C.c_int32, vp]
    if hasattr(L, "mz_select_stats_ex") or not os.environ.get("MZ_LIB_OVERRIDE"):
        # (an MZ_LIB_OVERRIDE build of an earlier round lacks these: A/B timing runs)
        L.mz_select_stats_ex.argtypes = [vp, vp, C.c_int32, C.c_int32, vp]
        L.mz_set_debug.argtypes = [vp, C.c_int32]
        L.mz_screen_batch.argtypes = [vp, vp, C.c_int32, vp, vp, vp]
    L.mz_set_regen_dims.argtypes = [vp, vp]
    L.mz_bank_use.argtypes = [vp, C.c_int32]
    L.mz_bank_consumed.argtypes = [vp, C.c_int32, vp, vp]
    L.mz_state_bytes.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.mz_state_save.argtypes = [vp, vp, C.c_uint64, vp]
    L.mz_state_load.argtypes = [vp, vp, C.c_uint64, vp]
    L.mz_q_front.argtypes = [vp, vp, C.c_int32, vp, vp, C.c_float, C.c_uint64, C.c_uint64, vp,
                             C.c_int32, vp]
    L.mz_q_front_rows.argtypes = [vp, vp, vp, vp, C.c_int32, vp, vp, C.c_float, C.c_uint64,
                                  C.c_uint64, vp, C.c_int32, vp]
    L.mz_greedy_rows.argtypes = [vp, C.c_float, C.c_uint64, C.c_uint64, C.c_int32, vp, vp, vp, vp,
                                 vp]
    L.mz_trainer_tick.argtypes = [vp, vp, vp, C.c_double, C.c_double, C.c_double, vp, vp, vp,
                                  C.c_uint64, C.c_uint64, C.c_int32, vp, vp, vp, vp]
    L.mz_greedy_scatter.argtypes = [vp, C.c_int32, vp, vp, C.c_int32, vp, vp]
    L.mz_head_bf16.argtypes = [vp] * 6 + [C.c_int32] * 9 + [vp] * 7
    L.mz_replay_push.argtypes = [C.c_int32, C.c_int64, C.c_int64] + [vp] * 12 + [C.c_int32,
                                                                                 C.c_int32, vp]
    L.mz_replay_sample_idx.argtypes = [C.c_uint64, C.c_uint64, C.c_int64, C.c_int64, C.c_int64,
                                       vp, C.c_int32, vp]
    L.mz_q_loss.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, C.c_int32, vp, vp, C.c_double,
                            C.c_int32, vp, vp, vp]
    L.mz_q_loss_backward.argtypes = [vp, vp, vp, C.c_int32, C.c_int32, vp, vp]
    L.mz_head_loss.argtypes = [vp, C.c_int32, vp, vp, vp, C.c_int32, vp, vp, C.c_int32, C.c_int32,
                               C.c_int32, vp, vp, C.c_double, C.c_int32, vp, vp, vp, vp, vp]
    L.mz_head_loss_backward.argtypes = [vp, vp, vp, C.c_int32, vp, C.c_int32, vp, C.c_int32,
                                        C.c_int32, vp, C.c_int32, vp, vp]
    L.mz_head_loss_workspace_floats.argtypes = [C.c_int32]
    L.mz_head_loss_backward_workspace_floats.argtypes = [C.c_int32, C.c_int32]
    L.mz_stem_forward.argtypes = [vp, vp, C.c_int32, vp, vp, C.c_float, vp, C.c_uint32, vp,
                                  C.c_int32, vp, vp]
    L.mz_stem_backward.argtypes = [vp, vp, vp, C.c_int32, C.c_int32, C.c_float, vp, vp, vp, vp]
    if hasattr(L, "mz_stem_backward_ex"):
        L.mz_stem_backward_ex.argtypes = [vp, vp, vp, C.c_int32, C.c_int32, C.c_float, vp, vp, vp,
                                          vp, vp]
    L.mz_stem_workspace_floats.argtypes = [C.c_int32]
    L.mz_qact_workspace_floats.argtypes = [C.c_int32]
    L.mz_leaky_relu_bf16.argtypes = [vp, C.c_int64, C.c_float, vp]
    L.mz_colsum_f32.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, vp]
    L.mz_replay_gather.argtypes = [vp, C.c_int32, C.c_int64] + [vp] * 11
    L.mz_pair_surrogate.argtypes = [vp, vp, vp, C.c_int32, C.c_float, vp, vp, vp]
    L.mz_adamw_flat.argtypes = [vp, vp, vp, vp, vp, C.c_int32, vp, vp, C.c_double, C.c_double,
                                C.c_double, C.c_double, C.c_float, C.c_float, C.c_int32, vp]
    L.mz_adamw_groups.argtypes = [vp, vp, vp, vp, vp, vp, C.c_int32, vp, vp, C.c_double,
                                  C.c_double, C.c_double, C.c_double, C.c_float, vp, vp]
    L.mz_ppo_act.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, vp, C.c_int32, C.c_int32,
                             C.c_uint64, C.c_uint64] + [vp] * 8
    L.mz_ppo_scan.argtypes = [vp, vp, vp, C.c_int32, C.c_int32] + [vp] * 10
    L.mz_ppo_head_loss.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp, vp, C.c_int32,
                                   C.c_float, vp, vp, vp, C.c_int32, vp, C.c_int32, vp]
    L.mz_ppo_finish.argtypes = [vp] * 6 + [C.c_int32, C.c_int32] + [vp] * 4 + \
        [C.c_double, C.c_int64] + [vp] * 7
    L.mz_qact_prepare.argtypes = [vp] * 7
    L.mz_qact.argtypes = [vp, vp, vp, vp, C.c_int32] + [vp] * 10 + [C.c_int32, C.c_float,
                                                                   C.c_uint64, C.c_uint64] + [vp] * 4
    L.mz_host_alloc.argtypes = [C.c_uint64, C.c_int32, C.POINTER(vp), C.POINTER(vp)]
    L.mz_host_free.argtypes = [vp]
    for f in EXPORTS:
        if f != "mz_last_error" and (hasattr(L, f) or not os.environ.get("MZ_LIB_OVERRIDE")):
            getattr(L, f).restype = C.c_int
    L.mz_qact_workspace_floats.restype = C.c_int64
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = load().mz_last_error().decode(errors="replace")
        raise MZ_ERRORS.get(rc, RuntimeError)(f"libmazerl error {rc}: {msg}")
    return rc
