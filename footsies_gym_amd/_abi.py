"""ctypes mirror of ``include/footsies.h`` (the libfootsies.so C-ABI).

Only plain ABI types live here: the structs, constants and the move tables the
Python side needs.  Kept in one place so the product binding (``_lib.py``) and
the test-side oracle binding (``oracle/binding.py``) agree on layouts.
"""
import ctypes as C

FS_ABI_VERSION = 7

FS_OK = 0
FS_E_INVALID = -1
FS_E_DEVICE = -2
FS_E_UNSUPPORTED = -3
FS_E_OOM = -4
FS_E_RUNTIME = -5

FS_P2_EXTERNAL = 0
FS_P2_BOT = 1
FS_P2_NOOP = 2

FS_P1_EXTERNAL = 0
FS_P1_BOT = 1

FS_FLOAT_STRICT32 = 0
FS_FLOAT_DOUBLE = 1

FS_AUTORESET_SAME_STEP = 0
FS_AUTORESET_NEXT_STEP = 1

FS_ACT_HOST = 0
FS_ACT_DEVICE = 1

FS_STREAM_OWN = C.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF)

FS_RESET_HARD = 0
FS_RESET_IF_NEEDED = 1
FS_RESET_SEED_ONLY = 2
FS_MAX_FRAME_DELAY = 4096
FS_RECORD_BYTES = 40
FS_KERNEL_HASHED = 1
FS_KERNEL_POLICY = 2
FS_KERNEL_PACKED = 4
FS_PACKED_LANE_BYTES = 16
FS_PPO_ACTOR_PARAMS = 5256
FS_PPO_CRITIC_PARAMS = 4801
FS_PPO_FP32 = 0
FS_PPO_SPLIT_BF16 = 1

# InputDefine (Assets/Script/InputData.cs:8-14)
IN_LEFT, IN_RIGHT, IN_ATTACK = 1, 2, 4

# FootsiesMove (footsies-gym/footsies_gym/moves.py:12-29): (name, actionID, duration)
MOVES = (
    ("STAND", 0, 24), ("FORWARD", 1, 24), ("BACKWARD", 2, 24), ("DASH_FORWARD", 10, 16),
    ("DASH_BACKWARD", 11, 22), ("N_ATTACK", 100, 22), ("B_ATTACK", 105, 21), ("N_SPECIAL", 110, 44),
    ("B_SPECIAL", 115, 55), ("DAMAGE", 200, 17), ("GUARD_M", 301, 23), ("GUARD_STAND", 305, 15),
    ("GUARD_CROUCH", 306, 15), ("GUARD_BREAK", 310, 36), ("GUARD_PROXIMITY", 350, 1), ("DEAD", 500, 500),
    ("WIN", 510, 33),
)
MOVE_ID_TO_INDEX = {mid: i for i, (_, mid, _) in enumerate(MOVES)}  # moves.py:41-42
MOVE_INDEX_TO_ID = tuple(mid for _, mid, _ in MOVES)


class fs_config(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("device_id", C.c_int32), ("p2_mode", C.c_int32),
        ("dense_reward", C.c_int32), ("frame_delay", C.c_int32), ("float_mode", C.c_int32),
        ("autoreset_mode", C.c_int32), ("p1_mode", C.c_int32), ("base_seed", C.c_uint64),
        ("arena_base", C.c_uint64),
    ]


_OUT_FIELDS = [
    ("guard", C.c_void_p), ("move", C.c_void_p), ("move_frame", C.c_void_p), ("position", C.c_void_p),
    ("reward", C.c_void_p), ("terminated", C.c_void_p), ("truncated", C.c_void_p), ("frame", C.c_void_p),
    ("action", C.c_void_p), ("hitstun", C.c_void_p),
    ("final_guard", C.c_void_p), ("final_move", C.c_void_p), ("final_move_frame", C.c_void_p),
    ("final_position", C.c_void_p), ("final_frame", C.c_void_p), ("final_action", C.c_void_p),
    ("final_hitstun", C.c_void_p),
]


class fs_outputs(C.Structure):
    _fields_ = _OUT_FIELDS


# name -> (numpy dtype string, columns per arena)
OUTPUT_SPEC = {
    "guard": ("u1", 2), "move": ("u1", 2), "move_frame": ("f4", 2), "position": ("f4", 2),
    "reward": ("f8", 1), "terminated": ("u1", 1), "truncated": ("u1", 1), "frame": ("i4", 1),
    "action": ("u1", 2), "hitstun": ("u1", 2),
    "final_guard": ("u1", 2), "final_move": ("u1", 2), "final_move_frame": ("f4", 2),
    "final_position": ("f4", 2), "final_frame": ("i4", 1), "final_action": ("u1", 2),
    "final_hitstun": ("u1", 2),
}


class fs_host_arrays(C.Structure):
    _fields_ = [(name, C.c_void_p) for name in (
        "guard", "move", "move_frame", "position", "info_guard", "info_move", "info_move_frame", "info_position",
        "frame", "p1_action", "p2_action", "p1_hitstun", "p2_hitstun", "reward", "terminated", "truncated")]


class fs_packed_traj(C.Structure):
    _fields_ = [("lanes", C.c_void_p), ("reward", C.c_void_p), ("final_lanes", C.c_void_p)]


class fs_policy(C.Structure):
    _fields_ = [
        ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p), ("b2", C.c_void_p), ("w3", C.c_void_p),
        ("b3", C.c_void_p), ("seed", C.c_uint64), ("actions_out", C.c_void_p), ("logp_out", C.c_void_p),
    ]


class fs_mlp(C.Structure):
    _fields_ = [("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p), ("b2", C.c_void_p), ("w3", C.c_void_p),
                ("b3", C.c_void_p)]


class fs_env_state(C.Structure):
    _fields_ = [
        ("p1Vital", C.c_int32), ("p2Vital", C.c_int32), ("p1Guard", C.c_int32), ("p2Guard", C.c_int32),
        ("p1Move", C.c_int32), ("p1MoveFrame", C.c_int32), ("p2Move", C.c_int32), ("p2MoveFrame", C.c_int32),
        ("p1Position", C.c_float), ("p2Position", C.c_float), ("globalFrame", C.c_int32),
        ("p1MostRecentAction", C.c_int32), ("p2MostRecentAction", C.c_int32),
        ("p1Hitstun", C.c_int32), ("p2Hitstun", C.c_int32),
    ]


class fs_fighter_state(C.Structure):
    _fields_ = [
        ("position_x", C.c_float), ("action_id", C.c_int32), ("action_frame", C.c_int32),
        ("hit_count", C.c_int32), ("hitstun", C.c_int32), ("vital", C.c_int32), ("guard", C.c_int32),
        ("buffer_action_id", C.c_int32), ("reserve_action_id", C.c_int32),
        ("input_dir_history", C.c_uint32), ("attack_hold", C.c_int32),
        ("is_input_backward", C.c_uint8), ("is_reserve_proximity_guard", C.c_uint8),
        ("has_won", C.c_uint8), ("facing_flipped", C.c_uint8), ("position_y", C.c_float),
    ]


class fs_arena_state(C.Structure):
    _fields_ = [
        ("f", fs_fighter_state * 2), ("frame_count", C.c_int32), ("recording_count", C.c_int32),
        ("recording_last", C.c_uint8 * 2), ("actor_input", C.c_uint8 * 2), ("reset_pending", C.c_uint8),
        ("has_terminated", C.c_uint8), ("pad0", C.c_uint8 * 2), ("cumulative_reward", C.c_double),
        ("rng", C.c_uint32 * 4), ("move_plan", C.c_int32), ("move_index", C.c_int32),
        ("attack_plan", C.c_int32), ("attack_index", C.c_int32), ("prev_distance", C.c_float),
        ("prev_opponent_action", C.c_int32),
        ("p2_bot", C.c_uint8), ("bot_ready", C.c_uint8 * 2), ("bot_input", C.c_uint8 * 2), ("pad1", C.c_uint8 * 3),
        ("p1_move_plan", C.c_int32), ("p1_move_index", C.c_int32), ("p1_attack_plan", C.c_int32),
        ("p1_attack_index", C.c_int32), ("p1_prev_distance", C.c_float), ("p1_prev_opponent_action", C.c_int32),
    ]


# functions exported by libfootsies.so: name -> (restype, argtypes)
LIB_FUNCTIONS = {
    "fs_abi_version": (C.c_int, []),
    "fs_runtime_images": (C.c_int, [C.c_char_p, C.c_size_t]),
    "fs_host_alloc": (C.c_int, [C.c_int, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "fs_host_free": (C.c_int, [C.c_void_p]),
    "fs_memcpy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "fs_runtime_version": (C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "fs_create": (C.c_int, [C.POINTER(fs_config), C.POINTER(C.c_void_p)]),
    "fs_reset": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "fs_set_p2_mode": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "fs_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "fs_step_masked": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "fs_step_n": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(fs_outputs)]),
    "fs_step_n_packed": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(fs_packed_traj)]),
    "fs_step_n_policy": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(fs_policy), C.c_void_p, C.POINTER(fs_outputs)]),
    "fs_ppo_workspace_bytes": (C.c_size_t, []),
    "fs_ppo_eval": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(fs_mlp), C.POINTER(fs_mlp),
                              C.c_void_p, C.c_void_p, C.c_void_p]),
    "fs_ppo_grad": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(fs_mlp), C.POINTER(fs_mlp), C.c_float, C.c_float,
                              C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "fs_ppo_grad_ex": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(fs_mlp), C.POINTER(fs_mlp), C.c_float, C.c_float,
                                 C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]),
    "fs_ppo_grad_runs": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int, C.POINTER(fs_mlp),
                                   C.POINTER(fs_mlp), C.c_float, C.c_float, C.c_float, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]),
    "fs_ppo_eval_ex": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(fs_mlp), C.POINTER(fs_mlp),
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]),
    "fs_ppo_gae": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_float,
                             C.c_void_p, C.c_void_p, C.c_void_p]),
    "fs_ppo_features": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]),
    "fs_ppo_pack": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                              C.c_void_p, C.c_void_p]),
    "fs_hash_actions": (C.c_int, [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]),
    "fs_outputs_get": (C.c_int, [C.c_void_p, C.POINTER(fs_outputs)]),
    "fs_pack_outputs": (C.c_int, [C.c_void_p, C.c_void_p]),
    "fs_step_rec": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "fs_bind_outputs": (C.c_int, [C.c_void_p, C.POINTER(fs_outputs)]),
    "fs_get_env_state": (C.c_int, [C.c_void_p, C.POINTER(fs_env_state)]),
    "fs_get_state": (C.c_int, [C.c_void_p, C.POINTER(fs_arena_state)]),
    "fs_set_state": (C.c_int, [C.c_void_p, C.POINTER(fs_arena_state)]),
    "fs_sync": (C.c_int, [C.c_void_p]),
    "fs_stream": (C.c_void_p, [C.c_void_p]),
    "fs_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "fs_num_envs": (C.c_int, [C.c_void_p]),
    "fs_steps_taken": (C.c_uint64, [C.c_void_p]),
    "fs_step_kernel": (C.c_char_p, [C.c_void_p, C.c_int, C.c_int]),
    "fs_host_convert": (C.c_int, [C.POINTER(fs_outputs), C.c_int64, C.c_void_p, C.c_int64, C.POINTER(fs_host_arrays),
                                  C.c_int]),
    "fs_host_convert_start": (C.c_int, [C.POINTER(fs_outputs), C.c_int64, C.c_void_p, C.c_int64,
                                        C.POINTER(fs_host_arrays), C.c_int]),
    "fs_host_convert_wait": (C.c_int, []),
    "fs_destroy": (None, [C.c_void_p]),
    "fs_last_error": (C.c_char_p, [C.c_void_p]),
}


def structs_to_numpy(arr, n):
    """View a ctypes struct array as a numpy structured array (no copy)."""
    import numpy as np
    return np.ctypeslib.as_array(arr, shape=(n,))
