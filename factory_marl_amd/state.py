"""Pack / unpack the per-arena state record of fm_get_state / fm_set_state (include/factorysim.h).

Record = float64 [qpos nq | qvel nv | qpos_stage nq | qvel_stage nv | qacc_warmstart nv | ctrl_target nu |
spawn_freq | conveyor_speed | play_time | last_grip_dist A | last_bucket_dist A | episode_return |
A x (ik last_ctrl 8 | move_start 3 | ik_actions 8 | pause_last 8)]
+ int32 [in_scene K | out_scene K | n_in n_out step_counter steps_since_spawn failure_counter
hidden_counter score0 score1 last_score0 last_score1 episode_length | A x (ik state counter target ignore[A])]
+ uint64 [PCG64 state_hi state_lo inc_hi inc_lo].
"""
import numpy as np


def sizes(A, K):
    nq, nv, nu = 1 + 7 * K + 9 * A, 1 + 6 * K + 9 * A, 1 + 8 * A
    nd = 2 * nq + 3 * nv + nu + 3 + 2 * A + 1 + 27 * A
    ni = 2 * K + 11 + (3 + A) * A
    return nq, nv, nu, nd, ni


def record_bytes(A, K):
    *_, nd, ni = sizes(A, K)
    return 8 * nd + 4 * ni + 32


def pack(A, K, dbl, ints, rng):
    nq, nv, nu, nd, ni = sizes(A, K)
    out = np.zeros(record_bytes(A, K), np.uint8)
    out[:8 * nd] = np.ascontiguousarray(dbl, dtype=np.float64).view(np.uint8)
    out[8 * nd:8 * nd + 4 * ni] = np.ascontiguousarray(ints, dtype=np.int32).view(np.uint8)
    out[8 * nd + 4 * ni:] = np.ascontiguousarray(rng, dtype=np.uint64).view(np.uint8)
    return out


def unpack(A, K, rec):
    nq, nv, nu, nd, ni = sizes(A, K)
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    dbl = rec[:8 * nd].view(np.float64).copy()
    ints = rec[8 * nd:8 * nd + 4 * ni].view(np.int32).copy()
    rng = rec[8 * nd + 4 * ni:].view(np.uint64).copy()
    return dbl, ints, rng


def fields(A, K, dbl):
    """named views of the float64 block"""
    nq, nv, nu, nd, ni = sizes(A, K)
    o = 0
    f = {}
    for name, n in [("qpos", nq), ("qvel", nv), ("qpos_stage", nq), ("qvel_stage", nv), ("qacc_warmstart", nv),
                    ("ctrl_target", nu), ("spawn_freq", 1), ("conveyor_speed", 1), ("play_time", 1),
                    ("last_grip_dist", A), ("last_bucket_dist", A), ("episode_return", 1), ("ik", 27 * A)]:
        f[name] = dbl[o:o + n]
        o += n
    return f
