/*
 * hrl_env.h — C ABI of the batched Geister rules and of the self-play ply tail (libhrl.so).
 *
 * Replaces the per-game rules of handyrl/envs/geister.py (Environment.legal_actions :460-487,
 * Environment.observation :495-535, Environment.play :359-394), which generation.py:20-88 calls
 * once per ply per worker process, by three launches over E games held in HBM in the layout of
 * handyrl_amd.envs.geister.GeisterBatch:
 *   board (E,36) int8: -1 empty, colour*2 + type (0 blue, 1 red), absolute cell x*6 + y;
 *   color, turn_count, win (E,) int64; cnt (E,4) int64 pieces per (colour, type).
 * Action labels are the reference's: 0..143 = direction*36 + cell in the mover's frame (white's
 * frame is the board rotated 180 degrees), 144 + k = initial layout k of combinations(range(8), 4).
 * All pointers are device pointers; bool tensors are one byte per element.  Asynchronous on
 * `stream`, no allocation, no synchronisation (graph-capturable).
 * Returns 0, HRL_EINVAL or HRL_ELAUNCH_BASE - hipError_t (hrl_targets.h).
 */
#ifndef HRL_ENV_H
#define HRL_ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* legal (E, 214) bytes: 1 where the side to move may play the label (geister.py:460-487). */
int hrl_geister_legal(const int8_t *board, const int64_t *color, const int64_t *turn_count, int64_t E,
                      uint8_t *legal, void *stream);

/* The view of `player` (E,): planes (E,7,6,6) fp32 [ones, own, opponent, own blue, own red, opponent
 * blue, opponent red] rotated for white, scalar (E,18) fp32 [me is black, turn view, one-hot 1..4 of
 * the four piece counts]; `full` != 0 shows the opponent's colours (observation(None), CIGeister)
 * (geister.py:495-535). */
int hrl_geister_observation(const int8_t *board, const int64_t *color, const int64_t *cnt, const int64_t *player,
                            int64_t E, int full, float *planes, float *scalar, void *stream);

/* hrl_geister_observation that also records the view for DeviceGenerator's episode: slot t (read from
 * device memory) of rec_planes (E,Tm,7,6,6) / rec_scalar (E,Tm,18) gets the view where active[e], zeros
 * elsewhere (the record of generation.py:55-62 with its reset value for finished games); rec_planes NULL:
 * no record. */
int hrl_geister_observation_record(const int8_t *board, const int64_t *color, const int64_t *cnt,
                                   const int64_t *player, int64_t E, int full, float *planes, float *scalar,
                                   const uint8_t *active, const int64_t *t, int64_t Tm, float *rec_planes,
                                   float *rec_scalar, void *stream);

/* Play action (E,) in every game whose active byte is set (geister.py:359-394): layouts, moves,
 * captures, escapes, piece counts, winner, the 200-move draw; the side to move flips.
 * layout_type (70,8) int8 piece type per initial slot, opos (2,8) int64 initial cells per colour.
 * live (E,) bytes or NULL: set to (win < 0) for every played game (the next ply's active mask; may be
 * the same array as `active`). */
int hrl_geister_step(int8_t *board, int64_t *color, int64_t *turn_count, int64_t *win, int64_t *cnt,
                     const int64_t *action, const uint8_t *active, const int8_t *layout_type, const int64_t *opos,
                     int64_t E, uint8_t *live, void *stream);

/* The sampling and recording tail of a self-play ply (generation.py:43-62), one wave per game:
 * m = legal ? 0 : 1e32, p = logits - m, action = argmax(p - log(-log(U[t]))) (torch.argmax's tie order);
 * slot t (read from device memory) of policy_buf / amask_buf (E,Tm,A), action_buf / value_buf / turn_buf
 * (E,Tm) and reward_buf (E,Tm,P) fp64 gets the game's p, m, action, value, player, reward when `active`,
 * else 0, 1e32, 0, 0, 0, 0.  logits (E, >=A) rows of stride logit_stride; U (Tm,E,A) uniforms in (0,1];
 * reward / reward_buf both NULL when the env has no per-ply reward.  action (E,) gets the sample. */
int hrl_selfplay_sample_record(const float *logits, int64_t logit_stride, const uint8_t *legal, const float *U,
                               const int64_t *t, const float *value, const uint8_t *active, const int64_t *player,
                               const double *reward, int64_t E, int64_t A, int64_t Tm, int64_t P, int64_t *action,
                               float *policy_buf, float *amask_buf, int64_t *action_buf, float *value_buf,
                               int64_t *turn_buf, double *reward_buf, void *stream);

/* Masked row copy for the movers' recurrent state (generation.py:38-41: only the mover's hidden state
 * advances): for each of nleaves (<= 16) fp32 tensors, row e of dst[l] (E rows of F[l] contiguous floats,
 * row stride dst_stride[l] elements) becomes row e of src[l] where mask[e] != 0; other rows are untouched.
 * One launch for every state tensor, exactly torch.where(mask, src, dst). */
int hrl_masked_rows_copy(int nleaves, float *const *dst, const int64_t *dst_stride, const float *const *src,
                         const int64_t *src_stride, const int64_t *F, const uint8_t *mask, int64_t E, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HRL_ENV_H */
