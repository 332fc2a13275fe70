/*
 * hrl_loss.h — C ABI of the fused learner loss (libhrl.so).
 *
 * Replaces, for one learner step, the body of compute_loss after the network
 * forward (handyrl/train.py:220-258) and compose_losses (train.py:188-215):
 *   importance ratios      log_softmax+gather of behaviour/target policies,
 *                          rho = exp(lt - lb), clipped_rhos = cs = clamp(rho,0,1)
 *   value preparation      zero-sum symmetrisation (2-player turn-based) and
 *                          outcome padding  v*emask + outcome*(1-emask)
 *   return targets         the fused scans of hrl_targets.h, value and return head
 *   policy advantages      clipped_rhos * (adv_value + adv_return), summed over
 *                          players under turn_mask
 *   losses                 p, v, r, ent and total as SUMS (train.py:202-213),
 *                          plus dcnt = sum(turn_mask)
 * and its backward: closed-form gradients w.r.t. the target policy logits,
 * the value head and the return head for any upstream gradients of the five
 * losses (the targets and advantages are detached, as in the reference).
 *
 * Layout (fp32 unless noted, C-contiguous, device pointers):
 *   tpol, bpol (B,T,Pp,A)   target (network) / behaviour logits, already masked
 *   action     (B,T,Pp) int64
 *   emask      (B,T)        tmask, omask (B,T,P)     progress (B,T)
 *   value      (B,T,P) or NULL     outcome (B,P)
 *   ret_out    (B,T,P) or NULL     ret (B,T,P)   reward (B,T,P)
 *   Pp == 1 or Pp == P (policy-side player slots; SURVEY §8 notation)
 * Sums accumulate in fp64 and reduce in a fixed order (deterministic).
 * workspace: caller-allocated, hrl_loss_workspace_bytes() bytes, kept
 * between forward and backward of the same step.
 * losses (device, 6 floats): p, v, r, ent, total, dcnt.
 * dlosses (device, 5 floats): upstream gradients of p, v, r, ent, total.
 * Returns 0, HRL_EINVAL or HRL_ELAUNCH_BASE - hipError_t (hrl_targets.h).
 */
#ifndef HRL_LOSS_H
#define HRL_LOSS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int64_t hrl_loss_workspace_bytes(int64_t B, int64_t T, int64_t P, int64_t Pp);

int hrl_loss_forward(const float *tpol, const float *bpol, const int64_t *action,
                     int64_t B, int64_t T, int64_t P, int64_t Pp, int64_t A,
                     const float *emask, const float *tmask, const float *omask, const float *progress,
                     const float *value, const float *outcome,
                     const float *ret_out, const float *ret, const float *reward,
                     int value_target, int policy_target, int symmetrize,
                     double lmb, double gamma, double ent_coef, double ent_decay,
                     void *workspace, int64_t workspace_bytes, float *losses, void *stream);

int hrl_loss_backward(const float *tpol, const int64_t *action,
                      int64_t B, int64_t T, int64_t P, int64_t Pp, int64_t A,
                      const float *emask, const float *tmask, const float *omask, const float *progress,
                      const float *value, const float *ret_out,
                      double ent_coef, double ent_decay,
                      const void *workspace, int64_t workspace_bytes, const float *dlosses,
                      float *g_tpol, float *g_value, float *g_ret, void *stream);

/*
 * forward_prediction's masking of a feed-forward net's outputs (handyrl/train.py:176-183), one launch each way:
 *   policy (BT, A)    = sum_p opol[bt, p|0, :] * tmask[bt, p] - amask[bt, :]   (opol (BT, Pq, A), amask (BT, 1, A))
 *   value  (BT, P)    = oval[bt, p|0] * omask[bt, p]                          (oval (BT, Pq, 1); NULL: no value head)
 * Pq = 1 or P; tmask, omask (BT, P).  The backward forms dL/dopol (BT, Pq, A) and dL/doval (BT, Pq) from
 * dL/dpolicy and dL/dvalue (gval NULL: no value head).  Float operations and sum order as torch's.
 */
int hrl_output_mask_forward(const float *opol, const float *oval, const float *tmask, const float *omask,
                            const float *amask, int64_t BT, int64_t P, int64_t Pq, int64_t A, float *pol,
                            float *val, void *stream);
int hrl_output_mask_backward(const float *gpol, const float *gval, const float *tmask, const float *omask,
                             int64_t BT, int64_t P, int64_t Pq, int64_t A, float *gopol, float *goval,
                             void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HRL_LOSS_H */
