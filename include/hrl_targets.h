/*
 * hrl_targets.h — C ABI of the MI355X return-target scans (libhrl.so).
 *
 * Replaces the reference operator
 *     handyrl.losses.compute_target(algorithm, values, returns, rewards,
 *                                   lmb, gamma, rhos, cs)
 * (reference: handyrl/losses.py:61-74, with the recurrences at
 *  losses.py:16-17 monte_carlo, :20-28 temporal_difference, :31-40 upgo,
 *  :43-58 vtrace) and its two/four call sites in compute_loss
 * (handyrl/train.py:245-253).
 *
 * Conventions (all pointers are DEVICE pointers, fp32, C-contiguous):
 *   values   (B, T, C)       C = P*K value columns (P players x K value dims)
 *   returns  (B, ret_T, C)   ret_T in {1, T}; TD/UPGO/VTRACE read only the
 *                            last time step (the bootstrap), MC reads all
 *   rewards  (B, T, C)       may be NULL  (reference: rewards=None -> 0)
 *   rhos, cs (B, T, rho_C)   rho_C in {1, P}; value column c reads rho column
 *                            c / rho_div  (rho_div = K when rho_C == P,
 *                            rho_div = C when rho_C == 1: broadcast)
 *   lmb, gamma               passed as double; the kernels use the same float
 *                            coefficients the reference's Python-scalar x
 *                            float32-tensor arithmetic uses: (float)(1-lmb),
 *                            (float)lmb, (float)gamma, (float)(gamma*lmb)
 * Outputs (caller-allocated, (B, T, C)):
 *   targets  may be NULL (MC's target is `returns` itself, losses.py:17)
 *   advantages
 *
 * Every entry point is asynchronous on `stream` (a hipStream_t; pass torch's
 * current stream), allocates nothing, never synchronises and reads nothing
 * back to the host, so it may be captured into a hipGraph.
 * Return value: 0 on success, HRL_EINVAL for a bad algorithm / shape /
 * pointer, HRL_ELAUNCH_BASE - hipError_t for a launch failure.
 */
#ifndef HRL_TARGETS_H
#define HRL_TARGETS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    HRL_ALG_MC = 0,      /* losses.py:16  */
    HRL_ALG_TD = 1,      /* losses.py:20  */
    HRL_ALG_UPGO = 2,    /* losses.py:31  */
    HRL_ALG_VTRACE = 3,  /* losses.py:43  */
};

#define HRL_OK 0
#define HRL_EINVAL (-22)
#define HRL_ELAUNCH_BASE (-1000)

/* ABI version, bumped on any signature change. */
int hrl_abi_version(void);

/* Human-readable text for a return code (static storage). */
const char *hrl_strerror(int code);

/* Kernel form of the scans for T <= 16: 2 one lane per (trajectory, column) straight from global memory (no
 * LDS), 0 the chunked LDS-transpose kernel every T uses, 1 (the default) the first for small batches
 * (B*C <= 32768) and the second otherwise.  Results are bit-identical.  Process-wide; returns the previous
 * setting. */
int hrl_targets_set_short_form(int form);

/*
 * One algorithm, one head: the drop-in for a single compute_target call
 * (losses.py:61).  targets may be NULL; for MC it must be NULL.
 */
int hrl_compute_target(int alg,
                       const float *values, const float *returns, const float *rewards,
                       const float *rhos, const float *cs,
                       int64_t B, int64_t T, int64_t C, int64_t ret_T,
                       int64_t rho_C, int64_t rho_div,
                       double lmb, double gamma,
                       float *targets, float *advantages,
                       void *stream);

/*
 * Fused learner form of train.py:248-253 for one head: ONE pass over the
 * inputs produces the value-target of `target_alg` (args['value_target'])
 * and the advantages of `adv_alg` (args['policy_target']; the reference
 * discards value_target's advantages when the two differ, train.py:251-253).
 * targets may be NULL (and must be for target_alg == MC).
 */
int hrl_compute_targets_fused(int target_alg, int adv_alg,
                              const float *values, const float *returns, const float *rewards,
                              const float *rhos, const float *cs,
                              int64_t B, int64_t T, int64_t C, int64_t ret_T,
                              int64_t rho_C, int64_t rho_div,
                              double lmb, double gamma,
                              float *targets, float *advantages,
                              void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HRL_TARGETS_H */
