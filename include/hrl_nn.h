/*
 * hrl_nn.h — C ABI of the MI355X kernels for the learner's network hot ops
 * (libhrl.so).
 *
 * Training-mode BatchNorm over (N, C, HW) NCHW activations, the op that
 * dominates the learner step of the board-game nets (TicTacToe
 * SimpleConv2dModel handyrl/envs/tictactoe.py:17-69, GeisterNet
 * handyrl/envs/geister.py:100-167, GeeseNet handyrl/envs/kaggle/
 * hungry_geese.py:23-57): their BatchNorm2d layers see N = B*T*P samples of a
 * tiny board (HW = 9 .. 77), a shape the vendor spatial BatchNorm handles at
 * ~3% of HBM bandwidth.  Replaces torch.nn.BatchNorm2d.forward/backward in
 * training mode (the reference calls it through nn.Module, train.py:380-383).
 *
 * Semantics follow torch.nn.functional.batch_norm(training=True):
 *   mean_c, var_c = biased statistics over (N, HW);  invstd = 1/sqrt(var+eps)
 *   y = x * alpha_c + beta_c,  alpha = invstd*weight, beta = bias - mean*alpha
 *   running_mean = (1-m)*running_mean + m*mean
 *   running_var  = (1-m)*running_var  + m*var*M/(M-1),  M = N*HW
 * Statistics accumulate in fp64; all reductions are in a fixed order
 * (deterministic).  All pointers are device pointers, fp32, contiguous;
 * weight/bias and running_* may be NULL.  Asynchronous on `stream`; no
 * allocation, no synchronisation (graph-capturable).
 * `workspace` is caller-allocated scratch of hrl_bn_workspace_bytes() bytes.
 * Returns 0, HRL_EINVAL or HRL_ELAUNCH_BASE - hipError_t (hrl_targets.h).
 */
#ifndef HRL_NN_H
#define HRL_NN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scratch bytes needed by hrl_bn_forward_train / hrl_bn_backward for this shape. */
int64_t hrl_bn_workspace_bytes(int64_t N, int64_t C, int64_t HW);

/* Training forward: y, save_mean, save_invstd (C floats each), running stats updated in place.
 * relu != 0 fuses the ReLU that follows the BatchNorm in the env nets
 * (F.relu(bn(conv(h))), tictactoe.py:62-65): y = relu(x*alpha + beta). */
int hrl_bn_forward_train(const float *x, int64_t N, int64_t C, int64_t HW,
                         const float *weight, const float *bias,
                         float *running_mean, float *running_var, double momentum, double eps, int relu,
                         float *y, float *save_mean, float *save_invstd,
                         void *workspace, int64_t workspace_bytes, void *stream);

/* Backward of the training forward: dx (may not alias dy), dweight/dbias (C floats, may be NULL).
 * With relu != 0 the ReLU mask is recomputed from x (no saved output needed);
 * bias is then required to rebuild the forward's per-channel shift. */
int hrl_bn_backward(const float *x, const float *dy, int64_t N, int64_t C, int64_t HW,
                    const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                    int relu, float *dx, float *dweight, float *dbias,
                    void *workspace, int64_t workspace_bytes, void *stream);

/* The forward in pieces, for producers that compute the statistics themselves
 * (hrl_conv3x3_forward_ex with stats): fold per-block partials part[nparts][C][2]
 * = (sum x, sum x^2) over `count` = N*HW values into save_mean / save_invstd,
 * the running statistics and the apply coefficients alpha = invstd*weight,
 * beta = bias - mean*alpha; and apply y = x*alpha + beta [relu]. */
int hrl_bn_finalize_stats(const double *part, int64_t nparts, int64_t C, int64_t count, const float *weight,
                          const float *bias, float *running_mean, float *running_var, double momentum, double eps,
                          float *save_mean, float *save_invstd, float *alpha, float *beta, void *stream);
int hrl_bn_apply(const float *x, int64_t N, int64_t C, int64_t HW, const float *alpha, const float *beta, int relu,
                 float *y, void *stream);
/* Eval-mode forward (inference, e.g. self-play): y = x*alpha + beta [relu] with
 * alpha = weight / sqrt(running_var + eps), beta = bias - running_mean*alpha
 * (the vendor inference BatchNorm takes ~0.5 ms on (2048, 32, 6, 6)).
 * coef: 2*C floats of scratch (alpha | beta). */
int hrl_bn_forward_eval(const float *x, int64_t N, int64_t C, int64_t HW, const float *weight, const float *bias,
                        const float *running_mean, const float *running_var, double eps, int relu, float *y,
                        float *coef, void *stream);
/* The backward in pieces: fold (sum g, sum g*(x-mean)) partials into dweight,
 * dbias and the apply coefficients kcoef, gmean (C floats each); then
 * dx = ((g - gmean) - (x - mean)*kcoef) * invstd * weight, g masked by the
 * recomputed ReLU when relu != 0 (hrl_bn_backward = reduce + these two). */
/* Grouped BatchNorm: rows [g*N/G, (g+1)*N/G) are group g (N % G == 0), with statistics of its own --
 * a recurrent net's per-time-step BatchNorm run over all T steps in one launch (rows time-major).
 * save_mean / save_invstd are (G, C); the running statistics advance once per group, in group order,
 * as G sequential hrl_bn_forward_train calls would; dweight / dbias are the groups' sums.
 * workspace: hrl_bn_workspace_bytes_grouped(N, C, HW, G). */
int64_t hrl_bn_workspace_bytes_grouped(int64_t N, int64_t C, int64_t HW, int64_t G);
int hrl_bn_forward_train_grouped(const float *x, int64_t N, int64_t C, int64_t HW, int64_t G, const float *weight,
                                 const float *bias, float *running_mean, float *running_var, double momentum,
                                 double eps, int relu, float *y, float *save_mean, float *save_invstd,
                                 void *workspace, int64_t workspace_bytes, void *stream);
int hrl_bn_backward_grouped(const float *x, const float *dy, int64_t N, int64_t C, int64_t HW, int64_t G,
                            const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                            int relu, float *dx, float *dweight, float *dbias, void *workspace,
                            int64_t workspace_bytes, void *stream);
int hrl_bn_finalize_backward(const double *part, int64_t nparts, int64_t C, int64_t count, const float *weight,
                             const float *save_invstd, float *dweight, float *dbias, float *kcoef, float *gmean,
                             void *stream);
int hrl_bn_backward_apply(const float *x, const float *dy, int64_t N, int64_t C, int64_t HW, const float *weight,
                          const float *bias, const float *save_mean, const float *save_invstd, int relu,
                          const float *kcoef, const float *gmean, float *dx, void *stream);

/* Residual blocks (GeeseNet, hungry_geese.py:50-51: h' = relu(h + bn(conv(h)))):
 * hrl_bn_apply_residual: y = relu(res + x*alpha + beta) (res NULL: relu(x*alpha + beta));
 * hrl_bn_backward_masked: the BatchNorm backward of such a block, the incoming gradient dy
 * (w.r.t. y) masked where out (= y) <= 0, i.e. dx = BNbwd(dy * [out > 0]); dweight/dbias may be NULL.
 * workspace: hrl_bn_workspace_bytes(N, C, HW). */
int hrl_bn_apply_residual(const float *x, const float *res, int64_t N, int64_t C, int64_t HW, const float *alpha,
                          const float *beta, float *y, void *stream);
int hrl_bn_backward_masked(const float *x, const float *dy, const float *out, int64_t N, int64_t C, int64_t HW,
                           const float *weight, const float *save_mean, const float *save_invstd, float *dx,
                           float *dweight, float *dbias, void *workspace, int64_t workspace_bytes, void *stream);
/* hrl_bn_backward_masked without its apply pass (round 5): the reduce and finalize only, the apply's per-channel
 * coefficients k and mean(dy [out > 0]) into kcoef / gmean (C floats each) for a consumer that applies them itself
 * (hrl_torus_conv_wgrad_bn).  workspace: hrl_bn_workspace_bytes(N, C, HW). */
int hrl_bn_backward_masked_coefs(const float *x, const float *dy, const float *out, int64_t N, int64_t C,
                                 int64_t HW, const float *weight, const float *save_mean, const float *save_invstd,
                                 float *kcoef, float *gmean, float *dweight, float *dbias, void *workspace,
                                 int64_t workspace_bytes, void *stream);
/* The apply half of hrl_bn_backward_masked with the coefficients of hrl_bn_finalize_backward
 * (sums from hrl_torus_unit_input_grad). */
int hrl_bn_backward_apply_masked(const float *x, const float *dy, const float *out, int64_t N, int64_t C, int64_t HW,
                                 const float *weight, const float *save_mean, const float *save_invstd,
                                 const float *kcoef, const float *gmean, float *dx, void *stream);

/*
 * Tiny-board convolution as one dense matrix (handyrl_amd/nn.py BoardConv2d):
 * W_board[(ci*H*W + p), (co*H*W + q)] = W[co, ci, dy, dx] where input cell p
 * is output cell q shifted by (dy - kh/2, dx - kw/2), zero off the board.
 * hrl_board_weight builds W_board (Cin*HW x Cout*HW); hrl_board_fold sums a
 * W_board-shaped gradient back onto W (deterministic, one thread per weight).
 * hrl_board_bias / hrl_board_bias_fold do the same for the bias: b_board[co*HW+q] = b[co].
 */
int hrl_board_weight(const float *w, int64_t Cout, int64_t Cin, int64_t kh, int64_t kw, int64_t H, int64_t W,
                     float *w_board, void *stream);
int hrl_board_fold(const float *g_board, int64_t Cout, int64_t Cin, int64_t kh, int64_t kw, int64_t H, int64_t W,
                   float *g_w, void *stream);
int hrl_board_bias(const float *b, int64_t Cout, int64_t HW, float *b_board, void *stream);
int hrl_board_bias_fold(const float *g_board, int64_t Cout, int64_t HW, float *g_b, void *stream);

/* out[c] = sum_r x[r, c] for a row-major (M, N) matrix, N <= 256 (bias gradients over
 * M = B*T*P rows); fp64 accumulation, fixed-order folds (deterministic). */
int64_t hrl_colsum_workspace_bytes(int64_t M, int64_t N);
int hrl_colsum(const float *x, int64_t M, int64_t N, float *out, void *workspace, int64_t workspace_bytes,
               void *stream);

/*
 * 3x3 'same' convolution of 32 -> 32 channels on a 3x3 board (TicTacToe body,
 * tictactoe.py:57-58) with fp32 MFMA, skipping the off-board taps
 * (csrc/hrl_conv.hip).  x, y: (M, 32*9) NCHW rows; weight (32, 32, 3, 3).
 * flip = 0: y = conv(x, W) + bias.  flip = 1: y = conv^T(x, W), the input
 * gradient of the forward (bias must be NULL).
 * hrl_conv3x3_wgrad: dweight (32, 32, 3, 3) = d conv / dW for input x and output gradient dy.
 * workspace: hrl_conv3x3_workspace_bytes(M) bytes.
 */
int64_t hrl_conv3x3_workspace_bytes(int64_t M);
int hrl_conv3x3_forward(const float *x, int64_t M, int64_t C_in, int64_t C_out, const float *weight,
                        const float *bias, int flip, float *y, void *workspace, int64_t workspace_bytes,
                        void *stream);
int hrl_conv3x3_wgrad(const float *x, const float *dy, int64_t M, int64_t C_in, int64_t C_out, float *dweight,
                      void *workspace, int64_t workspace_bytes, void *stream);

/*
 * The same kernels fused with the BatchNorm+ReLU around a conv -> BN -> ReLU
 * chain (conv3x3_kernel<PRO, EPI>, csrc/hrl_conv.hip):
 *   in_alpha / in_beta (32 floats, both or neither): x is the previous
 *     block's raw conv output; the kernel reads relu(x*in_alpha[c] + in_beta[c]);
 *   epilogue 0: none;
 *            1: forward statistics, part = per-workgroup fp64 (sum y, sum y^2)
 *               per output channel -> hrl_bn_finalize_stats;
 *            2: (input gradient of a chain) y is dL/d relu(ref*ep_alpha + ep_beta);
 *               part = (sum g, sum g*(ref - ep_mean)) with g = y masked where
 *               ref*ep_alpha + ep_beta <= 0 -> hrl_bn_finalize_backward;
 *            3: y *= [ref > 0] (backward of a ReLU on the chain input).
 *   part: hrl_conv3x3_stats_blocks(M) x 32 x 2 doubles; ref: (M, 288) like y.
 * hrl_conv3x3_forward / hrl_conv3x3_wgrad are these with nothing fused.
 */
int64_t hrl_conv3x3_stats_blocks(int64_t M);
/* Arithmetic of the forward / input-gradient kernel: on != 0 (the default) an exact three-way bf16 split of
 * both fp32 operands on v_mfma_f32_16x16x32_bf16 (six partial products, fp32 accumulation; error below one fp32
 * rounding per product), 0 the fp32 v_mfma_f32_16x16x4_f32.  Process-wide; returns the previous setting. */
int hrl_conv3x3_set_split(int on);
/* Kernel form of hrl_conv3x3_block_backward: 1 (the default) the 8-wave tile-shared, pipelined kernel (the next
 * tile staged in a second LDS buffer while the MFMAs run); 2 two independent 4-wave workgroups per CU, each
 * sharing a 16-row tile among its waves (single-buffered LDS images, ABI 25); 0 the per-wave kernel.
 * Forms 0 and 1 run the per-wave kernel without an input gradient.  The input gradient and the epilogue are the
 * same in all; the weight gradient sums the tiles in a different association per form.  Process-wide; returns
 * the previous setting. */
int hrl_conv3x3_set_block_form(int form);
/* Rows of epilogue-2 sums (32 x 2 doubles each) hrl_conv3x3_block_backward writes into `part` under the current
 * block form (ABI 25; form 2 writes more rows than hrl_conv3x3_stats_blocks). */
int64_t hrl_conv3x3_block_sum_blocks(int64_t M);
/* The chain's forward conv with BN statistics (hrl_conv3x3_forward_ex, epilogue 1, packed weights, no bias):
 * 2 (default) = the LDS-DMA ring form (every wave computes, x' staged from a raw ring), 3 = the same with y staged
 * through the ring slot into 1 KiB contiguous stores (round 6, bit-identical), 1 = the block backward's tile-shared
 * form, 0 = the per-wave conv3x3_kernel (tools/fwd_form_bench.py).  Returns the previous. */
int hrl_conv3x3_set_fwd_form(int form);
/* Both packed layouts of n <= 8 weights (32, 32, 3, 3) in one launch: packed[(l*2 + f) * 9216], f = 0 forward,
 * 1 input gradient (host array of device pointers).  hrl_conv3x3_forward_ex with flip | 2 takes `weight`
 * as such a packed layout and skips its own packing launch. */
int hrl_conv3x3_pack_n(const float *const *weights, int n, float *packed, void *stream);
int hrl_conv3x3_forward_ex(const float *x, int64_t M, const float *in_alpha, const float *in_beta,
                           const float *weight, const float *bias, int flip, float *y, int epilogue,
                           const float *ref, const float *ep_mean, const float *ep_alpha, const float *ep_beta,
                           double *part, void *workspace, int64_t workspace_bytes, void *stream);
int hrl_conv3x3_wgrad_ex(const float *x, const float *in_alpha, const float *in_beta, const float *dy, int64_t M,
                         float *dweight, void *workspace, int64_t workspace_bytes, void *stream);

/*
 * One conv -> BN -> ReLU chain block's whole backward in one launch (conv3x3_block_bwd_kernel), replacing
 * hrl_bn_backward_apply + hrl_conv3x3_wgrad_ex + hrl_conv3x3_forward_ex(flip) of that block:
 *   dY      = hrl_bn_backward_apply(y, g; bn_weight, bn_bias, save_mean, save_invstd, relu=1, kcoef, gmean),
 *             formed in registers (never stored);
 *   dweight = the weight gradient of conv(x') with x' = relu(x*in_alpha + in_beta) (or x; both or neither);
 *   gin     = (gin != NULL) the input gradient conv^T(dY) from packed_flip (hrl_conv3x3_pack_n's f = 1 layout)
 *             with the epilogue of hrl_conv3x3_forward_ex and ref = x: 0 none, 2 BN_{i-1}'s backward sums
 *             into part (ep_mean, ep_alpha, ep_beta), 3 gin *= [x > 0].
 * g, y, x, gin: (M, 288) rows; M * 1152 bytes < 4 GiB.  workspace: hrl_conv3x3_workspace_bytes(M) bytes;
 * part: hrl_conv3x3_block_sum_blocks(M) x 32 x 2 doubles.  Replaces, for the TicTacToe body
 * (tictactoe.py:57-65), the autograd backward of conv -> BatchNorm2d -> ReLU per block.
 */
/* dweight NULL: the weight gradient is left as per-workgroup partial rows in the workspace (9216 floats each,
 * [tap][ci][co]) for hrl_grad_fold_norm (fold mode 1); hrl_conv3x3_wgrad_partials(M, &offset_bytes) returns their
 * row count and byte offset in the workspace. */
int64_t hrl_conv3x3_wgrad_partials(int64_t M, int64_t *offset_bytes);
int hrl_conv3x3_block_backward(const float *g, const float *y, int64_t M, const float *bn_weight,
                               const float *bn_bias, const float *save_mean, const float *save_invstd,
                               const float *kcoef, const float *gmean, const float *x, const float *in_alpha,
                               const float *in_beta, const float *packed_flip, float *dweight, float *gin,
                               int epilogue, const float *ep_mean, const float *ep_alpha, const float *ep_beta,
                               double *part, void *workspace, int64_t workspace_bytes, void *stream);

/*
 * The BatchNorm finalize folded into the kernel that consumes it (ABI 26): the chain's kernels no longer wait on
 * a finalize launch of their own between them.
 *
 * hrl_conv3x3_forward_bnfold = hrl_bn_finalize_stats(prev_part, prev_nblocks, 32, M*9, gamma, beta, running_mean,
 *   running_var, momentum, eps, save_mean, save_invstd, alpha, beta_out) followed by hrl_conv3x3_forward_ex(x, M,
 *   alpha, beta_out, packed, NULL, 2, y, 1, ..., part): the previous conv's BN statistics -> its coefficients ->
 *   this conv's BN + ReLU prologue, epilogue 1 (this conv's statistics into part).  Under fwd form 2 (default) one
 *   launch: every workgroup folds the partial rows in bn_finalize_kernel's order (bit-identical coefficients),
 *   workgroup 0 writes the four outputs and advances the running statistics; other forms run the two launches.
 *   prev_part != part (the prologue reads every row the epilogue rewrites); prev_nblocks <= 512 for the fused form.
 * hrl_conv3x3_block_backward_bnfold = hrl_bn_finalize_backward(sums, sums_nblocks, 32, M*9, bn_weight,
 *   save_invstd, dgamma, dbeta, kcoef, gmean) followed by hrl_conv3x3_block_backward(... kcoef, gmean ...): one
 *   launch under block form 1 (default) with an input gradient, the two otherwise.  sums != part.
 * Both replace the finalize between two of the TicTacToe body's convs (tictactoe.py:57-65; BatchNorm2d's
 * statistics / backward reduction, train.py:383).
 */
int hrl_conv3x3_forward_bnfold(const float *x, int64_t M, const double *prev_part, int64_t prev_nblocks,
                               const float *gamma, const float *beta, float *running_mean, float *running_var,
                               double momentum, double eps, float *save_mean, float *save_invstd, float *alpha,
                               float *beta_out, const float *packed, float *y, double *part, void *workspace,
                               int64_t workspace_bytes, void *stream);
int hrl_conv3x3_block_backward_bnfold(const float *g, const float *y, int64_t M, const float *bn_weight,
                                      const float *bn_bias, const float *save_mean, const float *save_invstd,
                                      const double *sums, int64_t sums_nblocks, float *dgamma, float *dbeta,
                                      float *kcoef, float *gmean, const float *x, const float *in_alpha,
                                      const float *in_beta, const float *packed_flip, float *dweight, float *gin,
                                      int epilogue, const float *ep_mean, const float *ep_alpha, const float *ep_beta,
                                      double *part, void *workspace, int64_t workspace_bytes, void *stream);

/*
 * Fused ConvLSTM cell gates (GeisterNet DRC, handyrl/envs/geister.py:48-63;
 * replaces the split/sigmoid/tanh/mul/add chain of ConvLSTMCell.forward and
 * its autograd backward).  Gate pre-activations z = zx + zh in channel order
 * i, f, o, g: zh (N, 4H, HW) contiguous; zx the same shape with per-sample
 * stride zx_stride floats (a channel slice of a wider tensor) or NULL.
 * bias (bias_rows, 4H) or NULL: the x half's convolution bias, added as z = (zx + bias[n % bias_rows]) + zh
 * (the biased convolution's own order; bias_rows > 1 for layers stacked along N, sample n = e*rows + layer).
 * Forward: gates (N, 4H, HW) = (sigmoid i, sigmoid f, sigmoid o, tanh g) (NULL: not saved, inference);
 *          c_out = f*c + i*g; h_out = o*tanh(c_out).
 * Backward: dz (N, 4H, HW) and dc (N, H, HW) from dh / dc_out (either may be NULL = zero).
 */
int hrl_lstm_gates_forward(const float *zx, int64_t zx_stride, const float *zh, const float *c, int64_t N, int64_t H,
                           int64_t HW, const float *bias, int64_t bias_rows, float *h_out, float *c_out, float *gates,
                           void *stream);
/* hrl_lstm_gates_forward_grouped: the L (<= 4) cells of one DRC repeat in one launch; layer l's zh is channels
 * [l*4H, (l+1)*4H) of one grouped convolution's output (per-sample stride zh_stride floats), zx[l] its x half
 * (per-sample stride zx_strides[l]), c[l] its state; writes h_out[l], c_out[l] (contiguous (N, H, HW)) and, when
 * gates is given, gates[l] (N, 4H, HW).  hrl_lstm_gates_forward's float operations (z = zx + zh). */
int hrl_lstm_gates_forward_grouped(int L, const float *zh, int64_t zh_stride, const float *const *zx,
                                   const int64_t *zx_strides, const float *const *c, int64_t N, int64_t H, int64_t HW,
                                   float *const *h_out, float *const *c_out, float *const *gates, void *stream);
/* hrl_lstm_gates_backward_ex: hrl_lstm_gates_backward for the repeats of a recurrent unroll step -- dh (games
 * dh_stride floats apart) is the sum of dh_parts partial gradients dh_part_stride floats apart (added in order),
 * and with dzx given the gate gradient is also written (dzx_init) or added (else) into dzx (N, 4H, HW). */
int hrl_lstm_gates_backward_ex(const float *gates, const float *c, const float *c_out, const float *dh,
                               int64_t dh_stride, int dh_parts, int64_t dh_part_stride, const float *dc_out,
                               int64_t N, int64_t H, int64_t HW, float *dz, float *dc, float *dzx, int dzx_init,
                               void *stream);
int hrl_lstm_gates_backward(const float *gates, const float *c, const float *c_out, const float *dh,
                            const float *dc_out, int64_t N, int64_t H, int64_t HW, float *dz, float *dc,
                            void *stream);

/*
 * Recurrent state plumbing of forward_prediction (handyrl/train.py:155-174),
 * one launch for all state tensors (csrc/hrl_hidden.hip).  Each state tensor
 * l is (B, P, F[l]) floats (arrays of per-tensor device pointers; at most 16).
 * mask: (B, P) observation mask of the step.
 *   gather:  out[l] = sum_p H[l][:, p] * mask[:, p]  -> (B, F[l])      (sum != 0)
 *                     H[l] * mask                     -> (B, P, F[l])   (sum == 0)
 *   update:  out[l] = H[l] * (1 - mask) + nh[l] * mask, nh[l]: (B, Pn, F[l]), Pn = 1 or P
 * and their adjoints.  A tensor whose gradient is None is left out of the
 * backward call, so autograd's pruning is kept.
 */
int hrl_hidden_gather(const float *const *H, const float *mask, int64_t B, int64_t P, int nleaves, const int64_t *F,
                      int sum, float *const *out, void *stream);
int hrl_hidden_gather_backward(const float *const *dout, const float *mask, int64_t B, int64_t P, int nleaves,
                               const int64_t *F, int sum, float *const *dH, void *stream);
int hrl_hidden_update(const float *const *H, const float *const *nh, int64_t Pn, const float *mask, int64_t B,
                      int64_t P, int nleaves, const int64_t *F, float *const *out, void *stream);
int hrl_hidden_update_backward(const float *const *dout, const float *mask, int64_t B, int64_t P, int64_t Pn,
                               int nleaves, const int64_t *F, float *const *dH, float *const *dnh, void *stream);
/* The adjoints with an addend per state tensor (addend NULL, or per tensor NULL / rows of F[l] floats that are
 * addend_strides[l] floats apart, NULL: F[l]): gather: dH[l] = addend[l] + (the adjoint); update: dnh[l] =
 * addend[l] + (the adjoint).  The sum a state tensor with two consumers needs (the gather and the update of the
 * same step; the new state and the step's output) formed in the adjoint's launch instead of by autograd
 * (train._unroll_flat_hidden); the stride takes a channel slice of a wider gradient without a copy. */
int hrl_hidden_gather_backward_add(const float *const *dout, const float *mask, int64_t B, int64_t P, int nleaves,
                                   const int64_t *F, int sum, const float *const *addend,
                                   const int64_t *addend_strides, float *const *dH, void *stream);
int hrl_hidden_update_backward_add(const float *const *dout, const float *mask, int64_t B, int64_t P, int64_t Pn,
                                   int nleaves, const int64_t *F, const float *const *addend,
                                   const int64_t *addend_strides, float *const *dH, float *const *dnh,
                                   void *stream);
/* Step t's state update fused with step t+1's gather (round 5; the learner's recurrent unroll): out = H (1 - mask)
 * + nh mask (hrl_hidden_update) and gathered = the next step's input from out with mask_next (hrl_hidden_gather, sum
 * as there), one launch; bit for bit the two launches.  The adjoint: the gather's (dout = dgathered mask_next +
 * dstate, dstate the new state's other gradient, rows dstate_strides floats apart, NULL: none; a leaf's dgathered
 * may be NULL when its dstate is given) then the update's (dH, dnh = ... + dout_add, the step output's gradient,
 * rows dout_add_strides apart), one launch. */
int hrl_hidden_update_gather(const float *const *H, const float *const *nh, int64_t Pn, const float *mask,
                             const float *mask_next, int64_t B, int64_t P, int nleaves, const int64_t *F, int sum,
                             float *const *out, float *const *gathered, void *stream);
int hrl_hidden_update_gather_backward(const float *const *dgathered, const float *mask, const float *mask_next,
                                      int64_t B, int64_t P, int64_t Pn, int nleaves, const int64_t *F, int sum,
                                      const float *const *dstate, const int64_t *dstate_strides,
                                      const float *const *dout_add, const int64_t *dout_add_strides,
                                      float *const *dH, float *const *dnh, void *stream);

/*
 * 3x3 convolution on a torus board, 17 or 32 -> 32 channels, H*W <= 80
 * (GeeseNet's TorusConv2d, handyrl/envs/kaggle/hungry_geese.py:23-35: the
 * reference's wrap-around concatenation + 'valid' conv, with the wrap as
 * addressing) with fp32 MFMA (csrc/hrl_torus.hip).  x: (N, Cin, H, W),
 * y: (N, 32, H, W), weight (32, Cin, 3, 3), bias (32) or NULL.
 * flip = 0: y = conv(x, W) + bias.  flip = 1 (no bias): y = conv^T(x, W), the input
 * gradient of the forward: x is then (N, 32, H, W) and y (N, Cin, H, W).  part != NULL: also the per-workgroup
 * fp64 (sum y, sum y^2) per channel, hrl_torus_stats_blocks(N) x 32 x 2
 * doubles -> hrl_bn_finalize_stats (GeeseNet's BatchNorm after every conv).
 * add != NULL (flip = 1, the input gradient of a residual block): y += add * [add_mask > 0]
 * elementwise in the store (the residual branch's gradient, masked by the block's ReLU);
 * add and add_mask are shaped like y.
 * hrl_torus_conv_wgrad: dweight (32, Cin, 3, 3) and dbias (32, may be NULL)
 * for input x and output gradient dy; deterministic.
 * workspace: hrl_torus_workspace_bytes(N) bytes.
 */
int64_t hrl_torus_workspace_bytes(int64_t N);
/* Arithmetic of the torus forward / input-gradient kernel, as hrl_conv3x3_set_split: on != 0 (default) the exact
 * three-way bf16 split on v_mfma_f32_16x16x32_bf16, 0 fp32 MFMA.  Process-wide; returns the previous setting. */
int hrl_torus_set_split(int on);
/* Kernel form of the split 32-input-channel launches (hrl_torus_conv_forward with 32 input channels,
 * hrl_torus_unit_forward, hrl_torus_unit_input_grad): 2 (default) splits each input value once per sample into an
 * LDS image of bf16 parts, 1 splits the gathered values per tap.  The results are bit-identical.  1 or 2 sets the
 * form; any other value only queries.  Process-wide; returns the previous setting. */
int hrl_torus_set_form(int form);
int64_t hrl_torus_stats_blocks(int64_t N);
int hrl_torus_conv_forward(const float *x, int64_t N, int64_t Cin, int64_t Cout, int64_t H, int64_t W,
                           const float *weight, const float *bias, int flip, float *y, double *part,
                           const float *add, const float *add_mask, void *workspace, int64_t workspace_bytes,
                           void *stream);
int hrl_torus_conv_wgrad(const float *x, const float *dy, int64_t N, int64_t Cin, int64_t Cout, int64_t H, int64_t W,
                         float *dweight, float *dbias, void *workspace, int64_t workspace_bytes, void *stream);
/* The weight gradient of a torus conv followed by a training-mode BatchNorm and a ReLU (round 5), with the
 * BatchNorm's masked backward apply formed in the kernel's staging instead of a pass of its own:
 *   dy = (((g [o > 0] - gmean) - (y - save_mean) kcoef) save_invstd) gamma   per channel,
 *   o = [x +] (y alpha + beta)   (the block output relu(o) recomputed as the forward formed it; residual != 0:
 *                                 the block's input x is its residual, Cin 32)
 * (hrl_bn_backward_apply_masked's arithmetic, bit for bit; gamma NULL = 1) is written to dy (N, 32, H, W) for the
 * input gradient, and dweight (32, Cin, 3, 3) / dbias (32, may be NULL) are hrl_torus_conv_wgrad(x, dy).
 * y, g: (N, 32, H, W) float4-aligned (the conv output, the gradient w.r.t. the block output); alpha / beta the
 * forward's hrl_bn_finalize_stats coefficients; kcoef / gmean from hrl_bn_finalize_backward or
 * hrl_bn_backward_masked_coefs.  Cin 17 or 32 (32: x float4-aligned); split arithmetic only
 * (hrl_torus_set_split(1), else HRL_EINVAL).  workspace: hrl_torus_workspace_bytes(N). */
int hrl_torus_conv_wgrad_bn(const float *x, int64_t N, int64_t Cin, int64_t H, int64_t W, const float *y,
                            const float *g, const float *alpha, const float *beta, int residual, const float *gamma,
                            const float *save_mean, const float *save_invstd, const float *kcoef, const float *gmean,
                            float *dy, float *dweight, float *dbias, void *workspace, int64_t workspace_bytes,
                            void *stream);

/*
 * The GeeseNet unit chain (hungry_geese.py:48-51, h_{i+1} = relu(h_i + bn_i(conv_i(h_i)))) with the
 * BatchNorm passes folded into the torus convs:
 * hrl_torus_unit_forward: unit i's conv (32 -> 32, with the BN statistics in part) whose input
 *   h = relu([res +] y_prev*alpha[c] + beta[c]) is built in the prologue from the previous unit's conv
 *   output y_prev, its residual input res (NULL for the unit after the stem) and BN coefficients
 *   (hrl_bn_finalize_stats alpha/beta); h is also written (N, 32, H, W).  Same arithmetic as
 *   hrl_bn_apply_residual + hrl_torus_conv_forward, one pass less.
 * hrl_torus_unit_input_grad: dh = conv^T(dy) + g*[out > 0] (unit i's input gradient, the residual
 *   branch added) and, in the same pass, the previous unit's masked BatchNorm backward sums
 *   part[block][c] = (sum dh*[h_mask > 0], sum dh*[h_mask > 0]*(y_prev - mean_prev[c])) over
 *   hrl_torus_stats_blocks(N) blocks -> hrl_bn_finalize_backward -> hrl_bn_backward_apply_masked.
 *   h_mask is unit i's input (= unit i-1's output), y_prev unit i-1's conv output.
 * Both: float4-aligned tensors, workspace hrl_torus_workspace_bytes(N).
 */
int hrl_torus_unit_forward(const float *y_prev, const float *res, const float *alpha, const float *beta, float *h,
                           int64_t N, int64_t H, int64_t W, const float *weight, const float *bias, float *y,
                           double *part, void *workspace, int64_t workspace_bytes, void *stream);
/* A zero-padded 3x3 'same' nn.Conv2d, 32 input channels -> Cout (a multiple of 32) on a board of 4..80 cells,
 * on the torus kernel's MFMA path (GeisterNet's ConvLSTM h / x halves, geister.py:48-59): x (N, 32, H, W),
 * y (N, Cout, H, W); the weights are input channels [w_ci0, w_ci0 + 32) of a (Cout, w_cin_total, 3, 3)
 * tensor (a cell's conv([x, h]) split into its halves); bias (Cout) or NULL.
 * workspace: hrl_board_conv_workspace_bytes(Cout) bytes.  hrl_board_conv_pack + hrl_board_conv_forward_packed
 * split the weight packing out (a recurrent unroll packs each weight once per step). */
int64_t hrl_board_conv_workspace_bytes(int64_t Cout);
int hrl_board_conv_forward(const float *x, int64_t N, int64_t Cin, int64_t H, int64_t W, const float *weight,
                           int64_t w_cin_total, int64_t w_ci0, int64_t Cout, const float *bias, float *y,
                           void *workspace, int64_t workspace_bytes, void *stream);
int hrl_board_conv_pack(const float *weight, int64_t w_cin_total, int64_t w_ci0, int64_t Cout, void *packed,
                        int64_t packed_bytes, void *stream);
int hrl_board_conv_forward_packed(const float *x, int64_t N, int64_t Cin, int64_t H, int64_t W, const void *packed,
                                  int64_t Cout, const float *bias, float *y, void *stream);

/* GeisterNet's 3x3 'same' convolutions at self-play sizes (geister.py:17-63 ConvLSTMCell, :99-167 GeisterNet)
 * on the 6x6 board with games as the MFMA rows (csrc/hrl_gboard.hip): the stem, the cells' x halves, their
 * grouped h halves and the move head's first conv replace the vendor convolutions of the inference forward.
 * hrl_gboard_pack: input channels [w_ci0, w_ci0 + Cin_g) of weight (Cout, w_cin_total, 3, 3) -> split fragments
 *   (packed: hrl_gboard_pack_bytes(Cout, Cin_g) bytes; pack once, convolve many times).
 * hrl_gboard_forward: y[n, co] = conv(x[n, group(co) * Cin_g ..], W[co]) for N games, groups | Cout
 *   (groups > 1: Cout / groups a multiple of 16), Cin_g <= 64.  Game n of x starts at x + n * x_stride floats
 *   (channel c at + c * 36); x2 (or NULL; groups 1, Cin_g > 32 only): channels 32.. read from x2 instead
 *   (the head's [h_e, h_last] without the concatenation).  y: game n at y + n * y_stride.  Epilogue, in order:
 *   + bias[co] (or NULL), * alpha[co] + beta[co] (a BatchNorm's inference coefficients, or both NULL),
 *   relu.  x, x2, y 16-byte aligned, strides multiples of 4.  packed_bytes: the size of `packed` (hrl_gboard_forward
 *   and hrl_gboard_forward_groups return HRL_EINVAL before any launch when it is below
 *   hrl_gboard_pack_bytes(Cout, Cin_g), e.g. a buffer packed for another shape; ABI 19). */
int64_t hrl_gboard_pack_bytes(int64_t Cout, int64_t Cin_g);
int hrl_gboard_pack(const float *weight, int64_t Cout, int64_t Cin_g, int64_t w_cin_total, int64_t w_ci0,
                    void *packed, int64_t packed_bytes, void *stream);
/* hrl_gboard_pack_adjoint: the input-gradient conv of input channels [w_ci0, w_ci0 + Cin_slice) of weight
 * (Cout_fwd, w_cin_total, 3, 3) -- W'[co'][ci'][tap] = W[ci'][w_ci0 + co'][8 - tap], Cin_slice outputs from Cout_fwd
 * inputs -- packed for hrl_gboard_forward (packed: hrl_gboard_pack_bytes(Cin_slice, Cout_fwd) bytes).
 * Cin_g (input channels per group) may be <= 64 or 97..128 (1, 2 or 4 k-steps of 32). */
int hrl_gboard_pack_adjoint(const float *weight, int64_t Cout_fwd, int64_t w_cin_total, int64_t w_ci0,
                            int64_t Cin_slice, void *packed, int64_t packed_bytes, void *stream);
/* hrl_gboard_wgrad: the weight (and bias) gradient of a 3x3 'same' conv on the 6x6 board summed over nseg (<= 64)
 * recorded uses (x_i: ns[i] games of Cin input channels, x_strides[i] floats apart; dy_i: ns[i] games of Cout
 * output gradients), ADDED into input channels [w_ci0, w_ci0 + Cin) of dweight (Cout, w_cin_total, 3, 3) and, when
 * dbias is given, into dbias (Cout).  Games are the MFMA K (exact bf16 split, fp32-accurate); deterministic.
 * Replaces the deferred weight gradient's aten.convolution_backward (nn.DeferredGrads.flush).  32-channel tiles
 * (Cout, Cin): 4x1, 2x2, 2x1, 1x2, 1x1.  workspace: hrl_gboard_wgrad_workspace_bytes(Cout, Cin, G) bytes, G = the
 * sum over the segments of ns[i] rounded up to a multiple of 16 (one workgroup partial per 16-game tile). */
int64_t hrl_gboard_wgrad_workspace_bytes(int64_t Cout, int64_t Cin, int64_t total_games);
int hrl_gboard_wgrad(const float *const *xs, const int64_t *x_strides, const float *const *dys,
                     const int64_t *dy_strides, const int64_t *ns, int nseg, int64_t Cout, int64_t Cin,
                     float *dweight, int64_t w_cin_total, int64_t w_ci0, float *dbias, void *workspace,
                     int64_t workspace_bytes, void *stream);
/* hrl_gboard_set_whole_ring: 1 (default) = launches with one task per workgroup stage a whole 32-channel k-step
 * (9 quads) at once, 0 = the 3-quad ring always (measurement); returns the previous setting. */
int hrl_gboard_set_whole_ring(int on);
/* hrl_gboard_set_nctw: force the column tiles per workgroup (1, 2, 4; 0 = the launcher's choice), measurement
 * only; returns the previous setting. */
int hrl_gboard_set_nctw(int nctw);
/* hrl_gboard_launch_stats: the launch forms the gboard launchers chose since the last reset (host-side counters; a
 * graph replay does not count), so a test can assert which kernels a learner step at a given size ran.  Copies
 * min(n, total) counters into counts (NULL: none) and returns the total; reset != 0 zeroes them afterwards.  Order:
 * 0 conv launches, 1 of them whole-tile (one task per workgroup, the k-step staged at once), 2/3/4 with 1/2/4 column
 * tiles per workgroup, 5 with groups == 4 (the h halves' K-split adjoint), 6 hrl_gboard_forward_groups calls,
 * 7 hrl_gboard_wgrad launches, 8 the most segments in one, 9 the most 16-game tiles in one, 10 wgrad launches in
 * which workgroups carry their accumulators over several tiles (tiles > 256). */
int hrl_gboard_launch_stats(int64_t *counts, int n, int reset);
/* hrl_gboard_pointwise_wgrad: dweight (O, C) += sum over N games and the 36 cells of dy[n][o][q] x[n][c][q] -- the
 * weight gradient of a 1x1 conv on the 6x6 board (O <= 8, C <= 256; games x_stride / dy_stride floats apart,
 * float4-aligned).  Deterministic (per-workgroup partials folded in order).  workspace:
 * hrl_gboard_pointwise_wgrad_workspace_bytes(C, O, N) bytes. */
int64_t hrl_gboard_pointwise_wgrad_workspace_bytes(int64_t C, int64_t O, int64_t N);
int hrl_gboard_pointwise_wgrad(const float *x, int64_t x_stride, const float *dy, int64_t dy_stride, int64_t N,
                               int64_t C, int64_t O, float *dweight, void *workspace, int64_t workspace_bytes,
                               void *stream);
/* hrl_gboard_forward_groups: a grouped conv (groups <= 4, Cin_g <= 32 per group) whose groups read separate
 * inputs xs[g] (N games, x_strides[g] floats apart): the DRC layers' h halves of one repeat without stacking
 * their states.  No bias / epilogue. */
int hrl_gboard_forward_groups(const float *const *xs, const int64_t *x_strides, int64_t N, int64_t Cin_g,
                              int64_t groups, const void *packed, int64_t packed_bytes, int64_t Cout, float *y,
                              int64_t y_stride, void *stream);
int hrl_gboard_forward(const float *x, int64_t x_stride, const float *x2, int64_t x2_stride, int64_t N, int64_t Cin_g,
                       int64_t groups, const void *packed, int64_t packed_bytes, int64_t Cout, const float *bias,
                       const float *alpha, const float *beta, int relu, float *y, int64_t y_stride, void *stream);

/* A 1x1 convolution on the 6x6 board (no bias; GeisterNet's move-head conv2 and value / return head convs,
 * geister.py:238-264): y[n, o, q] = sum_c W[o, c] x[n, c, q] over x1's C1 channels, then x2's C2 (x2 NULL when
 * C2 = 0), then y*alpha[o] + beta[o] (both or neither) and relu.  weight (O, C1 + C2) row-major, O in
 * {1, 2, 4, 8}, C1 + C2 <= 128; games x1_stride / x2_stride / y_stride floats apart. */
int hrl_gboard_pointwise(const float *x1, int64_t x1_stride, int64_t C1, const float *x2, int64_t x2_stride,
                          int64_t C2, int64_t N, const float *weight, int64_t O, const float *alpha, const float *beta,
                          int relu, float *y, int64_t y_stride, void *stream);

/* GeeseNet's head pooling (hungry_geese.py:52-53) on h (N, 32, H, W) and the net input x (its plane 0,
 * samples x_stride floats apart): head[n, c] = sum_q h[n, c, q] * x[n, 0, q], avg[n, c] = mean_q h[n, c, q]
 * (both (N, 32)); hrl_torus_head_unpool: the gradient w.r.t. h, g = dhead * x0 + davg / (H*W). */
int hrl_torus_head_pool(const float *h, const float *x, int64_t N, int64_t H, int64_t W, int64_t x_stride,
                        float *head, float *avg, void *stream);
int hrl_torus_head_unpool(const float *dhead, const float *davg, const float *x, int64_t N, int64_t H, int64_t W,
                          int64_t x_stride, float *g, void *stream);
int hrl_torus_unit_input_grad(const float *dy, int64_t N, int64_t H, int64_t W, const float *weight, const float *g,
                              const float *out, float *dh, const float *h_mask, const float *y_prev,
                              const float *mean_prev, double *part, void *workspace, int64_t workspace_bytes,
                              void *stream);

/*
 * The TicTacToe net's two output heads fused (handyrl/envs/tictactoe.py:35-49, 59-60;
 * csrc/hrl_heads.hip): on h (N, 32, 3, 3),
 *   a_p = leaky_relu(conv1x1(h; w1p (2, 32), b1p (2)), 0.1)  (N, 18);  p = a_p @ wp^T, wp (9, 18)
 *   a_v = leaky_relu(conv1x1(h; w1v (1, 32), b1v (1)), 0.1)  (N, 9);   v = a_v @ wv^T, wv (1, 9)
 * hrl_heads_forward writes p (N, 9), v (N, 1) (the value before the model's tanh; tanh_v != 0: after it,
 * the model's torch.tanh folded in) and, when a_p / a_v are non-NULL, the activations the backward needs.
 * bn_alpha / bn_beta (32 each, both or neither): the input is the raw input y of the body's last
 * BatchNorm and the heads read h = relu(y*bn_alpha + bn_beta) (hrl_bn_finalize_stats' coefficients).
 * hrl_heads_backward: from dp (N, 9), dv (N, 1): dh (N, 288) = dL/dh and every parameter gradient;
 * v_tanh != NULL: dv is the gradient of tanh(v) and v_tanh that forward output (tanh_v = 1), the tanh
 * backward dv * (1 - v_tanh^2) is applied in the kernels
 * (deterministic); with bn_part (needs bn_alpha/beta and bn_mean) also that BatchNorm's backward sums
 * (sum dh*m, sum dh*m*(y - bn_mean)), m = [y*bn_alpha + bn_beta > 0], as fp64 partials
 * bn_part[hrl_heads_bn_parts(N)][32][2] -> hrl_bn_finalize_backward.
 * workspace: hrl_heads_workspace_bytes(N) bytes.
 */
int64_t hrl_heads_workspace_bytes(int64_t N);
int64_t hrl_heads_bn_parts(int64_t N);
int hrl_heads_forward(const float *h, int64_t N, const float *w1p, const float *b1p, const float *w1v,
                      const float *b1v, const float *wp, const float *wv, const float *bn_alpha, const float *bn_beta,
                      float *a_p, float *a_v, float *p_out, float *v_out, int tanh_v, void *stream);
/* hrl_heads_backward with all six weight-gradient pointers NULL (form 2): the parameter gradients are left as
 * hrl_heads_bn_parts(N) partial rows of 270 floats at the start of the workspace -- [dW1 (3 x 32: policy rows then
 * the value row) | db1 (3) | dWp (9 x 18) | dWv (9)] -- for hrl_grad_fold_norm. */
/* hrl_heads_set_bwd_form: 2 (default) = the lane-per-channel backward (4-wave workgroups, accumulators in registers,
 * the fc weight gradients in the same pass), 1 = the row-per-lane kernel + separate fc-gradient launch (measurement).
 * Process-wide; returns the previous setting (any other value only queries it).  hrl_heads_bn_parts /
 * hrl_heads_workspace_bytes follow the form; the deferred (NULL-gradient) mode needs form 2. */
int hrl_heads_set_bwd_form(int form);
int hrl_heads_backward(const float *h, int64_t N, const float *w1p, const float *w1v, const float *wp,
                       const float *wv, const float *bn_alpha, const float *bn_beta, const float *bn_mean,
                       double *bn_part, const float *a_p, const float *a_v, const float *dp, const float *dv,
                       const float *v_tanh, float *dh, float *dw1p, float *db1p, float *dw1v, float *db1v, float *dwp, float *dwv,
                       void *workspace, int64_t workspace_bytes, void *stream);

/* The 3x3-board stem conv, Cin <= 3 -> 32 channels, with bias (TicTacToe, tictactoe.py:57), as fp32
 * MFMA on the dense board matrix (csrc/hrl_stem.hip): x (N, Cin, 3, 3), y (N, 32, 3, 3),
 * weight (32, Cin, 3, 3), bias (32) or NULL.  hrl_stem_wgrad: dweight and dbias (may be NULL),
 * deterministic; workspace hrl_stem_workspace_bytes(N) bytes.  (No input gradient: the stem reads
 * the observation.) */
int64_t hrl_stem_workspace_bytes(int64_t N);
int hrl_stem_forward(const float *x, int64_t N, int64_t Cin, const float *weight, const float *bias, float *y,
                     void *stream);
int hrl_stem_wgrad(const float *x, const float *dy, int64_t N, int64_t Cin, float *dweight, float *dbias,
                   void *workspace, int64_t workspace_bytes, void *stream);
/* hrl_stem_wgrad with dweight and dbias NULL (form 2): the gradients are left as hrl_stem_wgrad_partials(N, &row)
 * partial rows of `row` floats at the start of the workspace, [dW (32, Cin, 3, 3) | db (32)], for
 * hrl_grad_fold_norm. */
int64_t hrl_stem_wgrad_partials(int64_t N, int64_t *row_floats);
/* hrl_stem_set_wgrad_form: 2 (default) = the lane-per-channel weight gradient (a lane owns one output channel's
 * Cin x 9 weights and its bias of a row; 4-wave workgroups, 4 per CU), 1 = the dense-board fp32 MFMA kernel
 * (measurement).  Process-wide; returns the previous setting (any other value only queries it).
 * hrl_stem_workspace_bytes covers both forms; the deferred (NULL-gradient) mode needs form 2. */
int hrl_stem_set_wgrad_form(int form);
/* hrl_stem_set_fwd_form: 2 (default) = the lane-per-channel forward (a lane owns one output channel of two rows as a
 * float2: packed fp32 FMAs, weights in registers, 36-byte output runs), 1 = the fp32 MFMA kernel on the dense board
 * matrix (measurement).  Process-wide; returns the previous setting (any other value only queries it). */
int hrl_stem_set_fwd_form(int form);

/* The learner step's tail on the flat gradient buffer `grads` (n floats; parameter gradients are views of it):
 * hrl_grad_fold_norm: for each of nfolds (<= 16) deferred weight-gradient folds, grads[dst + j] (j < count) =
 *   the fixed-order fp64 sum over nparts partial rows of parts[row * stride + col0 + col(j)] (mode 0: col(j) = j;
 *   mode 1: a 32x32x3x3 conv weight from the chain blocks' [tap][ci][co] rows, count 9216); then the fp64 sum of
 *   squares of every 64-element block of grads into norm_part (hrl_grad_fold_norm_blocks(n) doubles); and,
 *   once, *step += 1 (may be NULL) and *counters[k] += increments[k] (BatchNorm num_batches_tracked,
 *   ncounters <= 8; increments NULL: all 1, e.g. T for a recurrent unroll's per-step BatchNorm).
 * hrl_adam_clip: clip_grad_norm_(max_norm) from those block sums (every workgroup folds them in one fixed order;
 *   *total_norm = the norm; grads scaled in place) and torch.optim.Adam's step (fused_adam_utils.cuh adam_math,
 *   L2 weight decay, the same double / float promotions) on the tensors params[t] (elements offsets[t] ..
 *   offsets[t+1] of grads, offsets[ntensors] = n, ntensors <= 64) whose live[t] != 0; exp_avg / exp_avg_sq are n
 *   floats each; lr and step are device scalars (a graph replays with their current values).  Once per call
 *   acc_dst[k] += *acc_src[k] for k < nacc (<= 8; acc_src[k] NULL: the norm) -- the learner's running loss
 *   statistics, so their accumulation is no launch of its own.
 * Deterministic.  Replaces the reduce launches of the HIP backward Functions, the clip, torch's step-count and
 * batch-counter increments and torch's fused Adam (train.py:384-385). */
int64_t hrl_grad_fold_norm_blocks(int64_t n);
int hrl_grad_fold_norm(float *grads, int64_t n, const float *const *parts, const int64_t *strides,
                       const int64_t *col0, const int64_t *nparts, const int64_t *dst, const int64_t *count,
                       const int *modes, int nfolds, float *step, int64_t *const *counters,
                       const int64_t *increments, int ncounters, double *norm_part, int64_t norm_part_bytes,
                       void *stream);
int hrl_adam_clip(float *grads, int64_t n, const double *norm_part, double max_norm, float *total_norm,
                  float *const *params, const int64_t *offsets, const int *live, int ntensors, float *exp_avg,
                  float *exp_avg_sq, const float *lr, const float *step, double beta1, double beta2, double eps,
                  double weight_decay, const float *const *acc_src, int nacc, float *acc_dst, void *stream);

/* clip_grad_norm_(params, max_norm) on the learner's flat gradient buffer (handyrl/train.py:384)
 * in one launch: total = ||grads||_2 (fp64 fold) -> *total_norm; grads *= min(max_norm / (total + 1e-6), 1).
 * grads 16-byte aligned, n floats (csrc/hrl_optim.hip). */
int hrl_clip_grad_norm(float *grads, int64_t n, double max_norm, float *total_norm, void *stream);
/* The same with a workspace of hrl_clip_workspace_bytes(n) bytes (8-byte aligned): above 64 k floats it runs as
 * two launches over 64 workgroups (per-chunk fp64 partials, then every workgroup folds them in one fixed order and
 * scales its chunk) instead of one workgroup walking the whole buffer; deterministic, the same norm. */
int64_t hrl_clip_workspace_bytes(int64_t n);
int hrl_clip_grad_norm_ws(float *grads, int64_t n, double max_norm, float *total_norm, void *workspace,
                          int64_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HRL_NN_H */
