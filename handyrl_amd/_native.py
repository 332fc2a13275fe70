"""ctypes binding of the C ABI in ``include/*.h`` (libhrl.so).

The library is the ONLY compute path for the kernels it exports: if it is
missing or fails to load, every caller gets a RuntimeError — there is no CPU
or eager-PyTorch fallback.

torch is imported first so that the HIP runtime torch ships
(libamdhip64.so.7) is already in the process; libhrl.so's DT_NEEDED entry for
the same soname then binds to that copy, and the hipStream_t handles torch
hands us are valid in the library.
"""

import ctypes
import os

import torch  # noqa: F401  (must precede loading libhrl.so, see module doc)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib', 'libhrl.so')
# diagnostic builds (tools/*): HRL_LIB_PATH names another build of the same sources
LIB_PATH = os.environ.get('HRL_LIB_PATH', LIB_PATH)

HRL_OK = 0
HRL_EINVAL = -22

ALG = {'MC': 0, 'TD': 1, 'UPGO': 2, 'VTRACE': 3}

_f32p = ctypes.c_void_p
_i64 = ctypes.c_int64
_dbl = ctypes.c_double

# symbol -> (restype, argtypes); mirrors include/*.h exactly
SIGNATURES = {
    'hrl_abi_version': (ctypes.c_int, []),
    'hrl_targets_set_short_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_strerror': (ctypes.c_char_p, [ctypes.c_int]),
    'hrl_compute_target': (ctypes.c_int, [
        ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _f32p,
        _i64, _i64, _i64, _i64, _i64, _i64, _dbl, _dbl, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_compute_targets_fused': (ctypes.c_int, [
        ctypes.c_int, ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _f32p,
        _i64, _i64, _i64, _i64, _i64, _i64, _dbl, _dbl, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_bn_workspace_bytes': (ctypes.c_int64, [_i64, _i64, _i64]),
    'hrl_bn_forward_train': (ctypes.c_int, [
        _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p, _dbl, _dbl, ctypes.c_int, _f32p, _f32p, _f32p,
        ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_backward': (ctypes.c_int, [
        _f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p, ctypes.c_int, _f32p, _f32p, _f32p,
        ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_workspace_bytes_grouped': (ctypes.c_int64, [_i64, _i64, _i64, _i64]),
    'hrl_bn_forward_train_grouped': (ctypes.c_int, [
        _f32p, _i64, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p, _dbl, _dbl, ctypes.c_int, _f32p, _f32p, _f32p,
        ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_backward_grouped': (ctypes.c_int, [
        _f32p, _f32p, _i64, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p, ctypes.c_int, _f32p, _f32p, _f32p,
        ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_loss_workspace_bytes': (ctypes.c_int64, [_i64, _i64, _i64, _i64]),
    'hrl_loss_forward': (ctypes.c_int, [
        _f32p, _f32p, ctypes.c_void_p, _i64, _i64, _i64, _i64, _i64,
        _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
        ctypes.c_int, ctypes.c_int, ctypes.c_int, _dbl, _dbl, _dbl, _dbl,
        ctypes.c_void_p, _i64, _f32p, ctypes.c_void_p]),
    'hrl_loss_backward': (ctypes.c_int, [
        _f32p, ctypes.c_void_p, _i64, _i64, _i64, _i64, _i64,
        _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _dbl, _dbl,
        ctypes.c_void_p, _i64, _f32p, _f32p, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_output_mask_forward': (ctypes.c_int, [_f32p, _f32p, _f32p, _f32p, _f32p, _i64, _i64, _i64, _i64, _f32p,
                                               _f32p, ctypes.c_void_p]),
    'hrl_output_mask_backward': (ctypes.c_int, [_f32p, _f32p, _f32p, _f32p, _i64, _i64, _i64, _i64, _f32p, _f32p,
                                                ctypes.c_void_p]),
    'hrl_board_weight': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, _i64, _i64, _f32p, ctypes.c_void_p]),
    'hrl_board_fold': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, _i64, _i64, _f32p, ctypes.c_void_p]),
    'hrl_board_bias': (ctypes.c_int, [_f32p, _i64, _i64, _f32p, ctypes.c_void_p]),
    'hrl_board_bias_fold': (ctypes.c_int, [_f32p, _i64, _i64, _f32p, ctypes.c_void_p]),
    'hrl_conv3x3_workspace_bytes': (ctypes.c_int64, [_i64]),
    'hrl_conv3x3_forward': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _f32p, _f32p, ctypes.c_int, _f32p,
                                           ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_conv3x3_wgrad': (ctypes.c_int, [_f32p, _f32p, _i64, _i64, _i64, _f32p, ctypes.c_void_p, _i64,
                                         ctypes.c_void_p]),
    'hrl_colsum_workspace_bytes': (ctypes.c_int64, [_i64, _i64]),
    'hrl_colsum': (ctypes.c_int, [_f32p, _i64, _i64, _f32p, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_finalize_stats': (ctypes.c_int, [ctypes.c_void_p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p,
                                             ctypes.c_double, ctypes.c_double, _f32p, _f32p, _f32p, _f32p,
                                             ctypes.c_void_p]),
    'hrl_bn_forward_eval': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p, ctypes.c_double,
                                           ctypes.c_int, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_bn_apply': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _f32p, _f32p, ctypes.c_int, _f32p, ctypes.c_void_p]),
    'hrl_conv3x3_stats_blocks': (ctypes.c_int64, [_i64]),
    'hrl_conv3x3_block_sum_blocks': (ctypes.c_int64, [_i64]),
    'hrl_conv3x3_set_split': (ctypes.c_int, [ctypes.c_int]),
    'hrl_conv3x3_set_block_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_conv3x3_set_fwd_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_torus_set_split': (ctypes.c_int, [ctypes.c_int]),
    'hrl_torus_set_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_conv3x3_pack_n': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _f32p, ctypes.c_void_p]),
    'hrl_conv3x3_forward_ex': (ctypes.c_int, [_f32p, _i64, _f32p, _f32p, _f32p, _f32p, ctypes.c_int, _f32p,
                                              ctypes.c_int, _f32p, _f32p, _f32p, _f32p, ctypes.c_void_p,
                                              ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_finalize_backward': (ctypes.c_int, [ctypes.c_void_p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p,
                                                _f32p, _f32p, ctypes.c_void_p]),
    'hrl_bn_backward_apply': (ctypes.c_int, [_f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p,
                                             ctypes.c_int, _f32p, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_conv3x3_block_backward': (ctypes.c_int, [_f32p, _f32p, _i64, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                                  _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_int, _f32p,
                                                  _f32p, _f32p, ctypes.c_void_p, ctypes.c_void_p, _i64,
                                                  ctypes.c_void_p]),
    'hrl_conv3x3_forward_bnfold': (ctypes.c_int, [_f32p, _i64, ctypes.c_void_p, _i64, _f32p, _f32p, _f32p, _f32p,
                                                  ctypes.c_double, ctypes.c_double, _f32p, _f32p, _f32p, _f32p,
                                                  _f32p, _f32p, ctypes.c_void_p, ctypes.c_void_p, _i64,
                                                  ctypes.c_void_p]),
    'hrl_conv3x3_block_backward_bnfold': (ctypes.c_int, [_f32p, _f32p, _i64, _f32p, _f32p, _f32p, _f32p,
                                                         ctypes.c_void_p, _i64, _f32p, _f32p, _f32p, _f32p,
                                                         _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_int,
                                                         _f32p, _f32p, _f32p, ctypes.c_void_p, ctypes.c_void_p,
                                                         _i64, ctypes.c_void_p]),
    'hrl_conv3x3_wgrad_ex': (ctypes.c_int, [_f32p, _f32p, _f32p, _f32p, _i64, _f32p, ctypes.c_void_p, _i64,
                                            ctypes.c_void_p]),
    'hrl_hidden_gather': (ctypes.c_int, [ctypes.c_void_p, _f32p, _i64, _i64, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_gather_backward': (ctypes.c_int, [ctypes.c_void_p, _f32p, _i64, _i64, ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_gather_backward_add': (ctypes.c_int, [ctypes.c_void_p, _f32p, _i64, _i64, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_update_gather': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, _i64, _f32p, _f32p, _i64, _i64,
                                                ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_update_gather_backward': (ctypes.c_int, [ctypes.c_void_p, _f32p, _f32p, _i64, _i64, _i64,
                                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_update_backward_add': (ctypes.c_int, [ctypes.c_void_p, _f32p, _i64, _i64, _i64, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_update': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, _i64, _f32p, _i64, _i64, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_hidden_update_backward': (ctypes.c_int, [ctypes.c_void_p, _f32p, _i64, _i64, _i64, ctypes.c_int,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_lstm_gates_forward': (ctypes.c_int, [_f32p, _i64, _f32p, _f32p, _i64, _i64, _i64, _f32p, _i64, _f32p,
                                              _f32p, _f32p, ctypes.c_void_p]),
    'hrl_lstm_gates_backward': (ctypes.c_int, [_f32p, _f32p, _f32p, _f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p,
                                               ctypes.c_void_p]),
    'hrl_torus_workspace_bytes': (ctypes.c_int64, [_i64]),
    'hrl_torus_stats_blocks': (ctypes.c_int64, [_i64]),
    'hrl_torus_conv_forward': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, _i64, _f32p, _f32p, ctypes.c_int,
                                              _f32p, ctypes.c_void_p, _f32p, _f32p, ctypes.c_void_p, _i64,
                                              ctypes.c_void_p]),
    'hrl_stem_workspace_bytes': (ctypes.c_int64, [_i64]),
    'hrl_stem_forward': (ctypes.c_int, [_f32p, _i64, _i64, _f32p, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_stem_wgrad': (ctypes.c_int, [_f32p, _f32p, _i64, _i64, _f32p, _f32p, ctypes.c_void_p, _i64,
                                      ctypes.c_void_p]),
    'hrl_stem_set_wgrad_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_stem_set_fwd_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_clip_grad_norm': (ctypes.c_int, [_f32p, _i64, _dbl, _f32p, ctypes.c_void_p]),
    'hrl_clip_workspace_bytes': (ctypes.c_int64, [_i64]),
    'hrl_grad_fold_norm_blocks': (ctypes.c_int64, [_i64]),
    'hrl_grad_fold_norm': (ctypes.c_int, [_f32p, _i64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int, _f32p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_adam_clip': (ctypes.c_int, [_f32p, _i64, ctypes.c_void_p, _dbl, _f32p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _dbl, _dbl, _dbl,
                                     _dbl, ctypes.c_void_p, ctypes.c_int, _f32p, ctypes.c_void_p]),
    'hrl_conv3x3_wgrad_partials': (ctypes.c_int64, [_i64, ctypes.c_void_p]),
    'hrl_stem_wgrad_partials': (ctypes.c_int64, [_i64, ctypes.c_void_p]),
    'hrl_clip_grad_norm_ws': (ctypes.c_int, [_f32p, _i64, _dbl, _f32p, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_heads_workspace_bytes': (ctypes.c_int64, [_i64]),
    'hrl_heads_bn_parts': (ctypes.c_int64, [_i64]),
    'hrl_heads_set_bwd_form': (ctypes.c_int, [ctypes.c_int]),
    'hrl_heads_forward': (ctypes.c_int, [_f32p, _i64, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                         _f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_void_p]),
    'hrl_heads_backward': (ctypes.c_int, [_f32p, _i64, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                          ctypes.c_void_p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                          _f32p, _f32p, _f32p, _f32p, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_apply_residual': (ctypes.c_int, [_f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_bn_backward_masked': (ctypes.c_int, [_f32p, _f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p,
                                              _f32p, _f32p, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_torus_conv_wgrad': (ctypes.c_int, [_f32p, _f32p, _i64, _i64, _i64, _i64, _i64, _f32p, _f32p,
                                            ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_torus_conv_wgrad_bn': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p,
                                               ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                               ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_bn_backward_masked_coefs': (ctypes.c_int, [_f32p, _f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p,
                                                    _f32p, _f32p, _f32p, _f32p, ctypes.c_void_p, _i64,
                                                    ctypes.c_void_p]),
    'hrl_torus_unit_forward': (ctypes.c_int, [_f32p, _f32p, _f32p, _f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p,
                                              _f32p, ctypes.c_void_p, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_torus_unit_input_grad': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p, _f32p, _f32p,
                                                 _f32p, _f32p, ctypes.c_void_p, ctypes.c_void_p, _i64,
                                                 ctypes.c_void_p]),
    'hrl_board_conv_workspace_bytes': (ctypes.c_int64, [_i64]),
    'hrl_board_conv_forward': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, _f32p, _i64, _i64, _i64, _f32p, _f32p,
                                              ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_board_conv_pack': (ctypes.c_int, [_f32p, _i64, _i64, _i64, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_board_conv_forward_packed': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, ctypes.c_void_p, _i64, _f32p,
                                                     _f32p, ctypes.c_void_p]),
    'hrl_gboard_pack_bytes': (ctypes.c_int64, [_i64, _i64]),
    'hrl_gboard_pack': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_gboard_pack_adjoint': (ctypes.c_int, [_f32p, _i64, _i64, _i64, _i64, ctypes.c_void_p, _i64,
                                               ctypes.c_void_p]),
    'hrl_gboard_wgrad_workspace_bytes': (ctypes.c_int64, [_i64, _i64, _i64]),
    'hrl_gboard_wgrad': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int, _i64, _i64, _f32p, _i64, _i64, _f32p,
                                        ctypes.c_void_p, _i64, ctypes.c_void_p]),
    'hrl_gboard_set_whole_ring': (ctypes.c_int, [ctypes.c_int]),
    'hrl_gboard_set_nctw': (ctypes.c_int, [ctypes.c_int]),
    'hrl_gboard_launch_stats': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    'hrl_gboard_pointwise_wgrad_workspace_bytes': (_i64, [_i64, _i64, _i64]),
    'hrl_gboard_pointwise_wgrad': (ctypes.c_int, [_f32p, _i64, _f32p, _i64, _i64, _i64, _i64, _f32p, ctypes.c_void_p,
                                                  _i64, ctypes.c_void_p]),
    'hrl_gboard_forward_groups': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, _i64, _i64, _i64, ctypes.c_void_p,
                                                 _i64, _i64, _f32p, _i64, ctypes.c_void_p]),
    'hrl_lstm_gates_backward_ex': (ctypes.c_int, [_f32p, _f32p, _f32p, _f32p, _i64, ctypes.c_int, _i64, _f32p, _i64,
                                                  _i64, _i64, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_void_p]),
    'hrl_lstm_gates_forward_grouped': (ctypes.c_int, [ctypes.c_int, _f32p, _i64, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, _i64, _i64, _i64, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_gboard_forward': (ctypes.c_int, [_f32p, _i64, _f32p, _i64, _i64, _i64, _i64, ctypes.c_void_p, _i64, _i64,
                                          _f32p, _f32p, _f32p, ctypes.c_int, _f32p, _i64, ctypes.c_void_p]),
    'hrl_gboard_pointwise': (ctypes.c_int, [_f32p, _i64, _i64, _f32p, _i64, _i64, _i64, _f32p, _i64, _f32p, _f32p,
                                            ctypes.c_int, _f32p, _i64, ctypes.c_void_p]),
    'hrl_torus_head_pool': (ctypes.c_int, [_f32p, _f32p, _i64, _i64, _i64, _i64, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_torus_head_unpool': (ctypes.c_int, [_f32p, _f32p, _f32p, _i64, _i64, _i64, _i64, _f32p,
                                             ctypes.c_void_p]),
    'hrl_bn_backward_apply_masked': (ctypes.c_int, [_f32p, _f32p, _f32p, _i64, _i64, _i64, _f32p, _f32p, _f32p,
                                                    _f32p, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_geister_legal': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _i64, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    'hrl_geister_observation': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               _i64, ctypes.c_int, _f32p, _f32p, ctypes.c_void_p]),
    'hrl_geister_step': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, _i64, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_selfplay_sample_record': (ctypes.c_int, [_f32p, _i64, ctypes.c_void_p, _f32p, ctypes.c_void_p, _f32p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _i64, _i64,
                                                  _i64, _i64, ctypes.c_void_p, _f32p, _f32p, ctypes.c_void_p, _f32p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'hrl_masked_rows_copy': (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _i64,
                                            ctypes.c_void_p]),
    'hrl_geister_observation_record': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, _i64, ctypes.c_int, _f32p, _f32p,
                                                      ctypes.c_void_p, ctypes.c_void_p, _i64, _f32p, _f32p,
                                                      ctypes.c_void_p]),
}

ABI_VERSION = 26

_lib = None


def load():
    """Load libhrl.so (once) and bind every signature; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError('HIP library %s is missing: run `python -m handyrl_amd.build` '
                           '(there is no CPU fallback for the learner kernels)' % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.hrl_abi_version() != ABI_VERSION:
        raise RuntimeError('libhrl.so ABI %d != expected %d' % (lib.hrl_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(code, what):
    if code != HRL_OK:
        msg = load().hrl_strerror(code).decode()
        if code == HRL_EINVAL:
            raise ValueError('%s: %s' % (what, msg))
        raise RuntimeError('%s failed (%d): %s' % (what, code, msg))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def ptr_array(tensors):
    """A C array of device pointers (None -> NULL) for the multi-tensor entry points."""
    arr = (ctypes.c_void_p * len(tensors))(*[None if t is None else t.data_ptr() for t in tensors])
    return arr


def i64_array(values):
    return (ctypes.c_int64 * len(values))(*values)


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
