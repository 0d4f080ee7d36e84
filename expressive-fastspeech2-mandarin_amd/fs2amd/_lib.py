"""ctypes binding of libfs2hip.so (the C ABI declared in include/fs2hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950)
into ``fs2amd/_lib/libfs2hip.so``; ``FS2_LIB`` overrides the path. There is no CPU fallback:
if the library is missing the import of :mod:`fs2amd.ops` raises.

``import torch`` must happen before the library is loaded so that its libamdhip64.so.7
resolves (by SONAME) to the HIP runtime torch already mapped: one runtime per process.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first)

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(HERE, "_lib", "libfs2hip.so")

FS2_F32, FS2_BF16, FS2_FP8 = 0, 1, 2
FS2_OK, FS2_EINVAL, FS2_ELAUNCH, FS2_EUNSUPPORTED = 0, 1, 2, 3
(EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_TANH, EPI_BIAS_RES, EPI_RES_LN, EPI_RELU_LN, EPI_RELU_LN_DOT, EPI_BIAS_LRELU,
 EPI_RES_SUM, EPI_RELU_GRAD) = range(10)
DUR_I64, DUR_F32, DUR_LOGPRED = 0, 1, 2

_p = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float


class PackDesc(ctypes.Structure):
    """Mirror of ``fs2_pack_desc`` (include/fs2hip.h)."""

    _fields_ = [("src", _p), ("fwd", _p), ("tr", _p), ("N", _i), ("C", _i), ("KS", _i), ("n_off", _i),
                ("N_tot", _i), ("f32_copy", _i), ("C_tot", _i), ("tiles_c", _i), ("blk0", _i)]


class LossArgs(ctypes.Structure):
    """Mirror of ``fs2_loss_args`` (include/fs2hip.h)."""

    _fields_ = [("mel", _p), ("postnet", _p), ("mel_tgt", _p), ("tgt_bs", _i64), ("tgt_ts", _i64), ("mel_valid", _p),
                ("B", _i), ("T", _i), ("n_mel", _i), ("p_pred", _p), ("p_tgt", _p), ("p_mask", _p), ("n_p", _i64),
                ("e_pred", _p), ("e_tgt", _p), ("e_mask", _p), ("n_e", _i64), ("logd_pred", _p), ("d_tgt", _p),
                ("d_mask", _p), ("n_d", _i64)]


class AdamParam(ctypes.Structure):
    """Mirror of ``fs2_adam_param`` (include/fs2hip.h)."""

    _fields_ = [("p", _p), ("m", _p), ("v", _p), ("step", _p), ("off", _i64), ("numel", _i64)]


class ReduceDesc(ctypes.Structure):
    """Mirror of ``fs2_reduce_desc`` (include/fs2hip.h)."""

    _fields_ = [("part", _p), ("M", _i64), ("S", _i), ("kind", _i), ("KS", _i), ("N", _i), ("C", _i), ("split", _i),
                ("accumulate", _i), ("pad_", _i), ("out0", _p), ("out1", _p), ("out2", _p), ("blk0", _i64)]


REDUCE_BATCH_MAX = 32


class ReduceBatch(ctypes.Structure):
    """Mirror of ``fs2_reduce_batch`` (include/fs2hip.h)."""

    _fields_ = [("n", _i), ("pad_", _i), ("d", ReduceDesc * REDUCE_BATCH_MAX)]


class ConvDesc(ctypes.Structure):
    """Mirror of ``fs2_conv_desc`` (include/fs2hip.h)."""

    _fields_ = [
        ("x", _p), ("x_dtype", _i), ("x_row_stride", _i64),
        ("w", _p), ("bias", _p),
        ("B", _i), ("T", _i), ("Cin", _i), ("Cin_pad", _i), ("N", _i), ("KS", _i), ("pad", _i),
        ("compute", _i), ("epilogue", _i),
        ("residual", _p), ("res_dtype", _i), ("res_row_stride", _i64),
        ("ln_gamma", _p), ("ln_beta", _p), ("ln_eps", _f),
        ("lens", _p), ("addvec1", _p), ("addvec2", _p),
        ("dot_w", _p), ("dot_b", _f),
        ("out", _p), ("out_dtype", _i), ("out_row_stride", _i64),
        ("rows_dev", _p), ("row_pos", _p), ("a_rowmap", _p),
        ("col_scale", _p), ("out_scale", _f), ("out2", _p), ("out2_scale", _f),
        ("cin_block", _i), ("cin_src", _i * 4), ("out_split", _i),
        ("splitk_ws", _p), ("splitk_ws_bytes", _i64),
        ("dilation", _i), ("act_slope", _f), ("out2_act", _i), ("out2_slope", _f), ("out2_f32", _i),
        ("residual2", _p), ("out_div", _f),
        ("group_n", _i), ("group_cin", _i),
    ]


class Ffn8Desc(ctypes.Structure):
    """Mirror of ``fs2_ffn8_desc`` (include/fs2hip.h)."""

    _fields_ = [
        ("x8", _p), ("x8_row_stride", _i64), ("res", _p), ("res_row_stride", _i64), ("w", _p),
        ("cs1", _p), ("b1", _p), ("inv_sf", _f), ("cs2", _p), ("b2", _p),
        ("B", _i), ("T", _i), ("D", _i), ("F", _i), ("KS", _i), ("pad", _i),
        ("ln_gamma", _p), ("ln_beta", _p), ("ln_eps", _f),
        ("out", _p), ("out_row_stride", _i64), ("out8", _p), ("out8_row_stride", _i64), ("out8_scale", _f),
        ("rows_dev", _p), ("row_pos", _p), ("rows_max", _i),
    ]


class WconvDesc(ctypes.Structure):
    """Mirror of ``fs2_wconv_desc`` (include/fs2hip.h)."""

    _fields_ = [
        ("x", _p), ("x_row_stride", _i64), ("w", _p), ("bias", _p),
        ("B", _i), ("T", _i), ("Cin", _i), ("N", _i), ("KS", _i), ("pad", _i), ("epilogue", _i),
        ("out", _p), ("out_row_stride", _i64), ("w2", _p), ("bias2", _p), ("residual", _p), ("res_row_stride", _i64),
        ("rows_dev", _p), ("row_pos", _p), ("rows_max", _i),
    ]


class CondDesc(ctypes.Structure):
    """Mirror of ``fs2_cond_desc`` (include/fs2hip.h)."""

    _fields_ = [
        ("speakers", _p), ("speaker_table", _p), ("n_speaker", _i), ("emotions", _p), ("emo_table", _p),
        ("n_emo", _i), ("d_emo", _i), ("arousals", _p), ("aro_table", _p), ("n_aro", _i), ("d_aro", _i),
        ("valences", _p), ("val_table", _p), ("n_val", _i), ("d_val", _i), ("lin_w", _p), ("lin_b", _p),
        ("spk_out", _p), ("emo_out", _p),
    ]


class CondGrads(ctypes.Structure):
    """Mirror of ``fs2_cond_grads`` (include/fs2hip.h)."""

    _fields_ = [("d_speaker_table", _p), ("d_emo_table", _p), ("d_aro_table", _p), ("d_val_table", _p),
                ("d_lin_w", _p), ("d_lin_b", _p)]


class FfnDesc(ctypes.Structure):
    """Mirror of ``fs2_ffn_desc`` (include/fs2hip.h)."""

    _fields_ = [
        ("x", _p), ("x_row_stride", _i64),
        ("w", _p), ("b1", _p), ("b2", _p),
        ("B", _i), ("T", _i), ("D", _i), ("F", _i), ("KS", _i), ("pad", _i),
        ("ln_gamma", _p), ("ln_beta", _p), ("ln_eps", _f),
        ("lens", _p), ("addvec1", _p), ("addvec2", _p),
        ("out", _p), ("out_row_stride", _i64),
        ("rows_dev", _p), ("row_pos", _p),
        ("nsplit", _i), ("splitk_ws", _p), ("splitk_ws_bytes", _i64), ("rows_max", _i),
        ("tile_rows", _i),
        ("wqkv", _p), ("bqkv", _p), ("qkv_out", _p), ("qkv_row_stride", _i64), ("nqkv", _i),
        ("pre_att", _p), ("pre_att_row_stride", _i64), ("pre_w", _p), ("pre_b", _p), ("pre_gamma", _p),
        ("pre_beta", _p), ("pre_eps", _f),
    ]


class VpFusedDesc(ctypes.Structure):
    """Mirror of ``fs2_vp_fused_desc`` (include/fs2hip.h)."""

    _fields_ = [
        ("x", _p), ("x_row_stride", _i64), ("w", _p), ("vec", _p), ("lin_b", _p), ("ln_eps", _f),
        ("B", _i), ("L", _i), ("G", _i), ("lens", _p), ("pred", _p), ("embed_group", _i),
        ("x_out", _p), ("x_out_row_stride", _i64), ("target", _p), ("control", _f), ("bins", _p),
        ("n_bins", _i), ("table", _p),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "fs2_version": (ctypes.c_char_p, []),
    "fs2_build_id": (ctypes.c_char_p, []),
    "fs2_status_string": (ctypes.c_char_p, [_i]),
    "fs2_conv_cin_pad": (_i, [_i, _i]),
    "fs2_conv1d": (_i, [ctypes.POINTER(ConvDesc), _p]),
    "fs2_ffn": (_i, [ctypes.POINTER(FfnDesc), _p]),
    "fs2_ffn_wide": (_i, [ctypes.POINTER(FfnDesc), _p, ctypes.c_int64, _p]),
    "fs2_ffn_weight_elems": (ctypes.c_int64, [_i, _i]),
    "fs2_ffn8": (_i, [ctypes.POINTER(Ffn8Desc), _p]),
    "fs2_ffn8_weight_bytes": (ctypes.c_int64, [_i, _i]),
    "fs2_wconv": (_i, [ctypes.POINTER(WconvDesc), _p]),
    "fs2_wconv_weight_elems": (ctypes.c_int64, [_i, _i, _i]),
    "fs2_attention": (_i, [_p, _i, _i64, _p, _i, _i, _i, _i, _f, _p, _i64, _p, _p, _p]),
    "fs2_attention_ex": (_i, [_p, _i, _i64, _p, _i, _i, _i, _i, _f, _p, _i64, _p, _p, _i, _p, _i64, _i64, _p]),
    "fs2_attention_split_ws_bytes": (_i64, [_i, _i, _i, _i64]),
    "fs2_attention_items": (_i, [_p, _i, _i, _i, _p, _i64, _i64, _p]),
    "fs2_embed_pe": (_i, [_p, _p, _i, _p, _i, _i, _i, _p, _i, _p, _p]),
    "fs2_attention_bwd": (_i, [_p, _i, _i64, _p, _i64, _p, _i64, _p, _i, _i, _i, _i, _f, _p, _i64, _p, _p, _i64, _p,
                               _p]),
    "fs2_cond_vectors": (_i, [_p, _p, _i, _p, _p, _i, _i, _p, _p, _i, _i, _p, _p, _i, _i, _p, _p, _i, _i, _p, _p,
                              _p]),
    "fs2_variance_embed": (_i, [_p, _i, _p, _p, _f, _p, _i, _p, _i, _i, _p]),
    "fs2_variance_embed_ex": (_i, [_p, _i, _p, _p, _i, _p, _i, _i, _p, _p, _p]),
    "fs2_lr_backward": (_i, [_p, _p, _i, _i, _i, _i, _p, _p]),
    "fs2_lr_durations": (_i, [_p, _i, _f, _i, _i, _p, _p, _p, _p]),
    "fs2_lr_expand": (_i, [_p, _i, _p, _p, _i, _i, _i, _i, _p, _p, _i, _p, _p, _p]),
    "fs2_pack_rows": (_i, [_p, _i, _p, _p, _i, _p, _p, _i64, _p]),
    "fs2_postnet_assemble": (_i, [_p, _p, _p, _i, _i, _i, _p, _p, _i, _p, _p]),
    "fs2_seq_layout_margin": (_i, [_p, _i, _i, _i, _p, _p, _p, _p]),
    "fs2_len_stats": (_i, [_p, _i, _p, _p, _p]),
    "fs2_seq_layout": (_i, [_p, _i, _i, _p, _p, _p, _p]),
    "fs2_vp_norm": (_i, [_p, _i64, _i, _i, _i, _p, _p, _f, _p, _i64, _p]),
    "fs2_vp_head": (_i, [_p, _i64, _i, _i, _i, _i, _p, _p, _f, _p, _p, _p, _p, _i, _p, _i, _i64, _i, _p, _f, _p, _i, _p,
                         _p]),
    "fs2_vp_fused": (_i, [ctypes.POINTER(VpFusedDesc), _p]),
    "fs2_vp_fused_weight_elems": (ctypes.c_int64, [_i]),
    "fs2_lr_fused": (_i, [_p, _i, _p, _i, _f, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "fs2_enc_attn_block": (_i, [_p, _p, _i, _i, _p, _p, _p, _p, _p, _p, _f, _i, _i, _f, _p, _p, _i64, _p]),
    "fs2_enc_embed_attn_block": (_i, [_p, _p, _i, _p, _p, _p, _i, _i, _p, _p, _p, _p, _p, _p, _f, _i, _i, _f, _p, _p, _p,
                                      _i, _p, _p, _p, _i64, _p]),
    "fs2_lr_fused_proj": (_i, [_p, _i, _p, _i, _f, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p,
                               _p, _p, _i, _p, _p]),
    "fs2_hifigan_mrf": (_i, [_p, _p, _p, _p, _i, _i, _i, _f, _p, _p]),
    "fs2_hifigan_mrf_weight_elems": (ctypes.c_int64, [_i]),
    "fs2_hifigan_pair": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _f, _f, _i, _p, _p]),
    "fs2_hifigan_post": (_i, [_p, _p, _f, _i, _i, _i, _i, _p, _p]),
    "fs2_res_ln_fwd": (_i, [_p, _p, _i, _p, _p, _p, _i64, _i, _i, _f, _f, _p, _i, _p, _p, _p, _p, _p]),
    "fs2_res_ln_bwd_ws_bytes": (_i64, [_i]),
    "fs2_pack_train_plan": (_i, [_p, _i, _p]),
    "fs2_pack_train": (_i, [_p, _i, _i, _p]),
    "fs2_res_ln_bwd": (_i, [_p, _p, _p, _p, _p, _i64, _i, _i, _f, _p, _i, _p, _p, _p, _p, _p, _i, _i, _p, _i64, _p]),
    "fs2_relu_ln_fwd": (_i, [_p, _p, _p, _i64, _i, _f, _f, _p, _i, _p, _p, _p, _p, _p]),
    "fs2_relu_ln_bwd": (_i, [_p, _p, _p, _p, _p, _i64, _i, _f, _p, _i, _p, _p, _p, _p, _i, _i, _p, _i64, _p]),
    "fs2_relu_ln_head_fwd": (_i, [_p, _p, _p, _i64, _i, _f, _f, _p, _i, _p, _p, _p, _p, _p, _p, _p, _p]),
    "fs2_relu_ln_head_bwd_ws_bytes": (_i64, [_i]),
    "fs2_relu_ln_head_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _f, _p, _i, _p, _p, _p, _p, _p, _p, _i, _i,
                                  _p, _i64, _p]),
    "fs2_embedding_bwd": (_i, [_p, _i64, _p, _i64, _i, _i, _i, _p, _i, _p]),
    "fs2_loss_ws_bytes": (_i64, []),
    "fs2_loss_fwd": (_i, [_p, _p, _p, _p, _i64, _p]),
    "fs2_loss_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "fs2_bn_train_ws_bytes": (_i64, [_i]),
    "fs2_bn_train_fwd": (_i, [_p, _i64, _i, _p, _p, _f, _f, _p, _p, _i, _f, _p, _i, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "fs2_bn_train_bwd": (_i, [_p, _p, _i64, _i, _p, _p, _p, _p, _i, _f, _p, _i, _p, _p, _p, _i, _p, _i64, _p]),
    "fs2_adam_ws_bytes": (_i64, []),
    "fs2_adam_flat": (_i, [_p, _i64, _p, _i, _p, _f, _f, _f, _f, _f, _f, _p, _i64, _p]),
    "fs2_colsum_ws_bytes": (_i64, [_i]),
    "fs2_colsum": (_i, [_p, _i, _i64, _i, _i64, _p, _i, _p, _i64, _p]),
    "fs2_conv_wgrad_ws_bytes": (_i64, [_i, _i, _i, _i, _i]),
    "fs2_conv_wgrad": (_i, [_p, _i, _i64, _p, _i64, _i, _i, _i, _i, _i, _i, _p, _p, _i, _i, _p, _p, _p, _p, _i, _p,
                            _i64, _p]),
    "fs2_conv_wgrad_splits": (_i, [_i, _i, _i, _i, _i]),
    "fs2_ln_bwd_parts": (_i, [_i64]),
    "fs2_reduce_batch_launch": (_i, [_p, _p]),
    "fs2_cond_bwd_ws_bytes": (_i64, [_i, _i]),
    "fs2_cond_bwd": (_i, [_p, _i, _i, _i, _p, _p, _p, _i64, _p]),
    "fs2_length_masks": (_i, [_p, _i, _i, _p, _p]),
    "fs2_length_regulate": (_i, [_p, _i, _p, _i, _f, _i, _i, _i, _i, _p, _p, _i, _p, _p, _p, _p, _p]),
}


def header_symbols(header_path):
    """Every ``fs2_*`` function declared in include/fs2hip.h (for the export test)."""
    import re

    text = open(header_path).read()
    return sorted(set(re.findall(r"\b(fs2_[a-z0-9_]+)\s*\(", text)) - {"fs2_conv_desc"})


_LIB = None
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "fs2hip.h")


def source_build_id(csrc=CSRC, header=HEADER):
    """sha256 (first 16 hex digits) of csrc/*.hip, csrc/*.h and include/fs2hip.h, in name order:
    the id __graft_entry__.build_hip embeds as fs2_build_id(). None when the sources are absent."""
    import hashlib

    if not os.path.isdir(csrc) or not os.path.exists(header):
        return None
    h = hashlib.sha256()
    for name in sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h"))):
        h.update(name.encode())
        with open(os.path.join(csrc, name), "rb") as f:
            h.update(f.read())
    with open(header, "rb") as f:
        h.update(b"fs2hip.h")
        h.update(f.read())
    return h.hexdigest()[:16]


def lib_path():
    return os.environ.get("FS2_LIB", DEFAULT_LIB)


def load():
    """Load (once) and return the ctypes library; raises if it was not built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError(
            f"fs2amd: HIP library not found at {path}. Build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    # FS2_LIB_ALLOW_MISSING=1 (A/B runs against an older library build only): skip entry points
    # the override library does not export; calling one of them then raises AttributeError.
    allow_missing = "FS2_LIB" in os.environ and os.environ.get("FS2_LIB_ALLOW_MISSING") == "1"
    for name, (res, args) in SIGNATURES.items():
        if allow_missing and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # provenance: the default in-tree library must have been built from the sources beside it
    # (FS2_LIB overrides are A/B builds of other trees and are not checked)
    if "FS2_LIB" not in os.environ:
        want = source_build_id()
        got = lib.fs2_build_id().decode()
        if want is not None and got != want:
            raise RuntimeError(f"fs2amd: {path} was built from other sources (fs2_build_id {got}, sources "
                               f"{want}); rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    _LIB = lib
    return lib


def check(rc, what):
    if rc != FS2_OK:
        msg = load().fs2_status_string(rc).decode()
        raise RuntimeError(f"{what} failed: fs2 status {rc} ({msg})")
