"""ctypes binding of libcrnn_hip.so (include/crnn_hip.h).

The product path is the HIP library; there is no CPU or eager-PyTorch fallback.
If the shared object is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# CRNN_HIP_LIB: an alternative build of the same library (tuning A/B runs)
LIB_PATH = os.environ.get("CRNN_HIP_LIB", os.path.join(HERE, "libcrnn_hip.so"))
CSRC = os.path.join(PKG, "csrc")

F32, BF16 = 0, 1
F32_BF16MMA = 2   # gemm_nt / nn / tn: fp32 operands, bf16 MFMA, fp32 out (include/crnn_hip.h)

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_long
f32 = C.c_float
u64 = C.c_ulonglong
sz = C.c_size_t


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("B", "Hi", "Wi", "Ci", "Ho", "Wo", "Co", "KH", "KW", "sh", "sw", "ph", "pw", "Ci_real")]


class BnBwdDesc(C.Structure):
    _fields_ = [("dy", vp), ("z", vp), ("mean", vp), ("invstd", vp), ("scale", vp), ("shift", vp),
                ("y", vp), ("s", vp), ("dpool", vp), ("mode", C.c_int), ("M", C.c_long),
                ("C", C.c_int), ("HW", C.c_int)]


class PackJob(C.Structure):  # crnn_pack_job
    _fields_ = [("kind", C.c_int), ("out_f32", C.c_int), ("a", C.c_int), ("b", C.c_int), ("c", C.c_int),
                ("d", C.c_int), ("e", C.c_int), ("pad_", C.c_int), ("start", C.c_long), ("src", vp),
                ("src2", vp), ("perm", vp), ("dst", vp), ("dst2", vp)]


# crnn_set_option keys (include/crnn_hip.h)
(OPT_GEMM_STAGGER, OPT_GEMM_PERSISTENT, OPT_DEEP_LINEAR, OPT_WGRAD_TILE, OPT_LSTM_TILE, OPT_HALO_CONV, OPT_LSTM_HANDOFF,
 OPT_WGRAD_REDUCE, OPT_WGRAD_FAST, OPT_ROW_CLASS, OPT_QUANT_TILE, OPT_PAD_SKIP, OPT_LSTM_BWD_PART,
 OPT_LSTM_L2_HANDOFF, OPT_GEMM4W, OPT_DIAG, OPT_DGRAD_GROUP, OPT_FIN_TICKET,
 OPT_CONV_HALO_W, OPT_LSTM_PIPE, OPT_LINEAR_ROW8, OPT_HALO_ROW16, OPT_HALO_WG2, OPT_WGRAD_SLAB_BF16) = range(24)

PACK_CONV, PACK_ROWS, PACK_ROWS_SUM, PACK_TRANSPOSE, PACK_CONV_T = 0, 1, 2, 3, 4

_SIGS = {
    "crnn_pack_batch": ([i32, vp, i32, i64, vp], i32),
    "crnn_pack_conv_batch": ([i32, vp, i32, i64, i32, vp], i32),
    "crnn_pack_conv_t_batch": ([i32, vp, i32, i64, vp], i32),
    "crnn_pack_conv_t_tiles": ([i32, i32], i32),
    "crnn_version": ([], i32),
    "crnn_set_option": ([i32, i32], i32),
    "crnn_get_option": ([i32], i32),
    "crnn_last_error_string": ([], C.c_char_p),
    "crnn_nchw_to_nhwc": ([i32, vp, vp, i32, i32, i32, i32, i32, vp], i32),
    "crnn_cast_f32": ([i32, vp, vp, i64, vp], i32),
    "crnn_dropout": ([i32, vp, vp, i64, f32, C.c_ulonglong, vp], i32),
    "crnn_dropblock_mask": ([vp, vp, i32, i32, i32, i32, f32, i32, C.c_ulonglong, vp], i32),
    "crnn_dropblock_apply": ([i32, vp, vp, vp, vp, i64, vp], i32),
    "crnn_pack_conv_weight": ([i32, vp, vp, i32, i32, i32, i32, i32, vp], i32),
    "crnn_pack_rows": ([i32, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_conv_fwd": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, vp], i32),
    "crnn_conv_fwd_bnrelu_supported": ([i32, C.POINTER(ConvDesc)], i32),
    "crnn_conv_fwd_bnrelu": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, vp], i32),
    "crnn_conv_fwd_bnrelu_pool_supported": ([i32, C.POINTER(ConvDesc)], i32),
    "crnn_conv_fwd_bnrelu_pool": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, vp], i32),
    "crnn_conv_fwd_tile": ([i32, C.POINTER(ConvDesc), C.POINTER(C.c_int), C.POINTER(C.c_int)], None),
    "crnn_conv_wgrad_plan": ([i32, C.POINTER(ConvDesc), C.POINTER(C.c_int), C.POINTER(C.c_int),
                              C.POINTER(C.c_int)], None),
    "crnn_conv_stat_rows": ([i32, C.POINTER(ConvDesc)], i32),
    "crnn_conv_stat_rows_per_partial": ([i32, C.POINTER(ConvDesc)], i32),
    "crnn_conv_dgrad": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, i32, vp], i32),
    "crnn_conv_dgrad_ds_supported": ([i32, C.POINTER(ConvDesc), C.POINTER(ConvDesc)], i32),
    "crnn_conv_dgrad_ds": ([i32, C.POINTER(ConvDesc), C.POINTER(ConvDesc), vp, vp, vp, vp], i32),
    "crnn_conv_dgrad_bnrelu_rows": ([i32, C.POINTER(ConvDesc)], i32),
    "crnn_conv_dgrad_tw_rows": ([i32, C.POINTER(ConvDesc)], i32),
    "crnn_conv_dgrad_tw": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, i32, vp], i32),
    "crnn_conv_dgrad_bnrelu_tw": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "crnn_conv_dgrad_bnrelu": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "crnn_conv_wgrad": ([i32, C.POINTER(ConvDesc), vp, vp, vp, vp, sz, f32, vp], i32),
    "crnn_conv_wgrad_workspace": ([i32, C.POINTER(ConvDesc)], sz),
    "crnn_conv_wgrad_gemm": ([i32, C.POINTER(ConvDesc), vp, vp, vp, sz, vp], i32),
    "crnn_conv_wgrad_reduce": ([i32, C.POINTER(ConvDesc), vp, vp, sz, f32, vp], i32),
    "crnn_bn_finalize": ([vp, vp, i32, i64, i32, i64, vp, vp, vp, vp, f32, f32, i32, vp, vp, vp, vp, vp, vp], i32),
    "crnn_bn_finalize_workspace": ([i32], sz),
    "crnn_channel_stats": ([i32, vp, i64, i32, vp, vp, i32, vp], i32),
    "crnn_bn_act": ([i32, vp, vp, vp, vp, i64, i32, i32, vp], i32),
    "crnn_bn_relu_maxpool": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_maxpool_bwd": ([i32, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_bn_bwd_reduce": ([i32, C.POINTER(BnBwdDesc), vp, vp, i32, vp], i32),
    "crnn_bn_bwd_finalize": ([vp, vp, i32, i32, i64, vp, vp, vp, vp, i32, vp, vp], i32),
    "crnn_bn_bwd_apply": ([i32, C.POINTER(BnBwdDesc), vp, vp, vp, vp], i32),
    "crnn_bn_rows": ([i64], i32),
    "crnn_se_pool": ([i32, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_pool_partials": ([vp, i32, i64, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_bn_bwd_reduce": ([i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_bn_partials": ([vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_mlp_fwd": ([vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_pool_mlp_fwd": ([vp, i32, i64, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_se_residual_fwd": ([i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_residual_drop_fwd": ([i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, vp], i32),
    "crnn_se_bwd_reduce": ([i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_se_mlp_bwd": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp], i32),
    "crnn_se_mlp_bwd_partials": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
                                 i32),
    "crnn_hpool_fwd": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_hpool_bwd": ([i32, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_gemm_nt": ([i32, vp, i32, vp, i32, vp, i32, vp, i32, i32, i32, i32, i32, vp], i32),
    "crnn_gemm_nn": ([i32, vp, i32, vp, i32, vp, i32, i32, i32, i32, i32, i32, vp], i32),
    "crnn_gemm_tn": ([i32, vp, i32, vp, i32, vp, i32, i32, i32, i32, i32, vp], i32),
    "crnn_gemm_tn_workspace": ([i32, i32, i32], sz),
    "crnn_gemm_tn_slab": ([vp, i32, vp, i32, vp, i32, i32, i32, i32, i32, vp, sz, vp], i32),
    "crnn_colsum": ([i32, vp, i32, i64, i32, vp, i32, i32, vp], i32),
    "crnn_lstm_step_fwd": ([i32, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_lstm_step_bwd": ([i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_lstm_bptt_workspace": ([i32, i32], sz),
    "crnn_lstm_dwhh": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_lstm_dwih": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp], i32),
    "crnn_lstm_dbias": ([i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_lstm_dbias_workspace": ([i32], sz),
    "crnn_lstm_seq_supported": ([i32, i32, i32], i32),
    "crnn_lstm_seq_workspace": ([i32], sz),
    "crnn_lstm_seq_time_next": ([vp, vp], i32),
    "crnn_lstm_seq_status_offset": ([i32], sz),
    "crnn_lstm_seq_config": ([i32, i32, i32, vp, vp], i32),
    "crnn_lstm_seq_debug_stamps": ([vp], i32),
    "crnn_lstm_seq_fwd": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_lstm_seq_bwd": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp], i32),
    "crnn_lstm_wgrad_workspace": ([i32, i32, i32, i32], sz),
    "crnn_lstm_wgrad": ([vp, vp, vp, vp, vp, vp, vp, vp, sz, i32, i32, i32, i32, i32, vp], i32),
    "crnn_lstm_dx": ([i32, vp, vp, vp, i32, i32, i32, i32, vp], i32),
    "crnn_attn_context": ([vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, f32, u64, vp], i32),
    "crnn_attn_context_bf16": ([vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, f32, u64, vp], i32),
    "crnn_attn_cell": ([vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, i32, vp, i32, vp, vp, i32, i32, i32, vp], i32),
    "crnn_attn_cell_bwd": ([vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, i32, i32, vp], i32),
    "crnn_attn_gates_cell": ([i32, vp, i32, vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, i32, vp, vp, i32, i32,
                              i32, vp], i32),
    "crnn_attn_bwd": ([vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, u64, vp], i32),
    "crnn_attn_bwd_bf16": ([vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, u64, vp], i32),
    "crnn_attn_denc": ([vp, i32, vp, i32, i32, i32, i32, f32, u64, vp, vp], i32),
    "crnn_attn_dproj_enc": ([vp, vp, vp, vp, i32, i32, i32, i32, vp, vp], i32),
    "crnn_attn_dproj_enc_bf16": ([vp, vp, vp, vp, i32, i32, i32, i32, vp, vp], i32),
    "crnn_attn_onehot_rows": ([vp, i32, i32, i32, i32, vp, i32, i32, vp], i32),
    "crnn_attn_out": ([vp, i32, i32, i32, i32, vp, i32, vp, vp], i32),
    "crnn_preprocess": ([vp, vp, i32, i32, i32, i32, i32, vp, vp, i64, vp], i32),
    "crnn_preprocess_workspace": ([i32, i32, i32], i64),
    "crnn_attn_xent": ([vp, i32, vp, i32, i32, i32, vp, vp, i32, vp, vp], i32),
    "crnn_ctc_loss": ([vp, i32, i32, i32, i32, vp, i32, vp, vp, vp, i32, vp], i32),
    "crnn_ctc_reduce_mean": ([vp, vp, i32, vp, vp], i32),
    "crnn_ctc_greedy": ([vp, i32, i32, i32, i32, vp, vp, vp], i32),
    "crnn_adamw": ([vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, i32, f32, vp], i32),
    "crnn_adam_step": ([vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, i32, f32, i32, vp, vp], i32),
    "crnn_sgd_step": ([vp, vp, vp, i64, f32, f32, f32, f32, i32, vp, vp], i32),
}

_lib = None


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile libcrnn_hip.so for gfx950 with hipcc (in-tree)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], check=True)
    else:
        subprocess.run(["make", "-C", CSRC, f"-j{jobs}", "-q"], check=False)
        r = subprocess.run(["make", "-C", CSRC, "-q"], check=False)
        if r.returncode != 0:
            subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib():
    """Load (once) and return the ctypes handle. Raises if the library is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libcrnn_hip.so not built ({LIB_PATH}); run crnn_hip._lib.build() "
                               "or `make -C rcnn-ocr_amd/csrc`")
        h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (args, res) in _SIGS.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = res
        _lib = h
    return _lib


def source_hash() -> str:
    """sha256 (16 hex digits) over the sources that decide what the bench's kernels do: the HIP
    sources, the C header, the host package (rcnn-ocr_amd/**/*.py) and bench.py. Measured-counter
    files (profiles/*_pmc_traffic.json) carry the hash of the tree they were taken on; bench.py
    attaches them only when it equals the running tree's (no git on the GPU box)."""
    import hashlib
    repo = os.path.dirname(PKG)
    files = []
    for root, dirs, names in os.walk(PKG):
        dirs[:] = sorted(d for d in dirs if d != "__pycache__")
        for n in sorted(names):
            if n.endswith((".hip", ".hpp", ".cpp", ".h", ".py")) or n == "Makefile":
                files.append(os.path.join(root, n))
    files += [os.path.join(repo, "include", "crnn_hip.h"), os.path.join(repo, "bench.py")]
    h = hashlib.sha256()
    for f in files:
        if os.path.exists(f):
            h.update(os.path.relpath(f, repo).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def exported_symbols():
    return list(_SIGS.keys())


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().crnn_last_error_string()
        raise RuntimeError(f"{what} failed (hip error {rc}): {msg.decode() if msg else ''}")


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    check(rc, name)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    if t is None:
        return None
    return t.data_ptr()


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float32:
        return F32
    raise ValueError(f"unsupported compute dtype {dt}")


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise RuntimeError("crnn_hip ops run only on a HIP device (no CPU fallback); got a CPU tensor")
