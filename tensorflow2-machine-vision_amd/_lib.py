"""ctypes binding of libedet.so (the C-ABI declared in include/edet.h).

This is the only module that touches the shared library.  Every entry point returns an int
status; non-zero raises ``EdetError`` carrying ``edet_last_error()``.  There is no fallback:
if the library is missing the import of the package's compute modules fails loudly.
"""
from __future__ import annotations

import ctypes
import os

# libedet.so links libamdhip64.so.7; load torch first so the process has ONE HIP runtime
# (torch's) and libedet binds to it instead of bringing up a second one.
import torch  # noqa: F401
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t, c_uint64, c_void_p

MAX_SEG = 5
ABI_VERSION = 10  # must equal edet_abi_version() of the loaded library (struct layouts)
OPT_NORM_BLOCKS = 256  # EDET_OPT_NORM_BLOCKS: edet_opt_norm partial-sum slots per quantity
F32, BF16 = 0, 1
# replicated statistics vectors (include/edet.h, ABI 9): channel c of replica r at stat_idx(c, r)
STAT_REPLICAS = 4


def stat_len(C: int) -> int:
    """doubles of a replicated statistics vector of C channels (EDET_STAT_LEN)"""
    return (C + 15) // 16 * 16 * STAT_REPLICAS


def stat_idx(c, r=0):
    return (c // 16) * 16 * STAT_REPLICAS + r * 16 + c % 16


def stat_fold(t, C: int):
    """The values of a replicated statistics vector (last dimension stat_len(C)): replicas summed
    in the library's order, (r0 + r1) + (r2 + r3); a tensor of the leading shape x C."""
    lead = t.shape[:-1]
    v = t.reshape(*lead, -1, STAT_REPLICAS, 16)
    s = (v[..., 0, :] + v[..., 1, :]) + (v[..., 2, :] + v[..., 3, :])
    return s.reshape(*lead, -1)[..., :C]


def stat_unfold(v):
    """A replicated statistics vector holding the values v (last dimension C) in replica 0."""
    import torch as _t
    C = v.shape[-1]
    lead = v.shape[:-1]
    out = _t.zeros(*lead, stat_len(C), dtype=v.dtype, device=v.device)
    o = out.view(*lead, -1, STAT_REPLICAS, 16)
    pad = _t.zeros(*lead, (C + 15) // 16 * 16, dtype=v.dtype, device=v.device)
    pad[..., :C] = v
    o[..., 0, :] = pad.view(*lead, -1, 16)
    return out
ACT_NONE, ACT_SWISH = 0, 1
MODE_SAME, MODE_UPSAMPLE, MODE_MAXPOOL = 0, 1, 2

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EDET_LIB", os.path.join(_PKG_DIR, "lib", "libedet.so"))


class EdetError(RuntimeError):
    pass


class Pyramid(ctypes.Structure):
    _fields_ = [("nseg", c_int32), ("batch", c_int32), ("row_off", c_int32 * MAX_SEG),
                ("H", c_int32 * MAX_SEG), ("W", c_int32 * MAX_SEG)]


class BN(ctypes.Structure):
    _fields_ = [("sum", c_void_p * MAX_SEG), ("sq", c_void_p * MAX_SEG),
                ("gamma", c_void_p * MAX_SEG), ("beta", c_void_p * MAX_SEG),
                ("eps", c_float), ("enabled", c_int32)]


class Lazy(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("gate", c_void_p), ("bn", BN), ("ld", c_int32), ("act", c_int32)]


class SegOut(ctypes.Structure):
    _fields_ = [("a", c_void_p * MAX_SEG), ("b", c_void_p * MAX_SEG)]


class StatOut(ctypes.Structure):
    _fields_ = [("sum", c_void_p * MAX_SEG), ("sq", c_void_p * MAX_SEG)]


class BnGrad64(ctypes.Structure):
    _fields_ = [("dgamma", c_void_p * MAX_SEG), ("dbeta", c_void_p * MAX_SEG)]


class DgradLazy(ctypes.Structure):
    """edet_dgrad_lazy: d(raw y) of a lazy value, built by its consumer on load (ABI 8)."""
    _fields_ = [("dv", c_void_p), ("y", Lazy), ("dsq", c_void_p), ("acc", BnGrad64), ("grads", SegOut)]


class FuseInput(ctypes.Structure):
    _fields_ = [("v", Lazy), ("dx", c_void_p), ("H", c_int32), ("W", c_int32),
                ("mode", c_int32), ("accumulate", c_int32), ("pool_arg", c_void_p)]


class FuseFold(ctypes.Structure):
    """edet_fuse_fold: one BiFPN node's weight-gradient records (ABI 10)."""
    _fields_ = [("part", c_void_p), ("w", c_void_p), ("dw", c_void_p), ("nparts", c_int32), ("n_in", c_int32)]


FUSE_FOLD_MAX = 64  # EDET_FUSE_FOLD_MAX


class Sched(ctypes.Structure):
    _fields_ = [("adjusted_lr", c_float), ("warmup_init", c_float), ("warmup_steps", c_int32),
                ("total_steps", c_int32), ("momentum", c_float), ("ema_decay", c_float),
                ("clip_norm", c_float), ("l2_weight", c_float), ("fixed_lr", c_float),
                ("skip_nonfinite", c_int32)]


class AugParams(ctypes.Structure):
    """edet_aug_params: one image's augmentation (include/edet.h, csrc/augment.hip)."""
    _fields_ = [("warp", ctypes.c_double * 9), ("noise_seed", c_uint64), ("blur", c_int32), ("warp_border", c_int32),
                ("noise", c_int32), ("rw", c_int32), ("rh", c_int32), ("top", c_int32), ("left", c_int32),
                ("pad_border", c_int32), ("out_raw", c_int32), ("warp_bg", ctypes.c_uint8 * 4),
                ("pad_bg", ctypes.c_uint8 * 4)]


P = c_void_p
PPyr, PLazy, PSeg, PStat, PBnG, PFuse, PSched = (POINTER(Pyramid), POINTER(Lazy), POINTER(SegOut), POINTER(StatOut),
                                                 POINTER(BnGrad64), POINTER(FuseInput), POINTER(Sched))
PDgl = POINTER(DgradLazy)

# name -> argtypes (all return int unless listed in _RESTYPE)
SIGNATURES = {
    "edet_last_error": [],
    "edet_abi_version": [],
    "edet_memset_async": [P, c_int, c_size_t, P],
    "edet_memcpy_async": [P, P, c_size_t, P],
    "edet_zero_ranges": [c_int, P, P, P],
    "edet_set_workspace": [P, c_size_t],
    "edet_partials_defer": [P, c_size_t],
    "edet_partials_flush": [POINTER(c_size_t), P],
    "edet_probe": [P, c_int, P],
    "edet_wall_clock_khz": [P],
    "edet_launched_kernels": [c_char_p, c_size_t],
    "edet_dev_set": [c_int, c_int],
    "edet_conv1x1_fwd": [c_int, PLazy, PPyr, c_int, P, c_int, P, P, c_int, c_int, PStat, P],
    "edet_conv1x1_dgrad": [c_int, P, c_int, PPyr, c_int, P, c_int, P, c_int, c_int, P],
    "edet_conv1x1_dgrad_fold": [c_int, P, c_int, PPyr, c_int, P, c_int, P, c_int, PLazy, PBnG, P],
    "edet_conv1x1_dgrad_sesum": [c_int, P, c_int, PPyr, c_int, P, c_int, P, c_int, PLazy, P, P],
    "edet_conv1x1_wgrad": [c_int, PLazy, PPyr, c_int, P, c_int, c_int, P, P, P],
    "edet_dwconv_fwd": [c_int, PLazy, PPyr, c_int, c_int, c_int, P, P, PPyr, PStat, P],
    "edet_dwconv_dgrad": [c_int, P, PPyr, c_int, c_int, c_int, P, P, PPyr, c_int, P],
    "edet_dwconv_dgrad_fold": [c_int, P, PPyr, c_int, c_int, c_int, P, P, PPyr, PLazy, PBnG, P],
    "edet_dwconv_wgrad": [c_int, PLazy, PPyr, c_int, c_int, c_int, P, PPyr, P, P],
    "edet_dwconv_bwd": [c_int, PLazy, PPyr, c_int, c_int, c_int, P, PPyr, P, P, c_int, P, PBnG, P],
    "edet_dwconv_bwd_lazy": [c_int, PLazy, PPyr, c_int, c_int, PDgl, PPyr, P, P, c_int, P, PBnG, P],
    "edet_dwconv_fwd_squeeze": [c_int, PLazy, PPyr, c_int, c_int, c_int, P, P, PPyr, PLazy, P, P],
    "edet_stem_fwd": [c_int, P, c_int, c_int, c_int, P, c_int, P, P, P, P],
    "edet_stem_wgrad": [c_int, P, c_int, c_int, c_int, P, c_int, P, P],
    "edet_lazy_bwd_reduce": [c_int, PLazy, PPyr, c_int, P, P, P, PBnG, P],
    "edet_lazy_bwd_apply": [c_int, PLazy, PPyr, c_int, P, P, P, PBnG, PSeg, P, c_int, P],
    "edet_se_squeeze": [c_int, PLazy, c_int, c_int, c_int, P, P],
    "edet_se_fwd": [c_int, c_int, c_int, P, P, P, P, P, P, P, P],
    "edet_gate_grad": [c_int, PLazy, c_int, c_int, c_int, P, P, P],
    "edet_gate_bn_reduce": [c_int, PLazy, c_int, c_int, c_int, P, P, P],
    "edet_se_bn_combine": [c_int, c_int, P, P, P, PBnG, P],
    "edet_se_bwd": [c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "edet_se_bwd_bn": [c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, PBnG, P],
    "edet_residual_fwd": [c_int, PLazy, PLazy, PPyr, c_int, P, P, P],
    "edet_lazy_materialize": [c_int, PLazy, PPyr, c_int, P, P],
    "edet_maxpool_fwd": [c_int, PLazy, c_int, c_int, c_int, c_int, P, P],
    "edet_maxpool_bwd": [c_int, PLazy, c_int, c_int, c_int, c_int, P, P, c_int, P],
    "edet_maxpool_fwd_taps": [c_int, PLazy, c_int, c_int, c_int, c_int, P, P, P],
    "edet_maxpool_bwd_taps": [c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P],
    "edet_bifpn_fuse_fwd": [c_int, c_int, PFuse, P, c_int, c_int, c_int, c_int, P, P],
    "edet_bifpn_fuse_bwd": [c_int, c_int, PFuse, P, c_int, c_int, c_int, c_int, P, P, P, P],
    "edet_bifpn_fuse_bwd_dv_parts": [c_int, c_int, PFuse, c_int, c_int, c_int, c_int, POINTER(c_int)],
    "edet_bifpn_fuse_bwd_dv": [c_int, c_int, PFuse, P, c_int, c_int, c_int, c_int, P, P, c_int, P, c_int, P],
    "edet_bifpn_fuse_fold": [c_int, POINTER(FuseFold), P],
    "edet_detection_loss": [c_int, P, c_int, P, c_int, PPyr, c_int, c_int, P, P, P, c_float,
                            c_float, c_float, c_float, c_float, P, P, P, P, P],
    "edet_count_positives": [P, c_int64, P, P],
    "edet_onehot_to_index": [P, c_int64, c_int, P, P],
    "edet_anchor_boxes": [c_int, c_int, c_float, c_float, c_float, c_float, c_int, P, P, P],
    "edet_generate_targets": [P, PPyr, c_int, P, P, P, c_int, c_float, P, P, P, P],
    "edet_decode_boxes": [c_int, P, PPyr, c_int, P, c_int, P, P],
    "edet_detect_nms": [c_int, P, P, c_int, PPyr, c_int, c_int, c_int, c_float, c_float, P, P, P, P, P, P],
    "edet_opt_norm": [P, P, c_int64, c_int64, PSched, P, P, P, P],
    "edet_opt_apply": [P, P, P, P, c_int64, c_int64, PSched, P, P, c_int, P, P, P],
    "edet_cast_f32": [c_int, P, P, c_int64, P],
    "edet_transpose_cast": [c_int, P, P, P, c_int, c_int, P],
    "edet_bn_inference_stats": [c_int64, P, P, P, P, P, P],
    "edet_bn_update_moving": [c_int64, P, P, P, c_float, P, P, P, P],
    "edet_dropmask": [P, c_int, c_float, c_uint64, P, P],
    "edet_augment_image": [c_int, P, c_int, c_int, POINTER(AugParams), P, P, c_int, c_int, P],
}
_RESTYPE = {"edet_last_error": c_char_p}


class _Lib:
    def __init__(self, path: str):
        if not os.path.exists(path):
            raise ImportError(
                f"libedet.so not found at {path}: build it with `make -C "
                f"tensorflow2-machine-vision_amd` (or __graft_entry__.build()). There is no "
                f"CPU fallback for the EfficientDet hot path.")
        self.path = path
        self.dll = ctypes.CDLL(path)
        self.fns = {}
        # EDET_ALLOW_MISSING=1 (same-box A/B against an older build of the same ABI only): entry
        # points the library lacks are left unbound instead of failing the import
        allow_missing = os.environ.get("EDET_ALLOW_MISSING") == "1"
        for name, argtypes in SIGNATURES.items():
            if allow_missing and not hasattr(self.dll, name):
                continue
            fn = getattr(self.dll, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPE.get(name, c_int)
            self.fns[name] = fn
        abi = self.fns["edet_abi_version"]()
        # same-box timing A/B only: an ABI 9 build lacks the ABI 10 entry points (the callers
        # check has()); an ABI 8 build (plain statistics vectors) runs in the larger replicated
        # buffers of ABI 9 without leaving them, its values are not the model's
        if abi != ABI_VERSION and not (allow_missing and abi in (8, 9)):
            raise ImportError(f"{path} implements C-ABI version {abi}, this binding expects {ABI_VERSION}: "
                              f"rebuild it with `make -C tensorflow2-machine-vision_amd`")
        # development builds only (EDET_LIB=.../libedet_dev.so): plan slots for whole-step A/B runs,
        # EDET_DEV_SLOTS="29=2,30=1024"; the production library refuses them (edet_dev_set errors)
        for kv in filter(None, os.environ.get("EDET_DEV_SLOTS", "").split(",")):
            slot, val = (int(v) for v in kv.split("="))
            rc = self.fns["edet_dev_set"](slot, val)
            if rc == -2:  # EDET_EUNSUPPORTED
                raise ImportError(f"EDET_DEV_SLOTS needs a development build (make dev): {path}")
            if rc != 0:
                raise ImportError(f"EDET_DEV_SLOTS: {self.last_error()}")

    def has(self, name: str) -> bool:
        return name in self.fns

    def last_error(self) -> str:
        return self.fns["edet_last_error"]().decode(errors="replace")

    def call(self, name: str, *args):
        rc = self.fns[name](*args)
        if rc != 0:
            raise EdetError(f"{name} failed ({rc}): {self.last_error()}")
        return rc


_LIB: _Lib | None = None


def lib() -> _Lib:
    global _LIB
    if _LIB is None:
        _LIB = _Lib(LIB_PATH)
    return _LIB


def call(name: str, *args):
    return lib().call(name, *args)


def has(name: str) -> bool:
    return lib().has(name)


def launched_kernels() -> list:
    """Base names of the kernels launched since the previous query (measurement)."""
    buf = ctypes.create_string_buffer(512)
    lib().fns["edet_launched_kernels"](buf, 512)
    return [k for k in buf.value.decode().split(",") if k]
