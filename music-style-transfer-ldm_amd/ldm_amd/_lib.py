"""ctypes binding of libldm_amd.so (include/ldm_capi.h).

torch is imported first on purpose: its wheel ships libamdhip64.so with SONAME libamdhip64.so.7, and
loading it before libldm_amd.so makes the dynamic linker bind our library to the SAME HIP runtime
instance, so torch's streams, allocations and graph capture are valid in our launches.

There is no CPU fallback anywhere: if the library is missing or no HIP device is present, every
entry point raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("LDM_AMD_LIB", os.path.join(PKG_ROOT, "lib", "libldm_amd.so"))

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_float = ctypes.c_float
c_vp = ctypes.c_void_p
c_fp = ctypes.c_void_p  # device float* as raw address


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in
                ("B", "Cin", "Hin", "Win", "Cout", "Hout", "Wout", "kh", "kw", "stride", "pad", "out_pad", "transposed",
                 "layout")]

    def key(self):
        return tuple(getattr(self, f[0]) for f in self._fields_)


class Epilogue(ctypes.Structure):
    _fields_ = [("bias", c_fp), ("bn_weight", c_fp), ("bn_bias", c_fp), ("bn_mean", c_fp), ("bn_var", c_fp),
                ("bn_eps", c_float), ("act", c_int32), ("bcast_add", c_fp), ("skip_add", c_fp), ("act_out", c_fp),
                ("dtype", c_int32)]


class ConvPlan(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("tm", c_int32), ("tn", c_int32), ("wk", c_int32), ("ks", c_int32),
                ("balance", c_int32), ("packed_floats", c_int64), ("ws_floats", c_int64)]

    def key(self):
        return (self.kind, self.tm, self.tn, self.wk, -self.ks if self.balance else self.ks)


class ActFinJob(ctypes.Structure):
    """ldm_act_fin_job: one deferred bias-gradient finalize (ldm_act_backward_defer / ldm_act_finalize_many)."""
    _fields_ = [("part", c_fp), ("dbias", c_fp), ("B", c_int32), ("C", c_int32), ("Q", c_int32), ("kind", c_int32)]


class WgradRedJob(ctypes.Structure):
    """ldm_wgrad_red_job: one deferred weight-gradient reduction (ldm_conv_backward_weight_defer)."""
    _fields_ = [("partial", c_fp), ("dw", c_fp), ("S", c_int32), ("MN", c_int32), ("accumulate", c_int32)]


class UNetShape(ctypes.Structure):
    _fields_ = [("B", c_int32), ("C", c_int32), ("H", c_int32), ("W", c_int32), ("nf", c_int32)]


class UNetWeights(ctypes.Structure):
    _fields_ = [("conv_w", c_fp * 9), ("conv_b", c_fp * 9), ("conv_plan", ConvPlan * 9),
                ("ca_wq", c_fp * 2), ("ca_bq", c_fp * 2), ("ca_plan_q", ConvPlan * 2),
                ("ca_wkv", c_fp * 2), ("ca_bkv", c_fp * 2), ("ca_plan_kv", ConvPlan * 2),
                ("ca_wo", c_fp * 2), ("ca_bo", c_fp * 2), ("ca_plan_o", ConvPlan * 2),
                ("t_freqs", c_fp), ("t_w1", c_fp), ("t_b1", c_fp), ("t_w2", c_fp), ("t_b2", c_fp),
                ("ca_wq_raw", c_fp * 2), ("fold_w", c_fp * 2), ("fold_pb", c_fp * 2), ("use_fold", c_int32),
                ("step_w", c_fp * 9), ("step_pb", c_fp * 2), ("use_step", c_int32),
                ("step_dtype", c_int32), ("step_bneck_w", c_fp)]


ACT = {"none": 0, "relu": 1, "tanh": 2, "tanh_half": 3, "gelu": 4}
DT_ROUND_OUT = 0x100   # ldm_epilogue.dtype flag (ldm_capi.h LDM_DT_ROUND_OUT); act codes: LDM_ACT_ROUND_* = dt << 8
# 16-bit storage (ldm_capi.h): conv / wgrad dtype flags, and the BatchNorm / activation-backward act-code fields
DT_X16, DT_Y16, DT_DY16 = 0x200, 0x400, 0x800
ST_SHIFT, ST_X16, ST_Y16, ST_DY16, ST_DX16 = 16, 1 << 18, 1 << 19, 1 << 20, 1 << 21

# name -> (restype, argtypes).  Kept in one table so tests can check it against include/ldm_capi.h.
SIGNATURES = {
    "ldm_last_error": (ctypes.c_char_p, []),
    "ldm_capi_version": (c_int32, []),
    "ldm_device_count": (c_int32, [ctypes.POINTER(c_int32)]),
    "ldm_conv_make_plan": (c_int32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvPlan)]),
    "ldm_conv_make_plan_forced": (c_int32, [ctypes.POINTER(ConvDesc), c_int32, c_int32, c_int32, c_int32, c_int32,
                                            ctypes.POINTER(ConvPlan)]),
    "ldm_conv_pack_weight": (c_int32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvPlan), c_fp, c_fp, c_vp]),
    "ldm_conv_forward": (c_int32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvPlan), c_fp, c_fp,
                                   ctypes.POINTER(Epilogue), c_fp, c_vp]),
    "ldm_conv_forward_ws": (c_int32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvPlan), c_fp, c_fp,
                                      ctypes.POINTER(Epilogue), c_fp, c_fp, c_vp]),
    "ldm_reduce_workspace_floats": (c_int64, [c_int32, c_int32, c_int32]),
    "ldm_step_packed_floats": (c_int64, [c_int32]),
    "ldm_step_pack_weight": (c_int32, [c_int32, c_fp, c_fp, c_vp]),
    "ldm_step_pack_weight_dt": (c_int32, [c_int32, c_int32, c_fp, c_fp, c_vp]),
    "ldm_step_conv": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_vp]),
    "ldm_step_conv_dt": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32,
                                   c_vp]),
    "ldm_step_workspace_floats": (c_int64, [c_int32, c_int32, c_int32]),
    "ldm_step_workspace_counter_floats": (c_int64, [c_int32, c_int32, c_int32]),
    "ldm_step_layer_forms": (c_int32, [c_vp]),
    "ldm_step_dec1_ddim": (c_int32, [c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_float, c_fp, c_fp, c_fp,
                                     c_int32, c_vp]),
    "ldm_step_conv_ws": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32,
                                   c_fp, c_vp]),
    "ldm_mel_quantize": (c_int32, [c_fp, c_fp, c_int64, ctypes.c_float, c_vp]),
    "ldm_mel_dequantize": (c_int32, [c_fp, c_fp, c_int64, ctypes.c_float, c_vp]),
    "ldm_u8_to_unit": (c_int32, [c_fp, c_fp, c_int64, c_vp]),
    "ldm_batchnorm_train": (c_int32, [c_fp, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_float, c_float,
                                      c_int32, c_fp, c_fp, c_fp, c_vp]),
    "ldm_batchnorm_train_out": (c_int32, [c_fp, c_fp, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_float,
                                          c_float, c_int32, c_fp, c_fp, c_fp, c_vp]),
    "ldm_batchnorm_apply_out": (c_int32, [c_fp, c_fp, c_int32, c_int32, c_int32, c_vp, ctypes.c_double, c_fp, c_fp,
                                          c_fp, c_fp, c_float, c_float, c_int32, c_fp, c_fp, c_vp]),
    "ldm_maxpool2x2": (c_int32, [c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_vp]),
    "ldm_std_mse_workspace_floats": (c_int64, [c_int32, c_int64]),
    "ldm_std_mse_moments": (c_int32, [c_fp, c_fp, c_int32, c_int64, c_vp, c_fp, c_vp]),
    "ldm_std_mse_accumulate": (c_int32, [c_vp, c_int32, c_int64, ctypes.c_double, ctypes.c_double, c_vp, c_fp, c_vp]),
    "ldm_batchnorm_stats": (c_int32, [c_fp, c_int32, c_int32, c_int32, c_vp, c_fp, c_vp]),
    "ldm_batchnorm_apply": (c_int32, [c_fp, c_int32, c_int32, c_int32, c_vp, ctypes.c_double, c_fp, c_fp, c_fp, c_fp,
                                      c_float, c_float, c_int32, c_fp, c_fp, c_vp]),
    "ldm_batchnorm_eval": (c_int32, [c_fp, c_fp, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_float, c_int32,
                                     c_vp]),
    "ldm_activation": (c_int32, [c_fp, c_fp, c_int64, c_int32, c_vp]),
    "ldm_sinusoid_embed": (c_int32, [c_vp, c_int32, c_int32, c_int32, c_fp, c_fp, c_vp]),
    "ldm_time_mlp_forward": (c_int32, [c_vp, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_vp]),
    "ldm_attention_core": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_int32, c_float, c_vp]),
    "ldm_attention_flash_supported": (c_int32, [c_int32, c_int32]),
    "ldm_attention_forward_lse": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_int32,
                                            c_float, c_vp]),
    "ldm_attention_backward_flash": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32,
                                               c_int32, c_int32, c_int32, c_float, c_vp]),
    "ldm_pack_job_bytes": (c_int64, []),
    "ldm_pack_many_prepare": (c_int32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvPlan), ctypes.POINTER(c_vp),
                                        ctypes.POINTER(c_vp), c_int32, c_vp, ctypes.POINTER(c_int64)]),
    "ldm_pack_many": (c_int32, [c_vp, c_int32, c_int64, c_vp]),
    "ldm_im2col": (c_int32, [c_fp, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                             c_fp, c_fp, c_int32, c_int32, c_fp, c_vp]),
    "ldm_col2im": (c_int32, [c_fp, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                             c_fp, c_int32, c_int32, c_fp, c_vp]),
    "ldm_maxpool3s2": (c_int32, [c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_vp]),
    "ldm_maxpool3s2_backward": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_vp]),
    "ldm_lpips_layer": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_fp, c_fp, c_vp]),
    "ldm_lpips_layer_backward": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_int32, c_fp,
                                           c_vp]),
    "ldm_attention_fold_keys": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_float, c_fp, c_fp,
                                          c_vp]),
    "ldm_attention_folded": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_int32,
                                       c_vp]),
    "ldm_fold_conv_proj": (c_int32, [ctypes.POINTER(ConvDesc), c_fp, c_fp, c_fp, c_fp, c_int32, c_fp, c_fp, c_vp]),
    "ldm_attention_folded_probs": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_int32,
                                             c_vp]),
    "ldm_bneck_fold_supported": (c_int32, [c_int32, c_int32, c_int32]),
    "ldm_bneck_fold_values": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_vp]),
    "ldm_bneck_pv": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_vp]),
    "ldm_ca1_probs": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_int32, c_vp]),
    "ldm_ca1_probs_form": (c_int32, []),
    "ldm_set_cin1_packed": (c_int32, [c_int32]),
    "ldm_set_cin1_s1": (c_int32, [c_int32]),
    "ldm_set_flash_split": (c_int32, [c_int32]),
    "ldm_q_sample": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_vp, c_fp, c_int32, c_int64, c_vp]),
    "ldm_predict_start": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_vp, c_fp, c_int32, c_int64, c_vp]),
    "ldm_sched_backward": (c_int32, [c_int32, c_fp, c_fp, c_int32, c_vp, c_fp, c_fp, c_int32, c_int64, c_vp]),
    "ldm_ddim_step":(c_int32, [c_fp, c_fp, c_fp, c_float, c_fp, c_fp, c_int64, c_vp]),
    "ldm_loss_forward": (c_int32, [c_int32, c_fp, c_fp, c_int64, c_vp, c_fp, c_vp]),
    "ldm_loss_backward": (c_int32, [c_int32, c_fp, c_fp, c_int64, c_fp, c_fp, c_fp, c_vp]),
    "ldm_unet_workspace_floats": (c_int64, [ctypes.POINTER(UNetShape), ctypes.POINTER(UNetWeights)]),
    "ldm_ddim_workspace_floats": (c_int64, [ctypes.POINTER(UNetShape), ctypes.POINTER(UNetWeights), c_int32]),
    "ldm_unet_make_plans": (c_int32, [ctypes.POINTER(UNetShape), ctypes.POINTER(UNetWeights)]),
    "ldm_unet_layer_desc": (c_int32, [ctypes.POINTER(UNetShape), c_int32, ctypes.POINTER(ConvDesc)]),
    "ldm_unet_forward": (c_int32, [ctypes.POINTER(UNetShape), ctypes.POINTER(UNetWeights), c_fp, c_vp, c_int32,
                                   c_fp, c_fp, c_fp, c_fp, c_vp]),
    "ldm_ddim_sample": (c_int32, [ctypes.POINTER(UNetShape), ctypes.POINTER(UNetWeights), c_fp, c_fp, c_fp, c_vp,
                                  c_fp, c_int32, c_float, c_fp, c_fp, c_int64, c_fp, c_vp]),
    # backward / optimiser
    "ldm_conv_tiled_plan": (c_int32, [ctypes.POINTER(ConvDesc), c_int32, ctypes.POINTER(ConvPlan)]),
    "ldm_conv_sconv_plan": (c_int32, [ctypes.POINTER(ConvDesc), c_int32, ctypes.POINTER(ConvPlan)]),
    "ldm_conv_storage16": (c_int32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvPlan)]),
    "ldm_conv_wgrad_storage16": (c_int32, [ctypes.POINTER(ConvDesc)]),
    "ldm_batchnorm_stats_code": (c_int32, [c_fp, c_int32, c_int32, c_int32, c_int32, c_vp, c_fp, c_vp]),
    "ldm_conv_wgrad_workspace_floats": (c_int64, [ctypes.POINTER(ConvDesc)]),
    "ldm_conv_backward_weight_dt": (c_int32, [ctypes.POINTER(ConvDesc), c_fp, c_fp, c_fp, c_int32, c_fp, c_int32, c_vp]),
    "ldm_conv_backward_weight": (c_int32, [ctypes.POINTER(ConvDesc), c_fp, c_fp, c_fp, c_int32, c_fp, c_vp]),
    "ldm_act_backward_defer": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_vp,
                                         c_vp]),
    "ldm_act_partial_floats": (c_int64, [c_int32, c_int32, c_int32]),
    "ldm_batchnorm_backward_dxsum_defer": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32,
                                                     c_int32, c_fp, c_fp, c_fp, c_fp, c_vp, c_vp, c_fp, c_vp]),
    "ldm_bn_dxsum_partial_floats": (c_int64, [c_int32, c_int32, c_int32]),
    "ldm_conv_backward_weight_defer": (c_int32, [c_vp, c_fp, c_fp, c_fp, c_int32, c_fp, c_int32, c_vp, c_vp]),
    "ldm_wgrad_reduce_many": (c_int32, [c_vp, c_int32, c_vp]),
    "ldm_act_finalize_many": (c_int32, [c_vp, c_int32, c_vp]),
    "ldm_act_backward": (c_int32, [c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_fp, c_fp, c_fp, c_fp,
                                   c_vp]),
    "ldm_batchnorm_backward": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32,
                                         c_int32, c_fp, c_fp, c_fp, c_fp, c_vp]),
    "ldm_batchnorm_backward_dxsum": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32,
                                               c_int32, c_fp, c_fp, c_fp, c_fp, c_fp, c_vp]),
    "ldm_batchnorm_backward_reduce": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32,
                                                c_int32, c_vp, c_fp, c_fp, c_fp, c_vp]),
    "ldm_batchnorm_backward_apply": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32,
                                               c_int32, c_vp, ctypes.c_double, c_fp, c_vp]),
    "ldm_attention_backward": (c_int32, [c_fp, c_fp, c_fp, c_fp, c_fp, c_int32, c_int32, c_int32, c_int32, c_int32,
                                         c_float, c_vp]),
    "ldm_unscale_check": (c_int32, [c_vp, c_vp, c_vp, c_int32, c_int32, c_fp, c_vp, c_vp]),
    "ldm_adam_step": (c_int32, [c_vp, c_vp, c_vp, c_int32, c_int32, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, ctypes.c_double, c_int32, c_int32, c_vp, c_vp]),
    "ldm_adam_step_dev": (c_int32, [c_vp, c_vp, c_vp, c_int32, c_int32, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double, ctypes.c_double, c_int32, c_fp, c_vp, c_fp,
                                    c_vp]),
    "ldm_update_scale": (c_int32, [c_fp, c_vp, c_vp, c_float, c_float, c_int32, c_vp]),
}

# ldm_tensor_slot: 4 device pointers + int64 numel, packed into an int64 tensor on the device
TENSOR_SLOT_WORDS = 5

_LIB = None


class LDMError(RuntimeError):
    pass


def load(path=None):
    """Load (once) and return the CDLL with every prototype declared. Raises if absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise LDMError(f"libldm_amd.so not found at {p}: build it with `make -C music-style-transfer-ldm_amd/csrc` "
                       "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().ldm_last_error().decode(errors="replace")
        raise LDMError(f"{what} failed (code {rc}): {msg}")


def call(name, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc


def step_layer_forms():
    """Bit mask of the reverse-loop layers that run uconv.hip's K-split form (ldm_step_layer_forms)."""
    k = ctypes.c_int32(0)
    call("ldm_step_layer_forms", ctypes.byref(k))
    return int(k.value)
