"""ctypes binding of the C ABI in ``include/fastscnn.h`` (libfastscnn_hip.so).

There is no fallback: if the library is missing or fails to load, every entry point raises
``RuntimeError`` — the HIP path is the product, never a CPU restatement.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FSCNN_LIB", os.path.join(_HERE, "libfastscnn_hip.so"))

DT_F32, DT_BF16, DT_F16 = 0, 1, 2

c_int, c_ll, c_float, c_vp, c_char_p = (ctypes.c_int, ctypes.c_longlong, ctypes.c_float,
                                        ctypes.c_void_p, ctypes.c_char_p)
c_ull = ctypes.c_ulonglong
P_int, P_ll, P_vp = ctypes.POINTER(c_int), ctypes.POINTER(c_ll), ctypes.POINTER(c_vp)

# name -> (restype, argtypes)
SIGNATURES = {
    "fscnn_version": (c_char_p, []),
    "fscnn_last_error": (c_char_p, []),
    "fscnn_net_create": (c_int, [c_int, c_int, P_vp]),
    "fscnn_net_destroy": (None, [c_vp]),
    "fscnn_net_param_count": (c_int, [c_vp, P_int, P_ll]),
    "fscnn_net_param_info": (c_int, [c_vp, c_int, ctypes.POINTER(c_char_p), P_ll, P_ll]),
    "fscnn_net_buffer_count": (c_int, [c_vp, P_int, P_ll, P_int]),
    "fscnn_net_buffer_info": (c_int, [c_vp, c_int, ctypes.POINTER(c_char_p), P_ll, P_ll]),
    "fscnn_net_stage_range": (c_int, [c_vp, c_int, P_ll, P_ll]),
    "fscnn_plan_create": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, P_vp]),
    "fscnn_plan_destroy": (None, [c_vp]),
    "fscnn_plan_workspace": (c_int, [c_vp, P_ll, P_ll]),
    "fscnn_plan_shapes": (c_int, [c_vp, P_int]),
    "fscnn_plan_buffer": (c_int, [c_vp, c_char_p, P_ll, P_ll, P_int, P_int, P_int]),
    "fscnn_forward": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_ull,
                              c_float, c_float, c_vp]),
    "fscnn_backward": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_ull, c_float,
                               c_int, c_int, c_vp]),
    "fscnn_normalize_u8": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "fscnn_remap_labels": (c_int, [c_vp, c_ll, c_vp, c_int, c_int, c_ll, c_vp, c_vp]),
    "fscnn_ohem_prob": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_ll, c_float, c_vp, c_vp,
                                c_vp]),
    "fscnn_ohem_threshold": (c_int, [c_vp, c_ll, c_vp, c_ll, c_float, c_vp, c_vp, c_vp]),
    "fscnn_ce_weighted_fwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_ll, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_vp]),
    "fscnn_ce_weighted_bwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_ll, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fscnn_dice_fwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_float, c_float, c_int,
                               c_vp, c_vp, c_vp]),
    "fscnn_dice_bwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_float, c_float, c_int,
                               c_vp, c_vp, c_float, c_float, c_float, c_vp, c_vp]),
    "fscnn_predict": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fscnn_seg_metric": (c_int, [c_vp, c_int, c_vp, c_ll, c_int, c_vp, c_vp]),
    "fscnn_forward_aux": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                                  c_ull, c_float, c_float, c_vp]),
    "fscnn_backward_aux": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_ull,
                                   c_float, c_int, c_int, c_vp]),
    "fscnn_forward_loss": (c_int, [c_vp, c_vp, c_int, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_ull, c_float, c_float, c_vp]),
    "fscnn_backward_loss": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_ull,
                                    c_float, c_int, c_int, c_vp]),
    "fscnn_backward_dx": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
                                  c_vp, c_vp, c_vp, c_ull, c_float, c_int, c_int, c_vp]),
    "fscnn_prof_begin": (c_int, [c_int, c_int]),
    "fscnn_prof_end": (c_int, [ctypes.POINTER(ctypes.c_double), P_ll, ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double)]),
    "fscnn_prof_launch": (c_int, [c_ll, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_float),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(c_char_p)]),
    "fscnn_prof_kind_name": (c_char_p, [c_int]),
    "fscnn_ce_parts": (c_ll, [c_int, c_ll]),
    "fscnn_ce_fwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_ll, c_vp, c_vp, c_vp]),
    "fscnn_ce_bwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_ll, c_vp, c_vp, c_vp,
                             c_vp]),
    "fscnn_sgd": (c_int, [c_vp, c_vp, c_vp, c_ll, c_float, c_float, c_float, c_float, c_int,
                          c_int, c_float, c_vp]),
    "fscnn_conv0_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp,
                                c_int, c_vp]),
    "fscnn_conv0_wgrad_slab_floats": (c_ll, [c_int, c_int, c_int]),
    "fscnn_conv0_wgrad": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp]),
    "fscnn_dw3x3_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                c_int, c_vp, c_vp]),
    "fscnn_dw3x3_dgrad": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp,
                                  c_vp]),
    "fscnn_dw3x3_wgrad_slab_floats": (c_ll, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "fscnn_dw3x3_wgrad": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                                  c_vp, c_vp]),
    "fscnn_pw_gemm": (c_int, [c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp,
                              c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp]),
    "fscnn_pw_dgrad_bnbwd": (c_int, [c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_int,
                                     c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int,
                                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, P_int, c_vp]),
    "fscnn_kth_smallest": (c_int, [c_vp, c_ll, c_ll, c_vp, c_vp, c_vp]),
    "fscnn_debug_stamps": (c_int, [c_vp, c_int]),
    "fscnn_debug_stamp_count": (c_int, []),
    "fscnn_debug_stamp_tag": (c_char_p, [c_int]),
    "fscnn_pw_wgrad_slab_floats": (c_ll, [c_int, c_int, c_int]),
    "fscnn_pw_gemm_stats_parts": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "fscnn_pw_wgrad": (c_int, [c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int,
                               c_vp]),
    "fscnn_bn_finalize": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_float,
                                  c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fscnn_bilinear_ac_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_vp, c_int, c_int, c_vp]),
    "fscnn_bilinear_ac_bwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_vp, c_vp, c_vp]),
    "fscnn_pyramid_pool_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                                       c_vp]),
    "fscnn_block_ir_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                   c_vp, c_int, c_vp]),
    "fscnn_pyramid_pool_bwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_int,
                                       c_int, c_vp]),
    "fscnn_block_ir_s2_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_int, c_vp]),
    "fscnn_block_ltd_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "fscnn_block_dsconv_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp,
                                       c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "fscnn_block_dsconv_res_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                           c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                           c_vp, c_int, c_vp]),
    "fscnn_block_cls_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int] + [c_vp] * 14 + [c_int, c_vp, c_vp,
                                                                              c_int, c_vp]),
    "fscnn_block_ffm_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_int,
                                    c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_int, c_vp]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load (once) and return the ctypes library; raises RuntimeError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "libfastscnn_hip.so not found at %s — build it with "
                "`python -c 'import __graft_entry__; __graft_entry__.build()'` "
                "(there is no CPU fallback)" % LIB_PATH)
        # torch must be imported first so its bundled HIP runtime (same soname) is the one used
        import torch  # noqa: F401
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().fscnn_last_error().decode(errors="replace")
        raise RuntimeError("fastscnn HIP error %d in %s: %s" % (rc, what, msg))


def call(name, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc


def ptr(t):
    """Device pointer of a tensor (None → NULL)."""
    return None if t is None else c_vp(t.data_ptr())


def stream_ptr(device=None):
    import torch
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def dtype_code(dt):
    import torch
    if dt == torch.float32:
        return DT_F32
    if dt == torch.bfloat16:
        return DT_BF16
    if dt == torch.float16:
        return DT_F16
    raise RuntimeError("fastscnn: unsupported dtype %s (fp32 / bf16 / fp16)" % (dt,))
