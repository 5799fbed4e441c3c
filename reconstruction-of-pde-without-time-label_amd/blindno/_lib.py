"""ctypes binding of libblindno.so (the C ABI declared in include/blindno.h).

The library is loaded AFTER torch so that its HIP runtime dependency
(``libamdhip64.so.7``) resolves to the runtime torch already loaded: device
pointers and streams are then shared with PyTorch.  There is no fallback: if the
library or a GPU is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLINDNO_LIB", os.path.join(_HERE, "libblindno.so"))

# argument codes: p pointer, i int32, l int64, f float, d double, s stream
SIGNATURES = {
    "blindno_abi_version": "",
    "blindno_lift_fwd": "ppppiiiiiiis",
    "blindno_lift_bwd": "pppppiiiiiiiis",
    "blindno_project_fwd": "ppppppiiiiiiiiiis",
    "blindno_project_bwd": "pppppppiiiiiiiiiiiis",
    "blindno_rowdft": "pppiiiiiis",
    "blindno_rowdft_crop": "pppiiiiiiiis",
    "blindno_rowdft_bag_lift": "ppppppiiiiiiiiis",
    "blindno_rowdft_bag_lift_dg": "pppppppiiiiiiiiis",
    "blindno_rowidft_epi_lift": "ppppppppppiiiiiiiiis",
    "blindno_rowidft_bwd_lift": "ppppppppppiiiiiiiiis",
    "blindno_colpass": "pppppppiiiiiiiis",
    "blindno_colspec_ok": "iiiiii",
    "blindno_colspec_nchunk": "ii",
    "blindno_colspec_bwd_nchunk": "ii",
    "blindno_rowdft_cd": "ppppiiiiiiiis",
    "blindno_rowdft_bag_lift_cd": "pppppiiiiiiiis",
    "blindno_rowdft_bag_lift_cd_pack": "pppppiiiiiiiippppis",
    "blindno_colmix": "pipppiiiiiiiippps",
    "blindno_rowidft_epi_zc": "ppppppppp" + "iiiiiiiiii" + "s",
    "blindno_rowidft_epi_lift_zc": "ppppppppppppp" + "iiiiiiiiiii" + "s",
    "blindno_rowidft_bwd_zc": "pppppppppp" + "iiiiiiiii" + "s",
    "blindno_rowidft_bwd_lift_zc": "ppppppppppp" + "iiiiiiiiii" + "s",
    "blindno_rowidft_bwd_lift_zc_mix": "ppppppppppp" + "iiiiiiiiii" + "ppppi" + "s",
    "blindno_rowdft_cd_bag": "pppi" + "ppp" + "iiiiiii" + "s",
    "blindno_rowidft_bwd_zc_bag": "pppp" + "i" + "pppppppp" + "iiiiiiiii" + "s",
    "blindno_mix_wgrad": "ppppiiiiiis",
    "blindno_mix_wgrad_part": "pppiiiiiiis",
    "blindno_mix_wgrad_multi": "ppppis",
    "blindno_mix_wgrad_multi_u": "ppppppis",
    "blindno_mix1d": "ppppiiiiiis",
    "blindno_rowidft_epi": "ppppppiiiiiis",
    "blindno_rowidft_epi_crop": "pppppp" + "iiiiiiii" + "s",
    "blindno_rowidft_bwd": "pppppppiiiiiis",
    "blindno_rowidft_bwd_crop": "pppppppiiiiiiiis",
    "blindno_rowidft_bwd_rd": "pppppppiiiiiiiipps",
    "blindno_rowidft_epi_rd": "ppppppiiiiiippis",
    "blindno_rowidft_epi_lift_rd": "ppppppppppiiiiiiiiippis",
    "blindno_conv_wgrad": "pppiiiiiis",
    "blindno_reduce_partials": "ppiis",
    "blindno_spectrum_tile_layout": "iiiii",
    "blindno_pack_w2d": "pppiiiiis",
    "blindno_unpack_w2d": "pppiiiiis",
    "blindno_pack_w1d": "ppiiiis",
    "blindno_bagmean_fwd": "pppppiiiiis",
    "blindno_bagmean_bwd": "pppiiiiis",
    "blindno_mse": "pppplips",
    "blindno_mse_finish": "pilps",
    "blindno_mse_finish_acc": "pilpps",
    "blindno_mse_fwd": "ppplipppps",
    "blindno_rowsq": "pppiiiiiis",
    "blindno_adam": "pppplffffffs",
    "blindno_gpe_solve": "ppppddiiipppiiis",
    "blindno_trapz_rows": "ppppiis",
    # size queries (return a count, not an error code)
    "blindno_lift_bwd_nchunk": "iii",
    "blindno_conv_wgrad_nchunk": "iii",
    "blindno_rowidft_bwd_nchunk": "iiiii",
    "blindno_set_rowfuse": "i",
    "blindno_set_colfuse": "i",
    "blindno_project_bwd_nchunk": "iii",
    "blindno_project_bwd_nchunk_heads": "iii",
    "blindno_mix_wgrad_nsplit": "iiiii",
    "blindno_lift_fwd_g": "ppppiliiiiiiis",
    "blindno_lift_fwd_bag_g": "ppppiliiiiiiippppfs",
    "blindno_lift_bag_ok": "iiiiiiii",
    "blindno_lift_bwd_g": "pppppiiliiiiiiis",
    "blindno_lift_bwd_mix_g": "pppppiiliiiiiiippppiiis",
    "blindno_lift_bwd_bag_mix_g": "pppppiiliiiiiiippppiiippppffs",
    "blindno_project_fwd_g": "ppppppiliiiiiiiiiis",
    "blindno_project_bwd_g": "pppppppiiliiiiiiiiiis",
    "blindno_colpass_g": "pppppppiliiiiiiiis",
    "blindno_mix_wgrad_g": "ppppiiiiiiis",
    "blindno_rowidft_epi_g": "ppppppiliiiiiis",
    "blindno_rowidft_bwd_g": "ppppppiliiiiiis",
    "blindno_conv_wgrad_g": "pppiiiiiiis",
    "blindno_rowdft_wgrad_ok": "iiiii",
    "blindno_rowdft_wgrad_g": "pppppiippppiiiiiiiis",
    "blindno_bagmean_fwd_w": "pppppp" + "iiiii" + "s",
    "blindno_project_bwd_w": "pppppppp" + "i" + "iiiiiiiiiii" + "s",
    "blindno_project_bag_stats_floats": "iii",
    "blindno_project_bag_bwd_nchunk": "iii",
    "blindno_project_bag_fwd": "ppppppppp" + "iiiiiiii" + "s",
    "blindno_project_bag_bwd": "ppppppp" + "i" + "iiiiiiii" + "s",
    "blindno_pack_w2d_2": "ppppp" + "iiiii" + "s",
    "blindno_unpack_w2d_2": "ppppp" + "iiiii" + "s",
    "blindno_bn_act_nslices": "iii",
    "blindno_bn_act_fwd": "ppppppppiiiifffis",
    "blindno_bn_act_bwd": "pppppppppiiiifis",
    "blindno_gather_flat": "pppips",
    "blindno_gather_batch": "ppppipis",
    "blindno_reduce_partials_multi": "ppppis",
    "blindno_reduce_partials_pieces": "ppppppis",
    "blindno_reduce_partials_pieces_u": "pppppppppis",
    "blindno_finish_multi": "pppppppppippppis",
    "blindno_unpack_w2d_multi": "ppppis",
    "blindno_pack_w2d_multi": "ppppis",
    "blindno_fp_propagate": "pppiiiiiids",
    "blindno_bagattn_nchunk": "i",
    "blindno_bagattn_fwd": "pppppppp" + "iiii" + "s",
    "blindno_bagattn_bwd": "ppppppppppp" + "iiii" + "s",
    "blindno_conv2d_fwd": "pppp" + "iiiiiiiiiii" + "s",
    "blindno_conv2d_bwd_data": "ppp" + "iiiiiiiiiii" + "s",
    "blindno_conv2d_wgrad_nsplit": "iiiiiiiiiii",
    "blindno_conv2d_bwd_weight": "pppp" + "i" + "iiiiiiiiiii" + "s",
    "blindno_conv2d_fwd_nsplit": "iiiiiiiiiii",
    "blindno_conv2d_fwd_split": "ppppp" + "i" + "p" + "iiiiiiiiiii" + "s",
    "blindno_conv2d_bwd_data_nsplit": "iiiiiiiiiii",
    "blindno_conv2d_bwd_data_split": "pppp" + "i" + "p" + "iiiiiiiiiii" + "s",
    "blindno_conv2d_wscratch_floats": "i" + "iiiiiiiiiii",
    # whole-op spectral convolutions (C hosts); int64_t byte queries
    "blindno_spectral2d_tables_bytes": "iiii",
    "blindno_spectral2d_tables_init": "piiii",
    "blindno_spectral_conv2d_workspace_bytes": "iiiiiiii",
    "blindno_spectral_conv2d_saved_bytes": "iiiii",
    "blindno_spectral_conv2d_fwd": "ppppppp" + "iiiiiii" + "s",
    "blindno_spectral_conv2d_bwd": "ppppppppp" + "iiiiiii" + "s",
    "blindno_spectral1d_tables_bytes": "ii",
    "blindno_spectral1d_tables_init": "pii",
    "blindno_spectral_conv1d_workspace_bytes": "iiiiii",
    "blindno_spectral_conv1d_saved_bytes": "iii",
    "blindno_spectral_conv1d_fwd": "pppppp" + "iiiii" + "s",
    "blindno_spectral_conv1d_bwd": "ppppppp" + "iiiii" + "s",
    # PermInvUNet_attn (csrc/unet.hip)
    "blindno_dwconv_fwd": "pppp" + "iiiiii" + "s",
    "blindno_dwconv_bwd_data": "ppp" + "iiiiii" + "s",
    "blindno_dwconv_wgrad_nsplit": "iiii",
    "blindno_dwconv_bwd_weight": "pppp" + "i" + "iiiiii" + "s",
    "blindno_cnx_pw_fwd": "ppppppppp" + "iii" + "s",
    "blindno_cnx_pw_bwd_nblk": "iii",
    "blindno_cnx_pw_bwd": "pppppppppp" + "iiii" + "s",
    "blindno_maxpool_fwd": "ppp" + "iiiii" + "s",
    "blindno_maxpool_bwd": "ppp" + "iiiii" + "s",
    "blindno_convt_fwd": "pppp" + "iiiiiiiii" + "s",
    "blindno_convt_bwd_data": "ppp" + "iiiiiiiii" + "s",
    "blindno_convt_wgrad_nparts": "iii",
    "blindno_convt_bwd_weight": "pppp" + "iiiiiiiii" + "s",
    "blindno_tok_gram_nchunk": "l",
    "blindno_tok_attn_save_floats": "iil",
    "blindno_tok_attn_fwd": "ppppppp" + "iil" + "f" + "s",
    "blindno_tok_attn_bwd_scratch_floats": "ii",
    "blindno_tok_attn_bwd": "pppppppp" + "iil" + "s",
    # DeepONet combiner + bag mean (csrc/deeponet.hip)
    "blindno_deeponet_bag_nblk": "i",
    "blindno_deeponet_bag_fwd": "pppppp" + "iiii" + "f" + "s",
    "blindno_deeponet_bag_bwd": "pppppppp" + "iiiii" + "f" + "s",
}

# entry points returning int64_t (byte counts) instead of an error code / int count
RET64 = {n for n in SIGNATURES if n.endswith(("_bytes", "_floats"))}

_CT = {"p": ctypes.c_void_p, "i": ctypes.c_int, "l": ctypes.c_int64, "f": ctypes.c_float,
       "d": ctypes.c_double, "s": ctypes.c_void_p}

_lock = threading.Lock()
_lib = None


class BlindnoError(RuntimeError):
    pass


def load():
    """Load and type the library (idempotent).  Raises BlindnoError if absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise BlindnoError(
                f"libblindno.so not found at {LIB_PATH}; build it with "
                "`python reconstruction-of-pde-without-time-label_amd/build.py` "
                "(there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, sig in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = [_CT[c] for c in sig]
            fn.restype = ctypes.c_int64 if name in RET64 else ctypes.c_int
        lib.blindno_error_string.argtypes = [ctypes.c_int]
        lib.blindno_error_string.restype = ctypes.c_char_p
        _lib = lib
        return lib


def exported_symbols():
    return list(SIGNATURES) + ["blindno_error_string"]


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class _TensorPtr(ctypes.c_void_p):
    """A device pointer that keeps its tensor alive: ``call(name, ptr(x.contiguous()), ...)``
    must not hand the kernel a block the caching allocator already took back (and gave to the
    next temporary in the same argument list) before the launch is enqueued."""
    __slots__ = ("tensor",)


def ptr(t):
    if t is None:
        return None
    p = _TensorPtr(t.data_ptr())
    p.tensor = t
    return p


_HOOKS = {}   # kernel name -> object with before(args) / after(args) (blindno.timing)


def query(name, *args) -> int:
    """Call a size-query entry point (returns a count)."""
    return int(getattr(load(), name)(*args))


def call(name, *args):
    lib = load()
    hook = _HOOKS.get(name)
    if hook is not None:
        hook.before(args)
    rc = getattr(lib, name)(*args)
    if hook is not None:
        hook.after(args)
    if rc != 0:
        msg = lib.blindno_error_string(rc).decode(errors="replace")
        raise BlindnoError(f"{name} failed: hip error {rc} ({msg})")
    return rc
