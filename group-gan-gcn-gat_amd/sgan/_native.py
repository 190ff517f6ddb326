"""ctypes binding of libsgg.so (include/sgg.h).

The product path has NO CPU fallback: if the library is missing, or the
process has no GPU, every entry point raises.  `torch` is imported first so
libsgg.so binds to the HIP runtime torch already loaded (same SONAME
libamdhip64.so.7): one runtime, torch's caching allocator and streams are
ours.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below)

from ._srchash import source_hash

# SGG_LIB: another build of the same library (A/B runs of kernel variants,
# tools/); only such an explicit choice skips the source-hash check in load()
_LIB_EXPLICIT = bool(os.environ.get("SGG_LIB"))
_LIB_PATH = os.environ.get("SGG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libsgg.so")

_i = ctypes.c_int
_f = ctypes.c_float
_p = ctypes.c_void_p
_sz = ctypes.c_size_t

MAX_HEADS = 4   # SGG_GATENC_MAX_HEADS


class GatEncWeights(ctypes.Structure):
    """SggGatEncWeights (include/sgg.h)."""
    _fields_ = [("Wi", _p * MAX_HEADS), ("ai", _p * MAX_HEADS), ("Wio", _p), ("aio", _p),
                ("Wg", _p * MAX_HEADS), ("ag", _p * MAX_HEADS), ("Wgo", _p), ("ago", _p), ("Woe", _p), ("boe", _p)]


class GatEncArgs(ctypes.Structure):
    """SggGatEncArgs (include/sgg.h)."""
    _fields_ = [("X", _p), ("ldx", _i), ("labels", _p), ("scene_off", _p), ("S", _i), ("np", _i), ("nh", _i),
                ("alpha", _f), ("w", GatEncWeights), ("y", _p), ("ldy", _i), ("dy", _p), ("lddy", _i), ("dX", _p),
                ("lddx", _i), ("slab", _p), ("saved", _p), ("X2", _p), ("ldx2", _i), ("kx1", _i),
                ("dX2", _p), ("lddx2", _i), ("dy_copies", _i), ("dy_cstride", _i)]


_pargs = ctypes.POINTER(GatEncArgs)


class GcnModArgs(ctypes.Structure):
    """SggGcnModArgs (include/sgg.h)."""
    _fields_ = [("X", _p), ("ldx", _i), ("X2", _p), ("ldx2", _i), ("kx1", _i), ("labels", _p), ("scene_off", _p),
                ("S", _i), ("np", _i), ("fin", _i), ("fe", _i), ("bf16", _i), ("W0i", _p), ("W1i", _p), ("W0g", _p),
                ("W1g", _p), ("Woe", _p), ("boe", _p), ("y", _p), ("ldy", _i), ("dy", _p), ("lddy", _i),
                ("dy_copies", _i), ("dy_cstride", _i), ("dX", _p), ("lddx", _i), ("dX2", _p), ("lddx2", _i),
                ("slab", _p)]


_gargs = ctypes.POINTER(GcnModArgs)


class LstmSeg(ctypes.Structure):
    """SggLstmSeg (include/sgg.h): one encoder sequence segment."""
    _fields_ = [("rel", _p), ("A", _p), ("Whh", _p), ("bias", _p), ("h0", _p), ("c0", _p), ("T", _i), ("B", _i),
                ("Bl", _i), ("t0", _i), ("Tl", _i), ("Bsrc", _i), ("h_all", _p), ("c_all", _p), ("act_all", _p),
                ("Wu", _p), ("ldwu", _i), ("cu", _p), ("NU", _i), ("U", _p)]


_sargs = ctypes.POINTER(LstmSeg)

FOLD_MAX = 8   # SGG_FOLD_MAX


class Fold(ctypes.Structure):
    """SggFold (include/sgg.h)."""
    _fields_ = [("W", _p), ("ldw", _i), ("R", _i), ("E", _i), ("We", _p), ("be", _p), ("b1", _p), ("b2", _p),
                ("A", _p), ("bias", _p)]

RED_MAX = 24    # SGG_RED_MAX
FOLDB_MAX = 6   # SGG_FOLDB_MAX


class Red(ctypes.Structure):
    """SggRed (include/sgg.h): one slab row-sum job of sgg_grad_finish."""
    _fields_ = [("src", _p), ("rows", _i), ("ld", _i), ("col0", _i), ("cols", _i), ("out", _p), ("map", _i),
                ("N", _i), ("ldo", _i), ("trans", _i)]


class FoldBwd(ctypes.Structure):
    """SggFoldBwd (include/sgg.h): one fold backward of sgg_grad_finish."""
    _fields_ = [("W", _p), ("ldw", _i), ("R", _i), ("E", _i), ("We", _p), ("be", _p),
                ("dA_src", _p), ("dA_rows", _i), ("dA_ld", _i), ("dA_col0", _i),
                ("db_src", _p), ("db_rows", _i), ("db_ld", _i), ("db_col0", _i),
                ("dW", _p), ("lddw", _i), ("dWe", _p), ("dbe", _p), ("dbias_copy", _p)]


class DecInit(ctypes.Structure):
    """SggDecInit (include/sgg.h): the decoder's h0 / rel0 built in the LSTM prologue."""
    _fields_ = [("ctx", _p), ("ldc", _i), ("Dc", _i), ("z", _p), ("nz", _i), ("best", _p), ("first_k", _i),
                ("ped_scene", _p), ("S", _i), ("Bper", _i), ("last_rel", _p)]


LOSSJOB_MAX = 2   # SGG_LOSSJOB_MAX


class TrajOut(ctypes.Structure):
    """SggTrajOut (include/sgg.h): the discriminator input written by the decoder launch."""
    _fields_ = [("out", _p), ("NB", _i), ("T0", _i), ("col0", _i), ("ncol", _i), ("head", _p), ("ldh", _i),
                ("b", _p), ("ldb", _i), ("pos0", _p), ("start", _p)]


class PoolBatch(ctypes.Structure):
    """SggPoolBatch (include/sgg.h): one batch of sgg_pool_fwd2."""
    _fields_ = [("U", _p), ("pos", _p), ("scene_off", _p), ("chunks", _p), ("nchunks", _i), ("max_rows", _i),
                ("gpw", _i), ("B", _i), ("max_n", _i), ("out", _p), ("argmax", _p), ("nchunks_dev", _p)]


class GatLayerSet(ctypes.Structure):
    """SggGatLayerSet (include/sgg.h): one batch of sgg_gat_layer_fwd2."""
    _fields_ = [("x1", _p), ("ld1", _i), ("K1", _i), ("x2", _p), ("ld2", _i), ("K2", _i), ("seg_off", _p),
                ("nseg", _i), ("n", _i), ("max_seg", _i), ("xn", _p), ("rstd", _p), ("wh", _p), ("hp", _p), ("y", _p),
                ("ldy", _i)]


class L2Job(ctypes.Structure):
    """SggL2Job (include/sgg.h): an L2 loss value of sgg_grad_finish_losses."""
    _fields_ = [("term", _p), ("S", _i), ("loss", _p)]


class BceJob(ctypes.Structure):
    """SggBceJob (include/sgg.h): a BCE loss value of sgg_grad_finish_losses."""
    _fields_ = [("x", _p), ("n", _i), ("split", _i), ("ya", _p), ("yb", _p), ("w", _f), ("loss", _p),
                ("addend", _p), ("total", _p), ("nvalid", _p)]


# name -> (restype, argtypes); must mirror include/sgg.h exactly
SIGNATURES = {
    "sgg_version": (_i, []),
    "sgg_last_error": (ctypes.c_char_p, []),
    "sgg_source_hash": (ctypes.c_char_p, []),
    "sgg_xw": (_i, [_p, _i, _p, _i, _p, _i, _i, _p, _p, _i, _i, _i, _i, _i, _p]),
    "sgg_xw_bf16": (_i, [_p, _i, _p, _i, _p, _i, _i, _p, _p, _i, _i, _i, _i, _i, _p]),
    "sgg_pool_plan": (_i, [_p, _i, _i, _i, _i, _p, _i, _p, _p]),
    "sgg_pool_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p]),
    "sgg_pool_plan_bf16": (_i, [_p, _i, _i, _i, _p, _i, _p, _p]),
    "sgg_pool_fwd_bf16": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p]),
    "sgg_pool_fwd2": (_i, [ctypes.POINTER(PoolBatch), ctypes.POINTER(PoolBatch), _p, _p, _p, _i, _i, _p]),
    "sgg_pool_bwd_grid": (_i, [_i]),
    "sgg_pool_dh_dw": (_i, [_p, _i, _p, _i, _p, _i, _i, _p, _i, _i, _i, _p, _sz, _p]),
    "sgg_pool_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p]),
    "sgg_gat_fwd": (_i, [_p, _i, _p, _p, _p, _p, _i, _i, _i, _f, _i, _i, _i, _p, _p, _i, _p]),
    "sgg_gat_bwd": (_i, [_p, _i, _p, _p, _p, _i, _i, _i, _f, _i, _i, _i, _p, _p, _p, _i, _p, _p, _p, _p]),
    "sgg_gat_fwd_ex": (_i, [_p, _i, _p, _p, _p, _p, _p, _i, _i, _i, _f, _i, _i, _i, _p, _p, _i, _p]),
    "sgg_gat_bwd_ex": (_i, [_p, _i, _p, _p, _p, _p, _i, _i, _i, _f, _i, _i, _i, _p, _p, _p, _i, _p, _p, _p, _p, _p,
                            _p]),
    "sgg_gat_bwd_ex_work_bytes": (_sz, [_i, _i, _i]),
    "sgg_gat_layer_lds_bytes": (_sz, [_i, _i, _i]),
    "sgg_gat_layer_fwd": (_i, [_p, _i, _i, _p, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _f, _f, _i, _i, _i, _p, _p,
                               _p, _p, _p, _i, _p]),
    "sgg_gat_layer_fwd2": (_i, [ctypes.POINTER(GatLayerSet), ctypes.POINTER(GatLayerSet), _p, _p, _p, _p, _i, _i, _f,
                                _f, _i, _i, _p]),
    "sgg_seg_norm_fwd": (_i, [_p, _i, _i, _p, _i, _f, _p, _i, _p, _p]),
    "sgg_seg_norm_bwd": (_i, [_p, _i, _p, _i, _i, _p, _i, _p, _p, _i, _p]),
    "sgg_group_index_ws": (_sz, [_i, _i]),
    "sgg_group_index": (_i, [_p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p]),
    "sgg_seg_reduce": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _i, _i, _p, _i, _p]),
    "sgg_seg_gather": (_i, [_p, _i, _i, _p, _p, _p, _i, _p, _i, _p]),
    "sgg_xtw_splits": (_i, [_i, _i, _i]),
    "sgg_lstm_bwd_split": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p]),
    "sgg_lstm_bwd_tail": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p]),
    "sgg_lstm_fwd_seg": (_i, [_sargs, _i, _p]),
    "sgg_lstm_fwd_seg2": (_i, [_sargs, _i, _sargs, _i, _p]),
    "sgg_lstm_fwd_seg3": (_i, [_sargs, _i, _sargs, _i, _sargs, _i, _p]),
    "sgg_lstm_bwd_shared": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _p, _p]),
    "sgg_lstm_u_ok": (_i, [_i, _i, _i, _i, _i, _i]),
    "sgg_lstm_fwd_u": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _i, _p, _i, _p, _p]),
    "sgg_head_ok": (_i, [_i, _i]),
    "sgg_head_slab_cols": (_i, [_i, _i]),
    "sgg_head_fwd": (_i, [_p, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _p]),
    "sgg_head_bwd": (_i, [_p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i, _p, _i, _p, _p, _p, _p, _i, _f, _p, _p]),
    "sgg_head_fwdbwd": (_i, [_p, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _i, _p, _p, _p, _p, _i, _f, _p, _p]),
    "sgg_xtw_partial": (_i, [_p, _i, _p, _i, _p, _i, _i, _i, _i, _i, _p, _sz, _p]),
    "sgg_grad_finish": (_i, [ctypes.POINTER(Red), _i, ctypes.POINTER(FoldBwd), _i, _p, _sz, _p]),
    "sgg_lstm_fwd_dec": (_i, [ctypes.POINTER(DecInit), _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p,
                              ctypes.POINTER(TrajOut), _p]),
    "sgg_lstm_fwd_dec2": (_i, [ctypes.POINTER(DecInit), ctypes.POINTER(DecInit), _p, _p, _p, _p, _p, _i, _i, _i, _i,
                               _p, _p, ctypes.POINTER(TrajOut), _p]),
    "sgg_lstm_fwd_dec_seg": (_i, [ctypes.POINTER(DecInit), _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p,
                                  ctypes.POINTER(TrajOut), _sargs, _i, _p]),
    "sgg_grad_finish_losses": (_i, [ctypes.POINTER(Red), _i, ctypes.POINTER(FoldBwd), _i, _p, _sz,
                                    ctypes.POINTER(L2Job), _i, ctypes.POINTER(BceJob), _i, _p]),
    "sgg_adam_parts": (_i, [ctypes.c_longlong]),
    "sgg_adam_step": (_i, [_p, _p, _p, _p, _p, _i, ctypes.c_double, ctypes.c_double, ctypes.c_double, _f, _f, _p, _p,
                          _sz, _p]),
    "sgg_xtw": (_i, [_p, _i, _p, _i, _p, _i, _i, _i, _i, _p, _i, _i, _p, _p, _sz, _p]),
    "sgg_fold_fwd": (_i, [_p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p]),
    "sgg_fold_fwd_multi": (_i, [ctypes.POINTER(Fold), _i, _p]),
    "sgg_fold_bwd": (_i, [_p, _i, _i, _i, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "sgg_lstm_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p]),
    "sgg_lstm_state_floats": (ctypes.c_longlong, [_i, _i, _i, _i]),
    "sgg_lstm_wpart_rows": (_i, [_i, _i]),
    "sgg_lstm_kernel_name": (ctypes.c_char_p, [_i, _i, _i, _i, _i]),
    "sgg_lstm_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p]),
    "sgg_bce_fwd": (_i, [_p, _i, _i, _p, _p, _f, _p, _p, _p, _p, _p]),
    "sgg_bce_bwd": (_i, [_p, _i, _i, _p, _p, _f, _p, _p, _p, _p]),
    "sgg_gatenc_param_size": (_i, [_i]),
    "sgg_gatenc_lds_bytes": (ctypes.c_longlong, [_i, _i, _i]),
    "sgg_gatenc_saved_floats": (ctypes.c_longlong, [_i, _i, _i]),
    "sgg_gatenc_fwd": (_i, [_pargs, _p]),
    "sgg_gatenc_fwd2": (_i, [_pargs, _pargs, _p]),
    "sgg_gatenc_bwd": (_i, [_pargs, _p]),
    "sgg_gcnmod_param_size": (_i, [_i, _i]),
    "sgg_gcnmod_slab_rows": (_i, [_i]),
    "sgg_gcnmod_lds_bytes": (ctypes.c_longlong, [_i, _i, _i, _i]),
    "sgg_gcnmod_fwd": (_i, [_gargs, _p]),
    "sgg_gcnmod_fwd2": (_i, [_gargs, _gargs, _p]),
    "sgg_gcnmod_bwd": (_i, [_gargs, _p]),
    "sgg_slab_reduce": (_i, [_p, _i, _i, _p, _p]),
    "sgg_gather_batch_floats": (ctypes.c_longlong, [_i, _i, _i]),
    "sgg_gather_batch": (_i, [_p, _i, _p, _i, _i, _i, _p, _p]),
    "sgg_traj_cat": (_i, [_p, _i, _i, _p, _i, _p, _i, _i, _i, _p, _p, _p, _p]),
    "sgg_decoder_init": (_i, [_p, _i, _i, _p, _i, _p, _i, _i, _p, _i, _i, _p, _p, _p, _p]),
    "sgg_l2_select": (_i, [_p, _p, _p, _i, _p, _i, _i, _i, _i, _p, _p]),
    "sgg_l2_loss_fwd": (_i, [_p, _i, _p, _p, _i, _p, _i, _i, _i, _f, _p, _p, _p, _p]),
    "sgg_l2_loss_bwd": (_i, [_p, _i, _p, _p, _i, _p, _p, _i, _i, _f, _p, _p, _i, _p]),
    "sgg_l2_loss_bwd_scenes": (_i, [_p, _i, _p, _p, _i, _p, _i, _i, _i, _f, _p, _p, _i, _p, _p]),
}

_lib = None


class NativeError(RuntimeError):
    pass


def lib_path():
    return _LIB_PATH


def built_hash():
    """The source hash compiled into the loaded library."""
    return load(require_gpu=False).sgg_source_hash().decode()


def load(require_gpu=True):
    """Load libsgg.so (once).  Raises NativeError when it is missing, when it
    was built from other sources than this tree's (`sgg_source_hash()` vs
    `_srchash.source_hash()`; skipped only for an explicit SGG_LIB) or, with
    require_gpu, when no HIP device is visible: there is no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise NativeError("libsgg.so not built at %s -- run group-gan-gcn-gat_amd/build_native.py "
                              "(or __graft_entry__.build())" % _LIB_PATH)
        lib = ctypes.CDLL(_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if not _LIB_EXPLICIT:
            built, tree = lib.sgg_source_hash().decode(), source_hash()
            if built != tree:
                raise NativeError("%s was built from other sources (hash %s) than this tree's csrc/ + "
                                  "include/sgg.h (%s) -- rebuild with group-gan-gcn-gat_amd/build_native.py"
                                  % (_LIB_PATH, built[:16], tree[:16]))
        _lib = lib
    if require_gpu and not torch.cuda.is_available():
        raise NativeError("sgan: no HIP device visible; the MI355X kernels have no CPU fallback")
    return _lib


def check(rc, name):
    if rc != 0:
        msg = _lib.sgg_last_error().decode(errors="replace")
        raise NativeError("%s failed (rc=%d): %s" % (name, rc, msg))


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Asserts device + contiguity
    of the innermost dim; callers pass explicit leading dimensions."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())
