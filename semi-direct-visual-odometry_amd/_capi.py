"""ctypes binding of libsvo_hip.so (the C ABI declared in include/svo_c.h).

The library is the product: there is no fallback.  If it is missing, or no gfx950 device is visible,
every entry point raises — nothing silently runs on the CPU.
"""
import ctypes
import os

from . import _paths

c_int32, c_double, c_void_p, c_uint8 = ctypes.c_int32, ctypes.c_double, ctypes.c_void_p, ctypes.c_uint8
P_i32 = ctypes.POINTER(c_int32)
P_dbl = ctypes.POINTER(c_double)
P_u8 = ctypes.POINTER(c_uint8)

SVO_OK, SVO_ERR_ARG, SVO_ERR_HIP, SVO_ERR_NODEV, SVO_ERR_STATE = 0, -1, -2, -3, -4

STATUS_NAMES = {0: "Success", 1: "Max_Coff_Dx", 2: "Non_In_Dx", 3: "Small_Step_Size", 4: "Lambda_Value",
                5: "Norm_Inf_Diff", 6: "Non_Suff_Points", 7: "Increase_Chi_Squred_Error",
                8: "Small_Chi_Squred_Error", 9: "Failed"}


class SvoCamera(ctypes.Structure):
    _fields_ = [("fx", c_double), ("fy", c_double), ("cx", c_double), ("cy", c_double),
                ("width", c_int32), ("height", c_int32)]


class SvoAlignParams(ctypes.Structure):
    _fields_ = [("patch_size", c_int32), ("min_level", c_int32), ("max_level", c_int32), ("median_mode", c_int32)]


class SvoDepthSeed(ctypes.Structure):
    _fields_ = [("a", c_double), ("b", c_double), ("mu", c_double), ("sigma", c_double), ("var", c_double),
                ("max_depth", c_double), ("px", c_double * 2), ("bearing", c_double * 3), ("kf", c_int32),
                ("valid", c_int32)]


DEPTH_OUTCOMES = {0: "Rejected", 1: "No_Match", 2: "Updated", 3: "Converged", 4: "NaN"}


class SvoLevelTrace(ctypes.Structure):
    _fields_ = [("level", c_int32), ("n_ref_vis", c_int32), ("n_vis", c_int32), ("status", c_int32),
                ("median", c_double), ("mad", c_double), ("sigma", c_double), ("chi2", c_double),
                ("lambda_", c_double), ("err", c_double), ("H", c_double * 36), ("g", c_double * 6),
                ("dx", c_double * 6), ("scale_kernel", c_int32), ("reserved", c_int32)]


# (name, restype, argtypes) for every entry point of include/svo_c.h
_SIGNATURES = [
    ("svo_device_count", c_int32, [P_i32]),
    ("svo_ctx_create", c_int32, [c_int32, ctypes.POINTER(c_void_p)]),
    ("svo_ctx_destroy", c_int32, [c_void_p]),
    ("svo_ctx_synchronize", c_int32, [c_void_p]),
    ("svo_ctx_stream", c_void_p, [c_void_p]),
    ("svo_last_error", ctypes.c_char_p, []),
    ("svo_abi_version", c_int32, []),
    ("svo_ctx_event_record", c_int32, [c_void_p, c_int32]),
    ("svo_ctx_event_elapsed", c_int32, [c_void_p, c_int32, c_int32, ctypes.POINTER(ctypes.c_float)]),
    ("svo_pyramid_set_create", c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, ctypes.POINTER(c_void_p)]),
    ("svo_pyramid_set_destroy", c_int32, [c_void_p]),
    ("svo_pyramid_set_upload", c_int32, [c_void_p, c_int32, c_int32, c_void_p]),
    ("svo_pyramid_set_upload_device", c_int32, [c_void_p, c_int32, c_int32, c_void_p]),
    ("svo_pyramid_set_build", c_int32, [c_void_p, c_int32, c_int32]),
    ("svo_pyramid_set_build_async", c_int32, [c_void_p, c_int32, c_int32]),
    ("svo_pyramid_set_download", c_int32, [c_void_p, c_int32, c_int32, c_int32, c_void_p]),
    ("svo_pyramid_level_size", c_int32, [c_void_p, c_int32, P_i32, P_i32]),
    ("svo_align_batch_create", c_int32, [c_void_p, ctypes.POINTER(SvoCamera), ctypes.POINTER(SvoAlignParams),
                                         c_int32, c_int32, ctypes.POINTER(c_void_p)]),
    ("svo_align_batch_destroy", c_int32, [c_void_p]),
    ("svo_align_batch_set_pair", c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_int32,
                                           c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                           c_void_p, c_void_p]),
    ("svo_align_batch_set_pairs", c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32]),
    ("svo_align_batch_set_initial_poses", c_int32, [c_void_p, c_void_p]),
    ("svo_align_batch_run", c_int32, [c_void_p]),
    ("svo_align_batch_profile", c_int32, [c_void_p, ctypes.POINTER(ctypes.c_float)]),
    ("svo_align_batch_results", c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    ("svo_align_batch_traces", c_int32, [c_void_p, c_int32, c_void_p]),
    ("svo_robust_scale_capacity", c_int32, [c_int32, c_void_p]),
    ("svo_debug_robust_scale", c_int32, [c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int64, c_int32, c_void_p, ctypes.c_int64]),
    ("svo_feature_align", c_int32, [c_void_p, ctypes.POINTER(SvoCamera), c_int32, c_void_p, c_void_p, c_int32,
                                    c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("svo_feature_align_multi", c_int32, [c_void_p, ctypes.POINTER(SvoCamera), c_int32, c_void_p, c_void_p, c_void_p,
                                          c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("svo_world2image", c_int32, [ctypes.POINTER(SvoCamera), c_void_p, c_int32, c_void_p, c_void_p]),
    ("svo_map_reproject_plan", c_int32, [ctypes.POINTER(SvoCamera), c_int32, c_int32, c_void_p, c_void_p,
                                         ctypes.c_uint64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                         c_void_p, c_void_p, P_i32, c_void_p, c_void_p, c_void_p, P_i32, P_i32]),
    ("svo_depth_seed_init", c_int32, [c_double, c_double, c_void_p]),
    ("svo_depth_update", c_int32, [c_void_p, ctypes.POINTER(SvoCamera), c_int32, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_int32, c_void_p, c_int32, c_void_p, P_i32, c_void_p, c_void_p,
                                   c_void_p, P_i32]),
    ("svo_feature_grid_size", c_int32, [c_int32, c_int32, c_int32, P_i32, P_i32]),
    ("svo_feature_detect", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, P_i32]),
    ("svo_feature_select_ssc", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                         c_int32, c_void_p, c_void_p, P_i32, P_i32]),
    ("svo_feature_select_by_value", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32,
                                              c_void_p, c_void_p, P_i32]),
    ("svo_pose_matrix3x4_inverse", c_int32, [c_void_p, c_void_p]),
    ("svo_format_kitti_pose", c_int32, [c_void_p, ctypes.c_char_p, c_int32]),
    ("svo_pose_optimize", c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
]

EXPORTED = [s[0] for s in _SIGNATURES]
_lib = None


class SvoError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"svo error {code}: {msg}")
        self.code = code


def lib_path():
    return _paths.lib_path("libsvo_hip.so")


def lib():
    """Load libsvo_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise SvoError(SVO_ERR_STATE, f"{path} is missing: build it with __graft_entry__.build() or "
                                          f"`make -C semi-direct-visual-odometry_amd`")
        L = ctypes.CDLL(path)
        for name, res, args in _SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.svo_abi_version() != 2:  # include/svo_c.h SVO_ABI_VERSION
            raise SvoError(SVO_ERR_STATE, "ABI version mismatch")
        _lib = L
    return _lib


def check(rc):
    if rc != SVO_OK:
        msg = lib().svo_last_error()
        raise SvoError(rc, msg.decode() if msg else "")
    return rc


def ptr(a):
    """Raw data pointer of a numpy array (or None)."""
    return None if a is None else a.ctypes.data_as(c_void_p)
