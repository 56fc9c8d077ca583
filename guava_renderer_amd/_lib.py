"""Loader for the gfx950 rasterizer library (guava_renderer_amd/lib/libgsr.so, C ABI include/gsr.h).

There is no CPU fallback: if the library is missing or fails to load, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libgsr.so")

# every symbol declared in include/*.h
EXPORTS = ("gsr_version", "gsr_last_error", "gsr_geometry_bytes",
           "gsr_image_bytes", "gsr_binning_bytes", "gsr_mark_visible", "gsr_forward", "gsr_forward_ex",
           "gsr_forward_async_bound", "gsr_forward_async",
           "gsr_backward", "gsr_backward_ex", "gsr_batch_workspace_bytes", "gsr_forward_batch",
           "gsr_backward_batch", "gsr_backward_batch_shared", "gsr_batch_status", "gsr_profile_enable", "gsr_profile_read",
           "gsr_render_counters", "gsr_render_timeline", "gsr_forward_batch_refine",
           "gsr_refine_prepare", "gsr_batch_status_offset", "gsr_frames_to8b",
           "gsr_stream_create_cu_mask", "gsr_stream_destroy", "gsr_set_render_stream",
           # include/gsr_deform.h
           "gsr_lbs_workspace_bytes", "gsr_lbs", "gsr_lbs_sp", "gsr_blend_joints", "gsr_blend_joints_sp",
           "gsr_lbs_tiled_floats", "gsr_lbs_tile_bases",
           "gsr_scratch_geometry", "gsr_scratch_binning", "gsr_scratch_image", "gsr_forward_batch_deformed",
           "gsr_splice_head",
           "gsr_pack_rows", "gsr_deform_gaussians", "gsr_ehm_workspace_bytes", "gsr_ehm_forward",
           # include/gsr_ssim.h
           "gsr_fused_ssim", "gsr_fused_ssim_backward", "gsr_image_loss_partials", "gsr_image_loss")

# per-call numerics flags (include/gsr.h GSR_NUMERICS_*); 0 = bit-identical to the CPU oracle
NUMERICS_EXACT = 0
NUMERICS_FAST_EXP = 1
NUMERICS_SPLIT_BF16 = 2
# same flag word, batched forward only: no backward will read the workspace (include/gsr.h)
FORWARD_ONLY = 0x100


def numerics(fast_exp=False, split_bf16=False):
    """The `numerics` flag word of one call (include/gsr.h)."""
    return (NUMERICS_FAST_EXP if fast_exp else 0) | (NUMERICS_SPLIT_BF16 if split_bf16 else 0)


ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float
_sz = ctypes.c_size_t
_u32 = ctypes.c_uint32

_lib = None


class RefineEpilogue(ctypes.Structure):
    """gsr_refine_epilogue (include/gsr.h)."""
    _fields_ = [("weight", _vp), ("bias", _vp), ("n_out", _i), ("negative_slope", _f),
                ("out_refine", _vp), ("keep_channels", _i)]


class Scratch(ctypes.Structure):
    """gsr_scratch (include/gsr.h): preallocated buffers for the three forward resizers."""
    _fields_ = [("geometry", _vp), ("geometry_cap", _sz), ("binning", _vp), ("binning_cap", _sz),
                ("image", _vp), ("image_cap", _sz)]


class DeformInputs(ctypes.Structure):
    """GsrDeformInputs (include/gsr_deform.h): the assembly inputs of gsr_forward_batch_deformed."""
    _fields_ = [("V", _i), ("F", _i), ("N", _i), ("pad_", _i), ("verts", _vp), ("vert_transforms", _vp),
                ("faces", _vp), ("vtx_rotations", _vp), ("vtx_rot_stride", _i64), ("vtx_scales", _vp),
                ("vtx_scale_stride", _i64), ("binding_face", _vp), ("face_bary", _vp), ("local_xyz", _vp),
                ("local_stride", _i64), ("uv_rotations", _vp), ("uv_rot_stride", _i64), ("uv_scales", _vp),
                ("uv_scale_stride", _i64), ("bad_index_flag", _vp)]


class RowSegment(ctypes.Structure):
    """GsrRowSegment (include/gsr_deform.h)."""
    _fields_ = [("src", _vp), ("dst", _vp), ("src_stride", _i64), ("dst_stride", _i64), ("width", _i),
                ("pad_", _i)]


class LbsSparse(ctypes.Structure):
    """GsrLbsSparse (include/gsr_deform.h)."""
    _fields_ = [("jreg_row", _vp), ("jreg_col", _vp), ("jreg_val", _vp), ("skin_k", ctypes.c_int32),
                ("pad_", ctypes.c_int32), ("skin_joint", _vp), ("skin_weight", _vp),
                ("shapedirs_tiled", _vp), ("posedirs_tiled", _vp), ("shapedirs_tiled_k", ctypes.c_int32),
                ("shapedirs_tiled_m", ctypes.c_int32), ("posedirs_tiled_k", ctypes.c_int32),
                ("posedirs_tiled_m", ctypes.c_int32)]


class EhmModel(ctypes.Structure):
    """GsrEhmModel (include/gsr_deform.h)."""
    _fields_ = [("V", ctypes.c_int32), ("J", ctypes.c_int32), ("NB", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("v_template", _vp), ("shapedirs_t", _vp), ("posedirs", _vp), ("J_regressor", _vp),
                ("lbs_weights_t", _vp), ("parents_host", _vp), ("sparse", ctypes.POINTER(LbsSparse))]


class Ehm(ctypes.Structure):
    """GsrEhm (include/gsr_deform.h)."""
    _fields_ = [("flame", EhmModel), ("body", EhmModel), ("head_index", _vp), ("l_eyelid", _vp),
                ("r_eyelid", _vp), ("N_head", ctypes.c_int32), ("hj0", ctypes.c_int32), ("hj1", ctypes.c_int32),
                ("bj0", ctypes.c_int32), ("bj1", ctypes.c_int32), ("pad_", ctypes.c_int32), ("bad_index_flag", _vp)]


class EhmParam(ctypes.Structure):
    """GsrEhmParam (include/gsr_deform.h)."""
    _fields_ = [("p", _vp), ("row_stride", _i64), ("width", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class EhmOutputs(ctypes.Structure):
    """GsrEhmOutputs (include/gsr_deform.h)."""
    _fields_ = [("vertices", _vp), ("joints", _vp), ("joints_transform", _vp), ("ver_transform_mat", _vp),
                ("joint_transform_mat", _vp)]


# GsrEhmParam slots (include/gsr_deform.h GSR_EHM_*)
EHM_SLOTS = ("flame.shape_params", "flame.expression_params", "flame.jaw_params", "flame.eye_pose_params",
             "flame.eyelid_params", "body.shape", "body.exp", "body.global_pose", "body.body_pose",
             "body.left_hand_pose", "body.right_hand_pose", "body.head_scale", "body.joints_offset")


class GsrError(RuntimeError):
    pass


class CapacityError(GsrError):
    """A batched forward needed more Gaussian-tile instances than its workspace holds (that call's
    images were filled with NaN)."""


def load(path=None):
    """Load libgsr.so (building it first when hipcc is available and the .so is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("GSR_LIB") or LIB_PATH  # GSR_LIB: A/B builds (tools/gpu_abl.sh)
    # torch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7) and loads it by the
    # unversioned name; load torch first so libgsr.so binds to that same HIP runtime instead of
    # pulling /opt/rocm's copy into the process as a second runtime.
    import torch  # noqa: F401
    if not os.path.exists(path):
        try:
            from . import build as _build
            _build.build(verbose=False)
        except Exception as e:  # noqa: BLE001
            raise GsrError(f"libgsr.so not found at {path} and could not be built: {e}") from e
    L = ctypes.CDLL(path)
    L.gsr_version.restype = ctypes.c_char_p
    # stale-build guard: the library carries the hash of the sources it was built from
    built = L.gsr_version().decode().split()[-1]
    if path == LIB_PATH and os.environ.get("GSR_ALLOW_STALE") != "1":
        from . import build as _build
        if os.path.isdir(_build.CSRC) and built != _build.source_hash():
            raise GsrError(f"{path} was built from other sources (hash {built}, tree {_build.source_hash()}): "
                           "rebuild with `python -m guava_renderer_amd.build` (GSR_ALLOW_STALE=1 overrides)")
    L.gsr_last_error.restype = ctypes.c_char_p
    L.gsr_geometry_bytes.argtypes = [_i, _i, _i]
    L.gsr_geometry_bytes.restype = _sz
    L.gsr_image_bytes.argtypes = [_i, _i]
    L.gsr_image_bytes.restype = _sz
    L.gsr_binning_bytes.argtypes = [_i64]
    L.gsr_binning_bytes.restype = _sz
    L.gsr_mark_visible.argtypes = [_i, _vp, _vp, _vp, _vp, _vp]
    L.gsr_mark_visible.restype = _i
    L.gsr_forward.argtypes = [ALLOC_FN, ALLOC_FN, ALLOC_FN, _vp, _i, _i, _i, _vp, _i, _i, _vp, _vp,
                              _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, _vp, _i,
                              _vp, _i, _vp]
    L.gsr_forward.restype = _i
    L.gsr_forward_ex.argtypes = list(L.gsr_forward.argtypes[:-1]) + [_u32, _vp]
    L.gsr_forward_ex.restype = _i
    L.gsr_forward_async_bound.argtypes = [_i, _i, _i]
    L.gsr_forward_async_bound.restype = _i64
    L.gsr_forward_async.argtypes = list(L.gsr_forward.argtypes[:-1]) + [_vp, _u32, _vp]
    L.gsr_forward_async.restype = _i
    L.gsr_backward.argtypes = [_i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp,
                               _vp, _vp, _vp, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]
    L.gsr_backward.restype = _i
    L.gsr_backward_ex.argtypes = list(L.gsr_backward.argtypes[:-1]) + [_u32, _vp]
    L.gsr_backward_ex.restype = _i
    L.gsr_batch_workspace_bytes.argtypes = [_i, _i, _i, _i, _i64]
    L.gsr_batch_workspace_bytes.restype = _sz
    L.gsr_batch_status_offset.argtypes = [_i, _i, _i, _i, _i64]
    L.gsr_batch_status_offset.restype = _sz
    L.gsr_forward_batch.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                    _i64, _f, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i,
                                    _u32, _vp]
    L.gsr_forward_batch.restype = _i
    L.gsr_forward_batch_refine.argtypes = list(L.gsr_forward_batch.argtypes[:-2]) + [
        ctypes.POINTER(RefineEpilogue), _u32, _vp]
    L.gsr_forward_batch_refine.restype = _i
    L.gsr_forward_batch_deformed.argtypes = [_i, _i, _i, ctypes.POINTER(DeformInputs), _vp, _i64, _vp, _i64, _f,
                                             _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i, _u32, _vp]
    L.gsr_forward_batch_deformed.restype = _i
    L.gsr_refine_prepare.argtypes = [_i, _vp, _vp, _i, _i, _vp, _vp]
    L.gsr_refine_prepare.restype = _i
    L.gsr_backward_batch.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                     _i64, _f, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _u32, _vp]
    L.gsr_backward_batch.restype = _i
    L.gsr_backward_batch_shared.argtypes = list(L.gsr_backward_batch.argtypes[:24]) + [_vp, _vp, _vp, _vp, _vp,
                                                                                       _i, _u32, _vp]
    L.gsr_backward_batch_shared.restype = _i
    L.gsr_batch_status.argtypes = [_vp, _i, _i, ctypes.POINTER(_i64), ctypes.POINTER(_i), _vp]
    L.gsr_batch_status.restype = _i
    L.gsr_profile_enable.argtypes = [ctypes.c_uint32]
    L.gsr_profile_enable.restype = _i
    L.gsr_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i), _i]
    L.gsr_profile_read.restype = _i
    L.gsr_render_counters.argtypes = [_vp]
    L.gsr_render_counters.restype = _i
    L.gsr_render_timeline.argtypes = [_vp, ctypes.c_uint32]
    L.gsr_render_timeline.restype = _i
    L.gsr_frames_to8b.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _vp]
    L.gsr_frames_to8b.restype = _i
    L.gsr_stream_create_cu_mask.argtypes = [_u32, ctypes.POINTER(_u32), ctypes.POINTER(_vp)]
    L.gsr_stream_create_cu_mask.restype = _i
    L.gsr_stream_destroy.argtypes = [_vp]
    L.gsr_stream_destroy.restype = _i
    L.gsr_set_render_stream.argtypes = [_vp, _vp]
    L.gsr_set_render_stream.restype = _i
    L.gsr_lbs_workspace_bytes.argtypes = [_i, _i, _i, _i]
    L.gsr_lbs_workspace_bytes.restype = _sz
    L.gsr_lbs_tiled_floats.argtypes = [_i, _i]
    L.gsr_lbs_tiled_floats.restype = _sz
    L.gsr_lbs_tile_bases.argtypes = [_i, _i, _vp, _vp, _vp]
    L.gsr_lbs_tile_bases.restype = _i
    L.gsr_lbs.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                          _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.gsr_lbs.restype = _i
    L.gsr_lbs_sp.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                             _vp, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(LbsSparse), _vp]
    L.gsr_lbs_sp.restype = _i
    L.gsr_blend_joints.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.gsr_blend_joints.restype = _i
    L.gsr_blend_joints_sp.argtypes = [_i, _i, _i, _i, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                      ctypes.POINTER(LbsSparse), _vp]
    L.gsr_blend_joints_sp.restype = _i
    L.gsr_splice_head.argtypes = [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _i,
                                  _i, _i, _vp, _vp, _vp]
    L.gsr_splice_head.restype = _i
    L.gsr_pack_rows.argtypes = [_i, _i, ctypes.POINTER(RowSegment), _vp]
    L.gsr_pack_rows.restype = _i
    L.gsr_deform_gaussians.argtypes = [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp,
                                       _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp]
    L.gsr_deform_gaussians.restype = _i
    L.gsr_ehm_workspace_bytes.argtypes = [ctypes.POINTER(Ehm), _i]
    L.gsr_ehm_workspace_bytes.restype = _sz
    L.gsr_ehm_forward.argtypes = [ctypes.POINTER(Ehm), _i, ctypes.POINTER(EhmParam), ctypes.POINTER(EhmOutputs),
                                  _vp, _vp]
    L.gsr_ehm_forward.restype = _i
    L.gsr_fused_ssim.argtypes = [_i, _i, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.gsr_fused_ssim.restype = _i
    L.gsr_fused_ssim_backward.argtypes = [_i, _i, _i, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.gsr_fused_ssim_backward.restype = _i
    L.gsr_image_loss_partials.argtypes = [_i, _i, _i]
    L.gsr_image_loss_partials.restype = _i
    L.gsr_image_loss.argtypes = [_i, _i, _i, _vp, _vp, _vp, _f, _f, _vp, _vp, _vp, _vp]
    L.gsr_image_loss.restype = _i
    _lib = L
    return L


def check(rc, what):
    """Raise with the library's message for a negative return code; return rc otherwise."""
    if rc < 0:
        msg = load().gsr_last_error().decode(errors="replace")
        raise GsrError(f"{what} failed ({-rc}): {msg}")
    return rc

