"""ctypes binding of libofl_codec.so (include/ofl_codec.h).

The product path has no CPU fallback: if the library is missing or no GPU is
visible, the codec raises.  torch is imported before the library is loaded so
that the library binds to the HIP runtime torch already loaded (both carry the
SONAME libamdhip64.so.7), making torch streams and device pointers valid here.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libofl_codec.so")
_lock = threading.Lock()
_lib = None

OFL_OK = 0
OFL_EINVAL, OFL_EHIP, OFL_ESPACE, OFL_EFORMAT = -1, -2, -3, -4

EXPORTS = (
    "ofl_version", "ofl_last_error", "ofl_eden_slice_plan", "ofl_eden_plan_create",
    "ofl_eden_plan_destroy", "ofl_eden_plan_set_schedule", "ofl_eden_plan_num_waves",
    "ofl_eden_plan_get_schedule", "ofl_eden_plan_set_row2", "ofl_eden_plan_set_pair", "ofl_eden_plan_set_sset", "ofl_eden_plan_set_fuse", "ofl_eden_plan_num_slices", "ofl_eden_plan_planes_bytes",
    "ofl_eden_plan_workspace_bytes", "ofl_eden_plan_tensor_info", "ofl_eden_plan_tensor_dims",
    "ofl_eden_encode", "ofl_eden_encode_wavg", "ofl_eden_decode", "ofl_eden_decode_add", "ofl_eden_encode_host", "ofl_eden_decode_host", "ofl_eden_encode_mapped", "ofl_eden_decode_mapped", "ofl_eden_encode_seeded", "ofl_copy_h2d_chunked", "ofl_eden_encode_host_x", "ofl_eden_decode_host_x", "ofl_copy_h2d_async", "ofl_copy_h2d_staged", "ofl_eden_plan_profile", "ofl_eden_plan_num_launches",
    "ofl_eden_plan_launch_info", "ofl_eden_plan_profile_collect", "ofl_serial_sum_f32", "ofl_serial_sum_f32_mt", "ofl_serial_sum_copy_f32",
    "ofl_serial_sum_f64", "ofl_host_copy_many", "ofl_serial_sums_many", "ofl_lossy_last_error", "ofl_lossy_workspace_bytes", "ofl_kmeans1d_fit",
    "ofl_kmeans1d_batch_workspace_bytes", "ofl_kmeans1d_batch", "ofl_kmeans1d_batch_tab",
    "ofl_kmeans1d_label", "ofl_sparsify_topk", "ofl_ternary_stats", "ofl_ternary_ranks", "ofl_lut_decode",
    "ofl_lut_decode_batch_workspace_bytes", "ofl_lut_decode_batch",
    "ofl_sparsify_topk_batch_workspace_bytes", "ofl_sparsify_topk_batch",
    "ofl_ternary_ranks_batch_workspace_bytes", "ofl_ternary_ranks_batch",
    "ofl_agg_last_error", "ofl_wavg_delta", "ofl_wavg_ranges_workspace_bytes", "ofl_wavg_delta_ranges",
    "ofl_wavg_range_sums_workspace_bytes", "ofl_wavg_delta_range_sums", "ofl_wavg_delta_seeds",
    "ofl_py_hash_doubles",
    "ofl_wavg_points_workspace_bytes", "ofl_wavg_delta_points", "ofl_apply_delta",
    "ofl_apply_delta_ranges", "ofl_wavg_delta32_ranges", "ofl_sub_f32_f64",
    "ofl_gzip_last_error", "ofl_gzip_ranks_workspace_bytes", "ofl_gzip_ranks_bound", "ofl_gzip_ranks", "ofl_gzip_ranks_to", "ofl_gzip_label_to", "ofl_side_stream",
    "ofl_gunzip_members", "ofl_gzip_member_index", "ofl_inflate_members", "ofl_inflate_tlz_workspace_bytes",
    "ofl_inflate_tlz", "ofl_inflate_tlz_async", "ofl_inflate_tlz_wait", "ofl_inflate_tlz_launch", "ofl_inflate_tlz_launch_lut", "ofl_inflate_tlz_check", "ofl_gzip_profile", "ofl_gzip_profile_collect",
)


class CodecError(RuntimeError):
    pass


def _bind(L):
    i64, i32, vp, sz = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    L.ofl_version.restype = ctypes.c_char_p
    L.ofl_last_error.restype = ctypes.c_char_p
    L.ofl_eden_slice_plan.argtypes = [i64, vp, vp, i32]
    L.ofl_eden_slice_plan.restype = i32
    L.ofl_eden_plan_create.argtypes = [i32, vp, vp, vp, vp, i32, ctypes.POINTER(vp)]
    L.ofl_eden_plan_create.restype = i32
    L.ofl_eden_plan_destroy.argtypes = [vp]
    L.ofl_eden_plan_destroy.restype = None
    L.ofl_eden_plan_set_schedule.argtypes = [vp, i64, i32]
    L.ofl_eden_plan_set_schedule.restype = i32
    L.ofl_eden_plan_set_row2.argtypes = [vp, i32]
    L.ofl_eden_plan_set_row2.restype = i32
    L.ofl_eden_plan_set_pair.argtypes = [vp, i32]
    L.ofl_eden_plan_set_pair.restype = i32
    L.ofl_eden_plan_set_sset.argtypes = [vp, i32]
    L.ofl_eden_plan_set_sset.restype = i32
    L.ofl_eden_plan_set_fuse.argtypes = [vp, i32]
    L.ofl_eden_plan_set_fuse.restype = i32
    L.ofl_eden_plan_num_waves.argtypes = [vp]
    L.ofl_eden_plan_num_waves.restype = i32
    L.ofl_eden_plan_get_schedule.argtypes = [vp, vp, vp]
    L.ofl_eden_plan_get_schedule.restype = i32
    for f in ("ofl_eden_plan_num_slices", "ofl_eden_plan_planes_bytes", "ofl_eden_plan_workspace_bytes"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = i64
    L.ofl_eden_plan_tensor_info.argtypes = [vp, i32, vp, vp, vp, vp]
    L.ofl_eden_plan_tensor_info.restype = i32
    L.ofl_eden_plan_tensor_dims.argtypes = [vp, i32, vp]
    L.ofl_eden_plan_tensor_dims.restype = i32
    L.ofl_eden_encode.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_eden_encode_wavg.argtypes = [vp, vp, vp, i32, ctypes.c_double, vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_eden_encode_wavg.restype = i32
    L.ofl_eden_encode.restype = i32
    L.ofl_eden_decode.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_eden_decode.restype = i32
    L.ofl_eden_decode_add.argtypes = [vp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_eden_decode_add.restype = i32
    L.ofl_eden_encode_host.argtypes = [vp, vp, vp, sz, sz, vp, vp, sz, sz, vp, sz, vp]
    L.ofl_eden_encode_host.restype = i32
    L.ofl_eden_decode_host.argtypes = [vp, vp, vp, sz, sz, sz, vp, vp, sz, vp, sz, vp]
    L.ofl_eden_decode_host.restype = i32
    L.ofl_eden_encode_seeded.argtypes = [vp, vp, sz, ctypes.c_uint32, vp, vp, sz, sz, vp, sz, vp]
    L.ofl_eden_encode_seeded.restype = i32
    L.ofl_copy_h2d_chunked.argtypes = [vp, vp, vp, i64, i64, i32, vp, vp]
    L.ofl_copy_h2d_chunked.restype = i32
    L.ofl_eden_encode_mapped.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp]
    L.ofl_eden_encode_mapped.restype = i32
    L.ofl_eden_decode_mapped.argtypes = [vp, vp, sz, sz, vp, vp, sz, vp]
    L.ofl_eden_decode_mapped.restype = i32
    u32 = ctypes.c_uint32
    L.ofl_eden_encode_host_x.argtypes = [vp, vp, sz, u32, vp, sz, vp, vp, sz, sz, vp, sz, vp]
    L.ofl_eden_encode_host_x.restype = i32
    L.ofl_eden_decode_host_x.argtypes = [vp, vp, sz, vp, i32, u32, vp, sz, sz, vp, vp, sz, vp, sz, vp]
    L.ofl_eden_decode_host_x.restype = i32
    L.ofl_copy_h2d_async.argtypes = [vp, vp, sz, vp]
    L.ofl_copy_h2d_async.restype = i32
    L.ofl_copy_h2d_staged.argtypes = [vp, vp, sz, i32, vp]
    L.ofl_copy_h2d_staged.restype = i32
    L.ofl_eden_plan_profile.argtypes = [vp, i32]
    L.ofl_eden_plan_profile.restype = i32
    L.ofl_eden_plan_num_launches.argtypes = [vp, i32]
    L.ofl_eden_plan_num_launches.restype = i32
    L.ofl_eden_plan_launch_info.argtypes = [vp, i32, i32, ctypes.c_char_p, i32, vp, vp, vp]
    L.ofl_eden_plan_launch_info.restype = i32
    L.ofl_eden_plan_profile_collect.argtypes = [vp, i32, vp, i32, vp]
    L.ofl_eden_plan_profile_collect.restype = i32
    L.ofl_lossy_last_error.restype = ctypes.c_char_p
    L.ofl_lossy_workspace_bytes.argtypes = [i64]
    L.ofl_lossy_workspace_bytes.restype = sz
    L.ofl_kmeans1d_fit.argtypes = [vp, i64, i32, i32, ctypes.c_uint64, i32, vp, vp, vp, vp, sz, vp]
    L.ofl_kmeans1d_fit.restype = i32
    L.ofl_kmeans1d_batch_workspace_bytes.argtypes = [i32, vp]
    L.ofl_kmeans1d_batch_workspace_bytes.restype = sz
    L.ofl_kmeans1d_batch.argtypes = [i32, vp, vp, vp, i32, i32, ctypes.c_uint64, i32, i32, vp, vp, vp, vp, vp,
                                     vp, vp, sz, vp]
    L.ofl_kmeans1d_batch.restype = i32
    L.ofl_kmeans1d_batch_tab.argtypes = [i32, vp, vp, vp, i32, i32, ctypes.c_uint64, i32, i32, vp, vp, vp, vp, vp, vp,
                                         vp, vp, sz, vp]
    L.ofl_kmeans1d_batch_tab.restype = i32
    L.ofl_kmeans1d_label.argtypes = [vp, i64, vp, i32, vp, vp, vp]
    L.ofl_kmeans1d_label.restype = i32
    L.ofl_sparsify_topk.argtypes = [vp, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_sparsify_topk.restype = i32
    L.ofl_ternary_stats.argtypes = [vp, i64, vp, vp, vp, vp, sz, vp]
    L.ofl_ternary_stats.restype = i32
    L.ofl_ternary_ranks.argtypes = [vp, i64, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp, vp]
    L.ofl_ternary_ranks.restype = i32
    L.ofl_lut_decode.argtypes = [vp, i64, vp, vp, i32, vp, vp]
    L.ofl_lut_decode.restype = i32
    L.ofl_lut_decode_batch_workspace_bytes.argtypes = [i32, i32]
    L.ofl_lut_decode_batch_workspace_bytes.restype = sz
    L.ofl_lut_decode_batch.argtypes = [i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, sz, vp]
    L.ofl_lut_decode_batch.restype = i32
    L.ofl_sparsify_topk_batch_workspace_bytes.argtypes = [i32, vp]
    L.ofl_sparsify_topk_batch_workspace_bytes.restype = sz
    L.ofl_sparsify_topk_batch.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_sparsify_topk_batch.restype = i32
    L.ofl_ternary_ranks_batch_workspace_bytes.argtypes = [i32]
    L.ofl_ternary_ranks_batch_workspace_bytes.restype = sz
    L.ofl_ternary_ranks_batch.argtypes = [i32, vp, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_ternary_ranks_batch.restype = i32
    L.ofl_agg_last_error.restype = ctypes.c_char_p
    L.ofl_wavg_delta.argtypes = [i32, vp, vp, ctypes.c_double, vp, i64, vp, vp, vp, vp]
    L.ofl_wavg_delta.restype = i32
    L.ofl_wavg_ranges_workspace_bytes.argtypes = [i32, i32]
    L.ofl_wavg_ranges_workspace_bytes.restype = sz
    L.ofl_wavg_delta_ranges.argtypes = [i32, vp, vp, ctypes.c_double, vp, i32, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_wavg_delta_ranges.restype = i32
    L.ofl_wavg_range_sums_workspace_bytes.argtypes = [i32, i32, i64]
    L.ofl_wavg_range_sums_workspace_bytes.restype = sz
    L.ofl_wavg_delta_range_sums.argtypes = [i32, vp, vp, ctypes.c_double, vp, i32, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_wavg_delta_range_sums.restype = i32
    L.ofl_wavg_delta_seeds.argtypes = [i32, vp, vp, ctypes.c_double, vp, i32, vp, vp, vp, i64, vp, vp, vp, vp, vp]
    L.ofl_wavg_delta_seeds.restype = i32
    L.ofl_py_hash_doubles.argtypes = [vp, i32, vp, vp]
    L.ofl_py_hash_doubles.restype = i32
    L.ofl_wavg_points_workspace_bytes.argtypes = [i32, i32]
    L.ofl_wavg_points_workspace_bytes.restype = sz
    L.ofl_wavg_delta_points.argtypes = [i32, vp, vp, ctypes.c_double, vp, i32, vp, vp, vp, vp, vp, sz, vp]
    L.ofl_wavg_delta_points.restype = i32
    L.ofl_apply_delta.argtypes = [vp, vp, i64, vp, vp]
    L.ofl_apply_delta.restype = i32
    L.ofl_sub_f32_f64.argtypes = [vp, vp, i64, vp, vp]
    L.ofl_sub_f32_f64.restype = i32
    L.ofl_apply_delta_ranges.argtypes = [vp, vp, vp, i32, vp, vp, i64, vp]
    L.ofl_apply_delta_ranges.restype = i32
    L.ofl_wavg_delta32_ranges.argtypes = [i32, vp, vp, ctypes.c_double, vp, i32, vp, vp, i64, vp, vp]
    L.ofl_wavg_delta32_ranges.restype = i32
    L.ofl_gzip_last_error.restype = ctypes.c_char_p
    L.ofl_gzip_ranks_workspace_bytes.argtypes = [i64]
    L.ofl_gzip_ranks_workspace_bytes.restype = sz
    L.ofl_gzip_ranks_bound.argtypes = [i64]
    L.ofl_gzip_ranks_bound.restype = sz
    L.ofl_gzip_ranks.argtypes = [vp, i64, vp, sz, vp, vp, sz, vp]
    L.ofl_gzip_ranks.restype = i32
    L.ofl_gzip_ranks_to.argtypes = [vp, i64, vp, sz, vp, sz, i32, vp, vp, sz, vp]
    L.ofl_gzip_ranks_to.restype = i32
    L.ofl_gzip_label_to.argtypes = [vp, i64, vp, i32, vp, sz, vp, sz, i32, vp, vp, sz, vp]
    L.ofl_gzip_label_to.restype = i32
    L.ofl_side_stream.argtypes = [i32, ctypes.POINTER(ctypes.c_void_p)]
    L.ofl_side_stream.restype = i32
    L.ofl_gunzip_members.argtypes = [vp, sz, vp, sz, vp, i32]
    L.ofl_gunzip_members.restype = i32
    L.ofl_gzip_member_index.argtypes = [vp, sz, vp, i64, vp, vp, vp, vp]
    L.ofl_gzip_member_index.restype = i32
    L.ofl_inflate_members.argtypes = [vp, vp, i64, ctypes.c_uint32, vp, sz, vp, sz, vp]
    L.ofl_inflate_members.restype = i32
    L.ofl_inflate_tlz_workspace_bytes.argtypes = [i64]
    L.ofl_inflate_tlz_workspace_bytes.restype = sz
    L.ofl_inflate_tlz.argtypes = [vp, vp, i64, vp, sz, vp, sz, vp]
    L.ofl_inflate_tlz.restype = i32
    L.ofl_inflate_tlz_async.argtypes = [vp, vp, i64, i64, vp, sz, vp, sz, vp]
    L.ofl_inflate_tlz_async.restype = i32
    L.ofl_inflate_tlz_wait.argtypes = [vp, vp, i64, vp, sz, vp, sz, vp]
    L.ofl_inflate_tlz_wait.restype = i32
    L.ofl_inflate_tlz_launch.argtypes = [vp, vp, i64, i64, vp, sz, vp, sz, vp]
    L.ofl_inflate_tlz_launch.restype = i32
    L.ofl_inflate_tlz_launch_lut.argtypes = [vp, vp, i64, i64, vp, sz, vp, sz, vp, vp, vp, i32, vp]
    L.ofl_inflate_tlz_launch_lut.restype = i32
    L.ofl_inflate_tlz_check.argtypes = [i64, vp, sz, vp]
    L.ofl_inflate_tlz_check.restype = i32
    L.ofl_gzip_profile.argtypes = [i32]
    L.ofl_gzip_profile.restype = i32
    L.ofl_gzip_profile_collect.argtypes = [vp, sz, vp, vp, i32, vp]
    L.ofl_gzip_profile_collect.restype = i32
    L.ofl_serial_sum_f32.argtypes = [vp, i64]
    L.ofl_serial_sum_f32.restype = ctypes.c_float
    L.ofl_serial_sum_f32_mt.argtypes = [vp, i64, vp, i32]
    L.ofl_serial_sum_f32_mt.restype = ctypes.c_float
    L.ofl_serial_sum_copy_f32.argtypes = [vp, vp, i64]
    L.ofl_serial_sum_copy_f32.restype = ctypes.c_float
    L.ofl_serial_sum_f64.argtypes = [vp, i64]
    L.ofl_serial_sum_f64.restype = ctypes.c_double
    L.ofl_host_copy_many.argtypes = [i32, vp, vp, vp, i32]
    L.ofl_host_copy_many.restype = i32
    L.ofl_serial_sums_many.argtypes = [i32, vp, vp, i32, vp, i32]
    L.ofl_serial_sums_many.restype = i32
    return L


def lib():
    """Load (once) and return the bound library; raise if it is not built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                import torch  # noqa: F401  (HIP runtime first; see module doc)
                path = os.environ.get("OFL_CODEC_LIB", LIB_PATH)  # dev: A/B a kernel variant
                if not os.path.exists(path):
                    raise CodecError(
                        f"{path} is missing: build it with `python -m openfl_amd.build` "
                        "(hipcc --offload-arch=gfx950); openfl_amd has no CPU fallback")
                _lib = _bind(ctypes.CDLL(path))
    return _lib


def check_lossy(rc):
    if rc != OFL_OK:
        raise CodecError(lib().ofl_lossy_last_error().decode() or f"libofl_codec error {rc}")
    return rc


def check_gzip(rc):
    if rc != OFL_OK:
        raise CodecError(lib().ofl_gzip_last_error().decode() or f"libofl_codec error {rc}")
    return rc


def check_agg(rc):
    if rc != OFL_OK:
        raise CodecError(lib().ofl_agg_last_error().decode() or f"libofl_codec error {rc}")
    return rc


def check(rc):
    if rc != OFL_OK:
        raise CodecError(lib().ofl_last_error().decode() or f"libofl_codec error {rc}")
    return rc
