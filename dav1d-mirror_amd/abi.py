"""ctypes / numpy mirror of include/dav1d_gpu.h (the C-ABI boundary).

Only plain pointers and sizes cross the boundary; torch is used by callers
for device memory and streams, never in these signatures.
"""
import ctypes
import os

import numpy as np

# RectTxfmSize order (src/levels.h:44-78) -> (w, h)
TX_WH = [(4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (4, 8), (8, 4), (8, 16),
         (16, 8), (16, 32), (32, 16), (32, 64), (64, 32), (4, 16), (16, 4),
         (8, 32), (32, 8), (16, 64), (64, 16)]
TX_INDEX = {wh: i for i, wh in enumerate(TX_WH)}
N_TX = len(TX_WH)

DCT_DCT, IDTX, H_DCT, WHT_WHT = 0, 9, 11, 16
NO_RESIDUAL = 0xFF          # txtp value: prediction only (no inv_txfm_add)

PRED_NONE, PRED_INTER, PRED_INTER_AVG, PRED_INTRA, PRED_CFL = 0, 1, 2, 3, 4
PRED_INTER_WAVG, PRED_INTER_MASK, PRED_PAL, PRED_WARP, PRED_INTER_INTRA = 5, 6, 7, 8, 9
PRED_INTER_WMASK, PRED_INTER_OBMC, PRED_INTER_SCALED = 10, 11, 12
SECOND_LAUNCH_KINDS = (PRED_WARP, PRED_INTER_INTRA, PRED_INTER_WMASK, PRED_INTER_OBMC,
                       PRED_INTER_SCALED)   # the batch's class_warp sub-ranges
INTER_KINDS = (PRED_INTER, PRED_INTER_AVG, PRED_INTER_WAVG, PRED_INTER_MASK)
COMPOUND_KINDS = (PRED_INTER_AVG, PRED_INTER_WAVG, PRED_INTER_MASK)
FILTER_2D_BILINEAR = 9

(DC_PRED, VERT_PRED, HOR_PRED, LEFT_DC_PRED, TOP_DC_PRED, DC_128_PRED, Z1_PRED,
 Z2_PRED, Z3_PRED, SMOOTH_PRED, SMOOTH_V_PRED, SMOOTH_H_PRED, PAETH_PRED,
 FILTER_PRED) = range(14)

MAX_REFS = 8


def itx_supported(tx, tp):
    """The reference's instantiated (size, type) pairs, src/itx_tmpl.c:142-160."""
    if tp == WHT_WHT:
        return tx == 0
    w, h = TX_WH[tx]
    m = max(w, h)
    if m == 64:
        return tp == DCT_DCT
    if m == 32:
        return tp in (DCT_DCT, IDTX)
    if w == 16 and h == 16:
        return tp <= H_DCT
    return True


# Dav1dGpuUnit, 32 bytes, with the inter / intra union as overlapping fields;
# every byte belongs to a field so copies never carry uninitialised padding.
UNIT_DTYPE = np.dtype({
    "names": ["dst_off", "coef_off", "tx", "txtp", "plane", "pred", "nzw", "nzh",
              "bw4", "bh4",
              "src_off0", "src_off1", "mx0", "mx1", "my0", "my1", "filter2d", "ref0", "ref1",
              "weight", "edge_off", "angle", "mode", "pad_intra", "max_w", "max_h",
              "cfl_alpha", "cfl_pad_wh", "cfl_luma_off"],
    "formats": ["<i4", "<i4", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "u1",
                "<i4", "<i4", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "u1",
                "<i4", "<u2", "u1", "u1", "<u2", "<u2",
                "i1", "u1", "<i4"],
    "offsets": [0, 4, 8, 9, 10, 11, 12, 13, 14, 15,
                16, 20, 24, 25, 26, 27, 28, 29, 30, 31,
                16, 20, 22, 23, 24, 26,
                20, 21, 28],
    "itemsize": 32,
})


class Plane(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("stride", ctypes.c_int64),
                ("w", ctypes.c_int32), ("h", ctypes.c_int32)]


class FrameBatch(ctypes.Structure):
    _fields_ = [("dst", Plane * 3),
                ("ref", (Plane * 3) * MAX_REFS),
                ("units", ctypes.c_void_p),
                ("n_units", ctypes.c_int32),
                ("class_start", ctypes.c_int32 * (N_TX + 1)),
                ("coef", ctypes.c_void_p),
                ("edges", ctypes.c_void_p),
                ("bitdepth_max", ctypes.c_int32),
                ("zero_coefs", ctypes.c_int32),
                ("cfl_luma", Plane),
                ("cfl_ss", ctypes.c_int32),
                ("aux", ctypes.c_void_p),
                ("aux_pool", ctypes.c_void_p),
                ("class_warp", ctypes.c_int32 * N_TX)]


class TileBatch(ctypes.Structure):
    _fields_ = [("dst", Plane * 3),
                ("ref", (Plane * 3) * MAX_REFS),
                ("tiles", ctypes.c_void_p),
                ("n_tiles", ctypes.c_int32),
                ("n_tiles_huge", ctypes.c_int32),
                ("bitdepth_max", ctypes.c_int32),
                ("preds", ctypes.c_void_p),
                ("txs", ctypes.c_void_p),
                ("coef", ctypes.c_void_p),
                ("edges", ctypes.c_void_p),
                ("aux_pool", ctypes.c_void_p),
                ("cfl_luma", Plane),
                ("cfl_ss", ctypes.c_int32),
                ("zero_coefs", ctypes.c_int32)]


# Dav1dGpuIntraEdge (16 bytes) and its batch: device dav1d_prepare_intra_edges
INTRA_EDGE_DTYPE = np.dtype([("unit", "<i4"), ("x4", "<i2"), ("y4", "<i2"), ("w4", "<i2"), ("h4", "<i2"),
                             ("mode", "u1"), ("angle", "i1"), ("flags", "u1"), ("pad", "u1")])
IE_HAVE_LEFT, IE_HAVE_TOP, IE_TOP_HAS_RIGHT, IE_LEFT_HAS_BOTTOM = 1, 2, 4, 8
IE_FILTER_EDGE, IE_SMOOTH, IE_TOP_SB_EDGE = 16, 32, 64


class IntraEdgeBatch(ctypes.Structure):
    _fields_ = [("pic", Plane * 3),
                ("top_edge", Plane * 3),
                ("sb_log2", ctypes.c_int32 * 3),
                ("units", ctypes.c_void_p),
                ("edges", ctypes.c_void_p),
                ("recs", ctypes.c_void_p),
                ("n_recs", ctypes.c_int32),
                ("bitdepth_max", ctypes.c_int32)]


IS_FUSED, IS_PERSISTENT, IS_SB, IS_DEVICE_DEPS, IS_LEVEL0_BATCH = 1, 2, 4, 8, 16
EDGE_BACKUP_DTYPE = np.dtype([("plane", "<i4"), ("sby", "<i4"), ("x0", "<i4"), ("w", "<i4")])


class IntraSchedule(ctypes.Structure):
    _fields_ = [("n_levels", ctypes.c_int32),
                ("flags", ctypes.c_int32),
                ("unit_start", ctypes.c_void_p),
                ("class_start", ctypes.c_void_p),
                ("rec_start", ctypes.c_void_p),
                ("run_start", ctypes.c_void_p),
                ("runs", ctypes.c_void_p),
                ("workspace", ctypes.c_void_p),
                ("workspace_bytes", ctypes.c_int64),
                ("dep_start", ctypes.c_void_p),
                ("deps", ctypes.c_void_p),
                ("n_sb", ctypes.c_int32),
                ("sb_level_start", ctypes.c_void_p),
                ("sb_dep_start", ctypes.c_void_p),
                ("sb_deps", ctypes.c_void_p), ("task_group", ctypes.c_void_p)]


class RecBlock(ctypes.Structure):
    """Dav1dGpuRecBlock: one block of one plane, as recon_b_* would run it."""
    _fields_ = [("plane", ctypes.c_int32), ("x", ctypes.c_int32), ("y", ctypes.c_int32),
                ("w", ctypes.c_int32), ("h", ctypes.c_int32), ("tx", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("tile_x0", ctypes.c_int32), ("tile_y0", ctypes.c_int32), ("tile_x1", ctypes.c_int32),
                ("tile_y1", ctypes.c_int32), ("mvx", ctypes.c_int32 * 2), ("mvy", ctypes.c_int32 * 2),
                ("ref", ctypes.c_uint8 * 2), ("filter2d", ctypes.c_uint8), ("weight", ctypes.c_uint8),
                ("mode", ctypes.c_uint8), ("angle", ctypes.c_int8), ("cfl_alpha", ctypes.c_int8),
                ("flags", ctypes.c_uint8)]


class FilmGrainData(ctypes.Structure):
    """Dav1dGpuFilmGrainData: the layout of dav1d's Dav1dFilmGrainData."""
    _fields_ = [("seed", ctypes.c_uint), ("num_y_points", ctypes.c_int),
                ("y_points", (ctypes.c_uint8 * 2) * 14), ("chroma_scaling_from_luma", ctypes.c_int),
                ("num_uv_points", ctypes.c_int * 2), ("uv_points", ((ctypes.c_uint8 * 2) * 10) * 2),
                ("scaling_shift", ctypes.c_int), ("ar_coeff_lag", ctypes.c_int),
                ("ar_coeffs_y", ctypes.c_int8 * 24), ("ar_coeffs_uv", (ctypes.c_int8 * 28) * 2),
                ("ar_coeff_shift", ctypes.c_uint64), ("grain_scale_shift", ctypes.c_int),
                ("uv_mult", ctypes.c_int * 2), ("uv_luma_mult", ctypes.c_int * 2), ("uv_offset", ctypes.c_int * 2),
                ("overlap_flag", ctypes.c_int), ("clip_to_restricted_range", ctypes.c_int)]


class FilmGrainBatch(ctypes.Structure):
    _fields_ = [("in_", Plane * 3), ("out", Plane * 3), ("data", FilmGrainData), ("layout", ctypes.c_int32),
                ("bitdepth_max", ctypes.c_int32), ("is_id", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("scratch", ctypes.c_void_p)]


class CdefFrame(ctypes.Structure):
    """Dav1dGpuCdefFrame: one frame of bytefn(dav1d_cdef_brow) work."""
    _fields_ = [("in_", Plane * 3), ("out", Plane * 3), ("cdef_idx", ctypes.c_void_p), ("noskip", ctypes.c_void_p),
                ("layout", ctypes.c_int32), ("bitdepth_max", ctypes.c_int32), ("damping", ctypes.c_int32),
                ("pad_", ctypes.c_int32), ("y_strength", ctypes.c_uint8 * 8), ("uv_strength", ctypes.c_uint8 * 8),
                ("row_start", ctypes.c_int32), ("row_end", ctypes.c_int32)]


class FilterLUT(ctypes.Structure):
    """Dav1dGpuFilterLUT: Av1FilterLUT (src/lf_mask.h:35-39)."""
    _fields_ = [("e", ctypes.c_uint8 * 64), ("i", ctypes.c_uint8 * 64), ("sharp", ctypes.c_uint64 * 2)]


class LoopFilterFrame(ctypes.Structure):
    """Dav1dGpuLoopFilterFrame: one frame of deblocking."""
    _fields_ = [("pic", Plane * 3), ("masks", ctypes.c_void_p), ("level", ctypes.c_void_p),
                ("b4_stride", ctypes.c_int64), ("lut", FilterLUT), ("layout", ctypes.c_int32),
                ("bitdepth_max", ctypes.c_int32), ("filter_uv", ctypes.c_int32), ("row_start", ctypes.c_int32),
                ("row_end", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class _LrSgr(ctypes.Structure):
    _fields_ = [("s0", ctypes.c_uint32), ("s1", ctypes.c_uint32), ("w0", ctypes.c_int16), ("w1", ctypes.c_int16)]


class LrParams(ctypes.Union):
    """Dav1dGpuLrParams: LooprestorationParams (src/looprestoration.h:47-53)."""
    _fields_ = [("filter", (ctypes.c_int16 * 8) * 2), ("sgr", _LrSgr)]


class LrUnit(ctypes.Structure):
    """Dav1dGpuLrUnit: Av1RestorationUnit (src/lf_mask.h:41-47)."""
    _fields_ = [("type", ctypes.c_uint8), ("filter_h", ctypes.c_int8 * 3), ("filter_v", ctypes.c_int8 * 3),
                ("sgr_weights", ctypes.c_int8 * 2)]


class LrFrame(ctypes.Structure):
    _fields_ = [("in_", Plane * 3), ("lpf", Plane * 3), ("out", Plane * 3), ("units", ctypes.c_void_p * 3),
                ("unit_rows", ctypes.c_int32 * 3), ("unit_cols", ctypes.c_int32 * 3),
                ("unit_size_log2", ctypes.c_int32 * 2), ("layout", ctypes.c_int32), ("bitdepth_max", ctypes.c_int32),
                ("sb128", ctypes.c_int32), ("restore_planes", ctypes.c_int32), ("row_start", ctypes.c_int32),
                ("row_end", ctypes.c_int32)]


class ResizeFrame(ctypes.Structure):   # Dav1dGpuResizeFrame
    _fields_ = [("in_", Plane * 3), ("out", Plane * 3), ("step", ctypes.c_int32 * 2), ("start", ctypes.c_int32 * 2),
                ("layout", ctypes.c_int32), ("bitdepth_max", ctypes.c_int32), ("sb128", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


class PictureParameters(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int), ("h", ctypes.c_int), ("layout", ctypes.c_int), ("bpc", ctypes.c_int)]


class Picture(ctypes.Structure):   # Dav1dGpuPicture == Dav1dPicture (272 bytes)
    _fields_ = [("seq_hdr", ctypes.c_void_p), ("frame_hdr", ctypes.c_void_p), ("data", ctypes.c_void_p * 3),
                ("stride", ctypes.c_ssize_t * 2), ("p", PictureParameters), ("m_", ctypes.c_uint8 * 48),
                ("content_light", ctypes.c_void_p), ("mastering_display", ctypes.c_void_p),
                ("itut_t35", ctypes.c_void_p), ("n_itut_t35", ctypes.c_size_t), ("reserved", ctypes.c_size_t * 4),
                ("refs_", ctypes.c_void_p * 5), ("reserved_ref", ctypes.c_size_t * 4), ("ref", ctypes.c_void_p),
                ("allocator_data", ctypes.c_void_p)]


PIC_ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(Picture), ctypes.c_void_p)
PIC_RELEASE_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(Picture), ctypes.c_void_p)


class PicAllocator(ctypes.Structure):   # Dav1dGpuPicAllocator == Dav1dPicAllocator
    _fields_ = [("cookie", ctypes.c_void_p), ("alloc_picture_callback", PIC_ALLOC_FN),
                ("release_picture_callback", PIC_RELEASE_FN)]


PIC_DEVICE, PIC_HOST_MAPPED = 0, 1

GRAIN_W, GRAIN_H = 82, 73
GRAIN_SCRATCH_BYTES = 3 * GRAIN_H * GRAIN_W * 2 + 3 * 4096

_LIB = None


def lib_path():
    # DAV1D_GPU_LIB_VARIANT=<name> loads libdav1d_gpu.<name>.so: profiling
    # builds from tools/build_variants.sh (phase ablations), never a fallback
    v = os.environ.get("DAV1D_GPU_LIB_VARIANT")
    name = f"libdav1d_gpu.{v}.so" if v else "libdav1d_gpu.so"
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), name)


def load_lib():
    """Load the in-tree HIP library; raises (never falls back) if it is absent."""
    global _LIB
    if _LIB is None:
        p = lib_path()
        if not os.path.exists(p):
            raise RuntimeError(f"{p} missing: build it with __graft_entry__.build() "
                               "(there is no CPU fallback for the GPU DSP path)")
        L = ctypes.CDLL(p)
        L.dav1d_gpu_recon_8bpc.argtypes = [ctypes.POINTER(FrameBatch), ctypes.c_void_p]
        L.dav1d_gpu_recon_8bpc.restype = ctypes.c_int
        L.dav1d_gpu_recon_16bpc.argtypes = [ctypes.POINTER(FrameBatch), ctypes.c_void_p]
        L.dav1d_gpu_recon_16bpc.restype = ctypes.c_int
        L.dav1d_gpu_device_count.restype = ctypes.c_int
        L.dav1d_gpu_version.restype = ctypes.c_char_p
        L.dav1d_gpu_source_hash.restype = ctypes.c_char_p
        L.dav1d_gpu_debug_register_buffer.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.dav1d_gpu_debug_register_buffer.restype = ctypes.c_int
        for bpc in (8, 16):
            f = getattr(L, f"dav1d_gpu_recon_tiles_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(TileBatch), ctypes.c_void_p]
            f.restype = ctypes.c_int
        for bpc in (8, 16):
            f = getattr(L, f"dav1d_gpu_prepare_intra_edges_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(IntraEdgeBatch), ctypes.c_void_p]
            f.restype = ctypes.c_int
            f = getattr(L, f"dav1d_gpu_backup_ipred_edge_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(IntraEdgeBatch), ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
            f.restype = ctypes.c_int
            f = getattr(L, f"dav1d_gpu_recon_intra_frame_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(FrameBatch), ctypes.POINTER(IntraEdgeBatch),
                          ctypes.POINTER(IntraSchedule), ctypes.c_void_p]
            f.restype = ctypes.c_int
        for bpc in (8, 16):
            f = getattr(L, f"dav1d_gpu_apply_grain_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(FilmGrainBatch), ctypes.c_void_p]
            f.restype = ctypes.c_int
        for bpc in (8, 16):
            f = getattr(L, f"dav1d_gpu_lr_frame_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(LrFrame), ctypes.c_void_p]
            f.restype = ctypes.c_int
            f = getattr(L, f"dav1d_gpu_loopfilter_frame_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(LoopFilterFrame), ctypes.c_void_p]
            f.restype = ctypes.c_int
            f = getattr(L, f"dav1d_gpu_cdef_frame_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(CdefFrame), ctypes.c_void_p]
            f.restype = ctypes.c_int
        L.dav1d_gpu_recorder_new.argtypes = [ctypes.c_int] * 5
        L.dav1d_gpu_recorder_new.restype = ctypes.c_void_p
        L.dav1d_gpu_recorder_free.argtypes = [ctypes.c_void_p]
        L.dav1d_gpu_recorder_free.restype = None
        L.dav1d_gpu_rec_block.argtypes = [ctypes.c_void_p, ctypes.POINTER(RecBlock)]
        L.dav1d_gpu_rec_block.restype = ctypes.c_int
        L.dav1d_gpu_rec_block_aux.argtypes = [ctypes.c_void_p, ctypes.POINTER(RecBlock), ctypes.c_void_p,
                                              ctypes.c_size_t]
        L.dav1d_gpu_rec_block_aux.restype = ctypes.c_int
        L.dav1d_gpu_rec_residual.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p]
        L.dav1d_gpu_rec_residual.restype = ctypes.c_int
        L.dav1d_gpu_recorder_flush.argtypes = [ctypes.c_void_p, ctypes.POINTER(Plane * 3),
                                               ctypes.POINTER((Plane * 3) * MAX_REFS), ctypes.c_void_p]
        L.dav1d_gpu_recorder_flush.restype = ctypes.c_int
        L.dav1d_gpu_recorder_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                               ctypes.POINTER(ctypes.c_int32)]
        L.dav1d_gpu_recorder_stats.restype = ctypes.c_int
        L.dav1d_gpu_recorder_prep_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
        L.dav1d_gpu_recorder_prep_ms.restype = ctypes.c_int
        L.dav1d_gpu_recorder_status.argtypes = [ctypes.c_void_p]
        L.dav1d_gpu_recorder_status.restype = ctypes.c_int
        L.dav1d_gpu_recorder_set_top_edge.argtypes = [ctypes.c_void_p, ctypes.POINTER(Plane * 3), ctypes.c_int]
        L.dav1d_gpu_recorder_set_top_edge.restype = ctypes.c_int
        L.dav1d_gpu_get_error.restype = ctypes.c_int
        L.dav1d_gpu_pic_allocator_init.argtypes = [ctypes.POINTER(PicAllocator), ctypes.c_int, ctypes.c_int]
        L.dav1d_gpu_pic_allocator_init.restype = ctypes.c_int
        L.dav1d_gpu_pic_allocator_close.argtypes = [ctypes.POINTER(PicAllocator)]
        L.dav1d_gpu_pic_allocator_close.restype = ctypes.c_int
        L.dav1d_gpu_picture_plane.argtypes = [ctypes.POINTER(Picture), ctypes.c_int, ctypes.POINTER(Plane)]
        L.dav1d_gpu_picture_plane.restype = ctypes.c_int
        L.dav1d_gpu_clear_error.restype = ctypes.c_int
        L.dav1d_gpu_intra_workspace_bytes.argtypes = [ctypes.POINTER(IntraSchedule), ctypes.c_int]
        L.dav1d_gpu_intra_workspace_bytes.restype = ctypes.c_int64
        L.dav1d_gpu_recon_lds_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
        L.dav1d_gpu_recon_lds_bytes.restype = ctypes.c_int
        _LIB = L
    return _LIB


# every symbol include/dav1d_gpu.h declares
EXPORTED_SYMBOLS = [
    "dav1d_mc_dsp_init_8bpc", "dav1d_mc_dsp_init_16bpc",
    "dav1d_intra_pred_dsp_init_8bpc", "dav1d_intra_pred_dsp_init_16bpc",
    "dav1d_itx_dsp_init_8bpc", "dav1d_itx_dsp_init_16bpc",
    "dav1d_mc_dsp_init_gpu_8bpc", "dav1d_mc_dsp_init_gpu_16bpc",
    "dav1d_intra_pred_dsp_init_gpu_8bpc", "dav1d_intra_pred_dsp_init_gpu_16bpc",
    "dav1d_itx_dsp_init_gpu_8bpc", "dav1d_itx_dsp_init_gpu_16bpc",
    "dav1d_gpu_device_count", "dav1d_gpu_set_device", "dav1d_gpu_version", "dav1d_gpu_source_hash",
    "dav1d_gpu_get_error", "dav1d_gpu_clear_error", "dav1d_gpu_debug_register_buffer",
    "dav1d_gpu_pic_allocator_init", "dav1d_gpu_pic_allocator_close", "dav1d_gpu_picture_plane",
    "dav1d_gpu_recon_8bpc", "dav1d_gpu_recon_16bpc", "dav1d_gpu_recon_lds_bytes",
    "dav1d_gpu_recon_tiles_8bpc", "dav1d_gpu_recon_tiles_16bpc",
    "dav1d_gpu_prepare_intra_edges_8bpc", "dav1d_gpu_prepare_intra_edges_16bpc",
    "dav1d_gpu_backup_ipred_edge_8bpc", "dav1d_gpu_backup_ipred_edge_16bpc",
    "dav1d_gpu_recon_intra_frame_8bpc", "dav1d_gpu_recon_intra_frame_16bpc",
    "dav1d_gpu_intra_workspace_bytes",
    "dav1d_gpu_recorder_new", "dav1d_gpu_recorder_free", "dav1d_gpu_rec_block", "dav1d_gpu_rec_block_aux", "dav1d_gpu_rec_residual",
    "dav1d_gpu_recorder_flush", "dav1d_gpu_recorder_stats", "dav1d_gpu_recorder_status",
    "dav1d_gpu_recorder_prep_ms",
    "dav1d_gpu_recorder_set_top_edge",
    "dav1d_gpu_apply_grain_8bpc", "dav1d_gpu_apply_grain_16bpc",
    "dav1d_cdef_dsp_init_8bpc", "dav1d_cdef_dsp_init_16bpc",
    "dav1d_cdef_dsp_init_gpu_8bpc", "dav1d_cdef_dsp_init_gpu_16bpc",
    "dav1d_gpu_cdef_frame_8bpc", "dav1d_gpu_cdef_frame_16bpc",
    "dav1d_loop_filter_dsp_init_8bpc", "dav1d_loop_filter_dsp_init_16bpc",
    "dav1d_loop_filter_dsp_init_gpu_8bpc", "dav1d_loop_filter_dsp_init_gpu_16bpc",
    "dav1d_gpu_loopfilter_frame_8bpc", "dav1d_gpu_loopfilter_frame_16bpc",
    "dav1d_loop_restoration_dsp_init_8bpc", "dav1d_loop_restoration_dsp_init_16bpc",
    "dav1d_loop_restoration_dsp_init_gpu_8bpc", "dav1d_loop_restoration_dsp_init_gpu_16bpc",
    "dav1d_gpu_lr_frame_8bpc", "dav1d_gpu_lr_frame_16bpc",
    "dav1d_gpu_resize_frame_8bpc", "dav1d_gpu_resize_frame_16bpc",
]


def build_stamp():
    """(library source hash, hash of the sources in this tree, equal?): a
    library built from other sources than the tree's is stale."""
    import importlib.util
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("_dgpu_src_hash", root / "tools" / "src_hash.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    lib = load_lib().dav1d_gpu_source_hash().decode()
    tree = mod.source_hash(str(root))
    return lib, tree, lib == tree
