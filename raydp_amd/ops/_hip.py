"""ctypes front end of ``libhipkernels.so`` (gfx950 kernels in ``csrc/hip``).

The structs below mirror the C structs byte for byte (checked against the ``rx_*_size``
exports at load time). GPU ops never fall back to eager PyTorch silently: if the library is
missing or was built for another architecture the call raises.
"""
import ctypes

from raydp_amd.native import loader

MAXL = 8
MAXSEG = 4 * MAXL
MAXCOLS = 64


class MlpLayer(ctypes.Structure):
    _fields_ = [
        ("in_", ctypes.c_int), ("out", ctypes.c_int),
        ("in_k", ctypes.c_int), ("out_k", ctypes.c_int),
        ("in_n", ctypes.c_int), ("out_n", ctypes.c_int),
        ("w_img", ctypes.c_int), ("wt_img", ctypes.c_int),
        ("w_off", ctypes.c_int), ("b_off", ctypes.c_int),
        ("act", ctypes.c_int), ("bn", ctypes.c_int),
        ("g_off", ctypes.c_int), ("be_off", ctypes.c_int),
        ("rs_off", ctypes.c_int), ("mw_off", ctypes.c_int),
        ("eps", ctypes.c_float), ("momentum", ctypes.c_float),
        ("xt_off", ctypes.c_int), ("stat_off", ctypes.c_int), ("r_off", ctypes.c_int),
        ("pr_off", ctypes.c_int), ("xg_off", ctypes.c_int), ("gg_off", ctypes.c_int),
        ("sv_lds", ctypes.c_int),
    ]


class FrontCol(ctypes.Structure):
    """One column of an embedding front (csrc/hip/mlp_core.h FrontCol)."""
    _fields_ = [("src", ctypes.c_int), ("poff", ctypes.c_int), ("stride", ctypes.c_int), ("rows", ctypes.c_int)]


MAXF = 64


class MlpDesc(ctypes.Structure):
    _fields_ = [
        ("L", ctypes.c_int),
        ("r_lds_off", ctypes.c_int), ("gt_lds_off", ctypes.c_int),
        ("stats_lds_off", ctypes.c_int), ("lds_bytes", ctypes.c_int),
        ("max_k", ctypes.c_int), ("max_n", ctypes.c_int),
        ("loss", ctypes.c_int), ("beta", ctypes.c_float),
        ("out_dim", ctypes.c_int), ("feat_k", ctypes.c_int),
        ("layer", MlpLayer * MAXL),
        ("pr_lds_off", ctypes.c_int), ("pr_total", ctypes.c_int),
        ("act_off", ctypes.c_int), ("wgrad_mode", ctypes.c_int),
        ("front_n", ctypes.c_int), ("front_q", ctypes.c_int), ("acc_mode", ctypes.c_int),
        ("acc_thr", ctypes.c_float), ("front", FrontCol * MAXF), ("front_qbase", ctypes.c_int * MAXF),
        ("loss_lds_off", ctypes.c_int), ("w0s_lds_off", ctypes.c_int), ("x0c_lds_off", ctypes.c_int),
    ]


class StepBufs(ctypes.Structure):
    """Device buffers of one fused model (csrc/hip/fused_mlp.hip StepBufs)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("d_dev", "img", "rstats", "params", "grads", "scratch",
                                               "metrics", "stamps", "jit_step", "jit_eval",
                                               "jit_persist", "mw", "jit_step_mw")]


class MwArgs(ctypes.Structure):
    """Multi-workgroup step of one fused model (csrc/hip/fused_mlp.hip MwArgs)."""
    _fields_ = [("part", ctypes.c_void_p), ("ctl", ctypes.c_void_p), ("G", ctypes.c_int),
                ("resident_ok", ctypes.c_int), ("stride", ctypes.c_int), ("seq", ctypes.c_uint),
                ("scratch_stride", ctypes.c_longlong), ("ticks", ctypes.c_ulonglong),
                ("wpart", ctypes.c_void_p), ("wctr", ctypes.c_void_p), ("lcnt", ctypes.c_void_p),
                ("nopt", ctypes.c_int), ("fseq", ctypes.c_uint), ("share", ctypes.c_int)]


class OptSeg(ctypes.Structure):
    _fields_ = [
        ("start", ctypes.c_int), ("len", ctypes.c_int), ("kind", ctypes.c_int),
        ("out", ctypes.c_int), ("in_", ctypes.c_int), ("in_k", ctypes.c_int), ("out_k", ctypes.c_int),
        ("in_n", ctypes.c_int), ("out_n", ctypes.c_int), ("xg_off", ctypes.c_int), ("gg_off", ctypes.c_int),
        ("W", ctypes.c_void_p), ("Wt", ctypes.c_void_p),
    ]


class OptDesc(ctypes.Structure):
    _fields_ = [
        ("nseg", ctypes.c_int), ("total", ctypes.c_int), ("algo", ctypes.c_int),
        ("b1", ctypes.c_float), ("b2", ctypes.c_float), ("eps", ctypes.c_float),
        ("wd", ctypes.c_float), ("momentum", ctypes.c_float), ("dampening", ctypes.c_float),
        ("nesterov", ctypes.c_int), ("maximize", ctypes.c_int),
        ("seg", OptSeg * MAXSEG),
        ("act_off", ctypes.c_int), ("act_floats", ctypes.c_int), ("bp", ctypes.c_int),
        ("wgrad_mode", ctypes.c_int), ("ps_l0_inline", ctypes.c_int),
    ]


class IngestCol(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int), ("pad_", ctypes.c_int), ("vbit", ctypes.c_longlong),
        ("values", ctypes.c_void_p), ("valid", ctypes.c_void_p),
        ("fill", ctypes.c_float), ("pad2_", ctypes.c_int),
    ]


class DmaRegion(ctypes.Structure):
    """One host byte range DMA'd into a chunk's staging area (csrc/hip/arrow_ingest.hip)."""
    _fields_ = [("host", ctypes.c_uint64), ("bytes", ctypes.c_longlong), ("off", ctypes.c_longlong)]


class DmaCol(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int), ("has_valid", ctypes.c_int),
        ("vals_off", ctypes.c_longlong), ("valid_off", ctypes.c_longlong), ("vbit", ctypes.c_longlong),
        ("fill", ctypes.c_float), ("pad_", ctypes.c_int),
    ]


class DmaChunk(ctypes.Structure):
    _fields_ = [
        ("nrows", ctypes.c_longlong), ("out_row0", ctypes.c_longlong), ("bytes", ctypes.c_longlong),
        ("first_region", ctypes.c_int), ("nregions", ctypes.c_int), ("first_col", ctypes.c_int),
        ("pad_", ctypes.c_int),
    ]


class IngestArgs(ctypes.Structure):
    _fields_ = [
        ("ncols", ctypes.c_int), ("out_stride", ctypes.c_int), ("out_bf16", ctypes.c_int),
        ("pad_", ctypes.c_int), ("nrows", ctypes.c_longlong), ("out_row0", ctypes.c_longlong),
        ("col", IngestCol * MAXCOLS),
    ]


_lib = None


def lib():
    """Load the HIP kernel library (requires a ROCm PyTorch already initialised)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401 - torch's HIP runtime must be loaded first (shared SONAME)
    L = loader.load("hipkernels", build_if_missing=True)
    vp, i, f, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_longlong
    L.rx_mlp_desc_size.restype = i
    L.rx_opt_desc_size.restype = i
    L.rx_ingest_args_size.restype = i
    L.rx_step_bufs_size.restype = i
    # (desc, bufs, opt, opt_dev, mt, m, v, feats, labels, perm, n_rows, batch, first_step, nsteps,
    #  lrs, bc1s, bc2s, gscale, opt_first, stream, allreduce_fn, ar_ctx)
    L.rx_mlp_train_steps.argtypes = [vp, vp, vp, vp, i, vp, vp, vp, vp, vp, i, i, i, i, vp, vp, vp, f, i,
                                     vp, vp, vp]
    L.rx_mlp_fwdbwd.argtypes = [vp, vp, i, vp, vp, vp, i, i, i, vp]
    L.rx_opt_step.argtypes = [vp, vp, vp, vp, vp, vp, f, f, f, f, i, vp]
    L.rx_mlp_wgrad.argtypes = [vp, vp, vp, vp]
    L.rx_mlp_eval.argtypes = [vp, vp, i, vp, vp, i, i, vp]
    L.rx_jit_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                              ctypes.POINTER(vp), i]
    # (desc, bufs, opt, opt_dev, mt, m, v, feats, labels, perm, n_rows, batch, nsteps, sched, opt_first,
    #  sync, timeout_s, stream, xg ctx (world > 1, else null), gscale, ranks sharing the device)
    L.rx_mlp_train_persistent.argtypes = [vp, vp, vp, vp, i, vp, vp, vp, vp, vp, i, i, i, vp, i, vp,
                                          ctypes.c_double, vp, vp, f, i]
    L.rx_mlp_train_persistent.restype = i
    L.rx_ps_sync_words.restype = i
    L.rx_mw_args_size.restype = i
    L.rx_mw_resident.argtypes = [i, i, i]
    L.rx_mw_resident.restype = i
    L.rx_ps_err_index.restype = i
    L.rx_ps_grid_blocks.argtypes = [vp]
    L.rx_ps_grid_blocks.restype = i
    L.rx_jit_load.restype = i
    L.rx_mlp_refresh_images.argtypes = [vp, vp, vp, vp]
    L.rx_arrow_ingest.argtypes = [vp, vp, vp]
    L.rx_gather_rows.argtypes = [vp, vp, vp, ll, i, vp]
    u64 = ctypes.c_uint64
    L.rx_pin_range.argtypes = [u64, u64, u64, u64, u64]
    L.rx_pin_stats.argtypes = [vp]
    L.rx_unpin_arena.argtypes = [u64]
    L.rx_dma_sizes.argtypes = [vp]
    # (chunks, nchunks, regions, cols, ncols, out_stride, out_bf16, out, stage, stage_bytes,
    #  compute, copy, stats)
    L.rx_ingest_dma.argtypes = [vp, i, vp, vp, i, i, i, vp, vp, ll, vp, vp, vp]
    L.rx_feistel_perm.argtypes = [vp, ll, u64, vp]
    L.rx_comm_available.restype = i
    L.rx_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.rx_comm_allreduce.argtypes = [vp, i, vp, vp]
    L.rx_comm_broadcast.argtypes = [vp, i, i, vp, vp]
    L.rx_comm_destroy.argtypes = [vp]
    for fn in ("rx_mlp_train_steps", "rx_mlp_fwdbwd", "rx_opt_step", "rx_mlp_eval",
               "rx_mlp_refresh_images", "rx_arrow_ingest", "rx_gather_rows", "rx_comm_unique_id",
               "rx_pin_range", "rx_pin_stats", "rx_unpin_arena", "rx_dma_sizes", "rx_ingest_dma",
               "rx_feistel_perm",
               "rx_comm_allreduce", "rx_comm_broadcast", "rx_comm_destroy"):
        getattr(L, fn).restype = i
    for name, cls in (("rx_mlp_desc_size", MlpDesc), ("rx_opt_desc_size", OptDesc),
                      ("rx_ingest_args_size", IngestArgs), ("rx_step_bufs_size", StepBufs),
                      ("rx_mw_args_size", MwArgs)):
        got = getattr(L, name)()
        if got != ctypes.sizeof(cls):
            raise RuntimeError(f"ABI mismatch for {cls.__name__}: C {got} vs ctypes {ctypes.sizeof(cls)}")
    sizes = (ctypes.c_int * 3)()
    L.rx_dma_sizes(sizes)
    for got, cls in zip(sizes, (DmaRegion, DmaCol, DmaChunk)):
        if got != ctypes.sizeof(cls):
            raise RuntimeError(f"ABI mismatch for {cls.__name__}: C {got} vs ctypes {ctypes.sizeof(cls)}")
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")


def stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
