"""ggml_mi355x — Python host mirror of the ggml K-quant MUL_MAT operator surface,
bound to libggml_mi355x.so (HIP, gfx950) through its C-ABI (include/ggml_mi355x.h).

The names follow ggml: ``vec_dot_q4_K_q8_K`` (ggml_vec_dot_t, README.md:449),
``quantize_row_q8_K`` (from_float of Q8_K), ``mul_mat`` (ggml_compute_forward_mul_mat,
ggml-cpu.c:1389) and a ``Backend`` mirroring ggml-backend's device interface
(graph_compute, ggml-cpu.cpp:186). PyTorch is only plumbing here: device
buffers and the current HIP stream handle. There is no CPU fallback: if the
shared library or a gfx950 device is missing, every compute call raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("MI355X_LIB") or os.path.join(PKG_ROOT, "lib", "libggml_mi355x.so")

TYPE_F32, TYPE_F16, TYPE_Q4_K, TYPE_Q5_K, TYPE_Q6_K, TYPE_Q8_K, TYPE_I32 = 0, 1, 12, 13, 14, 15, 26
QK_K = 256
BLOCK_BYTES = {TYPE_Q4_K: 144, TYPE_Q5_K: 176, TYPE_Q6_K: 210, TYPE_Q8_K: 292}
TYPE_NAMES = {TYPE_Q4_K: "q4_K", TYPE_Q5_K: "q5_K", TYPE_Q6_K: "q6_K", TYPE_Q8_K: "q8_K", TYPE_F32: "f32"}
MAX_FUSED = 4
OP_NONE, OP_MUL_MAT, OP_GET_ROWS, OP_RMS_NORM, OP_MUL, OP_ADD, OP_SWIGLU, OP_ROPE, OP_ATTN_DECODE, OP_ALL_GATHER, \
    OP_ALL_REDUCE = range(11)
MAX_SRC = 8
FLAG_OUTPUT = 1
E_OK, E_INVAL, E_UNSUPPORTED, E_WORKSPACE, E_NODEVICE, E_COMM, E_LAYER = 0, -1, -2, -3, -4, -6, -7
PRO_NONE, PRO_RMS_NORM, PRO_SWIGLU = 0, 1, 2
EPI_NONE, EPI_SWIGLU = 0, 1
ATTN_GROUP, ATTN_HEAD, ATTN_SPLIT = 0, 1, 2
# mi355x_attn_path: the decode attention kernel a descriptor takes
ATTN_PATH_HEAD, ATTN_PATH_HEAD_BATCH, ATTN_PATH_SPLIT4, ATTN_PATH_SPLIT8, ATTN_PATH_CELLS, ATTN_PATH_GROUP, ATTN_PATH_KD1 = range(7)
MMQ_AUTO, MMQ_TILE64, MMQ_TILE128, MMQ_TILE128W, MMQ_TILE64W, MMQ_TILE128X, MMQ_TILE192 = 0, 1, 2, 3, 4, 5, 6
PREFILL_EXACT, PREFILL_F16, PREFILL_F16_ALL = 0, 1, 2

# Every symbol include/ggml_mi355x.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "mi355x_row_size", "mi355x_version", "mi355x_device_available",
    "mi355x_quantize_row_q8_K", "mi355x_vec_dot_q4_K_q8_K", "mi355x_vec_dot_q5_K_q8_K",
    "mi355x_vec_dot_q6_K_q8_K", "mi355x_quantize_q8_K", "mi355x_mul_mat_workspace_size",
    "mi355x_mul_mat", "mi355x_mul_mat_q8", "mi355x_gemv_fused", "mi355x_debug_block_partials", "mi355x_debug_stream",
    "mi355x_backend_init", "mi355x_backend_free", "mi355x_backend_name", "mi355x_backend_stream",
    "mi355x_backend_alloc", "mi355x_backend_free_buffer", "mi355x_backend_set_tensor",
    "mi355x_backend_get_tensor", "mi355x_backend_synchronize", "mi355x_backend_supports_op",
    "mi355x_backend_graph_compute", "mi355x_timing_enable", "mi355x_timing_read", "mi355x_diag_stamps",
    "mi355x_gemv_fused_workspace_size", "mi355x_gemv_impl",
    "mi355x_gguf_open", "mi355x_gguf_close", "mi355x_gguf_version", "mi355x_gguf_alignment",
    "mi355x_gguf_data_offset", "mi355x_gguf_n_tensors", "mi355x_gguf_find_tensor", "mi355x_gguf_get_tensor",
    "mi355x_gguf_tensor_data", "mi355x_gguf_upload", "mi355x_gguf_n_kv", "mi355x_gguf_find_key",
    "mi355x_gguf_key", "mi355x_gguf_kv_type", "mi355x_gguf_get_int", "mi355x_gguf_get_float",
    "mi355x_gguf_get_str", "mi355x_gguf_arr_n",
    "mi355x_gemv_ext_workspace_size", "mi355x_gemv_fused_ext", "mi355x_backend_set_fusion",
    "mi355x_get_rows", "mi355x_rms_norm", "mi355x_add", "mi355x_mul", "mi355x_swiglu",
    "mi355x_rope_table_size", "mi355x_rope_table", "mi355x_rope", "mi355x_attn_decode", "mi355x_attn_path",
    "mi355x_comm_id_size", "mi355x_comm_get_unique_id", "mi355x_backend_set_comm", "mi355x_backend_comm_world",
    "mi355x_backend_set_comm_loopback", "mi355x_lower_ggml_graph", "mi355x_attn_impl",
    "mi355x_mmq_impl",
    "mi355x_prefill_precision",
    "mi355x_gemv_waves",
    "mi355x_debug_knob",
    "mi355x_device_count", "mi355x_device_ordinal", "mi355x_device_memory", "mi355x_backend_memset", "mi355x_backend_set_attn_oproj",
    "mi355x_backend_set_layer_engine", "mi355x_backend_layer_error",
    "mi355x_attn_prompt",
    "mi355x_attn_prompt_impl",
)


class Mi355xError(RuntimeError):
    pass


class GemvDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("w", ctypes.c_void_p), ("n_rows", ctypes.c_int64),
                ("row_stride", ctypes.c_size_t), ("y", ctypes.c_void_p)]


class LaunchTiming(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_char * 96), ("bytes", ctypes.c_double), ("ms", ctypes.c_float)]


class Tensor(ctypes.Structure):
    pass


Tensor._fields_ = [("type", ctypes.c_int), ("op", ctypes.c_int), ("ne", ctypes.c_int64 * 4),
                   ("nb", ctypes.c_size_t * 4), ("src", ctypes.POINTER(Tensor) * MAX_SRC), ("data", ctypes.c_void_p),
                   ("op_params", ctypes.c_int32 * 8), ("flags", ctypes.c_int32)]


class GTensor(ctypes.Structure):
    """mi355x_gtensor: the ggml_tensor-shaped mirror the lowering reads."""
    pass


GTensor._fields_ = [("type", ctypes.c_int), ("op", ctypes.c_int), ("ne", ctypes.c_int64 * 4),
                    ("nb", ctypes.c_size_t * 4), ("op_params", ctypes.c_int32 * 16), ("flags", ctypes.c_int32),
                    ("src", ctypes.POINTER(GTensor) * 10), ("view_src", ctypes.POINTER(GTensor)),
                    ("view_offs", ctypes.c_size_t), ("data", ctypes.c_void_p), ("name", ctypes.c_char * 64)]


class LowerOpts(ctypes.Structure):
    _fields_ = [("rope_table", ctypes.c_void_p), ("rope_n_pos", ctypes.c_int), ("rope_freq_base", ctypes.c_float),
                ("rope_freq_scale", ctypes.c_float), ("cells_eq_pos", ctypes.c_int)]


(GOP_NONE, GOP_GET_ROWS, GOP_RMS_NORM, GOP_MUL, GOP_ADD, GOP_MUL_MAT, GOP_ROPE, GOP_SET_ROWS, GOP_SOFT_MAX, GOP_GLU,
 GOP_RESHAPE, GOP_VIEW, GOP_PERMUTE, GOP_TRANSPOSE, GOP_CONT, GOP_CPY) = range(16)
GLU_SWIGLU = 2


class AttnDesc(ctypes.Structure):
    _fields_ = [("q", ctypes.c_void_p), ("k", ctypes.c_void_p), ("v", ctypes.c_void_p), ("pos", ctypes.c_void_p),
                ("rope_table", ctypes.c_void_p), ("k_cache", ctypes.c_void_p), ("v_cache", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("n_ctx", ctypes.c_int), ("n_head", ctypes.c_int),
                ("n_head_kv", ctypes.c_int), ("head_dim", ctypes.c_int), ("scale", ctypes.c_float),
                ("rope_row", ctypes.c_int)]


class GemvExt(ctypes.Structure):
    _fields_ = [("prologue", ctypes.c_int), ("x2", ctypes.c_void_p), ("eps", ctypes.c_float),
                ("residual", ctypes.c_void_p * MAX_FUSED), ("epilogue", ctypes.c_int), ("epi_y", ctypes.c_void_p)]

_lib = None


def lib():
    """Load libggml_mi355x.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Mi355xError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C ggml-neon-opt_amd)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i64, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int
    L.mi355x_row_size.argtypes = [i32, i64]
    L.mi355x_row_size.restype = sz
    L.mi355x_version.restype = ctypes.c_char_p
    L.mi355x_device_available.restype = i32
    L.mi355x_device_count.restype = i32
    L.mi355x_device_ordinal.restype = i32
    L.mi355x_device_ordinal.argtypes = [i32]
    L.mi355x_device_memory.argtypes = [i32, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    L.mi355x_device_memory.restype = i32
    L.mi355x_backend_memset.argtypes = [ctypes.c_void_p, ctypes.c_void_p, i32, ctypes.c_size_t]
    L.mi355x_backend_memset.restype = i32
    L.mi355x_backend_set_attn_oproj.argtypes = [ctypes.c_void_p, i32]
    L.mi355x_backend_set_attn_oproj.restype = i32
    L.mi355x_backend_set_layer_engine.argtypes = [ctypes.c_void_p, i32]
    L.mi355x_backend_set_layer_engine.restype = i32
    L.mi355x_backend_layer_error.argtypes = [ctypes.c_void_p]
    L.mi355x_backend_layer_error.restype = i32
    L.mi355x_quantize_row_q8_K.argtypes = [vp, vp, i64]
    for n in ("q4_K", "q5_K", "q6_K"):
        getattr(L, f"mi355x_vec_dot_{n}_q8_K").argtypes = [i32, vp, sz, vp, sz, vp, sz, i32]
    L.mi355x_quantize_q8_K.argtypes = [vp, sz, vp, i64, i64, vp]
    L.mi355x_quantize_q8_K.restype = i32
    L.mi355x_mul_mat_workspace_size.argtypes = [i32, i64, i64, i64]
    L.mi355x_mul_mat_workspace_size.restype = sz
    L.mi355x_mul_mat.argtypes = [i32, vp, i64, i64, sz, vp, i64, sz, vp, sz, vp, sz, vp]
    L.mi355x_mul_mat.restype = i32
    L.mi355x_mul_mat_q8.argtypes = [i32, vp, i64, i64, sz, vp, i64, sz, vp, sz, vp]
    L.mi355x_mul_mat_q8.restype = i32
    L.mi355x_gemv_fused.argtypes = [ctypes.POINTER(GemvDesc), i32, vp, i64, vp, sz, vp]
    L.mi355x_gemv_fused_workspace_size.argtypes = [i64]
    L.mi355x_gemv_fused_workspace_size.restype = sz
    L.mi355x_gemv_fused.restype = i32
    L.mi355x_debug_block_partials.argtypes = [i32, vp, i64, i64, sz, vp, vp, vp]
    L.mi355x_debug_block_partials.restype = i32
    L.mi355x_debug_stream.argtypes = [vp, sz, vp, vp]
    L.mi355x_debug_stream.restype = i32
    L.mi355x_backend_init.argtypes = [i32]
    L.mi355x_backend_init.restype = vp
    L.mi355x_backend_free.argtypes = [vp]
    L.mi355x_backend_name.argtypes = [vp]
    L.mi355x_backend_name.restype = ctypes.c_char_p
    L.mi355x_backend_stream.argtypes = [vp]
    L.mi355x_backend_stream.restype = vp
    L.mi355x_backend_alloc.argtypes = [vp, sz]
    L.mi355x_backend_alloc.restype = vp
    L.mi355x_backend_free_buffer.argtypes = [vp, vp]
    L.mi355x_backend_set_tensor.argtypes = [vp, vp, vp, sz]
    L.mi355x_backend_set_tensor.restype = i32
    L.mi355x_backend_get_tensor.argtypes = [vp, vp, vp, sz]
    L.mi355x_backend_get_tensor.restype = i32
    L.mi355x_backend_synchronize.argtypes = [vp]
    L.mi355x_backend_synchronize.restype = i32
    L.mi355x_backend_supports_op.argtypes = [ctypes.POINTER(Tensor)]
    L.mi355x_backend_supports_op.restype = i32
    L.mi355x_backend_graph_compute.argtypes = [vp, ctypes.POINTER(ctypes.POINTER(Tensor)), i32, i32]
    L.mi355x_backend_graph_compute.restype = i32
    L.mi355x_timing_enable.argtypes = [i32]
    L.mi355x_timing_enable.restype = i32
    L.mi355x_timing_read.argtypes = [ctypes.POINTER(LaunchTiming), i32]
    L.mi355x_timing_read.restype = i32
    L.mi355x_gemv_impl.argtypes = [i32]
    L.mi355x_gemv_impl.restype = i32
    L.mi355x_diag_stamps.argtypes = [vp, sz]
    L.mi355x_diag_stamps.restype = i32
    f32 = ctypes.c_float
    L.mi355x_gemv_ext_workspace_size.argtypes = [i64]
    L.mi355x_gemv_ext_workspace_size.restype = sz
    L.mi355x_gemv_fused_ext.argtypes = [ctypes.POINTER(GemvDesc), i32, vp, i64, ctypes.POINTER(GemvExt), vp, sz, vp]
    L.mi355x_gemv_fused_ext.restype = i32
    L.mi355x_backend_set_fusion.argtypes = [vp, i32]
    L.mi355x_backend_set_fusion.restype = i32
    L.mi355x_get_rows.argtypes = [i32, vp, i64, sz, i64, vp, i64, vp, vp]
    L.mi355x_rms_norm.argtypes = [vp, vp, vp, i64, i64, f32, vp]
    L.mi355x_add.argtypes = [vp, vp, vp, i64, vp]
    L.mi355x_mul.argtypes = [vp, vp, vp, i64, vp]
    L.mi355x_swiglu.argtypes = [vp, vp, vp, i64, vp]
    L.mi355x_rope_table_size.argtypes = [i32, i32]
    L.mi355x_rope_table_size.restype = sz
    L.mi355x_rope_table.argtypes = [vp, i32, i32, f32, f32, vp]
    L.mi355x_rope.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32, vp]
    L.mi355x_attn_decode.argtypes = [ctypes.POINTER(AttnDesc), vp]
    L.mi355x_attn_path.argtypes = [ctypes.POINTER(AttnDesc)]
    L.mi355x_attn_path.restype = i32
    L.mi355x_attn_prompt.argtypes = [ctypes.POINTER(AttnDesc), i32, vp]
    L.mi355x_attn_prompt_impl.argtypes = [i32]
    L.mi355x_attn_prompt_impl.restype = i32
    L.mi355x_attn_impl.argtypes = [i32]
    L.mi355x_attn_impl.restype = i32
    L.mi355x_mmq_impl.argtypes = [i32]
    L.mi355x_mmq_impl.restype = i32
    L.mi355x_prefill_precision.argtypes = [i32]
    L.mi355x_prefill_precision.restype = i32
    L.mi355x_gemv_waves.argtypes = [i32]
    L.mi355x_gemv_waves.restype = i32
    L.mi355x_debug_knob.argtypes = [ctypes.c_char_p, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
    L.mi355x_debug_knob.restype = i32
    for n in ("mi355x_get_rows", "mi355x_rms_norm", "mi355x_add", "mi355x_mul", "mi355x_swiglu",
              "mi355x_rope_table", "mi355x_rope", "mi355x_attn_decode", "mi355x_attn_prompt"):
        getattr(L, n).restype = i32
    L.mi355x_lower_ggml_graph.argtypes = [ctypes.POINTER(ctypes.POINTER(GTensor)), i32, ctypes.POINTER(LowerOpts),
                                          ctypes.POINTER(Tensor), i32, ctypes.POINTER(ctypes.POINTER(Tensor)), i32,
                                          ctypes.POINTER(i32)]
    L.mi355x_lower_ggml_graph.restype = i32
    L.mi355x_comm_id_size.argtypes = []
    L.mi355x_comm_id_size.restype = sz
    L.mi355x_comm_get_unique_id.argtypes = [vp]
    L.mi355x_comm_get_unique_id.restype = i32
    L.mi355x_backend_set_comm.argtypes = [vp, i32, i32, vp]
    L.mi355x_backend_set_comm.restype = i32
    L.mi355x_backend_comm_world.argtypes = [vp]
    L.mi355x_backend_comm_world.restype = i32
    L.mi355x_backend_set_comm_loopback.argtypes = [vp, i32, i32]
    L.mi355x_backend_set_comm_loopback.restype = i32
    from . import gguf as _gguf
    _gguf.bind(L)
    _lib = L
    return L


GEMV_AUTO, GEMV_TASKS, GEMV_ROWS, GEMV_DYN = 0, 1, 2, 3


def gemv_impl(impl):
    """Select the decode GEMV kernel (GEMV_AUTO / GEMV_ROWS: row-stream kq_rows, one
    launch per stage, the claimed-row kq_rows_dyn where enough rows per wave; GEMV_TASKS:
    kq_gemv; GEMV_DYN: kq_rows_dyn for every one-type launch). Returns the previous selection."""
    prev = lib().mi355x_gemv_impl(impl)
    if prev < 0:
        raise Mi355xError(f"mi355x_gemv_impl failed with status {prev}")
    return prev


def timing_enable(enable=True):
    """Start (and clear) or stop per-launch kernel timing (hipExtLaunchKernelGGL events)."""
    lib().mi355x_timing_enable(1 if enable else 0)


def timing_read():
    """Synchronize the device; return [(kernel_name, algorithmic_bytes, ms), ...]."""
    n = lib().mi355x_timing_read(None, 0)
    if n < 0:
        raise Mi355xError(f"mi355x_timing_read failed ({n})")
    buf = (LaunchTiming * max(n, 1))()
    n = lib().mi355x_timing_read(buf, n)
    return [(buf[i].kernel.decode(), buf[i].bytes, buf[i].ms) for i in range(n)]


def version() -> str:
    return lib().mi355x_version().decode()


def device_available() -> bool:
    return bool(lib().mi355x_device_available())


def row_size(type_: int, k: int) -> int:
    return int(lib().mi355x_row_size(type_, k))


def _check(rc: int, what: str):
    if rc == E_LAYER:
        raise Mi355xError(f"{what}: a persistent-layer launch lost co-residency; that step's outputs "
                          "are invalid (counters re-armed)")
    if rc != 0:
        raise Mi355xError(f"{what} failed with status {rc}")


def _require_device():
    if not device_available():
        raise Mi355xError("no gfx950 device visible: the HIP path cannot run (there is no CPU fallback)")


def _stream(stream):
    if stream is not None:
        return ctypes.c_void_p(stream)
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# ----------------------------------------------------------- tensor helpers
def _torch():
    import torch
    return torch


def quantize_q8_K(x, out=None, stream=None):
    """x: (M, K) float32 cuda tensor -> (M, K/256*292) uint8 cuda tensor (Q8_K rows)."""
    torch = _torch()
    _require_device()
    if x.dim() == 1:
        x = x[None]
    assert x.dtype == torch.float32 and x.is_cuda and x.stride(1) == 1
    M, K = x.shape
    if out is None:
        out = torch.empty((M, K // QK_K * 292), dtype=torch.uint8, device=x.device)
    _check(lib().mi355x_quantize_q8_K(x.data_ptr(), x.stride(0) * 4, out.data_ptr(), K, M, _stream(stream)),
           "mi355x_quantize_q8_K")
    return out


def mul_mat(type_, w, K, x, out=None, workspace=None, stream=None):
    """dst (M, N) = mul_mat(w (N rows of `type_`), x (M, K) f32), ggml semantics."""
    torch = _torch()
    _require_device()
    if x.dim() == 1:
        x = x[None]
    M = x.shape[0]
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    ws = int(lib().mi355x_mul_mat_workspace_size(type_, K, N, M))
    if M == 1 and x.data_ptr() % 16:
        ws = max(ws, K // QK_K * 304)  # Q8L activation blocks (kq_rows)
    if ws and (workspace is None or workspace.numel() < ws):
        workspace = _workspace(ws, x.device, stream)
    _check(lib().mi355x_mul_mat(type_, w.data_ptr(), K, N, w.stride(0), x.data_ptr(), M, x.stride(0) * 4,
                                out.data_ptr(), out.stride(0) * 4,
                                workspace.data_ptr() if ws else None, ws, _stream(stream)), "mi355x_mul_mat")
    return out


def mul_mat_q8(type_, w, K, q8, out=None, stream=None):
    torch = _torch()
    _require_device()
    if q8.dim() == 1:
        q8 = q8[None]
    M = q8.shape[0]
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=q8.device)
    _check(lib().mi355x_mul_mat_q8(type_, w.data_ptr(), K, N, w.stride(0), q8.data_ptr(), M, q8.stride(0),
                                   out.data_ptr(), out.stride(0) * 4, _stream(stream)), "mi355x_mul_mat_q8")
    return out


_ws_cache = {}


def _workspace(nbytes, device, stream=None):
    """Scratch for the quantized activation, one per (device, stream): launches on one
    stream are ordered, those on different streams (other threads) may overlap."""
    torch = _torch()
    key = (str(device), _stream(stream).value or 0)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def gemv_fused(mats, x, stream=None, workspace=None):
    """mats: list of (type, w tensor (N, rowbytes), y tensor (N,) f32); x: (K,) f32. One launch
    (two when K > 8192: Q8_K quantization into a workspace first)."""
    _require_device()
    n = len(mats)
    descs = (GemvDesc * n)()
    for i, (t, w, y) in enumerate(mats):
        descs[i] = GemvDesc(t, w.data_ptr(), w.shape[0], w.stride(0), y.data_ptr())
    K = x.shape[-1]
    need = int(lib().mi355x_gemv_fused_workspace_size(K))
    if need and (workspace is None or workspace.numel() < need):
        workspace = _workspace(need, x.device, stream)
    _check(lib().mi355x_gemv_fused(descs, n, x.data_ptr(), K, workspace.data_ptr() if need else None, need,
                                   _stream(stream)), "mi355x_gemv_fused")


def mmq_impl(impl):
    """Prefill GEMM variant (MMQ_*); returns the previous."""
    return int(lib().mi355x_mmq_impl(impl))


def prefill_precision(p=-1):
    """Prefill (M >= 16) precision: PREFILL_EXACT (bit-exact kq_mmq), PREFILL_F16 (stated
    tolerance: kq_mmf where it is faster) or PREFILL_F16_ALL (kq_mmf on every shape); -1
    queries. Returns the previous value."""
    return int(lib().mi355x_prefill_precision(p))


def gemv_waves(waves):
    """kq_rows waves per workgroup: 0 = by launch size, else fixed (1..12); returns the previous."""
    return int(lib().mi355x_gemv_waves(waves))


DEBUG_KNOBS = ("GEMV_DIAG", "GEMV_RING", "GEMV_PRE0", "GEMV_PF", "GEMV_XMODE", "GEMV_SMALL_MB", "GEMV_WPC",
               "GEMV_SMALL_WG", "GEMV_FQMAX", "MMF_WAVES", "MMF_ORDER", "ATTN_DIAG", "LOOPBACK_NOCOPY",
               "ATTN_OPROJ", "AO_NRB", "GEMV_DYN", "GEMV_DYN_P", "GEMV_DYN_STEPS")


def debug_knob(name, value=float("nan")):
    """Experiment knob of A/B runs (mi355x_debug_knob; the library reads no environment):
    set `name` to `value` (NaN: back to the product default). Returns the previous value."""
    prev = ctypes.c_double(0.0)
    rc = lib().mi355x_debug_knob(name.encode(), float(value), ctypes.byref(prev))
    if rc != 0:
        raise Mi355xError(f"debug_knob: unknown knob {name!r}")
    return prev.value


def attn_prompt_impl(impl):
    """Prompt attention: ATTN_GROUP (per kv group and token, default) / ATTN_HEAD; returns the previous."""
    return int(lib().mi355x_attn_prompt_impl(impl))


def attn_impl(impl):
    """ATTN_SPLIT (default: per query head, split by output past 256 cache cells) / ATTN_HEAD
    (per query head) / ATTN_GROUP (per kv group); returns the previous."""
    return int(lib().mi355x_attn_impl(impl))


def gemv_fused_ext(mats, x, prologue=PRO_NONE, x2=None, eps=0.0, residual=None, epi_y=None, stream=None):
    """gemv_fused with the decode graph's neighbours fused (mi355x_gemv_fused_ext):
    prologue PRO_RMS_NORM (x2 = norm weight) / PRO_SWIGLU (x = gate, x2 = up),
    y_i = mul_mat_i + residual[i], and with epi_y (mats = [gate, up]) the SWIGLU
    epilogue epi_y = swiglu(y_0, y_1)."""
    _require_device()
    n = len(mats)
    descs = (GemvDesc * n)()
    for i, (t, w, y) in enumerate(mats):
        descs[i] = GemvDesc(t, w.data_ptr(), w.shape[0], w.stride(0), y.data_ptr())
    ext = GemvExt()
    ext.prologue = prologue
    ext.x2 = x2.data_ptr() if x2 is not None else None
    ext.eps = eps
    for i in range(MAX_FUSED):
        r = residual[i] if residual is not None and i < len(residual) else None
        ext.residual[i] = r.data_ptr() if r is not None else None
    ext.epilogue = EPI_SWIGLU if epi_y is not None else EPI_NONE
    ext.epi_y = epi_y.data_ptr() if epi_y is not None else None
    K = x.shape[-1]
    need = int(lib().mi355x_gemv_ext_workspace_size(K))
    ws = _workspace(need, x.device, stream)
    _check(lib().mi355x_gemv_fused_ext(descs, n, x.data_ptr(), K, ctypes.byref(ext), ws.data_ptr(), need,
                                       _stream(stream)), "mi355x_gemv_fused_ext")


# ------------------------------------------- decode ops (mi355x_get_rows ... attn)
def get_rows(type_, table, K, ids, out=None, stream=None):
    """table: (rows, rowbytes) uint8 (or (rows, K) f32); ids: int32 cuda -> (n, K) f32."""
    torch = _torch()
    _require_device()
    n = ids.numel()
    if out is None:
        out = torch.empty((n, K), dtype=torch.float32, device=ids.device)
    _check(lib().mi355x_get_rows(type_, table.data_ptr(), K, table.stride(0) * table.element_size(), table.shape[0],
                                 ids.data_ptr(), n, out.data_ptr(), _stream(stream)), "mi355x_get_rows")
    return out


def rms_norm(x, eps, w=None, out=None, stream=None):
    torch = _torch()
    _require_device()
    x2 = x if x.dim() == 2 else x[None]
    if out is None:
        out = torch.empty_like(x)
    _check(lib().mi355x_rms_norm(x.data_ptr(), w.data_ptr() if w is not None else None, out.data_ptr(),
                                 x2.shape[1], x2.shape[0], eps, _stream(stream)), "mi355x_rms_norm")
    return out


def add(a, b, out=None, stream=None):
    out = _torch().empty_like(a) if out is None else out
    _check(lib().mi355x_add(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _stream(stream)), "mi355x_add")
    return out


def mul(a, b, out=None, stream=None):
    out = _torch().empty_like(a) if out is None else out
    _check(lib().mi355x_mul(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _stream(stream)), "mi355x_mul")
    return out


def swiglu(g, u, out=None, stream=None):
    out = _torch().empty_like(g) if out is None else out
    _check(lib().mi355x_swiglu(g.data_ptr(), u.data_ptr(), out.data_ptr(), g.numel(), _stream(stream)),
           "mi355x_swiglu")
    return out


def rope_table(n_pos, n_dims, freq_base=10000.0, freq_scale=1.0, device="cuda", stream=None):
    torch = _torch()
    _require_device()
    t = torch.empty((n_pos, n_dims // 2, 2), dtype=torch.float32, device=device)
    _check(lib().mi355x_rope_table(t.data_ptr(), n_pos, n_dims, freq_base, freq_scale, _stream(stream)),
           "mi355x_rope_table")
    return t


def rope(x, head_dim, n_dims, pos, table, out=None, stream=None):
    """x: (n_heads*head_dim,) f32; pos: int32 cuda tensor (1,)."""
    out = _torch().empty_like(x) if out is None else out
    _check(lib().mi355x_rope(x.data_ptr(), out.data_ptr(), head_dim, n_dims, x.numel() // head_dim, pos.data_ptr(),
                             table.data_ptr(), table.shape[0], _stream(stream)), "mi355x_rope")
    return out


def attn_decode(q, k, v, pos, table, k_cache, v_cache, n_head, n_head_kv, head_dim, scale, out=None, stream=None,
                rope_row=False):
    """k_cache: (n_ctx, n_head_kv*hd) int16/uint16 view of f16; v_cache: (n_head_kv*hd, n_ctx).
    rope_row: `table` is only the rope row of *pos (staged by the caller with the position)."""
    out = _torch().empty(n_head * head_dim, dtype=_torch().float32, device=q.device) if out is None else out
    a = AttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), pos.data_ptr(), table.data_ptr(), k_cache.data_ptr(),
                 v_cache.data_ptr(), out.data_ptr(), k_cache.shape[0], n_head, n_head_kv, head_dim, scale,
                 1 if rope_row else 0)
    _check(lib().mi355x_attn_decode(ctypes.byref(a), _stream(stream)), "mi355x_attn_decode")
    return out


def attn_path(n_ctx, n_head, n_head_kv, head_dim, cache_offset=0, f32_offset=0, rope_row=True):
    """The decode attention kernel (ATTN_PATH_*) mi355x_attn_decode would run for this shape under
    the current selectors: no launch, no device access (the descriptor's addresses are synthetic,
    16-B aligned plus `cache_offset` for the caches and `f32_offset` for q / k / v / rope)."""
    base = 1 << 20
    f = base + f32_offset
    a = AttnDesc(f, f + 4096, f + 8192, base, f + 12288, base + (1 << 12) + cache_offset,
                 base + (1 << 13) + cache_offset, base + (1 << 14), n_ctx, n_head, n_head_kv, head_dim,
                 1.0 / float(head_dim) ** 0.5, 1 if rope_row else 0)
    return int(lib().mi355x_attn_path(ctypes.byref(a)))


def attn_prompt(q, k, v, pos, table, k_cache, v_cache, n_head, n_head_kv, head_dim, scale, out=None, stream=None):
    """A prompt batch of T tokens: q (T, n_head*hd), k, v (T, n_head_kv*hd) f32, pos int32 cuda (T,),
    table the whole rope table; writes the T cells, returns out (T, n_head*hd)."""
    T = pos.numel()
    out = _torch().empty((T, n_head * head_dim), dtype=_torch().float32, device=q.device) if out is None else out
    a = AttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), pos.data_ptr(), table.data_ptr(), k_cache.data_ptr(),
                 v_cache.data_ptr(), out.data_ptr(), k_cache.shape[0], n_head, n_head_kv, head_dim, scale, 0)
    _check(lib().mi355x_attn_prompt(ctypes.byref(a), T, _stream(stream)), "mi355x_attn_prompt")
    return out


def block_partials(type_, w, K, q8_row, stream=None):
    """Per-superblock integer partials -> (N, nb, 2) int32 cuda tensor."""
    torch = _torch()
    _require_device()
    N = w.shape[0]
    out = torch.zeros((N, K // QK_K, 2), dtype=torch.int32, device=w.device)
    _check(lib().mi355x_debug_block_partials(type_, w.data_ptr(), K, N, w.stride(0), q8_row.data_ptr(),
                                             out.data_ptr(), _stream(stream)), "mi355x_debug_block_partials")
    return out


# ------------------------------------------- raw ggml surface (device pointers)
def vec_dot_q4_K_q8_K(n, s, bs, vx, bx, vy, by, nrc):
    lib().mi355x_vec_dot_q4_K_q8_K(n, s, bs, vx, bx, vy, by, nrc)


def vec_dot_q5_K_q8_K(n, s, bs, vx, bx, vy, by, nrc):
    lib().mi355x_vec_dot_q5_K_q8_K(n, s, bs, vx, bx, vy, by, nrc)


def vec_dot_q6_K_q8_K(n, s, bs, vx, bx, vy, by, nrc):
    lib().mi355x_vec_dot_q6_K_q8_K(n, s, bs, vx, bx, vy, by, nrc)


def quantize_row_q8_K(x, y, k):
    lib().mi355x_quantize_row_q8_K(x, y, k)


# ------------------------------------------------------------ backend mirror
class Backend:
    """ggml-backend device mirror: own stream, device buffers, graph_compute."""

    def __init__(self, device=0):
        _require_device()
        self.h = lib().mi355x_backend_init(device)
        if not self.h:
            raise Mi355xError("mi355x_backend_init failed")
        self._keep = []

    @property
    def name(self):
        return lib().mi355x_backend_name(self.h).decode()

    @property
    def stream(self):
        return lib().mi355x_backend_stream(self.h)

    def alloc(self, size):
        p = lib().mi355x_backend_alloc(self.h, size)
        if not p:
            raise Mi355xError("alloc failed")
        return p

    def free_buffer(self, p):
        lib().mi355x_backend_free_buffer(self.h, p)

    def set_tensor(self, dst, host_array):
        import numpy as np
        a = np.ascontiguousarray(host_array)
        self._keep.append(a)  # keep alive until synchronize
        _check(lib().mi355x_backend_set_tensor(self.h, dst, a.ctypes.data, a.nbytes), "set_tensor")

    def get_tensor(self, host_array, src):
        _check(lib().mi355x_backend_get_tensor(self.h, host_array.ctypes.data, src, host_array.nbytes),
               "get_tensor")

    def synchronize(self):
        _check(lib().mi355x_backend_synchronize(self.h), "synchronize")
        self._keep.clear()

    def set_fusion(self, enable):
        return int(lib().mi355x_backend_set_fusion(self.h, 1 if enable else 0))

    def set_attn_oproj(self, enable):
        """Decode attention + o-proj GEMV in one launch (default off); returns the previous."""
        return int(lib().mi355x_backend_set_attn_oproj(self.h, 1 if enable else 0))

    def set_layer_engine(self, enable):
        """Each decode layer as one persistent launch (csrc/kq_layer.hip); returns the previous."""
        return int(lib().mi355x_backend_set_layer_engine(self.h, 1 if enable else 0))

    def layer_error(self):
        """Non-zero if a persistent-layer launch gave up waiting (results invalid); clears it."""
        return int(lib().mi355x_backend_layer_error(self.h))

    def set_comm(self, rank, world, unique_id: bytes):
        """Join the RCCL communicator of a row split (every rank, same id bytes)."""
        buf = ctypes.create_string_buffer(bytes(unique_id), len(unique_id))
        _check(lib().mi355x_backend_set_comm(self.h, rank, world, buf), "set_comm")

    def set_comm_loopback(self, rank, world):
        """Test emulation of one rank of a row split on this GPU (no communicator)."""
        _check(lib().mi355x_backend_set_comm_loopback(self.h, rank, world), "set_comm_loopback")

    @property
    def comm_world(self):
        return int(lib().mi355x_backend_comm_world(self.h))

    def graph_compute(self, nodes, use_graph=True):
        arr = (ctypes.POINTER(Tensor) * len(nodes))(*[ctypes.pointer(n) for n in nodes])
        return int(lib().mi355x_backend_graph_compute(self.h, arr, len(nodes), 1 if use_graph else 0))

    def close(self):
        if self.h:
            lib().mi355x_backend_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lower_ggml_graph(gnodes, rope_table_ptr, rope_n_pos, freq_base, freq_scale=1.0, arena_cap=None,
                     cells_eq_pos=True):
    """mi355x_lower_ggml_graph over a list of GTensor nodes (graph order). Returns
    (status, [Tensor node list], arena) — the arena keeps the nodes alive.
    cells_eq_pos: the adapter's promise (mi355x_lower_opts) that the batch is one
    sequence whose KV cells equal its positions under a causal mask."""
    n = len(gnodes)
    arr = (ctypes.POINTER(GTensor) * max(1, n))(*[ctypes.pointer(t) for t in gnodes])
    cap = arena_cap or (4 * n + 64)
    arena = (Tensor * cap)()
    out = (ctypes.POINTER(Tensor) * cap)()
    nn = ctypes.c_int(0)
    opts = LowerOpts(rope_table_ptr, rope_n_pos, freq_base, freq_scale, 1 if cells_eq_pos else 0)
    rc = int(lib().mi355x_lower_ggml_graph(arr, n, ctypes.byref(opts), arena, cap, out, cap, ctypes.byref(nn)))
    return rc, [out[i].contents for i in range(nn.value)], (arena, out)


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 of a row split creates it, the others receive it)."""
    n = int(lib().mi355x_comm_id_size())
    buf = ctypes.create_string_buffer(n)
    _check(lib().mi355x_comm_get_unique_id(buf), "comm_get_unique_id")
    return buf.raw


def supports_op(t: Tensor) -> bool:
    return bool(lib().mi355x_backend_supports_op(ctypes.byref(t)))


def make_tensor(type_, ne0, ne1, data, row_stride=None, op=OP_NONE, src0=None, src1=None, srcs=None,
                op_params=None, flags=0) -> Tensor:
    """2-D ggml-style tensor descriptor: ne0 elements per row, ne1 rows, row stride nb1 bytes.
    `srcs` (list) overrides src0/src1; op_params: up to 8 int32 (use f32_bits for floats)."""
    t = Tensor()
    t.type = type_
    t.op = op
    nb0 = BLOCK_BYTES.get(type_, 2 if type_ == TYPE_F16 else 4)
    nb1 = row_stride if row_stride is not None else (ne0 // QK_K * nb0 if type_ in BLOCK_BYTES else ne0 * nb0)
    t.ne[0], t.ne[1], t.ne[2], t.ne[3] = ne0, ne1, 1, 1
    t.nb[0], t.nb[1], t.nb[2], t.nb[3] = nb0, nb1, nb1 * ne1, nb1 * ne1
    srcs = list(srcs) if srcs is not None else [src0, src1]
    for i in range(MAX_SRC):
        s = srcs[i] if i < len(srcs) else None
        t.src[i] = ctypes.pointer(s) if s is not None else ctypes.POINTER(Tensor)()
    t.data = data
    for i, v in enumerate(op_params or []):
        t.op_params[i] = v
    t.flags = flags
    return t


def f32_bits(v: float) -> int:
    import struct
    return struct.unpack("<i", struct.pack("<f", v))[0]
