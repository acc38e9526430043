"""GGUF model files through the library's native reader (kq_gguf.cpp, C-ABI
mi355x_gguf_*): metadata, tensor infos, mapped tensor bytes, device upload.

Mirrors what llama-bench does before the first MUL_MAT (gguf_reader::read and
llama_model_loader, artifacts/perf/out.folded:2-3, 17-22, 39-46): the K-quant
blocks reach the kernels byte-for-byte as stored in the file (no repack).
"""
from __future__ import annotations

import ctypes

U8, I8, U16, I16, U32, I32, F32, BOOL, STRING, ARRAY, U64, I64, F64 = range(13)


class TensorInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("type", ctypes.c_int), ("n_dims", ctypes.c_int),
                ("ne", ctypes.c_int64 * 4), ("offset", ctypes.c_uint64), ("size", ctypes.c_uint64)]


def bind(L):
    vp, i32, i64, u32, u64, sz = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                  ctypes.c_uint64, ctypes.c_size_t)
    L.mi355x_gguf_open.argtypes = [ctypes.c_char_p]
    L.mi355x_gguf_open.restype = vp
    L.mi355x_gguf_close.argtypes = [vp]
    L.mi355x_gguf_version.argtypes = [vp]
    L.mi355x_gguf_version.restype = u32
    L.mi355x_gguf_alignment.argtypes = [vp]
    L.mi355x_gguf_alignment.restype = u64
    L.mi355x_gguf_data_offset.argtypes = [vp]
    L.mi355x_gguf_data_offset.restype = u64
    L.mi355x_gguf_n_tensors.argtypes = [vp]
    L.mi355x_gguf_n_tensors.restype = i64
    L.mi355x_gguf_find_tensor.argtypes = [vp, ctypes.c_char_p]
    L.mi355x_gguf_find_tensor.restype = i64
    L.mi355x_gguf_get_tensor.argtypes = [vp, i64, ctypes.POINTER(TensorInfo)]
    L.mi355x_gguf_get_tensor.restype = i32
    L.mi355x_gguf_tensor_data.argtypes = [vp, i64]
    L.mi355x_gguf_tensor_data.restype = vp
    L.mi355x_gguf_upload.argtypes = [vp, i64, vp, sz, vp]
    L.mi355x_gguf_upload.restype = i32
    L.mi355x_gguf_n_kv.argtypes = [vp]
    L.mi355x_gguf_n_kv.restype = i64
    L.mi355x_gguf_find_key.argtypes = [vp, ctypes.c_char_p]
    L.mi355x_gguf_find_key.restype = i64
    L.mi355x_gguf_key.argtypes = [vp, i64]
    L.mi355x_gguf_key.restype = ctypes.c_char_p
    L.mi355x_gguf_kv_type.argtypes = [vp, i64]
    L.mi355x_gguf_kv_type.restype = i32
    L.mi355x_gguf_get_int.argtypes = [vp, i64, ctypes.POINTER(ctypes.c_int64)]
    L.mi355x_gguf_get_int.restype = i32
    L.mi355x_gguf_get_float.argtypes = [vp, i64, ctypes.POINTER(ctypes.c_double)]
    L.mi355x_gguf_get_float.restype = i32
    L.mi355x_gguf_get_str.argtypes = [vp, i64]
    L.mi355x_gguf_get_str.restype = ctypes.c_char_p
    L.mi355x_gguf_arr_n.argtypes = [vp, i64]
    L.mi355x_gguf_arr_n.restype = i64


class GGUFFile:
    """An open GGUF file. `tensors` maps name -> info dict; `kv` maps key -> value
    (ints, floats, strings; arrays as their length)."""

    def __init__(self, path):
        from . import lib
        self.L = lib()
        self.path = str(path)
        self.h = self.L.mi355x_gguf_open(self.path.encode())
        if not self.h:
            raise ValueError(f"not a readable GGUF file: {self.path}")
        self.version = int(self.L.mi355x_gguf_version(self.h))
        self.alignment = int(self.L.mi355x_gguf_alignment(self.h))
        self.data_offset = int(self.L.mi355x_gguf_data_offset(self.h))
        self.kv = {}
        for i in range(self.L.mi355x_gguf_n_kv(self.h)):
            key = self.L.mi355x_gguf_key(self.h, i).decode()
            t = self.L.mi355x_gguf_kv_type(self.h, i)
            if t == STRING:
                v = self.L.mi355x_gguf_get_str(self.h, i).decode()
            elif t == ARRAY:
                v = ("array", int(self.L.mi355x_gguf_arr_n(self.h, i)))
            elif t in (F32, F64):
                d = ctypes.c_double()
                self.L.mi355x_gguf_get_float(self.h, i, ctypes.byref(d))
                v = d.value
            else:
                n = ctypes.c_int64()
                self.L.mi355x_gguf_get_int(self.h, i, ctypes.byref(n))
                v = bool(n.value) if t == BOOL else n.value
            self.kv[key] = v
        self.tensors = {}
        self._index = {}
        for i in range(self.L.mi355x_gguf_n_tensors(self.h)):
            ti = TensorInfo()
            rc = self.L.mi355x_gguf_get_tensor(self.h, i, ctypes.byref(ti))
            assert rc == 0, rc
            name = ti.name.decode()
            self.tensors[name] = {"type": ti.type, "n_dims": ti.n_dims, "ne": tuple(ti.ne[:ti.n_dims]),
                                  "offset": int(ti.offset), "size": int(ti.size)}
            self._index[name] = i

    def bytes(self, name):
        """The tensor's raw bytes (a copy out of the mapping) as a numpy uint8 array."""
        import numpy as np
        info = self.tensors[name]
        ptr = self.L.mi355x_gguf_tensor_data(self.h, self._index[name])
        return np.ctypeslib.as_array((ctypes.c_uint8 * info["size"]).from_address(ptr)).copy()

    def upload(self, name, dst_ptr, dst_size, stream=None):
        """Async copy of the tensor's bytes to device memory (no repack)."""
        rc = self.L.mi355x_gguf_upload(self.h, self._index[name], dst_ptr, dst_size, stream)
        if rc != 0:
            raise RuntimeError(f"gguf upload of {name} failed: {rc}")

    def to_device(self, name, device="cuda"):
        """The tensor's bytes in a new torch uint8 device tensor, rows x row_bytes."""
        import torch
        info = self.tensors[name]
        rows = 1
        for d in info["ne"][1:]:
            rows *= d
        t = torch.empty(info["size"], dtype=torch.uint8, device=device)
        self.upload(name, t.data_ptr(), info["size"], torch.cuda.current_stream(t.device).cuda_stream)
        return t.view(rows, info["size"] // rows)

    def close(self):
        if self.h:
            self.L.mi355x_gguf_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
