"""Test infrastructure: a minimal, independent GGUF v3 writer (pure struct packing),
used to make fixture files for the native reader (kq_gguf.cpp). Layout per the
published GGUF format [U] (the reference reads it with ggml's gguf_reader,
artifacts/perf/out.folded:2-3):
  "GGUF" u32 version | u64 n_tensors | u64 n_kv | KVs | tensor infos | pad | data
"""
import struct

import numpy as np

U8, I8, U16, I16, U32, I32, F32, BOOL, STRING, ARRAY, U64, I64, F64 = range(13)
_FMT = {U8: "<B", I8: "<b", U16: "<H", I16: "<h", U32: "<I", I32: "<i", F32: "<f", BOOL: "<?",
        U64: "<Q", I64: "<q", F64: "<d"}
# ggml type -> (block elements, block bytes)
TYPE_SIZE = {0: (1, 4), 1: (1, 2), 12: (256, 144), 13: (256, 176), 14: (256, 210), 15: (256, 292), 30: (1, 2)}


def _str(s):
    b = s.encode() if isinstance(s, str) else s
    return struct.pack("<Q", len(b)) + b


def _value(t, v):
    if t == STRING:
        return _str(v)
    if t == ARRAY:
        et, items = v
        out = struct.pack("<IQ", et, len(items))
        for it in items:
            out += _value(et, it)
        return out
    return struct.pack(_FMT[t], v)


def tensor_nbytes(ggml_type, ne):
    blck, nbytes = TYPE_SIZE[ggml_type]
    rows = 1
    for d in ne[1:]:
        rows *= d
    assert ne[0] % blck == 0
    return ne[0] // blck * nbytes * rows


def write_gguf(path, kv, tensors, alignment=32, version=3):
    """kv: list of (key, type, value) — ARRAY values are (elem_type, [items]);
    tensors: list of (name, ggml_type, ne tuple, uint8 bytes). Writes general.alignment
    when it is not the default. Returns the data section offset."""
    kv = list(kv)
    if alignment != 32 and not any(k == "general.alignment" for k, _, _ in kv):
        kv.append(("general.alignment", U32, alignment))
    head = b"GGUF" + struct.pack("<IQQ", version, len(tensors), len(kv))
    for key, t, v in kv:
        head += _str(key) + struct.pack("<I", t) + _value(t, v)
    offsets, off = [], 0
    for name, gt, ne, data in tensors:
        assert len(data) == tensor_nbytes(gt, ne), name
        offsets.append(off)
        off += len(data)
        off = (off + alignment - 1) // alignment * alignment
    for (name, gt, ne, data), o in zip(tensors, offsets):
        head += _str(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", d) for d in ne)
        head += struct.pack("<IQ", gt, o)
    data_off = (len(head) + alignment - 1) // alignment * alignment
    with open(path, "wb") as f:
        f.write(head)
        f.write(b"\0" * (data_off - len(head)))
        pos = 0
        for (name, gt, ne, data), o in zip(tensors, offsets):
            f.write(b"\0" * (o - pos))
            f.write(np.asarray(data, np.uint8).tobytes())
            pos = o + len(data)
    return data_off


def mini_llama(path, rng, npo, E=512, L=2, KV=256, FF=1024, V=1000, extra_kv=()):
    """A llama-architecture Q4_K_M-style model file with small shapes: token_embd
    Q4_K, per layer attn_q/k/v/output, ffn_gate/up/down (attn_v, ffn_down Q6_K in
    layer 0), f32 norms, output Q6_K. Returns {name: (ggml_type, ne, bytes)}."""
    kv = [("general.architecture", STRING, "llama"), ("general.name", STRING, "mini-llama"),
          ("llama.block_count", U32, L), ("llama.embedding_length", U32, E),
          ("llama.feed_forward_length", U32, FF), ("llama.attention.head_count", U32, E // 64),
          ("llama.attention.head_count_kv", U32, KV // 64), ("llama.context_length", U32, 2048),
          ("llama.attention.layer_norm_rms_epsilon", F32, 1e-5), ("general.file_type", U32, 15),
          ("tokenizer.ggml.tokens", ARRAY, (STRING, [f"t{i}" for i in range(8)]))] + list(extra_kv)
    spec = [("token_embd.weight", 12, (E, V))]
    for i in range(L):
        more = i == 0
        spec += [(f"blk.{i}.attn_norm.weight", 0, (E,)),
                 (f"blk.{i}.attn_q.weight", 12, (E, E)), (f"blk.{i}.attn_k.weight", 12, (E, KV)),
                 (f"blk.{i}.attn_v.weight", 14 if more else 12, (E, KV)),
                 (f"blk.{i}.attn_output.weight", 12, (E, E)), (f"blk.{i}.ffn_norm.weight", 0, (E,)),
                 (f"blk.{i}.ffn_gate.weight", 12, (E, FF)), (f"blk.{i}.ffn_up.weight", 12, (E, FF)),
                 (f"blk.{i}.ffn_down.weight", 14 if more else 12, (FF, E))]
    spec += [("output_norm.weight", 0, (E,)), ("output.weight", 14, (E, V))]
    tensors, out = [], {}
    for name, gt, ne in spec:
        if gt == 0:
            data = np.frombuffer(rng.standard_normal(ne[0]).astype(np.float32).tobytes(), np.uint8)
        else:
            data = npo.random_blocks(rng, gt, ne[1], ne[0]).reshape(-1)
        tensors.append((name, gt, ne, data))
        out[name] = (gt, ne, data)
    write_gguf(path, kv, tensors)
    return out
