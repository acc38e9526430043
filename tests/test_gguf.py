"""CPU checks of the native GGUF reader (kq_gguf.cpp through the C-ABI): metadata of
every value type, tensor infos and byte-identical tensor data for fixture files
written by an independent writer (tests/gguf_writer.py), custom alignment, and
that corrupt or truncated files are rejected without reading out of bounds."""
import os
import struct

import numpy as np
import pytest

from gguf_writer import (ARRAY, BOOL, F32, F64, I8, I16, I32, I64, STRING, U8, U16, U32, U64, mini_llama,
                         write_gguf)


def _tensors(rng, npo):
    return [("a.q4", 12, (512, 3), npo.random_blocks(rng, 12, 3, 512).reshape(-1)),
            ("b.q6", 14, (256, 5), npo.random_blocks(rng, 14, 5, 256).reshape(-1)),
            ("c.f32", 0, (7,), np.frombuffer(np.arange(7, dtype=np.float32).tobytes(), np.uint8)),
            ("d.q5", 13, (256, 2, 2), npo.random_blocks(rng, 13, 4, 256).reshape(-1))]


KV = [("u8", U8, 200), ("i8", I8, -5), ("u16", U16, 60000), ("i16", I16, -30000), ("u32", U32, 4000000000),
      ("i32", I32, -2000000000), ("f32", F32, 1.5), ("bool", BOOL, True), ("str", STRING, "héllo"),
      ("u64", U64, 2 ** 63 + 5), ("i64", I64, -(2 ** 62)), ("f64", F64, 2.0 ** -40),
      ("arr.u32", ARRAY, (U32, [1, 2, 3])), ("arr.str", ARRAY, (STRING, ["x", "yy", ""]))]


@pytest.mark.parametrize("alignment", [32, 64, 4096])
def test_roundtrip(tmp_path, npo, alignment):
    import ggml_mi355x.gguf as G
    rng = np.random.default_rng(alignment)
    tensors = _tensors(rng, npo)
    path = tmp_path / "t.gguf"
    data_off = write_gguf(path, KV, tensors, alignment=alignment)
    with G.GGUFFile(path) as f:
        assert f.version == 3 and f.alignment == alignment and f.data_offset == data_off
        assert f.kv["u8"] == 200 and f.kv["i8"] == -5 and f.kv["u16"] == 60000 and f.kv["i16"] == -30000
        assert f.kv["u32"] == 4000000000 and f.kv["i32"] == -2000000000 and f.kv["f32"] == 1.5
        assert f.kv["bool"] is True and f.kv["str"] == "héllo" and f.kv["f64"] == 2.0 ** -40
        assert f.kv["u64"] == (2 ** 63 + 5) - 2 ** 64 and f.kv["i64"] == -(2 ** 62)  # int64 view
        assert f.kv["arr.u32"] == ("array", 3) and f.kv["arr.str"] == ("array", 3)
        assert list(f.tensors) == [t[0] for t in tensors]
        for name, gt, ne, data in tensors:
            info = f.tensors[name]
            assert info["type"] == gt and info["ne"] == ne and info["size"] == len(data)
            assert info["offset"] % alignment == 0 and info["offset"] >= data_off
            assert np.array_equal(f.bytes(name), data)


def test_mini_llama_metadata(tmp_path, npo):
    import ggml_mi355x.gguf as G
    path = tmp_path / "m.gguf"
    want = mini_llama(path, np.random.default_rng(3), npo)
    with G.GGUFFile(path) as f:
        assert f.kv["general.architecture"] == "llama" and f.kv["llama.block_count"] == 2
        assert abs(f.kv["llama.attention.layer_norm_rms_epsilon"] - 1e-5) < 1e-12
        assert set(f.tensors) == set(want)
        for name, (gt, ne, data) in want.items():
            assert f.tensors[name]["type"] == gt and f.tensors[name]["ne"] == ne
            assert np.array_equal(f.bytes(name), data)


def _small_file(tmp_path, npo):
    path = tmp_path / "s.gguf"
    write_gguf(path, KV[:3] + [("arr.str", ARRAY, (STRING, ["ab"]))], _tensors(np.random.default_rng(1), npo)[:2])
    return path, path.read_bytes()


def test_truncated_files_rejected(tmp_path, npo):
    """Every prefix of a valid file (header, KV, tensor infos, data) fails to open."""
    import ggml_mi355x.gguf as G
    path, blob = _small_file(tmp_path, npo)
    G.GGUFFile(path).close()
    cut = tmp_path / "cut.gguf"
    for n in list(range(0, 200)) + list(range(200, len(blob), 97)) + [len(blob) - 1]:
        cut.write_bytes(blob[:n])
        with pytest.raises(ValueError):
            G.GGUFFile(cut)


def _patched(tmp_path, blob, off, fmt, value):
    b = bytearray(blob)
    struct.pack_into(fmt, b, off, value)
    p = tmp_path / "bad.gguf"
    p.write_bytes(bytes(b))
    return p


def test_corrupt_headers_rejected(tmp_path, npo):
    import ggml_mi355x.gguf as G
    _, blob = _small_file(tmp_path, npo)
    for off, fmt, v in [(0, "<I", 0x46554748),      # magic
                        (4, "<I", 1), (4, "<I", 4),  # versions
                        (8, "<Q", 2 ** 40),          # tensor count
                        (16, "<Q", 2 ** 40)]:        # kv count
        with pytest.raises(ValueError):
            G.GGUFFile(_patched(tmp_path, blob, off, fmt, v))
    # a string length running past the end of the file (first key's length)
    with pytest.raises(ValueError):
        G.GGUFFile(_patched(tmp_path, blob, 24, "<Q", 2 ** 31))


def test_bad_tensor_infos_rejected(tmp_path, npo):
    import ggml_mi355x.gguf as G
    rng = np.random.default_rng(2)
    t = _tensors(rng, npo)[0]
    p = tmp_path / "dup.gguf"
    write_gguf(p, [], [t, t])  # duplicate name
    with pytest.raises(ValueError):
        G.GGUFFile(p)
    # data beyond the end: write a valid file, then chop the data section
    p = tmp_path / "short.gguf"
    write_gguf(p, [], [t])
    p.write_bytes(p.read_bytes()[:-100])
    with pytest.raises(ValueError):
        G.GGUFFile(p)
    # misaligned offset: bump the tensor's offset field (last 8 bytes of the tensor info)
    p = tmp_path / "mis.gguf"
    write_gguf(p, [], [t])
    blob = p.read_bytes()
    name = t[0].encode()  # the offset field follows name, n_dims, dims and type
    pos = blob.index(name) + len(name) + 4 + 8 * len(t[2]) + 4
    with pytest.raises(ValueError):
        G.GGUFFile(_patched(tmp_path, blob, pos, "<Q", 8))
    # a row that is not a whole number of blocks (ne0 = 500 for Q4_K)
    pos_ne0 = blob.index(name) + len(name) + 4
    with pytest.raises(ValueError):
        G.GGUFFile(_patched(tmp_path, blob, pos_ne0, "<Q", 500))
    # ne = {2^40, 2^40}: (ne0/256)*144*ne1 wraps past 64 bits -- a wrapped small size
    # must not pass the end-of-file check (checked products)
    assert len(t[2]) == 2
    p2 = _patched(tmp_path, blob, pos_ne0, "<Q", 2 ** 40)
    with pytest.raises(ValueError):
        G.GGUFFile(_patched(tmp_path, p2.read_bytes(), pos_ne0 + 8, "<Q", 2 ** 40))
    # an unknown ggml type (its size cannot be bounded)
    with pytest.raises(ValueError):
        G.GGUFFile(_patched(tmp_path, blob, pos - 4, "<I", 99))


def test_missing_file():
    import ggml_mi355x.gguf as G
    with pytest.raises(ValueError):
        G.GGUFFile("/nonexistent/model.gguf")
    assert os.path.exists(os.path.dirname(os.path.abspath(__file__)))
