"""CPU: the library's GGUF reader (csrc/gguf.cpp; the gguf_* API src/gemma_model.cpp:19-229 and
583-648 load models through) against files written by tests/gguf_writer.py.

Parity note: the `gguf` package and real model files are absent, so the files are
written here from the published layout; every value read back must equal what was written, and
every malformed file must fail with a message (no crash, no over-read)."""
import os
import struct
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import gemma_hip as G  # noqa: E402
from gguf_writer import (ARR, BOOL, F32, F64, I8, I16, I32, I64, STR, U8, U16, U32, U64,  # noqa: E402
                         GGUFWriter)


def _sample(alignment=32, version=3):
    rng = np.random.default_rng(7)
    w = GGUFWriter(alignment=alignment, version=version)
    w.add("general.architecture", STR, "gemma")
    w.add("gemma.block_count", U32, 18)
    w.add("gemma.attention.layer_norm_rms_epsilon", F32, 1e-6)
    w.add("k.u8", U8, 200)
    w.add("k.i8", I8, -5)
    w.add("k.u16", U16, 65000)
    w.add("k.i16", I16, -32000)
    w.add("k.i32", I32, -123456)
    w.add("k.u64", U64, 2 ** 40 + 3)
    w.add("k.i64", I64, -(2 ** 40))
    w.add("k.f64", F64, 3.25)
    w.add("k.bool", BOOL, True)
    w.add("tokenizer.ggml.tokens", ARR, ["<pad>", "<eos>", "<bos>", "▁hello", "é"], STR)
    w.add("tokenizer.ggml.scores", ARR, [0.0, -1.5, 2.25, 3.0, 4.0], F32)
    w.add("tokenizer.ggml.token_type", ARR, [3, 3, 3, 1, 1], I32)
    w.add("k.empty", ARR, [], U32)
    tens = {
        "token_embd.weight": (2, (64, 5), rng.integers(0, 256, 5 * 2 * 18, dtype=np.uint8)),
        "output_norm.weight": (0, (64,), rng.standard_normal(64).astype(np.float32)),
        "blk.0.attn_q.weight": (8, (64, 3), rng.integers(0, 256, 3 * 2 * 34, dtype=np.uint8)),
        "blk.0.ffn_gate.weight": (12, (256, 2), rng.integers(0, 256, 2 * 144, dtype=np.uint8)),
        "blk.0.ffn_down.weight": (14, (512, 1), rng.integers(0, 256, 2 * 210, dtype=np.uint8)),
        "blk.0.kv.f16": (1, (3, 2, 2), rng.integers(0, 2 ** 16, 12, dtype=np.uint16)),
    }
    for name, (t, ne, data) in tens.items():
        w.add_tensor(name, t, ne, data)
    return w, tens


def test_round_trip(tmp_path):
    w, tens = _sample()
    p = str(tmp_path / "m.gguf")
    w.write(p)
    f = G.GGUF(p)
    assert f.version == 3 and f.alignment == 32 and f.data_offset % 32 == 0
    kv = f.kv
    assert kv["general.architecture"] == "gemma" and kv["gemma.block_count"] == 18
    assert kv["gemma.attention.layer_norm_rms_epsilon"] == np.float32(1e-6)
    assert (kv["k.u8"], kv["k.i8"], kv["k.u16"], kv["k.i16"], kv["k.i32"]) == (200, -5, 65000, -32000, -123456)
    assert (kv["k.u64"], kv["k.i64"], kv["k.f64"], kv["k.bool"]) == (2 ** 40 + 3, -(2 ** 40), 3.25, True)
    assert kv["tokenizer.ggml.tokens"] == ["<pad>", "<eos>", "<bos>", "▁hello", "é"]
    assert kv["tokenizer.ggml.scores"] == [0.0, -1.5, 2.25, 3.0, 4.0]
    assert kv["tokenizer.ggml.token_type"] == [3, 3, 3, 1, 1]
    assert kv["k.empty"] == []
    assert list(f.tensors) == list(tens)
    for name, (t, ne, data) in tens.items():
        rt, rne, rdata, off = f.tensors[name]
        assert rt == t and rne[:len(ne)] == tuple(ne) and all(x == 1 for x in rne[len(ne):])
        assert rdata == data.tobytes(), name
        assert off % 32 == 0


@pytest.mark.parametrize("alignment,version", [(64, 3), (128, 2), (32, 2)])
def test_alignment_and_v2(tmp_path, alignment, version):
    w, tens = _sample(alignment, version)
    p = str(tmp_path / "m.gguf")
    w.write(p)
    f = G.GGUF(p)
    assert f.alignment == alignment and f.version == version and f.data_offset % alignment == 0
    for name, (_, _, data) in tens.items():
        assert f.tensors[name][2] == data.tobytes()


def test_no_alloc_reads_metadata_only(tmp_path):
    w, tens = _sample()
    p = str(tmp_path / "m.gguf")
    w.write(p)
    f = G.GGUF(p, load_tensors=False)
    assert set(f.tensors) == set(tens) and all(v[2] is None for v in f.tensors.values())


def _expect_error(path, fragment):
    with pytest.raises(ValueError) as e:
        G.GGUF(path)
    assert fragment in str(e.value), str(e.value)


def test_malformed_files_fail_with_a_message(tmp_path):
    w, _ = _sample()
    good = w.to_bytes()
    cases = {
        "magic": (b"GGUX" + good[4:], "bad magic"),
        "v1": (good[:4] + struct.pack("<I", 1) + good[8:], "v1"),
        "v9": (good[:4] + struct.pack("<I", 9) + good[8:], "newer"),
        "counts": (good[:8] + struct.pack("<QQ", 2 ** 40, 2 ** 40) + good[24:], "exceed"),
        "empty": (b"", "end of file"),
    }
    for name, (blob, frag) in cases.items():
        p = str(tmp_path / f"{name}.gguf")
        open(p, "wb").write(blob)
        _expect_error(p, frag)
    # every truncation point fails cleanly (header, kv pairs, tensor infos, data)
    step = max(1, len(good) // 97)
    for cut in list(range(0, len(good) - 32, step)) + [len(good) - 40]:  # (the last 8 bytes are padding)
        p = str(tmp_path / "cut.gguf")
        open(p, "wb").write(good[:cut])
        with pytest.raises(ValueError):
            G.GGUF(p)
    _expect_error(str(tmp_path / "missing.gguf"), "cannot open")


def test_bad_tensor_infos(tmp_path):
    def one(t, ne, data, offsets=None, **kw):
        w = GGUFWriter()
        w.add("a", U32, 1)
        w.tensors.append(("x", t, list(ne), data))
        p = str(tmp_path / "t.gguf")
        w.write(p, offsets=offsets)
        return p
    _expect_error(one(99, (4,), b"\0" * 16), "unsupported ggml type")
    _expect_error(one(2, (33,), b"\0" * 18), "block size")
    _expect_error(one(0, (4,), b"\0" * 16, offsets=[8]), "not aligned")
    _expect_error(one(0, (1 << 30,), b"\0" * 16), "past the end")
    # an offset near UINT64_MAX (aligned): offset + bytes wraps; must still be rejected
    _expect_error(one(0, (4,), b"\0" * 16, offsets=[(1 << 64) - 32]), "past the end")
    # dimensions whose byte count overflows size_t
    _expect_error(one(0, (1 << 40, 1 << 40, 1 << 40), b"\0" * 16), "too many elements")
    w = GGUFWriter()
    w.add("dup", U32, 1)
    w.add("dup", U32, 2)
    p = str(tmp_path / "dup.gguf")
    w.write(p)
    _expect_error(p, "duplicate key")
    w = GGUFWriter()
    w.add_tensor("t", 0, (4,), np.zeros(4, np.float32))
    w.add_tensor("t", 0, (4,), np.zeros(4, np.float32))
    w.write(p)
    _expect_error(p, "duplicate tensor")


def test_length_bombs_are_rejected_before_allocating(tmp_path):
    # a key whose string length claims 2^62 bytes, and an array claiming 2^60 elements
    head = struct.pack("<4sIQQ", b"GGUF", 3, 0, 1)
    p = str(tmp_path / "bomb.gguf")
    open(p, "wb").write(head + struct.pack("<Q", 2 ** 62) + b"abc")
    _expect_error(p, "past the end")
    open(p, "wb").write(head + struct.pack("<Q", 1) + b"k" + struct.pack("<IIQ", ARR, U32, 2 ** 60))
    _expect_error(p, "longer than the file")
    open(p, "wb").write(head + struct.pack("<Q", 1) + b"k" + struct.pack("<IIQ", ARR, STR, 2 ** 60))
    _expect_error(p, "longer than the file")


def _model_file(tmp_path, kmix, wtype=2, drop=None):
    import oracle_ctypes as O
    from test_gpu_ggml_graph import write_gguf
    shape = dict(n_layer=1, n_embd=256, n_head=2, n_head_kv=1, head_dim=128, n_ff=512, n_vocab=512)
    m = O.Model(O.make_config(shape, n_ctx=64, wtype=wtype, kmix=kmix))
    p = str(tmp_path / "m.gguf")
    write_gguf(m, shape, p, kmix)
    m.close()
    return p


def test_engine_from_gguf_rejects_unsupported_layouts(tmp_path):
    """The engine's GGUF loader validates before touching the GPU (runs on the CPU)."""
    import ctypes as C
    L = G.lib()
    # a Q5_K layer matrix (Q4_K_M files never hold one; Q5_K_M files do): rejected with a message
    E, V, F = 256, 512, 512
    w = GGUFWriter()
    for k, v in (("block_count", 1), ("embedding_length", E), ("attention.head_count", 2),
                 ("attention.head_count_kv", 1), ("attention.key_length", 128)):
        w.add("gemma." + k, U32, v)
    w.add_tensor("token_embd.weight", 14, [E, V], np.zeros(V * E // 256 * 210, np.uint8))
    w.add_tensor("output_norm.weight", 0, [E], np.ones(E, np.float32))
    GGUF_BLOCK_Q5_K = (13, 176)
    import gguf_writer
    gguf_writer.GGML_BLOCK.setdefault(13, (176, 256))
    w.add_tensor("blk.0.attn_q.weight", GGUF_BLOCK_Q5_K[0], [E, 256], np.zeros(256 * E // 256 * 176, np.uint8))
    w.add_tensor("blk.0.ffn_gate.weight", 12, [E, F], np.zeros(F * E // 256 * 144, np.uint8))
    p = str(tmp_path / "q5k.gguf")
    w.write(p)
    assert not L.gemma_engine_create_from_gguf(p.encode(), 64, 0)
    assert "Q4_K" in G.last_error(), G.last_error()
    bad = str(tmp_path / "bad.gguf")
    w = GGUFWriter()
    w.add("gemma.block_count", U32, 1)
    w.write(bad)
    assert not L.gemma_engine_create_from_gguf(bad.encode(), 64, 0)
    assert "missing u32 key gemma.embedding_length" in G.last_error()
    assert not L.gemma_engine_create_from_gguf(str(tmp_path / "none.gguf").encode(), 64, 0)
    assert "cannot open" in G.last_error()
    del C
