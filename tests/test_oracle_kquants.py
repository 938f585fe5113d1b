"""CPU oracle for the K-quant path: Q4_K / Q6_K weights x Q8_K activations.

Pins: (1) known answers built by hand (constant blocks, analytic dots); (2) the portable
AVX2-order emulation equals the AVX2-intrinsics form bit for bit; (3) both agree with the scalar
generic form (src/kernals.cl:48-111 for q4_K) to fp32 reordering; (4) quantize_row_q8_K known
answers.  The ggml AVX2 arithmetic itself is "parity unpinned" (ggml is absent)."""
import struct

import numpy as np
import pytest

import oracle_ctypes as O


def _f16(x):
    return int(O.lib().orc_fp32_to_fp16(x))


def _q8k_const(value, n_blocks):
    """Q8_K blocks with all qs = value, d = 1.0, bsums consistent."""
    out = b""
    for _ in range(n_blocks):
        out += struct.pack("<f", 1.0) + bytes([value & 0xFF]) * 256 + struct.pack("<16h", *([value * 16] * 16))
    return np.frombuffer(out, dtype=np.uint8).copy()


def test_q4_K_known_answer():
    # d = 1, dmin = 0, every 6-bit scale 1, mins 0, every nibble 1; q8 = 1 -> 256 per super-block
    scales = bytes([1, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1])  # sc 0..3 and 4..7 low nibbles = 1, mins 0
    blk = struct.pack("<HH", _f16(1.0), _f16(0.0)) + scales + bytes([0x11]) * 128
    w = np.frombuffer(blk * 2, dtype=np.uint8).copy()
    a = _q8k_const(1, 2)
    for form in ("ordered", "avx2", "generic"):
        assert O.vec_dot_k(O.Q4_K, w, a, 512, form) == 512.0, form
    # mins: dmin = 1, min 1 everywhere, q8 = 1 -> subtracts 256 per super-block
    scales_m = bytes([1, 1, 1, 1, 1, 1, 1, 1, 0x11, 0x11, 0x11, 0x11])
    blk = struct.pack("<HH", _f16(1.0), _f16(1.0)) + scales_m + bytes([0x11]) * 128
    w = np.frombuffer(blk, dtype=np.uint8).copy()
    for form in ("ordered", "avx2", "generic"):
        assert O.vec_dot_k(O.Q4_K, w, _q8k_const(1, 1), 256, form) == 0.0, form


def test_q6_K_known_answer():
    # q6 = 33 everywhere (ql nibbles 1, qh bits 2 -> 1 | 2<<4 = 33) -> (33-32) = 1; scales 1; d = 1
    blk = bytes([0x11]) * 128 + bytes([0xAA]) * 64 + bytes([1]) * 16 + struct.pack("<H", _f16(1.0))
    w = np.frombuffer(blk, dtype=np.uint8).copy()
    for form in ("ordered", "avx2", "generic"):
        assert O.vec_dot_k(O.Q6_K, w, _q8k_const(2, 1), 256, form) == 512.0, form


def test_q8_K_quantizer_known_answers():
    x = np.full((1, 256), 0.5, np.float32)
    q = O.quantize_q8_K(x)
    d = struct.unpack("<f", q[0, :4].tobytes())[0]
    qs = q[0, 4:260].view(np.int8)
    bs = q[0, 260:292].view(np.int16)
    assert np.all(qs == -127) and np.all(bs == -127 * 16)
    assert d == np.float32(1.0) / (np.float32(-127.0) / np.float32(0.5))
    z = O.quantize_q8_K(np.zeros((1, 256), np.float32))
    assert not z.any()


@pytest.mark.parametrize("wtype", [O.Q4_K, O.Q6_K], ids=["q4_K", "q6_K"])
@pytest.mark.parametrize("k", [256, 2048, 16384])
def test_kquant_avx2_equals_ordered_and_generic(wtype, k):
    rng = np.random.default_rng(k + wtype)
    W = O.synth_kquant(wtype, 7 + k, 6, k)
    X = (rng.standard_normal((3, k)) * rng.uniform(0.1, 4.0, (3, 1))).astype(np.float32)
    A = O.quantize_q8_K(X)
    for r in range(W.shape[0]):
        for c in range(A.shape[0]):
            o = O.vec_dot_k(wtype, W[r], A[c], k, "ordered")
            v = O.vec_dot_k(wtype, W[r], A[c], k, "avx2")
            g = O.vec_dot_k(wtype, W[r], A[c], k, "generic")
            assert np.float32(o).tobytes() == np.float32(v).tobytes(), (r, c, o, v)
            assert abs(o - g) <= 1e-5 * max(1.0, abs(g)) + 1e-4, (o, g)


def test_kquant_mul_mat_matches_vec_dot():
    k, rows = 2048, 40
    W = O.synth_kquant(O.Q4_K, 3, rows, k)
    X = np.random.default_rng(0).standard_normal((2, k)).astype(np.float32)
    wdata, rs = O.mul_mat_init(O.Q4_K, X)
    assert rs == k // 256 * 292
    Y = O.mul_mat(W, O.Q4_K, rows, W.shape[1], k, wdata, rs, 2)
    for c in range(2):
        for r in range(rows):
            assert Y[c, r] == np.float32(O.vec_dot_k(O.Q4_K, W[r], wdata[c], k, "avx2"))


# ---- dequantize_row_q4_K / q6_K (get_rows on a K-quant token_embd) -------------------------------
def _q4_K_scale_min(scales, j):
    """get_scale_min_k4 of ggml (the 6-bit packing src/kernals.cl:79-84 unpacks), written out."""
    if j < 4:
        return scales[j] & 63, scales[j + 4] & 63
    return (scales[j + 4] & 0xF) | ((scales[j - 4] >> 6) << 4), (scales[j + 4] >> 4) | ((scales[j] >> 6) << 4)


def _deq_q4_K_np(blocks):
    """numpy float32 restatement (same op order: d1 = d*sc, m1 = dmin*m, y = d1*q - m1)."""
    out = []
    for b in blocks.reshape(-1, 144):
        d = np.frombuffer(b[0:2].tobytes(), np.float16)[0].astype(np.float32)
        dmin = np.frombuffer(b[2:4].tobytes(), np.float16)[0].astype(np.float32)
        sc = b[4:16]
        q = b[16:]
        for j in range(4):
            s1, m1 = _q4_K_scale_min(sc, 2 * j)
            s2, m2 = _q4_K_scale_min(sc, 2 * j + 1)
            d1, mm1 = np.float32(d * np.float32(s1)), np.float32(dmin * np.float32(m1))
            d2, mm2 = np.float32(d * np.float32(s2)), np.float32(dmin * np.float32(m2))
            qq = q[32 * j:32 * j + 32]
            out.append((d1 * (qq & 15).astype(np.float32)).astype(np.float32) - mm1)
            out.append((d2 * (qq >> 4).astype(np.float32)).astype(np.float32) - mm2)
    return np.concatenate(out).astype(np.float32)


def _deq_q6_K_np(blocks):
    out = []
    for b in blocks.reshape(-1, 210):
        ql, qh = b[0:128].astype(np.int32), b[128:192].astype(np.int32)
        sc = b[192:208].view(np.int8).astype(np.float32)
        d = np.frombuffer(b[208:210].tobytes(), np.float16)[0].astype(np.float32)
        y = np.zeros(256, np.float32)
        for n in range(2):
            L, H, S = ql[64 * n:64 * n + 64], qh[32 * n:32 * n + 32], sc[8 * n:8 * n + 8]
            l = np.arange(32)
            is_ = l // 16
            qs = [(L[l] & 15) | ((H >> 0) & 3) << 4, (L[l + 32] & 15) | ((H >> 2) & 3) << 4,
                  (L[l] >> 4) | ((H >> 4) & 3) << 4, (L[l + 32] >> 4) | ((H >> 6) & 3) << 4]
            for g in range(4):
                y[128 * n + 32 * g + l] = (d * S[is_ + 2 * g]).astype(np.float32) * (qs[g] - 32).astype(np.float32)
        out.append(y)
    return np.concatenate(out)


@pytest.mark.parametrize("wtype", [O.Q4_K, O.Q6_K])
def test_dequantize_k_matches_numpy_restatement(wtype):
    k = 1024
    blocks = O.synth_kquant(wtype, 11, 1, k)
    got = O.dequantize(wtype, blocks, k)
    ref = _deq_q4_K_np(blocks) if wtype == O.Q4_K else _deq_q6_K_np(blocks)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_dequantize_k_known_answers():
    # Q4_K: d = 1, dmin = 0.5, scales all 1 / mins all 2 -> y = q - 1 exactly
    b = np.zeros(144, np.uint8)
    b[0:2] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
    b[2:4] = np.frombuffer(np.float16(0.5).tobytes(), np.uint8)
    b[4:8], b[8:12] = 1, 2          # j < 4: sc = scales[j] & 63, m = scales[j+4] & 63
    b[12:16] = 0x21                 # j >= 4: sc = low nibble | ..., m = high nibble | ...
    b[16:] = np.arange(128, dtype=np.uint8)
    y = O.dequantize(O.Q4_K, b, 256)
    q = np.concatenate([np.r_[np.arange(32 * j, 32 * j + 32) & 15, np.arange(32 * j, 32 * j + 32) >> 4]
                        for j in range(4)]).astype(np.float32)
    assert np.array_equal(y, q - 1.0)
    # Q6_K: d = 1, scales = 1: y = q6 - 32; all-zero quants -> -32
    b = np.zeros(210, np.uint8)
    b[192:208] = 1
    b[208:210] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
    assert np.all(O.dequantize(O.Q6_K, b, 256) == -32.0)
    b[0:128] = 0xFF
    b[128:192] = 0xFF
    assert np.all(O.dequantize(O.Q6_K, b, 256) == 31.0)


KMIX = dict(n_layer=2, n_embd=256, n_head=2, n_head_kv=1, head_dim=128, n_ff=512, n_vocab=1024)


def test_kmix_model_avx2_equals_ordered_and_prefill_equals_decode():
    cfg = O.make_config(KMIX, n_ctx=64, kmix=1)
    m = O.Model(cfg)
    prompt = O.make_prompt(9, KMIX["n_vocab"])
    seq, logits = m.generate(prompt, 4, avx2=True)
    seq_o, logits_o = m.generate(prompt, 4, avx2=False)
    assert seq == seq_o and np.array_equal(logits, logits_o)
    assert np.all(np.isfinite(logits)) and np.std(logits[-1]) > 0
    # the whole sequence in one PREFILL reproduces each decode step's last row
    m.reset()
    _, _, allv = m.inference(np.array(seq[:-1], np.int32), 0, want_all=True)
    for i in range(5):
        assert np.array_equal(allv[len(prompt) - 1 + i], logits[i])
    m.close()


def test_kmix_rejects_unaligned_shapes():
    with pytest.raises(ValueError):
        O.Model(O.make_config(dict(KMIX, n_embd=384), n_ctx=64, kmix=1))


def test_q6_K_output_layout_model_runs_and_is_consistent():
    """kmix = 2: llama.cpp's Q4_0 file layout (Q4_0 layers, Q6_K token_embd / output)."""
    shape = dict(KMIX, n_ff=384)
    m = O.Model(O.make_config(shape, n_ctx=64, kmix=2))
    prompt = O.make_prompt(6, shape["n_vocab"])
    seq, logits = m.generate(prompt, 3, avx2=True)
    seq_o, logits_o = m.generate(prompt, 3, avx2=False)
    assert seq == seq_o and np.array_equal(logits, logits_o) and np.all(np.isfinite(logits))
    assert len(m.tensor(16 + 1)) == 256 * shape["n_embd"] // 32 * 18   # a Q4_0 layer matrix
    assert len(m.tensor(0)) == shape["n_vocab"] * shape["n_embd"] // 256 * 210  # Q6_K token_embd
    m.close()
