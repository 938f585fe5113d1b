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
