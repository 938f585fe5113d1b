"""ctypes binding of the CPU ORACLE (oracle/lib/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "lib", "liboracle.so")

F32, F16, Q4_0, Q8_0 = 0, 1, 2, 8
Q4_K, Q6_K, Q8_K = 12, 14, 15


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


class OrcConfig(C.Structure):
    _fields_ = [("n_layer", C.c_int), ("n_embd", C.c_int), ("n_head", C.c_int), ("n_head_kv", C.c_int),
                ("head_dim", C.c_int), ("n_ff", C.c_int), ("n_vocab", C.c_int), ("n_ctx", C.c_int),
                ("wtype", C.c_int), ("eps", C.c_float), ("rope_base", C.c_float), ("seed", C.c_uint64),
                ("gelu_clamp", C.c_int), ("kmix", C.c_int), ("out_gain", C.c_float)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    vp, i64, f32p = C.c_void_p, C.c_int64, C.POINTER(C.c_float)
    L.orc_fp32_to_fp16.restype = C.c_uint16
    L.orc_fp32_to_fp16.argtypes = [C.c_float]
    L.orc_fp16_to_fp32.restype = C.c_float
    L.orc_fp16_to_fp32.argtypes = [C.c_uint16]
    L.orc_fp16_selfcheck.restype = C.c_int64
    L.orc_fp16_selfcheck.argtypes = [C.c_uint32]
    L.orc_init_tables.argtypes = [C.c_int]
    L.orc_table_exp_f16.restype = vp
    L.orc_table_gelu_f16.restype = vp
    for fn in ("orc_quantize_row_q4_0_ref", "orc_quantize_row_q8_0_ref", "orc_quantize_row_q8_0"):
        getattr(L, fn).argtypes = [vp, vp, C.c_int]
    for fn in ("orc_dequantize_row_q4_0", "orc_dequantize_row_q8_0", "orc_dequantize_row_q4_K",
               "orc_dequantize_row_q6_K"):
        getattr(L, fn).argtypes = [vp, vp, C.c_int]
    L.orc_row_size.restype = C.c_size_t
    L.orc_row_size.argtypes = [C.c_int, i64]
    for fn in ("orc_vec_dot_q4_0_q8_0", "orc_vec_dot_q8_0_q8_0", "orc_vec_dot_f16",
               "orc_vec_dot_q4_0_q8_0_avx2", "orc_vec_dot_q8_0_q8_0_avx2", "orc_vec_dot_f16_avx2"):
        getattr(L, fn).argtypes = [C.c_int, f32p, vp, vp]
    L.orc_block_lane_sums.argtypes = [C.c_int, vp, vp, vp]
    L.orc_quantize_row_q8_K.argtypes = [vp, vp, C.c_int]
    for fn in ("orc_vec_dot_q4_K_q8_K", "orc_vec_dot_q6_K_q8_K", "orc_vec_dot_q4_K_q8_K_avx2",
               "orc_vec_dot_q6_K_q8_K_avx2", "orc_vec_dot_q4_K_q8_K_generic", "orc_vec_dot_q6_K_q8_K_generic"):
        getattr(L, fn).argtypes = [C.c_int, f32p, vp, vp]
    L.orc_synth_kquant.argtypes = [C.c_int, C.c_uint64, i64, i64, vp]
    L.orc_rms_norm.argtypes = [vp, vp, C.c_int, C.c_float]
    L.orc_soft_max_row.argtypes = [vp, vp, vp, C.c_int, C.c_float]
    L.orc_rope_neox.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_float]
    L.orc_rope_cos_sin.argtypes = [C.c_int, C.c_int, C.c_float, vp, vp]
    L.orc_gelu.argtypes = [vp, vp, C.c_int]
    L.orc_set_threads.argtypes = [C.c_int]
    L.orc_mul_mat.argtypes = [i64, i64, i64, i64, i64, i64, i64, C.c_size_t, i64, vp, vp, C.c_int, vp, C.c_int]
    L.orc_mul_mat_init.argtypes = [C.c_int, vp, i64, i64, i64, vp]
    L.orc_model_create.restype = vp
    L.orc_model_create.argtypes = [C.POINTER(OrcConfig)]
    L.orc_model_free.argtypes = [vp]
    L.orc_model_tensor.restype = vp
    L.orc_model_tensor.argtypes = [vp, C.c_int, C.POINTER(C.c_int64)]
    L.orc_model_reset_kv.argtypes = [vp]
    L.orc_model_inference.restype = C.c_int
    L.orc_model_inference.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, C.c_int]
    L.orc_model_hidden.restype = C.c_int
    L.orc_model_hidden.argtypes = [vp, C.c_int, vp, i64]
    L.orc_bench_run.restype = C.c_double
    L.orc_bench_run.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, vp, C.POINTER(C.c_double), vp]
    L.orc_set_pool.argtypes = [C.c_int]
    L.orc_prof.argtypes = [C.c_int, vp]
    L.orc_make_prompt.argtypes = [C.c_uint64, C.c_int, C.c_int, vp]
    L.orc_synth_value.restype = C.c_float
    L.orc_synth_value.argtypes = [C.c_uint64, C.c_int, C.c_uint64, C.c_double]
    _lib = L
    return L


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def fp32_to_fp16_bits(x):
    L = lib()
    x = np.asarray(x, dtype=np.float32).ravel()
    return np.array([L.orc_fp32_to_fp16(float(v)) for v in x], dtype=np.uint16)


def quantize(x, kind):
    """kind: 'q4_0_ref', 'q8_0_ref', 'q8_0' (AVX2 activation quantizer). x: [rows, k] f32."""
    L = lib()
    x = np.ascontiguousarray(x, dtype=np.float32)
    rows, k = x.shape
    bpb = 18 if kind == "q4_0_ref" else 34
    out = np.zeros((rows, k // 32 * bpb), dtype=np.uint8)
    fn = {"q4_0_ref": L.orc_quantize_row_q4_0_ref, "q8_0_ref": L.orc_quantize_row_q8_0_ref,
          "q8_0": L.orc_quantize_row_q8_0}[kind]
    for r in range(rows):
        fn(ptr(x[r]), ptr(out[r]), k)
    return out


KQ_BLOCK = {12: 144, 14: 210}   # Q4_K, Q6_K bytes per 256 values


def synth_kquant(wtype, seed, rows, k):
    """Random valid Q4_K / Q6_K blocks, [rows, k/256*bpb] bytes (ggml layout)."""
    out = np.zeros((rows, k // 256 * KQ_BLOCK[wtype]), dtype=np.uint8)
    lib().orc_synth_kquant(wtype, seed, rows, k, ptr(out))
    return out


def quantize_q8_K(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    rows, k = x.shape
    out = np.zeros((rows, k // 256 * 292), dtype=np.uint8)
    for r in range(rows):
        lib().orc_quantize_row_q8_K(ptr(x[r]), ptr(out[r]), k)
    return out


def vec_dot_k(wtype, wrow, arow, k, form="ordered"):
    """form: 'ordered' (AVX2-order emulation), 'avx2', 'generic'."""
    L = lib()
    name = {12: "q4_K", 14: "q6_K"}[wtype]
    sfx = {"ordered": "", "avx2": "_avx2", "generic": "_generic"}[form]
    s = C.c_float()
    getattr(L, f"orc_vec_dot_{name}_q8_K{sfx}")(k, C.byref(s), ptr(wrow), ptr(arow))
    return s.value


def vec_dot(wtype, wrow, arow, k, avx2=False):
    L = lib()
    s = C.c_float()
    if wtype == Q4_0:
        fn = L.orc_vec_dot_q4_0_q8_0_avx2 if avx2 else L.orc_vec_dot_q4_0_q8_0
    elif wtype == Q8_0:
        fn = L.orc_vec_dot_q8_0_q8_0_avx2 if avx2 else L.orc_vec_dot_q8_0_q8_0
    else:
        fn = L.orc_vec_dot_f16_avx2 if avx2 else L.orc_vec_dot_f16
    fn(k, C.byref(s), ptr(wrow), ptr(arow))
    return s.value


def mul_mat(src0, src0_type, ne01, nb01, k, wdata, row_size, ncols, avx2=True):
    """Plain 2-D case: dst[ncols][ne01]."""
    L = lib()
    dst = np.zeros((ncols, ne01), dtype=np.float32)
    L.orc_mul_mat(ne01, ncols, 1, nb01, ncols, ne01 * 4, ne01 * 4 * ncols, row_size, k, ptr(src0), ptr(dst),
                  src0_type, ptr(wdata), 1 if avx2 else 0)
    return dst


def mul_mat_init(src0_type, x):
    L = lib()
    x = np.ascontiguousarray(x, dtype=np.float32)
    ncols, k = x.shape
    rs = k * 2 if src0_type == F16 else (k // 256 * 292 if src0_type in (Q4_K, Q6_K) else k // 32 * 34)
    out = np.zeros((ncols, rs), dtype=np.uint8)
    L.orc_mul_mat_init(src0_type, ptr(x), k, ncols, k, ptr(out))
    return out, rs


GEMMA_2B = dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
GEMMA_7B = dict(n_layer=28, n_embd=3072, n_head=16, n_head_kv=16, head_dim=256, n_ff=24576, n_vocab=256000)
TINY = dict(n_layer=2, n_embd=512, n_head=2, n_head_kv=1, head_dim=256, n_ff=2048, n_vocab=4096)


def make_config(shape, n_ctx=512, wtype=Q4_0, seed=0x6E6D6D61, eps=1e-6, rope_base=10000.0, gelu_clamp=0, kmix=0,
                out_gain=0.0):
    return OrcConfig(n_ctx=n_ctx, wtype=wtype, eps=eps, rope_base=rope_base, seed=seed, gelu_clamp=gelu_clamp,
                     kmix=kmix, out_gain=out_gain, **shape)


def dequantize(wtype, row_bytes, k):
    """ggml dequantize_row_{q4_0,q8_0,q4_K,q6_K} of one row (get_rows)."""
    fn = {Q4_0: "orc_dequantize_row_q4_0", Q8_0: "orc_dequantize_row_q8_0", Q4_K: "orc_dequantize_row_q4_K",
          Q6_K: "orc_dequantize_row_q6_K"}[wtype]
    src = np.ascontiguousarray(row_bytes, dtype=np.uint8)
    out = np.zeros(k, dtype=np.float32)
    getattr(lib(), fn)(ptr(src), ptr(out), k)
    return out


class Model:
    def __init__(self, cfg):
        self.cfg = cfg
        self.L = lib()
        self.h = self.L.orc_model_create(C.byref(cfg))
        if not self.h:
            raise ValueError("orc_model_create rejected the config")

    def close(self):
        if self.h:
            self.L.orc_model_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def tensor(self, tid):
        n = C.c_int64()
        p = self.L.orc_model_tensor(self.h, tid, C.byref(n))
        return np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p)).copy()

    def poke(self, tid, offset, data):
        """Overwrite bytes of one of the model's tensors in place (test construction of adversarial
        weights; the oracle then computes with them as with its own)."""
        n = C.c_int64()
        p = self.L.orc_model_tensor(self.h, tid, C.byref(n))
        data = np.ascontiguousarray(data).view(np.uint8).ravel()
        assert p and 0 <= offset and offset + data.size <= n.value, (tid, offset, data.size, n.value)
        C.memmove(p + offset, data.ctypes.data, data.size)

    def reset(self):
        self.L.orc_model_reset_kv(self.h)

    def inference(self, tokens, stage, want_all=False, avx2=True):
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        last = np.zeros(self.cfg.n_vocab, dtype=np.float32)
        T = len(toks) if stage == 0 else 1
        allv = np.zeros((T, self.cfg.n_vocab), dtype=np.float32) if want_all else None
        tok = self.L.orc_model_inference(self.h, ptr(toks), len(toks), stage, ptr(last),
                                         ptr(allv) if want_all else None, 1 if avx2 else 0)
        return tok, last, allv

    def hidden(self, il, T):
        out = np.zeros(T * self.cfg.n_embd, dtype=np.float32)
        self.L.orc_model_hidden(self.h, il, ptr(out), out.size)
        return out.reshape(T, self.cfg.n_embd)

    def generate(self, prompt, n_decode, avx2=True):
        """Reference loop (src/gemma_model.cpp:548-575): PREFILL then greedy DECODE steps."""
        self.reset()
        seq = list(int(t) for t in prompt)
        logits = []
        tok, last, _ = self.inference(seq, 0, avx2=avx2)
        seq.append(tok)
        logits.append(last)
        for _ in range(n_decode):
            tok, last, _ = self.inference(seq, 1, avx2=avx2)
            seq.append(tok)
            logits.append(last)
        return seq, np.stack(logits)


def make_prompt(n, n_vocab, seed=1):
    out = np.zeros(n, dtype=np.int32)
    lib().orc_make_prompt(seed, n, n_vocab, ptr(out))
    return out
