"""ctypes binding of libgemma_hip.so — the MI355X hot path behind the C-ABI in include/gemma_hpc.h.

Product-side host mirror: it only forwards to the HIP library and never falls back to CPU code.
Loading fails loudly if the library is missing or was not built for gfx950.
"""
import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libgemma_hip.so")
# GHIP_LIB: an alternative build of the same library, for A/B timing of two builds on one box
# (scripts/lib_ab.sh).  Honoured only with GHIP_ALLOW_ALT_LIB=1, so a stray variable can never make
# a test, smoke() or bench.py load anything but the in-tree build.
if os.environ.get("GHIP_LIB"):
    if os.environ.get("GHIP_ALLOW_ALT_LIB") != "1":
        raise RuntimeError("GHIP_LIB is set but GHIP_ALLOW_ALT_LIB=1 is not: refusing to load a non-tree library")
    LIB_PATH = os.environ["GHIP_LIB"]

GGML_TYPE_F32, GGML_TYPE_F16, GGML_TYPE_Q4_0, GGML_TYPE_Q8_0 = 0, 1, 2, 8
GGML_TYPE_Q4_K, GGML_TYPE_Q6_K, GGML_TYPE_Q8_K = 12, 14, 15

# exported symbols (checked against include/gemma_hpc.h by tests/test_capi_symbols.py)
EXPORTS = ["mul_mat", "hpc_init", "hpc_shutdown", "hpc_register_weight", "hpc_last_error", "hpc_set_error_mode",
           "hpc_weight_cache_entries", "hpc_set_matvec_ks", "hpc_set_gemm_x4", "gemma_engine_debug_step", "gemma_engine_stamp_step", "gemma_engine_create", "gemma_engine_free", "gemma_engine_begin",
           "gemma_engine_step", "gemma_engine_tokens", "gemma_engine_pos", "gemma_engine_prefill",
           "gemma_engine_prefill_fast", "gemma_engine_prefill_taps", "gemma_test_gemm", "gemma_test_gemm_exact", "gemma_kq_time", "hpc_graph_compute",
           "ggml_init", "ggml_free", "ggml_new_tensor_2d", "ggml_mul_mat", "ggml_graph_compute_with_ctx",
           "gemma_engine_tensor", "gemma_engine_time", "gemma_engine_sync", "gemma_engine_tune",
           "gemma_engine_plan", "gemma_engine_set_plan", "gemma_engine_set_fuse", "gemma_engine_set_att_o", "gemma_engine_set_option", "gemma_engine_set_persist", "gemma_engine_persist_err", "gemma_engine_graph_kernels", "gemma_hbm_read_gbs", "gemma_hbm_read_probe",
           "gemma_tp_unique_id", "gemma_engine_create_tp", "gemma_engine_create_tp2", "gemma_engine_tp_flags", "gemma_engine_p2p_handle", "gemma_engine_p2p_open", "gemma_engine_p2p_err", "gemma_engine_tp_info", "gemma_engine_set_persist_timeout",
           "gguf_init_from_file", "gguf_free", "gguf_get_n_kv", "gguf_get_key", "gguf_get_kv_type",
           "gguf_get_arr_type", "gguf_get_arr_n", "gguf_get_arr_data", "gguf_get_arr_str", "gguf_get_val_str",
           "gguf_get_val_data", "gguf_get_n_tensors", "gguf_get_tensor_name", "gguf_get_tensor_type",
           "gguf_get_tensor_offset", "gguf_get_version", "gguf_get_alignment", "gguf_get_data_offset",
           "gguf_find_key", "gguf_find_tensor", "ggml_get_tensor", "ggml_nbytes",
           "gemma_engine_create_from_gguf", "gemma_engine_config"]


def build():
    subprocess.run(["make", "-s", "-j8", "-C", PKG_DIR], check=True)


TP_REP_ATTN = 1  # include/gemma_hpc.h GEMMA_TP_REP_ATTN
TP_P2P = 2       # include/gemma_hpc.h GEMMA_TP_P2P: peer-to-peer gathers instead of RCCL (tp id None)


class GemmaConfig(C.Structure):
    _fields_ = [("n_layer", C.c_int), ("n_embd", C.c_int), ("n_head", C.c_int), ("n_head_kv", C.c_int),
                ("head_dim", C.c_int), ("n_ff", C.c_int), ("n_vocab", C.c_int), ("n_ctx", C.c_int),
                ("wtype", C.c_int), ("eps", C.c_float), ("rope_base", C.c_float), ("seed", C.c_uint64),
                ("gelu_clamp", C.c_int), ("out_type", C.c_int), ("out_gain", C.c_float)]


class GgmlTensor(C.Structure):
    """struct ggml_tensor as declared in include/ggml.h (only `data` is read by mul_mat)."""
    _fields_ = [("type", C.c_int), ("backend", C.c_int), ("buffer", C.c_void_p), ("ne", C.c_int64 * 4),
                ("nb", C.c_size_t * 4), ("op", C.c_int32), ("op_params", C.c_int32 * 16), ("flags", C.c_int32),
                ("grad", C.c_void_p), ("src", C.c_void_p * 10), ("perf_runs", C.c_int), ("perf_cycles", C.c_int64),
                ("perf_time_us", C.c_int64), ("view_src", C.c_void_p), ("view_offs", C.c_size_t),
                ("data", C.c_void_p), ("name", C.c_char * 64), ("extra", C.c_void_p), ("padding", C.c_char * 8)]


class GGUFInitParams(C.Structure):
    _fields_ = [("no_alloc", C.c_bool), ("ctx", C.POINTER(C.c_void_p))]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libgemma_hip.so not built ({LIB_PATH}); run `make -C {PKG_DIR}` or "
                           "__graft_entry__.build() — there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, i64 = C.c_void_p, C.c_int64
    L.mul_mat.restype = None
    L.mul_mat.argtypes = [i64, i64, i64, i64, i64, i64, i64, C.c_size_t, i64, vp, vp, vp, vp, C.c_int, vp]
    L.hpc_init.restype = C.c_int
    L.hpc_init.argtypes = [C.c_int]
    L.hpc_register_weight.restype = C.c_int
    L.hpc_register_weight.argtypes = [vp, C.c_int, i64, i64, C.c_size_t]
    L.hpc_last_error.restype = C.c_int
    L.hpc_last_error.argtypes = [C.c_char_p, C.c_size_t]
    L.hpc_set_error_mode.argtypes = [C.c_int]
    L.hpc_weight_cache_entries.restype = C.c_int
    L.hpc_set_matvec_ks.argtypes = [C.c_int]
    L.hpc_set_gemm_x4.argtypes = [C.c_int]
    L.hpc_set_gemm_x4.restype = None
    L.gemma_engine_debug_step.restype = C.c_int
    L.gemma_engine_debug_step.argtypes = [vp, vp, vp]
    L.gemma_engine_stamp_step.restype = C.c_int
    L.gemma_engine_stamp_step.argtypes = [vp, C.c_int, vp]
    L.gemma_tp_unique_id.restype = C.c_int
    L.gemma_tp_unique_id.argtypes = [vp, C.c_int]
    L.gemma_engine_create_tp.restype = vp
    L.gemma_engine_create_tp.argtypes = [C.POINTER(GemmaConfig), C.c_int, C.c_int, C.c_int, vp]
    L.gemma_engine_create_tp2.restype = vp
    L.gemma_engine_create_tp2.argtypes = [C.POINTER(GemmaConfig), C.c_int, C.c_int, C.c_int, vp, C.c_int]
    L.gemma_engine_tp_flags.restype = C.c_int
    L.gemma_engine_tp_flags.argtypes = [vp]
    L.gemma_engine_p2p_handle.restype = C.c_int
    L.gemma_engine_p2p_handle.argtypes = [vp, vp, C.c_int]
    L.gemma_engine_p2p_open.restype = C.c_int
    L.gemma_engine_p2p_open.argtypes = [vp, vp, C.c_int]
    L.gemma_engine_p2p_err.restype = C.c_int
    L.gemma_engine_p2p_err.argtypes = [vp, C.c_int]
    L.gemma_engine_create.restype = vp
    L.gemma_engine_create.argtypes = [C.POINTER(GemmaConfig), C.c_int]
    L.gemma_engine_free.argtypes = [vp]
    L.gemma_engine_begin.restype = C.c_int
    L.gemma_engine_begin.argtypes = [vp, vp, C.c_int]
    L.gemma_engine_step.restype = C.c_int
    L.gemma_engine_step.argtypes = [vp, C.c_int, vp, C.c_int]
    L.gemma_engine_tokens.restype = C.c_int
    L.gemma_engine_tokens.argtypes = [vp, vp, C.c_int]
    L.gemma_engine_pos.restype = C.c_int
    L.gemma_engine_pos.argtypes = [vp]
    L.gemma_engine_prefill.restype = C.c_int
    L.gemma_engine_prefill.argtypes = [vp, vp, vp]
    L.gemma_engine_prefill_fast.restype = C.c_int
    L.gemma_engine_prefill_fast.argtypes = [vp, vp, vp]
    L.gemma_engine_prefill_taps.restype = C.c_int
    L.gemma_engine_prefill_taps.argtypes = [vp, vp, C.c_int]
    L.gemma_engine_tensor.restype = C.c_int64
    L.gemma_engine_tensor.argtypes = [vp, C.c_int, vp, i64]
    L.gemma_engine_tune.argtypes = [vp, C.c_int]
    L.gemma_engine_plan.argtypes = [vp, C.POINTER(C.c_int), C.c_int]
    L.gemma_engine_set_plan.argtypes = [vp, C.POINTER(C.c_int), C.c_int]
    L.gemma_engine_set_fuse.argtypes = [vp, C.c_int]
    L.gemma_engine_set_att_o.argtypes = [vp, C.c_int]
    L.gemma_engine_set_option.restype = C.c_int
    L.gemma_engine_set_option.argtypes = [vp, C.c_char_p, C.c_int]
    L.gemma_engine_set_persist.argtypes = [vp, C.c_int]
    L.gemma_engine_persist_err.argtypes = [vp, vp, C.c_int]
    L.gemma_engine_set_persist_timeout.argtypes = [vp, C.c_uint]
    L.gemma_engine_tp_info.argtypes = [vp, vp]
    L.gemma_engine_graph_kernels.argtypes = [vp]
    L.gemma_engine_time.restype = C.c_double
    L.gemma_engine_time.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_double)]
    L.gemma_kq_time.restype = C.c_double
    L.gemma_kq_time.argtypes = [C.c_int, i64, i64, C.c_int, C.POINTER(C.c_double)]
    L.gemma_hbm_read_gbs.restype = C.c_double
    L.gemma_hbm_read_gbs.argtypes = [C.c_int, C.c_size_t, C.c_int]
    L.gemma_hbm_read_probe.restype = C.c_double
    L.gemma_hbm_read_probe.argtypes = [C.c_int, C.c_size_t, C.c_int, C.c_int]
    L.gemma_engine_sync.restype = C.c_int
    L.gemma_engine_sync.argtypes = [vp]
    L.gemma_engine_create_from_gguf.restype = vp
    L.gemma_engine_create_from_gguf.argtypes = [C.c_char_p, C.c_int, C.c_int]
    L.gemma_engine_config.restype = C.c_int
    L.gemma_engine_config.argtypes = [vp, C.POINTER(GemmaConfig)]
    # GGUF reader (include/ggml.h)
    L.gguf_init_from_file.restype = vp
    L.gguf_init_from_file.argtypes = [C.c_char_p, GGUFInitParams]
    L.gguf_free.argtypes = [vp]
    for fn in ("gguf_get_n_kv", "gguf_get_n_tensors", "gguf_get_version"):
        getattr(L, fn).restype = C.c_int
        getattr(L, fn).argtypes = [vp]
    for fn in ("gguf_get_alignment", "gguf_get_data_offset"):
        getattr(L, fn).restype = C.c_size_t
        getattr(L, fn).argtypes = [vp]
    for fn, rt in (("gguf_get_key", C.c_char_p), ("gguf_get_kv_type", C.c_int), ("gguf_get_arr_type", C.c_int),
                   ("gguf_get_arr_n", C.c_int), ("gguf_get_arr_data", vp), ("gguf_get_val_str", C.c_char_p),
                   ("gguf_get_val_data", vp), ("gguf_get_tensor_name", C.c_char_p),
                   ("gguf_get_tensor_type", C.c_int), ("gguf_get_tensor_offset", C.c_size_t)):
        getattr(L, fn).restype = rt
        getattr(L, fn).argtypes = [vp, C.c_int]
    L.gguf_get_arr_str.restype = C.c_char_p
    L.gguf_get_arr_str.argtypes = [vp, C.c_int, C.c_int]
    L.gguf_find_key.restype = C.c_int
    L.gguf_find_key.argtypes = [vp, C.c_char_p]
    L.gguf_find_tensor.restype = C.c_int
    L.gguf_find_tensor.argtypes = [vp, C.c_char_p]
    L.ggml_get_tensor.restype = C.POINTER(GgmlTensor)
    L.ggml_get_tensor.argtypes = [vp, C.c_char_p]
    L.ggml_nbytes.restype = C.c_size_t
    L.ggml_nbytes.argtypes = [C.POINTER(GgmlTensor)]
    L.ggml_free.restype = None
    L.ggml_free.argtypes = [vp]
    _lib = L
    return L


def last_error():
    buf = C.create_string_buffer(1024)
    lib().hpc_last_error(buf, 1024)
    return buf.value.decode()


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def mul_mat(src0_bytes, src0_type, ne01, nb01, shared_edge, wdata, row_size, ncols, ne1=None, nb1=None, nb2=None):
    """Call the drop-in `mul_mat` (src/hpc.h:22-32 signature) on host buffers; returns dst [ncols][ne01]."""
    L = lib()
    ne1 = ncols if ne1 is None else ne1
    nb1 = ne01 * 4 if nb1 is None else nb1
    nb2 = nb1 * ne1 if nb2 is None else nb2
    ne12 = ncols // ne1
    span = max((c % ne1) * nb1 + (c // ne1) * nb2 for c in range(ncols)) + ne01 * 4
    raw = np.zeros((span + 3) // 4, dtype=np.float32)
    dst = raw
    t0, t1 = GgmlTensor(), GgmlTensor()
    t0.data = src0_bytes.ctypes.data
    t0.type = src0_type
    t1.data = dst.ctypes.data
    t1.type = GGML_TYPE_F32
    L.mul_mat(ne01, ne1, ne12, nb01, ne1, nb1, nb2, row_size, shared_edge, C.byref(t0), None, C.byref(t1), None,
              src0_type, _p(wdata))
    out = np.empty((ncols, ne01), dtype=np.float32)
    for c in range(ncols):
        off = ((c % ne1) * nb1 + (c // ne1) * nb2) // 4
        out[c] = raw[off:off + ne01]
    return out


class Engine:
    def __init__(self, shape, n_ctx=512, wtype=GGML_TYPE_Q4_0, seed=0x6E6D6D61, eps=1e-6, rope_base=10000.0,
                 gelu_clamp=0, device=0, tp=None, out_type=0, out_gain=0.0, tp_flags=0):
        """tp = (n_ranks, rank, rccl_id_bytes) for the row-split engine (one process per GPU);
        rccl_id_bytes None = all ranks' shards virtual in this engine (single-GPU parity mode).
        tp_flags: TP_REP_ATTN keeps the attention block (Wq|Wk|Wv, Wo) whole on every rank."""
        self.cfg = GemmaConfig(n_ctx=n_ctx, wtype=wtype, eps=eps, rope_base=rope_base, seed=seed,
                               gelu_clamp=gelu_clamp, out_type=out_type, out_gain=out_gain, **shape)
        self.L = lib()
        if tp is not None and (tp[0] > 1 or tp[2] is not None):  # n_ranks 1 + id: a 1-rank RCCL comm
            idbuf = C.create_string_buffer(bytes(tp[2]), len(tp[2])) if tp[2] is not None else None
            self.h = self.L.gemma_engine_create_tp2(C.byref(self.cfg), device, tp[0], tp[1], idbuf, tp_flags)
        else:
            self.h = self.L.gemma_engine_create(C.byref(self.cfg), device)
        if not self.h:
            raise RuntimeError("gemma_engine_create failed: " + last_error())

    @classmethod
    def from_gguf(cls, path, n_ctx=512, device=0):
        """An engine on a Gemma GGUF file's weights (gemma_engine_create_from_gguf)."""
        self = cls.__new__(cls)
        self.L = lib()
        self.h = self.L.gemma_engine_create_from_gguf(path.encode(), n_ctx, device)
        if not self.h:
            raise RuntimeError("gemma_engine_create_from_gguf failed: " + last_error())
        self.cfg = GemmaConfig()
        self.L.gemma_engine_config(self.h, C.byref(self.cfg))
        return self

    def close(self):
        if self.h:
            self.L.gemma_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, r, what):
        if r != 0:
            raise RuntimeError(f"{what} failed: {last_error()}")

    def begin(self, prompt):
        p = np.ascontiguousarray(prompt, dtype=np.int32)
        self._chk(self.L.gemma_engine_begin(self.h, _p(p), len(p)), "begin")

    def step(self, n, want_logits=False, use_graph=True):
        lg = np.zeros((n, self.cfg.n_vocab), dtype=np.float32) if want_logits else None
        self._chk(self.L.gemma_engine_step(self.h, n, _p(lg) if want_logits else None, 1 if use_graph else 0), "step")
        return lg

    def sync(self):
        """wait for the engine's stream"""
        self._chk(self.L.gemma_engine_sync(self.h), "sync")

    def tokens(self):
        out = np.zeros(self.cfg.n_ctx + 1, dtype=np.int32)
        n = self.L.gemma_engine_tokens(self.h, _p(out), len(out))
        return out[:n]

    def prefill(self, n_prompt=None, want_all=False, exact=True):
        """Batched prefill of the prompt given to begin(); returns (token, last-row logits[, all rows]).
        exact=True: bit-identical to the CPU path; False: the MFMA tolerance path."""
        last = np.zeros(self.cfg.n_vocab, dtype=np.float32)
        allv = np.zeros((n_prompt, self.cfg.n_vocab), dtype=np.float32) if want_all else None
        fn = self.L.gemma_engine_prefill if exact else self.L.gemma_engine_prefill_fast
        tok = fn(self.h, _p(last), _p(allv) if want_all else None)
        if tok < 0:
            raise RuntimeError("prefill failed: " + last_error())
        return (tok, last, allv) if want_all else (tok, last)

    def tensor(self, tid, nbytes):
        out = np.zeros(nbytes, dtype=np.uint8)
        n = self.L.gemma_engine_tensor(self.h, tid, _p(out), nbytes)
        if n < 0:
            raise RuntimeError("tensor failed: " + last_error())
        return out[:n]

    def stamp_step(self, layer):
        """Diagnostics: one eager step; returns u64 stamps [6 regions][4096 workgroups][16 phases]."""
        out = np.zeros(6 * 4096 * 16, dtype=np.uint64)
        self._chk(self.L.gemma_engine_stamp_step(self.h, layer, _p(out)), "stamp_step")
        return out.reshape(6, 4096, 16)

    PLAN_CLASSES = ("qkv", "attn_out", "gate_up", "down", "logits")

    def tune(self, iters=8):
        """measure the launch plan (clobbers the decode state: begin() afterwards); returns it"""
        if self.L.gemma_engine_tune(self.h, iters) != 0:
            raise RuntimeError("tune failed: " + last_error())
        return self.plan()

    def plan(self):
        """{class: (k_split, rows_per_wg, image)} plus "attention": form (0 per head, 1 split)"""
        buf = (C.c_int * 16)()
        n = self.L.gemma_engine_plan(self.h, buf, 16)
        p = {k: (buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i, k in enumerate(self.PLAN_CLASSES[: n // 3])}
        if n > 15:
            p["attention"] = buf[15]
        return p

    def set_plan(self, plan):
        flat = []
        for k in self.PLAN_CLASSES:
            v = list(plan[k])
            flat += v + [0] * (3 - len(v))
        if "attention" in plan:
            flat.append(int(plan["attention"]))
        arr = (C.c_int * len(flat))(*flat)
        if self.L.gemma_engine_set_plan(self.h, arr, len(flat)) != 0:
            raise RuntimeError("set_plan failed: " + last_error())

    def set_fuse(self, front=-1):
        """fused layer front on (1) / off (0) / unchanged (-1); returns the sticky hand-off timeout
        word (0 = every in-launch hand-off completed in time)"""
        return self.L.gemma_engine_set_fuse(self.h, front)

    def set_option(self, name, value):
        """a selectable variant (include/gemma_hpc.h gemma_engine_set_option); drops the decode graph"""
        self._chk(self.L.gemma_engine_set_option(self.h, name.encode(), int(value)), f"set_option({name})")

    def set_att_o(self, on=-1):
        """decode attention + attn-out in one launch per layer: on 1 / off 0 / keep -1; returns the setting"""
        return self.L.gemma_engine_set_att_o(self.h, on) == 1

    def set_persist(self, on=-1):
        """The decode step's layers as one persistent launch (token.hip): on 1/0, -1 keep; returns
        True when it runs this engine's steps."""
        return self.L.gemma_engine_set_persist(self.h, on) == 1

    def set_persist_timeout(self, ticks):
        """the persistent launch's per-wait bound in 100 MHz ticks (0 = default; tests force timeouts)"""
        return self.L.gemma_engine_set_persist_timeout(self.h, ticks)

    def p2p_handle(self):
        """this rank's inbox arena as IPC handle bytes (GEMMA_TP_P2P engines)"""
        buf = C.create_string_buffer(128)
        n = self.L.gemma_engine_p2p_handle(self.h, buf, 128)
        if n <= 0:
            raise RuntimeError("gemma_engine_p2p_handle: " + last_error())
        return buf.raw[:n]

    def p2p_open(self, handles):
        """every rank's handle (rank order); then a host barrier before the first step"""
        raw = b"".join(handles)
        if self.L.gemma_engine_p2p_open(self.h, C.create_string_buffer(raw, len(raw)), len(handles)) != 0:
            raise RuntimeError("gemma_engine_p2p_open: " + last_error())

    def p2p_err(self, reset=False):
        """the sticky flag-wait timeout word of the p2p gathers"""
        return self.L.gemma_engine_p2p_err(self.h, 1 if reset else 0)

    def tp_flags(self):
        """layout flags of a row-split engine (TP_REP_ATTN)"""
        return self.L.gemma_engine_tp_flags(self.h)

    def tp_info(self):
        """[ranks, rank, RCCL communicator present, shard slots in this engine]"""
        out = (C.c_int * 4)()
        self.L.gemma_engine_tp_info(self.h, out)
        return list(out)

    def persist_err(self, reset=False):
        """Sticky hand-off timeout words [flag, site, layer] of the persistent launch."""
        out = (C.c_int * 3)()
        self.L.gemma_engine_persist_err(self.h, out, 1 if reset else 0)
        return list(out)

    def graph_kernels(self):
        """kernel launches per decode token (the captured decode graph's kernel nodes)"""
        n = self.L.gemma_engine_graph_kernels(self.h)
        if n < 0:
            raise RuntimeError("graph_kernels failed: " + last_error())
        return n

    def time_kernel(self, which, iters):
        b = C.c_double()
        us = self.L.gemma_engine_time(self.h, which, iters, C.byref(b))
        if us < 0:
            raise RuntimeError("time failed: " + last_error())
        return us, b.value


def tp_unique_id():
    """RCCL unique id for gemma_engine_create_tp (call on rank 0, broadcast the bytes)."""
    buf = C.create_string_buffer(256)
    n = lib().gemma_tp_unique_id(buf, 256)
    if n <= 0:
        raise RuntimeError("gemma_tp_unique_id failed: " + last_error())
    return buf.raw[:n]


_GGUF_SCALAR = {0: C.c_uint8, 1: C.c_int8, 2: C.c_uint16, 3: C.c_int16, 4: C.c_uint32, 5: C.c_int32, 6: C.c_float,
                7: C.c_bool, 10: C.c_uint64, 11: C.c_int64, 12: C.c_double}


class GGUF:
    """A GGUF file read by the library's gguf_init_from_file (include/ggml.h): `kv` maps keys to
    values (scalars, str, lists), `tensors` maps names to (ggml type, ne, bytes) when load_tensors."""

    def __init__(self, path, load_tensors=True):
        L = lib()
        ctx = C.c_void_p()
        self.g = L.gguf_init_from_file(path.encode(), GGUFInitParams(not load_tensors, C.pointer(ctx)))
        if not self.g:
            raise ValueError(last_error())
        self.version = L.gguf_get_version(self.g)
        self.alignment = L.gguf_get_alignment(self.g)
        self.data_offset = L.gguf_get_data_offset(self.g)
        self.kv = {}
        for i in range(L.gguf_get_n_kv(self.g)):
            key = L.gguf_get_key(self.g, i).decode()
            t = L.gguf_get_kv_type(self.g, i)
            if t == 8:
                v = L.gguf_get_val_str(self.g, i).decode()
            elif t == 9:
                at, n = L.gguf_get_arr_type(self.g, i), L.gguf_get_arr_n(self.g, i)
                if at == 8:
                    v = [L.gguf_get_arr_str(self.g, i, j).decode() for j in range(n)]
                else:
                    ct = _GGUF_SCALAR[at]
                    v = list((ct * n).from_address(L.gguf_get_arr_data(self.g, i))) if n else []
            else:
                v = _GGUF_SCALAR[t].from_address(L.gguf_get_val_data(self.g, i)).value
            self.kv[key] = v
        self.tensors = {}
        for i in range(L.gguf_get_n_tensors(self.g)):
            name = L.gguf_get_tensor_name(self.g, i)
            t = L.ggml_get_tensor(ctx, name)
            data = None
            if load_tensors:
                data = C.string_at(t.contents.data, L.ggml_nbytes(t))
            self.tensors[name.decode()] = (L.gguf_get_tensor_type(self.g, i), tuple(t.contents.ne), data,
                                           L.gguf_get_tensor_offset(self.g, i))
        L.ggml_free(ctx)
        L.gguf_free(self.g)
        self.g = None
