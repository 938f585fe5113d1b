"""The decode engine on llama.cpp-layout weights (SURVEY §8(f) rank 3 and the Q6_K output that
SURVEY §8 notes for real Q4_0 files): a Q6_K token_embd / tied output (embedding dequantized on the
device, logits through Q8_K INIT + the K-quant matvec + row argmax), and engines loaded from GGUF
files (gemma_engine_create_from_gguf).  Tokens and every logit bit-identical to the CPU oracle
(kmix = 2: Q4_0 / Q8_0 layers, Q6_K token_embd)."""
import numpy as np
import pytest

import gemma_hip as G
import oracle_ctypes as O
from test_gpu_ggml_graph import write_gguf

gpu = pytest.mark.gpu
SMALL = dict(n_layer=2, n_embd=512, n_head=2, n_head_kv=1, head_dim=256, n_ff=1024, n_vocab=2048)


def _compare(e, m, shape, n_prompt, n_decode):
    prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    seq_ref, lg_ref = m.generate(prompt, n_decode)
    e.begin(prompt)
    lg = e.step(n_prompt + n_decode, want_logits=True)
    assert list(e.tokens()[: len(seq_ref)]) == list(seq_ref)
    got = lg[n_prompt - 1:]
    bad = np.argwhere(got.view(np.uint32) != lg_ref.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} logits differ, first {bad[:5]}"
    return prompt


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_0, O.Q8_0])
def test_synthetic_q6K_output_matches_oracle(wtype):
    m = O.Model(O.make_config(SMALL, n_ctx=128, wtype=wtype, kmix=2))
    e = G.Engine(SMALL, n_ctx=128, wtype=wtype, out_type=G.GGML_TYPE_Q6_K)
    ref = m.tensor(0)  # Q6_K token_embd generated on the device == the oracle's bytes
    assert np.array_equal(e.tensor(0, ref.size), ref)
    _compare(e, m, SMALL, 9, 20)
    e.close()
    m.close()


@gpu
def test_q6K_output_gemma2b_shapes():
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=16384)
    m = O.Model(O.make_config(shape, n_ctx=256, kmix=2))
    e = G.Engine(shape, n_ctx=256, out_type=G.GGML_TYPE_Q6_K)
    _compare(e, m, shape, 17, 6)
    e.close()
    m.close()


@gpu
def test_q6K_output_exact_prefill():
    m = O.Model(O.make_config(SMALL, n_ctx=128, kmix=2))
    e = G.Engine(SMALL, n_ctx=128, out_type=G.GGML_TYPE_Q6_K)
    prompt = O.make_prompt(45, SMALL["n_vocab"])
    m.reset()
    tok_ref, _, all_ref = m.inference(prompt, 0, want_all=True)
    e.begin(prompt)
    tok, last, allv = e.prefill(len(prompt), want_all=True)
    assert tok == tok_ref
    assert np.array_equal(allv.view(np.uint32), all_ref.view(np.uint32))
    # decode continues from the KV cache the prefill wrote
    seq = list(prompt) + [tok]
    lg = e.step(3, want_logits=True)
    for i in range(3):
        t, ref, _ = m.inference(seq, 1)
        assert np.array_equal(lg[i].view(np.uint32), ref.view(np.uint32))
        seq.append(t)
    e.close()
    m.close()


@gpu
@pytest.mark.parametrize("wtype,kmix", [(O.Q4_0, 0), (O.Q4_0, 2), (O.Q8_0, 2)])
def test_engine_from_gguf(tmp_path, wtype, kmix):
    shape = dict(SMALL, n_head=4, n_head_kv=2, head_dim=128)
    m = O.Model(O.make_config(shape, n_ctx=128, wtype=wtype, kmix=kmix))
    path = tmp_path / "m.gguf"
    if kmix == 2:  # token_embd is Q6_K in this layout
        write_gguf_q6k(m, shape, path)
    else:
        write_gguf(m, shape, path, 0)
    e = G.Engine.from_gguf(str(path), n_ctx=128)
    for k in ("n_layer", "n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab"):
        assert getattr(e.cfg, k) == shape[k], k
    assert e.cfg.wtype == wtype and e.cfg.out_type == (G.GGML_TYPE_Q6_K if kmix == 2 else 0)
    _compare(e, m, shape, 11, 10)
    e.close()
    m.close()


def write_gguf_q6k(m, shape, path):
    """write_gguf with token_embd typed Q6_K (the oracle's kmix = 2 bytes) and wtype layers."""
    import test_gpu_ggml_graph as T
    orig = T.GGUFWriter.add_tensor

    def add_tensor(self, name, t, ne, data):
        return orig(self, name, O.Q6_K if name == "token_embd.weight" else t, ne, data)
    T.GGUFWriter.add_tensor = add_tensor
    try:
        T.write_gguf(m, shape, path, 0)
    finally:
        T.GGUFWriter.add_tensor = orig


# ---- K-quant layers (llama.cpp Q4_K_M layout: Q4_K q/k/o/gate/up, Q6_K v/down/token_embd) ----------
KSHAPE = dict(n_layer=2, n_embd=256, n_head=2, n_head_kv=1, head_dim=128, n_ff=512, n_vocab=1024)


@gpu
def test_kquant_engine_synthetic_matches_oracle():
    m = O.Model(O.make_config(KSHAPE, n_ctx=128, kmix=1))
    e = G.Engine(KSHAPE, n_ctx=128, wtype=G.GGML_TYPE_Q4_K)
    for tid in [0, 1] + [16 + il * 16 + k for il in range(2) for k in range(9)]:
        ref = m.tensor(tid)
        assert np.array_equal(e.tensor(tid, ref.size), ref), tid
    _compare(e, m, KSHAPE, 7, 16)
    with pytest.raises(RuntimeError):  # the approximate MFMA prefill is Q4_0 / Q8_0 only
        e.begin(O.make_prompt(5, KSHAPE["n_vocab"]))
        e.prefill(5, exact=False)
    e.close()
    m.close()


def _prefill_compare(e, m, shape, n_prompt, n_decode):
    prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    m.reset()
    tok_ref, _, all_ref = m.inference(prompt, 0, want_all=True)
    e.begin(prompt)
    tok, last, allv = e.prefill(len(prompt), want_all=True)
    assert tok == tok_ref
    bad = np.argwhere(allv.view(np.uint32) != all_ref.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} prefill logits differ, first {bad[:5]}"
    # decode continues from the KV cache the batched prefill wrote
    seq = list(prompt) + [tok]
    lg = e.step(n_decode, want_logits=True)
    for i in range(n_decode):
        t, ref, _ = m.inference(seq, 1)
        assert np.array_equal(lg[i].view(np.uint32), ref.view(np.uint32)), i
        seq.append(t)


@gpu
@pytest.mark.parametrize("n_prompt", [1, 7, 33, 64, 100])
def test_kquant_engine_batched_prefill_matches_oracle(n_prompt):
    # every prompt row's logits of the batched K-quant prefill (all T columns per launch) equal the
    # CPU path's, and decode continues bit-exactly from its KV cache
    m = O.Model(O.make_config(KSHAPE, n_ctx=128, kmix=1))
    e = G.Engine(KSHAPE, n_ctx=128, wtype=G.GGML_TYPE_Q4_K)
    _prefill_compare(e, m, KSHAPE, n_prompt, 3)
    e.close()
    m.close()


@gpu
@pytest.mark.parametrize("mfma", [1, 0])
def test_kquant_engine_batched_prefill_gemma2b_layer_shapes(mfma):
    # mfma = 1: the lane-tiled Q4_K / Q6_K matrices through the MFMA GEMM (prefill_kq.hip), = 0: the
    # dot4 T-column kernel
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=8192)
    m = O.Model(O.make_config(shape, n_ctx=256, kmix=1))
    e = G.Engine(shape, n_ctx=256, wtype=G.GGML_TYPE_Q4_K)
    G.lib().hpc_set_kq_gemm_min(-1 if mfma else 1 << 30)
    try:
        _prefill_compare(e, m, shape, 40, 2)
    finally:
        G.lib().hpc_set_kq_gemm_min(-1)
    e.close()
    m.close()


@gpu
@pytest.mark.parametrize("fuse,dual,pair", [(5, 1, 1), (5, 0, 0), (6, 1, 1), (3, 1, 1), (3, 1, 0), (3, 0, 1),
                                           (4, 1, 1), (2, 1, 1), (1, 1, 1), (0, 0, 0)])
def test_kquant_engine_gemma2b_layer_shapes(fuse, dual, pair):
    # fuse: the Q8_K INIT plan (enqueue_step_kq; 5 default) — 3 norms in prologues + quantizations handed off,
    # 2 the producer tails (hand-off), 1 the consumer prologues,
    # 0 separate norm / quantize launches; dual: gate and up in one launch; pair: q|k and v in one launch
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=8192)
    m = O.Model(O.make_config(shape, n_ctx=256, kmix=1))
    e = G.Engine(shape, n_ctx=256, wtype=G.GGML_TYPE_Q4_K)
    e.set_option("kq_fuse", fuse)
    e.set_option("kq_dual", dual)
    e.set_option("kq_pair", pair)
    _compare(e, m, shape, 13, 6)
    e.close()
    m.close()


@gpu
def test_kquant_engine_from_gguf(tmp_path):
    m = O.Model(O.make_config(KSHAPE, n_ctx=128, kmix=1))
    path = tmp_path / "k.gguf"
    write_gguf(m, KSHAPE, path, 1)
    e = G.Engine.from_gguf(str(path), n_ctx=128)
    assert e.cfg.wtype == G.GGML_TYPE_Q4_K
    _compare(e, m, KSHAPE, 9, 12)
    e.close()
    m.close()
