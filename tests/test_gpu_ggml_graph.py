"""The ggml operator surface: the reference's graph code restated against
include/ggml.h (tests/ggml_driver/gemma_graph_driver.cpp, same API calls as src/gemma_model.cpp)
runs on the MI355X graph executor, and its logits — prefill (last row) and every decode step — and
greedy tokens are bit-identical to the CPU oracle.

The GGUF cases write the oracle's model as a GGUF file (tests/gguf_writer.py: the tensor names and
metadata keys src/gemma_model.cpp:145-214 / 403-415 read) and the driver loads it the way
load_model_from_file does (gguf_init_from_file into a weight context).  The K-quant mix (Q4_K and
Q6_K matrices, Q6_K token_embd, as llama.cpp's Q4_K_M files hold them) runs get_rows / mul_mat on
the K-quant kernels; parity is against the oracle's restatement (ggml absent: unpinned, §7)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_ctypes as O
from gguf_writer import ARR, F32, STR, U32, GGUFWriter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "ggml_driver", "gemma_graph_driver")
gpu = pytest.mark.gpu


def test_driver_built():
    assert os.path.exists(DRIVER), "make -C gemma.ggml_amd builds the ggml graph driver"


LAYER_TENSORS = ["attn_norm", "attn_q", "attn_k", "attn_v", "attn_output", "ffn_norm", "ffn_gate", "ffn_up",
                 "ffn_down"]  # oracle tensor ids 16 + 16*il + k, k = 0..8


def _token_text(i):
    return {0: "<pad>", 1: "<eos>", 2: "<bos>"}.get(i, "\u2581t%d" % i)


def write_gguf(m, shape, path, kmix):
    """The oracle's model as a Gemma GGUF file (ggml dims: ne[0] = row length)."""
    E, V, F = shape["n_embd"], shape["n_vocab"], shape["n_ff"]
    qw, kvw = shape["n_head"] * shape["head_dim"], shape["n_head_kv"] * shape["head_dim"]
    wt = m.cfg.wtype
    kt = {"attn_q": O.Q4_K, "attn_k": O.Q4_K, "attn_v": O.Q6_K, "attn_output": O.Q4_K, "ffn_gate": O.Q4_K,
          "ffn_up": O.Q4_K, "ffn_down": O.Q6_K}
    dims = {"attn_norm": [E], "ffn_norm": [E], "attn_q": [E, qw], "attn_k": [E, kvw], "attn_v": [E, kvw],
            "attn_output": [qw, E], "ffn_gate": [E, F], "ffn_up": [E, F], "ffn_down": [F, E]}
    w = GGUFWriter()
    w.add("general.architecture", STR, "gemma")
    w.add("gemma.context_length", U32, 8192)
    w.add("gemma.embedding_length", U32, E)
    w.add("gemma.block_count", U32, shape["n_layer"])
    w.add("gemma.feed_forward_length", U32, F)
    w.add("gemma.attention.head_count", U32, shape["n_head"])
    w.add("gemma.attention.head_count_kv", U32, shape["n_head_kv"])
    w.add("gemma.attention.key_length", U32, shape["head_dim"])
    w.add("gemma.attention.value_length", U32, shape["head_dim"])
    w.add("gemma.attention.layer_norm_rms_epsilon", F32, 1e-6)
    w.add("tokenizer.ggml.model", STR, "llama")
    w.add("tokenizer.ggml.tokens", ARR, [_token_text(i) for i in range(V)], STR)
    w.add("tokenizer.ggml.scores", ARR, [0.0] * V, F32)
    w.add("tokenizer.ggml.token_type", ARR, [1] * V, 5)
    for k, v in (("bos", 2), ("eos", 1), ("unknown", 3), ("padding", 0)):
        w.add(f"tokenizer.ggml.{k}_token_id", U32, v)
    w.add_tensor("token_embd.weight", O.Q6_K if kmix else wt, [E, V], m.tensor(0))
    w.add_tensor("output_norm.weight", 0, [E], m.tensor(1))
    for il in range(shape["n_layer"]):
        for k, name in enumerate(LAYER_TENSORS):
            t = 0 if name.endswith("norm") else (kt[name] if kmix else wt)
            w.add_tensor(f"blk.{il}.{name}.weight", t, dims[name], m.tensor(16 + il * 16 + k))
    w.write(str(path))


def _write_weights(m, shape, path):
    with open(path, "wb") as f:
        f.write(m.tensor(0).tobytes())  # token_embd (also the tied output)
        f.write(m.tensor(1).tobytes())  # output_norm
        for il in range(shape["n_layer"]):
            for k in range(9):  # attn_norm q k v o ffn_norm gate up down
                f.write(m.tensor(16 + il * 16 + k).tobytes())


def _check_out(m, prompt, n_decode, V, opath):
    """the driver's logits rows and tokens against the oracle's inference() sequence"""
    raw = np.fromfile(opath, dtype=np.float32)
    logits = raw[: (n_decode + 1) * V].reshape(n_decode + 1, V)
    toks = raw[(n_decode + 1) * V:].view(np.int32)
    seq = list(prompt)
    t0, l0, _ = m.inference(seq, 0)
    refs, rtoks = [l0], [t0]
    seq.append(t0)
    for _ in range(n_decode):
        t, lg, _ = m.inference(seq, 1)
        refs.append(lg)
        rtoks.append(t)
        seq.append(t)
    for i, ref in enumerate(refs):
        assert np.array_equal(logits[i].view(np.uint32), ref.view(np.uint32)), (i, np.abs(logits[i] - ref).max())
    assert list(toks) == rtoks
    return seq


def _run(tmp_path, shape, wtype, n_prompt, n_decode, ctx, gguf=False, kmix=0, fast=1, second_seed=None, register=1,
         poke=None, prompt=None):
    """fast=1: the executor recognises the Gemma graph and runs the device-resident engine over the
    graph's weights and KV-cache mirrors (ggml_api.cpp try_fast); fast=0: node by node.
    second_seed: a second model of the same shapes (other weights) run after the first in the same
    driver process, whose pooled host arenas likely land at the first model's addresses.
    register (GGUF): the driver pre-uploads every quantized weight at load (hpc_register_weight) and
    the fast path's engine copies them device to device; 0: the engine uploads from the host."""
    m = O.Model(O.make_config(shape, n_ctx=ctx, wtype=wtype, kmix=kmix))
    if poke is not None:  # adversarial weights (tests/test_gpu_norm_exact.py), oracle and file alike
        poke(m)
    wpath, ppath, opath = tmp_path / ("m.gguf" if gguf else "w.bin"), tmp_path / "p.bin", tmp_path / "o.bin"
    if gguf:
        write_gguf(m, shape, wpath, kmix)
    else:
        _write_weights(m, shape, wpath)
    m2 = None
    if second_seed is not None:
        m2 = O.Model(O.make_config(shape, n_ctx=ctx, wtype=wtype, kmix=kmix, seed=second_seed))
        _write_weights(m2, shape, tmp_path / "w2.bin")
    if prompt is None:
        prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    prompt = np.array(prompt, dtype=np.int32)
    prompt.tofile(ppath)
    if gguf:
        args = [DRIVER, str(wpath), str(ppath), str(opath), str(ctx), str(n_decode)]
    else:
        args = [DRIVER, str(wpath), str(ppath), str(opath)] + [str(shape[k]) for k in
                ("n_layer", "n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab")] + [str(ctx), str(wtype),
                                                                                              str(n_decode)]
    env = dict(os.environ, GHIP_GGML_FAST=str(fast), GHIP_GGML_DEBUG="1", DRIVER_NO_REGISTER=str(1 - register))
    if m2 is not None:
        env["DRIVER_SECOND"] = str(tmp_path / "w2.bin")
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    if fast and not kmix:  # the Gemma graph must take the engine path (K-quant layers: node by node)
        assert "fast path not taken" not in r.stderr, r.stderr[-500:]
    # oracle: the reference's inference() sequence (PREFILL, then DECODE per token)
    V = shape["n_vocab"]
    seq = _check_out(m, prompt, n_decode, V, opath)
    m.close()
    if m2 is not None:
        _check_out(m2, prompt, n_decode, V, str(opath) + ".2")
        m2.close()
    if gguf:  # print_tokens through the GGUF tokenizer table
        want = "".join(_token_text(int(i)) for i in seq).replace("<bos>", "", 1).replace("\u2581", " ")
        assert open(str(opath) + ".txt", encoding="utf-8").read() == want


@gpu
@pytest.mark.parametrize("fast", [1, 0])
def test_ggml_graph_tiny_q4_0(tmp_path, fast):
    _run(tmp_path, dict(O.TINY), O.Q4_0, 20, 4, 128, fast=fast)


@gpu
@pytest.mark.parametrize("fast", [1, 0])
def test_ggml_graph_gqa_q8_0(tmp_path, fast):
    _run(tmp_path, dict(O.TINY, n_head=4, n_head_kv=2), O.Q8_0, 37, 3, 128, fast=fast)


@gpu
@pytest.mark.parametrize("fast", [1, 0])
def test_ggml_graph_gemma2b_layers(tmp_path, fast):
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=8192)
    _run(tmp_path, shape, O.Q4_0, 40, 2, 128, fast=fast)


@gpu
@pytest.mark.parametrize("fast", [1, 0])
@pytest.mark.parametrize("register", [1, 0])
def test_ggml_graph_gguf_q4_0(tmp_path, fast, register):
    _run(tmp_path, dict(O.TINY), O.Q4_0, 20, 4, 128, gguf=True, fast=fast, register=register)


@gpu
@pytest.mark.parametrize("fast", [1, 0])
def test_ggml_graph_gguf_kquant_mix_tiny(tmp_path, fast):
    shape = dict(n_layer=2, n_embd=256, n_head=2, n_head_kv=1, head_dim=128, n_ff=512, n_vocab=1024)
    _run(tmp_path, shape, O.Q4_0, 23, 4, 128, gguf=True, kmix=1, fast=fast)


@gpu
@pytest.mark.parametrize("fast", [1, 0])
def test_ggml_graph_gguf_kquant_mix_gemma2b_layers(tmp_path, fast):
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=8192)
    _run(tmp_path, shape, O.Q4_0, 33, 2, 128, gguf=True, kmix=1, fast=fast)


@gpu
def test_ggml_graph_two_models_one_process(tmp_path):
    """a second model of the same size in the same process: the fast path's engine (keyed by the
    graph's host weight addresses) must not serve the first model's device copy"""
    _run(tmp_path, dict(O.TINY), O.Q4_0, 12, 3, 128, fast=1, second_seed=0x1234567)
