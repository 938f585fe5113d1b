"""Generates tests/golden/hf_wiring_tiny.npz — the FLOAT graph-wiring fixture for the oracle.

Test infrastructure only (run in the build container; the GPU box never runs it).  The oracle's
synthetic weights (dequantized from its Q8_0 tensors) are loaded into a locally constructed
`transformers` GemmaForCausalLM (GemmaConfig built here, nothing downloaded) and its float
forward pass over a synthetic prompt is recorded.  tests/test_oracle_kat.py then checks the
oracle's own quantized forward pass (ggml semantics: Q8_0 activations, fp16 tables) against these
logits within a tolerance that covers activation quantization: this pins the wiring of
src/gemma_model.cpp:665-747 (embedding scale, RMSNorm placement and the GGUF '+1' norm weights,
RoPE-NEOX pairs, MQA grouping, q scaling, GeGLU-tanh, residuals, tied output) to an independent
implementation.

usage: python tests/golden/make_hf_wiring_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ctypes as O  # noqa: E402

SHAPE = dict(n_layer=2, n_embd=256, n_head=4, n_head_kv=1, head_dim=64, n_ff=512, n_vocab=512)
T = 12


def dequant(m, tid, rows, cols):
    raw = m.tensor(tid).reshape(rows, cols // 32 * 34)
    L = O.lib()
    out = np.zeros((rows, cols), np.float32)
    for r in range(rows):
        L.orc_dequantize_row_q8_0(O.ptr(np.ascontiguousarray(raw[r])), O.ptr(out[r]), cols)
    return out


def f32(m, tid):
    return m.tensor(tid).view(np.float32).copy()


def main():
    from transformers import GemmaConfig, GemmaForCausalLM
    cfg = O.make_config(SHAPE, n_ctx=64, wtype=O.Q8_0)
    m = O.Model(cfg)
    E, H, Hkv, hd, F, V = (SHAPE[k] for k in ("n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab"))
    prompt = np.zeros(T, np.int32)
    O.lib().orc_make_prompt(1, T, V, O.ptr(prompt))

    hc = GemmaConfig(vocab_size=V, hidden_size=E, intermediate_size=F, num_hidden_layers=SHAPE["n_layer"],
                     num_attention_heads=H, num_key_value_heads=Hkv, head_dim=hd, hidden_act="gelu_pytorch_tanh",
                     hidden_activation="gelu_pytorch_tanh", max_position_embeddings=64, rms_norm_eps=1e-6,
                     rope_theta=10000.0, attention_bias=False, tie_word_embeddings=True)
    hc._attn_implementation = "eager"
    model = GemmaForCausalLM(hc).float().eval()
    sd = model.state_dict()
    sd["model.embed_tokens.weight"] = torch.from_numpy(dequant(m, 0, V, E))
    sd["model.norm.weight"] = torch.from_numpy(f32(m, 1) - 1.0)  # HF Gemma RMSNorm scales by (1 + w)
    for il in range(SHAPE["n_layer"]):
        t = lambda k: 16 + il * 16 + k  # noqa: E731  (tensor ids: DESIGN.md §Synthetic weights)
        p = f"model.layers.{il}."
        sd[p + "input_layernorm.weight"] = torch.from_numpy(f32(m, t(0)) - 1.0)
        sd[p + "self_attn.q_proj.weight"] = torch.from_numpy(dequant(m, t(1), H * hd, E))
        sd[p + "self_attn.k_proj.weight"] = torch.from_numpy(dequant(m, t(2), Hkv * hd, E))
        sd[p + "self_attn.v_proj.weight"] = torch.from_numpy(dequant(m, t(3), Hkv * hd, E))
        sd[p + "self_attn.o_proj.weight"] = torch.from_numpy(dequant(m, t(4), E, H * hd))
        sd[p + "post_attention_layernorm.weight"] = torch.from_numpy(f32(m, t(5)) - 1.0)
        sd[p + "mlp.gate_proj.weight"] = torch.from_numpy(dequant(m, t(6), F, E))
        sd[p + "mlp.up_proj.weight"] = torch.from_numpy(dequant(m, t(7), F, E))
        sd[p + "mlp.down_proj.weight"] = torch.from_numpy(dequant(m, t(8), E, F))
    if "lm_head.weight" in sd:
        sd["lm_head.weight"] = sd["model.embed_tokens.weight"]
    model.load_state_dict(sd)
    with torch.no_grad():
        logits = model(torch.from_numpy(prompt.astype(np.int64))[None]).logits[0].numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "hf_wiring_tiny.npz"), prompt=prompt, logits=logits,
                        shape=np.array([SHAPE[k] for k in ("n_layer", "n_embd", "n_head", "n_head_kv", "head_dim",
                                                             "n_ff", "n_vocab")], np.int64),
                        seed=np.array([cfg.seed], np.uint64))
    _, _, ours = m.inference(prompt, 0, want_all=True)
    d = np.abs(ours - logits)
    print("max|diff|", d.max(), "logit std", logits.std(), "argmax agree", (ours.argmax(1) == logits.argmax(1)).mean(),
          "min row corr", min(np.corrcoef(ours[i], logits[i])[0, 1] for i in range(T)))


if __name__ == "__main__":
    main()
