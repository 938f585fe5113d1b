"""Timing of the ggml-API drop-in path: the reference's graph code restated against
include/ggml.h (tests/ggml_driver/gemma_graph_driver) on a full Gemma-2B Q4_0 GGUF file written from
the engine's synthetic weights, prefill of a 128-token prompt then greedy decode through
ggml_graph_compute_with_ctx, as src/gemma_model.cpp:548-575 times it.
usage: python scripts/ggml_path_bench.py [n_decode] [out_dir]"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402
from gguf_writer import ARR, F32, STR, U32, GGUFWriter  # noqa: E402

n_decode = int(sys.argv[1]) if len(sys.argv) > 1 else 32
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "ggml_path")
os.makedirs(out, exist_ok=True)
S = GEMMA_2B
E, V, F, L = S["n_embd"], S["n_vocab"], S["n_ff"], S["n_layer"]
qw, kvw = S["n_head"] * S["head_dim"], S["n_head_kv"] * S["head_dim"]
t0 = time.time()
e = G.Engine(S, n_ctx=512)
q4 = lambda rows, k: rows * k // 32 * 18  # noqa: E731
w = GGUFWriter()
w.add("general.architecture", STR, "gemma")
for key, v in (("block_count", L), ("embedding_length", E), ("feed_forward_length", F), ("context_length", 8192),
               ("attention.head_count", S["n_head"]), ("attention.head_count_kv", S["n_head_kv"]),
               ("attention.key_length", S["head_dim"]), ("attention.value_length", S["head_dim"])):
    w.add("gemma." + key, U32, v)
w.add("gemma.attention.layer_norm_rms_epsilon", F32, 1e-6)
w.add("tokenizer.ggml.tokens", ARR, ["<pad>", "<eos>", "<bos>"] + ["▁t%d" % i for i in range(3, V)], STR)
for k, v in (("bos", 2), ("eos", 1), ("unknown", 3), ("padding", 0)):
    w.add(f"tokenizer.ggml.{k}_token_id", U32, v)
w.add_tensor("token_embd.weight", 2, [E, V], e.tensor(0, q4(V, E)))
w.add_tensor("output_norm.weight", 0, [E], e.tensor(1, E * 4))
names = [("attn_norm", 0, [E], E * 4), ("attn_q", 2, [E, qw], q4(qw, E)), ("attn_k", 2, [E, kvw], q4(kvw, E)),
         ("attn_v", 2, [E, kvw], q4(kvw, E)), ("attn_output", 2, [qw, E], q4(E, qw)), ("ffn_norm", 0, [E], E * 4),
         ("ffn_gate", 2, [E, F], q4(F, E)), ("ffn_up", 2, [E, F], q4(F, E)), ("ffn_down", 2, [F, E], q4(E, F))]
for il in range(L):
    for k, (nm, t, ne, nb) in enumerate(names):
        w.add_tensor(f"blk.{il}.{nm}.weight", t, ne, e.tensor(16 + il * 16 + k, nb))
e.close()
path = os.path.join(out, "gemma2b_q4_0.gguf")
w.write(path)
del w
prompt = np.array(make_prompt(128, V), dtype=np.int32)
prompt.tofile(os.path.join(out, "prompt.bin"))
print(f"gguf written ({os.path.getsize(path) / 1e9:.2f} GB, {time.time() - t0:.1f} s)", flush=True)
if os.environ.get("GGML_PATH_WRITE_ONLY"):  # keep the file for an external (profiled) driver run
    sys.exit(0)
drv = os.path.join(ROOT, "tests", "ggml_driver", "gemma_graph_driver")
# logits rows not written out per step (not part of the reference loop); two rounds of the reference's
# begin_one_round_inference on the loaded model: the second round's prefill is compute only
env = dict(os.environ, DRIVER_BENCH="1", DRIVER_ROUNDS=os.environ.get("DRIVER_ROUNDS", "2"))
r = subprocess.run([drv, path, os.path.join(out, "prompt.bin"), os.path.join(out, "o.bin"), "512", str(n_decode)],
                   capture_output=True, text=True, timeout=900, env=env)
open(os.path.join(out, "driver.err"), "w").write(r.stderr)
print(r.stderr.strip().splitlines()[-1] if r.stderr.strip() else "", flush=True)
os.remove(path)
sys.exit(r.returncode)
