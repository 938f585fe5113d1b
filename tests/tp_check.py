"""Row-split TP parity run: `torchrun --nproc-per-node N tests/tp_check.py [tiny|2b] [ngpus]`.

Each rank builds the row-split engine (RCCL id broadcast over gloo), decodes greedily, and rank 0
checks tokens and every step's gathered logits bit-for-bit against the CPU oracle (row split has
no cross-rank reduction, so the N-rank result must equal the 1-GPU one exactly)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gemma_hip as G  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "tiny"
ngpus = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = rank % ngpus
idt = torch.zeros(256, dtype=torch.uint8)
if rank == 0:
    raw = G.tp_unique_id()
    idt[: len(raw)] = torch.tensor(list(raw), dtype=torch.uint8)
dist.broadcast(idt, 0)
shape = dict(n_layer=2, n_embd=512, n_head=2, n_head_kv=1, head_dim=256, n_ff=2048, n_vocab=4096) if which == "tiny" \
    else dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
n_ctx = 128
e = G.Engine(shape, n_ctx=n_ctx, device=dev, tp=(world, rank, bytes(idt.numpy())))
import oracle_ctypes as O  # noqa: E402  (checker only)
prompt = O.make_prompt(6, shape["n_vocab"])
e.begin(prompt)
n_dec = 6
lg = e.step(len(prompt) + n_dec, want_logits=True, use_graph=True)
toks = list(e.tokens())
e.close()
if rank == 0:
    m = O.Model(O.make_config(shape, n_ctx=n_ctx))
    seq_ref, lg_ref = m.generate(prompt, n_dec)
    ok_t = toks[: len(seq_ref)] == list(seq_ref)
    got = lg[len(prompt) - 1:]
    ok_l = np.array_equal(got.view(np.uint32), lg_ref.view(np.uint32))
    print(f"TP world={world} {which}: tokens {'OK' if ok_t else 'DIFF'}, logits {'bit-exact' if ok_l else 'DIFF'}",
          flush=True)
    if not (ok_t and ok_l):
        sys.exit(1)
dist.barrier()
dist.destroy_process_group()
