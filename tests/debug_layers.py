"""Debug helper (not a test): per-layer GPU vs oracle comparison for one configuration."""
import sys

import numpy as np

import oracle_ctypes as O
import gemma_hip as G
import ctypes as C


def run(shape, n_prompt, n_steps, n_ctx, wtype):
    L = O.lib()
    L.orc_model_taps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    m = O.Model(O.make_config(shape, n_ctx=n_ctx, wtype=wtype))
    e = G.Engine(shape, n_ctx=n_ctx, wtype=wtype)
    G.lib().gemma_engine_debug_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    e.begin(prompt)
    m.reset()
    qw = shape["n_head"] * shape["head_dim"]
    kvw = shape["n_head_kv"] * shape["head_dim"]
    E = shape["n_embd"]
    per = qw + 2 * kvw + qw + E
    seq = list(prompt)
    for step in range(n_steps):
        taps = np.zeros(per * shape["n_layer"], dtype=np.float32)
        lg = np.zeros(shape["n_vocab"], dtype=np.float32)
        r = G.lib().gemma_engine_debug_step(e.h, taps.ctypes.data, lg.ctypes.data)
        assert r == 0, G.last_error()
        tok, last, _ = m.inference(np.array(seq[:step + 1], dtype=np.int32), 0 if step == 0 else 1)
        if step + 1 >= len(seq):
            seq.append(tok)
        taps = taps.reshape(shape["n_layer"], per)
        worst = []
        for il in range(shape["n_layer"]):
            q = np.zeros(qw + 2 * kvw, dtype=np.float32)
            a = np.zeros(qw, dtype=np.float32)
            x = np.zeros(E, dtype=np.float32)
            L.orc_model_taps(m.h, il, q.ctypes.data, a.ctypes.data, x.ctypes.data)
            g = taps[il]
            dq = np.abs(g[:qw + 2 * kvw] - q).max()
            da = np.abs(g[qw + 2 * kvw:qw + 2 * kvw + qw] - a).max()
            dx = np.abs(g[-E:] - x).max()
            nq = int((g[:qw + 2 * kvw].view(np.uint32) != q.view(np.uint32)).sum())
            na = int((g[qw + 2 * kvw:qw + 2 * kvw + qw].view(np.uint32) != a.view(np.uint32)).sum())
            nx = int((g[-E:].view(np.uint32) != x.view(np.uint32)).sum())
            worst.append((il, nq, na, nx, dq, da, dx))
        nl = int((lg.view(np.uint32) != last.view(np.uint32)).sum())
        bad = [w for w in worst if w[1] or w[2] or w[3]]
        print(f"step {step} pos {step} logits_diff={nl} first_bad_layer={bad[0] if bad else None}", flush=True)
        if bad:
            for w in bad[:3]:
                print("   ", w)
            break


def run_graph(shape, n_prompt, n_steps, n_ctx, wtype):
    m = O.Model(O.make_config(shape, n_ctx=n_ctx, wtype=wtype))
    prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    for use_graph in (0, 1):
        e = G.Engine(shape, n_ctx=n_ctx, wtype=wtype)
        e.begin(prompt)
        lg = e.step(n_steps, want_logits=True, use_graph=use_graph)
        toks = e.tokens()
        m.reset()
        for step in range(n_steps):
            tok, last, _ = m.inference(toks[:step + 1], 0 if step == 0 else 1)
            nd = int((lg[step].view(np.uint32) != last.view(np.uint32)).sum())
            if nd:
                print(f"graph={use_graph} first diff at step {step}: {nd} logits, max {np.abs(lg[step]-last).max()}")
                break
        else:
            print(f"graph={use_graph} all {n_steps} steps bit-exact")
        e.close()


if __name__ == "__main__":
    which = sys.argv[1]
    if which == "tiny_q8":
        run(O.TINY, 7, 40, 128, O.Q8_0)
    elif which == "tiny_q8_long":
        run(O.TINY, 7, 36, 128, O.Q8_0)
    elif which == "tiny_q4":
        run(O.TINY, 7, 40, 128, O.Q4_0)
    elif which == "2b_graph":
        O.lib().orc_set_threads(16)
        run_graph(O.GEMMA_2B, 6, 10, 256, O.Q4_0)
    elif which == "tiny_q8_graph":
        run_graph(O.TINY, 7, 40, 128, O.Q8_0)
    elif which == "2b":
        O.lib().orc_set_threads(16)
        run(O.GEMMA_2B, 6, 8, 256, O.Q4_0)
