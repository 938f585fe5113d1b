"""Per-class matvec timing under explicit plans (hipEvents, back-to-back launches rotating over the
layers, as bench.py's roofline leg): python scripts/kern_ab.py 'down=9,1,1;down=8,1,1' ..."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gemma.ggml_amd", "python"))
import gemma_hip as G  # noqa: E402

SH = dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
IDS = {"gate_up": 0, "down": 1, "qkv": 2, "attn_out": 3, "logits": 4}
e = G.Engine(SH, n_ctx=256, device=0, wtype=int(os.environ.get("WTYPE", "2")))
base = e.plan()
for spec in sys.argv[1:]:
    p = dict(base)
    for item in spec.split(";"):
        k, v = item.split("=")
        p[k] = int(v) if k == "attention" else tuple(int(t) for t in v.split(","))
    e.set_plan(p)
    res = {}
    for k in [k for k in IDS if k in spec] + ["step"]:
        if k == "step":
            e.begin([2, 100, 200, 300])
            us, _ = e.time_kernel(5, 60)
        else:
            us, algo = e.time_kernel(IDS[k], 60)
        res[k] = round(us, 2)
    print(spec, res, flush=True)
e.close()
