"""The Gemma-2B graph built through this repo's ggml surface (include/ggml.h, csrc/ggml_api.cpp) by
the restated driver (tests/ggml_driver/gemma_graph_driver.cpp, the API calls of
src/gemma_model.cpp:665-747) against the reference's only held fixture for this path:
tests/golden/tensor_in_target_cgraph.txt, a verbatim copy of the data file
/root/reference/tensor_dump/tensor_in_target_cgraph (the node listing of the llama.cpp Gemma-2B graph
the author compared the reference's graph with, src/gemma_model.cpp:240-248 / tensor_dump.cpp).

What it pins (CPU only, no weights, no device):
* node count (620 for 18 layers) and, node by node, the op: ggml's own names ("node_<i>" of unnamed
  nodes, "<src> (view)", " (reshaped)", "(copy of node_<i>)") must be identical, and llama.cpp's
  callback names (norm-<il>, kq-<il>, ffn_gelu-<il>, ...) must be the op that callback names;
* the copies into the cache views and the K / V views of each layer read that layer's cache;
* both stages (the listing is one graph; the reference builds the same structure for PREFILL and
  DECODE, only the shapes differ).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "ggml_driver", "gemma_graph_driver")
FIXTURE = os.path.join(ROOT, "tests", "golden", "tensor_in_target_cgraph.txt")

# llama.cpp callback name (without the layer suffix) -> the op that tensor is
CB_OP = {"norm": "RMS_NORM", "k_cache_view": "VIEW", "v_cache_view": "VIEW", "v_cur_t": "TRANSPOSE", "v": "VIEW",
         "k": "VIEW", "q": "PERMUTE", "kq": "MUL_MAT", "kq_soft_max_ext": "SOFT_MAX", "kqv": "MUL_MAT",
         "kqv_merged": "PERMUTE", "kqv_merged_cont": "CONT", "kqv_out": "MUL_MAT", "ffn_gate": "MUL_MAT",
         "ffn_gelu": "GELU", "ffn_up": "MUL_MAT", "ffn_gate_par": "MUL", "result_norm": "MUL",
         "result_output": "MUL_MAT"}
GEMMA_2B = ["18", "2048", "8", "1", "256", "16384", "256000", "512", "2"]  # n_layer E H Hkv hd F V ctx Q4_0


def _target():
    rows = []
    with open(FIXTURE) as f:
        for line in f:
            m = re.match(r"node\[(\d+)\]: (.*)$", line.rstrip("\n"))
            if m:
                assert int(m.group(1)) == len(rows)
                rows.append(m.group(2))
    return rows


def _ours(T, decode):
    if not os.path.exists(DRIVER):
        pytest.skip("driver not built (make -C gemma.ggml_amd)")
    out = subprocess.run([DRIVER, "--graph-listing", *GEMMA_2B, str(T), "1" if decode else "0"], capture_output=True,
                         text=True, timeout=120, check=True).stdout
    rows = []
    for line in out.splitlines():
        m = re.match(r"node\[(\d+)\]: (.*)\t(\w+)$", line)
        assert m, line
        assert int(m.group(1)) == len(rows)
        rows.append((m.group(2), m.group(3)))
    return rows


def _expected_op(name):
    if name.endswith("(view)"):
        return "VIEW"
    if name.endswith("(reshaped)"):
        return "RESHAPE"
    if "(copy of" in name:
        return "CPY"
    if re.fullmatch(r"node_\d+", name):
        return None  # unnamed in both graphs: the name itself must match
    base = re.sub(r"-\d+$", "", name)
    assert base in CB_OP, f"unknown fixture name {name!r}"
    return CB_OP[base]


def test_fixture_shape():
    t = _target()
    assert len(t) == 620 and t[0] == "inp_tokens (view)" and t[-1] == "result_output"


@pytest.mark.parametrize("T,decode", [(5, False), (1, True)])
def test_gemma2b_graph_matches_reference_listing(T, decode):
    target, ours = _target(), _ours(T, decode)
    assert len(ours) == len(target), f"{len(ours)} nodes vs the fixture's {len(target)}"
    for i, (tn, (on, op)) in enumerate(zip(target, ours)):
        exp = _expected_op(tn)
        where = f"node[{i}]: fixture {tn!r}, ours {on!r} {op}"
        layer = re.search(r"-(\d+)", tn)
        if exp is None:
            assert on == tn, where  # ggml's node_<index> of an unnamed node: same position, same op chain
            continue
        assert op == exp, where
        if tn.endswith("(view)") or tn.endswith("(reshaped)"):
            if not tn.startswith(("k_cache_view", "v_cache_view")):
                assert on == tn, where
        if "(copy of" in tn:
            src = tn.split("(copy of ", 1)[1].rstrip(")")
            cache = "cache_k_l" if tn.startswith("k_cache_view") else "cache_v_l"
            assert on.startswith(f"{cache}{layer.group(1)} (view) (copy of "), where
            if re.fullmatch(r"node_\d+", src):
                assert on.endswith(f"(copy of {src})"), where
        base = re.sub(r"-\d+$", "", tn)
        if base in ("k_cache_view", "k"):
            assert on == f"cache_k_l{layer.group(1)} (view)", where
        if base in ("v_cache_view", "v"):
            assert on == f"cache_v_l{layer.group(1)} (view)", where
