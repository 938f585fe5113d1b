"""K-quant matvec timing at Gemma-2B shapes (gemma_kq_time): avg µs and GB/s per launch."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gemma.ggml_amd", "python"))
import gemma_hip as G  # noqa: E402

L = G.lib()
for t, n in ((12, "q4_K"), (14, "q6_K")):
    for rows, K in ((16384, 2048), (2048, 16384), (2560, 2048), (256000, 2048)):
        ab = C.c_double()
        us = L.gemma_kq_time(t, rows, K, 50, C.byref(ab))
        print(f"{n} rows {rows} K {K}: {us:.2f} us {ab.value / us / 1e3:.1f} GB/s", flush=True)
