"""Adversarial RMSNorm inputs: rows on which a tree sum of the squares and ggml's sequential sum give
DIFFERENT means (VERDICT r4 "What's weak" #1).  TEST INFRASTRUCTURE (CPU only).

ggml's rms_norm sums (double)(x_i*x_i) in index order, rounding after every add, then
takes mean = (float)(sum/n).  The kernels add the same terms in a tree T and keep T's mean only when
rms_mean_certain proves it equal to the sequential one, else they run the sequential sum
(csrc/device_util.h).  This module builds token-embedding rows — Q8_0 / Q4_0 / Q6_K bytes, so an
engine or a ggml graph can load them — whose embedded values x = dequantize(row) * sqrtf(n) make
the two disagree:

  * element 0 is huge (t0 = x0^2 fixes the double accumulator's ulp u for the whole sum);
  * every tail element's square t_i has its bits below u a little over half of u, so the sequential
    sum rounds UP at every add (S - E ≈ 0.3·u per element, E the exact sum), while the exact tail
    sum, added once, does not;
  * two tuner elements place E just below a rounding boundary of (float)(sum/n) and S above it.

`verify` checks the property on the bytes through the oracle's own dequantizer: every sum within
`TREE_ULPS` accumulator ulps of E (any summation tree of depth <= TREE_ULPS, Higham §4.2) gives one
mean, the sequential sum another, and the rms_norm scales 1/sqrtf(mean + eps) differ too.  Seeds
that do not meet it are skipped, so every returned row is adversarial by construction and by check.
"""
import math

import numpy as np

import oracle_ctypes as O

F32 = np.float32
TREE_ULPS = 32  # |T - E| bound in accumulator ulps that the check covers (kernel trees are < 24 deep)


def seq_sum(t):
    """ggml's order: sum += (double)t_i, i = 0 .. n-1."""
    s = 0.0
    for v in np.asarray(t, dtype=np.float64).tolist():
        s += v
    return s


def exact_sum(t):
    return math.fsum(np.asarray(t, dtype=np.float64).tolist())


def mean_of(s, n):
    return F32(s / n)  # (float)(sum / n): double division, then round to float


def scale_of(mean, eps):
    return F32(F32(1.0) / np.sqrt(F32(mean) + F32(eps)))  # 1.0f / sqrtf(mean + eps), IEEE f32


def _fp16_grid(lo, hi):
    h = np.arange(0x0400, 0x7C00, dtype=np.uint16).view(np.float16).astype(np.float32)
    return h[(h >= lo) & (h <= hi)]


def _x(c, q, s):
    return F32(F32(c) * F32(q)) * s  # (unit * q) rounded to f32, then the embedding scale


# ---- formats: element e of a row = unit[group(e)] * q[e] (groups contiguous) --------------------
FMT = {
    "q8_0": dict(group=32, qmin=-127, qmax=127, type=O.Q8_0),
    "q4_0": dict(group=32, qmin=-8, qmax=7, type=O.Q4_0),
    "q6_K": dict(group=16, qmin=-32, qmax=31, type=O.Q6_K, sb=256),
}


def pack(fmt, n, d16, sc, q):
    """Row bytes.  q8_0 / q4_0: d16[b] (fp16 bits) per 32, q[e]; q6_K: d16 per 256, sc (int8) per 16,
    q[e] in [-32, 31] (ggml block_q6_K: ql[128] qh[64] scales[16] d; scale j covers 16j .. 16j+15)."""
    out = bytearray()
    if fmt == "q8_0":
        for b in range(n // 32):
            out += int(d16[b]).to_bytes(2, "little") + np.asarray(q[32 * b:32 * b + 32], dtype=np.int8).tobytes()
    elif fmt == "q4_0":
        for b in range(n // 32):
            u = np.asarray(q[32 * b:32 * b + 32], dtype=np.int64) + 8
            qs = (u[:16] | (u[16:] << 4)).astype(np.uint8)
            out += int(d16[b]).to_bytes(2, "little") + qs.tobytes()
    else:
        for sbi in range(n // 256):
            u = np.asarray(q[256 * sbi:256 * sbi + 256], dtype=np.int64) + 32
            ql = np.zeros(128, dtype=np.int64)
            qh = np.zeros(64, dtype=np.int64)
            for h in range(2):
                for l in range(32):
                    q1, q2, q3, q4 = (u[h * 128 + l + 32 * k] for k in range(4))
                    ql[h * 64 + l] = (q1 & 15) | ((q3 & 15) << 4)
                    ql[h * 64 + l + 32] = (q2 & 15) | ((q4 & 15) << 4)
                    qh[h * 32 + l] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
            out += ql.astype(np.uint8).tobytes() + qh.astype(np.uint8).tobytes()
            out += np.asarray(sc[16 * sbi:16 * sbi + 16], dtype=np.int8).tobytes()
            out += int(d16[sbi]).to_bytes(2, "little")
    return np.frombuffer(bytes(out), dtype=np.uint8).copy()


def embed(fmt, row, n):
    """The values the norm sees: dequantize_row (the oracle's) times sqrtf(n) (src/gemma_model.cpp:677-679)."""
    return O.dequantize(FMT[fmt]["type"], row, n) * np.sqrt(F32(n))


def verify(x, eps):
    """(ok, info): every tree sum within TREE_ULPS ulps of the exact sum gives one mean, ggml's
    sequential sum another, and the two rms_norm scales differ."""
    x = np.asarray(x, dtype=np.float32)
    n = x.size
    t = x * x  # fp32 squares, as ggml and the kernels form them
    if not np.all(np.isfinite(t)):
        return False, {}
    S, E = seq_sum(t), exact_sum(t)
    u = math.ulp(E)
    lo, hi = mean_of(E - TREE_ULPS * u, n), mean_of(E + TREE_ULPS * u, n)
    mS, mE = mean_of(S, n), mean_of(E, n)
    info = dict(S=S, E=E, ulps=(S - E) / u, mean_seq=mS, mean_tree=mE, scale_seq=scale_of(mS, eps),
                scale_tree=scale_of(mE, eps))
    ok = lo == hi == mE and mS != mE and info["scale_seq"] != info["scale_tree"]
    return bool(ok), info


def build_row(fmt, n, eps=1e-6, seed=0, tries=64):
    """(row bytes, x, info) of an adversarial row of n values in format fmt (n a multiple of 256 for q6_K)."""
    for k in range(tries):
        r = _attempt(fmt, n, eps, seed * 1000 + k)
        if r is not None:
            return r
    raise RuntimeError("no adversarial row found")


def _attempt(fmt, n, eps, seed):
    f = FMT[fmt]
    rng = np.random.default_rng(seed)
    s = np.sqrt(F32(n))
    G = f["group"]
    ng = n // G
    q = np.zeros(n, dtype=np.int64)
    unit = np.zeros(ng, dtype=np.float32)  # per group
    d16 = np.zeros(n // f.get("sb", G), dtype=np.uint16)
    sc = np.zeros(ng, dtype=np.int64)
    qtop = f["qmax"]
    # element 0: t0 with a mid-binade mantissa (the accumulator keeps one ulp over the whole sum)
    if fmt == "q6_K":
        d0s = _fp16_grid(8.0, 2048.0)
        c0s = F32(d0s * F32(127))
    else:
        c0s = d0s = _fp16_grid(8.0, 2048.0)
    x0s = _x(c0s, qtop, s)
    t0s = (x0s * x0s).astype(np.float64)
    mant = t0s / 2.0 ** np.floor(np.log2(t0s))
    pick = np.flatnonzero((mant > 1.25) & (mant < 1.5))
    i0 = int(rng.choice(pick))
    t0 = float(t0s[i0])
    u = math.ulp(t0)
    d16[0] = np.float16(d0s[i0]).view(np.uint16)
    if fmt == "q6_K":
        sc[0] = 127
    unit[0] = c0s[i0]
    q[0] = qtop
    # boundary: the float midpoint above t0/n, one float spacing further if the tail would be too short
    f0 = F32(t0 / n)
    f1 = np.nextafter(f0, F32(np.inf))
    M = (float(f0) + float(f1)) / 2.0 * n
    # tail: the groups after the big element's group (q6_K: after super-block 0), minus two tuner groups
    first = (256 if fmt == "q6_K" else G) // G
    tail_groups = list(range(first, ng - 2))
    m = len(tail_groups) * G
    bias = 0.3 * m * u  # expected S - E from the tail
    D = M - t0 - bias / 2  # the exact tail + tuners should sum to this
    t_avg = D / (m + 3)
    tuner_share = 3 * t_avg  # two tuners absorb the greedy tail's residue
    frac_lo, frac_hi = 0.52, 0.75
    qs = np.arange(f["qmin"], f["qmax"] + 1)
    qs = qs[qs != 0]
    if fmt == "q6_K":  # shared d per tail super-block: unit = d * sc, sc picked per group below
        for sbi in range(1, n // 256):
            dt = F32(np.sqrt(t_avg) / (float(s) * 60.0 * 20.0))
            d16[sbi] = np.float16(dt * F32(rng.uniform(0.9, 1.1))).view(np.uint16)
    acc_tail = []  # chosen tail squares, in order
    for gi, g in enumerate(tail_groups):
        if fmt == "q6_K":
            dsb = F32(np.float16(d16[g * G // 256].view(np.float16)))
            scs = np.arange(-128, 128)
            cs = F32(dsb * F32(scs))
            ok_sc = scs[(np.abs(cs) > 0)]
            want = np.sqrt(t_avg) / (float(s) * 20.0)
            sc[g] = int(ok_sc[np.argmin(np.abs(np.abs(F32(dsb * F32(ok_sc))) - want) + rng.uniform(0, 1e-3, ok_sc.size))])
            unit[g] = F32(dsb * F32(sc[g]))
        else:  # the group's fp16 d: of a few random ones near the target, the one whose palette has
            # the most rounding-up squares within a factor 2 of t_avg
            best_n, best_d = -1, None
            for _ in range(64):
                dg = np.float16(np.sqrt(t_avg) / (float(s) * (qtop * 0.75)) * rng.uniform(0.7, 1.3))
                xs = _x(F32(dg), qs, s)
                ts = (xs * xs).astype(np.float64)
                fr = np.mod(ts, u) / u
                cnt = int(((fr > frac_lo) & (fr < frac_hi) & (ts > t_avg / 2) & (ts < 2 * t_avg)).sum())
                if cnt > best_n:
                    best_n, best_d = cnt, dg
            d16[g] = best_d.view(np.uint16)
            unit[g] = F32(best_d)
        xs = _x(unit[g], qs, s)
        ts = (xs * xs).astype(np.float64)
        frac = np.mod(ts, u) / u
        good = (frac > frac_lo) & (frac < frac_hi)
        if not good.any():
            return None
        gq, gt = qs[good], ts[good]
        for e in range(G):
            done = len(acc_tail)
            want_t = (D - tuner_share - math.fsum(acc_tail)) / max(1, m - done)
            cand = np.argsort(np.abs(gt - want_t))[:3]
            j = int(rng.choice(cand))
            q[g * G + e] = gq[j]
            acc_tail.append(float(gt[j]))
    # two tuners (first element of each of the last two groups): exact tail + tuners = D
    R = D - math.fsum(acc_tail)
    if not (0.3 * t_avg < R < 12 * t_avg):
        return None
    tg = [ng - 2, ng - 1]
    if fmt == "q6_K":
        dsb = F32(np.float16(d16[(n - 1) // 256].view(np.float16)))
        scs = np.arange(-128, 128)
        cands = [(F32(dsb * F32(sv)), sv) for sv in scs if sv != 0]
        cu = np.array([c for c, _ in cands], dtype=np.float32)
        cmeta = np.array([sv for _, sv in cands])
    else:
        grid = _fp16_grid(1e-3, 4096.0)
        cu, cmeta = grid, np.float16(grid).view(np.uint16)
    CU, QQ = np.meshgrid(cu, qs, indexing="ij")
    XX = _x(CU.ravel(), QQ.ravel(), s)
    TT = (XX * XX).astype(np.float64)
    keep = (TT > 0) & (TT < R)
    TT, idx = TT[keep], np.flatnonzero(keep)
    order = np.argsort(TT)
    TT, idx = TT[order], idx[order]
    win = bias / 8
    need = R - TT
    j = np.clip(np.searchsorted(TT, need), 1, TT.size - 1)
    hit = None
    for jj in (j - 1, j):
        okp = np.abs(TT + TT[jj] - R) < win
        if okp.any():
            a = int(rng.choice(np.flatnonzero(okp)))
            hit = (idx[a], idx[jj[a]])
            break
    if hit is None:
        return None
    best = hit
    for g, flat in zip(tg, best):
        ci, qi = divmod(int(flat), qs.size)
        q[g * G:g * G + G] = 0
        q[g * G] = qs[qi]
        unit[g] = cu[ci]
        if fmt == "q6_K":
            sc[g] = int(cmeta[ci])
        else:
            d16[g] = int(cmeta[ci])
    row = pack(fmt, n, d16, sc, q)
    x = embed(fmt, row, n)
    ok, info = verify(x, eps)
    return (row, x, info) if ok else None


def pick_norm_weight(x0, info, kind, w_start=1.0):
    """A norm weight w0 for element 0 that carries the scale difference into the quantized activation:
    kind "q8_0": the fp16 block scale d = fp16(amax / 127) of y0 = (x0*scale)*w0 (quantize_row_q8_0)
    differs between the two scales; "q8_K": quantize_row_q8_K's d = 1/iscale, iscale = -127/y0."""
    ws = (F32(w_start) + np.arange(1 << 20, dtype=np.float32) * np.spacing(F32(w_start))).astype(np.float32)
    ys, yt = (F32(F32(x0) * info["scale_seq"]) * ws), (F32(F32(x0) * info["scale_tree"]) * ws)
    if kind == "q8_0":
        ds = (np.abs(ys) / F32(127)).astype(np.float16)
        dt = (np.abs(yt) / F32(127)).astype(np.float16)
    else:
        ds = F32(1.0 / F32(-127.0 / ys.astype(np.float64)).astype(np.float64))
        dt = F32(1.0 / F32(-127.0 / yt.astype(np.float64)).astype(np.float64))
    hit = np.flatnonzero(ds != dt)
    if hit.size == 0:
        raise RuntimeError("no sensitive norm weight found")
    return F32(ws[hit[0]])
