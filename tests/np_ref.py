"""TEST INFRASTRUCTURE — an independent numpy restatement of the decode step.

A second restatement, written from the public ggml block spec and the
llama.cpp graph the reference calls (`llama_decode`, test-to-speech.cpp:178-185), that
shares no code with oracle/llm_ref.c + quant_ref.c: it cross-checks the C oracle (SURVEY §7
step 1), so a misreading shared by the C oracle and the HIP kernels cannot pass unseen.

Semantics restated (ggml CPU, parity unpinned):
  * weights: Q8_0 {f16 d, i8 q[32]}; Q4_K {f16 d, dmin, 12 B of 6-bit scales/mins, 4-bit q};
    Q6_K {ql, qh, i8 scales[16], f16 d}; dequantized values are exact in float64;
  * mul_mat re-quantizes the activation to the weight's vec_dot_type (Q8_0 for Q8_0
    weights: d = amax / 127 kept as f16, q = roundf(x / d); Q8_K for the K-quants: the
    signed value of largest |x| gives iscale = -127 / max, q = nearest-even, <= 127). The
    integer block dot ggml evaluates equals dot(dequant(w), dequant(a)) exactly, so it is
    float64 `@` here;
  * rms_norm: sum of f32 squares in double, scale = 1 / sqrtf(mean + eps) in f32;
  * RoPE: ggml rope cache (theta *= base^(-2/hd) in f32), NORM (2i, 2i+1) for llama,
    NEOX (i, i + hd/2) for qwen2 / qwen3; qwen3 q/k RMSNorm per head before it; qwen2
    q/k/v biases added after the projections;
  * F16 K/V cache; q rounded to f16 for Q.K^T; softmax(s / sqrt(hd)); out = sum p v;
  * ffn: down(silu(gate h) * up h); final output_norm + lm_head (tied to token_embd when
    output.weight is absent);
  * lfm2 (llama.cpp build_lfm2): attention layers with q/k RMSNorm and NEOX RoPE; the other
    layers a gated short conv: bcx = in_proj(norm x) = B | C | X, bx = B * X, a depthwise
    causal conv of width l_cache over the sequence's bx (ggml_ssm_conv, zero before the
    sequence), y = C * conv, out_proj(y); final norm token_embd_norm.
"""
from __future__ import annotations

import numpy as np

from miotts_amd import gguf_np


def _f16(a) -> np.ndarray:
    return np.asarray(a, np.uint8).view(np.float16).astype(np.float64)


def dequant(qtype: int, raw: np.ndarray, rows: int, k: int) -> np.ndarray:
    """GGUF rows (raw bytes, `rows` x row_bytes) -> float64 [rows, k]."""
    raw = np.asarray(raw, np.uint8)
    if qtype == 0:
        return raw.view(np.float32).reshape(rows, k).astype(np.float64)
    if qtype == 8:
        b = raw.reshape(rows, k // 32, 34)
        d = _f16(b[:, :, 0:2].copy()).reshape(rows, k // 32, 1)
        q = b[:, :, 2:].view(np.int8).astype(np.float64)
        return (d * q).reshape(rows, k)
    if qtype == 12:
        b = raw.reshape(rows, k // 256, 144)
        d = _f16(b[:, :, 0:2].copy()).reshape(rows, -1, 1)
        dmin = _f16(b[:, :, 2:4].copy()).reshape(rows, -1, 1)
        sc = b[:, :, 4:16].astype(np.int64)
        qs = b[:, :, 16:].astype(np.int64)
        # 6-bit scale / min of sub-block j (ggml get_scale_min_k4)
        scl, mn = np.zeros(sc.shape[:2] + (8,)), np.zeros(sc.shape[:2] + (8,))
        for j in range(8):
            if j < 4:
                scl[..., j] = sc[..., j] & 63
                mn[..., j] = sc[..., j + 4] & 63
            else:
                scl[..., j] = (sc[..., j + 4] & 0xF) | ((sc[..., j - 4] >> 6) << 4)
                mn[..., j] = (sc[..., j + 4] >> 4) | ((sc[..., j] >> 6) << 4)
        out = np.zeros((rows, k // 256, 256))
        for c in range(4):  # 64-weight chunk c: low nibbles (sub-block 2c), then high (2c+1)
            q = qs[:, :, 32 * c:32 * c + 32]
            out[:, :, 64 * c:64 * c + 32] = (d * scl[..., 2 * c:2 * c + 1]) * (q & 0xF) - dmin * mn[..., 2 * c:2 * c + 1]
            out[:, :, 64 * c + 32:64 * c + 64] = (d * scl[..., 2 * c + 1:2 * c + 2]) * (q >> 4) - dmin * mn[..., 2 * c + 1:2 * c + 2]
        return out.reshape(rows, k)
    if qtype == 14:
        b = raw.reshape(rows, k // 256, 210)
        ql = b[:, :, 0:128].astype(np.int64)
        qh = b[:, :, 128:192].astype(np.int64)
        sc = b[:, :, 192:208].view(np.int8).astype(np.float64)
        d = _f16(b[:, :, 208:210].copy()).reshape(rows, -1, 1)
        out = np.zeros((rows, k // 256, 256))
        for h in range(2):  # two 128-weight halves
            L = ql[:, :, 64 * h:64 * h + 64]
            H = qh[:, :, 32 * h:32 * h + 32]
            S = sc[:, :, 8 * h:8 * h + 8]
            q1 = ((L[..., :32] & 0xF) | ((H & 3) << 4)) - 32
            q2 = ((L[..., 32:] & 0xF) | (((H >> 2) & 3) << 4)) - 32
            q3 = ((L[..., :32] >> 4) | (((H >> 4) & 3) << 4)) - 32
            q4 = ((L[..., 32:] >> 4) | (((H >> 6) & 3) << 4)) - 32
            for n, q in enumerate((q1, q2, q3, q4)):
                s = np.repeat(S[..., [2 * n, 2 * n + 1]], 16, axis=-1)  # sub-blocks of 16
                out[:, :, 128 * h + 32 * n:128 * h + 32 * n + 32] = d * s * q
        return out.reshape(rows, k)
    if qtype in (2, 6):  # Q4_0 / Q5_0: 32 codes per block, x - 8 / (nibble | fifth bit) - 16
        bb = 18 if qtype == 2 else 22
        b = raw.reshape(rows, k // 32, bb)
        d = _f16(b[:, :, 0:2].copy()).reshape(rows, -1, 1)
        qs = b[:, :, bb - 16:].astype(np.int64)
        lo, hi = qs & 0xF, qs >> 4
        if qtype == 2:
            lo, hi = lo - 8, hi - 8
        else:
            qh = b[:, :, 2:6].copy().view(np.uint32).astype(np.int64)  # [rows, blocks, 1]
            j = np.arange(16)
            lo = (lo | (((qh >> j) & 1) << 4)) - 16
            hi = (hi | (((qh >> (j + 16)) & 1) << 4)) - 16
        return (d * np.concatenate([lo, hi], axis=2)).reshape(rows, k)
    if qtype == 30:  # BF16: the high half of an f32
        return (raw.view(np.uint16).astype(np.uint32) << 16).view(np.float32).reshape(rows, k).astype(np.float64)
    raise ValueError(f"np_ref: weight type {qtype}")


def _roundf(v: np.ndarray) -> np.ndarray:
    return np.sign(v) * np.floor(np.abs(v) + 0.5)  # C roundf: half away from zero


def act_q8_0(x: np.ndarray) -> np.ndarray:
    """quantize_row_q8_0_ref, returned dequantized (f16 scale)."""
    x = x.astype(np.float32).reshape(-1, 32)
    amax = np.abs(x).max(1, keepdims=True)
    d = (amax / np.float32(127)).astype(np.float32)
    idv = np.where(d != 0, np.float32(1) / np.where(d != 0, d, 1), 0).astype(np.float32)
    q = _roundf((x * idv).astype(np.float32).astype(np.float64))
    return (d.astype(np.float16).astype(np.float64) * q).reshape(-1)


def act_bf16(x: np.ndarray) -> np.ndarray:
    """ggml_compute_fp32_to_bf16 (nearest even), returned as float64."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    h = ((u + (0x7FFF + ((u >> 16) & 1))) >> 16).astype(np.uint32)
    return (h << 16).view(np.float32).astype(np.float64)


def act_q8_k(x: np.ndarray) -> np.ndarray:
    """quantize_row_q8_K_ref, returned dequantized."""
    x = x.astype(np.float32).reshape(-1, 256)
    out = np.zeros(x.shape)
    for i, blk in enumerate(x):
        j = int(np.argmax(np.abs(blk)))
        if blk[j] == 0:
            continue
        iscale = np.float32(-127.0) / blk[j]
        q = np.minimum(np.rint((iscale * blk).astype(np.float32)).astype(np.float64), 127)
        out[i] = np.float64(np.float32(1) / iscale) * q
    return out.reshape(-1)


class Mat:
    def __init__(self, t: gguf_np.Tensor):
        self.type, self.k, self.rows = t.type, t.ne[0], t.ne[1] if len(t.ne) > 1 else 1
        self.w = dequant(t.type, t.raw(), self.rows, self.k)

    def __matmul__(self, x: np.ndarray) -> np.ndarray:
        # the vec_dot_type: Q8_0 for Q8_0 / Q5_0 / Q4_0, Q8_K for the K-quants, BF16 for BF16
        if self.type in (2, 6, 8):
            a = act_q8_0(x)
        elif self.type in (12, 14):
            a = act_q8_k(x)
        elif self.type == 30:
            a = act_bf16(x)
        else:
            a = x.astype(np.float64)
        return (self.w @ a).astype(np.float32)


def rms_norm(x: np.ndarray, w: np.ndarray, eps: float) -> np.ndarray:
    x = x.astype(np.float32)
    mean = np.float32(np.sum((x * x).astype(np.float64)) / x.size)
    scale = np.float32(1.0) / np.sqrt(np.float32(mean + np.float32(eps)))
    return ((x * scale).astype(np.float32) * w.astype(np.float32)).astype(np.float32)


def rope_table(n_ctx: int, hd: int, base: float) -> np.ndarray:
    ts = np.float32(np.float32(base) ** np.float32(-2.0 / hd))
    out = np.zeros((n_ctx, hd // 2, 2), np.float32)
    for p in range(n_ctx):
        th = np.float32(p)
        for i in range(hd // 2):
            out[p, i] = (np.cos(th), np.sin(th))
            th = np.float32(th * ts)
    return out


class DecodeStep:
    """One llama_decode token step at a time, its own F16 K/V cache."""

    def __init__(self, path: str, n_ctx: int = 256):
        g = gguf_np.GGUFReader(path)
        a = g.kv["general.architecture"]
        kv = lambda k, d=None: g.kv.get(f"{a}.{k}", d)
        self.arch = a
        self.n_embd, self.n_layer = kv("embedding_length"), kv("block_count")
        self.n_head = kv("attention.head_count")
        hkv = kv("attention.head_count_kv", self.n_head)
        self.kv_per_layer = list(hkv) if isinstance(hkv, list) else [hkv] * self.n_layer
        self.n_kv = max(self.kv_per_layer) or self.n_head
        self.l_cache = kv("shortconv.l_cache", 3)
        self.hd = kv("attention.key_length", self.n_embd // self.n_head)
        self.eps = np.float32(kv("attention.layer_norm_rms_epsilon", 1e-6))
        self.neox = a in ("qwen2", "qwen3", "lfm2")
        self.rope = rope_table(n_ctx, self.hd, kv("rope.freq_base", 10000.0))
        f32 = lambda n: g.tensor(n).array().astype(np.float32).reshape(-1) if n in g.by_name else None
        self.tok = Mat(g.tensor("token_embd.weight"))
        self.out = Mat(g.tensor("output.weight")) if "output.weight" in g.by_name else self.tok
        self.out_norm = f32("token_embd_norm.weight" if a == "lfm2" else "output_norm.weight")
        self.L = []
        for i in range(self.n_layer):
            p = f"blk.{i}."
            conv = p + "shortconv.in_proj.weight" in g.by_name
            mats = ("shortconv.in_proj", "shortconv.out_proj") if conv else ("attn_q", "attn_k", "attn_v", "attn_output")
            self.L.append({
                "attn_norm": f32(p + "attn_norm.weight"), "ffn_norm": f32(p + "ffn_norm.weight"),
                "q_norm": f32(p + "attn_q_norm.weight"), "k_norm": f32(p + "attn_k_norm.weight"),
                "bq": f32(p + "attn_q.bias"), "bk": f32(p + "attn_k.bias"), "bv": f32(p + "attn_v.bias"),
                "conv": g.tensor(p + "shortconv.conv.weight").array().astype(np.float32) if conv else None,
                **{n: Mat(g.tensor(p + n + ".weight")) for n in mats + ("ffn_gate", "ffn_up", "ffn_down")}})
        self.kc = np.zeros((self.n_layer, self.n_kv, n_ctx, self.hd), np.float16)
        self.vc = np.zeros_like(self.kc)
        self.bx = np.zeros((self.n_layer, n_ctx, self.n_embd), np.float32)  # short-conv inputs

    def _rope(self, x: np.ndarray, pos: int) -> np.ndarray:
        cs = self.rope[pos]
        h = self.hd
        i0 = np.arange(h // 2) if self.neox else 2 * np.arange(h // 2)
        i1 = i0 + h // 2 if self.neox else i0 + 1
        y = x.copy()
        x0, x1 = x[..., i0], x[..., i1]
        y[..., i0] = x0 * cs[:, 0] - x1 * cs[:, 1]
        y[..., i1] = x0 * cs[:, 1] + x1 * cs[:, 0]
        return y.astype(np.float32)

    def layer(self, il: int, x: np.ndarray, pos: int) -> np.ndarray:
        """Residual stream after layer il for input x at position pos (writes the K/V row)."""
        L, H, Hk, hd = self.L[il], self.n_head, self.n_kv, self.hd
        h = rms_norm(x, L["attn_norm"], self.eps)
        if L["conv"] is not None:
            D = self.n_embd
            bcx = L["shortconv.in_proj"] @ h
            bx = (bcx[:D] * bcx[2 * D:]).astype(np.float32)
            self.bx[il, pos] = bx
            w = L["conv"]  # [D][l_cache]
            acc = np.zeros(D, np.float32)
            for j in range(self.l_cache):
                p = pos - (self.l_cache - 1) + j
                v = self.bx[il, p] if p >= 0 else np.zeros(D, np.float32)
                acc = (acc + (v * w[:, j]).astype(np.float32)).astype(np.float32)
            y = (bcx[D:2 * D] * acc).astype(np.float32)
            x = (x + (L["shortconv.out_proj"] @ y)).astype(np.float32)
            return self._ffn(L, x)
        q, k, v = L["attn_q"] @ h, L["attn_k"] @ h, L["attn_v"] @ h
        if L["bq"] is not None:
            q, k, v = (q + L["bq"]).astype(np.float32), (k + L["bk"]).astype(np.float32), (v + L["bv"]).astype(np.float32)
        q, k = q.reshape(H, hd), k.reshape(Hk, hd)
        if L["q_norm"] is not None:
            q = np.stack([rms_norm(r, L["q_norm"], self.eps) for r in q])
            k = np.stack([rms_norm(r, L["k_norm"], self.eps) for r in k])
        q, k = self._rope(q, pos), self._rope(k, pos)
        self.kc[il, :, pos] = k.astype(np.float16)
        self.vc[il, :, pos] = v.reshape(Hk, hd).astype(np.float16)
        G = H // Hk
        att = np.zeros((H, hd))
        for hh in range(H):
            K = self.kc[il, hh // G, :pos + 1].astype(np.float64)
            V = self.vc[il, hh // G, :pos + 1].astype(np.float64)
            s = (K @ q[hh].astype(np.float16).astype(np.float64)) / np.sqrt(hd)
            p = np.exp(s - s.max())
            att[hh] = (p / p.sum()) @ V
        x = (x + (L["attn_output"] @ att.reshape(-1).astype(np.float32))).astype(np.float32)
        return self._ffn(L, x)

    def _ffn(self, L, x):
        h = rms_norm(x, L["ffn_norm"], self.eps)
        g, u = (L["ffn_gate"] @ h).astype(np.float64), (L["ffn_up"] @ h).astype(np.float64)
        a = (g / (1.0 + np.exp(-g)) * u).astype(np.float32)
        return (x + (L["ffn_down"] @ a)).astype(np.float32)

    def embed(self, token: int) -> np.ndarray:
        return self.tok.w[token].astype(np.float32)

    def eval(self, token: int, pos: int) -> np.ndarray:
        x = self.embed(token)
        for il in range(self.n_layer):
            x = self.layer(il, x, pos)
        return self.out @ rms_norm(x, self.out_norm, self.eps)
