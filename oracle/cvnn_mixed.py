"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the network half of the training step (``_torch_step``, reference
gbm_trainer.py:819-835, on the ComplexLinear / modReLU / zReLU chain of cvnn.py:65-210) with the
operand precision of the MFMA kernels (spectralmc_amd/csrc/cvnn_mfma.hip) made explicit:

* every GEMM operand (activations Z, packed weights, output gradients dU) is rounded to the
  operand type first — ``"bf16"``: round to nearest even (torch's ``float.bfloat16()``);
  ``"f32"``: unchanged;
* products are summed exactly (float64 here) and the sum is rounded to f32, where the GPU sums in
  f32 on the matrix cores — the only difference the parity tests allow for;
* bias, activation, loss, activation backward run in f32 (loss summed in f64), as the kernels do.

The bf16 mode is the build's extension for BASELINE.json configs[2] ("bf16 CVNN"); the reference
asserts full precision (gbm_trainer.py:679-686), so its parity is against this restatement.

    layers: sequence of (in_features, out_features, activation, w_re, w_im, b_re, b_im, act_bias)
            with element offsets into the flat parameter vector (-1 = absent); activation
            0 none, 1 modReLU, 2 zReLU (include/spectralmc_hip.h)
"""

from __future__ import annotations

import numpy as np

ACT_NONE, ACT_MODRELU, ACT_ZRELU = 0, 1, 2


def bf16_round(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest-even bfloat16, returned as float32 (finite inputs)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def _rounder(operand: str):
    if operand == "bf16":
        return bf16_round
    if operand == "f32":
        return lambda x: np.asarray(x, dtype=np.float32)
    raise ValueError(operand)


def _interleave(re: np.ndarray, im: np.ndarray) -> np.ndarray:
    out = np.empty((re.shape[0], 2 * re.shape[1]), dtype=np.float32)
    out[:, 0::2] = re
    out[:, 1::2] = im
    return out


def _wc(params: np.ndarray, ni: int, no: int, w_re: int, w_im: int) -> np.ndarray:
    """Real [2 no][2 ni] map of the complex weight A + iB: blocks [[A, -B], [B, A]]."""
    A = params[w_re:w_re + no * ni].reshape(no, ni)
    Bm = params[w_im:w_im + no * ni].reshape(no, ni)
    W = np.empty((2 * no, 2 * ni), dtype=np.float32)
    W[0::2, 0::2] = A
    W[0::2, 1::2] = -Bm
    W[1::2, 0::2] = Bm
    W[1::2, 1::2] = A
    return W


def _act_fwd(act: int, c: np.ndarray, u: np.ndarray, v: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    f = np.float32
    if act == ACT_MODRELU:
        m = np.sqrt(u * u + v * v + f(1e-9))
        g = np.maximum(m + c, f(0)) / m
        return g * u, g * v
    if act == ACT_ZRELU:
        keep = (u >= 0) & (v >= 0)
        return np.where(keep, u, f(0)), np.where(keep, v, f(0))
    return u, v


def _act_bwd(act: int, c: np.ndarray, u: np.ndarray, v: np.ndarray, gr: np.ndarray,
             gi: np.ndarray) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    f = np.float32
    if act == ACT_MODRELU:
        m = np.sqrt(u * u + v * v + f(1e-9))
        on = m + c > 0
        dot = gr * u + gi * v
        dc = np.where(on, dot / m, f(0))
        g = (m + c) / m
        k = -dot * c / (m * m * m)
        return np.where(on, gr * g + k * u, f(0)), np.where(on, gi * g + k * v, f(0)), dc
    if act == ACT_ZRELU:
        keep = (u >= 0) & (v >= 0)
        return np.where(keep, gr, f(0)), np.where(keep, gi, f(0)), np.zeros_like(u)
    return gr, gi, np.zeros_like(u)


def cvnn_step(layers, params: np.ndarray, x_re: np.ndarray, x_im: np.ndarray | None, targets: np.ndarray,
              operand: str = "bf16") -> tuple[float, np.ndarray]:
    """Loss and the flat f32 gradient of one network step (before Adam)."""
    rnd = _rounder(operand)
    f = np.float32
    params = np.asarray(params, dtype=np.float32)
    x_re = np.asarray(x_re, dtype=np.float32)
    x_im = np.zeros_like(x_re) if x_im is None else np.asarray(x_im, dtype=np.float32)
    B = x_re.shape[0]
    N = layers[-1][1]
    z = rnd(_interleave(x_re, x_im))
    zs, pres, wcs = [], [], []
    for (ni, no, act, w_re, w_im, b_re, b_im, act_bias) in layers:
        wc = rnd(_wc(params, ni, no, w_re, w_im))
        pre = (z.astype(np.float64) @ wc.astype(np.float64).T).astype(f)
        u, v = pre[:, 0::2].copy(), pre[:, 1::2].copy()
        if b_re >= 0:
            u += params[b_re:b_re + no]
        if b_im >= 0:
            v += params[b_im:b_im + no]
        c = params[act_bias:act_bias + no] if act == ACT_MODRELU else np.zeros(no, f)
        ou, ov = _act_fwd(act, c, u, v)
        zs.append(z)
        pres.append((u, v, c))
        wcs.append(wc)
        z = rnd(_interleave(ou, ov))
    t = np.asarray(targets).astype(np.complex64)
    dr, di = ou - t.real, ov - t.imag
    loss = float((dr.astype(np.float64) ** 2).sum() + (di.astype(np.float64) ** 2).sum()) / (B * N)
    scale = f(2.0 / (float(B) * N))
    gr, gi = scale * dr, scale * di
    grads = np.zeros(params.shape[0], dtype=f)
    for l in range(len(layers) - 1, -1, -1):
        ni, no, act, w_re, w_im, b_re, b_im, act_bias = layers[l]
        u, v, c = pres[l]
        gu, gv, dc = _act_bwd(act, c, u, v, gr, gi)
        if act == ACT_MODRELU:
            grads[act_bias:act_bias + no] = dc.astype(np.float64).sum(axis=0).astype(f)
        gU = rnd(_interleave(gu, gv)).astype(np.float64)
        dW = (gU.T @ zs[l].astype(np.float64)).astype(f)  # [2 no][2 ni]
        grads[w_re:w_re + no * ni] = (dW[0::2, 0::2] + dW[1::2, 1::2]).reshape(-1)
        grads[w_im:w_im + no * ni] = (dW[1::2, 0::2] - dW[0::2, 1::2]).reshape(-1)
        db = gU.sum(axis=0).astype(f)
        if b_re >= 0:
            grads[b_re:b_re + no] = db[0::2]
        if b_im >= 0:
            grads[b_im:b_im + no] = db[1::2]
        if l > 0:
            gz = (gU @ wcs[l].astype(np.float64)).astype(f)
            gr, gi = gz[:, 0::2], gz[:, 1::2]
    return loss, grads


__all__ = ["bf16_round", "cvnn_step"]
