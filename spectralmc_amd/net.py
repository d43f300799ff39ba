"""Fused network half of the training step on the HIP kernels of csrc/cvnn.hip.

``FusedNetworkStep`` replaces the torch-ROCm forward / spectral-MSE / backward / Adam of
``_torch_step`` (reference gbm_trainer.py:819-835) with a handful of launches when the CVNN is a
chain of ComplexLinear layers with optional modReLU / zReLU activations — the
architectures ``cvnn_factory`` builds without batch norm or residual blocks.  Other models
keep the torch path.

Kernels (``compute``):
  "auto"  f32 networks on the matrix cores (csrc/cvnn_mfma.hip, v_mfma_f32_16x16x4_f32) when the
          widths fit its LDS plan, else the VALU kernels of csrc/cvnn.hip; f64 on the VALU kernels
  "valu"  the VALU kernels (f32 / f64)
  "mfma"  the f32 MFMA kernels (error if the shape does not fit)
  "bf16"  bf16 operands on v_mfma_f32_16x16x32_bf16 with f32 accumulation and f32 master
          parameters / Adam (BASELINE.json configs[2]; an extension of the reference, which
          asserts full precision, gbm_trainer.py:679-686)

State stays where torch expects it: the model's parameters and the Adam moments become views
into flat device buffers (the kernels' layout), the Adam state dict keeps its keys
(``step`` is one shared capturable f32 counter), so ``state_dict()`` / snapshots / resume
are unchanged.
"""

from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib
from .cvnn import ComplexLinear, ComplexSequential, modReLU, zReLU


class UnsupportedNetwork(ValueError):
    """The model or optimiser configuration is outside what the fused kernels implement."""


def _flatten(m: nn.Module):
    if isinstance(m, ComplexSequential):
        for c in m.layers:
            yield from _flatten(c)
    else:
        yield m


def lower(model: nn.Module, params: list[nn.Parameter]) -> list[_lib.CvnnLayer]:
    """Layer table of ``model`` with element offsets into the flat ``params`` layout."""
    offsets, off = {}, 0
    for p in params:
        offsets[id(p)] = off
        off += p.numel()
    covered: set[int] = set()

    def at(p: nn.Parameter | None) -> int:
        if p is None:
            return -1
        covered.add(id(p))
        return offsets[id(p)]

    mods = list(_flatten(model))
    table: list[_lib.CvnnLayer] = []
    i = 0
    while i < len(mods):
        lin = mods[i]
        if not isinstance(lin, ComplexLinear):
            raise UnsupportedNetwork(f"expected ComplexLinear, got {type(lin).__name__}")
        act, act_bias = _lib.ACT_NONE, -1
        if i + 1 < len(mods) and isinstance(mods[i + 1], (modReLU, zReLU)):
            nxt = mods[i + 1]
            if isinstance(nxt, modReLU):
                act, act_bias = _lib.ACT_MODRELU, at(nxt.bias)
            else:
                act = _lib.ACT_ZRELU
            i += 1
        table.append(_lib.CvnnLayer(in_features=lin.in_features, out_features=lin.out_features, activation=act,
                                    reserved=0, w_re=at(lin.real_weight), w_im=at(lin.imag_weight),
                                    b_re=at(lin.real_bias), b_im=at(lin.imag_bias), act_bias=act_bias))
        i += 1
    if not table or len(table) > _lib.CVNN_MAX_LAYERS:
        raise UnsupportedNetwork(f"{len(table)} layers (1..{_lib.CVNN_MAX_LAYERS} supported)")
    if covered != {id(p) for p in params}:
        raise UnsupportedNetwork("model has parameters outside its ComplexLinear / modReLU chain")
    return table


class FusedNetworkStep:
    """Device buffers + launches of one network step; ``fwd_bwd`` then (DP) ``adam``."""

    def __init__(self, model: nn.Module, adam: torch.optim.Optimizer, params: list[nn.Parameter],
                 flat_grads: torch.Tensor, loss_out: torch.Tensor, grad_norm_out: torch.Tensor, batch: int,
                 fuse_adam: bool, compute: str = "auto") -> None:
        if len(adam.param_groups) != 1:
            raise UnsupportedNetwork("one Adam parameter group expected")
        g = adam.param_groups[0]
        if g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or g.get("decoupled_weight_decay"):
            raise UnsupportedNetwork("amsgrad / maximize / differentiable / decoupled Adam not fused")
        if [id(p) for p in g["params"]] != [id(p) for p in params]:
            raise UnsupportedNetwork("optimizer parameters differ from the model's")
        dtype = params[0].dtype
        if dtype not in (torch.float32, torch.float64) or any(p.dtype != dtype for p in params):
            raise UnsupportedNetwork(f"parameter dtype {dtype}")
        self.table = lower(model, params)
        self.dtype_code = _lib.DTYPE_F32 if dtype == torch.float32 else _lib.DTYPE_F64
        self.n = sum(p.numel() for p in params)
        self.batch = batch
        dev = params[0].device
        L = _lib.lib()
        self._layers = (_lib.CvnnLayer * len(self.table))(*self.table)
        if compute not in ("auto", "valu", "mfma", "bf16"):
            raise ValueError(f"compute must be auto / valu / mfma / bf16, not {compute!r}")
        self.mode = 0  # 0: VALU kernels, else SMC_CVNN_MFMA_F32 / SMC_CVNN_MFMA_BF16
        blocks, ws_bytes = ctypes.c_int64(), ctypes.c_int64()
        if compute != "valu" and dtype == torch.float32:
            mode = _lib.CVNN_MFMA_BF16 if compute == "bf16" else _lib.CVNN_MFMA_F32
            st = L.smc_cvnn_mfma_plan(self._layers, len(self.table), mode, batch, ctypes.byref(blocks),
                                      ctypes.byref(ws_bytes))
            if st == _lib.SMC_OK:
                self.mode = mode
            elif compute != "auto":
                raise UnsupportedNetwork(f"MFMA network kernels: {_lib.last_error()}")
        elif compute in ("mfma", "bf16"):
            raise UnsupportedNetwork(f"MFMA network kernels take f32 parameters, not {dtype}")
        if self.mode:
            self.workspace = torch.empty(ws_bytes.value, dtype=torch.uint8, device=dev)
        else:
            _lib.check(L.smc_cvnn_plan(self._layers, len(self.table), self.dtype_code, batch, ctypes.byref(blocks)))
            self.workspace = None
        self.blocks = blocks.value
        self.partials = torch.empty((self.blocks, self.n + 1), dtype=dtype, device=dev)
        # (zeroed: its last slot is the fused finalize's arrival counter, which every update leaves at zero)
        self.norm_partials = torch.zeros(int(L.smc_adam_norm_partials(self.n)), dtype=torch.float64, device=dev)
        self.grads = flat_grads
        # parameters and Adam moments -> flat buffers (views keep torch's objects valid)
        self.params_flat = torch.empty(self.n, dtype=dtype, device=dev)
        self.exp_avg = torch.zeros(self.n, dtype=dtype, device=dev)
        self.exp_avg_sq = torch.zeros(self.n, dtype=dtype, device=dev)
        step0 = 0.0
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                st = adam.state.get(p, {})
                self.params_flat[off:off + k].copy_(p.detach().reshape(-1))
                if "exp_avg" in st:
                    self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                    self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                    step0 = float(st["step"])
                p.data = self.params_flat[off:off + k].view_as(p)
                off += k
        self.step = torch.tensor(step0, dtype=torch.float32, device=dev)
        off = 0
        for p in params:
            k = p.numel()
            adam.state[p] = {"step": self.step, "exp_avg": self.exp_avg[off:off + k].view_as(p),
                             "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p)}
            off += k
        b1, b2 = g["betas"]
        self.adam_args = _lib.AdamArgs(params=_lib.ptr(self.params_flat), exp_avg=_lib.ptr(self.exp_avg),
                                       exp_avg_sq=_lib.ptr(self.exp_avg_sq), step=_lib.ptr(self.step),
                                       lr=float(g["lr"]), beta1=float(b1), beta2=float(b2), eps=float(g["eps"]),
                                       weight_decay=float(g["weight_decay"]),
                                       norm_partials=_lib.ptr(self.norm_partials), grad_norm=_lib.ptr(grad_norm_out),
                                       loss=_lib.ptr(loss_out))
        self.fuse_adam = fuse_adam
        # MFMA (non-layered plans): Adam also writes the packed operand copies of the weights it updates, so
        # every fwd_bwd after the first skips its pack launch (SMC_CVNN_MFMA_PACKED; the e2e network chain's
        # 9 us pack_kernel, profiles/r05/).  The model's parameters are views of params_flat: any write to them
        # other than Adam's must be followed by invalidate_pack()
        self._pack = None
        self._packed = False
        if self.mode:
            pk = _lib.CvnnPack()
            _lib.check(L.smc_cvnn_mfma_pack_plan(self._layers, len(self.table), self.mode, batch,
                                                 _lib.ptr(self.workspace), ctypes.byref(pk)))
            if pk.n_layers > 0:
                self._pack = pk
                self.adam_args.pack = ctypes.addressof(pk)

    def fwd_bwd(self, real_in: torch.Tensor, imag_in: torch.Tensor | None, targets: torch.Tensor,
                stream: int | None = None) -> None:
        """Gradients + loss into the flat buffer (and, fused, the Adam step) on the current stream (or the
        hipStream_t ``stream``)."""
        L = _lib.lib()
        stream = stream if stream is not None else _lib.stream_handle()
        if self.mode:
            mode = self.mode | (_lib.CVNN_MFMA_PACKED if self._packed else 0)
            _lib.check(L.smc_cvnn_mfma_forward_backward(
                self._layers, len(self.table), mode, _lib.ptr(self.params_flat), self.n, _lib.ptr(real_in),
                _lib.ptr(imag_in) if imag_in is not None else None, _lib.ptr(targets), self.batch,
                _lib.ptr(self.partials), self.blocks, _lib.ptr(self.workspace), self.workspace.numel(), stream))
        else:
            _lib.check(L.smc_cvnn_forward_backward(self._layers, len(self.table), self.dtype_code,
                                                   _lib.ptr(self.params_flat), self.n, _lib.ptr(real_in),
                                                   _lib.ptr(imag_in) if imag_in is not None else None,
                                                   _lib.ptr(targets), self.batch, _lib.ptr(self.partials),
                                                   self.blocks, stream))
        _lib.check(L.smc_cvnn_reduce_grads(self.dtype_code, _lib.ptr(self.partials), self.blocks, self.n,
                                           _lib.ptr(self.grads),
                                           ctypes.byref(self.adam_args) if self.fuse_adam else None, stream))
        if self.fuse_adam and self._pack is not None:
            self._packed = True  # this update wrote the operand copies the next forward_backward reads

    def invalidate_pack(self) -> None:
        """The parameters changed other than through this step's Adam update (a state_dict load into the live
        model, a broadcast into params_flat): the next fwd_bwd runs its pack launch again instead of reading
        the packed operand copies the last update wrote (SMC_CVNN_MFMA_PACKED, include/spectralmc_hip.h)."""
        self._packed = False

    @property
    def kernels(self) -> str:
        return {0: "valu", _lib.CVNN_MFMA_F32: "mfma_f32", _lib.CVNN_MFMA_BF16: "mfma_bf16"}[self.mode]

    def adam(self, stream: int | None = None) -> None:
        """Adam + grad norm + loss copy from the (all-reduced) flat buffer."""
        _lib.check(_lib.lib().smc_adam_step(self.dtype_code, self.n, _lib.ptr(self.grads),
                                            ctypes.byref(self.adam_args),
                                            stream if stream is not None else _lib.stream_handle()))
        if self._pack is not None:
            self._packed = True


__all__ = ["FusedNetworkStep", "UnsupportedNetwork", "lower"]
