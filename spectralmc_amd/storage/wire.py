"""Checkpoint wire format: the reference's ``ModelCheckpointProto`` family, byte-compatible.

The reference compiles ``src/spectralmc/proto/{common,tensors}.proto`` with protoc at image
build time (``proto/__init__.py:1-20``); there is no protoc here, so the same messages are
declared programmatically (same package ``spectralmc.proto``, message names, field numbers
and types, proto3), which yields the identical encoding.  Converters follow
``serialization/tensors.py:33-593`` (TensorState / Adam / RNG / ModelCheckpoint) and
``serialization/common.py:19-110`` (dtype and device enums).
"""

from __future__ import annotations

from functools import lru_cache

import numpy as np
import torch
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from ..models.torch import (
    AdamOptimizerState,
    AdamParamState,
    Device,
    FullPrecisionDType,
    ReducedPrecisionDType,
    build_adam_optimizer_state,
    build_adam_param_group,
)
from ..result import Failure, Result, Success
from .errors import SerializationFailure

_PKG = "spectralmc.proto"
_FD = descriptor_pb2.FieldDescriptorProto

# enum values (common.proto)
DTYPE_FLOAT32, DTYPE_FLOAT64, DTYPE_FLOAT16, DTYPE_BFLOAT16, DTYPE_COMPLEX64, DTYPE_COMPLEX128 = 1, 2, 3, 4, 5, 6
DEVICE_CPU, DEVICE_CUDA = 1, 2

_DTYPES: tuple[tuple[int, object, torch.dtype, type], ...] = (
    (DTYPE_FLOAT32, FullPrecisionDType.float32, torch.float32, np.float32),
    (DTYPE_FLOAT64, FullPrecisionDType.float64, torch.float64, np.float64),
    (DTYPE_COMPLEX64, FullPrecisionDType.complex64, torch.complex64, np.complex64),
    (DTYPE_COMPLEX128, FullPrecisionDType.complex128, torch.complex128, np.complex128),
    (DTYPE_FLOAT16, ReducedPrecisionDType.float16, torch.float16, np.float16),
    (DTYPE_BFLOAT16, ReducedPrecisionDType.bfloat16, torch.bfloat16, np.uint16),
)


def _add_field(msg: descriptor_pb2.DescriptorProto, name: str, number: int, ftype: int, *,
               repeated: bool = False, type_name: str | None = None) -> None:
    f = msg.field.add(name=name, number=number, type=ftype,
                      label=_FD.LABEL_REPEATED if repeated else _FD.LABEL_OPTIONAL)
    if type_name is not None:
        f.type_name = type_name


def _add_map(msg: descriptor_pb2.DescriptorProto, name: str, number: int, key_type: int, value_type: int,
             value_type_name: str | None = None) -> None:
    entry = msg.nested_type.add(name="".join(w.capitalize() for w in name.split("_")) + "Entry")
    entry.options.map_entry = True
    _add_field(entry, "key", 1, key_type)
    _add_field(entry, "value", 2, value_type, type_name=value_type_name)
    _add_field(msg, name, number, _FD.TYPE_MESSAGE, repeated=True, type_name=f".{_PKG}.{msg.name}.{entry.name}")


def _common_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="common.proto", package=_PKG, syntax="proto3")
    for ename, values in (("PrecisionProto", ("PRECISION_UNSPECIFIED", "PRECISION_FLOAT32", "PRECISION_FLOAT64")),
                          ("DeviceProto", ("DEVICE_UNSPECIFIED", "DEVICE_CPU", "DEVICE_CUDA")),
                          ("DTypeProto", ("DTYPE_UNSPECIFIED", "DTYPE_FLOAT32", "DTYPE_FLOAT64", "DTYPE_FLOAT16",
                                          "DTYPE_BFLOAT16", "DTYPE_COMPLEX64", "DTYPE_COMPLEX128"))):
        e = fd.enum_type.add(name=ename)
        for i, v in enumerate(values):
            e.value.add(name=v, number=i)
    mv = fd.message_type.add(name="ModelVersionProto")
    _add_field(mv, "counter", 1, _FD.TYPE_UINT32)
    for i, n in enumerate(("semantic_version", "parent_hash", "content_hash", "commit_timestamp", "commit_message"), 2):
        _add_field(mv, n, i, _FD.TYPE_STRING)
    te = fd.message_type.add(name="TorchEnvProto")
    for i, n in enumerate(("python_version", "torch_version", "cuda_version"), 1):
        _add_field(te, n, i, _FD.TYPE_STRING)
    _add_field(te, "cudnn_enabled", 4, _FD.TYPE_BOOL)
    _add_field(te, "platform", 5, _FD.TYPE_STRING)
    af = fd.message_type.add(name="ArchitectureFingerprintProto")
    _add_field(af, "cvnn_structure_hash", 1, _FD.TYPE_STRING)
    _add_field(af, "total_parameters", 2, _FD.TYPE_UINT32)
    _add_field(af, "activation_kinds", 3, _FD.TYPE_STRING)
    return fd


def _tensors_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="tensors.proto", package=_PKG, syntax="proto3",
                                            dependency=["common.proto"])
    ts = fd.message_type.add(name="TensorStateProto")
    _add_field(ts, "shape", 1, _FD.TYPE_INT64, repeated=True)
    _add_field(ts, "dtype", 2, _FD.TYPE_ENUM, type_name=f".{_PKG}.DTypeProto")
    _add_field(ts, "device", 3, _FD.TYPE_ENUM, type_name=f".{_PKG}.DeviceProto")
    _add_field(ts, "data", 4, _FD.TYPE_BYTES)
    _add_field(ts, "requires_grad", 5, _FD.TYPE_BOOL)
    ps = fd.message_type.add(name="AdamParamStateProto")
    _add_field(ps, "step", 1, _FD.TYPE_INT32)
    _add_field(ps, "exp_avg", 2, _FD.TYPE_MESSAGE, type_name=f".{_PKG}.TensorStateProto")
    _add_field(ps, "exp_avg_sq", 3, _FD.TYPE_MESSAGE, type_name=f".{_PKG}.TensorStateProto")
    pg = fd.message_type.add(name="AdamParamGroupProto")
    for i, n in enumerate(("lr", "beta1", "beta2", "eps", "weight_decay"), 1):
        _add_field(pg, n, i, _FD.TYPE_DOUBLE)
    _add_field(pg, "amsgrad", 6, _FD.TYPE_BOOL)
    os_ = fd.message_type.add(name="AdamOptimizerStateProto")
    _add_map(os_, "state", 1, _FD.TYPE_INT32, _FD.TYPE_MESSAGE, f".{_PKG}.AdamParamStateProto")
    _add_field(os_, "param_groups", 2, _FD.TYPE_MESSAGE, repeated=True, type_name=f".{_PKG}.AdamParamGroupProto")
    rng = fd.message_type.add(name="RNGStateProto")
    _add_field(rng, "torch_cpu_rng_state", 1, _FD.TYPE_BYTES)
    _add_field(rng, "torch_cuda_rng_states", 2, _FD.TYPE_BYTES, repeated=True)
    ck = fd.message_type.add(name="ModelCheckpointProto")
    _add_map(ck, "model_state_dict", 1, _FD.TYPE_STRING, _FD.TYPE_MESSAGE, f".{_PKG}.TensorStateProto")
    _add_field(ck, "optimizer_state", 2, _FD.TYPE_MESSAGE, type_name=f".{_PKG}.AdamOptimizerStateProto")
    _add_field(ck, "rng_state", 3, _FD.TYPE_MESSAGE, type_name=f".{_PKG}.RNGStateProto")
    _add_field(ck, "global_step", 4, _FD.TYPE_UINT64)
    _add_field(ck, "torch_env", 5, _FD.TYPE_MESSAGE, type_name=f".{_PKG}.TorchEnvProto")
    _add_field(ck, "architecture", 6, _FD.TYPE_MESSAGE, type_name=f".{_PKG}.ArchitectureFingerprintProto")
    return fd


@lru_cache(maxsize=1)
def messages() -> dict[str, type]:
    """Message classes by name, from a private descriptor pool."""
    pool = descriptor_pool.DescriptorPool()
    pool.Add(_common_file())
    pool.Add(_tensors_file())
    names = ("ModelVersionProto", "TorchEnvProto", "ArchitectureFingerprintProto", "TensorStateProto",
             "AdamParamStateProto", "AdamParamGroupProto", "AdamOptimizerStateProto", "RNGStateProto",
             "ModelCheckpointProto")
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{n}")) for n in names}


# --------------------------------------------------------------------------- converters
def tensor_to_proto(t: torch.Tensor):
    """serialization/tensors.py:36-87: shape, dtype enum, device enum, raw little-endian bytes."""
    row = next((r for r in _DTYPES if r[2] == t.dtype), None)
    if row is None:
        return Failure(SerializationFailure(message=f"Unsupported dtype: {t.dtype}"))
    dev = Device.from_torch(t.device)
    if isinstance(dev, Failure):
        return Failure(SerializationFailure(message=str(dev.error)))
    msg = messages()["TensorStateProto"]()
    msg.shape.extend(t.shape)
    msg.dtype = row[0]
    msg.device = DEVICE_CUDA if dev.value is Device.cuda else DEVICE_CPU
    host = t.detach().cpu().contiguous()
    msg.data = (host.view(torch.uint16) if t.dtype == torch.bfloat16 else host).numpy().tobytes()
    msg.requires_grad = t.requires_grad
    return Success(msg)


def tensor_from_proto(msg) -> Result[torch.Tensor, SerializationFailure]:
    """serialization/tensors.py:89-160 (the tensor is placed on the recorded device)."""
    row = next((r for r in _DTYPES if r[0] == msg.dtype), None)
    if row is None:
        return Failure(SerializationFailure(message=f"Unknown dtype enum {msg.dtype}"))
    arr = np.frombuffer(msg.data, dtype=row[3]).reshape(tuple(msg.shape))
    t = torch.from_numpy(arr.copy())
    if row[2] == torch.bfloat16:
        t = t.view(torch.bfloat16)
    device = Device.cuda if msg.device == DEVICE_CUDA else Device.cpu
    t = t.to(device.to_torch())
    if msg.requires_grad:
        t.requires_grad_(True)
    return Success(t)


def adam_to_proto(state: AdamOptimizerState):
    msg = messages()["AdamOptimizerStateProto"]()
    for pid, ps in state.param_states.items():
        entry = msg.state[int(pid)]
        entry.step = int(ps.step)
        for name in ("exp_avg", "exp_avg_sq"):
            t = getattr(ps, name).to_torch()
            if isinstance(t, Failure):
                return Failure(SerializationFailure(message=str(t.error)))
            tp = tensor_to_proto(t.value)
            if isinstance(tp, Failure):
                return tp
            getattr(entry, name).CopyFrom(tp.value)
    for g in state.param_groups:
        msg.param_groups.add(lr=g.lr, beta1=g.betas[0], beta2=g.betas[1], eps=g.eps, weight_decay=g.weight_decay,
                             amsgrad=g.amsgrad)
    return Success(msg)


def adam_from_proto(msg) -> Result[AdamOptimizerState, SerializationFailure]:
    """serialization/tensors.py:321-411.  The proto carries no param-id lists; with a single
    group every stateful parameter id is assigned to it so the state can be loaded back into
    an optimizer (the reference leaves the list empty)."""
    states: dict[int, AdamParamState] = {}
    for pid in sorted(msg.state):
        entry = msg.state[pid]
        tensors = {}
        for name in ("exp_avg", "exp_avg_sq"):
            t = tensor_from_proto(getattr(entry, name))
            if isinstance(t, Failure):
                return t
            tensors[name] = t.value.cpu()
        ps = AdamParamState.from_torch({"step": int(entry.step), **tensors})
        if isinstance(ps, Failure):
            return Failure(SerializationFailure(message=str(ps.error)))
        states[int(pid)] = ps.value
    groups = []
    ids = sorted(states) if len(msg.param_groups) == 1 else []
    for g in msg.param_groups:
        built = build_adam_param_group({"params": ids, "lr": g.lr, "betas": (g.beta1, g.beta2), "eps": g.eps,
                                        "weight_decay": g.weight_decay, "amsgrad": g.amsgrad})
        if isinstance(built, Failure):
            return Failure(SerializationFailure(message=f"Invalid AdamParamGroup: {built.error}"))
        groups.append(built.value)
    out = build_adam_optimizer_state(param_states=states, param_groups=groups)
    if isinstance(out, Failure):
        return Failure(SerializationFailure(message=f"Invalid AdamOptimizerState: {out.error}"))
    return out


def checkpoint_to_proto(model_state_dict: dict[str, torch.Tensor], optimizer_state: AdamOptimizerState,
                        cpu_rng: bytes, cuda_rngs: list[bytes], global_step: int):
    """ModelCheckpointConverter.to_proto (serialization/tensors.py:458-527)."""
    msg = messages()["ModelCheckpointProto"]()
    for name, t in model_state_dict.items():
        tp = tensor_to_proto(t)
        if isinstance(tp, Failure):
            return tp
        msg.model_state_dict[name].CopyFrom(tp.value)
    op = adam_to_proto(optimizer_state)
    if isinstance(op, Failure):
        return op
    msg.optimizer_state.CopyFrom(op.value)
    msg.rng_state.torch_cpu_rng_state = cpu_rng
    msg.rng_state.torch_cuda_rng_states.extend(cuda_rngs)
    msg.global_step = int(global_step)
    return Success(msg)


def checkpoint_from_proto(msg):
    """ModelCheckpointConverter.from_proto (serialization/tensors.py:529-593)."""
    state: dict[str, torch.Tensor] = {}
    for name, tp in msg.model_state_dict.items():
        t = tensor_from_proto(tp)
        if isinstance(t, Failure):
            return t
        state[name] = t.value
    opt = adam_from_proto(msg.optimizer_state)
    if isinstance(opt, Failure):
        return opt
    return Success((state, opt.value, bytes(msg.rng_state.torch_cpu_rng_state),
                    [bytes(b) for b in msg.rng_state.torch_cuda_rng_states], int(msg.global_step)))


__all__ = ["messages", "tensor_to_proto", "tensor_from_proto", "adam_to_proto", "adam_from_proto",
           "checkpoint_to_proto", "checkpoint_from_proto"]
